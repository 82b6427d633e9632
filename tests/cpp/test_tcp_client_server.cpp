// GpuTcpClient talking to GpuTcpServer: both of the reference's example programs' handlers
// (example/tcpclient.cc:68-95 and example/tcpserver.cc:61-90, extracted verbatim into
// oracle/_ref/ by oracle/ref.mk) compiled unchanged against the two drop-ins, connected by an
// in-memory wire that loses frames in both directions, under a simulated clock advancing one
// millisecond per poll.  The example client writes a 16-B Packet {ts, val} on every send
// timeout (1 s); the example server echoes it; the client prints each echo's value and
// latency.  `cout`, `exit`, `getns()` and the globals the handlers name (`client`, `server`,
// `pack`) are test-local: getns() is the simulated clock.
//
// Runs: twin (both ends on the sequential oracle backend) and, with `gpu`, both ends on the
// GPU backend — every poll of either end one pn_classify launch for what it received and one
// pn_tx_fill launch for what it sent.  Checks: the client connects, gets every value echoed
// in order (the stream is reliable over the lossy wire), both handler logs and every frame on
// the wire equal between the two runs; then the client closes (RST), the server sees it go, and
// the client reconnects (its retry interval has passed).
//   argv: twin | gpu  [runs]  [show]   exit 0 = pass (runs: loss patterns, seed 0..runs-1)
#include <arpa/inet.h>

#include <cstdio>
#include <cstring>
#include <iostream>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/pollnet_amd/tcp_client.hpp"
#include "../../oracle/ref_server.hpp"
#include "../../include/pollnet_amd/tcp_server.hpp"
#include "segframes.hpp"
#include "server_harness.hpp"

using namespace std;
using namespace pollnet_amd;

struct ServerConf { // example/tcpserver.cc:4-14
  static const uint32_t RecvBufSize = 4096;
  static const uint32_t MaxConns = 10;
  static const uint32_t SendTimeoutSec = 0;
  static const uint32_t RecvTimeoutSec = 10;
  static const uint32_t ConnSendBufCnt = 64;
  static const uint32_t RxBatch = 256;
  static const uint32_t TxBatch = 64;
  struct UserData {
    struct sockaddr_in addr;
  };
};
struct ClientConf { // example/tcpclient.cc:3-14
  static const uint32_t RecvBufSize = 4096;
  static const uint32_t ConnRetrySec = 5;
  static const uint32_t ConnTimeoutSec = 5;
  static const uint32_t SendTimeoutSec = 1;
  static const uint32_t RecvTimeoutSec = 3;
  static const uint32_t ConnSendBufCnt = 64;
  static const uint32_t RxBatch = 256;
  static const uint32_t TxBatch = 64;
  struct UserData {};
};

// Two queues; what one end sends reaches the other end's next fill, unless lost.
struct Wire {
  std::vector<std::vector<uint8_t>> to_server, to_client, log; // log: every frame sent, both ways
  std::mt19937 loss;
  explicit Wire(uint32_t seed = 0) : loss(0x10553u + 0x9E3779B9u * seed) {}
  uint32_t drops = 0;
  uint32_t loss_pct = 4;
  void carry(std::vector<std::vector<uint8_t>>& q, const uint8_t* eth, uint32_t len) {
    log.emplace_back(eth, eth + len);
    if (loss() % 100 < loss_pct) {
      drops++;
      return;
    }
    q.emplace_back(eth, eth + len);
  }
};
static Wire* g_wire = nullptr;

static const uint8_t kServerMac[6] = {2, 0, 0, 0, 0, 1}, kClientMac[6] = {2, 0, 0, 0, 0, 2};

template <bool kServerSide>
struct WireLink {
  const char* open(const char*) { return nullptr; }
  uint32_t fill(uint8_t* slots, uint32_t stride, uint32_t off, uint32_t cap) {
    auto& q = kServerSide ? g_wire->to_server : g_wire->to_client;
    uint32_t n = 0;
    for (; n < cap && n < q.size(); n++) {
      uint8_t* s = slots + (size_t)n * stride;
      std::memset(s, 0, stride);
      std::memcpy(s + off, q[n].data(), q[n].size());
    }
    q.erase(q.begin(), q.begin() + n);
    return n;
  }
  void send(const uint8_t* eth, uint32_t len) { g_wire->carry(kServerSide ? g_wire->to_client : g_wire->to_server, eth, len); }
  uint32_t localIp() const { return htonl(kServerSide ? 0x0a000001 : 0x0a000002); }
  const uint8_t* localMac() const { return kServerSide ? kServerMac : kClientMac; }
  const char* resolveMac(uint32_t, uint8_t* mac) {
    std::memcpy(mac, kServerSide ? kClientMac : kServerMac, 6);
    return nullptr;
  }
};

static const int64_t kT0 = (int64_t)1700000000 << 30; // simulated clock origin (ns)
static int64_t g_now = kT0;

// The example client's `Packet` and `getns()` (example/tcpclient.cc:32-36, timestamp.h)
struct Packet {
  uint64_t ts = 0;
  uint64_t val = 0;
};
static uint64_t getns() { return (uint64_t)g_now; }

// the same ends in the pipelined RX mode (each poll's frames dispatched in the next poll)
struct ServerConfPipe : ServerConf {
  static const bool RxPipeline = true;
};
struct ClientConfPipe : ClientConf {
  static const bool RxPipeline = true;
};

#define PN_DEFINE_ENDS(NS, BACKEND, SCONF, CCONF)                                   \
  namespace NS {                                                                    \
  using TcpServer = GpuTcpServer<SCONF, WireLink<true>, BACKEND>;                   \
  using TcpClient = GpuTcpClient<CCONF, WireLink<false>, BACKEND>;                  \
  TcpServer& server = *new TcpServer;                                               \
  TcpClient& client = *new TcpClient;                                               \
  Packet pack;                                                                      \
  namespace srv {                                                                   \
  LogStream cout;                                                                   \
  int exits = 0;                                                                    \
  void exit(int) { ++exits; }                                                       \
  void pollOnce() {
#define PN_END_SERVER                                                               \
  server.poll(handler, g_now);                                                      \
  }                                                                                 \
  }                                                                                 \
  namespace cli {                                                                   \
  LogStream cout;                                                                   \
  int exits = 0;                                                                    \
  void exit(int) { ++exits; }                                                       \
  void pollOnce() {
#define PN_END_CLIENT                                                               \
  client.poll(handler, g_now);                                                      \
  }                                                                                 \
  }                                                                                 \
  }

PN_DEFINE_ENDS(on_twin, OracleBackend, ServerConf, ClientConf)
#include "../../oracle/_ref/tcpserver_handler.inc"
PN_END_SERVER
#include "../../oracle/_ref/tcpclient_handler.inc"
PN_END_CLIENT

PN_DEFINE_ENDS(on_gpu, GpuBackend, ServerConf, ClientConf)
#include "../../oracle/_ref/tcpserver_handler.inc"
PN_END_SERVER
#include "../../oracle/_ref/tcpclient_handler.inc"
PN_END_CLIENT

PN_DEFINE_ENDS(on_twin_pipe, OracleBackend, ServerConfPipe, ClientConfPipe)
#include "../../oracle/_ref/tcpserver_handler.inc"
PN_END_SERVER
#include "../../oracle/_ref/tcpclient_handler.inc"
PN_END_CLIENT

PN_DEFINE_ENDS(on_gpu_pipe, GpuBackend, ServerConfPipe, ClientConfPipe)
#include "../../oracle/_ref/tcpserver_handler.inc"
PN_END_SERVER
#include "../../oracle/_ref/tcpclient_handler.inc"
PN_END_CLIENT

// Both ends as the reference's own EfviTcpServer / EfviTcpClient (oracle/ref_server.hpp: efvitcp's
// TcpServer, TcpClient, TcpConn and Core compiled from /root/reference, ef_vi plumbing restated)
#define PN_DEFINE_REF_ENDS(NS)                                                      \
  namespace NS {                                                                    \
  using TcpServer = efvitcp::EfviTcpServer<ServerConf>;                             \
  using TcpClient = efvitcp::EfviTcpClient<ClientConf>;                             \
  TcpServer& server = *new TcpServer;                                               \
  TcpClient& client = *new TcpClient;                                               \
  Packet pack;                                                                      \
  namespace srv {                                                                   \
  LogStream cout;                                                                   \
  int exits = 0;                                                                    \
  void exit(int) { ++exits; }                                                       \
  void pollOnce() {

PN_DEFINE_REF_ENDS(on_ref)
#include "../../oracle/_ref/tcpserver_handler.inc"
PN_END_SERVER
#include "../../oracle/_ref/tcpclient_handler.inc"
PN_END_CLIENT

struct Result {
  std::string srv_log, cli_log;
  std::vector<std::vector<uint8_t>> wire;
  uint32_t drops = 0, echoed = 0, conns_after = 0;
  bool connected = false, closed_seen = false;
};

template <class S, class C>
static bool run(S& server, C& client, void (*poll_srv)(), void (*poll_cli)(), LogStream& slog, LogStream& clog,
                Result& out, uint32_t seed) {
  Wire w(seed);
  slog.os.str(std::string());
  clog.os.str(std::string());
  static Wire drain; // a re-init closes the previous run's connections (RSTs): not part of this run
  g_wire = &drain;
  g_now = kT0;
  if (!server.initWithLink("10.0.0.1", 1234, g_now)) return std::printf("server init: %s\n", server.getLastError()), false;
  if (!client.initWithLink("10.0.0.2", "10.0.0.1", 1234, 40000, g_now))
    return std::printf("client init: %s\n", client.getLastError()), false;
  g_wire = &w;
  const int64_t ms = 1 << 20; // one tick (ns >> 20)
  for (int t = 0; t < 22000; t++) {  // ~22 s of simulated time: ~20 send timeouts
    g_now += ms;
    poll_cli();
    poll_srv();
  }
  out.connected = client.isConnected();
  // the client closes (RST): the server must see the connection go
  client.close("bye");
  for (int t = 0; t < 3000; t++) { // the reconnect, and its first send timeout
    g_now += ms;
    poll_cli();
    poll_srv();
  }
  out.conns_after = server.getConnCnt();
  out.srv_log = slog.os.str();
  out.cli_log = clog.os.str();
  out.wire = w.log;
  out.drops = w.drops;
  static Wire sink; // frames sent after the run (the ends' destructors RST open connections)
  g_wire = &sink;
  return true;
}

// The reference ends: the same wire, clock and script; their ef_vi plumbing goes to WireLinks.
static bool run_ref(Result& out, uint32_t seed, bool wall_clock = false) {
  using namespace on_ref;
  static WireLink<true> slink;
  static WireLink<false> clink;
  // fresh ends for every run: the reference's init re-arms nothing (its timer lists, ids and table
  // are set up for one init per object), so a second init over live connections is not meaningful
  static Wire drain;
  g_wire = &drain; // the old ends' destructors RST their connections
  server.~TcpServer();
  client.~TcpClient();
  new (&server) TcpServer;
  new (&client) TcpClient;
  Wire w(seed);
  srv::cout.os.str(std::string());
  cli::cout.os.str(std::string());
  g_wire = &w;
  g_now = kT0;
  efvitcp::RefEnv& env = efvitcp::refEnv();
  env.now_ns = g_now;
  env.init_ns = g_now;
  env.wall_clock_time = wall_clock;
  env.link = &slink;
  env.fill = [](void* l, uint8_t* s, uint32_t st, uint32_t off, uint32_t cap) {
    return static_cast<WireLink<true>*>(l)->fill(s, st, off, cap);
  };
  env.send = [](void* l, const uint8_t* eth, uint32_t len) { static_cast<WireLink<true>*>(l)->send(eth, len); };
  env.local_ip = slink.localIp();
  std::memcpy(env.local_mac, kServerMac, 6);
  if (!server.init("wire", "10.0.0.1", 1234)) return std::printf("ref server init: %s\n", server.getLastError()), false;
  env.link = &clink;
  env.fill = [](void* l, uint8_t* s, uint32_t st, uint32_t off, uint32_t cap) {
    return static_cast<WireLink<false>*>(l)->fill(s, st, off, cap);
  };
  env.send = [](void* l, const uint8_t* eth, uint32_t len) { static_cast<WireLink<false>*>(l)->send(eth, len); };
  env.local_ip = clink.localIp();
  std::memcpy(env.local_mac, kClientMac, 6);
  std::memcpy(env.peer_mac, kServerMac, 6);
  if (!client.init("wire", "10.0.0.1", 1234, 40000)) return std::printf("ref client init: %s\n", client.getLastError()), false;
  const int64_t ms = 1 << 20;
  for (int t = 0; t < 22000; t++) {
    g_now += ms;
    env.now_ns = g_now;
    cli::pollOnce();
    srv::pollOnce();
  }
  out.connected = client.isConnected();
  client.close("bye");
  for (int t = 0; t < 3000; t++) {
    g_now += ms;
    env.now_ns = g_now;
    cli::pollOnce();
    srv::pollOnce();
  }
  out.conns_after = server.getConnCnt();
  out.srv_log = srv::cout.os.str();
  out.cli_log = cli::cout.os.str();
  out.wire = w.log;
  out.drops = w.drops;
  static Wire sink;
  g_wire = &sink;
  env.wall_clock_time = false;
  return true;
}

// The reconnect clock, the one other intended difference: EfviTcpClient::poll times its reconnect
// interval with time(0), the host's wall clock (EfviTcp.h:116-121), whatever `ns` the caller polls
// with; GpuTcpClient times it on the poll's clock.  Under a simulated clock (25 s of polls in well
// under a second of wall time) the reference client with the real time(0) does not reconnect after
// close("bye") (5-s ConnRetrySec not yet passed on the wall clock); the product does, as the
// reference does when its time(0) follows the same clock (the runs above).
static int reconnect_clock_divergence() {
  Result r;
  if (!run_ref(r, 0, true)) return 1;
  size_t conns = 0;
  for (size_t p = 0; (p = r.srv_log.find("new connection from", p)) != std::string::npos; p++) conns++;
  const bool ok = conns == 1 && r.conns_after == 0;
  std::printf("reconnect clock: reference client on the wall clock made %zu connection(s), %u open after the close "
              "(product on the poll clock: 2, 1) -> %s\n",
              conns, r.conns_after, ok ? "as documented" : "UNEXPECTED");
  return ok ? 0 : 1;
}

static int check(const char* tag, const Result& r) {
  int fail = 0;
  // the client printed "recv val: k ..." for k = 1, 2, ... in order
  uint32_t expect = 1;
  std::istringstream is(r.cli_log);
  std::string line;
  while (std::getline(is, line)) {
    unsigned v;
    if (std::sscanf(line.c_str(), "recv val: %u", &v) == 1) {
      if (v != expect) fail++;
      expect++;
    }
  }
  const uint32_t echoed = expect - 1;
  uint32_t bad = 0;
  for (auto& f0 : r.wire) {
    std::vector<uint8_t> f(f0);
    f.resize(f0.size() + 2, 0);
    const pn_result x = segtest::classify(f.data(), (uint32_t)f.size());
    bad += (x.flags & (PN_F_IP_OK | PN_F_TCP_OK)) != (PN_F_IP_OK | PN_F_TCP_OK);
  }
  const bool disc = r.srv_log.find("client disconnected") != std::string::npos;
  size_t conns = 0;
  for (size_t p = 0; (p = r.srv_log.find("new connection from", p)) != std::string::npos; p++) conns++;
  std::printf("%s: %zu frames on the wire (%u lost, %u bad checksums), client connected %d, %u values echoed in "
              "order, server saw the close %d, connections accepted %zu, open after the close %u\n",
              tag, r.wire.size(), r.drops, bad, r.connected, echoed, disc, conns, r.conns_after);
  // after close("bye") the client reconnects at once (ConnRetrySec = 5 s have long passed,
  // EfviTcp.h:92-104): the server sees the old connection go and a new one arrive
  if (!r.connected || echoed < 18 || bad || !disc || conns != 2 || r.conns_after != 1) fail++;
  if (r.cli_log.find("onTcpConnected") == std::string::npos) fail++;
  return fail;
}

int main(int argc, char** argv) {
  const bool gpu = argc > 1 && std::strcmp(argv[1], "gpu") == 0;
  const uint32_t runs = argc > 2 ? (uint32_t)std::atoi(argv[2]) : 1; // loss patterns (run k: seed k)
  const bool show = argc > 3;
  int fail = 0;
  // one mode: the twin run, then (gpu) the GPU run, which must equal it frame for frame
  auto mode = [&](const char* name, auto& ts, auto& tc, void (*tps)(), void (*tpc)(), LogStream& tsl, LogStream& tcl,
                  Packet& tpack, auto& gs, auto& gc, void (*gps)(), void (*gpc)(), LogStream& gsl, LogStream& gcl,
                  Packet& gpack, uint32_t seed) -> int {
    int f = 0;
    tpack = Packet{}; // the example client's running counter starts over
    gpack = Packet{};
    Result tw;
    if (!run(ts, tc, tps, tpc, tsl, tcl, tw, seed)) return 100;
    f += check((std::string("twin") + name).c_str(), tw);
    if (!name[0]) { // the classify-every-poll ends against the reference's own ends
      on_ref::pack = Packet{};
      Result rr;
      if (!run_ref(rr, seed)) return 100;
      f += check("reference", rr);
      const bool logs = rr.srv_log == tw.srv_log && rr.cli_log == tw.cli_log;
      size_t same = 0;
      while (same < rr.wire.size() && same < tw.wire.size() && rr.wire[same] == tw.wire[same]) same++;
      const bool wire = same == rr.wire.size() && same == tw.wire.size();
      std::printf("twin vs reference EfviTcpServer/EfviTcpClient: handler logs %s, wire frames %s (%zu vs %zu%s)\n",
                  logs ? "identical" : "DIFFERENT", wire ? "identical" : "DIFFERENT", tw.wire.size(), rr.wire.size(),
                  wire ? "" : (", first difference at " + std::to_string(same)).c_str());
      f += !logs + !wire;
      if (!wire) {
        auto dump = [](const char* t, const std::vector<uint8_t>& x) {
          std::printf("  %s %zu B:", t, x.size());
          for (size_t i = 0; i < x.size() && i < 64; i++) std::printf(" %02x", x[i]);
          std::printf("\n");
        };
        if (same < tw.wire.size()) dump("twin", tw.wire[same]);
        if (same < rr.wire.size()) dump("ref ", rr.wire[same]);
      }
    }
    if (show) std::printf("server log:\n%s\nclient log:\n%s\n", tw.srv_log.c_str(), tw.cli_log.c_str());
    if (gpu) {
      Result g;
      if (!run(gs, gc, gps, gpc, gsl, gcl, g, seed)) return 100;
      f += check((std::string("gpu") + name).c_str(), g);
      const bool logs = g.srv_log == tw.srv_log && g.cli_log == tw.cli_log;
      const bool wire = g.wire == tw.wire;
      std::printf("gpu%s: handler logs %s, wire frames %s (%zu)\n", name, logs ? "identical" : "DIFFERENT",
                  wire ? "identical" : "DIFFERENT", g.wire.size());
      f += !logs + !wire;
    }
    return f;
  };
  fail += reconnect_clock_divergence();
  for (uint32_t seed = 0; seed < runs; seed++) {
    if (runs > 1) std::printf("== loss pattern %u ==\n", seed);
    fail += mode("", on_twin::server, on_twin::client, on_twin::srv::pollOnce, on_twin::cli::pollOnce,
                 on_twin::srv::cout, on_twin::cli::cout, on_twin::pack, on_gpu::server, on_gpu::client,
                 on_gpu::srv::pollOnce, on_gpu::cli::pollOnce, on_gpu::srv::cout, on_gpu::cli::cout, on_gpu::pack, seed);
    fail += mode(" (pipelined)", on_twin_pipe::server, on_twin_pipe::client, on_twin_pipe::srv::pollOnce,
                 on_twin_pipe::cli::pollOnce, on_twin_pipe::srv::cout, on_twin_pipe::cli::cout, on_twin_pipe::pack,
                 on_gpu_pipe::server, on_gpu_pipe::client, on_gpu_pipe::srv::pollOnce, on_gpu_pipe::cli::pollOnce,
                 on_gpu_pipe::srv::cout, on_gpu_pipe::cli::cout, on_gpu_pipe::pack, seed);
  }
  if (gpu) {
    delete &on_gpu::client;
    delete &on_gpu::server;
    delete &on_gpu_pipe::client;
    delete &on_gpu_pipe::server;
  }
  std::printf("%s\n", fail ? "FAIL" : "PASS");
  return fail ? 1 : 0;
}
