// GpuTcpClient against the reference's OWN EfviTcpClient / efvitcp::TcpClient (oracle/ref_server.hpp),
// both facing the same scripted, adversarial server on a simulated clock (one millisecond per poll).
//
// The server script answers each SYN in one of six ways (SYN-ACK; SYN-ACK with a wrong ack number; RST|ACK
// acknowledging the SYN; a bare RST; a bare SYN; silence), so the client's SYN-SENT branch
// (TcpClient.h:85-98: RST to a bad ACK, "connection refused", SYN retransmission, connect failure) and its
// reconnect interval (EfviTcp.h:113-126) all run.  Once a connection is up, the server sends the client a
// stream in adversarial segments (reordered into 5+ extents, duplicated, overlapping, without ACK, with SYN,
// far out of the window, RSTs in and out of it), ACKs what the client writes, then FINs.  The client's
// handler writes on connect and on every 3rd data delivery and consumes whole 8-byte words only.
// The script is a deterministic function of what it receives, so any difference in the clients' behaviour
// shows up as a different frame sequence: every frame the client sends (byte for byte) and the handler log
// must be identical.   argv: twin | gpu [scripts]     exit 0 = pass
#include <sys/uio.h>
#include <arpa/inet.h>

#include <cstdio>
#include <cstring>
#include <memory>
#include <random>
#include <string>
#include <vector>

#include "../../include/pollnet_amd/tcp_client.hpp"
#include "../../oracle/ref_server.hpp"
#include "segframes.hpp"
#include "server_harness.hpp"

using pollnet_amd::GpuBackend;
using pollnet_amd::GpuTcpClient;

static const int64_t kT0 = (int64_t)901234 << 20;
static const uint32_t kSrvIp = 0x0a000001, kCliIp = 0x0a000002;
static const uint16_t kSrvPort = 1234, kCliPort = 40000;
static const uint8_t kSrvMac[6] = {2, 0, 0, 0, 0, 1}, kCliMac[6] = {2, 0, 0, 0, 0, 2};

struct RefCliConf { // pollnet's EfviTcpClient Conf
  static const uint32_t RecvBufSize = 8192;
  static const uint32_t ConnRetrySec = 1;
  static const uint32_t SendTimeoutSec = 0;
  static const uint32_t RecvTimeoutSec = 2;
  struct UserData {
    uint32_t deliveries = 0;
  };
};
struct ProdCliConf : RefCliConf {
  static const uint32_t RxBatch = 64; // the reference's 64 events per pollNet (Core.h:498)
};
struct ProdCliConfResident : ProdCliConf {
  static const bool RxResident = true; // each poll's classify posted to the resident service (pn_service_*)
};

// The scripted server, as the client's link: fill() = the server's frames for this tick, send() = a client
// frame (handled when the poll ends: a wire one poll long).
struct ScriptServer {
  std::mt19937_64 rng;
  uint32_t tick = 0, conns = 0;
  enum { kListen, kSynAcked, kEst, kClosed } st = kListen;
  uint32_t srv_isn = 0, cli_nxt = 0;  // client's next expected seq (what the server has received in order)
  uint32_t srv_una = 0;               // server stream bytes the client acknowledged
  std::vector<uint8_t> stream;        // server -> client
  struct Sg {
    uint32_t off, len;
    uint8_t flags;
    int32_t shift;
  };
  std::vector<Sg> sched;
  size_t pos = 0;
  uint32_t last_tx = 0, fin_tries = 0;
  std::vector<std::vector<uint8_t>> q, in_flight, out; // to the client; client frames in flight; every client frame

  explicit ScriptServer(uint64_t seed = 0) : rng(seed) {}
  const char* open(const char*) { return nullptr; }
  uint32_t localIp() const { return htonl(kCliIp); }
  const uint8_t* localMac() const { return kCliMac; }
  const char* resolveMac(uint32_t, uint8_t* mac) {
    std::memcpy(mac, kSrvMac, 6);
    return nullptr;
  }

  void emit(uint32_t seq, uint32_t ack, uint8_t flags, const uint8_t* p = nullptr, uint32_t len = 0, bool mss = false) {
    segtest::Seg s;
    s.src_ip = kSrvIp;
    s.src_port = kSrvPort;
    s.seq = seq;
    s.ack = ack;
    s.flags = flags;
    s.payload = p;
    s.len = len;
    if (mss) s.opts = {2, 4, 0x05, 0xb4};
    uint8_t buf[2048];
    uint32_t n = segtest::build(buf, s);
    // segtest builds client -> server frames: swap the addresses and ports, then fix both checksums
    std::memcpy(buf, kCliMac, 6);
    std::memcpy(buf + 6, kSrvMac, 6);
    segtest::put32(buf + 26, kSrvIp);
    segtest::put32(buf + 30, kCliIp);
    segtest::put16(buf + 34, kSrvPort);
    segtest::put16(buf + 36, kCliPort);
    segtest::put16(buf + 24, 0);
    segtest::put16(buf + 24, segtest::rfc_sum(buf + 14, 20, 0));
    segtest::put16(buf + 48, 30000); // the server's window
    segtest::put16(buf + 50, 0);
    const uint32_t tcp_len = n - 34;
    const uint32_t ph = (kSrvIp >> 16) + (kSrvIp & 0xffff) + (kCliIp >> 16) + (kCliIp & 0xffff) + 6 + tcp_len;
    segtest::put16(buf + 50, segtest::rfc_sum(buf + 34, tcp_len, ph));
    q.emplace_back(buf, buf + n);
  }

  void newStream() {
    auto U = [&](uint32_t lo, uint32_t hi) { return lo + (uint32_t)(rng() % (hi - lo + 1)); };
    stream.resize(U(1, 20000));
    for (auto& b : stream) b = (uint8_t)rng();
    sched.clear();
    pos = 0;
    const uint32_t L = (uint32_t)stream.size();
    std::vector<std::pair<uint32_t, uint32_t>> pk;
    for (uint32_t o = 0; o < L;) {
      const uint32_t n = std::min(L - o, U(1, 1460));
      pk.push_back({o, n});
      o += n;
    }
    const uint32_t W = U(1, 7);
    for (size_t b = 0; b < pk.size(); b += W) {
      std::vector<std::pair<uint32_t, uint32_t>> blk(pk.begin() + b, pk.begin() + std::min(pk.size(), b + W));
      std::shuffle(blk.begin(), blk.end(), rng);
      for (auto& x : blk) {
        Sg g{x.first, x.second, (uint8_t)(segtest::ACK | segtest::PSH), 0};
        const uint32_t r = (uint32_t)(rng() % 100);
        if (r < 3) g.flags = segtest::PSH;
        else if (r < 5) g.flags |= segtest::SYN;
        else if (r < 8) g.shift = 30000 + (int32_t)(rng() % 50000);
        else if (r < 10) g.shift = -(int32_t)(10000 + rng() % 30000);
        sched.push_back(g);
        if (rng() % 8 == 0) sched.push_back(sched[rng() % sched.size()]);
        if (rng() % 10 == 0) sched.push_back({x.first / 2, std::min(L - x.first / 2, U(1, 1460)), (uint8_t)(segtest::ACK | segtest::PSH), 0});
        if (rng() % 200 == 0) sched.push_back({x.first, 0, (uint8_t)(segtest::RST | segtest::ACK), 90000}); // out of window
      }
    }
    if (rng() % 6 == 0) sched.insert(sched.begin() + rng() % sched.size(), Sg{0, 0, segtest::RST, 0}); // may reset
  }

  // what the server sends this tick
  void step() {
    if (st != kEst) return;
    const uint32_t base = srv_isn + 1, L = (uint32_t)stream.size();
    if (pos < sched.size()) {
      for (int k = 0; k < 3 && pos < sched.size(); k++) {
        const Sg& g = sched[pos++];
        const uint32_t seq = base + g.off + (uint32_t)g.shift;
        if (g.flags & segtest::RST) {
          emit(seq + (g.shift ? 0 : srv_una - g.off), cli_nxt, g.flags);
          if (!g.shift) st = kClosed;
        } else {
          emit(seq, cli_nxt, g.flags, stream.data() + g.off, g.len);
        }
      }
      last_tx = tick;
      return;
    }
    if (tick - last_tx < 30) return;
    last_tx = tick;
    if (++fin_tries > 20) {
      st = kClosed;
      return;
    }
    // go-back-N from what the client acknowledged, FIN on the last piece
    uint32_t off = std::min(srv_una, L);
    do {
      const uint32_t n = std::min<uint32_t>(L - off, 1000);
      emit(base + off, cli_nxt, (uint8_t)(segtest::ACK | segtest::PSH | (off + n == L ? segtest::FIN : 0)),
           stream.data() + off, n);
      off += n;
    } while (off < L);
  }

  uint32_t fill(uint8_t* slots, uint32_t stride, uint32_t off, uint32_t cap) {
    ++tick;
    step();
    uint32_t n = 0;
    for (; n < cap && n < q.size(); n++) {
      std::memset(slots + (size_t)n * stride, 0, stride);
      std::memcpy(slots + (size_t)n * stride + off, q[n].data(), q[n].size());
    }
    q.erase(q.begin(), q.begin() + n);
    return n;
  }
  void send(const uint8_t* eth, uint32_t len) { in_flight.emplace_back(eth, eth + len); }
  void endPoll() {
    std::vector<std::vector<uint8_t>> f;
    f.swap(in_flight);
    for (auto& x : f) receive(x.data(), (uint32_t)x.size());
  }
  void receive(const uint8_t* eth, uint32_t len) {
    out.emplace_back(eth, eth + len);
    const uint8_t fl = eth[47];
    const uint32_t seq = pollnet_amd::srv_detail::rd32(eth + 38), ack = pollnet_amd::srv_detail::rd32(eth + 42);
    const uint32_t plen = len - 34 - (eth[46] >> 4) * 4;
    if (fl & segtest::RST) {
      if (st != kListen) st = kListen; // the client aborted: wait for its next SYN
      return;
    }
    if ((fl & segtest::SYN) && !(fl & segtest::ACK)) { // a (re)connect
      if (conns >= 4) return; // enough: silence from here
      const uint32_t what = (uint32_t)(rng() % 10);
      srv_isn = (uint32_t)rng();
      cli_nxt = seq + 1;
      if (what < 5) {
        emit(srv_isn, seq + 1, segtest::SYN | segtest::ACK, nullptr, 0, true);
        st = kSynAcked;
      } else if (what == 5) {
        emit(srv_isn, seq + 7, segtest::SYN | segtest::ACK, nullptr, 0, true); // wrong ack: the client RSTs
      } else if (what == 6) {
        emit(0, seq + 1, segtest::RST | segtest::ACK); // refused
        ++conns;
      } else if (what == 7) {
        emit(0, 0, segtest::RST); // no ACK: the client ignores it
      } else if (what == 8) {
        emit(srv_isn, 0, segtest::SYN, nullptr, 0, true); // simultaneous-open SYN: RST from the client
      } // 9: silence (the client retransmits its SYN)
      return;
    }
    if (st == kSynAcked && (fl & segtest::ACK) && ack == srv_isn + 1) {
      st = kEst;
      ++conns;
      srv_una = 0;
      fin_tries = 0;
      newStream();
    }
    if (st != kEst) return;
    if (fl & segtest::ACK) {
      const uint32_t a = ack - (srv_isn + 1);
      if ((int32_t)(a - srv_una) > 0 && a <= stream.size() + 1) srv_una = a;
    }
    if (plen && seq == cli_nxt) { // the client's data, in order: ACK it
      cli_nxt += plen;
      emit(srv_isn + 1 + std::min<uint32_t>(srv_una, (uint32_t)stream.size()), cli_nxt, segtest::ACK);
    }
  }
};

template <class Conn>
struct CliHandler {
  std::string* log;
  static uint32_t pat;
  void line(const char* what, Conn& c, uint32_t n = 0) {
    char b[160];
    std::snprintf(b, sizeof b, "%s n=%u err=%s connected=%d\n", what, n, c.getLastError() ? c.getLastError() : "-",
                  (int)c.isConnected());
    *log += b;
  }
  void onTcpConnectFailed() { *log += "connect failed\n"; }
  void onTcpConnected(Conn& c) {
    line("connected", c);
    uint8_t msg[300];
    for (auto& b : msg) b = (uint8_t)(pat++ * 131);
    c.writeNonblock(msg, sizeof msg);
  }
  uint32_t onTcpData(Conn& c, const uint8_t* d, uint32_t n) {
    line("data", c, n);
    char b[96];
    std::snprintf(b, sizeof b, "  first %02x last %02x sendable=%u now=%u\n", d[0], d[n - 1], c.getSendable(),
                  c.getImmediatelySendable());
    *log += b;
    const uint32_t k = ++c.deliveries % 3, m = std::min<uint32_t>(n, 700);
    if (k == 0) {
      c.writeNonblock(d, m);
    } else if (k == 1) { // two pieces through sendv (TcpConn.h:63-70)
      iovec iov[2] = {{(void*)d, m / 2}, {(void*)(d + m / 2), m - m / 2}};
      std::snprintf(b, sizeof b, "  sendv %u\n", c.sendv(iov, 2));
      *log += b;
    } else { // writeSome: what fits, and the send timeout re-armed (EfviTcp.h:66-70)
      std::snprintf(b, sizeof b, "  writeSome %d\n", c.writeSome(d, std::min<uint32_t>(n, 300)));
      *log += b;
    }
    return n & 7; // whole 8-byte words consumed
  }
  void onTcpDisconnect(Conn& c) { line("disconnect", c); }
  void onSendTimeout(Conn& c) { line("send timeout", c); }
  void onRecvTimeout(Conn& c) {
    line("recv timeout", c);
    c.close("timeout");
  }
};
template <class Conn>
uint32_t CliHandler<Conn>::pat = 0;

struct Run {
  std::vector<std::vector<uint8_t>> out;
  std::string log;
  uint32_t conns = 0;
};

static const int kPolls = 12000;

static Run runRef(uint64_t seed) {
  using Cli = efvitcp::EfviTcpClient<RefCliConf>;
  auto link = std::make_unique<ScriptServer>(seed);
  efvitcp::RefEnv& env = efvitcp::refEnv();
  env.link = link.get();
  env.fill = [](void* l, uint8_t* s, uint32_t st, uint32_t off, uint32_t cap) {
    return static_cast<ScriptServer*>(l)->fill(s, st, off, cap);
  };
  env.send = [](void* l, const uint8_t* eth, uint32_t len) { static_cast<ScriptServer*>(l)->send(eth, len); };
  env.init_ns = env.now_ns = kT0;
  env.local_ip = htonl(kCliIp);
  std::memcpy(env.local_mac, kCliMac, 6);
  std::memcpy(env.peer_mac, kSrvMac, 6);
  std::unique_ptr<Cli> cli(new Cli());
  Run r;
  CliHandler<Cli::Conn>::pat = 0;
  if (!cli->init("script", "10.0.0.1", kSrvPort, kCliPort)) {
    std::printf("ref init: %s\n", cli->getLastError());
    return r;
  }
  CliHandler<Cli::Conn> h{&r.log};
  for (int t = 1; t <= kPolls; t++) {
    env.now_ns = kT0 + ((int64_t)t << 20);
    cli->poll(h, env.now_ns);
    link->endPoll();
  }
  r.out = link->out;
  r.conns = link->conns;
  static ScriptServer sink(0); // the destructor's RST
  env.link = &sink;
  return r;
}

template <class Backend, class Conf = ProdCliConf>
static Run runProd(uint64_t seed, bool drop_bad = true) {
  using Cli = GpuTcpClient<Conf, ScriptServer, Backend>;
  auto cli = std::make_unique<Cli>();
  Run r;
  CliHandler<typename Cli::Conn>::pat = 0;
  cli->link() = ScriptServer(seed);
  if (!cli->initWithLink("10.0.0.2", "10.0.0.1", kSrvPort, kCliPort, kT0)) {
    std::printf("init: %s\n", cli->getLastError());
    return r;
  }
  cli->setDropBadChecksum(drop_bad); // off: the GPU backend classifies from the header lines only (pn_set_verify)
  CliHandler<typename Cli::Conn> h{&r.log};
  for (int t = 1; t <= kPolls; t++) {
    cli->poll(h, kT0 + ((int64_t)t << 20));
    cli->link().endPoll();
  }
  r.out = cli->link().out;
  r.conns = cli->link().conns;
  return r;
}

static int compare(const char* what, const Run& ref, const Run& p) {
  size_t same = 0;
  while (same < ref.out.size() && same < p.out.size() && ref.out[same] == p.out[same]) same++;
  const bool fr = same == ref.out.size() && same == p.out.size(), lg = ref.log == p.log;
  std::printf("%s: %zu client frames (reference %zu) %s, handler log %s (%zu B)\n", what, p.out.size(), ref.out.size(),
              fr ? "identical" : "DIFFERENT", lg ? "identical" : "DIFFERENT", ref.log.size());
  if (!fr && same < ref.out.size() && same < p.out.size()) {
    const uint8_t *a = ref.out[same].data() + 34, *b = p.out[same].data() + 34;
    std::printf("  first difference at frame %zu: reference seq %u ack %u flags 0x%02x, product seq %u ack %u flags 0x%02x\n",
                same, pollnet_amd::srv_detail::rd32(a + 4), pollnet_amd::srv_detail::rd32(a + 8), a[13],
                pollnet_amd::srv_detail::rd32(b + 4), pollnet_amd::srv_detail::rd32(b + 8), b[13]);
  }
  if (!lg) {
    size_t d = 0;
    while (d < ref.log.size() && d < p.log.size() && ref.log[d] == p.log[d]) d++;
    std::printf("  log differs at byte %zu: reference '%.60s' product '%.60s'\n", d, ref.log.c_str() + d,
                p.log.c_str() + std::min(d, p.log.size()));
  }
  return fr && lg ? 0 : 1;
}

int main(int argc, char** argv) {
  const bool gpu = argc > 1 && std::strcmp(argv[1], "gpu") == 0;
  const uint32_t runs = argc > 2 ? (uint32_t)std::atoi(argv[2]) : 8;
  int fail = 0;
  size_t connected = 0, failed = 0, rsts = 0, data = 0;
  for (uint32_t k = 0; k < runs; k++) {
    const uint64_t seed = 0xC11E47ull + 0x9E3779B97F4A7C15ull * k;
    const Run ref = runRef(seed);
    for (size_t p = 0; (p = ref.log.find("connected n", p)) != std::string::npos; p++) connected++;
    for (size_t p = 0; (p = ref.log.find("connect failed", p)) != std::string::npos; p++) failed++;
    for (auto& f : ref.out) rsts += (f[47] & 4) != 0, data += f.size() > 54;
    char what[96];
    std::snprintf(what, sizeof what, "script %u: twin vs reference", k);
    fail += compare(what, ref, runProd<OracleBackend>(seed));
    if (gpu) {
      std::snprintf(what, sizeof what, "script %u: GpuTcpClient (GPU) vs reference", k);
      fail += compare(what, ref, runProd<GpuBackend>(seed));
      std::snprintf(what, sizeof what, "script %u: GpuTcpClient (GPU, release path) vs reference", k);
      fail += compare(what, ref, runProd<GpuBackend>(seed, false));
      std::snprintf(what, sizeof what, "script %u: GpuTcpClient (GPU, resident service) vs reference", k);
      fail += compare(what, ref, runProd<GpuBackend, ProdCliConfResident>(seed));
      std::snprintf(what, sizeof what, "script %u: GpuTcpClient (GPU, resident, release path) vs reference", k);
      fail += compare(what, ref, runProd<GpuBackend, ProdCliConfResident>(seed, false));
    }
  }
  std::printf("exercised (reference side): %zu connections, %zu connect failures, %zu client RSTs, %zu data frames\n",
              connected, failed, rsts, data);
  if (!connected || !failed || !rsts || !data) fail++, std::printf("FAIL: a path was not exercised\n");
  std::printf("%s\n", fail ? "FAIL" : "PASS");
  return fail ? 1 : 0;
}
