// GpuTcpServer (include/pollnet_amd/tcp_server.hpp) as a drop-in for pollnet's
// EfviTcpServer: the handler of the reference's own example server
// (/root/reference/example/tcpserver.cc:61-90, extracted verbatim into
// oracle/_ref/tcpserver_handler.inc by oracle/ref.mk) is compiled unchanged against it
// and polls a mixed ring of 200 TCP flows (SYN with MSS option, handshake, reordered /
// duplicated / corrupted-then-resent data, FIN, segments after close) and 16 unknown
// flows.  Its `cout` lines go into a log, `exit` would be recorded.
//
// Two instances run the identical traffic:
//   gpu : GpuBackend — one pn_classify launch per poll over the pinned RX ring, records
//         walked against the table snapshot with host re-resolution after changes, one
//         pn_tx_fill launch per poll for the TX checksums;
//   twin: a sequential backend with the reference's semantics — each frame classified by
//         the C oracle against the live table at the moment the reference's loop would
//         reach it, TX checksums by the oracle (test infrastructure, never the product).
// Checks: identical handler logs and identical TX frames (byte for byte); every TX frame
// verifies (IP and TCP checksums); every accepted flow's echo, reassembled from the
// server's data segments, equals the stream the flow sent; every unknown-flow segment is
// answered by an RST; no connection is left open.
//   argv: twin | gpu <frames per poll>          exit 0 = pass
#include <arpa/inet.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <iostream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/pollnet_amd/tcp_server.hpp"
#include "segframes.hpp"
#include "server_harness.hpp"

using namespace std;
using namespace pollnet_amd;

struct ServerConf { // tcpserver.cc:4-14 with room for 200 concurrent flows
  static const uint32_t RecvBufSize = 40960;
  static const uint32_t MaxConns = 256;
  static const uint32_t SendTimeoutSec = 0;
  static const uint32_t RecvTimeoutSec = 10;
  static const uint32_t ConnSendBufCnt = 64;
  static const uint32_t RxBatch = 8192;
  static const uint32_t TxBatch = 256;
  struct UserData {
    struct sockaddr_in addr;
  };
};

static const int64_t kNowNs = (int64_t)123456 << 20; // fixed clock: no timer fires in this scenario

namespace on_gpu {
using TcpServer = GpuTcpServer<ServerConf, ScriptLink, GpuBackend>;
TcpServer& server = *new TcpServer;
LogStream cout;
int exits = 0;
void exit(int) { ++exits; }
void pollOnce() {
#include "../../oracle/_ref/tcpserver_handler.inc"
  server.poll(handler, kNowNs);
}
} // namespace on_gpu

namespace on_twin {
using TcpServer = GpuTcpServer<ServerConf, ScriptLink, OracleBackend>;
TcpServer& server = *new TcpServer;
LogStream cout;
int exits = 0;
void exit(int) { ++exits; }
void pollOnce() {
#include "../../oracle/_ref/tcpserver_handler.inc"
  server.poll(handler, kNowNs);
}
} // namespace on_twin

struct Flow {
  uint32_t ip;
  uint16_t port;
  uint32_t isn;
  std::vector<uint8_t> stream;
};

static std::vector<std::vector<uint8_t>> make_traffic(std::vector<Flow>& flows, uint32_t n_data, uint32_t n_unknown) {
  using namespace segtest;
  std::mt19937_64 rng(0x5E12BE12ull);
  auto U = [&](uint32_t lo, uint32_t hi) { return lo + (uint32_t)(rng() % (hi - lo + 1)); };
  flows.resize(n_data + n_unknown);
  std::vector<std::vector<Seg>> per(flows.size());
  for (uint32_t f = 0; f < flows.size(); f++) {
    Flow& F = flows[f];
    F.ip = 0x0a010000 | (f + 1);
    F.port = (uint16_t)(32768 + (f * 7919) % 28000);
    F.isn = (uint32_t)rng();
    // the server's ISN: connHashKey(peer) + now_ts (TcpConn::genISN, TcpConn.h:856-858)
    const uint32_t srv_isn = (uint32_t)pn_conn_hash_key(htonl(F.ip), htons(F.port)) + (uint32_t)(kNowNs >> 20);
    auto mk = [&](uint32_t a, uint32_t b, uint8_t fl) {
      Seg s;
      s.src_ip = F.ip;
      s.src_port = F.port;
      s.seq = F.isn + 1 + a;
      s.ack = srv_isn + 1;
      s.flags = fl;
      s.payload = F.stream.data() + a;
      s.len = b - a;
      return s;
    };
    if (f < n_data) {
      F.stream.resize(U(0, 30000));
      for (auto& b : F.stream) b = (uint8_t)rng();
      Seg syn;
      syn.src_ip = F.ip;
      syn.src_port = F.port;
      syn.seq = F.isn;
      syn.flags = SYN;
      syn.opts = {2, 4, 0x05, 0xb4}; // MSS 1460
      per[f].push_back(syn);
      std::vector<std::pair<uint32_t, uint32_t>> pk;
      for (uint32_t o = 0; o < F.stream.size();) {
        const uint32_t n = std::min<uint32_t>((uint32_t)F.stream.size() - o, U(1, 1460));
        pk.push_back({o, o + n});
        o += n;
      }
      if (pk.empty() || rng() % 4 == 0) per[f].push_back(mk(0, 0, ACK)); // a bare handshake ACK
      const uint32_t W = U(1, 3);
      for (size_t b = 0; b < pk.size(); b += W) {
        std::vector<std::pair<uint32_t, uint32_t>> blk(pk.begin() + b, pk.begin() + std::min(pk.size(), b + W));
        std::shuffle(blk.begin(), blk.end(), rng);
        for (auto& x : blk) {
          Seg s = mk(x.first, x.second, ACK | PSH);
          if (rng() % 16 == 0) { // corrupted copy first (dropped), the clean resend right after
            Seg bad = s;
            bad.corrupt = true;
            per[f].push_back(bad);
          }
          per[f].push_back(s);
          if (rng() % 20 == 0) per[f].push_back(s); // duplicate
        }
      }
      per[f].push_back(mk((uint32_t)F.stream.size(), (uint32_t)F.stream.size(), ACK | FIN));
      per[f].push_back(mk((uint32_t)F.stream.size() + 1, (uint32_t)F.stream.size() + 1, ACK)); // after close
    } else { // unknown flows: ACK-only and one bare data segment -> RST each
      for (int k = 0; k < 3; k++) {
        Seg s;
        s.src_ip = F.ip;
        s.src_port = F.port;
        s.seq = F.isn + k;
        s.ack = 777 + k;
        s.flags = (k == 2) ? PSH : ACK;
        per[f].push_back(s);
      }
    }
  }
  std::vector<std::vector<uint8_t>> frames;
  std::vector<uint32_t> pos(flows.size(), 0), live;
  for (uint32_t f = 0; f < flows.size(); f++) live.push_back(f);
  uint8_t buf[2048];
  while (!live.empty()) {
    const uint32_t k = (uint32_t)(rng() % live.size()), f = live[k];
    const uint32_t len = build(buf, per[f][pos[f]++]);
    frames.emplace_back(buf, buf + len);
    if (pos[f] == per[f].size()) {
      live[k] = live.back();
      live.pop_back();
    }
  }
  return frames;
}

// Checks on one run's TX frames; returns the number of failures.
static int check_tx(const char* tag, const std::vector<std::vector<uint8_t>>& out, const std::vector<Flow>& flows,
                    uint32_t n_data, uint32_t n_unknown_segs) {
  using segtest::classify;
  int fail = 0;
  std::map<uint16_t, const Flow*> by_port;
  for (auto& F : flows) by_port[htons(F.port)] = &F;
  std::map<uint16_t, std::map<uint32_t, std::vector<uint8_t>>> data; // port -> seq -> payload
  std::map<uint16_t, uint32_t> isn;
  uint32_t bad_sum = 0, syn_acks = 0, rsts = 0, rst_unknown = 0;
  for (auto& f0 : out) {
    std::vector<uint8_t> f(f0);
    f.resize(f0.size() + 2, 0); // the oracle reads an odd segment's pad byte (Core.h:113-117)
    const pn_result r = classify(f.data(), (uint32_t)f.size());
    if ((r.flags & (PN_F_IP_OK | PN_F_TCP_OK)) != (PN_F_IP_OK | PN_F_TCP_OK)) bad_sum++;
    uint16_t dport;
    std::memcpy(&dport, f.data() + 36, 2);
    const uint8_t fl = f[47];
    const uint32_t seq = r.seq - ((fl & 2) ? 1 : 0);
    if ((fl & 0x12) == 0x12) {
      syn_acks++;
      isn[dport] = seq;
    }
    if (fl & 4) {
      rsts++;
      auto it = by_port.find(dport);
      if (it != by_port.end() && (uint32_t)(it->second - flows.data()) >= n_data) rst_unknown++;
    }
    if (r.payload_len > 0) data[dport][seq].assign(f.begin() + r.payload_off, f.begin() + r.payload_off + r.payload_len);
  }
  uint32_t echo_ok = 0;
  for (uint32_t i = 0; i < n_data; i++) {
    const uint16_t p = htons(flows[i].port);
    std::vector<uint8_t> got;
    if (isn.count(p)) {
      for (auto& kv : data[p]) {
        const uint32_t off = kv.first - (isn[p] + 1);
        if (off > got.size()) break; // hole
        if (off + kv.second.size() > got.size()) got.resize(off + kv.second.size());
        std::copy(kv.second.begin(), kv.second.end(), got.begin() + off);
      }
    }
    echo_ok += got == flows[i].stream;
  }
  std::printf("%s: %zu TX frames (%u SYN-ACK, %u RST, %u RST to unknown flows), %u/%u echoes intact, %u bad checksums\n",
              tag, out.size(), syn_acks, rsts, rst_unknown, echo_ok, n_data, bad_sum);
  if (bad_sum) fail++, std::printf("FAIL %s: TX frames with bad checksums\n", tag);
  if (syn_acks != n_data) fail++, std::printf("FAIL %s: expected %u SYN-ACKs\n", tag, n_data);
  if (echo_ok != n_data) fail++, std::printf("FAIL %s: echoes differ from the streams\n", tag);
  if (rst_unknown != n_unknown_segs) fail++, std::printf("FAIL %s: expected %u RSTs to unknown flows\n", tag, n_unknown_segs);
  return fail;
}

template <class S>
static bool run(S& server, void (*poll_once)(), const std::vector<std::vector<uint8_t>>& frames, uint32_t per_poll) {
  server.setDropBadChecksum(true);
  if (!server.initWithLink("10.0.0.1", 1234, kNowNs)) {
    std::printf("init: %s\n", server.getLastError());
    return false;
  }
  server.link().in = frames;
  server.link().per_poll = per_poll;
  while (server.link().pos < frames.size()) {
    poll_once();
    if (server.getLastError()) {
      std::printf("poll: %s\n", server.getLastError());
      return false;
    }
  }
  return true;
}

int main(int argc, char** argv) {
  const bool gpu = argc > 1 && std::strcmp(argv[1], "gpu") == 0;
  const uint32_t per_poll = argc > 2 ? (uint32_t)std::atoi(argv[2]) : 512;
  const uint32_t n_data = 200, n_unknown = 16;
  std::vector<Flow> flows;
  const auto frames = make_traffic(flows, n_data, n_unknown);
  int fail = 0;

  if (!run(on_twin::server, on_twin::pollOnce, frames, per_poll)) return 3;
  const std::string tlog = on_twin::cout.os.str();
  const auto tout = on_twin::server.link().out;
  size_t lines = std::count(tlog.begin(), tlog.end(), '\n');
  std::printf("twin: %zu frames polled %u per poll, %zu handler lines, conns left %u\n", frames.size(), per_poll, lines,
              on_twin::server.getConnCnt());
  fail += check_tx("twin", tout, flows, n_data, 3 * n_unknown);
  if (lines != 2 * n_data || on_twin::server.getConnCnt() != 0 || on_twin::exits) {
    std::printf("FAIL twin: expected %u handler lines, no open connection, no exit()\n", 2 * n_data);
    fail++;
  }

  if (gpu) {
    if (!run(on_gpu::server, on_gpu::pollOnce, frames, per_poll)) return 5;
    const std::string glog = on_gpu::cout.os.str();
    const auto& gout = on_gpu::server.link().out;
    fail += check_tx("gpu", gout, flows, n_data, 3 * n_unknown);
    if (glog != tlog) {
      size_t d = 0;
      while (d < glog.size() && d < tlog.size() && glog[d] == tlog[d]) d++;
      std::printf("FAIL: handler logs differ at byte %zu:\n  gpu:  %.120s\n  twin: %.120s\n", d, glog.c_str() + d,
                  tlog.c_str() + d);
      fail++;
    }
    size_t same = 0;
    while (same < gout.size() && same < tout.size() && gout[same] == tout[same]) same++;
    if (gout.size() != tout.size() || same != gout.size()) {
      std::printf("FAIL: TX frames differ: gpu %zu, twin %zu, first difference at %zu\n", gout.size(), tout.size(), same);
      fail++;
    }
    std::printf("gpu: handler log %s, TX frames %s (%zu)\n", glog == tlog ? "identical" : "DIFFERENT",
                same == gout.size() && gout.size() == tout.size() ? "identical" : "DIFFERENT", gout.size());
    delete &on_gpu::server; // GPU resources go before the runtime tears down
  }
  delete &on_twin::server;
  std::printf("%s\n", fail ? "FAIL" : "PASS");
  return fail ? 1 : 0;
}
