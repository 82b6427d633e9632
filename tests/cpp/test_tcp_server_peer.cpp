// GpuTcpServer against live TCP peers: a deterministic in-memory client population that
// reacts to every frame the server sends, with loss in both directions and a clock that
// advances one millisecond per poll.  This drives the parts of the server a replayed
// ring cannot: SYN-ACK retransmission, RTO retransmission and its back-off, duplicate-ACK
// fast retransmit, delayed ACKs, window-limited sending (segments queued until the peer's
// ACK opens the window, TcpConn.h:646-660), the receive timeout (onRecvTimeout ->
// close("timeout") -> RST), admission refusal (allowNewConnection / MaxConns -> RST),
// the server's own FIN (Conn::sendFin), RSTs from the peer and the pollnet wrapper's
// close on a remote FIN (EfviTcp.h:283-288).
//
// The same population runs twice — GpuBackend (pn_classify + pn_tx_fill on the GPU) and
// the sequential oracle backend — and, the peers being deterministic functions of what
// they receive, the two runs must match frame for frame and callback for callback.
// Independently: every flow that completes echoes its stream exactly, every TX frame
// verifies, idle flows are timed out, and nothing is left open.
//   argv: twin | gpu            exit 0 = pass
#include <arpa/inet.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <random>
#include <string>
#include <tuple>
#include <vector>

#include "segframes.hpp"
#include "server_harness.hpp"
#include "peer_population.hpp"

using namespace pollnet_amd;

struct PeerConf {
  static const bool RxPipeline = false;
  static const uint32_t RecvBufSize = 8192;
  static const uint32_t MaxConns = 48;
  static const uint32_t SendTimeoutSec = 0;
  static const uint32_t RecvTimeoutSec = 1;
  static const uint32_t ConnSendBufCnt = 64;
  static const uint32_t RxBatch = 1024;
  static const uint32_t TxBatch = 128;
  static const uint32_t DelayedAckMS = 10;
  static const bool UseAllowNewConnection = true; // efvitcp::TcpServer's admission event (TcpServer.h:84)
  struct UserData {
    uint32_t echoed = 0;
    bool fin_asked = false;
  };
};

// the same with received frames held up to 3 ms for a fuller GPU batch
struct PeerConfBudget : PeerConf {
  static const uint32_t RxLatencyBudgetUs = 3000;
};
// a poll's frames classified in launches of 16 (the next on the GPU while one is dispatched)
struct PeerConfChunk : PeerConf {
  static const uint32_t RxChunk = 16;
};
// throughput mode: each poll's frames dispatched in the next poll, classified meanwhile
// against the table as it was at their launch (re-resolved where it has changed since)
struct PeerConfPipe : PeerConf {
  static const bool RxPipeline = true;
};
// the classify in the resident service (pn_service_*: a post per poll, no launch), every poll and pipelined
// (two posts outstanding)
struct PeerConfResident : PeerConf {
  static const bool RxResident = true;
};
struct PeerConfPipeResident : PeerConfPipe {
  static const bool RxResident = true;
};
// pipelined two polls deep (Conf::RxPipelineDepth 2: three RX rings, two batches in flight)
struct PeerConfPipe2 : PeerConfPipe {
  static const uint32_t RxPipelineDepth = 2;
};
struct PeerConfPipe2Resident : PeerConfPipe2 {
  static const bool RxResident = true;
};

template <class Backend, class Conf = PeerConf>
struct Run {
  using Server = GpuTcpServer<Conf, PeerLink, Backend>;
  std::unique_ptr<Server> srv = std::make_unique<Server>();
  std::string log;
  uint32_t polls = 0;

  bool go(const std::vector<Client>& population) {
    if (!srv->initWithLink("10.0.0.1", 1234, kT0)) {
      std::printf("init: %s\n", srv->getLastError());
      return false;
    }
    srv->link().clients = population;
    PeerHandler<typename Server::Conn> h{&log};
    for (polls = 1; polls < 30000; polls++) {
      srv->poll(h, kT0 + ((int64_t)polls << 20));
      if (srv->getLastError()) {
        std::printf("poll: %s\n", srv->getLastError());
        return false;
      }
      bool done = true;
      for (auto& c : srv->link().clients) done &= c.st == Client::kDone;
      if (done && srv->getConnCnt() == 0) break;
    }
    return true;
  }
};

template <class R>
static int check(const char* tag, R& r) {
  int fail = 0;
  uint32_t bad = 0;
  for (auto& f0 : r.srv->link().out) {
    std::vector<uint8_t> f(f0);
    f.resize(f0.size() + 2, 0);
    const pn_result x = segtest::classify(f.data(), (uint32_t)f.size());
    if ((x.flags & (PN_F_IP_OK | PN_F_TCP_OK)) != (PN_F_IP_OK | PN_F_TCP_OK)) bad++;
  }
  uint32_t est = 0, echo_ok = 0, echo_due = 0, refused = 0, timed_out = 0, idle = 0, not_done = 0;
  for (auto& c : r.srv->link().clients) {
    est += c.established;
    refused += c.refused;
    not_done += c.st != Client::kDone;
    if (c.kind == kIdle && c.established) {
      idle++;
      timed_out += c.got_rst;
    }
    if (c.established && (c.kind == kFinEnd || c.kind == kRstEnd) && c.port % 5 != 0) {
      echo_due++;
      echo_ok += c.echo == c.stream;
      if (c.echo != c.stream) {
        size_t d = 0;
        while (d < c.echo.size() && d < c.stream.size() && c.echo[d] == c.stream[d]) d++;
        std::printf("  echo port %u kind %d: %zu of %zu bytes, first difference %zu, rst %d fin %d win %u\n", c.port,
                    (int)c.kind, c.echo.size(), c.stream.size(), d, c.got_rst, c.got_fin, c.window);
      }
    }
  }
  const size_t timeouts = [&] {
    size_t n = 0, p = 0;
    while ((p = r.log.find("recv timeout", p)) != std::string::npos) n++, p++;
    return n;
  }();
  auto& L = r.srv->link();
  // exercised paths: retransmitted segments (same port/seq/flags seen before), SYN-ACKs, server FINs
  std::map<std::tuple<uint16_t, uint32_t, uint8_t>, int> seen;
  uint32_t retx = 0, synacks = 0, fins = 0, pure_acks = 0;
  for (auto& f : L.out) {
    uint16_t dport;
    std::memcpy(&dport, f.data() + 36, 2);
    const uint8_t fl = f[47];
    if ((fl & 0x12) == 0x12) synacks++;
    if (fl & 1) fins++;
    if (f.size() == 54 && fl == 0x18) pure_acks++;
    if (f.size() > 54 || (fl & 0x03)) retx += seen[{dport, srv_detail::rd32(f.data() + 38), fl}]++ > 0;
  }
  std::printf("%s: %u retransmitted segments, %u SYN-ACKs, %u FINs, %u pure ACKs; log: %zu sendFin\n", tag, retx,
              synacks, fins, pure_acks, [&] {
                size_t n = 0, p = 0;
                while ((p = r.log.find("sendFin", p)) != std::string::npos) n++, p++;
                return n;
              }());
  if (retx == 0 || fins == 0) fail++, std::printf("FAIL %s: retransmission / FIN paths not exercised\n", tag);
  std::printf("%s: %u polls, %zu TX frames (%u bad checksums), drops c2s %u s2c %u; %u established, %u refused, "
              "%u/%u echoes intact, %u/%u idle flows timed out (%zu recv timeouts), %u not done, conns left %u\n",
              tag, r.polls, L.out.size(), bad, L.drops_c2s, L.drops_s2c, est, refused, echo_ok, echo_due, timed_out,
              idle, timeouts, not_done, r.srv->getConnCnt());
  if (bad) fail++, std::printf("FAIL %s: TX frames with bad checksums\n", tag);
  if (echo_ok != echo_due || echo_due < 30) fail++, std::printf("FAIL %s: echoes\n", tag);
  if (timed_out != idle || idle == 0 || timeouts < idle) fail++, std::printf("FAIL %s: idle flows\n", tag);
  if (not_done || r.srv->getConnCnt()) {
    fail++;
    std::printf("FAIL %s: flows left\n", tag);
    for (auto& c : r.srv->link().clients)
      if (c.st != Client::kDone)
        std::printf("  port %u kind %d st %d una %u nxt %u len %zu echo %zu got_fin %d fin_sent %d wnd %u\n", c.port,
                    (int)c.kind, (int)c.st, c.snd_una, c.snd_nxt, c.stream.size(), c.echo.size(), c.got_fin,
                    c.fin_sent, c.srv_wnd);
  }
  if (refused == 0) fail++, std::printf("FAIL %s: no admission refusal exercised\n", tag);
  return fail;
}

// the same Conf with every TX batch through the backend's fill (pn_tx_fill on the GPU, the
// oracle's fill in the twin) instead of the host for batches with few payload frames
template <class Conf>
struct AllTxOnBackend : Conf {
  static const uint32_t TxGpuMinDataFrames = 0;
};
// ... and a mixed policy: batches with 2+ payload frames through the backend, the rest on the host
template <class Conf>
struct MixedTx : Conf {
  static const uint32_t TxGpuMinDataFrames = 2;
};

template <class A, class B>
static int same_frames(const char* what, A& a, B& b) {
  const auto &x = a.srv->link().out, &y = b.srv->link().out;
  const bool eq = x == y && a.log == b.log;
  std::printf("%s: TX frames %s (%zu vs %zu), logs %s\n", what, eq ? "identical" : "DIFFERENT", x.size(), y.size(),
              a.log == b.log ? "identical" : "DIFFERENT");
  return eq ? 0 : 1;
}

template <class Conf>
static int scenario(bool gpu, const std::vector<Client>& pop, const char* name) {
  int fail = 0;
  Run<OracleBackend, Conf> twin;
  if (!twin.go(pop)) return 100;
  {
    // TX policies: host sums for small batches (default), the oracle's fill for every batch, mixed
    Run<OracleBackend, AllTxOnBackend<Conf>> twin_b;
    Run<OracleBackend, MixedTx<Conf>> twin_m;
    if (!twin_b.go(pop) || !twin_m.go(pop)) return 100;
    std::printf("[%s] TX policies: default %llu frames summed on the host; mixed %llu host + %llu backend fill\n",
                name, (unsigned long long)twin.srv->txHostFrames(), (unsigned long long)twin_m.srv->txHostFrames(),
                (unsigned long long)twin_m.srv->txGpuFrames());
    if (!twin_m.srv->txHostFrames() || !twin_m.srv->txGpuFrames() || twin_b.srv->txHostFrames())
      fail++, std::printf("FAIL: both TX policies not exercised\n");
    fail += same_frames("twin host-fill vs twin backend-fill", twin, twin_b);
    fail += same_frames("twin mixed vs twin backend-fill", twin_m, twin_b);
  }
  std::printf("[%s] twin: %llu records re-resolved against the live table\n", name,
              (unsigned long long)twin.srv->reResolved());
  fail += check("twin", twin);
  // pipelined, connections are accepted between a batch's launch and its dispatch
  if (Conf::RxPipeline && !twin.srv->reResolved()) fail++, std::printf("FAIL: no re-resolved record\n");
  if (gpu) {
    Run<GpuBackend, Conf> g;
    if (!g.go(pop)) return 100;
    fail += check("gpu", g);
    const auto &a = g.srv->link().out, &b = twin.srv->link().out;
    size_t same = 0;
    while (same < a.size() && same < b.size() && a[same] == b[same]) same++;
    const bool frames_eq = a.size() == b.size() && same == a.size();
    if (!frames_eq) std::printf("FAIL: TX frames differ: gpu %zu, twin %zu, first difference at %zu\n", a.size(), b.size(), same);
    if (g.log != twin.log) std::printf("FAIL: handler logs differ\n");
    fail += !frames_eq + (g.log != twin.log);
    std::printf("gpu: handler log %s, TX frames %s (%zu)\n", g.log == twin.log ? "identical" : "DIFFERENT",
                frames_eq ? "identical" : "DIFFERENT", a.size());
    Run<GpuBackend, MixedTx<Conf>> g_mixed; // batches with payload through pn_tx_fill, the rest on the host
    if (!g_mixed.go(pop)) return 100;
    if (!g_mixed.srv->txGpuFrames() || !g_mixed.srv->txHostFrames())
      fail++, std::printf("FAIL: gpu mixed TX policy not exercised\n");
    fail += same_frames("gpu mixed TX policy vs twin", g_mixed, twin);
  }
  return fail;
}

// pollnet's EfviTcpServer wrapper never consults the handler's allowNewConnection (its TmpHandler
// returns true, EfviTcp.h:270): without Conf::UseAllowNewConnection the same handler, which would
// refuse every port divisible by 7, gets no refusal at all (room for every client).
struct PeerConfWrapper : PeerConf {
  static const bool UseAllowNewConnection = false;
  static const uint32_t MaxConns = 128;
};
static int wrapper_admission(bool gpu, const std::vector<Client>& pop) {
  auto one = [&](auto& r, const char* tag) {
    if (!r.go(pop)) return 100;
    uint32_t refused = 0, est = 0, by7 = 0;
    for (auto& c : r.srv->link().clients) {
      refused += c.refused;
      est += c.established;
      by7 += c.established && c.port % 7 == 0;
    }
    std::printf("%s (allowNewConnection not consulted): %u established (%u on ports divisible by 7), %u refused\n", tag,
                est, by7, refused);
    return (refused != 0 || by7 == 0) ? (std::printf("FAIL %s: wrapper admission\n", tag), 1) : 0;
  };
  Run<OracleBackend, PeerConfWrapper> twin;
  int fail = one(twin, "twin");
  if (gpu) {
    Run<GpuBackend, PeerConfWrapper> g;
    fail += one(g, "gpu");
  }
  return fail;
}

int main(int argc, char** argv) {
  const bool gpu = argc > 1 && std::strcmp(argv[1], "gpu") == 0;
  const uint32_t runs = argc > 2 ? (uint32_t)std::atoi(argv[2]) : 1; // soak: more populations and loss patterns
  int fail = 0;
  for (g_seed = 0; g_seed < runs; g_seed++) {
    if (runs > 1) std::printf("== population %u ==\n", g_seed);
    const auto pop = population();
    fail += scenario<PeerConf>(gpu, pop, "classify every poll");
    fail += scenario<PeerConfBudget>(gpu, pop, "3-ms RX latency budget");
    fail += scenario<PeerConfChunk>(gpu, pop, "RX chunks of 16");
    fail += scenario<PeerConfPipe>(gpu, pop, "pipelined RX (dispatch one poll later)");
    fail += scenario<PeerConfResident>(gpu, pop, "resident service, every poll");
    fail += scenario<PeerConfPipeResident>(gpu, pop, "resident service, pipelined RX");
    fail += scenario<PeerConfPipe2>(gpu, pop, "pipelined RX two polls deep");
    fail += scenario<PeerConfPipe2Resident>(gpu, pop, "resident service, pipelined RX two polls deep");
    if (g_seed == 0) fail += wrapper_admission(gpu, pop);
  }
  std::printf("%s\n", fail ? "FAIL" : "PASS");
  return fail ? 1 : 0;
}
