// Throughput of the receive-side server loop (include/pollnet_amd/gpu_tcp_rx.hpp):
// frames from a pinned host ring -> GpuTcpRx::poll -> onTcpData, against the same
// host-side loop fed by the CPU restatement of the reference's release RX path
// (oracle orc_release_batch: parse + key + probe + payload math, no checksum —
// what efvitcp's pollNet does per frame in a release build) on one thread.
//
// Workload: n_flows established connections, each receiving in-order MSS segments
// (tot_len 1500, 1460-B payload, ACK|PSH); the handler reads each delivery's first
// 8 bytes and consumes everything (zero-copy path).  The ring holds `batches`
// batches of `batch` frames; between passes the sequence numbers are advanced in
// place (untimed) so every pass delivers new data.  Prints one JSON line.
#include <arpa/inet.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../include/pollnet_amd/gpu_tcp_rx.hpp"
#include "../oracle/pn_oracle.h"
#include "../tests/cpp/segframes.hpp"

using namespace pollnet_amd;
using Clock = std::chrono::steady_clock;

struct Conf {
  static const uint32_t MaxConnCnt = 1024;
  static const uint32_t MaxTimeWaitConnCnt = 1024;
  static const uint32_t ConnRecvBufSize = 40960;
  static const bool TimestampOption = false;
};

struct H {
  uint64_t bytes = 0, calls = 0, sink = 0;
  template <class C>
  uint32_t onTcpData(C&, const uint8_t* d, uint32_t n) {
    uint64_t w;
    std::memcpy(&w, d, 8);
    sink ^= w;
    bytes += n;
    calls++;
    return 0;
  }
  template <class C>
  void onTcpDisconnect(C&) {}
  template <class C>
  void onAckOwed(C& c, const RxAck& a) {
    if (a.immediate) c.ackSent();
  }
  void onNewSegment(uint64_t, const uint8_t*, const pn_result&) {}
  void onTimeWaitSegment(uint64_t, uint32_t, const uint8_t*, const pn_result&) {}
};

static double secs(Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double>(b - a).count(); }

int main(int argc, char** argv) {
  const uint32_t n_flows = argc > 1 ? std::atoi(argv[1]) : 1024;
  const uint32_t batch = argc > 2 ? std::atoi(argv[2]) : 65536;
  const uint32_t batches = argc > 3 ? std::atoi(argv[3]) : 8;
  const uint32_t passes = argc > 4 ? std::atoi(argv[4]) : 4;
  const uint32_t stride = 2048, off = 2, n = batch * batches;
  if (n % n_flows) {
    std::fprintf(stderr, "batch*batches must be a multiple of n_flows\n");
    return 2;
  }
  uint8_t* ring = nullptr;
  if (hipHostMalloc((void**)&ring, (size_t)stride * n, hipHostMallocDefault) != hipSuccess) return 3;
  std::vector<uint8_t> payload(1460);
  for (uint32_t i = 0; i < 1460; i++) payload[i] = (uint8_t)(i * 31 + 7);
  std::vector<uint32_t> isn(n_flows);
  for (uint32_t f = 0; f < n_flows; f++) isn[f] = 0x10000000u * (f & 15) + f * 7919u;
  auto flow_ip = [](uint32_t f) { return 0x0a010000u | f; };
  auto flow_port = [](uint32_t f) { return (uint16_t)(32768 + (f * 7919) % 28000); };
  const uint32_t per_flow = n / n_flows; // segments per flow per pass
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t f = i % n_flows, k = i / n_flows;
    segtest::Seg s;
    s.src_ip = flow_ip(f);
    s.src_port = flow_port(f);
    s.seq = isn[f] + 1 + k * 1460u;
    s.flags = segtest::ACK | segtest::PSH;
    s.payload = payload.data();
    s.len = 1460;
    segtest::build(ring + (size_t)i * stride + off, s);
  }
  auto advance = [&](uint32_t pass) { // pass p carries stream bytes [p*per_flow*1460, ...)
    for (uint32_t i = 0; i < n; i++) {
      const uint32_t f = i % n_flows, k = i / n_flows;
      segtest::put32(ring + (size_t)i * stride + off + 14 + 20 + 4, isn[f] + 1 + (pass * per_flow + k) * 1460u);
    }
  };
  auto open_all = [&](auto& srv) {
    for (uint32_t f = 0; f < n_flows; f++)
      if (!srv.accept(pn_conn_hash_key(htonl(flow_ip(f)), htons(flow_port(f))), isn[f])) return false;
    return true;
  };

  // ---- GPU path: poll() over the whole ring per pass, chunks of `batch` pipelined ----
  struct GpuRun {
    double mfps = 0, ms_chunk = 0, classify_ms_chunk = 0;
    bool ok = false;
  };
  auto run_gpu = [&](GpuRx::Mode mode, GpuRun& out) -> int {
    auto srv = std::make_unique<GpuTcpRx<Conf>>();
    if (const char* e = srv->init(0, stride, off, batch, mode)) {
      std::fprintf(stderr, "init: %s\n", e);
      return 4;
    }
    if (!open_all(*srv)) return 5;
    H h;
    double t_poll = 0;
    for (uint32_t p = 0; p < passes + 1; p++) { // pass 0 = warm-up
      advance(p);
      const auto t0 = Clock::now();
      if (const char* e = srv->poll(h, ring, n)) {
        std::fprintf(stderr, "poll: %s\n", e);
        return 6;
      }
      if (p) t_poll += secs(t0, Clock::now());
    }
    out.ok = h.bytes == (uint64_t)(passes + 1) * n * 1460;
    // the GPU share alone (transfer + classify, records ignored), same pipeline
    const auto t0 = Clock::now();
    for (uint32_t p = 0; p < passes; p++)
      srv->rx().pollBatch(ring, n, srv->table(), [](uint64_t, const pn_result&, const uint8_t*, uint32_t) {},
                          [](uint64_t, uint32_t, const uint8_t*, const pn_result&) {});
    out.classify_ms_chunk = secs(t0, Clock::now()) * 1e3 / (passes * batches);
    out.mfps = (double)passes * n / t_poll / 1e6;
    out.ms_chunk = t_poll * 1e3 / (passes * batches);
    return 0;
  };
  GpuRun copy_run, zc_run;
  if (int rc = run_gpu(GpuRx::Mode::Copy, copy_run)) return rc;
  if (int rc = run_gpu(GpuRx::Mode::ZeroCopy, zc_run)) return rc;

  // ---- CPU path: release-path records (oracle) + the same host loop, one thread ----
  // sequential twin of poll(): classify the batch on the CPU, then dispatch identically
  struct CpuSrv {
    ConnTable table;
    std::vector<GpuTcpRx<Conf>::Conn> conns = std::vector<GpuTcpRx<Conf>::Conn>(Conf::MaxConnCnt);
    uint32_t next = 0;
    CpuSrv() { table.init(Conf::MaxConnCnt, Conf::MaxTimeWaitConnCnt); }
    GpuTcpRx<Conf>::Conn* accept(uint64_t key, uint32_t syn_seq) {
      const uint32_t id = next++;
      if (table.add(key, id) != PN_OK) return nullptr;
      conns[id].open(syn_seq);
      conns[id].key = key;
      conns[id].id = id;
      return &conns[id];
    }
  };
  auto cpu = std::make_unique<CpuSrv>();
  if (!open_all(*cpu)) return 6;
  std::vector<pn_result> rec(batch);
  H hc;
  double t_cpu = 0, t_cpu_cls = 0;
  const uint32_t cpu_passes = std::max(1u, passes / 2);
  for (uint32_t p = 0; p < cpu_passes + 1; p++) {
    advance(p);
    const auto t0 = Clock::now();
    for (uint32_t b = 0; b < batches; b++) {
      uint32_t ne = 0;
      uint64_t mask = 0;
      const pn_conn_entry* e = cpu->table.entries(&ne, &mask);
      const uint8_t* slots = ring + (size_t)b * batch * stride;
      const auto c0 = Clock::now();
      orc_release_batch(slots, stride, off, batch, e, ne, mask, Conf::MaxConnCnt, rec.data(), 1);
      if (p) t_cpu_cls += secs(c0, Clock::now());
      for (uint32_t i = 0; i < batch; i++) {
        const pn_result& r = rec[i];
        if (!(r.flags & PN_F_HIT) || (r.flags & PN_F_TW)) continue;
        auto& c = cpu->conns[r.conn_id];
        struct A {
          H& h;
          GpuTcpRx<Conf>::Conn& c;
          uint32_t onData(RxConn<Conf>&, const uint8_t* d, uint32_t s) { return h.onTcpData(c, d, s); }
          void onFin(RxConn<Conf>&, const uint8_t*, uint32_t) {}
          void onReset(RxConn<Conf>&) {}
        } a{hc, c};
        const RxAck ack = c.onSegment(a, slots + (size_t)i * stride + off, r);
        if (ack.immediate) c.ackSent();
      }
    }
    if (p) t_cpu += secs(t0, Clock::now());
  }
  const bool ok_cpu = hc.bytes == (uint64_t)(cpu_passes + 1) * n * 1460;

  const double f_cpu = (double)cpu_passes * n / t_cpu;
  auto line = [](const GpuRun& r) {
    char b[256];
    std::snprintf(b, sizeof b,
                  "{\"mframes_per_s\": %.2f, \"gbit_per_s\": %.1f, \"ms_per_chunk\": %.3f, "
                  "\"transfer_classify_ms_per_chunk\": %.3f}",
                  r.mfps, r.mfps * 1514 * 8 / 1e3, r.ms_chunk, r.classify_ms_chunk);
    return std::string(b);
  };
  const bool ok = copy_run.ok && zc_run.ok && ok_cpu;
  std::printf("{\"bench\": \"tcp_rx_poll\", \"workload\": \"%u flows, in-order 1514-B frames (1460-B payload), "
              "pinned host ring of %u slots, poll() over the ring in chunks of %u\", \"frames\": %llu, "
              "\"gpu_poll_copy\": %s, \"gpu_poll_zero_copy\": %s, "
              "\"cpu_release_path_1thread\": {\"mframes_per_s\": %.2f, \"gbit_per_s\": %.1f, \"classify_share\": %.3f}, "
              "\"delivered_ok\": %s}\n",
              n_flows, n, batch, (unsigned long long)passes * n, line(copy_run).c_str(), line(zc_run).c_str(),
              f_cpu / 1e6, f_cpu * 1514 * 8 / 1e9, t_cpu_cls / t_cpu, ok ? "true" : "false");
  return ok ? 0 : 1;
}
