// Throughput of the drop-in server itself (include/pollnet_amd/tcp_server.hpp): frames in
// the RX ring -> GpuTcpServer::poll(handler) -> onTcpData, with the server's own ACKs built,
// checksummed (pn_tx_fill) and handed to the link — the whole EfviTcpServer::poll path
// (EfviTcp.h:258-307 -> TcpServer::poll, TcpServer.h:70-112 -> TcpConn::onPack), against the
// same server on the sequential backend (every frame classified by the CPU restatement of
// Core::pollNet's per-frame work, checksums included, TX checksums on the CPU; one thread).
//
// Workload: n_flows peers connect (SYN, SYN-ACK, ACK through the server's own handshake),
// then each poll hands the server RxBatch in-order MSS segments (1514-B frames, 1460-B
// payload, ACK|PSH), RxBatch / n_flows per flow; the handler reads each delivery's first 8
// bytes and consumes it.  The server ACKs every second segment (TcpConn.h:745-755).  The link
// plays the NIC: the ring slots keep their frames between polls and only the sequence number
// and TCP checksum are rewritten (6 bytes per frame; timed separately as `link_fill_share`).
//   argv: n_flows (256)  polls (400)  [cpu|quick|release_pair|resident_pair|resident_pair_l3|resident_pair_cold|twin_timed|echo]
//         prints one JSON line; exit 0 = all data delivered
//         (cpu: the sequential-backend legs only, no GPU needed; quick: GPU RxBatch 512 (also pipelined),
//         GPU pipelined 16384 and CPU 512, each verified and on the release path (discard off, no
//         checksum summed) — bench.py's secondary.tcp_server_poll; resident_pair*: the best GPU leg beside the
//         reference with the frames where a NIC's DMA leaves them: hot (written by the server's own core),
//         _l3 (written by another core of the same CCD, as DDIO / cache injection leaves them in the L3 or a
//         neighbour's L2), _cold (flushed to DRAM))
#include <arpa/inet.h>
#include <emmintrin.h>

#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <type_traits>
#include <vector>

#include "../include/pollnet_amd/tcp_server.hpp"
#include "../tests/cpp/segframes.hpp"
#include "../tests/cpp/server_harness.hpp"
#include "sampler.hpp"
// The reference's own server (pollnet's EfviTcpServer over efvitcp's TcpServer / TcpConn, compiled from the text
// oracle/ref.mk extracts from /root/reference; only the ef_vi plumbing is restated, oracle/ref_server.hpp) as the
// CPU baseline of the release-path legs, where that text was present at build time.
#if __has_include("../oracle/_ref/conn_efvitcpserver.inc")
#define PN_BENCH_REF 1
#include "../oracle/ref_server.hpp"
#endif

using namespace pollnet_amd;
using Clock = std::chrono::steady_clock;
static double secs(Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double>(b - a).count(); }

static const uint8_t kServerMac[6] = {2, 0, 0, 0, 0, 1};
static const uint32_t kPayload = 1460;

// The peers and the NIC: n_flows clients, frames written into the server's RX ring.
static bool g_cold = false; // resident_pair_cold: every leg's link leaves its frames out of the caches

// resident_pair_l3: the link's writes run on another core (the next allowed CPU after the server's, normally a core
// of the same CCD), so the lines the server then reads come from the shared L3 / that core's L2, as a NIC with
// DDIO or cache injection leaves them -- between a hot ring (the server's own writes) and a cold one (DRAM).
struct RemoteWriter {
  std::thread th;
  std::atomic<uint64_t> req{0}, done{0};
  std::atomic<bool> stop{false};
  void (*fn)(void*) = nullptr;
  void* arg = nullptr;
  int cpu_server = -1, cpu_writer = -1;
  bool start() {
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) != 0) return false;
    for (int c = 0; c < CPU_SETSIZE; c++)
      if (CPU_ISSET(c, &set)) {
        if (cpu_server < 0) cpu_server = c;
        else if (cpu_writer < 0) cpu_writer = c;
      }
    if (cpu_writer < 0) return false;
    cpu_set_t one;
    CPU_ZERO(&one);
    CPU_SET(cpu_server, &one);
    if (pthread_setaffinity_np(pthread_self(), sizeof one, &one) != 0) return false;
    th = std::thread([this] {
      cpu_set_t w;
      CPU_ZERO(&w);
      CPU_SET(cpu_writer, &w);
      pthread_setaffinity_np(pthread_self(), sizeof w, &w);
      uint64_t seen = 0;
      while (!stop.load(std::memory_order_acquire)) {
        const uint64_t r = req.load(std::memory_order_acquire);
        if (r == seen) {
          _mm_pause();
          continue;
        }
        fn(arg);
        seen = r;
        done.store(r, std::memory_order_release);
      }
    });
    return true;
  }
  void run(void (*f)(void*), void* a) { // f(a) on the writer's core; returns when it is done
    fn = f;
    arg = a;
    const uint64_t r = req.load(std::memory_order_relaxed) + 1;
    req.store(r, std::memory_order_release);
    while (done.load(std::memory_order_acquire) != r) _mm_pause();
  }
  ~RemoteWriter() {
    stop.store(true, std::memory_order_release);
    if (th.joinable()) th.join();
  }
};
static RemoteWriter* g_writer = nullptr;

struct BenchLink {
  enum Phase { Syn, Ack, Data, Idle } phase = Idle;
  uint32_t n_flows = 0;
  std::vector<uint32_t> cli_isn, srv_isn, sum_base; // sum_base: TCP sum of the data frame with seq = 0
  std::vector<uint8_t> payload = std::vector<uint8_t>(kPayload);
  uint64_t poll_no = 0;           // data polls so far
  uint8_t* written[3] = {nullptr, nullptr, nullptr}; // rings (pipelined: 2 or 3) whose slots hold full data frames
  uint32_t written_n = 0;
  uint64_t acks = 0, rsts = 0, synacks = 0, other = 0;
  // echo workload: the peers acknowledge every byte the server sent them (their next frames carry it)
  bool echo = false;
  bool cold = false; // frames flushed from the CPU caches after each fill (resident_pair_cold)
  std::vector<uint32_t> flow_of_port; // port -> flow + 1
  std::vector<uint64_t> srv_data;     // payload bytes the server sent each flow
  uint64_t echo_bytes = 0, echo_frames = 0;
  uint8_t other_flags = 0;
  double fill_s = 0;
  // a poll smaller than the flow count (the reference's 64 events per pollNet): handshakes continue over polls
  // from hs_next, data frames rotate over the flows (each slot gets its flow's 54-B header from hdr, payload
  // written once per slot), seg_k counts each flow's segments
  uint32_t hs_next = 0, cursor = 0;
  std::vector<uint8_t> hdr;
  std::vector<uint64_t> seg_k;
  const uint8_t* paid_base = nullptr; // the slots [0, paid_n) of that ring already hold the payload
  uint32_t paid_n = 0;
  uint64_t data_frames = 0;

  static uint32_t ip(uint32_t f) { return 0x0a010000u | f; }
  static uint16_t port(uint32_t f) { return (uint16_t)(32768 + (f * 7919) % 28000); }
  void setup(uint32_t n) {
    n_flows = n;
    flow_of_port.assign(65536, 0);
    for (uint32_t f = 0; f < n; f++) flow_of_port[port(f)] = f + 1;
    srv_data.assign(n, 0);
    cli_isn.resize(n);
    srv_isn.assign(n, 0);
    sum_base.resize(n);
    for (uint32_t f = 0; f < n; f++) cli_isn[f] = 0x10000000u * (f & 15) + f * 7919u;
    for (uint32_t i = 0; i < kPayload; i++) payload[i] = (uint8_t)(i * 31 + 7);
  }
  segtest::Seg seg(uint32_t f, uint8_t flags, uint32_t seq, uint32_t ack) const {
    segtest::Seg s;
    s.src_ip = ip(f);
    s.src_port = port(f);
    s.seq = seq;
    s.ack = ack;
    s.flags = flags;
    return s;
  }
  uint32_t dataSeq(uint32_t f, uint64_t k) const { return cli_isn[f] + 1 + (uint32_t)(k * kPayload); }
  uint32_t ackOf(uint32_t f) const { return srv_isn[f] + 1 + (uint32_t)srv_data[f]; }
  // a data frame's seq and ack (and its TCP checksum from the flow's base sum, built with both 0)
  void patch(uint8_t* eth, uint32_t f, uint32_t seq) const {
    const uint32_t ack = ackOf(f);
    segtest::put32(eth + 38, seq);
    segtest::put32(eth + 42, ack);
    uint32_t acc = sum_base[f] + (seq >> 16) + (seq & 0xffff) + (ack >> 16) + (ack & 0xffff);
    acc = (acc & 0xffff) + (acc >> 16);
    acc = (acc & 0xffff) + (acc >> 16);
    segtest::put16(eth + 50, (uint16_t)~acc);
  }

  const char* open(const char*) { return nullptr; }
  uint32_t fill(uint8_t* slots, uint32_t stride, uint32_t off, uint32_t cap) {
    if (!g_writer) return fillHere(slots, stride, off, cap);
    struct Job {
      BenchLink* l;
      uint8_t* slots;
      uint32_t stride, off, cap, n;
    } j{this, slots, stride, off, cap, 0};
    const double before = fill_s;
    const auto t0 = Clock::now();
    g_writer->run([](void* a) { auto* x = static_cast<Job*>(a); x->n = x->l->fillHere(x->slots, x->stride, x->off, x->cap); }, &j);
    fill_s = before + secs(t0, Clock::now()); // the link's time as the server's core sees it (handshake included)
    return j.n;
  }
  uint32_t fillHere(uint8_t* slots, uint32_t stride, uint32_t off, uint32_t cap) {
    const auto t0 = Clock::now();
    uint32_t n = 0;
    if (phase == Syn || phase == Ack) {
      for (; hs_next < n_flows && n < cap; hs_next++, n++) {
        const uint32_t f = hs_next;
        segtest::Seg s = phase == Syn ? seg(f, segtest::SYN, cli_isn[f], 0)
                                      : seg(f, segtest::ACK, cli_isn[f] + 1, srv_isn[f] + 1);
        if (phase == Syn) s.opts = {2, 4, 0x05, 0xb4}; // MSS 1460
        segtest::build(slots + (size_t)n * stride + off, s);
      }
      if (hs_next == n_flows) phase = Idle, hs_next = 0;
    } else if (phase == Data && cap < n_flows) {
      if (hdr.empty()) { // each flow's data-frame header with seq 0, and its TCP sum without the checksum field
        hdr.resize((size_t)n_flows * 54);
        seg_k.assign(n_flows, 0);
        std::vector<uint8_t> fr(2048);
        for (uint32_t f = 0; f < n_flows; f++) {
          segtest::Seg s = seg(f, segtest::ACK | segtest::PSH, 0, 0);
          s.payload = payload.data();
          s.len = kPayload;
          segtest::build(fr.data(), s);
          std::memcpy(&hdr[(size_t)f * 54], fr.data(), 54);
          sum_base[f] = (uint16_t)~(uint16_t)(fr[50] << 8 | fr[51]);
        }
      }
      for (; n < cap; n++) {
        const uint32_t f = cursor;
        cursor = cursor + 1 == n_flows ? 0 : cursor + 1;
        uint8_t* eth = slots + (size_t)n * stride + off;
        if (slots != paid_base) paid_base = slots, paid_n = 0;
        if (n >= paid_n) {
          std::memcpy(eth + 54, payload.data(), kPayload);
          paid_n = n + 1;
        }
        std::memcpy(eth, &hdr[(size_t)f * 54], 54);
        patch(eth, f, dataSeq(f, seg_k[f]++));
      }
      data_frames += n;
    } else if (phase == Data) {
      const uint32_t per_flow = cap / n_flows;
      n = per_flow * n_flows;
      if ((written[0] != slots && written[1] != slots && written[2] != slots) || written_n != n) { // whole frames
        for (uint32_t i = 0; i < n; i++) {
          const uint32_t f = i % n_flows;
          segtest::Seg s = seg(f, segtest::ACK | segtest::PSH, 0, 0);
          s.payload = payload.data();
          s.len = kPayload;
          uint8_t* eth = slots + (size_t)i * stride + off;
          segtest::build(eth, s);
          if (i < n_flows) { // the sum without the checksum field, with seq and ack 0
            const uint16_t c = (uint16_t)(eth[50] << 8 | eth[51]);
            sum_base[f] = (uint16_t)~c;
          }
        }
        if (written_n != n) written[0] = written[1] = written[2] = nullptr;
        (written[0] ? written[1] ? written[2] : written[1] : written[0]) = slots;
        written_n = n;
      }
      for (uint32_t i = 0; i < n; i++) { // seq, ack and checksum of segment k of flow f
        const uint32_t f = i % n_flows;
        patch(slots + (size_t)i * stride + off, f, dataSeq(f, poll_no * per_flow + i / n_flows));
      }
      poll_no++;
      data_frames += n;
    }
    if (cold) // as a NIC's DMA leaves them: every line of the frames written this fill out of the caches
      for (uint32_t i = 0; i < n; i++)
        for (uint32_t b = 0; b < off + 1514; b += 64) _mm_clflush(slots + (size_t)i * stride + b);
    if (cold) _mm_mfence(); // the flushes done inside the fill (the link's time), not in the server's
    fill_s += secs(t0, Clock::now());
    return n;
  }
  void send(const uint8_t* eth, uint32_t) {
    const uint8_t flags = eth[47];
    if (flags & segtest::RST) {
      rsts++;
    } else if ((flags & (segtest::SYN | segtest::ACK)) == (segtest::SYN | segtest::ACK)) {
      const uint16_t dport = (uint16_t)(eth[36] << 8 | eth[37]);
      for (uint32_t f = 0; f < n_flows; f++)
        if (port(f) == dport) srv_isn[f] = (uint32_t)eth[38] << 24 | eth[39] << 16 | eth[40] << 8 | eth[41];
      synacks++;
    } else if ((flags & ~segtest::PSH) == segtest::ACK) { // pure ACKs carry PSH, as all of efvitcp's frames (TcpConn.h:427)
      const uint32_t tot = (uint32_t)(eth[16] << 8 | eth[17]), payload = tot - 20 - (eth[46] >> 4) * 4;
      if (payload == 0) {
        acks++;
      } else if (echo) { // echoed data: the peer acknowledges it in its next frames
        const uint32_t f = flow_of_port[(uint16_t)(eth[36] << 8 | eth[37])];
        if (f) srv_data[f - 1] += payload;
        echo_bytes += payload;
        echo_frames++;
      } else {
        other++;
        other_flags = flags;
      }
    } else {
      other++;
      other_flags = flags;
    }
  }
  uint32_t localIp() const { return htonl(0x0a000001); }
  const uint8_t* localMac() const { return kServerMac; }
  const char* resolveMac(uint32_t, uint8_t*) { return "not used by a server"; }
};

struct Handler {
  uint64_t bytes = 0, calls = 0, sink = 0, connected = 0, disconnected = 0, echo_refused = 0;
  bool echo = false; // the reference example's echo server (example/tcpserver.cc): every delivery written back
  template <class C>
  uint32_t onTcpData(C& c, const uint8_t* d, uint32_t n) {
    uint64_t w;
    std::memcpy(&w, d, 8);
    sink ^= w;
    bytes += n;
    calls++;
    if (echo && !c.writeNonblock(d, n)) echo_refused++;
    return 0;
  }
  template <class C>
  void onTcpConnected(C&) {
    connected++;
  }
  template <class C>
  void onTcpDisconnect(C&) {
    disconnected++;
  }
  template <class C>
  void onSendTimeout(C&) {}
  template <class C>
  void onRecvTimeout(C&) {}
};

// The sequential backend with its legs timed: pipelined, a poll's frames are classified in launch() and dispatched
// (the engine's per-record host work: NIC filter, connection, onPack, handler, ACK decisions) in collect(), so the
// host dispatch cost per frame is measured on its own -- the part of a poll the GPU backend leaves on the host.
struct TimedOracleBackend : OracleBackend {
  double launch_s = 0, collect_s = 0, tx_s = 0;
  uint64_t collected = 0;
  const char* launch(uint32_t half, uint32_t n, const ConnTable& t) {
    const auto t0 = Clock::now();
    const char* e = OracleBackend::launch(half, n, t);
    launch_s += secs(t0, Clock::now());
    return e;
  }
  template <class F>
  const char* collect(uint32_t half, uint32_t n, const ConnTable& t, F&& f) {
    const auto t0 = Clock::now();
    const char* e = OracleBackend::collect(half, n, t, f);
    collect_s += secs(t0, Clock::now());
    collected += n;
    return e;
  }
  const char* fillTxLaunch(uint32_t n, uint32_t half) {
    const auto t0 = Clock::now();
    const char* e = OracleBackend::fillTxLaunch(n, half);
    tx_s += secs(t0, Clock::now());
    return e;
  }
};

// The GPU backend with the host's wait for each batch's records timed (pipelined: ready() before the dispatch).
struct TimedGpuBackend : GpuBackend {
  double wait_s = 0;
  const char* ready(uint32_t half) {
    const auto t0 = Clock::now();
    const char* e = GpuBackend::ready(half);
    wait_s += secs(t0, Clock::now());
    return e;
  }
};

template <uint32_t kBatch, uint32_t kChunk = 0, bool kPipe = false, bool kResident = false, bool kEcho = false,
          bool kLinks = false, uint32_t kDepth = 1>
struct Conf {
  static const uint32_t RecvBufSize = 65536;
  static const uint32_t MaxConns = 1024;
  static const uint32_t SendTimeoutSec = 0;
  static const uint32_t RecvTimeoutSec = 0;
  // echo: every 1,460-B delivery goes back as two segments (SMSS 956 with 1-KiB send buffers), acknowledged a
  // poll or two later; otherwise the server sends no data
  static const uint32_t ConnSendBufCnt = kEcho ? 64 : 16;
  static const uint32_t RxBatch = kBatch;
  static const uint32_t TxBatch = kEcho ? 4 * kBatch : kBatch;
  static const uint32_t RxChunk = kChunk;
  static const bool RxPipeline = kPipe;
  static const uint32_t RxPipelineDepth = kDepth; // with kPipe: polls a batch stays in flight (1 or 2)
  static const bool RxResident = kResident;
  static const bool RxLinks = kLinks; // with RxResident: the chain links and the in-order fast path
  struct UserData {};
};

struct Run {
  double mfps = 0, us_poll = 0, acks_per_frame = 0, fill_share = 0, classify_share = 0, tx_share = 0;
  double ns_classify = -1, ns_dispatch = -1; // TimedOracleBackend: per frame, in launch() / collect()
  double in_order_share = -1;                 // frames through the in-order fast path (chain links), of all
  double echo_gbps = -1;                      // echo workload: payload bits the server sent back per second
  double wait_us = -1;                        // TimedGpuBackend: host time per poll waiting for a batch's records
  bool ok = false;
  std::string err;
};

// verify = false: the checksum discard off, as the reference's release build runs (no checksum verified);
// the GPU backend then classifies from each frame's header lines only (pn_set_verify)
template <uint32_t kBatch, class Backend, uint32_t kChunk = 0, bool kPipe = false, bool kResident = false,
          bool kEcho = false, bool kLinks = false, uint32_t kDepth = 1>
static Run runOne(uint32_t n_flows, uint32_t polls, bool verify = true) {
  Run out;
  using Server = GpuTcpServer<Conf<kBatch, kChunk, kPipe, kResident, kEcho, kLinks, kDepth>, BenchLink, Backend>;
  auto srv = std::make_unique<Server>();
  srv->link().setup(n_flows);
  if (!srv->initWithLink("10.0.0.1", 1234)) {
    out.err = srv->getLastError();
    return out;
  }
  srv->setDropBadChecksum(verify);
  Handler h;
  BenchLink& link = srv->link();
  link.cold = g_cold;
  h.echo = link.echo = kEcho;
  link.phase = BenchLink::Syn;
  srv->poll(h);
  // (pipelined: frames are dispatched one poll later and the replies sent one poll after that)
  for (int k = 0; k < 8 && link.synacks < n_flows; k++) srv->poll(h);
  link.phase = BenchLink::Ack;
  srv->poll(h);
  for (int k = 0; k < 8 && h.connected < n_flows; k++) srv->poll(h);
  if (h.connected != n_flows || link.rsts) {
    out.err = "handshake: " + std::to_string(h.connected) + " connected, " + std::to_string(link.rsts) + " RSTs";
    return out;
  }
  link.phase = BenchLink::Data;
  const uint32_t warm = 8;
  for (uint32_t p = 0; p < warm; p++) srv->poll(h);
  const uint64_t bytes0 = h.bytes, acks0 = link.acks, echo0 = link.echo_bytes;
  link.fill_s = 0;
  if constexpr (std::is_same_v<Backend, TimedGpuBackend>) srv->backend().wait_s = 0;
  pn_sampler::start(std::is_base_of_v<GpuBackend, Backend> ? "gpu" : "twin");
  const auto t0 = Clock::now();
  for (uint32_t p = 0; p < polls; p++) srv->poll(h);
  const double t = secs(t0, Clock::now());
  if constexpr (std::is_same_v<Backend, TimedGpuBackend>) out.wait_us = srv->backend().wait_s * 1e6 / polls;
  pn_sampler::stop();
  const uint64_t timed_bytes = h.bytes - bytes0;
  if (kEcho) out.echo_gbps = (link.echo_bytes - echo0) * 8.0 / t / 1e9;
  link.phase = BenchLink::Idle;
  // pipelined: the last batch is still in flight (echo: its replies leave a poll after their dispatch)
  for (int k = 0; k < (kEcho ? 6 : 3); k++) srv->poll(h);
  const uint64_t frames = (uint64_t)polls * (kBatch / n_flows) * n_flows;
  out.mfps = frames / t / 1e6;
  out.us_poll = t * 1e6 / polls;
  out.acks_per_frame = (double)(link.acks - acks0) / frames;
  out.fill_share = link.fill_s / t;
  if (kResident && kLinks) out.in_order_share = (double)srv->inOrderFrames() / (double)link.data_frames;
  // the legs on their own, same frames: classify (+ the record walk, no dispatch) and the
  // TX checksum fill of one poll's ACKs
  const uint32_t n = (kBatch / n_flows) * n_flows, acks = (uint32_t)(out.acks_per_frame * n + 0.5);
  auto& be = srv->backend();
  const auto c0 = Clock::now();
  for (uint32_t p = 0; p < polls; p++)
    if (be.classify(n, srv->table(), [](uint64_t, const pn_result&, const uint8_t*, uint16_t = 0) {})) break;
  const auto c1 = Clock::now();
  // the TX leg as the engine runs it for a poll's ACKs: header-only frames get their sums as they are built (part
  // of the dispatch), so only a batch for pn_tx_fill (TxGpuMinDataFrames 0) is timed here
  for (uint32_t p = 0; p < polls && acks && Server::kTxGpuMin == 0; p++)
    if (be.fillTx(acks)) break;
  out.classify_share = secs(c0, c1) / t;
  out.tx_share = secs(c1, Clock::now()) / t;
  if constexpr (std::is_same_v<Backend, TimedOracleBackend>) {
    out.ns_classify = be.collected ? be.launch_s * 1e9 / be.collected : 0;
    out.ns_dispatch = be.collected ? be.collect_s * 1e9 / be.collected : 0;
  }
  out.ok = timed_bytes == frames * kPayload && h.bytes == (uint64_t)link.poll_no * (kBatch / n_flows) * n_flows * kPayload &&
           !link.rsts && !link.other && !h.disconnected && srv->getLastError() == nullptr &&
           (!kEcho || (link.echo_bytes == h.bytes && !h.echo_refused));
  if (!out.ok)
    out.err = srv->getLastError() ? srv->getLastError()
                                  : "delivered " + std::to_string(timed_bytes) + " of " + std::to_string(frames * kPayload) +
                                        " B, " + std::to_string(link.rsts) + " RSTs, " + std::to_string(link.other) +
                                        " other frames (flags " + std::to_string(link.other_flags) + "), " + std::to_string(h.disconnected) + " disconnects" +
                                        (kEcho ? ", echoed " + std::to_string(link.echo_bytes) + " of " + std::to_string(h.bytes) +
                                                     " B, " + std::to_string(h.echo_refused) + " refused writes"
                                               : std::string());
  return out;
}

#ifdef PN_BENCH_REF
// pollnet's EfviTcpServer Conf for the same server (its ServerConf fixes the rest, EfviTcp.h:191-212: 512 RX slots,
// 64 events per pollNet, 1024 1-KiB send buffers per connection -- ~1 GiB at MaxConns 1024)
struct RefBenchConf {
  static const uint32_t RecvBufSize = 65536;
  static const uint32_t MaxConns = 1024;
  static const uint32_t SendTimeoutSec = 0;
  static const uint32_t RecvTimeoutSec = 0;
  struct UserData {};
};

// The reference's own server on the same workload, one core: each poll takes at most 64 frames (Core.h:496-498),
// so the same frames as `polls` polls of 512 take 8x the polls.  Built without EFVITCP_DEBUG, as pollnet ships it:
// no checksum is verified (the release path).
static Run runRef(uint32_t n_flows, uint32_t polls, bool echo = false) {
  Run out;
  using Srv = efvitcp::EfviTcpServer<RefBenchConf>;
  auto link = std::make_unique<BenchLink>();
  link->cold = g_cold;
  link->setup(n_flows);
  efvitcp::RefEnv& env = efvitcp::refEnv();
  env.link = link.get();
  env.fill = [](void* l, uint8_t* slots, uint32_t stride, uint32_t off, uint32_t cap) {
    return static_cast<BenchLink*>(l)->fill(slots, stride, off, cap);
  };
  env.send = [](void* l, const uint8_t* eth, uint32_t len) { static_cast<BenchLink*>(l)->send(eth, len); };
  timespec ts;
  ::clock_gettime(CLOCK_REALTIME, &ts); // the reference's clock (Core::getns)
  env.init_ns = ts.tv_sec * 1000000000LL + ts.tv_nsec;
  env.local_ip = link->localIp();
  std::memcpy(env.local_mac, link->localMac(), 6);
  std::unique_ptr<Srv> srv(new Srv());
  if (!srv->init("bench", "10.0.0.1", 1234)) {
    out.err = srv->getLastError();
    return out;
  }
  Handler h;
  h.echo = link->echo = echo;
  link->phase = BenchLink::Syn;
  for (int k = 0; k < 64 && link->synacks < n_flows; k++) srv->poll(h);
  link->phase = BenchLink::Ack;
  for (int k = 0; k < 64 && h.connected < n_flows; k++) srv->poll(h);
  if (h.connected != n_flows || link->rsts) {
    out.err = "reference handshake: " + std::to_string(h.connected) + " connected, " + std::to_string(link->rsts) + " RSTs";
    return out;
  }
  link->phase = BenchLink::Data;
  const uint32_t ref_polls = polls * 8, warm = 64;
  for (uint32_t p = 0; p < warm; p++) srv->poll(h);
  const uint64_t bytes0 = h.bytes, acks0 = link->acks, frames0 = link->data_frames, echo0 = link->echo_bytes;
  link->fill_s = 0;
  pn_sampler::start("reference");
  const auto t0 = Clock::now();
  for (uint32_t p = 0; p < ref_polls; p++) srv->poll(h);
  const double t = secs(t0, Clock::now());
  pn_sampler::stop();
  const uint64_t frames = link->data_frames - frames0;
  if (echo) out.echo_gbps = (link->echo_bytes - echo0) * 8.0 / t / 1e9;
  out.mfps = frames / t / 1e6;
  out.us_poll = t * 1e6 / ref_polls;
  out.acks_per_frame = (double)(link->acks - acks0) / frames;
  out.fill_share = link->fill_s / t;
  out.ok = frames == (uint64_t)ref_polls * 64 && h.bytes - bytes0 == frames * kPayload &&
           h.bytes == link->data_frames * kPayload && !link->rsts && !link->other && !h.disconnected &&
           (!echo || (link->echo_bytes == h.bytes && !h.echo_refused));
  if (!out.ok)
    out.err = "reference: delivered " + std::to_string(h.bytes - bytes0) + " B of " + std::to_string(frames) + " frames, " +
              std::to_string(link->rsts) + " RSTs, " + std::to_string(link->other) + " other frames, " +
              std::to_string(h.disconnected) + " disconnects";
  return out;
}
#endif

static std::string json(const Run& r) {
  char b[448];
  if (!r.err.empty() && !r.ok) { // the message whole, quotes and backslashes escaped (it may quote a frame or a path)
    std::string e = "{\"error\": \"";
    for (const char ch : r.err) {
      if (ch == '"' || ch == '\\') e += '\\';
      e += (ch >= 0x20 ? ch : ' ');
    }
    return e + "\"}";
  }
  std::snprintf(b, sizeof b,
                "{\"mframes_per_s\": %.3f, \"gbit_per_s\": %.1f, \"us_per_poll\": %.1f, \"acks_per_frame\": %.3f, "
                "\"link_fill_share\": %.3f, \"mframes_per_s_server_only\": %.3f, \"classify_share\": %.3f, "
                "\"tx_fill_share\": %.3f}",
                r.mfps, r.mfps * 1514 * 8 / 1e3, r.us_poll, r.acks_per_frame, r.fill_share,
                r.fill_share < 1 ? r.mfps / (1 - r.fill_share) : 0.0, r.classify_share, r.tx_share);
  std::string o(b);
  if (r.in_order_share >= 0) {
    o.pop_back();
    char x[96];
    std::snprintf(x, sizeof x, ", \"in_order_fast_path_share\": %.3f}", r.in_order_share);
    o += x;
  }
  if (r.wait_us >= 0) {
    o.pop_back();
    char x[64];
    std::snprintf(x, sizeof x, ", \"wait_us_per_poll\": %.3f}", r.wait_us);
    o += x;
  }
  if (r.echo_gbps >= 0) {
    o.pop_back();
    char x[96];
    std::snprintf(x, sizeof x, ", \"echo_payload_gbit_per_s\": %.2f}", r.echo_gbps);
    return o + x;
  }
  if (r.ns_dispatch >= 0) {
    o.pop_back();
    char x[160];
    std::snprintf(x, sizeof x, ", \"ns_per_frame_total\": %.2f, \"ns_per_frame_classify\": %.2f, \"ns_per_frame_dispatch\": %.2f}",
                  r.mfps > 0 ? 1e3 / r.mfps : 0.0, r.ns_classify, r.ns_dispatch);
    return o + x;
  }
  return o;
}

int main(int argc, char** argv) {
  const uint32_t n_flows = argc > 1 ? std::atoi(argv[1]) : 256;
  const uint32_t polls = argc > 2 ? std::atoi(argv[2]) : 400;
  if (n_flows == 0 || n_flows > 512 || 512 % n_flows) {
    std::fprintf(stderr, "n_flows must divide 512\n");
    return 2;
  }
  std::string lines;
  bool ok = true;
  auto leg = [&](const char* name, const Run& r) {
    lines += std::string(lines.empty() ? "" : ", ") + "\"" + name + "\": " + json(r);
    ok = ok && r.ok;
  };
  const bool cpu_only = argc > 3 && std::strcmp(argv[3], "cpu") == 0;
  if (argc > 3 && std::strcmp(argv[3], "echo") == 0) {
    // the reference example's server (example/tcpserver.cc): every delivery written back, the peers acknowledging
    // it; TX batches of data frames take pn_tx_fill (GPU) / the oracle's fill (twin) / copyAndSum (reference)
    leg("gpu_echo_512_release_path", runOne<512, GpuBackend, 0, false, false, true>(n_flows, polls, false));
    leg("gpu_echo_512_pipelined_release_path", runOne<512, GpuBackend, 0, true, false, true>(n_flows, polls, false));
    leg("gpu_echo_512_pipelined_resident_release_path", runOne<512, GpuBackend, 0, true, true, true>(n_flows, polls, false));
    leg("cpu_echo_512_release_path", runOne<512, OracleBackend, 0, false, false, true>(n_flows, polls, false));
#ifdef PN_BENCH_REF
    leg("reference_server_echo_release_build", runRef(n_flows, polls, true));
#endif
  } else if (argc > 3 && std::strcmp(argv[3], "depth_ab") == 0) {
    // the best leg pipelined one and two polls deep (Conf::RxPipelineDepth), the host's wait per poll timed, beside
    // the reference's server
    leg("gpu_rxbatch_512_pipelined_resident_release_path_timed",
        runOne<512, TimedGpuBackend, 0, true, true>(n_flows, polls, false));
    leg("gpu_rxbatch_512_pipelined2_resident_release_path_timed",
        runOne<512, TimedGpuBackend, 0, true, true, false, false, 2>(n_flows, polls, false));
    leg("gpu_rxbatch_512_pipelined2_resident_release_path",
        runOne<512, GpuBackend, 0, true, true, false, false, 2>(n_flows, polls, false));
#ifdef PN_BENCH_REF
    leg("reference_server_release_build", runRef(n_flows, polls));
#endif
  } else if (argc > 3 && std::strcmp(argv[3], "twin_timed") == 0) { // the host dispatch alone (profiling)
    leg("cpu_rxbatch_512_pipelined_release_path_timed", runOne<512, TimedOracleBackend, 0, true>(n_flows, polls, false));
    // the same with the chain links (the oracle's, as the resident service's linked posts): the in-order fast path
    leg("cpu_rxbatch_512_pipelined_linked_release_path_timed",
        runOne<512, TimedOracleBackend, 0, true, true, false, true>(n_flows, polls, false));
  } else if (argc > 3 && std::strcmp(argv[3], "release_pair") == 0) { // one pair on its own (profiling the host side)
    leg("cpu_rxbatch_512_release_path", runOne<512, OracleBackend>(n_flows, polls, false));
    leg("cpu_rxbatch_512_pipelined_release_path_timed", runOne<512, TimedOracleBackend, 0, true>(n_flows, polls, false));
#ifdef PN_BENCH_REF
    leg("reference_server_release_build", runRef(n_flows, polls));
#endif
  } else if (argc > 3 && (std::strcmp(argv[3], "resident_pair") == 0 || std::strcmp(argv[3], "resident_pair_cold") == 0 ||
                           std::strcmp(argv[3], "resident_pair_l3") == 0)) {
    // the drop-in's best leg beside the reference, with the frames hot (the link writes them on the server's core),
    // _l3: written by another core (as a NIC with DDIO / cache injection leaves them), _cold: out of the CPU caches
    // after each fill (a NIC's DMA without DDIO); the same for both legs
    g_cold = std::strcmp(argv[3], "resident_pair_cold") == 0;
    static RemoteWriter writer;
    if (std::strcmp(argv[3], "resident_pair_l3") == 0) {
      if (!writer.start()) {
        std::fprintf(stderr, "resident_pair_l3: needs two allowed CPUs\n");
        return 2;
      }
      g_writer = &writer;
      lines += "\"cpus_server_writer\": [" + std::to_string(writer.cpu_server) + ", " + std::to_string(writer.cpu_writer) + "]";
    }
    leg("gpu_rxbatch_512_pipelined_resident_release_path", runOne<512, GpuBackend, 0, true, true>(n_flows, polls, false));
    // the same with the chain links (Conf::RxLinks): the GPU's chain pass in each post, the in-order fast path
    leg("gpu_rxbatch_512_pipelined_resident_linked_release_path",
        runOne<512, GpuBackend, 0, true, true, false, true>(n_flows, polls, false));
#ifdef PN_BENCH_REF
    leg("reference_server_release_build", runRef(n_flows, polls));
#endif
  } else if (argc > 3 && std::strcmp(argv[3], "quick") == 0) { // bench.py's secondary leg
    leg("gpu_rxbatch_512", runOne<512, GpuBackend>(n_flows, polls));
    leg("gpu_rxbatch_16384_pipelined", runOne<16384, GpuBackend, 0, true>(n_flows, polls / 4));
    leg("gpu_rxbatch_512_release_path", runOne<512, GpuBackend>(n_flows, polls, false));
    leg("gpu_rxbatch_16384_pipelined_release_path", runOne<16384, GpuBackend, 0, true>(n_flows, polls / 4, false));
    // the reference's batch in throughput mode (Conf::RxPipeline: each poll's frames dispatched in the next poll,
    // their classify overlapped with this poll's host work), both paths
    leg("gpu_rxbatch_512_pipelined", runOne<512, GpuBackend, 0, true>(n_flows, polls));
    leg("gpu_rxbatch_512_pipelined_release_path", runOne<512, GpuBackend, 0, true>(n_flows, polls, false));
    // the classify in the resident service (Conf::RxResident: a post per poll, no launch), both paths
    leg("gpu_rxbatch_512_resident", runOne<512, GpuBackend, 0, false, true>(n_flows, polls));
    leg("gpu_rxbatch_512_resident_release_path", runOne<512, GpuBackend, 0, false, true>(n_flows, polls, false));
    leg("gpu_rxbatch_512_pipelined_resident", runOne<512, GpuBackend, 0, true, true>(n_flows, polls));
    leg("gpu_rxbatch_512_pipelined_resident_release_path", runOne<512, GpuBackend, 0, true, true>(n_flows, polls, false));
    leg("cpu_rxbatch_512", runOne<512, OracleBackend>(n_flows, polls));
    // the same sequential server with the discard off: the reference's release build (no checksum summed per frame)
    leg("cpu_rxbatch_512_release_path", runOne<512, OracleBackend>(n_flows, polls, false));
#ifdef PN_BENCH_REF
    leg("reference_server_release_build", runRef(n_flows, polls));
#endif
  } else if (!cpu_only) {
    leg("gpu_rxbatch_512", runOne<512, GpuBackend>(n_flows, polls));
    leg("gpu_rxbatch_4096", runOne<4096, GpuBackend>(n_flows, polls));
    leg("gpu_rxbatch_16384", runOne<16384, GpuBackend>(n_flows, polls / 4));
    leg("gpu_rxbatch_512_chunk_128", runOne<512, GpuBackend, 128>(n_flows, polls));
    leg("gpu_rxbatch_512_chunk_256", runOne<512, GpuBackend, 256>(n_flows, polls));
    leg("gpu_rxbatch_4096_chunk_512", runOne<4096, GpuBackend, 512>(n_flows, polls));
    leg("gpu_rxbatch_4096_chunk_1024", runOne<4096, GpuBackend, 1024>(n_flows, polls));
    leg("gpu_rxbatch_16384_chunk_2048", runOne<16384, GpuBackend, 2048>(n_flows, polls / 4));
    leg("gpu_rxbatch_16384_chunk_4096", runOne<16384, GpuBackend, 4096>(n_flows, polls / 4));
    leg("gpu_rxbatch_512_pipelined", runOne<512, GpuBackend, 0, true>(n_flows, polls));
    leg("gpu_rxbatch_4096_pipelined", runOne<4096, GpuBackend, 0, true>(n_flows, polls));
    leg("gpu_rxbatch_16384_pipelined", runOne<16384, GpuBackend, 0, true>(n_flows, polls / 4));
  }
  if (argc <= 3 || (std::strcmp(argv[3], "quick") != 0 && std::strcmp(argv[3], "release_pair") != 0 &&
                    std::strcmp(argv[3], "resident_pair") != 0 && std::strcmp(argv[3], "resident_pair_cold") != 0 &&
                    std::strcmp(argv[3], "resident_pair_l3") != 0 &&
                    std::strcmp(argv[3], "twin_timed") != 0 && std::strcmp(argv[3], "echo") != 0 &&
                    std::strcmp(argv[3], "depth_ab") != 0)) {
    leg("cpu_rxbatch_512", runOne<512, OracleBackend>(n_flows, polls));
    leg("cpu_rxbatch_512_release_path", runOne<512, OracleBackend>(n_flows, polls, false));
    leg("cpu_rxbatch_4096", runOne<4096, OracleBackend>(n_flows, polls / 4));
    leg("cpu_rxbatch_4096_pipelined", runOne<4096, OracleBackend, 0, true>(n_flows, polls / 4));
#ifdef PN_BENCH_REF
    leg("reference_server_release_build", runRef(n_flows, polls));
#endif
  }
  std::printf("{\"bench\": \"tcp_server_poll\", \"workload\": \"%u flows connected through the server's handshake, "
              "in-order 1514-B frames (1460-B payload), RxBatch frames per poll, handler consumes, server ACKs\", "
              "%s, \"delivered_ok\": %s}\n",
              n_flows, lines.c_str(), ok ? "true" : "false");
  return ok ? 0 : 1;
}
