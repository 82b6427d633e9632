// gpu_rx.hpp — header-only C++ host adapter over the pn_* C-ABI.
//
// Mirrors the RX branch of efvitcp's Core<Conf>::pollNet (efvitcp/Core.h:494-552)
// for a run of ring slots: GPU launches classify it chunk by chunk (chunk k+1 on the
// GPU while chunk k is dispatched), and the records are dispatched on the host in
// ring order exactly where the reference would have branched:
//   - TIME_WAIT hit (entry->key == key && conn_id >= MaxConnCnt, Core.h:510)
//       -> tw_handler(key, tw_id, eth, rec)            (reference: :511-523)
//   - otherwise -> recv_handler(key, entry_index, eth, rec)   (reference: :526)
// `eth` points into the caller's host ring (zero-copy, valid during the call, as
// TcpConn::onPack's payload pointer is, TcpConn.h:715); `rec` carries the
// payload offset/length, seq, TCP flags and the checksum verdicts the reference
// computes in onPack (TcpConn.h:469-473) and Core::checksum (Core.h:448-472).
// The conn table stays host-owned (ConnTable below wraps pn_table_*, the
// reference's addConnEntry/delConnEntry/enterTW) and is re-snapshotted to the
// device with syncTable() after control-plane changes.
//
// Errors follow the reference: const char* (nullptr = ok), Core.h:253-383.
#pragma once

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <type_traits>

#include "../pollnet_amd.h"

namespace pollnet_amd {

// connHashKey (Core.h:167-172), inline for the per-record host walk: the remote ip (host order) << 15 | the low 15
// port bits, the port's msb at bit 47.  pn_conn_hash_key is the same function behind the C ABI (conn_table.cpp);
// tests/cpp/test_tx_host.cpp checks it against the oracle's.
inline uint64_t conn_hash_key(uint32_t ip_be, uint16_t port_be) {
  const uint64_t ip = __builtin_bswap32(ip_be), p = __builtin_bswap16(port_be);
  return (ip << 15) | (p & 0x7fff) | ((p & 0x8000) << 32);
}

// The key of a frame's remote end: its IP source address and TCP source port (ip_hdr + 12, tcp_hdr = ip + 20).
inline uint64_t frame_key(const uint8_t* eth) {
  uint32_t ip_be;
  uint16_t port_be;
  std::memcpy(&ip_be, eth + 14 + 12, 4);
  std::memcpy(&port_be, eth + 14 + 20, 2);
  return conn_hash_key(ip_be, port_be);
}

// A record's checksum verdicts: both OK, or the IP one OK where the TCP sum was not computed (the release
// path, pn_set_verify(ctx, 0): PN_F_TCP_UNCHECKED).
inline bool checksums_ok(uint16_t flags) {
  const uint16_t need = PN_F_IP_OK | ((flags & PN_F_TCP_UNCHECKED) ? 0 : PN_F_TCP_OK);
  return (flags & need) == need;
}

// Wait for a pn_*_notify launch: spin on its host-visible word (an acquire load, the
// reference's busy-poll style).  Every 4096 polls the stream is queried; if it has drained (or
// failed) without the token, that is an error -- the caller synchronises the stream to report it.
inline const char* wait_word(const uint32_t* word, uint32_t token, hipStream_t s) {
  for (uint32_t i = 1;; ++i) {
    if (__atomic_load_n(word, __ATOMIC_ACQUIRE) == token) return nullptr;
    if ((i & 4095) == 0) {
      const hipError_t q = hipStreamQuery(s);
      if (q != hipErrorNotReady) {
        if (__atomic_load_n(word, __ATOMIC_ACQUIRE) == token) return nullptr;
        return q == hipSuccess ? "notify word not written" : "notify launch failed";
      }
    }
  }
}

class ConnTable {
 public:
  ConnTable() = default;
  ConnTable(const ConnTable&) = delete;
  ConnTable& operator=(const ConnTable&) = delete;
  ~ConnTable() { pn_table_destroy(t_); }

  // reference_literal: PN_TABLE_REFERENCE_LITERAL (the reference's rehash kept as is, defect included)
  const char* init(uint32_t max_conn_cnt, uint32_t max_tw_cnt, bool reference_literal = false) {
    pn_table_destroy(t_);
    t_ = nullptr;
    return pn_table_create_ex(max_conn_cnt, max_tw_cnt, reference_literal ? PN_TABLE_REFERENCE_LITERAL : 0u, &t_)
               ? "pn_table_create failed"
               : nullptr;
  }
  static uint64_t key(uint32_t ip_be, uint16_t port_be) { return conn_hash_key(ip_be, port_be); } // Core.h:167
  bool find(uint64_t key, uint32_t* entry_idx, uint32_t* conn_id) const {                              // Core.h:558
    int hit = 0;
    pn_table_find(t_, key, entry_idx, &hit, conn_id);
    return hit != 0;
  }
  int add(uint64_t key, uint32_t conn_id) { return pn_table_add(t_, key, conn_id); }                 // Core.h:566
  int del(uint64_t key) { return pn_table_del(t_, key); }                                           // Core.h:578
  int enterTW(uint64_t key, uint32_t tw_id) {                                                       // Core.h:627
    return pn_table_set_conn_id(t_, key, pn_table_max_conn_cnt(t_) + tw_id);
  }
  uint32_t size() const { return pn_table_size(t_); } // getTblSize(), Core.h:564
  uint32_t maxConnCnt() const { return pn_table_max_conn_cnt(t_); }
  const pn_conn_entry* entries(uint32_t* n, uint64_t* mask) const { return pn_table_entries(t_, n, mask); }

 private:
  pn_conn_table* t_ = nullptr;
};

class GpuRx {
 public:
  // Copy: pollBatch copies the slots H2D, classifies in device memory and copies the
  //   records back (any host memory; pinned copies fastest).
  // ZeroCopy: the kernel reads the slots straight from pinned host memory over PCIe
  //   (hipHostMalloc / hipHostRegister'd) and writes the records to pinned memory —
  //   only the frames' own cache lines cross the bus, no slot padding, no copy stage.
  //   Measured faster at every batch size (64 frames: 19 vs 27 us; 1 Mi C2 frames: 443 vs
  //   326 Gbit/s; mixed C3: 392 vs 175 Gbit/s — DESIGN.md §7, §13); Copy stays the default
  //   because it accepts any host memory.  Chunks of up to PN_NOTIFY_MAX_FRAMES go through
  //   pn_classify_notify: the host polls a pinned word instead of synchronising (≈4 us sooner).
  enum class Mode { Copy, ZeroCopy };

  GpuRx() = default;
  GpuRx(const GpuRx&) = delete;
  GpuRx& operator=(const GpuRx&) = delete;
  ~GpuRx() { destruct(); }

  // device: GPU ordinal; slot_stride/frame_off: the ring layout (RecvBufSize = 2048,
  // frame_off = sizeof(RecvBuf) + receive_prefix_len in the reference); max_batch:
  // the chunk pollBatch() classifies per launch (two chunks are in flight at once).
  // resident (ZeroCopy only): the chunks go to the resident classify service (pn_service_*: one launch, then a post
  // per chunk through its mailbox) instead of a launch each; resident_idle_ms: how long it stays without a post.
  // links (resident, max_batch <= PN_LINK_MAX_FRAMES): each post also returns its chain links
  // (pn_service_post_linked), handed to a recv_handler that takes a fifth argument.
  const char* init(int device, uint32_t slot_stride, uint32_t frame_off, uint32_t max_batch, Mode mode = Mode::Copy,
                   bool resident = false, uint32_t resident_idle_ms = 100, bool links = false) {
    destruct();
    if (max_batch == 0) return "max_batch must be > 0";
    if (pn_open(device, &ctx_)) return pn_last_error(nullptr);
    stride_ = slot_stride;
    off_ = frame_off;
    cap_ = max_batch;
    mode_ = mode;
    if (hipSetDevice(device) != hipSuccess) return "hipSetDevice failed";
    if (hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking) != hipSuccess) return "hipStreamCreate failed";
    if (mode == Mode::ZeroCopy) {
      if (hipHostMalloc((void**)&h_word_, 64 * kBufs, hipHostMallocDefault) != hipSuccess)
        return "hipHostMalloc(notify words) failed";
      std::memset(h_word_, 0, 64 * kBufs);
    }
    if (resident && mode == Mode::ZeroCopy && pn_service_open(ctx_, slot_stride, frame_off, resident_idle_ms, &svc_))
      return pn_last_error(ctx_);
    for (uint32_t b = 0; b < kBufs; b++) {
      if (mode == Mode::Copy) {
        if (hipMalloc(&d_frames_[b], (size_t)slot_stride * max_batch) != hipSuccess) return "hipMalloc(frames) failed";
        if (hipMalloc(&d_res_[b], sizeof(pn_result) * (size_t)max_batch) != hipSuccess)
          return "hipMalloc(results) failed";
      }
      if (hipHostMalloc(&h_res_[b], sizeof(pn_result) * (size_t)max_batch, hipHostMallocDefault) != hipSuccess)
        return "hipHostMalloc(results) failed";
      if (mode == Mode::ZeroCopy &&
          hipHostMalloc(&h_offs_[b], sizeof(uint64_t) * (size_t)max_batch, hipHostMallocDefault) != hipSuccess)
        return "hipHostMalloc(offsets) failed";
      use_word_[b] = waited_[b] = false;
      if (hipEventCreateWithFlags(&done_[b], hipEventDisableTiming) != hipSuccess) return "hipEventCreate failed";
    }
    links_ = links && svc_ && max_batch <= PN_LINK_MAX_FRAMES;
    for (uint32_t b = 0; b < kBufs && links_; b++)
      if (hipHostMalloc((void**)&h_links_[b], sizeof(uint16_t) * (size_t)max_batch, hipHostMallocDefault) != hipSuccess)
        return "hipHostMalloc(links) failed";
    return nullptr;
  }
  bool links() const { return links_; }

  // Snapshot the host table to the device (after add/del/enterTW).
  const char* syncTable(const ConnTable& t) {
    uint32_t n = 0;
    uint64_t mask = 0;
    const pn_conn_entry* e = t.entries(&n, &mask);
    max_conn_ = t.maxConnCnt();
    return pn_set_conn_table(ctx_, e, n, mask, max_conn_) ? pn_last_error(ctx_) : nullptr;
  }

  // Classify n slots of the host ring and dispatch every record in ring order.  The
  // slots go in chunks of max_batch; chunk k+1 is on the GPU while chunk k is
  // dispatched on the host.
  // recv_handler(uint64_t key, const pn_result& rec, const uint8_t* eth, uint32_t miss_entry_idx)
  // tw_handler(uint64_t key, uint32_t tw_id, const uint8_t* eth, const pn_result& rec)
  // kHitKey = false: a hit's key is not computed (0 is passed; the caller derives it from eth if it needs it)
  template <bool kHitKey = true, class RecvHandler, class TwHandler>
  const char* pollBatch(const uint8_t* host_slots, uint32_t n, const ConnTable& table, RecvHandler&& recv_handler,
                        TwHandler&& tw_handler) {
    if (mode_ == Mode::ZeroCopy)
      if (const char* e = check_pinned(host_slots)) return e;
    return run<kHitKey>(
        n, table, [&](uint32_t k) { return launch(host_slots, n, k); },
        [&](uint32_t i) { return host_slots + (size_t)i * stride_ + off_; }, recv_handler, tw_handler);
  }

  // RX events instead of a contiguous run: frame i's Ethernet
  // header is at ring + offsets[i] — for ef_vi, id * RecvBufSize + sizeof(RecvBuf) +
  // receive_prefix_len of each RX event in event order (Core.h:503-505), wrapping
  // round the ring and skipping discarded slots.  ZeroCopy mode only (the ring stays
  // where the NIC wrote it; it must be pinned or hipHostRegister'd).  eth_mod16 =
  // offsets[i] % 16 for every i; avail = readable bytes from each Ethernet header.
  // Records are dispatched in offsets order.
  template <class RecvHandler, class TwHandler>
  const char* pollIndexed(const uint8_t* ring, const uint64_t* offsets, uint32_t n, uint32_t eth_mod16, uint32_t avail,
                          const ConnTable& table, RecvHandler&& recv_handler, TwHandler&& tw_handler) {
    if (mode_ != Mode::ZeroCopy) return "pollIndexed needs Mode::ZeroCopy";
    if (const char* e = check_pinned(ring)) return e;
    auto launch_k = [&](uint32_t k) -> const char* {
      const uint32_t base = k * cap_, m = std::min(cap_, n - base), b = k & 1;
      std::memcpy(h_offs_[b], offsets + base, sizeof(uint64_t) * m); // buffer b is free: chunk k-2 was dispatched
      if (pn_classify_indexed(ctx_, ring, h_offs_[b], eth_mod16, m, avail, h_res_[b], stream_)) return pn_last_error(ctx_);
      if (hipEventRecord(done_[b], stream_) != hipSuccess) return "hipEventRecord failed";
      use_word_[b] = false;
      linked_[b] = false;
      return nullptr;
    };
    return run(
        n, table, launch_k, [&](uint32_t i) { return ring + offsets[i]; }, recv_handler, tw_handler);
  }

  // The two halves of pollBatch, for a caller that overlaps one batch's classify with other
  // host work (e.g. dispatching the previous batch): submit issues the classify of n <=
  // max_batch slots into record buffer b (0 .. kBufs - 1; at most one batch per buffer in flight),
  // complete waits for it and dispatches its records exactly as pollBatch does; ready waits only
  // (complete then dispatches at once).  The slots must stay untouched in between.
  static constexpr uint32_t kBufs = 3;
  const char* submit(const uint8_t* host_slots, uint32_t n, uint32_t b) {
    if (n > cap_ || b >= kBufs) return "submit: n > max_batch or buffer out of range";
    if (mode_ == Mode::ZeroCopy)
      if (const char* e = check_pinned(host_slots)) return e;
    const char* e = launch_at(host_slots, n, b);
    if (e) drain();
    return e;
  }
  const char* ready(uint32_t b) {
    if (b >= kBufs) return "ready: buffer out of range";
    if (waited_[b]) return nullptr;
    if (const char* e = wait_done(b)) {
      drain();
      return e;
    }
    waited_[b] = true;
    return nullptr;
  }
  template <bool kHitKey = true, class RecvHandler, class TwHandler>
  const char* complete(const uint8_t* host_slots, uint32_t n, uint32_t b, const ConnTable& table,
                       RecvHandler&& recv_handler, TwHandler&& tw_handler) {
    if (n > cap_ || b >= kBufs) return "complete: n > max_batch or buffer out of range";
    if (const char* e = ready(b)) return e;
    waited_[b] = false;
    auto eth_of = [&](uint32_t i) { return host_slots + (size_t)i * stride_ + off_; };
    walk<kHitKey>(h_res_[b], linked_[b] ? h_links_[b] : nullptr, 0, n, table, eth_of, recv_handler, tw_handler);
    return nullptr;
  }

  pn_ctx* ctx() { return ctx_; }
  bool resident() const { return svc_ != nullptr; }
  hipStream_t stream() { return stream_; }
  Mode mode() const { return mode_; }

 private:
  static const char* check_pinned(const void* p) {
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) != hipSuccess || attr.type != hipMemoryTypeHost)
      return "zero-copy ring must be pinned host memory (hipHostMalloc / hipHostRegister)";
    return nullptr;
  }

  // Chunked pipeline shared by pollBatch / pollIndexed: chunk k+1 is launched before
  // chunk k is dispatched; eth_of(i) = frame i's Ethernet header in host memory.
  // An error leaves no chunk in flight: the stream is drained before returning, so the
  // next call may reuse the pinned buffers at once.
  template <bool kHitKey = true, class Launch, class EthOf, class RecvHandler, class TwHandler>
  const char* run(uint32_t n, const ConnTable& table, Launch&& launch_k, EthOf&& eth_of, RecvHandler& recv_handler,
                  TwHandler& tw_handler) {
    const char* e = run_chunks<kHitKey>(n, table, launch_k, eth_of, recv_handler, tw_handler);
    if (e) drain();
    return e;
  }
  template <bool kHitKey, class Launch, class EthOf, class RecvHandler, class TwHandler>
  const char* run_chunks(uint32_t n, const ConnTable& table, Launch& launch_k, EthOf& eth_of, RecvHandler& recv_handler,
                         TwHandler& tw_handler) {
    if (n == 0) return nullptr;
    const uint32_t chunks = (n + cap_ - 1) / cap_;
    if (const char* e = launch_k(0)) return e;
    for (uint32_t k = 0; k < chunks; k++) {
      if (k + 1 < chunks)
        if (const char* e = launch_k(k + 1)) return e;
      if (const char* e = wait_done(k & 1)) return e;
      const uint32_t base = k * cap_, m = std::min(cap_, n - base);
      walk<kHitKey>(h_res_[k & 1], linked_[k & 1] ? h_links_[k & 1] : nullptr, base, m, table, eth_of, recv_handler, tw_handler);
    }
    return nullptr;
  }
  // Dispatch records res[0, m) of frames base.. in order (with their chain links, when the post returned them and
  // the handler takes them: recv_handler(key, rec, eth, miss_entry_idx, link)).
  template <bool kHitKey, class EthOf, class RecvHandler, class TwHandler>
  void walk(const pn_result* res, const uint16_t* links, uint32_t base, uint32_t m, const ConnTable& table,
            EthOf& eth_of, RecvHandler& recv_handler, TwHandler& tw_handler) {
    constexpr bool kTakesLink =
        std::is_invocable_v<RecvHandler&, uint64_t, const pn_result&, const uint8_t*, uint32_t, uint16_t>;
    for (uint32_t i = 0; i < m; i++) {
      const uint8_t* eth = eth_of(base + i);
      const pn_result& r = res[i];
      const uint64_t key = (kHitKey || (r.flags & (PN_F_HIT | PN_F_TW)) != PN_F_HIT) ? frame_key(eth) : 0;
      if (r.flags & PN_F_TW) {
        tw_handler(key, r.conn_id - max_conn_, eth, r);
      } else {
        uint32_t idx = PN_MISS;
        if (!(r.flags & PN_F_HIT)) table.find(key, &idx, nullptr);
        if constexpr (kTakesLink) recv_handler(key, r, eth, idx, links ? links[i] : (uint16_t)0);
        else recv_handler(key, r, eth, idx);
      }
    }
  }

  // Issue chunk k (H2D + classify + D2H, or one zero-copy classify) into buffer k&1.
  const char* launch(const uint8_t* host_slots, uint32_t n, uint32_t k) {
    const uint32_t base = k * cap_;
    return launch_at(host_slots + (size_t)base * stride_, std::min(cap_, n - base), k & 1);
  }
  // After an error: nothing of this GpuRx left in flight (service posts waited for, the stream drained).
  void drain() {
    for (uint32_t b = 0; b < kBufs; b++) {
      if (posted_[b]) (void)wait_done(b);
      waited_[b] = false;
    }
    (void)hipStreamSynchronize(stream_);
  }
  // Wait for buffer b's launch: its service post, its notify word, or its event.
  const char* wait_done(uint32_t b) {
    if (posted_[b]) {
      posted_[b] = false;
      return pn_service_wait(svc_, post_[b]) ? pn_last_error(ctx_) : nullptr;
    }
    if (use_word_[b]) return wait_word(&h_word_[16 * b], tok_[b], stream_);
    return hipEventSynchronize(done_[b]) == hipSuccess ? nullptr : "hipEventSynchronize failed";
  }
  // Issue the m slots at src into buffer b.
  const char* launch_at(const uint8_t* src, uint32_t m, uint32_t b) {
    use_word_[b] = waited_[b] = false;
    posted_[b] = false;
    linked_[b] = svc_ && links_;
    if (svc_) { // resident service: a post, no launch
      if (pn_service_post_linked(svc_, src, m, h_res_[b], links_ ? h_links_[b] : nullptr, &post_[b]))
        return pn_last_error(ctx_);
      posted_[b] = true;
      return nullptr;
    }
    if (mode_ == Mode::ZeroCopy && m <= PN_NOTIFY_MAX_FRAMES) { // small batch: completion by a pinned word
      tok_[b] = ++next_tok_;
      if (pn_classify_notify(ctx_, src, stride_, off_, m, h_res_[b], stream_, &h_word_[16 * b], tok_[b]))
        return pn_last_error(ctx_);
      use_word_[b] = true;
      return nullptr;
    }
    if (mode_ == Mode::ZeroCopy) {
      if (pn_classify(ctx_, src, stride_, off_, m, h_res_[b], stream_)) return pn_last_error(ctx_);
    } else {
      if (hipMemcpyAsync(d_frames_[b], src, (size_t)stride_ * m, hipMemcpyHostToDevice, stream_) != hipSuccess)
        return "hipMemcpyAsync H2D failed";
      if (pn_classify(ctx_, d_frames_[b], stride_, off_, m, d_res_[b], stream_)) return pn_last_error(ctx_);
      if (hipMemcpyAsync(h_res_[b], d_res_[b], sizeof(pn_result) * m, hipMemcpyDeviceToHost, stream_) != hipSuccess)
        return "hipMemcpyAsync D2H failed";
    }
    if (hipEventRecord(done_[b], stream_) != hipSuccess) return "hipEventRecord failed";
    return nullptr;
  }

  void destruct() {
    if (svc_) (void)pn_service_close(svc_);
    svc_ = nullptr;
    for (uint32_t b = 0; b < kBufs; b++) posted_[b] = false;
    if (stream_) (void)hipStreamSynchronize(stream_);
    for (uint32_t b = 0; b < kBufs; b++) {
      if (done_[b]) (void)hipEventDestroy(done_[b]);
      if (h_res_[b]) (void)hipHostFree(h_res_[b]);
      if (h_offs_[b]) (void)hipHostFree(h_offs_[b]);
      h_offs_[b] = nullptr;
      if (h_links_[b]) (void)hipHostFree(h_links_[b]);
      h_links_[b] = nullptr;
      if (d_res_[b]) (void)hipFree(d_res_[b]);
      if (d_frames_[b]) (void)hipFree(d_frames_[b]);
      done_[b] = nullptr;
      h_res_[b] = nullptr;
      d_res_[b] = nullptr;
      d_frames_[b] = nullptr;
    }
    if (stream_) (void)hipStreamDestroy(stream_);
    if (h_word_) (void)hipHostFree(h_word_);
    h_word_ = nullptr;
    pn_close(ctx_);
    stream_ = nullptr;
    ctx_ = nullptr;
  }

  pn_ctx* ctx_ = nullptr;
  hipStream_t stream_ = nullptr;
  Mode mode_ = Mode::Copy;
  void* d_frames_[kBufs] = {};
  pn_result* d_res_[kBufs] = {};
  pn_result* h_res_[kBufs] = {};
  uint64_t* h_offs_[kBufs] = {}; // ZeroCopy: pinned offsets the indexed kernel reads
  hipEvent_t done_[kBufs] = {};
  uint32_t* h_word_ = nullptr; // ZeroCopy: pinned notify words of the buffers (64 B apart)
  uint32_t tok_[kBufs] = {}, next_tok_ = 0;
  bool use_word_[kBufs] = {};
  bool waited_[kBufs] = {};      // buffer b's batch is complete (ready), not yet dispatched
  pn_service* svc_ = nullptr;       // resident classify service (ZeroCopy, init's `resident`)
  uint16_t* h_links_[kBufs] = {}; // pinned: each buffer's chain links (init's `links`)
  bool links_ = false, linked_[kBufs] = {}; // links on; buffer b's batch came with them
  uint32_t post_[kBufs] = {};       // buffer b's service post (every 32-bit id is one: the counter wraps)
  bool posted_[kBufs] = {};         // ... and whether it is outstanding
  uint32_t stride_ = 0, off_ = 0, cap_ = 0, max_conn_ = 0;
};

} // namespace pollnet_amd
