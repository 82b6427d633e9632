// gpu_rx.hpp — header-only C++ host adapter over the pn_* C-ABI.
//
// Mirrors the RX branch of efvitcp's Core<Conf>::pollNet (efvitcp/Core.h:494-552)
// for a batch of ring slots: one GPU launch classifies the whole batch, then the
// records are dispatched on the host in ring order exactly where the reference
// would have branched:
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

#include <cstdint>
#include <cstring>

#include "../pollnet_amd.h"

namespace pollnet_amd {

class ConnTable {
 public:
  ConnTable() = default;
  ConnTable(const ConnTable&) = delete;
  ConnTable& operator=(const ConnTable&) = delete;
  ~ConnTable() { pn_table_destroy(t_); }

  const char* init(uint32_t max_conn_cnt, uint32_t max_tw_cnt) {
    pn_table_destroy(t_);
    t_ = nullptr;
    return pn_table_create(max_conn_cnt, max_tw_cnt, &t_) ? "pn_table_create failed" : nullptr;
  }
  static uint64_t key(uint32_t ip_be, uint16_t port_be) { return pn_conn_hash_key(ip_be, port_be); } // Core.h:167
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
  GpuRx() = default;
  GpuRx(const GpuRx&) = delete;
  GpuRx& operator=(const GpuRx&) = delete;
  ~GpuRx() { destruct(); }

  // device: GPU ordinal; slot_stride/frame_off: the ring layout (RecvBufSize = 2048,
  // frame_off = sizeof(RecvBuf) + receive_prefix_len in the reference); max_batch:
  // the largest n passed to pollBatch().
  const char* init(int device, uint32_t slot_stride, uint32_t frame_off, uint32_t max_batch) {
    destruct();
    if (pn_open(device, &ctx_)) return pn_last_error(nullptr);
    stride_ = slot_stride;
    off_ = frame_off;
    cap_ = max_batch;
    if (hipSetDevice(device) != hipSuccess) return "hipSetDevice failed";
    if (hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking) != hipSuccess) return "hipStreamCreate failed";
    if (hipMalloc(&d_frames_, (size_t)slot_stride * max_batch) != hipSuccess) return "hipMalloc(frames) failed";
    if (hipMalloc(&d_res_, sizeof(pn_result) * (size_t)max_batch) != hipSuccess) return "hipMalloc(results) failed";
    if (hipHostMalloc(&h_res_, sizeof(pn_result) * (size_t)max_batch, hipHostMallocDefault) != hipSuccess)
      return "hipHostMalloc(results) failed";
    return nullptr;
  }

  // Snapshot the host table to the device (after add/del/enterTW).
  const char* syncTable(const ConnTable& t) {
    uint32_t n = 0;
    uint64_t mask = 0;
    const pn_conn_entry* e = t.entries(&n, &mask);
    max_conn_ = t.maxConnCnt();
    return pn_set_conn_table(ctx_, e, n, mask, max_conn_) ? pn_last_error(ctx_) : nullptr;
  }

  // Classify n slots of the host ring (pinned memory copies fastest) and dispatch.
  // recv_handler(uint64_t key, const pn_result& rec, const uint8_t* eth, uint32_t miss_entry_idx)
  // tw_handler(uint64_t key, uint32_t tw_id, const uint8_t* eth, const pn_result& rec)
  template <class RecvHandler, class TwHandler>
  const char* pollBatch(const uint8_t* host_slots, uint32_t n, const ConnTable& table, RecvHandler&& recv_handler,
                        TwHandler&& tw_handler) {
    if (n > cap_) return "batch larger than max_batch";
    if (n == 0) return nullptr;
    if (hipMemcpyAsync(d_frames_, host_slots, (size_t)stride_ * n, hipMemcpyHostToDevice, stream_) != hipSuccess)
      return "hipMemcpyAsync H2D failed";
    if (pn_classify(ctx_, d_frames_, stride_, off_, n, d_res_, stream_)) return pn_last_error(ctx_);
    if (hipMemcpyAsync(h_res_, d_res_, sizeof(pn_result) * n, hipMemcpyDeviceToHost, stream_) != hipSuccess)
      return "hipMemcpyAsync D2H failed";
    if (hipStreamSynchronize(stream_) != hipSuccess) return "hipStreamSynchronize failed";
    for (uint32_t i = 0; i < n; i++) {
      const uint8_t* eth = host_slots + (size_t)i * stride_ + off_;
      const pn_result& r = h_res_[i];
      uint32_t ip_be;
      uint16_t port_be;
      std::memcpy(&ip_be, eth + 14 + 12, 4);  // ip_hdr->src_ip
      std::memcpy(&port_be, eth + 14 + 20, 2); // tcp_hdr->src_port (tcp = ip + 20)
      const uint64_t key = pn_conn_hash_key(ip_be, port_be);
      if (r.flags & PN_F_TW) {
        tw_handler(key, r.conn_id - max_conn_, eth, r);
      } else {
        uint32_t idx = PN_MISS;
        if (!(r.flags & PN_F_HIT)) table.find(key, &idx, nullptr);
        recv_handler(key, r, eth, idx);
      }
    }
    return nullptr;
  }

  pn_ctx* ctx() { return ctx_; }
  hipStream_t stream() { return stream_; }

 private:
  void destruct() {
    if (h_res_) (void)hipHostFree(h_res_);
    if (d_res_) (void)hipFree(d_res_);
    if (d_frames_) (void)hipFree(d_frames_);
    if (stream_) (void)hipStreamDestroy(stream_);
    pn_close(ctx_);
    h_res_ = nullptr;
    d_res_ = nullptr;
    d_frames_ = nullptr;
    stream_ = nullptr;
    ctx_ = nullptr;
  }

  pn_ctx* ctx_ = nullptr;
  hipStream_t stream_ = nullptr;
  void* d_frames_ = nullptr;
  pn_result* d_res_ = nullptr;
  pn_result* h_res_ = nullptr;
  uint32_t stride_ = 0, off_ = 0, cap_ = 0, max_conn_ = 0;
};

} // namespace pollnet_amd
