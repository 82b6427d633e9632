// Host-side internals shared by the library's translation units: the pn_ctx
// definition (opaque in include/pollnet_amd.h) and the error plumbing behind
// pn_last_error (the reference's const char* / getLastError convention, Core.h:253-383).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/pollnet_amd.h"

// The last launch that used a ctx-owned resource (a notify counter, the TX patch scratch): its stream while that
// handle is known valid (until the ctx's next pn_set_conn_table / pn_sync), then an event.
struct pn_fence {
  hipStream_t s = nullptr;
  hipEvent_t ev = nullptr; // created on first need, owned
  uint8_t state = 0;       // 0: nothing pending, 1: pending on s, 2: pending behind ev
};

struct pn_ctx {
  int device = 0;
  // Conn table: two device buffers.  Launches read tbl_buf[cur] (tbl_dev); pn_set_conn_table
  // uploads into the other one, whose readers (launches issued before the previous set) it
  // waits for through `retired`, then flips.  It never waits for the table it replaces.
  pn_conn_entry* tbl_buf[2] = {nullptr, nullptr};
  uint32_t tbl_cap[2] = {0, 0};
  int cur = 0;
  pn_conn_entry* tbl_dev = nullptr; // tbl_buf[cur] once a table is set
  uint32_t n_entries = 0;
  uint64_t mask = 0;
  uint32_t max_conn = 0;
  bool verify_tcp = true; // pn_set_verify: false = header lines only (the reference's release path)
  std::vector<hipStream_t> streams; // distinct streams launched on since the last set / sync
  std::vector<hipEvent_t> retired;  // recorded on those streams at the last set (pooled)
  size_t n_retired = 0;
  hipStream_t copy_stream = nullptr; // internal, non-blocking: table uploads
  void* tx_patch = nullptr;          // pn_tx_fill's per-frame patch records (8 B each)
  uint32_t tx_patch_n = 0;
  pn_fence tx;                       // the last launch that used tx_patch
  void* sig_count = nullptr;         // pn_*_notify workgroup counters: [0] classify, [16] tx_fill (64-B apart)
  pn_fence sig[2];
  std::vector<pn_service*> services; // open resident services (pn_service_*): their posts capture table buffers
  std::string err;
};

namespace pn_internal {

inline thread_local std::string g_err; // last error of calls made without a ctx

inline int set_err(pn_ctx* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  g_err = msg;
  return code;
}

// Before pn_set_conn_table overwrites or frees table buffer `buf`: wait for every resident-service post that
// captured it (rx_service.hip).
int svc_release_table(pn_ctx* ctx, int buf);

inline int hip_err(pn_ctx* ctx, hipError_t e, const char* what) {
  return set_err(ctx, PN_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

// Every launch of the ctx names its stream here (no per-launch event: a compare with the
// last stream).  The handle must stay valid until the ctx's next
// pn_set_conn_table or pn_sync returns (include/pollnet_amd.h).
inline void note_stream(pn_ctx* ctx, hipStream_t s) {
  if (!ctx->streams.empty() && ctx->streams.back() == s) return;
  for (size_t i = 0; i < ctx->streams.size(); ++i)
    if (ctx->streams[i] == s) {
      std::swap(ctx->streams[i], ctx->streams.back());
      return;
    }
  ctx->streams.push_back(s);
}

inline int ensure_event(pn_ctx* ctx, hipEvent_t* ev) {
  if (*ev) return PN_OK;
  hipError_t e = hipEventCreateWithFlags(ev, hipEventDisableTiming);
  if (e != hipSuccess) return hip_err(ctx, e, "hipEventCreate");
  return PN_OK;
}

// Before the fenced resource is freed: the host waits for its last user.
inline int fence_host_wait(pn_ctx* ctx, pn_fence& f) {
  hipError_t e = hipSuccess;
  if (f.state == 1) e = hipStreamSynchronize(f.s);
  else if (f.state == 2) e = hipEventSynchronize(f.ev);
  if (e != hipSuccess) return hip_err(ctx, e, "waiting for the last user of ctx scratch");
  f.state = 0;
  return PN_OK;
}

// Before a launch on `s` uses the fenced resource: order it after the previous user, on the
// device (hipStreamWaitEvent), without blocking the host.
inline int fence_use(pn_ctx* ctx, pn_fence& f, hipStream_t s) {
  hipError_t e = hipSuccess;
  if (f.state == 1 && f.s != s) {
    int rc = ensure_event(ctx, &f.ev);
    if (rc) return rc;
    e = hipEventRecord(f.ev, f.s);
    if (e == hipSuccess) e = hipStreamWaitEvent(s, f.ev, 0);
  } else if (f.state == 2) {
    e = hipStreamWaitEvent(s, f.ev, 0);
  }
  if (e != hipSuccess) return hip_err(ctx, e, "ordering after the previous user of ctx scratch");
  f.s = s;
  f.state = 1;
  return PN_OK;
}

// pn_set_conn_table: stop holding stream handles; what is pending becomes an event.
inline int fence_detach(pn_ctx* ctx, pn_fence& f) {
  if (f.state != 1) return PN_OK;
  int rc = ensure_event(ctx, &f.ev);
  if (rc) return rc;
  hipError_t e = hipEventRecord(f.ev, f.s);
  if (e != hipSuccess) return hip_err(ctx, e, "hipEventRecord(ctx scratch fence)");
  f.state = 2;
  f.s = nullptr;
  return PN_OK;
}

// Readers of the inactive table buffer (every launch issued before the previous
// pn_set_conn_table) have finished.  Normally long done: the wait returns at once.
inline int wait_retired(pn_ctx* ctx) {
  for (size_t i = 0; i < ctx->n_retired; ++i) {
    hipError_t e = hipEventSynchronize(ctx->retired[i]);
    if (e != hipSuccess) return hip_err(ctx, e, "hipEventSynchronize(previous table readers)");
  }
  ctx->n_retired = 0;
  return PN_OK;
}

// Mark the end of everything launched since the last set: one event per stream seen (the
// only place stream handles are used after their launch), then forget the handles.
inline int retire_streams(pn_ctx* ctx) {
  for (size_t i = 0; i < ctx->streams.size(); ++i) {
    if (ctx->retired.size() <= i) ctx->retired.push_back(nullptr);
    int rc = ensure_event(ctx, &ctx->retired[i]);
    if (rc) return rc;
    hipError_t e = hipEventRecord(ctx->retired[i], ctx->streams[i]);
    if (e != hipSuccess) return hip_err(ctx, e, "hipEventRecord(table readers)");
  }
  ctx->n_retired = ctx->streams.size();
  ctx->streams.clear();
  for (pn_fence* f : {&ctx->sig[0], &ctx->sig[1], &ctx->tx}) {
    int rc = fence_detach(ctx, *f);
    if (rc) return rc;
  }
  return PN_OK;
}

// The workgroup counter of a notify launch of `kind` (0 classify, 1 tx_fill), device memory,
// zero between launches (the last workgroup resets it).  The next launch of that kind reuses it:
// one on another stream is ordered after the previous one on the device.
inline int notify_counter(pn_ctx* ctx, int kind, hipStream_t s, uint32_t** out) {
  hipError_t e;
  if (!ctx->sig_count) {
    e = hipMalloc(&ctx->sig_count, 128);
    if (e == hipSuccess) e = hipMemsetAsync(ctx->sig_count, 0, 128, s); // ordered before this first launch
    if (e != hipSuccess) return hip_err(ctx, e, "hipMalloc(notify counters)");
    // both counters were zeroed on s: a first launch of the other kind on another stream waits for it
    for (pn_fence& f : ctx->sig) {
      f.s = s;
      f.state = 1;
    }
    note_stream(ctx, s);
  }
  int rc = fence_use(ctx, ctx->sig[kind], s);
  if (rc) return rc;
  *out = (uint32_t*)ctx->sig_count + 16 * kind;
  return PN_OK;
}

} // namespace pn_internal
