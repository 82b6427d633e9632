// Host-side internals shared by the library's translation units: the pn_ctx
// definition (opaque in include/pollnet_amd.h) and the error plumbing behind
// pn_last_error (the reference's const char* / getLastError convention, Core.h:253-383).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "../../include/pollnet_amd.h"

struct pn_ctx {
  int device = 0;
  pn_conn_entry* tbl_dev = nullptr;
  uint32_t n_entries = 0;
  uint64_t mask = 0;
  uint32_t max_conn = 0;
  hipStream_t last_stream = nullptr;
  void* tx_patch = nullptr;       // pn_tx_fill's per-frame patch records (8 B each)
  uint32_t tx_patch_n = 0;
  hipStream_t tx_stream = nullptr; // stream of the last pn_tx_fill (the scratch is reused)
  void* sig_count = nullptr;       // pn_*_notify workgroup counters: [0] classify, [16] tx_fill (64-B apart)
  hipStream_t sig_stream[2] = {nullptr, nullptr}; // stream of the last notify launch of each kind
  bool sig_used[2] = {false, false};
  std::string err;
};

namespace pn_internal {

inline thread_local std::string g_err; // last error of calls made without a ctx

inline int set_err(pn_ctx* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  g_err = msg;
  return code;
}

inline int hip_err(pn_ctx* ctx, hipError_t e, const char* what) {
  return set_err(ctx, PN_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

// Before the device table is overwritten or freed: every launch that may read it has finished.
// Classify launches can be on any stream of the process (the caller's), so this waits for the
// whole device: a control-plane call, kept off the launch path (a per-launch event record
// costs ≈3-5 µs of idle GPU between back-to-back launches).
inline int wait_table_readers(pn_ctx* ctx) {
  hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) return hip_err(ctx, e, "hipDeviceSynchronize(table readers)");
  return PN_OK;
}

// The workgroup counter of a notify launch of `kind` (0 classify, 1 tx_fill), device memory,
// zero between launches (the last workgroup resets it).  The next launch of that kind reuses it,
// so a launch on another stream than the previous one first waits for the device (the previous
// stream may be gone; a rare path).
inline int notify_counter(pn_ctx* ctx, int kind, hipStream_t s, uint32_t** out) {
  hipError_t e;
  if (!ctx->sig_count) {
    e = hipMalloc(&ctx->sig_count, 128);
    if (e == hipSuccess) e = hipMemset(ctx->sig_count, 0, 128);
    if (e != hipSuccess) return hip_err(ctx, e, "hipMalloc(notify counters)");
  }
  if (ctx->sig_used[kind] && ctx->sig_stream[kind] != s) {
    e = hipDeviceSynchronize();
    if (e != hipSuccess) return hip_err(ctx, e, "hipDeviceSynchronize(notify counter)");
  }
  ctx->sig_stream[kind] = s;
  ctx->sig_used[kind] = true;
  *out = (uint32_t*)ctx->sig_count + 16 * kind;
  return PN_OK;
}

} // namespace pn_internal
