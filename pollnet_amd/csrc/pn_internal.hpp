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

} // namespace pn_internal
