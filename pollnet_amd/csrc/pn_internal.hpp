// Host-side internals shared by the library's translation units: the pn_ctx
// definition (opaque in include/pollnet_amd.h) and the error plumbing behind
// pn_last_error (the reference's const char* / getLastError convention, Core.h:253-383).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <utility>
#include <vector>

#include "../../include/pollnet_amd.h"

struct pn_ctx {
  int device = 0;
  pn_conn_entry* tbl_dev = nullptr;
  uint32_t n_entries = 0;
  uint64_t mask = 0;
  uint32_t max_conn = 0;
  hipStream_t last_stream = nullptr;
  // Streams with classify launches that read tbl_dev, each with an event recorded after
  // its latest such launch: pn_set_conn_table waits for all of them before replacing
  // the table (a launch on any stream may still be reading it).
  std::vector<std::pair<hipStream_t, hipEvent_t>> table_readers;
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

// After a launch that reads the device conn table on stream s.
inline int note_table_reader(pn_ctx* ctx, hipStream_t s) {
  hipEvent_t ev = nullptr;
  for (auto& r : ctx->table_readers)
    if (r.first == s) ev = r.second;
  if (!ev) {
    hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (e != hipSuccess) return hip_err(ctx, e, "hipEventCreate(table reader)");
    ctx->table_readers.emplace_back(s, ev);
  }
  hipError_t e = hipEventRecord(ev, s);
  if (e != hipSuccess) return hip_err(ctx, e, "hipEventRecord(table reader)");
  return PN_OK;
}

// Before the device table is overwritten: every launch that may read it has finished.
inline int wait_table_readers(pn_ctx* ctx) {
  for (auto& r : ctx->table_readers) {
    hipError_t e = hipEventSynchronize(r.second);
    if (e != hipSuccess) return hip_err(ctx, e, "hipEventSynchronize(table reader)");
  }
  return PN_OK;
}

} // namespace pn_internal
