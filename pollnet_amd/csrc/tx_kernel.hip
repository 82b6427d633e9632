// TX checksum fill: the product entry points pn_tx_fill and
// pn_tx_fill_notify.  Kernels and their design notes are in tx_fill.hpp; tuning variants in
// tx_tuning.hip (tuning library).
#include "tx_fill.hpp"

namespace {
TArgs tx_args(pn_ctx* ctx, void* frames, uint32_t slot_stride, uint32_t frame_off, uint32_t n, const uint16_t* lens) {
  TArgs a;
  a.frames = (uint8_t*)frames;
  a.lens = lens;
  a.n = n;
  a.stride = slot_stride;
  a.ipa_off = (frame_off + 14) & ~15u;
  a.avail = slot_stride - frame_off;
  a.frame_off = frame_off;
  a.patch = (uint2*)ctx->tx_patch;
  a.fpw = frames_per_wave(n);
  return a;
}
} // namespace

extern "C" int pn_tx_fill(pn_ctx* ctx, void* frames, uint32_t slot_stride, uint32_t frame_off, uint32_t n,
                          const uint16_t* lens, uint32_t mode, void* stream) {
  if (!ctx) return set_err(nullptr, PN_EINVAL, "pn_tx_fill: ctx is NULL");
  if (mode != PN_TX_TCP && mode != PN_TX_UDP_EFVI && mode != PN_TX_UDP) return set_err(ctx, PN_EINVAL, "pn_tx_fill: unknown mode");
  if (n == 0) return PN_OK;
  int rc = check_args(ctx, frames, slot_stride, frame_off, lens);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return hip_err(ctx, e, "hipSetDevice");
  if (n > kTxInPlaceMaxFrames) { // the two-phase form's patch records (ctx scratch)
    rc = ensure_patch(ctx, n, s);
    if (rc) return rc;
  }
  const TArgs a = tx_args(ctx, frames, slot_stride, frame_off, n, lens);
  const uint32_t mis = (frame_off + 14) & 15;
  if (mode == PN_TX_TCP) launch_mode<PN_TX_TCP>(a, mis, s);
  else if (mode == PN_TX_UDP_EFVI) launch_mode<PN_TX_UDP_EFVI>(a, mis, s);
  else launch_mode<PN_TX_UDP>(a, mis, s);
  e = hipGetLastError();
  if (e != hipSuccess) return hip_err(ctx, e, "tx_fill launch");
  pn_internal::note_stream(ctx, s);
  return PN_OK;
}

// The one-launch in-place form with a completion word (signal_done, frame_pass.hpp).
extern "C" int pn_tx_fill_notify(pn_ctx* ctx, void* frames, uint32_t slot_stride, uint32_t frame_off, uint32_t n,
                                 const uint16_t* lens, uint32_t mode, void* stream, uint32_t* done_word, uint32_t token) {
  if (!ctx) return set_err(nullptr, PN_EINVAL, "pn_tx_fill_notify: ctx is NULL");
  if (mode != PN_TX_TCP && mode != PN_TX_UDP_EFVI && mode != PN_TX_UDP)
    return set_err(ctx, PN_EINVAL, "pn_tx_fill_notify: unknown mode");
  if (n == 0 || n > PN_NOTIFY_MAX_FRAMES || !done_word || ((uintptr_t)done_word & 3))
    return set_err(ctx, PN_EINVAL, "pn_tx_fill_notify: n must be in [1, PN_NOTIFY_MAX_FRAMES], done_word 4-byte aligned");
  int rc = check_args(ctx, frames, slot_stride, frame_off, lens);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return hip_err(ctx, e, "hipSetDevice");
  TArgs a = tx_args(ctx, frames, slot_stride, frame_off, n, lens);
  rc = pn_internal::notify_counter(ctx, 1, s, &a.sig_count);
  if (rc) return rc;
  a.sig_flag = done_word;
  a.sig_token = token;
  const uint32_t mis = (frame_off + 14) & 15;
  static_assert(PN_NOTIFY_MAX_FRAMES <= kTxInPlaceMaxFrames, "notify batches take the one-launch in-place form");
  if (mode == PN_TX_TCP) launch_mis<PN_TX_TCP, 0, true>(a, mis, s);
  else if (mode == PN_TX_UDP_EFVI) launch_mis<PN_TX_UDP_EFVI, 0, true>(a, mis, s);
  else launch_mis<PN_TX_UDP, 0, true>(a, mis, s);
  e = hipGetLastError();
  if (e != hipSuccess) return hip_err(ctx, e, "tx_fill (notify) launch");
  pn_internal::note_stream(ctx, s);
  return PN_OK;
}
