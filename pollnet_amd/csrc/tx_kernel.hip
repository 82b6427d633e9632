// TX checksum fill: the product entry point pn_tx_fill.  Kernels and
// their design notes are in tx_fill.hpp; tuning variants in tx_tuning.hip (tuning library).
#include "tx_fill.hpp"

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
  const uint32_t mis = (frame_off + 14) & 15;
  if (mode == PN_TX_TCP) launch_mode<PN_TX_TCP>(a, mis, s);
  else if (mode == PN_TX_UDP_EFVI) launch_mode<PN_TX_UDP_EFVI>(a, mis, s);
  else launch_mode<PN_TX_UDP>(a, mis, s);
  e = hipGetLastError();
  if (e != hipSuccess) return hip_err(ctx, e, "tx_fill launch");
  ctx->last_stream = s;
  return PN_OK;
}
