// Tuning library: A/B variants of the TX fill (scripts/tx_variants.py), compiled only with
// `make` (TUNING=1 by default).  Never part of the product library.
#include "tx_fill.hpp"

// Tuning: after a phase-2 kernel with ordinary stores, a short launch whose workgroups each end with a
// system-scope release, which writes the L2's dirty lines back (one workgroup per XCD suffices; 64 cover the
// round-robin placement), so the patch's dirty sectors leave before the next call's read stream.
__global__ __launch_bounds__(64) void tx_l2_release_kernel(uint32_t* sink) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  if (threadIdx.x == 0 && sink[blockIdx.x] == 0x7fffffffu) sink[blockIdx.x] = 0; // never true: keeps the launch
}


// Same-run ceiling for pn_tx_fill (bench.py): the production launches (the fill kernel with
// its header window and stream loads, the patch records, the patch kernel's 2-byte stores) with
// the stream phase's lane reduction ablated -- the same loads and stores, next to no arithmetic.
// Timing only: the fields it writes are wrong.  Batches above kTxInPlaceMaxFrames (two launches),
// frame_off 2 or 14, cooperative layout.
extern "C" int pn_calib_tx_ablated(pn_ctx* ctx, void* frames, uint32_t slot_stride, uint32_t frame_off, uint32_t n,
                                   void* stream) {
  if (!ctx || !frames || n <= kTxInPlaceMaxFrames || (frame_off != 2 && frame_off != 14))
    return set_err(ctx, PN_EINVAL, "pn_calib_tx_ablated: bad arguments");
  TArgs a;
  a.frames = (uint8_t*)frames;
  a.lens = nullptr;
  a.n = n;
  a.stride = slot_stride;
  a.ipa_off = (frame_off + 14) & ~15u;
  a.avail = slot_stride - frame_off;
  a.frame_off = frame_off;
  a.fpw = frames_per_wave(n);
  if (!coop_layout(a) || slot_stride < frame_off + 96 || (slot_stride & 15))
    return set_err(ctx, PN_EINVAL, "pn_calib_tx_ablated: needs the cooperative layout");
  hipStream_t s = (hipStream_t)stream;
  int rc = ensure_patch(ctx, n, s);
  if (rc) return rc;
  a.patch = (uint2*)ctx->tx_patch;
  const dim3 grid((n + a.fpw - 1) / a.fpw), block(kWave);
  constexpr int SABL = kTxStream | kAblNoReduce;
  if (frame_off == 2)
    hipLaunchKernelGGL((tx_fill_kernel<0, 1, PN_TX_TCP, kWbPatch, 0, 0, 0, true, SABL>), grid, block, 0, s, a);
  else
    hipLaunchKernelGGL((tx_fill_kernel<12, 1, PN_TX_TCP, kWbPatch, 0, 0, 0, true, SABL>), grid, block, 0, s, a);
  hipLaunchKernelGGL((tx_patch_kernel<PN_TX_TCP>), dim3((n + 255) / 256), dim3(256), 0, s, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hip_err(ctx, e, "pn_calib_tx_ablated launch");
  pn_internal::note_stream(ctx, s);
  return PN_OK;
}

#ifdef PN_TUNING_VARIANTS

// Tuning variants (TCP mode, cooperative layouts, no lens), A/B-timed by
// scripts/tx_variants.py; not part of the public header.  History:
// profiles/r01_experiments/tx_variants_*.json.
extern "C" int pn_tx_fill_variant(pn_ctx* ctx, void* frames, uint32_t slot_stride, uint32_t frame_off, uint32_t n,
                                  const uint16_t* lens, int variant, void* stream) {
  if (!ctx || !frames || n == 0 || lens || (frame_off != 2 && frame_off != 14))
    return set_err(ctx, PN_EINVAL, "tx variant: bad args");
  TArgs a;
  a.frames = (uint8_t*)frames;
  a.lens = nullptr;
  a.n = n;
  a.stride = slot_stride;
  a.ipa_off = (frame_off + 14) & ~15u;
  a.avail = slot_stride - frame_off;
  a.frame_off = frame_off;
  // block write-back variants: the block is the slot's first line (every part loaded) inside the slot
  if (!coop_layout(a) || a.stride < a.ipa_off + kWinBytes || (a.stride % 128) || (((uintptr_t)a.frames + a.ipa_off) & 127u) != 16)
    return set_err(ctx, PN_EINVAL, "tx variant: needs the cooperative layout");
  hipStream_t s = (hipStream_t)stream;
  int rc = ensure_patch(ctx, variant >= 15 ? 2 * n : n, s); // 16-B record variants need 2 patch slots per frame
  if (rc) return rc;
  a.patch = (uint2*)ctx->tx_patch;
  const dim3 grid((n + kFramesPerWave - 1) / kFramesPerWave), block(kWave), pgrid((n + 255) / 256), pblock(256);
  auto go = [&](auto mis_tag) {
    constexpr int M = decltype(mis_tag)::value;
    constexpr int T = PN_TX_TCP;
    switch (variant) {
      case 0: hipLaunchKernelGGL((tx_fill_kernel<M, 1, T, 0, 0, kLoadAux>), grid, block, 0, s, a); return 0;     // in place, u16
      case 2: hipLaunchKernelGGL((tx_fill_kernel<M, 1, T, 128, 16, kLoadAux>), grid, block, 0, s, a); return 0;  // in place, line wb
      case 9: hipLaunchKernelGGL((tx_fill_kernel<M, 1, T, -1, 0, kLoadAux>), grid, block, 0, s, a); return 0;    // no writes
      case 10: // two-phase, line-0 window nt
        hipLaunchKernelGGL((tx_fill_kernel<M, 1, T, kWbPatch, 0, kLoadAux>), grid, block, 0, s, a);
        hipLaunchKernelGGL((tx_patch_kernel<T>), pgrid, pblock, 0, s, a);
        return 0;
      case 11: // two-phase, blockIdx order (production before the XCD order)
        hipLaunchKernelGGL((tx_fill_kernel<M, 1, T>), grid, block, 0, s, a);
        hipLaunchKernelGGL((tx_patch_kernel<T>), pgrid, pblock, 0, s, a);
        return 0;
      case 20: // two-phase, fill kernel at 4 waves/SIMD (2-KiB LDS pad)
        hipLaunchKernelGGL((tx_fill_kernel<M, 1, T, kWbPatch, 0, 0, 2>), grid, block, 0, s, a);
        hipLaunchKernelGGL((tx_patch_kernel<T>), pgrid, pblock, 0, s, a);
        return 0;
      case 21: // two-phase, fill kernel in XCD-contiguous order
        hipLaunchKernelGGL((tx_fill_kernel<M, 1, T, kWbPatch, 0, 0, 0, true>), grid, block, 0, s, a);
        hipLaunchKernelGGL((tx_patch_kernel<T>), pgrid, pblock, 0, s, a);
        return 0;
      // phase-2 store forms after the production phase 1 (line-0 window default policy, XCD order)
      case 30: case 32: case 33:
        hipLaunchKernelGGL((tx_fill_kernel<M, 1, T, kWbPatch, 0, 0, 0, true>), grid, block, 0, s, a);
        if (variant == 30) hipLaunchKernelGGL((tx_patch_kernel<T, 1>), pgrid, pblock, 0, s, a);      // 2-byte nt
        else if (variant == 32) hipLaunchKernelGGL((tx_patch_sector_kernel<0>), dim3((8 * n + 255) / 256), pblock, 0, s, a);
        else if (variant == 33) hipLaunchKernelGGL((tx_patch_sector_kernel<2>), dim3((8 * n + 255) / 256), pblock, 0, s, a);
        else return -1;
        return 0;
      case 35: hipLaunchKernelGGL((tx_probe_fullwrite_kernel<64>), dim3((4 * n + 255) / 256), pblock, 0, s, a); return 0;
      case 36: hipLaunchKernelGGL((tx_probe_fullwrite_kernel<128>), dim3((8 * n + 255) / 256), pblock, 0, s, a); return 0;
      case 13: hipLaunchKernelGGL((tx_fill_kernel<M, 1, T>), grid, block, 0, s, a); return 0; // phase 1 only
      case 14: hipLaunchKernelGGL((tx_patch_kernel<T>), pgrid, pblock, 0, s, a); return 0;    // phase 2 only
      case 15: hipLaunchKernelGGL((tx_fill_kernel<M, 1, T, -3>), grid, block, 0, s, a); return 0;  // phase 1, 16-B records
      case 16: hipLaunchKernelGGL((tx_fill_kernel<M, 1, T, -4>), grid, block, 0, s, a); return 0;  // phase 1, RX-style store
      // in place with the line-0 window at the default policy: the line is still in L2 when its
      // fields are written, so the 2-byte stores (or the patched line) merge there
      case 17: hipLaunchKernelGGL((tx_fill_kernel<M, 1, T, 0, 0, 0>), grid, block, 0, s, a); return 0;
      case 18: hipLaunchKernelGGL((tx_fill_kernel<M, 1, T, 128, 0, 0>), grid, block, 0, s, a); return 0;
      case 19: hipLaunchKernelGGL((tx_fill_kernel<M, 1, T, 128, 16, 0>), grid, block, 0, s, a); return 0;
      // the product's launch shape (frames_per_wave(n) per wave, XCD order): 40 = pn_tx_fill's
      // two phases, 41 = one launch writing the fields in place (small batches: one launch fewer)
      case 42: { // pn_tx_fill's two phases with empty stream loads skipped (kSkipEmptyLoads, measured, not adopted)
        TArgs b = a;
        b.fpw = frames_per_wave(n);
        hipLaunchKernelGGL((tx_fill_kernel<M, 1, T, kWbPatch, 0, 0, 0, true, kTxStream | kSkipEmptyLoads>), dim3((n + b.fpw - 1) / b.fpw), block,
                           0, s, b);
        hipLaunchKernelGGL((tx_patch_kernel<T>), pgrid, pblock, 0, s, b);
        return 0;
      }
      case 43: { // pn_tx_fill's two phases with the 8 window loads in flight at once (the RX kernel's form; slower here)
        TArgs b = a;
        b.fpw = frames_per_wave(n);
        hipLaunchKernelGGL((tx_fill_kernel<M, 1, T, kWbPatch, 0, 0, 0, true, kExactRange>),
                           dim3((n + b.fpw - 1) / b.fpw), block, 0, s, b);
        hipLaunchKernelGGL((tx_patch_kernel<T>), pgrid, pblock, 0, s, b);
        return 0;
      }
      // round 5 (the SendBuf layout's write pattern): the product's launch shape with a write-through
      // phase 2 (50: 2-byte fields, 51: whole 64-B sectors from a re-read), or the production phase 2 followed by
      // an L2 write-back launch (52)
      case 50: case 51: case 52: {
        TArgs b = a;
        b.fpw = frames_per_wave(n);
        hipLaunchKernelGGL((tx_fill_kernel<M, 1, T, kWbPatch, 0, 0, 0, true>), dim3((n + b.fpw - 1) / b.fpw), block, 0, s, b);
        if (variant == 50) {
          hipLaunchKernelGGL((tx_patch_wt_kernel<T, 0>), pgrid, pblock, 0, s, b);
        } else if (variant == 51) {
          hipLaunchKernelGGL((tx_patch_wt_kernel<T, 1>), dim3((8 * n + 255) / 256), pblock, 0, s, b);
        } else {
          hipLaunchKernelGGL((tx_patch_kernel<T>), pgrid, pblock, 0, s, b);
          hipLaunchKernelGGL(tx_l2_release_kernel, dim3(64), dim3(64), 0, s, reinterpret_cast<uint32_t*>(b.patch));
        }
        return 0;
      }
      case 40: case 41: {
        TArgs b = a;
        b.fpw = frames_per_wave(n);
        const dim3 g((n + b.fpw - 1) / b.fpw);
        if (variant == 41) {
          hipLaunchKernelGGL((tx_fill_kernel<M, 1, T, 0, 0, 0, 0, true>), g, block, 0, s, b);
        } else {
          hipLaunchKernelGGL((tx_fill_kernel<M, 1, T, kWbPatch, 0, 0, 0, true>), g, block, 0, s, b);
          hipLaunchKernelGGL((tx_patch_kernel<T>), pgrid, pblock, 0, s, b);
        }
        return 0;
      }
      default: return -1;
    }
  };
  rc = frame_off == 2 ? go(std::integral_constant<int, 0>{}) : go(std::integral_constant<int, 12>{});
  if (rc) return set_err(ctx, PN_EINVAL, "tx variant: unknown");
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hip_err(ctx, e, "tx variant launch");
  pn_internal::note_stream(ctx, s);
  return PN_OK;
}
#endif // PN_TUNING_VARIANTS
