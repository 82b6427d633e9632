// Device-side helpers shared by the gfx950 kernels (rx_kernel.hip, stream_kernel.hip):
// exact u16-word sums with v_dot2_u32_u16, CSum::fold, DPP moves, raw buffer
// descriptors, and fixed-offset field access into a register-resident header window.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace pn_dev {

using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;
using u16x2 = __attribute__((ext_vector_type(2))) unsigned short;

__device__ __forceinline__ uint32_t dot2(uint32_t w, uint32_t sel, uint32_t acc) {
  // acc + w.lo*sel.lo + w.hi*sel.hi ; sel halves are 0/1 -> masked sum of u16 halves
  return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, w), __builtin_bit_cast(u16x2, sel), acc, false);
}

__device__ __forceinline__ uint32_t bswap16(uint32_t v) { return ((v & 0xff) << 8) | ((v >> 8) & 0xff); }

// CSum::fold (Core.h:94-98) on an exact (non-overflowing) u32 sum.
__device__ __forceinline__ uint32_t csum_fold(uint32_t s) {
  uint32_t r = (s >> 16) + (s & 0xffff);
  r += r >> 16;
  return (~r) & 0xffff;
}

template <int DPP>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, DPP, 0xf, 0xf, false);
}

// Between a wave's writes to its own LDS tile and other lanes' reads of them (and back): a
// wavefront-scope release, the wave barrier, a wavefront-scope acquire.  LDS ops of one wave
// execute in order on the hardware, so this costs at most an lgkmcnt wait; what it buys is the
// ordering under the memory model, so the compiler may not move a read above the write it needs.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// A buffer-load offset past every descriptor's range (at most a few MiB here): the load returns zeros and
// fetches nothing.  Used instead of a branch around a load, so that loads stay in flight together.
constexpr uint32_t kNoFetch = 0x80000000u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t frame_rsrc(const uint8_t* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)bytes, 0x00020000);
}

// Header-window accessors at compile-time byte offsets O relative to the
// 16-B aligned window start (MIS + field offset).
template <int NW>
struct Win {
  uint32_t d[NW];
  template <int O>
  __device__ __forceinline__ uint32_t b8() const { return (d[O / 4] >> (8 * (O % 4))) & 0xff; }
  template <int O>
  __device__ __forceinline__ uint32_t u16() const {
    static_assert(O % 2 == 0, "even offset");
    return (d[O / 4] >> (8 * (O % 4))) & 0xffff;
  }
  template <int O>
  __device__ __forceinline__ uint32_t u32() const {
    static_assert(O % 2 == 0, "even offset");
    if constexpr (O % 4 == 0) return d[O / 4];
    else return __builtin_amdgcn_alignbyte(d[O / 4 + 1], d[O / 4], 2);
  }
  // exact sum of the u16 words in [LO, HI) (both even, compile-time)
  template <int LO, int HI>
  __device__ __forceinline__ uint32_t sum16() const {
    uint32_t acc = 0;
#pragma unroll
    for (int q = LO / 4; q < (HI + 3) / 4; ++q) {
      const uint32_t sel = ((4 * q >= LO && 4 * q < HI) ? 1u : 0u) | ((4 * q + 2 >= LO && 4 * q + 2 < HI) ? 0x10000u : 0u);
      acc = dot2(d[q], sel, acc);
    }
    return acc;
  }
  // sum of u16 words in [LO, lim) for runtime lim <= HI (RFC option bytes)
  template <int LO, int HI>
  __device__ __forceinline__ uint32_t sum16_upto(uint32_t lim) const {
    uint32_t acc = 0;
#pragma unroll
    for (int q = LO / 4; q < (HI + 3) / 4; ++q) {
      const uint32_t o0 = 4 * q, o1 = 4 * q + 2;
      const uint32_t sel = ((o0 >= LO && o0 < lim) ? 1u : 0u) | ((o1 >= LO && o1 < lim) ? 0x10000u : 0u);
      acc = dot2(d[q], sel, acc);
    }
    return acc;
  }
};

// Masked dot2 selector for dword k of a chunk whose first byte is `o` bytes into
// the window; halves at window offsets >= end are excluded.  end and o even.
__device__ __forceinline__ uint32_t tail_sel(int end, int o) {
  int t = end - o;
  t = t < 0 ? 0 : (t > 4 ? 4 : t); // 0, 2 or 4 valid bytes
  return (uint32_t)((t >> 1) + (t >> 2) * 0xffff);
}

} // namespace pn_dev
