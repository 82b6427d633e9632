// Tuning library (libpollnet_amd_tuning.so, include/pollnet_amd_tuning.h): the RX kernel's
// A/B variants (scripts/variants.py, history in profiles/r01_experiments) and the
// same-run bandwidth ceilings bench.py reports beside the production kernel.  Never
// linked into or loaded by the product path; the variants are compiled only with
// `make` (TUNING=1 by default: -DPN_TUNING_VARIANTS; `make TUNING=0` leaves them out).
#include "rx_classify.hpp"
#include "stream_match.hpp"

namespace {
using pn_internal::g_err;
using pn_internal::hip_err;
using pn_internal::set_err;

__global__ __launch_bounds__(256) void calib_stream_read_kernel(const u32x4* src, uint64_t n16, uint32_t* sink) {
  // the whole grid sweeps the buffer front to back, one 16-B coalesced load per lane per step
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) {
    const u32x4 v = src[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9E3779B9u) sink[blockIdx.x] = acc; // keeps the loads live; practically never stores
}

// Test helper: one lane holds its stream until the host stores non-zero to *go (pinned host
// memory) or max_ticks of the device wall clock pass (always exits), then stores 1 (released)
// or 2 (timed out) to *done.  Stands for unrelated work in flight on a foreign stream.
__global__ __launch_bounds__(64) void spin_wait_kernel(const uint32_t* go, uint32_t* done, uint64_t max_ticks) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = wall_clock64();
  uint32_t r = 2;
  while (wall_clock64() - t0 < max_ticks) {
    if (__hip_atomic_load(go, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != 0) {
      r = 1;
      break;
    }
    __builtin_amdgcn_s_sleep(8);
  }
  __hip_atomic_store(done, r, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Latency probe (round 5, bench/bench_doorbell): how fast can a resident kernel answer the host?  One lane
// watches *bell (pinned host memory) and copies every new value to *echo; it ends at the value 0xFFFFFFFF or
// after max_idle_ticks of the device wall clock without a new value (always exits).  once = 1: answer the
// value already there and end (the launch-per-request form the product uses today).
__global__ __launch_bounds__(64) void doorbell_echo_kernel(const uint32_t* bell, uint32_t* echo, uint64_t max_idle_ticks,
                                                            uint32_t once, uint32_t sleep) {
  if (threadIdx.x != 0) return;
  uint32_t last = 0;
  uint64_t t_last = wall_clock64();
  for (;;) {
    // relaxed in the loop (a system-scope load reads memory; an acquire would invalidate the caches every
    // iteration); the acquire fence once a new value has arrived
    const uint32_t v = __hip_atomic_load(bell, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (v == 0xFFFFFFFFu) break;
    if (v != last || once) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      last = v;
      __hip_atomic_store(echo, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      if (once) break;
      t_last = wall_clock64();
    } else if (wall_clock64() - t_last > max_idle_ticks) {
      break;
    }
    if (sleep) __builtin_amdgcn_s_sleep(1);
  }
}

// The doorbell answered from a pipelined poll: K relaxed system-scope reads of the bell's 64-B line in flight (lane
// i reads word i & 15: the service mailbox's shape, no branch around the load), issued `gap` x 64 clocks apart; each is checked when it returns (the
// value stays in a VGPR until its readlane, so the compiler waits for the oldest read only: vmcnt(K - 1)).  A new
// value is seen about one gap after it lands rather than up to one read round trip later.  Reads issued before a value
// arrived return older values: only a larger value counts.
template <int K>
__global__ __launch_bounds__(64) void doorbell_echo_pipe_kernel(const uint32_t* bell, uint32_t* echo,
                                                                uint64_t max_idle_ticks, uint32_t gap) {
  const int lane = threadIdx.x;
  uint32_t last = 0;
  uint64_t t_last = wall_clock64();
  uint32_t q[K];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    q[j] = __hip_atomic_load(bell + (lane & 15), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    for (uint32_t g = 0; g < gap; ++g) __builtin_amdgcn_s_sleep(1);
  }
  // no return inside the loop: an exit path there makes the compiler drain every read at the loop head (vmcnt(0))
  bool go = true;
  while (go) {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const uint32_t v = (uint32_t)__builtin_amdgcn_readlane(q[j], 0);
      if (v == 0xFFFFFFFFu) {
        go = false;
      } else if ((int32_t)(v - last) > 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        last = v;
        if (lane == 0) __hip_atomic_store(echo, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        t_last = wall_clock64();
      } else if (wall_clock64() - t_last > max_idle_ticks) {
        go = false;
      }
      q[j] = __hip_atomic_load(bell + (lane & 15), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      for (uint32_t g = 0; g < gap; ++g) __builtin_amdgcn_s_sleep(1);
    }
  }
}

// Read-only ceilings for the slot layout (no header work, no arithmetic): each wave
// streams the first `bytes` of each of its 64 slots with the RX kernel's 1-KiB
// buffer loads, 8 slots per batch.  STORE = 16 / 8: plus a per-slot record store
// of that many bytes at the wave's end (sink holds n x 16 B), the RX kernel's
// write pattern.
template <int STORE>
__global__ __launch_bounds__(kWave) void calib_slot_read_kernel(const uint8_t* base, uint32_t n, uint32_t stride,
                                                               uint32_t bytes, uint32_t* sink) {
  const int lane = threadIdx.x;
  const uint32_t wave_base = blockIdx.x * kFramesPerWave;
  if (wave_base >= n) return;
  const uint32_t n_here = min((uint32_t)kFramesPerWave, n - wave_base);
  const uint8_t* wb = base + (uint64_t)wave_base * stride;
  uint32_t acc = 0;
  for (uint32_t b0 = 0; b0 < n_here; b0 += kBatch) {
    u32x4 w0s[kBatch], w1s[kBatch];
#pragma unroll
    for (int j = 0; j < kBatch; ++j) {
      const uint32_t nb = (b0 + j < n_here) ? bytes : 0u;
      const __amdgpu_buffer_rsrc_t rs = frame_rsrc(wb + (uint64_t)(b0 + j) * stride, nb);
      w0s[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, 0, 0);
      w1s[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, 1024 + lane * 16, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < kBatch; ++j) acc ^= w0s[j].x ^ w0s[j].y ^ w0s[j].z ^ w0s[j].w ^ w1s[j].x ^ w1s[j].y ^ w1s[j].z ^ w1s[j].w;
  }
  if constexpr (STORE == 16) {
    if (lane < (int)n_here) {
      u32x4 r = {acc, acc ^ 1u, acc ^ 2u, acc ^ 3u};
      *reinterpret_cast<u32x4*>(sink + 4 * (uint64_t)(wave_base + lane)) = r;
    }
  } else if constexpr (STORE == 8) {
    if (lane < (int)n_here) *reinterpret_cast<uint64_t*>(sink + 2 * (uint64_t)(wave_base + lane)) = ((uint64_t)acc << 32) | acc;
  } else {
    if (acc == 0x9E3779B9u) sink[blockIdx.x] = acc;
  }
}

// Ceiling for variable-length frames (C3/C5 slot rings): slot i's first lens[i] bytes (the
// frame's lines, from the slot start to the frame's pad byte), read with the RX kernel's load
// pattern, workgroup order (each XCD a contiguous eighth) and LDS occupancy cap, no arithmetic;
// STORE = 16 adds the 16-B records.  Out-of-range dwords of a line cost no extra traffic.
template <int STORE>
__global__ __launch_bounds__(kWave) void calib_slot_read_var_kernel(const uint8_t* base, uint32_t n, uint32_t stride,
                                                                   const uint32_t* lens, uint32_t* sink) {
  __shared__ uint32_t pad_lds[512];
  const int lane = threadIdx.x;
  pad_lds[lane] = lane;
  // never true: keeps the padding allocated (wave-uniform, so n and the descriptors stay scalar)
  if (__builtin_amdgcn_readfirstlane(pad_lds[(lane + 1) & 63]) == 0x7fffffffu) n = 0;
  const uint32_t wave_base = xcd_group(blockIdx.x, gridDim.x) * kFramesPerWave;
  if (wave_base >= n) return;
  const uint32_t n_here = min((uint32_t)kFramesPerWave, n - wave_base);
  const uint8_t* wb = base + (uint64_t)wave_base * stride;
  uint32_t acc = 0;
  for (uint32_t b0 = 0; b0 < n_here; b0 += kBatch) {
    u32x4 w0s[kBatch], w1s[kBatch];
#pragma unroll
    for (int j = 0; j < kBatch; ++j) {
      // one frame per load: its length is the same on every lane (scalar descriptor)
      const uint32_t nb = __builtin_amdgcn_readfirstlane(
          (b0 + j < n_here) ? min(lens[wave_base + b0 + j], min(stride, 2048u)) : 0u);
      const __amdgpu_buffer_rsrc_t rs = frame_rsrc(wb + (uint64_t)(b0 + j) * stride, nb);
      w0s[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, 0, 0);
      w1s[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, 1024 + lane * 16, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < kBatch; ++j) acc ^= w0s[j].x ^ w0s[j].y ^ w0s[j].z ^ w0s[j].w ^ w1s[j].x ^ w1s[j].y ^ w1s[j].z ^ w1s[j].w;
  }
  if constexpr (STORE == 16) {
    if (lane < (int)n_here) {
      u32x4 r = {acc, acc ^ 1u, acc ^ 2u, acc ^ 3u};
      *reinterpret_cast<u32x4*>(sink + 4 * (uint64_t)(wave_base + lane)) = r;
    }
  } else {
    if (acc == 0x9E3779B9u) sink[blockIdx.x] = acc;
  }
}

// Write-grouping probe: the slot-read ceiling with each 64-thread workgroup owning G
// consecutive 64-slot groups and writing their G x 64 16-B records (G KiB, contiguous) in
// one burst at the end instead of 1 KiB after each group.
// EACH = true: the same G-group loop, records written after each group (separates the
// effect of fewer, longer workgroups from that of the write bursts).
template <int G, bool EACH = false>
__global__ __launch_bounds__(kWave) void calib_slot_read_grouped_kernel(const uint8_t* base, uint32_t n, uint32_t stride,
                                                                       uint32_t bytes, uint32_t* sink) {
  __shared__ u32x4 recs[EACH ? 1 : G * kFramesPerWave];
  const int lane = threadIdx.x;
  for (int g = 0; g < G; ++g) {
    const uint32_t wave_base = (blockIdx.x * G + g) * kFramesPerWave;
    uint32_t acc = 0;
    if (wave_base < n) {
      const uint32_t n_here = min((uint32_t)kFramesPerWave, n - wave_base);
      const uint8_t* wb = base + (uint64_t)wave_base * stride;
      for (uint32_t b0 = 0; b0 < n_here; b0 += kBatch) {
        u32x4 w0s[kBatch], w1s[kBatch];
#pragma unroll
        for (int j = 0; j < kBatch; ++j) {
          const uint32_t nb = (b0 + j < n_here) ? bytes : 0u;
          const __amdgpu_buffer_rsrc_t rs = frame_rsrc(wb + (uint64_t)(b0 + j) * stride, nb);
          w0s[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, 0, kLoadAux);
          w1s[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, 1024 + lane * 16, 0, kLoadAux);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int j = 0; j < kBatch; ++j) acc ^= w0s[j].x ^ w0s[j].y ^ w0s[j].z ^ w0s[j].w ^ w1s[j].x ^ w1s[j].y ^ w1s[j].z ^ w1s[j].w;
      }
    }
    if constexpr (EACH) {
      if (wave_base + lane < n) {
        const __amdgpu_buffer_rsrc_t ro = frame_rsrc((const uint8_t*)(sink + 4 * (uint64_t)wave_base), 64 * 16);
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{acc, acc ^ 1u, acc ^ 2u, acc ^ 3u}, ro, lane * 16, 0, kStoreAux);
      }
    } else {
      recs[g * kFramesPerWave + lane] = u32x4{acc, acc ^ 1u, acc ^ 2u, acc ^ 3u};
    }
  }
  if constexpr (EACH) return;
  __syncthreads();
  const uint32_t first = blockIdx.x * G * kFramesPerWave;
  const __amdgpu_buffer_rsrc_t ro = frame_rsrc((const uint8_t*)(sink + 4 * (uint64_t)first),
                                               16 * min((uint32_t)(G * kFramesPerWave), n - first));
#pragma unroll
  for (int g = 0; g < G; ++g)
    __builtin_amdgcn_raw_buffer_store_b128(recs[g * kFramesPerWave + lane], ro, (g * kFramesPerWave + lane) * 16, 0, kStoreAux);
}

// The production launch's arguments (rx_kernel.hip strided_args) for the ceilings below.
int strided_args_calib(pn_ctx* ctx, const void* frames_dev, uint32_t slot_stride, uint32_t frame_off, uint32_t n,
                       void* results_dev, KArgs& a) {
  if (((uintptr_t)frames_dev & 15) || ((uintptr_t)results_dev & 15) || (slot_stride & 15) || slot_stride > 65536 ||
      slot_stride < frame_off + 96)
    return set_err(ctx, PN_EINVAL, "ceiling: layout contract");
  a.frames = (const uint8_t*)frames_dev;
  a.out = (pn_result*)results_dev;
  a.tbl = ctx->tbl_dev;
  a.mask = ctx->mask;
  a.n_entries = ctx->n_entries;
  a.max_conn = ctx->max_conn;
  a.n = n;
  a.stride = slot_stride;
  a.ipa_off = (frame_off + 14) & ~15u;
  a.avail = slot_stride - frame_off;
  a.offs = nullptr;
  a.fpw = frames_per_wave(n);
  if (!coop_layout(a)) return set_err(ctx, PN_EINVAL, "ceiling: needs the cooperative layout");
  return PN_OK;
}

} // namespace

extern "C" {


#ifdef PN_TUNING_VARIANTS
// Tuning: the indexed kernel with the cooperative line window (variant 1) or without (0),
// A/B-timed by scripts/bench_indexed.py; not part of the public header.
int pn_classify_indexed_variant(pn_ctx* ctx, const void* base, const uint64_t* offsets, uint32_t eth_mod16, uint32_t n,
                                uint32_t avail, void* results_dev, void* stream, int variant) {
  if (!ctx || !ctx->tbl_dev || n == 0 || eth_mod16 != 2 || variant < 0 || variant > 5)
    return set_err(ctx, PN_EINVAL, "indexed variant: bad args");
  KArgs a;
  a.frames = (const uint8_t*)base;
  a.out = (pn_result*)results_dev;
  a.tbl = ctx->tbl_dev;
  a.mask = ctx->mask;
  a.n_entries = ctx->n_entries;
  a.max_conn = ctx->max_conn;
  a.n = n;
  a.stride = 0;
  a.ipa_off = 0;
  a.avail = avail;
  a.offs = offsets;
  a.fpw = frames_per_wave(n);
  hipStream_t s = (hipStream_t)stream;
  if (variant == 1) launch_one<0, 1, kProdAbl, kLoadAux, kStoreAux, 1, kLoadAux, 1, kXcdOrder>(a, s); // window non-temporal
  else if (variant == 2) launch_one<0, 1, kProdAbl, kLoadAux, kStoreAux, 1, 0, 1, 0>(a, s);  // production window, blockIdx order
  else if (variant == 3) launch_one<0, 1, kProdAbl, 0, kStoreAux, 1, 0, 1, 0>(a, s);         // + stream at default policy
  else if (variant == 4) // timing only (packed captures): the wave's frames streamed as one contiguous range
    launch_one<0, 1, kProdAbl | kAblContigStream, kLoadAux, kStoreAux, 1, kIdxWin, 1, kXcdOrder>(a, s);
  else if (variant == 5) // production without kSkipEmptyLoads (every stream load issued)
    launch_one<0, 1, kProdAbl & ~kSkipEmptyLoads, kLoadAux, kStoreAux, 1, kIdxWin, 1, kXcdOrder>(a, s);
  else launch_one<0, 0, kProdAbl, kLoadAux, kStoreAux, 1, kLoadAux, 1, 0>(a, s);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hip_err(ctx, e, "indexed variant launch");
  pn_internal::note_stream(ctx, s);
  return PN_OK;
}


int pn_classify_variant(pn_ctx* ctx, const void* frames_dev, uint32_t slot_stride, uint32_t frame_off, uint32_t n,
                        void* results_dev, void* stream, int variant) {
  if (!ctx || !ctx->tbl_dev || (frame_off + 14) % 16 != 0 || n == 0) return set_err(ctx, PN_EINVAL, "variant: bad args");
  KArgs a;
  a.frames = (const uint8_t*)frames_dev;
  a.out = (pn_result*)results_dev;
  a.tbl = ctx->tbl_dev;
  a.mask = ctx->mask;
  a.n_entries = ctx->n_entries;
  a.max_conn = ctx->max_conn;
  a.offs = nullptr;
  a.n = n;
  a.stride = slot_stride;
  a.ipa_off = (frame_off + 14) & ~15u;
  a.avail = slot_stride - frame_off;
  a.offs = nullptr;
  a.fpw = frames_per_wave(n); // the product's launch shape
  hipStream_t s = (hipStream_t)stream;
  if ((variant & 1) && !coop_layout(a)) return set_err(ctx, PN_EINVAL, "variant: needs the cooperative layout");
  // Tuning variants of the MIS = 0 (ip at slot+16) kernel, A/B-timed in one process by
  // scripts/variants.py; not part of the public header.  History: profiles/r01_experiments.
  switch (variant) {
    case 0: launch_one<0, 0>(a, s); break;                         // per-lane window
    case 1: launch_one<0, 1>(a, s); break;                         // cooperative window (production here)
    case 2: launch_one<0, 0, kProdAbl, 0, 0>(a, s); break;                // per-lane, default cache policy
    case 3: launch_one<0, 1, kProdAbl, 0, 0>(a, s); break;                // cooperative, default cache policy
    case 4: launch_one<0, 1, kProdAbl, kLoadAux, kStoreAux, 0, 0>(a, s); break; // line-0 window default policy
    case 5: launch_one<0, 1, kProdAbl, kLoadAux, 0>(a, s); break;         // default-policy record stores
    case 6: launch_one<0, 1, kProdAbl, kLoadAux, 0, 0, 0>(a, s); break;   // both
    case 7: launch_one<0, 1, kProdAbl, kLoadAux, 2>(a, s); break;         // nt record stores
    case 8: launch_one<0, 1, kAblGlobalStore | kProdAbl>(a, s); break;        // plain global record store
    case 9: launch_one<0, 1, 0>(a, s); break;                      // 16-B stream descriptors + per-dword tail masks
    case 19: launch_one<0, 1, kAblStore8 | kProdAbl>(a, s); break;            // timing only: 8-B stores
    case 22: launch_one<0, 1, kExactRange>(a, s); break;                         // scalar probe walk (before kCoopProbe)
    case 23: launch_one<0, 1, kProdAbl, kLoadAux, kStoreAux, 0, kLoadAux, 2, 0>(a, s); break;  // 2 groups per WG, burst records
    case 24: launch_one<0, 1, kProdAbl, kLoadAux, kStoreAux, 0, kLoadAux, 4, 0>(a, s); break;  // 4
    case 25: launch_one<0, 1, kProdAbl, kLoadAux, kStoreAux, 0, kLoadAux, 8, 0>(a, s); break;  // 8
    case 26: launch_one<0, 1, kProdAbl, kLoadAux, kStoreAux, 0, kLoadAux, 16, 0>(a, s); break; // 16
    case 27: launch_one<0, 1, kProdAbl, kLoadAux, kStoreAux, 0, kLoadAux, 8, 1>(a, s); break;  // 8 groups, records per group
    case 28: launch_one<0, 1, kProdAbl, kLoadAux, kStoreAux, 0, kLoadAux, 1, 2 << 4>(a, s); break;  // 1 group, +2 KiB LDS
    case 29: launch_one<0, 1, kProdAbl, kLoadAux, kStoreAux, 0, kLoadAux, 1, 6 << 4>(a, s); break;  // 1 group, +6 KiB LDS
    case 30: launch_one<0, 1, kProdAbl, kLoadAux, kStoreAux, 0, kLoadAux, 8, (2 << 4) | 1>(a, s); break;  // 27 + 2 KiB
    case 31: launch_one<0, 1, kProdAbl, kLoadAux, kStoreAux, 0, kLoadAux, 1, 2>(a, s); break;  // 1 group, 3-wave budget
    case 32: launch_one<0, 1, kProdAbl, kLoadAux, kStoreAux, 0, kLoadAux, 1, 4>(a, s); break;  // 1 group, 2-wave budget
    case 33: launch_one<0, 1, kProdAbl, kLoadAux, kStoreAux, 0, kLoadAux, 2, 4>(a, s); break;  // 2 groups burst, 2-wave budget
    case 34: launch_one<0, 1, kProdAbl, kLoadAux, kStoreAux, 0, kLoadAux, 1, 0>(a, s); break;  // no LDS pad: 5 waves/SIMD
    case 35: launch_one<0, 1, kProdAbl, kLoadAux, kStoreAux, 0, kLoadAux, 1, kProdGopt | 8>(a, s); break;  // XCD-contiguous (production)
    case 36: launch_one<0, 1, kProdAbl, kLoadAux, kStoreAux, 0, kLoadAux, 1, 2 << 4>(a, s); break;  // blockIdx order
    case 37: launch_one<0, 1, kProdAbl & ~kSkipEmptyLoads>(a, s); break;  // every stream load issued (before kSkipEmptyLoads;
    // the per-lane EXEC mask, per-batch gate and per-frame pair branch forms measured against it are
    // in the history)
    case 38: launch_one<0, 1, kProdAbl | kGroupProbe>(a, s); break;  // cluster lanes resolved per run position
    case 39: launch_one<0, 1, kProdAbl & ~kGroupProbe>(a, s); break; // one lane per round trip past kAhead
    case 42: launch_one<0, 1, kProdAbl | kLateProbe>(a, s); break;   // walk finished after phase 2
    case 43: launch_one<0, 1, kProdAbl | kAblNoWalk>(a, s); break;   // timing only: home slot decides
    case 45: launch_one<0, 1, kProdAbl | kAblNoWalk | kAblUniformProbe>(a, s); break; // timing only: one line per probe
    case 47: launch_one<0, 1, kProdAbl | kSerialWindow>(a, s); break; // window loads one round trip each (before round 3)
    case 48: launch_one<0, 1, kProdAbl & ~kPipeStream>(a, s); break;  // phase 2 not pipelined (before round 3)
    case 11: launch_one<0, 1, kAblNoProbe | kProdAbl>(a, s); break;           // timing-only ablations from here
    case 12: launch_one<0, 1, kAblNoReduce | kProdAbl>(a, s); break;
    case 14: launch_one<0, 1, kAblNoMask>(a, s); break;
    case 18: launch_one<0, 1, kAblNoStore | kProdAbl>(a, s); break;
    case 49: launch_one<0, 1, kAblSmallStore | kProdAbl>(a, s); break;   // stores into 16 KiB
    case 55: launch_one<0, 1, kAblEarlyStore | kProdAbl>(a, s); break;   // store issued first, none at the end
    case 50: launch_one<0, 1, kProdAbl, kLoadAux, 1>(a, s); break;   // record stores sc0
    case 51: launch_one<0, 1, kProdAbl, kLoadAux, 3>(a, s); break;   // sc0 nt
    case 52: launch_one<0, 1, kProdAbl, kLoadAux, 17>(a, s); break;  // sc0 sc1
    case 53: launch_one<0, 1, kProdAbl, kLoadAux, 18>(a, s); break;  // sc1 nt
    case 54: launch_one<0, 1, kProdAbl, kLoadAux, 19>(a, s); break;  // sc0 sc1 nt
    case 56: launch_one<0, 1, kProdAbl, kLoadAux, kStoreAux, 0, kLoadAux, 2, kProdGopt | kGroupLoopXcd | kOpaqueLane>(a, s); break;
    case 57: launch_one<0, 1, kProdAbl, kLoadAux, kStoreAux, 0, kLoadAux, 4, kProdGopt | kGroupLoopXcd | kOpaqueLane>(a, s); break;
    case 58: launch_one<0, 1, kProdAbl, kLoadAux, kStoreAux, 0, kLoadAux, 2, kProdGopt | kGroupLoopXcd>(a, s); break;
    case 59: launch_one<0, 1, kProdAbl, kLoadAux, kStoreAux, 0, kLoadAux, 8, kProdGopt | kGroupLoopXcd | kOpaqueLane>(a, s); break;
    default: return set_err(ctx, PN_EINVAL, "variant: unknown");
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hip_err(ctx, e, "variant launch");
  pn_internal::note_stream(ctx, s);
  return PN_OK;
}


#endif // PN_TUNING_VARIANTS

// Same-run ceiling for pn_classify (bench.py): the production kernel -- its window loads, stream
// loads, record stores, occupancy and workgroup order -- with the conn-table probe and the stream
// phase's lane reduction ablated.  Timing only: the records are wrong.  frame_off 2 or 18 (the
// MIS = 0 class, the bench's layout), cooperative layout.
int pn_calib_classify_ablated(pn_ctx* ctx, const void* frames_dev, uint32_t slot_stride, uint32_t frame_off, uint32_t n,
                              void* results_dev, void* stream) {
  if (!ctx || !ctx->tbl_dev || !frames_dev || !results_dev || n == 0 || (frame_off + 14) % 16 != 0)
    return set_err(ctx, PN_EINVAL, "pn_calib_classify_ablated: bad arguments");
  KArgs a;
  int rc = strided_args_calib(ctx, frames_dev, slot_stride, frame_off, n, results_dev, a);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  launch_one<0, 1, kProdAbl | kAblNoProbe | kAblNoReduce>(a, s);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hip_err(ctx, e, "pn_calib_classify_ablated launch");
  pn_internal::note_stream(ctx, s);
  return PN_OK;
}

int pn_calib_slot_read(pn_ctx* ctx, const void* src_dev, uint32_t n_slots, uint32_t stride, uint32_t bytes,
                       int store_bytes, void* sink_dev, void* stream) {
  if (!ctx || !src_dev || !sink_dev || (stride & 15) || bytes > stride || bytes > 2048 || n_slots == 0)
    return set_err(ctx, PN_EINVAL, "pn_calib_slot_read: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  const uint32_t waves = (n_slots + kFramesPerWave - 1) / kFramesPerWave;
  const uint8_t* src = (const uint8_t*)src_dev;
  uint32_t* sink = (uint32_t*)sink_dev;
  switch (store_bytes) {
    // 16 B records written per G groups (probe): store_bytes = 16 | G << 8
    case 16 | (4 << 8): hipLaunchKernelGGL((calib_slot_read_grouped_kernel<4>), dim3((waves + 3) / 4), dim3(64), 0, s, src, n_slots, stride, bytes, sink); break;
    case 16 | (16 << 8): hipLaunchKernelGGL((calib_slot_read_grouped_kernel<16>), dim3((waves + 15) / 16), dim3(64), 0, s, src, n_slots, stride, bytes, sink); break;
    case 16 | (1 << 8): hipLaunchKernelGGL((calib_slot_read_grouped_kernel<1>), dim3(waves), dim3(64), 0, s, src, n_slots, stride, bytes, sink); break;
    case 16 | (4 << 8) | (1 << 16): hipLaunchKernelGGL((calib_slot_read_grouped_kernel<4, true>), dim3((waves + 3) / 4), dim3(64), 0, s, src, n_slots, stride, bytes, sink); break;
    case 16 | (16 << 8) | (1 << 16): hipLaunchKernelGGL((calib_slot_read_grouped_kernel<16, true>), dim3((waves + 15) / 16), dim3(64), 0, s, src, n_slots, stride, bytes, sink); break;
    case 16: hipLaunchKernelGGL((calib_slot_read_kernel<16>), dim3(waves), dim3(64), 0, s, src, n_slots, stride, bytes, sink); break;
    case 8: hipLaunchKernelGGL((calib_slot_read_kernel<8>), dim3(waves), dim3(64), 0, s, src, n_slots, stride, bytes, sink); break;
    default: hipLaunchKernelGGL((calib_slot_read_kernel<0>), dim3(waves), dim3(64), 0, s, src, n_slots, stride, bytes, sink);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hip_err(ctx, e, "calib slot launch");
  pn_internal::note_stream(ctx, s);
  return PN_OK;
}


int pn_calib_slot_read_var(pn_ctx* ctx, const void* src_dev, uint32_t n_slots, uint32_t stride, const void* lens_dev,
                           int store_bytes, void* sink_dev, void* stream) {
  if (!ctx || !src_dev || !lens_dev || !sink_dev || (stride & 15) || n_slots == 0 ||
      (store_bytes != 0 && store_bytes != 16))
    return set_err(ctx, PN_EINVAL, "pn_calib_slot_read_var: bad arguments");
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return hip_err(ctx, e, "hipSetDevice");
  hipStream_t s = (hipStream_t)stream;
  const uint32_t waves = (n_slots + kFramesPerWave - 1) / kFramesPerWave;
  const uint8_t* src = (const uint8_t*)src_dev;
  const uint32_t* lens = (const uint32_t*)lens_dev;
  uint32_t* sink = (uint32_t*)sink_dev;
  if (store_bytes == 16)
    hipLaunchKernelGGL((calib_slot_read_var_kernel<16>), dim3(waves), dim3(64), 0, s, src, n_slots, stride, lens, sink);
  else
    hipLaunchKernelGGL((calib_slot_read_var_kernel<0>), dim3(waves), dim3(64), 0, s, src, n_slots, stride, lens, sink);
  e = hipGetLastError();
  if (e != hipSuccess) return hip_err(ctx, e, "calib slot var launch");
  pn_internal::note_stream(ctx, s);
  return PN_OK;
}


// pn_match_streams in either form (stream_match.hpp): 1 cooperative chunks through LDS, 0 one lane
// per frame; 2-4 the cooperative form with nt / sc0 / sc1 loads; 5 its loads alone (a ceiling); 6-8 the id
// stores write-through / nt (7: with nt loads).  A/B by scripts/bench_streams.py.
int pn_match_streams_variant(pn_ctx* ctx, const void* frames, uint32_t slot_stride, uint32_t frame_off, uint32_t n,
                             const pn_stream_filter* filters, uint32_t n_filters, uint32_t* stream_ids, void* stream,
                             int variant) {
  if (n == 0 || variant < 0 || variant > 40) return set_err(ctx, PN_EINVAL, "match variant: bad arguments");
  MatchArgs a;
  int rc = match_args(ctx, frames, slot_stride, frame_off, n, filters, n_filters, stream_ids, a);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  switch (variant) {
    case 1: launch_match<kMatchProd, kMatchLoadAux>(a, frame_off, s); break; // round-3 production
    case 9: launch_match<1>(a, frame_off, s); break;     // cooperative, default-policy loads
    case 2: launch_match<1, 2>(a, frame_off, s); break;  // cooperative, nt loads
    case 3: launch_match<1, 1>(a, frame_off, s); break;  // cooperative, sc0 loads
    case 4: launch_match<1, 16>(a, frame_off, s); break; // cooperative, sc1 loads
    case 5: launch_match<2, kMatchLoadAux>(a, frame_off, s); break;     // timing-only ceiling: the same loads, no compare or store
    case 6: launch_match<1, 0, 16>(a, frame_off, s); break; // ids stored write-through (sc1)
    case 7: launch_match<1, 2, 16>(a, frame_off, s); break; // nt loads + sc1 id stores
    case 8: launch_match<1, 0, 2>(a, frame_off, s); break;  // ids stored nt
    // round 4: wave-ordered tile, mask compare, G groups per wave, W waves per workgroup
    // (match_streams_mask_kernel<.., G, .., OPT, W>); the odd-numbered-after-19 / 15-19 ids: loads + tile only
    case 10: launch_match_mask<1, kMatchLoadAux, 0, 4>(a, frame_off, s); break;
    case 11: launch_match_mask<2, kMatchLoadAux, 0, 4>(a, frame_off, s); break;
    case 12: launch_match_mask<4, kMatchLoadAux, 0, 4>(a, frame_off, s); break;
    case 13: launch_match_mask<1, kMatchLoadAux, 0, 1>(a, frame_off, s); break;
    case 14: launch_match_mask<2, kMatchLoadAux, 0, 1>(a, frame_off, s); break;
    case 15: launch_match_mask<1, kMatchLoadAux, 2, 4>(a, frame_off, s); break;  // timing only: 10's loads + tile
    case 16: launch_match_mask<2, kMatchLoadAux, 2, 4>(a, frame_off, s); break;  // 11's
    case 17: launch_match_mask<4, kMatchLoadAux, 2, 4>(a, frame_off, s); break;  // 12's
    case 18: launch_match_mask<1, kMatchLoadAux, 2, 1>(a, frame_off, s); break;  // 13's
    case 19: launch_match_mask<2, kMatchLoadAux, 2, 1>(a, frame_off, s); break;  // 14's
    case 20: launch_match_mask<4, kMatchLoadAux, 0, 1>(a, frame_off, s); break;
    case 21: launch_match_mask<4, kMatchLoadAux, 2, 1>(a, frame_off, s); break;  // 20's
    case 22: launch_match_mask<4, kMatchLoadAux, 0, 2>(a, frame_off, s); break;
    case 23: launch_match_mask<4, kMatchLoadAux, 2, 2>(a, frame_off, s); break;  // 22's
    case 24: launch_match_mask<8, kMatchLoadAux, 0, 4>(a, frame_off, s); break;
    case 25: launch_match_mask<8, kMatchLoadAux, 2, 4>(a, frame_off, s); break;  // 24's
    case 26: launch_match_mask<8, kMatchLoadAux, 0, 1>(a, frame_off, s); break;
    case 27: launch_match_mask<8, kMatchLoadAux, 2, 1>(a, frame_off, s); break;  // 26's
    case 28: launch_match_mask<2, kMatchLoadAux, 0, 2>(a, frame_off, s); break;
    case 29: launch_match_mask<2, kMatchLoadAux, 2, 2>(a, frame_off, s); break;  // 28's
    case 30: launch_match_mask<1, kMatchLoadAux, 4, 1>(a, frame_off, s); break;  // production + s_setprio 2 after the loads
    case 31: launch_match_mask<1, kMatchLoadAux, 8, 1>(a, frame_off, s); break;  // production, needed chunks only to the tile
    case 32: launch_match_mask<1, kMatchLoadAux, 12, 1>(a, frame_off, s); break; // both
    case 33: launch_match_mask<1, kMatchLoadAux, 16, 1>(a, frame_off, s); break; // production, and-compare form
    case 34: launch_match_mask<1, kMatchLoadAux, 32, 1>(a, frame_off, s); break; // timing only: no compare
    case 35: launch_match_mask<1, kMatchLoadAux, 64, 1>(a, frame_off, s); break; // timing only: no id store
    case 36: launch_match_mask<1, kMatchLoadAux, 128, 1>(a, frame_off, s); break; // production, nt id stores
    case 37: launch_match_mask<1, kMatchLoadAux, 256, 1>(a, frame_off, s); break; // production, masks loaded first
    case 38: launch_match_mask<1, kMatchLoadAux, 512, 1>(a, frame_off, s); break; // timing only: stores into 4 KiB
    case 39: launch_match_mask<1, kMatchLoadAux, 1024, 1>(a, frame_off, s); break; // no tile: quad DPP exchange
    case 40: launch_match_mask<1, kMatchLoadAux, 1024 | 2, 1>(a, frame_off, s); break; // 39's loads + exchange alone
    default: launch_match<0>(a, frame_off, s);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hip_err(ctx, e, "match variant launch");
  pn_internal::note_stream(ctx, s);
  return PN_OK;
}

int pn_test_spin_wait(const uint32_t* go_host, uint32_t* done_host, uint32_t max_ms, void* stream) {
  if (!go_host || !done_host || max_ms == 0 || max_ms > 10000)
    return set_err(nullptr, PN_EINVAL, "pn_test_spin_wait: go/done must be set, max_ms in [1, 10000]");
  int dev = 0, khz = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev);
  if (e != hipSuccess || khz <= 0) return hip_err(nullptr, e, "wall clock rate");
  hipLaunchKernelGGL(spin_wait_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, go_host, done_host,
                     (uint64_t)khz * max_ms);
  e = hipGetLastError();
  return e == hipSuccess ? PN_OK : hip_err(nullptr, e, "spin_wait launch");
}

int pn_test_doorbell_echo(const uint32_t* bell_host, uint32_t* echo_host, uint32_t max_idle_ms, int once, int sleep,
                          void* stream) {
  if (!bell_host || !echo_host || max_idle_ms == 0 || max_idle_ms > 10000)
    return set_err(nullptr, PN_EINVAL, "pn_test_doorbell_echo: bell/echo must be set, max_idle_ms in [1, 10000]");
  int dev = 0, khz = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev);
  if (e != hipSuccess || khz <= 0) return hip_err(nullptr, e, "wall clock rate");
  hipLaunchKernelGGL(doorbell_echo_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, bell_host, echo_host,
                     (uint64_t)khz * max_idle_ms, (uint32_t)(once != 0), (uint32_t)(sleep != 0));
  e = hipGetLastError();
  return e == hipSuccess ? PN_OK : hip_err(nullptr, e, "doorbell_echo launch");
}

int pn_test_doorbell_echo_pipe(const uint32_t* bell_host, uint32_t* echo_host, uint32_t max_idle_ms, int depth,
                               uint32_t gap, void* stream) {
  if (!bell_host || !echo_host || max_idle_ms == 0 || max_idle_ms > 10000 || gap > 64 ||
      (depth != 1 && depth != 2 && depth != 4 && depth != 8))
    return set_err(nullptr, PN_EINVAL, "pn_test_doorbell_echo_pipe: bell/echo, max_idle_ms in [1, 10000], depth 1/2/4/8, gap <= 64");
  int dev = 0, khz = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev);
  if (e != hipSuccess || khz <= 0) return hip_err(nullptr, e, "wall clock rate");
  const uint64_t t = (uint64_t)khz * max_idle_ms;
  const hipStream_t s = (hipStream_t)stream;
  switch (depth) {
    case 1: hipLaunchKernelGGL(doorbell_echo_pipe_kernel<1>, dim3(1), dim3(64), 0, s, bell_host, echo_host, t, gap); break;
    case 2: hipLaunchKernelGGL(doorbell_echo_pipe_kernel<2>, dim3(1), dim3(64), 0, s, bell_host, echo_host, t, gap); break;
    case 4: hipLaunchKernelGGL(doorbell_echo_pipe_kernel<4>, dim3(1), dim3(64), 0, s, bell_host, echo_host, t, gap); break;
    default: hipLaunchKernelGGL(doorbell_echo_pipe_kernel<8>, dim3(1), dim3(64), 0, s, bell_host, echo_host, t, gap);
  }
  e = hipGetLastError();
  return e == hipSuccess ? PN_OK : hip_err(nullptr, e, "doorbell_echo_pipe launch");
}

int pn_calib_stream_read(pn_ctx* ctx, const void* src_dev, uint64_t bytes, void* sink_dev, void* stream) {
  if (!ctx || !src_dev || !sink_dev || (bytes & 15) || ((uintptr_t)src_dev & 15))
    return set_err(ctx, PN_EINVAL, "pn_calib_stream_read: bad arguments");
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return hip_err(ctx, e, "hipSetDevice");
  hipLaunchKernelGGL(calib_stream_read_kernel, dim3(2048), dim3(256), 0, (hipStream_t)stream, (const u32x4*)src_dev,
                     bytes / 16, (uint32_t*)sink_dev);
  e = hipGetLastError();
  if (e != hipSuccess) return hip_err(ctx, e, "calib launch");
  pn_internal::note_stream(ctx, (hipStream_t)stream);
  return PN_OK;
}

} // extern "C"
