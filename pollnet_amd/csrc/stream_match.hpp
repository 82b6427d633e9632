// stream_match.hpp — the TcpStream filter kernel (device code + launch helper), shared by the
// product library (stream_kernel.hip: pn_match_streams) and the tuning library (rx_tuning.hip:
// the A/B variant).  Internal linkage; one including translation unit per library.
#pragma once
// TcpStream's packet filter for a whole batch, many streams at once (SURVEY §8(f)
// rank 3).  Reference, per frame and per stream (TcpStream.h:39-52):
//   etherType == 0x0008 (0x0800 read little-endian) && ip.protocol == 6 &&
//   (filter_src_ip == 0 || == ip.ipSrc) && (filter_dst_ip == 0 || == ip.ipDst) &&
//   (filter_src_port == 0 || == tcp.portSrc) && (filter_dst_port == 0 || == tcp.portDst)
// with the IP header assumed 20 bytes (TcpHeaderPos = 14 + 20, TcpStream.h:213-214).
//
// Each frame's header bytes (ethertype .. TCP ports) are read once -- one 64-B segment of
// its slot, a gather at the slot stride -- and the frame's lane compares them against every
// filter in the kernel-argument segment (scalar loads, wave-uniform) and writes the index of
// the first stream the frame belongs to.  V = 1 (production): 4 lanes per frame load its
// segment's 16-B chunks with one instruction for 16 frames (one 64-B request per frame per
// instruction, only the chunks the fields touch) into an LDS tile each frame's lane reads back.
// V = 0 (tuning): each lane loads its own frame's 4 chunks, 4 instructions each touching 64
// slots.
#include <hip/hip_runtime.h>

#include "../../include/pollnet_amd.h"
#include "device_common.hpp"
#include "pn_internal.hpp"

namespace {

using namespace pn_dev;
using pn_internal::hip_err;
using pn_internal::set_err;

// A filter as values and care-masks: frame passes it iff ((field ^ v) & m) == 0 for its three words
// (a zero filter field is a wildcard: mask 0).  ports = src_port | dst_port << 16, both as stored.
struct MatchMask {
  uint32_t vs, vd, vp; // src ip, dst ip, ports
  uint32_t ms, md, mp;
};
constexpr uint32_t kMaskBlock = 8; // filters compared per block of kernel-argument loads

struct MatchArgs {
  const uint8_t* frames;
  uint32_t* out;
  uint32_t n;
  uint32_t stride;
  uint32_t ipa_off; // (frame_off + 14) & ~15
  uint32_t n_filters;
  uint32_t n_blocks; // ceil(n_filters / kMaskBlock): m[] is padded to whole blocks
  pn_stream_filter f[PN_MAX_STREAM_FILTERS];
  MatchMask m[PN_MAX_STREAM_FILTERS];
};

// MIS = (frame_off + 14) % 16: the IP header's offset in its 16-B chunk.  The window
// is the chunk before it (ethertype when MIS < 2) and the 3 chunks from it.
constexpr int kPre = 16; // window starts one chunk before the IP header's chunk
// whether window chunk c holds any byte of ethertype .. the TCP ports ([IP - 2, IP + 24))
template <int MIS>
__device__ __host__ constexpr bool chunk_needed(int c) {
  return 16 * c < kPre + MIS + 24 && 16 * c + 16 > kPre + MIS - 2;
}

// LAUX: the cooperative loads' cache policy (tuning: whether L2 then fetches 64-B sectors, not lines).
// SAUX >= 0 (tuning): the ids through a buffer store with that cache policy instead of a plain store.
template <int MIS, int V, int LAUX = 0, int SAUX = -1>
__global__ __launch_bounds__(256) void match_streams_kernel(MatchArgs a) {
  const uint32_t f = blockIdx.x * 256 + threadIdx.x;
  Win<16> h;
  if constexpr (V >= 1) {
    // wave w of the workgroup: frames f0 .. f0 + 63; instruction i: lane l loads chunk l & 3 of
    // frame f0 + 16 i + (l >> 2)
    __shared__ u32x4 tile[256 * 4];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // wave-uniform (readfirstlane): a descriptor built from a per-lane value is a waterfall loop
    const uint32_t f0 = __builtin_amdgcn_readfirstlane(blockIdx.x * 256 + w * 64);
    u32x4* wt = tile + w * 256;
    const uint32_t c = lane & 3;
    const uint32_t n_here = f0 < a.n ? min(64u, a.n - f0) : 0u;
    const uint32_t nrec = __builtin_amdgcn_readfirstlane(n_here ? (n_here - 1) * a.stride + 64 : 0u); // kept scalar
    const __amdgpu_buffer_rsrc_t rs = frame_rsrc(a.frames + (uint64_t)f0 * a.stride + a.ipa_off - kPre, nrec);
    // all 4 loads in flight before the LDS writes: a chunk that is not needed gets an offset past the
    // range (zeros, no fetch) instead of a branch around its load (which serialized the loads)
    const bool need = (c == 0 && chunk_needed<MIS>(0)) || (c == 1 && chunk_needed<MIS>(1)) ||
                      (c == 2 && chunk_needed<MIS>(2)) || (c == 3 && chunk_needed<MIS>(3));
    u32x4 v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t r = 16 * i + (lane >> 2);
      const uint32_t off = (r * a.stride + 16 * c) | (need ? 0u : kNoFetch); // past n or not needed: zeros
      v[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, LAUX);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t r = 16 * i + (lane >> 2);
      wt[r * 4 + (c ^ (r & 3))] = v[i];
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const u32x4 v = wt[lane * 4 + (q ^ (lane & 3))];
      h.d[4 * q + 0] = v.x;
      h.d[4 * q + 1] = v.y;
      h.d[4 * q + 2] = v.z;
      h.d[4 * q + 3] = v.w;
    }
    if (f >= a.n) return;
  } else {
    // one descriptor per wave (scalar), each lane at its own slot's offset
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t f0 = __builtin_amdgcn_readfirstlane(blockIdx.x * 256 + (threadIdx.x >> 6) * 64);
    const uint32_t n_here = f0 < a.n ? min(64u, a.n - f0) : 0u;
    const uint32_t nrec = __builtin_amdgcn_readfirstlane(n_here ? (n_here - 1) * a.stride + 64 : 0u);
    if (f >= a.n) return;
    const __amdgpu_buffer_rsrc_t rs = frame_rsrc(a.frames + (uint64_t)f0 * a.stride + a.ipa_off - kPre, nrec);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * a.stride + 16 * c, 0, 0);
      h.d[4 * c + 0] = v.x;
      h.d[4 * c + 1] = v.y;
      h.d[4 * c + 2] = v.z;
      h.d[4 * c + 3] = v.w;
    }
  }
  if constexpr (V == 2) { // timing only: the loads and the LDS round trip, no compare, (almost) no store
    uint32_t x = 0;
#pragma unroll
    for (int q = 0; q < 12; ++q) x ^= h.d[q];
    if (x == 0x9E3779B9u) a.out[f] = x;
    return;
  }
  constexpr int IP = kPre + MIS;
  const uint32_t ether_type = h.template u16<IP - 2>(); // as stored: 0x0008 for IPv4
  const uint32_t proto = h.template b8<IP + 9>();
  const uint32_t src_ip = h.template u32<IP + 12>(), dst_ip = h.template u32<IP + 16>();
  const uint32_t src_port = h.template u16<IP + 20>(), dst_port = h.template u16<IP + 22>();
  uint32_t id = PN_NO_STREAM;
  if (ether_type == 0x0008 && proto == 6) {
    for (uint32_t k = 0; k < a.n_filters; ++k) {
      const pn_stream_filter& q = a.f[k];
      if ((q.src_ip == 0 || q.src_ip == src_ip) && (q.dst_ip == 0 || q.dst_ip == dst_ip) &&
          (q.src_port == 0 || q.src_port == src_port) && (q.dst_port == 0 || q.dst_port == dst_port)) {
        id = k;
        break;
      }
    }
  }
  if constexpr (SAUX >= 0) {
    const __amdgpu_buffer_rsrc_t ro = frame_rsrc((const uint8_t*)(a.out + blockIdx.x * 256), 256 * 4); // scalar
    __builtin_amdgcn_raw_buffer_store_b32(id, ro, (f & 255u) * 4, 0, SAUX);
  } else {
    a.out[f] = id;
  }
}

// lane j of each quad's value, to all four lanes of the quad (DPP quad_perm [j, j, j, j]); j folds to a constant
__device__ __forceinline__ uint32_t quad_bcast(uint32_t v, int j) {
  switch (j) {
    case 0: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x00, 0xF, 0xF, false);
    case 1: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x55, 0xF, 0xF, false);
    case 2: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xAA, 0xF, 0xF, false);
    default: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xFF, 0xF, 0xF, false);
  }
}

// Round 4 form: the same cooperative 64-B loads (4 lanes per frame, one line request per frame), then
//   - each wave orders its own LDS tile round trip by itself: the DS instructions of one wave execute
//     in order, so a wave reads its tile right after writing it, without waiting at a workgroup barrier
//     for the other waves' loads;
//   - G groups of 64 frames per wave, all G x 4 loads in flight before the first group is compared;
//   - the filters as value / care-mask words (MatchMask): per filter 3 xor, 1 and, 2 and-or, 1 compare and
//     1 select per frame, no branch, last to first so the first passing filter wins.
// WPW waves per workgroup, each with its own 4-KiB tile.
// OPT & 2 (tuning): the loads and the tile round trip alone, no compare or store (its ceiling).
// OPT & 4 (tuning): raise the wave's priority once its loads are in (s_setprio 2), so the compare and store
// finish ahead of waves still issuing loads.  OPT & 8 (tuning): only the needed chunks written to the tile.
// OPT & 16: the filter test as (field & mask) == value per word instead of xor/and/or.
// OPT & 32 / 64 (tuning, timing only): no filter compare / no id store.  OPT & 128 (tuning): nt id stores.
// OPT & 256: the last filter block's masks loaded right after the frame loads, not at the compare (below).
// OPT & 512 (timing only): the id stores all land in the first 4 KiB of the output (store issue without the
// write volume).  OPT & 1024 (tuning): no LDS tile, the header words exchanged within each quad by DPP.
template <int MIS, int G, int LAUX, int OPT = 0, int WPW = 4>
__global__ __launch_bounds__(64 * WPW) void match_streams_mask_kernel(MatchArgs a) {
  constexpr uint32_t kWaveFrames = 64 * G;
  __shared__ u32x4 tile[WPW * 256];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t w = WPW == 1 ? 0u : __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t f0 = __builtin_amdgcn_readfirstlane((blockIdx.x * WPW + w) * kWaveFrames);
  if (f0 >= a.n) return; // wave-uniform, and no workgroup barrier below
  const uint32_t n_here = min(kWaveFrames, a.n - f0);
  const __amdgpu_buffer_rsrc_t rs =
      frame_rsrc(a.frames + (uint64_t)f0 * a.stride + a.ipa_off - kPre, (n_here - 1) * a.stride + 64);
  u32x4* wt = tile + w * 256;
  const uint32_t c = lane & 3;
  const bool need = (c == 0 && chunk_needed<MIS>(0)) || (c == 1 && chunk_needed<MIS>(1)) ||
                    (c == 2 && chunk_needed<MIS>(2)) || (c == 3 && chunk_needed<MIS>(3));
  const int b_last = (int)a.n_blocks - 1;
  const uint32_t last = a.n_filters - 1;
  MatchMask q0[kMaskBlock];
  // instruction (g, i): lane l loads chunk l & 3 of frame 64 g + 16 i + (l >> 2); rows past n_here
  // read zeros (the descriptor's range), unneeded chunks fetch nothing
  u32x4 v[G][4];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t r = 64 * g + 16 * i + (lane >> 2);
      v[g][i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (r * a.stride + 16 * c) | (need ? 0u : kNoFetch), 0, LAUX);
    }
  // OPT & 256: the last filter block's kernel-argument loads go out right after the frame loads and are in
  // registers while the frames are still on their way (a.m always holds kMaskBlock entries, so block 0 is
  // read even without filters; it is used only when n_blocks > 0).  The empty asm statements use the values
  // here, so the compiler cannot sink the loads to the compare, after the frames' wait.
  if constexpr ((OPT & 256) != 0) {
    __builtin_amdgcn_sched_barrier(0);
    const int b0 = b_last > 0 ? b_last : 0;
    asm volatile("" : : "s"(last));
#pragma unroll
    for (int j = 0; j < (int)kMaskBlock; ++j) {
      q0[j] = a.m[b0 * kMaskBlock + j];
      asm volatile("" : : "s"(q0[j].vs), "s"(q0[j].vd), "s"(q0[j].vp), "s"(q0[j].ms), "s"(q0[j].md), "s"(q0[j].mp));
    }
  }
#pragma unroll
  for (int g = 0; g < G; ++g) {
    Win<16> h;
    uint32_t f;
    if constexpr ((OPT & 1024) != 0) {
      // tuning: no tile.  Lane 4q + c takes frame 16c + q; each header word k of it is in lane 4q + k / 4 of its
      // quad, component k % 4 of load c: four quad broadcasts (DPP) of that component, one per load, and the
      // lane keeps the one of its own load
#pragma unroll
      for (int k = 0; k < 16; ++k) h.d[k] = 0;
      constexpr int kLo = (kPre + MIS - 2) / 4, kHi = (kPre + MIS + 23) / 4;
#pragma unroll
      for (int k = kLo; k <= kHi; ++k) {
        uint32_t x[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const u32x4 vv = v[g][i];
          const uint32_t comp = (k & 3) == 0 ? vv.x : (k & 3) == 1 ? vv.y : (k & 3) == 2 ? vv.z : vv.w;
          x[i] = quad_bcast(comp, k >> 2);
        }
        h.d[k] = c == 0 ? x[0] : c == 1 ? x[1] : c == 2 ? x[2] : x[3];
      }
      f = f0 + 64 * g + 16 * c + (lane >> 2);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t r = 16 * i + (lane >> 2);
        if (!(OPT & 8) || need) wt[r * 4 + (c ^ (r & 3))] = v[g][i];
      }
      // other lanes of this wave read what these lanes wrote: order the tile writes before the reads
      // for the compiler and the memory model (the tile is the wave's own, so a wavefront-scope
      // release/acquire pair around a wave barrier is the whole synchronisation)
      wave_lds_sync();
      if constexpr ((OPT & 4) != 0) {
        if (g == 0) __builtin_amdgcn_s_setprio(2);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const u32x4 x = wt[lane * 4 + (q ^ (lane & 3))];
        h.d[4 * q + 0] = x.x;
        h.d[4 * q + 1] = x.y;
        h.d[4 * q + 2] = x.z;
        h.d[4 * q + 3] = x.w;
      }
      if constexpr (G > 1) wave_lds_sync(); // group g's reads before group g + 1's writes
      f = f0 + 64 * g + lane;
    }
    if constexpr (OPT & 2) { // timing only
      uint32_t x = 0;
#pragma unroll
      for (int q = 0; q < 12; ++q) x ^= h.d[q];
      if (x == 0x9E3779B9u && f < a.n) a.out[f] = x;
      continue;
    }
    constexpr int IP = kPre + MIS;
    const uint32_t sip = h.template u32<IP + 12>(), dip = h.template u32<IP + 16>(), ports = h.template u32<IP + 20>();
    uint32_t id = PN_NO_STREAM;
    // blocks of kMaskBlock filters, last block first: each block's scalar loads go out together
    // (padding entries repeat the last filter; their index clamps to it, so they change nothing)
    if constexpr ((OPT & 32) != 0) id = sip ^ dip ^ ports; // timing only: no compare
    for (int b = (OPT & 32) ? -1 : b_last; b >= 0; --b) {
      MatchMask q[kMaskBlock];
#pragma unroll
      for (int j = 0; j < (int)kMaskBlock; ++j) q[j] = ((OPT & 256) != 0 && b == b_last) ? q0[j] : a.m[b * kMaskBlock + j];
#pragma unroll
      for (int j = kMaskBlock - 1; j >= 0; --j) {
        bool pass;
        if constexpr ((OPT & 16) != 0) { // and-compare form: 3 ands, 3 compares (a wildcard's value is 0 = its mask)
          pass = (sip & q[j].ms) == q[j].vs && (dip & q[j].md) == q[j].vd && (ports & q[j].mp) == q[j].vp;
        } else {
          pass = (((sip ^ q[j].vs) & q[j].ms) | ((dip ^ q[j].vd) & q[j].md) | ((ports ^ q[j].vp) & q[j].mp)) == 0;
        }
        id = pass ? min((uint32_t)(b * kMaskBlock + j), last) : id;
      }
    }
    if (h.template u16<IP - 2>() != 0x0008 || h.template b8<IP + 9>() != 6) id = PN_NO_STREAM;
    if constexpr ((OPT & 64) != 0) { // timing only: (almost) no id store
      if (id == 0x9E3779B9u && f < a.n) a.out[f] = id;
      continue;
    }
    if constexpr ((OPT & 512) != 0) { // timing only: every store, into 4 KiB of lines (no HBM write volume)
      if (f < a.n) a.out[(blockIdx.x & 15) * 64 + lane] = id;
      continue;
    }
    if constexpr ((OPT & 128) != 0) { // tuning: non-temporal id store
      if (f < a.n) __builtin_nontemporal_store(id, a.out + f);
    } else {
      if (f < a.n) a.out[f] = id;
    }
  }
}

// Production (round 4): one group of 64 frames per wave, one wave per workgroup (a 4-KiB tile each).
// Interleaved A/B, 9 rounds, 1 Mi resident slots x 4 batches, 8 filters (profiles/r04/match_streams/):
// 0.0269 -> 0.0219 ms on C2 and 0.0275 -> 0.0220 on C3 against the round-3 kernel (tuning variant 1),
// at 0.94 of its own loads + tile round trip (variant 18); more groups per wave (2, 4, 8) or more
// waves per workgroup (2, 4) measured 2-10 % slower.
constexpr int kMatchG = 1;
constexpr int kMatchWPW = 1;

template <int G, int LAUX, int OPT = 0, int WPW = 4>
void launch_match_mask(const MatchArgs& a, uint32_t frame_off, hipStream_t s) {
  constexpr uint32_t per_wg = 64 * G * WPW;
  const dim3 grid((a.n + per_wg - 1) / per_wg), block(64 * WPW);
  switch ((frame_off + 14) & 15) {
    case 0: hipLaunchKernelGGL((match_streams_mask_kernel<0, G, LAUX, OPT, WPW>), grid, block, 0, s, a); break;
    case 2: hipLaunchKernelGGL((match_streams_mask_kernel<2, G, LAUX, OPT, WPW>), grid, block, 0, s, a); break;
    case 4: hipLaunchKernelGGL((match_streams_mask_kernel<4, G, LAUX, OPT, WPW>), grid, block, 0, s, a); break;
    case 6: hipLaunchKernelGGL((match_streams_mask_kernel<6, G, LAUX, OPT, WPW>), grid, block, 0, s, a); break;
    case 8: hipLaunchKernelGGL((match_streams_mask_kernel<8, G, LAUX, OPT, WPW>), grid, block, 0, s, a); break;
    case 10: hipLaunchKernelGGL((match_streams_mask_kernel<10, G, LAUX, OPT, WPW>), grid, block, 0, s, a); break;
    case 12: hipLaunchKernelGGL((match_streams_mask_kernel<12, G, LAUX, OPT, WPW>), grid, block, 0, s, a); break;
    default: hipLaunchKernelGGL((match_streams_mask_kernel<14, G, LAUX, OPT, WPW>), grid, block, 0, s, a); break;
  }
}

// The round-3 production form, now tuning variant 1 (A/B: scripts/bench_streams.py, match_ab.py):
// cooperative loads, non-temporal (glc slc = 2).  Measured 5-7 % faster than the default policy on
// C2 and C3 (profiles/r03/match_streams_policies.json); the slot lines are read once here.
constexpr int kMatchProd = 1;
constexpr int kMatchLoadAux = 2;

template <int V, int LAUX = 0, int SAUX = -1>
void launch_match(const MatchArgs& a, uint32_t frame_off, hipStream_t s) {
  const dim3 grid((a.n + 255) / 256), block(256);
  switch ((frame_off + 14) & 15) {
    case 0: hipLaunchKernelGGL((match_streams_kernel<0, V, LAUX, SAUX>), grid, block, 0, s, a); break;
    case 2: hipLaunchKernelGGL((match_streams_kernel<2, V, LAUX, SAUX>), grid, block, 0, s, a); break;
    case 4: hipLaunchKernelGGL((match_streams_kernel<4, V, LAUX, SAUX>), grid, block, 0, s, a); break;
    case 6: hipLaunchKernelGGL((match_streams_kernel<6, V, LAUX, SAUX>), grid, block, 0, s, a); break;
    case 8: hipLaunchKernelGGL((match_streams_kernel<8, V, LAUX, SAUX>), grid, block, 0, s, a); break;
    case 10: hipLaunchKernelGGL((match_streams_kernel<10, V, LAUX, SAUX>), grid, block, 0, s, a); break;
    case 12: hipLaunchKernelGGL((match_streams_kernel<12, V, LAUX, SAUX>), grid, block, 0, s, a); break;
    default: hipLaunchKernelGGL((match_streams_kernel<14, V, LAUX, SAUX>), grid, block, 0, s, a); break;
  }
}

// Argument checks and kernel arguments of pn_match_streams.
inline int match_args(pn_ctx* ctx, const void* frames, uint32_t slot_stride, uint32_t frame_off, uint32_t n,
                      const pn_stream_filter* filters, uint32_t n_filters, uint32_t* stream_ids, MatchArgs& a) {
  if (!ctx) return set_err(nullptr, PN_EINVAL, "pn_match_streams: ctx is NULL");
  if (!frames || !stream_ids || (n_filters && !filters)) return set_err(ctx, PN_EINVAL, "pn_match_streams: NULL buffer");
  if (n_filters > PN_MAX_STREAM_FILTERS)
    return set_err(ctx, PN_EINVAL, "pn_match_streams: at most PN_MAX_STREAM_FILTERS filters");
  if (((uintptr_t)frames & 15) || ((uintptr_t)stream_ids & 3))
    return set_err(ctx, PN_EINVAL, "pn_match_streams: frames must be 16-byte, ids 4-byte aligned");
  if ((slot_stride & 15) || slot_stride > 65536 || (frame_off & 1) || frame_off < 2 || slot_stride < frame_off + 96)
    return set_err(ctx, PN_EINVAL, "pn_match_streams: slot_stride/frame_off violate the layout contract");
  a.frames = (const uint8_t*)frames;
  a.out = stream_ids;
  a.n = n;
  a.stride = slot_stride;
  a.ipa_off = (frame_off + 14) & ~15u;
  a.n_filters = n_filters;
  for (uint32_t k = 0; k < n_filters; ++k) { // host memory: copied into the kernel arguments
    const pn_stream_filter& q = filters[k];
    a.f[k] = q;
    a.m[k] = {q.src_ip, q.dst_ip, (uint32_t)q.src_port | (uint32_t)q.dst_port << 16, q.src_ip ? ~0u : 0u,
              q.dst_ip ? ~0u : 0u, (q.src_port ? 0xffffu : 0u) | (q.dst_port ? 0xffff0000u : 0u)};
  }
  a.n_blocks = (n_filters + kMaskBlock - 1) / kMaskBlock;
  for (uint32_t k = n_filters; k < a.n_blocks * kMaskBlock; ++k) a.m[k] = a.m[n_filters - 1]; // the same verdict
  return PN_OK;
}

} // namespace

