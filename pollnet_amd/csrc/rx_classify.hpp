// rx_classify.hpp — the RX classify kernel (device code + launch helpers), shared by the
// product library (rx_kernel.hip: the production instantiations behind pn_classify /
// pn_classify_indexed) and the tuning library (rx_tuning.hip: A/B variants, ceilings).
// Included by exactly one translation unit per library; everything is internal linkage.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <string>

#include "../../include/pollnet_amd.h"
#include "device_common.hpp"
#include "frame_pass.hpp"
#include "pn_internal.hpp"

// The MI355X (gfx950) receive-path per-frame transform: Ethernet/IPv4/TCP header
// parse, IP + TCP one's-complement verification, conn-table probe and
// payload off/len for a batch of RX-ring slots resident in HBM.
//
// Reference path (per frame, scalar): efvitcp/Core.h:503-526 (pointers, key,
// findConnEntry, TIME_WAIT test), Core.h:448-472 (checksum, debug build),
// Core.h:89-138 (CSum), TcpConn.h:469-473 (payload arithmetic).
//
// Execution model (one wavefront = 64 frames, 64-thread workgroups, no
// inter-wave communication):
//  phase 1  lane f owns frame f: gets a 112-B header window (either 8 lanes per
//           slot load its first 128-B line coalesced into a swizzled LDS tile, or
//           each lane loads its own window when the layout is not line-aligned),
//           decodes fields at compile-time offsets (kernel specialised on
//           (frame_off+14)%16), computes the 20-byte IP sum, the sum of the
//           frame's words inside the window, connHashKey and the ordered probe
//           of the (L2-resident) conn table.
//  phase 2  the wave streams the rest of each frame's summed region
//           [ip, ip+20+tcp_len(+pad)) from the window end on, with
//           1 KiB buffer_load_dwordx4 instructions (64 lanes x 16 B), summing
//           u16 halves with v_dot2_u32_u16 (exact integer sums, no folding),
//           8 frames per batch, reduced across lanes with permlane32/16 swaps
//           and DPP (one value per lane per batch) and parked on the frame's lane.
//  phase 3  lane f subtracts the IP-header words, adds the pseudo-header and
//           folds exactly like CSum::fold; one coalesced 16-B record per lane.
// HBM bytes per frame = the frame itself (+16 B result): the kernel is bound by
// HBM bandwidth (no MFMA: there is no contraction).  It runs within ~1 % of a
// no-arithmetic kernel with the same reads and record writes;
// the remaining gap to pure streaming is the DRAM cost of interleaving the
// record writes with the frame reads.
namespace {

using namespace pn_dev;
using pn_internal::g_err;
using pn_internal::hip_err;
using pn_internal::set_err;

struct KArgs {
  const uint8_t* frames;
  pn_result* out;
  const pn_conn_entry* tbl;
  uint64_t mask;
  uint32_t n_entries;
  uint32_t max_conn;
  uint32_t n;
  uint32_t stride;
  uint32_t ipa_off; // (frame_off + 14) & ~15: 16-B aligned start of the header window
  uint32_t avail;   // stride - frame_off: bytes from the Ethernet header to the slot end
  const uint64_t* offs; // indexed layout: frame i's Ethernet header at frames + offs[i] (nullptr: strided)
  uint32_t fpw = kFramesPerWave; // frames per wave (8..64): small batches spread over more waves (latency)
  uint32_t* sig_count = nullptr;  // kSignalDone: workgroups finished (device memory, 0 before the launch)
  uint32_t* sig_flag = nullptr;   // kSignalDone: host-visible word the last workgroup sets to sig_token
  uint32_t sig_token = 0;
};

// The resident service's arguments (kChainAux): KArgs and where each frame's chain entries go.  A classify
// instantiated with kChainAux is only ever given one of these (the production launches keep KArgs as it is, so their
// kernel arguments and code are unchanged).
struct KArgsAux : KArgs {
  u32x4* aux = nullptr; // two 16-B entries per frame (device scratch), or nullptr
};

// Conn-table lookup carried from the home-slot load to its resolution.
struct Probe {
  uint64_t key;
  uint32_t e;
  uint64_t k;   // key of entry e (PN_EMPTY_KEY when not loaded)
  uint32_t cid; // conn_id of entry e
};

// Per-frame state the header lane keeps from phase 1 to phase 3.
struct FrameState {
  uint32_t flags, ihl, tot_len, src_ip, dst_ip, seq_raw, doff, tflags, s_ip20, s_opt, tcp_len, conn_id;
  uint32_t t_all; // exact u16-word sum of [ip, ip+20+tcp_len(+pad)) accumulated so far
  int end_rel;    // summed extent relative to the window start (even), | 1 when tcp_len is odd; 0 = nothing to stream
  uint32_t pad;   // odd tcp_len: the byte after the segment (kPadUnknown until phase 2 captured it)
  bool trunc;
  Probe probe; // kLateProbe: the issued probe, finished after phase 2
};

// connHashKey (Core.h:167-172) and the load of the home slot `key & tbl_mask` (Core.h:558-559).
template <int ABL>
__device__ __forceinline__ Probe probe_issue(uint32_t src_ip, uint32_t src_port, bool live, const KArgs& a) {
  Probe p;
  const uint32_t ip_h = __builtin_bswap32(src_ip);
  const uint32_t port_h = bswap16(src_port);
  p.key = ((uint64_t)ip_h << 15) | (port_h & 0x7fff) | ((uint64_t)(port_h & 0x8000) << 32);
  p.e = (uint32_t)(p.key & a.mask);
  p.k = PN_EMPTY_KEY;
  p.cid = 0;
  if (live && p.e < a.n_entries) { // the home slot: almost every lookup ends here
    uint32_t eh = p.e;
    if constexpr (ABL & kAblUniformProbe) eh = __builtin_amdgcn_readfirstlane(eh); // timing only
    const u32x4 ent = *reinterpret_cast<const u32x4*>(a.tbl + eh);
    p.k = ((uint64_t)ent.y << 32) | ent.x;
    p.cid = ent.z;
  }
  return p;
}

// The rest of findConnEntry's ordered walk (Core.h:560-561) and the conn / TIME_WAIT / miss
// verdict (Core.h:510).  Every lane of the wave must call it (the cooperative walk ballots).
template <int ABL>
__device__ __forceinline__ void probe_finish(const Probe& p, bool live, const KArgs& a, uint32_t& conn_id, uint32_t& flags) {
  const uint64_t key = p.key;
  uint32_t e = p.e;
  uint64_t k = p.k;
  uint32_t cid = p.cid;
  if constexpr (ABL & kAblNoWalk) {
    // timing only: the home slot decides
  } else if constexpr (ABL & kCoopProbe) {
    // Lanes whose run continues past the home slot are served one at a time by the whole
    // wave (all 64 lanes reach here): 64 consecutive entries per round trip, the first with
    // key >= the lane's key (or the array end) found by a ballot -- the entry the scalar
    // walk stops at.
    const uint32_t lane = threadIdx.x;
    bool srch = live && e < a.n_entries && k < key;
    if (__ballot(srch) != 0) {
      // short runs (the common case past the home slot): every searching lane fetches its
      // next kAhead entries at once -- one round trip for all of them, in parallel
      constexpr int kAhead = 2;
      u32x4 nx[kAhead];
#pragma unroll
      for (int j = 0; j < kAhead; ++j) {
        nx[j] = u32x4{0u, 0u, 0u, 0u};
        if (srch && e + 1 + j < a.n_entries) nx[j] = *reinterpret_cast<const u32x4*>(a.tbl + e + 1 + j);
      }
      uint32_t step = 0, cid2 = 0;
      uint64_t k2 = 0;
#pragma unroll
      for (int j = kAhead - 1; j >= 0; --j) { // the first entry (in order) that stops the walk
        const uint64_t kk = ((uint64_t)nx[j].y << 32) | nx[j].x;
        if (e + 1 + j >= a.n_entries || kk >= key) {
          step = j + 1;
          k2 = kk;
          cid2 = nx[j].z;
        }
      }
      if (srch) {
        if (step != 0) {
          e += step;
          k = k2;
          cid = cid2;
          srch = false;
        } else {
          e += kAhead; // every fetched key < key: the run goes on
        }
      }
    }
    uint64_t need = __ballot(srch);
    if constexpr (ABL & kGroupProbe) {
      while (need != 0) { // wave-uniform
        // the lanes at the first searching lane's run position: one fetch serves them all
        const uint32_t e0 = __builtin_amdgcn_readlane(e, (uint32_t)__builtin_ctzll(need));
        uint64_t group = __ballot(srch && e == e0);
        for (uint32_t base = e0 + 1; group != 0; base += kWave) {
          const uint32_t idx = base + lane;
          u32x4 ent = {0u, 0u, 0u, 0u};
          if (idx < a.n_entries) ent = *reinterpret_cast<const u32x4*>(a.tbl + idx);
          const uint64_t kk = ((uint64_t)ent.y << 32) | ent.x;
          for (uint64_t pend = group; pend != 0; pend &= pend - 1) {
            const uint32_t L = (uint32_t)__builtin_ctzll(pend);
            const uint64_t kl = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(key >> 32), L) << 32) |
                                (uint32_t)__builtin_amdgcn_readlane((uint32_t)key, L);
            const uint64_t stop = __ballot(idx >= a.n_entries || kk >= kl);
            if (stop != 0) { // the entry lane L's scalar walk stops at
              const uint32_t first = (uint32_t)__builtin_ctzll(stop);
              const uint32_t klo = __builtin_amdgcn_readlane(ent.x, first), khi = __builtin_amdgcn_readlane(ent.y, first);
              const uint32_t c = __builtin_amdgcn_readlane(ent.z, first);
              if (lane == L) {
                e = base + first;
                k = ((uint64_t)khi << 32) | klo;
                cid = c;
                srch = false;
              }
              group &= ~(1ull << L);
            }
          }
        }
        need = __ballot(srch);
      }
    } else {
      while (need != 0) { // wave-uniform
        const uint32_t L = (uint32_t)__builtin_ctzll(need);
        need &= need - 1;
        const uint64_t kl = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(key >> 32), L) << 32) |
                            (uint32_t)__builtin_amdgcn_readlane((uint32_t)key, L); // readlane returns int
        for (uint32_t base = __builtin_amdgcn_readlane(e, L) + 1;; base += kWave) {
          const uint32_t idx = base + lane;
          u32x4 ent = {0u, 0u, 0u, 0u};
          if (idx < a.n_entries) ent = *reinterpret_cast<const u32x4*>(a.tbl + idx);
          const uint64_t kk = ((uint64_t)ent.y << 32) | ent.x;
          const uint64_t stop = __ballot(idx >= a.n_entries || kk >= kl);
          if (stop != 0) {
            const uint32_t first = (uint32_t)__builtin_ctzll(stop);
            const uint32_t klo = __builtin_amdgcn_readlane(ent.x, first), khi = __builtin_amdgcn_readlane(ent.y, first);
            const uint32_t c = __builtin_amdgcn_readlane(ent.z, first);
            if (lane == L) {
              e = base + first;
              k = ((uint64_t)khi << 32) | klo;
              cid = c;
            }
            break;
          }
        }
      }
    }
  } else {
    while (live && e < a.n_entries && k < key) {
      if (++e >= a.n_entries) break;
      const u32x4 ent = *reinterpret_cast<const u32x4*>(a.tbl + e);
      k = ((uint64_t)ent.y << 32) | ent.x;
      cid = ent.z;
    }
  }
  if (live && e < a.n_entries && k == key) {
    conn_id = cid;
    flags |= PN_F_HIT;
    if (cid >= a.max_conn) flags |= PN_F_TW;
  }
}

// ---- phase 1: decode one frame from its header window (lane f <-> frame f) ----
template <int MIS, int ABL>
__device__ __forceinline__ FrameState header_phase(const Window& h, uint32_t ether_type, bool live, uint32_t s0,
                                                   const KArgs& a) {
  static_assert(MIS + 64 <= kWinBytes, "window must cover ip .. ip+64");
  FrameState st;
  // IpHeader (Core.h:57-69), fields relative to ip = window + MIS
  const uint32_t ver_ihl = h.template b8<MIS + 0>();
  st.ihl = ver_ihl & 0xf;
  st.tot_len = bswap16(h.template u16<MIS + 2>());
  const uint32_t proto = h.template b8<MIS + 9>();
  st.src_ip = h.template u32<MIS + 12>();
  st.dst_ip = h.template u32<MIS + 16>();
  // TcpHeader at ip + 20 (IHL assumed 5: Core.h:507)
  const uint32_t src_port = h.template u16<MIS + 20>();
  st.seq_raw = h.template u32<MIS + 24>();
  st.doff = h.template b8<MIS + 32>() >> 4;
  st.tflags = h.template b8<MIS + 33>();

  uint32_t flags = (st.tflags & 0x1f) << 4; // fin,syn,rst,psh,ack -> PN_F_FIN..PN_F_ACK
  if (ether_type != 0x0008 || (ver_ihl >> 4) != 4 || proto != 6) flags |= PN_F_NOT_TCP;
  if (st.ihl != 5) flags |= PN_F_IHL_NE_5;

  // CSum.add<20>(ip).fold() (Core.h:451-453)
  st.s_ip20 = h.template sum16<MIS, MIS + 20>();
  if (csum_fold(st.s_ip20) == 0) flags |= PN_F_IP_OK;
  // RFC option words [20, 4*IHL)
  st.s_opt = 0;
  if (st.ihl > 5) st.s_opt = h.template sum16_upto<MIS + 20, MIS + 60>(MIS + 4 * st.ihl);

  // uint16_t tcp_len = ntohs(tot_len) - 20 ; CSum::add(tcp, tcp_len) reads ceil(tcp_len/2) words
  st.tcp_len = (st.tot_len - 20) & 0xffff;
  const uint32_t seg_even = (st.tcp_len + 1) & ~1u;
  st.trunc = 34 + seg_even > a.avail;
  if (st.trunc) flags |= PN_F_TRUNC;
  // summed region relative to the window: [MIS, MIS + 20 + seg_even); bit 0 flags an odd
  // tcp_len, whose last summed byte (end - 1) is the byte after the segment
  st.end_rel = (live && !st.trunc) ? (int)((MIS + 20 + seg_even) | (st.tcp_len & 1)) : 0;
  st.pad = kPadUnknown;

  // the part of the region in the window below the stream start, summed from registers
  st.t_all = window_part<MIS>(h, st.end_rel & ~1, s0);

  // connHashKey (Core.h:167-172) + findConnEntry (Core.h:558-562), bounded at n_entries.
  // (Resolving the probe after phase 2 instead, so the home-slot load overlaps the stream loads,
  // measured no faster: profiles/r02/s3/late_probe_ab.json.)
  st.conn_id = PN_MISS;
  if constexpr (ABL & kLateProbe) st.probe = probe_issue<ABL>(st.src_ip, src_port, live, a);
  else if constexpr (!(ABL & kAblNoProbe)) probe_finish<ABL>(probe_issue<ABL>(st.src_ip, src_port, live, a), live, a, st.conn_id, flags);
  st.flags = flags;
  return st;
}

// ---- phase 3: fold and write the record on the frame's lane ----
template <int MIS, int ABL, int SAUX>
__device__ __forceinline__ void finish(const KArgs& a, FrameState st, uint32_t f, const uint8_t* win, bool bad_off,
                                       u32x4* lds_rec, uint32_t cx_ack = 0, uint32_t cx_wport = 0) {
  uint32_t flags = st.flags;
  uint32_t tcp_fold = 0xffff;
  if constexpr ((ABL & kHeaderOnly) != 0) { // the release path: no TCP sum (the IP header is in the window)
    flags |= PN_F_TCP_UNCHECKED; // tcp_fold stays 0xFFFF: no fold was computed (never a fold value)
    if (!st.trunc && st.ihl >= 5 && 4 * st.ihl <= st.tot_len && csum_fold(st.s_ip20 + st.s_opt) == 0)
      flags |= PN_F_RFC_IP_OK;
  } else if (!st.trunc) {
    const uint32_t s_seg = st.t_all - st.s_ip20; // exact: both are exact word sums
    const uint32_t s_addr = (st.src_ip >> 16) + (st.src_ip & 0xffff) + (st.dst_ip >> 16) + (st.dst_ip & 0xffff);
    // sum.add(ntohs(0x6)) ; sum.add(htons(tcp_len))  (Core.h:462-464)
    tcp_fold = csum_fold(s_addr + 0x0600 + bswap16(st.tcp_len) + s_seg);
    if (tcp_fold == 0) flags |= PN_F_TCP_OK;
    const uint32_t hl = 4 * st.ihl;
    if (st.ihl >= 5 && hl <= st.tot_len) {
      if (csum_fold(st.s_ip20 + st.s_opt) == 0) flags |= PN_F_RFC_IP_OK;
      uint32_t pad = 0;
      if (st.tot_len & 1) { // the byte the reference sums past the segment (high half of the last word)
        uint32_t b = st.pad;
        if (b == kPadUnknown) b = (win + MIS)[st.tot_len]; // in-window / jumbo
        pad = b << 8;
      }
      const uint32_t rfc = s_addr + 0x0600 + bswap16(st.tot_len - hl) + (s_seg - st.s_opt - pad);
      if (csum_fold(rfc) == 0) flags |= PN_F_RFC_TCP_OK;
    }
  }
  // TcpConn::onPack (TcpConn.h:469-473)
  const int data_off = 34 + 4 * (int)st.doff;
  const int data_end = 14 + (int)min(st.tot_len, 1500u);
  u32x4 rec;
  rec.x = st.conn_id;
  rec.y = __builtin_bswap32(st.seq_raw) + ((st.tflags >> 1) & 1);
  rec.z = (uint32_t)data_off | ((uint32_t)(data_end - data_off) << 16);
  rec.w = flags | (tcp_fold << 16);
  if (bad_off) rec = u32x4{PN_MISS, 0, 0, PN_F_BADOFF}; // outside the launch's alignment class: not parsed
  if constexpr (ABL & kChainAux) {
    u32x4* aux = static_cast<const KArgsAux&>(a).aux;
    if (aux) {
      aux[2 * f] = rec;
      aux[2 * f + 1] = u32x4{cx_ack, st.dst_ip, cx_wport, 0u};
    }
  }
  if (lds_rec) { // grouped launches write the workgroup's records in one burst at its end
    *lds_rec = rec;
  } else if constexpr (ABL & (kAblNoStore | kAblEarlyStore)) {
    if (rec.x == 0x7eadbeefu && rec.y == 0x12345678u) *reinterpret_cast<u32x4*>(a.out + f) = rec; // ~never
  } else if constexpr (ABL & kAblSmallStore) { // timing only: 16 blocks of 64 records, rewritten by every wave
    const uint32_t blk = __builtin_amdgcn_readfirstlane((f & ~63u) & 0x3C0u);
    const __amdgpu_buffer_rsrc_t rs = frame_rsrc((const uint8_t*)(a.out + blk), 64 * 16);
    __builtin_amdgcn_raw_buffer_store_b128(rec, rs, (f & 63u) * 16, 0, SAUX);
  } else if constexpr (ABL & kAblStore8) { // timing only: half the record bytes
    reinterpret_cast<uint2*>(a.out)[f] = uint2{rec.x ^ rec.y, rec.z ^ rec.w};
  } else if constexpr (ABL & kAblGlobalStore) { // the record through a plain global store (SAUX ignored)
    *reinterpret_cast<u32x4*>(a.out + f) = rec;
  } else {
    // one coalesced 1-KiB store per wave; the descriptor covers this wave's 64 records.  The block is the
    // same on every lane (a wave's frames never cross a 64-frame boundary): readfirstlane makes the
    // descriptor scalar, where a per-lane one would be a waterfall loop around the store
    const uint32_t blk = __builtin_amdgcn_readfirstlane(f & ~63u);
    const __amdgpu_buffer_rsrc_t rs = frame_rsrc((const uint8_t*)(a.out + blk), 64 * 16);
    __builtin_amdgcn_raw_buffer_store_b128(rec, rs, (f & 63u) * 16, 0, SAUX);
  }
}

// ---- the kernel: one 64-frame group per 64-thread workgroup ----
// COOP = 1: 8 lanes per slot load its 128-B window block (the 16-B chunk before the
// window + the window; the slot's first line in the default layout) into an
// XOR-swizzled LDS tile that the header lanes read back (load_window_strided).
// COOP = 0: each lane loads its own 112-B window (frame_off = 0).
// IDX = 1: indexed layout (frame i at frames + offs[i], any place, same (offs+14)%16
// class); per-frame stream descriptors; with COOP, waves whose frames all have their
// block 16-B aligned inside the ring load blocks cooperatively, other waves per-lane
// bounds-checked windows.
// Register target: 4 waves/SIMD.  Until round 3 the MIS % 4 == 0 kernels fit 5 (<= 96 VGPRs) and the
// LDS pad below held them at 4; the grouped probe takes them to 102 VGPRs (104 with the pipelined phase 2), so registers and pad agree.
template <int MIS, int COOP, int ABL, int LAUX, int SAUX, int IDX, int LWIN>
__device__ __forceinline__ void classify_group(const KArgs& a, const uint32_t wave_base, const int lane, u32x4* lds_recs) {
  if (wave_base >= a.n) return;
  const uint32_t f = wave_base + lane;
  const uint32_t n_here = min(a.fpw, a.n - wave_base);
  const bool live = (uint32_t)lane < n_here;
  const uint8_t* wave_slot = a.frames + (uint64_t)wave_base * a.stride;
  // one wave-uniform descriptor over the wave's slots; lanes past n read zeros
  const __amdgpu_buffer_rsrc_t rs = frame_rsrc(wave_slot, n_here * a.stride);
  if constexpr (ABL & kAblEarlyStore) {
    const uint32_t blk = __builtin_amdgcn_readfirstlane(f & ~63u);
    const __amdgpu_buffer_rsrc_t ro = frame_rsrc((const uint8_t*)(a.out + blk), 64 * 16);
    __builtin_amdgcn_raw_buffer_store_b128(u32x4{f, 0u, 0u, 0u}, ro, (f & 63u) * 16, 0, SAUX);
  }

  Window h;
  uint32_t ether_type;
  const uint8_t* win = nullptr; // this lane's window start (ip - MIS)
  bool bad_off = false;
  if constexpr (IDX) {
    ether_type = 0;
#pragma unroll
    for (int q = 0; q < 4 * kWinChunks; ++q) h.d[q] = 0;
    const uint64_t o = live ? a.offs[f] : 0;
    bad_off = live && ((o + 14) & 15) != (uint64_t)MIS;
    win = a.frames + o + 14 - MIS;
    bool coop_done = false;
    if constexpr (COOP) {
      // Cooperative window: when every frame of the wave has its 128-B window block (the
      // 16-B chunk before the window, and the window) 16-B aligned inside [base, eth + avail),
      // 8 lanes per frame load the block coalesced into the LDS tile, as the strided kernel
      // does (one request per line; the second line of a straddling block only when the
      // header fields reach it); otherwise the wave falls back to per-lane windows.
      const bool use = live && !bad_off;
      const bool elig = !use || ((((uintptr_t)win & 15u) == 0) && o + 14 >= (uint64_t)(MIS + 16) &&
                                 (uint32_t)(14 - MIS + kWinBytes) <= a.avail);
      if (__all(elig)) {
        __shared__ uint64_t line_addr[kFramesPerWave];
        line_addr[lane] = use ? (uint64_t)(win - 16) : 0ull;
        __syncthreads();
        u32x4* tile = coop_tile();
        // all 8 loads in flight before the first LDS write (as load_window_strided): a part that is not
        // needed reads its block's first chunk instead -- a line the same instruction fetches anyway (or,
        // for an unused row, the first used frame's block) -- and is zeroed, rather than a branch around it
        const uint64_t used = __ballot(use);
        const uint32_t l0 = used ? (uint32_t)__builtin_ctzll(used) : 0u;
        const uint64_t wb = (uint64_t)(win - 16);
        const uint64_t safe = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(wb >> 32), l0) << 32) |
                              (uint32_t)__builtin_amdgcn_readlane((uint32_t)wb, l0);
        u32x4 v[8];
        bool need[8];
        const u32x4* src[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const uint32_t r = 8 * i + (lane >> 3), part = lane & 7;
          const uint64_t la = line_addr[r];
          need[i] = la && block_part_needed<MIS>((uint32_t)la, part);
          src[i] = need[i] ? reinterpret_cast<const u32x4*>(la) + part : reinterpret_cast<const u32x4*>(la ? la : safe);
          v[i] = u32x4{0u, 0u, 0u, 0u};
        }
        if (used != 0) { // wave-uniform: a wave with no frame to classify loads nothing
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            if constexpr (LWIN == 0) v[i] = *src[i]; // default policy (tuning)
            else v[i] = __builtin_nontemporal_load(src[i]);
          }
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const uint32_t r = 8 * i + (lane >> 3), part = lane & 7;
          tile[r * 8 + (part ^ (r & 7))] = need[i] ? v[i] : u32x4{0u, 0u, 0u, 0u};
        }
        __syncthreads();
#pragma unroll
        for (int c = 0; c < kWinChunks; ++c) {
          const u32x4 v = tile[lane * 8 + ((1 + c) ^ (lane & 7))];
          h.d[4 * c + 0] = v.x;
          h.d[4 * c + 1] = v.y;
          h.d[4 * c + 2] = v.z;
          h.d[4 * c + 3] = v.w;
        }
        if constexpr (MIS >= 2) ether_type = h.template u16<MIS - 2>();
        else ether_type = tile[lane * 8 + (0 ^ (lane & 7))].w >> 16;
        coop_done = true;
      }
    }
    if (live && !coop_done) {
      if (!bad_off) {
        // window chunk c spans eth + (14 - MIS) + 16c .. +16: used only inside avail.  A chunk past it
        // re-reads chunk 0 (a line this lane fetches anyway) and is dropped, rather than a branch around
        // its load, so the 7 loads are in flight together
        u32x4 v[kWinChunks];
#pragma unroll
        for (int c = 0; c < kWinChunks; ++c) {
          const bool in = (uint32_t)(14 - MIS + 16 * c + 16) <= a.avail;
          v[c] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(win) + (in ? c : 0));
        }
#pragma unroll
        for (int c = 0; c < kWinChunks; ++c) {
          if ((uint32_t)(14 - MIS + 16 * c + 16) <= a.avail) {
            h.d[4 * c + 0] = v[c].x;
            h.d[4 * c + 1] = v[c].y;
            h.d[4 * c + 2] = v[c].z;
            h.d[4 * c + 3] = v[c].w;
          }
        }
        if constexpr (MIS >= 2) ether_type = h.template u16<MIS - 2>();
        else ether_type = *reinterpret_cast<const uint32_t*>(win - 4) >> 16; // eth + 10 - MIS >= eth
      }
    }
  } else {
    ether_type = load_window_strided<MIS, COOP, LWIN, (ABL & kSerialWindow) != 0>(rs, lane, a.stride, a.ipa_off,
                                                                                    (uint32_t)(uintptr_t)wave_slot, h);
  }
  if constexpr (!IDX) win = wave_slot + (uint64_t)lane * a.stride + a.ipa_off;
  FrameState st = header_phase<MIS, ABL>(h, ether_type, live && !bad_off, stream_start((uint64_t)win), a);
  if constexpr (IDX && (ABL & kAblContigStream)) {
    // timing only: [first frame's stream start, last frame's extent end) as one range, 16 x 1 KiB per round
    const uint64_t w = (uint64_t)win;
    const uint64_t lo64 = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(w >> 32), 0) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane((uint32_t)w, 0);
    const uint32_t last = n_here - 1;
    const uint64_t hw = ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(w >> 32), last) << 32) |
                        (uint32_t)__builtin_amdgcn_readlane((uint32_t)w, last);
    const uint64_t lo = (lo64 + stream_start(lo64)) & ~15ull;
    const uint64_t hi = (hw + (uint32_t)(__builtin_amdgcn_readlane(st.end_rel, last) & ~1) + 15) & ~15ull;
    const uint32_t len = hi > lo ? (uint32_t)(hi - lo) : 0u;
    const __amdgpu_buffer_rsrc_t rc = frame_rsrc((const uint8_t*)lo, len);
    uint32_t sum = 0;
    for (uint32_t o = 0; o < len; o += 16 * 1024) {
      u32x4 v[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = __builtin_amdgcn_raw_buffer_load_b128(rc, o + j * 1024 + lane * 16, 0, LAUX);
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        sum = dot2(v[j].x, 0x10001u, sum);
        sum = dot2(v[j].y, 0x10001u, sum);
        sum = dot2(v[j].z, 0x10001u, sum);
        sum = dot2(v[j].w, 0x10001u, sum);
      }
    }
    st.t_all += sum;
  } else if constexpr ((ABL & kHeaderOnly) != 0) {
    // no segment stream: the record needs only the header lines
  } else {
    if constexpr ((ABL & kSkipWaveGate) && (ABL & kSkipEmptyLoads)) {
      // a frame whose extent ends before its second stream KiB: take the skipping form
      const uint32_t e16 = (uint32_t)((st.end_rel & ~1) + 3) & ~3u;
      const bool short_frame = live && e16 <= stream_start((uint64_t)win) + 1024;
      constexpr int kFull = ABL & ~(kSkipEmptyLoads | kSkipWaveGate);
      if (__ballot(short_frame) == 0) {
        if constexpr ((ABL & kPipeStream) && !IDX) {
          if (a.stride <= 2048) // no frame reaches past its two stream KiBs
            stream_phase_pipelined<kFull, LAUX, IDX>(a.stride, wave_slot + a.ipa_off, (uint64_t)win, n_here, lane,
                                                     st.end_rel, st.t_all, st.pad);
          else
            stream_phase<kFull, LAUX, IDX>(a.stride, wave_slot + a.ipa_off, (uint64_t)win, n_here, lane, st.end_rel,
                                           st.t_all, st.pad);
        } else {
          stream_phase<kFull, LAUX, IDX>(a.stride, wave_slot + a.ipa_off, (uint64_t)win, n_here, lane, st.end_rel,
                                         st.t_all, st.pad);
        }
      } else {
        stream_phase<ABL, LAUX, IDX>(a.stride, wave_slot + a.ipa_off, (uint64_t)win, n_here, lane, st.end_rel, st.t_all,
                                     st.pad);
      }
    } else {
      stream_phase<ABL, LAUX, IDX>(a.stride, wave_slot + a.ipa_off, (uint64_t)win, n_here, lane, st.end_rel, st.t_all,
                                   st.pad);
    }
  }
  if constexpr (ABL & kLateProbe) probe_finish<ABL>(st.probe, live && !bad_off, a, st.conn_id, st.flags);
  if constexpr (ABL & kChainAux) { // the ack number and window << 16 | destination port, as stored
    if (live)
      finish<MIS, ABL, SAUX>(a, st, f, win, bad_off, lds_recs ? lds_recs + lane : nullptr, h.template u32<MIS + 28>(),
                             h.template u16<MIS + 22>() | (h.template u16<MIS + 34>() << 16));
  } else {
    if (live) finish<MIS, ABL, SAUX>(a, st, f, win, bad_off, lds_recs ? lds_recs + lane : nullptr);
  }
}

// GRP = 1: one 64-frame group per workgroup, records stored as each group finishes.
// GRP > 1 (tuning variants): GRP consecutive groups per workgroup, their records kept in
// LDS and written in one GRP-KiB burst at the end (scripts/write_grouping.py probe).
// GOPT (tuning): bit 0 = GRP groups per workgroup but records stored per group (no LDS);
// bit 1 / bit 2 = register budget for 3 / 2 waves per SIMD instead of 4 (a budget for 5 spills and costs 8.6 %
// on the round-3 final tree, profiles/r03/window/five_waves_c*.json);
// GOPT >> 4 = KiB of LDS padding, which caps workgroups per CU.  Production pads 2 KiB:
// with the 8-KiB window tile that is 10 KiB per workgroup, 16 per CU = 4 waves/SIMD where
// registers allowed 5 before the grouped probe -- C2 -1.2 %, C3 -2.5 %, C5 -0.3 % (3 waves: C3 +9 %, C5 +13 %;
// profiles/r01_experiments/occupancy_c{2,3,5}.json).
// Bit 3: XCD-aware order.  Workgroup b is dispatched to XCD b % 8; mapping it to group
// (b % 8) * ceil(G / 8) + b / 8 gives every XCD one contiguous eighth of the batch (its own
// L2 and memory-side traffic stays in one region): C2 -1.2 %, C3 -4.2 %, C5 -3.4 %
// (profiles/r01_experiments/xcd_order_c{2,3,5}.json; records identical).
constexpr int kXcdOrder = 8;
constexpr int kProdGopt = (2 << 4) | kXcdOrder;
// Bit 12: completion word (pn_classify_notify; signal_done in frame_pass.hpp).  Above the LDS-padding
// field (bits 4-11).
constexpr int kSignalDone = 1 << 12;
// Bit 13 (tuning): GRP consecutive groups per workgroup in XCD order, each group's records stored as it
// finishes, so a group's store is in flight while the next group loads (only the last store is waited for at the
// wave's end).  Bit 14: the lane index made opaque per group, so the compiler cannot hoist lane-derived values
// out of the group loop (live across it they cost registers: 128-147 VGPRs in the GRP > 1 variants above).
constexpr int kGroupLoopXcd = 1 << 13;
constexpr int kOpaqueLane = 1 << 14;
template <int MIS, int COOP, int ABL = kProdAbl, int LAUX = kLoadAux, int SAUX = kStoreAux, int IDX = 0, int LWIN = LAUX,
          int GRP = 1, int GOPT = kProdGopt>
__global__ __launch_bounds__(kWave, (GOPT & 4) ? 2 : (GOPT & 2) ? 3 : 4) void rx_classify_kernel(KArgs a) {
  const int lane = threadIdx.x;
  static_assert(!(GOPT & kSignalDone) || ((GOPT & 8) && GRP == 1), "the completion word is set on the XCD-ordered one-group path");
  if constexpr (((GOPT >> 4) & 0xff) > 0) {
    __shared__ uint32_t pad_lds[((GOPT >> 4) & 0xff) * 256];
    pad_lds[lane] = lane;
    // never true: keeps the padding allocated.  The test is wave-uniform (readfirstlane), so a.n stays
    // a scalar: a per-lane write to it made every descriptor built from it divergent, and the compiler
    // then wrapped each buffer load in a waterfall loop and serialized the window loads.
    if (__builtin_amdgcn_readfirstlane(pad_lds[(lane + 1) & 63]) == 0x7fffffffu) a.n = 0;
  }
  if constexpr (GOPT & kGroupLoopXcd) {
    const uint32_t g0 = xcd_group(blockIdx.x, gridDim.x) * GRP;
#pragma nounroll
    for (int g = 0; g < GRP; ++g) {
      int l = lane;
      if constexpr (GOPT & kOpaqueLane) asm volatile("" : "+v"(l));
      classify_group<MIS, COOP, ABL, LAUX, SAUX, IDX, LWIN>(a, (g0 + g) * a.fpw, l, nullptr);
    }
  } else if constexpr (GOPT & 8) { // XCD-aware order (tuning): workgroup b runs on XCD b % 8; give each XCD a
    // contiguous eighth of the batch instead of every eighth group
    classify_group<MIS, COOP, ABL, LAUX, SAUX, IDX, LWIN>(a, xcd_group(blockIdx.x, gridDim.x) * a.fpw, lane, nullptr);
    if constexpr (GOPT & kSignalDone) signal_done(a.sig_count, a.sig_flag, a.sig_token, lane);
  } else if constexpr (GRP == 1 || (GOPT & 1)) {
#pragma nounroll
    for (int g = 0; g < GRP; ++g)
      classify_group<MIS, COOP, ABL, LAUX, SAUX, IDX, LWIN>(a, (blockIdx.x * GRP + g) * a.fpw, lane, nullptr);
  } else {
    __shared__ u32x4 recs[GRP * kFramesPerWave];
    const uint32_t first = blockIdx.x * GRP * kFramesPerWave;
#pragma nounroll
    for (int g = 0; g < GRP; ++g) // not unrolled: two groups' live ranges overlapping would halve occupancy
      classify_group<MIS, COOP, ABL, LAUX, SAUX, IDX, LWIN>(a, first + g * kFramesPerWave, lane, recs + g * kFramesPerWave);
    __syncthreads();
    if (first >= a.n) return;
    const uint32_t cnt = min((uint32_t)(GRP * kFramesPerWave), a.n - first);
    const __amdgpu_buffer_rsrc_t ro = frame_rsrc((const uint8_t*)(a.out + first), cnt * 16); // stores past n dropped
#pragma unroll
    for (int g = 0; g < GRP; ++g)
      __builtin_amdgcn_raw_buffer_store_b128(recs[g * kFramesPerWave + lane], ro, (g * kFramesPerWave + lane) * 16, 0, SAUX);
  }
}
} // namespace

namespace {
// Whether the cooperative header-window load applies: a 16-B chunk precedes the
// window inside the slot (frame_off >= 2) and blocks are 16-B aligned.  One request
// per block line: a single line for the default frame_off = 2 layout and ef_vi's
// 10 + prefix for prefix <= 5, two otherwise.
inline bool coop_layout(const KArgs& a) {
  return (a.stride % 16) == 0 && a.ipa_off >= 16 && ((uintptr_t)a.frames % 16) == 0;
}

// Indexed launches load the cooperative window blocks at the default cache policy: in a
// packed capture a frame's last line is the next frame's window line, and a block loaded
// with default policy is still in L2 when the previous frame's stream asks for it
// (packed C2/C3/C5 -8..-10 %, permuted ef_vi event runs -2 %, in-order slot runs +1 %;
// profiles/r01_experiments/indexed_window_policy_c{2,3,5}.json).
constexpr int kIdxWin = 0;

template <int MIS, int COOP, int ABL = kProdAbl, int LAUX = kLoadAux, int SAUX = kStoreAux, int IDX = 0, int LWIN = LAUX,
          int GRP = 1, int GOPT = kProdGopt>
void launch_one(const KArgs& a, hipStream_t s) {
  hipLaunchKernelGGL((rx_classify_kernel<MIS, COOP, ABL, LAUX, SAUX, IDX, LWIN, GRP, GOPT>),
                     dim3((a.n + GRP * a.fpw - 1) / (GRP * a.fpw)), dim3(kWave), 0, s, a);
}


template <int MIS, bool SIG = false, bool HO = false>
void launch(const KArgs& a, hipStream_t s) {
  constexpr int G = SIG ? (kProdGopt | kSignalDone) : kProdGopt;
  constexpr int A = HO ? (kProdAbl | kHeaderOnly) : kProdAbl;
  if (coop_layout(a)) return launch_one<MIS, 1, A, kLoadAux, kStoreAux, 0, kLoadAux, 1, G>(a, s);
  launch_one<MIS, 0, A, kLoadAux, kStoreAux, 0, kLoadAux, 1, G>(a, s);
}
} // namespace
