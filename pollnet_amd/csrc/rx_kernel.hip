// MI355X (gfx950) receive-path per-frame transform: Ethernet/IPv4/TCP header
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
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <string>

#include "../../include/pollnet_amd.h"
#include "device_common.hpp"
#include "frame_pass.hpp"
#include "pn_internal.hpp"

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
};

// Per-frame state the header lane keeps from phase 1 to phase 3.
struct FrameState {
  uint32_t flags, ihl, tot_len, src_ip, dst_ip, seq_raw, doff, tflags, s_ip20, s_opt, tcp_len, conn_id;
  uint32_t t_all; // exact u16-word sum of [ip, ip+20+tcp_len(+pad)) accumulated so far
  int end_rel;    // summed extent relative to the window start (even), | 1 when tcp_len is odd; 0 = nothing to stream
  uint32_t pad;   // odd tcp_len: the byte after the segment (kPadUnknown until phase 2 captured it)
  bool trunc;
};

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

  // connHashKey (Core.h:167-172) + findConnEntry (Core.h:558-562), bounded at n_entries
  st.conn_id = PN_MISS;
  if constexpr (!(ABL & kAblNoProbe)) {
    const uint32_t ip_h = __builtin_bswap32(st.src_ip);
    const uint32_t port_h = bswap16(src_port);
    const uint64_t key = ((uint64_t)ip_h << 15) | (port_h & 0x7fff) | ((uint64_t)(port_h & 0x8000) << 32);
    uint32_t e = (uint32_t)(key & a.mask);
    uint64_t k = PN_EMPTY_KEY;
    uint32_t cid = 0;
    if (live && e < a.n_entries) { // the home slot: almost every lookup ends here
      const u32x4 ent = *reinterpret_cast<const u32x4*>(a.tbl + e);
      k = ((uint64_t)ent.y << 32) | ent.x;
      cid = ent.z;
    }
    if constexpr (ABL & kCoopProbe) {
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
    } else {
      while (live && e < a.n_entries && k < key) {
        if (++e >= a.n_entries) break;
        const u32x4 ent = *reinterpret_cast<const u32x4*>(a.tbl + e);
        k = ((uint64_t)ent.y << 32) | ent.x;
        cid = ent.z;
      }
    }
    if (live && e < a.n_entries && k == key) {
      st.conn_id = cid;
      flags |= PN_F_HIT;
      if (cid >= a.max_conn) flags |= PN_F_TW;
    }
  }
  st.flags = flags;
  return st;
}

// ---- phase 3: fold and write the record on the frame's lane ----
template <int MIS, int ABL, int SAUX>
__device__ __forceinline__ void finish(const KArgs& a, FrameState st, uint32_t f, const uint8_t* win, bool bad_off,
                                       u32x4* lds_rec) {
  uint32_t flags = st.flags;
  uint32_t tcp_fold = 0xffff;
  if (!st.trunc) {
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
  if (lds_rec) { // grouped launches write the workgroup's records in one burst at its end
    *lds_rec = rec;
  } else if constexpr (ABL & kAblNoStore) {
    if (rec.x == 0x7eadbeefu && rec.y == 0x12345678u) *reinterpret_cast<u32x4*>(a.out + f) = rec; // ~never
  } else if constexpr (ABL & kAblStore8) { // timing only: half the record bytes
    reinterpret_cast<uint2*>(a.out)[f] = uint2{rec.x ^ rec.y, rec.z ^ rec.w};
  } else if constexpr (ABL & kAblGlobalStore) { // the record through a plain global store (SAUX ignored)
    *reinterpret_cast<u32x4*>(a.out + f) = rec;
  } else {
    // one coalesced 1-KiB store per wave; the descriptor covers this wave's 64 records
    const __amdgpu_buffer_rsrc_t rs = frame_rsrc((const uint8_t*)(a.out + (f & ~63u)), 64 * 16);
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
// 5 waves/SIMD (<= 96 VGPRs) where that compiles without spills (MIS % 4 == 0, incl. the
// default and ef_vi layouts); the 2-mod-4 alignments and the indexed path need a few more VGPRs and keep 4.
template <int MIS, int COOP, int ABL, int LAUX, int SAUX, int IDX, int LWIN>
__device__ __forceinline__ void classify_group(const KArgs& a, const uint32_t wave_base, const int lane, u32x4* lds_recs) {
  if (wave_base >= a.n) return;
  const uint32_t f = wave_base + lane;
  const uint32_t n_here = min(a.fpw, a.n - wave_base);
  const bool live = (uint32_t)lane < n_here;
  const uint8_t* wave_slot = a.frames + (uint64_t)wave_base * a.stride;
  // one wave-uniform descriptor over the wave's slots; lanes past n read zeros
  const __amdgpu_buffer_rsrc_t rs = frame_rsrc(wave_slot, n_here * a.stride);

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
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const uint32_t r = 8 * i + (lane >> 3), part = lane & 7;
          const uint64_t la = line_addr[r];
          u32x4 v = {0u, 0u, 0u, 0u};
          if (la && block_part_needed<MIS>((uint32_t)la, part)) {
            if constexpr (LWIN == 0) v = reinterpret_cast<const u32x4*>(la)[part]; // default policy (tuning)
            else v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(la) + part);
          }
          tile[r * 8 + (part ^ (r & 7))] = v;
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
        // window chunk c spans eth + (14 - MIS) + 16c .. +16: load it only inside avail
#pragma unroll
        for (int c = 0; c < kWinChunks; ++c) {
          if ((uint32_t)(14 - MIS + 16 * c + 16) <= a.avail) {
            const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(win) + c);
            h.d[4 * c + 0] = v.x;
            h.d[4 * c + 1] = v.y;
            h.d[4 * c + 2] = v.z;
            h.d[4 * c + 3] = v.w;
          }
        }
        if constexpr (MIS >= 2) ether_type = h.template u16<MIS - 2>();
        else ether_type = *reinterpret_cast<const uint32_t*>(win - 4) >> 16; // eth + 10 - MIS >= eth
      }
    }
  } else {
    ether_type = load_window_strided<MIS, COOP, LWIN>(rs, lane, a.stride, a.ipa_off, (uint32_t)(uintptr_t)wave_slot, h);
  }
  if constexpr (!IDX) win = wave_slot + (uint64_t)lane * a.stride + a.ipa_off;
  FrameState st = header_phase<MIS, ABL>(h, ether_type, live && !bad_off, stream_start((uint64_t)win), a);
  stream_phase<ABL, LAUX, IDX>(a.stride, wave_slot + a.ipa_off, (uint64_t)win, n_here, lane, st.end_rel, st.t_all, st.pad);
  if (live) finish<MIS, ABL, SAUX>(a, st, f, win, bad_off, lds_recs ? lds_recs + lane : nullptr);
}

// GRP = 1: one 64-frame group per workgroup, records stored as each group finishes.
// GRP > 1 (tuning variants): GRP consecutive groups per workgroup, their records kept in
// LDS and written in one GRP-KiB burst at the end (scripts/write_grouping.py probe).
// GOPT (tuning): bit 0 = GRP groups per workgroup but records stored per group (no LDS);
// bit 1 / bit 2 = register budget for 3 / 2 waves per SIMD instead of 5;
// GOPT >> 4 = KiB of LDS padding, which caps workgroups per CU.  Production pads 2 KiB:
// with the 8-KiB window tile that is 10 KiB per workgroup, 16 per CU = 4 waves/SIMD where
// registers would allow 5 -- C2 -1.2 %, C3 -2.5 %, C5 -0.3 % (3 waves: C3 +9 %, C5 +13 %;
// profiles/r01_experiments/occupancy_c{2,3,5}.json).
// Bit 3: XCD-aware order.  Workgroup b is dispatched to XCD b % 8; mapping it to group
// (b % 8) * ceil(G / 8) + b / 8 gives every XCD one contiguous eighth of the batch (its own
// L2 and memory-side traffic stays in one region): C2 -1.2 %, C3 -4.2 %, C5 -3.4 %
// (profiles/r01_experiments/xcd_order_c{2,3,5}.json; records identical).
constexpr int kXcdOrder = 8;
constexpr int kProdGopt = (2 << 4) | kXcdOrder;
template <int MIS, int COOP, int ABL = kProdAbl, int LAUX = kLoadAux, int SAUX = kStoreAux, int IDX = 0, int LWIN = LAUX,
          int GRP = 1, int GOPT = kProdGopt>
__global__ __launch_bounds__(kWave, (GOPT & 4) ? 2 : (GOPT & 2) ? 3 : (MIS % 4 == 0 && !IDX) ? 5 : 4) void rx_classify_kernel(KArgs a) {
  const int lane = threadIdx.x;
  if constexpr ((GOPT >> 4) > 0) {
    __shared__ uint32_t pad_lds[(GOPT >> 4) * 256];
    pad_lds[lane] = lane;
    if (pad_lds[(lane + 1) & 63] == 0x7fffffffu) a.n = 0; // never true: keeps the padding allocated
  }
  if constexpr (GOPT & 8) { // XCD-aware order (tuning): workgroup b runs on XCD b % 8; give each XCD a
    // contiguous eighth of the batch instead of every eighth group
    classify_group<MIS, COOP, ABL, LAUX, SAUX, IDX, LWIN>(a, xcd_group(blockIdx.x, gridDim.x) * a.fpw, lane, nullptr);
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

__global__ __launch_bounds__(256) void calib_stream_read_kernel(const u32x4* src, uint64_t n16, uint32_t* sink) {
  // the whole grid sweeps the buffer front to back, one 16-B coalesced load per lane per step
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) {
    const u32x4 v = src[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9E3779B9u) sink[blockIdx.x] = acc; // keeps the loads live; practically never stores
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
  if (pad_lds[(lane + 1) & 63] == 0x7fffffffu) n = 0; // never true: keeps the padding allocated
  const uint32_t wave_base = xcd_group(blockIdx.x, gridDim.x) * kFramesPerWave;
  if (wave_base >= n) return;
  const uint32_t n_here = min((uint32_t)kFramesPerWave, n - wave_base);
  const uint8_t* wb = base + (uint64_t)wave_base * stride;
  uint32_t acc = 0;
  for (uint32_t b0 = 0; b0 < n_here; b0 += kBatch) {
    u32x4 w0s[kBatch], w1s[kBatch];
#pragma unroll
    for (int j = 0; j < kBatch; ++j) {
      const uint32_t nb = (b0 + j < n_here) ? min(lens[wave_base + b0 + j], min(stride, 2048u)) : 0u;
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

} // namespace

// ============================ C-ABI ============================
namespace {
// Whether the cooperative header-window load applies: a 16-B chunk precedes the
// window inside the slot (frame_off >= 2) and blocks are 16-B aligned.  One request
// per block line: a single line for the default frame_off = 2 layout and ef_vi's
// 10 + prefix for prefix <= 5, two otherwise.
bool coop_layout(const KArgs& a) {
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


template <int MIS>
void launch(const KArgs& a, hipStream_t s) {
  if (coop_layout(a)) return launch_one<MIS, 1>(a, s);
  launch_one<MIS, 0>(a, s);
}
} // namespace

extern "C" {

int pn_device_count(int* n) {
  if (!n) return PN_EINVAL;
  hipError_t e = hipGetDeviceCount(n);
  if (e != hipSuccess) {
    *n = 0;
    return hip_err(nullptr, e, "hipGetDeviceCount");
  }
  return PN_OK;
}

int pn_open(int device, pn_ctx** out) {
  if (!out) return set_err(nullptr, PN_EINVAL, "pn_open: out is NULL");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) return hip_err(nullptr, e, "hipGetDeviceCount");
  if (device < 0 || device >= n) return set_err(nullptr, PN_EINVAL, "pn_open: no such device");
  pn_ctx* c = new pn_ctx();
  c->device = device;
  *out = c;
  return PN_OK;
}

void pn_close(pn_ctx* ctx) {
  if (!ctx) return;
  if (ctx->tbl_dev || ctx->tx_patch) {
    (void)hipSetDevice(ctx->device);
    if (ctx->tx_patch) (void)hipStreamSynchronize(ctx->tx_stream);
    if (ctx->tbl_dev) (void)hipFree(ctx->tbl_dev);
    if (ctx->tx_patch) (void)hipFree(ctx->tx_patch);
  }
  delete ctx;
}

const char* pn_last_error(const pn_ctx* ctx) { return ctx ? ctx->err.c_str() : g_err.c_str(); }

int pn_set_conn_table(pn_ctx* ctx, const pn_conn_entry* entries, uint32_t n_entries, uint64_t tbl_mask,
                      uint32_t max_conn_cnt) {
  if (!ctx || !entries || n_entries == 0) return set_err(ctx, PN_EINVAL, "pn_set_conn_table: bad arguments");
  if (tbl_mask >= n_entries || (tbl_mask & (tbl_mask + 1)) != 0)
    return set_err(ctx, PN_EINVAL, "pn_set_conn_table: tbl_mask must be 2^k-1 < n_entries");
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return hip_err(ctx, e, "hipSetDevice");
  // a classify launched on this ctx may still be reading the table: let it finish
  // before the snapshot is replaced (the copy below is not ordered against that stream)
  if (ctx->tbl_dev) {
    e = hipStreamSynchronize(ctx->last_stream);
    if (e != hipSuccess) return hip_err(ctx, e, "hipStreamSynchronize(last classify)");
  }
  if (n_entries > ctx->n_entries) {
    if (ctx->tbl_dev) (void)hipFree(ctx->tbl_dev);
    ctx->tbl_dev = nullptr;
    ctx->n_entries = 0;
    e = hipMalloc(&ctx->tbl_dev, (size_t)n_entries * sizeof(pn_conn_entry));
    if (e != hipSuccess) return hip_err(ctx, e, "hipMalloc(conn table)");
  }
  e = hipMemcpy(ctx->tbl_dev, entries, (size_t)n_entries * sizeof(pn_conn_entry), hipMemcpyHostToDevice);
  if (e != hipSuccess) return hip_err(ctx, e, "hipMemcpy(conn table)");
  ctx->n_entries = n_entries;
  ctx->mask = tbl_mask;
  ctx->max_conn = max_conn_cnt;
  return PN_OK;
}

int pn_classify(pn_ctx* ctx, const void* frames_dev, uint32_t slot_stride, uint32_t frame_off, uint32_t n,
                void* results_dev, void* stream) {
  if (!ctx) return set_err(nullptr, PN_EINVAL, "pn_classify: ctx is NULL");
  if (!ctx->tbl_dev) return set_err(ctx, PN_ENOTABLE, "pn_classify: no conn table (call pn_set_conn_table)");
  if (n == 0) return PN_OK;
  if (!frames_dev || !results_dev) return set_err(ctx, PN_EINVAL, "pn_classify: NULL buffer");
  if (((uintptr_t)frames_dev & 15) || ((uintptr_t)results_dev & 15))
    return set_err(ctx, PN_EINVAL, "pn_classify: frames/results must be 16-byte aligned");
  if ((slot_stride & 15) || slot_stride > 65536 || (frame_off & 1) || slot_stride < frame_off + 96)
    return set_err(ctx, PN_EINVAL, "pn_classify: slot_stride/frame_off violate the layout contract");
  KArgs a;
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
  hipStream_t s = (hipStream_t)stream;
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return hip_err(ctx, e, "hipSetDevice");
  switch ((frame_off + 14) & 15) {
    case 0: launch<0>(a, s); break;
    case 2: launch<2>(a, s); break;
    case 4: launch<4>(a, s); break;
    case 6: launch<6>(a, s); break;
    case 8: launch<8>(a, s); break;
    case 10: launch<10>(a, s); break;
    case 12: launch<12>(a, s); break;
    default: launch<14>(a, s); break;
  }
  e = hipGetLastError();
  if (e != hipSuccess) return hip_err(ctx, e, "rx_classify launch");
  ctx->last_stream = s;
  return PN_OK;
}

int pn_classify_indexed(pn_ctx* ctx, const void* base, const uint64_t* offsets, uint32_t eth_mod16, uint32_t n,
                        uint32_t avail, void* results_dev, void* stream) {
  if (!ctx) return set_err(nullptr, PN_EINVAL, "pn_classify_indexed: ctx is NULL");
  if (!ctx->tbl_dev) return set_err(ctx, PN_ENOTABLE, "pn_classify_indexed: no conn table (call pn_set_conn_table)");
  if (n == 0) return PN_OK;
  if (!base || !offsets || !results_dev) return set_err(ctx, PN_EINVAL, "pn_classify_indexed: NULL buffer");
  if (((uintptr_t)base & 15) || ((uintptr_t)results_dev & 15) || ((uintptr_t)offsets & 7))
    return set_err(ctx, PN_EINVAL, "pn_classify_indexed: base/results must be 16-byte, offsets 8-byte aligned");
  if (eth_mod16 > 15 || (eth_mod16 & 1) || avail < 96 || avail > 65536)
    return set_err(ctx, PN_EINVAL, "pn_classify_indexed: eth_mod16 must be even < 16, avail in [96, 65536]");
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
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return hip_err(ctx, e, "hipSetDevice");
  switch ((eth_mod16 + 14) & 15) {
    case 0: launch_one<0, 1, kProdAbl, kLoadAux, kStoreAux, 1, kIdxWin, 1, kXcdOrder>(a, s); break;
    case 2: launch_one<2, 1, kProdAbl, kLoadAux, kStoreAux, 1, kIdxWin, 1, kXcdOrder>(a, s); break;
    case 4: launch_one<4, 1, kProdAbl, kLoadAux, kStoreAux, 1, kIdxWin, 1, kXcdOrder>(a, s); break;
    case 6: launch_one<6, 1, kProdAbl, kLoadAux, kStoreAux, 1, kIdxWin, 1, kXcdOrder>(a, s); break;
    case 8: launch_one<8, 1, kProdAbl, kLoadAux, kStoreAux, 1, kIdxWin, 1, kXcdOrder>(a, s); break;
    case 10: launch_one<10, 1, kProdAbl, kLoadAux, kStoreAux, 1, kIdxWin, 1, kXcdOrder>(a, s); break;
    case 12: launch_one<12, 1, kProdAbl, kLoadAux, kStoreAux, 1, kIdxWin, 1, kXcdOrder>(a, s); break;
    default: launch_one<14, 1, kProdAbl, kLoadAux, kStoreAux, 1, kIdxWin, 1, kXcdOrder>(a, s); break;
  }
  e = hipGetLastError();
  if (e != hipSuccess) return hip_err(ctx, e, "rx_classify (indexed) launch");
  ctx->last_stream = s;
  return PN_OK;
}

// Tuning: the indexed kernel with the cooperative line window (variant 1) or without (0),
// A/B-timed by scripts/bench_indexed.py; not part of the public header.
int pn_classify_indexed_variant(pn_ctx* ctx, const void* base, const uint64_t* offsets, uint32_t eth_mod16, uint32_t n,
                                uint32_t avail, void* results_dev, void* stream, int variant) {
  if (!ctx || !ctx->tbl_dev || n == 0 || eth_mod16 != 2 || variant < 0 || variant > 3)
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
  hipStream_t s = (hipStream_t)stream;
  if (variant == 1) launch_one<0, 1, kProdAbl, kLoadAux, kStoreAux, 1, kLoadAux, 1, kXcdOrder>(a, s); // window non-temporal
  else if (variant == 2) launch_one<0, 1, kProdAbl, kLoadAux, kStoreAux, 1, 0, 1, 0>(a, s);  // production window, blockIdx order
  else if (variant == 3) launch_one<0, 1, kProdAbl, 0, kStoreAux, 1, 0, 1, 0>(a, s);         // + stream at default policy
  else launch_one<0, 0, kProdAbl, kLoadAux, kStoreAux, 1, kLoadAux, 1, 0>(a, s);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hip_err(ctx, e, "indexed variant launch");
  ctx->last_stream = s;
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
    case 11: launch_one<0, 1, kAblNoProbe | kProdAbl>(a, s); break;           // timing-only ablations from here
    case 12: launch_one<0, 1, kAblNoReduce | kProdAbl>(a, s); break;
    case 14: launch_one<0, 1, kAblNoMask>(a, s); break;
    case 18: launch_one<0, 1, kAblNoStore | kProdAbl>(a, s); break;
    default: return set_err(ctx, PN_EINVAL, "variant: unknown");
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hip_err(ctx, e, "variant launch");
  ctx->last_stream = s;
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
  ctx->last_stream = s;
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
  ctx->last_stream = s;
  return PN_OK;
}

int pn_sync(pn_ctx* ctx) {
  if (!ctx) return set_err(nullptr, PN_EINVAL, "pn_sync: ctx is NULL");
  hipError_t e = hipSetDevice(ctx->device);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->last_stream);
  if (e != hipSuccess) return hip_err(ctx, e, "hipStreamSynchronize");
  return PN_OK;
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
  ctx->last_stream = (hipStream_t)stream;
  return PN_OK;
}

} // extern "C"
