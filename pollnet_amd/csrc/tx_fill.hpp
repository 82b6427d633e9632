// tx_fill.hpp — the TX checksum-fill kernels (device code + launch helpers), shared by the
// product library (tx_kernel.hip: pn_tx_fill) and the tuning library (tx_tuning.hip:
// A/B variants).  Internal linkage; one including translation unit per library.
#pragma once
// MI355X (gfx950) TX checksum fill for a batch of outgoing frames.
//
// Reference: efvitcp never sums a frame in one pass; it carries one's-complement
// state per connection and per send buffer and folds it when the frame leaves:
//   TcpConn::reset / onEstablished cache the header sums (TcpConn.h:149-186, :422-428),
//   sendPartial adds each appended piece with copyAndSum (TcpConn.h:238-240, :257-299),
//   sendBuf adds seq/ack/window/timestamps (TcpConn.h:310-323),
//   SendBuf::setOptDataLen writes tot_len and folds both sums (Core.h:157-163);
//   resendUna patches the folded sum in place (TcpConn.h:771-785), sumRst builds
//   RST / TIME_WAIT ACKs the same way (Core.h:385-398).  Efvi's UDP sender caches the
//   IPv4 header sum once and folds it with each length (Efvi.h:405-411, 611-621).
// Every one of those sums is congruent (mod 0xFFFF) to the plain RFC 1071 word sum of
// the bytes that end up in the frame and is never 0, so CSum::fold of either gives the
// same 16 bits: the kernel recomputes both checksums from the frame
// bytes in one HBM pass and writes the values the reference's incremental path writes.
// Efvi's cached fold is not CSum::fold: when the first end-around step of the cached
// header sum carries, `cache += cache >> 16` keeps the carry bit and adds it again, so
// the cache is one too large and the header checksum written with it does not verify
// (DESIGN.md §12).  PN_TX_UDP_EFVI reproduces Efvi bit for bit, defect included;
// PN_TX_UDP writes the same fields with CSum::fold (equal to Efvi everywhere else).
//
// Two launches per call:
//  tx_fill_kernel   rx_kernel.hip's frame pass (frame_pass.hpp) — one wave per 64
//                   slots, header window per lane, wave-wide 1-KiB streaming of each
//                   frame's segment with exact dot2 word sums — then one 8-B patch
//                   record per frame (the field values), written coalesced to ctx
//                   scratch.  No write touches the frames here.
//  tx_patch_kernel  one lane per frame writes its 2-byte fields into the frame.
// Writing the fields in place from the first kernel costs 33-46 % of its time (DRAM
// read/write interleaving over 1 Mi partially written lines); as a separate short
// phase the same stores cost 22 % (profiles/r01_experiments/tx_variants_*.json).
// HBM-bound: reads tot_len bytes (+ the Ethernet line head), writes 4-8 bytes.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "../../include/pollnet_amd.h"
#include "device_common.hpp"
#include "frame_pass.hpp"
#include "pn_internal.hpp"

namespace {

using namespace pn_dev;
using pn_internal::hip_err;
using pn_internal::set_err;

struct TArgs {
  uint8_t* frames;
  const uint16_t* lens; // setOptDataLen's len / update_udp_pkt's paylen per frame, or nullptr
  uint32_t n;
  uint32_t stride;
  uint32_t ipa_off;  // (frame_off + 14) & ~15
  uint32_t avail;    // stride - frame_off
  uint32_t frame_off;
  uint2* patch;      // n patch records (ctx scratch)
  uint32_t fpw = kFramesPerWave; // frames per wave (8..64, frames_per_wave)
  uint32_t* sig_count = nullptr;  // SIG (pn_tx_fill_notify): workgroups finished, device memory
  uint32_t* sig_flag = nullptr;   // SIG: host-visible word the last workgroup sets to sig_token
  uint32_t sig_token = 0;
};

// Patch record: x = ip checksum | (tcp checksum or udp_len) << 16, y = tot_len word | flags << 16
constexpr uint32_t kPatchOk = 1u << 16, kPatchLen = 2u << 16;

__device__ __forceinline__ void st16(uint8_t* p, uint32_t v) { *reinterpret_cast<uint16_t*>(p) = (uint16_t)v; }

// Where the field values go.  WB = -2 (production above kTxInPlaceMaxFrames): the patch record.
// WB = 0 (production up to it): 2-byte stores straight into the frame.  Tuning variants
// (scripts/tx_variants.py): WB = 128 patch the cooperative LDS tile and write back the slot's
// whole first line; WB = -1 nothing.
constexpr int kWbPatch = -2;

// MODE: PN_TX_TCP, PN_TX_UDP_EFVI or PN_TX_UDP.
// PADK (tuning): KiB of LDS padding per workgroup (caps workgroups per CU, as the RX
// kernel's 2-KiB pad does: 10 KiB = 4 waves/SIMD).
// SABL: the stream phase's options.  Every stream load is issued (kExactRange): TX batches are
// mostly full-size frames, where skipping empty loads measured 1.8 % slower at frame_off 2 and
// equal at 14 (tuning variant 42 = with kSkipEmptyLoads, profiles/r02/s3/tx_skip_ab_off*.json).
// The window loads go out one round trip apart (kSerialWindow), not all at once as in the RX kernel:
// the fill measured 1.3 % faster that way at frame_off 2 and 2.5 % at 14, both variant orders, 4 rotating
// batches (tuning variants 40 vs 43, profiles/r03/window/tx_window_off*.json).  Phase 2 pipelined by half
// batches as in the RX kernel gained 0.1-0.2 % here (profiles/r03/pipe_stream/tx_pipe_*.json): not taken.
// SIG: completion word (pn_tx_fill_notify, signal_done in frame_pass.hpp).
constexpr int kTxStream = kExactRange | kSerialWindow;
template <int MIS, int COOP, int MODE, int WB = kWbPatch, int SAUX = 0, int LAUX0 = 0, int PADK = 0, bool XCD = false,
          int SABL = kTxStream, bool SIG = false>
__global__ __launch_bounds__(kWave, 5) void tx_fill_kernel(TArgs a) {
  const int lane = threadIdx.x;
  const uint32_t wave_base = (XCD ? xcd_group(blockIdx.x, gridDim.x) : blockIdx.x) * a.fpw;
  if constexpr (PADK > 0) {
    __shared__ uint32_t pad_lds[PADK * 256];
    pad_lds[lane] = lane;
    // never true: keeps the padding allocated.  Wave-uniform (readfirstlane) so a.n stays scalar: a
    // per-lane write would make the descriptors built from it divergent (waterfall loops, as in the RX
    // kernel's pad test before round 3)
    if (__builtin_amdgcn_readfirstlane(pad_lds[(lane + 1) & 63]) == 0x7fffffffu) a.n = 0;
  }
  if (wave_base >= a.n) return;
  const uint32_t f = wave_base + lane;
  const uint32_t n_here = min(a.fpw, a.n - wave_base);
  const bool live = (uint32_t)lane < n_here;
  uint8_t* wave_slot = a.frames + (uint64_t)wave_base * a.stride;
  const __amdgpu_buffer_rsrc_t rs = frame_rsrc(wave_slot, n_here * a.stride);

  // LAUX0: the line-0 window loads keep the default policy (not nt), so the line the
  // patch kernel later writes is still in the memory-side cache
  Window h;
  (void)load_window_strided<MIS, COOP, LAUX0, (SABL & kSerialWindow) != 0>(rs, lane, a.stride, a.ipa_off,
                                                                           (uint32_t)(uintptr_t)wave_slot, h);
  uint8_t* ip = wave_slot + (uint64_t)lane * a.stride + a.ipa_off + MIS;

  // IpHeader (Core.h:57-69): tot_len at ip+2, checksum at ip+10
  const uint32_t tot_word_old = h.template u16<MIS + 2>();
  const uint32_t ip_chk_old = h.template u16<MIS + 10>();
  uint32_t tot = bswap16(tot_word_old);
  constexpr bool UDP = MODE != PN_TX_TCP;
  constexpr uint32_t kHdr = UDP ? 28 : 40; // ip + udp / ip + tcp without options
  const bool has_len = a.lens != nullptr;
  uint32_t len = 0;
  if (has_len && live) {
    len = a.lens[f];
    tot = (kHdr + len) & 0xffff; // htons(40 + len) (Core.h:158), htons(28 + paylen) (Efvi.h:615)
  }
  const bool ok = live && tot >= kHdr && 14 + tot <= a.avail;
  const uint32_t tot_word = bswap16(tot);
  const uint32_t s_ip_stored = h.template sum16<MIS, MIS + 20>(); // the 20 bytes as they are in memory
  // the header's words with checksum 0 and the new tot_len (exact: both removed words are terms of s_ip_stored)
  const uint32_t s_ip = s_ip_stored - ip_chk_old - tot_word_old + tot_word;

  uint32_t ip_chk, l4; // l4: tcp checksum (TCP) or udp_len word (UDP)
  if constexpr (UDP) {
    if constexpr (MODE == PN_TX_UDP_EFVI) {
      // Efvi: ipsum_cache over the header with tot_len = check = 0 (Efvi.h:405-411), then
      // ipsum = cache + iplen; ipsum += ipsum >> 16; check = ~ipsum & 0xffff (Efvi.h:615-617)
      uint32_t cache = s_ip - tot_word;
      cache = (cache >> 16) + (cache & 0xffff);
      cache += cache >> 16;
      uint32_t ipsum = cache + tot_word;
      ipsum += ipsum >> 16;
      ip_chk = ~ipsum & 0xffff;
    } else {
      ip_chk = csum_fold(s_ip);
    }
    l4 = bswap16((8 + len) & 0xffff); // udp_len = htons(8 + paylen) (Efvi.h:618)
  } else {
    // summed extent [ip, ip + tot) rounded up to a whole word; bit 0 flags an odd tot_len,
    // whose last word holds the byte after the segment (zero-padded in the sum: copyAndSum
    // adds a trailing odd byte as the low byte of a word, TcpConn.h:291-295)
    const uint32_t even_end = MIS + ((tot + 1) & ~1u);
    const int end_rel = ok ? (int)(even_end | (tot & 1)) : 0;
    uint32_t t_all = window_part<MIS>(h, end_rel & ~1, stream_start((uint64_t)(ip - MIS)));
    uint32_t pad = kPadUnknown;
    stream_phase<SABL, kLoadAux, 0>(a.stride, wave_slot + a.ipa_off, 0, n_here, lane, end_rel, t_all, pad);
    if (ok && (tot & 1) && pad == kPadUnknown) pad = ip[tot]; // pad byte inside the window
    const uint32_t tcp_chk_old = h.template u16<MIS + 36>(); // TcpHeader.checksum at tcp+16 (Core.h:84)
    const uint32_t s_seg = t_all - s_ip_stored - tcp_chk_old - ((tot & 1) ? (pad << 8) : 0u);
    const uint32_t src_ip = h.template u32<MIS + 12>(), dst_ip = h.template u32<MIS + 16>();
    const uint32_t s_addr = (src_ip >> 16) + (src_ip & 0xffff) + (dst_ip >> 16) + (dst_ip & 0xffff);
    // pseudo-header: src, dst, ntohs(6), htons(20 + len) (TcpConn.h:165-167, Core.h:160)
    l4 = csum_fold(s_addr + 0x0600 + bswap16(tot - 20) + s_seg);
    ip_chk = csum_fold(s_ip);
  }

  if constexpr (WB == kWbPatch) {
    if (live) {
      const uint2 rec = {ip_chk | (l4 << 16), tot_word | (ok ? kPatchOk : 0u) | (has_len ? kPatchLen : 0u)};
      a.patch[f] = rec; // one coalesced 512-B store per wave
    }
  } else if constexpr (WB == -3) { // timing only: a 16-B record per frame (RX's record size), plain store
    if (live) reinterpret_cast<u32x4*>(a.patch)[f] = u32x4{ip_chk, l4, tot_word, f};
  } else if constexpr (WB == -4) { // timing only: the 16-B record through RX's buffer store (sc1)
    if (live) {
      // the wave's 64-record block: wave-uniform (readfirstlane), so the descriptor stays scalar
      const uint32_t blk = __builtin_amdgcn_readfirstlane(f & ~63u);
      const __amdgpu_buffer_rsrc_t ro = frame_rsrc((const uint8_t*)(a.patch + 2 * blk), 64 * 16);
      __builtin_amdgcn_raw_buffer_store_b128(u32x4{ip_chk, l4, tot_word, f}, ro, (f & 63u) * 16, 0, kStoreAux);
    }
  } else {
    constexpr int L4 = UDP ? 24 : 36;
    constexpr bool kTile = COOP && WB > 0;
    auto put = [&](auto o_tag, uint32_t v) {
      constexpr int O = decltype(o_tag)::value;
      if constexpr (WB < 0) {
        if (v == 0xbeefu) st16(ip + O, v); // rarely (writes the right value): keeps the sums live
      } else if constexpr (kTile) {
        constexpr int L = 16 + MIS + O; // line offset of the field
        uint16_t* row = reinterpret_cast<uint16_t*>(coop_tile() + lane * 8 + ((L >> 4) ^ (lane & 7)));
        row[(L & 15) >> 1] = (uint16_t)v;
      } else {
        st16(ip + O, v);
      }
    };
    if (ok) {
      if (has_len) put(std::integral_constant<int, 2>{}, tot_word);
      put(std::integral_constant<int, 10>{}, ip_chk);
      if (!UDP || has_len) put(std::integral_constant<int, L4>{}, l4);
    }
    if constexpr (kTile) { // write the patched lines back, 8 lanes per 128-B line
      __syncthreads();
      u32x4* tile = coop_tile();
      const uint32_t line0 = coop_block(a.ipa_off);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint32_t r = 8 * i + (lane >> 3), part = lane & 7;
        __builtin_amdgcn_raw_buffer_store_b128(tile[r * 8 + (part ^ (r & 7))], rs, r * a.stride + line0 + 16 * part, 0,
                                               SAUX);
      }
    }
  }
  if constexpr (SIG) signal_done(a.sig_count, a.sig_flag, a.sig_token, lane);
}

// Phase 2: one lane per frame writes the fields its patch record carries.
// PV (tuning, scripts/tx_variants.py): 0 plain 2-byte stores (production); 1 the same with
// the nt policy.  (Global stores: a per-lane buffer descriptor would be waterfalled.)
template <int MODE, int PV = 0>
__global__ __launch_bounds__(256) void tx_patch_kernel(TArgs a) {
  const uint32_t f = blockIdx.x * 256 + threadIdx.x;
  if (f >= a.n) return;
  const uint2 rec = a.patch[f];
  if (!(rec.y & kPatchOk)) return;
  uint8_t* ip = a.frames + (uint64_t)f * a.stride + a.frame_off + 14;
  if constexpr (PV == 0) {
    if (rec.y & kPatchLen) st16(ip + 2, rec.y);
    st16(ip + 10, rec.x);
    if constexpr (MODE == PN_TX_TCP) st16(ip + 36, rec.x >> 16);
    else if (rec.y & kPatchLen) st16(ip + 24, rec.x >> 16);
  } else { // nt 2-byte stores (PV == 1)
    if (rec.y & kPatchLen) __builtin_nontemporal_store((uint16_t)rec.y, reinterpret_cast<uint16_t*>(ip + 2));
    __builtin_nontemporal_store((uint16_t)rec.x, reinterpret_cast<uint16_t*>(ip + 10));
    if constexpr (MODE == PN_TX_TCP) __builtin_nontemporal_store((uint16_t)(rec.x >> 16), reinterpret_cast<uint16_t*>(ip + 36));
    else if (rec.y & kPatchLen) __builtin_nontemporal_store((uint16_t)(rec.x >> 16), reinterpret_cast<uint16_t*>(ip + 24));
  }
}

// Timing-only probe (tuning): each frame's first B bytes of the 64-B-aligned region holding
// ip+10 written in full (B/16 lanes per frame, 16 B each), no read, garbage values.
template <int B>
__global__ __launch_bounds__(256) void tx_probe_fullwrite_kernel(TArgs a) {
  constexpr int L = B / 16;
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  const uint32_t f = t / L, part = t % L;
  if (f >= a.n) return;
  const uint64_t ip = (uint64_t)(a.frames + (uint64_t)f * a.stride + a.frame_off + 14);
  const uint64_t q = ((ip + 10) & ~(uint64_t)(B - 1)) + 16 * part;
  *reinterpret_cast<u32x4*>(q) = u32x4{f, part, 0u, 0u};
}

// Phase 2, whole-sector form (tuning): 8 lanes per frame rewrite each 64-B sector that holds
// a field (the sector read back, the fields patched in registers, 16 B per lane), so the
// memory sees full-sector writes instead of 2-byte masked ones.  Valid only where those
// sectors lie inside the frame's own slot and nothing else writes them meanwhile.
// SAUX: store policy (0 plain, 2 nt).
template <int SAUX>
__global__ __launch_bounds__(256) void tx_patch_sector_kernel(TArgs a) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  const uint32_t f = t >> 3, part = t & 7;
  if (f >= a.n) return;
  const uint2 rec = a.patch[f];
  if (!(rec.y & kPatchOk)) return;
  uint8_t* slot = a.frames + (uint64_t)f * a.stride;
  const uint64_t ip = (uint64_t)(slot + a.frame_off + 14);
  const uint64_t sa = (ip + 10) & ~63ull, sb = (ip + 36) & ~63ull; // sectors of the two checksum fields
  const uint64_t sec = part < 4 ? sa : sb;
  if (part >= 4 && sb == sa) return;
  const uint64_t q = sec + 16 * (part & 3);
  u32x4 v = *reinterpret_cast<const u32x4*>(q);
  auto patch16 = [&](uint64_t at, uint32_t val) { // a 2-byte field at address `at`, if inside this quad
    if (at >= q && at < q + 16) {
      const uint32_t o = (uint32_t)(at - q), w = o >> 2, sh = (o & 2) * 8;
      uint32_t* d = reinterpret_cast<uint32_t*>(&v);
      d[w] = (d[w] & ~(0xffffu << sh)) | ((val & 0xffffu) << sh);
    }
  };
  if (rec.y & kPatchLen) patch16(ip + 2, rec.y);
  patch16(ip + 10, rec.x);
  patch16(ip + 36, rec.x >> 16);
  if constexpr (SAUX == 2) __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(q));
  else *reinterpret_cast<u32x4*>(q) = v;
}

// Phase 2 with write-through stores (tuning, round 5: the offset-14 write pattern).  System-scope
// stores (sc0 sc1) go through L2 to the memory side at once, so the dirty sectors leave during this short
// phase instead of being written back while the next call streams its reads.  FORM 0: the 2-byte fields;
// FORM 1: each 64-B sector holding a field rewritten whole from a re-read (8 lanes per frame, 16 B each), so
// every write request is a full aligned 64-B one.
__device__ __forceinline__ void st16_wt(uint8_t* p, uint32_t v) {
  asm volatile("global_store_short %0, %1, off sc0 sc1" : : "v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ void st128_wt(uint8_t* p, u32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" : : "v"(p), "v"(v) : "memory");
}
template <int MODE, int FORM>
__global__ __launch_bounds__(256) void tx_patch_wt_kernel(TArgs a) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  if constexpr (FORM == 0) {
    const uint32_t f = t;
    if (f >= a.n) return;
    const uint2 rec = a.patch[f];
    if (!(rec.y & kPatchOk)) return;
    uint8_t* ip = a.frames + (uint64_t)f * a.stride + a.frame_off + 14;
    if (rec.y & kPatchLen) st16_wt(ip + 2, rec.y & 0xffff);
    st16_wt(ip + 10, rec.x & 0xffff);
    if constexpr (MODE == PN_TX_TCP) st16_wt(ip + 36, rec.x >> 16);
  } else {
    const uint32_t f = t >> 3, part = t & 7;
    if (f >= a.n) return;
    const uint2 rec = a.patch[f];
    if (!(rec.y & kPatchOk)) return;
    uint8_t* slot = a.frames + (uint64_t)f * a.stride;
    const uint64_t ip = (uint64_t)(slot + a.frame_off + 14);
    const uint64_t sa = (ip + 10) & ~63ull, sb = (ip + 36) & ~63ull;
    const uint64_t sec = part < 4 ? sa : sb;
    if (part >= 4 && sb == sa) return;
    const uint64_t q = sec + 16 * (part & 3);
    u32x4 v = *reinterpret_cast<const u32x4*>(q);
    auto patch16 = [&](uint64_t at, uint32_t val) {
      if (at >= q && at < q + 16) {
        const uint32_t o = (uint32_t)(at - q), w = o >> 2, sh = (o & 2) * 8;
        uint32_t* d = reinterpret_cast<uint32_t*>(&v);
        d[w] = (d[w] & ~(0xffffu << sh)) | ((val & 0xffffu) << sh);
      }
    };
    if (rec.y & kPatchLen) patch16(ip + 2, rec.y);
    patch16(ip + 10, rec.x);
    patch16(ip + 36, rec.x >> 16);
    st128_wt(reinterpret_cast<uint8_t*>(q), v);
  }
}

inline bool coop_layout(const TArgs& a) {
  return (a.stride % 16) == 0 && a.ipa_off >= 16 && ((uintptr_t)a.frames % 16) == 0;
}

// Up to this many frames a call is ONE launch writing the fields in place: the batch's lines
// are still cached when they are written, and the patch launch's ≈2-µs boundary is the larger
// cost (1.5-4.6 µs less per call from 16 to 65,536 frames, pinned host or device memory,
// bench/bench_tx_small, profiles/r02/tx_fill_small_batches.json).  Above it the two phases
// (§12: the in-place writes' write-back would land in the rest of the stream).
constexpr uint32_t kTxInPlaceMaxFrames = 65536;

template <int MIS, int MODE, int WB, bool SIG = false>
void launch(const TArgs& a, hipStream_t s) {
  const dim3 grid((a.n + a.fpw - 1) / a.fpw), block(kWave);
  // XCD-contiguous group order, as the RX kernel: -1.7 % (profiles/r01_experiments/tx_xcd_order_off{2,14}.json)
  if (coop_layout(a)) {
    hipLaunchKernelGGL((tx_fill_kernel<MIS, 1, MODE, WB, 0, 0, 0, true, kTxStream, SIG>), grid, block, 0, s, a);
    return;
  }
  hipLaunchKernelGGL((tx_fill_kernel<MIS, 0, MODE, WB, 0, 0, 0, true, kTxStream, SIG>), grid, block, 0, s, a);
}

template <int MODE, int WB, bool SIG = false>
void launch_mis(const TArgs& a, uint32_t mis, hipStream_t s) {
  switch (mis) {
    case 0: launch<0, MODE, WB, SIG>(a, s); break;
    case 2: launch<2, MODE, WB, SIG>(a, s); break;
    case 4: launch<4, MODE, WB, SIG>(a, s); break;
    case 6: launch<6, MODE, WB, SIG>(a, s); break;
    case 8: launch<8, MODE, WB, SIG>(a, s); break;
    case 10: launch<10, MODE, WB, SIG>(a, s); break;
    case 12: launch<12, MODE, WB, SIG>(a, s); break;
    default: launch<14, MODE, WB, SIG>(a, s); break;
  }
}

template <int MODE>
void launch_mode(const TArgs& a, uint32_t mis, hipStream_t s) {
  if (a.n <= kTxInPlaceMaxFrames) {
    launch_mis<MODE, 0>(a, mis, s);
    return;
  }
  launch_mis<MODE, kWbPatch>(a, mis, s);
  hipLaunchKernelGGL((tx_patch_kernel<MODE>), dim3((a.n + 255) / 256), dim3(256), 0, s, a);
}

inline int check_args(pn_ctx* ctx, void* frames, uint32_t slot_stride, uint32_t frame_off, const uint16_t* lens) {
  if (!frames) return set_err(ctx, PN_EINVAL, "pn_tx_fill: NULL frames");
  if (((uintptr_t)frames & 15) || ((uintptr_t)lens & 1))
    return set_err(ctx, PN_EINVAL, "pn_tx_fill: frames must be 16-byte, lens 2-byte aligned");
  if ((slot_stride & 15) || slot_stride > 65536 || (frame_off & 1) || slot_stride < frame_off + 96)
    return set_err(ctx, PN_EINVAL, "pn_tx_fill: slot_stride/frame_off violate the layout contract");
  return PN_OK;
}

// ctx-owned patch scratch, grown on demand.  A call on another stream than the previous
// scratch user is ordered after it on the device (pn_fence: no per-launch event, no host wait);
// growing it waits on the host for that user before the old scratch is freed.
inline int ensure_patch(pn_ctx* ctx, uint32_t n, hipStream_t s) {
  if (n > ctx->tx_patch_n) {
    if (ctx->tx_patch) {
      const int rc = pn_internal::fence_host_wait(ctx, ctx->tx);
      if (rc) return rc;
      (void)hipFree(ctx->tx_patch);
      ctx->tx_patch = nullptr;
      ctx->tx_patch_n = 0;
    }
    const uint32_t cap = n < (1u << 16) ? (1u << 16) : n;
    hipError_t e = hipMalloc(&ctx->tx_patch, (size_t)cap * sizeof(uint2));
    if (e != hipSuccess) return hip_err(ctx, e, "hipMalloc(tx patch scratch)");
    ctx->tx_patch_n = cap;
  }
  return pn_internal::fence_use(ctx, ctx->tx, s);
}

} // namespace
