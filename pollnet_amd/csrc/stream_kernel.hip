// TcpStream's packet filter for a whole batch, many streams at once (SURVEY §8(f)
// rank 3).  Reference, per frame and per stream (TcpStream.h:39-52):
//   etherType == 0x0008 (0x0800 read little-endian) && ip.protocol == 6 &&
//   (filter_src_ip == 0 || == ip.ipSrc) && (filter_dst_ip == 0 || == ip.ipDst) &&
//   (filter_src_port == 0 || == tcp.portSrc) && (filter_dst_port == 0 || == tcp.portDst)
// with the IP header assumed 20 bytes (TcpHeaderPos = 14 + 20, TcpStream.h:213-214).
//
// One lane per frame reads only the frame's header bytes (ethertype .. TCP ports: one
// cache line per frame), compares against every filter in the kernel-argument segment
// (scalar loads, wave-uniform) and writes the index of the first stream the frame
// belongs to.  HBM-bound at one line per frame.
#include <hip/hip_runtime.h>

#include "../../include/pollnet_amd.h"
#include "device_common.hpp"
#include "pn_internal.hpp"

namespace {

using namespace pn_dev;
using pn_internal::hip_err;
using pn_internal::set_err;

struct MatchArgs {
  const uint8_t* frames;
  uint32_t* out;
  uint32_t n;
  uint32_t stride;
  uint32_t ipa_off; // (frame_off + 14) & ~15
  uint32_t n_filters;
  pn_stream_filter f[PN_MAX_STREAM_FILTERS];
};

// MIS = (frame_off + 14) % 16: the IP header's offset in its 16-B chunk.  The window
// is the chunk before it (ethertype when MIS < 2) and the 3 chunks from it.
template <int MIS>
__global__ __launch_bounds__(256) void match_streams_kernel(MatchArgs a) {
  const uint32_t f = blockIdx.x * 256 + threadIdx.x;
  if (f >= a.n) return;
  constexpr int kPre = 16; // window starts one chunk before the IP header's chunk
  const __amdgpu_buffer_rsrc_t rs =
      frame_rsrc(a.frames + (uint64_t)f * a.stride + a.ipa_off - kPre, kPre + 48);
  Win<16> h;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * c, 0, 0);
    h.d[4 * c + 0] = v.x;
    h.d[4 * c + 1] = v.y;
    h.d[4 * c + 2] = v.z;
    h.d[4 * c + 3] = v.w;
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
  a.out[f] = id;
}

} // namespace

extern "C" int pn_match_streams(pn_ctx* ctx, const void* frames, uint32_t slot_stride, uint32_t frame_off, uint32_t n,
                                const pn_stream_filter* filters, uint32_t n_filters, uint32_t* stream_ids,
                                void* stream) {
  if (!ctx) return set_err(nullptr, PN_EINVAL, "pn_match_streams: ctx is NULL");
  if (n == 0) return PN_OK;
  if (!frames || !stream_ids || (n_filters && !filters)) return set_err(ctx, PN_EINVAL, "pn_match_streams: NULL buffer");
  if (n_filters > PN_MAX_STREAM_FILTERS)
    return set_err(ctx, PN_EINVAL, "pn_match_streams: at most PN_MAX_STREAM_FILTERS filters");
  if (((uintptr_t)frames & 15) || ((uintptr_t)stream_ids & 3))
    return set_err(ctx, PN_EINVAL, "pn_match_streams: frames must be 16-byte, ids 4-byte aligned");
  if ((slot_stride & 15) || slot_stride > 65536 || (frame_off & 1) || frame_off < 2 || slot_stride < frame_off + 96)
    return set_err(ctx, PN_EINVAL, "pn_match_streams: slot_stride/frame_off violate the layout contract");
  MatchArgs a;
  a.frames = (const uint8_t*)frames;
  a.out = stream_ids;
  a.n = n;
  a.stride = slot_stride;
  a.ipa_off = (frame_off + 14) & ~15u;
  a.n_filters = n_filters;
  for (uint32_t k = 0; k < n_filters; ++k) a.f[k] = filters[k]; // host memory: copied into the kernel arguments
  hipStream_t s = (hipStream_t)stream;
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return hip_err(ctx, e, "hipSetDevice");
  const dim3 grid((n + 255) / 256), block(256);
  switch ((frame_off + 14) & 15) {
    case 0: hipLaunchKernelGGL(match_streams_kernel<0>, grid, block, 0, s, a); break;
    case 2: hipLaunchKernelGGL(match_streams_kernel<2>, grid, block, 0, s, a); break;
    case 4: hipLaunchKernelGGL(match_streams_kernel<4>, grid, block, 0, s, a); break;
    case 6: hipLaunchKernelGGL(match_streams_kernel<6>, grid, block, 0, s, a); break;
    case 8: hipLaunchKernelGGL(match_streams_kernel<8>, grid, block, 0, s, a); break;
    case 10: hipLaunchKernelGGL(match_streams_kernel<10>, grid, block, 0, s, a); break;
    case 12: hipLaunchKernelGGL(match_streams_kernel<12>, grid, block, 0, s, a); break;
    default: hipLaunchKernelGGL(match_streams_kernel<14>, grid, block, 0, s, a); break;
  }
  e = hipGetLastError();
  if (e != hipSuccess) return hip_err(ctx, e, "match_streams launch");
  pn_internal::note_stream(ctx, s);
  return PN_OK;
}
