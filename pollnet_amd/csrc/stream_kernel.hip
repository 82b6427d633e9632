// pn_match_streams: TcpStream's packet filter for a whole batch, many streams at once
// (TcpStream.h:39-52).  The kernel is in stream_match.hpp.
#include "stream_match.hpp"

extern "C" int pn_match_streams(pn_ctx* ctx, const void* frames, uint32_t slot_stride, uint32_t frame_off, uint32_t n,
                                const pn_stream_filter* filters, uint32_t n_filters, uint32_t* stream_ids,
                                void* stream) {
  if (ctx && n == 0) return PN_OK;
  MatchArgs a;
  int rc = match_args(ctx, frames, slot_stride, frame_off, n, filters, n_filters, stream_ids, a);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return hip_err(ctx, e, "hipSetDevice");
  launch_match_mask<kMatchG, kMatchLoadAux, 0, kMatchWPW>(a, frame_off, s);
  e = hipGetLastError();
  if (e != hipSuccess) return hip_err(ctx, e, "match_streams launch");
  pn_internal::note_stream(ctx, s);
  return PN_OK;
}
