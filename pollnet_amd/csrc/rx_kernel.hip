// MI355X (gfx950) receive-path per-frame transform: the product C-ABI (pn_open /
// pn_set_conn_table / pn_classify / pn_classify_indexed / pn_sync).  The kernel itself
// and its execution model are in rx_classify.hpp; the tuning variants and bandwidth
// ceilings live in the separate libpollnet_amd_tuning.so (rx_tuning.hip).
#include "rx_classify.hpp"

namespace {
using pn_internal::g_err;
using pn_internal::hip_err;
using pn_internal::set_err;

// Argument checks and kernel arguments shared by pn_classify and pn_classify_notify.
int strided_args(pn_ctx* ctx, const char* fn, const void* frames_dev, uint32_t slot_stride, uint32_t frame_off,
                 uint32_t n, void* results_dev, KArgs& a) {
  if (!ctx) return set_err(nullptr, PN_EINVAL, std::string(fn) + ": ctx is NULL");
  if (!ctx->tbl_dev) return set_err(ctx, PN_ENOTABLE, std::string(fn) + ": no conn table (call pn_set_conn_table)");
  if (!frames_dev || !results_dev) return set_err(ctx, PN_EINVAL, std::string(fn) + ": NULL buffer");
  if (((uintptr_t)frames_dev & 15) || ((uintptr_t)results_dev & 15))
    return set_err(ctx, PN_EINVAL, std::string(fn) + ": frames/results must be 16-byte aligned");
  if ((slot_stride & 15) || slot_stride > 65536 || (frame_off & 1) || slot_stride < frame_off + 96)
    return set_err(ctx, PN_EINVAL, std::string(fn) + ": slot_stride/frame_off violate the layout contract");
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
  return PN_OK;
}

template <bool SIG, bool HO>
void launch_strided_as(const KArgs& a, uint32_t frame_off, hipStream_t s) {
  switch ((frame_off + 14) & 15) {
    case 0: launch<0, SIG, HO>(a, s); break;
    case 2: launch<2, SIG, HO>(a, s); break;
    case 4: launch<4, SIG, HO>(a, s); break;
    case 6: launch<6, SIG, HO>(a, s); break;
    case 8: launch<8, SIG, HO>(a, s); break;
    case 10: launch<10, SIG, HO>(a, s); break;
    case 12: launch<12, SIG, HO>(a, s); break;
    default: launch<14, SIG, HO>(a, s); break;
  }
}

// the ctx's verify setting picks the full kernel or the header-only one (pn_set_verify)
template <bool SIG>
void launch_strided(const pn_ctx* ctx, const KArgs& a, uint32_t frame_off, hipStream_t s) {
  if (ctx->verify_tcp) launch_strided_as<SIG, false>(a, frame_off, s);
  else launch_strided_as<SIG, true>(a, frame_off, s);
}

template <int A>
void launch_indexed(const KArgs& a, uint32_t eth_mod16, hipStream_t s) {
  switch ((eth_mod16 + 14) & 15) {
    case 0: launch_one<0, 1, A, kLoadAux, kStoreAux, 1, kIdxWin, 1, kXcdOrder>(a, s); break;
    case 2: launch_one<2, 1, A, kLoadAux, kStoreAux, 1, kIdxWin, 1, kXcdOrder>(a, s); break;
    case 4: launch_one<4, 1, A, kLoadAux, kStoreAux, 1, kIdxWin, 1, kXcdOrder>(a, s); break;
    case 6: launch_one<6, 1, A, kLoadAux, kStoreAux, 1, kIdxWin, 1, kXcdOrder>(a, s); break;
    case 8: launch_one<8, 1, A, kLoadAux, kStoreAux, 1, kIdxWin, 1, kXcdOrder>(a, s); break;
    case 10: launch_one<10, 1, A, kLoadAux, kStoreAux, 1, kIdxWin, 1, kXcdOrder>(a, s); break;
    case 12: launch_one<12, 1, A, kLoadAux, kStoreAux, 1, kIdxWin, 1, kXcdOrder>(a, s); break;
    default: launch_one<14, 1, A, kLoadAux, kStoreAux, 1, kIdxWin, 1, kXcdOrder>(a, s); break;
  }
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
  (void)hipSetDevice(ctx->device);
  // teardown: every launch that may still read ctx memory has finished.  A device-wide wait, so
  // that no stream handle is touched (the caller may have destroyed its streams already)
  if (ctx->tbl_buf[0] || ctx->tbl_buf[1] || ctx->tx_patch || ctx->sig_count) (void)hipDeviceSynchronize();
  for (pn_conn_entry* b : ctx->tbl_buf)
    if (b) (void)hipFree(b);
  if (ctx->tx_patch) (void)hipFree(ctx->tx_patch);
  if (ctx->sig_count) (void)hipFree(ctx->sig_count);
  for (hipEvent_t ev : ctx->retired)
    if (ev) (void)hipEventDestroy(ev);
  for (pn_fence* f : {&ctx->sig[0], &ctx->sig[1], &ctx->tx})
    if (f->ev) (void)hipEventDestroy(f->ev);
  if (ctx->copy_stream) (void)hipStreamDestroy(ctx->copy_stream);
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
  // the snapshot goes to the buffer launches are NOT reading now; its own readers (launches
  // issued before the previous set) are waited for by event — normally long done — as are the
  // resident-service posts that captured it (by their done words; the service's kernel never
  // ends between posts, so no event on its stream could say it), and the launches and posts
  // reading the current buffer, on any stream, keep running untouched
  const int nxt = ctx->tbl_dev ? ctx->cur ^ 1 : ctx->cur;
  int rc = pn_internal::svc_release_table(ctx, nxt);
  if (rc) return rc;
  rc = pn_internal::wait_retired(ctx);
  if (rc) return rc;
  if (n_entries > ctx->tbl_cap[nxt]) {
    if (ctx->tbl_buf[nxt]) (void)hipFree(ctx->tbl_buf[nxt]);
    ctx->tbl_buf[nxt] = nullptr;
    ctx->tbl_cap[nxt] = 0;
    e = hipMalloc(&ctx->tbl_buf[nxt], (size_t)n_entries * sizeof(pn_conn_entry));
    if (e != hipSuccess) return hip_err(ctx, e, "hipMalloc(conn table)");
    ctx->tbl_cap[nxt] = n_entries;
  }
  if (!ctx->copy_stream) {
    e = hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking);
    if (e != hipSuccess) return hip_err(ctx, e, "hipStreamCreate(table uploads)");
  }
  e = hipMemcpyAsync(ctx->tbl_buf[nxt], entries, (size_t)n_entries * sizeof(pn_conn_entry), hipMemcpyHostToDevice,
                     ctx->copy_stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->copy_stream);
  if (e != hipSuccess) return hip_err(ctx, e, "hipMemcpyAsync(conn table)");
  // everything launched so far reads (at most) the buffer being retired: mark its end
  rc = pn_internal::retire_streams(ctx);
  if (rc) return rc;
  ctx->cur = nxt;
  ctx->tbl_dev = ctx->tbl_buf[nxt];
  ctx->n_entries = n_entries;
  ctx->mask = tbl_mask;
  ctx->max_conn = max_conn_cnt;
  return PN_OK;
}


int pn_classify(pn_ctx* ctx, const void* frames_dev, uint32_t slot_stride, uint32_t frame_off, uint32_t n,
                void* results_dev, void* stream) {
  if (ctx && n == 0 && ctx->tbl_dev) return PN_OK;
  KArgs a;
  int rc = strided_args(ctx, "pn_classify", frames_dev, slot_stride, frame_off, n, results_dev, a);
  if (rc) return rc;
  if (n == 0) return PN_OK;
  hipStream_t s = (hipStream_t)stream;
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return hip_err(ctx, e, "hipSetDevice");
  launch_strided<false>(ctx, a, frame_off, s);
  e = hipGetLastError();
  if (e != hipSuccess) return hip_err(ctx, e, "rx_classify launch");
  pn_internal::note_stream(ctx, s);
  return PN_OK;
}

int pn_classify_notify(pn_ctx* ctx, const void* frames, uint32_t slot_stride, uint32_t frame_off, uint32_t n,
                       void* results, void* stream, uint32_t* done_word, uint32_t token) {
  KArgs a;
  int rc = strided_args(ctx, "pn_classify_notify", frames, slot_stride, frame_off, n, results, a);
  if (rc) return rc;
  if (n == 0 || n > PN_NOTIFY_MAX_FRAMES || !done_word || ((uintptr_t)done_word & 3))
    return set_err(ctx, PN_EINVAL, "pn_classify_notify: n must be in [1, PN_NOTIFY_MAX_FRAMES], done_word 4-byte aligned");
  hipStream_t s = (hipStream_t)stream;
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return hip_err(ctx, e, "hipSetDevice");
  rc = pn_internal::notify_counter(ctx, 0, s, &a.sig_count);
  if (rc) return rc;
  a.sig_flag = done_word;
  a.sig_token = token;
  launch_strided<true>(ctx, a, frame_off, s);
  e = hipGetLastError();
  if (e != hipSuccess) return hip_err(ctx, e, "rx_classify (notify) launch");
  pn_internal::note_stream(ctx, s);
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
  if (ctx->verify_tcp) launch_indexed<kProdAbl>(a, eth_mod16, s);
  else launch_indexed<kProdAbl | kHeaderOnly>(a, eth_mod16, s);
  e = hipGetLastError();
  if (e != hipSuccess) return hip_err(ctx, e, "rx_classify (indexed) launch");
  pn_internal::note_stream(ctx, s);
  return PN_OK;
}

int pn_set_verify(pn_ctx* ctx, int verify_tcp) {
  if (!ctx) return set_err(nullptr, PN_EINVAL, "pn_set_verify: ctx is NULL");
  ctx->verify_tcp = verify_tcp != 0;
  return PN_OK;
}

int pn_sync(pn_ctx* ctx) {
  if (!ctx) return set_err(nullptr, PN_EINVAL, "pn_sync: ctx is NULL");
  hipError_t e = hipSetDevice(ctx->device);
  if (e != hipSuccess) return hip_err(ctx, e, "hipSetDevice");
  // every stream launched on since the last set, and (by event) everything before it
  for (hipStream_t s : ctx->streams) {
    e = hipStreamSynchronize(s);
    if (e != hipSuccess) return hip_err(ctx, e, "hipStreamSynchronize");
  }
  ctx->streams.clear();
  int rc = pn_internal::wait_retired(ctx);
  if (rc) return rc;
  for (pn_fence* f : {&ctx->sig[0], &ctx->sig[1], &ctx->tx}) f->state = 0;
  return PN_OK;
}

} // extern "C"
