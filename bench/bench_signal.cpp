// Completion by a polled word vs stream synchronisation, for small batches.
//   sync    pn_classify + hipStreamSynchronize (what GpuRx / the drop-in server do)
//   signal  pn_classify_notify: the kernel's last workgroup stores a token to a host-visible
//           word once every record is stored and visible; the host spins on it
//   service the resident classify service (pn_service_post + pn_service_wait): no launch per batch
// C2 frames (1514 B) and the generator's table; batches of 64..1024 frames, device-resident
// (records to device memory) and zero-copy (pinned slots, records to pinned memory).  Host wall
// clock per batch, median of `reps`, the two forms interleaved; records compared.  One JSON line.
// (built by `make bench/bench_signal`)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../include/pollnet_amd_gen.h"
#include "../include/pollnet_amd/gpu_rx.hpp"

using Clock = std::chrono::steady_clock;

static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char** argv) {
  const uint32_t reps = argc > 1 ? std::atoi(argv[1]) : 400;
  const uint32_t stride = 2048, off = 2, nmax = 1024;
  pn_gen_params gp{2, 1, 0, 1024, 7};
  std::vector<uint8_t> frames((size_t)stride * nmax);
  if (pn_gen_frames(&gp, 0, nmax, frames.data(), stride, off, 8)) return 3;
  pn_conn_table* t = nullptr;
  if (pn_table_create(1024, 1024, &t) || pn_gen_conn_table(&gp, t)) return 3;
  pn_ctx* ctx = nullptr;
  if (pn_open(0, &ctx)) return std::fprintf(stderr, "%s\n", pn_last_error(nullptr)), 4;
  uint32_t ne = 0;
  uint64_t mask = 0;
  const pn_conn_entry* e = pn_table_entries(t, &ne, &mask);
  if (pn_set_conn_table(ctx, e, ne, mask, 1024)) return 4;
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 4;
  uint8_t *d_frames = nullptr, *h_frames = nullptr;
  pn_result *d_rec = nullptr, *h_rec = nullptr, *h_rec2 = nullptr;
  uint32_t* flag = nullptr;
  if (hipMalloc((void**)&d_frames, frames.size()) != hipSuccess || hipMalloc((void**)&d_rec, 16 * nmax) != hipSuccess ||
      hipHostMalloc((void**)&h_frames, frames.size(), hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc((void**)&h_rec, 16 * nmax, hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc((void**)&h_rec2, 16 * nmax, hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc((void**)&flag, 64, hipHostMallocDefault) != hipSuccess)
    return 5;
  std::memcpy(h_frames, frames.data(), frames.size());
  if (hipMemcpy(d_frames, frames.data(), frames.size(), hipMemcpyHostToDevice) != hipSuccess) return 5;
  *flag = 0;
  uint32_t token = 0;
  pn_service* svc = nullptr;
  if (pn_service_open(ctx, stride, off, 2000, &svc)) return std::fprintf(stderr, "%s\n", pn_last_error(ctx)), 4;
  uint16_t* h_links = nullptr; // the chain links of a linked post (pn_service_post_linked)
  if (hipHostMalloc((void**)&h_links, 2 * 1024, hipHostMallocDefault) != hipSuccess) return 3;
  bool ok = true;
  std::string out = "{\"bench\": \"completion_word_vs_stream_sync\", \"frames\": \"C2 1514-B\"";
  // both checksums verified, then the release path (pn_set_verify(ctx, 0): header lines only)
  for (int verify = 1; verify >= 0 && ok; verify--)
  for (int zc = 0; zc < 2; zc++) {
    if (pn_set_verify(ctx, verify)) return 4;
    const uint8_t* fr = zc ? h_frames : d_frames;
    pn_result* rec = zc ? h_rec : d_rec;
    auto sync_once = [&](uint32_t n) {
      return pn_classify(ctx, fr, stride, off, n, rec, s) == 0 && hipStreamSynchronize(s) == hipSuccess;
    };
    auto signal_once = [&](uint32_t n) {
      const uint32_t tok = ++token;
      if (pn_classify_notify(ctx, fr, stride, off, n, rec, s, flag, tok)) return false;
      return pollnet_amd::wait_word(flag, tok, s) == nullptr;
    };
    auto service_once = [&](uint32_t n) { return pn_service_post(svc, fr, n, rec, nullptr) == 0 && pn_service_wait(svc, 0) == 0; };
    auto linked_once = [&](uint32_t n) {
      return pn_service_post_linked(svc, fr, n, rec, h_links, nullptr) == 0 && pn_service_wait(svc, 0) == 0;
    };
    std::string legs;
    for (uint32_t n : {64u, 512u, 1024u}) {
      // records equal: the signalled batch's records (zero-copy: read right after the word) vs sync's
      ok = ok && sync_once(n);
      if (zc) std::memcpy(h_rec2, h_rec, 16 * n);
      else ok = ok && hipMemcpy(h_rec2, d_rec, 16 * n, hipMemcpyDeviceToHost) == hipSuccess;
      std::memset(h_rec, 0, 16 * n);
      if (!zc) ok = ok && hipMemset(d_rec, 0, 16 * n) == hipSuccess && hipDeviceSynchronize() == hipSuccess;
      ok = ok && signal_once(n);
      bool same;
      if (zc) {
        same = std::memcmp(h_rec, h_rec2, 16 * n) == 0;
      } else {
        std::vector<pn_result> tmp(n);
        ok = ok && hipStreamSynchronize(s) == hipSuccess &&
             hipMemcpy(tmp.data(), d_rec, 16 * n, hipMemcpyDeviceToHost) == hipSuccess;
        same = std::memcmp(tmp.data(), h_rec2, 16 * n) == 0;
      }
      ok = ok && same;
      ok = ok && hipStreamSynchronize(s) == hipSuccess;
      // the service's records for the same batch
      std::memset(h_rec, 0, 16 * n);
      if (!zc) ok = ok && hipMemset(d_rec, 0, 16 * n) == hipSuccess && hipDeviceSynchronize() == hipSuccess;
      ok = ok && service_once(n);
      bool same_svc;
      if (zc) {
        same_svc = std::memcmp(h_rec, h_rec2, 16 * n) == 0;
      } else {
        std::vector<pn_result> tmp(n);
        ok = ok && hipMemcpy(tmp.data(), d_rec, 16 * n, hipMemcpyDeviceToHost) == hipSuccess;
        same_svc = std::memcmp(tmp.data(), h_rec2, 16 * n) == 0;
      }
      ok = ok && same_svc;
      std::vector<double> ts, tg, tv, tl;
      for (int w = 0; w < 20; w++) ok = ok && sync_once(n) && signal_once(n) && service_once(n) && linked_once(n);
      ok = ok && hipStreamSynchronize(s) == hipSuccess;
      for (uint32_t r = 0; r < reps && ok; r++) {
        auto t0 = Clock::now();
        ok = ok && sync_once(n);
        auto t1 = Clock::now();
        ok = ok && signal_once(n);
        auto t2 = Clock::now();
        ok = ok && hipStreamSynchronize(s) == hipSuccess; // the signalled launch has drained
        auto t3 = Clock::now();
        ok = ok && service_once(n);
        auto t4 = Clock::now();
        ok = ok && linked_once(n);
        auto t5 = Clock::now();
        tl.push_back(std::chrono::duration<double, std::micro>(t5 - t4).count());
        ts.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
        tg.push_back(std::chrono::duration<double, std::micro>(t2 - t1).count());
        tv.push_back(std::chrono::duration<double, std::micro>(t4 - t3).count());
      }
      if (!ok) break;
      char buf[384];
      std::snprintf(buf, sizeof buf,
                    "%s\"%u\": {\"sync_us\": %.2f, \"signal_us\": %.2f, \"service_us\": %.2f, \"service_linked_us\": %.2f, "
                    "\"records_equal\": %s}",
                    legs.empty() ? "" : ", ", n, median(ts), median(tg), median(tv), median(tl),
                    same && same_svc ? "true" : "false");
      legs += buf;
    }
    out += std::string(", \"") + (zc ? "zero_copy" : "resident") + (verify ? "" : "_release_path") + "\": {" + legs + "}";
  }
  out += std::string(", \"ok\": ") + (ok ? "true" : "false") + "}";
  std::printf("%s\n", out.c_str());
  (void)hipStreamSynchronize(s);
  if (pn_service_close(svc)) ok = false;
  (void)hipHostFree(h_links);
  pn_close(ctx);
  return ok ? 0 : 1;
}
