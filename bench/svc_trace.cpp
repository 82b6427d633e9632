// Where a resident-service post spends its time on the GPU (measurement build only: `make svc_trace` builds
// ab_libs/trace/libpollnet_amd.so with -DPN_SVC_TRACE, whose service kernels store the device wall clock at each
// step of the post protocol, and this driver against it).  Per post kind: the host's post-to-complete time and the
// device steps relative to wave 0 seeing the post (medians over reps, µs).  Round 6 protocol (every wave reads the
// mailbox itself):
//   w0_acq     wave 0's acquire fence after its mailbox read matched
//   oth_seen   the last of the post's other waves seeing the post;  oth_acq its acquire fence;  oth_args its arguments
//   run_end    the last wave's classify + system fence + done word;  count_end  + its count (counted posts)
//   w0_pub, w0_next: steps of the round-5 protocol (wave 0's hand-off), -1 now
//   argv: reps (300)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../include/pollnet_amd.h"
#include "../include/pollnet_amd_gen.h"

extern "C" int pn_svc_trace_set(uint64_t* host_buf);

using Clock = std::chrono::steady_clock;

static double med(std::vector<double> v) {
  if (v.empty()) return -1;
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char** argv) {
  const uint32_t reps = argc > 1 ? std::atoi(argv[1]) : 300;
  const uint32_t stride = 2048, off = 2, nmax = 1024;
  pn_gen_params gp{2, 1, 0, 1024, 7};
  std::vector<uint8_t> frames((size_t)stride * nmax);
  if (pn_gen_frames(&gp, 0, nmax, frames.data(), stride, off, 8)) return 3;
  pn_conn_table* t = nullptr;
  if (pn_table_create(1024, 1024, &t) || pn_gen_conn_table(&gp, t)) return 3;
  pn_ctx* ctx = nullptr;
  if (pn_open(0, &ctx)) return 4;
  uint32_t ne = 0;
  uint64_t mask = 0;
  const pn_conn_entry* e = pn_table_entries(t, &ne, &mask);
  if (pn_set_conn_table(ctx, e, ne, mask, 1024)) return 4;
  uint8_t *d_frames = nullptr, *h_frames = nullptr;
  pn_result *d_rec = nullptr, *h_rec = nullptr;
  uint64_t* tr = nullptr;
  if (hipMalloc((void**)&d_frames, frames.size()) != hipSuccess || hipMalloc((void**)&d_rec, 16 * nmax) != hipSuccess ||
      hipHostMalloc((void**)&h_frames, frames.size(), hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc((void**)&h_rec, 16 * nmax, hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc((void**)&tr, 64 * 8 * 8, hipHostMallocDefault) != hipSuccess)
    return 5;
  std::memcpy(h_frames, frames.data(), frames.size());
  if (hipMemcpy(d_frames, frames.data(), frames.size(), hipMemcpyHostToDevice) != hipSuccess) return 5;
  if (pn_svc_trace_set(tr)) return 6;
  pn_service* svc = nullptr;
  if (pn_service_open(ctx, stride, off, 2000, &svc)) return std::fprintf(stderr, "%s\n", pn_last_error(ctx)), 4;
  std::string out = "{\"bench\": \"service_post_steps\", \"unit\": \"us, device wall clock, median\"";
  bool ok = true;
  struct Kind { const char* name; int verify; int zc; uint32_t n; };
  const Kind kinds[] = {{"resident_release_64", 0, 0, 64},  {"resident_release_512", 0, 0, 512},
                        {"resident_verified_64", 1, 0, 64}, {"resident_verified_512", 1, 0, 512},
                        {"zero_copy_release_64", 0, 1, 64}, {"zero_copy_release_512", 0, 1, 512},
                        {"zero_copy_verified_64", 1, 1, 64}};
  for (const Kind& kd : kinds) {
    if (pn_set_verify(ctx, kd.verify)) return 4;
    const uint8_t* fr = kd.zc ? h_frames : d_frames;
    pn_result* rec = kd.zc ? h_rec : d_rec;
    for (int w = 0; w < 20 && ok; w++) ok = pn_service_post(svc, fr, kd.n, rec, nullptr) == 0 && pn_service_wait(svc, 0) == 0;
    std::vector<double> host, w0_acq, w0_pub, oth_seen, oth_acq, oth_args, run_end, count_end, w0_next;
    uint32_t waves = 0;
    for (uint32_t r = 0; r < reps && ok; r++) {
      std::memset(tr, 0, 64 * 8 * 8);
      std::this_thread::sleep_for(std::chrono::microseconds(30)); // the memset reaches memory; the service idles
      const auto t0 = Clock::now();
      ok = pn_service_post(svc, fr, kd.n, rec, nullptr) == 0 && pn_service_wait(svc, 0) == 0;
      host.push_back(std::chrono::duration<double, std::micro>(Clock::now() - t0).count());
      std::this_thread::sleep_for(std::chrono::microseconds(60)); // the trailing clock stores arrive
      const auto T = [&](int w, int i) { return __atomic_load_n(tr + w * 8 + i, __ATOMIC_ACQUIRE); };
      const uint64_t base = T(0, 0);
      if (!base) continue;
      const auto us = [&](uint64_t x) { return x ? (double)(int64_t)(x - base) / 100.0 : -1.0; }; // 100 MHz
      w0_acq.push_back(us(T(0, 1)));
      if (T(0, 2)) w0_pub.push_back(us(T(0, 2)));
      if (T(0, 4)) w0_next.push_back(us(T(0, 4)));
      uint64_t seen = 0, acq = 0, args = 0, end = 0, cnt = 0;
      uint32_t n_w = 0;
      for (int w = 0; w < 64; w++) {
        if (!T(w, 6)) continue;
        n_w++;
        if (w) {
          seen = std::max(seen, T(w, 0));
          acq = std::max(acq, T(w, 1));
          args = std::max(args, T(w, 5));
        }
        end = std::max(end, T(w, 6));
        cnt = std::max(cnt, T(w, 7));
      }
      waves = std::max(waves, n_w);
      if (seen) oth_seen.push_back(us(seen)), oth_acq.push_back(us(acq)), oth_args.push_back(us(args));
      run_end.push_back(us(end));
      if (cnt) count_end.push_back(us(cnt));
    }
    char b[640];
    std::snprintf(b, sizeof b,
                  ", \"%s\": {\"waves\": %u, \"host_post_to_complete\": %.2f, \"w0_acq\": %.2f, \"w0_pub\": %.2f, "
                  "\"oth_seen\": %.2f, \"oth_acq\": %.2f, \"oth_args\": %.2f, \"run_end\": %.2f, \"count_end\": %.2f, "
                  "\"w0_next\": %.2f}",
                  kd.name, waves, med(host), med(w0_acq), med(w0_pub), med(oth_seen), med(oth_acq), med(oth_args),
                  med(run_end), med(count_end), med(w0_next));
    out += b;
  }
  out += std::string(", \"ok\": ") + (ok ? "true" : "false") + "}";
  std::printf("%s\n", out.c_str());
  if (pn_service_close(svc)) ok = false;
  pn_close(ctx);
  return ok ? 0 : 1;
}
