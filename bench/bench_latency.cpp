// Batch size vs throughput and latency of pn_classify (SURVEY §7 "latency vs throughput":
// the reference handles <= 64 RX events per pollNet call, Core.h:496-498; a GPU pays a launch
// and a completion wait per batch, so the drop-in must batch across polls).  For each batch
// size n, on one MI355X, with the C2 generator's 1514-B frames in 2-KiB slots:
//   kernel_us    : back-to-back launches over fresh (rotating) resident slots, HIP events / launch
//   resident_rt  : one pn_classify + hipStreamSynchronize, host wall clock (median, p99)
//   resident_spin: the same with the completion busy-polled (hipEventQuery loop)
//   e2e_rt       : pinned host slots -> H2D -> pn_classify -> D2H records -> sync (median, p99)
//   e2e_graph_rt : the same three operations captured once in a hipGraph, hipGraphLaunch + sync
//   zero_copy_rt : the kernel reads the pinned host slots and writes records to pinned host memory
// Prints one JSON line.  Test/bench tool: links the product library only.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../include/pollnet_amd_gen.h"

using Clock = std::chrono::steady_clock;

#define HIP_OK(x)                                                                      \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)
#define PN_OK_(x)                                                                      \
  do {                                                                                 \
    if ((x) != 0) {                                                                    \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, pn_last_error(ctx));   \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

static double us_since(Clock::time_point t0) {
  return std::chrono::duration<double, std::micro>(Clock::now() - t0).count();
}

struct Stat {
  double med, p99;
};
static Stat stat(std::vector<double>& v) {
  std::sort(v.begin(), v.end());
  return {v[v.size() / 2], v[std::min(v.size() - 1, (size_t)(v.size() * 0.99))]};
}

int main(int argc, char** argv) {
  const uint32_t kStride = 2048, kOff = 2;
  const uint32_t total = argc > 1 ? (uint32_t)atoi(argv[1]) : (1u << 20);  // resident slots
  const uint32_t sizes[] = {64, 256, 1024, 4096, 16384, 65536, 262144, 1048576};

  pn_ctx* ctx = nullptr;
  if (pn_open(0, &ctx) != 0) {
    fprintf(stderr, "pn_open: %s\n", pn_last_error(nullptr));
    return 1;
  }
  pn_gen_params gp{2, 1, 0, 1024, 0x5EED0002ull};
  pn_conn_table* tbl = nullptr;
  PN_OK_(pn_table_create(1024, 1024, &tbl));
  PN_OK_(pn_gen_conn_table(&gp, tbl));
  uint32_t n_entries = 0;
  uint64_t mask = 0;
  const pn_conn_entry* ents = pn_table_entries(tbl, &n_entries, &mask);
  PN_OK_(pn_set_conn_table(ctx, ents, n_entries, mask, pn_table_max_conn_cnt(tbl)));

  uint8_t* host = nullptr;
  HIP_OK(hipHostMalloc((void**)&host, (size_t)total * kStride, hipHostMallocDefault));
  PN_OK_(pn_gen_frames(&gp, 0, total, host, kStride, kOff, 16));
  uint8_t *dev = nullptr, *dev_e2e = nullptr;
  pn_result *res = nullptr, *res_host = nullptr;
  HIP_OK(hipMalloc((void**)&dev, (size_t)total * kStride));
  HIP_OK(hipMalloc((void**)&dev_e2e, (size_t)total * kStride));
  HIP_OK(hipMalloc((void**)&res, (size_t)total * sizeof(pn_result)));
  HIP_OK(hipHostMalloc((void**)&res_host, (size_t)total * sizeof(pn_result), hipHostMallocDefault));
  HIP_OK(hipMemcpy(dev, host, (size_t)total * kStride, hipMemcpyHostToDevice));
  hipStream_t s;
  HIP_OK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  HIP_OK(hipEventCreate(&e0));
  HIP_OK(hipEventCreate(&e1));
  hipEvent_t ed;
  HIP_OK(hipEventCreateWithFlags(&ed, hipEventDisableTiming));

  printf("{\"tool\": \"bench/bench_latency\", \"workload\": \"C2 1514-B frames, 2048-B slots, frame_off 2\", "
         "\"resident_slots\": %u, \"rows\": [",
         total);
  bool first = true;
  for (uint32_t n : sizes) {
    if (n > total) break;
    const uint32_t groups = total / n;
    // kernel time: back-to-back launches, each over the next n slots (fresh bytes, as a ring delivers)
    const int reps = (int)std::max<uint32_t>(8u, std::min<uint32_t>(400u, (64u << 20) / n));
    for (int w = 0; w < 4; ++w) PN_OK_(pn_classify(ctx, dev + (size_t)(w % groups) * n * kStride, kStride, kOff, n, res, s));
    HIP_OK(hipEventRecord(e0, s));
    for (int k = 0; k < reps; ++k)
      PN_OK_(pn_classify(ctx, dev + (size_t)(k % groups) * n * kStride, kStride, kOff, n, res, s));
    HIP_OK(hipEventRecord(e1, s));
    HIP_OK(hipEventSynchronize(e1));
    float ms = 0;
    HIP_OK(hipEventElapsedTime(&ms, e0, e1));
    const double kern_us = ms * 1e3 / reps;

    // one resident batch, host-visible completion
    const int iters = n >= 262144 ? 30 : 200;
    std::vector<double> rt, e2e, gr;
    for (int k = 0; k < iters + 5; ++k) {
      auto t0 = Clock::now();
      PN_OK_(pn_classify(ctx, dev + (size_t)(k % groups) * n * kStride, kStride, kOff, n, res, s));
      HIP_OK(hipStreamSynchronize(s));
      if (k >= 5) rt.push_back(us_since(t0));
    }
    // the same, completion busy-polled with hipEventQuery (pollnet's own style: spin, never block)
    std::vector<double> spin;
    for (int k = 0; k < iters + 5; ++k) {
      auto t0 = Clock::now();
      PN_OK_(pn_classify(ctx, dev + (size_t)(k % groups) * n * kStride, kStride, kOff, n, res, s));
      HIP_OK(hipEventRecord(ed, s));
      hipError_t q;
      while ((q = hipEventQuery(ed)) == hipErrorNotReady) {
      }
      HIP_OK(q);
      if (k >= 5) spin.push_back(us_since(t0));
    }
    // host ring in, records out
    for (int k = 0; k < iters + 5; ++k) {
      const size_t g = (size_t)(k % groups) * n;
      auto t0 = Clock::now();
      HIP_OK(hipMemcpyAsync(dev_e2e, host + g * kStride, (size_t)n * kStride, hipMemcpyHostToDevice, s));
      PN_OK_(pn_classify(ctx, dev_e2e, kStride, kOff, n, res, s));
      HIP_OK(hipMemcpyAsync(res_host, res, (size_t)n * sizeof(pn_result), hipMemcpyDeviceToHost, s));
      HIP_OK(hipStreamSynchronize(s));
      if (k >= 5) e2e.push_back(us_since(t0));
    }
    // zero copy: the kernel reads the pinned host slots over PCIe and writes the records into pinned
    // host memory (GpuRx's zero-copy mode): one launch + sync, no copies
    std::vector<double> zc;
    for (int k = 0; k < iters + 5; ++k) {
      const size_t g = (size_t)(k % groups) * n;
      auto t0 = Clock::now();
      PN_OK_(pn_classify(ctx, host + g * kStride, kStride, kOff, n, res_host, s));
      HIP_OK(hipStreamSynchronize(s));
      if (k >= 5) zc.push_back(us_since(t0));
    }
    // the same, captured once as a graph (fixed host slots: the ring's next batch would be a node update)
    hipGraph_t graph;
    hipGraphExec_t exec;
    HIP_OK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    HIP_OK(hipMemcpyAsync(dev_e2e, host, (size_t)n * kStride, hipMemcpyHostToDevice, s));
    PN_OK_(pn_classify(ctx, dev_e2e, kStride, kOff, n, res, s));
    HIP_OK(hipMemcpyAsync(res_host, res, (size_t)n * sizeof(pn_result), hipMemcpyDeviceToHost, s));
    HIP_OK(hipStreamEndCapture(s, &graph));
    HIP_OK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
    for (int k = 0; k < iters + 5; ++k) {
      auto t0 = Clock::now();
      HIP_OK(hipGraphLaunch(exec, s));
      HIP_OK(hipStreamSynchronize(s));
      if (k >= 5) gr.push_back(us_since(t0));
    }
    HIP_OK(hipGraphExecDestroy(exec));
    HIP_OK(hipGraphDestroy(graph));
    // the records of the last graph run must be those of the first n frames
    uint32_t bad = 0;
    for (uint32_t i = 0; i < n; ++i)
      bad += !(res_host[i].payload_off == 54 && res_host[i].conn_id == 0 && (res_host[i].flags & 0x4));

    Stat a = stat(rt), b = stat(e2e), c = stat(gr), d = stat(spin), z = stat(zc);
    const double wire = 1514.0 * 8 * n;
    printf("%s{\"frames\": %u, \"kernel_us\": %.2f, \"kernel_mframes_per_s\": %.1f, \"kernel_gbit_per_s\": %.1f, "
           "\"resident_rt_us_median\": %.2f, \"resident_rt_us_p99\": %.2f, \"resident_spin_rt_us_median\": %.2f, "
           "\"resident_spin_rt_us_p99\": %.2f, \"e2e_rt_us_median\": %.2f, "
           "\"e2e_rt_us_p99\": %.2f, \"e2e_graph_rt_us_median\": %.2f, \"e2e_graph_rt_us_p99\": %.2f, "
           "\"e2e_gbit_per_s\": %.1f, \"zero_copy_rt_us_median\": %.2f, \"zero_copy_rt_us_p99\": %.2f, "
           "\"zero_copy_gbit_per_s\": %.1f, \"records_unexpected\": %u}",
           first ? "" : ", ", n, kern_us, n / kern_us, wire / kern_us / 1e3, a.med, a.p99, d.med, d.p99, b.med, b.p99, c.med, c.p99,
           wire / b.med / 1e3, z.med, z.p99, wire / z.med / 1e3, bad);
    first = false;
    fflush(stdout);
  }
  printf("]}\n");
  HIP_OK(hipStreamDestroy(s));
  HIP_OK(hipFree(dev));
  HIP_OK(hipFree(dev_e2e));
  HIP_OK(hipFree(res));
  HIP_OK(hipHostFree(host));
  HIP_OK(hipHostFree(res_host));
  pn_table_destroy(tbl);
  pn_close(ctx);
  return 0;
}
