// Latency floor of a GPU round trip from the host (round 5): a value written to pinned host memory and
// answered by the GPU into pinned host memory, the host spinning on the answer.
//   launch:     one kernel launch per request (answers the value and ends) -- what pn_classify_notify pays
//   resident:   one resident kernel polling the doorbell (pn_test_doorbell_echo), with / without s_sleep
//   pipe_dK_gG: the pipelined poll (pn_test_doorbell_echo_pipe): K reads in flight, G x 64 clocks apart (round 6)
//   device_bell_*: the bell in device memory (hipExtMallocWithFlags, uncached or fine-grained) that the host writes
//     through the large BAR, the resident kernel polling HBM instead of host memory (round 6; argv[2] = "device" runs
//     only these legs)
// Prints one JSON line: median / p90 microseconds per round trip.   argv: iterations (2000) [device]
#include <hip/hip_runtime.h>

#include <immintrin.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../include/pollnet_amd.h"
#include "../include/pollnet_amd_tuning.h"

using Clock = std::chrono::steady_clock;

static void stats(const char* name, std::vector<double>& us, bool last) {
  std::sort(us.begin(), us.end());
  std::printf("\"%s\": {\"us_median\": %.2f, \"us_p10\": %.2f, \"us_p90\": %.2f}%s", name, us[us.size() / 2],
              us[us.size() / 10], us[us.size() * 9 / 10], last ? "" : ", ");
}

static bool spin(volatile uint32_t* w, uint32_t v) {
  const auto t0 = Clock::now();
  while (__atomic_load_n(w, __ATOMIC_ACQUIRE) != v)
    if (Clock::now() - t0 > std::chrono::seconds(2)) return false;
  return true;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 2000;
  uint32_t* words = nullptr;
  if (hipHostMalloc((void**)&words, 256, hipHostMallocDefault) != hipSuccess) return 2;
  uint32_t* bell = words;
  uint32_t* echo = words + 32; // another 128-B line
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 2;
  std::printf("{\"bench\": \"doorbell_round_trip\", \"iterations\": %d, ", iters);
  if (argc > 2 && std::strcmp(argv[2], "device") == 0) {
    int large_bar = 0;
    (void)hipDeviceGetAttribute(&large_bar, hipDeviceAttributeIsLargeBar, 0);
    std::printf("\"large_bar\": %d, ", large_bar);
    std::fflush(stdout);
    const struct { const char* name; unsigned flags; } kinds[] = {{"device_bell_uncached", hipDeviceMallocUncached},
                                                                 {"device_bell_finegrained", hipDeviceMallocFinegrained}};
    for (int kd = 0; kd < 2; kd++) {
      uint32_t* dbell = nullptr;
      if (hipExtMallocWithFlags((void**)&dbell, 4096, kinds[kd].flags) != hipSuccess) return 7;
      hipPointerAttribute_t attr{};
      (void)hipPointerGetAttributes(&attr, dbell);
      std::printf("\"%s_ptr\": {\"device\": \"%p\", \"host\": \"%p\", \"type\": %d}, ", kinds[kd].name, (void*)dbell,
                  attr.hostPointer, (int)attr.type);
      std::fflush(stdout);
      volatile uint32_t* hb = (volatile uint32_t*)(attr.hostPointer ? attr.hostPointer : dbell);
      *hb = 0u; // a host store into VRAM through the BAR (no large BAR: this faults on the host)
      _mm_sfence();
      if (*hb != 0u) return 8;
      __atomic_store_n(echo, 0u, __ATOMIC_RELEASE);
      if (pn_test_doorbell_echo(dbell, echo, 200, 0, 0, s)) return 3;
      std::vector<double> us;
      bool ok = true;
      uint32_t rnd = 777;
      for (int i = 1; i <= iters + 50 && ok; i++) {
        rnd = rnd * 1664525u + 1013904223u;
        const auto tw = Clock::now() + std::chrono::nanoseconds((rnd >> 8) % 3000);
        while (Clock::now() < tw) {
        }
        const auto t0 = Clock::now();
        *hb = (uint32_t)i;
        _mm_sfence(); // out of the write-combining buffer
        ok = spin(echo, (uint32_t)i);
        if (i > 50) us.push_back(std::chrono::duration<double, std::micro>(Clock::now() - t0).count());
      }
      *hb = 0xFFFFFFFFu; // stop
      _mm_sfence();
      if (hipStreamSynchronize(s) != hipSuccess) return 5;
      if (!ok) return 6;
      stats(kinds[kd].name, us, false);
      (void)hipFree(dbell);
    }
    // the host-memory bell beside them, same request pattern
    __atomic_store_n(bell, 0u, __ATOMIC_RELEASE);
    __atomic_store_n(echo, 0u, __ATOMIC_RELEASE);
    if (pn_test_doorbell_echo(bell, echo, 200, 0, 0, s)) return 3;
    std::vector<double> us;
    bool ok = true;
    uint32_t rnd = 777;
    for (int i = 1; i <= iters + 50 && ok; i++) {
      rnd = rnd * 1664525u + 1013904223u;
      const auto tw = Clock::now() + std::chrono::nanoseconds((rnd >> 8) % 3000);
      while (Clock::now() < tw) {
      }
      const auto t0 = Clock::now();
      __atomic_store_n(bell, (uint32_t)i, __ATOMIC_RELEASE);
      ok = spin(echo, (uint32_t)i);
      if (i > 50) us.push_back(std::chrono::duration<double, std::micro>(Clock::now() - t0).count());
    }
    __atomic_store_n(bell, 0xFFFFFFFFu, __ATOMIC_RELEASE);
    if (hipStreamSynchronize(s) != hipSuccess) return 5;
    if (!ok) return 6;
    stats("host_bell_same_pattern", us, true);
    std::printf("}\n");
    return 0;
  }
  // launch per request
  {
    std::vector<double> us;
    for (int i = 1; i <= iters + 50; i++) {
      __atomic_store_n(bell, (uint32_t)i, __ATOMIC_RELEASE);
      const auto t0 = Clock::now();
      if (pn_test_doorbell_echo(bell, echo, 100, 1, 0, s)) return 3;
      if (!spin(echo, (uint32_t)i)) return 4;
      if (i > 50) us.push_back(std::chrono::duration<double, std::micro>(Clock::now() - t0).count());
    }
    if (hipStreamSynchronize(s) != hipSuccess) return 5;
    stats("launch_per_request", us, false);
  }
  for (int sl = 0; sl < 2; sl++) {
    __atomic_store_n(bell, 0u, __ATOMIC_RELEASE);
    __atomic_store_n(echo, 0u, __ATOMIC_RELEASE);
    if (pn_test_doorbell_echo(bell, echo, 200, 0, sl, s)) return 3; // ends 200 ms after the last request
    std::vector<double> us;
    bool ok = true;
    for (int i = 1; i <= iters + 50 && ok; i++) {
      const auto t0 = Clock::now();
      __atomic_store_n(bell, (uint32_t)i, __ATOMIC_RELEASE);
      ok = spin(echo, (uint32_t)i);
      if (i > 50) us.push_back(std::chrono::duration<double, std::micro>(Clock::now() - t0).count());
    }
    __atomic_store_n(bell, 0xFFFFFFFFu, __ATOMIC_RELEASE); // stop
    if (hipStreamSynchronize(s) != hipSuccess) return 5;
    if (!ok) return 6;
    stats(sl ? "resident_sleep" : "resident_spin", us, false);
  }
  // the pipelined poll: the host waits a random 0-3 us between requests, so a request lands at any phase of the polls
  const struct { int depth; uint32_t gap; } grid[] = {{1, 0}, {2, 4}, {2, 8}, {4, 2}, {4, 4}, {4, 8}, {8, 1}, {8, 2}, {8, 4}};
  uint32_t rnd = 12345;
  const int n_grid = (int)(sizeof grid / sizeof grid[0]);
  for (int g = 0; g < n_grid; g++) {
    __atomic_store_n(bell, 0u, __ATOMIC_RELEASE);
    __atomic_store_n(echo, 0u, __ATOMIC_RELEASE);
    if (pn_test_doorbell_echo_pipe(bell, echo, 200, grid[g].depth, grid[g].gap, s)) return 3;
    std::vector<double> us;
    bool ok = true;
    for (int i = 1; i <= iters + 50 && ok; i++) {
      rnd = rnd * 1664525u + 1013904223u;
      const auto tw = Clock::now() + std::chrono::nanoseconds((rnd >> 8) % 3000);
      while (Clock::now() < tw) {
      }
      const auto t0 = Clock::now();
      __atomic_store_n(bell, (uint32_t)i, __ATOMIC_RELEASE);
      ok = spin(echo, (uint32_t)i);
      if (i > 50) us.push_back(std::chrono::duration<double, std::micro>(Clock::now() - t0).count());
    }
    __atomic_store_n(bell, 0xFFFFFFFFu, __ATOMIC_RELEASE); // stop
    if (hipStreamSynchronize(s) != hipSuccess) return 5;
    if (!ok) return 6;
    char name[32];
    std::snprintf(name, sizeof name, "pipe_d%d_g%u", grid[g].depth, grid[g].gap);
    stats(name, us, g == n_grid - 1);
  }
  std::printf("}\n");
  (void)hipStreamDestroy(s);
  (void)hipHostFree(words);
  return 0;
}
