// Zero-copy classify of a host ring: which pinned-memory kind reads fastest over PCIe, and is
// each one safe when the host rewrites the ring between launches (a NIC refilling slots)?
//   default      hipHostMalloc(hipHostMallocDefault)       (what GpuBackend / GpuRx use)
//   noncoherent  hipHostMalloc(hipHostMallocNonCoherent)
//   registered   aligned_alloc + hipHostRegister
// (built by `make bench/bench_pinned`)
// Frames: C4 (1514-B frames over 1024 flows, all hits).  Per batch size: host-visible time of
// pn_classify + stream sync (the server's classify leg).  Staleness: every frame's payload is
// corrupted, classified, repaired, classified — 4 rounds; each launch's verdicts must follow
// the bytes the host just wrote.  Prints one JSON line; exit 0 = every kind stayed correct.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../include/pollnet_amd_gen.h"

using Clock = std::chrono::steady_clock;

int main(int argc, char** argv) {
  const uint32_t reps = argc > 1 ? std::atoi(argv[1]) : 200;
  const uint32_t stride = 2048, off = 2, nmax = 16384;
  pn_gen_params gp{4, 1024, 0, 1024, 7};
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
  pn_result* rec = nullptr;
  if (hipHostMalloc((void**)&rec, sizeof(pn_result) * nmax, hipHostMallocDefault) != hipSuccess) return 4;

  std::string out = "{\"bench\": \"zero_copy_ring_kinds\"";
  bool all_ok = true;
  const char* kinds[] = {"default", "noncoherent", "registered"};
  for (int kind = 0; kind < 3; kind++) {
    uint8_t* ring = nullptr;
    bool ok = true;
    if (kind == 0) ok = hipHostMalloc((void**)&ring, frames.size(), hipHostMallocDefault) == hipSuccess;
    if (kind == 1) ok = hipHostMalloc((void**)&ring, frames.size(), hipHostMallocNonCoherent) == hipSuccess;
    if (kind == 2) {
      ring = (uint8_t*)std::aligned_alloc(4096, frames.size());
      ok = ring && hipHostRegister(ring, frames.size(), hipHostRegisterDefault) == hipSuccess;
    }
    if (!ok) {
      out += std::string(", \"") + kinds[kind] + "\": {\"error\": \"allocation failed\"}";
      all_ok = false;
      continue;
    }
    std::memcpy(ring, frames.data(), frames.size());
    auto classify = [&](uint32_t n) {
      return pn_classify(ctx, ring, stride, off, n, rec, s) == 0 && hipStreamSynchronize(s) == hipSuccess;
    };
    char buf[512];
    std::string legs;
    for (uint32_t n : {512u, 4096u, 16384u}) {
      for (int w = 0; w < 10; w++) ok = ok && classify(n);
      const auto t0 = Clock::now();
      for (uint32_t r = 0; r < reps; r++) ok = ok && classify(n);
      const double us = std::chrono::duration<double, std::micro>(Clock::now() - t0).count() / reps;
      std::snprintf(buf, sizeof buf, "%s\"us_%u\": %.1f, \"gbyte_per_s_%u\": %.1f", legs.empty() ? "" : ", ", n, us, n,
                    n * 1514.0 / us / 1e3);
      legs += buf;
    }
    // staleness: verdicts follow the host's rewrites (C4 damages 1 frame in 1024 itself)
    ok = ok && classify(nmax);
    std::vector<bool> clean(nmax);
    for (uint32_t i = 0; i < nmax; i++) clean[i] = (rec[i].flags & PN_F_TCP_OK) != 0;
    uint32_t wrong = 0;
    for (int round = 0; round < 4 && ok; round++) {
      for (int corrupt = 1; corrupt >= 0; corrupt--) {
        for (uint32_t i = 0; i < nmax; i++) ring[(size_t)i * stride + off + 1000] ^= 0x5a;
        ok = ok && classify(nmax);
        for (uint32_t i = 0; i < nmax; i++) wrong += ((rec[i].flags & PN_F_TCP_OK) != 0) != (clean[i] && !corrupt);
      }
    }
    std::snprintf(buf, sizeof buf, ", \"stale_verdicts\": %u, \"ok\": %s", wrong, ok && !wrong ? "true" : "false");
    legs += buf;
    out += std::string(", \"") + kinds[kind] + "\": {" + legs + "}";
    all_ok = all_ok && ok && !wrong;
    if (kind == 2) {
      (void)hipHostUnregister(ring);
      std::free(ring);
    } else {
      (void)hipHostFree(ring);
    }
  }
  std::printf("%s}\n", out.c_str());
  (void)hipHostFree(rec);
  (void)hipStreamDestroy(s);
  pn_close(ctx);
  pn_table_destroy(t);
  return all_ok ? 0 : 1;
}
