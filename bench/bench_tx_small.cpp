// TX checksum fill at small batch sizes (the drop-in server's per-poll ACK batches): host-
// visible time of one call + stream sync, the two-phase form (fill into patch records, then a
// patch launch; tuning variant 40) against the same fill writing the fields in place in one
// launch (variant 41) — both in pn_tx_fill's launch shape, `make TUNING=1` — and pn_tx_fill
// itself (which takes the one-launch form up to kTxInPlaceMaxFrames), frames in pinned host
// memory (the server's TX batch, zero copy) and in device memory.  The forms' frames are
// compared byte for byte after each size.
// Measurement only.  Prints one JSON line.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../include/pollnet_amd_gen.h"
#include "../include/pollnet_amd_tuning.h"

using Clock = std::chrono::steady_clock;

int main(int argc, char** argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 300;
  const uint32_t stride = 2048, off = 2, nmax = 65536;
  pn_gen_params gp{4, 1024, 0, 1024, 11};
  std::vector<uint8_t> src((size_t)stride * nmax);
  if (pn_gen_frames(&gp, 0, nmax, src.data(), stride, off, 8)) return 3;
  pn_ctx* ctx = nullptr;
  if (pn_open(0, &ctx)) return 4;
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 4;
  uint8_t *host_a = nullptr, *host_b = nullptr, *dev = nullptr;
  if (hipHostMalloc((void**)&host_a, src.size(), hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc((void**)&host_b, src.size(), hipHostMallocDefault) != hipSuccess ||
      hipMalloc((void**)&dev, src.size()) != hipSuccess)
    return 4;
  std::string out = "{\"bench\": \"tx_fill_small_batches\", \"unit\": \"us per call incl. sync\"";
  bool same_all = true;
  for (int where = 0; where < 2; where++) {
    for (uint32_t n : {16u, 64u, 256u, 1024u, 4096u, 16384u, 65536u}) {
      double us[3] = {0, 0, 0};
      for (int form = 2; form >= 0; form--) { // 2 = pn_tx_fill, 1 = in place (41), 0 = two-phase (40)
        uint8_t* buf = where == 0 ? (form == 1 ? host_b : host_a) : dev;
        if (where == 0) std::memcpy(buf, src.data(), (size_t)stride * n);
        else if (hipMemcpy(buf, src.data(), (size_t)stride * n, hipMemcpyHostToDevice) != hipSuccess) return 5;
        auto call = [&]() {
          int rc = form == 2 ? pn_tx_fill(ctx, buf, stride, off, n, nullptr, PN_TX_TCP, s)
                             : pn_tx_fill_variant(ctx, buf, stride, off, n, nullptr, form ? 41 : 40, s);
          return rc == 0 && hipStreamSynchronize(s) == hipSuccess;
        };
        for (int w = 0; w < 20; w++)
          if (!call()) return std::fprintf(stderr, "%s\n", pn_last_error(ctx)), 6;
        const auto t0 = Clock::now();
        for (int r = 0; r < reps; r++) call();
        us[form] = std::chrono::duration<double, std::micro>(Clock::now() - t0).count() / reps;
        if (where == 1 && form == 0 && hipMemcpy(host_a, dev, (size_t)stride * n, hipMemcpyDeviceToHost) != hipSuccess)
          return 5;
        if (where == 1 && form == 1 && hipMemcpy(host_b, dev, (size_t)stride * n, hipMemcpyDeviceToHost) != hipSuccess)
          return 5;
      }
      const bool same = std::memcmp(host_a, host_b, (size_t)stride * n) == 0;
      same_all &= same;
      char b[200];
      std::snprintf(b, sizeof b,
                    ", \"%s_n%u\": {\"two_phase\": %.1f, \"in_place_one_launch\": %.1f, \"pn_tx_fill\": %.1f, "
                    "\"same\": %s}",
                    where ? "device" : "pinned_host", n, us[0], us[1], us[2], same ? "true" : "false");
      out += b;
    }
  }
  std::printf("%s}\n", out.c_str());
  return same_all ? 0 : 1;
}
