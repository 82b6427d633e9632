// The sniffer path end to end: a captured ring in pinned host memory,
// S watched TCP streams among other traffic, every watched stream reassembled and handed to its handler.
//
//   CPU:  what pollnet's sniffer does with S TcpStreams on one core — for every frame, every stream's
//         filterPacket (TcpStream.h:39-52), and handlePacket (:54-142) where it passes.  The filter and the
//         reassembler are this repository's restatements (GpuTcpStreams::filterPacket, StreamReassembler),
//         which the tests hold equal to the reference's own TcpStream.
//   GPU:  GpuTcpStreams::poll — one pn_match_streams launch per chunk reading each frame's header line over
//         PCIe (zero copy), the host reassembling only the frames of a watched stream.
// Both deliver every stream's bytes to the same handler; the per-stream byte counts and a checksum of the
// delivered bytes must agree.  One JSON line on stdout.
//   bench_streams [frames=1048576] [streams=8] [watched_every=16] [reps=5] [chunk=262144]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <memory>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../include/pollnet_amd/tcp_stream.hpp"

using namespace pollnet_amd;

namespace {

constexpr uint32_t kStride = 2048, kOff = 2;

void put16(uint8_t* p, uint16_t v) {
  p[0] = v >> 8;
  p[1] = v & 0xff;
}
void put32(uint8_t* p, uint32_t v) {
  put16(p, v >> 16);
  put16(p + 2, v & 0xffff);
}

// One Ethernet/IPv4/TCP frame (IHL 5, doff 5, ACK|PSH) at eth; checksums are not needed on this path.
void frame(uint8_t* eth, uint32_t sip, uint16_t sport, uint32_t dip, uint16_t dport, uint32_t seq, const uint8_t* pay,
           uint32_t len) {
  std::memset(eth, 0, 54);
  eth[0] = 2, eth[5] = 1, eth[6] = 2, eth[11] = 2;
  put16(eth + 12, 0x0800);
  uint8_t* ip = eth + 14;
  ip[0] = 0x45;
  put16(ip + 2, (uint16_t)(40 + len));
  ip[8] = 64;
  ip[9] = 6;
  put32(ip + 12, sip);
  put32(ip + 16, dip);
  uint8_t* tcp = ip + 20;
  put16(tcp, sport);
  put16(tcp + 2, dport);
  put32(tcp + 4, seq);
  tcp[12] = 5 << 4;
  tcp[13] = 0x18;
  put16(tcp + 14, 65535);
  std::memcpy(tcp + 20, pay, len);
}

struct Sink {
  std::vector<uint64_t> bytes, sum;
  explicit Sink(uint32_t s) : bytes(s), sum(s) {}
  uint32_t operator()(int s, const uint8_t* d, uint32_t n) {
    bytes[s] += n;
    uint64_t h = sum[s];
    for (uint32_t i = 0; i < n; i += 64) h = h * 1099511628211ull + d[i]; // touch the payload, one byte a line
    sum[s] = h;
    return 0;
  }
};

double now_s() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

}  // namespace

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)std::atoi(argv[1]) : (1u << 20);
  const uint32_t S = argc > 2 ? (uint32_t)std::atoi(argv[2]) : 8;
  const uint32_t every = argc > 3 ? (uint32_t)std::atoi(argv[3]) : 16;
  const int reps = argc > 4 ? std::atoi(argv[4]) : 5;
  const uint32_t chunk = argc > 5 ? (uint32_t)std::atoi(argv[5]) : (1u << 18);
  if (!n || !S || S > PN_MAX_STREAM_FILTERS || !every || reps < 1 || !chunk) return 2;

  uint8_t* ring = nullptr;
  if (hipHostMalloc((void**)&ring, (size_t)n * kStride, hipHostMallocDefault) != hipSuccess) return 3;
  std::mt19937_64 rng(0x5EED57);
  std::vector<uint8_t> pay(1460);
  for (auto& b : pay) b = (uint8_t)rng();
  std::vector<uint32_t> seq(S);
  for (auto& q : seq) q = (uint32_t)rng();
  const uint32_t server = 0x0a000001;
  uint64_t watched = 0, wire = 0;
  for (uint32_t i = 0; i < n; i++) {
    uint8_t* eth = ring + (size_t)i * kStride + kOff;
    if (i % every == 0) { // the next segment of watched stream k, in order
      const uint32_t k = (i / every) % S, len = 1460;
      frame(eth, 0x0a070000 | k, (uint16_t)(5000 + k), server, 1234, seq[k], pay.data(), len);
      seq[k] += len;
      watched++;
      wire += 54 + len;
    } else { // other traffic: TCP from hosts no filter names, 64-1514-B frames
      const uint32_t len = 10 + (uint32_t)(rng() % 1451);
      frame(eth, 0x0a090000 | (uint32_t)(rng() & 0xffff), (uint16_t)(1024 + rng() % 60000), server, 1234,
            (uint32_t)rng(), pay.data(), len);
      wire += 54 + len;
    }
  }
  std::vector<pn_stream_filter> filters(S);
  std::vector<std::string> src(S);
  for (uint32_t k = 0; k < S; k++) {
    char b[32];
    std::snprintf(b, sizeof b, "10.7.0.%u", k);
    src[k] = b;
    pn_stream_filter f{};
    inet_pton(AF_INET, b, &f.src_ip);
    inet_pton(AF_INET, "10.0.0.1", &f.dst_ip);
    f.src_port = htons((uint16_t)(5000 + k));
    f.dst_port = htons(1234);
    filters[k] = f;
  }

  // CPU: every stream's filterPacket on every frame, handlePacket where it passes (one core)
  std::vector<double> cpu_s, gpu_s;
  Sink cpu_sink(S), gpu_sink(S);
  for (int r = 0; r < reps; r++) {
    std::vector<std::unique_ptr<StreamReassembler<>>> rs;
    for (uint32_t k = 0; k < S; k++) rs.push_back(std::make_unique<StreamReassembler<>>());
    Sink sink(S);
    const double t0 = now_s();
    for (uint32_t i = 0; i < n; i++) {
      const uint8_t* eth = ring + (size_t)i * kStride + kOff;
      for (uint32_t k = 0; k < S; k++)
        if (GpuTcpStreams<>::filterPacket(filters[k], eth))
          rs[k]->handlePacket(eth, [&](const uint8_t* d, uint32_t m) { return sink((int)k, d, m); });
    }
    cpu_s.push_back(now_s() - t0);
    if (r == 0) cpu_sink = sink;
  }
  // GPU: GpuTcpStreams::poll over the same ring, zero copy
  const char* err = nullptr;
  for (int r = 0; r < reps && !err; r++) {
    auto g = std::make_unique<GpuTcpStreams<>>();
    if ((err = g->init(0, kStride, kOff, chunk, GpuRx::Mode::ZeroCopy))) break;
    for (uint32_t k = 0; k < S; k++)
      if (g->addStream(src[k].c_str(), (uint16_t)(5000 + k), "10.0.0.1", 1234) < 0) err = "addStream failed";
    if (err) break;
    Sink sink(S);
    const double t0 = now_s();
    err = g->poll(ring, n, [&](int s, const uint8_t* d, uint32_t m) { return sink(s, d, m); });
    gpu_s.push_back(now_s() - t0);
    if (r == 0) gpu_sink = sink;
  }
  if (err) {
    std::printf("{\"error\": \"%s\"}\n", err);
    return 4;
  }
  const bool equal = cpu_sink.bytes == gpu_sink.bytes && cpu_sink.sum == gpu_sink.sum;
  uint64_t delivered = 0;
  for (auto b : cpu_sink.bytes) delivered += b;
  auto med = [](std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  const double c = med(cpu_s), g = med(gpu_s);
  std::printf("{\"bench\": \"sniffer_streams\", \"frames\": %u, \"streams\": %u, \"watched_every\": %u, "
              "\"watched_frames\": %llu, \"delivered_bytes\": %llu, \"cpu_one_core\": {\"ms\": %.3f, \"mframes_per_s\": %.2f, "
              "\"gbit_per_s\": %.1f}, \"gpu_zero_copy\": {\"ms\": %.3f, \"mframes_per_s\": %.2f, \"gbit_per_s\": %.1f}, "
              "\"gpu_over_cpu\": %.2f, \"delivery_equal\": %s, \"reps\": %d, \"chunk\": %u, \"note\": \"capture in pinned host "
              "memory (2-KiB slots); CPU: every stream's filterPacket per frame + handlePacket (restated, held equal to "
              "the reference TcpStream by the tests); GPU: GpuTcpStreams::poll (pn_match_streams over PCIe + host "
              "reassembly of the watched frames)\"}\n",
              n, S, every, (unsigned long long)watched, (unsigned long long)delivered, c * 1e3, n / c / 1e6,
              wire * 8 / c / 1e9, g * 1e3, n / g / 1e6, wire * 8 / g / 1e9, c / g, equal ? "true" : "false", reps, chunk);
  (void)hipHostFree(ring);
  return equal ? 0 : 1;
}
