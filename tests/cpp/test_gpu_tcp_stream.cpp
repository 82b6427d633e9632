// GPU: pn_match_streams + GpuTcpStreams (include/pollnet_amd/tcp_stream.hpp) against
// the reference's own TcpStream (oracle/_ref/libref_tcpstream.so).
//
// A captured ring of ~12,000 frames: 8 sniffed TCP streams (reordered, duplicated,
// with SYNs), other TCP flows, UDP, ARP and IPv6 frames, IHL=6 frames.  8 filters with
// wildcards that overlap (the last filter is all-wildcard).  Checks:
//   1. every frame's stream id == the index of the first filter the reference's
//      TcpStream::filterPacket accepts it for (copy and zero-copy, several chunk sizes);
//   2. GpuTcpStreams::poll's handler log per stream (sizes and bytes) == feeding each
//      frame, in ring order, to the reference TcpStream of every filter that accepts it
//      (independent TcpStreams, the default), and with setFirstMatchOnly(true) to that of
//      its first accepting filter only.
// argv[1] = libref_tcpstream.so.  Exit 0 = pass.
#include <dlfcn.h>

#include <cstdio>
#include <memory>
#include <random>
#include <string>
#include <vector>

#include "../../include/pollnet_amd/tcp_stream.hpp"
#include "segframes.hpp"

using namespace segtest;
using namespace pollnet_amd;

struct RefLog {
  uint8_t* bytes;
  uint64_t n_bytes, cap_bytes;
  uint32_t* call_sizes;
  uint32_t n_calls, cap_calls;
};

struct FilterSpec {
  std::string src_ip;
  uint16_t src_port;
  std::string dst_ip;
  uint16_t dst_port;
};

static std::string ip_str(uint32_t ip) {
  char b[32];
  std::snprintf(b, sizeof b, "%u.%u.%u.%u", ip >> 24, (ip >> 16) & 255, (ip >> 8) & 255, ip & 255);
  return b;
}

int main(int argc, char** argv) {
  void* h = dlopen(argc > 1 ? argv[1] : "oracle/_ref/libref_tcpstream.so", RTLD_NOW);
  if (!h) {
    std::printf("FAIL: reference not loadable (%s)\n", dlerror());
    return 1;
  }
  auto ref_filter = (int (*)(const uint8_t*, uint32_t, const char*, uint16_t, const char*, uint16_t))dlsym(
      h, "ref_filter_packet");
  auto ref_new = (void* (*)(int, int))dlsym(h, "ref_stream_new2");
  auto ref_free = (void (*)(void*))dlsym(h, "ref_stream_free");
  auto ref_handle = (int (*)(void*, const uint8_t*, uint32_t, uint32_t, RefLog*))dlsym(h, "ref_stream_handle");
  if (!ref_filter || !ref_new || !ref_free || !ref_handle) return 1;

  std::mt19937_64 rng(0x51FF);
  auto U = [&](uint32_t lo, uint32_t hi) { return lo + (uint32_t)(rng() % (hi - lo + 1)); };
  const uint32_t server = 0x0a000001; // 10.0.0.1, as segframes builds dst
  // 8 sniffed streams: client 10.7.0.k:5000+k -> 10.0.0.1:1234
  struct Sn {
    uint32_t ip;
    uint16_t port;
    uint32_t isn;
    std::vector<uint8_t> data;
    std::vector<Seg> segs;
    size_t next = 0;
  };
  std::vector<Sn> sn(8);
  for (uint32_t k = 0; k < 8; k++) {
    Sn& s = sn[k];
    s.ip = 0x0a070000 | k;
    s.port = (uint16_t)(5000 + k);
    s.isn = (uint32_t)rng();
    s.data.resize(U(200000, 1500000));
    for (auto& b : s.data) b = (uint8_t)rng();
    Seg syn;
    syn.src_ip = s.ip;
    syn.src_port = s.port;
    syn.seq = s.isn;
    syn.flags = SYN;
    s.segs.push_back(syn);
    std::vector<std::pair<uint32_t, uint32_t>> cuts;
    for (uint32_t o = 0; o < s.data.size();) {
      const uint32_t n = std::min<uint32_t>((uint32_t)s.data.size() - o, U(1, 1460));
      cuts.push_back({o, o + n});
      o += n;
    }
    for (size_t b = 0; b < cuts.size(); b += 3) {
      std::vector<std::pair<uint32_t, uint32_t>> blk(cuts.begin() + b, cuts.begin() + std::min(cuts.size(), b + 3));
      if (b) std::shuffle(blk.begin(), blk.end(), rng);
      for (auto& x : blk) {
        Seg d;
        d.src_ip = s.ip;
        d.src_port = s.port;
        d.seq = s.isn + 1 + x.first;
        d.flags = ACK | PSH;
        d.payload = s.data.data() + x.first;
        d.len = x.second - x.first;
        s.segs.push_back(d);
        if (rng() % 25 == 0) s.segs.push_back(d);
      }
    }
  }
  // the ring: sniffed segments interleaved with noise
  const uint32_t stride = 2048, off = 2;
  std::vector<std::pair<int, Seg>> order; // (kind, seg): kind 0 = sniffed, 1 tcp noise, 2 udp, 3 arp, 4 ipv6, 5 ihl6
  std::vector<uint8_t> noise(1460, 0x77);
  size_t left = 0;
  for (auto& s : sn) left += s.segs.size();
  while (left) {
    if (rng() % 4 == 0) {
      Seg z;
      z.src_ip = (rng() % 2) ? (0x0a070000 | U(0, 7)) : (0x0b000000 | U(0, 3)); // sniffed hosts (other ports) or 11.0.0.x
      z.src_port = (uint16_t)U(1, 65535);
      z.seq = (uint32_t)rng();
      z.payload = noise.data();
      z.len = U(0, 1460);
      order.push_back({(int)U(1, 5), z});
    } else {
      uint32_t k = U(0, 7);
      while (sn[k].next == sn[k].segs.size()) k = (k + 1) % 8;
      order.push_back({0, sn[k].segs[sn[k].next++]});
      left--;
    }
  }
  const uint32_t n = (uint32_t)order.size();
  uint8_t* ring = nullptr;
  if (hipHostMalloc((void**)&ring, (size_t)stride * n, hipHostMallocDefault) != hipSuccess) return 2;
  std::memset(ring, 0, (size_t)stride * n);
  std::vector<uint32_t> flen(n);
  for (uint32_t i = 0; i < n; i++) {
    uint8_t* eth = ring + (size_t)i * stride + off;
    flen[i] = build(eth, order[i].second);
    switch (order[i].first) {
      case 2: eth[23] = 17; break;               // UDP
      case 3: eth[12] = 0x08, eth[13] = 0x06; break; // ARP
      case 4: eth[12] = 0x86, eth[13] = 0xdd; break; // IPv6
      case 5: eth[14] = 0x46; break;             // IHL 6: the filter still reads fixed offsets
      default: break;
    }
    if (order[i].first) { // noise: vary the destination so every filter sees traffic
      if (rng() % 2) put16(eth + 36, (uint16_t)U(1, 65535));
      if (rng() % 3 == 0) put32(eth + 30, 0x0c000000 | U(0, 255));
    }
  }
  // filters: overlapping wildcards; the last catches every TCP frame
  std::vector<FilterSpec> fs = {
      {ip_str(0x0a070000), 5000, ip_str(server), 1234},      // stream 0 exactly
      {ip_str(0x0a070001), 0, "0.0.0.0", 0},                  // anything from host 1
      {"0.0.0.0", 5002, "0.0.0.0", 1234},                     // client port 5002
      {ip_str(0x0a070003), 5003, "0.0.0.0", 0},               // host 3 port 5003
      {"0.0.0.0", 0, ip_str(server), 1234},                   // the rest to the server
      {ip_str(0x0b000001), 0, "0.0.0.0", 0},                  // a noise host
      {"0.0.0.0", 0, "0.0.0.0", 1234},                        // shadowed by filter 4
      {"0.0.0.0", 0, "0.0.0.0", 0},                           // everything TCP/IPv4
  };
  // reference: the filters accepting each frame, and the first of them
  std::vector<uint32_t> want(n, PN_NO_STREAM), accept(n, 0);
  uint32_t multi = 0;
  for (uint32_t i = 0; i < n; i++) {
    const uint8_t* eth = ring + (size_t)i * stride + off;
    for (uint32_t k = 0; k < fs.size(); k++)
      if (ref_filter(eth, flen[i], fs[k].src_ip.c_str(), fs[k].src_port, fs[k].dst_ip.c_str(), fs[k].dst_port)) {
        accept[i] |= 1u << k;
        if (want[i] == PN_NO_STREAM) want[i] = k;
      }
    multi += __builtin_popcount(accept[i]) > 1;
  }
  std::printf("frames accepted by more than one filter: %u\n", multi);
  int fail_overlap = multi == 0;
  int fail = fail_overlap;
  uint32_t per_id[9] = {};
  for (uint32_t i = 0; i < n; i++) per_id[want[i] == PN_NO_STREAM ? 8 : want[i]]++;

  // 1. ids from the kernel (through GpuTcpStreams, both modes): capture via a probe handler
  //    is not possible for unmatched frames, so call pn_match_streams directly too
  {
    pn_ctx* ctx = nullptr;
    if (pn_open(0, &ctx)) return 3;
    std::vector<pn_stream_filter> pf;
    for (auto& f : fs) {
      pn_stream_filter q{};
      inet_pton(AF_INET, f.src_ip.c_str(), &q.src_ip);
      inet_pton(AF_INET, f.dst_ip.c_str(), &q.dst_ip);
      q.src_port = htons(f.src_port);
      q.dst_port = htons(f.dst_port);
      pf.push_back(q);
    }
    uint32_t* ids = nullptr;
    (void)hipHostMalloc((void**)&ids, sizeof(uint32_t) * n, hipHostMallocDefault);
    void* d_ring = nullptr;
    uint32_t* d_ids = nullptr;
    (void)hipMalloc(&d_ring, (size_t)stride * n);
    (void)hipMalloc((void**)&d_ids, sizeof(uint32_t) * n);
    (void)hipMemcpy(d_ring, ring, (size_t)stride * n, hipMemcpyHostToDevice);
    for (int zc = 0; zc < 2; zc++) {
      std::memset(ids, 0xAB, sizeof(uint32_t) * n);
      if (zc) {
        if (pn_match_streams(ctx, ring, stride, off, n, pf.data(), (uint32_t)pf.size(), ids, nullptr)) return 4;
      } else {
        if (pn_match_streams(ctx, d_ring, stride, off, n, pf.data(), (uint32_t)pf.size(), d_ids, nullptr)) return 4;
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(ids, d_ids, sizeof(uint32_t) * n, hipMemcpyDeviceToHost);
      }
      (void)hipDeviceSynchronize();
      uint32_t diff = 0;
      for (uint32_t i = 0; i < n; i++) diff += ids[i] != want[i];
      std::printf("match (%s): %u frames, %u ids differ from the reference filterPacket\n",
                  zc ? "zero-copy" : "device", n, diff);
      fail += diff != 0;
    }
    (void)hipFree(d_ring);
    (void)hipFree(d_ids);
    (void)hipHostFree(ids);
    pn_close(ctx);
  }
  std::printf("frames per stream id:");
  for (int k = 0; k < 9; k++) std::printf(" %u", per_id[k]);
  std::printf(" (last = none)\n");
  for (int k = 0; k < 9; k++) fail += per_id[k] == 0; // every filter (and "none") must be exercised

  // 2. reassembly: reference TcpStreams fed by the reference filter vs GpuTcpStreams
  const uint32_t msg_len[8] = {0, 100, 7, 0, 1000, 0, 3, 0};
  struct Log {
    std::vector<uint32_t> calls;
    std::vector<uint8_t> bytes;
  };
  std::vector<Log> ref_logs[2]; // [first-match only, every accepting stream]
  for (int all = 0; all < 2; all++) {
    std::vector<Log>& ref_log = ref_logs[all];
    ref_log.resize(8);
    std::vector<void*> rs(8);
    for (auto& r : rs) r = ref_new(1, 0);
    std::vector<uint8_t> rb(16u << 20);
    std::vector<uint32_t> rc(1u << 20);
    for (uint32_t k = 0; k < 8; k++) {
      RefLog rl{rb.data(), 0, rb.size(), rc.data(), 0, (uint32_t)rc.size()};
      for (uint32_t i = 0; i < n; i++)
        if (all ? (accept[i] >> k) & 1 : want[i] == k)
          ref_handle(rs[k], ring + (size_t)i * stride + off, flen[i], msg_len[k], &rl);
      ref_log[k].calls.assign(rc.begin(), rc.begin() + rl.n_calls);
      ref_log[k].bytes.assign(rb.begin(), rb.begin() + rl.n_bytes);
    }
    for (auto r : rs) ref_free(r);
  }
  for (int all = 0; all < 2; all++)
  for (int zc = 0; zc < 2; zc++)
    for (uint32_t chunk : {1000u, 4096u, 257u}) {
      const std::vector<Log>& ref_log = ref_logs[all];
      auto g = std::make_unique<GpuTcpStreams<>>();
      if (const char* e = g->init(0, stride, off, chunk, zc ? GpuRx::Mode::ZeroCopy : GpuRx::Mode::Copy)) {
        std::printf("init: %s\n", e);
        return 5;
      }
      g->setFirstMatchOnly(!all);
      for (auto& f : fs)
        if (g->addStream(f.src_ip.c_str(), f.src_port, f.dst_ip.c_str(), f.dst_port) < 0) return 6;
      std::vector<Log> got(8);
      const char* e = g->poll(ring, n, [&](int s, const uint8_t* d, uint32_t size) -> uint32_t {
        got[s].calls.push_back(size);
        const uint32_t keep = msg_len[s] ? size % msg_len[s] : 0;
        got[s].bytes.insert(got[s].bytes.end(), d, d + size - keep);
        return keep;
      });
      if (e) {
        std::printf("poll: %s\n", e);
        return 7;
      }
      uint32_t same = 0;
      uint64_t bytes = 0, calls = 0;
      for (int k = 0; k < 8; k++) {
        same += got[k].calls == ref_log[k].calls && got[k].bytes == ref_log[k].bytes;
        bytes += got[k].bytes.size();
        calls += got[k].calls.size();
      }
      std::printf("GpuTcpStreams (%s, chunk %u, %s): %u/8 streams identical to the reference (%llu calls, %llu bytes)\n",
                  zc ? "zero-copy" : "copy", chunk, all ? "every matching stream" : "first match only", same,
                  (unsigned long long)calls, (unsigned long long)bytes);
      fail += same != 8;
    }
  // the sniffed streams whose filter selects them alone are delivered intact
  for (int k : {0, 3}) {
    const auto& b = ref_logs[1][k].bytes;
    const bool whole = b.size() == sn[k].data.size() && std::equal(b.begin(), b.end(), sn[k].data.begin());
    std::printf("stream %d: %zu of %zu bytes, %s\n", k, b.size(), sn[k].data.size(), whole ? "intact" : "NOT intact");
    fail += !whole;
  }
  std::printf("%s\n", fail ? "FAIL" : "PASS");
  return fail ? 1 : 0;
}
