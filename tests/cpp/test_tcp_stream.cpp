// StreamReassembler (include/pollnet_amd/tcp_stream.hpp) against the reference itself:
// pollnet's TcpStream.h compiled unmodified into oracle/_ref/libref_tcpstream.so, in
// four instantiations — WaitForResend true/false x BUFSIZE 1 MiB / 4 KiB.
//
// Random sniffed streams drive both packet by packet: optional leading SYN, SYN
// restarts with a new ISN mid-capture, block reordering wide enough to exhaust the 5
// extents, duplicates, re-segmented retransmissions, lost segments (gaps WaitForResend
// = false skips), zero-length segments, streams longer than the 4-KiB buffer (drops
// and compaction), and handlers that consume whole messages only.  Every packet's
// return value, every handler call's size and every consumed byte must be identical.
// Exit 0 = pass.  argv[1] = libref_tcpstream.so, argv[2] = streams per instantiation.
#include <dlfcn.h>

#include <cstdio>
#include <cstdlib>
#include <memory>
#include <random>
#include <vector>

#include "../../include/pollnet_amd/tcp_stream.hpp"
#include "segframes.hpp"

using namespace segtest;

struct RefLog {
  uint8_t* bytes;
  uint64_t n_bytes, cap_bytes;
  uint32_t* call_sizes;
  uint32_t n_calls, cap_calls;
};
struct RefApi {
  void* (*mk)(int, int);
  void (*fr)(void*);
  int (*handle)(void*, const uint8_t*, uint32_t, uint32_t, RefLog*);
};

struct Stats {
  uint64_t packets = 0, taken = 0, calls = 0, bytes = 0, drops_full = 0;
};

template <bool W, uint32_t B>
static bool run_one(const RefApi& ref, uint64_t seed, Stats& st) {
  std::mt19937_64 rng(seed);
  auto U = [&](uint32_t lo, uint32_t hi) { return lo + (uint32_t)(rng() % (hi - lo + 1)); };
  const uint32_t L = U(0, B > 4096 ? 300000 : 20000);
  std::vector<uint8_t> stream(L + 1);
  for (auto& b : stream) b = (uint8_t)rng();
  uint32_t isn = (uint32_t)rng();
  std::vector<Seg> pk;
  auto data_seg = [&](uint32_t a, uint32_t b) {
    Seg s;
    s.seq = isn + 1 + a;
    s.flags = ACK | PSH;
    s.payload = stream.data() + a;
    s.len = b - a;
    return s;
  };
  if (rng() % 2) { // a SYN first: the stream starts at isn + 1
    Seg syn;
    syn.seq = isn;
    syn.flags = SYN;
    pk.push_back(syn);
  }
  std::vector<std::pair<uint32_t, uint32_t>> cuts;
  for (uint32_t o = 0; o < L;) {
    const uint32_t n = std::min(L - o, U(1, 1460));
    cuts.push_back({o, o + n});
    o += n;
  }
  const uint32_t W_ = U(1, 8); // reorder block: up to 8 -> more than 5 extents at times
  const bool lossy = rng() % 3 == 0;
  for (size_t b = 0; b < cuts.size(); b += W_) {
    std::vector<std::pair<uint32_t, uint32_t>> blk(cuts.begin() + b, cuts.begin() + std::min(cuts.size(), b + W_));
    if (b) std::shuffle(blk.begin(), blk.end(), rng); // keep the very first segment first
    for (auto& x : blk) {
      if (lossy && b && rng() % 25 == 0) continue; // lost
      pk.push_back(data_seg(x.first, x.second));
      if (rng() % 20 == 0) pk.push_back(pk[rng() % pk.size()]);
      if (rng() % 30 == 0) {
        const uint32_t a = U(0, x.second - 1);
        pk.push_back(data_seg(a, std::min(L, a + U(0, 1460))));
      }
    }
    if (rng() % 400 == 0) { // the stream restarts: SYN with a new ISN, offsets from 0 again
      isn = (uint32_t)rng();
      Seg syn;
      syn.seq = isn;
      syn.flags = SYN | (rng() % 2 ? ACK : 0);
      pk.push_back(syn);
      pk.push_back(data_seg(0, std::min<uint32_t>(L, 500)));
    }
  }
  const uint32_t msg_len = std::vector<uint32_t>{0, 1, 7, 100, 1000}[rng() % 5];

  pollnet_amd::StreamReassembler<W, B> mine;
  std::vector<uint32_t> my_calls;
  std::vector<uint8_t> my_bytes;
  std::vector<int> my_ret;
  void* rs = ref.mk(W, B == 4096);
  std::vector<uint8_t> rbytes(8u << 20);
  std::vector<uint32_t> rcalls(1u << 20);
  RefLog rl{rbytes.data(), 0, rbytes.size(), rcalls.data(), 0, (uint32_t)rcalls.size()};
  std::vector<int> ref_ret;
  std::vector<uint8_t> frame(2048);
  for (const Seg& s : pk) {
    const uint32_t flen = build(frame.data(), s);
    my_ret.push_back(mine.handlePacket(frame.data(), [&](const uint8_t* d, uint32_t n) -> uint32_t {
      my_calls.push_back(n);
      const uint32_t keep = msg_len ? n % msg_len : 0;
      my_bytes.insert(my_bytes.end(), d, d + (n - keep));
      return keep;
    }));
    ref_ret.push_back(ref.handle(rs, frame.data(), flen, msg_len, &rl));
  }
  ref.fr(rs);
  bool ok = my_ret == ref_ret && rl.n_calls == my_calls.size() &&
            std::equal(my_calls.begin(), my_calls.end(), rcalls.begin()) && rl.n_bytes == my_bytes.size() &&
            std::equal(my_bytes.begin(), my_bytes.end(), rbytes.begin());
  if (!ok) {
    size_t k = std::mismatch(my_ret.begin(), my_ret.end(), ref_ret.begin()).first - my_ret.begin();
    std::printf("W=%d B=%u seed %llu: first return difference at packet %zu/%zu; calls %zu vs %u; bytes %zu vs %llu\n",
                (int)W, B, (unsigned long long)seed, k, pk.size(), my_calls.size(), rl.n_calls, my_bytes.size(),
                (unsigned long long)rl.n_bytes);
  }
  st.packets += pk.size();
  for (int r : my_ret) st.taken += r;
  st.calls += my_calls.size();
  st.bytes += my_bytes.size();
  return ok;
}

int main(int argc, char** argv) {
  const char* so = argc > 1 ? argv[1] : "oracle/_ref/libref_tcpstream.so";
  void* h = dlopen(so, RTLD_NOW);
  if (!h) {
    std::printf("SKIPPED (%s)\n", dlerror());
    return 0;
  }
  RefApi ref{(void* (*)(int, int))dlsym(h, "ref_stream_new2"), (void (*)(void*))dlsym(h, "ref_stream_free"),
             (int (*)(void*, const uint8_t*, uint32_t, uint32_t, RefLog*))dlsym(h, "ref_stream_handle")};
  if (!ref.mk || !ref.fr || !ref.handle) {
    std::printf("missing ref_stream_* symbols\n");
    return 1;
  }
  const int n = argc > 2 ? std::atoi(argv[2]) : 200;
  int bad = 0;
  Stats st[4];
  for (int i = 0; i < n; i++) {
    bad += !run_one<true, (1u << 20)>(ref, 0x5717EA0000ull + i, st[0]);
    bad += !run_one<false, (1u << 20)>(ref, 0x5717EB0000ull + i, st[1]);
    bad += !run_one<true, 4096>(ref, 0x5717EC0000ull + i, st[2]);
    bad += !run_one<false, 4096>(ref, 0x5717ED0000ull + i, st[3]);
  }
  const char* names[4] = {"<true, 1 MiB>", "<false, 1 MiB>", "<true, 4 KiB>", "<false, 4 KiB>"};
  for (int k = 0; k < 4; k++)
    std::printf("TcpStream%s: %llu packets (%llu taken), %llu handler calls, %llu bytes consumed\n", names[k],
                (unsigned long long)st[k].packets, (unsigned long long)st[k].taken, (unsigned long long)st[k].calls,
                (unsigned long long)st[k].bytes);
  std::printf("%d/%d streams identical to the reference TcpStream\n", 4 * n - bad, 4 * n);

  // GpuTcpStreams::filterPacket (the host filter for a frame's later streams) vs the reference's filterPacket:
  // random headers drawn from small pools (so filters hit), non-IPv4 / non-TCP frames, wildcard filters
  auto ref_filter = (int (*)(const uint8_t*, uint32_t, const char*, uint16_t, const char*, uint16_t))dlsym(
      h, "ref_filter_packet");
  if (!ref_filter) {
    std::printf("missing ref_filter_packet\n");
    return 1;
  }
  std::mt19937_64 rng(0xF117E4);
  const uint32_t hosts[4] = {0x0a000001, 0x0a000002, 0xc0a80105, 0x7f000001};
  const uint16_t ports[4] = {1234, 40000, 80, 5000};
  uint32_t fdiff = 0, fpass = 0, fcases = 0;
  uint8_t fr[64];
  for (int i = 0; i < 200000; i++) {
    for (auto& b : fr) b = (uint8_t)rng();
    fr[12] = 0x08, fr[13] = rng() % 8 ? 0x00 : 0x06;
    fr[23] = rng() % 8 ? 6 : 17;
    const uint32_t sip = hosts[rng() % 4], dip = hosts[rng() % 4];
    const uint16_t sp = ports[rng() % 4], dp = ports[rng() % 4];
    for (int k = 0; k < 4; k++) fr[26 + k] = (uint8_t)(sip >> (24 - 8 * k)), fr[30 + k] = (uint8_t)(dip >> (24 - 8 * k));
    fr[34] = sp >> 8, fr[35] = sp & 255, fr[36] = dp >> 8, fr[37] = dp & 255;
    const uint32_t fs = rng() % 2 ? hosts[rng() % 4] : 0, fd = rng() % 2 ? hosts[rng() % 4] : 0;
    const uint16_t fsp = rng() % 2 ? ports[rng() % 4] : 0, fdp = rng() % 2 ? ports[rng() % 4] : 0;
    char s_ip[32], d_ip[32];
    std::snprintf(s_ip, sizeof s_ip, "%u.%u.%u.%u", fs >> 24, (fs >> 16) & 255, (fs >> 8) & 255, fs & 255);
    std::snprintf(d_ip, sizeof d_ip, "%u.%u.%u.%u", fd >> 24, (fd >> 16) & 255, (fd >> 8) & 255, fd & 255);
    pn_stream_filter f{};
    inet_pton(AF_INET, s_ip, &f.src_ip);
    inet_pton(AF_INET, d_ip, &f.dst_ip);
    f.src_port = htons(fsp);
    f.dst_port = htons(fdp);
    const bool want = ref_filter(fr, 64, s_ip, fsp, d_ip, fdp) != 0;
    const bool got = pollnet_amd::GpuTcpStreams<>::filterPacket(f, fr);
    fdiff += want != got;
    fpass += want;
    fcases++;
  }
  std::printf("filterPacket: %u frames, %u pass, %u differ from the reference\n", fcases, fpass, fdiff);
  return bad || fdiff ? 1 : 0;
}
