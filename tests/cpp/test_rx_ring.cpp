// RX-ring ingestion (include/pollnet_amd/rx_ring.hpp), SURVEY §8(f) rank 2.
//
//  cpu   SocketEthBatcher over a SOCK_SEQPACKET pair (message-preserving like a packet
//        socket): 5,000 C5 frames of 64..1514 B sent in bursts, drained into 2-KiB
//        slots; every frame's bytes and length must arrive intact and in order, and
//        a frame longer than its slot is cut at the slot (read(fd, buf, size) rule).
//  lo    AF_PACKET capture on "lo" (the reference's SocketEthReceiver use), when the
//        process may open a packet socket: a TCP connection over 127.0.0.1 sends 64
//        messages; the captured frames, classified by the oracle, must contain them
//        (loopback TCP checksums are left partial by the kernel: TCP_OK is not
//        expected; IP header checksums are valid).  SKIP when not permitted.
//  gpu   (when a device exists) the socket-filled pinned batch through GpuRx ZeroCopy
//        pollBatch, and an ef_vi-layout ring (512 RecvBuf slots, prefix 14) driven by a
//        wrapping RX-event run with discards through GpuRx::pollIndexed: every record
//        equal to the oracle's for the same bytes, dispatched in event order.
// argv[1]: "cpu" (no GPU part) or "all".  Exit 0 = pass.
#include <netinet/in.h>
#include <pthread.h>
#include <sys/socket.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "../../include/pollnet_amd/gpu_rx.hpp"
#include "../../include/pollnet_amd/rx_ring.hpp"
#include "../../include/pollnet_amd_gen.h"
#include "../../oracle/pn_oracle.h"

using namespace pollnet_amd;

static int g_fail = 0;
#define CHECK(c)                                               \
  do {                                                         \
    if (!(c)) {                                                \
      std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
      g_fail++;                                                \
    }                                                          \
  } while (0)

static uint32_t frame_len(const uint8_t* eth) { return 14u + ((uint32_t)eth[16] << 8 | eth[17]); }

// C5 frames (options, odd lengths) generated into 2-KiB slots at offset 2
static std::vector<uint8_t> gen(uint32_t cfg, uint32_t n) {
  pn_gen_params p{};
  p.cfg = cfg;
  p.n_flows = 1024;
  p.n_tw_flows = 32;
  p.max_conn_cnt = 1024;
  p.seed = 0x5EED0000u + cfg;
  std::vector<uint8_t> s((size_t)n * 2048);
  pn_gen_frames(&p, 0, n, s.data(), 2048, 2, 4);
  return s;
}

static void part_socketpair(uint8_t* batch, uint32_t stride, uint32_t off, uint32_t n, std::vector<uint32_t>& lens,
                            const std::vector<uint8_t>& src, uint32_t* filled) {
  int sv[2];
  CHECK(socketpair(AF_UNIX, SOCK_SEQPACKET, 0, sv) == 0);
  SocketEthBatcher b;
  CHECK(b.initFd(sv[1]));
  uint32_t got = 0, sent = 0;
  std::mt19937 rng(5);
  while (got < n) {
    const uint32_t burst = std::min<uint32_t>(n - sent, 1 + rng() % 64); // < the socket buffer
    for (uint32_t i = 0; i < burst; i++, sent++) {
      const uint8_t* eth = src.data() + (size_t)sent * 2048 + 2;
      CHECK(send(sv[0], eth, frame_len(eth), 0) == (ssize_t)frame_len(eth));
    }
    const uint32_t m = b.fill(batch + (size_t)got * stride, stride, off, n - got, lens.data() + got);
    got += m;
    if (sent == n && m == 0) break; // nothing more will come
  }
  CHECK(got == n);
  CHECK(b.fill(batch, stride, off, 1, nullptr) == 0); // drained
  uint32_t ok = 0;
  for (uint32_t i = 0; i < n; i++) {
    const uint8_t* eth = src.data() + (size_t)i * 2048 + 2;
    ok += lens[i] == frame_len(eth) && std::memcmp(batch + (size_t)i * stride + off, eth, lens[i]) == 0;
  }
  CHECK(ok == n);
  // a frame longer than the slot is cut at it
  std::vector<uint8_t> big(3000, 0x5a), small(256);
  CHECK(send(sv[0], big.data(), big.size(), 0) == 3000);
  uint32_t l = 0;
  CHECK(b.fill(small.data(), 256, 2, 1, &l) == 1 && l == 254);
  ::close(sv[0]);
  *filled = got;
  std::printf("socketpair: %u/%u frames intact (bursts, recvmmsg), oversize frame cut at the slot\n", ok, n);
}

static void part_loopback() {
  SocketEthBatcher cap;
  if (!cap.init("lo")) {
    std::printf("lo capture: SKIPPED (%s)\n", cap.getLastError());
    return;
  }
  // a TCP connection over loopback carrying 64 distinct messages
  int ls = socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  a.sin_port = 0;
  CHECK(bind(ls, (sockaddr*)&a, sizeof a) == 0 && listen(ls, 1) == 0);
  socklen_t al = sizeof a;
  getsockname(ls, (sockaddr*)&a, &al);
  const uint16_t port = ntohs(a.sin_port);
  int cs = socket(AF_INET, SOCK_STREAM, 0);
  CHECK(connect(cs, (sockaddr*)&a, sizeof a) == 0);
  int ss = accept(ls, nullptr, nullptr);
  int one = 1;
  setsockopt(cs, IPPROTO_TCP, 1 /*TCP_NODELAY*/, &one, sizeof one);
  cap.setRecvBuffer(8 << 20);
  std::vector<uint8_t> msg(1000);
  std::vector<uint8_t> rbuf(1 << 20);
  const uint32_t stride = 65536;
  std::vector<uint8_t> slots((size_t)stride * 64);
  std::vector<uint32_t> lens(64);
  uint32_t got = 0, data_frames = 0, ip_ok = 0;
  std::vector<std::pair<uint32_t, std::vector<uint8_t>>> segs; // (seq, payload) of data frames to the server
  auto drain = [&]() {
    for (;;) {
      const uint32_t m = cap.fill(slots.data(), stride, 2, 64, lens.data());
      if (m == 0) return;
      got += m;
      for (uint32_t i = 0; i < m; i++) {
        const uint8_t* eth = slots.data() + (size_t)i * stride + 2;
        pn_conn_entry empty{PN_EMPTY_KEY, 0, 0};
        pn_result r;
        orc_classify_frame(eth, stride - 2, &empty, 1, 0, 1, &r);
        if (r.flags & PN_F_NOT_TCP) continue;
        const uint16_t sport = (uint16_t)(eth[34] << 8 | eth[35]), dport = (uint16_t)(eth[36] << 8 | eth[37]);
        if (dport != port && sport != port) continue;
        ip_ok += (r.flags & PN_F_IP_OK) != 0;
        // lo's MTU is 64 KiB: coalesced segments may exceed efvitcp's 1500 clamp (TcpConn.h:472),
        // so take TcpStream's unclamped length tot_len - 20 - doff*4 (TcpStream.h:72-74)
        const int len = (int)((uint32_t)eth[16] << 8 | eth[17]) - 20 - 4 * (eth[46] >> 4);
        if (dport == port && len > 0) {
          data_frames++;
          segs.push_back({r.seq, std::vector<uint8_t>(eth + r.payload_off, eth + r.payload_off + len)});
        }
      }
    }
  };
  for (int k = 0; k < 64; k++) {
    for (size_t i = 0; i < msg.size(); i++) msg[i] = (uint8_t)(k * 31 + i);
    CHECK(send(cs, msg.data(), msg.size(), 0) == (ssize_t)msg.size());
    (void)recv(ss, rbuf.data(), rbuf.size(), MSG_DONTWAIT);
    drain();
  }
  for (int w = 0; w < 20; w++) { // let the tail reach the wire
    usleep(5000);
    (void)recv(ss, rbuf.data(), rbuf.size(), MSG_DONTWAIT);
    drain();
  }
  // the client's byte stream, rebuilt from the captured segments by sequence number
  std::vector<uint8_t> want;
  for (int k = 0; k < 64; k++)
    for (size_t i = 0; i < msg.size(); i++) want.push_back((uint8_t)(k * 31 + i));
  bool stream_ok = !segs.empty();
  if (stream_ok) {
    uint32_t base = segs[0].first;
    for (auto& x : segs) base = (int32_t)(x.first - base) < 0 ? x.first : base;
    std::vector<uint8_t> rebuilt(want.size(), 0);
    std::vector<bool> have(want.size(), false);
    for (auto& x : segs)
      for (size_t i = 0; i < x.second.size(); i++) {
        const uint32_t o = x.first - base + (uint32_t)i;
        if (o < rebuilt.size()) rebuilt[o] = x.second[i], have[o] = true;
      }
    stream_ok = rebuilt == want && std::all_of(have.begin(), have.end(), [](bool b) { return b; });
    if (!stream_ok && getenv("PN_DEBUG")) {
      for (auto& x : segs) std::printf("  seg seq+%u len %zu\n", x.first - base, x.second.size());
      size_t miss = 0, bad = 0;
      for (size_t i = 0; i < want.size(); i++) miss += !have[i], bad += have[i] && rebuilt[i] != want[i];
      std::printf("  missing %zu bytes, wrong %zu\n", miss, bad);
    }
  }
  std::printf("lo capture: %u frames, %u TCP data frames to port %u (IP_OK on %u), 64,000-B stream %s\n", got,
              data_frames, port, ip_ok, stream_ok ? "rebuilt intact" : "NOT rebuilt");
  CHECK(stream_ok);
  ::close(cs);
  ::close(ss);
  ::close(ls);
}

static void part_gpu(uint8_t* batch, uint32_t stride, uint32_t off, uint32_t n) {
  ConnTable t;
  CHECK(t.init(1024, 1024) == nullptr);
  pn_gen_params p{};
  p.cfg = 5;
  p.n_flows = 1024;
  p.n_tw_flows = 32;
  p.max_conn_cnt = 1024;
  p.seed = 0x5EED0005u;
  {
    pn_conn_table* raw = nullptr;
    pn_table_create(1024, 1024, &raw);
    pn_gen_conn_table(&p, raw);
    uint32_t ne = 0;
    uint64_t mask = 0;
    const pn_conn_entry* e = pn_table_entries(raw, &ne, &mask);
    for (uint32_t i = 0; i < ne; i++)
      if (e[i].key != PN_EMPTY_KEY) t.add(e[i].key, e[i].conn_id);
    pn_table_destroy(raw);
  }
  uint32_t tn = 0;
  uint64_t tm = 0;
  const pn_conn_entry* te = t.entries(&tn, &tm);
  auto oracle = [&](const uint8_t* eth, uint32_t avail) {
    pn_result r;
    orc_classify_frame(eth, avail, te, tn, tm, 1024, &r);
    return r;
  };
  { // the socket-filled batch, zero-copy
    GpuRx rx;
    CHECK(rx.init(0, stride, off, 1000, GpuRx::Mode::ZeroCopy) == nullptr);
    CHECK(rx.syncTable(t) == nullptr);
    uint32_t i = 0, diff = 0;
    auto chk = [&](const uint8_t* eth, const pn_result& r) {
      const pn_result e = oracle(eth, stride - off);
      diff += std::memcmp(&e, &r, sizeof r) != 0 || eth != batch + (size_t)i * stride + off;
      i++;
    };
    const char* err = rx.pollBatch(
        batch, n, t, [&](uint64_t, const pn_result& r, const uint8_t* eth, uint32_t) { chk(eth, r); },
        [&](uint64_t, uint32_t, const uint8_t* eth, const pn_result& r) { chk(eth, r); });
    CHECK(err == nullptr && i == n && diff == 0);
    std::printf("gpu: socket-filled pinned batch, zero-copy: %u records, %u differ from the oracle\n", i, diff);
  }
  { // ef_vi ring: 512 RecvBuf slots, prefix 14, RX events wrapping with discards
    EfviRingLayout lay;
    lay.prefix_len = 14;
    const uint32_t R = 512;
    uint8_t* ring = nullptr;
    CHECK(hipHostMalloc((void**)&ring, (size_t)R * lay.kRecvBufSize, hipHostMallocDefault) == hipSuccess);
    std::memset(ring, 0, (size_t)R * lay.kRecvBufSize);
    pn_gen_frames(&p, 777, R, ring, lay.kRecvBufSize, lay.frame_off(), 4);
    std::mt19937 rng(9);
    std::vector<uint32_t> ids;
    for (uint32_t k = 0; k < 3 * R; k++) // three laps of the ring, 7 % discards
      if (rng() % 100 >= 7) ids.push_back((400 + k) % R);
    std::vector<uint64_t> offs(ids.size());
    lay.offsets(ids.data(), (uint32_t)ids.size(), offs.data());
    GpuRx rx;
    CHECK(rx.init(0, lay.kRecvBufSize, lay.frame_off(), 300, GpuRx::Mode::ZeroCopy) == nullptr);
    CHECK(rx.syncTable(t) == nullptr);
    uint32_t i = 0, diff = 0;
    auto chk = [&](const uint8_t* eth, const pn_result& r) {
      const pn_result e = oracle(eth, lay.avail());
      diff += std::memcmp(&e, &r, sizeof r) != 0 || eth != ring + offs[i];
      i++;
    };
    const char* err = rx.pollIndexed(
        ring, offs.data(), (uint32_t)offs.size(), lay.eth_mod16(), lay.avail(), t,
        [&](uint64_t, const pn_result& r, const uint8_t* eth, uint32_t) { chk(eth, r); },
        [&](uint64_t, uint32_t, const uint8_t* eth, const pn_result& r) { chk(eth, r); });
    if (err) std::printf("pollIndexed: %s\n", err);
    CHECK(err == nullptr && i == offs.size() && diff == 0);
    std::printf("gpu: ef_vi ring (prefix %u), %zu RX events over 3 laps: %u records, %u differ from the oracle\n",
                lay.prefix_len, offs.size(), i, diff);
    (void)hipHostFree(ring);
  }
}

int main(int argc, char** argv) {
  const bool gpu = argc > 1 && std::strcmp(argv[1], "all") == 0;
  const uint32_t n = 5000, stride = 2048, off = 2;
  const std::vector<uint8_t> src = gen(5, n);
  uint8_t* batch = nullptr;
  std::vector<uint8_t> host_batch;
  if (gpu) {
    if (hipHostMalloc((void**)&batch, (size_t)stride * n, hipHostMallocDefault) != hipSuccess) return 2;
    std::memset(batch, 0, (size_t)stride * n);
  } else {
    host_batch.assign((size_t)stride * n, 0);
    batch = host_batch.data();
  }
  std::vector<uint32_t> lens(n);
  uint32_t filled = 0;
  part_socketpair(batch, stride, off, n, lens, src, &filled);
  part_loopback();
  if (gpu) part_gpu(batch, stride, off, filled);
  std::printf("%s\n", g_fail ? "FAIL" : "PASS");
  return g_fail ? 1 : 0;
}
