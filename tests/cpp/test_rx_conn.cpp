// CPU tests of the receive-side state machine (include/pollnet_amd/rx_conn.hpp).
//
// Part A — differential against the reference itself: the reassembly core shared by
// efvitcp's TcpConn::onPack (TcpConn.h:667-750) and pollnet's TcpStream::handlePacket
// (TcpStream.h:54-142) — ordered segment list, zero-copy delivery of the next
// in-order segment, buffered delivery otherwise, "remaining bytes" re-presented with
// the next data.  TcpStream.h compiles unmodified from /root/reference into
// oracle/_ref/libref_tcpstream.so; random segment streams (reordering, duplicates,
// re-segmented retransmissions, handlers that consume whole messages only) must
// produce the same sequence of handler calls (sizes) and the same consumed bytes.
// The scenarios stay inside the semantics both share: ACK set, no SYN/FIN/RST,
// <= 4 extents, stream < TcpStream's BUFSIZE/2.
//
// Part B — onPack-only rules, expected values worked out from TcpConn.h line by
// line: acceptability window, RST, ACK-less segments, FIN ordering, immediate-ACK
// rules, receive-buffer overrun, PAWS.
//
// Records come from the C oracle (the checker).  Exit 0 = pass; argv[1] = path of
// libref_tcpstream.so (Part A skipped, and reported, when it cannot be loaded).
#include <dlfcn.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>
#include <vector>

#include "../../include/pollnet_amd/rx_conn.hpp"
#include "segframes.hpp"

using namespace segtest;
using pollnet_amd::RxAck;
using pollnet_amd::RxConn;

static int g_fail = 0;
#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      std::printf("FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);          \
      g_fail++;                                                         \
    }                                                                   \
  } while (0)

template <uint32_t BUF, bool TS = false>
struct ConfT {
  static const uint32_t ConnRecvBufSize = BUF;
  static const bool TimestampOption = TS;
};

// handler consuming whole msg_len-byte messages (0: everything), logging like the ref shim
struct Log {
  std::vector<uint32_t> calls;
  std::vector<uint8_t> bytes;
  std::vector<uint32_t> fins;
  int resets = 0;
};
template <class C>
struct MsgHandler {
  uint32_t msg_len;
  Log* log;
  uint32_t onData(RxConn<C>&, const uint8_t* d, uint32_t n) {
    log->calls.push_back(n);
    const uint32_t keep = msg_len ? n % msg_len : 0;
    log->bytes.insert(log->bytes.end(), d, d + (n - keep));
    return keep;
  }
  void onFin(RxConn<C>&, const uint8_t* d, uint32_t n) {
    log->fins.push_back(n);
    log->bytes.insert(log->bytes.end(), d, d + n);
  }
  void onReset(RxConn<C>&) { log->resets++; }
};

// ---------------- Part A ----------------
struct RefLog {
  uint8_t* bytes;
  uint64_t n_bytes, cap_bytes;
  uint32_t* call_sizes;
  uint32_t n_calls, cap_calls;
};
struct RefApi {
  void* (*mk)();
  void (*fr)(void*);
  int (*handle)(void*, const uint8_t*, uint32_t, uint32_t, RefLog*);
};

static bool run_diff(const RefApi& ref, uint64_t seed, int* skipped) {
  std::mt19937_64 rng(seed);
  auto U = [&](uint32_t lo, uint32_t hi) { return lo + (uint32_t)(rng() % (hi - lo + 1)); };
  const uint32_t L = U(1, 200000);
  std::vector<uint8_t> stream(L);
  for (auto& b : stream) b = (uint8_t)rng();
  const uint32_t isn = (uint32_t)rng();
  // cut into packets
  std::vector<std::pair<uint32_t, uint32_t>> pk; // [begin, end) stream offsets
  for (uint32_t o = 0; o < L;) {
    const uint32_t n = std::min(L - o, U(1, 1460));
    pk.push_back({o, o + n});
    o += n;
  }
  // arrival: packet 0 first, then small block shuffles, duplicates, re-segmented resends
  const uint32_t W = U(1, 4);
  std::vector<std::pair<uint32_t, uint32_t>> arr{pk[0]};
  for (size_t b = 1; b < pk.size(); b += W) {
    const size_t e = std::min(pk.size(), b + W);
    std::vector<std::pair<uint32_t, uint32_t>> blk(pk.begin() + b, pk.begin() + e);
    std::shuffle(blk.begin(), blk.end(), rng);
    for (auto& x : blk) {
      arr.push_back(x);
      if (rng() % 20 == 0) arr.push_back(arr[rng() % arr.size()]); // duplicate of anything sent so far
      if (rng() % 30 == 0) {                                        // re-segmented retransmission
        const uint32_t a = U(0, x.second - 1), n = U(1, 1460);
        arr.push_back({a, std::min(L, a + n)});
      }
    }
  }
  const uint32_t msg_len = std::vector<uint32_t>{0, 1, 7, 100, 1000, 4096}[rng() % 6];

  using C = ConfT<(1u << 20)>;
  auto conn = std::make_unique<RxConn<C>>();
  conn->open(isn);
  Log mine;
  MsgHandler<C> h{msg_len, &mine};
  void* rs = ref.mk();
  std::vector<uint8_t> rbytes(L + 16);
  std::vector<uint32_t> rcalls(1 << 20);
  RefLog rl{rbytes.data(), 0, rbytes.size(), rcalls.data(), 0, (uint32_t)rcalls.size()};
  std::vector<uint8_t> frame(2048);
  bool ok = true;
  for (auto& x : arr) {
    Seg s;
    s.seq = isn + 1 + x.first;
    s.payload = stream.data() + x.first;
    s.len = x.second - x.first;
    const uint32_t flen = build(frame.data(), s);
    const pn_result r = classify(frame.data(), (uint32_t)frame.size());
    conn->onSegment(h, frame.data(), r);
    ref.handle(rs, frame.data(), flen, msg_len, &rl);
    if (conn->segCount() > 4) { // outside the shared semantics (TcpStream drops at 5 extents)
      ++*skipped;
      ref.fr(rs);
      return true;
    }
  }
  ref.fr(rs);
  if (rl.n_calls != mine.calls.size() || !std::equal(mine.calls.begin(), mine.calls.end(), rcalls.begin())) {
    std::printf("seed %llu: %zu calls vs ref %u\n", (unsigned long long)seed, mine.calls.size(), rl.n_calls);
    ok = false;
  }
  if (rl.n_bytes != mine.bytes.size() || !std::equal(mine.bytes.begin(), mine.bytes.end(), rbytes.begin())) {
    std::printf("seed %llu: %zu bytes vs ref %llu\n", (unsigned long long)seed, mine.bytes.size(),
                (unsigned long long)rl.n_bytes);
    ok = false;
  }
  // and both equal the stream prefix of whole messages
  const uint32_t whole = msg_len ? L - L % msg_len : L;
  if (mine.bytes.size() != whole || !std::equal(mine.bytes.begin(), mine.bytes.end(), stream.begin())) {
    std::printf("seed %llu: delivered %zu of %u bytes\n", (unsigned long long)seed, mine.bytes.size(), whole);
    ok = false;
  }
  return ok;
}

// ---------------- Part B ----------------
template <class C>
struct Rig {
  std::unique_ptr<RxConn<C>> c = std::make_unique<RxConn<C>>();
  Log log;
  MsgHandler<C> h{0, &log};
  std::vector<uint8_t> frame = std::vector<uint8_t>(2048);
  std::vector<uint8_t> data = std::vector<uint8_t>(1 << 16);
  uint32_t isn = 1000;
  Rig() {
    for (size_t i = 0; i < data.size(); i++) data[i] = (uint8_t)(i * 7 + 3);
    c->open(isn);
  }
  // segment carrying stream bytes [off, off+len)
  RxAck seg(uint32_t off, uint32_t len, uint8_t flags = ACK, std::vector<uint8_t> opts = {}) {
    Seg s;
    s.seq = isn + 1 + off;
    s.flags = flags;
    s.opts = std::move(opts);
    s.payload = data.data() + off;
    s.len = len;
    build(frame.data(), s);
    return c->onSegment(h, frame.data(), classify(frame.data(), (uint32_t)frame.size()));
  }
};

static std::vector<uint8_t> ts_opt(uint32_t tsval) {
  std::vector<uint8_t> o{1, 1, 8, 10, 0, 0, 0, 0, 0, 0, 0, 0};
  put32(o.data() + 4, tsval);
  return o;
}

static void part_b() {
  using C = ConfT<40960>; // efvitcp_server.cc's ConnRecvBufSize
  { // in-order delivery is zero-copy and the ACK is delayed until 2*RMSS unacked
    Rig<C> r;
    RxAck a = r.seg(0, 1000);
    CHECK(a.send && !a.immediate);
    CHECK(r.log.calls.size() == 1 && r.log.calls[0] == 1000);
    a = r.seg(1000, 1000);
    CHECK(a.send && !a.immediate); // 2000 < 2*1460
    a = r.seg(2000, 1000);
    CHECK(a.send && a.immediate); // 3000 >= 2920
    r.c->ackSent();
    CHECK(r.c->ackSeq() == r.isn + 1 + 3000 && !r.c->pendingAck());
    // the window was rebased after the second segment (2000 >= RMSS consumed, nothing
    // held), not after the third (1000 < RMSS since the rebase)
    CHECK(r.c->recvBufSeq() == r.isn + 1 + 2000 && r.c->segs()[0].second == 1000);
  }
  { // a hole: the later segment is buffered, an immediate ACK owed; filling delivers both
    Rig<C> r;
    RxAck a = r.seg(500, 500);
    CHECK(a.send && a.immediate && r.log.calls.empty() && r.c->segCount() == 2);
    a = r.seg(0, 500);
    CHECK(a.immediate); // a hole existed
    CHECK(r.log.calls.size() == 1 && r.log.calls[0] == 1000);
    CHECK(std::equal(r.log.bytes.begin(), r.log.bytes.end(), r.data.begin()) && r.log.bytes.size() == 1000);
  }
  { // old data only: not acceptable -> ACK (delayed), nothing delivered
    Rig<C> r;
    r.seg(0, 800);
    r.c->ackSent();
    RxAck a = r.seg(0, 800);
    CHECK(a.send && !a.immediate && r.log.calls.size() == 1);
    // partly old: trimmed, only the new bytes delivered
    a = r.seg(400, 800);
    CHECK(r.log.calls.size() == 2 && r.log.calls[1] == 400);
  }
  { // segment without ACK: no data processing
    Rig<C> r;
    RxAck a = r.seg(0, 100, PSH);
    CHECK(!a.send && r.log.calls.empty());
  }
  { // RST inside the window resets; outside it is ignored without an ACK
    Rig<C> r;
    RxAck a = r.seg(50000, 0, RST | ACK); // beyond the 40960-B window
    CHECK(!a.send && r.log.resets == 0 && !r.c->closed());
    a = r.seg(0, 0, RST);
    CHECK(r.log.resets == 1 && r.c->closed());
    a = r.seg(0, 100);
    CHECK(!a.send && r.log.calls.empty()); // closed: ignored
  }
  { // FIN with data in order: data, then onFin with what was left; FIN acked at once
    Rig<C> r;
    r.h.msg_len = 64; // leaves 1000 % 64 = 40 bytes
    RxAck a = r.seg(0, 1000, ACK | FIN);
    CHECK(r.log.calls.size() == 1 && r.log.calls[0] == 1000);
    CHECK(r.log.fins.size() == 1 && r.log.fins[0] == 40);
    CHECK(a.send && a.immediate && r.c->finReceived());
    CHECK(r.c->ackSeq() == r.isn + 1 + 1001);
    a = r.seg(1000, 10); // data after the FIN: no delivery
    CHECK(r.log.calls.size() == 1);
  }
  { // FIN beyond a hole is not processed; its retransmission after the fill is
    Rig<C> r;
    r.seg(500, 500, ACK | FIN);
    CHECK(!r.c->finReceived() && r.log.fins.empty());
    r.seg(0, 500);
    CHECK(!r.c->finReceived() && r.log.calls.size() == 1 && r.log.calls[0] == 1000);
    r.seg(1000, 0, ACK | FIN);
    CHECK(r.c->finReceived() && r.log.fins.size() == 1 && r.log.fins[0] == 0);
  }
  { // leftovers are re-presented with the next data (from recv_buf)
    Rig<C> r;
    r.h.msg_len = 300;
    r.seg(0, 1000); // consumes 900, keeps 100
    r.seg(1000, 1000);
    CHECK(r.log.calls.size() == 2 && r.log.calls[0] == 1000 && r.log.calls[1] == 1100);
    CHECK(r.log.bytes.size() == 1800 && std::equal(r.log.bytes.begin(), r.log.bytes.end(), r.data.begin()));
  }
  { // a handler that never consumes: buffer full -> reset + RST owed
    using S = ConfT<4096>;
    Rig<S> r;
    r.h.msg_len = 1u << 30; // keeps everything
    RxAck a;
    for (uint32_t off = 0; off < 4096 && !r.c->closed(); off += 1024) a = r.seg(off, 1024);
    CHECK(a.rst && r.log.resets == 1 && r.c->closed());
  }
  { // more than kMaxSegs holes: the last extent is evicted to make room
    Rig<C> r;
    for (int k = 5; k >= 1; k--) r.seg(k * 200, 100); // 5 extents: [0,0) + four... then a fifth
    CHECK(r.c->segCount() == 5);
    r.seg(100, 50); // new extent before the others: last one evicted
    CHECK(r.c->segCount() == 5 && r.c->segs()[1].first == 100 && r.c->segs()[4].first == 600);
  }
  { // PAWS: an older TSval is rejected (ACK owed), a newer one accepted and recorded
    using T = ConfT<40960, true>;
    Rig<T> r;
    r.c->open(r.isn, true, 5000);
    RxAck a = r.seg(0, 100, ACK, ts_opt(4000));
    CHECK(a.send && r.log.calls.empty());
    a = r.seg(0, 100, ACK, ts_opt(6000));
    CHECK(r.log.calls.size() == 1 && r.log.calls[0] == 100 && r.c->recentTs() == 6000);
  }
}

int main(int argc, char** argv) {
  part_b();
  std::printf("part B: %s\n", g_fail ? "FAIL" : "ok");
  const char* so = argc > 1 ? argv[1] : "oracle/_ref/libref_tcpstream.so";
  void* h = dlopen(so, RTLD_NOW);
  if (!h) {
    std::printf("part A: SKIPPED (%s)\n", dlerror());
    return g_fail ? 1 : 0;
  }
  RefApi ref{(void* (*)())dlsym(h, "ref_stream_new"), (void (*)(void*))dlsym(h, "ref_stream_free"),
             (int (*)(void*, const uint8_t*, uint32_t, uint32_t, RefLog*))dlsym(h, "ref_stream_handle")};
  if (!ref.mk || !ref.fr || !ref.handle) {
    std::printf("part A: missing ref_stream_* symbols\n");
    return 1;
  }
  const int n = argc > 2 ? std::atoi(argv[2]) : 300;
  int bad = 0, skipped = 0;
  for (int i = 0; i < n; i++)
    if (!run_diff(ref, 0xD1FF0000ull + i, &skipped)) bad++;
  std::printf("part A: %d/%d streams identical to the reference TcpStream (%d outside shared semantics)\n",
              n - bad - skipped, n - skipped, skipped);
  return (g_fail || bad) ? 1 : 0;
}
