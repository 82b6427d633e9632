// RxConn (include/pollnet_amd/rx_conn.hpp, the receive half of the engine's onPack) against the
// reference's OWN TcpConn::onPack (TcpConn.h:467-769, compiled from /root/reference by
// oracle/ref_server.hpp), segment by segment, over random segment streams.
//
// Per stream: one reference TcpConn is taken through reset / onSyn / sendSyn / onEstablished
// (TcpServer.h:88-93, 111-113) by a driver with TcpConn's friend access, then both it and an RxConn
// get the same frames.  After every segment the test compares
//   - the handler calls: onData / onFin (size and bytes, in order), onConnectionReset;
//   - the ACK owed: the frames the reference sent (ACK or RST: ack number and window) against
//     RxAck {send, immediate, rst}, and the delayed-ACK timer against the owed-but-delayed ACK;
//   - the state: recv_buf_seq, the extent list (segs, recv_seg_cnt), fin_received, pending_ack,
//     last_ack_seq, recent_ts, closed.
// Between segments the delayed ACK fires at random (onTimer, TcpConn.h:833-835 / ackSent()).
// Streams: reordering in blocks of up to 7 (5+ extents: the reference's MaxRecvSegs eviction),
// duplicates, overlapping re-segmented retransmissions, partly and wholly old data, data past the
// window, segments without ACK, with SYN, FIN in the middle / with the last data / beyond a hole,
// RSTs in and out of the window, handlers that consume everything, whole messages only (leaving
// bytes), or nothing (window full -> reset), oversize frames (tot_len > 1500, clamped), and with
// TimestampOption: stale / fresh TSvals (PAWS), aligned and walked option layouts.
//   argv: [streams per configuration] [seed]           exit 0 = pass
#include <arpa/inet.h>

#include <cstdio>
#include <cstdlib>
#include <memory>
#include <random>
#include <string>
#include <vector>

#include "../../include/pollnet_amd/rx_conn.hpp"
#include "../../oracle/ref_server.hpp"
#include "segframes.hpp"

using pollnet_amd::RxAck;
using pollnet_amd::RxConn;

template <uint32_t BUF, bool TS>
struct L1Conf {
  static const uint32_t ConnSendBufCnt = 64;
  static const bool SendBuf1K = true;
  static const uint32_t ConnRecvBufSize = BUF;
  static const uint32_t MaxConnCnt = 1;
  static const uint32_t MaxTimeWaitConnCnt = 1;
  static const uint32_t RecvBufCnt = 8;
  static const uint32_t SynRetries = 3;
  static const uint32_t TcpRetries = 10;
  static const uint32_t DelayedAckMS = 10;
  static const uint32_t MinRtoMS = 100;
  static const uint32_t MaxRtoMS = 30 * 1000;
  static const bool WindowScaleOption = false;
  static const bool TimestampOption = TS;
  static const int CongestionControlAlgo = 0;
  static const uint32_t UserTimerCnt = 2;
  struct UserData {};
};

// One handler event, as both sides report it.
struct Ev {
  char kind; // 'D' data, 'F' fin, 'R' reset
  std::vector<uint8_t> bytes;
  bool operator==(const Ev& o) const { return kind == o.kind && bytes == o.bytes; }
};
// An ACK / RST frame the connection sent: ack number, window, RST.
struct Ack {
  uint32_t ack;
  uint16_t win;
  bool rst;
  bool operator==(const Ack& o) const { return ack == o.ack && win == o.win && rst == o.rst; }
};

// Consumption policy shared by both handlers: consume whole msg-byte messages (0: all; ~0u: nothing).
static uint32_t keep(uint32_t msg, uint32_t n) {
  if (msg == 0) return 0;
  if (msg == ~0u) return n;
  return n % msg;
}

struct RefConnKey {};
namespace efvitcp {
// The driver: an explicit specialization of TcpConn's friend class template (TcpConn.h:138-139)
template <>
class TcpServer<RefConnKey> {
 public:
  template <class Conf>
  struct Drv {
    using Conn = TcpConn<Conf>;
    struct Handler {
      std::vector<Ev>* ev;
      uint32_t msg;
      void onConnectionEstablished(Conn&) {}
      void onMoreSendable(Conn&) {}
      void onConnectionClosed(Conn&) { ev->push_back({'C', {}}); }
      void onConnectionTimeout(Conn&) {}
      void onUserTimeout(Conn&, uint32_t) {}
      void onConnectionReset(Conn&) { ev->push_back({'R', {}}); }
      uint32_t onData(Conn&, const uint8_t* d, uint32_t n) {
        ev->push_back({'D', std::vector<uint8_t>(d, d + n)});
        return keep(msg, n);
      }
      void onFin(Conn&, uint8_t* d, uint32_t n) { ev->push_back({'F', std::vector<uint8_t>(d, d + n)}); }
    };
    std::unique_ptr<Core<Conf>> core{new Core<Conf>()};
    std::unique_ptr<Conn> conn{new Conn()};
    std::vector<Ack> sent;
    std::vector<Ev> ev;
    Handler h{&ev, 0};

    static uint32_t fill0(void*, uint8_t*, uint32_t, uint32_t, uint32_t) { return 0; }
    static void capture(void* self, const uint8_t* eth, uint32_t) {
      const uint8_t* tcp = eth + 34;
      static_cast<Drv*>(self)->sent.push_back(
          {(uint32_t)tcp[8] << 24 | (uint32_t)tcp[9] << 16 | (uint32_t)tcp[10] << 8 | tcp[11], (uint16_t)(tcp[14] << 8 | tcp[15]), (tcp[13] & 4) != 0});
    }
    // TcpServer.h:88-93: entry, reset, onSyn, sendSyn; then the handshake ACK (TcpServer.h:111-113)
    uint32_t open(uint8_t* syn_eth, uint32_t peer_ip_be, uint16_t peer_port_be) {
      RefEnv& env = refEnv();
      env.link = this;
      env.fill = fill0;
      env.send = capture;
      env.init_ns = (int64_t)4242 << 20;
      env.local_ip = htonl(0x0a000001);
      core->init("");
      conn->init(core.get(), (uint8_t*)core->getSendBuf(0), 0);
      const uint64_t key = connHashKey(peer_ip_be, peer_port_be);
      uint32_t conn_id = core->conns[core->conn_cnt++];
      core->addConnEntry(core->findConnEntry(key), key, conn_id);
      uint8_t mac[6] = {2, 0, 0, 0, 0, 2};
      conn->reset(htons(1234), mac, peer_ip_be, peer_port_be);
      conn->onSyn((IpHeader*)(syn_eth + 14));
      conn->sendSyn();
      const uint32_t srv_isn = ntohl(conn->getSendBuf(0)->tcp_hdr.seq_num);
      return srv_isn;
    }
    void established(uint8_t* ack_eth) {
      conn->onEstablished(h, (IpHeader*)(ack_eth + 14));
      conn->onPack(h, (IpHeader*)(ack_eth + 14));
    }
    void pack(uint8_t* eth) { conn->onPack(h, (IpHeader*)(eth + 14)); }
    bool delayedArmed() { return !conn->timers[1].isUnlinked(); }
    void fireDelayed() { // the delayed-ACK timer expiring (Core::pollTime -> TcpConn::onTimer)
      conn->timers[1].unlink();
      conn->onTimer(h, &conn->timers[1]);
    }
    bool closed() { return conn->isClosed(); }
    uint32_t recvBufSeq() { return conn->recv_buf_seq; }
    uint32_t segCnt() { return conn->recv_seg_cnt; }
    std::pair<uint32_t, uint32_t> seg(uint32_t i) { return conn->segs[i]; }
    bool finReceived() { return conn->fin_received; }
    bool pendingAck() { return conn->pending_ack; }
    uint32_t lastAckSeq() { return conn->last_ack_seq; }
    uint32_t recentTs() { return conn->recent_ts; }
  };
};
} // namespace efvitcp

template <class Conf>
struct Prod {
  struct H {
    std::vector<Ev>* ev;
    uint32_t msg;
    uint32_t onData(RxConn<Conf>&, const uint8_t* d, uint32_t n) {
      ev->push_back({'D', std::vector<uint8_t>(d, d + n)});
      return keep(msg, n);
    }
    void onFin(RxConn<Conf>&, const uint8_t* d, uint32_t n) { ev->push_back({'F', std::vector<uint8_t>(d, d + n)}); }
    void onReset(RxConn<Conf>&) { ev->push_back({'R', {}}); }
  };
  std::unique_ptr<RxConn<Conf>> c{new RxConn<Conf>()};
  std::vector<Ack> sent;
  std::vector<Ev> ev;
  H h{&ev, 0};
  bool delayed = false; // an ACK owed on the delayed-ACK timer
  void ackNow(bool rst = false) {
    sent.push_back({c->ackSeq(), (uint16_t)std::min<uint32_t>(65535u, c->window()), rst});
    c->ackSent();
    delayed = false;
  }
  // what the engine does with RxAck (tcp_engine.hpp onPack / sendAck)
  void apply(const RxAck& a) {
    if (c->closed()) delayed = false; // onClose unlinks every timer (TcpConn.h:455)
    if (a.rst) {
      ackNow(true); // close(): RST carrying the ACK (TcpConn.h:96-105)
      return;
    }
    if (!a.send) return;
    if (a.immediate) ackNow();
    else delayed = true;
  }
};

struct Stats {
  uint64_t streams = 0, segments = 0, max_extents_hit = 0, resets = 0, fins = 0, window_full = 0, paws_drops = 0,
           delayed_fired = 0, evicted = 0;
};

static int g_fail = 0;

template <uint32_t BUF, bool TS>
static bool one_stream(uint64_t seed, Stats& st) {
  using Conf = L1Conf<BUF, TS>;
  std::mt19937_64 rng(seed);
  auto U = [&](uint32_t lo, uint32_t hi) { return lo + (uint32_t)(rng() % ((uint64_t)hi - lo + 1)); };
  const uint32_t L = U(0, 1 + (uint32_t)(rng() % 4) * 20000);
  std::vector<uint8_t> stream(L + 4096);
  for (auto& b : stream) b = (uint8_t)rng();
  const uint32_t isn = (uint32_t)rng();
  const uint32_t peer_ip = 0x0a000002 + (uint32_t)(rng() % 1000);
  const uint16_t peer_port = (uint16_t)U(1024, 65535);
  const uint32_t msg = std::vector<uint32_t>{0, 0, 1, 7, 100, 1000, 4096, ~0u}[rng() % 8];
  uint32_t tsval = (uint32_t)rng(); // the peer's clock
  const bool use_ts = TS && rng() % 4 != 0;
  const uint32_t max_pay = use_ts ? 1448 : 1460;

  auto mkopts = [&](uint32_t tv) -> std::vector<uint8_t> {
    if (!use_ts) {
      if (rng() % 10 == 0) return {1, 1, 1, 0}; // NOPs + EOL (no timestamp)
      return {};
    }
    std::vector<uint8_t> o;
    switch (rng() % 4) {
      case 0: o = {8, 10}; break;                       // unaligned: found by the option walk
      case 1: o = {1, 8, 10}; break;
      case 2: o = {4, 2, 8, 10}; break;                 // SACK-permitted, then TS
      default: o = {1, 1, 8, 10}; break;                // the aligned layout (TcpConn.h:477)
    }
    const size_t p = o.size();
    o.resize(p + 8);
    segtest::put32(o.data() + p, tv);
    segtest::put32(o.data() + p + 4, 0);
    return o;
  };

  using Drv = efvitcp::TcpServer<RefConnKey>::Drv<Conf>;
  std::unique_ptr<Drv> ref(new Drv());
  Prod<Conf> prod;
  ref->h.msg = prod.h.msg = msg;
  std::vector<uint8_t> frame(4096);
  auto build = [&](uint32_t seq, uint32_t ack, uint8_t flags, const uint8_t* p, uint32_t n, std::vector<uint8_t> o,
                   uint32_t oversize = 0) {
    segtest::Seg s;
    s.src_ip = peer_ip;
    s.src_port = peer_port;
    s.seq = seq;
    s.ack = ack;
    s.flags = flags;
    s.opts = std::move(o);
    s.payload = p;
    s.len = n + oversize;
    std::memset(frame.data(), 0, frame.size());
    segtest::build(frame.data(), s);
  };
  // SYN (MSS, and the TS option when negotiated), the server's SYN-ACK, the handshake ACK
  {
    std::vector<uint8_t> o{2, 4, 0x05, 0xb4};
    if (use_ts) {
      o.insert(o.end(), {1, 1, 8, 10, 0, 0, 0, 0, 0, 0, 0, 0});
      segtest::put32(o.data() + 8, tsval);
    }
    build(isn, 0, segtest::SYN, nullptr, 0, o);
  }
  const uint32_t srv_isn = ref->open(frame.data(), htonl(peer_ip), htons(peer_port));
  prod.c->open(isn, use_ts, tsval);
  prod.c->ackSent(); // the SYN-ACK carried the ACK (sendSyn -> sendBuf -> updateLastAck)
  const uint32_t ack = srv_isn + 1;
  build(isn + 1, ack, segtest::ACK, nullptr, 0, mkopts(tsval));
  ref->sent.clear();
  ref->established(frame.data());
  prod.apply(prod.c->onSegment(prod.h, frame.data(), segtest::classify(frame.data(), (uint32_t)frame.size())));

  // the schedule: packets in blocks shuffled, duplicates, overlaps, odd flags and places
  struct S {
    uint32_t off, len;
    uint8_t flags;
    int32_t shift;
    int32_t ts_delta;
    uint32_t oversize;
  };
  std::vector<std::pair<uint32_t, uint32_t>> pk;
  for (uint32_t o = 0; o < L;) {
    const uint32_t n = std::min(L - o, U(1, max_pay));
    pk.push_back({o, n});
    o += n;
  }
  std::vector<S> sched;
  const uint32_t W = U(1, 8);
  for (size_t b = 0; b < pk.size(); b += W) {
    std::vector<std::pair<uint32_t, uint32_t>> blk(pk.begin() + b, pk.begin() + std::min(pk.size(), b + W));
    std::shuffle(blk.begin(), blk.end(), rng);
    for (auto& x : blk) {
      S s{x.first, x.second, (uint8_t)(segtest::ACK | segtest::PSH), 0, 1, 0};
      const uint32_t r = (uint32_t)(rng() % 1000);
      if (r < 25) s.flags = segtest::PSH;
      else if (r < 40) s.flags |= segtest::SYN;
      else if (r < 47) s.flags |= segtest::FIN;
      else if (r < 70) s.shift = (int32_t)(BUF + rng() % 100000);
      else if (r < 90) s.shift = -(int32_t)(1 + rng() % 70000);
      else if (r < 110) s.shift = (int32_t)(rng() % (2 * BUF)) - (int32_t)BUF;
      else if (r < 125) s.ts_delta = -(int32_t)(1 + rng() % 100000); // stale TSval (PAWS)
      else if (r < 135) s.oversize = U(1, 400);                     // tot_len > 1500: clamped
      if (x.first + x.second == L && rng() % 2) s.flags |= segtest::FIN; // FIN with the last data
      sched.push_back(s);
      if (rng() % 9 == 0) sched.push_back(sched[rng() % sched.size()]);
      if (rng() % 11 == 0) {
        const uint32_t a = U(0, x.first + x.second - 1);
        sched.push_back({a, std::min(L - a, U(1, max_pay)), (uint8_t)(segtest::ACK | segtest::PSH), 0, 1, 0});
      }
      const uint32_t q = (uint32_t)(rng() % 1000);
      if (q < 3) sched.push_back({x.first, 0, segtest::RST, 0, 1, 0});
      else if (q < 8) sched.push_back({x.first, 0, (uint8_t)(segtest::RST | segtest::ACK), (int32_t)(BUF + 5000), 1, 0});
    }
  }
  // the tail: the whole stream again in order with a FIN (repair), then a bare FIN
  for (uint32_t o = 0; o < L; o += max_pay)
    sched.push_back({o, std::min(max_pay, L - o), (uint8_t)(segtest::ACK | segtest::PSH | (o + max_pay >= L ? segtest::FIN : 0)), 0, 1, 0});
  sched.push_back({L, 0, (uint8_t)(segtest::ACK | segtest::FIN), 0, 1, 0});

  st.streams++;
  char why[200] = "";
  for (size_t k = 0; k < sched.size() && !ref->closed(); k++) {
    const S& s = sched[k];
    tsval += s.ts_delta > 0 ? (uint32_t)s.ts_delta : 0;
    const uint32_t tv = s.ts_delta < 0 ? tsval + (uint32_t)s.ts_delta : tsval;
    build(isn + 1 + s.off + (uint32_t)s.shift, (s.flags & segtest::ACK) ? ack : 0, s.flags, stream.data() + s.off, s.len,
          mkopts(tv), s.oversize);
    ref->sent.clear();
    prod.sent.clear();
    ref->ev.clear();
    prod.ev.clear();
    const uint32_t segs_before = ref->segCnt();
    ref->pack(frame.data());
    const pn_result rec = segtest::classify(frame.data(), (uint32_t)frame.size());
    prod.apply(prod.c->onSegment(prod.h, frame.data(), rec));
    st.segments++;
    if (ref->segCnt() == 5) st.max_extents_hit++;
    if (segs_before == 5 && ref->segCnt() == 5 && ref->ev.empty() && s.shift == 0) st.evicted++;
    for (auto& e : ref->ev) st.resets += e.kind == 'R', st.fins += e.kind == 'F';
    if (use_ts && s.ts_delta < 0 && s.shift == 0 && (s.flags & segtest::ACK) && s.len && ref->ev.empty()) st.paws_drops++;
    if (ref->closed() && ref->sent.size() == 1 && ref->sent[0].rst && ref->sent[0].win == 0) st.window_full++;
    // between segments the delayed ACK may fire
    if (rng() % 3 == 0 && ref->delayedArmed()) {
      st.delayed_fired++;
      ref->fireDelayed();
      if (prod.delayed) prod.ackNow();
    }
    if (ref->ev.size() != prod.ev.size() || !std::equal(ref->ev.begin(), ref->ev.end(), prod.ev.begin()))
      std::snprintf(why, sizeof why, "handler calls (%zu vs %zu)", ref->ev.size(), prod.ev.size());
    else if (ref->sent.size() != prod.sent.size() || !std::equal(ref->sent.begin(), ref->sent.end(), prod.sent.begin()))
      std::snprintf(why, sizeof why, "frames sent (%zu vs %zu%s)", ref->sent.size(), prod.sent.size(),
                    ref->sent.empty() ? "" : ref->sent[0].rst ? ", ref RST" : "");
    else if (ref->delayedArmed() != prod.delayed)
      std::snprintf(why, sizeof why, "delayed ACK timer %d vs owed %d", ref->delayedArmed(), prod.delayed);
    else if (ref->closed() != prod.c->closed())
      std::snprintf(why, sizeof why, "closed %d vs %d", ref->closed(), prod.c->closed());
    else if (!ref->closed()) {
      bool segs_eq = ref->segCnt() == prod.c->segCount();
      for (uint32_t i = 0; segs_eq && i < ref->segCnt(); i++)
        segs_eq = ref->seg(i).first == prod.c->segs()[i].first && ref->seg(i).second == prod.c->segs()[i].second;
      if (ref->recvBufSeq() != prod.c->recvBufSeq() || !segs_eq)
        std::snprintf(why, sizeof why, "extents (recv_buf_seq %u vs %u, %u vs %u extents)", ref->recvBufSeq(),
                      prod.c->recvBufSeq(), ref->segCnt(), prod.c->segCount());
      else if (ref->finReceived() != prod.c->finReceived())
        std::snprintf(why, sizeof why, "fin_received %d vs %d", ref->finReceived(), prod.c->finReceived());
      else if (ref->pendingAck() != prod.c->pendingAck())
        std::snprintf(why, sizeof why, "pending_ack %d vs %d", ref->pendingAck(), prod.c->pendingAck());
      else if (ref->lastAckSeq() != prod.c->lastAckSeq())
        std::snprintf(why, sizeof why, "last_ack_seq %u vs %u", ref->lastAckSeq(), prod.c->lastAckSeq());
      else if (use_ts && ref->recentTs() != prod.c->recentTs())
        std::snprintf(why, sizeof why, "recent_ts %u vs %u", ref->recentTs(), prod.c->recentTs());
    }
    if (why[0]) {
      std::printf("FAIL BUF %u TS %d seed %llu segment %zu (off %u len %u flags 0x%02x shift %d ts %d): %s\n", BUF, TS,
                  (unsigned long long)seed, k, s.off, s.len, s.flags, s.shift, s.ts_delta, why);
      g_fail++;
      return false;
    }
  }
  return true;
}

template <uint32_t BUF, bool TS>
static void config(uint32_t n, uint64_t seed0) {
  Stats st;
  uint32_t bad = 0;
  for (uint32_t i = 0; i < n; i++)
    if (!one_stream<BUF, TS>(seed0 + i * 0x9E3779B97F4A7C15ull + BUF * 2 + TS, st) && ++bad >= 5) break;
  std::printf("ConnRecvBufSize %6u TimestampOption %d: %llu streams, %llu segments, %s; 5 extents reached %llu times, "
              "%llu evictions, %llu resets, %llu FINs delivered, %llu window-full aborts, %llu PAWS drops, %llu delayed "
              "ACKs fired\n",
              BUF, TS, (unsigned long long)st.streams, (unsigned long long)st.segments, bad ? "FAIL" : "identical",
              (unsigned long long)st.max_extents_hit, (unsigned long long)st.evicted, (unsigned long long)st.resets,
              (unsigned long long)st.fins, (unsigned long long)st.window_full, (unsigned long long)st.paws_drops,
              (unsigned long long)st.delayed_fired);
}

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)std::atoi(argv[1]) : 1300;
  const uint64_t seed = argc > 2 ? std::strtoull(argv[2], nullptr, 0) : 0x5EEDC0DEull;
  config<4096, false>(n, seed);
  config<8192, false>(n, seed);
  config<40960, false>(n, seed);
  config<131072, false>(n, seed);
  config<4096, true>(n, seed);
  config<8192, true>(n, seed);
  config<40960, true>(n, seed);
  config<131072, true>(n, seed);
  std::printf("%s\n", g_fail ? "FAIL" : "PASS");
  return g_fail ? 1 : 0;
}
