// GPU end-to-end check of the receive-side server loop (include/pollnet_amd/gpu_tcp_rx.hpp):
// many TCP flows (SYN, reordered / duplicated / corrupted-then-resent data, FIN),
// TIME_WAIT flows and unknown flows, interleaved into one ring and polled in batches
// whose boundaries split flows (so connections open and close mid-batch).
//
// The checker is a sequential twin with the reference's semantics (Core::pollNet,
// Core.h:494-552): every frame is classified by the C oracle against the *live*
// table at that moment and dispatched at once — no batch snapshot.  The GPU path
// (one pn_classify per batch against a snapshot, host re-resolution after table
// changes) must produce the identical callback log: every record field, every
// onTcpData size and byte, every disconnect and ACK.  Independently, each flow's
// delivered bytes must equal the stream it sent.  Exit 0 = pass.
#include <arpa/inet.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <vector>

#include "../../include/pollnet_amd/gpu_tcp_rx.hpp"
#include "segframes.hpp"

using namespace segtest;
using namespace pollnet_amd;

struct Conf {
  static const uint32_t MaxConnCnt = 256;
  static const uint32_t MaxTimeWaitConnCnt = 64;
  static const uint32_t ConnRecvBufSize = 40960;
  static const bool TimestampOption = false;
};

struct Ev {
  uint8_t type; // 1 data, 2 disconnect, 3 ack owed, 4 new segment, 5 time-wait segment
  uint64_t key;
  uint32_t a, b;
  uint64_t h;
  bool operator==(const Ev& o) const { return type == o.type && key == o.key && a == o.a && b == o.b && h == o.h; }
};
static uint64_t fnv(const uint8_t* p, uint32_t n, uint64_t h = 1469598103934665603ull) {
  for (uint32_t i = 0; i < n; i++) h = (h ^ p[i]) * 1099511628211ull;
  return h;
}
static uint64_t rec_hash(const pn_result& r) { return fnv((const uint8_t*)&r, sizeof r); }

struct Flow {
  uint32_t ip;
  uint16_t port;
  uint32_t isn;
  uint32_t msg_len;
  std::vector<uint8_t> stream, got, tail; // tail: what the last onTcpData call left unconsumed
};

// The handler both paths drive; `Srv` is GpuTcpRx<Conf> or the twin.
template <class Srv>
struct Handler {
  Srv* srv;
  std::map<uint64_t, Flow*>* flows;
  std::vector<Ev> log;
  template <class C>
  uint32_t onTcpData(C& c, const uint8_t* d, uint32_t n) {
    Flow* f = (*flows)[c.key];
    const uint32_t keep = f->msg_len ? n % f->msg_len : 0;
    f->got.insert(f->got.end(), d, d + n - keep);
    f->tail.assign(d + n - keep, d + n);
    log.push_back({1, c.key, c.id, n, fnv(d, n)});
    return keep;
  }
  template <class C>
  void onTcpDisconnect(C& c) {
    // remote close: the reference wrapper presents the last bytes once more via onFin
    // and ignores what is left (EfviTcp.h:283-288); keep them as the stream's end
    Flow* f = (*flows)[c.key];
    f->got.insert(f->got.end(), f->tail.begin(), f->tail.end());
    f->tail.clear();
    log.push_back({2, c.key, c.id, 0, fnv((const uint8_t*)c.err, (uint32_t)std::strlen(c.err))});
  }
  template <class C>
  void onAckOwed(C& c, const RxAck& a) {
    log.push_back({3, c.key, c.ackSeq(), (uint32_t)(a.send | a.immediate << 1 | a.rst << 2), 0});
    if (a.immediate) c.ackSent();
  }
  void onNewSegment(uint64_t key, const uint8_t*, const pn_result& r) {
    log.push_back({4, key, r.conn_id, r.flags, rec_hash(r)});
    if ((r.flags & PN_F_SYN) && !(r.flags & PN_F_ACK)) srv->accept(key, r.seq - 1); // rec.seq = seq + syn
  }
  void onTimeWaitSegment(uint64_t key, uint32_t tw_id, const uint8_t*, const pn_result& r) {
    log.push_back({5, key, tw_id, r.flags, rec_hash(r)});
    if (r.flags & PN_F_RST) srv->removeTW(tw_id); // in-sequence RST ends TIME_WAIT (Core.h:513-517)
  }
};

// Sequential twin with reference semantics (same conn-id allocation and table ops as GpuTcpRx).
struct Twin {
  struct Conn : RxConn<Conf> {
    uint64_t key = 0;
    uint32_t id = 0;
    const char* err = nullptr;
    bool live = false;
    bool isClosed() const { return err != nullptr; }
  };
  ConnTable table;
  std::vector<Conn> conns = std::vector<Conn>(Conf::MaxConnCnt);
  std::vector<uint32_t> free_;
  bool drop_bad = true;
  Twin() {
    table.init(Conf::MaxConnCnt, Conf::MaxTimeWaitConnCnt);
    for (uint32_t i = Conf::MaxConnCnt; i-- > 0;) free_.push_back(i);
  }
  Conn* accept(uint64_t key, uint32_t syn_seq) {
    if (free_.empty()) return nullptr;
    const uint32_t id = free_.back();
    if (table.add(key, id) != PN_OK) return nullptr;
    free_.pop_back();
    Conn& c = conns[id];
    c.open(syn_seq);
    c.key = key;
    c.id = id;
    c.err = nullptr;
    c.live = true;
    return &c;
  }
  void remove(Conn& c) {
    if (c.live && table.del(c.key) == PN_OK) {
      c.live = false;
      free_.push_back(c.id);
    }
  }
  std::vector<uint32_t> free_tw = [] {
    std::vector<uint32_t> v;
    for (uint32_t i = Conf::MaxTimeWaitConnCnt; i-- > 0;) v.push_back(i);
    return v;
  }();
  std::vector<uint64_t> tw_keys = std::vector<uint64_t>(Conf::MaxTimeWaitConnCnt, PN_EMPTY_KEY);
  int removeTW(uint32_t tw_id) {
    if (table.del(tw_keys[tw_id]) != PN_OK) return PN_ENOENT;
    tw_keys[tw_id] = PN_EMPTY_KEY;
    free_tw.push_back(tw_id);
    return PN_OK;
  }
  int enterTW(Conn& c) {
    const uint32_t tw_id = free_tw.back();
    const int rc = table.enterTW(c.key, tw_id);
    if (rc == PN_OK) {
      free_tw.pop_back();
      tw_keys[tw_id] = c.key;
      c.live = false;
      free_.push_back(c.id);
      return (int)tw_id;
    }
    return rc;
  }
  template <class H>
  void poll(H& h, const uint8_t* slots, uint32_t n, uint32_t stride, uint32_t off) {
    for (uint32_t i = 0; i < n; i++) {
      const uint8_t* eth = slots + (size_t)i * stride + off;
      uint32_t ne = 0;
      uint64_t mask = 0;
      const pn_conn_entry* e = table.entries(&ne, &mask);
      pn_result r;
      orc_classify_frame(eth, stride - off, e, ne, mask, Conf::MaxConnCnt, &r);
      if (drop_bad && (r.flags & (PN_F_IP_OK | PN_F_TCP_OK)) != (PN_F_IP_OK | PN_F_TCP_OK)) continue;
      uint32_t ip_be;
      uint16_t port_be;
      std::memcpy(&ip_be, eth + 26, 4);
      std::memcpy(&port_be, eth + 34, 2);
      const uint64_t key = pn_conn_hash_key(ip_be, port_be);
      if (r.flags & PN_F_TW) {
        h.onTimeWaitSegment(key, r.conn_id - Conf::MaxConnCnt, eth, r);
      } else if (!(r.flags & PN_F_HIT)) {
        h.onNewSegment(key, eth, r);
      } else {
        Conn& c = conns[r.conn_id];
        struct A {
          H& h;
          Conn& c;
          uint32_t onData(RxConn<Conf>&, const uint8_t* d, uint32_t s) { return h.onTcpData(c, d, s); }
          void onFin(RxConn<Conf>&, const uint8_t* d, uint32_t s) {
            if (s) h.onTcpData(c, d, s);
            c.err = "remote close";
            h.onTcpDisconnect(c);
          }
          void onReset(RxConn<Conf>&) {
            c.err = "connection reset";
            h.onTcpDisconnect(c);
          }
        } a{h, c};
        const RxAck ack = c.onSegment(a, eth, r);
        if (ack.send || ack.rst) h.onAckOwed(c, ack);
        if (c.err) remove(c);
      }
    }
  }
};

int main(int argc, char** argv) {
  // argv: batch [twin | copy | zc] [span]: `span` polls the whole ring in one call
  // (chunks of `batch` pipelined inside GpuRx) instead of one poll per batch
  const uint32_t n_flows = 200, n_tw = 8, batch = argc > 1 ? (uint32_t)std::atoi(argv[1]) : 1000;
  const bool indexed = argc > 2 && std::strcmp(argv[2], "idx") == 0; // pollIndexed over event offsets
  const bool zero_copy = indexed || (argc > 2 && std::strcmp(argv[2], "zc") == 0);
  const bool span = argc > 3 && std::strcmp(argv[3], "span") == 0;
  const uint32_t stride = 2048, off = 2;
  std::mt19937_64 rng(0x7C9E5EEDull);
  auto U = [&](uint32_t lo, uint32_t hi) { return lo + (uint32_t)(rng() % (hi - lo + 1)); };

  // ---- build the traffic ----
  std::vector<Flow> flows(n_flows + n_tw + 16);
  std::vector<std::vector<Seg>> per(flows.size());
  for (uint32_t f = 0; f < flows.size(); f++) {
    Flow& F = flows[f];
    F.ip = 0x0a010000 | f;
    F.port = (uint16_t)(32768 + (f * 7919) % 28000);
    F.isn = (uint32_t)rng();
    F.msg_len = (f % 3 == 0) ? 100 : 0;
    if (f < n_flows) {
      F.stream.resize(U(0, 30000));
      for (auto& b : F.stream) b = (uint8_t)rng();
      auto mk = [&](uint32_t a, uint32_t b, uint8_t fl) {
        Seg s;
        s.src_ip = F.ip;
        s.src_port = F.port;
        s.seq = F.isn + 1 + a;
        s.flags = fl;
        s.payload = F.stream.data() + a;
        s.len = b - a;
        return s;
      };
      Seg syn;
      syn.src_ip = F.ip;
      syn.src_port = F.port;
      syn.seq = F.isn;
      syn.flags = SYN;
      per[f].push_back(syn);
      std::vector<std::pair<uint32_t, uint32_t>> pk;
      for (uint32_t o = 0; o < F.stream.size();) {
        const uint32_t n = std::min<uint32_t>((uint32_t)F.stream.size() - o, U(1, 1460));
        pk.push_back({o, o + n});
        o += n;
      }
      const uint32_t W = U(1, 3);
      for (size_t b = 0; b < pk.size(); b += W) {
        std::vector<std::pair<uint32_t, uint32_t>> blk(pk.begin() + b, pk.begin() + std::min(pk.size(), b + W));
        std::shuffle(blk.begin(), blk.end(), rng);
        for (auto& x : blk) {
          Seg s = mk(x.first, x.second, ACK | PSH);
          if (rng() % 16 == 0) { // corrupted copy first (dropped), the clean resend right after
            Seg bad = s;
            bad.corrupt = true;
            per[f].push_back(bad);
          }
          per[f].push_back(s);
          if (rng() % 20 == 0) per[f].push_back(s); // duplicate
        }
      }
      per[f].push_back(mk((uint32_t)F.stream.size(), (uint32_t)F.stream.size(), ACK | FIN));
      per[f].push_back(mk((uint32_t)F.stream.size() + 1, (uint32_t)F.stream.size() + 1, ACK)); // after close: unknown
    } else { // TIME_WAIT flows (n_tw) and unknown flows: a few ACK-only segments each; every
      // other TIME_WAIT flow ends it with an RST and reconnects with a SYN (delete-then-SYN)
      const bool reconnect = f < n_flows + n_tw && f % 2 == 0;
      for (int k = 0; k < 3; k++) {
        Seg s;
        s.src_ip = F.ip;
        s.src_port = F.port;
        s.seq = F.isn + k;
        s.flags = reconnect && k == 1 ? RST : reconnect && k == 2 ? SYN : ACK;
        per[f].push_back(s);
      }
    }
  }
  // interleave, keeping each flow's order
  std::vector<std::pair<uint32_t, uint32_t>> order; // (flow, index)
  {
    std::vector<uint32_t> pos(flows.size(), 0), live;
    for (uint32_t f = 0; f < flows.size(); f++) live.push_back(f);
    while (!live.empty()) {
      const uint32_t k = (uint32_t)(rng() % live.size()), f = live[k];
      order.push_back({f, pos[f]++});
      if (pos[f] == per[f].size()) {
        live[k] = live.back();
        live.pop_back();
      }
    }
  }
  const uint32_t n = (uint32_t)order.size();
  const bool twin_only = argc > 2 && std::strcmp(argv[2], "twin") == 0;
  uint8_t* ring = nullptr;
  std::vector<uint8_t> host_ring;
  if (twin_only) {
    host_ring.resize((size_t)stride * n);
    ring = host_ring.data();
  } else if (hipHostMalloc((void**)&ring, (size_t)stride * n, hipHostMallocDefault) != hipSuccess) {
    return 2;
  }
  std::memset(ring, 0, (size_t)stride * n);
  for (uint32_t i = 0; i < n; i++) build(ring + (size_t)i * stride + off, per[order[i].first][order[i].second]);

  auto run = [&](auto& srv, auto&& poll_fn, std::vector<Ev>& log_out, std::vector<std::vector<uint8_t>>& got) {
    std::map<uint64_t, Flow*> byk;
    for (auto& F : flows) {
      F.got.clear();
      F.tail.clear();
      uint32_t ip_be = htonl(F.ip);
      byk[pn_conn_hash_key(ip_be, htons(F.port))] = &F;
    }
    using S = std::remove_reference_t<decltype(srv)>;
    Handler<S> h{&srv, &byk, {}};
    for (uint32_t t = 0; t < n_tw; t++) { // pre-existing TIME_WAIT entries
      const Flow& F = flows[n_flows + t];
      auto* c = srv.accept(pn_conn_hash_key(htonl(F.ip), htons(F.port)), F.isn);
      if (!c || srv.enterTW(*c) != (int)t) return false;
    }
    const uint32_t step = span ? n : batch;
    for (uint32_t b = 0; b < n; b += step) {
      if (!poll_fn(h, ring + (size_t)b * stride, std::min(step, n - b))) return false;
    }
    log_out = std::move(h.log);
    got.clear();
    for (auto& F : flows) got.push_back(F.got);
    return true;
  };

  Twin twin;
  std::vector<Ev> tlog, glog;
  std::vector<std::vector<uint8_t>> tgot, ggot;
  if (!run(twin, [&](auto& h, const uint8_t* s, uint32_t m) { twin.poll(h, s, m, stride, off); return true; }, tlog, tgot))
    return 3;

  if (twin_only) { // CPU-only: the twin alone must deliver every stream
    uint32_t ok = 0;
    for (uint32_t f = 0; f < n_flows; f++) ok += tgot[f] == flows[f].stream;
    size_t disc = 0;
    for (auto& e : tlog) disc += e.type == 2;
    std::printf("twin: frames %u, %zu events, %u/%u streams intact, %zu disconnects\n", n, tlog.size(), ok, n_flows,
                disc);
    return (ok == n_flows && disc == n_flows) ? 0 : 1;
  }

  auto gpu = std::make_unique<GpuTcpRx<Conf>>();
  if (const char* e = gpu->init(0, stride, off, batch, zero_copy ? GpuRx::Mode::ZeroCopy : GpuRx::Mode::Copy)) {
    std::printf("init: %s\n", e);
    return 4;
  }
  gpu->setDropBadChecksum(true);
  std::vector<uint64_t> offs(n);
  for (uint32_t i = 0; i < n; i++) offs[i] = (uint64_t)i * stride + off;
  if (!run(*gpu,
           [&](auto& h, const uint8_t* s, uint32_t m) {
             const char* e = indexed ? gpu->pollIndexed(h, ring, offs.data() + (s - ring) / stride, m, off % 16, stride - off)
                                     : gpu->poll(h, s, m);
             if (e) std::printf("poll: %s\n", e);
             return e == nullptr;
           },
           glog, ggot))
    return 5;

  int fail = 0;
  size_t first_diff = std::mismatch(tlog.begin(), tlog.end(), glog.begin(), glog.end()).first - tlog.begin();
  if (tlog.size() != glog.size() || first_diff != tlog.size()) {
    std::printf("FAIL: callback logs differ: twin %zu events, gpu %zu, first difference at %zu\n", tlog.size(),
                glog.size(), first_diff);
    fail++;
  }
  uint32_t streams_ok = 0, bytes = 0;
  for (uint32_t f = 0; f < n_flows; f++) {
    if (ggot[f] == flows[f].stream) streams_ok++;
    bytes += (uint32_t)flows[f].stream.size();
  }
  if (streams_ok != n_flows) {
    std::printf("FAIL: %u/%u flows delivered their stream\n", streams_ok, n_flows);
    fail++;
  }
  uint32_t n_reconnect = 0; // TIME_WAIT flows with an even flow index: RST then SYN
  for (uint32_t f = n_flows; f < n_flows + n_tw; f++) n_reconnect += f % 2 == 0;
  size_t cnt[6] = {};
  for (auto& e : glog) cnt[e.type]++;
  std::printf("%s%s: ", indexed ? "indexed zero-copy" : zero_copy ? "zero-copy" : "copy",
              span ? ", one poll over the ring" : "");
  std::printf("frames %u in batches of %u: %zu events (data %zu, disconnect %zu, ack %zu, new %zu, tw %zu); "
              "%u/%u streams (%u B) intact; conns left %u\n",
              n, batch, glog.size(), cnt[1], cnt[2], cnt[3], cnt[4], cnt[5], streams_ok, n_flows, bytes,
              gpu->getConnCnt());
  std::printf("TIME_WAIT: %u ended by RST and reconnected by SYN, %u left\n", n_reconnect, gpu->getTimeWaitCnt());
  if (gpu->getConnCnt() != n_reconnect || gpu->getTimeWaitCnt() != n_tw - n_reconnect) {
    std::printf("FAIL: expected %u reconnected flows open and %u TIME_WAIT entries, have %u / %u\n", n_reconnect,
                n_tw - n_reconnect, gpu->getConnCnt(), gpu->getTimeWaitCnt());
    fail++;
  }
  if (cnt[2] != n_flows || cnt[5] != 3 * n_tw - n_reconnect) {
    std::printf("FAIL: expected %u disconnects and %u time-wait segments\n", n_flows, 3 * n_tw - n_reconnect);
    fail++;
  }
  std::printf("%s\n", fail ? "FAIL" : "PASS");
  return fail ? 1 : 0;
}
