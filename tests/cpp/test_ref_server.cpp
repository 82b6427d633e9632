// GpuTcpServer against the reference's OWN efvitcp server (F1 parity: the stateful onPack
// remainder, onTcpData delivery, ACK / RST / FIN / TIME_WAIT policy, timers).
//
// The reference side is pollnet's EfviTcpServer over efvitcp::TcpServer / TcpConn, compiled from
// the text of /root/reference (oracle/ref_server.hpp; only the ef_vi plumbing is restated there).
// Both servers run the same handler over the same deterministic client population
// (peer_population.hpp: handshakes, echo traffic, loss both ways, retransmissions, delayed ACKs,
// window-limited sends, receive timeouts, server FINs, peer FINs and RSTs, admission refusal at
// MaxConns) and a clock of one millisecond per poll.  The clients being deterministic functions
// of what they receive, any difference in behaviour shows up as a different frame sequence: the
// test requires every frame the server sends (byte for byte, checksums included) and the
// handler's log to be identical, and reports the first difference otherwise.
//   argv: twin | gpu  [populations]        exit 0 = pass
// twin: the product engine with the sequential oracle backend (CPU); gpu: with GpuBackend
// (pn_classify + pn_tx_fill on the device).
#include <arpa/inet.h>

#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../oracle/ref_server.hpp"
#include "peer_population.hpp"
#include "server_harness.hpp"

using pollnet_amd::GpuBackend;
using pollnet_amd::GpuTcpServer;

// pollnet's EfviTcpServer Conf (its ServerConf fixes the rest, EfviTcp.h:191-212)
struct RefConf {
  static const uint32_t RecvBufSize = 8192;
  static const uint32_t MaxConns = 48;
  static const uint32_t SendTimeoutSec = 0;
  static const uint32_t RecvTimeoutSec = 1;
  struct UserData {
    uint32_t echoed = 0;
    bool fin_asked = false;
  };
};
// the product with the same Conf; RxBatch 64 = the reference's 64 events per pollNet (Core.h:498)
struct ProdConf : RefConf {
  static const uint32_t RxBatch = 64;
};
// the same with the classify in the resident service (a post per poll, no launch)
struct ProdConfResident : ProdConf {
  static const bool RxResident = true;
};
// ... with the chain links of each post and the in-order fast path they drive (Conf::RxLinks)
struct ProdConfLinked : ProdConfResident {
  static const bool RxLinks = true;
};

static const uint32_t kMaxPolls = 30000;

static bool done(PeerLink& l) {
  for (auto& c : l.clients)
    if (c.st != Client::kDone) return false;
  return true;
}

struct Transcript {
  std::vector<std::vector<uint8_t>> out;
  std::string log;
  uint32_t polls = 0;
  std::vector<Client> clients;
  uint64_t in_order = 0; // frames the product took through the in-order fast path (chain links)
};

static Transcript runRef(const std::vector<Client>& pop) {
  using Srv = efvitcp::EfviTcpServer<RefConf>;
  auto link = std::make_unique<PeerLink>();
  link->defer = true;
  link->clients = pop;
  efvitcp::RefEnv& env = efvitcp::refEnv();
  env.link = link.get();
  env.fill = [](void* l, uint8_t* slots, uint32_t stride, uint32_t off, uint32_t cap) {
    return static_cast<PeerLink*>(l)->fill(slots, stride, off, cap);
  };
  env.send = [](void* l, const uint8_t* eth, uint32_t len) { static_cast<PeerLink*>(l)->send(eth, len); };
  env.init_ns = kT0;
  env.local_ip = link->localIp();
  std::memcpy(env.local_mac, link->localMac(), 6);
  std::unique_ptr<Srv> srv(new Srv()); // ~50 MiB of send buffers
  Transcript t;
  if (!srv->init("peer", "10.0.0.1", 1234)) {
    std::printf("ref init: %s\n", srv->getLastError());
    return t;
  }
  PeerHandler<Srv::Conn> h{&t.log};
  for (t.polls = 1; t.polls < kMaxPolls; t.polls++) {
    srv->poll(h, kT0 + ((int64_t)t.polls << 20));
    link->endPoll();
    if (done(*link) && srv->getConnCnt() == 0) break;
  }
  t.out = link->out;
  t.clients = link->clients;
  return t;
}

template <class Backend, class Conf = ProdConf>
static Transcript runProd(const std::vector<Client>& pop, bool drop_bad = true) {
  using Srv = GpuTcpServer<Conf, PeerLink, Backend>;
  auto srv = std::make_unique<Srv>();
  Transcript t;
  if (!srv->initWithLink("10.0.0.1", 1234, kT0)) {
    std::printf("init: %s\n", srv->getLastError());
    return t;
  }
  srv->link().defer = true;
  srv->link().clients = pop;
  srv->setDropBadChecksum(drop_bad); // off: the GPU backend classifies from the header lines only (pn_set_verify)
  PeerHandler<typename Srv::Conn> h{&t.log};
  for (t.polls = 1; t.polls < kMaxPolls; t.polls++) {
    srv->poll(h, kT0 + ((int64_t)t.polls << 20));
    srv->link().endPoll();
    if (srv->getLastError()) {
      std::printf("poll: %s\n", srv->getLastError());
      return t;
    }
    if (done(srv->link()) && srv->getConnCnt() == 0) break;
  }
  t.out = srv->link().out;
  t.clients = srv->link().clients;
  t.in_order = srv->inOrderFrames();
  return t;
}

static void dumpFrame(const char* tag, const std::vector<uint8_t>& f) {
  const uint8_t* tcp = f.data() + 34;
  std::printf("  %s: %zu B, port %u, seq %u ack %u flags 0x%02x win %u\n", tag, f.size(),
              (unsigned)(tcp[2] << 8 | tcp[3]), rd32(tcp + 4), rd32(tcp + 8), tcp[13], (unsigned)(tcp[14] << 8 | tcp[15]));
}

static int compare(const char* what, const Transcript& ref, const Transcript& p) {
  size_t same = 0;
  while (same < ref.out.size() && same < p.out.size() && ref.out[same] == p.out[same]) same++;
  const bool frames_eq = same == ref.out.size() && same == p.out.size();
  const bool log_eq = ref.log == p.log;
  std::printf("%s: %zu frames (reference %zu) %s, handler log %s (%zu B)", what, p.out.size(), ref.out.size(),
              frames_eq ? "identical" : "DIFFERENT", log_eq ? "identical" : "DIFFERENT", ref.log.size());
  if (p.in_order) std::printf(", %llu through the in-order fast path", (unsigned long long)p.in_order);
  std::printf("\n");
  if (!frames_eq) {
    std::printf("  first difference at frame %zu\n", same);
    if (same < ref.out.size()) dumpFrame("reference", ref.out[same]);
    if (same < p.out.size()) dumpFrame("product  ", p.out[same]);
  }
  if (!log_eq) {
    size_t d = 0;
    while (d < ref.log.size() && d < p.log.size() && ref.log[d] == p.log[d]) d++;
    const size_t b = ref.log.rfind('\n', d ? d - 1 : 0);
    const size_t s = b == std::string::npos ? 0 : b + 1;
    std::printf("  log differs at byte %zu:\n  reference: %.120s\n  product:   %.120s\n", d, ref.log.c_str() + s,
                p.log.c_str() + std::min(s, p.log.size()));
  }
  return frames_eq && log_eq ? 0 : 1;
}

// What the run exercised (so a pass is not vacuous).
static int coverage(const Transcript& t) {
  uint32_t synacks = 0, fins = 0, rsts = 0, data = 0, est = 0, refused = 0;
  for (auto& f : t.out) {
    const uint8_t fl = f[47];
    synacks += (fl & 0x12) == 0x12;
    fins += fl & 1;
    rsts += (fl & 4) != 0;
    data += f.size() > 54 + ((fl & 2) ? 4 : 0);
  }
  for (auto& c : t.clients) est += c.established, refused += c.refused;
  auto count = [&](const char* w) {
    size_t n = 0, p = 0;
    while ((p = t.log.find(w, p)) != std::string::npos) n++, p++;
    return n;
  };
  std::printf("  exercised: %u SYN-ACKs, %u data frames, %u FINs, %u RSTs; %u established, %u refused; "
              "log: %zu connected, %zu disconnect, %zu recv timeout, %zu sendFin; %u polls\n",
              synacks, data, fins, rsts, est, refused, count("connected"), count("disconnect"), count("recv timeout"),
              count("sendFin"), t.polls);
  auto disc = [&](const char* err) { // disconnect lines with that error
    size_t n = 0, p = 0;
    const std::string w = std::string("err=") + err + " ";
    while ((p = t.log.find("disconnect ", p)) != std::string::npos) {
      const size_t e = t.log.find('\n', p);
      if (t.log.compare(t.log.find("err=", p), w.size(), w) == 0) n++;
      p = e;
    }
    return n;
  };
  std::printf("  disconnects by cause: %zu connection reset, %zu remote close, %zu timeout, %zu connection closed, "
              "%zu send buffer full\n",
              disc("connection reset"), disc("remote close"), disc("timeout"), disc("connection closed"),
              disc("send buffer full"));
  // send-side samples (getSendable / getImmediatelySendable, logged by the handler): how many, and how many
  // limited by the peer's window rather than by free send buffers
  uint32_t samples = 0, wnd_limited = 0, zero_now = 0;
  for (size_t p = 0; (p = t.log.find("data ", p)) != std::string::npos; p++) {
    unsigned sendable = 0, now = 0;
    if (std::sscanf(t.log.c_str() + t.log.find("sendable=", p), "sendable=%u now=%u", &sendable, &now) != 2) continue;
    samples++;
    wnd_limited += now < sendable;
    zero_now += now == 0;
  }
  std::printf("  send side: %u getSendable/getImmediatelySendable samples, %u window-limited (%u zero)\n", samples,
              wnd_limited, zero_now);
  return (synacks && data && fins && rsts && est && count("recv timeout") && count("sendFin") &&
          disc("connection reset") && disc("remote close") && samples && wnd_limited)
             ? 0
             : 1;
}

// The one intended difference, shown: efvitcp answers unknown flows and TIME_WAIT segments from ONE
// shared send buffer and skips the answer while that buffer's previous frame is still in the NIC's
// TX queue (Core.h:404, 427); ACKs and close()'s RST likewise need a completed buffer from getAckBuf
// (TcpConn.h:851-860).  The engine sends every frame at flush and never holds one back.  With TX
// completions arriving one poll late, three unknown-flow segments in one poll get one RST from the
// reference and three from the product; with immediate completions both send three.
struct BurstLink {
  std::vector<std::vector<uint8_t>> in, out;
  const char* open(const char*) { return nullptr; }
  uint32_t fill(uint8_t* slots, uint32_t stride, uint32_t off, uint32_t cap) {
    uint32_t n = 0;
    for (; n < cap && n < in.size(); n++) {
      std::memset(slots + (size_t)n * stride, 0, stride);
      std::memcpy(slots + (size_t)n * stride + off, in[n].data(), in[n].size());
    }
    in.erase(in.begin(), in.begin() + n);
    return n;
  }
  void send(const uint8_t* eth, uint32_t len) { out.emplace_back(eth, eth + len); }
  uint32_t localIp() const { return htonl(0x0a000001); }
  const uint8_t* localMac() const {
    static const uint8_t m[6] = {2, 0, 0, 0, 0, 1};
    return m;
  }
};
static std::vector<std::vector<uint8_t>> burst(uint32_t n = 3, bool corrupt = false) {
  std::vector<std::vector<uint8_t>> f;
  for (uint32_t k = 0; k < n; k++) {
    segtest::Seg s;
    s.src_ip = 0x0a050000 + k;
    s.src_port = (uint16_t)(50000 + k);
    s.seq = 1000 * k;
    s.ack = 77 + k;
    s.flags = segtest::ACK;
    s.corrupt = corrupt;
    std::vector<uint8_t> b(128);
    b.resize(segtest::build(b.data(), s));
    f.push_back(b);
  }
  return f;
}
static int nic_queue_divergence() {
  int fail = 0;
  for (int late = 0; late < 2; late++) {
    using Srv = efvitcp::EfviTcpServer<RefConf>;
    BurstLink link;
    link.in = burst();
    efvitcp::RefEnv& env = efvitcp::refEnv();
    env.link = &link;
    env.fill = [](void* l, uint8_t* s, uint32_t st, uint32_t off, uint32_t cap) {
      return static_cast<BurstLink*>(l)->fill(s, st, off, cap);
    };
    env.send = [](void* l, const uint8_t* eth, uint32_t len) { static_cast<BurstLink*>(l)->send(eth, len); };
    env.init_ns = kT0;
    env.local_ip = link.localIp();
    std::memcpy(env.local_mac, link.localMac(), 6);
    env.tx_complete_next_poll = late;
    std::unique_ptr<Srv> ref(new Srv());
    ref->init("burst", "10.0.0.1", 1234);
    std::string log;
    PeerHandler<Srv::Conn> h{&log};
    ref->poll(h, kT0 + (1 << 20));
    env.tx_complete_next_poll = false;
    using P = GpuTcpServer<ProdConf, BurstLink, OracleBackend>;
    auto p = std::make_unique<P>();
    p->initWithLink("10.0.0.1", 1234, kT0);
    p->link().in = burst();
    PeerHandler<P::Conn> ph{&log};
    p->poll(ph, kT0 + (1 << 20));
    const size_t want_ref = late ? 1 : 3;
    const bool ok = link.out.size() == want_ref && p->link().out.size() == 3 &&
                    std::equal(link.out.begin(), link.out.end(), p->link().out.begin());
    std::printf("NIC-queue divergence, TX completions %s: reference %zu RSTs, product %zu RSTs%s -> %s\n",
                late ? "one poll late" : "immediate", link.out.size(), p->link().out.size(),
                late ? " (the reference's are the product's first)" : " (identical)", ok ? "as documented" : "UNEXPECTED");
    fail += !ok;
  }
  return fail;
}

// The reference server as the harness runs it, on one burst of frames; returns its frames after each poll.
static std::vector<size_t> ref_polls(std::vector<std::vector<uint8_t>> frames, int polls, BurstLink& link) {
  using Srv = efvitcp::EfviTcpServer<RefConf>;
  link.in = std::move(frames);
  efvitcp::RefEnv& env = efvitcp::refEnv();
  env.link = &link;
  env.fill = [](void* l, uint8_t* s, uint32_t st, uint32_t off, uint32_t cap) {
    return static_cast<BurstLink*>(l)->fill(s, st, off, cap);
  };
  env.send = [](void* l, const uint8_t* eth, uint32_t len) { static_cast<BurstLink*>(l)->send(eth, len); };
  env.init_ns = kT0;
  env.local_ip = link.localIp();
  std::memcpy(env.local_mac, link.localMac(), 6);
  env.tx_complete_next_poll = false;
  std::unique_ptr<Srv> ref(new Srv());
  ref->init("burst", "10.0.0.1", 1234);
  std::string log;
  PeerHandler<Srv::Conn> h{&log};
  std::vector<size_t> out;
  for (int k = 1; k <= polls; k++) {
    ref->poll(h, kT0 + ((int64_t)k << 20));
    out.push_back(link.out.size());
  }
  return out;
}
template <class Conf, class Backend = OracleBackend>
static std::vector<size_t> prod_polls(std::vector<std::vector<uint8_t>> frames, int polls, bool drop_bad,
                                      std::vector<std::vector<uint8_t>>* sent) {
  using P = GpuTcpServer<Conf, BurstLink, Backend>;
  auto p = std::make_unique<P>();
  p->initWithLink("10.0.0.1", 1234, kT0);
  p->setDropBadChecksum(drop_bad);
  p->link().in = std::move(frames);
  std::string log;
  PeerHandler<typename P::Conn> h{&log};
  std::vector<size_t> out;
  for (int k = 1; k <= polls; k++) {
    p->poll(h, kT0 + ((int64_t)k << 20));
    out.push_back(p->link().out.size());
  }
  *sent = p->link().out;
  return out;
}

// Frames per poll: the reference takes at most 64 RX events per pollNet (Core.h:496-498), the engine up to
// Conf::RxBatch (default 512).  100 unknown-flow segments in one burst: the reference answers 64 in the
// first poll and 36 in the second, the engine all 100 in the first (and with RxBatch = 64, as the reference);
// the 100 RSTs are the same frames in the same order.
static int rx_batch_divergence() {
  BurstLink link;
  const auto ref = ref_polls(burst(100), 2, link);
  std::vector<std::vector<uint8_t>> a, b;
  const auto def = prod_polls<RefConf>(burst(100), 2, true, &a);
  const auto b64 = prod_polls<ProdConf>(burst(100), 2, true, &b);
  const bool ok = ref == std::vector<size_t>{64, 100} && def == std::vector<size_t>{100, 100} && b64 == ref &&
                  a == link.out && b == link.out;
  std::printf("frames per poll: reference %zu then %zu RSTs, product (RxBatch 512) %zu then %zu, product (RxBatch 64) "
              "%zu then %zu; the same 100 frames -> %s\n",
              ref[0], ref[1], def[0], def[1], b64[0], b64[1], ok ? "as documented" : "UNEXPECTED");
  return ok ? 0 : 1;
}

// Bad checksums: the reference relies on the NIC to discard them (an ef_vi RX_DISCARD event); run without a
// NIC it answers a corrupted unknown-flow segment with an RST.  The engine discards it after pn_classify
// (setDropBadChecksum, default on); with the discard off it sends the reference's RST, byte for byte.
// On the GPU backend the discard off also switches the kernel to the header lines only (pn_set_verify(ctx, 0)).
template <class Backend = OracleBackend>
static int bad_checksum_divergence(const char* backend = "") {
  BurstLink link;
  const auto ref = ref_polls(burst(3, true), 1, link);
  std::vector<std::vector<uint8_t>> dropped, kept;
  const auto on = prod_polls<ProdConf, Backend>(burst(3, true), 1, true, &dropped);
  const auto off = prod_polls<ProdConf, Backend>(burst(3, true), 1, false, &kept);
  const bool ok = ref[0] == 3 && on[0] == 0 && off[0] == 3 && kept == link.out;
  std::printf("bad checksums%s: reference without a NIC %zu RSTs, product %zu (discard on) / %zu (discard off, the "
              "reference's frames) -> %s\n",
              backend, ref[0], on[0], off[0], ok ? "as documented" : "UNEXPECTED");
  return ok ? 0 : 1;
}

int main(int argc, char** argv) {
  const bool gpu = argc > 1 && std::strcmp(argv[1], "gpu") == 0;
  const uint32_t runs = argc > 2 ? (uint32_t)std::atoi(argv[2]) : 1;
  int fail = nic_queue_divergence() + rx_batch_divergence() + bad_checksum_divergence();
  if (gpu) fail += bad_checksum_divergence<GpuBackend>(" (GPU backend)");
  uint64_t in_order_total = 0;
  for (g_seed = 0; g_seed < runs; g_seed++) {
    for (int chaos = 0; chaos < 2; chaos++) {
      std::printf("== %s population %u ==\n", chaos ? "chaos" : "peer", g_seed);
      const auto pop = chaos ? chaos_population() : population();
      const Transcript ref = runRef(pop);
      if (ref.out.empty()) return 2;
      fail += coverage(ref);
      fail += compare("twin (sequential oracle backend) vs reference", ref, runProd<OracleBackend>(pop));
      // the twin with chain links (orc_chain_links, as the resident service's linked posts): the in-order fast path
      const Transcript tl = runProd<OracleBackend, ProdConfLinked>(pop);
      fail += compare("twin with chain links vs reference", ref, tl);
      in_order_total += tl.in_order;
      if (gpu) {
        fail += compare("GpuTcpServer (GPU backend) vs reference", ref, runProd<GpuBackend>(pop));
        fail += compare("GpuTcpServer (GPU backend, release path: no checksum verification) vs reference", ref,
                        runProd<GpuBackend>(pop, false));
        fail += compare("GpuTcpServer (GPU backend, resident service) vs reference", ref,
                        runProd<GpuBackend, ProdConfResident>(pop));
        fail += compare("GpuTcpServer (GPU backend, resident service, release path) vs reference", ref,
                        runProd<GpuBackend, ProdConfResident>(pop, false));
        fail += compare("GpuTcpServer (GPU backend, resident service, chain links) vs reference", ref,
                        runProd<GpuBackend, ProdConfLinked>(pop));
        fail += compare("GpuTcpServer (GPU backend, resident service, chain links, release path) vs reference", ref,
                        runProd<GpuBackend, ProdConfLinked>(pop, false));
      }
    }
  }
  if (!in_order_total) fail++, std::printf("FAIL: no frame took the in-order fast path\n");
  std::printf("%s\n", fail ? "FAIL" : "PASS");
  return fail ? 1 : 0;
}
