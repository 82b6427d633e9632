// GpuTcpServer against live TCP peers: a deterministic in-memory client population that
// reacts to every frame the server sends, with loss in both directions and a clock that
// advances one millisecond per poll.  This drives the parts of the server a replayed
// ring cannot: SYN-ACK retransmission, RTO retransmission and its back-off, duplicate-ACK
// fast retransmit, delayed ACKs, window-limited sending (segments queued until the peer's
// ACK opens the window, TcpConn.h:646-660), the receive timeout (onRecvTimeout ->
// close("timeout") -> RST), admission refusal (allowNewConnection / MaxConns -> RST),
// the server's own FIN (Conn::sendFin), RSTs from the peer and the pollnet wrapper's
// close on a remote FIN (EfviTcp.h:283-288).
//
// The same population runs twice — GpuBackend (pn_classify + pn_tx_fill on the GPU) and
// the sequential oracle backend — and, the peers being deterministic functions of what
// they receive, the two runs must match frame for frame and callback for callback.
// Independently: every flow that completes echoes its stream exactly, every TX frame
// verifies, idle flows are timed out, and nothing is left open.
//   argv: twin | gpu            exit 0 = pass
#include <arpa/inet.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <random>
#include <string>
#include <tuple>
#include <vector>

#include "segframes.hpp"
#include "server_harness.hpp"

using namespace pollnet_amd;

struct PeerConf {
  static const bool RxPipeline = false;
  static const uint32_t RecvBufSize = 8192;
  static const uint32_t MaxConns = 48;
  static const uint32_t SendTimeoutSec = 0;
  static const uint32_t RecvTimeoutSec = 1;
  static const uint32_t ConnSendBufCnt = 64;
  static const uint32_t RxBatch = 1024;
  static const uint32_t TxBatch = 128;
  static const uint32_t DelayedAckMS = 10;
  static const bool UseAllowNewConnection = true; // efvitcp::TcpServer's admission event (TcpServer.h:84)
  struct UserData {
    uint32_t echoed = 0;
    bool fin_asked = false;
  };
};

// the same with received frames held up to 3 ms for a fuller GPU batch
struct PeerConfBudget : PeerConf {
  static const uint32_t RxLatencyBudgetUs = 3000;
};
// a poll's frames classified in launches of 16 (the next on the GPU while one is dispatched)
struct PeerConfChunk : PeerConf {
  static const uint32_t RxChunk = 16;
};
// throughput mode: each poll's frames dispatched in the next poll, classified meanwhile
// against the table as it was at their launch (re-resolved where it has changed since)
struct PeerConfPipe : PeerConf {
  static const bool RxPipeline = true;
};

static const int64_t kT0 = (int64_t)777777 << 20;

enum Kind : uint8_t { kFinEnd, kRstEnd, kIdle, kServerFin };

struct Client {
  uint32_t ip;
  uint16_t port;
  Kind kind;
  uint32_t start, window;
  std::vector<uint8_t> stream;
  std::mt19937 rng;
  // state
  enum { kWait, kSynSent, kEst, kDone } st = kWait;
  uint32_t isn = 0, srv_isn = 0;
  uint32_t snd_una = 0, snd_nxt = 0, srv_wnd = 0, last_tx = 0, last_progress = 0;
  bool fin_sent = false, got_rst = false, got_fin = false, refused = false, established = false;
  std::vector<uint8_t> echo;
  std::map<uint32_t, std::vector<uint8_t>> ooo;
};

// Population and loss seeds: run k of a soak (argv[2] runs) perturbs both; 0 = the original.
static uint32_t g_seed = 0;

// The client population as a link: fill() = frames the clients send this tick,
// send() = a frame from the server, handed to its client.
struct PeerLink {
  std::vector<Client> clients;
  std::vector<std::vector<uint8_t>> q;   // client -> server, this tick
  std::vector<std::vector<uint8_t>> out; // every server frame (the comparison)
  std::mt19937 loss{0xD20Bu ^ g_seed};
  uint32_t tick = 0;
  uint32_t drops_c2s = 0, drops_s2c = 0;

  const char* open(const char*) { return nullptr; }
  uint32_t localIp() const { return htonl(0x0a000001); }
  const uint8_t* localMac() const {
    static const uint8_t m[6] = {2, 0, 0, 0, 0, 1};
    return m;
  }

  void emit(Client& c, uint32_t seq, uint32_t ack, uint8_t flags, const uint8_t* p = nullptr, uint32_t len = 0,
            bool mss = false) {
    segtest::Seg s;
    s.src_ip = c.ip;
    s.src_port = c.port;
    s.seq = seq;
    s.ack = ack;
    s.flags = flags;
    s.payload = p;
    s.len = len;
    if (mss) s.opts = {2, 4, 0x05, 0xb4};
    uint8_t buf[2048];
    const uint32_t n = segtest::build(buf, s);
    segtest::put16(buf + 48, (uint16_t)c.window); // the client's receive window
    segtest::put16(buf + 50, 0);
    {
      uint8_t* tcp = buf + 34;
      const uint32_t tcp_len = n - 34;
      uint32_t ph = (c.ip >> 16) + (c.ip & 0xffff) + (0x0a000001 >> 16) + (0x0a000001 & 0xffff) + 6 + tcp_len;
      segtest::put16(tcp + 16, segtest::rfc_sum(tcp, tcp_len, ph));
    }
    q.emplace_back(buf, buf + n);
  }
  uint32_t ackNum(const Client& c) const { return c.srv_isn + 1 + (uint32_t)c.echo.size() + (c.got_fin ? 1 : 0); }

  void step(Client& c) {
    const uint32_t base = c.isn + 1;
    switch (c.st) {
      case Client::kWait:
        if (tick >= c.start) {
          c.st = Client::kSynSent;
          c.last_tx = tick;
          emit(c, c.isn, 0, segtest::SYN, nullptr, 0, true);
        }
        break;
      case Client::kSynSent:
        if (tick - c.last_tx >= 300) {
          c.last_tx = tick;
          emit(c, c.isn, 0, segtest::SYN, nullptr, 0, true);
        }
        break;
      case Client::kEst: {
        const uint32_t limit = c.kind == kIdle ? (uint32_t)c.stream.size() / 2 : (uint32_t)c.stream.size();
        if (c.snd_una < c.snd_nxt && tick - c.last_progress >= 150 && tick - c.last_tx >= 150) { // RTO: resend una
          const uint32_t n = std::min<uint32_t>(c.snd_nxt - c.snd_una, 1000);
          emit(c, base + c.snd_una, ackNum(c), segtest::ACK | segtest::PSH, c.stream.data() + c.snd_una, n);
          c.last_tx = tick;
        }
        for (int k = 0; k < 3 && c.snd_nxt < limit && !c.fin_sent; k++) {
          const uint32_t room = c.srv_wnd - std::min(c.srv_wnd, c.snd_nxt - c.snd_una); // what the window admits
          const uint32_t n = std::min<uint32_t>({limit - c.snd_nxt, 1 + (uint32_t)(c.rng() % 1460), room});
          if (n == 0) break;
          emit(c, base + c.snd_nxt, ackNum(c), segtest::ACK | segtest::PSH, c.stream.data() + c.snd_nxt, n);
          if (c.snd_una == c.snd_nxt) c.last_progress = tick;
          c.snd_nxt += n;
          c.last_tx = tick;
        }
        const bool all_acked = c.snd_una == limit && c.snd_nxt == limit;
        // the handler echoes whole 8-byte words on ports divisible by 5 (the rest comes with the FIN)
        const uint32_t echo_due = c.port % 5 == 0 ? limit & ~7u : limit;
        if (c.kind == kRstEnd && all_acked && c.echo.size() >= echo_due) {
          emit(c, base + c.snd_nxt, 0, segtest::RST);
          c.st = Client::kDone;
        } else if ((c.kind == kFinEnd && all_acked && c.echo.size() >= echo_due) || (c.got_fin && !c.fin_sent)) {
          if (!c.fin_sent || tick - c.last_tx >= 200) { // (re)send our FIN until the server's RST
            emit(c, base + c.snd_nxt, ackNum(c), segtest::ACK | segtest::FIN);
            c.fin_sent = true;
            c.last_tx = tick;
          }
        } else if (c.fin_sent && tick - c.last_tx >= 200) {
          emit(c, base + c.snd_nxt, ackNum(c), segtest::ACK | segtest::FIN);
          c.last_tx = tick;
        } else if (tick - c.last_tx >= 300) { // keepalive / window probe: a live server ACKs, a closed one RSTs
          emit(c, base + c.snd_nxt - 1, ackNum(c), segtest::ACK);
          c.last_tx = tick;
        }
        break;
      }
      case Client::kDone: break;
    }
  }

  uint32_t fill(uint8_t* slots, uint32_t stride, uint32_t off, uint32_t cap) {
    ++tick;
    for (auto& c : clients) step(c);
    uint32_t n = 0;
    size_t i = 0;
    for (; i < q.size() && n < cap; i++) {
      if (loss() % 100 < 3) {
        drops_c2s++;
        continue;
      }
      uint8_t* s = slots + (size_t)n * stride;
      std::memset(s, 0, stride);
      std::memcpy(s + off, q[i].data(), q[i].size());
      n++;
    }
    q.erase(q.begin(), q.begin() + i);
    return n;
  }

  void send(const uint8_t* eth, uint32_t len) {
    out.emplace_back(eth, eth + len);
    if (loss() % 100 < 3) {
      drops_s2c++;
      return;
    }
    uint16_t dport;
    std::memcpy(&dport, eth + 36, 2);
    Client* cp = nullptr;
    for (auto& c : clients)
      if (htons(c.port) == dport) cp = &c;
    if (!cp || cp->st == Client::kDone) return;
    Client& c = *cp;
    const uint8_t fl = eth[47];
    const uint32_t seq = srv_detail::rd32(eth + 38), ack = srv_detail::rd32(eth + 42);
    const uint16_t wnd = (uint16_t)(eth[48] << 8 | eth[49]);
    const uint32_t plen = len - 54;
    if (fl & segtest::RST) {
      c.got_rst = true;
      if (c.st == Client::kSynSent) c.refused = true;
      c.st = Client::kDone;
      return;
    }
    if ((fl & segtest::SYN) && (fl & segtest::ACK)) {
      if (c.st == Client::kSynSent) {
        c.srv_isn = seq;
        c.st = Client::kEst;
        c.established = true;
        c.srv_wnd = wnd;
        c.last_progress = tick;
      }
      if (c.st == Client::kEst) emit(c, c.isn + 1 + c.snd_nxt, ackNum(c), segtest::ACK); // (re-)ACK the SYN-ACK
      return;
    }
    if (c.st != Client::kEst) return;
    // ACK field
    const uint32_t acked = ack - (c.isn + 1);
    if ((int32_t)(acked - c.snd_una) > 0 && acked <= c.snd_nxt) {
      c.snd_una = acked;
      c.last_progress = tick;
    }
    c.srv_wnd = wnd;
    // data + FIN from the server
    bool owe_ack = false;
    if (plen) {
      const uint32_t off = seq - (c.srv_isn + 1);
      if (off <= c.echo.size() && off + plen > c.echo.size()) {
        c.echo.insert(c.echo.end(), eth + 54 + (c.echo.size() - off), eth + 54 + plen);
        for (auto it = c.ooo.begin(); it != c.ooo.end() && it->first <= c.echo.size();) {
          if (it->first + it->second.size() > c.echo.size())
            c.echo.insert(c.echo.end(), it->second.begin() + (c.echo.size() - it->first), it->second.end());
          it = c.ooo.erase(it);
        }
      } else if (off > c.echo.size()) {
        c.ooo[off].assign(eth + 54, eth + 54 + plen);
      }
      owe_ack = true;
    }
    if ((fl & segtest::FIN) && seq + plen == c.srv_isn + 1 + c.echo.size() && !c.got_fin) {
      c.got_fin = true;
      owe_ack = true;
    }
    if (owe_ack) emit(c, c.isn + 1 + c.snd_nxt, ackNum(c), segtest::ACK);
  }
};

template <class Conn>
struct PeerHandler {
  std::string* log;
  void line(const char* what, Conn& c) {
    sockaddr_in a;
    c.getPeername(a);
    char b[160];
    std::snprintf(b, sizeof b, "%s %u:%u id=%u err=%s echoed=%u\n", what, ntohl(a.sin_addr.s_addr), ntohs(a.sin_port),
                  c.getConnId(), c.getLastError() ? c.getLastError() : "-", c.echoed);
    *log += b;
  }
  bool allowNewConnection(uint32_t ip, uint16_t port_be) { return ntohs(port_be) % 7 != 0; }
  void onTcpConnected(Conn& c) {
    c.echoed = 0;
    c.fin_asked = false;
    line("connected", c);
  }
  uint32_t onTcpData(Conn& c, const uint8_t* d, uint32_t n) {
    sockaddr_in a;
    c.getPeername(a);
    const uint16_t port = ntohs(a.sin_port);
    if (port % 5 == 0 && n > 7) { // consume only whole 8-byte words: the rest is re-presented
      const uint32_t take = n & ~7u;
      if (!c.fin_asked && c.writeNonblock(d, take)) c.echoed += take;
      return n - take;
    }
    if (!c.fin_asked && c.writeNonblock(d, n)) c.echoed += n;
    if (port % 11 == 0 && c.echoed >= 4000 && !c.fin_asked) { // half-close from the server
      c.fin_asked = true;
      c.sendFin();
      line("sendFin", c);
    }
    return 0;
  }
  void onTcpDisconnect(Conn& c) { line("disconnect", c); }
  void onRecvTimeout(Conn& c) {
    line("recv timeout", c);
    c.close("timeout");
  }
  void onSendTimeout(Conn& c) { line("send timeout", c); }
};

template <class Backend, class Conf = PeerConf>
struct Run {
  using Server = GpuTcpServer<Conf, PeerLink, Backend>;
  std::unique_ptr<Server> srv = std::make_unique<Server>();
  std::string log;
  uint32_t polls = 0;

  bool go(const std::vector<Client>& population) {
    if (!srv->initWithLink("10.0.0.1", 1234, kT0)) {
      std::printf("init: %s\n", srv->getLastError());
      return false;
    }
    srv->link().clients = population;
    PeerHandler<typename Server::Conn> h{&log};
    for (polls = 1; polls < 30000; polls++) {
      srv->poll(h, kT0 + ((int64_t)polls << 20));
      if (srv->getLastError()) {
        std::printf("poll: %s\n", srv->getLastError());
        return false;
      }
      bool done = true;
      for (auto& c : srv->link().clients) done &= c.st == Client::kDone;
      if (done && srv->getConnCnt() == 0) break;
    }
    return true;
  }
};

static std::vector<Client> population() {
  std::mt19937_64 rng(0xC11E27ull + 0x9E3779B97F4A7C15ull * g_seed);
  std::vector<Client> cs(120);
  for (uint32_t i = 0; i < cs.size(); i++) {
    Client& c = cs[i];
    c.ip = 0x0a020000 | (i + 1);
    c.port = (uint16_t)(20000 + i * 13);
    c.kind = (Kind)(i % 4 == 3 ? kIdle : i % 3 == 2 ? kRstEnd : kFinEnd);
    if (c.port % 11 == 0) c.kind = kServerFin;
    c.start = 1 + (uint32_t)(rng() % 400);
    c.window = (i % 6 == 1) ? 2500 : 60000;
    c.stream.resize(2000 + rng() % 20000);
    for (auto& b : c.stream) b = (uint8_t)rng();
    c.isn = (uint32_t)rng();
    c.rng.seed((uint32_t)rng());
  }
  return cs;
}

template <class R>
static int check(const char* tag, R& r) {
  int fail = 0;
  uint32_t bad = 0;
  for (auto& f0 : r.srv->link().out) {
    std::vector<uint8_t> f(f0);
    f.resize(f0.size() + 2, 0);
    const pn_result x = segtest::classify(f.data(), (uint32_t)f.size());
    if ((x.flags & (PN_F_IP_OK | PN_F_TCP_OK)) != (PN_F_IP_OK | PN_F_TCP_OK)) bad++;
  }
  uint32_t est = 0, echo_ok = 0, echo_due = 0, refused = 0, timed_out = 0, idle = 0, not_done = 0;
  for (auto& c : r.srv->link().clients) {
    est += c.established;
    refused += c.refused;
    not_done += c.st != Client::kDone;
    if (c.kind == kIdle && c.established) {
      idle++;
      timed_out += c.got_rst;
    }
    if (c.established && (c.kind == kFinEnd || c.kind == kRstEnd) && c.port % 5 != 0) {
      echo_due++;
      echo_ok += c.echo == c.stream;
      if (c.echo != c.stream) {
        size_t d = 0;
        while (d < c.echo.size() && d < c.stream.size() && c.echo[d] == c.stream[d]) d++;
        std::printf("  echo port %u kind %d: %zu of %zu bytes, first difference %zu, rst %d fin %d win %u\n", c.port,
                    (int)c.kind, c.echo.size(), c.stream.size(), d, c.got_rst, c.got_fin, c.window);
      }
    }
  }
  const size_t timeouts = [&] {
    size_t n = 0, p = 0;
    while ((p = r.log.find("recv timeout", p)) != std::string::npos) n++, p++;
    return n;
  }();
  auto& L = r.srv->link();
  // exercised paths: retransmitted segments (same port/seq/flags seen before), SYN-ACKs, server FINs
  std::map<std::tuple<uint16_t, uint32_t, uint8_t>, int> seen;
  uint32_t retx = 0, synacks = 0, fins = 0, pure_acks = 0;
  for (auto& f : L.out) {
    uint16_t dport;
    std::memcpy(&dport, f.data() + 36, 2);
    const uint8_t fl = f[47];
    if ((fl & 0x12) == 0x12) synacks++;
    if (fl & 1) fins++;
    if (f.size() == 54 && fl == 0x18) pure_acks++;
    if (f.size() > 54 || (fl & 0x03)) retx += seen[{dport, srv_detail::rd32(f.data() + 38), fl}]++ > 0;
  }
  std::printf("%s: %u retransmitted segments, %u SYN-ACKs, %u FINs, %u pure ACKs; log: %zu sendFin\n", tag, retx,
              synacks, fins, pure_acks, [&] {
                size_t n = 0, p = 0;
                while ((p = r.log.find("sendFin", p)) != std::string::npos) n++, p++;
                return n;
              }());
  if (retx == 0 || fins == 0) fail++, std::printf("FAIL %s: retransmission / FIN paths not exercised\n", tag);
  std::printf("%s: %u polls, %zu TX frames (%u bad checksums), drops c2s %u s2c %u; %u established, %u refused, "
              "%u/%u echoes intact, %u/%u idle flows timed out (%zu recv timeouts), %u not done, conns left %u\n",
              tag, r.polls, L.out.size(), bad, L.drops_c2s, L.drops_s2c, est, refused, echo_ok, echo_due, timed_out,
              idle, timeouts, not_done, r.srv->getConnCnt());
  if (bad) fail++, std::printf("FAIL %s: TX frames with bad checksums\n", tag);
  if (echo_ok != echo_due || echo_due < 30) fail++, std::printf("FAIL %s: echoes\n", tag);
  if (timed_out != idle || idle == 0 || timeouts < idle) fail++, std::printf("FAIL %s: idle flows\n", tag);
  if (not_done || r.srv->getConnCnt()) {
    fail++;
    std::printf("FAIL %s: flows left\n", tag);
    for (auto& c : r.srv->link().clients)
      if (c.st != Client::kDone)
        std::printf("  port %u kind %d st %d una %u nxt %u len %zu echo %zu got_fin %d fin_sent %d wnd %u\n", c.port,
                    (int)c.kind, (int)c.st, c.snd_una, c.snd_nxt, c.stream.size(), c.echo.size(), c.got_fin,
                    c.fin_sent, c.srv_wnd);
  }
  if (refused == 0) fail++, std::printf("FAIL %s: no admission refusal exercised\n", tag);
  return fail;
}

// the same Conf with every TX batch through the backend's fill (pn_tx_fill on the GPU, the
// oracle's fill in the twin) instead of the host for batches with few payload frames
template <class Conf>
struct AllTxOnBackend : Conf {
  static const uint32_t TxGpuMinDataFrames = 0;
};
// ... and a mixed policy: batches with 2+ payload frames through the backend, the rest on the host
template <class Conf>
struct MixedTx : Conf {
  static const uint32_t TxGpuMinDataFrames = 2;
};

template <class A, class B>
static int same_frames(const char* what, A& a, B& b) {
  const auto &x = a.srv->link().out, &y = b.srv->link().out;
  const bool eq = x == y && a.log == b.log;
  std::printf("%s: TX frames %s (%zu vs %zu), logs %s\n", what, eq ? "identical" : "DIFFERENT", x.size(), y.size(),
              a.log == b.log ? "identical" : "DIFFERENT");
  return eq ? 0 : 1;
}

template <class Conf>
static int scenario(bool gpu, const std::vector<Client>& pop, const char* name) {
  int fail = 0;
  Run<OracleBackend, Conf> twin;
  if (!twin.go(pop)) return 100;
  {
    // TX policies: host sums for small batches (default), the oracle's fill for every batch, mixed
    Run<OracleBackend, AllTxOnBackend<Conf>> twin_b;
    Run<OracleBackend, MixedTx<Conf>> twin_m;
    if (!twin_b.go(pop) || !twin_m.go(pop)) return 100;
    std::printf("[%s] TX policies: default %llu frames summed on the host; mixed %llu host + %llu backend fill\n",
                name, (unsigned long long)twin.srv->txHostFrames(), (unsigned long long)twin_m.srv->txHostFrames(),
                (unsigned long long)twin_m.srv->txGpuFrames());
    if (!twin_m.srv->txHostFrames() || !twin_m.srv->txGpuFrames() || twin_b.srv->txHostFrames())
      fail++, std::printf("FAIL: both TX policies not exercised\n");
    fail += same_frames("twin host-fill vs twin backend-fill", twin, twin_b);
    fail += same_frames("twin mixed vs twin backend-fill", twin_m, twin_b);
  }
  std::printf("[%s] twin: %llu records re-resolved against the live table\n", name,
              (unsigned long long)twin.srv->reResolved());
  fail += check("twin", twin);
  // pipelined, connections are accepted between a batch's launch and its dispatch
  if (Conf::RxPipeline && !twin.srv->reResolved()) fail++, std::printf("FAIL: no re-resolved record\n");
  if (gpu) {
    Run<GpuBackend, Conf> g;
    if (!g.go(pop)) return 100;
    fail += check("gpu", g);
    const auto &a = g.srv->link().out, &b = twin.srv->link().out;
    size_t same = 0;
    while (same < a.size() && same < b.size() && a[same] == b[same]) same++;
    const bool frames_eq = a.size() == b.size() && same == a.size();
    if (!frames_eq) std::printf("FAIL: TX frames differ: gpu %zu, twin %zu, first difference at %zu\n", a.size(), b.size(), same);
    if (g.log != twin.log) std::printf("FAIL: handler logs differ\n");
    fail += !frames_eq + (g.log != twin.log);
    std::printf("gpu: handler log %s, TX frames %s (%zu)\n", g.log == twin.log ? "identical" : "DIFFERENT",
                frames_eq ? "identical" : "DIFFERENT", a.size());
    Run<GpuBackend, MixedTx<Conf>> g_mixed; // batches with payload through pn_tx_fill, the rest on the host
    if (!g_mixed.go(pop)) return 100;
    if (!g_mixed.srv->txGpuFrames() || !g_mixed.srv->txHostFrames())
      fail++, std::printf("FAIL: gpu mixed TX policy not exercised\n");
    fail += same_frames("gpu mixed TX policy vs twin", g_mixed, twin);
  }
  return fail;
}

// pollnet's EfviTcpServer wrapper never consults the handler's allowNewConnection (its TmpHandler
// returns true, EfviTcp.h:270): without Conf::UseAllowNewConnection the same handler, which would
// refuse every port divisible by 7, gets no refusal at all (room for every client).
struct PeerConfWrapper : PeerConf {
  static const bool UseAllowNewConnection = false;
  static const uint32_t MaxConns = 128;
};
static int wrapper_admission(bool gpu, const std::vector<Client>& pop) {
  auto one = [&](auto& r, const char* tag) {
    if (!r.go(pop)) return 100;
    uint32_t refused = 0, est = 0, by7 = 0;
    for (auto& c : r.srv->link().clients) {
      refused += c.refused;
      est += c.established;
      by7 += c.established && c.port % 7 == 0;
    }
    std::printf("%s (allowNewConnection not consulted): %u established (%u on ports divisible by 7), %u refused\n", tag,
                est, by7, refused);
    return (refused != 0 || by7 == 0) ? (std::printf("FAIL %s: wrapper admission\n", tag), 1) : 0;
  };
  Run<OracleBackend, PeerConfWrapper> twin;
  int fail = one(twin, "twin");
  if (gpu) {
    Run<GpuBackend, PeerConfWrapper> g;
    fail += one(g, "gpu");
  }
  return fail;
}

int main(int argc, char** argv) {
  const bool gpu = argc > 1 && std::strcmp(argv[1], "gpu") == 0;
  const uint32_t runs = argc > 2 ? (uint32_t)std::atoi(argv[2]) : 1; // soak: more populations and loss patterns
  int fail = 0;
  for (g_seed = 0; g_seed < runs; g_seed++) {
    if (runs > 1) std::printf("== population %u ==\n", g_seed);
    const auto pop = population();
    fail += scenario<PeerConf>(gpu, pop, "classify every poll");
    fail += scenario<PeerConfBudget>(gpu, pop, "3-ms RX latency budget");
    fail += scenario<PeerConfChunk>(gpu, pop, "RX chunks of 16");
    fail += scenario<PeerConfPipe>(gpu, pop, "pipelined RX (dispatch one poll later)");
    if (g_seed == 0) fail += wrapper_admission(gpu, pop);
  }
  std::printf("%s\n", fail ? "FAIL" : "PASS");
  return fail ? 1 : 0;
}
