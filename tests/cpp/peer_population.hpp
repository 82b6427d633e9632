// A deterministic in-memory TCP client population (with loss in both directions) acting as a
// GpuTcpServer link, and the handler the server tests run over it.  Shared by
// test_tcp_server_peer.cpp (GPU vs sequential twin) and test_ref_server.cpp (both vs the
// reference's own efvitcp server, oracle/ref_server.hpp).
#pragma once

#include <sys/uio.h>
#include <arpa/inet.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <random>
#include <string>
#include <vector>

#include "segframes.hpp"
#include "../../include/pollnet_amd/tcp_engine.hpp"

using pollnet_amd::srv_detail::rd32;

static const int64_t kT0 = (int64_t)777777 << 20;

enum Kind : uint8_t { kFinEnd, kRstEnd, kIdle, kServerFin, kChaos };

// One segment of a kChaos client's schedule: stream bytes [off, off + len) sent with `flags`
// at sequence base + off + shift (shift != 0: outside the receive window, or RST probes).
struct ChaosSeg {
  uint32_t off, len;
  uint8_t flags;
  int32_t shift;
}; 

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
  // kChaos: the schedule, then go-back-N repair from the server's ACK with a FIN on the last piece
  std::vector<ChaosSeg> sched;
  size_t sched_pos = 0;
  uint32_t repairs = 0;
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
        if (c.kind == kChaos) {
          chaosStep(c);
          break;
        }
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

  // kChaos (chaos_population): after the handshake, the schedule at 4 segments a tick —
  // reordered, duplicated, overlapping, re-segmented, some without ACK, with SYN, out of the
  // window, RSTs in and out of it; then go-back-N from the server's ACK every 20 ticks, the last
  // piece carrying the FIN, until the server's RST (pollnet closes on a remote FIN) or 60 rounds.
  void chaosStep(Client& c) {
    const uint32_t base = c.isn + 1, L = (uint32_t)c.stream.size();
    if (c.sched_pos < c.sched.size()) {
      for (int k = 0; k < 4 && c.sched_pos < c.sched.size() && c.st == Client::kEst; k++) {
        const ChaosSeg& g = c.sched[c.sched_pos++];
        const uint32_t seq = base + g.off + (uint32_t)g.shift;
        if (g.flags & segtest::RST) {
          emit(c, seq, (g.flags & segtest::ACK) ? ackNum(c) : 0, g.flags);
          if (g.shift == 0) c.st = Client::kDone; // an RST that may land in the window: the client is gone
        } else {
          emit(c, seq, ackNum(c), g.flags, c.stream.data() + g.off, g.len);
        }
      }
      c.last_tx = tick;
      return;
    }
    if (tick - c.last_tx < 20) return;
    if (++c.repairs > 60) {
      c.st = Client::kDone;
      return;
    }
    c.last_tx = tick;
    uint32_t off = c.snd_una;
    const uint32_t end = std::min(L, off + std::max<uint32_t>(1, std::min<uint32_t>(c.srv_wnd, 3000)));
    do {
      const uint32_t n = std::min<uint32_t>(end - off, 1000);
      const bool last = off + n == L;
      emit(c, base + off, ackNum(c), (uint8_t)(segtest::ACK | segtest::PSH | (last ? segtest::FIN : 0)),
           c.stream.data() + off, n);
      off += n;
    } while (off < end);
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

  // Deferred (defer = true): the server's frames reach the clients when the poll ends
  // (endPoll), whenever within the poll they were sent — a wire one poll long.  The reference
  // sends each frame as it builds it, the engine at the end of its poll: with the wire in
  // between, both present the clients the same frames at the same tick.
  bool defer = false;
  std::vector<std::vector<uint8_t>> in_flight;
  void send(const uint8_t* eth, uint32_t len) {
    if (defer) {
      in_flight.emplace_back(eth, eth + len);
      return;
    }
    deliver(eth, len);
  }
  void endPoll() {
    std::vector<std::vector<uint8_t>> f;
    f.swap(in_flight);
    for (auto& x : f) deliver(x.data(), (uint32_t)x.size());
  }
  void deliver(const uint8_t* eth, uint32_t len) {
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
    const uint32_t seq = rd32(eth + 38), ack = rd32(eth + 42);
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
        if (c.kind == kChaos) c.snd_nxt = (uint32_t)c.stream.size();
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
    if (port >= 30000 && port % 13 == 0) return n; // a chaos client's handler that consumes nothing: window fills
    if (port % 4 == 1) { // the send side's state as the handler sees it (TcpConn.h:47-56)
      char b[96];
      std::snprintf(b, sizeof b, "data %u id=%u n=%u sendable=%u now=%u\n", port, c.getConnId(), n, c.getSendable(),
                    c.getImmediatelySendable());
      *log += b;
    }
    if (port % 8 == 3 && !c.fin_asked) { // echo in two pieces through sendv (TcpConn.h:63-70); what does not fit is dropped
      iovec iov[2] = {{(void*)d, n / 2}, {(void*)(d + n / 2), n - n / 2}};
      c.echoed += c.sendv(iov, 2);
      return 0;
    }
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


// Clients that send adversarial segment streams (kChaos, ports >= 30000) beside ordinary ones.
inline std::vector<Client> chaos_population(uint32_t n_chaos = 60, uint32_t n_plain = 20) {
  std::mt19937_64 rng(0xC4A05ull + 0x9E3779B97F4A7C15ull * g_seed);
  auto U = [&](uint32_t lo, uint32_t hi) { return lo + (uint32_t)(rng() % (hi - lo + 1)); };
  std::vector<Client> cs(n_chaos + n_plain);
  for (uint32_t i = 0; i < cs.size(); i++) {
    Client& c = cs[i];
    const bool chaos = i < n_chaos;
    c.ip = 0x0a030000 | (i + 1);
    c.port = (uint16_t)(chaos ? 30000 + i * 7 : 20000 + i * 13);
    c.kind = chaos ? kChaos : (Kind)(i % 3 == 2 ? kRstEnd : kFinEnd);
    if (!chaos && c.port % 11 == 0) c.kind = kServerFin;
    c.start = 1 + (uint32_t)(rng() % 300);
    c.window = (i % 5 == 1) ? 3000 : 60000;
    c.stream.resize(chaos ? U(1, 30000) : 2000 + rng() % 12000);
    for (auto& b : c.stream) b = (uint8_t)rng();
    c.isn = (uint32_t)rng();
    c.rng.seed((uint32_t)rng());
    if (!chaos) continue;
    // packets, then arrival order: block shuffles (up to 6 out of order: 5+ extents), duplicates,
    // overlapping re-segmented retransmissions, and per segment odd flags or sequence numbers
    const uint32_t L = (uint32_t)c.stream.size();
    std::vector<std::pair<uint32_t, uint32_t>> pk;
    for (uint32_t o = 0; o < L;) {
      const uint32_t n = std::min(L - o, U(1, 1460));
      pk.push_back({o, n});
      o += n;
    }
    const uint32_t W = U(1, 7);
    std::vector<std::pair<uint32_t, uint32_t>> arr;
    for (size_t b = 0; b < pk.size(); b += W) {
      std::vector<std::pair<uint32_t, uint32_t>> blk(pk.begin() + b, pk.begin() + std::min(pk.size(), b + W));
      std::shuffle(blk.begin(), blk.end(), rng);
      for (auto& x : blk) {
        arr.push_back(x);
        if (rng() % 10 == 0) arr.push_back(arr[rng() % arr.size()]);
        if (rng() % 12 == 0) {
          const uint32_t a = U(0, x.first + x.second - 1);
          arr.push_back({a, std::min(L - a, U(1, 1460))});
        }
      }
    }
    for (auto& x : arr) {
      ChaosSeg g{x.first, x.second, (uint8_t)(segtest::ACK | segtest::PSH), 0};
      const uint32_t r = (uint32_t)(rng() % 1000);
      if (r < 30) g.flags = segtest::PSH;                              // no ACK: dropped after the RST check
      else if (r < 45) g.flags |= segtest::SYN;                        // SYN on a data segment (seq + 1)
      else if (r < 50) g.flags |= segtest::FIN;                        // FIN in the middle of the stream
      else if (r < 75) g.shift = 20000 + (int32_t)(rng() % 100000);    // far beyond the window
      else if (r < 95) g.shift = -(int32_t)(9000 + rng() % 60000);     // long before it (old data)
      else if (r < 100) g.shift = (int32_t)(rng() % 9000) - 4000;      // near the window's edges
      c.sched.push_back(g);
      const uint32_t q = (uint32_t)(rng() % 1000);
      if (q < 4) c.sched.push_back({x.first, 0, segtest::RST, 0});                          // RST, maybe in window
      else if (q < 10) c.sched.push_back({x.first, 0, segtest::RST | segtest::ACK, 200000}); // RST out of window
    }
  }
  return cs;
}
