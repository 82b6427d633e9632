// Shared pieces of the GpuTcpServer tests: a scripted link, the sequential oracle
// backend (the reference's semantics: each frame classified against the live table when
// the loop reaches it; TX checksums by the oracle — test infrastructure only) and a
// stand-in for std::cout.
#pragma once

#include <arpa/inet.h>

#include <cstring>
#include <sstream>
#include <vector>

#include "../../include/pollnet_amd/tcp_server.hpp"
#include "../../oracle/pn_oracle.h"

// Frames in (a prepared list, per_poll at a time), frames out (recorded).
struct ScriptLink {
  std::vector<std::vector<uint8_t>> in, out;
  size_t pos = 0;
  uint32_t per_poll = 1u << 30;
  const char* open(const char*) { return nullptr; }
  uint32_t fill(uint8_t* slots, uint32_t stride, uint32_t off, uint32_t cap) {
    uint32_t n = 0;
    while (n < cap && n < per_poll && pos < in.size()) {
      uint8_t* s = slots + (size_t)n * stride;
      std::memset(s, 0, stride);
      std::memcpy(s + off, in[pos].data(), in[pos].size());
      ++pos;
      ++n;
    }
    return n;
  }
  void send(const uint8_t* eth, uint32_t len) { out.emplace_back(eth, eth + len); }
  uint32_t localIp() const { return htonl(0x0a000001); }
  const uint8_t* localMac() const {
    static const uint8_t m[6] = {2, 0, 0, 0, 0, 1};
    return m;
  }
};

// The reference's sequential semantics: classify each frame when the loop reaches it.
struct OracleBackend {
  static constexpr bool kSnapshot = false;
  static constexpr uint32_t kStride = 2048, kFrameOff = 2;
  // verify = false: the release path, as the GPU backend's pn_set_verify(ctx, 0) -- no segment sum per frame, the
  // records pn_classify writes then (orc_classify_frame_release); the reference's release build sums nothing
  bool verify = true;
  const char* setVerify(bool v) {
    verify = v;
    return nullptr;
  }
  std::vector<uint8_t> rx, tx;
  std::vector<pn_result> recs[3]; // pipelined: each ring's records, classified at launch
  std::vector<uint16_t> lk[3];     // links: each ring's chain links (orc_chain_links), as the GPU's linked post
  uint32_t cap = 0;
  uint32_t tcap = 0;
  bool links = false;
  const char* init(int, uint32_t rx_cap, uint32_t tx_cap, uint32_t = 0, uint32_t rx_halves = 1, uint32_t tx_halves = 1,
                   bool = false, bool with_links = false) {
    cap = rx_cap;
    tcap = tx_cap;
    links = with_links && rx_cap <= PN_LINK_MAX_FRAMES;
    if (rx_halves < 1 || rx_halves > 3) return "rx_halves out of range";
    rx.assign((size_t)kStride * rx_cap * rx_halves, 0);
    tx.assign((size_t)kStride * tx_cap * (tx_halves == 2 ? 2 : 1), 0);
    for (int b = 0; b < 3; b++) {
      recs[b].assign(rx_cap, pn_result{});
      lk[b].assign(rx_cap, 0);
    }
    return nullptr;
  }
  void chain(uint32_t half, uint32_t n, const pollnet_amd::ConnTable& t) {
    if (links)
      orc_chain_links(rxSlots(half), kStride, kFrameOff, n, recs[half].data(), t.maxConnCnt(), PN_LINK_MAX_FRAMES,
                      PN_LINK_MAX_CONNS, lk[half].data());
  }
  uint8_t* rxSlots(uint32_t half = 0) { return rx.data() + (size_t)half * cap * kStride; }
  uint8_t* txSlots(uint32_t half = 0) { return tx.data() + (size_t)half * tcap * kStride; }
  const char* syncTable(const pollnet_amd::ConnTable&) { return nullptr; }
  static uint64_t keyOf(const uint8_t* eth) {
    uint32_t ip_be;
    uint16_t port_be;
    std::memcpy(&ip_be, eth + 26, 4);
    std::memcpy(&port_be, eth + 34, 2);
    return pollnet_amd::conn_hash_key(ip_be, port_be);
  }
  void one(const uint8_t* eth, const pollnet_amd::ConnTable& t, pn_result* r) const {
    uint32_t ne = 0;
    uint64_t mask = 0;
    const pn_conn_entry* e = t.entries(&ne, &mask);
    if (verify) orc_classify_frame(eth, kStride - kFrameOff, e, ne, mask, t.maxConnCnt(), r);
    else orc_classify_frame_release(eth, kStride - kFrameOff, e, ne, mask, t.maxConnCnt(), r);
  }
  // sequential: each frame against the live table, just before its dispatch (with links: the batch's links from its
  // records against the table at the start, the GPU's snapshot -- the engine uses a link only while the table is the
  // snapshot's, when the live records are those records)
  template <class F>
  const char* classify(uint32_t n, const pollnet_amd::ConnTable& t, F&& f) {
    if (links) {
      for (uint32_t i = 0; i < n; i++) one(rx.data() + (size_t)i * kStride + kFrameOff, t, &recs[0][i]);
      chain(0, n, t);
    }
    for (uint32_t i = 0; i < n; i++) {
      const uint8_t* eth = rx.data() + (size_t)i * kStride + kFrameOff;
      pn_result r;
      one(eth, t, &r);
      f(keyOf(eth), r, eth, links ? lk[0][i] : (uint16_t)0);
    }
    return nullptr;
  }
  // pipelined: the whole half against the table as it is at launch (the GPU's snapshot)
  const char* launch(uint32_t half, uint32_t n, const pollnet_amd::ConnTable& t) {
    for (uint32_t i = 0; i < n; i++) one(rxSlots(half) + (size_t)i * kStride + kFrameOff, t, &recs[half][i]);
    chain(half, n, t);
    return nullptr;
  }
  const char* ready(uint32_t) { return nullptr; } // classified at launch
  template <class F>
  const char* collect(uint32_t half, uint32_t n, const pollnet_amd::ConnTable&, F&& f) {
    for (uint32_t i = 0; i < n; i++) { // as GpuBackend: a hit's key is not computed (the engine derives it)
      const uint8_t* eth = rxSlots(half) + (size_t)i * kStride + kFrameOff;
      const pn_result& r = recs[half][i];
      f((r.flags & (PN_F_HIT | PN_F_TW)) == PN_F_HIT ? 0 : keyOf(eth), r, eth, links ? lk[half][i] : (uint16_t)0);
    }
    return nullptr;
  }
  const char* fillTx(uint32_t n, uint32_t half = 0) {
    orc_tx_fill_batch(txSlots(half), kStride, kFrameOff, n, nullptr, PN_TX_TCP, 1);
    return nullptr;
  }
  // pipelined: filled at launch; the engine sends the batch a poll later, as with the GPU
  const char* fillTxLaunch(uint32_t n, uint32_t half) { return fillTx(n, half); }
  const char* fillTxWait() { return nullptr; }
};

struct LogStream { // stands in for std::cout in the example's handler
  std::ostringstream os;
  template <class T>
  LogStream& operator<<(const T& v) {
    os << v;
    return *this;
  }
  LogStream& operator<<(std::ostream& (*m)(std::ostream&)) {
    os << m;
    return *this;
  }
};

