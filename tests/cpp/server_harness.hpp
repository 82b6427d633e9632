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
  std::vector<uint8_t> rx, tx;
  const char* init(int, uint32_t rx_cap, uint32_t tx_cap, uint32_t = 0) {
    rx.assign((size_t)kStride * rx_cap, 0);
    tx.assign((size_t)kStride * tx_cap, 0);
    return nullptr;
  }
  uint8_t* rxSlots() { return rx.data(); }
  uint8_t* txSlots() { return tx.data(); }
  const char* syncTable(const pollnet_amd::ConnTable&) { return nullptr; }
  template <class F>
  const char* classify(uint32_t n, const pollnet_amd::ConnTable& t, F&& f) {
    for (uint32_t i = 0; i < n; i++) {
      const uint8_t* eth = rx.data() + (size_t)i * kStride + kFrameOff;
      uint32_t ne = 0;
      uint64_t mask = 0;
      const pn_conn_entry* e = t.entries(&ne, &mask);
      pn_result r;
      orc_classify_frame(eth, kStride - kFrameOff, e, ne, mask, t.maxConnCnt(), &r);
      uint32_t ip_be;
      uint16_t port_be;
      std::memcpy(&ip_be, eth + 26, 4);
      std::memcpy(&port_be, eth + 34, 2);
      f(pn_conn_hash_key(ip_be, port_be), r, eth);
    }
    return nullptr;
  }
  const char* fillTx(uint32_t n) {
    orc_tx_fill_batch(tx.data(), kStride, kFrameOff, n, nullptr, PN_TX_TCP, 1);
    return nullptr;
  }
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

