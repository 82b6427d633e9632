// Test helper: builds Ethernet/IPv4/TCP frames (valid RFC 1071 checksums) for
// segment-level scenarios, and classifies them with the C oracle (the checker).
#pragma once

#include <cstdint>
#include <cstring>
#include <random>
#include <vector>

#include "../../include/pollnet_amd.h"
#include "../../oracle/pn_oracle.h"

namespace segtest {

enum : uint8_t { FIN = 1, SYN = 2, RST = 4, PSH = 8, ACK = 16 };

struct Seg {
  uint32_t src_ip = 0x0a000002; // host order
  uint16_t src_port = 40000;
  uint32_t seq = 0;
  uint32_t ack = 0;
  uint8_t flags = ACK;
  std::vector<uint8_t> opts; // TCP options (padded to 4 B by the builder)
  const uint8_t* payload = nullptr;
  uint32_t len = 0;
  bool corrupt = false; // flip a payload (or header) bit after the checksums
};

inline void put16(uint8_t* p, uint16_t v) {
  p[0] = v >> 8;
  p[1] = v & 0xff;
}
inline void put32(uint8_t* p, uint32_t v) {
  put16(p, v >> 16);
  put16(p + 2, v & 0xffff);
}
inline uint16_t rfc_sum(const uint8_t* p, uint32_t n, uint32_t acc) {
  for (uint32_t i = 0; i + 1 < n; i += 2) acc += (uint32_t)p[i] << 8 | p[i + 1];
  if (n & 1) acc += (uint32_t)p[n - 1] << 8;
  while (acc >> 16) acc = (acc & 0xffff) + (acc >> 16);
  return (uint16_t)~acc;
}

// Writes the frame at eth (room for it required); returns its length (14 + tot_len).
inline uint32_t build(uint8_t* eth, const Seg& s) {
  const uint32_t olen = (uint32_t)((s.opts.size() + 3) & ~size_t(3));
  const uint32_t tcp_len = 20 + olen + s.len;
  const uint32_t tot = 20 + tcp_len;
  std::memset(eth, 0, 14 + 20 + 20 + olen);
  const uint8_t mac_dst[6] = {2, 0, 0, 0, 0, 1}, mac_src[6] = {2, 0, 0, 0, 0, 2};
  std::memcpy(eth, mac_dst, 6);
  std::memcpy(eth + 6, mac_src, 6);
  put16(eth + 12, 0x0800);
  uint8_t* ip = eth + 14;
  ip[0] = 0x45;
  put16(ip + 2, (uint16_t)tot);
  put16(ip + 6, 0x4000);
  ip[8] = 64;
  ip[9] = 6;
  put32(ip + 12, s.src_ip);
  put32(ip + 16, 0x0a000001);
  put16(ip + 10, rfc_sum(ip, 20, 0));
  uint8_t* tcp = ip + 20;
  put16(tcp, s.src_port);
  put16(tcp + 2, 1234);
  put32(tcp + 4, s.seq);
  put32(tcp + 8, s.ack);
  tcp[12] = (uint8_t)(((20 + olen) / 4) << 4);
  tcp[13] = s.flags;
  put16(tcp + 14, 65535);
  for (size_t i = 0; i < s.opts.size(); i++) tcp[20 + i] = s.opts[i];
  if (s.len) std::memcpy(tcp + 20 + olen, s.payload, s.len);
  uint32_t ph = (s.src_ip >> 16) + (s.src_ip & 0xffff) + (0x0a000001 >> 16) + (0x0a000001 & 0xffff) + 6 + tcp_len;
  put16(tcp + 16, rfc_sum(tcp, tcp_len, ph));
  if (s.corrupt) tcp[tcp_len - 1] ^= 0x10;
  return 14 + tot;
}

// The oracle's record for one frame against an empty table.
inline pn_result classify(const uint8_t* eth, uint32_t avail) {
  static const pn_conn_entry empty[1] = {{PN_EMPTY_KEY, 0, 0}};
  pn_result r;
  orc_classify_frame(eth, avail, empty, 1, 0, 1, &r);
  return r;
}

} // namespace segtest
