// The drop-in engine's host-side TX checksums (srv_detail::fill_tcp_checksums, tcp_engine.hpp: the
// header-only batches a poll sends) against the oracle's PN_TX_TCP fill (oracle/pn_tx_oracle.c, itself
// pinned to the reference's copyAndSum / setOptDataLen, tests/test_tx.py) over random frames: every
// tot_len from 40 to 1500 (odd and even), random header and payload bytes, random old checksum
// fields; frames with tot_len below the bare headers must be left untouched by both.  Also the sums a header-only
// frame gets as it is built (srv_detail::header_sums, from the field values) against fill_tcp_checksums over the
// same bytes, and the inline connHashKey (conn_hash_key) against the oracle's.  Host only.
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "../../include/pollnet_amd/tcp_engine.hpp"
#include "../../oracle/pn_oracle.h"

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)std::atoi(argv[1]) : 20000;
  const uint32_t stride = 2048, off = 2;
  std::mt19937_64 rng(0x7E57C0DEull);
  std::vector<uint8_t> a((size_t)n * stride), b;
  uint32_t short_frames = 0;
  for (uint32_t i = 0; i < n; i++) {
    uint8_t* s = a.data() + (size_t)i * stride;
    for (uint32_t k = 0; k < stride; k++) s[k] = (uint8_t)rng();
    uint8_t* ip = s + off + 14;
    uint32_t tot = i < 1461 ? 40 + i : 40 + (uint32_t)(rng() % 1461); // every length once, then random
    if (i % 97 == 5) tot = (uint32_t)(rng() % 40);                      // below the headers: untouched
    short_frames += tot < 40;
    ip[0] = 0x45;
    ip[2] = (uint8_t)(tot >> 8);
    ip[3] = (uint8_t)tot;
    ip[9] = 6;
  }
  b = a;
  for (uint32_t i = 0; i < n; i++) pollnet_amd::srv_detail::fill_tcp_checksums(a.data() + (size_t)i * stride + off);
  orc_tx_fill_batch(b.data(), stride, off, n, nullptr, PN_TX_TCP, 1);
  uint32_t diff = 0;
  for (uint32_t i = 0; i < n; i++)
    if (std::memcmp(a.data() + (size_t)i * stride, b.data() + (size_t)i * stride, stride)) {
      if (diff++ < 5) std::printf("frame %u differs\n", i);
    }
  std::printf("%u frames (%u below the headers): %u differ from the oracle's fill\n", n, short_frames, diff);

  // header-only frames as TcpEngine::header builds them: random addresses, ports, seq, ack, flags, window
  uint32_t hdiff = 0;
  for (uint32_t i = 0; i < n; i++) {
    uint8_t f[64] = {};
    uint8_t* ip = f + 14;
    const uint32_t src = (uint32_t)rng(), dst = (uint32_t)rng(), seq = (uint32_t)rng(), ack = (uint32_t)rng();
    const uint16_t sp = (uint16_t)rng(), dp = (uint16_t)rng(), win = (uint16_t)rng();
    const uint8_t flags = (uint8_t)rng();
    ip[0] = 0x45;
    pollnet_amd::srv_detail::wr16(ip + 2, 40);
    pollnet_amd::srv_detail::wr16(ip + 6, 0x4000);
    ip[8] = 64;
    ip[9] = 6;
    std::memcpy(ip + 12, &src, 4);
    std::memcpy(ip + 16, &dst, 4);
    uint8_t* tcp = ip + 20;
    std::memcpy(tcp, &sp, 2);
    std::memcpy(tcp + 2, &dp, 2);
    pollnet_amd::srv_detail::wr32(tcp + 4, seq);
    pollnet_amd::srv_detail::wr32(tcp + 8, ack);
    tcp[12] = 0x50;
    tcp[13] = flags;
    pollnet_amd::srv_detail::wr16(tcp + 14, win);
    uint8_t g[64];
    std::memcpy(g, f, 64);
    pollnet_amd::srv_detail::fill_tcp_checksums(g);
    const auto cs = pollnet_amd::srv_detail::header_sums(src, dst, sp, dp, seq, ack, flags, win);
    std::memcpy(ip + 10, &cs.ip, 2);
    std::memcpy(tcp + 16, &cs.tcp, 2);
    if (std::memcmp(f, g, 64)) {
      if (hdiff++ < 5) std::printf("header-only frame %u: built sums differ from fill_tcp_checksums\n", i);
    }
  }
  std::printf("%u header-only frames: %u built sums differ\n", n, hdiff);

  uint32_t kdiff = 0;
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t ipb = (uint32_t)rng();
    const uint16_t pb = (uint16_t)rng();
    kdiff += pollnet_amd::conn_hash_key(ipb, pb) != orc_conn_hash_key(ipb, pb);
  }
  std::printf("%u keys: %u differ from the oracle's connHashKey\n", n, kdiff);
  const bool fail = diff || hdiff || kdiff;
  std::printf("%s\n", fail ? "FAIL" : "PASS");
  return fail ? 1 : 0;
}
