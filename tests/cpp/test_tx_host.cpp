// The drop-in engine's host-side TX checksums (srv_detail::fill_tcp_checksums, tcp_engine.hpp: the
// header-only batches a poll sends) against the oracle's PN_TX_TCP fill (oracle/pn_tx_oracle.c, itself
// pinned to the reference's copyAndSum / setOptDataLen, tests/test_tx.py) over random frames: every
// tot_len from 40 to 1500 (odd and even), random header and payload bytes, random old checksum
// fields; frames with tot_len below the bare headers must be left untouched by both.  Host only.
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
  std::printf("%s\n", diff ? "FAIL" : "PASS");
  return diff ? 1 : 0;
}
