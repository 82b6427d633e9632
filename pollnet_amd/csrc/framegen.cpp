// Deterministic synthetic RX-ring generator for the BASELINE configs (libpollnet_amd_gen.so,
// include/pollnet_amd_gen.h: workload tooling, not the product ABI)
// (SURVEY.md §8d C2-C5).  Every frame is a pure function of (seed, global frame
// index), so threads and ranks can generate disjoint shards of one batch.
//
// Slot layout (the reference's RecvBuf ring, Core.h:140-145, 503-505): frame i's
// Ethernet header starts at slot + frame_off; bytes after the frame are zero
// (the reference's odd-length TCP sum reads one byte past the segment,
// Core.h:113-117, so the pad byte is part of the contract; C5 sets it on purpose
// for a slice of frames).
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/pollnet_amd_gen.h"

namespace {

inline uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

struct XorShift64 {
  uint64_t s;
  explicit XorShift64(uint64_t seed) : s(splitmix64(seed) | 1) {}
  uint64_t next() {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return s;
  }
  uint32_t below(uint32_t n) { return (uint32_t)((next() >> 11) % n); }
};

struct Flow {
  uint32_t ip_be;
  uint16_t port_be;
};

inline uint32_t ip4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  return __builtin_bswap32((a << 24) | (b << 16) | (c << 8) | d);
}

// Flow k of a config.  C3/C4/C5: 10.1.(k>>8).(k&255) with a distinct random
// ephemeral port in [32768, 60999]; C5 replaces the last 64 flows with an
// adversarial cluster whose ports share their low 12 bits (same home slot once
// tbl_mask = 4095, so one long sorted probe run).
std::vector<Flow> make_flows(const pn_gen_params& p) {
  std::vector<Flow> flows;
  if (p.cfg == 2) {
    flows.push_back({ip4(10, 0, 0, 2), __builtin_bswap16(40000)});
    return flows;
  }
  const uint32_t lo = 32768, span = 61000 - 32768;
  std::vector<uint16_t> ports(span);
  for (uint32_t i = 0; i < span; i++) ports[i] = (uint16_t)(lo + i);
  XorShift64 r(p.seed ^ 0xF10F10F1ull);
  for (uint32_t i = 0; i < span - 1; i++) std::swap(ports[i], ports[i + r.below(span - i)]);
  for (uint32_t k = 0; k < p.n_flows; k++) flows.push_back({ip4(10, 1, k >> 8, k & 255), __builtin_bswap16(ports[k % span])});
  if (p.cfg == 5 && p.n_flows >= 128) {
    for (uint32_t j = 0; j < 64; j++) {
      uint32_t k = p.n_flows - 64 + j;
      flows[k] = {ip4(10, 3, 0, j), __builtin_bswap16((uint16_t)(32768 + (j % 8) * 4096 + 777))};
    }
  }
  return flows;
}

bool is_tw_flow(const pn_gen_params& p, uint32_t k, uint32_t* tw_id) {
  if (p.n_tw_flows == 0 || p.n_flows == 0) return false;
  uint32_t stride = p.n_flows / p.n_tw_flows;
  if (stride == 0) stride = 1;
  if (k % stride != 1 % stride || k / stride >= p.n_tw_flows) return false;
  if (tw_id) *tw_id = k / stride;
  return true;
}

// RFC 1071 one's-complement sum over big-endian 16-bit words (odd tail padded).
uint32_t be_sum(const uint8_t* b, uint32_t len, uint32_t acc) {
  uint32_t i = 0;
  for (; i + 1 < len; i += 2) acc += ((uint32_t)b[i] << 8) | b[i + 1];
  if (len & 1) acc += (uint32_t)b[len - 1] << 8;
  return acc;
}
uint16_t be_fold_not(uint32_t acc) {
  while (acc >> 16) acc = (acc & 0xffff) + (acc >> 16);
  return (uint16_t)~acc;
}
inline void put16(uint8_t* p, uint16_t v) {
  p[0] = (uint8_t)(v >> 8);
  p[1] = (uint8_t)v;
}
inline void put32(uint8_t* p, uint32_t v) {
  p[0] = (uint8_t)(v >> 24);
  p[1] = (uint8_t)(v >> 16);
  p[2] = (uint8_t)(v >> 8);
  p[3] = (uint8_t)v;
}

void gen_one(const pn_gen_params& p, const std::vector<Flow>& flows, uint64_t gi, uint8_t* slot, uint32_t stride,
             uint32_t off) {
  memset(slot, 0, stride);
  XorShift64 r(p.seed ^ (gi * 0xD1B54A32D192ED03ull));
  uint8_t* eth = slot + off;
  uint8_t* ip = eth + 14;
  const uint32_t avail = stride - off;

  // flow
  Flow f;
  if ((p.cfg == 3 || p.cfg == 5) && r.below(64) == 0) {
    // one draw per statement: the frames must not depend on the compiler's argument order
    const uint32_t c = r.below(256);
    const uint32_t d = r.below(256);
    const uint32_t port = 1024 + r.below(64000);
    f = {ip4(10, 2, c, d), __builtin_bswap16((uint16_t)port)};
  } else if (p.cfg == 2) {
    f = flows[0];
  } else {
    f = flows[r.below((uint32_t)flows.size())];
  }

  // geometry
  uint32_t ihl = 5, doff = 5, tot_len = 1500;
  if (p.cfg == 3) tot_len = 50 + r.below(1451);
  if (p.cfg == 5) {
    if (r.below(4) == 0) ihl = 6 + r.below(10);
    doff = 5 + r.below(11);
    uint32_t mn = 4 * ihl + 4 * doff;
    tot_len = mn + r.below(1500 - mn + 1);
  }
  if (p.cfg == 3 && avail > 2048 && r.below(8) == 0) tot_len = 1500 + r.below(std::min<uint32_t>(avail, 65000) - 1515); // jumbo slots
  if (14 + tot_len + 1 > avail) tot_len = avail - 15; // keep the pad byte inside the slot
  if (tot_len < 4 * ihl + 4 * doff) { // tiny slots: drop options so the headers fit
    ihl = 5;
    doff = 5;
  }
  const uint32_t hl = 4 * ihl, th = 4 * doff;
  if (tot_len < hl + th) tot_len = hl + th;

  // Ethernet
  const uint8_t dmac[6] = {2, 0, 0, 0, 0, 1}, smac[6] = {2, 0, 0, 0, 0, 2};
  memcpy(eth, dmac, 6);
  memcpy(eth + 6, smac, 6);
  put16(eth + 12, 0x0800);

  // IPv4
  ip[0] = (uint8_t)(0x40 | ihl);
  ip[1] = 0;
  put16(ip + 2, (uint16_t)tot_len);
  put16(ip + 4, (uint16_t)gi);
  put16(ip + 6, 0x4000); // DF
  ip[8] = 64;
  ip[9] = 6;
  memcpy(ip + 12, &f.ip_be, 4);
  memcpy(ip + 16, "\x0a\x00\x00\x01", 4); // 10.0.0.1
  for (uint32_t i = 20; i < hl; i++) ip[i] = (uint8_t)r.below(2); // NOP / EOL option bytes

  // TCP at ip + IHL*4 (RFC placement)
  uint8_t* tcp = ip + hl;
  memcpy(tcp, &f.port_be, 2);
  put16(tcp + 2, 1234);
  uint32_t seq = p.cfg == 2 ? (uint32_t)(gi * 1460u) : (uint32_t)r.next();
  put32(tcp + 4, seq);
  put32(tcp + 8, (uint32_t)r.next());
  uint8_t fl = 0x18; // ACK|PSH
  if (p.cfg == 3 || p.cfg == 5) {
    uint32_t x = r.below(256);
    if (x == 0 || x == 1) fl = 0x02;      // SYN
    else if (x == 2 || x == 3) fl = 0x11; // FIN|ACK
    else if (x == 4) fl = 0x04;           // RST
    else if (x == 5) fl = 0x12;           // SYN|ACK
  }
  tcp[12] = (uint8_t)(doff << 4);
  tcp[13] = fl;
  put16(tcp + 14, 0xffff);
  for (uint32_t i = 20; i < th; i++) tcp[i] = 1; // NOP options

  // payload
  uint8_t* pay = tcp + th;
  const uint32_t plen = tot_len - hl - th;
  for (uint32_t i = 0; i < plen; i += 8) {
    uint64_t v = r.next();
    uint32_t n = std::min<uint32_t>(8, plen - i);
    memcpy(pay + i, &v, n);
  }

  // checksums (RFC 791 / 793)
  put16(ip + 10, be_fold_not(be_sum(ip, hl, 0)));
  uint8_t pseudo[12];
  memcpy(pseudo, ip + 12, 8);
  pseudo[8] = 0;
  pseudo[9] = 6;
  put16(pseudo + 10, (uint16_t)(tot_len - hl));
  put16(tcp + 16, be_fold_not(be_sum(tcp, tot_len - hl, be_sum(pseudo, 12, 0))));

  // deterministic damage so both verdicts occur
  if (p.cfg == 2 || p.cfg == 4) {
    if ((gi & 1023) == 1023) pay[(gi >> 10) % plen] ^= (uint8_t)(1u << (gi % 8));
  } else {
    uint32_t d = r.below(2048);
    if (d < 2) {
      if (plen) {
        const uint32_t bit = r.below(8); // (the committed goldens draw the bit before the byte)
        pay[r.below(plen)] ^= (uint8_t)(1u << bit);
      }
      else tcp[16] ^= 0x40;
    } else if (d == 2) {
      ip[8] ^= 0x10; // TTL: IP sum breaks, TCP (no TTL in pseudo-header) stays valid
    }
    if (p.cfg == 5 && (tot_len & 1) && r.below(16) == 0) ip[tot_len] = 0xA5; // non-zero byte after the frame
  }
}

} // namespace

extern "C" {

int pn_gen_frames(const pn_gen_params* p, uint64_t first_index, uint32_t n, void* slots_host, uint32_t slot_stride,
                  uint32_t frame_off, int n_threads) {
  if (!p || !slots_host || (p->cfg < 2 || p->cfg > 5)) return PN_EINVAL;
  if (slot_stride < frame_off + 96 || (frame_off & 1)) return PN_EINVAL;
  if (p->cfg != 2 && p->n_flows == 0) return PN_EINVAL;
  const std::vector<Flow> flows = make_flows(*p);
  if (n_threads < 1) n_threads = 1;
  n_threads = std::min<int>(n_threads, 64);
  if (n < 4096) n_threads = 1;
  uint8_t* base = (uint8_t*)slots_host;
  auto work = [&](uint32_t lo, uint32_t hi) {
    for (uint32_t i = lo; i < hi; i++) gen_one(*p, flows, first_index + i, base + (uint64_t)i * slot_stride, slot_stride, frame_off);
  };
  if (n_threads == 1) {
    work(0, n);
  } else {
    std::vector<std::thread> th;
    for (int t = 0; t < n_threads; t++)
      th.emplace_back(work, (uint32_t)((uint64_t)n * t / n_threads), (uint32_t)((uint64_t)n * (t + 1) / n_threads));
    for (auto& x : th) x.join();
  }
  return PN_OK;
}

int pn_gen_conn_table(const pn_gen_params* p, pn_conn_table* t) {
  if (!p || !t) return PN_EINVAL;
  const std::vector<Flow> flows = make_flows(*p);
  // addConnEntry in flow order (conn_id = flow index), then enterTW relabels
  // conn_id to MaxConnCnt + tw_id (Core.h:621-627).
  for (uint32_t k = 0; k < flows.size(); k++) {
    int rc = pn_table_add(t, pn_conn_hash_key(flows[k].ip_be, flows[k].port_be), k);
    if (rc) return rc;
  }
  for (uint32_t k = 0; k < flows.size(); k++) {
    uint32_t tw;
    if (is_tw_flow(*p, k, &tw)) {
      int rc = pn_table_set_conn_id(t, pn_conn_hash_key(flows[k].ip_be, flows[k].port_be), p->max_conn_cnt + tw);
      if (rc) return rc;
    }
  }
  return PN_OK;
}

uint64_t pn_wire_bytes(const void* slots_host, uint32_t slot_stride, uint32_t frame_off, uint32_t n) {
  const uint8_t* b = (const uint8_t*)slots_host;
  uint64_t s = 0;
  for (uint32_t i = 0; i < n; i++) {
    const uint8_t* ip = b + (uint64_t)i * slot_stride + frame_off + 14;
    s += 14 + (((uint32_t)ip[2] << 8) | ip[3]);
  }
  return s;
}

} // extern "C"
