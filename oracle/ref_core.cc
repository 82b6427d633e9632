// Test-only harness: compiles the reference's OWN efvitcp/Core.h code for the hot path,
// extracted verbatim from /root/reference at build time (oracle/ref.mk -> _ref/core_*.inc,
// git-ignored; no reference text is kept in the repository):
//   core_defs.inc     Core.h:44-138, 167-182  constants, EtherHeader/IpHeader/TcpHeader,
//                                             CSum, connHashKey, getMSB, ConnHashEntry
//   core_sizes.inc    Core.h:235-236          MaxTableSize, TotalTableSize
//   core_table.inc    Core.h:558-605, 640-682 findConnEntry, getTblSize, addConnEntry,
//                                             delConnEntry, printTbl, tryExpandConnTbl
//   core_checksum.inc Core.h:448-472          Core::checksum (EFVITCP_DEBUG)
//   onpack_head.inc   TcpConn.h:469-473       TcpConn::onPack's payload extent and seq
//   tx_copyandsum.inc TcpConn.h:257-299       TcpConn::copyAndSum (send path: append + sum)
//   tx_setoptdatalen.inc Core.h:157-163       SendBuf::setOptDataLen (tot_len, both folds)
//   efvi_hdrs.inc     Efvi.h:557-586          ci_ether_hdr / ci_ip4_hdr / ci_udp_hdr
//   efvi_ipsum_cache.inc Efvi.h:406-411       Efvi's cached IPv4 header sum
//   efvi_update_udp_pkt.inc Efvi.h:611-621    Efvi::update_udp_pkt (tot_len, checksum, udp_len)
// Those member functions are pasted, unchanged, into RefCore below, which supplies only
// the data members they read (conn_tbl, tbl_mask, conn_cnt, conns, tw_cnt, tw_ids) and
// takes the debug build's `cout` / `exit(1)` as members, so a failed check is recorded
// and execution continues (the reference process would end there).  No ef_vi header is
// needed or faked: none of these lines touches ef_vi.
// Nothing here is shipped or used by the product path; tests/test_ref_core.py pins the
// oracle (oracle/pn_oracle.c) and the product's conn table against it, and bench.py times
// ref_bench_batch as its CPU baseline (kind "reference": the reference's own code, run here).
#define EFVITCP_DEBUG
#include <arpa/inet.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <iostream>
#include <memory>
#include <sstream>
#include <string>
#include <thread>
#include <utility>
#include <vector>

namespace efvitcp {
using std::endl;
#include "_ref/core_defs.inc"

// The debug build's output and exit, captured.
struct Capture {
  std::ostringstream os;
  template <class T>
  Capture& operator<<(const T& v) {
    os << v;
    return *this;
  }
  Capture& operator<<(std::ostream& (*m)(std::ostream&)) {
    os << m;
    return *this;
  }
};

template <uint32_t MaxConn, uint32_t MaxTW>
struct RefCore {
  struct Conf {
    static const uint32_t MaxConnCnt = MaxConn;
    static const uint32_t MaxTimeWaitConnCnt = MaxTW;
  };
#include "_ref/core_sizes.inc"

  Capture cout;
  int exits = 0;
  void exit(int) { ++exits; }

  // the id stacks are sized for any mix of connection and TIME_WAIT ids up to the table's
  // capacity (random test histories do not keep the reference's per-class limits)
  uint32_t conn_cnt = 0;
  uint32_t conns[MaxConn + MaxTW];
  uint32_t tw_cnt = 0;
  uint32_t tw_ids[MaxConn + MaxTW];
  uint64_t tbl_mask = 0;
  ConnHashEntry conn_tbl[TotalTableSize];

  RefCore() { // Core::init's table part (Core.h:315-322)
    for (uint32_t i = 0; i < MaxConn; i++) conns[i] = i;
    for (uint32_t i = 0; i < MaxTW; i++) tw_ids[i] = i;
    for (auto& e : conn_tbl) e.key = EmptyKey;
    tbl_mask = std::min(MaxTableSize, 128u) - 1;
  }

#include "_ref/core_table.inc"
#include "_ref/core_checksum.inc"
};
// The send path's byte work.  SendBuf's header part (Core.h:147-156 without post_addr, send_ts,
// avail and pad, which setOptDataLen does not touch) with setOptDataLen pasted unchanged, and
// TcpConn's copyAndSum pasted unchanged into a holder (it reads no TcpConn member).
#pragma pack(push, 1)
struct RefSendHdr {
  EtherHeader eth_hdr;
  IpHeader ip_hdr;
  TcpHeader tcp_hdr;
#include "_ref/tx_setoptdatalen.inc"
};
#pragma pack(pop)
struct RefCopyAndSum {
#include "_ref/tx_copyandsum.inc"
};
} // namespace efvitcp

namespace {
using Ref = efvitcp::RefCore<256, 256>; // the oracle tests' table sizing (tests/test_oracle.py)
}

extern "C" {

uint16_t ref_csum_fold(uint32_t sum) { return efvitcp::CSum(sum).fold(); }

// CSum over n host-order u16 words via add(uint16_t), then fold().
uint16_t ref_csum_words(const uint16_t* w, uint32_t n) {
  efvitcp::CSum s = 0;
  for (uint32_t i = 0; i < n; i++) s.add(w[i]);
  return s.fold();
}

uint64_t ref_conn_hash_key(uint32_t ip_be, uint16_t port_be) { return efvitcp::connHashKey(ip_be, port_be); }

// Header fields as the reference's bitfield structs read them (IpHeader/TcpHeader, Core.h:57-87):
// out[0] ip header_len, [1] ip_ver, [2] tot_len (host order), [3] protocol,
// [4] data_offset, [5] fin, [6] syn, [7] rst, [8] psh, [9] ack, [10] seq (host order).
void ref_header_fields(const uint8_t* eth, uint32_t* out) {
  const auto* ip = reinterpret_cast<const efvitcp::IpHeader*>(eth + sizeof(efvitcp::EtherHeader));
  const auto* tcp = reinterpret_cast<const efvitcp::TcpHeader*>(ip + 1);
  out[0] = ip->header_len;
  out[1] = ip->ip_ver;
  out[2] = ntohs(ip->tot_len);
  out[3] = ip->protocol;
  out[4] = tcp->data_offset;
  out[5] = tcp->fin;
  out[6] = tcp->syn;
  out[7] = tcp->rst;
  out[8] = tcp->psh;
  out[9] = tcp->ack;
  out[10] = ntohl(tcp->seq_num);
}

// Core::checksum on one frame: bit 0 = the IP sum verified, bit 1 = the TCP sum verified
// (each exit(1) of the debug build is recorded instead of ending the process).
int ref_checksum(const uint8_t* eth) {
  std::unique_ptr<Ref> c(new Ref());
  c->checksum(reinterpret_cast<efvitcp::IpHeader*>(const_cast<uint8_t*>(eth) + sizeof(efvitcp::EtherHeader)));
  const std::string log = c->cout.os.str();
  const bool ip_bad = log.find("invalid ip sum") != std::string::npos;
  const bool tcp_bad = log.find("invalid tcp sum") != std::string::npos;
  return (ip_bad ? 0 : 1) | (tcp_bad ? 0 : 2);
}

// The same, plus the folded sums the check printed ("invalid ip sum: N" / "invalid tcp sum: N";
// 0 when it verified): the value pn_result.tcp_fold carries.
int ref_checksum_folds(const uint8_t* eth, uint32_t* ip_fold, uint32_t* tcp_fold) {
  std::unique_ptr<Ref> c(new Ref());
  c->checksum(reinterpret_cast<efvitcp::IpHeader*>(const_cast<uint8_t*>(eth) + sizeof(efvitcp::EtherHeader)));
  const std::string log = c->cout.os.str();
  auto value = [&](const char* what) -> uint32_t {
    const size_t p = log.find(what);
    return p == std::string::npos ? 0u : (uint32_t)std::stoul(log.substr(p + std::strlen(what)));
  };
  *ip_fold = value("invalid ip sum: ");
  *tcp_fold = value("invalid tcp sum: ");
  return (*ip_fold ? 0 : 1) | (*tcp_fold ? 0 : 2);
}

// TcpConn::onPack's first statements (TcpConn.h:469-473) on one frame: payload offset from
// the Ethernet header, payload length (data_end - data, signed), seq + syn.
void ref_onpack_head(uint8_t* eth, uint32_t* payload_off, int32_t* payload_len, uint32_t* seq) {
  using namespace efvitcp;
  IpHeader* ip_hdr = reinterpret_cast<IpHeader*>(eth + sizeof(EtherHeader));
#include "_ref/onpack_head.inc"
  (void)opt;
  *payload_off = (uint32_t)(data - eth);
  *payload_len = (int32_t)(data_end - data);
  *seq = seq_num;
}

// One data segment of an established connection without timestamps, built as TcpConn builds
// it, on a frame whose Ethernet / IP / TCP headers (data_offset 5, urgent pointer 0) are in
// place at eth: reset (TcpConn.h:149-168) caches ipsum over the IP header with tot_len and
// checksum zeroed and tcpsum = src + dst + ntohs(6) + both ports; onEstablished (:422-428)
// adds offset_flags; sendPartial (:232-256) appends the payload in the given pieces with
// copyAndSum, each piece at its real address (odd ones too), into data_sum; sendBuf
// (:310-323) adds seq, ack and window, then tcpsum, and setOptDataLen writes tot_len and the
// two checksums.  The glue is restated; copyAndSum, CSum and setOptDataLen are the reference's.
void ref_tx_data_segment(uint8_t* eth, const uint8_t* payload, uint32_t len, const uint32_t* pieces,
                         uint32_t n_pieces) {
  using namespace efvitcp;
  RefSendHdr* b = reinterpret_cast<RefSendHdr*>(eth);
  b->ip_hdr.tot_len = 0;
  b->ip_hdr.checksum = 0;
  CSum ipsum = 0;
  ipsum.add<sizeof(IpHeader)>(&b->ip_hdr);
  CSum tcpsum = 0;
  tcpsum.add(b->ip_hdr.src_ip);
  tcpsum.add(b->ip_hdr.dst_ip);
  tcpsum.add(ntohs(0x6));
  tcpsum.add(b->tcp_hdr.src_port);
  tcpsum.add(b->tcp_hdr.dst_port);
  tcpsum.add(b->tcp_hdr.offset_flags);
  CSum data_sum = 0;
  RefCopyAndSum c;
  uint8_t* data = eth + sizeof(RefSendHdr);
  uint32_t off = 0;
  for (uint32_t i = 0; i < n_pieces && off < len; i++) {
    const uint32_t m = std::min(pieces[i], len - off);
    data_sum.add(c.copyAndSum(data + off, payload + off, m));
    off += m;
  }
  if (off < len) data_sum.add(c.copyAndSum(data + off, payload + off, len - off));
  CSum sum = data_sum;
  sum.add(b->tcp_hdr.seq_num);
  sum.add(b->tcp_hdr.ack_num);
  sum.add(b->tcp_hdr.window_size);
  sum.add(tcpsum);
  b->setOptDataLen((uint16_t)len, ipsum, sum);
}

// Efvi's UDP sender (Efvi.h): the header structs, the cached IPv4 header sum and update_udp_pkt
// pasted unchanged; the cache is taken over the frame's own IPv4 header with tot_len and checksum
// zeroed, as init_udp_pkt's ci_ip4_hdr_init leaves them (Efvi.h:403-411, 625-640).
struct RefEfviUdp {
#include "_ref/efvi_hdrs.inc"
#pragma pack(pop)
  uint32_t ipsum_cache = 0;
  void cache(uint8_t* eth) {
    uint16_t* ip4 = (uint16_t*)(eth + 14);
#include "_ref/efvi_ipsum_cache.inc"
  }
#include "_ref/efvi_update_udp_pkt.inc"
};

// One Efvi datagram: header cached with tot_len = checksum = 0, then update_udp_pkt(paylen).
void ref_efvi_udp_datagram(uint8_t* eth, uint32_t paylen) {
  RefEfviUdp u;
  eth[16] = eth[17] = 0; // ip_tot_len_be16
  eth[24] = eth[25] = 0; // ip_check_be16
  u.cache(eth);
  u.update_udp_pkt(eth, paylen);
}

// ---- the conn table, driven the way the reference's callers drive it ----
void* ref_table_new() { return new Ref(); }
void ref_table_free(void* t) { delete static_cast<Ref*>(t); }

// TcpServer.h:88-90 / Core::enterTW's bookkeeping: a connection id takes a conn slot, an id
// >= MaxConnCnt a TIME_WAIT slot; then findConnEntry + addConnEntry.  -1 if the key is present.
int ref_table_add(void* tp, uint64_t key, uint32_t conn_id) {
  Ref* t = static_cast<Ref*>(tp);
  efvitcp::ConnHashEntry* e = t->findConnEntry(key);
  if (e->key == key) return -1;
  if (conn_id < 256) t->conn_cnt++;
  else t->tw_cnt++;
  t->addConnEntry(e, key, conn_id);
  return 0;
}
int ref_table_del(void* tp, uint64_t key) {
  Ref* t = static_cast<Ref*>(tp);
  if (t->findConnEntry(key)->key != key) return -1;
  t->delConnEntry(key);
  return 0;
}
// relabel (Core::enterTW's entry->conn_id = MaxConnCnt + tw_id, Core.h:626), moving the count
int ref_table_set_conn_id(void* tp, uint64_t key, uint32_t conn_id) {
  Ref* t = static_cast<Ref*>(tp);
  efvitcp::ConnHashEntry* e = t->findConnEntry(key);
  if (e->key != key) return -1;
  if (e->conn_id < 256 && conn_id >= 256) t->conn_cnt--, t->tw_cnt++;
  if (e->conn_id >= 256 && conn_id < 256) t->tw_cnt--, t->conn_cnt++;
  e->conn_id = conn_id;
  return 0;
}
uint32_t ref_table_find(void* tp, uint64_t key) {
  Ref* t = static_cast<Ref*>(tp);
  return (uint32_t)(t->findConnEntry(key) - t->conn_tbl);
}
// entries as 16-B {key, conn_id, pad} records (the product's pn_conn_entry layout)
uint32_t ref_table_entries(void* tp, uint64_t* keys, uint32_t* conn_ids, uint64_t* mask) {
  Ref* t = static_cast<Ref*>(tp);
  for (uint32_t i = 0; i < Ref::TotalTableSize; i++) {
    keys[i] = t->conn_tbl[i].key;
    conn_ids[i] = t->conn_tbl[i].conn_id;
  }
  *mask = t->tbl_mask;
  return Ref::TotalTableSize;
}
uint32_t ref_table_total_size() { return Ref::TotalTableSize; }

// ---- the CPU baseline: the reference's own per-frame code over a ring of slots ----
// Per frame, in pollNet's order (Core.h:503-510, debug build; the release build skips the first step):
// Core::checksum (Core.h:448-472),
// key = connHashKey(src_ip, src_port), entry = findConnEntry(key), the TIME_WAIT test, and
// TcpConn::onPack's payload extent and seq (TcpConn.h:469-473).  The table is the bench's
// (MaxConnCnt = MaxTimeWaitConnCnt = 1024, pollnet_amd.rx.GenParams), one copy per thread.
// Each frame folds into a digest over (verified, hit, tw, conn_id, payload_off, payload_len,
// seq) so the work is observable and comparable with the oracle's records
// (tests/test_ref_core.py).
using RefBench = efvitcp::RefCore<1024, 1024>;

void* ref_bench_new(const uint64_t* keys, const uint32_t* conn_ids, uint32_t n) {
  RefBench* t = new RefBench();
  for (uint32_t i = 0; i < n; i++) {
    efvitcp::ConnHashEntry* e = t->findConnEntry(keys[i]);
    if (e->key == keys[i]) continue;
    if (conn_ids[i] < 1024) t->conn_cnt++;
    else t->tw_cnt++;
    t->addConnEntry(e, keys[i], conn_ids[i]);
  }
  return t;
}
void ref_bench_free(void* t) { delete static_cast<RefBench*>(t); }

// CHECK = false: the release build's per-frame work (Core.h:503-510 without EFVITCP_DEBUG's Core::checksum,
// then onPack's head): the digest's verified bit is 0, as records_digest(release=True) computes it.
extern "C++" {
template <bool CHECK>
static inline uint64_t ref_frame_digest(RefBench& t, uint8_t* eth) {
  using namespace efvitcp;
  IpHeader* ip_hdr = reinterpret_cast<IpHeader*>(eth + sizeof(EtherHeader));
  bool verified = false;
  if constexpr (CHECK) {
    const int exits0 = t.exits;
    t.checksum(ip_hdr);
    verified = t.exits == exits0;
  }
  TcpHeader* th = reinterpret_cast<TcpHeader*>(ip_hdr + 1);
  const uint64_t key = connHashKey(ip_hdr->src_ip, th->src_port);
  ConnHashEntry* entry = t.findConnEntry(key);
  const bool hit = entry->key == key;
  const bool tw = hit && entry->conn_id >= 1024;
#include "_ref/onpack_head.inc"
  (void)opt;
  const uint64_t conn = hit ? entry->conn_id : 0xffffffffu;
  uint64_t x = (uint64_t)verified | (uint64_t)hit << 1 | (uint64_t)tw << 2 | conn << 3;
  x ^= ((uint64_t)(uint32_t)(data - eth) << 32 | (uint32_t)(int32_t)(data_end - data)) * 0x9E3779B97F4A7C15ull;
  x ^= (uint64_t)seq_num * 0xC2B2AE3D27D4EB4Full;
  return x * 0xD6E8FEB86659FD93ull ^ (x >> 29);
}

// Frames [0, n) of the slot ring, split into contiguous shards over `threads` threads (each
// with its own copy of the table).  Returns the digest (sum over frames, order-free); *n_valid
// = frames whose checksums verified (CHECK; 0 on the release path).
template <bool CHECK>
static uint64_t ref_batch(void* tp, uint8_t* slots, uint32_t stride, uint32_t off, uint32_t n, int threads,
                          uint32_t* n_valid) {
  RefBench* proto = static_cast<RefBench*>(tp);
  if (threads < 1) threads = 1;
  std::vector<uint64_t> dig(threads, 0);
  std::vector<uint32_t> valid(threads, 0);
  auto work = [&](int w) {
    std::unique_ptr<RefBench> t(new RefBench()); // the table members the functions read
    t->conn_cnt = proto->conn_cnt;
    t->tw_cnt = proto->tw_cnt;
    t->tbl_mask = proto->tbl_mask;
    std::memcpy(t->conn_tbl, proto->conn_tbl, sizeof(t->conn_tbl));
    const uint32_t b = (uint32_t)((uint64_t)n * w / threads), e = (uint32_t)((uint64_t)n * (w + 1) / threads);
    uint64_t d = 0;
    uint32_t v = 0;
    int exits_cleared = 0;
    for (uint32_t i = b; i < e; i++) {
      const int exits0 = t->exits;
      d += ref_frame_digest<CHECK>(*t, slots + (size_t)i * stride + off);
      if constexpr (CHECK) {
        if (t->exits == exits0) {
          v++;
        } else if (t->exits - exits_cleared > 256) { // drop the debug build's prints now and then
          t->cout.os.str(std::string());
          exits_cleared = t->exits;
        }
      }
    }
    dig[w] = d;
    valid[w] = v;
  };
  std::vector<std::thread> pool;
  for (int w = 1; w < threads; w++) pool.emplace_back(work, w);
  work(0);
  for (auto& th : pool) th.join();
  uint64_t d = 0;
  uint32_t v = 0;
  for (int w = 0; w < threads; w++) d += dig[w], v += valid[w];
  if (n_valid) *n_valid = v;
  return d;
}
} // extern "C++"
// The debug build's per-frame work (Core::checksum included): bench.py's cpu_baseline headline.
uint64_t ref_bench_batch(void* tp, uint8_t* slots, uint32_t stride, uint32_t off, uint32_t n, int threads,
                         uint32_t* n_valid) {
  return ref_batch<true>(tp, slots, stride, off, n, threads, n_valid);
}
// The release build's (no checksum): cpu_baseline.release_path, beside pn_set_verify(ctx, 0).
uint64_t ref_release_batch(void* tp, uint8_t* slots, uint32_t stride, uint32_t off, uint32_t n, int threads) {
  return ref_batch<false>(tp, slots, stride, off, n, threads, nullptr);
}
// how many times the debug build's rehash check fired (Core.h:665-669: it would have exited)
int ref_table_debug_exits(void* tp) { return static_cast<Ref*>(tp)->exits; }

} // extern "C"
