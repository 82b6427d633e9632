// tcp_engine.hpp — the TCP endpoint engine under GpuTcpServer / GpuTcpClient.
//
// pollnet's efvitcp endpoints (TcpServer.h, TcpClient.h over Core<Conf> and TcpConn<Conf>)
// run per poll: one timer tick (Core::pollTime, Core.h:710-748), then Core::pollNet over
// the RX events (Core.h:494-552) with the endpoint's recv handler, TcpConn::onPack for
// segments of known connections (TcpConn.h:466-769), and every frame they send finalised
// with its checksums (SendBuf::setOptDataLen, Core.h:157-163).  TcpEngine does the same
// with the per-frame work on the GPU:
//   - the link's pending frames land in a pinned ring; ONE pn_classify launch parses them,
//     verifies both checksums and probes the conn table for the whole batch;
//   - the records are walked in ring order on the host: the NIC filter, the checksum discard
//     a NIC applies, TIME_WAIT (Core.h:510-524), then the endpoint's own branches for unknown
//     flows and unestablished connections (Derived::onMiss / Derived::onHandshake: a server's
//     SYN accept and SYN-RECEIVED, a client's SYN-SENT), then onPack — its receive half is
//     RxConn (rx_conn.hpp), its ACK-field / send half is here;
//   - every frame the poll built gets its IP and TCP checksums — from ONE pn_tx_fill launch
//     over the pinned TX batch when it carries enough payload (TxGpuMinDataFrames), else on the
//     host (header-only ACKs: nanoseconds each) — and leaves through the link in generation order.
// The table snapshot on the device is refreshed before each classify; records after a table
// change within the same batch are re-resolved on the host (one ordered probe), so every
// frame sees the table the reference's sequential loop would have shown it.
//
// Send side: the reference's segment ring (ConnSendBufCnt segments of up to SMSS bytes,
// TcpConn.h:58-90, 232-256), window, RTO / fast retransmit and delayed ACK, restated for
// pollnet's configuration (EfviTcp.h:21-36, 180-199: no window scaling, no timestamps, no
// congestion window).  Time: now_ts = ns >> 20 (Core.h:46), from `ns` or CLOCK_REALTIME.
#pragma once

#include <arpa/inet.h>
#include <net/if.h>
#include <netinet/in.h>
#include <sys/ioctl.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <cstdio>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <type_traits>
#include <utility>
#include <vector>

#include "gpu_rx.hpp"
#include "rx_conn.hpp"
#include "rx_ring.hpp"

namespace pollnet_amd {

// ---------------------------------------------------------------------------
// Optional Conf members / handler callbacks, detected by name.
namespace srv_detail {
#define PN_CONF_OPT(name, type, dflt)                                                               \
  template <class C, class = void>                                                                  \
  struct opt_##name {                                                                               \
    static constexpr type value = dflt;                                                             \
  };                                                                                                \
  template <class C>                                                                                \
  struct opt_##name<C, decltype(void(C::name))> {                                                   \
    static constexpr type value = C::name;                                                          \
  };
PN_CONF_OPT(SendTimeoutSec, uint32_t, 0)
PN_CONF_OPT(RecvTimeoutSec, uint32_t, 0)
PN_CONF_OPT(ConnSendBufCnt, uint32_t, 1024) // EfviTcp.h:181
PN_CONF_OPT(RxBatch, uint32_t, 512)         // frames per poll (RecvBufCnt = 512, EfviTcp.h:186)
PN_CONF_OPT(RxLatencyBudgetUs, uint32_t, 0) // hold received frames up to this long for a fuller batch
PN_CONF_OPT(TxBatch, uint32_t, 1024)        // frames per pn_tx_fill launch
PN_CONF_OPT(TxGpuMinDataFrames, uint32_t, 64) // a TX batch goes to pn_tx_fill when it holds at least this many
                                            // payload-bearing frames; below, every frame of it is
                                            // checksummed on the host (0 = always the GPU)
PN_CONF_OPT(UseAllowNewConnection, bool, false) // consult the handler's allowNewConnection on a SYN, as
                                            // efvitcp::TcpServer does (TcpServer.h:84); pollnet's
                                            // EfviTcpServer wrapper never does (EfviTcp.h:270)
PN_CONF_OPT(RxChunk, uint32_t, 0)           // frames per classify launch within a poll (0 = RxBatch): chunk
                                            // k+1 is on the GPU while chunk k is dispatched
PN_CONF_OPT(RxPipeline, bool, false)        // throughput mode: a poll's frames are classified while the
                                            // previous poll's are dispatched (one poll of added latency)
PN_CONF_OPT(RxPipelineDepth, uint32_t, 1)   // with RxPipeline: the polls a batch stays in flight before its
                                            // dispatch, 1 or 2 (2: the GPU has two polls' host work to finish a
                                            // batch in, one poll more of latency)
PN_CONF_OPT(RxResident, bool, false)        // the classify runs in the resident service (pn_service_*): a post
                                            // per poll through its mailbox instead of a launch
PN_CONF_OPT(RxLinks, bool, false)           // with RxResident: each post also returns its chain links
                                            // (pn_service_post_linked) and a frame that continues its connection's
                                            // previous one takes the in-order fast path.  Off by default: the GPU's
                                            // chain pass lengthens a 512-frame post more than the fast path saves
                                            // on the host
PN_CONF_OPT(DelayedAckMS, uint32_t, 10)     // EfviTcp.h:189
PN_CONF_OPT(Device, int, 0)
PN_CONF_OPT(ReferenceLiteralTable, bool, false) // PN_TABLE_REFERENCE_LITERAL: the reference's rehash, defect kept
PN_CONF_OPT(ConnRetrySec, uint32_t, 0)          // client: reconnect interval (EfviTcp.h:94-98), 0 = never
#undef PN_CONF_OPT

#define PN_HANDLER_OPT(name, call)                                                                   \
  template <class H, class C, class = void>                                                          \
  struct has_##name : std::false_type {};                                                            \
  template <class H, class C>                                                                        \
  struct has_##name<H, C, decltype(void(std::declval<H&>().call))> : std::true_type {};
PN_HANDLER_OPT(onTcpConnected, onTcpConnected(std::declval<C&>()))
PN_HANDLER_OPT(onTcpDisconnect, onTcpDisconnect(std::declval<C&>()))
PN_HANDLER_OPT(onSendTimeout, onSendTimeout(std::declval<C&>()))
PN_HANDLER_OPT(onRecvTimeout, onRecvTimeout(std::declval<C&>()))
PN_HANDLER_OPT(allowNewConnection, allowNewConnection(uint32_t(0), uint16_t(0)))
PN_HANDLER_OPT(onTcpConnectFailed, onTcpConnectFailed())
#undef PN_HANDLER_OPT

template <class C, class = void>
struct user_data {
  struct type {};
};
template <class C>
struct user_data<C, std::void_t<typename C::UserData>> {
  using type = typename C::UserData;
};

inline uint16_t rd16(const uint8_t* p) { return (uint16_t)(p[0] << 8 | p[1]); }
inline uint32_t rd32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }
inline void wr16(uint8_t* p, uint16_t v) {
  p[0] = (uint8_t)(v >> 8);
  p[1] = (uint8_t)v;
}
inline void wr32(uint8_t* p, uint32_t v) {
  wr16(p, (uint16_t)(v >> 16));
  wr16(p + 2, (uint16_t)v);
}

// One's-complement sum of n bytes taken as big-endian 16-bit words (an odd tail byte padded
// with zero, as copyAndSum pads it, TcpConn.h:291-295), accumulated from native-order loads: the
// folded result is the byte-swapped sum (RFC 1071 §2(B)), stored back with a native store.
inline uint64_t csum_add(const uint8_t* p, uint32_t n, uint64_t s) {
  for (; n >= 8; p += 8, n -= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    s += (v & 0xffffffffu) + (v >> 32);
  }
  if (n >= 4) {
    uint32_t v;
    std::memcpy(&v, p, 4);
    s += v;
    p += 4;
    n -= 4;
  }
  if (n >= 2) {
    uint16_t v;
    std::memcpy(&v, p, 2);
    s += v;
    p += 2;
    n -= 2;
  }
  if (n) s += p[0];
  return s;
}
inline uint16_t csum_fold(uint64_t s) { // CSum::fold (Core.h:94-98), carries folded back until none
  while (s >> 16) s = (s & 0xffff) + (s >> 16);
  return (uint16_t)~s;
}
// Both checksums of a header-only frame (20-B IP header, 20-B TCP header, no payload) from the field values the
// engine writes (TcpEngine::header), without reading the frame back: the same native-order word sums
// fill_tcp_checksums takes over those bytes, so the same folded values (tests/cpp/test_tx_host.cpp), as the
// reference's SendBuf::setOptDataLen folds them from its cached header sums (Core.h:157-163).  Addresses and ports
// are given in memory (network) order, the rest as numbers.
struct HeaderSums {
  uint16_t ip, tcp;
};
inline HeaderSums header_sums(uint32_t src_ip_mem, uint32_t dst_ip_mem, uint16_t src_port_mem, uint16_t dst_port_mem,
                              uint32_t seq, uint32_t ack, uint8_t flags, uint16_t window) {
  auto halves = [](uint32_t x) -> uint64_t { return (x & 0xffffu) + (x >> 16); };
  const uint64_t addr = halves(src_ip_mem) + halves(dst_ip_mem);
  // 45 00 | tot_len 40 | id 0 | 40 00 (DF) | ttl 64, proto 6 | checksum | addresses, as native 16-bit loads
  const uint64_t ip = 0x0045u + 0x2800u + 0x0040u + 0x0640u + addr;
  // pseudo-header (addresses, protocol 6, TCP length 20), ports, seq, ack, doff 5 | flags, window
  const uint64_t tcp = addr + 0x0600u + 0x1400u + src_port_mem + dst_port_mem + halves(__builtin_bswap32(seq)) +
                       halves(__builtin_bswap32(ack)) + (0x50u | (uint32_t)flags << 8) + __builtin_bswap16(window);
  return {csum_fold(ip), csum_fold(tcp)};
}
// Both checksums of a built TCP/IPv4 frame (eth = Ethernet header; 20-B IP header, as every
// frame the engine builds): the values SendBuf::setOptDataLen folds from its cached header sums
// (Core.h:157-163, at the end of TcpConn::sendBuf, TcpConn.h:310-323) and pn_tx_fill(PN_TX_TCP)
// writes.  A sum over these fields is never zero (IP version, protocol 6), so the folded value
// is unique and any correct order of summation gives the same bytes.
// A frame whose tot_len is below the bare headers (40) is left untouched, as pn_tx_fill leaves it.
inline void fill_tcp_checksums(uint8_t* eth) {
  uint8_t* ip = eth + 14;
  const uint32_t tot_len = rd16(ip + 2), tcp_len = tot_len - 20;
  if (tot_len < 40) return;
  ip[10] = ip[11] = 0;
  const uint16_t ip_sum = csum_fold(csum_add(ip, 20, 0));
  std::memcpy(ip + 10, &ip_sum, 2);
  uint8_t* tcp = ip + 20;
  tcp[16] = tcp[17] = 0;
  const uint16_t len_be = (uint16_t)(tcp_len >> 8 | (tcp_len & 0xff) << 8);
  uint64_t s = csum_add(ip + 12, 8, 0x0600u + len_be); // pseudo-header: addresses, protocol 6, TCP length
  const uint16_t tcp_sum = csum_fold(csum_add(tcp, tcp_len, s));
  std::memcpy(tcp + 16, &tcp_sum, 2);
}
} // namespace srv_detail

// ---------------------------------------------------------------------------
// Hashed timer wheel with efvitcp's semantics (Core.h:184-200, 684-748): 256 one-tick
// slots plus 256 slots of 256 ticks, LIFO within a slot, advanced one tick per call.
struct TimerNode {
  TimerNode* prev = this;
  TimerNode* next = this;
  uint32_t owner = 0; // conn id (< MaxConnCnt) or MaxConnCnt + tw id
  uint32_t kind = 0;  // 0 resend, 1 delayed ACK, 2 + user timer id; TIME_WAIT nodes: 0
  uint32_t expire = 0;
  TimerNode() = default;
  TimerNode(const TimerNode&) : TimerNode() {} // nodes are never copied linked
  TimerNode& operator=(const TimerNode&) { return *this; }
  bool unlinked() const { return prev == this; }
  void unlink() {
    prev->next = next;
    next->prev = prev;
    prev = next = this;
  }
};

class TimerWheel {
 public:
  static constexpr uint32_t kSlots = 256;
  TimerWheel() = default;
  TimerWheel(const TimerWheel&) = delete;
  TimerWheel& operator=(const TimerWheel&) = delete;

  uint32_t now() const { return now_; }
  void reset(uint32_t now_ts) {
    now_ = now_ts;
    for (auto& s : near_) s.prev = s.next = &s;
    for (auto& s : far_) s.prev = s.next = &s;
  }
  void add(uint32_t dur, TimerNode* n) {
    TimerNode* slot;
    if (dur <= kSlots) {
      slot = &near_[(now_ + dur) % kSlots];
    } else {
      dur = std::min(dur, kSlots * (kSlots + 1) - 1 - (now_ % kSlots));
      n->expire = now_ + dur;
      slot = &far_[n->expire / kSlots % kSlots];
    }
    n->next = slot->next;
    n->prev = slot;
    slot->next->prev = n;
    slot->next = n;
  }
  // One tick if ts moved (time never goes back); fire(node) for each expired node, unlinked.
  template <class Fire>
  void tick(uint32_t ts, Fire&& fire) {
    if (ts == now_) return;
    if (++now_ % kSlots == 0) { // cascade the far slot that comes due
      TimerNode* slot = &far_[now_ / kSlots % kSlots];
      for (TimerNode* n = slot->next; n != slot;) {
        TimerNode* nx = n->next;
        n->prev = n->next = n;
        add(n->expire - now_, n);
        n = nx;
      }
      slot->prev = slot->next = slot;
    }
    TimerNode* slot = &near_[now_ % kSlots];
    if (slot->unlinked()) return;
    TimerNode due; // detach the slot so timers re-armed while firing land in a later tick
    due.next = slot->next;
    due.prev = slot->prev;
    slot->next->prev = &due;
    slot->prev->next = &due;
    slot->prev = slot->next = slot;
    while (due.next != &due) {
      TimerNode* n = due.next;
      n->unlink();
      fire(n);
    }
  }

 private:
  uint32_t now_ = 0;
  TimerNode near_[kSlots], far_[kSlots];
};

// ---------------------------------------------------------------------------
// Links: where received frames come from and where built frames go.
//   const char* open(const char* interface)       (nullptr = ok)
//   uint32_t fill(uint8_t* slots, uint32_t stride, uint32_t frame_off, uint32_t cap)
//   void send(const uint8_t* eth, uint32_t len)
//   uint32_t localIp() (network order), const uint8_t* localMac()
//   const char* resolveMac(uint32_t ip_be, uint8_t* mac)   (clients: the next hop's MAC)
//
// SocketLink: an AF_PACKET socket on `interface` (pollnet's SocketEthReceiver,
// Socket.h:567-629, drained by recvmmsg into the pinned ring) that also transmits the
// built frames.  Needs CAP_NET_RAW; the host stack must be kept off the server port
// (e.g. a firewall drop), as with any user-space TCP stack on a shared interface.
class SocketLink {
 public:
  const char* open(const char* interface) {
    int fd = ::socket(AF_INET, SOCK_DGRAM, 0);
    if (fd < 0) return "socket(AF_INET) failed";
    ifreq ifr;
    std::memset(&ifr, 0, sizeof ifr);
    std::strncpy(ifr.ifr_name, interface, IFNAMSIZ - 1);
    ifr.ifr_addr.sa_family = AF_INET;
    int rc = ioctl(fd, SIOCGIFADDR, &ifr); // Core.h:258-264
    if (rc == 0) local_ip_ = ((sockaddr_in*)&ifr.ifr_addr)->sin_addr.s_addr;
    if (rc == 0 && (rc = ioctl(fd, SIOCGIFHWADDR, &ifr)) == 0) std::memcpy(mac_, ifr.ifr_hwaddr.sa_data, 6);
    ::close(fd);
    if (rc != 0) return "ioctl SIOCGIFADDR/SIOCGIFHWADDR failed";
    if (!rx_.init(interface)) return rx_.getLastError();
    return nullptr;
  }
  uint32_t fill(uint8_t* slots, uint32_t stride, uint32_t frame_off, uint32_t cap) {
    return rx_.fill(slots, stride, frame_off, cap);
  }
  void send(const uint8_t* eth, uint32_t len) { (void)::send(rx_.fd(), eth, len, MSG_DONTWAIT); }
  uint32_t localIp() const { return local_ip_; }
  const uint8_t* localMac() const { return mac_; }
  // The MAC of the next hop toward ip (TcpClient::getDestMac, TcpClient.h:100-152): the gateway
  // `ip route get` names (or ip itself when on-link), looked up in the kernel's ARP table.
  const char* resolveMac(uint32_t ip_be, uint8_t* mac) {
    char ip[INET_ADDRSTRLEN], cmd[96], line[512], hop[64] = "";
    inet_ntop(AF_INET, &ip_be, ip, sizeof ip);
    std::snprintf(cmd, sizeof cmd, "/usr/sbin/ip route get %s", ip);
    FILE* p = popen(cmd, "r");
    if (!p) return "ip route get failed";
    while (!hop[0] && fgets(line, sizeof line, p)) {
      const char* via = std::strstr(line, " via ");
      if (std::sscanf(via ? via + 5 : line, "%63s", hop) != 1) hop[0] = 0;
    }
    pclose(p);
    if (!hop[0]) return "no route to the server";
    FILE* arp = std::fopen("/proc/net/arp", "r");
    if (!arp) return "cannot open /proc/net/arp";
    bool found = false;
    char aip[64], hw[64];
    while (!found && fgets(line, sizeof line, arp)) {
      unsigned m[6];
      if (std::sscanf(line, "%63s %*s %*s %63s", aip, hw) == 2 && std::strcmp(aip, hop) == 0 &&
          std::sscanf(hw, "%x:%x:%x:%x:%x:%x", &m[0], &m[1], &m[2], &m[3], &m[4], &m[5]) == 6) {
        for (int i = 0; i < 6; i++) mac[i] = (uint8_t)m[i];
        found = true;
      }
    }
    std::fclose(arp);
    return found ? nullptr : "next hop not in the ARP table";
  }

 private:
  SocketEthBatcher rx_;
  uint32_t local_ip_ = 0;
  uint8_t mac_[6] = {};
};

// ---------------------------------------------------------------------------
// GpuBackend: the per-frame work on the GPU.  The RX ring and the TX batch are pinned
// host memory read in place by the kernels (zero copy: only each frame's own lines
// cross PCIe, GpuRx::Mode::ZeroCopy).
class GpuBackend {
 public:
  static constexpr bool kSnapshot = true; // records are classified against a table snapshot
  static constexpr uint32_t kStride = 2048, kFrameOff = 2;

  GpuBackend() = default;
  GpuBackend(const GpuBackend&) = delete;
  GpuBackend& operator=(const GpuBackend&) = delete;
  ~GpuBackend() {
    drain(); // a pipelined batch may still be reading the ring
    if (tx_stream_) (void)hipStreamDestroy(tx_stream_);
    if (rx_ring_) (void)hipHostFree(rx_ring_);
    if (tx_ring_) (void)hipHostFree(tx_ring_);
    if (tx_word_) (void)hipHostFree(tx_word_);
  }

  // rx_chunk: frames per classify launch (a poll's frames go in chunks, the next one on the
  // GPU while the host dispatches the current one; 0 = one launch per poll).  rx_halves = 2 or 3:
  // that many RX rings of rx_cap slots for launch/collect (one or two in flight while another fills).
  // tx_halves = 2: two TX batches (one filled on the GPU while the other is built).
  // links (with resident): the service returns each post's chain links, passed to f as a fourth argument
  const char* init(int device, uint32_t rx_cap, uint32_t tx_cap, uint32_t rx_chunk = 0, uint32_t rx_halves = 1,
                   uint32_t tx_halves = 1, bool resident = false, bool links = false) {
    drain();
    if (rx_ring_) (void)hipHostFree(rx_ring_);
    if (tx_ring_) (void)hipHostFree(tx_ring_);
    rx_ring_ = tx_ring_ = nullptr;
    const uint32_t chunk = rx_chunk && rx_chunk < rx_cap ? rx_chunk : rx_cap;
    if (const char* e = rx_.init(device, kStride, kFrameOff, chunk, GpuRx::Mode::ZeroCopy, resident, 100, links))
      return e;
    if (pn_set_verify(rx_.ctx(), verify_ ? 1 : 0)) return pn_last_error(rx_.ctx());
    // the TX fill has a stream of its own: pipelined, it runs beside the next batch's classify
    if (!tx_stream_ && hipStreamCreateWithFlags(&tx_stream_, hipStreamNonBlocking) != hipSuccess)
      return "hipStreamCreate(tx) failed";
    rx_cap_ = rx_cap;
    tx_cap_ = tx_cap;
    if (rx_halves < 1 || rx_halves > GpuRx::kBufs) return "rx_halves out of range";
    const size_t rx_bytes = (size_t)kStride * rx_cap * rx_halves;
    const size_t tx_bytes = (size_t)kStride * tx_cap * (tx_halves == 2 ? 2 : 1);
    if (hipHostMalloc((void**)&rx_ring_, rx_bytes, hipHostMallocDefault) != hipSuccess)
      return "hipHostMalloc(rx ring) failed";
    if (hipHostMalloc((void**)&tx_ring_, tx_bytes, hipHostMallocDefault) != hipSuccess)
      return "hipHostMalloc(tx batch) failed";
    if (!tx_word_ && hipHostMalloc((void**)&tx_word_, 64, hipHostMallocDefault) != hipSuccess)
      return "hipHostMalloc(tx notify word) failed";
    *tx_word_ = tx_tok_;
    std::memset(rx_ring_, 0, rx_bytes);
    std::memset(tx_ring_, 0, tx_bytes);
    return nullptr;
  }
  uint8_t* rxSlots(uint32_t half = 0) { return rx_ring_ + (size_t)half * rx_cap_ * kStride; }
  // Whether classify verifies the TCP checksum (pn_set_verify).  Off, the kernel reads only each frame's
  // header lines over PCIe instead of the whole frame: the engine turns it off with its checksum discard.
  const char* setVerify(bool v) {
    verify_ = v;
    if (rx_.ctx() && pn_set_verify(rx_.ctx(), v ? 1 : 0)) return pn_last_error(rx_.ctx());
    return nullptr;
  }
  // Pipelined RX: launch classifies the first n slots of one half against the snapshot on the
  // device (syncTable); collect waits for it and calls f(key, rec, eth, link) in ring order (link: the frame's chain
  // link, 0 without links).
  const char* launch(uint32_t half, uint32_t n, const ConnTable&) { return rx_.submit(rxSlots(half), n, half); }
  // wait for a launched half without dispatching it (collect then dispatches at once)
  const char* ready(uint32_t half) { return rx_.ready(half); }
  template <class F>
  const char* collect(uint32_t half, uint32_t n, const ConnTable& t, F&& f) {
    return rx_.template complete<false>(
        rxSlots(half), n, half, t,
        [&](uint64_t key, const pn_result& r, const uint8_t* eth, uint32_t, uint16_t link) { f(key, r, eth, link); },
        [&](uint64_t key, uint32_t, const uint8_t* eth, const pn_result& r) { f(key, r, eth, (uint16_t)0); });
  }
  uint8_t* txSlots(uint32_t half = 0) { return tx_ring_ + (size_t)half * tx_cap_ * kStride; }
  const char* syncTable(const ConnTable& t) { return rx_.syncTable(t); }
  // f(key, rec, eth, link) for the n frames of the RX ring, in ring order.
  template <class F>
  const char* classify(uint32_t n, const ConnTable& t, F&& f) {
    return rx_.template pollBatch<false>(
        rx_ring_, n, t,
        [&](uint64_t key, const pn_result& r, const uint8_t* eth, uint32_t, uint16_t link) { f(key, r, eth, link); },
        [&](uint64_t key, uint32_t, const uint8_t* eth, const pn_result& r) { f(key, r, eth, (uint16_t)0); });
  }
  // IP + TCP checksums of the first n slots of a TX batch (PN_TX_TCP: SendBuf::setOptDataLen,
  // Core.h:157-163).  fillTx waits for them; fillTxLaunch / fillTxWait split the same call
  // (pipelined: the fill runs while the host dispatches the next batch).
  const char* fillTx(uint32_t n, uint32_t half = 0) {
    if (const char* e = fillTxLaunch(n, half)) return e;
    return fillTxWait();
  }
  // Batches of up to PN_NOTIFY_MAX_FRAMES (a poll's ACKs) complete through a pinned word
  // (pn_tx_fill_notify): the host sees the fill done ≈4 us before a stream sync would return.
  const char* fillTxLaunch(uint32_t n, uint32_t half) {
    tx_word_used_ = n <= PN_NOTIFY_MAX_FRAMES;
    if (tx_word_used_) {
      if (pn_tx_fill_notify(rx_.ctx(), txSlots(half), kStride, kFrameOff, n, nullptr, PN_TX_TCP, tx_stream_, tx_word_,
                            ++tx_tok_))
        return pn_last_error(rx_.ctx());
      return nullptr;
    }
    if (pn_tx_fill(rx_.ctx(), txSlots(half), kStride, kFrameOff, n, nullptr, PN_TX_TCP, tx_stream_))
      return pn_last_error(rx_.ctx());
    return nullptr;
  }
  const char* fillTxWait() {
    if (tx_word_used_ && wait_word(tx_word_, tx_tok_, tx_stream_) == nullptr) return nullptr;
    if (hipStreamSynchronize(tx_stream_) != hipSuccess) return "hipStreamSynchronize(tx_fill) failed";
    return tx_word_used_ ? "tx_fill notify word not written" : nullptr;
  }

 private:
  // Wait for every launch that may read the rings (before they are freed).
  void drain() {
    if (rx_.stream()) (void)hipStreamSynchronize(rx_.stream());
    if (tx_stream_) (void)hipStreamSynchronize(tx_stream_);
  }

  GpuRx rx_;
  bool verify_ = true;
  hipStream_t tx_stream_ = nullptr;
  uint8_t* rx_ring_ = nullptr;
  uint8_t* tx_ring_ = nullptr;
  uint32_t* tx_word_ = nullptr; // pinned notify word of the TX fill
  uint32_t tx_tok_ = 0;
  bool tx_word_used_ = false;   // the fill in flight completes through tx_word_
  uint32_t rx_cap_ = 0, tx_cap_ = 0;
};


// ---------------------------------------------------------------------------
// TcpEngine<Conf, IConf, Link, Backend, Derived>: connections, timers, segments, frames.
//   IConf   MaxConnCnt / MaxTimeWaitConnCnt / ConnRecvBufSize / TimestampOption (the efvitcp
//           Conf the pollnet wrapper derives, EfviTcp.h:21-36, 180-199)
//   Derived (CRTP) supplies the endpoint's branches:
//     static constexpr bool kClient;
//     bool accepts(const uint8_t* eth)                                   the NIC filter
//     template <class HH> void onMiss(HH&, uint64_t key, const pn_result&, const uint8_t* eth)
//     template <class HH> bool onHandshake(HH&, Conn&, const pn_result&, const uint8_t* eth)
//                                   (an unestablished connection's segment; true: go on to onPack)
template <class Conf, class IConfT, class Link, class Backend, class Derived>
class TcpEngine {
 public:
  using IConf = IConfT;
  static constexpr uint32_t kMaxConn = IConf::MaxConnCnt;
  static constexpr uint32_t kMaxTw = IConf::MaxTimeWaitConnCnt;
  static constexpr uint32_t kSendBufCnt = srv_detail::opt_ConnSendBufCnt<Conf>::value;
  static constexpr uint32_t kSendMTU = 1024 - 28;      // SendBuf1K: SendBufSize - offsetof(ip_hdr), Core.h:232-234
  static constexpr uint32_t kSegCap = kSendMTU - 40;   // largest SMSS (onSyn's clamp, TcpConn.h:357)
  static constexpr uint32_t kSynRetries = 3, kTcpRetries = 10, kMinRtoMS = 100, kMaxRtoMS = 30 * 1000;
  static constexpr uint32_t kDelayedAckMS = srv_detail::opt_DelayedAckMS<Conf>::value;
  static constexpr uint32_t kTimeWaitTimeout = 60 * 1000; // Core.h:48
  static constexpr uint32_t kRxBatch = srv_detail::opt_RxBatch<Conf>::value;
  static constexpr uint32_t kTxBatch = srv_detail::opt_TxBatch<Conf>::value;
  static constexpr uint32_t kTxGpuMin = srv_detail::opt_TxGpuMinDataFrames<Conf>::value;
  static constexpr uint32_t kRxBudgetUs = srv_detail::opt_RxLatencyBudgetUs<Conf>::value;
  static constexpr uint32_t kRxChunk = srv_detail::opt_RxChunk<Conf>::value;
  static constexpr bool kRxPipeline = srv_detail::opt_RxPipeline<Conf>::value;
  static_assert(!(kRxPipeline && kRxChunk), "RxPipeline and RxChunk are alternatives");
  static constexpr uint32_t kRxDepth = kRxPipeline ? srv_detail::opt_RxPipelineDepth<Conf>::value : 0;
  static_assert(!kRxPipeline || kRxDepth == 1 || kRxDepth == 2, "RxPipelineDepth is 1 or 2");
  static constexpr uint32_t kRxBufs = kRxDepth + 1; // RX rings: the one filling, the batches in flight
  static constexpr uint32_t kSendTimeoutMs = srv_detail::opt_SendTimeoutSec<Conf>::value * 1000;
  static constexpr uint32_t kRecvTimeoutMs = srv_detail::opt_RecvTimeoutSec<Conf>::value * 1000;
  static_assert(kSendBufCnt >= 4 && !(kSendBufCnt & (kSendBufCnt - 1)), "ConnSendBufCnt must be a power of 2");
  static_assert(Conf::RecvBufSize >= 2 * 1460, "RecvBufSize below two RMSS");

  class Conn : public srv_detail::user_data<Conf>::type {
   public:
    const char* err_ = nullptr; // EfviTcp.h:54 / 197 (UserData::err_)

    uint32_t getConnId() const { return id_; }
    void getPeername(sockaddr_in& addr) const { // TcpConn.h:37-41
      addr.sin_addr.s_addr = peer_ip_;
      addr.sin_port = peer_port_;
    }
    bool isEstablished() const { return established_; }
    bool isConnected() const { return established_; }
    bool isClosed() const { return fin_received_ && !established_; } // TcpConn.h:45
    const char* getLastError() const { return err_; }
    void close(const char* reason) { // EfviTcp.h:61-64, 230-233
      err_ = reason;
      eng_->closeConn(*this);
    }
    // EfviTcpClient::Conn::writeSome (EfviTcp.h:66-70): send, and re-arm the send timeout.
    int writeSome(const void* data, uint32_t size, bool more = false) {
      const int ret = (int)send(data, size, more);
      if (kSendTimeoutMs) setUserTimer(0, kSendTimeoutMs);
      return ret;
    }
    // All or nothing, else the connection is closed: EfviTcp.h:73-79 (client: through
    // writeSome, the timer re-armed either way) and 236-244 (server: re-armed on success).
    bool writeNonblock(const void* data, uint32_t size, bool more = false) {
      if constexpr (Derived::kClient) {
        if ((uint32_t)writeSome(data, size, more) != size) {
          close("send buffer full");
          return false;
        }
      } else {
        if (send(data, size, more) != size) {
          close("send buffer full");
          return false;
        }
        if (kSendTimeoutMs) setUserTimer(0, kSendTimeoutMs);
      }
      return true;
    }
    // TcpConn::send (TcpConn.h:58-61): bytes accepted into the send buffer.
    uint32_t send(const void* data, uint32_t size, bool more = false) {
      if (fin_sent_) return 0;
      return eng_->sendPartial(*this, (const uint8_t*)data, size, !more);
    }
    uint32_t getSendable() const { // TcpConn.h:47-50
      if (fin_sent_) return 0;
      return (send_una_ + kSendBufCnt - 1 - data_next_) * smss_ - data_next_size_;
    }
    // TcpConn::getImmediatelySendable (TcpConn.h:52-56): what fits the peer's window now.  pollnet's wrappers
    // run without a congestion window (CongestionControlAlgo = 0, EfviTcp.h:48, 206), so both_wnd_seq is the
    // peer's window edge (TcpConn.h:189-192).
    uint32_t getImmediatelySendable() const {
      if (data_next_ != send_next_) return 0;
      const int32_t wnd = (int32_t)(send_wnd_seq_ - next_seq_ - data_next_size_);
      return std::min((uint32_t)std::max(0, wnd), getSendable());
    }
    // TcpConn::sendv (TcpConn.h:63-70): the pieces appended in order, the last one pushed.
    uint32_t sendv(const iovec* iov, int iovcnt) {
      if (fin_sent_) return 0;
      uint32_t total = 0;
      for (int i = 0; i < iovcnt; i++)
        total += eng_->sendPartial(*this, (const uint8_t*)iov[i].iov_base, (uint32_t)iov[i].iov_len, i + 1 == iovcnt);
      return total;
    }
    void sendFin() { eng_->sendFin(*this); }
    void setUserTimer(uint32_t timer_id, uint32_t duration_ms) { eng_->setUserTimer(*this, timer_id, duration_ms); }
#ifdef EFVITCP_DEBUG
    // TcpConn::dump / shortDump (TcpConn.h:107-128, debug builds): the reference's fields in the reference's
    // order.  cwnd, ssthresh and cong_av print 0: with pollnet's wrappers (CongestionControlAlgo = 0,
    // EfviTcp.h:48, 206) the reference never writes them (TcpConn.h:418-421, 583-664, 788-791, 816-824), so
    // its zero-initialised server prints 0.  ack_seq / ack_end_seq are recv_buf_seq plus the first / last
    // reassembly extent's end (TcpConn.h:115-116), from the receive half.
    void dump(const char* note) const {
      const uint32_t cwnd = 0, ssthresh = 0, cong_av = 0;
      const uint32_t ack_seq = rx_.recvBufSeq() + rx_.segs()[0].second;
      const uint32_t ack_end_seq = rx_.recvBufSeq() + rx_.segs()[rx_.segCount() ? rx_.segCount() - 1 : 0].second;
      std::printf("%s: conn_id: %u, key: %llu, established: %d, fin_sent: %d, fin_received: %d, cwnd: %u, "
                  "ssthresh: %u, cong_av: %u, fast_re: %d, dup_ack_cnt: %u, send_una: %u, send_next: %u, "
                  "data_next: %u, data_next_size: %u, ack_seq: %u, ack_end_seq: %u, send_next_seq: %u, "
                  "both_wnd_seq: %u, rto: %u, srtt: %u, rttvar: %u, recent_ts: %u, in_recover: %d, recover: %u, "
                  "retries: %u, src port: %u, dst port: %u\n",
                  note, id_, (unsigned long long)key_, established_, fin_sent_, fin_received_, cwnd, ssthresh, cong_av,
                  fast_re_, dup_ack_cnt_, send_una_, send_next_, data_next_, data_next_size_, ack_seq, ack_end_seq,
                  segs_[send_next_ & (kSendBufCnt - 1)].seq, send_wnd_seq_, rto_, srtt_, rttvar_, rx_.recentTs(),
                  in_recover_, recover_, retries_, ntohs(local_port_), ntohs(peer_port_));
    }
    void shortDump(const char* note = "") const {
      std::printf("%s, src port: %u, dst port: %u\n", note, ntohs(local_port_), ntohs(peer_port_));
    }
#endif

   private:
    friend class TcpEngine;
    friend Derived;
    struct Seg {
      uint32_t seq = 0;
      uint32_t send_ts = 0;
      uint16_t len = 0; // payload bytes
      bool fin = false;
      bool syn_ack = false; // the SYN segment carried ACK (a server's SYN-ACK)
    };
    Seg& seg(uint32_t idx) { return segs_[idx & (kSendBufCnt - 1)]; }
    uint8_t* segData(uint32_t idx) { return data_.get() + (size_t)(idx & (kSendBufCnt - 1)) * kSegCap; }

    TcpEngine* eng_ = nullptr;
    uint32_t id_ = 0;
    uint64_t key_ = 0;
    // every frame of this connection starts from these 54 bytes (Ethernet, IPv4 and TCP headers with the
    // connection's addresses and ports, the rest zero), as the reference's SendBufs are pre-filled (Core.h:291-301);
    // hdr_ip_sum_ / hdr_tcp_sum_: their fixed words summed (TcpEngine::connHeader)
    alignas(64) uint8_t hdr_[64] = {};
    uint32_t hdr_ip_sum_ = 0, hdr_tcp_sum_ = 0;
    uint32_t peer_ip_ = 0;     // network order
    uint16_t peer_port_ = 0;   // network order
    uint16_t local_port_ = 0;  // network order
    uint8_t peer_mac_[6] = {};
    // send side (TcpConn.h:861-898)
    std::unique_ptr<Seg[]> segs_;
    std::unique_ptr<uint8_t[]> data_;
    uint32_t send_una_ = 0, send_next_ = 0, data_next_ = 0, data_next_size_ = 0, recover_ = 0;
    uint32_t next_seq_ = 0; // seg(send_next_).seq, kept here so that an ACK reads no segment entry
    uint64_t ack_frame_ = ~0ull; // frame_idx_ of the last frame whose ACK field this connection processed (inOrder)
    uint32_t ack_in_ = 0;        // that frame's ack number
    uint32_t smss_ = 536, send_wnd_seq_ = 0, rto_ = 1000, srtt_ = 0, rttvar_ = 0, dup_ack_cnt_ = 0, retries_ = 0;
    bool established_ = false, fin_sent_ = true, fin_received_ = true, fast_re_ = false, in_recover_ = false;
    TimerNode timers_[4]; // resend, delayed ACK, user 0 (send timeout), user 1 (recv timeout)
    // last: the receive half's state leads its 64-KiB buffer, so everything a segment touches on the common path
    // (the fields above and the receive state) sits in the connection's first few cache lines
    RxConn<IConf> rx_;
  };

  TcpEngine() : conns_(kMaxConn), tws_(kMaxTw) {}
  TcpEngine(const TcpEngine&) = delete;
  TcpEngine& operator=(const TcpEngine&) = delete;

  Link& link() { return link_; }
  Backend& backend() { return be_; } // measurement: the per-frame legs timed on their own
  // Records re-resolved on the host because the table changed after their snapshot.
  uint64_t reResolved() const { return re_resolved_; }
  // Frames that took the in-order fast path on their chain link (RxLinks).
  uint64_t inOrderFrames() const { return in_order_; }
  // Drop checksum-failed frames before they touch any state (what the NIC's RX checksum
  // offload does for efvitcp: ef_vi delivers them as RX_DISCARD).  Default on.  Off, the frames
  // are trusted as the reference's release build trusts them (Core::checksum is debug-only,
  // Core.h:448-478), and the GPU backend also stops verifying the TCP checksum: its classify
  // reads only each frame's header lines (pn_set_verify), so the records a hook sees carry no
  // TCP verdict (PN_F_TCP_UNCHECKED set, PN_F_TCP_OK / PN_F_RFC_TCP_OK clear, tcp_fold 0xFFFF).
  // To keep the verdict in the records with the discard off, call setVerify(true) after this.
  // Returns the backend's error (pn_set_verify), nullptr on success.
  const char* setDropBadChecksum(bool drop) {
    drop_bad_ = drop;
    return be_.setVerify(drop);
  }
  // Whether the backend computes the TCP verdict (pn_set_verify), on its own.  The discard needs it:
  // setVerify(false) while setDropBadChecksum(true) is in force is refused.
  const char* setVerify(bool verify) {
    if (!verify && drop_bad_) return "setVerify(false): the checksum discard (setDropBadChecksum(true)) needs the TCP verdict";
    return be_.setVerify(verify);
  }
  const ConnTable& table() const { return table_; }
  uint32_t nowTs() const { return wheel_.now(); }
  // Frames built since the last flush (checksums not yet filled), plus (pipelined) those whose
  // fill is still running.
  uint32_t pendingTx() const { return tx_n_ + tx_fl_n_; }
  // Fill the pending frames' checksums and send them in order; a pipelined batch still being
  // filled goes first.  A batch of at least TxGpuMinDataFrames payload-bearing frames takes one
  // pn_tx_fill launch; a smaller one (a poll's ACKs, the odd data segment) is summed on the host,
  // where a header-only frame costs nanoseconds and a launch ~10 us.
  const char* flushTx() {
    const char* e = completeTx();
    if (!tx_n_) return e;
    if (txOnHost()) {
      fillTxHost(tx_cur_, tx_n_);
    } else if (const char* e2 = be_.fillTx(tx_n_, tx_cur_)) {
      err_ = e2;
      tx_n_ = tx_data_n_ = 0;
      tx_fill_[tx_cur_].clear();
      return e2;
    } else {
      tx_gpu_frames_ += tx_n_;
      tx_fill_[tx_cur_].clear(); // pn_tx_fill writes every frame's checksums
    }
    sendTx(tx_cur_, tx_n_);
    tx_n_ = tx_data_n_ = 0;
    return e;
  }
  // TX frames summed on the host / filled by pn_tx_fill since init (measurement)
  uint64_t txHostFrames() const { return tx_host_frames_; }
  uint64_t txGpuFrames() const { return tx_gpu_frames_; }

 protected:
  struct Tw { // Core.h:186-197 TimeWaitConn
    uint64_t key = 0;
    uint8_t peer_mac[6] = {};
    uint32_t peer_ip = 0;
    uint16_t peer_port = 0, local_port = 0;
    uint32_t seq_num = 0, ack_num = 0;
    TimerNode timer;
  };

  // The pollnet wrapper's TmpHandler (EfviTcp.h:107-147 client, 264-307 server): the reference's
  // event callbacks mapped onto the user's handler; callbacks it does not define are skipped.
  template <class Handler>
  struct H {
    Handler& u;
    void connected(Conn& c) {
      if constexpr (srv_detail::has_onTcpConnected<Handler, Conn>::value) u.onTcpConnected(c);
    }
    void disconnect(Conn& c) {
      if constexpr (srv_detail::has_onTcpDisconnect<Handler, Conn>::value) u.onTcpDisconnect(c);
    }
    void connectFailed() {
      if constexpr (srv_detail::has_onTcpConnectFailed<Handler, Conn>::value) u.onTcpConnectFailed();
    }
    void sendTimeout(Conn& c) {
      if constexpr (srv_detail::has_onSendTimeout<Handler, Conn>::value) u.onSendTimeout(c);
    }
    void recvTimeout(Conn& c) {
      if constexpr (srv_detail::has_onRecvTimeout<Handler, Conn>::value) u.onRecvTimeout(c);
    }
    bool allow(uint32_t ip_be, uint16_t port_be) {
      if constexpr (srv_detail::opt_UseAllowNewConnection<Conf>::value &&
                    srv_detail::has_allowNewConnection<Handler, Conn>::value)
        return u.allowNewConnection(ip_be, port_be);
      return true; // EfviTcp.h:270: the wrapper's TmpHandler accepts every connection
    }
    uint32_t data(Conn& c, const uint8_t* d, uint32_t n) { return u.onTcpData(c, d, n); }
  };

  Derived& self() { return static_cast<Derived&>(*this); }

  static int64_t getns() {
    timespec ts;
    ::clock_gettime(CLOCK_REALTIME, &ts);
    return (int64_t)ts.tv_sec * 1000000000 + ts.tv_nsec;
  }

  // Core::init's state (Core.h:253-330): local address, table, id stacks, timer wheel, buffers.
  const char* initEngine(const char* local_ip, int64_t now_ns) {
    closeAll();
    ready_ = false;
    local_ip_ = link_.localIp();
    if (local_ip && std::strcmp(local_ip, "0.0.0.0") != 0) {
      in_addr a;
      if (inet_pton(AF_INET, local_ip, &a) != 1) return "invalid local ip";
      local_ip_ = a.s_addr;
    }
    std::memcpy(local_mac_, link_.localMac(), 6);
    if (const char* e = table_.init(kMaxConn, kMaxTw, srv_detail::opt_ReferenceLiteralTable<Conf>::value)) return e;
    if (const char* e = be_.init(srv_detail::opt_Device<Conf>::value, kRxBatch, kTxBatch, kRxChunk, kRxBufs,
                                 kRxPipeline ? 2 : 1, srv_detail::opt_RxResident<Conf>::value,
                                 srv_detail::opt_RxResident<Conf>::value && srv_detail::opt_RxLinks<Conf>::value))
      return e;
    tx_base_[0] = be_.txSlots(0) + Backend::kFrameOff; // each TX batch's first frame
    tx_base_[1] = kRxPipeline ? be_.txSlots(1) + Backend::kFrameOff : tx_base_[0];
    free_conns_.clear();
    for (uint32_t i = kMaxConn; i-- > 0;) free_conns_.push_back(i); // Core.h:315: conns[i] = i
    free_tws_.clear();
    for (uint32_t i = kMaxTw; i-- > 0;) free_tws_.push_back(i);
    conn_cnt_ = tw_cnt_ = 0;
    for (auto& c : conns_) // unlink before the wheel's heads are reset
      for (auto& t : c.timers_) t.unlink();
    for (auto& tw : tws_) tw.timer.unlink();
    wheel_.reset((uint32_t)(now_ns >> 20));
    for (uint32_t i = 0; i < kMaxConn; i++) {
      Conn& c = conns_[i];
      c.eng_ = this;
      c.id_ = i;
      if (!c.segs_) {
        c.segs_.reset(new typename Conn::Seg[kSendBufCnt]);
        c.data_.reset(new uint8_t[(size_t)kSendBufCnt * kSegCap]);
      }
      for (uint32_t k = 0; k < 4; k++) {
        c.timers_[k].owner = i;
        c.timers_[k].kind = k;
      }
      c.established_ = false;
      c.fin_sent_ = c.fin_received_ = true;
    }
    for (uint32_t i = 0; i < kMaxTw; i++) tws_[i].timer.owner = kMaxConn + i;
    tx_n_ = tx_data_n_ = rx_pending_ = cur_ = tx_cur_ = tx_fl_n_ = 0;
    for (auto& v : tx_fill_) {
      v.clear();
      v.reserve(kTxBatch);
    }
    for (auto& f : fl_n_) f = 0;
    fl_head_ = fl_cnt_ = 0;
    ++tver_;
    ready_ = true;
    return nullptr;
  }

  void closeAll() { // TcpServer::close / TcpClient::close: close() every connection (RST if established)
    if (!ready_) return;
    for (auto& c : conns_)
      if (c.eng_ && !c.isClosed()) closeConn(c);
    flushTx();
  }

  // The link gets frames [0, n) of a TX batch, in order.
  void sendTx(uint32_t half, uint32_t n) {
    for (uint32_t i = 0; i < n; i++) {
      const uint8_t* f = tx_base_[half] + (size_t)i * Backend::kStride;
      link_.send(f, 14 + srv_detail::rd16(f + 16));
    }
  }
  bool txOnHost() const { return tx_data_n_ < kTxGpuMin; }
  void fillTxHost(uint32_t half, uint32_t n) { // the frames header() left unsummed (header-only ones are done)
    for (const uint32_t i : tx_fill_[half])
      srv_detail::fill_tcp_checksums(tx_base_[half] + (size_t)i * Backend::kStride);
    tx_fill_[half].clear();
    tx_host_frames_ += n;
  }
  // Pipelined TX: start filling the frames built so far and switch to the other batch ...
  void launchTx() {
    if (!tx_n_) return;
    tx_fl_host_ = txOnHost();
    if (tx_fl_host_) {
      fillTxHost(tx_cur_, tx_n_);
    } else if (const char* e = be_.fillTxLaunch(tx_n_, tx_cur_)) {
      err_ = e;
      tx_n_ = tx_data_n_ = 0;
      tx_fill_[tx_cur_].clear();
      return;
    } else {
      tx_gpu_frames_ += tx_n_;
      tx_fill_[tx_cur_].clear(); // pn_tx_fill writes every frame's checksums
    }
    tx_fl_n_ = tx_n_;
    tx_n_ = tx_data_n_ = 0;
    tx_cur_ ^= 1;
  }
  // ... and, a poll later, wait for that fill and send its frames.
  const char* completeTx() {
    if (!tx_fl_n_) return nullptr;
    const uint32_t n = tx_fl_n_;
    tx_fl_n_ = 0;
    if (!tx_fl_host_)
      if (const char* e = be_.fillTxWait()) return err_ = e;
    sendTx(tx_cur_ ^ 1, n);
    return nullptr;
  }

  // One poll: a timer tick, the RX batch (classified on the GPU, dispatched in ring order),
  // the TX batch (checksums on the GPU).  With a latency budget the frames of several polls
  // accumulate in the ring (timers and TX still run every poll) until the ring is full or
  // the oldest has waited the budget: one launch per budget instead of one per poll.
  template <class HH>
  void pollEngine(HH& h, int64_t now) {
    wheel_.tick((uint32_t)(now >> 20), [&](TimerNode* n) { onTimer(h, n); }); // Core::pollTime
    const uint32_t got = link_.fill(be_.rxSlots(cur_) + (size_t)rx_pending_ * Backend::kStride, Backend::kStride,
                                    Backend::kFrameOff, kRxBatch - rx_pending_);
    if (got && rx_pending_ == 0) rx_first_ns_ = now;
    rx_pending_ += got;
    const bool due = rx_pending_ == kRxBatch || now - rx_first_ns_ >= (int64_t)kRxBudgetUs * 1000;
    const uint32_t n = due ? rx_pending_ : 0;
    if (n) {
      rx_pending_ = 0;
      if (Backend::kSnapshot && tver_ != synced_ver_) {
        if ((err_ = be_.syncTable(table_))) return;
        synced_ver_ = tver_;
      }
    }
    auto frame = [&](uint64_t key, const pn_result& r, const uint8_t* eth, uint16_t link = 0) {
      onFrame(h, key, r, eth, link);
    };
    if constexpr (kRxPipeline) {
      // launch this poll's frames; send what the previous poll built (its checksum fill ran
      // meanwhile); dispatch the oldest batch in flight -- launched kRxDepth polls ago, or any
      // when no frames came -- while the newer ones are classified; start the fill of what this
      // poll built.  At depth 2 the oldest batch is waited for before the launch: a resident
      // service takes a post only with at most one other outstanding.
      if (n) {
        if (kRxDepth == 2 && fl_cnt_ == 2)
          if ((err_ = be_.ready(fl_head_))) return;
        if ((err_ = be_.launch(cur_, n, table_))) return;
        fl_n_[cur_] = n;
        fl_ver_[cur_] = tver_;
        ++fl_cnt_;
      }
      completeTx();
      if (fl_cnt_ > (n ? kRxDepth : 0)) {
        const uint32_t old = fl_head_, m = fl_n_[old];
        fl_n_[old] = 0;
        fl_head_ = old + 1 == kRxBufs ? 0 : old + 1;
        --fl_cnt_;
        disp_ver_ = fl_ver_[old];
        if (const char* e = be_.ready(old)) err_ = e;
        else if (const char* e2 = be_.collect(old, m, table_, frame)) err_ = e2;
      }
      cur_ = fl_head_ + fl_cnt_;
      if (cur_ >= kRxBufs) cur_ -= kRxBufs;
      launchTx();
    } else {
      if (n) {
        disp_ver_ = tver_;
        if (const char* e = be_.classify(n, table_, frame)) err_ = e;
      }
      flushTx();
    }
  }

  // ---- one received frame (Core::pollNet RX branch + the endpoint's recv handler) ----
  // key: the frame's connHashKey, which the backends pass for TIME_WAIT records and misses only (a hit's connection
  // is its conn_id; the key is derived from the frame here where a hit needs it)
  // link: the frame's chain link (pn_service_post_linked), 0 = none
  template <class HH>
  PN_HOT void onFrame(HH& h, uint64_t key, const pn_result& rec, const uint8_t* eth, uint16_t link = 0) {
    ++frame_idx_;
    if (link && inOrder(h, rec, eth, link)) return;
    if (rec.flags & (PN_F_NOT_TCP | PN_F_TRUNC | PN_F_BADOFF)) return;
    if (!self().accepts(eth)) return; // the NIC filter (Core.h:335-383)
    if (drop_bad_ && !checksums_ok(rec.flags)) return;
    pn_result r = rec;
    // the record came from a table snapshot that has changed since (earlier in this batch, or,
    // pipelined, after the launch): probe the live table
    if ((Backend::kSnapshot || kRxPipeline) && tver_ != disp_ver_) {
      ++re_resolved_;
      key = frame_key(eth);
      uint32_t conn_id = PN_MISS;
      const bool hit = table_.find(key, nullptr, &conn_id);
      r.conn_id = conn_id;
      r.flags = (uint16_t)((r.flags & ~(PN_F_HIT | PN_F_TW)) | (hit ? PN_F_HIT : 0) |
                           (hit && conn_id >= kMaxConn ? PN_F_TW : 0));
    }
    if (r.flags & PN_F_TW) { // Core.h:510-524
      Tw& tw = tws_[r.conn_id - kMaxConn];
      const bool seq_expected = seqRaw(r) == tw.ack_num;
      if (r.flags & PN_F_RST) {
        if (seq_expected) {
          tw.timer.unlink();
          delEntry(key);
        }
      } else if (!seq_expected || segLen(eth, r)) {
        ackTW(tw);
      }
      return;
    }
    if (!(r.flags & PN_F_HIT)) {
      self().onMiss(h, key, r, eth);
      return;
    }
    Conn& c = conns_[r.conn_id];
    if (!c.established_ && !self().onHandshake(h, c, r, eth)) return;
    onPack(h, c, eth, r);
  }

  static uint32_t seqRaw(const pn_result& r) { return r.seq - ((r.flags & PN_F_SYN) ? 1u : 0u); } // rec.seq = seq + syn
  static uint32_t ackNum(const uint8_t* eth) { return srv_detail::rd32(eth + 34 + 8); }
  static uint32_t segLen(const uint8_t* eth, const pn_result& r) { // tot_len - 20 - doff*4 + syn + fin
    const uint32_t tot = srv_detail::rd16(eth + 16), doff = eth[34 + 12] >> 4;
    return tot - 20 - doff * 4 + ((r.flags & PN_F_SYN) ? 1 : 0) + ((r.flags & PN_F_FIN) ? 1 : 0);
  }

  // ---- connection setup (TcpConn::reset / onSyn / sendSyn / onEstablished) ----
  // Take a connection id and a table entry for key (TcpServer.h:88-89, TcpClient.h:67-69).
  Conn* newConn(uint64_t key) {
    if (free_conns_.empty()) return nullptr;
    const uint32_t id = free_conns_.back();
    free_conns_.pop_back();
    ++conn_cnt_;
    table_.add(key, id);
    ++tver_;
    return &conns_[id];
  }
  void resetConn(Conn& c, uint64_t key, const uint8_t* peer_mac, uint32_t peer_ip, uint16_t peer_port,
                 uint16_t local_port) { // TcpConn.h:150-186
    c.key_ = key;
    std::memcpy(c.peer_mac_, peer_mac, 6);
    c.peer_ip_ = peer_ip;
    c.peer_port_ = peer_port;
    c.local_port_ = local_port;
    // err_ is left as the slot's last connection left it: TcpConn::reset does not touch UserData
    // (EfviTcp.h:208-211), so a server's new connection reports the previous one's error until
    // its own (the client's is set by connect's result, EfviTcp.h:122)
    c.established_ = c.fin_sent_ = c.fin_received_ = c.fast_re_ = c.in_recover_ = false;
    c.ack_frame_ = ~0ull;
    c.send_una_ = c.send_next_ = c.data_next_size_ = c.dup_ack_cnt_ = c.retries_ = 0;
    c.data_next_ = 1;
    c.smss_ = 536;
    c.rx_.resetRecv();
    // genISN (TcpConn.h:856-858): connHashKey(peer) + now_ts; keeps send window 0 until established
    c.send_wnd_seq_ = (uint32_t)key + wheel_.now();
    c.seg(0).seq = c.next_seq_ = c.send_wnd_seq_;
    buildConnHeader(c);
  }
  // The connection's frame template and its fixed words' sums (native-order 16-bit words, as header_sums).
  void buildConnHeader(Conn& c) {
    using namespace srv_detail;
    uint8_t* f = c.hdr_;
    std::memset(f, 0, sizeof c.hdr_);
    std::memcpy(f, c.peer_mac_, 6);
    std::memcpy(f + 6, local_mac_, 6);
    f[12] = 0x08;
    uint8_t* ip = f + 14;
    ip[0] = 0x45;
    wr16(ip + 6, 0x4000);
    ip[8] = 64;
    ip[9] = 6;
    std::memcpy(ip + 12, &local_ip_, 4);
    std::memcpy(ip + 16, &c.peer_ip_, 4);
    std::memcpy(ip + 20, &c.local_port_, 2);
    std::memcpy(ip + 22, &c.peer_port_, 2);
    auto halves = [](uint32_t x) { return (x & 0xffffu) + (x >> 16); };
    const uint32_t addr = halves(local_ip_) + halves(c.peer_ip_);
    c.hdr_ip_sum_ = 0x0045u + 0x0040u + 0x0640u + addr;
    c.hdr_tcp_sum_ = addr + 0x0600u + c.local_port_ + c.peer_port_;
  }
  void onSyn(Conn& c, const uint8_t* eth, const pn_result& r) { // TcpConn.h:339-375
    const uint8_t* opt = eth + 54;
    const uint8_t* data = eth + 34 + (eth[46] >> 4) * 4;
    while (opt < data) {
      const uint8_t kind = *opt++;
      if (kind <= 1) continue;
      const uint8_t len = *opt++;
      if (kind == 2 && len == 4) c.smss_ = std::min<uint32_t>(kSendMTU - 40, srv_detail::rd16(opt));
      if (len > 2) opt += len - 2;
    }
    c.rx_.open(seqRaw(r));
    c.fin_received_ = false;
  }
  void sendSyn(Conn& c) { // TcpConn.h:197-230: SYN, with ACK when a SYN was received (pending_ack)
    c.rto_ = 1000;
    typename Conn::Seg& s = c.seg(c.send_next_);
    s.len = 0;
    s.fin = false;
    s.syn_ack = c.rx_.pendingAck();
    emit(c, s.seq, s.syn_ack ? kSynAck : kSyn, nullptr, 0);
    advanceNext(c, 1);
  }
  template <class HH>
  void onEstablished(HH& h, Conn& c, const uint8_t* eth) { // TcpConn.h:377-418
    c.send_wnd_seq_ = ackNum(eth) + srv_detail::rd16(eth + 34 + 14);
    c.established_ = true;
    c.srtt_ = std::max(1u, wheel_.now() - c.seg(c.send_una_).send_ts);
    c.rttvar_ = c.srtt_ >> 1;
    updateRto(c);
    // onConnectionEstablished (EfviTcp.h:131-135, 296-300)
    if (kSendTimeoutMs) setUserTimer(c, 0, kSendTimeoutMs);
    if (kRecvTimeoutMs) setUserTimer(c, 1, kRecvTimeoutMs);
    h.connected(c);
  }
  void updateRto(Conn& c) { c.rto_ = std::max(kMinRtoMS, c.srtt_ + std::max(1u, c.rttvar_ << 2)); }

  // ---- segment processing of a connection (TcpConn::onPack) ----
  template <class HH>
  struct PackAdapter {
    TcpEngine& s;
    HH& h;
    Conn& c;
    const uint8_t* eth;
    PN_HOT uint32_t onData(RxConn<IConf>&, const uint8_t* d, uint32_t n) { // EfviTcp.h:136-139, 301-304
      if (kRecvTimeoutMs) s.setUserTimer(c, 1, kRecvTimeoutMs);
      return h.data(c, d, n);
    }
    void onFin(RxConn<IConf>&, const uint8_t* d, uint32_t n) { // EfviTcp.h:121-125, 283-288
      c.fin_received_ = true;
      if (n) h.data(c, d, n);
      c.err_ = "remote close";
      s.closeConn(c); // RST (the wrapper's Conn::close -> TcpConn::close)
      h.disconnect(c);
    }
    void onReset(RxConn<IConf>&) { // onConnectionReset (EfviTcp.h:111-114, 269-272)
      c.err_ = "connection reset";
      h.disconnect(c);
    }
    PN_HOT void onAckField(RxConn<IConf>&, bool no_text) {
      c.ack_frame_ = s.frame_idx_; // the in-order fast path's proof that this frame's ack field was applied
      s.onAck(c, eth, no_text);
    }
  };

  template <class HH>
  PN_HOT void onPack(HH& h, Conn& c, const uint8_t* eth, const pn_result& r) {
    PackAdapter<HH> a{*this, h, c, eth};
    afterSegment(h, c, c.rx_.onSegment(a, eth, r));
  }

  // The in-order fast path (round 6).  The GPU's chain link says this frame continues frame
  // j = frame_idx_ - link, the previous frame of the same connection in the batch, exactly: clean flags, payload,
  // seq = j's seq + payload_len, and the same payload offset, ack number, window and destination.  When j's ACK field
  // was processed (ack_frame_: so j also passed the NIC filter and the checksum discard), the record is the
  // snapshot's and the table unchanged, and the connection is still where an in-order segment leaves it --
  // established, no FIN either way, nothing held or out of order -- and the same ack field changes nothing
  // (TcpConn.h:536-665: the window no wider than j's made it, una not advanced by j's ack number, nothing queued
  // that the window admits; what j's own handler sent since is checked here, not assumed), then TcpConn::onPack's
  // remaining steps are exactly: the payload to onData zero-copy, the window slide, the ACK decision
  // (TcpConn.h:700-764).  Anything else takes the full path (false).
  template <class HH>
  PN_HOT bool inOrder(HH& h, const pn_result& r, const uint8_t* eth, uint16_t link) {
    if (tver_ != disp_ver_ || r.conn_id >= kMaxConn) return false; // the links are the batch-start table's
    Conn& c = conns_[r.conn_id];
    if (c.ack_frame_ != frame_idx_ - link || !c.established_ || c.fin_sent_) return false;
    // onAck with j's ack number again: una would not move, and sendQueued would send nothing
    if (c.send_una_ != c.send_next_ && (int32_t)(c.ack_in_ - c.seg(c.send_una_ + 1).seq) >= 0) return false;
    const uint32_t queued = c.data_next_ == c.send_next_ ? c.data_next_size_ : c.smss_;
    if (queued && (int32_t)(c.next_seq_ + queued - c.send_wnd_seq_) <= 0) return false;
    const uint32_t len = (uint32_t)(int32_t)r.payload_len;
    if (!c.rx_.inOrderReady(r.seq, len)) return false;
    PackAdapter<HH> a{*this, h, c, eth};
    c.ack_frame_ = frame_idx_; // its ACK field is j's: processed (as a no-op)
    afterSegment(h, c, c.rx_.onInOrder(a, eth + r.payload_off, len));
    ++in_order_;
    return true;
  }

  template <class HH>
  PN_HOT void afterSegment(HH& h, Conn& c, const RxAck ack) {
    if (c.rx_.closed() && !c.isClosed()) { // RST accepted, or receive buffer full (TcpConn.h:526-531, 741-745)
      if (ack.rst)
        closeConn(c); // close(): RST to the peer
      else
        onClose(c, false);
      return;
    }
    // as in the reference, an ACK still owed is sent even when a callback closed the
    // connection (a close() sends an RST first, which clears the owed ACK)
    if (ack.send) sendAck(c, ack.immediate);
    // TcpConn.h:765-768: both FINs exchanged and everything acknowledged -> TIME_WAIT
    if (c.fin_sent_ && c.rx_.finReceived() && c.established_ && c.send_una_ == c.data_next_) {
      c.err_ = "connection closed"; // onConnectionClosed (EfviTcp.h:116-119, 278-281)
      h.disconnect(c);
      onClose(c, true);
    }
  }

  // Step 5: the ACK field (TcpConn.h:536-665; pollnet: no cwnd, no window scaling).
  PN_HOT void onAck(Conn& c, const uint8_t* eth, bool no_text) {
    const uint32_t ack_num = ackNum(eth);
    c.ack_in_ = ack_num; // (inOrder)
    bool window_updated = false;
    if (!c.fin_sent_) {
      const uint32_t w = ack_num + srv_detail::rd16(eth + 34 + 14);
      if ((int32_t)(w - c.send_wnd_seq_) > 0) {
        window_updated = true;
        c.send_wnd_seq_ = w;
      }
    }
    const uint32_t old_una = c.send_una_;
    while (c.send_una_ != c.send_next_ && (int32_t)(ack_num - c.seg(c.send_una_ + 1).seq) >= 0) c.send_una_++;
    if (old_una != c.send_una_) { // new data acknowledged
      c.dup_ack_cnt_ = 0;
      c.retries_ = 0;
      const int rtt = std::max(1, (int)(wheel_.now() - c.seg(old_una).send_ts));
      c.rttvar_ -= (int)(c.rttvar_ - std::abs(rtt - (int)c.srtt_)) >> 2;
      c.srtt_ -= (int)(c.srtt_ - rtt) >> 3;
      updateRto(c);
      c.timers_[0].unlink();
      if (c.send_una_ != c.send_next_) wheel_.add(c.rto_, &c.timers_[0]);
      if (c.in_recover_) {
        if ((int32_t)(c.send_una_ - c.recover_) < 0) {
          resendUna(c); // partial ACK
        } else {
          if ((int32_t)(c.send_una_ - c.recover_) > 0) c.in_recover_ = false;
          c.fast_re_ = false;
        }
      }
    } else if (c.send_una_ != c.send_next_ && !window_updated && no_text) { // duplicate ACK
      if (++c.dup_ack_cnt_ == 3 && !c.in_recover_) {
        c.fast_re_ = c.in_recover_ = true;
        c.recover_ = c.send_next_;
        resendUna(c);
      }
    }
    sendQueued(c);
  }

  // Transmit queued segments the window now admits (TcpConn.h:646-660).  Nothing queued (the common case: the
  // segment being built is the next to send and empty) ends it before the loop, inline.
  PN_HOT void sendQueued(Conn& c) {
    if (c.data_next_ == c.send_next_ && !c.data_next_size_) return;
    sendQueuedLoop(c);
  }
  void sendQueuedLoop(Conn& c) {
    while (uint32_t size = (c.data_next_ == c.send_next_ ? c.data_next_size_ : c.smss_)) {
      typename Conn::Seg& s = c.seg(c.send_next_);
      if ((int32_t)(s.seq + size - c.send_wnd_seq_) > 0) break;
      if (c.data_next_ == c.send_next_) {
        s.fin = c.fin_sent_;
        s.len = (uint16_t)(size - (s.fin ? 1 : 0));
        emit(c, s.seq, s.fin ? kFinAck : kData, c.segData(c.send_next_), s.len);
        advanceData(c);
      } else {
        s.len = (uint16_t)size;
        s.fin = false;
        emit(c, s.seq, kData, c.segData(c.send_next_), s.len);
      }
      advanceNext(c, size);
    }
  }

  void advanceNext(Conn& c, uint32_t inc) { // TcpConn.h:327-333
    typename Conn::Seg& s = c.seg(c.send_next_);
    s.send_ts = wheel_.now();
    if (c.send_next_ == c.send_una_) wheel_.add(c.rto_, &c.timers_[0]);
    const uint32_t seq = s.seq;
    c.seg(++c.send_next_).seq = c.next_seq_ = seq + inc;
  }
  void advanceData(Conn& c) {
    c.data_next_++;
    c.data_next_size_ = 0;
  }

  // TcpConn::sendPartial (TcpConn.h:232-256): append, cut segments at SMSS, send what fits.
  uint32_t sendPartial(Conn& c, const uint8_t* d, uint32_t size, bool last) {
    const uint8_t* p = d;
    while (size && c.send_una_ + kSendBufCnt - 1 != c.data_next_) {
      const uint32_t n = std::min(c.smss_ - c.data_next_size_, size);
      std::memcpy(c.segData(c.data_next_) + c.data_next_size_, p, n);
      p += n;
      size -= n;
      c.data_next_size_ += n;
      typename Conn::Seg& s = c.seg(c.data_next_);
      const bool can_send =
          c.data_next_ == c.send_next_ && (int32_t)(s.seq + c.data_next_size_ - c.send_wnd_seq_) <= 0;
      if (c.data_next_size_ == c.smss_ || (last && can_send)) {
        if (can_send) {
          s.len = (uint16_t)c.data_next_size_;
          s.fin = false;
          emit(c, s.seq, kData, c.segData(c.data_next_), s.len);
          advanceNext(c, c.data_next_size_);
        }
        advanceData(c);
      }
    }
    return (uint32_t)(p - d);
  }

  void sendFin(Conn& c) { // TcpConn.h:69-84
    if (c.fin_sent_ || !c.eng_) return;
    if (c.send_una_ + kSendBufCnt - 1 == c.data_next_) {
      closeConn(c);
      return;
    }
    c.fin_sent_ = true;
    c.rx_.setFinSent();
    c.data_next_size_++;
    if (c.data_next_ == c.send_next_ && c.data_next_size_ == 1) {
      typename Conn::Seg& s = c.seg(c.data_next_);
      s.fin = true;
      s.len = 0;
      emit(c, s.seq, kFinAck, nullptr, 0);
      advanceNext(c, 1);
      advanceData(c);
    }
  }

  // TcpConn.h:335-343.  The reference takes the ACK's buffer from getAckBuf (TcpConn.h:851-860):
  // a free SendBuf in [data_next, send_una + ConnSendBufCnt - 1] whose previous frame the NIC has
  // completed (avail).  Here every frame leaves through the link at flush, so every buffer is
  // complete, and sendPartial / sendFin keep data_next <= send_una + ConnSendBufCnt - 1: that range
  // is never empty and getAckBuf never fails — the ACK (and close()'s RST) always goes out.  The one
  // case the reference would drop, a buffer still in the NIC's TX queue, does not exist here.
  PN_HOT void sendAck(Conn& c, bool immediate) {
    if (kDelayedAckMS == 0 || immediate) {
      emit(c, c.next_seq_, kAck, nullptr, 0);
      return;
    }
    if (c.timers_[1].unlinked()) wheel_.add(std::max(1u, kDelayedAckMS), &c.timers_[1]);
  }

  void resendUna(Conn& c) { // TcpConn.h:771-790 (pollnet: no ssthresh)
    c.retries_++;
    typename Conn::Seg& s = c.seg(c.send_una_);
    if (!c.established_ && c.send_una_ == 0)
      emit(c, s.seq, s.syn_ack ? kSynAck : kSyn, nullptr, 0);
    else
      emit(c, s.seq, s.fin ? kFinAck : kData, c.segData(c.send_una_), s.len);
    s.send_ts = wheel_.now();
  }

  void setUserTimer(Conn& c, uint32_t id, uint32_t ms) { // TcpConn.h:86-90
    TimerNode& t = c.timers_[2 + id];
    t.unlink();
    if (ms) wheel_.add(ms, &t);
  }

  // TcpConn::close (TcpConn.h:92-102): RST if established, then release the entry.
  void closeConn(Conn& c) {
    if (c.isClosed()) return;
    if (c.established_) emit(c, c.next_seq_, kRstAck, nullptr, 0);
    onClose(c, false);
  }

  // TcpConn::onClose (TcpConn.h:420-435): leave the table, or enter TIME_WAIT.
  void onClose(Conn& c, bool enter_tw) {
    if (c.isClosed()) return;
    c.fin_sent_ = c.fin_received_ = true;
    c.established_ = false;
    for (auto& t : c.timers_) t.unlink();
    if (!enter_tw || tw_cnt_ == kMaxTw) { // Core::enterTW: TIME_WAIT table full -> delete (Core.h:608-611)
      releaseEntry(c);
      return;
    }
    // Core::enterTW (Core.h:607-638)
    const uint32_t tw_id = free_tws_.back();
    if (table_.enterTW(c.key_, tw_id) != 0) { // the key is not in the table (a reference-literal rehash
      releaseEntry(c);                        // stranded it): no TIME_WAIT, the ids stay consistent
      return;
    }
    free_tws_.pop_back();
    ++tw_cnt_;
    free_conns_.push_back(c.id_);
    --conn_cnt_;
    ++tver_;
    Tw& tw = tws_[tw_id];
    tw.key = c.key_;
    std::memcpy(tw.peer_mac, c.peer_mac_, 6);
    tw.peer_ip = c.peer_ip_;
    tw.peer_port = c.peer_port_;
    tw.local_port = c.local_port_;
    tw.seq_num = c.next_seq_;
    tw.ack_num = c.rx_.ackSeq();
    wheel_.add(kTimeWaitTimeout, &tw.timer);
  }

  // A closing connection leaves the table (delConnEntry); its id is returned even when its key
  // cannot be found (stranded by a reference-literal rehash, PN_TABLE_REFERENCE_LITERAL).
  void releaseEntry(Conn& c) {
    uint32_t id = PN_MISS;
    if (table_.find(c.key_, nullptr, &id) && id == c.id_) {
      delEntry(c.key_);
      return;
    }
    free_conns_.push_back(c.id_);
    --conn_cnt_;
  }

  // Core::delConnEntry (Core.h:578-605) with its id bookkeeping.
  void delEntry(uint64_t key) {
    uint32_t id = PN_MISS;
    if (!table_.find(key, nullptr, &id)) return;
    if (id < kMaxConn) {
      free_conns_.push_back(id);
      --conn_cnt_;
    } else {
      free_tws_.push_back(id - kMaxConn);
      --tw_cnt_;
    }
    table_.del(key);
    ++tver_;
  }

  template <class HH>
  void onTimer(HH& h, TimerNode* n) { // TcpConn::onTimer (TcpConn.h:792-836), TIME_WAIT expiry (Core.h:740-744)
    if (n->owner >= kMaxConn) {
      delEntry(tws_[n->owner - kMaxConn].key);
      return;
    }
    Conn& c = conns_[n->owner];
    switch (n->kind) {
      case 0: { // retransmission
        if (c.retries_ >= std::min(31u, !c.established_ ? kSynRetries : kTcpRetries)) {
          c.err_ = "connection timeout"; // onConnectionTimeout (EfviTcp.h:115-119, 273-276)
          if (c.established_) h.disconnect(c);
          else if (Derived::kClient) h.connectFailed();
          closeConn(c);
          break;
        }
        resendUna(c);
        c.fast_re_ = false;
        c.in_recover_ = true;
        c.recover_ = c.send_next_;
        c.rto_ = std::min(c.rto_ << 1, kMaxRtoMS);
        wheel_.add(c.rto_, &c.timers_[0]);
        break;
      }
      case 1: sendAck(c, true); break;
      case 2: h.sendTimeout(c); break;
      default: h.recvTimeout(c); break;
    }
  }

  // ---- frame building: a header-only frame gets both checksums as it is built; one with options or payload at
  // flush (flushTx: on the host, or the whole batch by pn_tx_fill) ----
  enum Kind { kSyn, kSynAck, kData, kFinAck, kAck, kRstAck };
  uint8_t* txFrame() {
    if (tx_n_ == kTxBatch) flushTx();
    return tx_base_[tx_cur_] + (size_t)tx_n_++ * Backend::kStride;
  }
  void header(uint8_t* f, const uint8_t* dst_mac, uint32_t dst_ip, uint16_t src_port, uint16_t dst_port, uint32_t seq,
              uint32_t ack, uint8_t doff_words, uint8_t flags, uint16_t window, uint32_t tcp_len) {
    using namespace srv_detail;
    std::memcpy(f, dst_mac, 6);
    std::memcpy(f + 6, local_mac_, 6);
    f[12] = 0x08;
    f[13] = 0x00;
    uint8_t* ip = f + 14; // SendBuf's fixed IP header (Core.h:291-301)
    ip[0] = 0x45;
    ip[1] = 0;
    wr16(ip + 2, (uint16_t)(20 + tcp_len));
    wr16(ip + 4, 0);
    wr16(ip + 6, 0x4000);
    ip[8] = 64;
    ip[9] = 6;
    wr16(ip + 10, 0);
    std::memcpy(ip + 12, &local_ip_, 4);
    std::memcpy(ip + 16, &dst_ip, 4);
    uint8_t* tcp = ip + 20;
    std::memcpy(tcp, &src_port, 2);
    std::memcpy(tcp + 2, &dst_port, 2);
    wr32(tcp + 4, seq);
    wr32(tcp + 8, ack);
    tcp[12] = (uint8_t)(doff_words << 4);
    tcp[13] = flags;
    wr16(tcp + 14, window);
    wr32(tcp + 16, 0); // checksum, urgent pointer
    if (doff_words == 5 && tcp_len == 20) { // header only: both checksums now, from the values
      const HeaderSums cs = header_sums(local_ip_, dst_ip, src_port, dst_port, seq, ack, flags, window);
      std::memcpy(ip + 10, &cs.ip, 2);
      std::memcpy(tcp + 16, &cs.tcp, 2);
    } else { // options or payload follow: summed at flush, on the host or by pn_tx_fill
      tx_fill_[tx_cur_].push_back(tx_n_ - 1);
    }
  }
  // header() for a frame of connection c, from its template: the fields that vary written over it, and (header only)
  // both checksums from the template's fixed sums plus those fields.  The same bytes as header().
  void connHeader(const Conn& c, uint8_t* f, uint32_t seq, uint32_t ack, uint8_t doff_words, uint8_t flags,
                  uint16_t window, uint32_t tcp_len) {
    using namespace srv_detail;
    std::memcpy(f, c.hdr_, sizeof c.hdr_);
    uint8_t* ip = f + 14;
    uint8_t* tcp = ip + 20;
    wr16(ip + 2, (uint16_t)(20 + tcp_len));
    wr32(tcp + 4, seq);
    wr32(tcp + 8, ack);
    tcp[12] = (uint8_t)(doff_words << 4);
    tcp[13] = flags;
    wr16(tcp + 14, window);
    if (doff_words == 5 && tcp_len == 20) {
      auto halves = [](uint32_t x) -> uint64_t { return (x & 0xffffu) + (x >> 16); };
      const uint16_t ip_sum = csum_fold(c.hdr_ip_sum_ + 0x2800u);
      const uint16_t tcp_sum = csum_fold(c.hdr_tcp_sum_ + 0x1400u + halves(__builtin_bswap32(seq)) +
                                         halves(__builtin_bswap32(ack)) + (0x50u | (uint32_t)flags << 8) +
                                         __builtin_bswap16(window));
      std::memcpy(ip + 10, &ip_sum, 2);
      std::memcpy(tcp + 16, &tcp_sum, 2);
    } else {
      tx_fill_[tx_cur_].push_back(tx_n_ - 1);
    }
  }
  // A segment of connection c (TcpConn::sendBuf, TcpConn.h:310-323): ack = what was received
  // so far (updateLastAck, TcpConn.h:838-843), window = free receive buffer.
  void emit(Conn& c, uint32_t seq, Kind k, const uint8_t* payload, uint32_t len) {
    c.timers_[1].unlink();
    c.rx_.ackSent();
    const uint32_t ack = c.rx_.ackSeq();
    const uint16_t win = (uint16_t)std::min<uint32_t>(65535u, c.rx_.window());
    uint8_t* f = txFrame();
    enum : uint8_t { FIN = 1, SYN = 2, RST = 4, PSH = 8, ACK = 16 };
    switch (k) {
      case kSyn:
      case kSynAck: // MSS option (TcpConn.h:207-214)
        connHeader(c, f, seq, ack, 6, (uint8_t)(SYN | (k == kSynAck ? ACK : 0)), win, 24);
        f[54] = 2;
        f[55] = 4;
        srv_detail::wr16(f + 56, (uint16_t)PN_RECV_MSS);
        break;
      case kData:
      case kFinAck:
        connHeader(c, f, seq, ack, 5, (uint8_t)(PSH | ACK | (k == kFinAck ? FIN : 0)), win, 20 + len);
        if (len) {
          std::memcpy(f + 54, payload, len);
          ++tx_data_n_;
        }
        break;
      case kAck: connHeader(c, f, seq, ack, 5, PSH | ACK, win, 20); break;
      case kRstAck: connHeader(c, f, seq, ack, 5, RST | PSH | ACK, win, 20); break;
    }
  }
  // Core::rspRst (Core.h:400-423): answer a segment nobody owns.  RSTs and TIME_WAIT ACKs
  // share one send buffer in the reference (the last SendBuf), whose window field is never
  // written (0) and whose ack_num an ACK-less RST does not rewrite: rst_ack_ is that field.
  // (One difference: the reference skips the RST while that buffer's previous frame is
  // still in the NIC's TX queue, Core.h:404; here every RST goes out.)
  void rspRst(const uint8_t* eth, const pn_result& r) {
    using namespace srv_detail;
    if (r.flags & PN_F_RST) return;
    const uint8_t* tcp = eth + 34;
    uint32_t src_ip;
    uint16_t src_port, dst_port;
    std::memcpy(&src_ip, eth + 26, 4);
    std::memcpy(&src_port, tcp, 2);
    std::memcpy(&dst_port, tcp + 2, 2);
    uint8_t* f = txFrame();
    if (r.flags & PN_F_ACK) { // ack_num keeps what the shared buffer last carried
      header(f, eth + 6, src_ip, dst_port, src_port, rd32(tcp + 8), rst_ack_, 5, 0x04, 0, 20);
    } else {
      rst_ack_ = rd32(tcp + 4) + segLen(eth, r);
      header(f, eth + 6, src_ip, dst_port, src_port, 0, rst_ack_, 5, 0x14, 0, 20);
    }
  }
  // Core::ackTW (Core.h:425-446)
  void ackTW(const Tw& tw) {
    uint8_t* f = txFrame();
    rst_ack_ = tw.ack_num;
    header(f, tw.peer_mac, tw.peer_ip, tw.local_port, tw.peer_port, tw.seq_num, tw.ack_num, 5, 0x10, 0, 20);
  }

  Link link_;
  Backend be_;
  ConnTable table_;
  TimerWheel wheel_;
  std::vector<Conn> conns_;
  std::vector<Tw> tws_;
  std::vector<uint32_t> free_conns_, free_tws_;
  uint32_t conn_cnt_ = 0, tw_cnt_ = 0, tx_n_ = 0, rx_pending_ = 0;
  int64_t rx_first_ns_ = 0;
  uint32_t local_ip_ = 0, rst_ack_ = 0;
  uint8_t local_mac_[6] = {};
  // table versions: tver_ counts table changes; synced_ver_ is the device snapshot's, disp_ver_
  // that of the records being dispatched; fl_* the pipelined batch in flight per ring half
  uint64_t tver_ = 1, synced_ver_ = 0, disp_ver_ = 0, fl_ver_[3] = {0, 0, 0};
  // RX rings: cur_ is filling; fl_cnt_ batches in flight from fl_head_ on (pipelined), fl_n_ frames each
  uint32_t cur_ = 0, fl_n_[3] = {0, 0, 0}, fl_head_ = 0, fl_cnt_ = 0;
  uint32_t tx_cur_ = 0, tx_fl_n_ = 0; // TX batch being built; frames of the other one in its fill (pipelined)
  uint8_t* tx_base_[2] = {nullptr, nullptr}; // be_.txSlots(half) + kFrameOff, set at init
  uint32_t tx_data_n_ = 0;            // payload-bearing frames in the batch being built
  std::vector<uint32_t> tx_fill_[2];  // per TX batch: the frames whose checksums are filled at flush
  bool tx_fl_host_ = false;           // the batch in its fill was summed on the host
  uint64_t tx_host_frames_ = 0, tx_gpu_frames_ = 0;
  uint64_t re_resolved_ = 0;
  uint64_t frame_idx_ = 0; // frames dispatched (onFrame) since init: a frame's place for the chain links
  uint64_t in_order_ = 0;  // frames that took the in-order fast path
  bool ready_ = false, drop_bad_ = true;
  const char* err_ = "Closed";
};

} // namespace pollnet_amd
