// tcp_server.hpp — GpuTcpServer<Conf>: pollnet's TCP server surface over the GPU RX path.
//
// A drop-in for pollnet's EfviTcpServer<Conf> (/root/reference/efvitcp/EfviTcp.h:177-309)
// with the same user surface:
//   bool init(const char* interface, const char* server_ip, uint16_t server_port);
//   const char* getLastError();  void close(const char* reason);  bool isClosed();
//   uint32_t getConnCnt();  void foreachConn(F);
//   template <class Handler> void poll(Handler& handler, int64_t ns = 0);
// and the same Conn (EfviTcp.h:225-241 over TcpConn, efvitcp/TcpConn.h:30-113):
//   getPeername, isConnected/isEstablished/isClosed, getLastError, close(reason),
//   writeNonblock(data, size, more), send, getSendable, sendFin, setUserTimer, getConnId,
//   plus the user's Conf::UserData fields (Conn derives from it, as TcpConn does).
// Handler callbacks, found by name as the reference's TmpHandler calls them
// (EfviTcp.h:264-307; README.md:81-104):
//   uint32_t onTcpData(Conn&, const uint8_t* data, uint32_t size)   required; returns the
//            bytes NOT consumed, re-presented with the next data (TcpConn.h:715-724)
//   void onTcpConnected(Conn&), onTcpDisconnect(Conn&), onSendTimeout(Conn&),
//        onRecvTimeout(Conn&)                                         optional
//   bool allowNewConnection(uint32_t ip_be, uint16_t port_be)          optional (accept all)
// so a handler written for EfviTcpServer (example/tcpserver.cc:61-91) compiles unchanged.
//
// What poll() does, in the reference's order (TcpServer.h:70-112 over Core::pollTime /
// Core::pollNet, Core.h:494-552, 710-748):
//   1. one timer tick (Core::pollTime: now_ts advances by at most one ms per call):
//      retransmission, delayed ACK, the user send/recv timeouts, TIME_WAIT expiry;
//   2. the link's pending frames land in a pinned ring of slots; ONE pn_classify launch
//      (zero-copy over PCIe) parses them, verifies the IP/TCP checksums and probes the
//      conn table for the whole batch (the per-frame hot path, on the GPU);
//   3. the records are walked in ring order on the host, each through the reference's
//      branches: the NIC filter (dst ip/port, Core.h:335-383), the checksum discard a NIC
//      applies (ef_vi RX_DISCARD), TIME_WAIT (Core.h:510-524: in-sequence RST deletes,
//      data or out-of-sequence -> ACK), unknown flow (TcpServer.h:80-96: SYN accepted
//      while conn_cnt < MaxConnCnt, else RST), SYN-RECEIVED (TcpServer.h:97-111) and the
//      connection's segment processing (TcpConn::onPack, TcpConn.h:466-769: the receive
//      half is RxConn, rx_conn.hpp; the ACK field / send half is here);
//   4. every frame the poll produced (SYN-ACK, ACKs, data, RST, TIME_WAIT ACKs,
//      retransmissions) gets its IP and TCP checksums from ONE pn_tx_fill launch over the
//      pinned TX batch, then goes out through the link in generation order.
// Conf::RxLatencyBudgetUs (default 0: every poll with frames classifies them) lets frames of
// consecutive polls accumulate for up to that long before one launch takes them all.
// Sends issued outside poll() (a writeNonblock from the user's own loop) are built at once
// and leave with the next poll's TX batch.  The table snapshot on the device is refreshed
// before each classify; records after a table change within the same batch are
// re-resolved on the host (one ordered probe), so every frame sees the table the
// reference's sequential loop would have shown it.
//
// Send side: the reference's segment ring (ConnSendBufCnt segments of up to SMSS bytes,
// TcpConn.h:58-90, 232-256), window, RTO/fast retransmit and delayed ACK, restated for
// pollnet's configuration (EfviTcp.h:180-199: no window scaling, no timestamps, no
// congestion window).  Time: now_ts = ns >> 20 (Core.h:46), from `ns` or CLOCK_REALTIME.
#pragma once

#include <arpa/inet.h>
#include <net/if.h>
#include <netinet/in.h>
#include <sys/ioctl.h>
#include <sys/socket.h>
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
PN_CONF_OPT(DelayedAckMS, uint32_t, 10)     // EfviTcp.h:189
PN_CONF_OPT(Device, int, 0)
PN_CONF_OPT(ReferenceLiteralTable, bool, false) // PN_TABLE_REFERENCE_LITERAL: the reference's rehash, defect kept
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
    if (rx_ring_) (void)hipHostFree(rx_ring_);
    if (tx_ring_) (void)hipHostFree(tx_ring_);
  }

  const char* init(int device, uint32_t rx_cap, uint32_t tx_cap) {
    if (const char* e = rx_.init(device, kStride, kFrameOff, rx_cap, GpuRx::Mode::ZeroCopy)) return e;
    if (hipHostMalloc((void**)&rx_ring_, (size_t)kStride * rx_cap, hipHostMallocDefault) != hipSuccess)
      return "hipHostMalloc(rx ring) failed";
    if (hipHostMalloc((void**)&tx_ring_, (size_t)kStride * tx_cap, hipHostMallocDefault) != hipSuccess)
      return "hipHostMalloc(tx batch) failed";
    std::memset(rx_ring_, 0, (size_t)kStride * rx_cap);
    std::memset(tx_ring_, 0, (size_t)kStride * tx_cap);
    return nullptr;
  }
  uint8_t* rxSlots() { return rx_ring_; }
  uint8_t* txSlots() { return tx_ring_; }
  const char* syncTable(const ConnTable& t) { return rx_.syncTable(t); }
  // f(key, rec, eth) for the n frames of the RX ring, in ring order.
  template <class F>
  const char* classify(uint32_t n, const ConnTable& t, F&& f) {
    return rx_.pollBatch(
        rx_ring_, n, t, [&](uint64_t key, const pn_result& r, const uint8_t* eth, uint32_t) { f(key, r, eth); },
        [&](uint64_t key, uint32_t, const uint8_t* eth, const pn_result& r) { f(key, r, eth); });
  }
  // IP + TCP checksums of the first n TX slots (PN_TX_TCP: SendBuf::setOptDataLen, Core.h:157-163).
  const char* fillTx(uint32_t n) {
    if (pn_tx_fill(rx_.ctx(), tx_ring_, kStride, kFrameOff, n, nullptr, PN_TX_TCP, rx_.stream()))
      return pn_last_error(rx_.ctx());
    if (hipStreamSynchronize(rx_.stream()) != hipSuccess) return "hipStreamSynchronize(tx_fill) failed";
    return nullptr;
  }

 private:
  GpuRx rx_;
  uint8_t* rx_ring_ = nullptr;
  uint8_t* tx_ring_ = nullptr;
};

// ---------------------------------------------------------------------------
template <class Conf, class Link = SocketLink, class Backend = GpuBackend>
class GpuTcpServer {
 public:
  // EfviTcpServer's ServerConf (EfviTcp.h:180-199), as RxConn reads it.
  struct IConf {
    static const uint32_t ConnRecvBufSize = Conf::RecvBufSize;
    static const uint32_t MaxConnCnt = Conf::MaxConns;
    static const uint32_t MaxTimeWaitConnCnt = Conf::MaxConns;
    static const bool TimestampOption = false;
  };
  static constexpr uint32_t kMaxConn = Conf::MaxConns;
  static constexpr uint32_t kSendBufCnt = srv_detail::opt_ConnSendBufCnt<Conf>::value;
  static constexpr uint32_t kSendMTU = 1024 - 28;      // SendBuf1K: SendBufSize - offsetof(ip_hdr), Core.h:232-234
  static constexpr uint32_t kSegCap = kSendMTU - 40;   // largest SMSS (onSyn's clamp, TcpConn.h:357)
  static constexpr uint32_t kSynRetries = 3, kTcpRetries = 10, kMinRtoMS = 100, kMaxRtoMS = 30 * 1000;
  static constexpr uint32_t kDelayedAckMS = srv_detail::opt_DelayedAckMS<Conf>::value;
  static constexpr uint32_t kTimeWaitTimeout = 60 * 1000; // Core.h:48
  static constexpr uint32_t kRxBatch = srv_detail::opt_RxBatch<Conf>::value;
  static constexpr uint32_t kTxBatch = srv_detail::opt_TxBatch<Conf>::value;
  static constexpr uint32_t kRxBudgetUs = srv_detail::opt_RxLatencyBudgetUs<Conf>::value;
  static_assert(kSendBufCnt >= 4 && !(kSendBufCnt & (kSendBufCnt - 1)), "ConnSendBufCnt must be a power of 2");
  static_assert(Conf::RecvBufSize >= 2 * 1460, "RecvBufSize below two RMSS");

  class Conn : public srv_detail::user_data<Conf>::type {
   public:
    const char* err_ = nullptr; // EfviTcp.h:197 (UserData::err_)

    uint32_t getConnId() const { return id_; }
    void getPeername(sockaddr_in& addr) const { // TcpConn.h:37-41
      addr.sin_addr.s_addr = peer_ip_;
      addr.sin_port = peer_port_;
    }
    bool isEstablished() const { return established_; }
    bool isConnected() const { return established_; }
    bool isClosed() const { return fin_received_ && !established_; } // TcpConn.h:45
    const char* getLastError() const { return err_; }
    void close(const char* reason) { // EfviTcp.h:230-233
      err_ = reason;
      srv_->closeConn(*this);
    }
    // EfviTcp.h:236-244: all or nothing, else the connection is closed.
    bool writeNonblock(const void* data, uint32_t size, bool more = false) {
      if (send(data, size, more) != size) {
        close("send buffer full");
        return false;
      }
      if (srv_detail::opt_SendTimeoutSec<Conf>::value) setUserTimer(0, srv_detail::opt_SendTimeoutSec<Conf>::value * 1000);
      return true;
    }
    // TcpConn::send (TcpConn.h:58-61): bytes accepted into the send buffer.
    uint32_t send(const void* data, uint32_t size, bool more = false) {
      if (fin_sent_) return 0;
      return srv_->sendPartial(*this, (const uint8_t*)data, size, !more);
    }
    uint32_t getSendable() const { // TcpConn.h:47-50
      if (fin_sent_) return 0;
      return (send_una_ + kSendBufCnt - 1 - data_next_) * smss_ - data_next_size_;
    }
    void sendFin() { srv_->sendFin(*this); }
    void setUserTimer(uint32_t timer_id, uint32_t duration_ms) { srv_->setUserTimer(*this, timer_id, duration_ms); }

   private:
    friend class GpuTcpServer;
    struct Seg {
      uint32_t seq = 0;
      uint32_t send_ts = 0;
      uint16_t len = 0; // payload bytes
      bool fin = false;
    };
    Seg& seg(uint32_t idx) { return segs_[idx & (kSendBufCnt - 1)]; }
    uint8_t* segData(uint32_t idx) { return data_.get() + (size_t)(idx & (kSendBufCnt - 1)) * kSegCap; }

    GpuTcpServer* srv_ = nullptr;
    uint32_t id_ = 0;
    uint64_t key_ = 0;
    uint32_t peer_ip_ = 0;    // network order
    uint16_t peer_port_ = 0;  // network order
    uint8_t peer_mac_[6] = {};
    RxConn<IConf> rx_;
    // send side (TcpConn.h:861-898)
    std::unique_ptr<Seg[]> segs_;
    std::unique_ptr<uint8_t[]> data_;
    uint32_t send_una_ = 0, send_next_ = 0, data_next_ = 0, data_next_size_ = 0, recover_ = 0;
    uint32_t smss_ = 536, send_wnd_seq_ = 0, rto_ = 1000, srtt_ = 0, rttvar_ = 0, dup_ack_cnt_ = 0, retries_ = 0;
    bool established_ = false, fin_sent_ = true, fin_received_ = true, fast_re_ = false, in_recover_ = false;
    TimerNode timers_[4]; // resend, delayed ACK, user 0 (send timeout), user 1 (recv timeout)
  };

  GpuTcpServer() : conns_(kMaxConn), tws_(kMaxConn) {}
  GpuTcpServer(const GpuTcpServer&) = delete;
  GpuTcpServer& operator=(const GpuTcpServer&) = delete;
  ~GpuTcpServer() { close(nullptr); }  // RSTs to open connections, as TcpServer's destructor

  // EfviTcpServer::init (EfviTcp.h:246-250): open the interface, listen on server_port.
  // server_ip is the address the server answers on (the NIC filter's local ip,
  // Core.h:335-383); nullptr or "0.0.0.0" takes the interface's address.
  bool init(const char* interface, const char* server_ip, uint16_t server_port) {
    if ((err_ = link_.open(interface))) return false;
    return initCommon(server_ip, server_port, getns());
  }
  // The same over a link the caller has opened (a capture replay, a test peer, a
  // ring fed by another process); now_ns fixes the clock origin (0 = CLOCK_REALTIME).
  bool initWithLink(const char* server_ip, uint16_t server_port, int64_t now_ns = 0) {
    return initCommon(server_ip, server_port, now_ns ? now_ns : getns());
  }
  Link& link() { return link_; }

  const char* getLastError() { return err_; }
  void close(const char* reason) { // EfviTcp.h:252-255 / TcpServer::close
    if (reason) err_ = reason;
    if (!ready_) return;
    for (auto& c : conns_)
      if (c.srv_ && !c.isClosed()) closeConn(c);
    flushTx();
  }
  bool isClosed() { return err_ != nullptr; }
  uint32_t getConnCnt() { return conn_cnt_; } // TcpServer.h:53 (SYN-RECEIVED included)
  template <class F>
  void foreachConn(F f) { // TcpServer.h:55-60
    for (auto& c : conns_)
      if (c.established_) f(c);
  }
  // Drop checksum-failed frames before they touch any state (what the NIC's RX
  // checksum offload does for efvitcp: ef_vi delivers them as RX_DISCARD).  Default on.
  void setDropBadChecksum(bool drop) { drop_bad_ = drop; }
  const ConnTable& table() const { return table_; }
  uint32_t nowTs() const { return wheel_.now(); }

  template <class Handler>
  void poll(Handler& handler, int64_t ns = 0) {
    if (!ready_) return;
    H<Handler> h{handler};
    const int64_t now = ns ? ns : getns();
    // 1. timers (Core::pollTime, Core.h:710-748)
    wheel_.tick((uint32_t)(now >> 20), [&](TimerNode* n) { onTimer(h, n); });
    // 2./3. RX batch: classify on the GPU, dispatch in ring order.  With a latency budget the
    // frames of several polls accumulate in the ring (timers and TX still run every poll) until
    // the ring is full or the oldest has waited the budget: one launch per budget instead of
    // one per poll.
    const uint32_t got = link_.fill(be_.rxSlots() + (size_t)rx_pending_ * Backend::kStride, Backend::kStride,
                                    Backend::kFrameOff, kRxBatch - rx_pending_);
    if (got && rx_pending_ == 0) rx_first_ns_ = now;
    rx_pending_ += got;
    const bool due = rx_pending_ == kRxBatch || now - rx_first_ns_ >= (int64_t)kRxBudgetUs * 1000;
    const uint32_t n = due ? rx_pending_ : 0;
    if (n) {
      rx_pending_ = 0;
      if (dirty_ && Backend::kSnapshot) {
        if ((err_ = be_.syncTable(table_))) return;
      }
      dirty_ = false;
      const char* e = be_.classify(n, table_, [&](uint64_t key, const pn_result& r, const uint8_t* eth) {
        onFrame(h, key, r, eth);
      });
      if (e) err_ = e;
    }
    // 4. TX batch: checksums on the GPU, then out in order
    flushTx();
  }

  // Frames built since the last flush (checksums not yet filled).
  uint32_t pendingTx() const { return tx_n_; }
  // Fill the pending frames' checksums (one pn_tx_fill launch) and send them.
  const char* flushTx() {
    if (!tx_n_) return nullptr;
    const char* e = be_.fillTx(tx_n_);
    if (e) {
      err_ = e;
    } else {
      for (uint32_t i = 0; i < tx_n_; i++) {
        const uint8_t* f = be_.txSlots() + (size_t)i * Backend::kStride + Backend::kFrameOff;
        link_.send(f, 14 + srv_detail::rd16(f + 16));
      }
    }
    tx_n_ = 0;
    return e;
  }

 private:
  struct Tw { // Core.h:186-197 TimeWaitConn
    uint64_t key = 0;
    uint8_t peer_mac[6] = {};
    uint32_t peer_ip = 0;
    uint16_t peer_port = 0;
    uint32_t seq_num = 0, ack_num = 0;
    TimerNode timer;
  };

  template <class Handler>
  struct H { // EfviTcpServer's TmpHandler (EfviTcp.h:264-307)
    Handler& u;
    void connected(Conn& c) {
      if constexpr (srv_detail::has_onTcpConnected<Handler, Conn>::value) u.onTcpConnected(c);
    }
    void disconnect(Conn& c) {
      if constexpr (srv_detail::has_onTcpDisconnect<Handler, Conn>::value) u.onTcpDisconnect(c);
    }
    void sendTimeout(Conn& c) {
      if constexpr (srv_detail::has_onSendTimeout<Handler, Conn>::value) u.onSendTimeout(c);
    }
    void recvTimeout(Conn& c) {
      if constexpr (srv_detail::has_onRecvTimeout<Handler, Conn>::value) u.onRecvTimeout(c);
    }
    bool allow(uint32_t ip_be, uint16_t port_be) {
      if constexpr (srv_detail::has_allowNewConnection<Handler, Conn>::value) return u.allowNewConnection(ip_be, port_be);
      return true;
    }
    uint32_t data(Conn& c, const uint8_t* d, uint32_t n) { return u.onTcpData(c, d, n); }
  };

  static int64_t getns() {
    timespec ts;
    ::clock_gettime(CLOCK_REALTIME, &ts);
    return (int64_t)ts.tv_sec * 1000000000 + ts.tv_nsec;
  }

  bool initCommon(const char* server_ip, uint16_t server_port, int64_t now_ns) {
    close(nullptr);
    ready_ = false;
    local_ip_ = link_.localIp();
    if (server_ip && std::strcmp(server_ip, "0.0.0.0") != 0) {
      in_addr a;
      if (inet_pton(AF_INET, server_ip, &a) != 1) return (err_ = "invalid server_ip"), false;
      local_ip_ = a.s_addr;
    }
    std::memcpy(local_mac_, link_.localMac(), 6);
    port_be_ = htons(server_port);
    if ((err_ = table_.init(kMaxConn, kMaxConn, srv_detail::opt_ReferenceLiteralTable<Conf>::value))) return false;
    if ((err_ = be_.init(srv_detail::opt_Device<Conf>::value, kRxBatch, kTxBatch))) return false;
    free_conns_.clear();
    for (uint32_t i = kMaxConn; i-- > 0;) free_conns_.push_back(i); // Core.h:315: conns[i] = i
    free_tws_.clear();
    for (uint32_t i = kMaxConn; i-- > 0;) free_tws_.push_back(i);
    conn_cnt_ = tw_cnt_ = 0;
    for (uint32_t i = 0; i < kMaxConn; i++) { // unlink before the wheel's heads are reset
      for (auto& t : conns_[i].timers_) t.unlink();
      tws_[i].timer.unlink();
    }
    wheel_.reset((uint32_t)(now_ns >> 20));
    for (uint32_t i = 0; i < kMaxConn; i++) {
      Conn& c = conns_[i];
      c.srv_ = this;
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
      tws_[i].timer.owner = kMaxConn + i;
    }
    tx_n_ = rx_pending_ = 0;
    dirty_ = true;
    ready_ = true;
    err_ = nullptr;
    return true;
  }

  // ---- one received frame (Core::pollNet RX branch + TcpServer::poll's recv handler) ----
  template <class HH>
  void onFrame(HH& h, uint64_t key, const pn_result& rec, const uint8_t* eth) {
    using namespace srv_detail;
    if (rec.flags & (PN_F_NOT_TCP | PN_F_TRUNC | PN_F_BADOFF)) return;
    if (std::memcmp(eth + 30, &local_ip_, 4) != 0 || std::memcmp(eth + 36, &port_be_, 2) != 0) return; // NIC filter
    if (drop_bad_ && (rec.flags & (PN_F_IP_OK | PN_F_TCP_OK)) != (PN_F_IP_OK | PN_F_TCP_OK)) return;
    pn_result r = rec;
    if (dirty_ && Backend::kSnapshot) { // the table changed earlier in this batch: probe the live one
      uint32_t conn_id = PN_MISS;
      const bool hit = table_.find(key, nullptr, &conn_id);
      r.conn_id = conn_id;
      r.flags = (uint16_t)((r.flags & ~(PN_F_HIT | PN_F_TW)) | (hit ? PN_F_HIT : 0) |
                           (hit && conn_id >= kMaxConn ? PN_F_TW : 0));
    }
    const uint8_t* tcp = eth + 34;
    const uint32_t seq_raw = r.seq - ((r.flags & PN_F_SYN) ? 1u : 0u); // rec.seq = ntohl(seq_num) + syn
    if (r.flags & PN_F_TW) { // Core.h:510-524
      Tw& tw = tws_[r.conn_id - kMaxConn];
      const bool seq_expected = seq_raw == tw.ack_num;
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
    if (!(r.flags & PN_F_HIT)) { // TcpServer.h:80-96
      if (r.flags & PN_F_RST) return;
      uint32_t src_ip;
      uint16_t src_port;
      std::memcpy(&src_ip, eth + 26, 4);
      std::memcpy(&src_port, tcp, 2);
      if ((r.flags & PN_F_ACK) || !(r.flags & PN_F_SYN) || conn_cnt_ == kMaxConn || !h.allow(src_ip, src_port)) {
        rspRst(eth, r);
        return;
      }
      const uint32_t id = free_conns_.back();
      free_conns_.pop_back();
      ++conn_cnt_;
      table_.add(key, id);
      dirty_ = true;
      Conn& c = conns_[id];
      resetConn(c, key, eth);
      onSyn(c, eth, r);
      sendSyn(c);
      return;
    }
    Conn& c = conns_[r.conn_id];
    if (!c.established_) { // SYN-RECEIVED (TcpServer.h:97-111)
      if ((r.flags & PN_F_SYN) && !(r.flags & PN_F_ACK)) {
        resendUna(c, false);
        return;
      }
      if ((r.flags & PN_F_RST) && seq_raw == c.rx_.ackSeq()) {
        onClose(c, false);
        return;
      }
      if (!(r.flags & PN_F_ACK)) return;
      if (rd32(tcp + 8) != c.seg(c.send_next_).seq) {
        rspRst(eth, r);
        return;
      }
      onEstablished(h, c, eth);
    }
    onPack(h, c, eth, r);
  }

  static uint32_t segLen(const uint8_t* eth, const pn_result& r) { // tot_len - 20 - doff*4 + syn + fin
    const uint32_t tot = srv_detail::rd16(eth + 16), doff = eth[34 + 12] >> 4;
    return tot - 20 - doff * 4 + ((r.flags & PN_F_SYN) ? 1 : 0) + ((r.flags & PN_F_FIN) ? 1 : 0);
  }

  // ---- connection setup (TcpConn::reset / onSyn / sendSyn / onEstablished) ----
  void resetConn(Conn& c, uint64_t key, const uint8_t* eth) { // TcpConn.h:150-186
    c.key_ = key;
    std::memcpy(c.peer_mac_, eth + 6, 6);
    std::memcpy(&c.peer_ip_, eth + 26, 4);
    std::memcpy(&c.peer_port_, eth + 34, 2);
    c.err_ = nullptr;
    c.established_ = c.fin_sent_ = c.fin_received_ = c.fast_re_ = c.in_recover_ = false;
    c.send_una_ = c.send_next_ = c.data_next_size_ = c.dup_ack_cnt_ = c.retries_ = 0;
    c.data_next_ = 1;
    c.smss_ = 536;
    // genISN (TcpConn.h:856-858): connHashKey(peer) + now_ts; keeps send window 0 until established
    c.send_wnd_seq_ = (uint32_t)key + wheel_.now();
    c.seg(0).seq = c.send_wnd_seq_;
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
    c.rx_.open(r.seq - 1);
    c.fin_received_ = false;
  }
  void sendSyn(Conn& c) { // TcpConn.h:197-230
    c.rto_ = 1000;
    typename Conn::Seg& s = c.seg(c.send_next_);
    s.len = 0;
    s.fin = false;
    emit(c, s.seq, kSynAck, nullptr, 0);
    advanceNext(c, 1);
  }
  template <class HH>
  void onEstablished(HH& h, Conn& c, const uint8_t* eth) { // TcpConn.h:377-418
    using namespace srv_detail;
    c.send_wnd_seq_ = rd32(eth + 34 + 8) + rd16(eth + 34 + 14);
    c.established_ = true;
    c.srtt_ = std::max(1u, wheel_.now() - c.seg(c.send_una_).send_ts);
    c.rttvar_ = c.srtt_ >> 1;
    updateRto(c);
    // onConnectionEstablished (EfviTcp.h:296-300)
    if (opt_SendTimeoutSec<Conf>::value) setUserTimer(c, 0, opt_SendTimeoutSec<Conf>::value * 1000);
    if (opt_RecvTimeoutSec<Conf>::value) setUserTimer(c, 1, opt_RecvTimeoutSec<Conf>::value * 1000);
    h.connected(c);
  }
  void updateRto(Conn& c) { c.rto_ = std::max(kMinRtoMS, c.srtt_ + std::max(1u, c.rttvar_ << 2)); }

  // ---- segment processing of a connection (TcpConn::onPack) ----
  template <class HH>
  struct PackAdapter {
    GpuTcpServer& s;
    HH& h;
    Conn& c;
    const uint8_t* eth;
    uint32_t onData(RxConn<IConf>&, const uint8_t* d, uint32_t n) { // EfviTcp.h:301-304
      if (srv_detail::opt_RecvTimeoutSec<Conf>::value)
        s.setUserTimer(c, 1, srv_detail::opt_RecvTimeoutSec<Conf>::value * 1000);
      return h.data(c, d, n);
    }
    void onFin(RxConn<IConf>&, const uint8_t* d, uint32_t n) { // EfviTcp.h:283-288
      c.fin_received_ = true;
      if (n) h.data(c, d, n);
      c.err_ = "remote close";
      s.closeConn(c); // RST (EfviTcp.h's Conn::close -> TcpConn::close)
      h.disconnect(c);
    }
    void onReset(RxConn<IConf>&) { // onConnectionReset (EfviTcp.h:269-272)
      c.err_ = "connection reset";
      h.disconnect(c);
    }
    void onAckField(RxConn<IConf>&, bool no_text) { s.onAck(c, eth, no_text); }
  };

  template <class HH>
  void onPack(HH& h, Conn& c, const uint8_t* eth, const pn_result& r) {
    PackAdapter<HH> a{*this, h, c, eth};
    const RxAck ack = c.rx_.onSegment(a, eth, r);
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
      c.err_ = "connection closed"; // onConnectionClosed (EfviTcp.h:278-281)
      h.disconnect(c);
      onClose(c, true);
    }
  }

  // Step 5: the ACK field (TcpConn.h:536-665; pollnet: no cwnd, no window scaling).
  void onAck(Conn& c, const uint8_t* eth, bool no_text) {
    using namespace srv_detail;
    const uint32_t ack_num = rd32(eth + 34 + 8);
    bool window_updated = false;
    if (!c.fin_sent_) {
      const uint32_t w = ack_num + rd16(eth + 34 + 14);
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
          resendUna(c, false); // partial ACK
        } else {
          if ((int32_t)(c.send_una_ - c.recover_) > 0) c.in_recover_ = false;
          c.fast_re_ = false;
        }
      }
    } else if (c.send_una_ != c.send_next_ && !window_updated && no_text) { // duplicate ACK
      if (++c.dup_ack_cnt_ == 3 && !c.in_recover_) {
        c.fast_re_ = c.in_recover_ = true;
        c.recover_ = c.send_next_;
        resendUna(c, true);
      }
    }
    sendQueued(c);
  }

  // Transmit queued segments the window now admits (TcpConn.h:646-660).
  void sendQueued(Conn& c) {
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
    c.seg(++c.send_next_).seq = seq + inc;
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
    if (c.fin_sent_ || !c.srv_) return;
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

  void sendAck(Conn& c, bool immediate) { // TcpConn.h:335-343
    if (kDelayedAckMS == 0 || immediate) {
      emit(c, c.seg(c.send_next_).seq, kAck, nullptr, 0);
      return;
    }
    if (c.timers_[1].unlinked()) wheel_.add(std::max(1u, kDelayedAckMS), &c.timers_[1]);
  }

  void resendUna(Conn& c, bool) { // TcpConn.h:771-790 (pollnet: no ssthresh)
    c.retries_++;
    typename Conn::Seg& s = c.seg(c.send_una_);
    if (!c.established_ && c.send_una_ == 0)
      emit(c, s.seq, kSynAck, nullptr, 0);
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
    if (c.established_) emit(c, c.seg(c.send_next_).seq, kRstAck, nullptr, 0);
    onClose(c, false);
  }

  // TcpConn::onClose (TcpConn.h:420-435): leave the table, or enter TIME_WAIT.
  void onClose(Conn& c, bool enter_tw) {
    if (c.isClosed()) return;
    c.fin_sent_ = c.fin_received_ = true;
    c.established_ = false;
    for (auto& t : c.timers_) t.unlink();
    if (!enter_tw) {
      delEntry(c.key_);
      return;
    }
    // Core::enterTW (Core.h:607-638)
    if (tw_cnt_ == kMaxConn) {
      delEntry(c.key_);
      return;
    }
    free_conns_.push_back(c.id_);
    --conn_cnt_;
    const uint32_t tw_id = free_tws_.back();
    free_tws_.pop_back();
    ++tw_cnt_;
    table_.enterTW(c.key_, tw_id);
    dirty_ = true;
    Tw& tw = tws_[tw_id];
    tw.key = c.key_;
    std::memcpy(tw.peer_mac, c.peer_mac_, 6);
    tw.peer_ip = c.peer_ip_;
    tw.peer_port = c.peer_port_;
    tw.seq_num = c.seg(c.send_next_).seq;
    tw.ack_num = c.rx_.ackSeq();
    wheel_.add(kTimeWaitTimeout, &tw.timer);
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
    dirty_ = true;
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
          c.err_ = "connection timeout"; // onConnectionTimeout (EfviTcp.h:273-276)
          if (c.established_) h.disconnect(c);
          closeConn(c);
          break;
        }
        resendUna(c, c.retries_ == 0);
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

  // ---- frame building: headers only; pn_tx_fill writes both checksums at flush ----
  enum Kind { kSynAck, kData, kFinAck, kAck, kRstAck };
  uint8_t* txFrame() {
    if (tx_n_ == kTxBatch) flushTx();
    uint8_t* f = be_.txSlots() + (size_t)tx_n_++ * Backend::kStride + Backend::kFrameOff;
    return f;
  }
  void header(uint8_t* f, const uint8_t* dst_mac, uint32_t dst_ip, uint16_t dst_port, uint32_t seq, uint32_t ack,
              uint8_t doff_words, uint8_t flags, uint16_t window, uint32_t tcp_len) {
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
    std::memcpy(tcp, &port_be_, 2);
    std::memcpy(tcp + 2, &dst_port, 2);
    wr32(tcp + 4, seq);
    wr32(tcp + 8, ack);
    tcp[12] = (uint8_t)(doff_words << 4);
    tcp[13] = flags;
    wr16(tcp + 14, window);
    wr32(tcp + 16, 0); // checksum (filled on the GPU), urgent pointer
  }
  // A segment of connection c (TcpConn::sendBuf, TcpConn.h:310-323): ack = what was
  // received so far (updateLastAck, TcpConn.h:838-843), window = free receive buffer.
  void emit(Conn& c, uint32_t seq, Kind k, const uint8_t* payload, uint32_t len) {
    c.timers_[1].unlink();
    c.rx_.ackSent();
    const uint32_t ack = c.rx_.ackSeq();
    const uint16_t win = (uint16_t)std::min<uint32_t>(65535u, c.rx_.window());
    uint8_t* f = txFrame();
    enum : uint8_t { FIN = 1, SYN = 2, RST = 4, PSH = 8, ACK = 16 };
    switch (k) {
      case kSynAck: // MSS option (TcpConn.h:207-214)
        header(f, c.peer_mac_, c.peer_ip_, c.peer_port_, seq, ack, 6, SYN | ACK, win, 24);
        f[54] = 2;
        f[55] = 4;
        srv_detail::wr16(f + 56, (uint16_t)PN_RECV_MSS);
        break;
      case kData:
      case kFinAck:
        header(f, c.peer_mac_, c.peer_ip_, c.peer_port_, seq, ack, 5, (uint8_t)(PSH | ACK | (k == kFinAck ? FIN : 0)),
               win, 20 + len);
        if (len) std::memcpy(f + 54, payload, len);
        break;
      case kAck: header(f, c.peer_mac_, c.peer_ip_, c.peer_port_, seq, ack, 5, PSH | ACK, win, 20); break;
      case kRstAck: header(f, c.peer_mac_, c.peer_ip_, c.peer_port_, seq, ack, 5, RST | PSH | ACK, win, 20); break;
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
    uint16_t src_port;
    std::memcpy(&src_ip, eth + 26, 4);
    std::memcpy(&src_port, tcp, 2);
    uint8_t* f = txFrame();
    if (r.flags & PN_F_ACK) { // ack_num keeps what the shared buffer last carried
      header(f, eth + 6, src_ip, src_port, rd32(tcp + 8), rst_ack_, 5, 0x04, 0, 20);
    } else {
      rst_ack_ = rd32(tcp + 4) + segLen(eth, r);
      header(f, eth + 6, src_ip, src_port, 0, rst_ack_, 5, 0x14, 0, 20);
    }
  }
  // Core::ackTW (Core.h:425-446)
  void ackTW(const Tw& tw) {
    uint8_t* f = txFrame();
    rst_ack_ = tw.ack_num;
    header(f, tw.peer_mac, tw.peer_ip, tw.peer_port, tw.seq_num, tw.ack_num, 5, 0x10, 0, 20);
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
  uint16_t port_be_ = 0;
  uint8_t local_mac_[6] = {};
  bool ready_ = false, dirty_ = true, drop_bad_ = true;
  const char* err_ = "Closed";
};

} // namespace pollnet_amd
