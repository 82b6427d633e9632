// tcp_server.hpp — GpuTcpServer<Conf>: pollnet's TCP server surface over the GPU RX/TX paths.
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
//   bool allowNewConnection(uint32_t ip_be, uint16_t port_be)          consulted only with
//        Conf::UseAllowNewConnection = true (efvitcp::TcpServer's event, TcpServer.h:84); by
//        default every SYN is allowed, as pollnet's EfviTcpServer wrapper does (EfviTcp.h:270)
// so a handler written for EfviTcpServer (example/tcpserver.cc:61-91) compiles unchanged.
//
// The poll itself — one timer tick, one pn_classify launch over the received frames, the
// records walked through the reference's branches, the checksums of the frames it sends (one
// pn_tx_fill launch, or the host for a batch of header-only frames) — is TcpEngine's (tcp_engine.hpp).  The server's own branches (TcpServer.h:80-111):
//   - unknown flow: a SYN is accepted while conn_cnt < MaxConnCnt and allowNewConnection
//     agrees (entry added, SYN-ACK with the MSS option sent), anything else but an RST is
//     answered with an RST;
//   - SYN-RECEIVED: a repeated SYN re-sends the SYN-ACK, an in-sequence RST releases the
//     entry, the handshake ACK must acknowledge the ISN (else RST), then the connection is
//     established and the same segment goes on to onPack.
// Conf::RxLatencyBudgetUs (default 0: every poll with frames classifies them) lets frames of
// consecutive polls accumulate for up to that long before one launch takes them all;
// Conf::RxChunk splits a poll's classify into launches overlapped with dispatch; Conf::RxPipeline
// dispatches each poll's frames in the next poll, their classify overlapped with this poll's
// dispatch (throughput mode).
#pragma once

#include "tcp_engine.hpp"

namespace pollnet_amd {

// EfviTcpServer's ServerConf (EfviTcp.h:180-199), as the engine and RxConn read it.
template <class Conf>
struct ServerIConf {
  static const uint32_t ConnRecvBufSize = Conf::RecvBufSize;
  static const uint32_t MaxConnCnt = Conf::MaxConns;
  static const uint32_t MaxTimeWaitConnCnt = Conf::MaxConns;
  static const bool TimestampOption = false;
};

template <class Conf, class Link = SocketLink, class Backend = GpuBackend>
class GpuTcpServer : public TcpEngine<Conf, ServerIConf<Conf>, Link, Backend, GpuTcpServer<Conf, Link, Backend>> {
  using Base = TcpEngine<Conf, ServerIConf<Conf>, Link, Backend, GpuTcpServer<Conf, Link, Backend>>;
  friend Base;

 public:
  using Conn = typename Base::Conn;
  static constexpr bool kClient = false;

  GpuTcpServer() = default;
  ~GpuTcpServer() { this->closeAll(); } // RSTs to open connections, as TcpServer's destructor

  // EfviTcpServer::init (EfviTcp.h:246-250): open the interface, listen on server_port.
  // server_ip is the address the server answers on (the NIC filter's local ip,
  // Core.h:335-383); nullptr or "0.0.0.0" takes the interface's address.
  bool init(const char* interface, const char* server_ip, uint16_t server_port) {
    if ((this->err_ = this->link_.open(interface))) return false;
    return setup(server_ip, server_port, Base::getns());
  }
  // The same over a link the caller has opened (a capture replay, a test peer, a ring fed
  // by another process); now_ns fixes the clock origin (0 = CLOCK_REALTIME).
  bool initWithLink(const char* server_ip, uint16_t server_port, int64_t now_ns = 0) {
    return setup(server_ip, server_port, now_ns ? now_ns : Base::getns());
  }

  const char* getLastError() { return this->err_; }
  void close(const char* reason) { // EfviTcp.h:252-255 / TcpServer::close
    if (reason) this->err_ = reason;
    this->closeAll();
  }
  bool isClosed() { return this->err_ != nullptr; }
  uint32_t getConnCnt() { return this->conn_cnt_; } // TcpServer.h:53 (SYN-RECEIVED included)
  template <class F>
  void foreachConn(F f) { // TcpServer.h:55-60
    for (auto& c : this->conns_)
      if (c.isEstablished()) f(c);
  }

  template <class Handler>
  void poll(Handler& handler, int64_t ns = 0) { // TcpServer::poll (TcpServer.h:70-112)
    if (!this->ready_) return;
    typename Base::template H<Handler> h{handler};
    this->pollEngine(h, ns ? ns : Base::getns());
  }

 private:
  bool setup(const char* server_ip, uint16_t server_port, int64_t now_ns) {
    if ((this->err_ = this->initEngine(server_ip, now_ns))) return false;
    port_be_ = htons(server_port);
    this->err_ = nullptr;
    return true;
  }
  // setServerFilter (Core.h:375-383): TCP to local_ip:port
  bool accepts(const uint8_t* eth) const {
    return std::memcmp(eth + 30, &this->local_ip_, 4) == 0 && std::memcmp(eth + 36, &port_be_, 2) == 0;
  }
  template <class HH>
  void onMiss(HH& h, uint64_t key, const pn_result& r, const uint8_t* eth) { // TcpServer.h:80-96
    if (r.flags & PN_F_RST) return;
    uint32_t src_ip;
    uint16_t src_port;
    std::memcpy(&src_ip, eth + 26, 4);
    std::memcpy(&src_port, eth + 34, 2);
    if ((r.flags & PN_F_ACK) || !(r.flags & PN_F_SYN) || this->conn_cnt_ == Base::kMaxConn ||
        !h.allow(src_ip, src_port)) {
      this->rspRst(eth, r);
      return;
    }
    Conn* c = this->newConn(key);
    this->resetConn(*c, key, eth + 6, src_ip, src_port, port_be_);
    this->onSyn(*c, eth, r);
    this->sendSyn(*c);
  }
  template <class HH>
  bool onHandshake(HH& h, Conn& c, const pn_result& r, const uint8_t* eth) { // SYN-RECEIVED, TcpServer.h:97-111
    if ((r.flags & PN_F_SYN) && !(r.flags & PN_F_ACK)) {
      this->resendUna(c);
      return false;
    }
    if ((r.flags & PN_F_RST) && Base::seqRaw(r) == c.rx_.ackSeq()) {
      this->onClose(c, false);
      return false;
    }
    if (!(r.flags & PN_F_ACK)) return false;
    if (Base::ackNum(eth) != c.next_seq_) {
      this->rspRst(eth, r);
      return false;
    }
    this->onEstablished(h, c, eth);
    return true;
  }

  uint16_t port_be_ = 0;
};

} // namespace pollnet_amd
