// tcp_client.hpp — GpuTcpClient<Conf>: pollnet's TCP client surface over the GPU RX/TX paths.
//
// A drop-in for pollnet's EfviTcpClient<Conf> (/root/reference/efvitcp/EfviTcp.h:11-173):
//   bool init(const char* interface, const char* server_ip, uint16_t server_port, uint16_t local_port = 0);
//   const char* getLastError();  bool isConnected();  void close(const char* reason);
//   int writeSome(data, size, more);  bool writeNonblock(data, size, more);  void allowReconnect();
//   template <class Handler> void poll(Handler& handler, int64_t ns = 0);
//   Conn& conn;                                   (the one connection, EfviTcp.h:170)
// Handler callbacks, found by name (EfviTcp.h:107-147; README.md:81-104):
//   uint32_t onTcpData(Conn&, const uint8_t*, uint32_t)   required
//   void onTcpConnectFailed(), onTcpConnected(Conn&), onTcpDisconnect(Conn&),
//        onSendTimeout(Conn&), onRecvTimeout(Conn&)        optional
// so a handler written for EfviTcpClient (example/tcpclient.cc) compiles unchanged.
//
// poll(): while the connection is closed, a connect is attempted at most every
// Conf::ConnRetrySec seconds (0: once; EfviTcp.h:92-104) — a SYN with the MSS option to the
// server, from local_port (0: an ephemeral port the kernel hands out, Core::autoGetPort); a
// failure to start one reports onTcpConnectFailed.  Then TcpEngine's poll (tcp_engine.hpp)
// with the client's branches (TcpClient.h:78-100): frames that pass the 5-tuple filter but
// miss the table get an RST; in SYN-SENT the segment must acknowledge the SYN (else RST), an
// RST means "connection refused" (onTcpConnectFailed), a SYN-ACK establishes the connection
// and goes on to onPack.  The retry clock is the poll's `ns` when given (the reference reads
// time(0)), so a test can drive it.
#pragma once

#include <limits>

#include "tcp_engine.hpp"

namespace pollnet_amd {

// EfviTcpClient's ClientConf (EfviTcp.h:15-36), as the engine and RxConn read it.
template <class Conf>
struct ClientIConf {
  static const uint32_t ConnRecvBufSize = Conf::RecvBufSize;
  static const uint32_t MaxConnCnt = 1;
  static const uint32_t MaxTimeWaitConnCnt = 1;
  static const bool TimestampOption = false;
};

template <class Conf, class Link = SocketLink, class Backend = GpuBackend>
class GpuTcpClient : public TcpEngine<Conf, ClientIConf<Conf>, Link, Backend, GpuTcpClient<Conf, Link, Backend>> {
  using Base = TcpEngine<Conf, ClientIConf<Conf>, Link, Backend, GpuTcpClient<Conf, Link, Backend>>;
  friend Base;

 public:
  using Conn = typename Base::Conn;
  static constexpr bool kClient = true;

  GpuTcpClient() : conn(this->conns_[0]) {}
  ~GpuTcpClient() { this->closeAll(); }

  const char* getLastError() { return conn.err_; }
  bool isConnected() { return conn.isEstablished(); }

  // EfviTcpClient::init (EfviTcp.h:82-89): open the interface; the connection is made by poll().
  bool init(const char* interface, const char* server_ip, uint16_t server_port, uint16_t local_port = 0) {
    if ((conn.err_ = this->link_.open(interface))) return false;
    return setup(nullptr, server_ip, server_port, local_port, Base::getns());
  }
  // The same over a link the caller has opened; local_ip names this end (nullptr: the
  // link's address), now_ns fixes the clock origin (0 = CLOCK_REALTIME).
  bool initWithLink(const char* local_ip, const char* server_ip, uint16_t server_port, uint16_t local_port = 0,
                    int64_t now_ns = 0) {
    return setup(local_ip, server_ip, server_port, local_port, now_ns ? now_ns : Base::getns());
  }

  int writeSome(const void* data, uint32_t size, bool more = false) { return conn.writeSome(data, size, more); }
  bool writeNonblock(const void* data, uint32_t size, bool more = false) { return conn.writeNonblock(data, size, more); }
  void close(const char* reason) { conn.close(reason); }
  void allowReconnect() { next_conn_ts_ = 0; }

  template <class Handler>
  void poll(Handler& handler, int64_t ns = 0) { // EfviTcpClient::poll (EfviTcp.h:91-148)
    if (!this->ready_) return;
    typename Base::template H<Handler> h{handler};
    const int64_t now = ns ? ns : Base::getns();
    if (conn.isClosed()) {
      const int64_t now_s = now / 1000000000;
      if (now_s >= next_conn_ts_) {
        constexpr uint32_t retry = srv_detail::opt_ConnRetrySec<Conf>::value;
        next_conn_ts_ = retry ? now_s + retry : std::numeric_limits<int64_t>::max(); // 0: no reconnect
        if ((conn.err_ = connect())) h.connectFailed();
      }
    }
    this->pollEngine(h, now);
  }

  Conn& conn;

 private:
  bool setup(const char* local_ip, const char* server_ip, uint16_t server_port, uint16_t local_port, int64_t now_ns) {
    if ((conn.err_ = this->initEngine(local_ip, now_ns))) return false;
    in_addr a;
    if (!server_ip || inet_pton(AF_INET, server_ip, &a) != 1) return (conn.err_ = "invalid server_ip"), false;
    server_ip_ = a.s_addr;
    server_port_ = htons(server_port);
    local_port_ = htons(local_port);
    next_conn_ts_ = 0;
    conn.err_ = nullptr;
    return true;
  }

  // TcpClient::connect (TcpClient.h:50-72): next hop's MAC, the local port, the SYN, the entry.
  const char* connect() {
    if (this->conn_cnt_) return "Connection already exists";
    uint8_t mac[6];
    if (const char* e = this->link_.resolveMac(server_ip_, mac)) return e;
    uint16_t lp = local_port_;
    if (!lp) {
      if (const char* e = autoGetPort(&lp)) return e;
    }
    cur_local_port_ = lp;
    const uint64_t key = pn_conn_hash_key(server_ip_, server_port_);
    Conn* c = this->newConn(key);
    this->resetConn(*c, key, mac, server_ip_, server_port_, lp);
    this->sendSyn(*c);
    return nullptr;
  }
  // Core::autoGetPort (Core.h:357-371): an ephemeral port bound and released through the kernel.
  const char* autoGetPort(uint16_t* port) {
    const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) return "socket failed";
    sockaddr_in sa;
    std::memset(&sa, 0, sizeof sa);
    sa.sin_family = AF_INET;
    sa.sin_addr.s_addr = this->local_ip_;
    if (::bind(fd, (sockaddr*)&sa, sizeof sa) < 0) { // the link's address may not be the kernel's
      sa.sin_addr.s_addr = INADDR_ANY;
      if (::bind(fd, (sockaddr*)&sa, sizeof sa) < 0) {
        ::close(fd);
        return "bind failed";
      }
    }
    socklen_t len = sizeof sa;
    getsockname(fd, (sockaddr*)&sa, &len);
    ::close(fd);
    *port = sa.sin_port;
    return nullptr;
  }

  // setClientFilter (Core.h:335-355): the full 5-tuple of the connection
  bool accepts(const uint8_t* eth) const {
    return std::memcmp(eth + 30, &this->local_ip_, 4) == 0 && std::memcmp(eth + 36, &cur_local_port_, 2) == 0 &&
           std::memcmp(eth + 26, &server_ip_, 4) == 0 && std::memcmp(eth + 34, &server_port_, 2) == 0;
  }
  template <class HH>
  void onMiss(HH&, uint64_t, const pn_result& r, const uint8_t* eth) { // TcpClient.h:82-85
    this->rspRst(eth, r);
  }
  template <class HH>
  bool onHandshake(HH& h, Conn& c, const pn_result& r, const uint8_t* eth) { // SYN-SENT, TcpClient.h:86-98
    const bool ack_ok = (r.flags & PN_F_ACK) && Base::ackNum(eth) == c.next_seq_;
    if (!ack_ok) {
      this->rspRst(eth, r);
      return false;
    }
    if (r.flags & PN_F_RST) { // onConnectionRefused (EfviTcp.h:107-110)
      c.err_ = "connection refused";
      h.connectFailed();
      this->onClose(c, false);
      return false;
    }
    if (!(r.flags & PN_F_SYN)) return false;
    this->onSyn(c, eth, r);
    c.rx_.setLastAckSeq(0); // the SYN went out with ack 0 (TcpConn::reset + updateLastAck)
    this->onEstablished(h, c, eth);
    return true;
  }

  uint32_t server_ip_ = 0;
  uint16_t server_port_ = 0, local_port_ = 0, cur_local_port_ = 0;
  int64_t next_conn_ts_ = 0;
};

} // namespace pollnet_amd
