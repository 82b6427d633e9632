// Test-only harness: the reference's own efvitcp TCP endpoint, compiled from the text of
// /root/reference extracted at build time (oracle/ref.mk, target `conn` -> oracle/_ref/conn_*.inc,
// git-ignored; no reference text is kept in the repository):
//   conn_tcpconn.inc        TcpConn.h:29-914    class TcpConn, whole (onPack, onTimer, send path, ...)
//   conn_tcpserver.inc      TcpServer.h:29-121  class TcpServer, whole (its poll's recv handler)
//   conn_efvitcpserver.inc  EfviTcp.h:188-313   pollnet's EfviTcpServer wrapper, whole
//   conn_tcpclient_*.inc    TcpClient.h:30-104, 166-168  class TcpClient less getDestMac
//   conn_efvitcpclient.inc  EfviTcp.h:30-186    pollnet's EfviTcpClient wrapper, whole
//   conn_timer_types.inc    Core.h:184-214      TimerNode, TimeWaitConn
//   conn_sendbuf.inc        Core.h:150-163      SendBuf's members after its ef_addr
//   conn_core_*.inc         Core.h:232-236, 290-291 + 293-322, 327-331, 385-446, 504-527, 554-682,
//                           357-373, 684-751, 753-762 + 769-782: every Core member that touches no
//                           ef_vi type
//   core_defs.inc           Core.h:44-138, 167-182  constants, header structs, CSum, connHashKey
// The one thing not taken from the reference is what needs ef_vi (not installed; no stand-in
// headers are written for it): the harness Core below restates
//   - Core::init's driver / NIC calls (Core.h:253-289): the local address, MAC and clock come
//     from RefEnv (the test's link and its clock) instead of ioctl / ef_vi, the receive prefix is 0;
//   - Core::send (Core.h:474-492): the frame goes to RefEnv's link; its TX completion is taken as
//     immediate (the buffer stays `avail`, the state Core.h:540-547 returns it to), or, with
//     RefEnv::tx_complete_next_poll, arrives with the next pollNet (`avail` false until then);
//   - Core::pollNet's event loop (Core.h:494-552): up to 64 frames (ef_eventq_poll's 64 events,
//     :498) are taken from the link into the RX slots, and each runs the reference's own RX body
//     (:504-527);
//   - setServerFilter / setClientFilter / delFilter (Core.h:333-355, 375-383): the test link only
//     carries the endpoint's own flow (setClientFilter keeps its port choice, autoGetPort, :337-342);
//   - TcpClient::getDestMac (TcpClient.h:105-164, the host's route and ARP tables): RefEnv's peer MAC;
//   - EfviTcpClient::poll's reconnect clock `time(0)` (EfviTcp.h:116): efvitcp::time below reads the
//     test's clock (RefEnv::now_ns), so the wrapper's reconnect interval runs on the polls' time.
// Each Core keeps the RefEnv current at its init (a client and a server can share a process).
// RecvBuf / SendBuf keep the reference layout with their ef_addr as a plain 8-byte member.
// Built without EFVITCP_DEBUG, as pollnet ships it.  Nothing here is shipped or used by the
// product; tests/cpp/test_ref_conn.cpp and test_ref_server.cpp compare the product against it.
#pragma once

#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <limits>
#include <string>
#include <utility>
#include <vector>

namespace efvitcp {
using std::cout;
using std::endl;
#include "_ref/core_defs.inc"

#pragma pack(push, 1)
struct RecvBuf { // Core.h:141-145
  uint64_t post_addr;
  uint16_t __pad;
};
struct SendBuf { // Core.h:147-164
  uint64_t post_addr;
#include "_ref/conn_sendbuf.inc"
};
#pragma pack(pop)

#include "_ref/conn_timer_types.inc"

// Where the harness Core's restated ef_vi parts go: the test's link and clock.
struct RefEnv {
  void* link = nullptr;
  // frames into the RX slots (stride, frame offset, at most cap); returns how many
  uint32_t (*fill)(void* link, uint8_t* slots, uint32_t stride, uint32_t off, uint32_t cap) = nullptr;
  void (*send)(void* link, const uint8_t* eth, uint32_t len) = nullptr;
  int64_t init_ns = 0;    // Core::init's clock (now_ts = ns >> TsScale)
  uint32_t local_ip = 0;  // network order
  uint8_t local_mac[6] = {};
  uint8_t peer_mac[6] = {}; // TcpClient::getDestMac's answer
  int64_t now_ns = 0;       // the test's clock, for EfviTcpClient's time(0)
  // false: every TX completion is immediate (a sent buffer stays `avail`);
  // true: completions arrive with the next pollNet (Core.h:491 clears `avail`, :540-547 sets it back)
  bool tx_complete_next_poll = false;
  bool wall_clock_time = false; // time(0) as the reference has it: the host's wall clock
};
inline RefEnv& refEnv() {
  static RefEnv e;
  return e;
}
inline time_t time(time_t* t) {
  return refEnv().wall_clock_time ? ::time(t) : (time_t)(refEnv().now_ns / 1000000000);
}

template<typename Conf>
class Core
{
public:
#include "_ref/conn_core_consts.inc"

  Core() = default;
  Core(const Core&) = delete;
  Core& operator=(const Core&) = delete;

  const char* init(const char*) {
    env_ = refEnv();
    const RefEnv& env = env_;
    now_ts = env.init_ns >> TsScale;
    local_ip = env.local_ip;
    std::memcpy(local_mac, env.local_mac, 6);
    receive_prefix_len = 0;
    pkt_buf = (uint8_t*)((uint64_t)(pkt_buf_blk + TotalBufAlign) & ~(TotalBufAlign - 1));
#include "_ref/conn_core_init.inc"
    return nullptr;
  }

#include "_ref/conn_core_getns.inc"

  void delFilter() {}
  const char* setServerFilter(uint16_t) { return nullptr; }
  const char* setClientFilter(uint16_t& local_port_be, uint32_t, uint16_t) {
    if (local_port_be == 0) return autoGetPort(local_port_be);
    return nullptr;
  }
#include "_ref/conn_core_autoport.inc"

#include "_ref/conn_core_rst.inc"

  void send(SendBuf* buf) {
    const uint32_t frame_len = 14 + ntohs(buf->ip_hdr.tot_len);
    const RefEnv& env = env_;
    env.send(env.link, (const uint8_t*)&buf->eth_hdr, frame_len);
    if (env.tx_complete_next_poll) {
      buf->avail = false;
      tx_queued_.push_back(buf);
    }
  }

  template<typename RecvHandler>
  void pollNet(RecvHandler recv_handler) {
    const RefEnv& env = env_;
    for (SendBuf* b : tx_queued_) b->avail = true; // the TX completion events of the last poll's frames
    tx_queued_.clear();
    const uint32_t n = env.fill(env.link, pkt_buf, RecvBufSize, sizeof(RecvBuf) + receive_prefix_len,
                                std::min<uint32_t>(64, Conf::RecvBufCnt));
    for (uint32_t id = 0; id < n; id++) {
#include "_ref/conn_core_rx.inc"
    }
  }

#include "_ref/conn_core_tbl.inc"
#include "_ref/conn_core_timer.inc"
#include "_ref/conn_core_members.inc"
  RefEnv env_;
  std::vector<SendBuf*> tx_queued_;
};

#include "_ref/conn_tcpconn.inc"
#include "_ref/conn_tcpserver.inc"
#include "_ref/conn_efvitcpserver.inc"

#include "_ref/conn_tcpclient_head.inc"
  const char* getDestMac(const char*, uint8_t* dest_mac) {
    std::memcpy(dest_mac, core.env_.peer_mac, 6);
    return nullptr;
  }
#include "_ref/conn_tcpclient_tail.inc"
#include "_ref/conn_efvitcpclient.inc"

} // namespace efvitcp
