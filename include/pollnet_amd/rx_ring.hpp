// rx_ring.hpp — getting received frames into the layouts pn_classify /
// pn_classify_indexed read (RX-ring ingestion).
//
//  EfviRingLayout   ef_vi's receive ring as efvitcp lays it out: RecvBufCnt slots of
//                   RecvBufSize = 2048 B (Core.h:45), each a RecvBuf header
//                   {ef_addr post_addr; uint16_t __pad} (10 B, Core.h:140-145) then
//                   receive_prefix_len NIC-prefix bytes (Core.h:285) then the frame;
//                   RX events name slots by id (Core.h:503-505).  The ring is
//                   classified where the NIC wrote it: hipHostRegister it once, then
//                   GpuRx/GpuTcpRx::pollIndexed(ring, offsets(ids), ...).
//  SocketEthBatcher pollnet's SocketEthReceiver (Socket.h:567-629): an AF_PACKET
//                   SOCK_RAW ETH_P_ALL socket, non-blocking, bound to an interface,
//                   optionally promiscuous; instead of one read() into one buffer per
//                   call it drains the socket into consecutive slots of a pinned batch
//                   (recvmmsg, up to `cap` frames per call), recording each frame's
//                   received length.  Frames longer than a slot are cut at the slot as
//                   the reference's read(fd, buf, RecvBufSize) cuts them.
#pragma once

#include <errno.h>
#include <fcntl.h>
#include <linux/if_packet.h>
#include <net/ethernet.h>
#include <net/if.h>
#include <sys/socket.h>
#include <unistd.h>

#include <arpa/inet.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

namespace pollnet_amd {

struct EfviRingLayout {
  static constexpr uint32_t kRecvBufSize = 2048; // Core.h:45
  static constexpr uint32_t kRecvBufHdr = 10;    // sizeof(RecvBuf), packed (Core.h:140-145)
  uint32_t prefix_len = 0;                       // ef_vi_receive_prefix_len(&vi) (Core.h:285)

  uint32_t frame_off() const { return kRecvBufHdr + prefix_len; } // Core.h:505
  uint32_t eth_mod16() const { return frame_off() % 16; }
  uint32_t avail() const { return kRecvBufSize - frame_off(); }
  uint64_t offset(uint32_t id) const { return (uint64_t)id * kRecvBufSize + frame_off(); }
  // offsets of a run of RX event ids (event order; wraps and gaps as the events have them)
  void offsets(const uint32_t* ids, uint32_t n, uint64_t* out) const {
    for (uint32_t i = 0; i < n; i++) out[i] = offset(ids[i]);
  }
};

class SocketEthBatcher {
 public:
  SocketEthBatcher() = default;
  SocketEthBatcher(const SocketEthBatcher&) = delete;
  SocketEthBatcher& operator=(const SocketEthBatcher&) = delete;
  ~SocketEthBatcher() { close("destruct"); }

  // SocketEthReceiver::init (Socket.h:570-605); false + getLastError() on failure.
  bool init(const char* interface, bool promiscuous = false) {
    fd_ = socket(AF_PACKET, SOCK_RAW, htons(ETH_P_ALL));
    if (fd_ < 0) return fail("socket error");
    if (!nonblock()) return false;
    sockaddr_ll sa;
    std::memset(&sa, 0, sizeof(sa));
    sa.sll_family = PF_PACKET;
    sa.sll_ifindex = (int)if_nametoindex(interface);
    sa.sll_protocol = htons(ETH_P_ALL);
    if (bind(fd_, (sockaddr*)&sa, sizeof(sa)) < 0) return close("bind error"), false;
    if (promiscuous) {
      packet_mreq mreq;
      std::memset(&mreq, 0, sizeof(mreq));
      mreq.mr_ifindex = (int)if_nametoindex(interface);
      mreq.mr_type = PACKET_MR_PROMISC;
      if (setsockopt(fd_, SOL_PACKET, PACKET_ADD_MEMBERSHIP, &mreq, sizeof(mreq)) < 0)
        return close("setsockopt PACKET_ADD_MEMBERSHIP"), false;
    }
    return true;
  }
  // Kernel-side queue for bursts between fills (SO_RCVBUF; capped by net.core.rmem_max).
  bool setRecvBuffer(int bytes) {
    if (setsockopt(fd_, SOL_SOCKET, SO_RCVBUF, &bytes, sizeof bytes) < 0) return fail("setsockopt SO_RCVBUF");
    return true;
  }
  // Any message-preserving socket (a SOCK_SEQPACKET / SOCK_DGRAM pair in tests).
  bool initFd(int fd) {
    fd_ = fd;
    return nonblock();
  }

  // Drain up to `cap` frames into slots + i*stride + frame_off (i = 0..); lens[i] =
  // bytes received (cut at stride - frame_off).  Returns the number of frames; 0 when
  // nothing was pending.
  uint32_t fill(uint8_t* slots, uint32_t stride, uint32_t frame_off, uint32_t cap, uint32_t* lens = nullptr) {
    uint32_t got = 0;
    while (got < cap && fd_ >= 0) {
      const uint32_t want = std::min<uint32_t>(cap - got, kVec);
      for (uint32_t i = 0; i < want; i++) {
        iov_[i].iov_base = slots + (size_t)(got + i) * stride + frame_off;
        iov_[i].iov_len = stride - frame_off;
        std::memset(&msg_[i], 0, sizeof(mmsghdr));
        msg_[i].msg_hdr.msg_iov = &iov_[i];
        msg_[i].msg_hdr.msg_iovlen = 1;
      }
      const int r = recvmmsg(fd_, msg_, want, MSG_DONTWAIT, nullptr);
      if (r <= 0) {
        if (r < 0 && errno != EAGAIN && errno != EWOULDBLOCK) saveError("recvmmsg error");
        break;
      }
      for (int i = 0; i < r; i++)
        if (lens) lens[got + i] = msg_[i].msg_len;
      got += (uint32_t)r;
      if ((uint32_t)r < want) break; // drained
    }
    return got;
  }

  const char* getLastError() const { return last_error_; }
  bool isClosed() const { return fd_ < 0; }
  int fd() const { return fd_; }
  void close(const char* reason) {
    if (fd_ >= 0) {
      saveError(reason);
      ::close(fd_);
      fd_ = -1;
    }
  }

 private:
  static constexpr uint32_t kVec = 1024;
  bool nonblock() {
    const int flags = fcntl(fd_, F_GETFL, 0);
    if (flags < 0 || fcntl(fd_, F_SETFL, flags | O_NONBLOCK) < 0) return close("fcntl O_NONBLOCK error"), false;
    return true;
  }
  bool fail(const char* msg) {
    saveError(msg);
    return false;
  }
  void saveError(const char* msg) { std::snprintf(last_error_, sizeof(last_error_), "%s %s", msg, std::strerror(errno)); }

  int fd_ = -1;
  iovec iov_[kVec];
  mmsghdr msg_[kVec];
  char last_error_[64] = "";
};

} // namespace pollnet_amd
