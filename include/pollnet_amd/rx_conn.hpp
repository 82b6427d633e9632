// rx_conn.hpp — the receive half of an efvitcp connection, driven by pn_result records.
//
// After pn_classify has parsed a frame on the GPU (payload offset/length, seq+syn,
// flags), everything efvitcp's TcpConn::onPack (efvitcp/TcpConn.h:466-769) still
// does with it is sequential per-connection state.  This class restates the part
// that belongs to the receiver, in the reference's order:
//   1. sequence acceptability + PAWS            TcpConn.h:475-497, 516-524
//   2. RST                                      TcpConn.h:526-531
//   5. "no ACK bit, no further processing"      TcpConn.h:533-535
//   7. segment text: out-of-order segment list, zero-copy delivery of in-order
//      data, leftovers ("remaining") kept in recv_buf, receive-window slide
//                                               TcpConn.h:667-750
//   8. FIN                                      TcpConn.h:752-762
//   ACK policy (immediate vs delayed)           TcpConn.h:764
// The ACK-field processing of step 5 (send window, una, RTT, congestion control),
// the send path and timers are the TX side's (out of scope): the
// caller learns what the TX side owes from the returned RxAck and tells this class
// when an ACK went out (ackSent()) and whether its own FIN was sent (setFinSent()).
//
// Handler (duck-typed, as the reference's):
//   uint32_t onData(RxConn&, const uint8_t* data, uint32_t size)  -> bytes NOT consumed
//   void     onFin(RxConn&, const uint8_t* data, uint32_t size)   (data still unconsumed)
//   void     onReset(RxConn&)                                      (RST, or recv buffer full)
//   void     onAckField(RxConn&, bool no_text)   optional: the point of step 5 where
//            the reference processes the ACK field (TcpConn.h:536-665), after the ACK
//            bit check and before the segment text; no_text = the segment occupies no
//            sequence space (its duplicate-ACK test, TcpConn.h:622).  A full TCP
//            endpoint (tcp_server.hpp) advances its send side here.
// Delivered pointers are zero-copy into the caller's frame when the segment is the
// next in-order one, else into recv_buf; valid only during the call (TcpConn.h:715).
#pragma once

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <type_traits>
#include <utility>

#include "../pollnet_amd.h"

// The per-segment path is a handful of small steps called once per frame; forced inline, it is one straight run
// of code per frame (the host dispatch).
#ifndef PN_HOT
#define PN_HOT __attribute__((always_inline))
#endif

namespace pollnet_amd {

namespace detail {
template <class H, class C, class = void>
struct has_on_ack_field : std::false_type {};
template <class H, class C>
struct has_on_ack_field<H, C, decltype(void(std::declval<H&>().onAckField(std::declval<C&>(), false)))>
    : std::true_type {};
} // namespace detail

// What the TX side owes after a segment.
struct RxAck {
  bool send = false;      // an ACK is owed (the reference's sendAck())
  bool immediate = false; // ... and may not be delayed (sendAck(true))
  bool rst = false;       // abort: recv buffer full of unconsumed data (close(): RST, TcpConn.h:96-105, 741-745)
};

template <class Conf>
class RxConn {
 public:
  static constexpr uint32_t kBufSize = Conf::ConnRecvBufSize;
  static constexpr uint32_t kMaxSegs = 5;    // TcpConn::MaxRecvSegs, TcpConn.h:909
  static constexpr uint32_t kRecvMSS = 1460; // Core.h:44

  // Received-data extents [first, second) relative to recvBufSeq(); segs()[0] is the
  // in-order run, its [first, second) the bytes held but not yet consumed.
  struct Seg {
    uint32_t first, second;
  };

  // A SYN was accepted (TcpConn::reset + onSyn, TcpConn.h:150-156, 351-356): stream
  // byte 0 is syn_seq + 1.  has_ts: timestamps negotiated, ts_val the SYN's TSval.
  void open(uint32_t syn_seq, bool has_ts = false, uint32_t ts_val = 0) {
    recv_buf_seq_ = syn_seq + 1;
    n_segs_ = 1;
    segs_[0] = {0, 0};
    fin_received_ = fin_sent_ = false;
    closed_ = false;
    pending_ack_ = true;
    has_ts_ = Conf::TimestampOption && has_ts;
    recent_ts_ = ts_val;
    last_ack_seq_ = recv_buf_seq_; // the SYN-ACK acknowledged the SYN
  }

  // A fresh connection before any SYN was received (TcpConn::reset, TcpConn.h:150-153): stream
  // offset 0, nothing owed, the ack field 0 — what a client's SYN carries.
  void resetRecv() {
    recv_buf_seq_ = 0;
    n_segs_ = 1;
    segs_[0] = {0, 0};
    fin_received_ = fin_sent_ = false;
    closed_ = false;
    pending_ack_ = false;
    has_ts_ = false;
    last_ack_seq_ = 0;
  }
  // The last ACK sent (a client's SYN carried ack 0 before the SYN-ACK set recv_buf_seq).
  void setLastAckSeq(uint32_t s) { last_ack_seq_ = s; }

  // TX side: an ACK carrying ackSeq() went out (TcpConn::updateLastAck, TcpConn.h:844-849).
  void ackSent() {
    pending_ack_ = false;
    last_ack_seq_ = ackSeq();
  }
  void setFinSent() { fin_sent_ = true; }

  uint32_t ackSeq() const { return recv_buf_seq_ + segs_[0].second; }
  // advertised window before scaling (getRecvWindowSize, TcpConn.h:301-307)
  uint32_t window() const { return kBufSize - segs_[0].second; }
  uint32_t recvBufSeq() const { return recv_buf_seq_; }
  const Seg* segs() const { return segs_; }
  uint32_t segCount() const { return n_segs_; }
  bool finReceived() const { return fin_received_; }
  bool pendingAck() const { return pending_ack_; }
  bool closed() const { return closed_; }
  uint32_t recentTs() const { return recent_ts_; }
  uint32_t lastAckSeq() const { return last_ack_seq_; } // the ack number last sent (updateLastAck)

  // The in-order fast path's state test (TcpEngine::inOrder): a segment of len > 0 payload bytes starting at seq is
  // exactly the next in-order data with nothing held, no hole, no FIN, no timestamps, and fits the buffer -- the case
  // onSegment hands to onData zero-copy without touching its extent list.
  bool inOrderReady(uint32_t seq, uint32_t len) const {
    return !closed_ && !fin_received_ && !hasTs() && n_segs_ == 1 && segs_[0].first == segs_[0].second &&
           seq == recv_buf_seq_ + segs_[0].second && len - 1 < kBufSize - segs_[0].second;
  }
  // onSegment for a segment that passed inOrderReady and whose ACK field changes nothing (the caller's proof): steps
  // 7 and the ACK policy only, as onSegment runs them for it (TcpConn.h:700-764).
  template <class Handler>
  PN_HOT RxAck onInOrder(Handler& h, const uint8_t* data, uint32_t n) {
    RxAck out;
    pending_ack_ = true;
    segs_[0].second += n;
    const uint32_t left = h.onData(*this, data, n);
    segs_[0].first = segs_[0].second - left;
    if (left) std::memcpy(recv_buf_ + segs_[0].first, data + n - left, left);
    slide();
    if (segs_[0].second == kBufSize) { // full of unconsumed data: cannot proceed
      h.onReset(*this);
      out.rst = true;
      close();
      return out;
    }
    if (pending_ack_) { // (a reply onData sent carried the ACK: ackSent() cleared it)
      out.send = true;
      out.immediate = ackSeq() - last_ack_seq_ >= 2 * rmss();
    }
    return out;
  }

  // One classified segment of this connection.  eth: the frame (host memory);
  // rec: its pn_result.
  template <class Handler>
  PN_HOT RxAck onSegment(Handler& h, const uint8_t* eth, const pn_result& rec) {
    RxAck out;
    if (closed_) return out;
    const bool fin = rec.flags & PN_F_FIN, rst = rec.flags & PN_F_RST;
    const uint8_t* data = eth + rec.payload_off;
    const uint32_t seq = rec.seq; // ntohl(seq_num) + syn

    bool got_ts = false;
    uint32_t tsval = 0;
    if (hasTs()) {
      got_ts = parse_ts(eth + 14 + 20 + 20, data, &tsval);
      if (got_ts && (int32_t)(seq - last_ack_seq_) <= 0 && (int32_t)(tsval - recent_ts_) >= 0) recent_ts_ = tsval;
    }

    // 1. acceptability: neither the first nor the last sequence number of the
    // segment (FIN counts) falls in [rcv_nxt, rcv_nxt + buffer) -> ACK and drop
    uint32_t loc = seq - recv_buf_seq_;
    uint32_t loc_end = loc + (uint32_t)(int32_t)rec.payload_len + (fin ? 1u : 0u);
    const uint32_t nxt = segs_[0].second;
    const bool start_out = (int32_t)(loc - nxt) < 0 || (int32_t)(loc - kBufSize) >= 0;
    const bool end_out = (int32_t)(loc_end - nxt) <= 0 || (int32_t)(loc_end - kBufSize) > 0;
    if ((start_out && end_out) || (Conf::TimestampOption && got_ts && (int32_t)(tsval - recent_ts_) < 0)) {
      out.send = !rst;
      return out;
    }
    // 2. RST
    if (rst) {
      if (!fin_sent_ || !fin_received_) h.onReset(*this);
      close();
      return out;
    }
    // 5. without ACK the segment goes no further (the ACK field itself is the TX side's)
    if (!(rec.flags & PN_F_ACK)) return out;
    if constexpr (detail::has_on_ack_field<Handler, RxConn>::value) h.onAckField(*this, loc == loc_end);

    // 7. segment text
    const int32_t behind = (int32_t)(loc - nxt);
    if (behind < 0) { // drop what was received already
      loc -= behind;
      data -= behind;
    }
    bool immediate = false;
    if (!fin_received_) {
      loc_end -= fin ? 1u : 0u;
      bool fin_ok = fin;
      if (loc_end > kBufSize) { // clipped at the buffer: the FIN is not in it
        loc_end = kBufSize;
        fin_ok = false;
      }
      const int32_t n = (int32_t)(loc_end - loc);
      if (n > 0) {
        pending_ack_ = true;
        if (n_segs_ > 1) immediate = true; // a hole existed
        uint32_t i = 0;
        if (n_segs_ == 1 && loc == segs_[0].second) segs_[0].second = loc_end; // in order, no hole: merge's result
        else if (merge(loc, loc_end, &i)) immediate = true;                   // a new hole was opened
        if (segs_[0].second != loc_end) fin_ok = false;
        if (segs_[0].first == loc && segs_[0].second == loc_end) {
          // exactly the next bytes and nothing pending: hand over the frame's own bytes
          const uint32_t left = h.onData(*this, data, (uint32_t)n);
          segs_[0].first = segs_[0].second - left;
          if (left) std::memcpy(recv_buf_ + segs_[0].first, data + n - left, left); // the common case keeps nothing
        } else {
          std::memcpy(recv_buf_ + loc, data, (uint32_t)n);
          if (i == 0) {
            const uint32_t left = h.onData(*this, recv_buf_ + segs_[0].first, segs_[0].second - segs_[0].first);
            segs_[0].first = segs_[0].second - left;
          }
        }
        slide();
        if (segs_[0].second == kBufSize) { // full of unconsumed data: cannot proceed
          h.onReset(*this);
          out.rst = true;
          close();
          return out;
        }
      } else if (loc != segs_[0].second) {
        fin_ok = false;
      }
      // 8. FIN
      if (fin_ok) {
        pending_ack_ = fin_received_ = true;
        immediate = true;
        segs_[0].second++; // the FIN occupies one sequence number
        h.onFin(*this, recv_buf_ + segs_[0].first, segs_[0].second - segs_[0].first - 1);
      }
    }
    if (pending_ack_) {
      out.send = true;
      out.immediate = immediate || ackSeq() - last_ack_seq_ >= 2 * rmss();
    }
    return out;
  }

 private:
  bool hasTs() const { return Conf::TimestampOption && has_ts_; }
  uint32_t rmss() const { return kRecvMSS - (hasTs() ? 12 : 0); } // getRMSS, TcpConn.h:408

  // TSval of a timestamp option in [opt, data) (TcpConn.h:475-494): the aligned
  // NOP,NOP,TS,10 layout first, else a walk over the options.
  static bool parse_ts(const uint8_t* opt, const uint8_t* data, uint32_t* tsval) {
    auto be32 = [](const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; };
    if (opt + 12 <= data && be32(opt) == 0x0101080a) {
      *tsval = be32(opt + 4);
      return true;
    }
    while (opt + 10 <= data) {
      const uint8_t kind = *opt++;
      if (kind <= 1) continue;
      const uint8_t len = *opt++;
      if (kind == 8 && len == 10) {
        *tsval = be32(opt);
        return true;
      }
      if (len > 2) opt += len - 2;
    }
    return false;
  }

  // Insert [b, e) into the ordered extent list, merging what it touches.  *first_idx
  // = the extent it landed in.  Returns true when it opened a new hole (TcpConn.h:685-711:
  // a new extent is dropped when kMaxSegs extents precede it, else the last one is
  // evicted to make room).
  bool merge(uint32_t b, uint32_t e, uint32_t* first_idx) {
    uint32_t i = 0;
    while (i < n_segs_ && segs_[i].second < b) ++i;
    uint32_t j = i;
    while (j < n_segs_ && segs_[j].first <= e) ++j;
    *first_idx = i;
    if (i == j) {
      if (i >= kMaxSegs) return false;
      if (n_segs_ == kMaxSegs) --n_segs_;
      std::copy_backward(segs_ + i, segs_ + n_segs_, segs_ + n_segs_ + 1);
      segs_[i] = {b, e};
      ++n_segs_;
      return true;
    }
    segs_[i].first = std::min(segs_[i].first, b);
    segs_[i].second = std::max(segs_[j - 1].second, e);
    if (j > i + 1) { // extents i+1 .. j-1 were swallowed
      std::copy(segs_ + j, segs_ + n_segs_, segs_ + i + 1);
      n_segs_ -= j - i - 1;
    }
    return false;
  }

  // Advance the window once at least one RMSS was consumed (receiver-side SWS
  // avoidance, TcpConn.h:726-740): rebase to 0 when nothing is held, else shift the
  // held bytes down once half the buffer is consumed.
  PN_HOT void slide() {
    const uint32_t consumed = segs_[0].first;
    if (consumed < rmss()) return;
    if (consumed == segs_[n_segs_ - 1].second) {
      recv_buf_seq_ += consumed;
      segs_[0] = {0, 0};
    } else if (consumed >= kBufSize / 2) {
      std::memmove(recv_buf_, recv_buf_ + consumed, segs_[n_segs_ - 1].second - consumed);
      recv_buf_seq_ += consumed;
      for (uint32_t k = 0; k < n_segs_; ++k) {
        segs_[k].first -= consumed;
        segs_[k].second -= consumed;
      }
    }
  }

  void close() { // TcpConn::onClose (TcpConn.h:451-465), receive side
    fin_received_ = fin_sent_ = true;
    closed_ = true;
  }

  uint32_t recv_buf_seq_ = 0;
  uint32_t n_segs_ = 1;
  Seg segs_[kMaxSegs] = {};
  uint32_t last_ack_seq_ = 0;
  uint32_t recent_ts_ = 0;
  bool fin_received_ = true, fin_sent_ = true, closed_ = true; // a fresh object is closed until open()
  bool pending_ack_ = false, has_ts_ = false;
  uint8_t recv_buf_[kBufSize];
};

} // namespace pollnet_amd
