// gpu_tcp_rx.hpp — the receive side of a GPU-classified TCP server: batch in, onTcpData out.
//
// The reference's server loop (efvitcp/TcpServer.h:70-112 over Core::pollNet,
// Core.h:494-552, wrapped by pollnet's EfviTcpServer::poll, efvitcp/EfviTcp.h:263-309)
// per RX frame: key -> conn table -> TIME_WAIT / unknown flow / connection ->
// TcpConn::onPack -> handler.onTcpData.  Here one pn_classify launch does the
// per-frame part for a whole batch (parse, checksums, table probe, payload
// extent) and poll() walks the records in ring order on the host:
//   - TIME_WAIT hit                    -> handler.onTimeWaitSegment(key, tw_id, eth, rec)
//   - unknown flow (miss)              -> handler.onNewSegment(key, eth, rec)
//     (the control plane: a SYN it accepts becomes a connection via accept())
//   - connection                        -> RxConn::onSegment (rx_conn.hpp), whose
//     callbacks are adapted as EfviTcp.h's TmpHandler does:
//       onData  -> handler.onTcpData(conn, data, size)            (returns bytes left)
//       onFin   -> onTcpData(conn, data, size) if size, then onTcpDisconnect(conn)
//       onReset -> onTcpDisconnect(conn)
//     and the ACK the TX side owes -> handler.onAckOwed(conn, RxAck)
// Handler surface (duck-typed, pollnet's names where they exist):
//   uint32_t onTcpData(Conn&, const uint8_t* data, uint32_t size);
//   void onTcpDisconnect(Conn&);
//   void onAckOwed(Conn&, const RxAck&);
//   void onNewSegment(uint64_t key, const uint8_t* eth, const pn_result& rec);
//   void onTimeWaitSegment(uint64_t key, uint32_t tw_id, const uint8_t* eth, const pn_result& rec);
// (GpuTcpServer, tcp_server.hpp, builds pollnet's own surface on the same records and
// decides the TIME_WAIT and unknown-flow branches itself; this class leaves them to the
// caller's control plane.)
//
// Table changes made during a poll (accept()/remove()/enterTW() from a callback) are
// seen by the records after them, as in the reference's sequential loop: once the
// host table diverges from the snapshot the batch was classified against, the
// remaining records of that batch are re-resolved on the host (6 header bytes + one
// ordered probe each); the next poll() re-snapshots the table to the device.
//
// Checksums: the reference's release build does not verify them (Core::checksum is
// EFVITCP_DEBUG-only, Core.h:448-472); setDropBadChecksum(true) drops frames whose
// IP or TCP verdict (reference semantics) failed before any state is touched.
#pragma once

#include <cstdint>
#include <cstring>
#include <vector>

#include "gpu_rx.hpp"
#include "rx_conn.hpp"

namespace pollnet_amd {

template <class Conf>
class GpuTcpRx {
 public:
  struct Conn : RxConn<Conf> {
    uint64_t key = 0;
    uint32_t id = 0;
    const char* err = nullptr; // why it closed (EfviTcp.h's conn.err_), nullptr while open
    bool live = false;         // holds a conn-table entry
    bool isClosed() const { return err != nullptr; }
  };

  GpuTcpRx() : conns_(Conf::MaxConnCnt) {}

  // device / ring layout / chunk / mode as GpuRx::init; the table holds MaxConnCnt
  // connections and MaxTimeWaitConnCnt TIME_WAIT entries (Core.h:780-781).
  // reference_literal: the conn table keeps the reference's rehash as is (PN_TABLE_REFERENCE_LITERAL).
  const char* init(int device, uint32_t slot_stride, uint32_t frame_off, uint32_t max_batch,
                   GpuRx::Mode mode = GpuRx::Mode::Copy, bool reference_literal = false) {
    const char* e = table_.init(Conf::MaxConnCnt, Conf::MaxTimeWaitConnCnt, reference_literal);
    if (e) return e;
    if ((e = rx_.init(device, slot_stride, frame_off, max_batch, mode))) return e;
    free_.clear();
    for (uint32_t i = Conf::MaxConnCnt; i-- > 0;) free_.push_back(i);
    free_tw_.clear();
    for (uint32_t i = Conf::MaxTimeWaitConnCnt; i-- > 0;) free_tw_.push_back(i);
    tw_keys_.assign(Conf::MaxTimeWaitConnCnt, PN_EMPTY_KEY);
    dirty_ = true;
    return nullptr;
  }
  void setDropBadChecksum(bool drop) { drop_bad_ = drop; }
  // Whether classify verifies the TCP checksum (pn_set_verify; default on).  Off, the records carry no TCP
  // verdict and the kernel reads only each frame's header lines — the reference's release path; then
  // setDropBadChecksum(true) has no TCP verdict to act on.
  const char* setVerify(bool v) { return pn_set_verify(rx_.ctx(), v ? 1 : 0) ? pn_last_error(rx_.ctx()) : nullptr; }

  // Control plane: a SYN from `key` was accepted (TcpServer.h:85-96 + TcpConn::onSyn).
  Conn* accept(uint64_t key, uint32_t syn_seq, bool has_ts = false, uint32_t ts_val = 0) {
    if (free_.empty()) return nullptr;
    const uint32_t id = free_.back();
    if (table_.add(key, id) != PN_OK) return nullptr;
    free_.pop_back();
    Conn& c = conns_[id];
    c.open(syn_seq, has_ts, ts_val);
    c.key = key;
    c.id = id;
    c.err = nullptr;
    c.live = true;
    ++conn_cnt_;
    dirty_ = true;
    return &c;
  }
  // Drop the connection's table entry (Core::delConnEntry, Core.h:578-598).
  void remove(Conn& c) {
    if (c.live && table_.del(c.key) == PN_OK) {
      c.live = false;
      free_.push_back(c.id);
      --conn_cnt_;
      dirty_ = true;
    }
  }
  // The connection enters TIME_WAIT (Core::enterTW, Core.h:607-638): its entry is relabelled
  // MaxConnCnt + tw_id with a TIME_WAIT id taken here.  Returns the tw_id; when all
  // MaxTimeWaitConnCnt ids are taken the entry is deleted instead, as the reference does
  // (Core.h:608-611), and PN_EFULL is returned.  PN_ENOENT: the connection holds no entry.
  int enterTW(Conn& c) {
    if (!c.live) return PN_ENOENT;
    if (free_tw_.empty()) {
      remove(c);
      return PN_EFULL;
    }
    const uint32_t tw_id = free_tw_.back();
    const int rc = table_.enterTW(c.key, tw_id);
    if (rc != PN_OK) return rc;
    free_tw_.pop_back();
    tw_keys_[tw_id] = c.key;
    c.live = false;
    free_.push_back(c.id);
    --conn_cnt_;
    dirty_ = true;
    return (int)tw_id;
  }
  // A TIME_WAIT entry ends (Core::delConnEntry on an in-sequence RST, Core.h:513-517, or
  // when the TIME_WAIT timer fires, Core.h:740-744): the key is free for a new SYN.  The
  // snapshot is marked stale, so later records of the same poll are re-resolved.
  int removeTW(uint32_t tw_id) {
    if (tw_id >= Conf::MaxTimeWaitConnCnt || tw_keys_[tw_id] == PN_EMPTY_KEY) return PN_ENOENT;
    const int rc = table_.del(tw_keys_[tw_id]);
    if (rc != PN_OK) return rc;
    tw_keys_[tw_id] = PN_EMPTY_KEY;
    free_tw_.push_back(tw_id);
    dirty_ = true;
    return PN_OK;
  }
  uint32_t getTimeWaitCnt() const { return Conf::MaxTimeWaitConnCnt - (uint32_t)free_tw_.size(); }

  uint32_t getConnCnt() const { return conn_cnt_; } // EfviTcp.h:256
  template <class F>
  void foreachConn(F f) { // EfviTcp.h:258-261
    for (Conn& c : conns_)
      if (c.live) f(c);
  }
  const ConnTable& table() const { return table_; } // changes go through accept/remove/enterTW/removeTW
  GpuRx& rx() { return rx_; }

  // Classify n ring slots (host memory) on the GPU and dispatch them in ring order.
  // The table snapshot is refreshed here, never while a chunk is in flight; chunks
  // classified before a change made during this poll are re-resolved on the host.
  template <class Handler>
  const char* poll(Handler& h, const uint8_t* slots, uint32_t n) {
    if (const char* e = refresh()) return e;
    Dispatch<Handler> d{this, h};
    return rx_.pollBatch(
        slots, n, table_, [&](uint64_t key, const pn_result& r, const uint8_t* eth, uint32_t) { d(key, r, eth); },
        [&](uint64_t key, uint32_t, const uint8_t* eth, const pn_result& r) { d(key, r, eth); });
  }
  // The same over RX events (GpuRx::pollIndexed: ZeroCopy mode, frame i at ring + offsets[i]).
  template <class Handler>
  const char* pollIndexed(Handler& h, const uint8_t* ring, const uint64_t* offsets, uint32_t n, uint32_t eth_mod16,
                          uint32_t avail) {
    if (const char* e = refresh()) return e;
    Dispatch<Handler> d{this, h};
    return rx_.pollIndexed(
        ring, offsets, n, eth_mod16, avail, table_,
        [&](uint64_t key, const pn_result& r, const uint8_t* eth, uint32_t) { d(key, r, eth); },
        [&](uint64_t key, uint32_t, const uint8_t* eth, const pn_result& r) { d(key, r, eth); });
  }

 private:
  const char* refresh() {
    if (dirty_) {
      if (const char* e = rx_.syncTable(table_)) return e;
      dirty_ = false;
    }
    return nullptr;
  }

  template <class Handler>
  struct Dispatch {
    GpuTcpRx* self;
    Handler& h;
    void operator()(uint64_t key, const pn_result& rec, const uint8_t* eth) {
      // a frame cut at its slot (or outside the indexed call's class) has no trustworthy
      // payload extent: never delivered, whatever drop_bad_ says
      if (rec.flags & (PN_F_TRUNC | PN_F_BADOFF)) return;
      if (self->drop_bad_ && !checksums_ok(rec.flags)) return;
      pn_result r = rec;
      if (self->dirty_) { // the table changed earlier in this poll: resolve on the host, fix the record
        uint32_t conn_id = PN_MISS;
        const bool hit = self->table_.find(key, nullptr, &conn_id);
        r.conn_id = conn_id;
        r.flags = (uint16_t)((r.flags & ~(PN_F_HIT | PN_F_TW)) | (hit ? PN_F_HIT : 0) |
                             (hit && conn_id >= Conf::MaxConnCnt ? PN_F_TW : 0));
      }
      if (r.flags & PN_F_TW)
        h.onTimeWaitSegment(key, r.conn_id - Conf::MaxConnCnt, eth, r);
      else if (!(r.flags & PN_F_HIT))
        h.onNewSegment(key, eth, r);
      else
        self->deliver(h, self->conns_[r.conn_id], eth, r);
    }
  };
  // One segment of a live connection.  A connection that closes (remote FIN, RST,
  // buffer overrun) leaves the table at once, as TcpConn::onClose does
  // (TcpConn.h:451-465 -> Core::delConnEntry).
  template <class Handler>
  void deliver(Handler& h, Conn& c, const uint8_t* eth, const pn_result& rec) {
    struct Adapter { // EfviTcp.h:283-305
      Handler& h;
      Conn& c;
      uint32_t onData(RxConn<Conf>&, const uint8_t* d, uint32_t s) { return h.onTcpData(c, d, s); }
      void onFin(RxConn<Conf>&, const uint8_t* d, uint32_t s) {
        if (s) h.onTcpData(c, d, s);
        c.err = "remote close";
        h.onTcpDisconnect(c);
      }
      void onReset(RxConn<Conf>&) {
        c.err = "connection reset";
        h.onTcpDisconnect(c);
      }
    } a{h, c};
    const RxAck ack = c.onSegment(a, eth, rec);
    if (ack.send || ack.rst) h.onAckOwed(c, ack);
    if (c.err) remove(c);
  }

  GpuRx rx_;
  ConnTable table_;
  std::vector<Conn> conns_;
  std::vector<uint32_t> free_, free_tw_;
  std::vector<uint64_t> tw_keys_; // key of each TIME_WAIT id in use (PN_EMPTY_KEY: free)
  uint32_t conn_cnt_ = 0;
  bool dirty_ = true;
  bool drop_bad_ = false;
};

} // namespace pollnet_amd
