// tcp_stream.hpp — pollnet's TcpStream (sniffed TCP stream reassembly) over
// GPU-filtered batches.
//
//  StreamReassembler<WaitForResend, BUFSIZE>  TcpStream::handlePacket (TcpStream.h:54-142)
//      restated: the stream starts at its first packet or a SYN (seq + 1); payload =
//      ip + 20 + doff*4 .. ip + tot_len (no 1500 clamp); bytes already delivered are
//      trimmed; a segment past the buffer is dropped; up to 5 ordered extents; the next
//      in-order segment goes to the handler zero-copy, anything else through the
//      buffer; the handler returns the bytes it did not consume, which are kept and
//      re-presented; the buffer is compacted once half of it is consumed.  With
//      WaitForResend = false a gap is skipped instead of waited for.
//  GpuTcpStreams<WaitForResend, BUFSIZE>  up to PN_MAX_STREAM_FILTERS streams, each with
//      TcpStream::initFilter's 4-tuple (0 = wildcard).  poll() matches a batch of ring
//      slots against every filter in one pn_match_streams launch (one header line per
//      frame; zero-copy from a pinned ring), then hands each matching frame, in ring
//      order, to its streams' reassemblers — the frames of no stream are never touched
//      by the host.  As with independent TcpStreams (each running its own filterPacket),
//      a frame goes to every stream whose filter it passes, in stream order: the kernel
//      names the first, the host tests the later filters on that frame only.
//      setFirstMatchOnly(true): the first stream only (overlapping filters as priorities).
// Handler: uint32_t h(int stream, const uint8_t* data, uint32_t size) -> bytes not consumed.
#pragma once

#include <arpa/inet.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <memory>
#include <vector>

#include "gpu_rx.hpp"

// GpuTcpStreams::poll prefetches this many matched frames ahead of the one it reassembles (4 measured best of
// 0/1/2/4/8, profiles/r04/sniffer/prefetch_pf*.jsonl); overridable for A/B builds.
#ifndef PN_STREAM_PREFETCH_AHEAD
#define PN_STREAM_PREFETCH_AHEAD 4
#endif

namespace pollnet_amd {

template <bool WaitForResend = true, uint32_t BUFSIZE = (1u << 20)>
class StreamReassembler {
 public:
  static constexpr uint32_t kMaxSegs = 5; // TcpStream::MAX_SEG (TcpStream.h:225)
  struct Seg {
    uint32_t first, second; // [first, second) relative to the buffer start
  };

  // One frame of this stream (eth = its Ethernet header).  Returns what
  // TcpStream::handlePacket returns: true when the segment was taken.
  template <class Handler>
  bool handlePacket(const uint8_t* eth, Handler&& h) {
    const uint8_t* ip = eth + 14;
    const uint8_t* tcp = ip + 20; // IP header assumed 20 B (TcpStream.h:214)
    uint32_t seq = be32(tcp + 4);
    if (tcp[13] & 0x02) { // SYN: a new stream begins after it
      started_ = false;
      ++seq;
    }
    if (!started_) {
      started_ = true;
      base_seq_ = seq;
      n_ = 1;
      segs_[0] = {0, 0};
    }
    const uint32_t hdr = 20 + 4u * (tcp[12] >> 4);
    const uint8_t* data = ip + hdr;
    uint32_t len = be16(ip + 2) - hdr; // u32 arithmetic, as the reference's
    uint32_t loc = seq - base_seq_;
    const uint32_t loc_end = loc + len;
    const int32_t behind = (int32_t)(loc - segs_[0].second);
    if (behind < 0) { // drop what was delivered already
      loc -= behind;
      data -= behind;
      len += behind;
    }
    if ((int32_t)len <= 0) return false; // nothing new
    if (loc_end > BUFSIZE) return false;  // beyond the buffer
    if (!WaitForResend && loc > segs_[0].second) segs_[0] = {loc, loc}; // skip the gap

    uint32_t i = 0;
    while (i < n_ && segs_[i].second < loc) ++i;
    uint32_t j = i;
    while (j < n_ && segs_[j].first <= loc_end) ++j;
    if (i == j) { // a new extent
      if (n_ == kMaxSegs) return false;
      std::copy_backward(segs_ + i, segs_ + n_, segs_ + n_ + 1);
      segs_[i] = {loc, loc_end};
      ++n_;
    } else { // merge extents i .. j-1 with it
      segs_[i].first = std::min(segs_[i].first, loc);
      segs_[i].second = std::max(segs_[j - 1].second, loc_end);
      if (j > i + 1) {
        std::copy(segs_ + j, segs_ + n_, segs_ + i + 1);
        n_ -= j - i - 1;
      }
    }

    if (segs_[0].first == loc && segs_[0].second == loc_end) { // exactly the next bytes: zero copy
      const uint32_t left = h(data, len);
      segs_[0].first = segs_[0].second - left;
      if (left) std::memcpy(buf_.get() + segs_[0].first, data + (len - left), left);
    } else {
      std::memcpy(buf_.get() + loc, data, len);
      if (i != 0) return false; // landed beyond a gap: nothing new for the handler
      const uint32_t left = h(buf_.get() + segs_[0].first, segs_[0].second - segs_[0].first);
      segs_[0].first = segs_[0].second - left;
    }

    if (segs_[0].first >= BUFSIZE / 2) { // compact: move the held bytes to the front
      const uint32_t shift = segs_[0].first;
      const uint32_t held = segs_[n_ - 1].second - shift;
      if (held) std::memmove(buf_.get(), buf_.get() + shift, held);
      base_seq_ += shift;
      for (uint32_t k = 0; k < n_; ++k) {
        segs_[k].first -= shift;
        segs_[k].second -= shift;
      }
    }
    return true;
  }

  uint32_t segCount() const { return n_; }
  const Seg* segs() const { return segs_; }

 private:
  static uint32_t be16(const uint8_t* p) { return (uint32_t)p[0] << 8 | p[1]; }
  static uint32_t be32(const uint8_t* p) { return be16(p) << 16 | be16(p + 2); }

  bool started_ = false;
  uint32_t base_seq_ = 0;
  uint32_t n_ = 1;
  Seg segs_[kMaxSegs] = {};
  std::unique_ptr<uint8_t[]> buf_ = std::make_unique<uint8_t[]>(BUFSIZE);
};

template <bool WaitForResend = true, uint32_t BUFSIZE = (1u << 20)>
class GpuTcpStreams {
 public:
  using Stream = StreamReassembler<WaitForResend, BUFSIZE>;

  GpuTcpStreams() = default;
  GpuTcpStreams(const GpuTcpStreams&) = delete;
  GpuTcpStreams& operator=(const GpuTcpStreams&) = delete;
  ~GpuTcpStreams() { destruct(); }

  const char* init(int device, uint32_t slot_stride, uint32_t frame_off, uint32_t max_batch,
                   GpuRx::Mode mode = GpuRx::Mode::ZeroCopy) {
    destruct();
    if (max_batch == 0) return "max_batch must be > 0";
    if (pn_open(device, &ctx_)) return pn_last_error(nullptr);
    stride_ = slot_stride;
    off_ = frame_off;
    cap_ = max_batch;
    mode_ = mode;
    if (hipSetDevice(device) != hipSuccess) return "hipSetDevice failed";
    if (hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking) != hipSuccess) return "hipStreamCreate failed";
    for (int b = 0; b < 2; b++) {
      if (mode == GpuRx::Mode::Copy) {
        if (hipMalloc(&d_frames_[b], (size_t)slot_stride * max_batch) != hipSuccess) return "hipMalloc(frames) failed";
        if (hipMalloc(&d_ids_[b], sizeof(uint32_t) * max_batch) != hipSuccess) return "hipMalloc(ids) failed";
      }
      if (hipHostMalloc(&h_ids_[b], sizeof(uint32_t) * max_batch, hipHostMallocDefault) != hipSuccess)
        return "hipHostMalloc(ids) failed";
      if (hipEventCreateWithFlags(&done_[b], hipEventDisableTiming) != hipSuccess) return "hipEventCreate failed";
    }
    return nullptr;
  }

  // TcpStream::initFilter (TcpStream.h:32-37) for a new stream: "0.0.0.0" / port 0 are
  // wildcards.  Returns the stream's index, or -1 (bad address, or all streams in use).
  int addStream(const char* src_ip, uint16_t src_port, const char* dst_ip, uint16_t dst_port) {
    if (filters_.size() >= PN_MAX_STREAM_FILTERS) return -1;
    pn_stream_filter f{};
    if (inet_pton(AF_INET, src_ip, &f.src_ip) != 1 || inet_pton(AF_INET, dst_ip, &f.dst_ip) != 1) return -1;
    f.src_port = htons(src_port);
    f.dst_port = htons(dst_port);
    filters_.push_back(f);
    streams_.push_back(std::make_unique<Stream>());
    return (int)filters_.size() - 1;
  }
  Stream& stream(int i) { return *streams_[i]; }
  uint32_t streamCount() const { return (uint32_t)filters_.size(); }
  // true: a frame goes to the first stream it passes only (default false: every stream it passes)
  void setFirstMatchOnly(bool v) { first_only_ = v; }

  // TcpStream::filterPacket (TcpStream.h:39-52) on the host, for the filters after a frame's first
  // match: IPv4 (etherType read little-endian, 0x0008) and TCP, IHL assumed 5 (TcpStream.h:213-214),
  // each non-zero field equal to the frame's, all in network order as stored
  static bool filterPacket(const pn_stream_filter& f, const uint8_t* eth) {
    uint16_t ether_type, src_port, dst_port;
    uint32_t src_ip, dst_ip;
    std::memcpy(&ether_type, eth + 12, 2);
    std::memcpy(&src_ip, eth + 26, 4);
    std::memcpy(&dst_ip, eth + 30, 4);
    std::memcpy(&src_port, eth + 34, 2);
    std::memcpy(&dst_port, eth + 36, 2);
    return ether_type == 0x0008 && eth[23] == 6 && (!f.src_ip || f.src_ip == src_ip) &&
           (!f.dst_ip || f.dst_ip == dst_ip) && (!f.src_port || f.src_port == src_port) &&
           (!f.dst_port || f.dst_port == dst_port);
  }

  // Match n ring slots on the GPU (chunks of max_batch, chunk k+1 on the GPU while
  // chunk k is reassembled) and feed every matching frame to its stream in ring order.
  template <class Handler>
  const char* poll(const uint8_t* slots, uint32_t n, Handler&& h) {
    if (n == 0 || filters_.empty()) return nullptr;
    if (mode_ == GpuRx::Mode::ZeroCopy) {
      hipPointerAttribute_t attr;
      if (hipPointerGetAttributes(&attr, slots) != hipSuccess || attr.type != hipMemoryTypeHost)
        return "zero-copy ring must be pinned host memory (hipHostMalloc / hipHostRegister)";
    }
    const uint32_t chunks = (n + cap_ - 1) / cap_, nf = (uint32_t)filters_.size();
    if (const char* e = launch(slots, n, 0)) return e;
    for (uint32_t k = 0; k < chunks; k++) {
      if (k + 1 < chunks)
        if (const char* e = launch(slots, n, k + 1)) return e;
      if (hipEventSynchronize(done_[k & 1]) != hipSuccess) return "hipEventSynchronize failed";
      const uint32_t base = k * cap_, m = std::min(cap_, n - base);
      const uint32_t* ids = h_ids_[k & 1];
      // The host touches only the matched frames, spread over the ring, so each is a run of cold lines:
      // prefetch the next kPrefetchAhead matched frames (the first 1536 B of each slot's frame: reading its
      // length first would stall on that line) while this one is reassembled.
      const uint32_t span = std::min<uint32_t>(1536u, stride_ - off_);
      uint32_t ahead = 0, inflight = 0; // next index to look at for a prefetch; matched frames prefetched past i
      for (uint32_t i = 0; i < m; i++) {
        const uint32_t s = ids[i];
        if (s == PN_NO_STREAM) continue;
        if (ahead <= i) ahead = i + 1, inflight = 0;
        else if (inflight) inflight--;
        for (; inflight < kPrefetchAhead && ahead < m; ahead++) {
          if (ids[ahead] == PN_NO_STREAM) continue;
          const uint8_t* e = slots + (size_t)(base + ahead) * stride_ + off_;
          for (uint32_t o = 0; o < span; o += 64) __builtin_prefetch(e + o);
          inflight++;
        }
        const uint8_t* eth = slots + (size_t)(base + i) * stride_ + off_;
        streams_[s]->handlePacket(eth, [&](const uint8_t* d, uint32_t size) { return h((int)s, d, size); });
        if (first_only_) continue;
        for (uint32_t t = s + 1; t < nf; t++)
          if (filterPacket(filters_[t], eth))
            streams_[t]->handlePacket(eth, [&](const uint8_t* d, uint32_t size) { return h((int)t, d, size); });
      }
    }
    return nullptr;
  }

 private:
  const char* launch(const uint8_t* slots, uint32_t n, uint32_t k) {
    const uint32_t base = k * cap_, m = std::min(cap_, n - base), b = k & 1;
    const uint8_t* src = slots + (size_t)base * stride_;
    const pn_stream_filter* f = filters_.data();
    const uint32_t nf = (uint32_t)filters_.size();
    if (mode_ == GpuRx::Mode::ZeroCopy) {
      if (pn_match_streams(ctx_, src, stride_, off_, m, f, nf, h_ids_[b], stream_)) return pn_last_error(ctx_);
    } else {
      if (hipMemcpyAsync(d_frames_[b], src, (size_t)stride_ * m, hipMemcpyHostToDevice, stream_) != hipSuccess)
        return "hipMemcpyAsync H2D failed";
      if (pn_match_streams(ctx_, d_frames_[b], stride_, off_, m, f, nf, d_ids_[b], stream_)) return pn_last_error(ctx_);
      if (hipMemcpyAsync(h_ids_[b], d_ids_[b], sizeof(uint32_t) * m, hipMemcpyDeviceToHost, stream_) != hipSuccess)
        return "hipMemcpyAsync D2H failed";
    }
    if (hipEventRecord(done_[b], stream_) != hipSuccess) return "hipEventRecord failed";
    return nullptr;
  }

  void destruct() {
    if (stream_) (void)hipStreamSynchronize(stream_);
    for (int b = 0; b < 2; b++) {
      if (done_[b]) (void)hipEventDestroy(done_[b]);
      if (h_ids_[b]) (void)hipHostFree(h_ids_[b]);
      if (d_ids_[b]) (void)hipFree(d_ids_[b]);
      if (d_frames_[b]) (void)hipFree(d_frames_[b]);
      done_[b] = nullptr;
      h_ids_[b] = d_ids_[b] = nullptr;
      d_frames_[b] = nullptr;
    }
    if (stream_) (void)hipStreamDestroy(stream_);
    pn_close(ctx_);
    stream_ = nullptr;
    ctx_ = nullptr;
  }

  pn_ctx* ctx_ = nullptr;
  hipStream_t stream_ = nullptr;
  GpuRx::Mode mode_ = GpuRx::Mode::ZeroCopy;
  bool first_only_ = false;
  static constexpr uint32_t kPrefetchAhead = PN_STREAM_PREFETCH_AHEAD;
  void* d_frames_[2] = {nullptr, nullptr};
  uint32_t* d_ids_[2] = {nullptr, nullptr};
  uint32_t* h_ids_[2] = {nullptr, nullptr};
  hipEvent_t done_[2] = {nullptr, nullptr};
  uint32_t stride_ = 0, off_ = 0, cap_ = 0;
  std::vector<pn_stream_filter> filters_;
  std::vector<std::unique_ptr<Stream>> streams_;
};

} // namespace pollnet_amd
