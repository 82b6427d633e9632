// Test-only harness: compiles the reference's own TcpStream.h
// (/root/reference/TcpStream.h, header-only, no external deps) into
// oracle/_ref/libref_tcpstream.so so the oracle's parse rules can be checked
// against the reference itself:
//   - TcpStream::filterPacket (TcpStream.h:39-52): ether_type == 0x0800 (LE
//     0x0008) && protocol == 6, 4-tuple wildcard filter;
//   - TcpStream::handlePacket (TcpStream.h:54-142): the IHL=5 payload split
//     header_len = 20 + doff*4 (:72-74), zero-copy payload pointer (:115).
// Nothing here is shipped or used by the product path.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <memory>
#include <utility>

#include "TcpStream.h"

namespace {
using Stream = TcpStream<true, (1u << 20)>;
}

extern "C" {

// Wildcard filter ("0.0.0.0", port 0) unless given; returns filterPacket().
int ref_filter_packet(const uint8_t* eth, uint32_t size, const char* src_ip, uint16_t src_port, const char* dst_ip,
                      uint16_t dst_port) {
  std::unique_ptr<Stream> s(new Stream());
  s->initFilter(src_ip ? src_ip : "0.0.0.0", src_port, dst_ip ? dst_ip : "0.0.0.0", dst_port);
  return s->filterPacket(eth, size) ? 1 : 0;
}

// First packet of a fresh stream: handlePacket() hands the whole payload to the
// handler zero-copy.  Returns 1 and the payload offset/size the reference
// computed, 0 if the reference dropped it (obsolete/empty or too large).
int ref_handle_packet(const uint8_t* eth, uint32_t size, uint32_t* payload_off, uint32_t* payload_len) {
  std::unique_ptr<Stream> s(new Stream());
  const uint8_t* got = nullptr;
  uint32_t got_size = 0;
  bool ok = s->handlePacket(eth, size, [&](const uint8_t* data, uint32_t n) -> uint32_t {
    got = data;
    got_size = n;
    return 0;
  });
  if (!ok || !got) return 0;
  *payload_off = (uint32_t)(got - eth);
  *payload_len = got_size;
  return 1;
}
}

// ---- stateful stream (test-only): the reference's reassembly driven packet by packet ----
// The handler consumes whole msg_len-byte messages (msg_len 0: everything) and logs
// each call's size and the consumed bytes, so a test can compare the exact sequence
// of deliveries with another implementation.
extern "C" {
struct ref_stream_log {
  uint8_t* bytes;      // consumed bytes, appended
  uint64_t n_bytes;
  uint64_t cap_bytes;
  uint32_t* call_sizes; // size presented by each handler call
  uint32_t n_calls;
  uint32_t cap_calls;
};

}

namespace {
// The reference's TcpStream in the instantiations the tests drive, behind one interface.
struct AnyStream {
  virtual ~AnyStream() = default;
  virtual int handle(const uint8_t* eth, uint32_t size, uint32_t msg_len, ref_stream_log* log) = 0;
};
template <bool W, uint32_t B>
struct StreamT final : AnyStream {
  TcpStream<W, B> s;
  int handle(const uint8_t* eth, uint32_t size, uint32_t msg_len, ref_stream_log* log) override {
    return s.handlePacket(eth, size, [&](const uint8_t* data, uint32_t n) -> uint32_t {
      const uint32_t keep = msg_len ? n % msg_len : 0;
      if (log->n_calls < log->cap_calls) log->call_sizes[log->n_calls] = n;
      log->n_calls++;
      const uint32_t take = n - keep;
      if (log->n_bytes + take <= log->cap_bytes) std::memcpy(log->bytes + log->n_bytes, data, take);
      log->n_bytes += take;
      return keep;
    }) ? 1 : 0;
  }
};
} // namespace

extern "C" {
// TcpStream<true, 1 MiB>
void* ref_stream_new(void) { return static_cast<AnyStream*>(new StreamT<true, (1u << 20)>()); }
// TcpStream<wait_for_resend, small_buf ? 4 KiB : 1 MiB>
void* ref_stream_new2(int wait_for_resend, int small_buf) {
  AnyStream* s;
  if (wait_for_resend) s = small_buf ? (AnyStream*)new StreamT<true, 4096>() : new StreamT<true, (1u << 20)>();
  else s = small_buf ? (AnyStream*)new StreamT<false, 4096>() : new StreamT<false, (1u << 20)>();
  return s;
}
void ref_stream_free(void* s) { delete static_cast<AnyStream*>(s); }
int ref_stream_handle(void* s, const uint8_t* eth, uint32_t size, uint32_t msg_len, ref_stream_log* log) {
  return static_cast<AnyStream*>(s)->handle(eth, size, msg_len, log);
}
}
