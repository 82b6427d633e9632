// BASELINE config C1 (CPU plumbing, no GPU): the reference's own Socket.h TCP server and
// client (Socket.h:40-392, compiled unmodified from /root/reference by oracle/ref.mk) echoing
// 1500-B application messages over 127.0.0.1, one connection -- example/tcpserver.cc's echo
// handler (writeNonblock(data, size), return 0) against a client that keeps `window`
// messages in flight (example/tcpclient.cc, with 1500-B messages instead of 16-B pings).
// Test/baseline infrastructure only: nothing of the product links or runs it.
//
//   ref_socket_c1 [seconds] [window] [port]   -> one JSON line
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "Socket.h"

namespace {

constexpr uint32_t kMsg = 1500;

struct ServerConf {
  static const uint32_t RecvBufSize = 4096;
  static const uint32_t MaxConns = 10;
  static const uint32_t SendTimeoutSec = 0;
  static const uint32_t RecvTimeoutSec = 10;
  struct UserData {};
};

struct ClientConf {
  static const uint32_t RecvBufSize = 4096;
  static const uint32_t ConnRetrySec = 1;
  static const uint32_t ConnTimeoutSec = 5;
  static const uint32_t SendTimeoutSec = 0;
  static const uint32_t RecvTimeoutSec = 10;
  struct UserData {};
};

using Server = SocketTcpServer<ServerConf>;
using Client = SocketTcpClient<ClientConf>;

std::atomic<bool> running{true};

uint64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

} // namespace

int main(int argc, char** argv) {
  const double seconds = argc > 1 ? atof(argv[1]) : 3.0;
  const uint32_t window = argc > 2 ? (uint32_t)atoi(argv[2]) : 8;
  const uint16_t port = argc > 3 ? (uint16_t)atoi(argv[3]) : 1234;

  static Server server;
  if (!server.init("lo", "127.0.0.1", port)) {
    printf("{\"error\": \"server init: %s\"}\n", server.getLastError());
    return 1;
  }
  std::thread srv([&] {
    struct {
      void onTcpConnected(Server::Conn&) {}
      void onSendTimeout(Server::Conn&) {}
      uint32_t onTcpData(Server::Conn& conn, const uint8_t* data, uint32_t size) {
        conn.writeNonblock(data, size); // example/tcpserver.cc's echo
        return 0;
      }
      void onRecvTimeout(Server::Conn& conn) { conn.close("timeout"); }
      void onTcpDisconnect(Server::Conn&) {}
    } handler;
    while (running.load(std::memory_order_relaxed)) server.poll(handler);
  });

  static Client client;
  client.init("lo", "127.0.0.1", port);
  static uint8_t msg[kMsg];
  for (uint32_t i = 0; i < kMsg; i++) msg[i] = (uint8_t)(i * 131 + 7);
  uint64_t echoed = 0, t_start = 0, t_end = 0, lat_sum = 0, lat_n = 0;
  bool connected = false, failed = false;
  static uint64_t sent_ts[1 << 16];
  uint64_t sent = 0;
  struct Handler {
    Client* c;
    uint64_t *echoed, *sent, *lat_sum, *lat_n, *t_start;
    uint32_t window;
    bool *connected, *failed;
    void onTcpConnectFailed() { *failed = true; }
    void onTcpConnected(Client::Conn& conn) {
      *connected = true;
      *t_start = now_ns();
      for (uint32_t i = 0; i < window; i++) {
        sent_ts[(*sent)++ & 0xffff] = now_ns();
        conn.writeNonblock(msg, kMsg);
      }
    }
    void onSendTimeout(Client::Conn&) {}
    uint32_t onTcpData(Client::Conn& conn, const uint8_t* data, uint32_t size) {
      const uint64_t t = now_ns();
      uint32_t whole = size / kMsg;
      for (uint32_t i = 0; i < whole; i++) { // every echoed message releases the next one
        lat_sum[0] += t - sent_ts[*echoed & 0xffff];
        ++*lat_n;
        ++*echoed;
        sent_ts[(*sent)++ & 0xffff] = now_ns();
        conn.writeNonblock(msg, kMsg);
      }
      return size - whole * kMsg; // the unfinished message is re-presented (README.md:117-129)
    }
    void onRecvTimeout(Client::Conn& conn) { conn.close("timeout"); }
    void onTcpDisconnect(Client::Conn&) {}
  } h{&client, &echoed, &sent, &lat_sum, &lat_n, &t_start, window, &connected, &failed};

  const uint64_t deadline_connect = now_ns() + 5000000000ull;
  while (!connected && !failed && now_ns() < deadline_connect) {
    client.poll(h);
    if (!connected) std::this_thread::sleep_for(std::chrono::milliseconds(1));
  }
  if (!connected) {
    running = false;
    srv.join();
    printf("{\"error\": \"connect failed\"}\n");
    return 1;
  }
  const uint64_t deadline = t_start + (uint64_t)(seconds * 1e9);
  while ((t_end = now_ns()) < deadline) client.poll(h);
  running = false;
  srv.join();
  const double el = (t_end - t_start) * 1e-9;
  const double msgs = echoed / el;
  printf("{\"config\": \"C1: Socket.h loopback TCP echo, 1 conn, 1500-B messages\", \"window\": %u, \"seconds\": %.3f, "
         "\"messages_echoed\": %llu, \"round_trips_per_s\": %.1f, \"payload_gbit_per_s_each_way\": %.3f, "
         "\"mean_rtt_us\": %.2f, \"threads\": 2, \"recv_buf_size\": 4096}\n",
         window, el, (unsigned long long)echoed, msgs, msgs * kMsg * 8 / 1e9, lat_n ? lat_sum * 1e-3 / lat_n : 0.0);
  return 0;
}
