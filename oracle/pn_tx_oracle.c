/*
 * pn_tx_oracle.c — plain-C restatement of pollnet's TX checksum generation
 * (SURVEY §8(f) rank 4).  TEST INFRASTRUCTURE: the checker for pn_tx_fill and the
 * timed CPU baseline of the TX leg; never linked into libpollnet_amd.
 *
 * Two halves, deliberately different formulations:
 *  (1) the reference's OWN way — incremental CSum state carried by the connection and
 *      the send buffers, folded when a frame leaves — restated function by function:
 *        Core::init send-buffer template + RST/TW cache   Core.h:290-311
 *        TcpConn::reset                                   TcpConn.h:149-186
 *        sendSyn                                          TcpConn.h:198-230
 *        onEstablished (offset_flags into tcpsum)         TcpConn.h:422-428
 *        the no-timestamp fix-up of tcpsum                TcpConn.h:396-399
 *        sendPartial's appends + copyAndSum               TcpConn.h:238-240, 257-299
 *        sendBuf                                          TcpConn.h:310-323
 *        SendBuf::setOptDataLen                           Core.h:157-163
 *        resendUna's in-place patch                       TcpConn.h:771-785
 *        rspRst / ackTW / sumRst                          Core.h:385-446
 *        Efvi UDP: init_udp_pkt, ipsum_cache, update_udp_pkt  Efvi.h:405-411, 590-636
 *      orc_tx_build_batch drives them to produce the frames a reference sender puts on
 *      the wire: the expected bytes for pn_tx_fill.
 *  (2) orc_tx_fill_*: a straight recomputation from the frame bytes (RFC 1071 sums, the
 *      same contract as pn_tx_fill), the CPU baseline.
 * Pinning: Core.h / TcpConn.h / Efvi.h need the absent ef_vi headers (unbuildable here,
 * DESIGN.md §5); half (1) is pinned by the reference's own debug self-check — every frame
 * it sends must pass Core::checksum (Core.h:448-472, called from Core::send :478) — which
 * tests/test_tx.py applies to every built frame through the RX oracle, and by RFC 1071.
 */
#define _GNU_SOURCE
#include "pn_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

static inline uint16_t ld16(const uint8_t* p) {
  uint16_t v;
  memcpy(&v, p, 2);
  return v;
}
static inline uint32_t ld32(const uint8_t* p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}
static inline void st16(uint8_t* p, uint16_t v) { memcpy(p, &v, 2); }
static inline void st32(uint8_t* p, uint32_t v) { memcpy(p, &v, 4); }
static inline uint16_t htons_(uint16_t v) { return (uint16_t)((v >> 8) | (v << 8)); }
static inline uint32_t htonl_(uint32_t v) { return __builtin_bswap32(v); }

static void orc_csum_add(orc_csum* s, orc_csum o) { s->sum += o.sum; } /* CSum::add(CSum) (Core.h:105) */

/* CSum::sub (Core.h:119-127) and setVar (Core.h:129-134) */
static void csum_sub16(orc_csum* s, uint16_t a) {
  s->sum += 0xffff;
  s->sum -= a;
}
static void csum_sub32(orc_csum* s, uint32_t a) {
  s->sum += 0x1fffe;
  s->sum -= a >> 16;
  s->sum -= a & 0xffff;
}
static void setvar16(orc_csum* s, int reset, uint8_t* var, uint16_t val) {
  if (reset) csum_sub16(s, ld16(var));
  st16(var, val);
  orc_csum_add16(s, val);
}
static void setvar32(orc_csum* s, int reset, uint8_t* var, uint32_t val) {
  if (reset) csum_sub32(s, ld32(var));
  st32(var, val);
  orc_csum_add32(s, val);
}

/* frame offsets: eth 0, ip 14, tcp 34, SendBuf+1 (options / payload) 54 */
enum { IP = 14, TCP = 34, OPT = 54 };
/* TcpHeader.offset_flags bitfield (Core.h:78-81): reserved:4, data_offset:4, fin, syn, rst, psh, ack */
static void set_doff(uint8_t* eth, uint32_t doff) { eth[TCP + 12] = (uint8_t)((eth[TCP + 12] & 0x0f) | (doff << 4)); }
static void set_flag(uint8_t* eth, int bit, int v) {
  eth[TCP + 13] = (uint8_t)(v ? (eth[TCP + 13] | (1u << bit)) : (eth[TCP + 13] & ~(1u << bit)));
}
enum { FIN = 0, SYN = 1, RST = 2, PSH = 3, ACK = 4 };

/* SendBuf::setOptDataLen (Core.h:157-163) */
static void set_opt_data_len(uint8_t* eth, uint16_t len, orc_csum ipsum, orc_csum tcpsum) {
  st16(eth + IP + 2, htons_((uint16_t)(40 + len)));
  orc_csum_add16(&ipsum, ld16(eth + IP + 2));
  st16(eth + IP + 10, orc_csum_fold(ipsum));
  orc_csum_add16(&tcpsum, htons_((uint16_t)(20 + len)));
  st16(eth + TCP + 16, orc_csum_fold(tcpsum));
}

/* Core::init's send-buffer template (Core.h:290-304); other bytes are the zeroed pkt_buf */
static void send_template(uint8_t* eth, const uint8_t* src_mac, uint32_t local_ip) {
  memcpy(eth + 6, src_mac, 6);
  st16(eth + 12, htons_(0x0800));
  eth[IP + 0] = 0x45; /* header_len 5, ip_ver 4 */
  eth[IP + 1] = 0;
  st16(eth + IP + 4, 0);
  st16(eth + IP + 6, htons_(0x4000)); /* DF */
  eth[IP + 8] = 64;
  eth[IP + 9] = 6;
  st32(eth + IP + 12, local_ip);
}

/* copyAndSum (TcpConn.h:257-299), literally: u64 words, odd-destination fix-up */
static orc_csum copy_and_sum(uint8_t* dst, const uint8_t* src, uint32_t size) {
  uint64_t sum = 0;
  if ((uintptr_t)dst & 1) {
    uint8_t n = *src++;
    *dst++ = n;
    sum += (uint64_t)n << 8; /* IsLittle */
    size--;
  }
  while (size >= 8) {
    uint64_t n;
    memcpy(&n, src, 8);
    memcpy(dst, &n, 8);
    sum += n >> 32;
    sum += n & 0xffffffff;
    src += 8;
    dst += 8;
    size -= 8;
  }
  if (size >= 4) {
    uint32_t n = ld32(src);
    st32(dst, n);
    sum += n;
    src += 4;
    dst += 4;
    size -= 4;
  }
  if (size >= 2) {
    uint16_t n = ld16(src);
    st16(dst, n);
    sum += n;
    src += 2;
    dst += 2;
    size -= 2;
  }
  if (size) {
    uint8_t n = *src;
    *dst = n;
    sum += n; /* IsLittle: low byte */
  }
  orc_csum ret = {(uint32_t)(sum >> 32)};
  orc_csum_add32(&ret, (uint32_t)sum);
  return ret;
}

/* ---- one connection's cached sums (TcpConn.h:907-908) and the header fields its buffers share ---- */
typedef struct tx_conn {
  uint8_t src_mac[6], dst_mac[6];
  uint32_t local_ip, dst_ip;       /* network order */
  uint16_t src_port, dst_port;     /* network order */
  int has_ts, has_ws, established;
  uint32_t recv_wnd_shift;
  orc_csum ipsum, tcpsum;
  uint8_t hdr[OPT + 4];            /* the connection's header template (SYN buffer) */
} tx_conn;

/* TcpConn::reset (TcpConn.h:149-186) on the connection's send buffer 0 */
static void conn_reset(tx_conn* c, uint32_t isn) {
  uint8_t* syn = c->hdr;
  memset(syn, 0, sizeof(c->hdr));
  send_template(syn, c->src_mac, c->local_ip);
  memcpy(syn, c->dst_mac, 6);
  st32(syn + IP + 16, c->dst_ip);
  st16(syn + IP + 2, 0);
  st16(syn + IP + 10, 0);
  c->ipsum.sum = 0;
  orc_csum_add_bytes(&c->ipsum, syn + IP, 20); /* add<sizeof(IpHeader)> */
  c->tcpsum.sum = 0;
  orc_csum_add32(&c->tcpsum, ld32(syn + IP + 12));
  orc_csum_add32(&c->tcpsum, ld32(syn + IP + 16));
  orc_csum_add16(&c->tcpsum, htons_(0x6));
  setvar16(&c->tcpsum, 0, syn + TCP + 0, c->src_port);
  setvar16(&c->tcpsum, 0, syn + TCP + 2, c->dst_port);
  st32(syn + TCP + 4, htonl_(isn));
  /* Conf::TimestampOption: the TS option header goes in now (has_ts = 1 until the peer says otherwise) */
  syn[OPT + 0] = 1;
  syn[OPT + 1] = 1;
  syn[OPT + 2] = 8;
  syn[OPT + 3] = 10;
  orc_csum_add_bytes(&c->tcpsum, syn + OPT, 4);
  c->established = 0;
}

/* sendBuf (TcpConn.h:310-323) */
static void send_buf(const tx_conn* c, uint8_t* buf, uint32_t opt_data_size, orc_csum sum, uint32_t ack, uint16_t window,
                     uint32_t now_ts, uint32_t recent_ts) {
  orc_csum_add32(&sum, ld32(buf + TCP + 4)); /* seq_num */
  setvar32(&sum, 0, buf + TCP + 8, htonl_(ack));
  setvar16(&sum, 0, buf + TCP + 14, htons_(window));
  if (c->has_ts) {
    setvar32(&sum, 0, buf + OPT + 4, htonl_(now_ts));
    setvar32(&sum, 0, buf + OPT + 8, htonl_(recent_ts));
    opt_data_size += 12;
  }
  orc_csum_add(&sum, c->tcpsum);
  set_opt_data_len(buf, (uint16_t)opt_data_size, c->ipsum, sum);
}

/* sendSyn (TcpConn.h:198-230) into buf (a copy of the connection's buffer 0) */
static uint32_t send_syn(const tx_conn* c, uint8_t* buf, int pending_ack, uint32_t ack, uint16_t window, uint32_t now_ts,
                         uint32_t recent_ts) {
  orc_csum sum = {0};
  st16(buf + TCP + 12, 0);
  set_flag(buf, SYN, 1);
  set_flag(buf, ACK, pending_ack);
  uint8_t* opt = buf + OPT;
  if (c->has_ts) opt += 12;
  uint8_t* additional_opt = opt;
  opt[0] = 2;
  opt[1] = 4;
  st16(opt + 2, htons_(PN_RECV_MSS));
  orc_csum_add_bytes(&sum, opt, 4);
  opt += 4;
  if (c->has_ws) {
    opt[0] = 1;
    opt[1] = 3;
    opt[2] = 3;
    opt[3] = (uint8_t)c->recv_wnd_shift;
    orc_csum_add_bytes(&sum, opt, 4);
    opt += 4;
  }
  uint16_t opt_len = (uint16_t)(opt - (buf + OPT));
  set_doff(buf, (uint32_t)(opt_len + 20) >> 2);
  orc_csum_add16(&sum, ld16(buf + TCP + 12));
  send_buf(c, buf, (uint32_t)(opt - additional_opt), sum, ack, window, now_ts, recent_ts);
  return (uint32_t)(opt - additional_opt) + (c->has_ts ? 12u : 0u);
}

/* option parse outcome (TcpConn.h:396-399) + onEstablished (TcpConn.h:422-428) */
static void conn_establish(tx_conn* c, int peer_ts) {
  if (!peer_ts) {
    c->has_ts = 0;
    csum_sub32(&c->tcpsum, ld32(c->hdr + OPT)); /* sub ts opt header */
  }
  st16(c->hdr + TCP + 12, 0);
  set_doff(c->hdr, c->has_ts ? 8 : 5);
  set_flag(c->hdr, PSH, 1);
  set_flag(c->hdr, ACK, 1);
  orc_csum_add16(&c->tcpsum, ld16(c->hdr + TCP + 12));
  c->established = 1;
}

/* sendPartial's appends (TcpConn.h:238-240, data_sum reset by advanceData :333-337) +
 * sendBuf: one data segment of len bytes, appended in n_pieces copyAndSum calls. */
static uint32_t send_data(const tx_conn* c, uint8_t* buf, uint32_t seq, const uint8_t* data, uint32_t len,
                          const uint32_t* pieces, uint32_t n_pieces, uint32_t ack, uint16_t window, uint32_t now_ts,
                          uint32_t recent_ts) {
  memcpy(buf, c->hdr, OPT + 4); /* the buffer's headers as onEstablished copied them, ts option header incl. */
  st32(buf + TCP + 4, htonl_(seq)); /* advanceNext (TcpConn.h:341-342) */
  orc_csum data_sum = {0};
  uint8_t* dst = buf + OPT + (c->has_ts ? 12 : 0);
  uint32_t off = 0;
  for (uint32_t k = 0; k < n_pieces && off < len; k++) {
    uint32_t m = pieces[k] < len - off ? pieces[k] : len - off;
    if (m == 0) continue; /* sendPartial never appends 0 bytes (TcpConn.h:234-236) */
    orc_csum_add(&data_sum, copy_and_sum(dst + off, data + off, m));
    off += m;
  }
  if (off < len) orc_csum_add(&data_sum, copy_and_sum(dst + off, data + off, len - off));
  send_buf(c, buf, len, data_sum, ack, window, now_ts, recent_ts);
  return len + (c->has_ts ? 12u : 0u);
}

/* resendUna (TcpConn.h:771-785): patch the folded sum of an already-sent buffer */
static void resend_una(const tx_conn* c, uint8_t* una, uint32_t ack, uint16_t window, uint32_t now_ts, uint32_t recent_ts) {
  orc_csum sum = {(uint16_t)~ld16(una + TCP + 16)};
  setvar32(&sum, 1, una + TCP + 8, htonl_(ack));
  setvar16(&sum, 1, una + TCP + 14, htons_(window));
  if (c->has_ts) {
    setvar32(&sum, 1, una + OPT + 4, htonl_(now_ts));
    setvar32(&sum, 1, una + OPT + 8, htonl_(recent_ts));
  }
  st16(una + TCP + 16, orc_csum_fold(sum));
}

/* ---- the RST / TIME_WAIT-ACK buffer (Core.h:305-311, 385-446) ---- */
typedef struct rst_buf {
  uint8_t f[OPT + 12];
  orc_csum rst_ipsum, rst_tcpsum;
} rst_buf;

static void rst_init(rst_buf* r, const uint8_t* src_mac, uint32_t local_ip) {
  memset(r->f, 0, sizeof(r->f));
  send_template(r->f, src_mac, local_ip);
  r->rst_ipsum.sum = 0;
  orc_csum_add_bytes(&r->rst_ipsum, r->f + IP, 20);
  r->rst_tcpsum.sum = 0;
  orc_csum_add32(&r->rst_tcpsum, ld32(r->f + IP + 12));
  orc_csum_add16(&r->rst_tcpsum, htons_(0x6));
  st32(r->f + OPT, htonl_(0x0101080a)); /* ts header */
}

static void sum_rst(rst_buf* r, int has_ts) { /* Core.h:385-398 */
  orc_csum ipsum = r->rst_ipsum;
  orc_csum_add32(&ipsum, ld32(r->f + IP + 16));
  orc_csum tcpsum = r->rst_tcpsum;
  orc_csum_add32(&tcpsum, ld32(r->f + IP + 16));
  orc_csum_add16(&tcpsum, ld16(r->f + TCP + 0));
  orc_csum_add16(&tcpsum, ld16(r->f + TCP + 2));
  orc_csum_add32(&tcpsum, ld32(r->f + TCP + 4));
  orc_csum_add32(&tcpsum, ld32(r->f + TCP + 8));
  orc_csum_add16(&tcpsum, ld16(r->f + TCP + 12));
  if (has_ts) orc_csum_add_bytes(&tcpsum, r->f + OPT, 12);
  set_opt_data_len(r->f, has_ts ? 12 : 0, ipsum, tcpsum);
}

/* rspRst (Core.h:400-421); returns 0 when the reference sends nothing (incoming RST) */
static int rsp_rst(rst_buf* r, const uint8_t* in) {
  const uint8_t* ip = in + IP;
  const uint8_t* tcp = in + TCP;
  if (tcp[13] & 0x04) return 0;
  memcpy(r->f, in + 6, 6);
  st32(r->f + IP + 16, ld32(ip + 12));
  st16(r->f + TCP + 0, ld16(tcp + 2));
  st16(r->f + TCP + 2, ld16(tcp + 0));
  set_flag(r->f, RST, 1);
  set_doff(r->f, 5);
  if (tcp[13] & 0x10) {
    set_flag(r->f, ACK, 0);
    st32(r->f + TCP + 4, ld32(tcp + 8));
  } else {
    set_flag(r->f, ACK, 1);
    st32(r->f + TCP + 4, 0);
    uint32_t seg_len = (uint32_t)htons_(ld16(ip + 2)) - 20 - ((uint32_t)(tcp[12] >> 4) << 2) + ((tcp[13] >> 1) & 1) +
                       (tcp[13] & 1);
    st32(r->f + TCP + 8, htonl_(htonl_(ld32(tcp + 4)) + seg_len));
  }
  sum_rst(r, 0);
  return 1;
}

/* ackTW (Core.h:423-446); TimeWaitConn fields as stored there (network order, now_ts raw) */
static void ack_tw(rst_buf* r, const uint8_t* dst_mac, uint32_t dst_ip, uint16_t src_port, uint16_t dst_port,
                   uint32_t seq_num, uint32_t ack_num, int has_ts, uint32_t now_ts, uint32_t tsecr) {
  memcpy(r->f, dst_mac, 6);
  st32(r->f + IP + 16, dst_ip);
  st16(r->f + TCP + 0, src_port);
  st16(r->f + TCP + 2, dst_port);
  set_flag(r->f, RST, 0);
  set_flag(r->f, ACK, 1);
  st32(r->f + TCP + 4, seq_num);
  st32(r->f + TCP + 8, ack_num);
  if (has_ts) {
    set_doff(r->f, 8);
    st32(r->f + OPT + 4, now_ts);
    st32(r->f + OPT + 8, tsecr);
  } else {
    set_doff(r->f, 5);
  }
  sum_rst(r, has_ts);
}

/* ---- Efvi's UDP sender (Efvi.h:405-411, 590-636) ---- */
static uint32_t udp_init_pkt(uint8_t* eth, const uint8_t* local_mac, const uint8_t* dest_mac, uint32_t saddr,
                             uint32_t daddr, uint16_t sport, uint16_t dport) {
  memset(eth, 0, 42);
  st16(eth + 12, htons_(0x0800));
  memcpy(eth + 6, local_mac, 6);
  memcpy(eth, dest_mac, 6);
  uint8_t* ip4 = eth + 14;
  ip4[0] = (4u << 4) | (20u >> 2); /* CI_IP4_IHL_VERSION */
  ip4[1] = 0;
  st16(ip4 + 2, htons_(0));
  st16(ip4 + 4, 0);
  st16(ip4 + 6, 0x0040);
  ip4[8] = 64;
  ip4[9] = 17;
  st32(ip4 + 12, saddr);
  st32(ip4 + 16, daddr);
  st16(ip4 + 10, 0);
  uint8_t* udp = ip4 + 20;
  st16(udp + 0, sport);
  st16(udp + 2, dport);
  st16(udp + 4, htons_(8));
  st16(udp + 6, 0);
  uint32_t cache = 0;
  for (int i = 0; i < 10; i++) cache += ld16(ip4 + 2 * i);
  cache = (cache >> 16u) + (cache & 0xffff);
  cache += (cache >> 16u);
  return cache;
}

static void udp_update_pkt(uint8_t* eth, uint32_t ipsum_cache, uint32_t paylen) { /* Efvi.h:611-621 */
  uint8_t* ip4 = eth + 14;
  uint16_t iplen = htons_((uint16_t)(28 + paylen));
  st16(ip4 + 2, iplen);
  uint32_t ipsum = ipsum_cache + iplen;
  ipsum += (ipsum >> 16u);
  st16(ip4 + 10, (uint16_t)(~ipsum & 0xffff));
  st16(ip4 + 20 + 4, htons_((uint16_t)(8 + paylen)));
}

/* ---- the batch a reference sender produces ---- */
static uint64_t splitmix(uint64_t* s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

int orc_tx_build_batch(uint64_t seed, uint32_t n, uint8_t* slots, uint32_t stride, uint32_t frame_off, uint32_t mode,
                       uint16_t* lens, uint8_t* kinds) {
  const uint32_t avail = stride - frame_off;
  if (avail < OPT + 12 + 64 || (frame_off & 1)) return -1;
  uint64_t s = seed;
  enum { NCONN = 64 };
  static const uint8_t local_mac[6] = {0x02, 0, 0, 0, 0, 0x01};
  const uint32_t local_ip = htonl_(0x0A000001u);
  tx_conn conns[NCONN];
  for (int k = 0; k < NCONN; k++) {
    tx_conn* c = &conns[k];
    memset(c, 0, sizeof(*c));
    memcpy(c->src_mac, local_mac, 6);
    for (int b = 0; b < 6; b++) c->dst_mac[b] = (uint8_t)splitmix(&s);
    c->local_ip = local_ip;
    c->dst_ip = (uint32_t)splitmix(&s);
    c->src_port = (uint16_t)splitmix(&s);
    c->dst_port = (uint16_t)splitmix(&s);
    c->has_ts = 1; /* Conf::TimestampOption */
    c->has_ws = (int)(splitmix(&s) & 1);
    c->recv_wnd_shift = (uint32_t)(splitmix(&s) % 15);
    conn_reset(c, (uint32_t)splitmix(&s));
  }
  rst_buf rb;
  rst_init(&rb, local_mac, local_ip);
  uint8_t* data = (uint8_t*)malloc(avail);
  if (!data) return -1;
  uint32_t udp_cache = 0;
  uint8_t udp_hdr[42];
  for (uint32_t i = 0; i < n; i++) {
    uint8_t* eth = slots + (uint64_t)i * stride + frame_off;
    memset(eth, 0, avail);
    const uint64_t r = splitmix(&s);
    if (mode == PN_TX_UDP_EFVI) {
      if (i % 97 == 0) /* a new destination every so often: init_udp_pkt + its cache */
        udp_cache = udp_init_pkt(udp_hdr, local_mac, conns[r % NCONN].dst_mac, local_ip, (uint32_t)splitmix(&s),
                                 (uint16_t)splitmix(&s), (uint16_t)splitmix(&s));
      uint32_t paylen = (uint32_t)(splitmix(&s) % 1473);
      if (14 + 28 + paylen > avail) paylen = avail - 42;
      memcpy(eth, udp_hdr, 42);
      for (uint32_t b = 0; b < paylen; b++) eth[42 + b] = (uint8_t)splitmix(&s);
      udp_update_pkt(eth, udp_cache, paylen);
      lens[i] = (uint16_t)paylen;
      kinds[i] = 5;
      continue;
    }
    tx_conn* c = &conns[r % NCONN];
    const uint32_t ack = (uint32_t)splitmix(&s), now_ts = (uint32_t)splitmix(&s), recent = (uint32_t)splitmix(&s);
    const uint16_t window = (uint16_t)splitmix(&s);
    uint32_t kind = (uint32_t)((r >> 8) % 100);
    kind = kind < 65 ? 0 : kind < 75 ? 1 : kind < 85 ? 2 : kind < 93 ? 3 : 4;
    if (kind == 1 && c->established) kind = 0;
    if (kind != 1 && !c->established) { /* handshake first: SYN, then the peer's answer */
      memcpy(eth, c->hdr, OPT + 4);
      lens[i] = (uint16_t)send_syn(c, eth, (int)((r >> 40) & 1), ack, window, now_ts, recent);
      kinds[i] = 1;
      conn_establish(c, (int)((r >> 41) % 4 != 0));
      continue;
    }
    if (kind == 0 || kind == 2) {
      const uint32_t smss = PN_RECV_MSS - (c->has_ts ? 12 : 0);
      uint32_t len = (uint32_t)(splitmix(&s) % (smss + 1));
      if ((r >> 44) % 16 == 0) len = (uint32_t)((r >> 48) % 8); /* tiny segments */
      if (OPT + 12 + len > avail) len = avail - OPT - 12;
      for (uint32_t b = 0; b < len; b++) data[b] = (uint8_t)splitmix(&s);
      uint32_t pieces[4], np = 1 + (uint32_t)((r >> 52) % 4);
      for (uint32_t k = 0; k < np; k++) pieces[k] = (uint32_t)(splitmix(&s) % (len + 1));
      lens[i] = (uint16_t)send_data(c, eth, (uint32_t)splitmix(&s), data, len, pieces, np, ack, window, now_ts, recent);
      kinds[i] = 0;
      if (kind == 2) { /* later retransmitted with fresh ack / window / timestamps */
        resend_una(c, eth, (uint32_t)splitmix(&s), (uint16_t)splitmix(&s), (uint32_t)splitmix(&s), (uint32_t)splitmix(&s));
        kinds[i] = 2;
      }
    } else if (kind == 1) {
      memcpy(eth, c->hdr, OPT + 4);
      lens[i] = (uint16_t)send_syn(c, eth, (int)((r >> 40) & 1), ack, window, now_ts, recent);
      kinds[i] = 1;
    } else if (kind == 3) { /* RST answering an incoming segment */
      uint8_t in[OPT];
      memset(in, 0, sizeof(in));
      for (int b = 0; b < OPT; b++) in[b] = (uint8_t)splitmix(&s);
      in[TCP + 13] &= (uint8_t)~0x04; /* not itself a RST */
      st16(in + IP + 2, htons_((uint16_t)(40 + splitmix(&s) % 1461)));
      in[TCP + 12] = (uint8_t)((5 + splitmix(&s) % 11) << 4);
      rsp_rst(&rb, in);
      memcpy(eth, rb.f, OPT + 12);
      lens[i] = 0;
      kinds[i] = 3;
    } else { /* TIME_WAIT ACK */
      const int ts = (int)((r >> 40) & 1);
      ack_tw(&rb, c->dst_mac, c->dst_ip, c->src_port, c->dst_port, (uint32_t)splitmix(&s), (uint32_t)splitmix(&s), ts,
             now_ts, recent);
      memcpy(eth, rb.f, OPT + 12);
      lens[i] = ts ? 12 : 0;
      kinds[i] = 4;
    }
  }
  free(data);
  return 0;
}

/* ---- (2) the fill restated from the frame bytes: pn_tx_fill's contract ---- */
static uint32_t word_sum(const uint8_t* p, uint32_t len) { /* RFC 1071, odd tail zero-padded */
  uint32_t s = 0;
  for (uint32_t k = 0; k + 1 < len; k += 2) s += ld16(p + k);
  if (len & 1) s += p[len - 1];
  return s;
}

int orc_tx_fill_frame(uint8_t* eth, uint32_t avail, int has_len, uint16_t len, uint32_t mode) {
  uint8_t* ip = eth + IP;
  const uint32_t hdr = mode == PN_TX_TCP ? 40 : 28;
  uint32_t tot = has_len ? ((hdr + len) & 0xffff) : htons_(ld16(ip + 2));
  if (tot < hdr || 14 + tot > avail) return 0; /* left untouched */
  if (mode == PN_TX_UDP) { /* CSum::fold of the 20-byte header */
    if (has_len) {
      st16(ip + 2, htons_((uint16_t)tot));
      st16(ip + 24, htons_((uint16_t)(8 + len)));
    }
    st16(ip + 10, 0);
    orc_csum a = {word_sum(ip, 20)};
    st16(ip + 10, orc_csum_fold(a));
    return 1;
  }
  if (mode == PN_TX_UDP_EFVI) {
    if (has_len) {
      st16(ip + 2, htons_((uint16_t)tot));
      st16(ip + 24, htons_((uint16_t)(8 + len)));
    }
    uint32_t cache = word_sum(ip, 20) - ld16(ip + 2) - ld16(ip + 10);
    cache = (cache >> 16) + (cache & 0xffff);
    cache += cache >> 16;
    uint32_t ipsum = cache + ld16(ip + 2);
    ipsum += ipsum >> 16;
    st16(ip + 10, (uint16_t)(~ipsum & 0xffff));
    return 1;
  }
  if (has_len) st16(ip + 2, htons_((uint16_t)tot));
  st16(ip + 10, 0);
  orc_csum a = {word_sum(ip, 20)};
  st16(ip + 10, orc_csum_fold(a));
  uint8_t* tcp = ip + 20;
  st16(tcp + 16, 0);
  orc_csum b = {0};
  orc_csum_add32(&b, ld32(ip + 12));
  orc_csum_add32(&b, ld32(ip + 16));
  orc_csum_add16(&b, htons_(6));
  orc_csum_add16(&b, htons_((uint16_t)(tot - 20)));
  b.sum += word_sum(tcp, tot - 20);
  st16(tcp + 16, orc_csum_fold(b));
  return 1;
}

typedef struct fill_job {
  uint8_t* slots;
  uint32_t stride, off, lo, hi, mode;
  const uint16_t* lens;
} fill_job;

static void* run_fill(void* arg) {
  fill_job* j = (fill_job*)arg;
  for (uint32_t i = j->lo; i < j->hi; i++)
    orc_tx_fill_frame(j->slots + (uint64_t)i * j->stride + j->off, j->stride - j->off, j->lens != NULL,
                      j->lens ? j->lens[i] : 0, j->mode);
  return NULL;
}

void orc_tx_fill_batch(uint8_t* slots, uint32_t stride, uint32_t frame_off, uint32_t n, const uint16_t* lens,
                       uint32_t mode, int n_threads) {
  if (n_threads < 1) n_threads = 1;
  if (n_threads > 256) n_threads = 256;
  fill_job jobs[256];
  pthread_t th[256];
  for (int t = 0; t < n_threads; t++) {
    jobs[t] = (fill_job){slots, stride, frame_off, (uint32_t)((uint64_t)n * t / n_threads),
                         (uint32_t)((uint64_t)n * (t + 1) / n_threads), mode, lens};
    if (n_threads == 1) run_fill(&jobs[0]);
    else pthread_create(&th[t], NULL, run_fill, &jobs[t]);
  }
  if (n_threads > 1)
    for (int t = 0; t < n_threads; t++) pthread_join(th[t], NULL);
}

/* The reference's own per-segment TX byte work on the same batch: copyAndSum of each
 * frame's segment into a send buffer + setOptDataLen (TcpConn.h:238-240, Core.h:157-163)
 * — the CPU figure pn_tx_fill's device rate is set beside (bench.py --path tx). */
typedef struct cas_job {
  const uint8_t* slots;
  uint8_t* out;
  uint32_t stride, off, lo, hi;
} cas_job;

static void* run_cas(void* arg) {
  cas_job* j = (cas_job*)arg;
  for (uint32_t i = j->lo; i < j->hi; i++) {
    const uint8_t* eth = j->slots + (uint64_t)i * j->stride + j->off;
    uint8_t* dst = j->out + (uint64_t)i * j->stride + j->off;
    uint32_t tot = htons_(ld16(eth + IP + 2));
    if (tot < 40 || 14 + tot > j->stride - j->off) continue;
    memcpy(dst, eth, OPT);
    orc_csum sum = copy_and_sum(dst + OPT, eth + OPT, tot - 40);
    orc_csum ipsum = {word_sum(eth + IP, 20) - ld16(eth + IP + 2) - ld16(eth + IP + 10)};
    orc_csum_add32(&sum, ld32(eth + IP + 12));
    orc_csum_add32(&sum, ld32(eth + IP + 16));
    orc_csum_add16(&sum, htons_(6));
    sum.sum += word_sum(eth + TCP, 20) - ld16(eth + TCP + 16);
    set_opt_data_len(dst, (uint16_t)(tot - 40), ipsum, sum);
  }
  return NULL;
}

void orc_tx_copy_and_sum_batch(const uint8_t* slots, uint8_t* out, uint32_t stride, uint32_t frame_off, uint32_t n,
                               int n_threads) {
  if (n_threads < 1) n_threads = 1;
  if (n_threads > 256) n_threads = 256;
  cas_job jobs[256];
  pthread_t th[256];
  for (int t = 0; t < n_threads; t++) {
    jobs[t] = (cas_job){slots, out, stride, frame_off, (uint32_t)((uint64_t)n * t / n_threads),
                        (uint32_t)((uint64_t)n * (t + 1) / n_threads)};
    if (n_threads == 1) run_cas(&jobs[0]);
    else pthread_create(&th[t], NULL, run_cas, &jobs[t]);
  }
  if (n_threads > 1)
    for (int t = 0; t < n_threads; t++) pthread_join(th[t], NULL);
}
