/*
 * pn_oracle.c — plain-C restatement of efvitcp's receive-path per-frame
 * transform.  TEST INFRASTRUCTURE: the checker for the HIP kernel and the timed
 * CPU baseline ("port"); never linked into libpollnet_amd.  Header pinning notes
 * are in pn_oracle.h.
 *
 * Deliberately written as literal scalar loops in the reference's own order
 * (u16 loads, u32 accumulator, per-entry probing) so that it shares no
 * formulation with the GPU kernel (dword dot-products, lane reductions).
 */
#define _GNU_SOURCE
#include "pn_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

static inline uint16_t ld16(const uint8_t* p) { /* *(uint16_t*)p on little-endian x86 */
  uint16_t v;
  memcpy(&v, p, 2);
  return v;
}
static inline uint32_t ld32(const uint8_t* p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}
static inline uint16_t bswap16(uint16_t v) { return (uint16_t)((v >> 8) | (v << 8)); }
static inline uint32_t bswap32(uint32_t v) { return __builtin_bswap32(v); }

/* ---------------- CSum, Core.h:89-138 ---------------- */
uint16_t orc_csum_fold(orc_csum s) { /* Core.h:94-98 */
  uint32_t res = (s.sum >> 16) + (s.sum & 0xffff);
  res += res >> 16;
  return (uint16_t)~res;
}
void orc_csum_add16(orc_csum* s, uint16_t a) { s->sum += a; } /* Core.h:100 */
void orc_csum_add32(orc_csum* s, uint32_t a) {                /* Core.h:101-104 */
  s->sum += a >> 16;
  s->sum += a & 0xffff;
}
void orc_csum_add_bytes(orc_csum* s, const void* p, uint32_t len) { /* Core.h:106-117 */
  /* The reference's loop `add(*(uint16_t*)(p + i))` keeps `sum` in a register
   * (a uint16_t load cannot alias the uint32_t member); accumulate locally so this
   * restatement compiles to the same vectorised loop. */
  const uint8_t* b = (const uint8_t*)p;
  uint32_t sum = s->sum;
  const uint32_t words = (uint32_t)(((uint64_t)len + 1) >> 1); /* odd len: the last word reads b[len] too */
  for (uint32_t k = 0; k < words; k++) sum += ld16(b + 2 * (uint64_t)k);
  s->sum = sum;
}

/* ---------------- connHashKey, Core.h:167-172 ---------------- */
uint64_t orc_conn_hash_key(uint32_t ip_be, uint16_t port_be) {
  uint64_t key = bswap32(ip_be);
  uint64_t p = bswap16(port_be);
  return (key << 15) | (p & 0x7fff) | ((p & 0x8000) << 32);
}

/* ---------------- conn table ---------------- */
static int get_msb(uint32_t n) { return n == 0 ? 0 : get_msb(n >> 1) + 1; } /* Core.h:174-176 */

int orc_table_init(orc_table* t, uint32_t max_conn, uint32_t max_tw) { /* Core.h:235-236, 321-322 */
  memset(t, 0, sizeof(*t));
  t->max_conn = max_conn;
  t->max_tw = max_tw;
  t->max_table_size = 1u << (1 + get_msb(max_conn + max_tw));
  t->total = t->max_table_size + max_conn + max_tw;
  t->tbl = (pn_conn_entry*)calloc(t->total, sizeof(pn_conn_entry));
  if (!t->tbl) return -1;
  for (uint32_t i = 0; i < t->total; i++) t->tbl[i].key = PN_EMPTY_KEY;
  t->mask = (t->max_table_size < 128 ? t->max_table_size : 128) - 1;
  t->size = 0;
  return 0;
}
void orc_table_free(orc_table* t) {
  free(t->tbl);
  t->tbl = NULL;
}

static uint32_t find_raw(const pn_conn_entry* tbl, uint32_t n, uint64_t mask, uint64_t key) {
  /* Core.h:558-562.  Bounded at n (the reference relies on an EmptyKey sentinel). */
  uint32_t e = (uint32_t)(key & mask);
  while (e < n && tbl[e].key < key) e++;
  return e;
}
uint32_t orc_table_find(const orc_table* t, uint64_t key) { return find_raw(t->tbl, t->total, t->mask, key); }

static void swap_entry(pn_conn_entry* a, pn_conn_entry* b) {
  pn_conn_entry x = *a;
  *a = *b;
  *b = x;
}

static void try_expand(orc_table* t) { /* Core.h:650-682 */
  if ((uint64_t)t->size * 2 <= t->mask) return;
  uint64_t end = t->mask + 1;
  t->mask = t->mask * 2 + 1;
  uint64_t new_end = t->mask + 1;
  while (t->tbl[end].key != PN_EMPTY_KEY) swap_entry(&t->tbl[new_end++], &t->tbl[end++]);
  uint64_t end_cnt = new_end - (t->mask + 1);
  uint64_t starts[2] = {0, t->mask + 1};
  uint64_t cnts[2] = {t->size - end_cnt, end_cnt};
  for (int r = 0; r < 2; r++) { /* the `rehash` lambda, Core.h:660-675 */
    uint64_t e = starts[r], cnt = cnts[r];
    for (; cnt; e++) {
      if (t->tbl[e].key == PN_EMPTY_KEY) continue;
      uint32_t ne = orc_table_find(t, t->tbl[e].key);
      uint64_t k = t->tbl[e].key;
      t->tbl[e].key = t->tbl[ne].key;
      t->tbl[ne].key = k;
      t->tbl[ne].conn_id = t->tbl[e].conn_id;
      cnt--;
    }
  }
}

int orc_table_add(orc_table* t, uint64_t key, uint32_t conn_id) { /* Core.h:566-576 */
  uint32_t e = orc_table_find(t, key);
  if (e < t->total && t->tbl[e].key == key) return -1;
  if (t->size >= t->max_conn + t->max_tw) return -2;
  t->size++; /* callers bump conn_cnt/tw_cnt before addConnEntry (TcpServer.h:88-89) */
  while (t->tbl[e].key != PN_EMPTY_KEY) {
    uint64_t k = t->tbl[e].key;
    uint32_t c = t->tbl[e].conn_id;
    t->tbl[e].key = key;
    t->tbl[e].conn_id = conn_id;
    key = k;
    conn_id = c;
    while (t->tbl[++e].key < key)
      ;
  }
  t->tbl[e].key = key;
  t->tbl[e].conn_id = conn_id;
  try_expand(t);
  return 0;
}

int orc_table_del(orc_table* t, uint64_t key) { /* Core.h:578-605 */
  uint32_t e = orc_table_find(t, key);
  if (e >= t->total || t->tbl[e].key != key) return -1;
  t->size--;
  for (;;) {
    uint32_t next = e + 1;
    while ((t->tbl[next].key & t->mask) > e) next++;
    if (t->tbl[next].key == PN_EMPTY_KEY) break;
    t->tbl[e] = t->tbl[next];
    e = next;
  }
  t->tbl[e].key = PN_EMPTY_KEY;
  return 0;
}

/* ---------------- per-frame transform ---------------- */
/* verify_tcp = 0: the record pn_classify writes under pn_set_verify(ctx, 0) -- everything but the TCP
 * verdict (no segment sum: PN_F_TCP_UNCHECKED, tcp_fold 0xFFFF), the IP verdicts from the header alone */
static void classify_frame(const uint8_t* eth, uint32_t avail, const pn_conn_entry* tbl, uint32_t n_entries,
                           uint64_t mask, uint32_t max_conn, pn_result* out, int with_rfc, int verify_tcp) {
  const uint8_t* ip = eth + 14;  /* Core.h:506 */
  const uint8_t* tcp = ip + 20;  /* Core.h:507: IHL assumed 5 */
  uint32_t flags = 0;

  uint16_t ether_type = ld16(eth + 12);
  uint8_t ver_ihl = ip[0];
  uint32_t ihl = ver_ihl & 0xf; /* IpHeader::header_len, low nibble (Core.h:59) */
  uint32_t tot_len = bswap16(ld16(ip + 2));
  if (ether_type != 0x0008 || (ver_ihl >> 4) != 4 || ip[9] != 6) flags |= PN_F_NOT_TCP; /* TcpStream.h:45-46 */
  if (ihl != 5) flags |= PN_F_IHL_NE_5;

  /* TcpHeader bitfields (Core.h:80): byte 12 high nibble = data_offset, byte 13 = fin/syn/rst/psh/ack */
  uint32_t doff = tcp[12] >> 4;
  uint8_t fl = tcp[13];
  uint32_t fin = fl & 1, syn = (fl >> 1) & 1, rst = (fl >> 2) & 1, psh = (fl >> 3) & 1, ack = (fl >> 4) & 1;
  if (fin) flags |= PN_F_FIN;
  if (syn) flags |= PN_F_SYN;
  if (rst) flags |= PN_F_RST;
  if (psh) flags |= PN_F_PSH;
  if (ack) flags |= PN_F_ACK;

  /* Core::checksum, Core.h:449-466 (EFVITCP_DEBUG), restated non-exiting */
  orc_csum s = {0};
  orc_csum_add_bytes(&s, ip, 20); /* add<sizeof(IpHeader)> */
  uint16_t ip_fold = orc_csum_fold(s);
  if (ip_fold == 0) flags |= PN_F_IP_OK;

  uint16_t tcp_len = (uint16_t)(tot_len - 20); /* uint16_t tcp_len = ntohs(tot_len) - 20 */
  uint32_t tcp_len_even = ((uint32_t)tcp_len + 1) & ~1u;
  uint16_t tcp_fold = 0xFFFF;
  int trunc = (14u + 20u + tcp_len_even) > avail;
  if (trunc) {
    flags |= PN_F_TRUNC;
    if (!verify_tcp) flags |= PN_F_TCP_UNCHECKED;
  } else if (!verify_tcp) {
    flags |= PN_F_TCP_UNCHECKED;
    uint32_t hl = ihl * 4;
    if (with_rfc && ihl >= 5 && hl <= tot_len) {
      orc_csum r = {0};
      orc_csum_add_bytes(&r, ip, hl);
      if (orc_csum_fold(r) == 0) flags |= PN_F_RFC_IP_OK;
    }
  } else {
    orc_csum t = {0};
    orc_csum_add32(&t, ld32(ip + 12)); /* src_ip */
    orc_csum_add32(&t, ld32(ip + 16)); /* dst_ip */
    orc_csum_add16(&t, bswap16(6));    /* ntohs(0x6) */
    orc_csum_add16(&t, bswap16(tcp_len));
    orc_csum_add_bytes(&t, tcp, tcp_len); /* CSum::add(p, len) */
    tcp_fold = orc_csum_fold(t);
    if (tcp_fold == 0) flags |= PN_F_TCP_OK;

    /* RFC 791 / 793 verdicts (not part of the reference; C5's ihl_ne_5 companion) */
    uint32_t hl = ihl * 4;
    if (with_rfc && ihl >= 5 && hl <= tot_len) {
      orc_csum r = {0};
      orc_csum_add_bytes(&r, ip, hl);
      if (orc_csum_fold(r) == 0) flags |= PN_F_RFC_IP_OK;
      uint32_t seg = tot_len - hl;
      orc_csum q = {0};
      orc_csum_add32(&q, ld32(ip + 12));
      orc_csum_add32(&q, ld32(ip + 16));
      orc_csum_add16(&q, bswap16(6));
      orc_csum_add16(&q, bswap16((uint16_t)seg));
      const uint8_t* sp = ip + hl;
      orc_csum_add_bytes(&q, sp, seg & ~1u);
      if (seg & 1) orc_csum_add16(&q, (uint16_t)sp[seg - 1]); /* zero-padded odd byte */
      if (orc_csum_fold(q) == 0) flags |= PN_F_RFC_TCP_OK;
    }
  }

  /* connHashKey + findConnEntry + TIME_WAIT test, Core.h:508-510 */
  uint64_t key = orc_conn_hash_key(ld32(ip + 12), ld16(tcp + 0));
  uint32_t e = find_raw(tbl, n_entries, mask, key);
  uint32_t conn_id = PN_MISS;
  if (e < n_entries && tbl[e].key == key) {
    conn_id = tbl[e].conn_id;
    flags |= PN_F_HIT;
    if (conn_id >= max_conn) flags |= PN_F_TW;
  }

  /* TcpConn::onPack header part, TcpConn.h:469-473 */
  int data_off = 14 + 20 + (int)doff * 4;
  int end = 14 + (int)(tot_len < 1500 ? tot_len : 1500);
  out->conn_id = conn_id;
  out->seq = bswap32(ld32(tcp + 4)) + syn;
  out->payload_off = (uint16_t)data_off;
  out->payload_len = (int16_t)(end - data_off);
  out->flags = (uint16_t)flags;
  out->tcp_fold = tcp_fold;
}

void orc_classify_frame(const uint8_t* eth, uint32_t avail, const pn_conn_entry* tbl, uint32_t n_entries,
                        uint64_t mask, uint32_t max_conn, pn_result* out) {
  classify_frame(eth, avail, tbl, n_entries, mask, max_conn, out, 1, 1);
}
void orc_classify_frame_release(const uint8_t* eth, uint32_t avail, const pn_conn_entry* tbl, uint32_t n_entries,
                                uint64_t mask, uint32_t max_conn, pn_result* out) {
  classify_frame(eth, avail, tbl, n_entries, mask, max_conn, out, 1, 0);
}

static void release_frame(const uint8_t* eth, const pn_conn_entry* tbl, uint32_t n_entries, uint64_t mask,
                          uint32_t max_conn, pn_result* out) {
  /* Core.h:503-510 + TcpConn.h:469-473 only: what the release build does per RX event */
  const uint8_t* ip = eth + 14;
  const uint8_t* tcp = ip + 20;
  uint64_t key = orc_conn_hash_key(ld32(ip + 12), ld16(tcp));
  uint32_t e = find_raw(tbl, n_entries, mask, key);
  uint32_t conn_id = PN_MISS, flags = 0;
  if (e < n_entries && tbl[e].key == key) {
    conn_id = tbl[e].conn_id;
    flags |= PN_F_HIT | (conn_id >= max_conn ? PN_F_TW : 0);
  }
  uint32_t tot_len = bswap16(ld16(ip + 2));
  uint32_t doff = tcp[12] >> 4;
  uint8_t fl = tcp[13];
  flags |= (uint32_t)(fl & 0x1f) << 4; /* fin..ack -> PN_F_FIN..PN_F_ACK */
  int data_off = 34 + (int)doff * 4;
  out->conn_id = conn_id;
  out->seq = bswap32(ld32(tcp + 4)) + ((fl >> 1) & 1);
  out->payload_off = (uint16_t)data_off;
  out->payload_len = (int16_t)(14 + (int)(tot_len < 1500 ? tot_len : 1500) - data_off);
  out->flags = (uint16_t)flags;
  out->tcp_fold = 0xFFFF; /* not computed (the GPU release path's sentinel) */
}

typedef struct job {
  const uint8_t* slots;
  uint32_t stride, off, lo, hi;
  const pn_conn_entry* tbl;
  uint32_t n_entries;
  uint64_t mask;
  uint32_t max_conn;
  pn_result* out;
  int mode; /* 0 full (REF + RFC), 1 release path, 2 REF checksum path only, 3 pn_set_verify(ctx, 0) records */
} job;

static void* run_job(void* arg) {
  job* j = (job*)arg;
  uint32_t avail = j->stride - j->off;
  for (uint32_t i = j->lo; i < j->hi; i++) {
    const uint8_t* eth = j->slots + (uint64_t)i * j->stride + j->off;
    if (j->mode == 1)
      release_frame(eth, j->tbl, j->n_entries, j->mask, j->max_conn, &j->out[i]);
    else
      classify_frame(eth, avail, j->tbl, j->n_entries, j->mask, j->max_conn, &j->out[i], j->mode != 2, j->mode != 3);
  }
  return NULL;
}

static void run_batch(const uint8_t* slots, uint32_t stride, uint32_t off, uint32_t n, const pn_conn_entry* tbl,
                      uint32_t n_entries, uint64_t mask, uint32_t max_conn, pn_result* out, int n_threads,
                      int mode) {
  if (n_threads < 1) n_threads = 1;
  if (n_threads > 256) n_threads = 256;
  job jobs[256];
  pthread_t th[256];
  for (int k = 0; k < n_threads; k++) { /* contiguous index shards */
    jobs[k] = (job){slots, stride, off, (uint32_t)((uint64_t)n * k / n_threads),
                    (uint32_t)((uint64_t)n * (k + 1) / n_threads), tbl, n_entries, mask, max_conn, out, mode};
  }
  if (n_threads == 1) {
    run_job(&jobs[0]);
    return;
  }
  for (int k = 0; k < n_threads; k++) pthread_create(&th[k], NULL, run_job, &jobs[k]);
  for (int k = 0; k < n_threads; k++) pthread_join(th[k], NULL);
}

void orc_classify_batch(const uint8_t* slots, uint32_t slot_stride, uint32_t frame_off, uint32_t n,
                        const pn_conn_entry* tbl, uint32_t n_entries, uint64_t mask, uint32_t max_conn,
                        pn_result* out, int n_threads) {
  run_batch(slots, slot_stride, frame_off, n, tbl, n_entries, mask, max_conn, out, n_threads, 0);
}

void orc_release_batch(const uint8_t* slots, uint32_t slot_stride, uint32_t frame_off, uint32_t n,
                       const pn_conn_entry* tbl, uint32_t n_entries, uint64_t mask, uint32_t max_conn,
                       pn_result* out, int n_threads) {
  run_batch(slots, slot_stride, frame_off, n, tbl, n_entries, mask, max_conn, out, n_threads, 1);
}

void orc_refsum_batch(const uint8_t* slots, uint32_t slot_stride, uint32_t frame_off, uint32_t n,
                      const pn_conn_entry* tbl, uint32_t n_entries, uint64_t mask, uint32_t max_conn,
                      pn_result* out, int n_threads) {
  run_batch(slots, slot_stride, frame_off, n, tbl, n_entries, mask, max_conn, out, n_threads, 2);
}

void orc_classify_batch_unverified(const uint8_t* slots, uint32_t slot_stride, uint32_t frame_off, uint32_t n,
                                   const pn_conn_entry* tbl, uint32_t n_entries, uint64_t mask, uint32_t max_conn,
                                   pn_result* out, int n_threads) {
  run_batch(slots, slot_stride, frame_off, n, tbl, n_entries, mask, max_conn, out, n_threads, 3);
}

/* ---- chain links (pn_service_post_linked) ---- */
static int orc_chain_usable(const pn_result* r) {
  const uint32_t f = r->flags;
  const uint32_t need = PN_F_HIT | PN_F_ACK | PN_F_IP_OK;
  const uint32_t none = PN_F_TW | PN_F_SYN | PN_F_FIN | PN_F_RST | PN_F_NOT_TCP | PN_F_TRUNC | PN_F_BADOFF | PN_F_IHL_NE_5;
  return (f & need) == need && (f & none) == 0 && (f & (PN_F_TCP_OK | PN_F_TCP_UNCHECKED)) != 0 && r->payload_len > 0;
}

void orc_chain_links(const uint8_t* slots, uint32_t slot_stride, uint32_t frame_off, uint32_t n, const pn_result* recs,
                     uint32_t max_conn, uint32_t max_frames, uint32_t max_conns, uint16_t* links) {
  memset(links, 0, (size_t)n * sizeof(uint16_t));
  if (n > max_frames || max_conn > max_conns || n == 0) return;
  uint32_t* last = (uint32_t*)malloc((size_t)(max_conn ? max_conn : 1) * sizeof(uint32_t)); /* 1 + index, 0 = none */
  memset(last, 0, (size_t)(max_conn ? max_conn : 1) * sizeof(uint32_t));
  for (uint32_t i = 0; i < n; i++) {
    const pn_result* r = &recs[i];
    if ((r->flags & (PN_F_HIT | PN_F_TW)) != PN_F_HIT || r->conn_id >= max_conn) continue;
    const uint32_t pj = last[r->conn_id];
    last[r->conn_id] = i + 1;
    if (!pj) continue;
    const uint32_t j = pj - 1;
    const pn_result* q = &recs[j];
    if (!orc_chain_usable(r) || !orc_chain_usable(q)) continue;
    if (r->seq != q->seq + (uint32_t)q->payload_len || r->payload_off != q->payload_off) continue;
    const uint8_t* ei = slots + (size_t)i * slot_stride + frame_off;
    const uint8_t* ej = slots + (size_t)j * slot_stride + frame_off;
    /* ack number (tcp + 8), window (tcp + 14), destination address (ip + 16) and port (tcp + 2), IHL 5 */
    if (memcmp(ei + 42, ej + 42, 4) || memcmp(ei + 48, ej + 48, 2) || memcmp(ei + 30, ej + 30, 4) ||
        memcmp(ei + 36, ej + 36, 2))
      continue;
    links[i] = (uint16_t)(i - j);
  }
  free(last);
}
