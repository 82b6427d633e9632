/*
 * pn_oracle.h — CPU restatement of efvitcp's RX per-frame transform.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load or call this code, and only as the
 * checker / the timed CPU baseline — never as the product path.
 *
 * Parity pinning:
 *   - the reference's OWN efvitcp/Core.h code for this path, compiled verbatim from
 *     /root/reference (oracle/ref_core.cc -> oracle/_ref/libref_core.so, line ranges
 *     extracted by oracle/ref.mk; no ef_vi header needed or faked): CSum, the header
 *     bitfield layouts, connHashKey, Core::checksum, the conn table's member
 *     functions and TcpConn::onPack's payload statements (TcpConn.h:469-473) —
 *     tests/test_ref_core.py checks this restatement against them on the committed
 *     fixtures, the config slices, random inputs and table histories;
 *   - the reference's own TcpStream.h compiled the same way (oracle/_ref/libref_tcpstream.so:
 *     ethertype/protocol filter, IHL=5 payload split);
 *   - RFC 1071 known answers (tests/golden/known_answers.json) and real kernel-generated
 *     IPv4 headers captured on loopback.
 * Every function cites the reference line it restates.
 */
#ifndef PN_ORACLE_H
#define PN_ORACLE_H
#include <stdint.h>
#include "../include/pollnet_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* CSum (Core.h:89-138): u32 accumulator of host-order u16 words. */
typedef struct orc_csum { uint32_t sum; } orc_csum;
uint16_t orc_csum_fold(orc_csum s);                               /* Core.h:94-98 */
void orc_csum_add16(orc_csum* s, uint16_t a);                     /* Core.h:100 */
void orc_csum_add32(orc_csum* s, uint32_t a);                     /* Core.h:101-104 */
void orc_csum_add_bytes(orc_csum* s, const void* p, uint32_t len); /* Core.h:106-117 (reads ceil(len/2) words) */

uint64_t orc_conn_hash_key(uint32_t ip_be, uint16_t port_be); /* Core.h:167-172 */

/* Ordered linear-probe conn table (Core.h:178-182, 235-236, 321-322, 558-682). */
typedef struct orc_table {
  pn_conn_entry* tbl;
  uint32_t total;          /* TotalTableSize */
  uint32_t max_table_size; /* MaxTableSize */
  uint32_t max_conn, max_tw;
  uint64_t mask;           /* tbl_mask */
  uint32_t size;           /* conn_cnt + tw_cnt */
} orc_table;
int orc_table_init(orc_table* t, uint32_t max_conn, uint32_t max_tw);
void orc_table_free(orc_table* t);
uint32_t orc_table_find(const orc_table* t, uint64_t key);               /* Core.h:558-562 (bounded) */
int orc_table_add(orc_table* t, uint64_t key, uint32_t conn_id);         /* Core.h:566-576 + 650-682 */
int orc_table_del(orc_table* t, uint64_t key);                           /* Core.h:578-605 */

/* One frame: eth points at the Ethernet header; `avail` = readable bytes from eth
 * to the end of its slot.  Table may be described by raw entries + mask. */
void orc_classify_frame(const uint8_t* eth, uint32_t avail, const pn_conn_entry* tbl, uint32_t n_entries,
                        uint64_t mask, uint32_t max_conn, pn_result* out);
/* The record pn_classify writes under pn_set_verify(ctx, 0): every field and verdict of
 * orc_classify_frame but the TCP one (no segment sum; PN_F_TCP_UNCHECKED, tcp_fold 0xFFFF). */
void orc_classify_frame_release(const uint8_t* eth, uint32_t avail, const pn_conn_entry* tbl, uint32_t n_entries,
                                uint64_t mask, uint32_t max_conn, pn_result* out);

/* Batch over strided slots; n_threads <= 1 runs single-threaded (pthreads otherwise). */
void orc_classify_batch(const uint8_t* slots, uint32_t slot_stride, uint32_t frame_off, uint32_t n,
                        const pn_conn_entry* tbl, uint32_t n_entries, uint64_t mask, uint32_t max_conn,
                        pn_result* out, int n_threads);

/* The reference's *release* RX path only (no checksum): parse + key + probe +
 * onPack payload math (Core.h:503-509, TcpConn.h:469-473).  Timed as the second
 * CPU-baseline variant.  Writes the same records with the two *_OK bits clear. */
void orc_release_batch(const uint8_t* slots, uint32_t slot_stride, uint32_t frame_off, uint32_t n,
                       const pn_conn_entry* tbl, uint32_t n_entries, uint64_t mask, uint32_t max_conn,
                       pn_result* out, int n_threads);

/* "ref parse + checksum": exactly the reference's work (Core::checksum + pollNet +
 * onPack header) without this oracle's RFC extras; RFC bits left clear.  Timed as
 * the primary CPU baseline. */
void orc_refsum_batch(const uint8_t* slots, uint32_t slot_stride, uint32_t frame_off, uint32_t n,
                      const pn_conn_entry* tbl, uint32_t n_entries, uint64_t mask, uint32_t max_conn,
                      pn_result* out, int n_threads);

/* orc_classify_frame_release over a batch: the expected records of pn_set_verify(ctx, 0). */
void orc_classify_batch_unverified(const uint8_t* slots, uint32_t slot_stride, uint32_t frame_off, uint32_t n,
                                   const pn_conn_entry* tbl, uint32_t n_entries, uint64_t mask, uint32_t max_conn,
                                   pn_result* out, int n_threads);

/* Chain links over a classified batch (pn_service_post_linked): links[i] = d > 0 when frame i - d is
 * the previous frame of frame i's connection in the batch (records with PN_F_HIT and not PN_F_TW) and frame i
 * continues it in order -- the case TcpConn::onPack hands to onData zero-copy without touching its segment list
 * (TcpConn.h:650-725): both clean, both with payload, seq contiguous, equal payload offset, ack number, window,
 * destination address and port.  Frame i at slots + i * slot_stride + frame_off.  All 0 when n > max_frames or
 * max_conn > max_conns (the GPU pass's LDS bounds, PN_LINK_MAX_FRAMES / PN_LINK_MAX_CONNS). */
void orc_chain_links(const uint8_t* slots, uint32_t slot_stride, uint32_t frame_off, uint32_t n, const pn_result* recs,
                     uint32_t max_conn, uint32_t max_frames, uint32_t max_conns, uint16_t* links);

/* ---- TX checksum generation (pn_tx_oracle.c) ---- */
/* n frames built the way a reference sender builds them (incremental CSum state:
 * TcpConn.h:149-323, 771-785; Core.h:157-163, 385-446; Efvi.h:405-411, 590-636).
 * mode PN_TX_TCP mixes SYNs, data segments (copyAndSum pieces), retransmissions,
 * RSTs and TIME_WAIT ACKs over 64 connections; PN_TX_UDP_EFVI builds Efvi UDP frames.
 * lens[i] = setOptDataLen's len (tot_len - 40) / update_udp_pkt's paylen;
 * kinds[i] = 0 data, 1 SYN, 2 retransmitted data, 3 RST, 4 TW ACK, 5 UDP.
 * Bytes of each slot past the frame are zero except what the reference's buffers leave
 * there.  0 on success. */
int orc_tx_build_batch(uint64_t seed, uint32_t n, uint8_t* slots, uint32_t stride, uint32_t frame_off, uint32_t mode,
                       uint16_t* lens, uint8_t* kinds);
/* pn_tx_fill's contract recomputed from the bytes (RFC 1071); 1 = filled, 0 = untouched. */
int orc_tx_fill_frame(uint8_t* eth, uint32_t avail, int has_len, uint16_t len, uint32_t mode);
void orc_tx_fill_batch(uint8_t* slots, uint32_t stride, uint32_t frame_off, uint32_t n, const uint16_t* lens,
                       uint32_t mode, int n_threads);
/* The reference's own TX byte work per segment (copyAndSum into a send buffer +
 * setOptDataLen) over a batch: the CPU baseline of the TX leg. */
void orc_tx_copy_and_sum_batch(const uint8_t* slots, uint8_t* out, uint32_t stride, uint32_t frame_off, uint32_t n,
                               int n_threads);

#ifdef __cplusplus
}
#endif
#endif
