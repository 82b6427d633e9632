/*
 * pollnet_amd.h — C-ABI of the MI355X receive-path per-frame transform.
 *
 * This is the drop-in seam for efvitcp's RX hot path.  In the reference every
 * raw frame taken off the ef_vi ring goes through `Core::pollNet`
 * (/root/reference/efvitcp/Core.h:494-552): header pointers (:503-507),
 * `connHashKey` (:508 -> :167-172), `findConnEntry` (:509 -> :558-562), the
 * TIME_WAIT test (:510), and then `recv_handler(key, entry, eth)` (:526) whose
 * stateless part is `TcpConn::onPack`'s payload arithmetic
 * (/root/reference/efvitcp/TcpConn.h:469-473).  The IP/TCP one's-complement
 * verification is `Core::checksum` (Core.h:448-472, EFVITCP_DEBUG only in the
 * reference) built on `CSum` (Core.h:89-138).
 *
 * Here that per-frame work runs as one batched HIP kernel over frames resident
 * in HBM and produces one 16-byte `pn_result` per frame.  Everything stateful
 * (TCP state machine, TIME_WAIT bookkeeping, timers, TX) stays on the host.
 *
 * Conventions (mirroring the reference's error style, Core.h:253-383 returns
 * `const char*`, Socket.h:47 `getLastError()`):
 *   - every function returns 0 on success and a negative PN_E* code on error;
 *   - `pn_last_error(ctx)` returns a static/ctx-owned message for the last error;
 *   - no C++ types, no exceptions cross this ABI; pointers + sizes only;
 *   - device pointers are plain `void*` from hipMalloc (or torch), streams are
 *     `hipStream_t` passed as `void*` (NULL = the null stream).
 */
#ifndef POLLNET_AMD_H
#define POLLNET_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PN_ABI_VERSION 1

/* ---- constants taken from the reference (Core.h) ---- */
#define PN_RECV_BUF_SIZE 2048u         /* RecvBufSize, Core.h:45 (ring slot stride) */
#define PN_RECV_MSS 1460u              /* RecvMSS, Core.h:44 */
#define PN_EMPTY_KEY (1ull << 63)      /* EmptyKey, Core.h:49 */
#define PN_MISS 0xFFFFFFFFu            /* pn_result.conn_id when findConnEntry misses */

/* ---- error codes ---- */
#define PN_OK 0
#define PN_EINVAL -1    /* bad argument (shape/alignment contract violated) */
#define PN_EHIP -2      /* a HIP runtime call failed (see pn_last_error) */
#define PN_ENOMEM -3    /* allocation failed */
#define PN_ENOTABLE -4  /* pn_classify before pn_set_conn_table */
#define PN_EFULL -5     /* conn table full */
#define PN_ENOENT -6    /* key not in conn table */

/* ---- per-frame output record (16 bytes, written coalesced) ---- */
typedef struct pn_result {
  uint32_t conn_id;     /* entry->conn_id on hit (Core.h:510/TcpServer.h:96), PN_MISS on miss.
                           conn_id >= max_conn_cnt means TIME_WAIT (tw_id = conn_id - max_conn_cnt) */
  uint32_t seq;         /* ntohl(tcp->seq_num) + tcp->syn                 (TcpConn.h:473) */
  uint16_t payload_off; /* (tcp + doff*4) - eth, tcp = ip + 20            (TcpConn.h:471, Core.h:507) */
  int16_t payload_len;  /* ip + min(tot_len,1500) - (tcp + doff*4)        (TcpConn.h:472, signed) */
  uint16_t flags;       /* PN_F_* below */
  uint16_t tcp_fold;    /* CSum::fold() of the reference TCP sum (Core.h:459-466); 0 <=> valid.
                           0xFFFF = no fold computed: PN_F_TRUNC (segment runs past the slot) or
                           PN_F_TCP_UNCHECKED (release path).  A real fold is never 0xFFFF (~r, r >= 1). */
} pn_result;

/* flags */
#define PN_F_IP_OK 0x0001u      /* CSum.add<20>(ip).fold() == 0            (Core.h:451-453) */
#define PN_F_TCP_OK 0x0002u     /* pseudo-header + segment fold == 0      (Core.h:459-466) */
#define PN_F_HIT 0x0004u        /* findConnEntry(key)->key == key          (Core.h:510, TcpServer.h:81) */
#define PN_F_TW 0x0008u         /* hit && conn_id >= MaxConnCnt            (Core.h:510) */
#define PN_F_FIN 0x0010u        /* TcpHeader bitfields                     (Core.h:80) */
#define PN_F_SYN 0x0020u
#define PN_F_RST 0x0040u
#define PN_F_PSH 0x0080u
#define PN_F_ACK 0x0100u
#define PN_F_IHL_NE_5 0x0200u   /* ip->header_len != 5 (reference assumes 5: Core.h:507, TcpConn.h:469) */
#define PN_F_RFC_IP_OK 0x0400u  /* RFC 791 header checksum over header_len*4 bytes */
#define PN_F_RFC_TCP_OK 0x0800u /* RFC 793 checksum: TCP at ip+IHL*4, odd tail zero-padded */
#define PN_F_NOT_TCP 0x1000u    /* ether_type != 0x0800 || ip_ver != 4 || protocol != 6
                                   (TcpStream.h:45-46; efvitcp itself trusts the NIC filter, Core.h:375-383) */
#define PN_F_TRUNC 0x2000u      /* ip+20+tcp_len(+pad) exceeds the slot: the reference would read past
                                   the frame (undefined); TCP_OK/RFC_TCP_OK cleared, tcp_fold=0xFFFF */
#define PN_F_BADOFF 0x4000u     /* pn_classify_indexed: offset outside the call's eth_mod16 class; the
                                   frame was not read and the record is {PN_MISS, 0, 0, 0, BADOFF, 0} */
#define PN_F_TCP_UNCHECKED 0x8000u /* pn_set_verify(ctx, 0): the reference's release path, which verifies no
                                   checksum (Core::checksum is debug-only, Core.h:448-478): only the frame's
                                   header lines were read; TCP_OK / RFC_TCP_OK never set, tcp_fold = 0xFFFF */

/* ---- 16-byte conn-table entry, identical layout to ConnHashEntry (Core.h:178-182) ---- */
typedef struct pn_conn_entry {
  uint64_t key;     /* connHashKey(), or PN_EMPTY_KEY */
  uint32_t conn_id;
  uint32_t _pad;
} pn_conn_entry;

/* ======================= host conn table (control plane) =======================
 * Restates Core's ordered-linear-probe table so the host builds the exact
 * `conn_tbl`/`tbl_mask` bytes the GPU reads.  Sizing as Core.h:235-236, initial
 * mask as Core.h:322.  Not thread-safe (reference: single thread). */
typedef struct pn_conn_table pn_conn_table;

/* connHashKey(ip, port) with ip/port in network byte order (Core.h:167-172). */
uint64_t pn_conn_hash_key(uint32_t ip_be, uint16_t port_be);

int pn_table_create(uint32_t max_conn_cnt, uint32_t max_tw_cnt, pn_conn_table** out);
/* The same with flags:
 *   PN_TABLE_REFERENCE_LITERAL  run Core::tryExpandConnTbl's in-place rehash (Core.h:650-682)
 *   exactly, without the product's repair: under the histories where that rehash strands keys
 *   (its debug build exits there, Core.h:665-669) the table, and so every pn_classify record,
 *   is what the reference's would be, lost connections included.  Default (0): the defect is
 *   detected and the table rebuilt canonically (pn_table_repairs counts it). */
#define PN_TABLE_REFERENCE_LITERAL 1u
int pn_table_create_ex(uint32_t max_conn_cnt, uint32_t max_tw_cnt, uint32_t flags, pn_conn_table** out);
uint32_t pn_table_flags(const pn_conn_table* t);
void pn_table_destroy(pn_conn_table* t);
/* findConnEntry (Core.h:558-562): index of the entry the probe stops at; *hit = key matched. */
int pn_table_find(const pn_conn_table* t, uint64_t key, uint32_t* entry_idx, int* hit, uint32_t* conn_id);
/* findConnEntry + addConnEntry + tryExpandConnTbl (Core.h:566-576, 650-682).
 * The reference's callers only add keys that missed; PN_EINVAL if key present. */
int pn_table_add(pn_conn_table* t, uint64_t key, uint32_t conn_id);
/* delConnEntry (Core.h:578-605): backward-shift delete. */
int pn_table_del(pn_conn_table* t, uint64_t key);
/* enterTW relabel (Core.h:612-627): conn_id -> max_conn_cnt + tw_id. */
int pn_table_set_conn_id(pn_conn_table* t, uint64_t key, uint32_t conn_id);
/* Snapshot view: entries (TotalTableSize of them), current tbl_mask, sizing. */
const pn_conn_entry* pn_table_entries(const pn_conn_table* t, uint32_t* n_entries, uint64_t* tbl_mask);
uint32_t pn_table_max_conn_cnt(const pn_conn_table* t);
uint32_t pn_table_size(const pn_conn_table* t); /* getTblSize() (Core.h:564) */
/* How many expansions hit the reference's rehash defect (Core.h:665-669 debug
 * exit) and were rebuilt canonically instead of losing keys. */
uint32_t pn_table_repairs(const pn_conn_table* t);

/* ======================= device context =======================
 * One ctx per (host thread, device).  Owns the device copy of the conn table.
 * Streams: every launch call takes the caller's stream; the ctx keeps that handle until its
 * next pn_set_conn_table or pn_sync returns, so a stream passed to a launch call must stay
 * valid until then (pn_close touches no stream handle). */
typedef struct pn_ctx pn_ctx;

int pn_open(int device, pn_ctx** out);
void pn_close(pn_ctx* ctx);
const char* pn_last_error(const pn_ctx* ctx); /* ctx may be NULL: last global error */
int pn_device_count(int* n);

/* Snapshot the conn table into device memory (H2D on the ctx's own stream, <=160 KiB for
 * 1024+1024 conns; returns when the copy is done).  `entries` is host memory laid out as
 * pn_conn_entry[n].  Double-buffered: the snapshot goes to the buffer no launch is reading
 * now, so launches already issued (on any stream, running or queued) keep the snapshot they
 * were issued against, and launches issued after this returns see the new one.  It waits
 * only for the launches issued before the PREVIOUS set (by events recorded then; normally long
 * done) — never for the device, other streams or other contexts.  The launch path records
 * nothing. */
int pn_set_conn_table(pn_ctx* ctx, const pn_conn_entry* entries, uint32_t n_entries, uint64_t tbl_mask,
                      uint32_t max_conn_cnt);

/* What the classify entry points verify on this ctx (default 1: both checksums, as the reference's debug
 * build does before every frame it sends or receives, Core.h:448-478).  verify_tcp = 0: the reference's
 * release path — the TCP checksum is neither computed nor read for (the kernel reads only each frame's
 * header lines: one 128-B line in the default layout instead of the whole frame); every other record field,
 * PN_F_IP_OK and PN_F_RFC_IP_OK included, is the same, and PN_F_TCP_UNCHECKED marks the record.  Applies to
 * launches issued after the call. */
int pn_set_verify(pn_ctx* ctx, int verify_tcp);

/* Classify n frames resident in device memory (asynchronous on `stream`).
 *   frames_dev : base of n slots, 16-byte aligned; frame i's Ethernet header is at
 *                frames_dev + i*slot_stride + frame_off (Core.h:503-505: slot +
 *                sizeof(RecvBuf) + receive_prefix_len).
 *   slot_stride: multiple of 16, >= frame_off + 96 (the header window), <= 65536.
 *   frame_off  : even; (frame_off + 14) % 16 selects a specialised kernel.
 *   results_dev: n pn_result records (16-byte aligned).
 * Frame length is taken from ip->tot_len only, as the reference does (Core.h:463, TcpConn.h:472). */
int pn_classify(pn_ctx* ctx, const void* frames_dev, uint32_t slot_stride, uint32_t frame_off, uint32_t n,
                void* results_dev, void* stream);

/* Classify n frames at arbitrary places — a ring whose slots are named by RX events
 * (ef_vi: slot id * RecvBufSize + sizeof(RecvBuf) + receive_prefix_len, Core.h:503-505,
 * wrapping and skipping discarded slots), a packet-mmap block, a packed capture:
 * frame i's Ethernet header is at base + offsets[i].
 *   base      : 16-byte aligned; device memory or pinned host memory (zero-copy).
 *   offsets   : n u64, readable by the device (device or pinned host memory).
 *   eth_mod16 : offsets[i] % 16, the same for every frame (even): the kernel is
 *               specialised on it; a frame outside the class gets a PN_F_BADOFF record.
 *   avail     : readable bytes from each Ethernet header, in [96, 65536] (ef_vi:
 *               RecvBufSize - sizeof(RecvBuf) - receive_prefix_len); bounds every read
 *               past the header.  A frame whose header window starts 16 B into a
 *               128-B line (2-KiB slots with frame_off 2, ef_vi with a prefix <= 7) may
 *               also be read from that line's start, never below base.
 * Records are written in offsets order, identical to pn_classify's for the same frame
 * bytes and avail.  Asynchronous on `stream`. */
int pn_classify_indexed(pn_ctx* ctx, const void* base, const uint64_t* offsets, uint32_t eth_mod16, uint32_t n,
                        uint32_t avail, void* results, void* stream);

/* ---- TcpStream's packet filter over a batch (TcpStream.h:32-52), many streams ---- */
#define PN_MAX_STREAM_FILTERS 64
#define PN_NO_STREAM 0xFFFFFFFFu
typedef struct pn_stream_filter { /* TcpStream::initFilter's four fields (TcpStream.h:32-37) */
  uint32_t src_ip;                /* network order (inet_pton); 0 = wildcard ("0.0.0.0") */
  uint32_t dst_ip;
  uint16_t src_port;              /* network order (htons); 0 = wildcard */
  uint16_t dst_port;
  uint32_t _pad;
} pn_stream_filter;

/* stream_ids[i] = index of the first filter frame i passes, PN_NO_STREAM if none.  A
 * frame passes filter k exactly when TcpStream::filterPacket would (TcpStream.h:39-52):
 * etherType 0x0800, protocol 6, and every non-zero field of filter k equal to the
 * frame's (IP header assumed 20 B).  frames/slot_stride/frame_off as pn_classify
 * (frame_off >= 2); frames in device or pinned host memory; filters in host memory
 * (copied into the launch), n_filters <= PN_MAX_STREAM_FILTERS.  Reads one header line
 * per frame.  Asynchronous on `stream`; needs no conn table. */
int pn_match_streams(pn_ctx* ctx, const void* frames, uint32_t slot_stride, uint32_t frame_off, uint32_t n,
                     const pn_stream_filter* filters, uint32_t n_filters, uint32_t* stream_ids, void* stream);

/* ---- TX checksum fill over a batch of outgoing frames ----
 * Replaces the reference's per-frame checksum finalisation on the send side:
 *   PN_TX_TCP      efvitcp: SendBuf::setOptDataLen (Core.h:157-163) at the end of
 *                  TcpConn::sendBuf (TcpConn.h:310-323), of sumRst for RST / TIME_WAIT
 *                  ACKs (Core.h:385-398), and resendUna's in-place patch
 *                  (TcpConn.h:771-785).  Writes ip->checksum (IP header assumed 20 B, as
 *                  every efvitcp frame is) and tcp->checksum over the pseudo-header and
 *                  tot_len - 20 bytes at ip + 20 (odd length zero-padded, as copyAndSum
 *                  sums it, TcpConn.h:291-295).  The values equal the reference's
 *                  incrementally folded ones for every frame its send path builds
 *                  (DESIGN.md §12).
 *   PN_TX_UDP_EFVI Efvi's UDP sender: update_udp_pkt (Efvi.h:611-621) with the cached
 *                  IPv4 header sum (Efvi.h:405-411), its fold reproduced exactly — including
 *                  the carry it counts twice when the cached sum's first fold carries,
 *                  which leaves those headers with a checksum that does not verify
 *                  (DESIGN.md §12).  Writes ip->checksum; the UDP checksum is left as is
 *                  (Efvi sends 0).
 *   PN_TX_UDP      the same fields with CSum::fold (Core.h:94-98): a verifying IPv4
 *                  header checksum for every header; equal to PN_TX_UDP_EFVI wherever
 *                  Efvi's own is valid.
 * lens (optional, device-readable u16 per frame): when given, tot_len is set first —
 * htons(40 + lens[i]) for TCP (setOptDataLen's opt + data length), htons(28 + lens[i])
 * and udp_len = htons(8 + lens[i]) for the UDP modes (update_udp_pkt's paylen); otherwise the
 * frame's own tot_len is used.  A frame whose tot_len is below the bare headers
 * (40 / 28) or runs past its slot (14 + tot_len > slot_stride - frame_off) is left
 * untouched.  Only the length and checksum fields are written.
 * Layout as pn_classify (frames in device memory or pinned host memory read and patched in
 * place, 16-byte aligned; SendBuf slots: frame_off = 14, slot_stride = SendBufSize,
 * Core.h:147-156, 232).  Asynchronous.  Up to 65,536 frames one launch; above, two (the
 * fields through ctx scratch; a two-launch call on another stream than the
 * previous one is ordered after it on the device). */
#define PN_TX_TCP 0u
#define PN_TX_UDP_EFVI 1u
#define PN_TX_UDP 2u
int pn_tx_fill(pn_ctx* ctx, void* frames, uint32_t slot_stride, uint32_t frame_off, uint32_t n, const uint16_t* lens,
               uint32_t mode, void* stream);

/* Small batches, latency: pn_classify / pn_tx_fill whose launch also stores `token` to
 * *done_word (4-byte aligned, host-visible: pinned host memory) once every record / field it
 * writes is stored and visible to the host.  A host that polls the word (an acquire load)
 * sees a 64..1024-frame batch done ≈3-4 µs sooner than hipStreamSynchronize returns (DESIGN.md
 * §13); the stream orders later work as usual, and pn_sync / hipStreamSynchronize still apply.
 * The same arguments as pn_classify (strided slots) / pn_tx_fill, plus: n in
 * [1, PN_NOTIFY_MAX_FRAMES] (every workgroup makes its stores system-visible, which only pays
 * off for small batches).  The per-ctx counter behind the word is reused: a notify call on
 * another stream than the previous one of the same kind is ordered after it on the device
 * (an event and hipStreamWaitEvent; the host does not wait).
 * Replaces the completion step of the reference's poll (ef_eventq_poll's RX/TX events,
 * Core.h:496-498): the host learns the batch is done from one memory word. */
#define PN_NOTIFY_MAX_FRAMES 1024u
int pn_classify_notify(pn_ctx* ctx, const void* frames, uint32_t slot_stride, uint32_t frame_off, uint32_t n,
                       void* results, void* stream, uint32_t* done_word, uint32_t token);
int pn_tx_fill_notify(pn_ctx* ctx, void* frames, uint32_t slot_stride, uint32_t frame_off, uint32_t n,
                      const uint16_t* lens, uint32_t mode, void* stream, uint32_t* done_word, uint32_t token);

/* ---- resident classify service: no launch per batch (round 5) ----
 * pn_service_open launches a kernel that stays on the GPU (PN_SERVICE_WAVES one-wave workgroups on a stream of its
 * own, the latency tier) and classifies every batch the host posts afterwards, with the same code and records as
 * pn_classify on the layout given at open (strided slots).  A post is one 64-B line the host writes into a mailbox
 * that every wave of the kernel polls -- device memory written through the large BAR (pinned host memory on a device
 * without one, or with PN_SERVICE_HOST_MAILBOX set in the environment at open) -- so a batch starts ~1-2 us after it
 * is posted instead of a launch's ~7 us (bench/bench_doorbell).
 *   pn_service_post: frames (pinned host or device memory, 16-B aligned), n in [1, PN_SERVICE_MAX_FRAMES], results
 *     (pinned host or device memory, 16-B aligned).  The ctx's conn table and pn_set_verify setting at the post are
 *     used.  At most two posts outstanding (a third is refused, PN_EINVAL); non-blocking; *post_id (may be NULL)
 *     names the post.  Frames and results must stay valid until the post completes.
 *   pn_service_wait: spins until post post_id's records are visible to the host (as pn_classify_notify's word);
 *     posts complete in order; post_id 0 = the last post.
 *   Post ids count up by one per post and wrap at 2^32: every value, 0 included, is a post's id (so "0 = the last
 *     post" waits at least as long as the post named 0).  PN_SERVICE_FIRST_POST in the environment at open sets the
 *     count's start (tests start it just below 2^32).
 *   pn_service_close: waits for outstanding posts, stops the kernel, frees the service (before pn_close).
 * Post size.  Up to 4096 frames a post runs on the latency tier (a 64-frame post on one wave, no cross-wave step).
 * Above, the post also runs on helper waves, a grid launched with the post on a second stream of the service (in all
 * PN_SERVICE_WAVES_PER_CU waves per CU, 64-frame groups; the helpers take the post from their launch and wait for
 * nothing): the chip is not held while the service idles.  Measured on MI355X (scripts/service_sizing.py, DESIGN.md
 * §13): a 1-Mi-frame post of device-resident C2 frames, post to records complete, takes 1.15x pn_classify's launch
 * to stream sync verified (0.300 vs 0.262 ms) and 1.27x on the release path (0.047 vs 0.037 ms); the latency tier
 * alone (large_waves = PN_SERVICE_WAVES) takes 10x.
 * Timers.  After idle_ms (1..10000) without a post the kernel ends by itself; the next post (or wait) relaunches it.
 * A post in flight has its own limit (8 s from its acceptance): should one of its waves never finish, the kernel ends
 * and the host's next wait relaunches it, which runs the post again.  So the kernel always ends.
 * Conn table.  pn_set_conn_table may be called at any time, posts outstanding or not: each post keeps classifying
 * against the table it was posted with; a set that would overwrite or free the buffer an outstanding post reads waits
 * for that post first (at most one post's run).  One thread per service, as per ctx.
 * pn_service_open_ex: the same with a large post's wave count given (0 = the default above; else in
 * [PN_SERVICE_WAVES, PN_SERVICE_MAX_WAVES]; PN_SERVICE_WAVES = no helpers, the latency tier alone).
 * Replaces the launch of the reference's per-poll work with its own busy-poll style (Core.h:494-498). */
typedef struct pn_service pn_service;
#define PN_SERVICE_WAVES 64u        /* the latency tier: every post of up to 4096 frames */
#define PN_SERVICE_WAVES_PER_CU 12u /* a large post's default wave count: this many per CU (3072 on a 256-CU MI355X) */
#define PN_SERVICE_MAX_WAVES 4096u
#define PN_SERVICE_MAX_FRAMES (1u << 20)
#define PN_SERVICE_STOP 0xFFFFFFFFu /* internal: the stop post */
int pn_service_open(pn_ctx* ctx, uint32_t slot_stride, uint32_t frame_off, uint32_t idle_ms, pn_service** out);
int pn_service_open_ex(pn_ctx* ctx, uint32_t slot_stride, uint32_t frame_off, uint32_t idle_ms, uint32_t large_waves,
                       pn_service** out);
int pn_service_post(pn_service* svc, const void* frames, uint32_t n, void* results, uint32_t* post_id);
/* pn_service_post with the post's chain links (round 6): links (host or device memory, n u16, 2-B aligned) gets, per
 * frame i, d > 0 when frame i - d is the previous frame of the same connection in the post (among records with
 * PN_F_HIT and not PN_F_TW) and frame i continues it in order: both frames clean (PN_F_ACK, PN_F_IP_OK and PN_F_TCP_OK
 * or PN_F_TCP_UNCHECKED; no SYN, FIN, RST, NOT_TCP, TRUNC, BADOFF, IHL_NE_5), both with payload, seq_i = seq_j +
 * payload_len_j, and equal payload_off, ack number, window, destination address and port; else 0.  A host that
 * processed frame i - d and left the connection untouched since can take frame i's data without re-checking it
 * against the connection.  Computed on the GPU after the records, in the same post (the links are
 * visible when pn_service_wait returns); n <= PN_LINK_MAX_FRAMES; with max_conn_cnt > PN_LINK_MAX_CONNS every link
 * is 0.  The chain's statement: oracle/pn_oracle.c orc_chain_links. */
#define PN_LINK_MAX_FRAMES 1024u
#define PN_LINK_MAX_CONNS 4096u
int pn_service_post_linked(pn_service* svc, const void* frames, uint32_t n, void* results, uint16_t* links,
                           uint32_t* post_id);
int pn_service_wait(pn_service* svc, uint32_t post_id);
int pn_service_close(pn_service* svc);

/* Wait until every launch this ctx issued (on any stream) has finished: synchronizes each
 * stream launched on since the last pn_set_conn_table, and the events that set recorded
 * for the launches before it.  Not a device-wide wait. */
int pn_sync(pn_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* POLLNET_AMD_H */
