/*
 * pollnet_amd_tuning.h — measurement-only entry points (libpollnet_amd_tuning.so).
 *
 * NOT part of the product ABI (include/pollnet_amd.h) and never loaded by the product
 * path: same-run bandwidth ceilings that bench.py reports beside the production kernel,
 * and (unless built with `make TUNING=0`) the A/B variants of the RX and TX kernels that
 * scripts/variants.py / scripts/tx_variants.py time.  Contexts come from pn_open().
 */
#ifndef POLLNET_AMD_TUNING_H
#define POLLNET_AMD_TUNING_H

#include "pollnet_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* HBM streaming-read calibration kernel (used by bench/profiling only): reads
 * `bytes` (multiple of 16) from src and writes one u32 per workgroup to sink. */
int pn_calib_stream_read(pn_ctx* ctx, const void* src_dev, uint64_t bytes, void* sink_dev, void* stream);
/* Ceiling for a slot layout: the first `bytes` (<= 2048) of each of n_slots slots,
 * read with the RX kernel's own load pattern and no arithmetic; store_bytes = 16 / 8
 * also writes that many bytes per slot to sink_dev (n_slots x 16 B) like the RX
 * kernel's records, 0 writes nothing; 16 | G << 8 (G = 1, 4, 16) writes the 16-B records of
 * G consecutive 64-slot groups in one burst per workgroup (write-grouping probe). */
int pn_calib_slot_read(pn_ctx* ctx, const void* src_dev, uint32_t n_slots, uint32_t stride, uint32_t bytes,
                       int store_bytes, void* sink_dev, void* stream);
/* Ceiling for variable-length frames: slot i's first lens_dev[i] bytes (u32 per slot, device
 * memory; clamped to min(stride, 2048)), same load pattern, workgroup order and occupancy as
 * the RX kernel, no arithmetic; store_bytes 16 also writes a 16-B record per slot, 0 none. */
int pn_calib_slot_read_var(pn_ctx* ctx, const void* src_dev, uint32_t n_slots, uint32_t stride, const void* lens_dev,
                           int store_bytes, void* sink_dev, void* stream);

/* Same-run ceilings that the product kernels cannot beat (bench.py): the production RX kernel
 * with the conn-table probe and the stream-phase lane reduction ablated (same loads, record
 * stores, occupancy and order; frame_off 2 or 18), and the production two-launch TX fill
 * (n > 65,536; frame_off 2 or 14) with its lane reduction ablated.  Timing only: their
 * records / fields are wrong. */
int pn_calib_classify_ablated(pn_ctx* ctx, const void* frames_dev, uint32_t slot_stride, uint32_t frame_off, uint32_t n,
                              void* results_dev, void* stream);
int pn_calib_tx_ablated(pn_ctx* ctx, void* frames, uint32_t slot_stride, uint32_t frame_off, uint32_t n, void* stream);

/* pn_match_streams in either kernel form: variant 1 = 4 lanes per frame load its header chunks
 * through LDS with nt loads (production), 0 = one lane per frame loads its own, 9 = variant 1 with
 * default-policy loads, 2-4 = nt / sc0 / sc1 loads, 5 = the production loads alone (timing-only
 * same-pattern ceiling; ids not written), 6 / 7 / 8 = sc1 id stores / nt loads + sc1 stores / nt stores. */
int pn_match_streams_variant(pn_ctx* ctx, const void* frames, uint32_t slot_stride, uint32_t frame_off, uint32_t n,
                             const pn_stream_filter* filters, uint32_t n_filters, uint32_t* stream_ids, void* stream,
                             int variant);

/* Test helper (no ctx): holds `stream` with one lane until the host stores non-zero to *go_host
 * or max_ms (<= 10000) pass, then stores 1 (released) / 2 (timed out) to *done_host; both in
 * pinned host memory.  Unrelated work in flight on a foreign stream (tests/test_gpu_notify.py). */
int pn_test_spin_wait(const uint32_t* go_host, uint32_t* done_host, uint32_t max_ms, void* stream);

/* Latency probe (no ctx; bench/bench_doorbell): one lane copies each new value of *bell_host to *echo_host (both
 * pinned host memory) until the value 0xFFFFFFFF or max_idle_ms (<= 10000) without a new value; once != 0: answer
 * the current value and end.  sleep != 0: s_sleep between polls. */
int pn_test_doorbell_echo(const uint32_t* bell_host, uint32_t* echo_host, uint32_t max_idle_ms, int once, int sleep,
                          void* stream);
/* The same answered from a pipelined poll (round 6): `depth` (1, 2, 4 or 8) reads of *bell_host in flight, a new one
 * issued `gap` x 64 clocks after the last, each checked when it returns -- a new value is seen within about one gap
 * of its arrival instead of up to a whole PCIe read round trip.  Values must increase (stale reads are ignored). */
int pn_test_doorbell_echo_pipe(const uint32_t* bell_host, uint32_t* echo_host, uint32_t max_idle_ms, int depth,
                               uint32_t gap, void* stream);

/* ---- A/B variants (built by default, TUNING=1; ids documented at their definitions) ---- */
int pn_classify_variant(pn_ctx* ctx, const void* frames_dev, uint32_t slot_stride, uint32_t frame_off, uint32_t n,
                        void* results_dev, void* stream, int variant);
int pn_classify_indexed_variant(pn_ctx* ctx, const void* base, const uint64_t* offsets, uint32_t eth_mod16, uint32_t n,
                                uint32_t avail, void* results_dev, void* stream, int variant);
int pn_tx_fill_variant(pn_ctx* ctx, void* frames, uint32_t slot_stride, uint32_t frame_off, uint32_t n,
                       const uint16_t* lens, int variant, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* POLLNET_AMD_TUNING_H */
