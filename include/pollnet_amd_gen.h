/*
 * pollnet_amd_gen.h — the synthetic workload generator (libpollnet_amd_gen.so).
 *
 * NOT part of the product ABI (include/pollnet_amd.h): the seeded frame / conn-table
 * generator behind the BASELINE configs that the tests, bench.py and the bench programs use to
 * build their rings.  Depends on the product library only for the conn-table calls.
 */
#ifndef POLLNET_AMD_GEN_H
#define POLLNET_AMD_GEN_H

#include "pollnet_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ======================= synthetic frame generator =======================
 * Deterministic (seed, frame index) generator for the BASELINE configs; writes
 * slots into host memory with bytes after each frame zero-filled.  Multi-threaded.
 *   cfg: 2 = C2 (1514-B frames, 1 flow), 3 = C3 (64..1514-B mixed, 1024 flows,
 *        TW + miss flows), 4 = C4 (1514-B frames over 1024 flows), 5 = C5
 *        (IPv4 options + odd lengths + bad-checksum + adversarial cluster).
 * first_index lets ranks generate disjoint shards of one global batch. */
typedef struct pn_gen_params {
  uint32_t cfg;
  uint32_t n_flows;       /* flows with a conn entry (conn_id = flow index) */
  uint32_t n_tw_flows;    /* of those, how many are moved to TIME_WAIT */
  uint32_t max_conn_cnt;  /* Conf::MaxConnCnt (= MaxTimeWaitConnCnt) */
  uint64_t seed;
} pn_gen_params;

int pn_gen_frames(const pn_gen_params* p, uint64_t first_index, uint32_t n, void* slots_host, uint32_t slot_stride,
                  uint32_t frame_off, int n_threads);
/* Build the conn table the generator's flows imply (add in flow order, TW relabel). */
int pn_gen_conn_table(const pn_gen_params* p, pn_conn_table* t);
/* Wire bytes (14 + tot_len) summed over the n generated frames (metric numerator). */
uint64_t pn_wire_bytes(const void* slots_host, uint32_t slot_stride, uint32_t frame_off, uint32_t n);

#ifdef __cplusplus
}
#endif
#endif /* POLLNET_AMD_GEN_H */
