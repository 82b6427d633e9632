// Standalone C++ check of the drop-in adapter (include/pollnet_amd/gpu_rx.hpp) with
// no Python/torch in the process: /opt/rocm's HIP runtime only.  Generates C2/C3/C5
// batches, classifies them through GpuRx::pollBatch, and compares every record and
// the TW/recv dispatch against the C oracle (test infrastructure, linked here only
// as the checker).  Exit 0 = pass.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/pollnet_amd/gpu_rx.hpp"
#include "../../include/pollnet_amd_gen.h"
#include "../../oracle/pn_oracle.h"

static int run(uint32_t cfg, uint32_t n, pollnet_amd::GpuRx::Mode mode, uint32_t chunk) {
  pn_gen_params p{};
  p.cfg = cfg;
  p.n_flows = cfg == 2 ? 1 : 1024;
  p.n_tw_flows = (cfg == 3 || cfg == 5) ? 32 : 0;
  p.max_conn_cnt = 1024;
  p.seed = 0x5EED0000u + cfg;
  const uint32_t stride = 2048, off = 2;
  uint8_t* ring = nullptr;
  if (hipHostMalloc((void**)&ring, (size_t)stride * n, hipHostMallocDefault) != hipSuccess) return 2;
  if (pn_gen_frames(&p, 0, n, ring, stride, off, 8)) return 3;
  pollnet_amd::ConnTable table;
  if (table.init(1024, 1024)) return 4;
  // pn_gen_conn_table needs the raw handle; rebuild the same table through the adapter API
  pn_conn_table* raw = nullptr;
  pn_table_create(1024, 1024, &raw);
  if (pn_gen_conn_table(&p, raw)) return 5;
  uint32_t ne = 0;
  uint64_t mask = 0;
  const pn_conn_entry* ents = pn_table_entries(raw, &ne, &mask);
  for (uint32_t i = 0; i < ne; i++)
    if (ents[i].key != PN_EMPTY_KEY) table.add(ents[i].key, ents[i].conn_id);
  pn_table_destroy(raw);
  pollnet_amd::GpuRx rx;
  if (const char* err = rx.init(0, stride, off, chunk, mode)) {
    std::printf("init: %s\n", err);
    return 6;
  }
  if (const char* err = rx.syncTable(table)) {
    std::printf("syncTable: %s\n", err);
    return 7;
  }
  std::vector<pn_result> got(n), exp(n);
  uint32_t tw_calls = 0, recv_calls = 0, misses = 0, bad_idx = 0;
  uint32_t i = 0;
  const char* err = rx.pollBatch(
      ring, n, table,
      [&](uint64_t key, const pn_result& r, const uint8_t* eth, uint32_t miss_idx) {
        recv_calls++;
        if (!(r.flags & PN_F_HIT)) {
          misses++;
          uint32_t idx = 0;
          if (table.find(key, &idx, nullptr) || idx != miss_idx) bad_idx++;
        }
        got[(eth - ring - off) / stride] = r;
        i++;
      },
      [&](uint64_t, uint32_t tw_id, const uint8_t* eth, const pn_result& r) {
        tw_calls++;
        if (tw_id >= 1024) bad_idx++;
        got[(eth - ring - off) / stride] = r;
        i++;
      });
  if (err) {
    std::printf("pollBatch: %s\n", err);
    return 8;
  }
  uint32_t tn = 0;
  uint64_t tm = 0;
  const pn_conn_entry* te = table.entries(&tn, &tm);
  orc_classify_batch(ring, stride, off, n, te, tn, tm, 1024, exp.data(), 8);
  uint32_t diff = 0, exp_tw = 0;
  for (uint32_t k = 0; k < n; k++) {
    if (std::memcmp(&got[k], &exp[k], sizeof(pn_result))) diff++;
    if (exp[k].flags & PN_F_TW) exp_tw++;
  }
  std::printf("cfg %u (%s, chunk %u): n=%u recv=%u tw=%u (expected tw %u) misses=%u diff=%u bad_idx=%u\n", cfg,
              mode == pollnet_amd::GpuRx::Mode::ZeroCopy ? "zero-copy" : "copy", chunk, n, recv_calls, tw_calls, exp_tw,
              misses, diff, bad_idx);
  (void)hipHostFree(ring);
  return (diff || bad_idx || tw_calls != exp_tw || i != n) ? 1 : 0;
}

int main() {
  int rc = 0;
  using M = pollnet_amd::GpuRx::Mode;
  rc |= run(2, 100000, M::Copy, 100000);
  rc |= run(3, 100000, M::Copy, 100000);
  rc |= run(5, 50000, M::Copy, 50000);
  // chunked pipeline (ragged last chunk) and the zero-copy mode
  rc |= run(3, 100000, M::Copy, 7777);
  rc |= run(3, 100000, M::ZeroCopy, 100000);
  rc |= run(5, 50000, M::ZeroCopy, 4096);
  rc |= run(2, 100000, M::ZeroCopy, 333);
  std::printf(rc ? "FAIL\n" : "PASS\n");
  return rc;
}
