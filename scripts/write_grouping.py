#!/usr/bin/env python3
"""Does writing the 16-B records in larger bursts cut their cost?  The RX kernel's load
pattern with no arithmetic (calib slot read, 1536 B per 2-KiB slot, C2 batch), interleaved
rounds: no records, records after every 64-slot group (the RX kernel's pattern), and
records of G = 1, 4, 16 groups written in one burst per workgroup."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import pollnet_amd as pa
    from pollnet_amd import tuning as tn

    n = 1 << 20
    p = pa.rx.GenParams.for_config(2)
    batches = [torch.from_numpy(pa.gen_frames(p, n, first_index=b * n).reshape(-1)).cuda() for b in range(4)]
    ctx = pa.RxContext(0)
    ctx.set_conn_table(pa.gen_conn_table(p))
    sink = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream()
    modes = {"no_records": 0, "records_per_group": 16, "grouped_G1": 16 | (1 << 8), "grouped_G4": 16 | (4 << 8),
             "grouped_G16": 16 | (16 << 8), "loop_G4_write_each": 16 | (4 << 8) | (1 << 16),
             "loop_G16_write_each": 16 | (16 << 8) | (1 << 16)}
    times = {k: [] for k in modes}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for _ in range(12):
        for k, m in modes.items():
            for b in batches[:2]:
                tn.calib_slot_read(ctx, b, n, 2048, 1536, sink, st, m)
            ev[0].record(st)
            for r in range(8):
                tn.calib_slot_read(ctx, batches[r % 4], n, 2048, 1536, sink, st, m)
            ev[1].record(st)
            torch.cuda.synchronize()
            times[k].append(ev[0].elapsed_time(ev[1]) / 8)
    out = {k: {"ms_median": round(statistics.median(v), 4), "read_tbps": round(1536 * n / (statistics.median(v) * 1e-3) / 1e12, 3)}
           for k, v in times.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
