#!/usr/bin/env python3
"""Packed capture (C3 frames back to back, pn_classify_indexed): how much faster could phase 2
run if a wave streamed its 64 frames as ONE contiguous byte range with fully used 1-KiB loads?
Timing-only ablation (tuning variant 4, records wrong) against the production kernel and a plain
stream read of the same bytes.  Interleaved rounds, HIP events on the launch stream.  Needs
`make TUNING=1`."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    import pollnet_amd as pa
    from pollnet_amd import tuning as tn

    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    n, stride, off = 1 << 20, 2048, 2
    p = pa.rx.GenParams.for_config(cfg)
    s = pa.gen_frames(p, n)
    ctx = pa.RxContext(0)
    ctx.set_conn_table(pa.gen_conn_table(p))
    tl = (s[:, off + 16].astype(np.int64) << 8) | s[:, off + 17]
    ln = 14 + tl + 1
    starts = np.empty(n, np.int64)
    pos = off
    for i in range(n):
        starts[i] = pos
        pos = ((pos + int(ln[i]) + 15) & ~15) + off
    packed = np.zeros(pos + stride, np.uint8)
    for i in range(n):
        packed[starts[i]:starts[i] + ln[i]] = s[i, off:off + ln[i]]
    dev = torch.from_numpy(packed).cuda()
    offs = torch.from_numpy(starts.astype(np.uint64).view(np.int64)).cuda()
    out = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
    sink = torch.zeros(4096, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream()
    runs = {
        "production": lambda: ctx.classify_indexed(dev, offs, off, n, stride - off, out, st),
        "contig_stream_ablation": lambda: tn.classify_indexed_variant(ctx, dev, offs, off, n, stride - off, out, st, 4),
        "stream_read_packed_bytes": lambda: tn.calib_stream_read(ctx, dev, (pos // 1024) * 1024, sink, st),
    }
    times = {k: [] for k in runs}
    for _ in range(12):
        for k, f in runs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(5):
                f()
            e1.record(st)
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1) / 5)
    algo = int(np.sum(ln - 1)) + 16 * n
    res = {"config": cfg, "frames": n, "packed_bytes": int(pos), "algo_bytes": algo}
    for k, v in times.items():
        ms = statistics.median(v)
        res[k] = {"ms_median": round(ms, 5), "frac_of_8TBs": round(algo / (ms * 1e-3) / 8e12, 4)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
