#!/usr/bin/env python3
"""Why does bench.py time C3 slower than the A/B harness?  One process: the bench's own setup
(frames through a reused host buffer, the gate's torch ops on the records), then the same
resident batch timed bench-style (W warmup, one event pair over K launches) and A/B-style
(rounds of 1 + 10 launches, median), then a second copy of the frames in a new buffer and a
new records buffer, each timed both ways.  A measurement, not part of any product path."""
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

    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    n, stride, off = 1 << 20, 2048, 2
    p = pa.rx.GenParams.for_config(cfg)
    table = pa.gen_conn_table(p)
    ctx = pa.RxContext(0)
    ctx.set_conn_table(table)
    host = np.empty((n, stride), dtype=np.uint8)
    pa.gen_frames(p, n, stride, off, first_index=0, threads=16, out=host)
    frames = torch.from_numpy(host.reshape(-1)).to("cuda:0")
    res = torch.empty(n * 16, dtype=torch.uint8, device="cuda:0")
    st = torch.cuda.current_stream()
    ctx.classify(frames, stride, off, n, res, st)
    torch.cuda.synchronize()
    rec = res.view(n, 16)
    flags = rec[:, 12].to(torch.int32) | (rec[:, 13].to(torch.int32) << 8)
    _ = bool(torch.all((flags & 0x4000) == 0))

    def bench_style(fr, rs, w=5, k=50):
        for _ in range(w):
            ctx.classify(fr, stride, off, n, rs, st)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(k):
            ctx.classify(fr, stride, off, n, rs, st)
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / k

    def ab_style(fr, rs, rounds=10):
        ts = []
        for _ in range(rounds):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ctx.classify(fr, stride, off, n, rs, st)
            e0.record(st)
            for _ in range(10):
                ctx.classify(fr, stride, off, n, rs, st)
            e1.record(st)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) / 10)
        return statistics.median(ts)

    out = {"config": cfg}
    frames2 = frames.clone()
    res2 = torch.empty_like(res)
    combos = {"bench_frames+bench_res": (frames, res), "bench_frames+new_res": (frames, res2),
              "new_frames+bench_res": (frames2, res), "new_frames+new_res": (frames2, res2)}
    for rep in range(2):
        for name, (fr, rs) in combos.items():
            out.setdefault(name, []).append({"bench_style": round(bench_style(fr, rs), 5), "ab_style": round(ab_style(fr, rs), 5)})
    out["addr_gib"] = {"frames": round(frames.data_ptr() / 2**30, 3), "frames2": round(frames2.data_ptr() / 2**30, 3),
                       "res": round(res.data_ptr() / 2**30, 4), "res2": round(res2.data_ptr() / 2**30, 4)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
