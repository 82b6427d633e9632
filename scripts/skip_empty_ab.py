#!/usr/bin/env python3
"""A/B of the stream-load forms in ONE process, interleaved rounds, HIP events on the launch stream.

  product        pn_classify / pn_classify_indexed (the product library's launch path)
  prod_tuning    the same production kernel launched from the tuning library (variant 35) --
                 isolates the launch path from the kernel
  every_load     every stream load issued (the form before kSkipEmptyLoads; variant 37 / indexed 5)
(The per-lane EXEC mask, per-batch gate and per-frame pair-branch forms this script also timed are in
the history: commit c98da75)

Strided 2-KiB slots for C2/C3/C5; packed captures (frames back to back, indexed kernel) for
C3/C5.  Every form's records must equal the product's.  Needs `make TUNING=1`.  One JSON line."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def packed_layout(np, s, n, off):
    tl = (s[:, off + 16].astype(np.int64) << 8) | s[:, off + 17]
    ln = 14 + tl + 1
    starts = np.empty(n, np.int64)
    pos = off
    for i in range(n):
        starts[i] = pos
        pos = ((pos + int(ln[i]) + 15) & ~15) + off
    packed = np.zeros(pos + 2048, np.uint8)
    for i in range(n):
        packed[starts[i]:starts[i] + ln[i]] = s[i, off:off + ln[i]]
    return packed, starts, int(np.sum(ln - 1))


def main():
    import numpy as np
    import torch

    import pollnet_amd as pa
    from pollnet_amd import tuning as tn

    n, stride, off = 1 << 20, 2048, 2
    rounds = int(os.environ.get("AB_ROUNDS", "10"))
    st = torch.cuda.current_stream()
    out = {"frames": n}
    for cfg in (2, 3, 5):
        p = pa.rx.GenParams.for_config(cfg)
        s = pa.gen_frames(p, n, stride, off)
        wire = pa.wire_bytes(s, stride, off, n)
        ctx = pa.RxContext(0)
        ctx.set_conn_table(pa.gen_conn_table(p))
        frames = torch.from_numpy(s.reshape(-1)).cuda()
        ref = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
        res = torch.empty_like(ref)
        ctx.classify(frames, stride, off, n, ref, st)

        def sv(v):
            return lambda: tn.classify_variant(ctx, frames, stride, off, n, res, st, v)

        runs = {"strided_product": lambda: ctx.classify(frames, stride, off, n, res, st),
                "strided_prod_tuning": sv(35), "strided_every_load": sv(37)}
        algo = {k: wire + 16 * n for k in runs}
        if cfg != 2:
            packed, starts, pbytes = packed_layout(np, s, n, off)
            dev = torch.from_numpy(packed).cuda()
            offs = torch.from_numpy(starts.astype(np.uint64).view(np.int64)).cuda()

            def iv(v):
                return lambda: tn.classify_indexed_variant(ctx, dev, offs, off, n, stride - off, res, st, v)

            runs.update({"packed_product": lambda: ctx.classify_indexed(dev, offs, off, n, stride - off, res, st),
                         "packed_every_load": iv(5)})
            for k in runs:
                algo.setdefault(k, pbytes + 16 * n)
        equal = {}
        for k, f in runs.items():
            res.zero_()
            f()
            torch.cuda.synchronize()
            equal[k] = bool(torch.equal(res, ref))
        times = {k: [] for k in runs}
        for _ in range(rounds):
            for k, f in runs.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                f()
                e0.record(st)
                for _ in range(10):
                    f()
                e1.record(st)
                e1.synchronize()
                times[k].append(e0.elapsed_time(e1) / 10)
        r = {"records_equal": equal}
        for k, v in times.items():
            ms = statistics.median(v)
            r[k] = {"ms_median": round(ms, 5), "ms_min": round(min(v), 5), "frac_of_8TBs": round(algo[k] / (ms * 1e-3) / 8e12, 4)}
        out[f"c{cfg}"] = r
        ctx.close()
        del frames, ref, res
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
