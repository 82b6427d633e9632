#!/usr/bin/env python3
"""Interleaved A/B of pn_match_streams forms (tuning library variants) on the bench's workload: 1 Mi
resident 2-KiB C2 slots x 4 rotating batches, the bench's 8 filters (7 flows not in the batch, then a
dst-port filter every frame passes), plus C3 with 7 single-flow filters and the dst-port filter.
Variant ids must equal the production kernel's (and numpy's filterPacket on batch 0).

  python scripts/match_ab.py [--rounds 9] [--variants 1,5,10,...]   -> one JSON object on stdout"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

TIMING_ONLY = {5, 15, 16, 17, 18, 19, 21, 23, 25, 27, 29, 34, 35, 38, 40}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--variants", default="1,5,12,13,17,18,20,21,22,23,24,25,26,27,28,29")
    ap.add_argument("--configs", default="2,3")
    args = ap.parse_args()
    import numpy as np
    import torch

    import pollnet_amd as pa
    from pollnet_amd import tuning as tn
    from streams_np import match_streams_np

    variants = [int(v) for v in args.variants.split(",")]
    n, off = 1 << 20, 2
    out = {"note": __doc__.splitlines()[0], "rounds": args.rounds}
    for cfg in [int(c) for c in args.configs.split(",")]:
        p = pa.rx.GenParams.for_config(cfg)
        host = [pa.gen_frames(p, n, 2048, off, first_index=b * n) for b in range(4)]
        dev = [torch.from_numpy(h.reshape(-1)).cuda() for h in host]
        flt = np.zeros(8, pa.STREAM_FILTER_DTYPE)
        if cfg == 2:  # bench.py secondary_streams: 7 flows not in the batch, then dst port 1234
            for k in range(7):
                flt[k] = (int.from_bytes(bytes([10, 9, k, 1]), "little"), 0,
                          int.from_bytes((5000 + k).to_bytes(2, "big"), "little"), 0, 0)
        else:  # 7 flows of the batch (single-flow filters), then dst port 1234
            for k in range(7):
                e = host[0][k * 997, off:]
                flt[k] = (int.from_bytes(bytes(e[26:30]), "little"), 0, int.from_bytes(bytes(e[34:36]), "little"), 0, 0)
        flt[7] = (0, 0, 0, int.from_bytes((1234).to_bytes(2, "big"), "little"), 0)
        ctx = pa.RxContext(0)
        st = torch.cuda.current_stream()
        ids = torch.empty(n, dtype=torch.int32, device="cuda")
        ctx.match_streams(dev[0], 2048, off, n, flt, ids, st)
        torch.cuda.synchronize()
        ref = ids.clone()
        np_ok = bool(np.array_equal(ref.cpu().numpy().view(np.uint32), match_streams_np(host[0], off, flt)))
        same = {}
        for v in variants:
            if v in TIMING_ONLY:
                continue
            got = torch.full_like(ids, 7)
            for b in range(4):  # every batch: the variants against the product
                ctx.match_streams(dev[b], 2048, off, n, flt, ids, st)
                tn.match_streams_variant(ctx, dev[b], 2048, off, n, flt, got, v, st)
                torch.cuda.synchronize()
                same[v] = same.get(v, True) and bool(torch.equal(got, ids))
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        sink = torch.empty_like(ids)

        def timed(fn, reps=40):
            for r in range(8):
                fn(dev[r % 4])
            ev[0].record(st)
            for r in range(reps):
                fn(dev[r % 4])
            ev[1].record(st)
            torch.cuda.synchronize()
            return ev[0].elapsed_time(ev[1]) / reps

        times = {v: [] for v in variants}
        for _ in range(args.rounds):
            for v in variants:
                buf = sink if v in TIMING_ONLY else ids
                times[v].append(timed(lambda d: tn.match_streams_variant(ctx, d, 2048, off, n, flt, buf, v, st)))
        res = {}
        for v in variants:
            ms = statistics.median(times[v])
            res[str(v)] = {"ms": round(ms, 5), "min_ms": round(min(times[v]), 5),
                           "frac": round(n * 68 / (ms * 1e-3) / 1e9 / 8000, 4),
                           "ids_equal_product": same.get(v)}
        out[f"c{cfg}"] = {"numpy_ok": np_ok, "variants": res}
        ctx.close()
        del dev
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
