#!/usr/bin/env python3
"""Device-resident rate of pn_match_streams (TcpStream::filterPacket on the GPU,
SURVEY §8(f) rank 3) over 1 Mi resident slots: 8 wildcard filters, HIP events on the
launch stream, 4 rotating batches.  Algorithmic bytes per frame: the 64-B header window
read + the 4-B stream id written.  Ids checked against the numpy restatement."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="2,3")
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--policies", action="store_true", help="also time the cooperative form with other load / store cache policies")
    args = ap.parse_args()
    import numpy as np
    import torch

    import pollnet_amd as pa
    from pollnet_amd import tuning as tn
    from streams_np import match_streams_np

    n, off = 1 << 20, 2
    out = {}
    for cfg in [int(c) for c in args.configs.split(",")]:
        p = pa.rx.GenParams.for_config(cfg)
        host = [pa.gen_frames(p, n, 2048, off, first_index=b * n) for b in range(4)]
        dev = [torch.from_numpy(h.reshape(-1)).cuda() for h in host]
        flt = np.zeros(8, pa.STREAM_FILTER_DTYPE)
        for k in range(8):  # 7 single-flow filters + a dst-port filter
            e = host[0][k * 997, off:]
            flt[k] = (int.from_bytes(bytes(e[26:30]), "little"), 0, int.from_bytes(bytes(e[34:36]), "little"), 0, 0)
        flt[7] = (0, 0, 0, int.from_bytes((1234).to_bytes(2, "big"), "little"), 0)
        ctx = pa.RxContext(0)
        ids = torch.empty(n, dtype=torch.int32, device="cuda")
        st = torch.cuda.current_stream()
        ctx.match_streams(dev[0], 2048, off, n, flt, ids, st)
        torch.cuda.synchronize()
        ok = np.array_equal(ids.cpu().numpy().view(np.uint32), match_streams_np(host[0], off, flt))
        # the per-lane form (tuning variant 0) gives the same ids
        ids0 = torch.empty_like(ids)
        tn.match_streams_variant(ctx, dev[0], 2048, off, n, flt, ids0, 0, st)
        torch.cuda.synchronize()
        ok = ok and bool(torch.equal(ids0, ids))
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

        def timed(fn, reps=20):
            ev[0].record(st)
            for r in range(reps):
                fn(dev[r % 4])
            ev[1].record(st)
            torch.cuda.synchronize()
            return ev[0].elapsed_time(ev[1]) / reps

        ts, ts0, tg = [], [], []
        for _ in range(args.rounds):  # interleaved: production, per-lane form, the production loads alone
            ts.append(timed(lambda d: ctx.match_streams(d, 2048, off, n, flt, ids, st)))
            ts0.append(timed(lambda d: tn.match_streams_variant(ctx, d, 2048, off, n, flt, ids0, 0, st)))
            tg.append(timed(lambda d: tn.match_streams_variant(ctx, d, 2048, off, n, flt, ids0, 5, st)))
        ms, ms0, mg = statistics.median(ts), statistics.median(ts0), statistics.median(tg)
        pol = {}
        ctx.match_streams(dev[0], 2048, off, n, flt, ids, st)  # the timed loops left another batch's ids
        if args.policies:
            for v, name in ((9, "default"), (2, "nt"), (3, "sc0"), (4, "sc1"), (6, "store_sc1"), (7, "nt_load_store_sc1"), (8, "store_nt")):
                ids_v = torch.empty_like(ids)
                tn.match_streams_variant(ctx, dev[0], 2048, off, n, flt, ids_v, v, st)
                torch.cuda.synchronize()
                assert torch.equal(ids_v, ids)
                pol[name] = round(statistics.median(
                    timed(lambda d: tn.match_streams_variant(ctx, d, 2048, off, n, flt, ids_v, v, st)) for _ in range(args.rounds)), 5)
        # same-run ceiling for this access pattern: the first 64 / 128 B of every 2-KiB slot,
        # the RX kernel's load pattern, no arithmetic, nothing written
        sink = torch.zeros(4096, dtype=torch.int32, device="cuda")
        ceil = {}
        for nb in (64, 128):
            cs = []
            for _ in range(max(3, args.rounds // 2)):
                ev[0].record(st)
                for r in range(20):
                    tn.calib_slot_read(ctx, dev[r % 4], n, 2048, nb, sink, st, 0)
                ev[1].record(st)
                torch.cuda.synchronize()
                cs.append(ev[0].elapsed_time(ev[1]) / 20)
            ceil[f"slot_read_first_{nb}B_ms"] = round(statistics.median(cs), 5)
        algo = n * (64 + 4)
        out[f"c{cfg}"] = {"ids_equal_numpy": ok, "ms_median": round(ms, 5), "per_lane_form_ms_median": round(ms0, 5),
                          "cooperative_load_policies_ms": pol,
                          "mframes_per_s": round(n / (ms * 1e-3) / 1e6, 1),
                          "algo_gbs": round(algo / (ms * 1e-3) / 1e9, 1),
                          "line_gbs": round(n * (128 + 4) / (ms * 1e-3) / 1e9, 1),
                          "same_run_ceilings": dict(ceil, gather_loads_only_ms=round(mg, 5),
                                                    kernel_vs_gather_ceiling=round(mg / ms, 4)),
                          "note": "algo = 64-B header window + 4-B id per frame; line = the 128-B line it lives in"}
        ctx.close()
        del dev
    print(json.dumps(out))


if __name__ == "__main__":
    main()
