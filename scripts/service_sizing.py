#!/usr/bin/env python3
"""Resident service large-post sizing (measurement only): a 1-Mi-frame post of device-resident C2 frames
against pn_classify on the same buffers, verified and release path, for several large_waves (pn_service_open_ex),
host wall clock post -> complete, median of --reps.  One JSON line.
    python scripts/service_sizing.py [--waves 64,1088,2112,3136] [--reps 15]"""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pollnet_amd as pa  # noqa: E402

STRIDE, OFF = 2048, 2


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--waves", default="64,1088,2112,3136")
    ap.add_argument("--reps", type=int, default=15)
    a = ap.parse_args()
    import torch

    n = 1 << 20
    p = pa.rx.GenParams.for_config(2)
    host = np.empty((n, STRIDE), np.uint8)
    pa.gen_frames(p, n, STRIDE, OFF, threads=16, out=host)
    bufs = [torch.from_numpy(host.reshape(-1)).cuda()]
    bufs.append(bufs[0].clone())
    del host
    ctx = pa.RxContext(0)
    ctx.set_conn_table(pa.gen_conn_table(p))
    ref = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
    out = torch.empty_like(ref)
    stream = torch.cuda.current_stream()
    res = {}
    for verify in (True, False):
        ctx.set_verify(verify)
        leg = {}

        def cls(k):
            t = time.perf_counter()
            ctx.classify(bufs[k & 1], STRIDE, OFF, n, ref, stream)
            torch.cuda.synchronize()
            return time.perf_counter() - t

        for k in range(3):
            cls(k)
        base = statistics.median(cls(k) for k in range(a.reps))
        leg["pn_classify_ms"] = round(base * 1e3, 4)
        for lw in [int(x) for x in a.waves.split(",")]:
            svc = pa.RxService(ctx, STRIDE, OFF, idle_ms=1000, large_waves=lw)
            try:
                def post(k):
                    t = time.perf_counter()
                    svc.post(bufs[k & 1], n, out)
                    svc.wait()
                    return time.perf_counter() - t

                for k in range(3):
                    post(k)
                ms = statistics.median(post(k) for k in range(a.reps))
                ctx.classify(bufs[0], STRIDE, OFF, n, ref, stream)
                torch.cuda.synchronize()
                svc.post(bufs[0], n, out)
                svc.wait()
                leg[str(lw)] = {"ms": round(ms * 1e3, 4), "vs_pn_classify": round(ms / base, 3),
                                "records_equal": bool(torch.equal(out, ref))}
            finally:
                svc.close()
        res["verified" if verify else "release_path"] = leg
    print(json.dumps(res))


if __name__ == "__main__":
    main()
