#!/usr/bin/env python3
"""Does where the CPU baseline's frames live change the reference's speed?  The same 256 Ki C2 frames in a private
anonymous array (round 4's `host.copy()`) and in the shared host ring's shard (round 5's e2e leg generates batch 0
there), the reference's own code (oracle/_ref/libref_core.so) and the oracle's port timed on each, 1 thread and the
box's share, passes interleaved round-robin.  Also the kernel's transparent-huge-page settings.  No GPU is touched.

  python3 scripts/cpu_placement_probe.py  ->  one JSON object"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np

    import bench
    import pollnet_amd as pa
    from oracle import pyoracle as orc
    from pollnet_amd.host_ring import SharedHostRing

    n, th = 1 << 18, bench.cpu_threads()
    p = pa.rx.GenParams.for_config(2)
    private = pa.gen_frames(p, n, threads=min(16, th))
    ring = SharedHostRing(None, 0, 1, n, 2048)
    shared = ring.shard()
    shared[:] = private
    t = pa.gen_conn_table(p)
    e, m = t.snapshot()
    ref = orc.RefBench(e)
    legs = {}
    for where, arr in (("private", private), ("shared_ring", shared)):
        for threads in (1, th):
            legs[f"ref_{where}_{threads}t"] = (lambda a, k: ref.batch(a, 2048, 2, n, k), arr, threads)
            legs[f"port_{where}_{threads}t"] = (
                lambda a, k: orc.classify_batch(a, 2048, 2, n, e, m, t.max_conn_cnt, threads=k, ref_only=True), arr, threads)
    runs = {k: [] for k in legs}
    for _ in range(5):
        for k, (fn, arr, threads) in legs.items():
            t0 = time.perf_counter()
            passes = 0
            while time.perf_counter() - t0 < 0.3:
                fn(arr, threads)
                passes += 1
            runs[k].append(passes * n / (time.perf_counter() - t0) / 1e6)
    out = {"frames": n, "threads": th, "unit": "M frames/s (median of 5 interleaved passes)",
           **{k: round(statistics.median(v), 3) for k, v in runs.items()}}
    for f in ("enabled", "shmem_enabled", "defrag"):
        try:
            with open(f"/sys/kernel/mm/transparent_hugepage/{f}") as fh:
                out[f"thp_{f}"] = fh.read().strip()
        except OSError:
            pass
    print(json.dumps(out, indent=1))
    del shared
    ring.close()


if __name__ == "__main__":
    main()
