#!/usr/bin/env python3
"""Does a narrower header read cut the zero-copy release path's PCIe bytes?  Frames in pinned host memory (2-KiB
slots, 1 Mi C2 frames), read in place over PCIe by the tuning library's slot-read ceiling (the RX kernel's load
pattern, no arithmetic) with the first 64, 128 or 256 bytes of each slot, 16-B records written to pinned host
memory; beside it the product's release-path classify (pn_set_verify(ctx, 0)) on the same slots.  Host wall clock
per pass (best of 5) and the implied PCIe read rate.

  python3 scripts/zc_narrow_probe.py  ->  one JSON object"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    import pollnet_amd as pa
    from pollnet_amd import tuning as tn

    n, stride, off = 1 << 20, 2048, 2
    p = pa.rx.GenParams.for_config(2)
    host = torch.empty(n * stride, dtype=torch.uint8).pin_memory()
    pa.gen_frames(p, n, stride, off, first_index=0, threads=16, out=host.numpy().reshape(n, stride))
    rec = torch.empty(n * 16, dtype=torch.uint8).pin_memory()
    ctx = pa.RxContext(0)
    ctx.set_conn_table(pa.gen_conn_table(p))
    st = torch.cuda.current_stream()
    out = {"frames": n, "slot_stride": stride, "unit": "M slots/s (host wall clock, best of 5)"}

    def best(fn, passes=5):
        fn()
        torch.cuda.synchronize()
        b = None
        for _ in range(passes):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            b = el if b is None else min(b, el)
        return b

    for nbytes in (64, 128, 256):
        t = best(lambda: tn.calib_slot_read(ctx, host, n, stride, nbytes, rec, st, store_bytes=16))
        out[f"slot_read_{nbytes}B"] = {"mslots_per_s": round(n / t / 1e6, 1), "read_gb_per_s": round(n * nbytes / t / 1e9, 2)}
    ctx.set_verify(False)
    t = best(lambda: ctx.classify(host, stride, off, n, rec, st))
    out["product_release_path_classify"] = {"mframes_per_s": round(n / t / 1e6, 1)}
    ctx.set_verify(True)
    print(json.dumps(out, indent=1))
    ctx.close()


if __name__ == "__main__":
    main()
