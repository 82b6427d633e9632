#!/usr/bin/env python3
"""Workload for rocprofv3 --pmc passes (run under the profiler, one counter set per pass):
  - pn_calib_stream_read over the whole frame buffer (a known byte count, 16-B
    coalesced loads) -> calibrates FETCH_SIZE for this box (gfx950 reports about
    half the bytes of wide streaming reads: MI355X_MICROARCH.md §HBM);
  - pn_classify over the same buffer (the measured kernel).
Each is launched --reps times; the buffer (2 GiB) exceeds the 256 MiB Infinity
Cache, so every pass streams from HBM."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--frames", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--variant", type=int, default=-1, help="tuning variant instead of the production kernel")
    a = ap.parse_args()
    import torch

    import pollnet_amd as pa
    from pollnet_amd import tuning as tn

    p = pa.rx.GenParams.for_config(a.config)
    s = pa.gen_frames(p, a.frames)
    t = pa.gen_conn_table(p)
    ctx = pa.RxContext(0)
    ctx.set_conn_table(t)
    frames = torch.from_numpy(s.reshape(-1)).cuda()
    res = torch.empty(a.frames * 16, dtype=torch.uint8, device="cuda")
    sink = torch.zeros(4096, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream()
    for _ in range(a.reps):
        tn.calib_stream_read(ctx, frames, frames.numel(), sink, st)
        if a.variant < 0:
            ctx.classify(frames, 2048, 2, a.frames, res, st)
        else:
            tn.classify_variant(ctx, frames, 2048, 2, a.frames, res, st, a.variant)
    torch.cuda.synchronize()
    print(f"calib_bytes={frames.numel()} wire_bytes={pa.wire_bytes(s, 2048, 2, a.frames)} frames={a.frames}")


if __name__ == "__main__":
    main()
