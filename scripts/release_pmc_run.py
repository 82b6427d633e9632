#!/usr/bin/env python3
"""The release-path classify (pn_set_verify(ctx, 0)) on C2, for rocprofv3 --pmc passes: 4 rotating resident 1-Mi
batches, 10 launches each, plus the 16-B streaming-read calibration kernel over a known byte count (the FETCH_SIZE
correction, as scripts/gpu_pmc.sh does for the full path).  scripts/release_pmc.sh runs the passes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import pollnet_amd as pa
    from pollnet_amd import tuning as tn

    n, stride, off = 1 << 20, 2048, 2
    p = pa.rx.GenParams.for_config(2)
    t = pa.gen_conn_table(p)
    ctx = pa.RxContext(0)
    ctx.set_conn_table(t)
    ctx.set_verify(False)
    bufs = [torch.from_numpy(pa.gen_frames(p, n, stride, off, first_index=b * n).reshape(-1)).cuda() for b in range(4)]
    res = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
    sink = torch.zeros(4096, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream()
    for k in range(40):
        ctx.classify(bufs[k % 4], stride, off, n, res, st)
    for _ in range(10):
        tn.calib_stream_read(ctx, bufs[0], bufs[0].numel(), sink, st)
    torch.cuda.synchronize()
    ctx.close()
    print("release-path classify: 40 launches of 1 Mi C2 frames; calibration: 10 reads of", bufs[0].numel(), "B")


if __name__ == "__main__":
    main()
