#!/usr/bin/env python3
"""Three C2 classify launches on one resident batch: the target of a rocprofv3 --pmc run whose JSON output is
inspected for per-instance (per TCC channel / XCD) counter values (a measurement, not a product path)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import pollnet_amd as pa

    n = 1 << 20
    p = pa.rx.GenParams.for_config(2)
    s = pa.gen_frames(p, n)
    ctx = pa.RxContext(0)
    ctx.set_conn_table(pa.gen_conn_table(p))
    frames = torch.from_numpy(s.reshape(-1)).cuda()
    res = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
    for _ in range(3):
        ctx.classify(frames, 2048, 2, n, res, torch.cuda.current_stream())
    torch.cuda.synchronize()
    ctx.close()
    print("ok")


if __name__ == "__main__":
    main()
