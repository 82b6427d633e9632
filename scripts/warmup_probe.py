#!/usr/bin/env python3
"""How long after an idle stretch does pn_classify reach its steady-state time?  The resident
batch is classified once (touching every page), the host sleeps IDLE seconds, then 300
back-to-back launches run with an event pair around each one.  Prints per-launch ms in groups.
A measurement, not part of any product path."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import pollnet_amd as pa

    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    idle = float(sys.argv[2]) if len(sys.argv) > 2 else 2.0
    tx_off = int(sys.argv[3]) if len(sys.argv) > 3 else -1  # >= 0: time pn_tx_fill at this frame_off instead
    n, stride, off = 1 << 20, 2048, 2
    p = pa.rx.GenParams.for_config(cfg)
    ctx = pa.RxContext(0)
    ctx.set_conn_table(pa.gen_conn_table(p))
    if tx_off >= 0:
        off = tx_off
    frames = torch.from_numpy(pa.gen_frames(p, n, stride, off).reshape(-1)).cuda()
    frames2 = frames.clone()  # TX: two rotating batches, as the bench's TX leg
    res = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream()

    def launch(i):
        if tx_off >= 0:
            ctx.tx_fill(frames if i % 2 == 0 else frames2, stride, off, n, None, pa.PN_TX_TCP, st)
        else:
            ctx.classify(frames, stride, off, n, res, st)

    launch(0)
    torch.cuda.synchronize()
    out = {"config": cfg, "idle_s": idle, "tx_frame_off": tx_off if tx_off >= 0 else None}
    for trial in range(2):
        time.sleep(idle)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(301)]
        ev[0].record(st)
        for i in range(300):
            launch(i)
            ev[i + 1].record(st)
        torch.cuda.synchronize()
        ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(300)]
        groups = [round(sum(ms[g:g + 10]) / 10, 4) for g in range(0, 300, 10)]
        out[f"trial{trial}_per10"] = groups
        out[f"trial{trial}_cum_ms_to_steady"] = round(sum(ms[:next((i for i, m in enumerate(ms) if m < 1.02 * min(ms[200:])), 300)]), 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
