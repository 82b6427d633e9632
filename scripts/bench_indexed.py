#!/usr/bin/env python3
"""Device-resident cost of the indexed layout (pn_classify_indexed) vs the strided
kernel on the same C2/C3 batch: identity offsets (an in-order event run) and a
random permutation (events scattered over the ring).  Interleaved rounds, HIP events
on the launch stream; records must equal the strided kernel's."""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--frames", type=int, default=1 << 20)
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import numpy as np
    import torch

    import pollnet_amd as pa
    from pollnet_amd import tuning as tn

    n, stride, off = a.frames, 2048, 2
    p = pa.rx.GenParams.for_config(a.config)
    s = pa.gen_frames(p, n)
    wire = pa.wire_bytes(s, stride, off, n)
    ctx = pa.RxContext(0)
    ctx.set_conn_table(pa.gen_conn_table(p))
    frames = torch.from_numpy(s.reshape(-1)).cuda()
    st = torch.cuda.current_stream()
    ident = torch.from_numpy((np.arange(n, dtype=np.uint64) * stride + off).view(np.int64)).cuda()
    perm_ids = np.random.default_rng(1).permutation(n)
    perm = torch.from_numpy((perm_ids.astype(np.uint64) * stride + off).view(np.int64)).cuda()
    ref = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
    out = torch.empty_like(ref)
    ctx.classify(frames, stride, off, n, ref, st)
    torch.cuda.synchronize()
    r = ref.cpu().numpy().view(pa.RESULT_DTYPE)
    # packed capture layout: each frame (+ its pad byte, zero) copied back to back, the next
    # Ethernet header at the next 16-B boundary + 2 (same alignment class as the slots)
    tl = (s[:, off + 16].astype(np.int64) << 8) | s[:, off + 17]
    ln = 14 + tl + 1
    starts = np.empty(n, np.int64)
    pos = off
    for i in range(n):
        starts[i] = pos
        pos = ((pos + int(ln[i]) + 15) & ~15) + off
    packed = np.zeros(pos + stride, np.uint8)
    for i in range(n):
        packed[starts[i]:starts[i] + ln[i]] = s[i, off:off + ln[i]]
    packed_dev = torch.from_numpy(packed).cuda()
    poffs = torch.from_numpy(starts.astype(np.uint64).view(np.int64)).cuda()
    runs = {
        "indexed_packed": lambda: ctx.classify_indexed(packed_dev, poffs, off, n, stride - off, out, st),
        "indexed_packed_all_default": lambda: tn.classify_indexed_variant(ctx, packed_dev, poffs, off, n, stride - off, out, st, 3),
        "indexed_packed_blockidx_order": lambda: tn.classify_indexed_variant(ctx, packed_dev, poffs, off, n, stride - off, out, st, 2),
        "indexed_permuted_blockidx_order": lambda: tn.classify_indexed_variant(ctx, frames, perm, off, n, stride - off, out, st, 2),
        "strided": lambda: ctx.classify(frames, stride, off, n, out, st),
        "indexed_in_order": lambda: ctx.classify_indexed(frames, ident, off, n, stride - off, out, st),
        "indexed_permuted": lambda: ctx.classify_indexed(frames, perm, off, n, stride - off, out, st),
        "indexed_in_order_perlane": lambda: tn.classify_indexed_variant(ctx, frames, ident, off, n, stride - off, out, st, 0),
        "indexed_in_order_coop_win_nt": lambda: tn.classify_indexed_variant(ctx, frames, ident, off, n, stride - off, out, st, 1),
        "indexed_permuted_coop_win_nt": lambda: tn.classify_indexed_variant(ctx, frames, perm, off, n, stride - off, out, st, 1),
        "indexed_packed_win_nt": lambda: tn.classify_indexed_variant(ctx, packed_dev, poffs, off, n, stride - off, out, st, 1),
    }
    for name, f in runs.items():  # parity first
        f()
        torch.cuda.synchronize()
        g = out.cpu().numpy().view(pa.RESULT_DTYPE)
        exp = r[perm_ids] if "permuted" in name else r
        assert np.array_equal(g, exp), name
    times = {k: [] for k in runs}
    for _ in range(a.rounds):
        for k, f in runs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(a.reps):
                f()
            e1.record(st)
            e1.synchronize()
            times[k].append(e0.elapsed_time(e1) / a.reps)
    algo = wire + 16 * n
    res = {"config": a.config, "frames": n, "records_equal": True, "packed_bytes": int(pos), "slot_bytes": n * stride}
    for k, v in times.items():
        ms = statistics.median(v)
        res[k] = {"ms_median": round(ms, 4), "algo_tbps": round(algo / (ms * 1e-3) / 1e12, 3),
                  "gbit_per_s": round(8 * wire / (ms * 1e-3) / 1e9, 1)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
