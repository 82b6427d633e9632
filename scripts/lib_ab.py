#!/usr/bin/env python3
"""Two builds of the product library side by side in ONE process (interleaved rounds, HIP events): the current
pollnet_amd/libpollnet_amd.so against an earlier build of the same C-ABI (e.g. scripts/_ab/*.so, made from an
older commit with `make pollnet_amd/libpollnet_amd.so` in a git worktree).  Each library gets its own pn_ctx;
every workload's records / filled frames must be identical between the two.  A measurement, not a product path.

  lib_ab.py <other.so> [--rounds R] [--workloads c2,c3,c5,packed3,tx2,tx14,streams]
"""
import argparse
import ctypes as C
import json
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
STRIDE, OFF = 2048, 2


class Lib:
    def __init__(self, path, table):
        self.path = path
        self.lib = C.CDLL(path)  # RTLD_LOCAL: each build keeps its own symbols and kernels
        L = self.lib
        vp, u32, u64, i32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int
        for name, res, args in [("pn_open", i32, [i32, C.POINTER(vp)]), ("pn_close", None, [vp]),
                                ("pn_set_conn_table", i32, [vp, vp, u32, u64, u32]),
                                ("pn_classify", i32, [vp, vp, u32, u32, u32, vp, vp]),
                                ("pn_classify_indexed", i32, [vp, vp, vp, u32, u32, u32, vp, vp]),
                                ("pn_tx_fill", i32, [vp, vp, u32, u32, u32, vp, u32, vp]),
                                ("pn_match_streams", i32, [vp, vp, u32, u32, u32, vp, u32, vp, vp])]:
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        self.ctx = vp()
        assert L.pn_open(0, C.byref(self.ctx)) == 0
        entries, mask, max_conn = table
        assert L.pn_set_conn_table(self.ctx, entries.ctypes.data, len(entries), mask, max_conn) == 0

    def close(self):
        self.lib.pn_close(self.ctx)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("other")
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--workloads", default="c2,c3,c5,packed3,tx2,tx14,streams")
    a = ap.parse_args()
    import torch

    import pollnet_amd as pa
    from bench import time_launches

    n = 1 << 20
    st = torch.cuda.current_stream()
    sp = st.cuda_stream
    out = {"current": os.path.join(ROOT, "pollnet_amd", "libpollnet_amd.so"), "other": a.other, "frames": n}
    for wl in a.workloads.split(","):
        cfg = {"c2": 2, "c3": 3, "c5": 5, "packed3": 3, "tx2": 2, "tx14": 2, "streams": 2}[wl]
        p = pa.rx.GenParams.for_config(cfg)
        t = pa.gen_conn_table(p)
        e, m = t.snapshot()
        libs = [Lib(out["current"], (e, m, t.max_conn_cnt)), Lib(a.other, (e, m, t.max_conn_cnt))]
        off = 14 if wl == "tx14" else OFF
        host = [pa.gen_frames(p, n, STRIDE, off, first_index=b * n) for b in range(2)]
        bufs = [torch.from_numpy(h.reshape(-1)).cuda() for h in host]
        res = [torch.empty(n * 16, dtype=torch.uint8, device="cuda") for _ in libs]
        if wl in ("c2", "c3", "c5"):
            fns = [lambda d, L=L, r=r: L.lib.pn_classify(L.ctx, d.data_ptr(), STRIDE, OFF, n, r.data_ptr(), sp)
                   for L, r in zip(libs, res)]
            for f in fns:
                f(bufs[0])
            torch.cuda.synchronize()
            same = torch.equal(res[0], res[1])
            tbufs = bufs
        elif wl == "packed3":
            s0 = host[0]
            tl = (s0[:, OFF + 16].astype(np.int64) << 8) | s0[:, OFF + 17]
            ln = 14 + tl + 1
            step = (ln + 17) & ~15
            starts = OFF + np.concatenate(([0], np.cumsum(step[:-1])))
            packed = np.zeros(int(starts[-1] + step[-1] + STRIDE), np.uint8)
            for i in range(n):
                packed[starts[i]:starts[i] + ln[i]] = s0[i, OFF:OFF + ln[i]]
            pk = torch.from_numpy(packed).cuda()
            offs = torch.from_numpy(starts.astype(np.uint64).view(np.int64)).cuda()
            fns = [lambda d, L=L, r=r: L.lib.pn_classify_indexed(L.ctx, d.data_ptr(), offs.data_ptr(), OFF, n,
                                                                 STRIDE - OFF, r.data_ptr(), sp)
                   for L, r in zip(libs, res)]
            for f in fns:
                f(pk)
            torch.cuda.synchronize()
            same = torch.equal(res[0], res[1])
            tbufs = [pk]
        elif wl in ("tx2", "tx14"):
            work = [[b.clone() for b in bufs] for _ in libs]
            fns = [lambda d, L=L: L.lib.pn_tx_fill(L.ctx, d.data_ptr(), STRIDE, off, n, None, 0, sp) for L in libs]
            for f, w in zip(fns, work):
                f(w[0])
            torch.cuda.synchronize()
            same = torch.equal(work[0][0], work[1][0])
            # timed on the SAME buffers (the fill is idempotent): a TX fill's time follows where its frames sit in
            # HBM (the write-back of its dirty sectors), so separate copies would compare placements, not builds
            tbufs = work[0]
        else:  # streams: pn_match_streams with 8 wildcard filters
            flt = np.zeros(8, dtype=pa.rx.STREAM_FILTER_DTYPE)
            flt["dst_port"] = np.array([1234, 80, 443, 22, 1235, 8080, 53, 25], np.uint16).byteswap()
            ids = [torch.empty(n * 4, dtype=torch.uint8, device="cuda") for _ in libs]
            fns = [lambda d, L=L, i=i: L.lib.pn_match_streams(L.ctx, d.data_ptr(), STRIDE, OFF, n, flt.ctypes.data,
                                                              len(flt), i.data_ptr(), sp)
                   for L, i in zip(libs, ids)]
            for f in fns:
                f(bufs[0])
            torch.cuda.synchronize()
            same = torch.equal(ids[0], ids[1])
            tbufs = bufs
        times = [[], []]
        for _ in range(a.rounds):
            for k, f in enumerate(fns):
                times[k].append(time_launches(torch, f, tbufs, a.steps, st))
        med = [statistics.median(t) for t in times]
        out[wl] = {"current_ms": round(med[0], 5), "other_ms": round(med[1], 5),
                   "current_over_other": round(med[0] / med[1], 4), "outputs_identical": bool(same)}
        print(wl, out[wl], flush=True)
        for L in libs:
            L.close()
        del bufs, res
        torch.cuda.empty_cache()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
