"""Optional GPU soak (PN_SOAK=<seeds> to run; skipped otherwise): random slot contents and generated C3/C5 frames
over many seeds, random layouts (frame_off, stride, n), through the full path and the release path
(pn_set_verify(ctx, 0)), every record against the oracle.  The suite's parity tests fix their seeds; this widens
them without slowing the suite."""
import os

import numpy as np
import pytest

import pollnet_amd as pa
from oracle import pyoracle as orc

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not os.environ.get("PN_SOAK"), reason="soak: set PN_SOAK=<number of seeds>")]
F = pa.rx.F


def release(exp):
    r = exp.copy()
    r["flags"] = (r["flags"] & ~np.uint16(F.TCP_OK | F.RFC_TCP_OK)) | np.uint16(F.TCP_UNCHECKED)
    r["tcp_fold"] = 0
    return r


def test_random_layout_soak():
    import torch

    assert torch.cuda.is_available()
    seeds = int(os.environ["PN_SOAK"])
    ctx = pa.RxContext(0)
    offs = [0, 2, 4, 6, 8, 10, 12, 14, 18, 34, 50, 98, 126]
    strides = [112, 128, 256, 1536, 2048, 4096, 9216]
    checked = 0
    for seed in range(seeds):
        rng = np.random.default_rng(0x50A4 + seed)
        cfg = int(rng.choice([3, 5]))
        stride = int(rng.choice(strides))
        off = int(rng.choice([o for o in offs if o + 96 <= stride]))
        n = int(rng.integers(1, 40000 if stride <= 2048 else 4000))
        p = pa.rx.GenParams.for_config(cfg)
        t = pa.gen_conn_table(p)
        e, m = t.snapshot()
        s = pa.gen_frames(p, n, stride, off)
        # a quarter of the slots overwritten with random bytes (garbage headers, any tot_len / IHL / doff)
        junk = rng.random(n) < 0.25
        s[junk] = rng.integers(0, 256, size=(int(junk.sum()), stride), dtype=np.uint8)
        exp = orc.classify_batch(s, stride, off, n, e, m, t.max_conn_cnt, threads=8)
        ctx.set_conn_table(t)
        frames = torch.from_numpy(np.ascontiguousarray(s).reshape(-1)).cuda()
        res = torch.full(((n + 7) * 16,), 0xAB, dtype=torch.uint8, device="cuda")
        for verify in (True, False):
            ctx.set_verify(verify)
            ctx.classify(frames, stride, off, n, res, torch.cuda.current_stream())
            torch.cuda.synchronize()
            out = res.cpu().numpy()
            assert (out[n * 16:] == 0xAB).all(), f"seed {seed}: wrote past n"
            got = out[: n * 16].view(pa.RESULT_DTYPE)
            want = exp if verify else release(exp)
            bad = np.nonzero(got != want)[0]
            assert len(bad) == 0, (f"seed {seed} cfg {cfg} stride {stride} off {off} n {n} verify {verify}: "
                                   f"{len(bad)} records differ, first #{bad[0]}: {got[bad[0]]} vs {want[bad[0]]}")
            checked += n
        ctx.set_verify(True)
    ctx.close()
    print(f"soak: {seeds} seeds, {checked} records checked")
