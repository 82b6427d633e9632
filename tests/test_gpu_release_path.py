"""GPU: pn_set_verify(ctx, 0) — the reference's release path (Core::checksum is debug-only, Core.h:448-478), so
the kernel reads only each frame's header lines.  Every record must equal the oracle's full record with its TCP
verdict taken out: TCP_OK and RFC_TCP_OK cleared, PN_F_TCP_UNCHECKED set, tcp_fold 0xFFFF (no fold computed); every other field (conn id,
seq, payload offset/length, the IP verdicts, TRUNC, NOT_TCP, IHL_NE_5, the flags) bit-exact.  Strided (all 8
alignment classes, strides 112 B..64 KiB, every frames-per-wave split), notify, indexed/packed, random bytes."""
import numpy as np
import pytest

import pollnet_amd as pa
from oracle import pyoracle as orc

from frames import FRAME_OFF, STRIDE

pytestmark = pytest.mark.gpu
F = pa.rx.F


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


@pytest.fixture
def ctx(torch_cuda):
    c = pa.RxContext(0)
    c.set_verify(False)
    yield c
    c.close()


def release(exp):
    """The oracle's full records as the release path reports them."""
    r = exp.copy()
    r["flags"] = (r["flags"] & ~np.uint16(F.TCP_OK | F.RFC_TCP_OK)) | np.uint16(F.TCP_UNCHECKED)
    r["tcp_fold"] = 0xFFFF
    return r


def classify(torch, ctx, slots, stride, off, n, table, canary=0):
    ctx.set_conn_table(table)
    frames = torch.from_numpy(np.ascontiguousarray(slots).reshape(-1)).cuda()
    res = torch.full(((n + canary) * 16,), 0xAB, dtype=torch.uint8, device="cuda")
    ctx.classify(frames, stride, off, n, res, torch.cuda.current_stream())
    torch.cuda.synchronize()
    out = res.cpu().numpy()
    if canary:
        assert (out[n * 16:] == 0xAB).all(), "kernel wrote past n records"
    return out[: n * 16].view(pa.RESULT_DTYPE).copy()


def same(got, exp):
    if np.array_equal(got, exp):
        return
    bad = np.nonzero(got != exp)[0]
    raise AssertionError(f"{len(bad)} records differ; first #{bad[0]}: gpu={got[bad[0]]} expected={exp[bad[0]]}")


@pytest.mark.parametrize("frame_off", [0, 2, 4, 6, 8, 10, 12, 14, 18, 50, 98, 126])
def test_every_alignment_class(torch_cuda, ctx, frame_off):
    p = pa.rx.GenParams.for_config(5)
    t = pa.gen_conn_table(p)
    e, m = t.snapshot()
    n = 3000
    s = pa.gen_frames(p, n, STRIDE, frame_off)
    exp = orc.classify_batch(s, STRIDE, frame_off, n, e, m, t.max_conn_cnt, threads=8)
    same(classify(torch_cuda, ctx, s, STRIDE, frame_off, n, t, canary=3), release(exp))


@pytest.mark.parametrize("stride,frame_off", [(112, 2), (1536, 2), (4096, 2), (9216, 8), (65536, 2)])
def test_slot_strides(torch_cuda, ctx, stride, frame_off):
    p = pa.rx.GenParams.for_config(3)
    t = pa.gen_conn_table(p)
    e, m = t.snapshot()
    n = 700 if stride < 65536 else 64
    s = pa.gen_frames(p, n, stride, frame_off)
    exp = orc.classify_batch(s, stride, frame_off, n, e, m, t.max_conn_cnt)
    same(classify(torch_cuda, ctx, s, stride, frame_off, n, t), release(exp))


@pytest.mark.parametrize("n", [1, 9, 64, 65, 1000, 16369, 65473])
@pytest.mark.parametrize("cfg", [2, 3])
def test_batch_sizes(torch_cuda, ctx, n, cfg):
    p = pa.rx.GenParams.for_config(cfg)
    t = pa.gen_conn_table(p)
    e, m = t.snapshot()
    s = pa.gen_frames(p, n)
    exp = orc.classify_batch(s, STRIDE, FRAME_OFF, n, e, m, t.max_conn_cnt, threads=8)
    got = classify(torch_cuda, ctx, s, STRIDE, FRAME_OFF, n, t, canary=65)
    same(got, release(exp))
    if cfg == 2 and n >= 1024:  # C2 flips a payload bit in every 1024th frame: the full path fails those frames
        assert (exp["flags"] & F.TCP_OK == 0).any() and (got["flags"] & F.TCP_UNCHECKED).all()


def test_random_bytes(torch_cuda, ctx):
    rng = np.random.default_rng(4321)
    n = 20000
    s = rng.integers(0, 256, size=(n, STRIDE), dtype=np.uint8)
    p = pa.rx.GenParams.for_config(5)
    t = pa.gen_conn_table(p)
    e, m = t.snapshot()
    s[: n // 3] = pa.gen_frames(p, n // 3)
    idx = rng.integers(0, n, 3000)
    tl = rng.integers(0, 2100, 3000).astype(np.uint16)
    s[idx, FRAME_OFF + 16] = (tl >> 8).astype(np.uint8)
    s[idx, FRAME_OFF + 17] = (tl & 255).astype(np.uint8)
    exp = orc.classify_batch(s, STRIDE, FRAME_OFF, n, e, m, t.max_conn_cnt, threads=8)
    got = classify(torch_cuda, ctx, s, STRIDE, FRAME_OFF, n, t)
    same(got, release(exp))
    assert (got["flags"] & F.TRUNC).any() and (got["flags"] & F.RFC_IP_OK).any()


def test_notify(torch_cuda, ctx):
    torch = torch_cuda
    p = pa.rx.GenParams.for_config(3)
    t = pa.gen_conn_table(p)
    e, m = t.snapshot()
    ctx.set_conn_table(t)
    n = 1000
    s = pa.gen_frames(p, n)
    exp = release(orc.classify_batch(s, STRIDE, FRAME_OFF, n, e, m, t.max_conn_cnt))
    frames = torch.from_numpy(s.reshape(-1)).cuda()
    res = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    word = torch.zeros(1, dtype=torch.int32).pin_memory()
    ctx.classify_notify(frames, STRIDE, FRAME_OFF, n, res, word, 7, torch.cuda.current_stream())
    torch.cuda.synchronize()
    assert int(word[0]) == 7
    same(res.cpu().numpy().view(pa.RESULT_DTYPE), exp)


@pytest.mark.parametrize("eth_mod16", [2, 14])
def test_packed_capture(torch_cuda, ctx, eth_mod16):
    torch = torch_cuda
    n, avail = 2000, 1600
    p = pa.rx.GenParams.for_config(3)
    t = pa.gen_conn_table(p)
    e, m = t.snapshot()
    ctx.set_conn_table(t)
    src = pa.gen_frames(p, n, 2048, 2)
    flen = 14 + ((src[:, 18].astype(np.int64) << 8) | src[:, 19])
    offs = np.zeros(n, dtype=np.uint64)
    pos = 0
    for i in range(n):
        o = ((pos + 15) & ~15) + eth_mod16
        offs[i] = o
        pos = o + int(flen[i])
    buf = np.zeros(pos + avail + 64, dtype=np.uint8)
    for i in range(n):
        o = int(offs[i])
        buf[o:o + int(flen[i])] = src[i, 2:2 + int(flen[i])]
    res = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    ctx.classify_indexed(torch.from_numpy(buf).cuda(), torch.from_numpy(offs.view(np.int64)).cuda(), eth_mod16, n,
                         avail, res, torch.cuda.current_stream())
    torch.cuda.synchronize()
    exp = np.empty(n, dtype=pa.RESULT_DTYPE)
    for i in range(n):
        o = int(offs[i])
        exp[i] = orc.classify_frame(buf[o:o + avail].tobytes(), avail, e, m, t.max_conn_cnt)
    same(res.cpu().numpy().view(pa.RESULT_DTYPE), release(exp))


def test_verify_switches_back(torch_cuda, ctx):
    """The setting applies to later launches: back on, the full records return."""
    p = pa.rx.GenParams.for_config(2)
    t = pa.gen_conn_table(p)
    e, m = t.snapshot()
    n = 4096
    s = pa.gen_frames(p, n)
    exp = orc.classify_batch(s, STRIDE, FRAME_OFF, n, e, m, t.max_conn_cnt)
    same(classify(torch_cuda, ctx, s, STRIDE, FRAME_OFF, n, t), release(exp))
    ctx.set_verify(True)
    same(classify(torch_cuda, ctx, s, STRIDE, FRAME_OFF, n, t), exp)


def test_zero_copy_pinned_host(torch_cuda, ctx):
    """Frames and records in pinned host memory (the kernel reads the header lines over PCIe)."""
    torch = torch_cuda
    p = pa.rx.GenParams.for_config(5)
    t = pa.gen_conn_table(p)
    e, m = t.snapshot()
    ctx.set_conn_table(t)
    n = 5000
    s = pa.gen_frames(p, n)
    exp = release(orc.classify_batch(s, STRIDE, FRAME_OFF, n, e, m, t.max_conn_cnt, threads=8))
    host = torch.from_numpy(s.reshape(-1)).pin_memory()
    res = torch.zeros(n * 16, dtype=torch.uint8).pin_memory()
    ctx.classify(host, STRIDE, FRAME_OFF, n, res, torch.cuda.current_stream())
    torch.cuda.synchronize()
    same(res.numpy().view(pa.RESULT_DTYPE), exp)
