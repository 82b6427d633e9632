"""GPU: pn_classify_indexed — frames named by offsets instead of a stride (SURVEY §8(f)
rank 2, RX-ring ingestion).

An ef_vi RX event batch names slots by id (Core.h:503-505): the run wraps around the
ring and skips discarded slots (EF_EVENT_TYPE_RX_DISCARD, Core.h:534-539), so the
frames to classify are base + id*RecvBufSize + sizeof(RecvBuf) + prefix.  Packed
captures place frames back to back.  Every record must equal what pn_classify (and
the oracle) produce for the same frame bytes and the same readable extent."""
import numpy as np
import pytest

import pollnet_amd as pa
from oracle import pyoracle as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


@pytest.fixture(scope="module")
def ctx(torch_cuda):
    c = pa.RxContext(0)
    yield c
    c.close()


def _strided(torch, ctx, slots, stride, off, n):
    frames = torch.from_numpy(slots.reshape(-1)).cuda()
    res = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
    ctx.classify(frames, stride, off, n, res, torch.cuda.current_stream())
    torch.cuda.synchronize()
    return res.cpu().numpy().view(pa.RESULT_DTYPE).copy(), frames


def _indexed(torch, ctx, base_dev, offsets, eth_mod16, avail, canary=13):
    n = len(offsets)
    offs = torch.from_numpy(np.asarray(offsets, dtype=np.uint64).view(np.int64)).cuda()
    res = torch.full(((n + canary) * 16,), 0xAB, dtype=torch.uint8, device="cuda")
    ctx.classify_indexed(base_dev, offs, eth_mod16, n, avail, res, torch.cuda.current_stream())
    torch.cuda.synchronize()
    out = res.cpu().numpy()
    assert (out[n * 16:] == 0xAB).all(), "kernel wrote past n records"
    return out[: n * 16].view(pa.RESULT_DTYPE).copy()


def _first_diff(got, exp):
    bad = np.nonzero(got != exp)[0]
    return f"{len(bad)} records differ; first #{bad[0]}: gpu={got[bad[0]]} expected={exp[bad[0]]}" if len(bad) else ""


@pytest.mark.parametrize("prefix", [0, 14, 4])
def test_efvi_event_ring_wraps_and_skips_discards(torch_cuda, ctx, prefix):
    """Ring of 4096 2-KiB RecvBuf slots, frame at 10 + prefix (Core.h:140-145, 505); an
    event run from slot 3000 wrapping to 1903 with 5 % discards."""
    R, stride = 4096, 2048
    off = 10 + prefix
    p = pa.rx.GenParams.for_config(5)
    t = pa.gen_conn_table(p)
    ctx.set_conn_table(t)
    slots = pa.gen_frames(p, R, stride, off)
    ref, frames = _strided(torch_cuda, ctx, slots, stride, off, R)
    rng = np.random.default_rng(prefix + 1)
    ids = (3000 + np.arange(3000)) % R
    ids = ids[rng.random(len(ids)) >= 0.05]
    got = _indexed(torch_cuda, ctx, frames, ids.astype(np.uint64) * stride + off, off % 16, stride - off)
    assert np.array_equal(got, ref[ids]), _first_diff(got, ref[ids])


def test_shuffled_jumbo_slots(torch_cuda, ctx):
    """C3 frames in 16-KiB slots (jumbo tot_len up to the slot), visited in a random
    order: per-frame stream descriptors and the KiB loop past 2 KiB."""
    R, stride, off = 8192, 16384, 2
    p = pa.rx.GenParams.for_config(3)
    t = pa.gen_conn_table(p)
    ctx.set_conn_table(t)
    slots = pa.gen_frames(p, R, stride, off)
    ref, frames = _strided(torch_cuda, ctx, slots, stride, off, R)
    ids = np.random.default_rng(7).permutation(R)
    got = _indexed(torch_cuda, ctx, frames, ids.astype(np.uint64) * stride + off, off, stride - off)
    assert np.array_equal(got, ref[ids]), _first_diff(got, ref[ids])
    tot = (slots[:, off + 16].astype(int) << 8) | slots[:, off + 17]
    assert (tot > 2048).any(), "workload should contain jumbo frames"


@pytest.mark.parametrize("eth_mod16", [2, 0, 6, 14])
def test_packed_layout_vs_oracle(torch_cuda, ctx, eth_mod16):
    """Frames packed back to back (each at the next 16-B boundary + eth_mod16), the
    readable extent running into the following frames: GPU == oracle on the same bytes."""
    n, avail = 3000, 1600
    p = pa.rx.GenParams.for_config(3)
    t = pa.gen_conn_table(p)
    e, m = t.snapshot()
    ctx.set_conn_table(t)
    src = pa.gen_frames(p, n, 2048, 2)
    tot = (src[:, 18].astype(np.int64) << 8) | src[:, 19]
    flen = 14 + tot
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
    base = torch_cuda.from_numpy(buf).cuda()
    got = _indexed(torch_cuda, ctx, base, offs, eth_mod16, avail)
    exp = np.empty(n, dtype=pa.RESULT_DTYPE)
    for i in range(n):
        o = int(offs[i])
        exp[i] = orc.classify_frame(buf[o:o + avail].tobytes(), avail, e, m, t.max_conn_cnt)
    assert np.array_equal(got, exp), _first_diff(got, exp)


def test_cooperative_window_eligibility(torch_cuda, ctx):
    """The indexed kernel loads each frame's 128-B window block (from the 16-B chunk before
    the IP header's) cooperatively when every frame of a wave has that block 16-B aligned
    inside [base, eth + avail); otherwise that wave loads per-lane windows.  Waves with
    the block on the line grid, off it (line + 32), mixed, the ring base off the 128-B
    grid, and a first frame whose block starts at base: every record equals the oracle's."""
    R, stride, avail = 4096, 2048, 2048 - 18
    p = pa.rx.GenParams.for_config(5)
    t = pa.gen_conn_table(p)
    e, m = t.snapshot()
    ctx.set_conn_table(t)
    a = pa.gen_frames(p, R, stride, 2)
    b = pa.gen_frames(p, R, stride, 18, first_index=R)
    rng = np.random.default_rng(11)
    use_b = np.zeros(R, dtype=bool)
    use_b[64 * 16:] = rng.random(R - 64 * 16) < 0.3  # first 16 waves all eligible, the rest mixed
    use_b[64 * 40:64 * 41] = True                     # one wave all at line + 32
    slots = np.where(use_b[:, None], b, a)
    offs = np.arange(R, dtype=np.uint64) * stride + np.where(use_b, 18, 2).astype(np.uint64)
    exp = np.empty(R, dtype=pa.RESULT_DTYPE)
    flat = slots.reshape(-1)
    for i in range(R):
        o = int(offs[i])
        exp[i] = orc.classify_frame(flat[o:o + avail].tobytes(), avail, e, m, t.max_conn_cnt)
    dev = torch_cuda.from_numpy(np.concatenate([np.zeros(16, np.uint8), flat])).cuda()
    got = _indexed(torch_cuda, ctx, dev[16:], offs, 2, avail)  # base 16 B off the allocation's 128-B grid
    assert np.array_equal(got, exp), _first_diff(got, exp)
    got = _indexed(torch_cuda, ctx, torch_cuda.from_numpy(flat).cuda(), offs, 2, avail)
    assert np.array_equal(got, exp), _first_diff(got, exp)


def test_window_fallback_at_ring_start(torch_cuda, ctx):
    """eth_mod16 = 0 puts the IP header's chunk at eth + 14 - 14: frame 0 at base + 0 has no
    16 B before its window inside the ring, so its wave falls back to per-lane windows
    (bounds-checked at base); the other waves load cooperatively.  Records equal the
    oracle's and the strided kernel's."""
    R, stride = 2048, 2048
    p = pa.rx.GenParams.for_config(3)
    t = pa.gen_conn_table(p)
    e, m = t.snapshot()
    ctx.set_conn_table(t)
    slots = pa.gen_frames(p, R, stride, 0)
    offs = np.arange(R, dtype=np.uint64) * stride
    flat = slots.reshape(-1)
    exp = np.empty(R, dtype=pa.RESULT_DTYPE)
    for i in range(R):
        o = int(offs[i])
        exp[i] = orc.classify_frame(flat[o:o + stride].tobytes(), stride, e, m, t.max_conn_cnt)
    got = _indexed(torch_cuda, ctx, torch_cuda.from_numpy(flat).cuda(), offs, 0, stride)
    assert np.array_equal(got, exp), _first_diff(got, exp)
    ref, _ = _strided(torch_cuda, ctx, slots, stride, 0, R)
    assert np.array_equal(got, ref), _first_diff(got, ref)


def test_offsets_outside_the_class_get_badoff(torch_cuda, ctx):
    R, stride, off = 512, 2048, 2
    p = pa.rx.GenParams.for_config(2)
    t = pa.gen_conn_table(p)
    ctx.set_conn_table(t)
    slots = pa.gen_frames(p, R, stride, off)
    ref, frames = _strided(torch_cuda, ctx, slots, stride, off, R)
    offs = np.arange(R, dtype=np.uint64) * stride + off
    offs[::7] += 4  # wrong class
    got = _indexed(torch_cuda, ctx, frames, offs, off, stride - off - 4)
    bad = np.zeros(R, dtype=bool)
    bad[::7] = True
    assert (got["flags"][bad] == pa.F.BADOFF).all() and (got["conn_id"][bad] == 0xFFFFFFFF).all()
    assert (got["seq"][bad] == 0).all() and (got["payload_len"][bad] == 0).all()
    # the others are the frames' records at the smaller readable extent (no frame reaches it)
    assert np.array_equal(got[~bad], ref[~bad]), _first_diff(got[~bad], ref[~bad])


def test_zero_copy_pinned_ring_and_offsets(torch_cuda, ctx):
    """base, offsets and records all in pinned host memory: the kernel reads the ring
    over PCIe (a NIC-DMA'd, HIP-registered ring needs no copy)."""
    R, stride, off = 4096, 2048, 12
    p = pa.rx.GenParams.for_config(3)
    t = pa.gen_conn_table(p)
    ctx.set_conn_table(t)
    slots = pa.gen_frames(p, R, stride, off)
    ref, _ = _strided(torch_cuda, ctx, slots, stride, off, R)
    ring = torch_cuda.from_numpy(slots.reshape(-1)).pin_memory()
    ids = (1000 + np.arange(R - 10)) % R
    offs = torch_cuda.from_numpy((ids.astype(np.uint64) * stride + off).view(np.int64)).pin_memory()
    res = torch_cuda.empty(len(ids) * 16, dtype=torch_cuda.uint8).pin_memory()
    ctx.classify_indexed(ring, offs, off % 16, len(ids), stride - off, res, torch_cuda.cuda.current_stream())
    torch_cuda.cuda.synchronize()
    got = res.numpy().view(pa.RESULT_DTYPE)
    assert np.array_equal(got, ref[ids]), _first_diff(got, ref[ids])


def test_indexed_argument_errors(torch_cuda, ctx):
    p = pa.rx.GenParams.for_config(2)
    ctx.set_conn_table(pa.gen_conn_table(p))
    buf = torch_cuda.zeros(4096, dtype=torch_cuda.uint8, device="cuda")
    offs = torch_cuda.zeros(4, dtype=torch_cuda.int64, device="cuda")
    res = torch_cuda.zeros(64, dtype=torch_cuda.uint8, device="cuda")
    for mod, avail in ((3, 2000), (16, 2000), (2, 95), (2, 70000)):
        with pytest.raises(pa.PollnetError):
            ctx.classify_indexed(buf, offs, mod, 4, avail, res)
    ctx.classify_indexed(buf, offs, 2, 0, 2000, res)  # n = 0 is a no-op


@pytest.mark.parametrize("n", [5, 100, 20000, 70000])
def test_permuted_ring_every_wave_split(torch_cuda, ctx, n):
    """A permuted event run over a 2-KiB slot ring at sizes that give 8, 16 and 64 frames per
    wave (frames_per_wave in rx_kernel.hip): records in event order == the oracle's."""
    p = pa.rx.GenParams.for_config(5)
    t = pa.gen_conn_table(p)
    e, m = t.snapshot()
    ctx.set_conn_table(t)
    slots = pa.gen_frames(p, n, 2048, 2)
    perm = np.random.default_rng(n).permutation(n)
    base = torch_cuda.from_numpy(slots.reshape(-1)).cuda()
    got = _indexed(torch_cuda, ctx, base, perm.astype(np.uint64) * 2048 + 2, 2, 2046)
    exp = orc.classify_batch(np.ascontiguousarray(slots[perm]), 2048, 2, n, e, m, t.max_conn_cnt)
    assert np.array_equal(got, exp), _first_diff(got, exp)
