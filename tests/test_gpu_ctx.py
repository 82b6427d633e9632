"""pn_ctx stream semantics (include/pollnet_amd.h): pn_set_conn_table never waits
for the device or for streams it did not launch on, a launch already queued keeps the table
snapshot it was issued against (double-buffered table), the TX scratch and notify counters are
ordered across streams on the device, and pn_sync waits for every stream the ctx used.

"Unrelated work in flight" is a one-lane kernel that holds a stream until the host releases it
(pn_test_spin_wait, tuning library, no ctx; it always exits after its time limit)."""
import time

import numpy as np
import pytest

import pollnet_amd as pa
from oracle import pyoracle as orc

from frames import FRAME_OFF, STRIDE

pytestmark = pytest.mark.gpu

SPIN_MS = 4000  # the spin kernel's own limit: a stuck test ends, and says so, after 4 s


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


class Spin:
    """A spin kernel on `stream`; release() lets it finish; done() is 0 while it runs."""

    def __init__(self, torch, stream):
        from pollnet_amd import tuning as tn

        self.torch = torch
        self.go = torch.zeros(16, dtype=torch.int32, pin_memory=True)
        self.fin = torch.zeros(16, dtype=torch.int32, pin_memory=True)
        self.stream = stream
        tn.spin_wait(self.go, self.fin, SPIN_MS, stream)
        time.sleep(0.02)  # let it start

    def done(self):
        return int(self.fin.numpy()[0])

    def release(self):
        self.go.numpy()[0] = 1
        self.stream.synchronize()
        return self.done()


def tables(cfg=3):
    p = pa.rx.GenParams.for_config(cfg)
    t = pa.gen_conn_table(p)
    e, m = t.snapshot()
    empty = np.zeros(len(e), pa.ENTRY_DTYPE)
    empty["key"] = pa.PN_EMPTY_KEY  # every frame would miss
    return p, t, e, m, empty


def test_set_conn_table_does_not_wait_for_a_foreign_stream(torch_cuda):
    """A stream the ctx never launched on holds a kernel waiting for host input: replacing the table
    (three times, with classify launches between) returns at once — the old hipDeviceSynchronize
    would have waited for that kernel (a deadlock had the host only released it afterwards)."""
    torch = torch_cuda
    p, t, e, m, empty = tables()
    n = 4096
    s = pa.gen_frames(p, n)
    exp = orc.classify_batch(s, STRIDE, FRAME_OFF, n, e, m, t.max_conn_cnt, threads=8)
    c = pa.RxContext(0)
    c.set_conn_entries(e, m, t.max_conn_cnt)
    frames = torch.from_numpy(s.reshape(-1)).cuda()
    res = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
    mine, foreign = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    spin = Spin(torch, foreign)
    try:
        lat = []
        for tbl in (empty, e, empty, e):
            c.classify(frames, STRIDE, FRAME_OFF, n, res, mine)
            t0 = time.perf_counter()
            c.set_conn_entries(tbl, m, t.max_conn_cnt)
            lat.append(time.perf_counter() - t0)
        c.classify(frames, STRIDE, FRAME_OFF, n, res, mine)  # against e, the last table set
        mine.synchronize()
        still_running = spin.done() == 0
    finally:
        released = spin.release()
    assert still_running, "the foreign kernel ended before the sets returned (timed out?)"
    assert max(lat) < 0.5, f"pn_set_conn_table waited: {lat}"
    assert released == 1  # released by the host, not by its time limit
    got = res.cpu().numpy().view(pa.RESULT_DTYPE)
    assert np.array_equal(got, exp)
    c.close()


def test_queued_launch_keeps_its_snapshot(torch_cuda):
    """classify queued behind a held stream, then the table replaced (returns at once), then a
    classify on another stream that runs immediately: the queued launch — which runs only after
    the host releases its stream, i.e. after the replacement — still sees the table it was issued
    against, the later one the new table; pn_sync then waits for both streams."""
    torch = torch_cuda
    p, t, e, m, empty = tables(5)
    n = 8192
    s = pa.gen_frames(p, n, first_index=123)
    exp_e = orc.classify_batch(s, STRIDE, FRAME_OFF, n, e, m, t.max_conn_cnt, threads=8)
    exp_empty = orc.classify_batch(s, STRIDE, FRAME_OFF, n, empty, m, t.max_conn_cnt, threads=8)
    assert not np.array_equal(exp_e, exp_empty)
    c = pa.RxContext(0)
    c.set_conn_entries(e, m, t.max_conn_cnt)
    frames = torch.from_numpy(s.reshape(-1)).cuda()
    r_queued = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    r_now = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    held, other = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    spin = Spin(torch, held)
    try:
        c.classify(frames, STRIDE, FRAME_OFF, n, r_queued, held)  # queued behind the spin
        t0 = time.perf_counter()
        c.set_conn_entries(empty, m, t.max_conn_cnt)
        lat = time.perf_counter() - t0
        c.classify(frames, STRIDE, FRAME_OFF, n, r_now, other)
        other.synchronize()
        queued_pending = spin.done() == 0
        now = r_now.cpu().numpy().view(pa.RESULT_DTYPE).copy()
    finally:
        spin.release()
    c.sync()
    assert queued_pending and lat < 0.5, lat
    assert np.array_equal(now, exp_empty)
    assert np.array_equal(r_queued.cpu().numpy().view(pa.RESULT_DTYPE), exp_e)
    # the next replacement waits (by event) for that queued launch, which is done now
    t0 = time.perf_counter()
    c.set_conn_entries(e, m, t.max_conn_cnt)
    assert time.perf_counter() - t0 < 0.5
    c.close()


def test_sync_waits_for_every_stream(torch_cuda):
    """pn_sync covers all the streams the ctx launched on (it used to wait for the last one only)."""
    torch = torch_cuda
    p, t, e, m, _ = tables(2)
    n = 4096
    s = pa.gen_frames(p, n)
    exp = orc.classify_batch(s, STRIDE, FRAME_OFF, n, e, m, t.max_conn_cnt, threads=8)
    c = pa.RxContext(0)
    c.set_conn_entries(e, m, t.max_conn_cnt)
    frames = torch.from_numpy(s.reshape(-1)).cuda()
    ra = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    rb = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    spin = Spin(torch, sa)
    c.classify(frames, STRIDE, FRAME_OFF, n, ra, sa)  # behind the spin
    c.classify(frames, STRIDE, FRAME_OFF, n, rb, sb)  # the ctx's last stream
    sb.synchronize()
    spin.go.numpy()[0] = 1  # release from the host, then pn_sync must wait for sa as well
    c.sync()
    assert np.array_equal(ra.cpu().numpy().view(pa.RESULT_DTYPE), exp)
    assert np.array_equal(rb.cpu().numpy().view(pa.RESULT_DTYPE), exp)
    assert spin.done() == 1
    c.close()


def test_tx_scratch_across_streams(torch_cuda):
    """Two-launch TX fills (> 65,536 frames use ctx scratch) on a stream, small fills on others, the
    first stream dropped, then a large fill on a new stream queued behind a held one and another on a
    third: every frame equals the oracle's fill (the scratch user on the new stream is ordered after
    the previous one on the device)."""
    torch = torch_cuda
    n = 70000
    p = pa.rx.GenParams.for_config(3)
    base = pa.gen_frames(p, n, first_index=5)
    exp = base.copy()
    orc.tx_fill_batch(exp, STRIDE, FRAME_OFF, n, None, orc.TX_TCP)
    c = pa.RxContext(0)

    def scrambled():
        v = base.copy()
        v[:, FRAME_OFF + 24:FRAME_OFF + 26] = 0x5A
        v[:, FRAME_OFF + 50:FRAME_OFF + 52] = 0xA5
        return torch.from_numpy(v.reshape(-1)).cuda()

    a, b, small = scrambled(), scrambled(), scrambled()
    torch.cuda.synchronize()
    s1 = torch.cuda.Stream()
    c.tx_fill(a, STRIDE, FRAME_OFF, n, stream=s1)
    del s1  # the binding keeps it alive until the next set / sync, as the C-ABI contract asks
    s_small = torch.cuda.Stream()
    for k in range(3):
        c.tx_fill(small[k * 4096 * STRIDE:], STRIDE, FRAME_OFF, 4096, stream=s_small)
    held, s3 = torch.cuda.Stream(), torch.cuda.Stream()
    spin = Spin(torch, held)
    try:
        c.tx_fill(b, STRIDE, FRAME_OFF, n, stream=held)  # queued: uses the scratch later
        c.tx_fill(a, STRIDE, FRAME_OFF, n, stream=s3)  # must wait (on the device) for the queued one
        time.sleep(0.05)
        ordered = s3.query() is False  # s3's fill has not run: it waits for the held stream's
    finally:
        spin.release()
    c.sync()
    assert ordered
    for buf in (a, b):
        assert np.array_equal(buf.cpu().numpy().reshape(n, STRIDE), exp)
    got_small = small.cpu().numpy().reshape(n, STRIDE)[: 3 * 4096]
    assert np.array_equal(got_small, exp[: 3 * 4096])
    c.close()


def test_notify_counters_zeroed_before_either_kind(torch_cuda):
    """The notify counters are zeroed on the stream of the ctx's first notify launch.  A first
    launch of the OTHER kind on another stream must wait for that zeroing: with the first
    classify_notify queued behind a spin, a tx_fill_notify on a free stream does not complete until
    the spin is released; then both words arrive, and again on a repeat of both."""
    torch = torch_cuda
    p = pa.rx.GenParams.for_config(3)
    t = pa.gen_conn_table(p)
    e, m = t.snapshot()
    n = 512
    s = pa.gen_frames(p, n, STRIDE, FRAME_OFF)
    exp = orc.classify_batch(s, STRIDE, FRAME_OFF, n, e, m, t.max_conn_cnt, threads=8)
    ref_tx = torch.from_numpy(s.reshape(-1).copy()).cuda()
    c0 = pa.RxContext(0)
    c0.tx_fill(ref_tx, STRIDE, FRAME_OFF, n)
    torch.cuda.synchronize()
    c0.close()
    exp_tx = ref_tx.cpu().numpy()
    c = pa.RxContext(0)
    c.set_conn_table(t)
    slots = torch.zeros(n * STRIDE, dtype=torch.uint8, pin_memory=True)
    slots.numpy()[:] = s.reshape(-1)
    txf = torch.zeros(n * STRIDE, dtype=torch.uint8, pin_memory=True)
    rec = torch.zeros(n * 16, dtype=torch.uint8, pin_memory=True)
    words = torch.zeros(64, dtype=torch.int32, pin_memory=True)
    wnp = words.numpy()
    held, free = torch.cuda.Stream(), torch.cuda.Stream()
    spin = Spin(torch, held)
    try:
        txf.numpy()[:] = s.reshape(-1)
        c.classify_notify(slots, STRIDE, FRAME_OFF, n, rec, words[0:], 5, held)   # first notify: zeroing on held
        c.tx_fill_notify(txf, STRIDE, FRAME_OFF, n, words[16:], 6, stream=free)  # other kind, other stream
        time.sleep(0.1)
        tx_waited = int(wnp[16]) == 0 and spin.done() == 0
    finally:
        spin.release()
    assert tx_waited, "tx_fill_notify ran before the counters were zeroed"
    for rnd in range(2):
        tok_c, tok_t = 5 + 10 * rnd, 6 + 10 * rnd
        if rnd:
            rec.zero_()
            txf.numpy()[:] = s.reshape(-1)
            c.classify_notify(slots, STRIDE, FRAME_OFF, n, rec, words[0:], tok_c, held)
            c.tx_fill_notify(txf, STRIDE, FRAME_OFF, n, words[16:], tok_t, stream=free)
        t0 = time.time()
        while int(wnp[0]) != tok_c or int(wnp[16]) != tok_t:
            assert time.time() - t0 < 10, f"round {rnd}: words {int(wnp[0])}, {int(wnp[16])}"
        assert np.array_equal(rec.numpy().view(pa.RESULT_DTYPE), exp)
        assert np.array_equal(txf.numpy(), exp_tx)
    torch.cuda.synchronize()
    c.close()
