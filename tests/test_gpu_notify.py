"""pn_classify_notify / pn_tx_fill_notify: the launch stores a token to a pinned host word once
every record / field it writes is visible; records and frames equal the plain entry points'
and the oracle's (bit-exact).  Zero-copy layout (pinned slots and records), as GpuRx and the
drop-in server use it for small batches."""
import time

import numpy as np
import pytest

import pollnet_amd as pa
from oracle import pyoracle as orc

from frames import STRIDE

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


def pinned(torch, nbytes):
    return torch.zeros(nbytes, dtype=torch.uint8, pin_memory=True)


def wait_token(word_np, token, torch, timeout_s=10.0):
    t0 = time.time()
    while int(word_np[0]) != token:  # the acquire side: records are read only after this
        if time.time() - t0 > timeout_s:
            torch.cuda.synchronize()
            raise AssertionError(f"notify word {int(word_np[0])} never became {token}")
    return True


@pytest.mark.parametrize("frame_off", [2, 0, 18])
@pytest.mark.parametrize("n", [1, 63, 64, 500, 1024])
def test_classify_notify_records_and_word(torch_cuda, frame_off, n):
    torch = torch_cuda
    p = pa.rx.GenParams.for_config(5)
    t = pa.gen_conn_table(p)
    e, m = t.snapshot()
    s = pa.gen_frames(p, n, STRIDE, frame_off, first_index=977)
    exp = orc.classify_batch(s, STRIDE, frame_off, n, e, m, t.max_conn_cnt, threads=8)
    ctx = pa.RxContext(0)
    ctx.set_conn_table(t)
    slots = pinned(torch, n * STRIDE)
    slots.numpy()[:] = s.reshape(-1)
    rec = pinned(torch, n * 16)
    word = torch.zeros(16, dtype=torch.int32, pin_memory=True)
    wnp = word.numpy()
    st = torch.cuda.Stream()
    for tok in (7, 8, 9):  # the counter behind the word is reused launch after launch
        rec.zero_()
        ctx.classify_notify(slots, STRIDE, frame_off, n, rec, word, tok, st)
        wait_token(wnp, tok, torch)
        got = rec.numpy().view(pa.RESULT_DTYPE).copy()
        assert np.array_equal(got, exp), f"token {tok}: {np.count_nonzero(got != exp)} records differ"
    st.synchronize()
    ctx.close()


def test_notify_limits(torch_cuda):
    torch = torch_cuda
    ctx = pa.RxContext(0)
    ctx.set_conn_table(pa.gen_conn_table(pa.rx.GenParams.for_config(2)))
    n = pa.rx.PN_NOTIFY_MAX_FRAMES + 1
    slots = pinned(torch, n * STRIDE)
    rec = pinned(torch, n * 16)
    word = torch.zeros(16, dtype=torch.int32, pin_memory=True)
    with pytest.raises(pa.PollnetError, match="PN_NOTIFY_MAX_FRAMES"):
        ctx.classify_notify(slots, STRIDE, 2, n, rec, word, 1)
    with pytest.raises(pa.PollnetError, match="PN_NOTIFY_MAX_FRAMES"):
        ctx.classify_notify(slots, STRIDE, 2, 0, rec, word, 1)
    with pytest.raises(pa.PollnetError, match="PN_NOTIFY_MAX_FRAMES"):
        ctx.tx_fill_notify(slots, STRIDE, 2, n, word, 1)
    ctx.close()


@pytest.mark.parametrize("frame_off,mode", [(14, pa.rx.PN_TX_TCP), (2, pa.rx.PN_TX_TCP), (2, pa.rx.PN_TX_UDP_EFVI)])
def test_tx_fill_notify_equals_tx_fill(torch_cuda, frame_off, mode):
    torch = torch_cuda
    n = 1000
    rng = np.random.default_rng(frame_off * 10 + mode)
    s = pa.gen_frames(pa.rx.GenParams.for_config(3), n, STRIDE, frame_off)
    # scramble both checksum fields so the fill has to write them
    ip = frame_off + 14
    s[:, ip + 10:ip + 12] = rng.integers(0, 256, (n, 2), dtype=np.uint8)
    s[:, ip + 36:ip + 38] = rng.integers(0, 256, (n, 2), dtype=np.uint8)
    ctx = pa.RxContext(0)
    a = torch.from_numpy(s.reshape(-1).copy()).cuda()
    ctx.tx_fill(a, STRIDE, frame_off, n, None, mode)
    torch.cuda.synchronize()
    b = pinned(torch, n * STRIDE)
    word = torch.zeros(16, dtype=torch.int32, pin_memory=True)
    wnp = word.numpy()
    for tok in (11, 12):
        b.numpy()[:] = s.reshape(-1)
        ctx.tx_fill_notify(b, STRIDE, frame_off, n, word, tok, mode=mode)
        wait_token(wnp, tok, torch)
        assert np.array_equal(b.numpy(), a.cpu().numpy()), f"token {tok}: filled frames differ"
    torch.cuda.synchronize()
    ctx.close()


def test_notify_kinds_on_several_streams(torch_cuda):
    """Classify and TX notifies in flight together on two streams (one counter per kind), then
    a classify notify on a third stream (its counter's previous stream is waited for)."""
    torch = torch_cuda
    p = pa.rx.GenParams.for_config(4)
    t = pa.gen_conn_table(p)
    e, m = t.snapshot()
    n = 1024
    s = pa.gen_frames(p, n, STRIDE, 2)
    exp = orc.classify_batch(s, STRIDE, 2, n, e, m, t.max_conn_cnt, threads=8)
    ctx = pa.RxContext(0)
    ctx.set_conn_table(t)
    slots = pinned(torch, n * STRIDE)
    slots.numpy()[:] = s.reshape(-1)
    txf = pinned(torch, n * STRIDE)
    txf.numpy()[:] = s.reshape(-1)
    ref_tx = torch.from_numpy(s.reshape(-1).copy()).cuda()  # C4 corrupts 1 frame in 1024: the fill rewrites it
    ctx.tx_fill(ref_tx, STRIDE, 2, n)
    exp_tx = ref_tx.cpu().numpy()
    rec = pinned(torch, n * 16)
    words = torch.zeros(64, dtype=torch.int32, pin_memory=True)
    wnp = words.numpy()
    s1, s2, s3 = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    for rnd in range(4):
        rec.zero_()
        ctx.classify_notify(slots, STRIDE, 2, n, rec, words[0:], 100 + rnd, s1 if rnd % 2 == 0 else s3)
        ctx.tx_fill_notify(txf, STRIDE, 2, n, words[16:], 200 + rnd, stream=s2)
        wait_token(wnp[0:], 100 + rnd, torch)
        wait_token(wnp[16:], 200 + rnd, torch)
        assert np.array_equal(rec.numpy().view(pa.RESULT_DTYPE), exp)
        assert np.array_equal(txf.numpy(), exp_tx)
    torch.cuda.synchronize()
    ctx.close()
