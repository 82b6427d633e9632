"""GPU: the resident classify service (pn_service_*, pollnet_amd/csrc/rx_service.hip): one launch, batches posted
through pinned host memory.  Every post's records must equal the oracle's (and, on the release path, the records
pn_set_verify(ctx, 0) writes): small and large posts (1 .. 70,000 frames: every wave count, the group loop), frames
and records in pinned host memory (zero copy) or device memory, two posts outstanding, a table change between
posts, the kernel ending by itself after idle_ms and the next post relaunching it, every alignment class of the
strided layout, and close.  Every wait inside the kernel has a wall-clock limit (it always ends)."""
import time

import numpy as np
import pytest

import pollnet_amd as pa
from oracle import pyoracle as orc

from frames import FRAME_OFF, STRIDE

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t

    assert t.cuda.is_available(), "GPU tests need an MI355X"
    return t


def _frames(cfg, n, first=0, off=FRAME_OFF, stride=STRIDE):
    p = pa.rx.GenParams.for_config(cfg)
    s = np.ascontiguousarray(pa.gen_frames(p, n, stride, off, first_index=first, threads=8))
    return p, s


def _expected(s, n, table, off=FRAME_OFF, stride=STRIDE, verify=True):
    e, m = table.snapshot()
    return orc.classify_batch(s, stride, off, n, e, m, table.max_conn_cnt, threads=8, unverified=not verify)


def _pinned(torch, arr):
    return torch.from_numpy(np.ascontiguousarray(arr).reshape(-1)).pin_memory()


@pytest.mark.parametrize("cfg", [3, 5])
def test_service_posts_equal_oracle_zero_copy(torch, cfg):
    p, s = _frames(cfg, 70000)
    table = pa.gen_conn_table(p)
    ctx = pa.RxContext(0)
    try:
        ctx.set_conn_table(table)
        svc = pa.RxService(ctx, STRIDE, FRAME_OFF)
        try:
            host = _pinned(torch, s)
            res = torch.zeros(70000 * 16, dtype=torch.uint8).pin_memory()
            exp_all = _expected(s, 70000, table)
            unv_all = _expected(s, 70000, table, verify=False)
            for n in (1, 7, 64, 65, 511, 512, 513, 4096, 4097, 70000):
                for verify in (True, False):
                    ctx.set_verify(verify)
                    res.zero_()
                    svc.classify(host, n, res)
                    got = res.numpy()[: n * 16].view(pa.RESULT_DTYPE)
                    exp = (exp_all if verify else unv_all)[:n]
                    assert np.array_equal(got, exp), (n, verify, np.nonzero(got != exp)[0][:5])
                    assert not res.numpy()[n * 16:].any(), "records written past n"
        finally:
            svc.close()
    finally:
        ctx.close()


def test_service_device_memory_and_two_outstanding(torch):
    p, s = _frames(2, 8192)
    table = pa.gen_conn_table(p)
    exp = _expected(s, 8192, table)
    ctx = pa.RxContext(0)
    try:
        ctx.set_conn_table(table)
        svc = pa.RxService(ctx, STRIDE, FRAME_OFF)
        try:
            dev = torch.from_numpy(s.reshape(-1)).cuda()
            r = [torch.zeros(4096 * 16, dtype=torch.uint8, device="cuda") for _ in range(2)]
            # two posts in flight: the halves of the batch, then wait for the second (posts complete in order)
            a = svc.post(dev, 4096, r[0])
            b = svc.post(dev[4096 * STRIDE:], 4096, r[1])
            assert b == a + 1
            svc.wait(a)
            assert np.array_equal(r[0].cpu().numpy().view(pa.RESULT_DTYPE), exp[:4096])
            svc.wait(b)
            got = np.concatenate([x.cpu().numpy() for x in r]).view(pa.RESULT_DTYPE)
            assert np.array_equal(got, exp)
            # 200 back-to-back posts, alternating halves
            for k in range(200):
                svc.post(dev[(k & 1) * 4096 * STRIDE:], 4096, r[k & 1])
                if k & 1:
                    svc.wait()
            svc.wait()
            got = np.concatenate([x.cpu().numpy() for x in r]).view(pa.RESULT_DTYPE)
            assert np.array_equal(got, exp)
        finally:
            svc.close()
    finally:
        ctx.close()


def test_service_table_change_and_idle_relaunch(torch):
    p, s = _frames(3, 2048)
    table = pa.gen_conn_table(p)
    ctx = pa.RxContext(0)
    try:
        ctx.set_conn_table(table)
        svc = pa.RxService(ctx, STRIDE, FRAME_OFF, idle_ms=5)
        try:
            host = _pinned(torch, s)
            res = torch.zeros(2048 * 16, dtype=torch.uint8).pin_memory()
            svc.classify(host, 2048, res)
            assert np.array_equal(res.numpy().view(pa.RESULT_DTYPE), _expected(s, 2048, table))
            # a table change between posts: every frame of the flow of frame 0 now misses
            key = int(pa.conn_hash_key(int(s[0, FRAME_OFF + 26:FRAME_OFF + 30].view("<u4")[0]),
                                       int(s[0, FRAME_OFF + 34:FRAME_OFF + 36].view("<u2")[0])))
            table.delete(key)
            ctx.set_conn_table(table)
            svc.classify(host, 2048, res)
            exp = _expected(s, 2048, table)
            assert np.array_equal(res.numpy().view(pa.RESULT_DTYPE), exp)
            assert (exp["conn_id"] == pa.PN_MISS).sum() > 0
            # idle: the kernel ends by itself after 5 ms; the next posts relaunch it
            for _ in range(3):
                time.sleep(0.03)
                res.zero_()
                svc.classify(host, 2048, res)
                assert np.array_equal(res.numpy().view(pa.RESULT_DTYPE), exp)
        finally:
            svc.close()
    finally:
        ctx.close()


@pytest.mark.parametrize("off", [0, 2, 6, 10, 14, 18])
def test_service_alignment_classes(torch, off):
    stride = 2048 if off != 18 else 1664
    p, s = _frames(5, 3000, off=off, stride=stride)
    table = pa.gen_conn_table(p)
    ctx = pa.RxContext(0)
    try:
        ctx.set_conn_table(table)
        svc = pa.RxService(ctx, stride, off)
        try:
            host = _pinned(torch, s)
            res = torch.zeros(3000 * 16, dtype=torch.uint8).pin_memory()
            svc.classify(host, 3000, res)
            assert np.array_equal(res.numpy().view(pa.RESULT_DTYPE), _expected(s, 3000, table, off=off, stride=stride))
        finally:
            svc.close()
    finally:
        ctx.close()


def test_service_argument_checks(torch):
    ctx = pa.RxContext(0)
    try:
        with pytest.raises(pa.PollnetError, match="idle_ms"):
            pa.RxService(ctx, STRIDE, FRAME_OFF, idle_ms=0)
        with pytest.raises(pa.PollnetError, match="layout"):
            pa.RxService(ctx, 100, FRAME_OFF)
        svc = pa.RxService(ctx, STRIDE, FRAME_OFF)
        try:
            buf = torch.zeros(STRIDE, dtype=torch.uint8).pin_memory()
            with pytest.raises(pa.PollnetError, match="conn table"):
                svc.post(buf, 1, buf)
        finally:
            svc.close()
    finally:
        ctx.close()


def test_service_soak_random_posts_and_relaunches(torch):
    """1,500 posts of random size (1 .. 4,096 frames) at random offsets into one pinned ring, verified or release
    path at random (switched with posts in flight: each post carries the setting at its post), one or two outstanding, with idle gaps longer than idle_ms (2 ms) between some of them so the
    kernel ends and is relaunched many times, some posts landing while it ends.  Every post's records equal the
    oracle's, and every launch ended by itself or at close."""
    rng = np.random.default_rng(0x50A4)
    N = 16384
    p, s = _frames(3, N)
    table = pa.gen_conn_table(p)
    exp = {True: _expected(s, N, table), False: _expected(s, N, table, verify=False)}
    ctx = pa.RxContext(0)
    try:
        ctx.set_conn_table(table)
        svc = pa.RxService(ctx, STRIDE, FRAME_OFF, idle_ms=2)
        try:
            host = _pinned(torch, s)
            outs = [torch.zeros(4096 * 16, dtype=torch.uint8).pin_memory() for _ in range(2)]
            pending = []  # (post id, out index, first frame, n, verify)

            def check(item):
                pid, o, first, n, verify = item
                svc.wait(pid)
                got = outs[o].numpy()[: n * 16].view(pa.RESULT_DTYPE)
                assert np.array_equal(got, exp[verify][first:first + n]), (pid, first, n, verify)

            relaunch_gaps = 0
            for k in range(1500):
                if len(pending) == 2 or (pending and rng.random() < 0.5):
                    check(pending.pop(0))
                verify = bool(rng.random() < 0.5)
                ctx.set_verify(verify)  # each post carries the setting at its post, posts in flight included
                n = int(rng.integers(1, 4097))
                first = int(rng.integers(0, N - n + 1))
                o = k & 1
                if pending and pending[0][1] == o:
                    check(pending.pop(0))
                pid = svc.post(host[first * STRIDE:], n, outs[o])
                pending.append((pid, o, first, n, verify))
                if rng.random() < 0.04:  # longer than idle_ms: the kernel ends before or while the next post arrives
                    time.sleep(float(rng.uniform(0.001, 0.006)))
                    relaunch_gaps += 1
            while pending:
                check(pending.pop(0))
            assert relaunch_gaps > 20
        finally:
            svc.close()
    finally:
        ctx.close()


def test_service_table_change_with_a_post_in_flight(torch):
    """pn_set_conn_table with one post outstanding (allowed: the table is double-buffered): the post in flight is
    classified against the table it was posted with, the next post against the new one."""
    p, s = _frames(3, 4096)
    table = pa.gen_conn_table(p)
    ctx = pa.RxContext(0)
    try:
        ctx.set_conn_table(table)
        svc = pa.RxService(ctx, STRIDE, FRAME_OFF)
        try:
            host = _pinned(torch, s)
            r = [torch.zeros(4096 * 16, dtype=torch.uint8).pin_memory() for _ in range(2)]
            exp_old = _expected(s, 4096, table)
            for _ in range(20):  # repeated, so some of the changes land while the first post is still running
                old = svc.post(host, 4096, r[0])
                key = int(pa.conn_hash_key(int(s[0, FRAME_OFF + 26:FRAME_OFF + 30].view("<u4")[0]),
                                           int(s[0, FRAME_OFF + 34:FRAME_OFF + 36].view("<u2")[0])))
                t2 = pa.gen_conn_table(p)
                t2.delete(key)
                ctx.set_conn_table(t2)
                new = svc.post(host, 4096, r[1])
                svc.wait(old)
                svc.wait(new)
                assert np.array_equal(r[0].numpy().view(pa.RESULT_DTYPE), exp_old)
                exp_new = _expected(s, 4096, t2)
                assert np.array_equal(r[1].numpy().view(pa.RESULT_DTYPE), exp_new)
                assert not np.array_equal(exp_new, exp_old)
                ctx.set_conn_table(table)
        finally:
            svc.close()
    finally:
        ctx.close()


@pytest.mark.parametrize("cfg", [2, 3])
def test_service_max_post_equals_pn_classify(torch, cfg):
    """One post of PN_SERVICE_MAX_FRAMES (1 Mi) frames in device memory, both paths: its records equal pn_classify's
    on the same frames (the bench's full-size parity is pinned to the oracle through pn_classify)."""
    n = 1 << 20
    p = pa.rx.GenParams.for_config(cfg)
    host = np.empty((n, STRIDE), np.uint8)
    pa.gen_frames(p, n, STRIDE, FRAME_OFF, first_index=0, threads=16, out=host)
    ctx = pa.RxContext(0)
    try:
        ctx.set_conn_table(pa.gen_conn_table(p))
        dev = torch.from_numpy(host.reshape(-1)).cuda()
        del host
        a = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
        b = torch.empty_like(a)
        svc = pa.RxService(ctx, STRIDE, FRAME_OFF)
        try:
            for verify in (True, False):
                ctx.set_verify(verify)
                a.fill_(0x5A)
                b.fill_(0xA5)
                ctx.classify(dev, STRIDE, FRAME_OFF, n, a, torch.cuda.current_stream())
                torch.cuda.synchronize()
                svc.classify(dev, n, b)
                assert torch.equal(a, b), verify
        finally:
            svc.close()
    finally:
        ctx.close()


# ---- round 6: the conn-table contract with posts outstanding, the post limit, large posts ----

@pytest.fixture(scope="module")
def big(torch):
    """1 Mi C3 frames in pinned host memory (zero copy: a verified post of them runs for tens of ms over PCIe)."""
    n = 1 << 20
    p = pa.rx.GenParams.for_config(3)
    host = _pinned(torch, np.zeros((n, STRIDE), np.uint8))
    pa.gen_frames(p, n, STRIDE, FRAME_OFF, first_index=0, threads=16, out=host.numpy().reshape(n, STRIDE))
    return p, host, n


def _flow_key(s, i):
    return int(pa.conn_hash_key(int(s[i, FRAME_OFF + 26:FRAME_OFF + 30].view("<u4")[0]),
                                int(s[i, FRAME_OFF + 34:FRAME_OFF + 36].view("<u2")[0])))


def test_service_table_changes_during_a_large_post(torch, big):
    """pn_set_conn_table during outstanding 1-Mi posts: two changes during one post (the second lands on the buffer
    the post reads: it waits for the post), then three changes during two posts, the last one growing n_entries (a
    new, larger buffer: the old one is freed only once the post reading it is done).  Every post's records equal the
    oracle's under the table it was posted with (rx_service.hip svc_release_table; Core.h:178-182, 558-682)."""
    p, host, n = big
    s = host.numpy().reshape(n, STRIDE)
    t0 = pa.gen_conn_table(p)
    tables = [t0]
    for i in (0, 1, 2):  # each drops a different flow: every change is visible throughout the batch
        t = pa.gen_conn_table(p, max_tw_cnt=4 * p.max_conn_cnt) if i == 2 else pa.gen_conn_table(p)
        t.delete(_flow_key(s, 1 + 7 * i))
        tables.append(t)
    assert len(tables[3].snapshot()[0]) > len(t0.snapshot()[0])  # the last change grows n_entries
    exp = {i: _expected(s, n, t) for i, t in enumerate(tables)}
    for i in range(1, 4):
        assert not np.array_equal(exp[i], exp[0])
    res = [torch.zeros(n * 16, dtype=torch.uint8).pin_memory() for _ in range(3)]
    got = lambda r: r.numpy().view(pa.RESULT_DTYPE)
    ctx = pa.RxContext(0)
    try:
        ctx.set_conn_table(t0)
        svc = pa.RxService(ctx, STRIDE, FRAME_OFF)
        try:
            # two changes during one post: T1 into the other buffer, T2 back into the post's own
            a = svc.post(host, n, res[0])
            ctx.set_conn_table(tables[1])
            ctx.set_conn_table(tables[2])
            b = svc.post(host, n, res[1])
            svc.wait(a)
            svc.wait(b)
            assert np.array_equal(got(res[0]), exp[0])
            assert np.array_equal(got(res[1]), exp[2])
            # three changes during two posts, the last one growing n_entries
            ctx.set_conn_table(t0)
            a = svc.post(host, n, res[0])           # T0
            ctx.set_conn_table(tables[1])
            b = svc.post(host, n, res[1])           # T1, two outstanding
            ctx.set_conn_table(tables[2])           # over T0's buffer: waits for a
            ctx.set_conn_table(tables[3])           # over T1's buffer, reallocated larger: waits for b
            svc.wait(a)
            c = svc.post(host, n, res[2])           # T3
            svc.wait(b)
            svc.wait(c)
            assert np.array_equal(got(res[0]), exp[0])
            assert np.array_equal(got(res[1]), exp[1])
            assert np.array_equal(got(res[2]), exp[3])
        finally:
            svc.close()
    finally:
        ctx.close()


def test_service_third_post_refused(torch, big):
    """At most two posts outstanding: with two verified 1-Mi posts from pinned host memory in flight (tens of ms of
    PCIe reads each) a third is refused at once, and the two complete with the oracle's records."""
    p, host, n = big
    s = host.numpy().reshape(n, STRIDE)
    table = pa.gen_conn_table(p)
    exp = _expected(s, n, table)
    res = [torch.zeros(n * 16, dtype=torch.uint8).pin_memory() for _ in range(3)]
    ctx = pa.RxContext(0)
    try:
        ctx.set_conn_table(table)
        svc = pa.RxService(ctx, STRIDE, FRAME_OFF)
        try:
            a = svc.post(host, n, res[0])
            b = svc.post(host, n, res[1])
            with pytest.raises(pa.PollnetError, match="two posts already outstanding"):
                svc.post(host, n, res[2])
            svc.wait(b)
            assert svc.wait(a) is None  # an id of a completed post returns at once
            for r in res[:2]:
                assert np.array_equal(r.numpy().view(pa.RESULT_DTYPE), exp)
            c = svc.post(host, 4096, res[2])  # both done: posting works again
            svc.wait(c)
            assert np.array_equal(res[2].numpy()[: 4096 * 16].view(pa.RESULT_DTYPE), exp[:4096])
        finally:
            svc.close()
    finally:
        ctx.close()


def test_service_large_post_late_in_the_idle_window(torch, big):
    """idle_ms = 1: a post arriving ~0.9 ms into the idle window that runs longer than the idle limit (a verified
    64 Ki-frame post from pinned host memory, ~2 ms) completes -- a post's limit runs from its acceptance, not from
    the last post -- and the next post after it completes too (the advisor's round-5 finding)."""
    p, host, n = big
    s = host.numpy().reshape(n, STRIDE)
    table = pa.gen_conn_table(p)
    m = 1 << 16
    exp = _expected(s[:m], m, table)
    res = torch.zeros(m * 16, dtype=torch.uint8).pin_memory()
    ctx = pa.RxContext(0)
    try:
        ctx.set_conn_table(table)
        svc = pa.RxService(ctx, STRIDE, FRAME_OFF, idle_ms=1)
        try:
            for rep in range(6):
                svc.classify(host, 64, res)  # the kernel is running, its idle timer just restarted
                t = time.perf_counter()
                while time.perf_counter() - t < 0.0009:
                    pass
                res.zero_()
                svc.classify(host, m, res)
                assert np.array_equal(res.numpy().view(pa.RESULT_DTYPE), exp), rep
                res.zero_()
                svc.classify(host, 4096, res)
                assert np.array_equal(res.numpy()[: 4096 * 16].view(pa.RESULT_DTYPE), exp[:4096]), rep
        finally:
            svc.close()
    finally:
        ctx.close()


@pytest.mark.parametrize("large_waves", [64, 96, 0])
def test_service_large_posts_with_helpers(torch, big, large_waves):
    """Posts above the latency tier's 4096 frames run on helper waves launched with them (pn_service_open_ex:
    large_waves 64 = the tier alone, 96 = 32 helpers, 0 = the default per-CU count): sizes around every boundary,
    both paths, device-resident and zero copy, two outstanding; records equal the oracle's."""
    p, host, n = big
    s = host.numpy().reshape(n, STRIDE)
    table = pa.gen_conn_table(p)
    m = 200_000
    exp = {True: _expected(s[:m], m, table), False: _expected(s[:m], m, table, verify=False)}
    dev = host[: m * STRIDE].cuda()
    outs = [torch.zeros(m * 16, dtype=torch.uint8).pin_memory() for _ in range(2)]
    ctx = pa.RxContext(0)
    try:
        ctx.set_conn_table(table)
        svc = pa.RxService(ctx, STRIDE, FRAME_OFF, large_waves=large_waves)
        try:
            k = 0
            for size in (4096, 4097, 4160, 4161, 8192, 65 * 64 * 33 + 5, 131072, m):
                for verify in (True, False):
                    for src in (host, dev):
                        ctx.set_verify(verify)
                        o = outs[k & 1]
                        o.zero_()
                        pid = svc.post(src, size, o)
                        svc.wait(pid)
                        got = o.numpy()[: size * 16].view(pa.RESULT_DTYPE)
                        assert np.array_equal(got, exp[verify][:size]), (size, verify, src.is_cuda)
                        assert not o.numpy()[size * 16:].any(), "records written past n"
                        k += 1
            # two large posts outstanding, then a small one behind them
            ctx.set_verify(True)
            a = svc.post(host, m, outs[0])
            b = svc.post(dev, m, outs[1])
            svc.wait(a)
            small = torch.zeros(64 * 16, dtype=torch.uint8).pin_memory()
            c = svc.post(host, 64, small)
            svc.wait(c)
            svc.wait(b)
            for o in outs:
                assert np.array_equal(o.numpy().view(pa.RESULT_DTYPE), exp[True])
            assert np.array_equal(small.numpy().view(pa.RESULT_DTYPE), exp[True][:64])
        finally:
            svc.close()
    finally:
        ctx.close()


def test_service_soak_large_posts_and_relaunches(torch, big):
    """300 posts of random size up to 40,000 frames (helpers above 4096) with idle gaps past idle_ms (2 ms), so
    launches end and are relaunched with large posts pending (their helpers relaunched with them): every post's
    records equal the oracle's."""
    rng = np.random.default_rng(0x6A11)
    p, host, n = big
    N = 1 << 17
    s = host.numpy().reshape(n, STRIDE)
    table = pa.gen_conn_table(p)
    exp = {True: _expected(s[:N], N, table), False: _expected(s[:N], N, table, verify=False)}
    ctx = pa.RxContext(0)
    try:
        ctx.set_conn_table(table)
        svc = pa.RxService(ctx, STRIDE, FRAME_OFF, idle_ms=2)
        try:
            outs = [torch.zeros(40000 * 16, dtype=torch.uint8).pin_memory() for _ in range(2)]
            pending = []

            def check(item):
                pid, o, first, size, verify = item
                svc.wait(pid)
                got = outs[o].numpy()[: size * 16].view(pa.RESULT_DTYPE)
                assert np.array_equal(got, exp[verify][first:first + size]), (pid, first, size, verify)

            gaps = 0
            for k in range(300):
                if len(pending) == 2 or (pending and rng.random() < 0.5):
                    check(pending.pop(0))
                verify = bool(rng.random() < 0.5)
                ctx.set_verify(verify)
                size = int(rng.integers(1, 40001)) if rng.random() < 0.7 else int(rng.integers(1, 4097))
                first = int(rng.integers(0, N - size + 1))
                o = k & 1
                if pending and pending[0][1] == o:
                    check(pending.pop(0))
                pid = svc.post(host[first * STRIDE:], size, outs[o])
                pending.append((pid, o, first, size, verify))
                if rng.random() < 0.1:
                    time.sleep(float(rng.uniform(0.001, 0.006)))
                    gaps += 1
            while pending:
                check(pending.pop(0))
            assert gaps > 10
        finally:
            svc.close()
    finally:
        ctx.close()


def test_service_post_ids_wrap(torch, big, monkeypatch):
    """The post counter wraps at 2^32 (11 hours of posts at 100k a second): a service started just below it
    (PN_SERVICE_FIRST_POST) takes posts 0xFFFFFFF1 .. 0x30 -- ids 0xFFFFFFFE and 0xFFFFFFFF (once the idle and stop
    marks' values) and 0 included -- of every kind: one wave, the latency tier, helper grids, two outstanding, and idle
    relaunches across the wrap.  Every post's records equal the oracle's."""
    p, host, n = big
    s = host.numpy().reshape(n, STRIDE)
    table = pa.gen_conn_table(p)
    m = 20000
    exp = _expected(s[:m], m, table)
    monkeypatch.setenv("PN_SERVICE_FIRST_POST", str(0xFFFFFFF0))
    outs = [torch.zeros(m * 16, dtype=torch.uint8).pin_memory() for _ in range(2)]
    ctx = pa.RxContext(0)
    try:
        ctx.set_conn_table(table)
        svc = pa.RxService(ctx, STRIDE, FRAME_OFF, idle_ms=2)
        try:
            sizes = [1, 64, 4096, m, 700]
            ids, pending = [], []
            for k in range(64):
                size = sizes[k % len(sizes)]
                o = k & 1
                if pending and pending[0][1] == o:
                    pid, oo, sz = pending.pop(0)
                    svc.wait(pid)
                    assert np.array_equal(outs[oo].numpy()[: sz * 16].view(pa.RESULT_DTYPE), exp[:sz]), (hex(pid), sz)
                outs[o].zero_()
                pid = svc.post(host, size, outs[o])
                ids.append(pid)
                pending.append((pid, o, size))
                if k % 7 == 3:  # past idle_ms: the kernel ends, the next post relaunches it
                    time.sleep(0.005)
            for pid, oo, sz in pending:
                svc.wait(pid)
                assert np.array_equal(outs[oo].numpy()[: sz * 16].view(pa.RESULT_DTYPE), exp[:sz]), (hex(pid), sz)
            assert ids[0] == 0xFFFFFFF1 and 0 in ids and 0xFFFFFFFF in ids and 0xFFFFFFFE in ids
            assert all(((b - a) & 0xFFFFFFFF) == 1 for a, b in zip(ids, ids[1:]))
        finally:
            svc.close()
    finally:
        ctx.close()


def test_service_host_mailbox_fallback(torch, big, monkeypatch):
    """Without a large BAR the mailbox is pinned host memory (PN_SERVICE_HOST_MAILBOX forces it here): the same
    protocol, the waves reading the mailbox over PCIe.  Posts of every kind -- one wave, the latency tier, helper
    grids, linked, two outstanding, idle relaunches -- give the oracle's records and links."""
    p, host, n = big
    s = host.numpy().reshape(n, STRIDE)
    table = pa.gen_conn_table(p)
    m = 20000
    exp = _expected(s[:m], m, table)
    links_exp = orc.chain_links(np.ascontiguousarray(s[:1000]), STRIDE, FRAME_OFF, 1000, exp[:1000], table.max_conn_cnt)
    monkeypatch.setenv("PN_SERVICE_HOST_MAILBOX", "1")
    outs = [torch.zeros(m * 16, dtype=torch.uint8).pin_memory() for _ in range(2)]
    lk = [torch.zeros(1024, dtype=torch.int16).pin_memory() for _ in range(2)]
    ctx = pa.RxContext(0)
    try:
        ctx.set_conn_table(table)
        svc = pa.RxService(ctx, STRIDE, FRAME_OFF, idle_ms=2)
        try:
            sizes = [1, 64, 1000, 4096, m, 700]
            pending = []
            for k in range(48):
                size = sizes[k % len(sizes)]
                o = k & 1
                if pending and pending[0][1] == o:
                    pid, oo, sz, linked = pending.pop(0)
                    svc.wait(pid)
                    assert np.array_equal(outs[oo].numpy()[: sz * 16].view(pa.RESULT_DTYPE), exp[:sz]), (pid, sz)
                    if linked:
                        assert np.array_equal(lk[oo].numpy()[:sz].view(np.uint16), links_exp[:sz]), (pid, sz)
                outs[o].zero_()
                linked = size == 1000
                pid = svc.post(host, size, outs[o], lk[o] if linked else None)
                pending.append((pid, o, size, linked))
                if k % 9 == 4:
                    time.sleep(0.005)
            for pid, oo, sz, linked in pending:
                svc.wait(pid)
                assert np.array_equal(outs[oo].numpy()[: sz * 16].view(pa.RESULT_DTYPE), exp[:sz]), (pid, sz)
                if linked:
                    assert np.array_equal(lk[oo].numpy()[:sz].view(np.uint16), links_exp[:sz]), (pid, sz)
        finally:
            svc.close()
    finally:
        ctx.close()


@pytest.mark.parametrize("mailbox", ["device", "host"])
def test_service_ring_reuse_with_table_changes(torch, monkeypatch, mailbox):
    """The drop-in server's pattern, as a soak: a pinned ring of two halves, each rewritten by the CPU with other frames
    once its previous post is done, two posts outstanding, conn-table changes with a post in flight, both paths, random
    sizes.  Every post's records equal the oracle's for the frames and table it was posted with -- with the mailbox in
    device memory and in pinned host memory (PN_SERVICE_HOST_MAILBOX)."""
    if mailbox == "host":
        monkeypatch.setenv("PN_SERVICE_HOST_MAILBOX", "1")
    rng = np.random.default_rng(0x7AB1E)
    m = 512
    p = pa.rx.GenParams.for_config(3)
    sets = [_frames(3, m, first=m * i)[1] for i in range(8)]
    t0 = pa.gen_conn_table(p)
    t1 = pa.gen_conn_table(p)
    for i in range(0, 64, 3):
        t1.delete(_flow_key(sets[0], i))
    tables = [t0, t1]
    exp = {(si, ti, v): _expected(sets[si], m, tables[ti], verify=v) for si in range(8) for ti in range(2)
           for v in (True, False)}
    assert not np.array_equal(exp[(0, 0, True)], exp[(0, 1, True)])
    ring = torch.zeros(2 * m * STRIDE, dtype=torch.uint8).pin_memory()
    ring_np = ring.numpy().reshape(2 * m, STRIDE)
    outs = [torch.zeros(m * 16, dtype=torch.uint8).pin_memory() for _ in range(2)]
    ctx = pa.RxContext(0)
    try:
        ti = 0
        ctx.set_conn_table(tables[ti])
        svc = pa.RxService(ctx, STRIDE, FRAME_OFF)
        try:
            pending = {}  # half -> (post id, set, table, n, verify)
            for it in range(600):
                h = it & 1
                if h in pending:
                    pid, si, tj, n, v = pending.pop(h)
                    svc.wait(pid)
                    got = outs[h].numpy()[: n * 16].view(pa.RESULT_DTYPE)
                    assert np.array_equal(got, exp[(si, tj, v)][:n]), (it, pid, si, tj, n, v)
                si = int(rng.integers(0, 8))
                ring_np[h * m:(h + 1) * m] = sets[si]
                if rng.random() < 0.15:  # a table change with the other half's post in flight
                    ti ^= 1
                    ctx.set_conn_table(tables[ti])
                v = bool(rng.random() < 0.5)
                ctx.set_verify(v)
                n = int(rng.integers(1, m + 1))
                outs[h].zero_()
                pid = svc.post(ring[h * m * STRIDE:], n, outs[h])
                pending[h] = (pid, si, ti, n, v)
            for h, (pid, si, tj, n, v) in pending.items():
                svc.wait(pid)
                got = outs[h].numpy()[: n * 16].view(pa.RESULT_DTYPE)
                assert np.array_equal(got, exp[(si, tj, v)][:n]), ("tail", pid, si, tj, n, v)
        finally:
            svc.close()
    finally:
        ctx.close()
