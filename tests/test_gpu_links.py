"""GPU: the chain links of a resident-service post (pn_service_post_linked, rx_service.hip chain_pass) against the
oracle's statement (orc_chain_links, pinned by hand cases in tests/test_oracle.py): crafted chain workloads with
every kind of break, interleaved flows (the drop-in server's 256 x 2 per poll), one flow (a connection repeating in
every 64-frame step), the generator's C2 / C3 / C5 batches, both paths, zero copy and device memory, two posts
outstanding, linked and plain posts interleaved, the bounds."""
import numpy as np
import pytest

import pollnet_amd as pa
from oracle import pyoracle as orc

import chainframes as cf
from frames import FRAME_OFF, STRIDE

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t

    assert t.cuda.is_available(), "GPU tests need an MI355X"
    return t


def _expect(s, n, table, verify):
    e, m = table.snapshot()
    r = orc.classify_batch(s, STRIDE, FRAME_OFF, n, e, m, table.max_conn_cnt, threads=8, unverified=not verify)
    return r, orc.chain_links(s, STRIDE, FRAME_OFF, n, r, table.max_conn_cnt)


def _run(torch, svc, ctx, s, n, table, verify, device=False):
    ctx.set_verify(verify)
    host = torch.from_numpy(np.ascontiguousarray(s).reshape(-1)).pin_memory()
    src = host.cuda() if device else host
    res = torch.zeros(n * 16, dtype=torch.uint8).pin_memory()
    links = torch.full((n,), -16657, dtype=torch.int16).pin_memory()  # 0xBEEF: overwritten everywhere
    svc.classify(src, n, res, links)
    return res.numpy().view(pa.RESULT_DTYPE), links.numpy().view(np.uint16)


PERTURB = [(9, "fin"), (13, "ack"), (18, "hole"), (26, "retrans"), (35, "pure_ack"), (41, "rst"), (50, "syn"),
           (57, "noack"), (66, "window"), (73, "dport"), (82, "bad_tcp"), (90, "bad_ip")]


@pytest.mark.parametrize("verify", [True, False])
@pytest.mark.parametrize("device", [False, True])
def test_links_crafted_chains(torch, verify, device):
    fr, flows = cf.build(8, 16, perturb=PERTURB, unknown=(6,))
    s = cf.slots_of(fr)
    table = cf.table_for(pa, flows, tw=(7,))
    ctx = pa.RxContext(0)
    try:
        ctx.set_conn_table(table)
        svc = pa.RxService(ctx, STRIDE, FRAME_OFF)
        try:
            got_r, got_l = _run(torch, svc, ctx, s, len(fr), table, verify, device)
            exp_r, exp_l = _expect(s, len(fr), table, verify)
            assert np.array_equal(got_r, exp_r)
            assert np.array_equal(got_l, exp_l), (np.nonzero(got_l != exp_l)[0][:8], got_l[:24], exp_l[:24])
            assert (exp_l != 0).sum() > len(fr) // 2  # the workload is mostly chains
        finally:
            svc.close()
    finally:
        ctx.close()


@pytest.mark.parametrize("n_flows,per_flow", [(256, 2), (256, 4), (1, 1024), (3, 300), (64, 16), (1000, 1)])
def test_links_interleaved_flows(torch, n_flows, per_flow):
    """The drop-in server's poll (256 flows x 2 segments), more segments per flow, one flow (its connection repeats
    in every lane of every 64-frame step), a few flows (repeats inside steps), one frame per flow (no chain)."""
    fr, flows = cf.build(n_flows, per_flow, seed=n_flows * 7 + per_flow)
    s = cf.slots_of(fr)
    table = cf.table_for(pa, flows, max_conn=max(1024, n_flows))
    ctx = pa.RxContext(0)
    try:
        ctx.set_conn_table(table)
        svc = pa.RxService(ctx, STRIDE, FRAME_OFF)
        try:
            for verify in (True, False):
                got_r, got_l = _run(torch, svc, ctx, s, len(fr), table, verify)
                exp_r, exp_l = _expect(s, len(fr), table, verify)
                assert np.array_equal(got_r, exp_r)
                assert np.array_equal(got_l, exp_l), (verify, np.nonzero(got_l != exp_l)[0][:8])
                assert (exp_l != 0).sum() == n_flows * (per_flow - 1)
        finally:
            svc.close()
    finally:
        ctx.close()


@pytest.mark.parametrize("cfg", [2, 3, 5])
def test_links_generator_batches(torch, cfg):
    """The generator's batches at every post size class: links equal the oracle's (C2 is one flow; its links are
    whatever its sequence numbers make them)."""
    p = pa.rx.GenParams.for_config(cfg)
    N = 1024
    s = np.ascontiguousarray(pa.gen_frames(p, N, STRIDE, FRAME_OFF, threads=8))
    table = pa.gen_conn_table(p)
    ctx = pa.RxContext(0)
    try:
        ctx.set_conn_table(table)
        svc = pa.RxService(ctx, STRIDE, FRAME_OFF)
        try:
            for n in (1, 7, 63, 64, 65, 129, 511, 512, 1000, 1024):
                for verify in (True, False):
                    got_r, got_l = _run(torch, svc, ctx, s[:n], n, table, verify)
                    exp_r, exp_l = _expect(s[:n], n, table, verify)
                    assert np.array_equal(got_r, exp_r), (n, verify)
                    assert np.array_equal(got_l, exp_l), (n, verify, np.nonzero(got_l != exp_l)[0][:8])
        finally:
            svc.close()
    finally:
        ctx.close()


def test_links_outstanding_interleaved_and_bounds(torch):
    """Two linked posts outstanding (each slot has its own scratch), plain posts between them, a post of more than
    PN_LINK_MAX_FRAMES refused, and a table with max_conn_cnt above PN_LINK_MAX_CONNS: every link 0."""
    fr, flows = cf.build(256, 4, seed=5)
    s = cf.slots_of(fr)
    n = len(fr)
    table = cf.table_for(pa, flows)
    exp_r, exp_l = _expect(s, n, table, False)
    ctx = pa.RxContext(0)
    try:
        ctx.set_conn_table(table)
        ctx.set_verify(False)
        svc = pa.RxService(ctx, STRIDE, FRAME_OFF, idle_ms=2)
        try:
            host = torch.from_numpy(s.reshape(-1)).pin_memory()
            res = [torch.zeros(n * 16, dtype=torch.uint8).pin_memory() for _ in range(2)]
            lk = [torch.zeros(n, dtype=torch.int16).pin_memory() for _ in range(2)]
            for rep in range(30):
                a = svc.post(host, n, res[0], lk[0] if rep % 3 else None)
                b = svc.post(host, n, res[1], lk[1])
                svc.wait(a)
                svc.wait(b)
                for r in res:
                    assert np.array_equal(r.numpy().view(pa.RESULT_DTYPE), exp_r)
                assert np.array_equal(lk[1].numpy().view(np.uint16), exp_l)
                if rep % 3:
                    assert np.array_equal(lk[0].numpy().view(np.uint16), exp_l)
                lk[0].zero_()
                lk[1].zero_()
                if rep % 10 == 9:
                    import time

                    time.sleep(0.005)  # past idle_ms: the next post relaunches the kernel
            big = torch.zeros((pa.PN_LINK_MAX_FRAMES + 1) * STRIDE, dtype=torch.uint8).pin_memory()
            with pytest.raises(pa.PollnetError, match="PN_LINK_MAX_FRAMES"):
                svc.post(big, pa.PN_LINK_MAX_FRAMES + 1, torch.zeros((pa.PN_LINK_MAX_FRAMES + 1) * 16,
                                                                    dtype=torch.uint8).pin_memory(),
                         torch.zeros(pa.PN_LINK_MAX_FRAMES + 1, dtype=torch.int16).pin_memory())
            wide = cf.table_for(pa, flows, max_conn=8192)
            ctx.set_conn_table(wide)
            lk[0].fill_(7)
            svc.classify(host, n, res[0], lk[0])
            assert not lk[0].numpy().any()
            e, m = wide.snapshot()
            r = orc.classify_batch(s, STRIDE, FRAME_OFF, n, e, m, wide.max_conn_cnt, unverified=True)
            assert np.array_equal(res[0].numpy().view(pa.RESULT_DTYPE), r)
        finally:
            svc.close()
    finally:
        ctx.close()
