"""pn_match_streams (TcpStream filter on the GPU) through the Python binding: C3/C5 batches
and random bytes, 1..64 overlapping wildcard filters, vs a numpy filterPacket."""
import numpy as np
import pytest

import pollnet_amd as pa

from streams_np import match_streams_np

pytestmark = pytest.mark.gpu


def _ip(s):
    return int.from_bytes(bytes(int(x) for x in s.split(".")), "little")


def _port(p):
    return int.from_bytes(p.to_bytes(2, "big"), "little")


def _filters(rng, slots, frame_off, k):
    """k filters: some copied from frames in the batch (with random wildcards), some random."""
    f = np.zeros(k, pa.STREAM_FILTER_DTYPE)
    for i in range(k):
        j = int(rng.integers(len(slots)))
        eth = slots[j, frame_off:]
        f[i]["src_ip"] = int.from_bytes(bytes(eth[26:30]), "little") if rng.random() < 0.7 else 0
        f[i]["dst_ip"] = int.from_bytes(bytes(eth[30:34]), "little") if rng.random() < 0.5 else 0
        f[i]["src_port"] = int.from_bytes(bytes(eth[34:36]), "little") if rng.random() < 0.7 else 0
        f[i]["dst_port"] = int.from_bytes(bytes(eth[36:38]), "little") if rng.random() < 0.5 else 0
        if rng.random() < 0.2:
            f[i]["src_ip"] = _ip(f"10.9.{i}.1")
    f[0] = (0, _ip("10.0.0.1"), 0, _port(1234), 0)  # dst-only filter: every TCP frame to the server
    return f


@pytest.mark.parametrize("cfg,frame_off", [(3, 2), (5, 10), (3, 24), (5, 16)])
def test_match_streams_vs_numpy(cfg, frame_off):
    import torch

    rng = np.random.default_rng(cfg * 100 + frame_off)
    n = 20000
    p = pa.rx.GenParams.for_config(cfg)
    slots = pa.gen_frames(p, n, 2048, frame_off)
    junk = rng.integers(0, 256, (n // 4, 2048), dtype=np.uint8)  # non-IPv4/non-TCP and garbage
    slots[rng.choice(n, n // 4, replace=False)] = junk
    ctx = pa.RxContext(0)
    dev = torch.from_numpy(slots.reshape(-1)).cuda()
    out = torch.full((n + 7,), 0xAB, dtype=torch.int32, device="cuda")
    for k in (1, 8, 64):
        flt = _filters(rng, slots, frame_off, k) if k > 1 else np.array([(0, _ip("10.0.0.1"), 0, 0, 0)],
                                                                        pa.STREAM_FILTER_DTYPE)
        ctx.match_streams(dev, 2048, frame_off, n, flt, out, torch.cuda.current_stream())
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint32)
        assert (got[n:] == 0xAB).all(), "wrote past n"
        exp = match_streams_np(slots, frame_off, flt)
        assert np.array_equal(got[:n], exp), (k, int(np.count_nonzero(got[:n] != exp)))
        assert (exp != pa.PN_NO_STREAM).any() and (exp == pa.PN_NO_STREAM).any()
    ctx.close()


# Every IP-header class (frame_off + 14) % 16 the kernel is instantiated for, slot strides from the
# contract's minimum (frame_off + 96, on the 16-B grid) to 64 KiB, and batches that end inside a wave
# (the per-wave buffer range and the no-fetch offsets of the cooperative loads).
@pytest.mark.parametrize("frame_off,stride,n", [(2, 112, 1), (4, 112, 63), (6, 1536, 1000), (8, 2048, 65),
                                                (12, 4096, 130), (14, 128, 257), (16, 65536, 200),
                                                (26, 2048, 4097)])
def test_match_streams_layouts(frame_off, stride, n):
    import torch

    rng = np.random.default_rng(frame_off * 7 + n)
    p = pa.rx.GenParams.for_config(3)
    full = pa.gen_frames(p, n, 2048, frame_off)
    slots = np.zeros((n, stride), np.uint8)
    w = min(stride, 2048)
    slots[:, :w] = full[:, :w]  # the filter reads only the first frame_off + 38 bytes of a slot
    slots[rng.random(n) < 0.2, frame_off + 23] = 17  # some UDP frames
    ctx = pa.RxContext(0)
    dev = torch.from_numpy(slots.reshape(-1)).cuda()
    out = torch.full((n + 64,), 0xAB, dtype=torch.int32, device="cuda")
    flt = np.roll(_filters(rng, slots, frame_off, 8), -1)  # the catch-all dst filter last: every id can win
    ctx.match_streams(dev, stride, frame_off, n, flt, out, torch.cuda.current_stream())
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    assert (got[n:] == 0xAB).all(), "wrote past n"
    exp = match_streams_np(slots, frame_off, flt)
    assert np.array_equal(got[:n], exp), int(np.count_nonzero(got[:n] != exp))
    # no filters: every frame gets PN_NO_STREAM; n = 0 writes nothing
    ctx.match_streams(dev, stride, frame_off, n, np.zeros(0, pa.STREAM_FILTER_DTYPE), out,
                      torch.cuda.current_stream())
    ctx.match_streams(dev, stride, frame_off, 0, flt, out[n:], torch.cuda.current_stream())
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    assert (got[:n] == pa.PN_NO_STREAM).all() and (got[n:] == 0xAB).all()
    ctx.close()


# The round-4 kernel forms (match_streams_mask_kernel, tuning variants 10-14: wave-ordered tile, mask
# compare in blocks of 8 filters, 1-4 groups of 64 frames per wave, 1 or 4 waves per workgroup) on
# the same layouts and 0, 1, 7, 8, 9 and 64 filters (padded blocks), against numpy.
@pytest.mark.parametrize("variant", [10, 11, 12, 13, 14, 20, 22, 24, 26, 28, 30, 31, 32, 33, 36, 37, 39])
@pytest.mark.parametrize("frame_off,stride,n", [(2, 112, 1), (4, 2048, 700), (14, 128, 257), (16, 65536, 200),
                                                (26, 2048, 4097)])
def test_match_streams_mask_variants(variant, frame_off, stride, n):
    import torch

    from pollnet_amd import tuning as tn

    rng = np.random.default_rng(frame_off * 7 + n + variant)
    p = pa.rx.GenParams.for_config(5)
    full = pa.gen_frames(p, n, 2048, frame_off)
    slots = np.zeros((n, stride), np.uint8)
    w = min(stride, 2048)
    slots[:, :w] = full[:, :w]
    slots[rng.random(n) < 0.2, frame_off + 23] = 17  # some UDP frames
    slots[rng.random(n) < 0.1, frame_off + 12] = 0x86  # some non-IPv4 ethertypes
    ctx = pa.RxContext(0)
    dev = torch.from_numpy(slots.reshape(-1)).cuda()
    out = torch.full((n + 300,), 0xAB, dtype=torch.int32, device="cuda")
    for k in (0, 1, 7, 8, 9, 64):
        flt = np.roll(_filters(rng, slots, frame_off, k), -1) if k else np.zeros(0, pa.STREAM_FILTER_DTYPE)
        out.fill_(0xAB)
        tn.match_streams_variant(ctx, dev, stride, frame_off, n, flt, out, variant, torch.cuda.current_stream())
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint32)
        assert (got[n:] == 0xAB).all(), ("wrote past n", k)
        exp = match_streams_np(slots, frame_off, flt)
        assert np.array_equal(got[:n], exp), (k, int(np.count_nonzero(got[:n] != exp)))
    ctx.close()
