"""HIP path (libpollnet_amd.so, gfx950) vs the oracle and the committed golden
fixtures: bit-exact on every pn_result field (integer work, no tolerance)."""
import hashlib
import json
import os

import numpy as np
import pytest

import pollnet_amd as pa
from pollnet_amd import tuning as tn
from oracle import pyoracle as orc

from frames import FRAME_OFF, STRIDE, make_frame, to_slots

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


def gpu_classify(torch, ctx, slots, stride, off, n, entries, mask, max_conn, canary=0):
    ctx.set_conn_entries(entries, mask, max_conn)
    frames = torch.from_numpy(np.ascontiguousarray(slots).reshape(-1)).cuda()
    res = torch.full(((n + canary) * 16,), 0xAB, dtype=torch.uint8, device="cuda")
    ctx.classify(frames, stride, off, n, res, torch.cuda.current_stream())
    torch.cuda.synchronize()
    out = res.cpu().numpy()
    if canary:
        assert (out[n * 16:] == 0xAB).all(), "kernel wrote past n records"
    return out[: n * 16].view(pa.RESULT_DTYPE).copy()


def assert_same(got, exp, names=None):
    if np.array_equal(got, exp):
        return
    bad = np.nonzero(got != exp)[0]
    i = int(bad[0])
    nm = names[i] if names is not None else i
    raise AssertionError(f"{len(bad)} records differ; first #{i} ({nm}): gpu={got[i]} oracle={exp[i]}")


def test_edge_frames_bit_exact(torch_cuda, ctx, golden_dir):
    d = np.load(os.path.join(golden_dir, "edge_frames.npz"))
    n = len(d["expected"])
    got = gpu_classify(torch_cuda, ctx, d["slots"], int(d["stride"]), int(d["frame_off"]), n, d["entries"], int(d["mask"]),
                       int(d["max_conn"]), canary=17)
    assert_same(got, d["expected"], d["names"])


def test_loopback_frames_bit_exact(torch_cuda, ctx, golden_dir):
    d = np.load(os.path.join(golden_dir, "loopback_frames.npz"))
    n = len(d["lengths"])
    ents = np.zeros(16, pa.ENTRY_DTYPE)
    ents["key"] = pa.PN_EMPTY_KEY
    exp = orc.classify_batch(d["slots"], int(d["stride"]), int(d["frame_off"]), n, ents, 15, 8)
    got = gpu_classify(torch_cuda, ctx, d["slots"], int(d["stride"]), int(d["frame_off"]), n, ents, 15, 8)
    assert_same(got, exp)
    assert np.all(got["flags"] & pa.F.IP_OK)


@pytest.mark.parametrize("cfg", [2, 3, 4, 5])
def test_config_slices_vs_committed(torch_cuda, ctx, golden_dir, cfg):
    d = np.load(os.path.join(golden_dir, "config_slices.npz"))
    p = pa.rx.GenParams.for_config(cfg)
    t = pa.gen_conn_table(p)
    e, m = t.snapshot()
    s = pa.gen_frames(p, 4096, STRIDE, FRAME_OFF)
    assert hashlib.sha256(s.tobytes()).hexdigest() == str(d[f"c{cfg}_slots_sha256"])
    got = gpu_classify(torch_cuda, ctx, s, STRIDE, FRAME_OFF, 4096, e, m, t.max_conn_cnt)
    assert_same(got, d[f"c{cfg}_expected"])


@pytest.mark.parametrize("cfg", [2, 3, 5, 4])
def test_full_size_digest(torch_cuda, ctx, golden_dir, cfg):
    """BASELINE sizes (C2/C3/C5: 1 Mi frames; C4: one 2 Mi-frame shard of 8): the sha256
    of the GPU's records equals the oracle's (computed when the fixtures were made),
    plus size-independent counts."""
    with open(os.path.join(golden_dir, "full_digests.json")) as f:
        ref = json.load(f)[f"c{cfg}"]
    p = pa.rx.GenParams.for_config(cfg)
    t = pa.gen_conn_table(p)
    e, m = t.snapshot()
    n = ref["n"]
    s = pa.gen_frames(p, n, STRIDE, FRAME_OFF)
    assert pa.wire_bytes(s, STRIDE, FRAME_OFF, n) == ref["wire_bytes"]
    got = gpu_classify(torch_cuda, ctx, s, STRIDE, FRAME_OFF, n, e, m, t.max_conn_cnt)
    counts = [int(((got["flags"] >> b) & 1).sum()) for b in range(14)]
    assert counts == ref["flag_bit_counts"]
    assert hashlib.sha256(got.tobytes()).hexdigest() == ref["records_sha256"]
    if cfg in (2, 4):  # every 1024th frame carries a flipped payload bit
        assert counts[1] == n - n // 1024


def test_every_c4_shard_digest(torch_cuda, ctx, golden_dir):
    """All 8 index shards of BASELINE configs[3] (C4: 16 Mi frames, 2 Mi per GPU), one after another on
    this GPU: each shard's records hash to the digest the N=8 bench line gates that rank on."""
    with open(os.path.join(golden_dir, "full_digests.json")) as f:
        shards = json.load(f)["c4_shards"]
    assert len(shards) == 8
    p = pa.rx.GenParams.for_config(4)
    t = pa.gen_conn_table(p)
    ctx.set_conn_table(t)
    n = shards[0]["n"]
    host = np.empty((n, STRIDE), dtype=np.uint8)
    frames = torch_cuda.empty(n * STRIDE, dtype=torch_cuda.uint8, device="cuda")
    res = torch_cuda.empty(n * 16, dtype=torch_cuda.uint8, device="cuda")
    for r, ref in enumerate(shards):
        assert ref["first_index"] == r * n and ref["n"] == n
        pa.gen_frames(p, n, STRIDE, FRAME_OFF, first_index=ref["first_index"], out=host)
        assert pa.wire_bytes(host, STRIDE, FRAME_OFF, n) == ref["wire_bytes"]
        frames.copy_(torch_cuda.from_numpy(host.reshape(-1)))
        ctx.classify(frames, STRIDE, FRAME_OFF, n, res, torch_cuda.cuda.current_stream())
        torch_cuda.cuda.synchronize()
        assert hashlib.sha256(res.cpu().numpy().tobytes()).hexdigest() == ref["records_sha256"], f"shard {r}"


@pytest.mark.parametrize("frame_off", [0, 2, 4, 6, 8, 10, 12, 14, 16, 24, 34, 38, 18, 50, 66, 82, 98, 114, 120, 126])
def test_every_alignment_specialisation(torch_cuda, ctx, frame_off):
    """(frame_off + 14) % 16 selects one of 8 kernel specialisations; ef_vi's layout is
    frame_off = 10 + receive_prefix_len (Core.h:505).  frame_off >= 18 moves the window
    block off the line grid: the stream starts at the next line, and the block's
    second-line parts are skipped (header fields in the first line: 18, 34, 38, 50) or
    loaded (66 .. 98); at 114 .. 126 the block starts at line + 112 (stream start 0)."""
    p = pa.rx.GenParams.for_config(5)
    t = pa.gen_conn_table(p)
    e, m = t.snapshot()
    n = 3000
    s = pa.gen_frames(p, n, STRIDE, frame_off)
    exp = orc.classify_batch(s, STRIDE, frame_off, n, e, m, t.max_conn_cnt, threads=8)
    got = gpu_classify(torch_cuda, ctx, s, STRIDE, frame_off, n, e, m, t.max_conn_cnt, canary=3)
    assert_same(got, exp)


@pytest.mark.parametrize("stride,frame_off", [(112, 2), (128, 2), (256, 10), (1536, 2), (4096, 2), (9216, 8), (65536, 2)])
def test_slot_strides(torch_cuda, ctx, stride, frame_off):
    p = pa.rx.GenParams.for_config(3)
    t = pa.gen_conn_table(p)
    e, m = t.snapshot()
    n = 700 if stride < 65536 else 64
    s = pa.gen_frames(p, n, stride, frame_off)
    exp = orc.classify_batch(s, stride, frame_off, n, e, m, t.max_conn_cnt)
    got = gpu_classify(torch_cuda, ctx, s, stride, frame_off, n, e, m, t.max_conn_cnt)
    assert_same(got, exp)


# pn_classify picks 8/16/32/64 frames per wave from n (frames_per_wave, rx_kernel.hip): the sizes
# cover every choice and both sides of each threshold (16368/32736/65472 = 1023 waves' worth)
@pytest.mark.parametrize("n", [1, 2, 7, 8, 9, 63, 64, 65, 255, 256, 257, 1000, 4099, 16368, 16369, 32736, 32737,
                               65472, 65473])
def test_ragged_batch_sizes(torch_cuda, ctx, n):
    p = pa.rx.GenParams.for_config(3)
    t = pa.gen_conn_table(p)
    e, m = t.snapshot()
    s = pa.gen_frames(p, n)
    exp = orc.classify_batch(s, STRIDE, FRAME_OFF, n, e, m, t.max_conn_cnt)
    got = gpu_classify(torch_cuda, ctx, s, STRIDE, FRAME_OFF, n, e, m, t.max_conn_cnt, canary=65)
    assert_same(got, exp)


@pytest.mark.parametrize("n", [8, 9, 64, 100, 1000, 16369, 32737, 65473])
@pytest.mark.parametrize("frame_off,stride", [(2, 2048), (18, 2048), (2, 1536), (0, 2048), (2, 4096)])
def test_full_size_waves_ragged_extents(torch_cuda, ctx, n, frame_off, stride):
    """Waves whose every frame reaches its second stream KiB take the full-size form of phase 2, which
    is software-pipelined by half batches at strides up to 2048 (frame_pass.hpp stream_phase_pipelined):
    C4 frames (1024 flows) cut to random tot_len in [1300, 1500] -- odd lengths with a non-zero byte after
    the segment, 2-mod-4 extents, stale checksums -- at every frames-per-wave choice and ragged n."""
    p = pa.rx.GenParams.for_config(4)
    t = pa.gen_conn_table(p)
    e, m = t.snapshot()
    s = pa.gen_frames(p, n, stride, frame_off)
    rng = np.random.default_rng(n * 131 + frame_off * 7 + stride)
    tot = rng.integers(1300, 1501, n)
    ip = frame_off + 14
    s[:, ip + 2] = (tot >> 8).astype(np.uint8)
    s[:, ip + 3] = (tot & 0xFF).astype(np.uint8)
    s[np.arange(n), ip + tot] = rng.integers(1, 256, n).astype(np.uint8)  # the byte after the segment
    exp = orc.classify_batch(s, stride, frame_off, n, e, m, t.max_conn_cnt)
    assert (exp["flags"] & 0x2000).sum() == 0  # nothing truncated: every frame streams both KiBs' worth
    got = gpu_classify(torch_cuda, ctx, s, stride, frame_off, n, e, m, t.max_conn_cnt, canary=64)
    assert_same(got, exp)


@pytest.mark.parametrize("n,frame_off,stride", [(9, 18, 2048), (100, 18, 2048), (20000, 18, 2048), (333, 2, 1536),
                                                (20001, 0, 4096)])
def test_small_batch_wave_split_layouts(torch_cuda, ctx, n, frame_off, stride):
    """Small batches (fewer than 64 frames per wave) on other layouts: C5 frames (options, odd
    lengths, probe cluster) at the ef_vi-style frame_off 18, a tight 1536-B ring, per-lane windows."""
    p = pa.rx.GenParams.for_config(5)
    t = pa.gen_conn_table(p)
    e, m = t.snapshot()
    s = pa.gen_frames(p, n, stride, frame_off)
    exp = orc.classify_batch(s, stride, frame_off, n, e, m, t.max_conn_cnt)
    got = gpu_classify(torch_cuda, ctx, s, stride, frame_off, n, e, m, t.max_conn_cnt, canary=64)
    assert_same(got, exp)


def test_empty_batch_is_noop(torch_cuda, ctx):
    p = pa.rx.GenParams.for_config(2)
    t = pa.gen_conn_table(p)
    ctx.set_conn_table(t)
    frames = torch_cuda.zeros(4096, dtype=torch_cuda.uint8, device="cuda")
    res = torch_cuda.full((64,), 7, dtype=torch_cuda.uint8, device="cuda")
    ctx.classify(frames, STRIDE, FRAME_OFF, 0, res)
    torch_cuda.cuda.synchronize()
    assert (res.cpu().numpy() == 7).all()


def test_random_bytes_fuzz(torch_cuda, ctx):
    """Arbitrary slot contents (garbage headers, any tot_len/IHL/doff, stale bytes after
    the frame): the kernel must agree with the oracle on every record."""
    rng = np.random.default_rng(1234)
    n = 20000
    s = rng.integers(0, 256, size=(n, STRIDE), dtype=np.uint8)
    # make a third of them plausible IPv4/TCP so checksums and lookups see structure
    p = pa.rx.GenParams.for_config(5)
    t = pa.gen_conn_table(p)
    e, m = t.snapshot()
    plaus = pa.gen_frames(p, n // 3)
    s[: n // 3] = plaus
    # random small tot_len on some, to land near the TRUNC/odd boundaries
    idx = rng.integers(0, n, 3000)
    tl = rng.integers(0, 2100, 3000).astype(np.uint16)
    s[idx, FRAME_OFF + 16] = (tl >> 8).astype(np.uint8)
    s[idx, FRAME_OFF + 17] = (tl & 255).astype(np.uint8)
    exp = orc.classify_batch(s, STRIDE, FRAME_OFF, n, e, m, t.max_conn_cnt, threads=8)
    got = gpu_classify(torch_cuda, ctx, s, STRIDE, FRAME_OFF, n, e, m, t.max_conn_cnt)
    assert_same(got, exp)


def test_probe_runs_to_array_end_and_tiny_tables(torch_cuda, ctx):
    """A run that reaches the last entry with no EmptyKey sentinel (the reference would
    walk off the array; both sides stop at n_entries), an all-empty table, a 1-conn Conf."""
    frames, keys = [], []
    for j in range(40):
        ip = f"10.7.{j}.1"
        frames.append(make_frame(ip, 33333, payload=bytes(50)))
        keys.append(pa.conn_hash_key(int.from_bytes(bytes([10, 7, j, 1]), "little"),
                                     int.from_bytes((33333).to_bytes(2, "big"), "little")))
    slots = to_slots(frames)
    n = len(frames)
    # same home slot for all (mask 0), sorted, filling the array to the end
    ents = np.zeros(24, pa.ENTRY_DTYPE)
    ks = sorted(keys)[:24]
    ents["key"] = ks
    ents["conn_id"] = np.arange(24)
    for e, m, mc in ((ents, 0, 16), (ents, 7, 16)):
        exp = orc.classify_batch(slots, STRIDE, FRAME_OFF, n, e, m, mc)
        got = gpu_classify(torch_cuda, ctx, slots, STRIDE, FRAME_OFF, n, e, m, mc)
        assert_same(got, exp)
    empty = np.zeros(8, pa.ENTRY_DTYPE)
    empty["key"] = pa.PN_EMPTY_KEY
    got = gpu_classify(torch_cuda, ctx, slots, STRIDE, FRAME_OFF, n, empty, 7, 1)
    assert (got["conn_id"] == pa.PN_MISS).all() and not (got["flags"] & pa.F.HIT).any()
    tiny = pa.ConnTable(1, 1)
    tiny.add(keys[3], 0)
    e, m = tiny.snapshot()
    got = gpu_classify(torch_cuda, ctx, slots, STRIDE, FRAME_OFF, n, e, m, 1)
    assert got[3]["conn_id"] == 0 and np.count_nonzero(got["flags"] & pa.F.HIT) == 1


def _key_to_src(key):
    """Inverse of connHashKey (Core.h:167-172): (ip, port) in host order for a 48-bit key."""
    ip = (key >> 15) & 0xFFFFFFFF
    port = (key & 0x7FFF) | (((key >> 47) & 1) << 15)
    return f"{ip >> 24}.{(ip >> 16) & 255}.{(ip >> 8) & 255}.{ip & 255}", port


@pytest.mark.parametrize("layout", ["sentinel", "array_end", "ordered_table"])
def test_long_probe_runs(torch_cuda, ctx, layout):
    """Probe runs far longer than one wave-cooperative pass (the kernel walks a run past
    the home slot 2 entries per lane, then 64 entries per round trip for the whole wave):
    hits at every depth of 300-entry runs, misses that stop on a larger key, runs that end
    on the EmptyKey sentinel or at the array end, every lane of a wave searching at once."""
    rng = np.random.default_rng(77)
    keys = sorted({int(k) for k in rng.integers(1, 1 << 48, 420, dtype=np.int64)})[:400]
    ip, port = _key_to_src(keys[5])
    ip_be = int.from_bytes(bytes(int(x) for x in ip.split(".")), "little")
    assert pa.conn_hash_key(ip_be, int.from_bytes(port.to_bytes(2, "big"), "little")) == keys[5]
    present = keys[:300] if layout != "ordered_table" else keys[:320]
    max_conn = 1 << 12
    if layout == "ordered_table":  # the product table (addConnEntry): 4 clusters of one home slot each
        t = pa.ConnTable(1024, 1024)
        clustered = []
        for i, k in enumerate(present):
            k = (k & ~0xFFF) | (0x100 * (i % 4) + 7)  # same low 12 bits per cluster
            clustered.append(k)
            t.add(k, i)
        present = clustered
        ents, mask = t.snapshot()
        max_conn = t.max_conn_cnt
    else:
        n_ent = len(present) + (20 if layout == "sentinel" else 0)
        ents = np.zeros(n_ent, pa.ENTRY_DTYPE)
        ents["key"] = pa.PN_EMPTY_KEY
        ents["key"][: len(present)] = present
        ents["conn_id"][: len(present)] = np.arange(len(present))
        mask = 0  # every key's home is entry 0: one run of 300
    pset = set(present)
    absent = [k for k in keys if k not in pset]
    pick = []
    for i in range(4096):
        r = i % 10
        if r < 5:
            pick.append(present[int(rng.integers(len(present)))])
        elif r < 8:
            pick.append(absent[int(rng.integers(len(absent)))])
        else:
            pick.append(int(rng.integers(1, 1 << 48)))
    pick[:64] = [present[-1 - j] for j in range(64)]  # one wave whose 64 lanes all walk deep
    frames = []
    for k in pick:
        ip, port = _key_to_src(k)
        frames.append(make_frame(ip, port, payload=bytes(10)))
    slots = to_slots(frames)
    n = len(frames)
    exp = orc.classify_batch(slots, STRIDE, FRAME_OFF, n, ents, mask, max_conn, threads=8)
    got = gpu_classify(torch_cuda, ctx, slots, STRIDE, FRAME_OFF, n, ents, mask, max_conn, canary=5)
    assert_same(got, exp)
    hits = got["conn_id"][(got["flags"] & pa.F.HIT) != 0]
    assert len(hits) > 1500 and int(hits.max()) >= 250  # hits deep in the runs happened
    assert np.count_nonzero((got["flags"] & pa.F.HIT) == 0) > 1000


def test_boundary_errors(torch_cuda, ctx):
    c = pa.RxContext(0)
    frames = torch_cuda.zeros(8192, dtype=torch_cuda.uint8, device="cuda")
    res = torch_cuda.zeros(64, dtype=torch_cuda.uint8, device="cuda")
    with pytest.raises(pa.PollnetError, match="conn table"):
        c.classify(frames, STRIDE, FRAME_OFF, 1, res)
    c.set_conn_table(pa.gen_conn_table(pa.rx.GenParams.for_config(2)))
    with pytest.raises(pa.PollnetError, match="aligned"):
        c.classify(frames.data_ptr() + 2, STRIDE, FRAME_OFF, 1, res)
    with pytest.raises(pa.PollnetError, match="layout"):
        c.classify(frames, 100, FRAME_OFF, 1, res)
    with pytest.raises(pa.PollnetError, match="layout"):
        c.classify(frames, STRIDE, 3, 1, res)
    c.close()


def test_side_stream_and_sync(torch_cuda, ctx):
    p = pa.rx.GenParams.for_config(3)
    t = pa.gen_conn_table(p)
    e, m = t.snapshot()
    n = 5000
    s = pa.gen_frames(p, n)
    exp = orc.classify_batch(s, STRIDE, FRAME_OFF, n, e, m, t.max_conn_cnt, threads=8)
    ctx.set_conn_entries(e, m, t.max_conn_cnt)
    frames = torch_cuda.from_numpy(s.reshape(-1)).cuda()
    torch_cuda.cuda.synchronize()
    st = torch_cuda.cuda.Stream()
    with torch_cuda.cuda.stream(st):
        res = torch_cuda.empty(n * 16, dtype=torch_cuda.uint8, device="cuda")
        ctx.classify(frames, STRIDE, FRAME_OFF, n, res, st)
    ctx.sync()
    assert_same(res.cpu().numpy().view(pa.RESULT_DTYPE), exp)


def test_table_replaced_while_classify_in_flight(torch_cuda):
    """pn_set_conn_table right after classify launches on two side streams (and a TX fill on
    a third): every launch still sees the snapshot it was issued against -- the replacement
    goes to the other table buffer, the launches record nothing."""
    torch = torch_cuda
    c = pa.RxContext(0)
    p = pa.rx.GenParams.for_config(3)
    t = pa.gen_conn_table(p)
    e, m = t.snapshot()
    n = 1 << 20
    s = pa.gen_frames(p, n)
    exp = orc.classify_batch(s[:8192], STRIDE, FRAME_OFF, 8192, e, m, t.max_conn_cnt, threads=8)
    other = np.zeros(len(e), pa.ENTRY_DTYPE)
    other["key"] = pa.PN_EMPTY_KEY  # an empty table: every record would become a miss
    c.set_conn_entries(e, m, t.max_conn_cnt)
    frames = torch.from_numpy(s.reshape(-1)).cuda()
    tx = torch.from_numpy(pa.gen_frames(pa.rx.GenParams.for_config(2), 4096).reshape(-1)).cuda()
    torch.cuda.synchronize()
    sa, sb, stx = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    ra = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
    rb = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
    for _ in range(3):
        c.classify(frames, STRIDE, FRAME_OFF, n, ra, sa)
        c.classify(frames, STRIDE, FRAME_OFF, n, rb, sb)
        c.tx_fill(tx, STRIDE, FRAME_OFF, 4096, stream=stx)
        c.set_conn_entries(other, m, t.max_conn_cnt)  # no sync before it
        torch.cuda.synchronize()
        for r in (ra, rb):
            got = r.cpu().numpy().view(pa.RESULT_DTYPE)
            assert_same(got[:8192], exp)
            assert np.count_nonzero(got["flags"] & pa.F.HIT) > n // 2
        c.set_conn_entries(e, m, t.max_conn_cnt)
    c.close()


def test_cpp_adapter_without_torch():
    """include/pollnet_amd/gpu_rx.hpp driven from a plain C++ process (only /opt/rocm's
    HIP runtime loaded): records and the pollNet-style TW/recv dispatch vs the oracle."""
    import subprocess

    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cpp", "test_gpu_rx")
    assert os.path.exists(exe), "build with `make` first"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "PASS" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("cfg", [3, 5])
def test_cooperative_and_per_lane_windows_agree(torch_cuda, ctx, cfg):
    """The kernel loads the header window cooperatively (one request per 128-B line) when
    slot lines are 128-B aligned with ip at line+16, else per lane.  Shift the same ring
    by 16 bytes to force the other path: records must be identical (and match the oracle)."""
    p = pa.rx.GenParams.for_config(cfg)
    t = pa.gen_conn_table(p)
    e, m = t.snapshot()
    n = 3000
    s = pa.gen_frames(p, n)
    exp = orc.classify_batch(s, STRIDE, FRAME_OFF, n, e, m, t.max_conn_cnt, threads=8)
    ctx.set_conn_entries(e, m, t.max_conn_cnt)
    outs = []
    for shift in (0, 16, 32, 48):
        buf = torch_cuda.zeros(n * STRIDE + 256, dtype=torch_cuda.uint8, device="cuda")
        base = buf.data_ptr()
        pad = (-base) % 128 + shift  # slots start `shift` bytes past a 128-B boundary
        buf[pad:pad + n * STRIDE].copy_(torch_cuda.from_numpy(s.reshape(-1)))
        res = torch_cuda.empty(n * 16, dtype=torch_cuda.uint8, device="cuda")
        ctx.classify(base + pad, STRIDE, FRAME_OFF, n, res, torch_cuda.cuda.current_stream())
        torch_cuda.cuda.synchronize()
        outs.append(res.cpu().numpy().view(pa.RESULT_DTYPE).copy())
    for o in outs:
        assert_same(o, exp)


def test_calib_slot_read_var(torch_cuda, ctx):
    """The mixed-size ceiling kernel (bench.py's frame_lines leg): writes exactly one 16-B record per
    slot, nothing past n, and rejects bad arguments."""
    n, stride = 1000, STRIDE
    frames = torch_cuda.randint(0, 256, (n * stride,), dtype=torch_cuda.uint8, device="cuda")
    lens = torch_cuda.randint(64, 1600, (n,), dtype=torch_cuda.int32, device="cuda")
    sink = torch_cuda.full(((n + 64) * 16,), 0xAB, dtype=torch_cuda.uint8, device="cuda")
    tn.calib_slot_read_var(ctx, frames, n, stride, lens, sink, torch_cuda.cuda.current_stream(), 16)
    torch_cuda.cuda.synchronize()
    out = sink.cpu().numpy()
    assert (out[n * 16:] == 0xAB).all()
    recs = out[: n * 16].view("<u4").reshape(n, 4)
    assert (recs[:, 1] == recs[:, 0] ^ 1).all() and (recs[:, 3] == recs[:, 0] ^ 3).all()
    with pytest.raises(pa.PollnetError, match="bad arguments"):
        tn.calib_slot_read_var(ctx, frames, n, 100, lens, sink, None, 16)
    with pytest.raises(pa.PollnetError, match="bad arguments"):
        tn.calib_slot_read_var(ctx, frames, n, stride, lens, sink, None, 8)


def test_reference_literal_table_records(torch_cuda, ctx):
    """PN_TABLE_REFERENCE_LITERAL on the rehash-defect history (tests/test_oracle.py): frames
    from every live flow — the stranded ones included — classified on the GPU against the
    literal table equal the oracle's records against the oracle's own table, bit for bit;
    the stranded flows come back as misses, as they would from the reference."""
    import socket
    import struct

    from test_oracle import _apply, _random_history

    ops, live = _random_history(7, 400, 0.5)
    ot, lt = orc.Table(256, 256), pa.ConnTable(256, 256, reference_literal=True)
    for op, k, c in ops:
        _apply(ot, op, k, c)
        _apply(lt, op, k, c)
    frames = []
    for k in list(live) + [(0x0A0B0C0D << 15) | 0x1234]:  # + one unknown flow
        ip = (k >> 15) & 0xFFFFFFFF
        port = (k & 0x7FFF) | ((k >> 32) & 0x8000)  # connHashKey inverted (Core.h:167-172)
        frames.append(make_frame(src=socket.inet_ntoa(struct.pack("!I", ip)), sport=port, payload=b"x" * (k % 97)))
    slots = to_slots(frames)
    n = len(frames)
    e, m = lt.snapshot()
    got = gpu_classify(torch_cuda, ctx, slots, STRIDE, FRAME_OFF, n, e, m, lt.max_conn_cnt)
    oe = ot.entries()
    exp = orc.classify_batch(slots, STRIDE, FRAME_OFF, n, oe, ot.mask, 256)
    assert_same(got, exp)
    lost = [i for i, k in enumerate(live) if oe[ot.find(k)]["key"] != k]
    assert lost and all(got["conn_id"][i] == pa.PN_MISS for i in lost)


def test_gpu_verdicts_equal_reference_core_checksum(torch_cuda, ctx, golden_dir):
    """GPU IP_OK / TCP_OK against the reference's own Core::checksum (Core.h:448-472, compiled
    from /root/reference into oracle/_ref/libref_core.so) directly, on the committed edge
    fixture: every frame whose summed bytes lie inside its slot."""
    ref = orc.ref_core()
    if ref is None:
        pytest.skip("oracle/_ref/libref_core.so not built")
    d = np.load(os.path.join(golden_dir, "edge_frames.npz"))
    slots, stride, off = d["slots"], int(d["stride"]), int(d["frame_off"])
    n = len(slots)
    got = gpu_classify(torch_cuda, ctx, slots, stride, off, n, d["entries"], int(d["mask"]), int(d["max_conn"]))
    checked = 0
    for i in range(n):
        eth = np.ascontiguousarray(slots[i, off:])
        tot = (int(eth[16]) << 8) | int(eth[17])
        if tot < 20 or 14 + tot + (tot & 1) > stride - off:
            continue
        v = ref.ref_checksum(eth.ctypes.data)
        f = int(got["flags"][i])
        assert bool(v & 1) == bool(f & pa.F.IP_OK) and bool(v & 2) == bool(f & pa.F.TCP_OK), i
        checked += 1
    assert checked > 1500
