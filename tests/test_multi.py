"""N>1 path on CPU: world_size-2 gloo ranks each own a contiguous index shard of one
global batch (no data exchange), results aggregate to the single-process answer,
and the bench's timing reduction (barrier + MAX over ranks) behaves.  The per-shard
compute here is the oracle (no GPU in this container); on the GPU box the same
sharding drives pn_classify (bench.py)."""
import hashlib
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_per_rank, cfg, out_dir):
    import sys

    sys.path.insert(0, ROOT)
    import torch

    import pollnet_amd as pa
    from oracle import pyoracle as orc
    from pollnet_amd.shard import shard_range

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    p = pa.rx.GenParams.for_config(cfg)
    lo, hi = shard_range(rank, world, n_per_rank)
    slots = pa.gen_frames(p, hi - lo, first_index=lo, threads=2)
    t = pa.gen_conn_table(p)
    e, m = t.snapshot()
    dist.barrier()
    rec = orc.classify_batch(slots, 2048, 2, hi - lo, e, m, t.max_conn_cnt)
    wall = torch.tensor([float(rank + 1)], dtype=torch.float64)  # stand-in per-rank time
    dist.all_reduce(wall, op=dist.ReduceOp.MAX)
    wire = torch.tensor([float(pa.wire_bytes(slots, 2048, 2, hi - lo))], dtype=torch.float64)
    dist.all_reduce(wire, op=dist.ReduceOp.SUM)
    np.save(os.path.join(out_dir, f"rank{rank}.npy"), rec)
    if rank == 0:
        with open(os.path.join(out_dir, "reduced.txt"), "w") as f:
            f.write(f"{wall.item()} {wire.item()}")
    dist.destroy_process_group()


@pytest.mark.parametrize("cfg", [3, 4])
def test_two_rank_shards_match_single_process(tmp_path, cfg):
    import sys

    sys.path.insert(0, ROOT)
    import pollnet_amd as pa
    from oracle import pyoracle as orc

    world, n = 2, 3000
    mp.spawn(_worker, args=(world, _free_port(), n, cfg, str(tmp_path)), nprocs=world, join=True)
    parts = [np.load(tmp_path / f"rank{r}.npy") for r in range(world)]
    p = pa.rx.GenParams.for_config(cfg)
    full = pa.gen_frames(p, world * n, threads=4)
    t = pa.gen_conn_table(p)
    e, m = t.snapshot()
    exp = orc.classify_batch(full, 2048, 2, world * n, e, m, t.max_conn_cnt)
    got = np.concatenate(parts)
    assert np.array_equal(got, exp)
    wall, wire = map(float, open(tmp_path / "reduced.txt").read().split())
    assert wall == float(world)  # MAX over ranks
    assert wire == float(pa.wire_bytes(full, 2048, 2, world * n))


def _window_worker(rank, world, port, flag, out_dir, shm=False):
    """Rank 1's work cannot start until rank 0's is done (a file flag): the two ran one after the
    other, so the common window must cover both (>= 0.4 s), while each rank's own body is ~0.2 s
    of work plus, on rank 1, the wait."""
    import time

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys

    sys.path.insert(0, ROOT)
    from pollnet_amd.shard import common_window

    def body():
        if rank == 1:
            while not os.path.exists(flag):
                time.sleep(0.005)
        time.sleep(0.2)
        if rank == 0:
            open(flag, "w").close()

    barrier = None
    if shm:
        from pollnet_amd.shard import ShmBarrier

        barrier = ShmBarrier(dist, rank, world)
    wall, own = common_window(body, dist, barrier)
    if barrier is not None:
        ts = []
        for _ in range(200):
            t0 = time.perf_counter()
            barrier()
            ts.append(time.perf_counter() - t0)
        per = sorted(ts)[len(ts) // 2]  # median: a rank descheduled by a busy host does not skew it
        barrier.close(dist)
    else:
        per = 0.0
    with open(os.path.join(out_dir, f"win{rank}.txt"), "w") as f:
        f.write(f"{wall} {own} {per}")
    dist.destroy_process_group()


@pytest.mark.parametrize("shm", [False, True])
def test_common_window_covers_serialised_ranks(tmp_path, shm):
    """bench.py's aggregate timing (shard.common_window): ranks that ran one after another cannot
    look parallel — every rank reports the same max window, and it spans both ranks' work; with gloo's
    barrier and with the shared-memory barrier the bench uses on one node (which must also be fast)."""
    world = 2
    mp.spawn(_window_worker, args=(world, _free_port(), str(tmp_path / "flag"), str(tmp_path), shm), nprocs=world,
             join=True)
    res = [tuple(map(float, open(tmp_path / f"win{r}.txt").read().split())) for r in range(world)]
    assert res[0][:2] == res[1][:2]  # max over ranks, identical everywhere
    wall, own, per = res[0]
    assert wall >= 0.4 and own >= 0.4 and wall >= own
    if shm:
        assert per < 2e-3, per  # a spin on shared memory, not a socket round trip
    assert not [f for f in os.listdir("/dev/shm") if f.startswith("pn_barrier_")]


def test_common_window_single_process():
    import time

    from pollnet_amd.shard import common_window

    wall, own = common_window(lambda: time.sleep(0.05), None)
    assert 0.05 <= own <= wall < 1.0


def test_bench_golden_covers_every_c4_shard_and_c2_batch():
    """The N>1 bench gates each rank's C4 shard (8 shards of 2 Mi = BASELINE configs[3]) and the N=1
    bench every rotating C2 batch against a committed oracle digest (tests/golden/make_golden.py)."""
    import importlib.util
    import sys

    sys.path.insert(0, ROOT)
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    for r in range(8):
        d = bench.golden_digest(4, r << 21, 1 << 21)
        assert d is not None and d["wire_bytes"] == (1 << 21) * 1514
    assert bench.golden_digest(4, 0, 1 << 21)["records_sha256"] == bench.golden_digest(4)["records_sha256"]
    for b in range(4):
        assert bench.golden_digest(2, b << 20, 1 << 20) is not None
    assert bench.golden_digest(4, 8 << 21, 1 << 21) is None and bench.golden_digest(4, 0, 4096) is None


def test_c4_shard_digest_regenerates():
    """One C4 shard (shard 5) recomputed here by generator + oracle equals the committed digest."""
    import json
    import sys

    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    sys.path.insert(0, ROOT)
    import make_golden

    with open(os.path.join(ROOT, "tests", "golden", "full_digests.json")) as f:
        ref = json.load(f)["c4_shards"][5]
    got = make_golden.records_digest(4, ref["first_index"], ref["n"], threads=min(8, os.cpu_count() or 1))
    assert got["records_sha256"] == ref["records_sha256"] and got["wire_bytes"] == ref["wire_bytes"]


def test_shard_ranges():
    from pollnet_amd.shard import shard_range, split_range

    assert [shard_range(r, 4, 10) for r in range(4)] == [(0, 10), (10, 20), (20, 30), (30, 40)]
    spans = [split_range(r, 3, 10) for r in range(3)]
    assert spans[0][0] == 0 and spans[-1][1] == 10 and all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
    with pytest.raises(ValueError):
        shard_range(4, 4, 10)


def _gpu_worker(rank, world, port, n_per_rank, out_dir):
    """One rank on the box's GPU: its contiguous C4 shard through pn_classify (the C-ABI)."""
    import sys

    sys.path.insert(0, ROOT)
    import torch

    import pollnet_amd as pa
    from pollnet_amd.shard import shard_range

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(rank % torch.cuda.device_count())
    p = pa.rx.GenParams.for_config(4)
    lo, hi = shard_range(rank, world, n_per_rank)
    slots = pa.gen_frames(p, hi - lo, first_index=lo, threads=4)
    ctx = pa.RxContext(torch.cuda.current_device())
    ctx.set_conn_table(pa.gen_conn_table(p))
    frames = torch.from_numpy(slots.reshape(-1)).cuda()
    res = torch.empty((hi - lo) * 16, dtype=torch.uint8, device="cuda")
    dist.barrier()
    ctx.classify(frames, 2048, 2, hi - lo, res, torch.cuda.current_stream())
    torch.cuda.synchronize()
    dist.barrier()
    np.save(os.path.join(out_dir, f"gpu_rank{rank}.npy"), res.cpu().numpy())
    ctx.close()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_gpu_two_rank_shards_equal_c4_digest(tmp_path, golden_dir):
    """Two gloo ranks share the box's GPU, each classifying its contiguous half of the C4
    shard (2 Mi frames) through pn_classify; the concatenated records hash to the committed
    single-process C4 digest (made by the oracle)."""
    import json

    with open(os.path.join(golden_dir, "full_digests.json")) as f:
        ref = json.load(f)["c4"]
    world = 2
    mp.spawn(_gpu_worker, args=(world, _free_port(), ref["n"] // world, str(tmp_path)), nprocs=world, join=True)
    got = np.concatenate([np.load(tmp_path / f"gpu_rank{r}.npy") for r in range(world)])
    assert hashlib.sha256(got.tobytes()).hexdigest() == ref["records_sha256"]


@pytest.mark.gpu
def test_bench_spawns_ranks_itself():
    """`bench.py --gpus 2` without torchrun starts its 2 ranks (spawn) and reports n_gpus 2;
    on a 1-GPU box the ranks share the device (a rehearsal of the N>1 flow)."""
    import json
    import subprocess
    import sys

    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
                        "--frames", "65536", "--batches", "2", "--no-cpu-baseline", "--no-e2e", "--no-secondary"],
                       capture_output=True, text=True, timeout=240, env={k: v for k, v in os.environ.items()
                                                                        if k not in ("WORLD_SIZE", "RANK")})
    assert p.returncode == 0, p.stderr[-3000:]
    lines = p.stdout.strip().splitlines()
    assert len(lines) == 1, lines  # stdout is the JSON line alone (gloo's own log goes to stderr)
    line = json.loads(lines[0])
    # a --frames override has no committed digest: checked by invariants + 4096 oracle records only
    assert line["n_gpus"] == 2 and line["verified_vs_oracle"] == "partial"
    assert line["correctness_gate"]["every_rank_verified"] is True
    assert line["correctness_gate"]["every_rank_sha256_gated"] is False
    assert line["config"]["global_frames"] == 2 * 65536
    assert line["config"]["workload"].startswith("C4")  # N>1 defaults to BASELINE configs[3]


@pytest.mark.gpu
def test_bench_under_the_drivers_torchrun_command():
    """The driver's own N>1 launch (`python -m torch.distributed.run --nnodes=1 --nproc-per-node N
    --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...`), N = 2 on this box's GPU:
    rank 0 alone prints one JSON line, n_gpus 2, the aggregate over both ranks.  Full C4 shards
    (2 Mi frames per rank, BASELINE configs[3]): each rank sha256-gates both of its batches against
    its own shard's committed digest."""
    import json
    import socket
    import subprocess
    import sys

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3",
           "--warmup", "1", "--batches", "2", "--no-cpu-baseline", "--no-e2e", "--no-secondary"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.strip().splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["verified_vs_oracle"] is True
    assert line["config"]["workload"].startswith("C4") and line["config"]["global_frames"] == 2 * (1 << 21)
    ranks = line["correctness_gate"]["ranks"]
    assert [g["shard"] for g in ranks] == [[0, 1 << 21], [1 << 21, 2 << 21]]
    for r, g in enumerate(ranks):
        assert g["batches_sha256_gated"] == "2/2" and g["gated_batches_sha256_match_golden"] is True
        assert g["all_batches_invariants"] is True and g["batch0_first_4096_vs_oracle"] is True
        # which physical device the rank ran on, its own kernel time, its setup time and host memory
        assert g["rank"] == r and g["device_ordinal"] == 0  # one GPU on this box: both ranks on device 0
        assert len(g["pci_bus_id"].split(":")) == 3 and g["kernel_ms"] > 0
        assert g["setup_s"] > 0 and g["peak_rss_mib"] > 0
    cg = line["correctness_gate"]
    assert cg["distinct_devices"] == 1 and cg["every_rank_sha256_gated"] is True
    assert cg["setup_s_max"] >= max(g["setup_s"] for g in ranks)
    assert line["value"] > 0 and line["scaling"] == "weak"


def _ring_worker(rank, world, port, n, cfg, out_dir):
    """Each rank generates its index shard straight into the node's shared host ring (the e2e leg's layout,
    pollnet_amd/host_ring.py), from CPUs of its NUMA node when known, then writes the oracle's records for its
    shard into its slice of the ring's record array.  No exchange."""
    import sys

    sys.path.insert(0, ROOT)
    import pollnet_amd as pa
    from oracle import pyoracle as orc
    from pollnet_amd.host_ring import SharedHostRing, cpu_affinity
    from pollnet_amd.shard import shard_range

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ring = SharedHostRing(dist, rank, world, n, 2048)
    p = pa.rx.GenParams.for_config(cfg)
    lo, hi = shard_range(rank, world, n)
    cpus = sorted(os.sched_getaffinity(0))[rank::world]  # a stand-in for the GPU's node: a distinct CPU subset
    with cpu_affinity(cpus):
        assert set(os.sched_getaffinity(0)) == set(cpus)
        pa.gen_frames(p, n, first_index=lo, threads=2, out=ring.shard())
    assert set(os.sched_getaffinity(0)) != set(cpus) or len(cpus) == len(os.sched_getaffinity(0))
    t = pa.gen_conn_table(p)
    e, m = t.snapshot()
    rec = orc.classify_batch(ring.shard(), 2048, 2, n, e, m, t.max_conn_cnt)
    ring.records()[:] = rec.view(np.uint8)
    dist.barrier()
    if rank == 0:  # the whole ring and record array, as one process on the node sees them
        np.save(os.path.join(out_dir, "ring.npy"), ring.slots().copy())
        np.save(os.path.join(out_dir, "records.npy"), np.concatenate([ring.records(r) for r in range(world)]))
        with open(os.path.join(out_dir, "name.txt"), "w") as f:
            f.write(ring.shm.name)
    ring.close(dist)
    dist.destroy_process_group()


def test_shared_host_ring_shards_assemble(tmp_path):
    """World-size-2 gloo: the ranks' shards of the shared host ring assemble into the global ring the generator
    makes in one process, the record slices into the single-process records, and the segment is unlinked at close."""
    import sys

    sys.path.insert(0, ROOT)
    import pollnet_amd as pa
    from oracle import pyoracle as orc

    world, n, cfg = 2, 2048, 4
    mp.spawn(_ring_worker, args=(world, _free_port(), n, cfg, str(tmp_path)), nprocs=world, join=True)
    p = pa.rx.GenParams.for_config(cfg)
    full = pa.gen_frames(p, world * n, threads=4)
    assert np.array_equal(np.load(tmp_path / "ring.npy"), full)
    t = pa.gen_conn_table(p)
    e, m = t.snapshot()
    exp = orc.classify_batch(full, 2048, 2, world * n, e, m, t.max_conn_cnt)
    assert np.array_equal(np.load(tmp_path / "records.npy"), exp.view(np.uint8))
    assert not os.path.exists("/dev/shm/" + open(tmp_path / "name.txt").read().strip())


def test_device_numa_lookup():
    """sysfs lookup of a PCI device's node: an absent device is (-1, []), never an exception."""
    import sys

    sys.path.insert(0, ROOT)
    from pollnet_amd.host_ring import _cpulist, device_numa

    assert device_numa(0xffff, 0xff, 0x1f) == (-1, [])
    assert _cpulist("0-3,8,10-11") == [0, 1, 2, 3, 8, 10, 11]


@pytest.mark.gpu
def test_bench_e2e_host_ring_two_ranks():
    """`bench.py --gpus 2 --e2e` under the driver's torchrun command on this box's one GPU: the end-to-end leg's
    plumbing (one shared host ring, each rank's C4 shard of 2 Mi frames first-touched on its GPU's NUMA node,
    hipHostRegister-ed and classified in place, records into the ring) with every shard gated: each rank's batches
    hash to its shard's committed digest, and its ring records equal its device-resident records, in both modes.
    Both ranks share one GPU and one PCIe link here, so the aggregate says nothing about 2 GPUs' PCIe."""
    import json
    import socket
    import subprocess
    import sys

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3",
           "--warmup", "1", "--batches", "2", "--e2e"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.strip().splitlines() if ln.startswith("{")]
    line = json.loads(lines[-1])
    assert line["verified_vs_oracle"] is True and line["correctness_gate"]["every_rank_sha256_gated"] is True
    e2e = line["e2e_host_ring"]
    assert "error" not in e2e, e2e
    for mode in ("verified", "release_path"):
        assert e2e[mode]["every_rank_records_ok"] is True, e2e[mode]
        assert [r["rank"] for r in e2e[mode]["ranks"]] == [0, 1]
        assert e2e[mode]["gbit_per_s"] > 0
    assert e2e["frames_per_rank"] == 1 << 21
    assert line["summary"]["e2e_host_ring_records_ok"] is True
    assert list(line)[-1] == "summary"


def test_shared_host_ring_refuses_what_does_not_fit():
    """A ring larger than /dev/shm's free space (or half the host's available memory) is refused before anything is
    created (a tmpfs filling up under a mapping would kill the writer with SIGBUS); bench.py then skips the e2e leg."""
    import sys

    sys.path.insert(0, ROOT)
    from pollnet_amd.host_ring import SharedHostRing, room_for

    assert room_for(1 << 20) is None
    assert "GiB" in room_for(1 << 50)
    with pytest.raises(RuntimeError, match="no shared host ring"):
        SharedHostRing(None, 0, 1, 1 << 40, 2048)


def test_server_rounds_median_legs():
    """bench.py's server placements run in rounds; each leg is reported from its median round with every round's
    rate beside it, `delivered_ok` only if every round delivered, and the summary takes the hot pair from them."""
    import importlib.util
    import sys

    sys.path.insert(0, ROOT)
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    leg = "gpu_rxbatch_512_pipelined_resident_release_path"
    ref = "reference_server_release_build"
    rows = [{leg: {"mframes_per_s": g, "mframes_per_s_server_only": g + 10}, ref: {"mframes_per_s": r,
             "mframes_per_s_server_only": r + 10}, "delivered_ok": ok}
            for g, r, ok in ((58.0, 54.0, True), (12.0, 53.0, True), (61.0, 55.0, True))]
    m = bench.median_legs(rows)
    assert m[leg]["mframes_per_s"] == 58.0 and m[leg]["rounds_mframes_per_s"] == [58.0, 12.0, 61.0]
    assert m[ref]["mframes_per_s"] == 54.0 and m["delivered_ok"] is True and m["rounds"] == 3
    rows[1]["delivered_ok"] = False
    assert bench.median_legs(rows)["delivered_ok"] is False
    s = bench.summary({"value": 1.0, "unit": "Gbit/s", "n_gpus": 1, "secondary": {"tcp_server_poll": {"hot": m}}})
    assert s["server_hot_pair_median3_mfps"] == [58.0, 54.0]
    assert s["server_hot_frames_resident_vs_reference_mfps"] == [68.0, 64.0]
