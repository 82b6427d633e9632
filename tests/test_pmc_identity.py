"""The committed PMC traffic (profiles/pmc_traffic.json) belongs to the code it was measured on (CPU only).

Every entry bench.py reports `roofline.traffic` / `traffic` from records the sha256 of each kernel's gfx950 machine
code in the library that ran (pollnet_amd/codehash.py, written by scripts/pmc_refresh.py).  This test fails when a
production kernel changed without a PMC refresh (scripts/pmc_refresh.sh on a GPU box, then scripts/pmc_refresh.py):
the bench would then report the entry's bytes as null with traffic_stale true."""
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "pollnet_amd", "libpollnet_amd.so")
# every entry bench.py reads (load_pmc): the headline (C2; C4 at N > 1), C3, C5, the release path, the filter, TX
BENCH_KEYS = ["c2_n1048576", "c4_n2097152", "c3_n1048576", "c5_n1048576", "c2_release_path_n1048576",
              "match_streams_c2_n1048576", "tx_c2_n1048576/frame_off_2", "tx_c2_n1048576/frame_off_14"]


def _entries():
    with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
        d = json.load(f)
    out = {}
    for k in BENCH_KEYS:
        key, _, sub = k.partition("/")
        e = d.get(key)
        out[k] = e.get(sub) if (e is not None and sub) else e
    return out


pytestmark = pytest.mark.skipif(not os.path.exists(LIB), reason="libpollnet_amd.so not built (make)")


@pytest.mark.parametrize("key", BENCH_KEYS)
def test_pmc_entry_is_of_the_built_kernels(key):
    from pollnet_amd import codehash

    e = _entries()[key]
    assert e is not None, f"no committed PMC entry {key}"
    ok, why = codehash.check_entry(e)
    assert ok, f"{key}: {why} -- refresh with scripts/pmc_refresh.sh on a GPU box"
    assert e["hbm_bytes_per_launch"] > 0 and e["frames_per_launch"] > 0


def test_kernel_hashes_cover_the_product_and_tuning_kernels():
    from pollnet_amd import codehash

    h = codehash.kernel_hashes(LIB)
    fams = ("rx_classify_kernel<", "match_streams_mask_kernel<", "tx_fill_kernel<", "tx_patch_kernel<")
    for f in fams:
        assert any(f in k for k in h), f
    assert all(len(v) == 16 for v in h.values())
    t = codehash.kernel_hashes(os.path.join(ROOT, "pollnet_amd", "libpollnet_amd_tuning.so"))
    assert any("calib_stream_read_kernel" in k for k in t)


def test_a_changed_kernel_is_reported_stale():
    from pollnet_amd import codehash

    e = dict(_entries()["c2_n1048576"])
    name = next(iter(e["kernels"]))
    e["kernels"] = dict(e["kernels"], **{name: "0" * 16})
    ok, why = codehash.check_entry(e)
    assert not ok and "changed" in why
    ok, why = codehash.check_entry({k: v for k, v in e.items() if k != "kernels"})
    assert not ok and "no kernel code hashes" in why


def test_bench_reports_stale_traffic_as_null(monkeypatch):
    """bench.py's pmc_fields: current code -> the committed bytes; changed code -> null, traffic_stale true."""
    import sys

    sys.path.insert(0, ROOT)
    import bench

    cur = bench.load_pmc("c2_n1048576")
    f = bench.pmc_fields(cur, 0.25)
    assert f["traffic"] == cur["hbm_bytes_per_launch"] and f["traffic_stale"] is False and f["traffic_gbs"] > 0
    stale = dict(cur, code_current=False, code_check="1 of 1 kernels changed")
    f = bench.pmc_fields(stale, 0.25)
    assert f["traffic"] is None and f["traffic_over_algorithmic"] is None and f["traffic_stale"] is True
    assert f["traffic_gbs"] is None
    assert bench.pmc_fields(None)["traffic"] is None
