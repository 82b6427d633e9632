"""Code-generation checks on the product kernels (CPU only: hipcc cross-compiles gfx950 device code to
assembly).  They pin two round-3 findings against regressions the parity tests cannot see:

- no waterfall loops: a buffer descriptor built from a value the compiler thinks is per-lane is wrapped in a
  readfirstlane / v_cmp_eq_u64 / exec-mask loop around every load and store that uses it (the LDS-pad test's
  per-lane write to a.n did that to every RX descriptor);
- the RX cooperative window's 8 loads go out before the first wait (with a branch around each load the
  compiler waited for each one before issuing the next: 8 dependent HBM round trips per wave)."""
import functools
import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


@functools.lru_cache(maxsize=None)
def _asm(src):
    # the tuning library is built with its A/B variants (Makefile TUNING=1: -DPN_TUNING_VARIANTS)
    extra = ["-DPN_TUNING_VARIANTS"] if "tuning" in src else []
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, os.path.basename(src) + ".s")
        subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "--cuda-device-only", "-S",
                        *extra, os.path.join(ROOT, "pollnet_amd", "csrc", src), "-o", out], check=True,
                       capture_output=True)
        with open(out) as f:
            return f.read()


def _kernels(asm):
    """{symbol: body lines} for every kernel in an assembly listing."""
    out, cur = {}, None
    for line in asm.splitlines():
        m = re.match(r"^(_Z\S+):", line)
        if m and "kernel" in m.group(1):
            cur = m.group(1)
            out[cur] = []
            continue
        if cur and line.startswith(".Lfunc_end"):
            cur = None
        elif cur:
            out[cur].append(line)
    return out


pytestmark = pytest.mark.skipif(not os.path.exists(HIPCC), reason="needs hipcc")


@pytest.mark.parametrize("src", ["rx_kernel.hip", "stream_kernel.hip", "tx_kernel.hip", "rx_tuning.hip",
                                 "tx_tuning.hip"])
def test_no_waterfall_loops(src):
    """Product kernels and the measurement library's ceilings and A/B variants alike: a variant with a
    waterfall loop would time that defect instead of the change it is meant to measure."""
    ks = _kernels(_asm(src))
    assert ks
    bad = [k for k, body in ks.items() if any(re.match(r"\s+v_cmp_eq_u64_e\d+ vcc, s\[", l) for l in body)]
    assert not bad, f"{len(bad)} kernels with a divergent descriptor (waterfall loop), e.g. {bad[0]}"


def test_service_kernel_waterfalls_only_its_record_store():
    """The resident service kernel (rx_service.hip) inlines the classify of both paths beside its own loop state, and
    at that SGPR pressure the compiler keeps the record store's block index in a VGPR: one waterfall loop per kernel,
    around that store, one iteration (the value is uniform).  Taking the classify out of line removes it but costs
    more: 64 frames 3.5-3.8 -> 4.8-5.2 us on the release path, 7.5-8.2 -> 9.7-10.5 verified
    (profiles/r05/service/inline_vs_call_ab.txt).  Pinned here so that a second one shows up.  Round 6: the large
    posts' helper kernel (the same classify call) is held to the same."""
    ks = _kernels(_asm("rx_service.hip"))
    assert len(ks) == 32
    assert sum("rx_service_helper_kernel" in k for k in ks) == 16
    for k, body in ks.items():
        at = [i for i, l in enumerate(body) if re.match(r"\s+v_cmp_eq_u64_e\d+ vcc, s\[", l)]
        assert len(at) <= 1, (k, len(at))
        for i in at:
            assert any("buffer_store_dwordx4" in l for l in body[i:i + 14]), k


def test_rx_window_loads_issued_together():
    ks = _kernels(_asm("rx_kernel.hip"))
    # the strided production kernels with the cooperative window (COOP = 1, IDX = 0)
    coop = {k: b for k, b in ks.items() if re.search(r"rx_classify_kernelILi\d+ELi1ELi\d+ELi2ELi16ELi0E", k)}
    assert len(coop) >= 8
    for k, body in coop.items():
        first_wait = next(i for i, l in enumerate(body) if "s_waitcnt vmcnt" in l)
        loads = [l for l in body[:first_wait] if "buffer_load_dwordx4" in l]
        assert len(loads) == 8, (k, len(loads))
