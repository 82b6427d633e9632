"""The C-ABI library loads and exports every symbol include/pollnet_amd.h declares;
host-side (no GPU) behaviour of the boundary."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import pollnet_amd as pa

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions(header="pollnet_amd.h"):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pn_[a-z0-9_]+)\s*\(", src)))


def exported_functions(lib_path):
    out = subprocess.run(["nm", "-D", "--defined-only", lib_path], capture_output=True, text=True, check=True).stdout
    return sorted({ln.split()[-1] for ln in out.splitlines() if " T " in ln and ln.split()[-1].startswith("pn_")})


def test_header_declares_and_library_exports_all():
    names = declared_functions()
    assert len(names) >= 20
    lib = ctypes.CDLL(pa.LIB_PATH)
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_product_exports_exactly_the_header():
    """The product library exports the C-ABI of include/pollnet_amd.h and nothing else:
    tuning variants and bandwidth ceilings live in libpollnet_amd_tuning.so."""
    assert exported_functions(pa.LIB_PATH) == declared_functions()


def test_generator_library_is_separate():
    """The seeded workload generator is its own library (include/pollnet_amd_gen.h), outside the
    product ABI."""
    gen = set(exported_functions(pa.rx.GEN_LIB_PATH))
    assert gen == set(declared_functions("pollnet_amd_gen.h")) == {"pn_gen_frames", "pn_gen_conn_table", "pn_wire_bytes"}
    assert not gen & set(exported_functions(pa.LIB_PATH))


def test_tuning_library_is_separate():
    from pollnet_amd import tuning

    tuned = set(exported_functions(tuning.LIB_PATH))
    declared = set(declared_functions("pollnet_amd_tuning.h"))
    assert {"pn_calib_stream_read", "pn_calib_slot_read", "pn_calib_slot_read_var"} <= tuned <= declared
    assert not tuned & set(declared_functions())
    src = open(os.path.join(ROOT, "pollnet_amd", "rx.py")).read() + open(os.path.join(ROOT, "pollnet_amd", "__init__.py")).read()
    assert "tuning" not in src  # the product package never loads the tuning library


def test_default_build_covers_every_native_binary():
    """`make` (what build() runs) builds every executable that bench.py and the tests start:
    the GPU box only gets what was built here."""
    out = subprocess.run(["make", "-C", ROOT, "-pn", "all"], capture_output=True, text=True).stdout
    all_line = next(ln for ln in out.splitlines() if ln.startswith("all:") and "libpollnet_amd.so" in ln)
    prereqs = set(all_line.split(":", 1)[1].split())
    used = set()
    for f in ["bench.py"] + [os.path.join("tests", t) for t in os.listdir(os.path.join(ROOT, "tests")) if t.endswith(".py")]:
        src = open(os.path.join(ROOT, f)).read()
        used |= {f"bench/{m}" for m in re.findall(r'"bench", "(bench_[a-z_]+)"', src)}
        used |= {f"tests/cpp/{m}" for m in re.findall(r'"cpp", "(test_[a-z_]+)"', src)}
    assert {"bench/bench_signal", "bench/bench_tcp_server", "tests/cpp/test_gpu_rx"} <= used
    assert used <= prereqs, sorted(used - prereqs)


def test_result_layout():
    assert pa.RESULT_DTYPE.itemsize == 16
    assert [pa.RESULT_DTYPE.fields[k][1] for k in ("conn_id", "seq", "payload_off", "payload_len", "flags", "tcp_fold")] == [
        0, 4, 8, 10, 12, 14]


def test_errors_follow_reference_convention():
    # negative rc + message, no exception across the ABI
    with pytest.raises(pa.PollnetError):
        pa.ConnTable(0, 0)
    t = pa.ConnTable(4, 4)
    t.add(5, 1)
    with pytest.raises(pa.PollnetError):
        t.add(5, 2)  # addConnEntry is only ever called for a missing key
    with pytest.raises(pa.PollnetError):
        t.delete(6)
    with pytest.raises(pa.PollnetError):
        t.add(pa.PN_EMPTY_KEY, 0)
    for i in range(7):
        t.add(100 + i, i)
    with pytest.raises(pa.PollnetError):
        t.add(1000, 9)  # MaxConn + MaxTW full


def test_set_verify_without_ctx_is_an_error():
    lib = ctypes.CDLL(pa.LIB_PATH)
    lib.pn_set_verify.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.pn_set_verify.restype = ctypes.c_int
    lib.pn_last_error.argtypes = [ctypes.c_void_p]
    lib.pn_last_error.restype = ctypes.c_char_p
    assert lib.pn_set_verify(None, 0) == -1  # PN_EINVAL
    assert b"pn_set_verify" in lib.pn_last_error(None)
    assert pa.rx.F.TCP_UNCHECKED == 0x8000  # PN_F_TCP_UNCHECKED, the flag the release path sets


def test_no_device_open_fails_loudly():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(pa.PollnetError):
        pa.RxContext(0)


def test_generator_rejects_bad_layout():
    with pytest.raises(pa.PollnetError):
        pa.gen_frames(pa.rx.GenParams.for_config(2), 4, slot_stride=64)


def test_product_never_reaches_the_oracle():
    """The product library links no oracle / reference code, and no product source names the
    oracle outside comments: the checker stays test infrastructure (tests/, smoke(), bench.py's
    cpu_baseline)."""
    out = subprocess.run(["readelf", "-d", pa.LIB_PATH], capture_output=True, text=True, check=True).stdout
    needed = re.findall(r"NEEDED\)\s+Shared library: \[([^\]]+)\]", out)
    assert needed and not [n for n in needed if "oracle" in n or "ref" in n], needed
    srcs = [os.path.join(d, f) for d in ("pollnet_amd", "pollnet_amd/csrc", "include", "include/pollnet_amd")
            for f in os.listdir(os.path.join(ROOT, d)) if f.endswith((".py", ".hip", ".hpp", ".cpp", ".h"))]
    assert len(srcs) > 15
    for f in srcs:
        src = open(os.path.join(ROOT, f)).read()
        if f.endswith(".py"):  # comments and docstrings may cite the oracle; code may not
            code = re.sub(r'#[^\n]*|""".*?"""', "", src, flags=re.S)
        else:  # C/C++: comments stripped, preprocessor lines (an #include) kept
            code = re.sub(r"//[^\n]*|/\*.*?\*/", "", src, flags=re.S)
        assert "oracle" not in code.lower(), f
