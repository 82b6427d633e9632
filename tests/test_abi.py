"""The C-ABI library loads and exports every symbol include/pollnet_amd.h declares;
host-side (no GPU) behaviour of the boundary."""
import ctypes
import os
import re

import numpy as np
import pytest

import pollnet_amd as pa

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "pollnet_amd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pn_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_and_library_exports_all():
    names = declared_functions()
    assert len(names) >= 20
    lib = ctypes.CDLL(pa.LIB_PATH)
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


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


def test_no_device_open_fails_loudly():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(pa.PollnetError):
        pa.RxContext(0)


def test_generator_rejects_bad_layout():
    with pytest.raises(pa.PollnetError):
        pa.gen_frames(pa.rx.GenParams.for_config(2), 4, slot_stride=64)
