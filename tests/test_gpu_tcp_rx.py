"""GPU: the receive-side server loop (include/pollnet_amd/gpu_tcp_rx.hpp) against a
sequential twin with the reference's semantics (tests/cpp/test_gpu_tcp_rx.cpp).

Batch sizes cut flows at different places so that connections open (SYN ->
accept) and close (FIN -> table delete) mid-batch, which exercises the host
re-resolution of records classified against an older table snapshot.  The callback
logs must be identical event for event, and every stream must arrive intact."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "test_gpu_tcp_rx")


@pytest.mark.gpu
@pytest.mark.parametrize("batch,mode,span", [(1000, "copy", ""), (64, "copy", ""), (1, "copy", ""),
                                             (8192, "zc", ""), (1000, "zc", ""), (64, "zc", "span"),
                                             (700, "copy", "span"), (500, "idx", ""), (128, "idx", "span")])
def test_gpu_tcp_rx_matches_sequential_twin(batch, mode, span):
    assert os.path.exists(BIN), "tests/cpp/test_gpu_tcp_rx not built (make)"
    p = subprocess.run([BIN, str(batch), mode] + ([span] if span else []), capture_output=True, text=True,
                       timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "PASS" in p.stdout and "200/200 streams" in p.stdout, p.stdout
