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
@pytest.mark.parametrize("batch", [1000, 64, 1, 8192])
def test_gpu_tcp_rx_matches_sequential_twin(batch):
    assert os.path.exists(BIN), "tests/cpp/test_gpu_tcp_rx not built (make)"
    p = subprocess.run([BIN, str(batch)], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "PASS" in p.stdout and "200/200 streams" in p.stdout, p.stdout
