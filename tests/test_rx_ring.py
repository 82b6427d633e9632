"""RX-ring ingestion (include/pollnet_amd/rx_ring.hpp) via
tests/cpp/test_rx_ring: the SocketEthReceiver-style batcher over a message-preserving
socket pair (5,000 C5 frames intact, oversize frames cut at the slot), live AF_PACKET
capture of a loopback TCP stream when the process may open packet sockets (the
64,000-B stream rebuilt from the captured frames), and on a GPU the zero-copy
classification of the socket-filled batch and of an ef_vi RecvBuf ring driven by a
wrapping RX-event run with discards (pn_classify_indexed), record for record against
the oracle."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "test_rx_ring")


def _run(mode):
    if not os.path.exists(BIN):
        subprocess.run(["make", "-C", ROOT, "tests/cpp/test_rx_ring"], check=True, capture_output=True)
    return subprocess.run([BIN, mode], capture_output=True, text=True, timeout=300)


def test_socket_batcher_and_loopback_capture():
    p = _run("cpu")
    assert p.returncode == 0, p.stdout + p.stderr
    assert "5000/5000 frames intact" in p.stdout
    assert "stream rebuilt intact" in p.stdout or "lo capture: SKIPPED" in p.stdout, p.stdout


@pytest.mark.gpu
def test_ingested_batches_on_gpu():
    p = _run("all")
    assert p.returncode == 0, p.stdout + p.stderr
    assert "zero-copy: 5000 records, 0 differ" in p.stdout, p.stdout
    assert "RX events over 3 laps" in p.stdout and ", 0 differ" in p.stdout.split("ef_vi ring")[1], p.stdout
