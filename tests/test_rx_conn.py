"""Receive-side state machine (include/pollnet_amd/rx_conn.hpp), host only.

Runs tests/cpp/test_rx_conn: onPack-only scenarios (TcpConn.h:475-764, expected
values worked out line by line) and a differential of the shared reassembly core
against the reference's own TcpStream.h compiled into oracle/_ref (300 random
segment streams with reordering, duplicates, re-segmented retransmissions and
message-granular handlers)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "test_rx_conn")
REF = os.path.join(ROOT, "oracle", "_ref", "libref_tcpstream.so")


def _run(*args):
    if not os.path.exists(BIN):
        subprocess.run(["make", "-C", ROOT, "tests/cpp/test_rx_conn"], check=True, capture_output=True)
    return subprocess.run([BIN, *args], capture_output=True, text=True, timeout=300)


def test_rx_conn_scenarios_and_reference_differential():
    if not os.path.exists(REF):
        pytest.skip("oracle/_ref/libref_tcpstream.so not built (needs /root/reference)")
    p = _run(REF, "300")
    assert p.returncode == 0, p.stdout + p.stderr
    assert "part B: ok" in p.stdout
    assert "part A: 300/300 streams identical" in p.stdout, p.stdout


def test_sequential_server_twin_delivers_every_stream():
    """The reference-semantics twin of tests/cpp/test_gpu_tcp_rx alone (no GPU): 200
    flows with SYN / reordered, duplicated, corrupted-then-resent data / FIN, TIME_WAIT
    and unknown flows — every stream delivered intact, every flow disconnected."""
    b = os.path.join(ROOT, "tests", "cpp", "test_gpu_tcp_rx")
    if not os.path.exists(b):
        subprocess.run(["make", "-C", ROOT, "tests/cpp/test_gpu_tcp_rx"], check=True, capture_output=True)
    p = subprocess.run([b, "1000", "twin"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "200/200 streams intact, 200 disconnects" in p.stdout
