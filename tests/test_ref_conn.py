"""F1 parity: the stateful onPack remainder and onTcpData delivery against the reference's OWN
efvitcp code (TcpConn.h:467-769, TcpServer.h:69-115, EfviTcp.h:188-313), compiled from
/root/reference into the test binaries by oracle/ref_server.hpp (only the ef_vi plumbing is
restated there; the text itself never leaves this container, the binaries do).

- tests/cpp/test_ref_conn: RxConn (the receive half) vs TcpConn::onPack, segment by segment,
  over 8 x 1300 random segment streams (4 receive-buffer sizes, TimestampOption on/off):
  reordering to 5+ extents, duplicates, overlaps, old data, data past the window, no-ACK / SYN /
  mid-stream FIN segments, FIN with data and beyond a hole, RSTs in and out of the window,
  handlers leaving bytes or consuming nothing (window full), oversize frames, stale TSvals
  (PAWS).  Handler calls, ACK / RST frames, the delayed-ACK timer and the state (extents,
  recv_buf_seq, fin_received, pending_ack, recent_ts) must be identical after every segment.
- tests/cpp/test_ref_server: GpuTcpServer vs the reference EfviTcpServer over reactive client
  populations (ordinary peers with loss; adversarial segment streams): every frame sent, byte
  for byte, and the handler log identical.  CPU: the engine on the sequential oracle backend;
  GPU: on GpuBackend (pn_classify + pn_tx_fill)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bin(name):
    b = os.path.join(ROOT, "tests", "cpp", name)
    if not os.path.exists(b):
        if not os.path.isdir("/root/reference"):
            pytest.skip(f"tests/cpp/{name} not built (the reference's text comes from /root/reference)")
        subprocess.run(["make", "-C", ROOT, f"tests/cpp/{name}"], check=True, capture_output=True)
    return b


def test_rx_conn_equals_reference_onpack():
    p = subprocess.run([_bin("test_ref_conn"), "1300"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    lines = [l for l in p.stdout.splitlines() if l.startswith("ConnRecvBufSize")]
    assert len(lines) == 8 and all("1300 streams" in l and "identical" in l for l in lines), p.stdout
    # the adversarial paths were taken (counts from the reference's own state)
    assert all("0 evictions" not in l and " 0 resets" not in l for l in lines), p.stdout
    assert sum("0 PAWS drops" not in l for l in lines) == 4, p.stdout


def test_server_twin_equals_reference_server():
    p = subprocess.run([_bin("test_ref_server"), "twin", "4"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert p.stdout.count("vs reference:") == 16, p.stdout
    # round 6: the twin with the chain links (orc_chain_links): frames through the in-order fast path, identical
    links = [l for l in p.stdout.splitlines() if l.startswith("twin with chain links vs reference:")]
    assert len(links) == 8 and all("through the in-order fast path" in l for l in links), p.stdout
    assert "DIFFERENT" not in p.stdout and p.stdout.rstrip().endswith("PASS"), p.stdout
    # the intended differences, each shown: NIC-queue buffers (2 cases), frames per poll, bad checksums
    assert p.stdout.count("-> as documented") == 4, p.stdout


@pytest.mark.gpu
def test_gpu_server_equals_reference_server():
    p = subprocess.run([_bin("test_ref_server"), "gpu", "3"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert p.stdout.count("GpuTcpServer (GPU backend) vs reference") == 6, p.stdout
    # and with the checksum discard off: the header-only kernel (pn_set_verify(ctx, 0)), the reference's release path
    assert p.stdout.count("GpuTcpServer (GPU backend, release path: no checksum verification) vs reference") == 6, p.stdout
    # and with the classify in the resident service (Conf::RxResident, pn_service_*), both paths
    assert p.stdout.count("GpuTcpServer (GPU backend, resident service) vs reference") == 6, p.stdout
    assert p.stdout.count("GpuTcpServer (GPU backend, resident service, release path) vs reference") == 6, p.stdout
    # and with the chain links of each post (Conf::RxLinks): the GPU's links drive the in-order fast path
    res = [l for l in p.stdout.splitlines() if l.startswith("GpuTcpServer (GPU backend, resident service, chain links")]
    assert len(res) == 12 and all("through the in-order fast path" in l for l in res), p.stdout
    assert "bad checksums (GPU backend):" in p.stdout and p.stdout.count("-> as documented") == 5, p.stdout
    assert "DIFFERENT" not in p.stdout and p.stdout.rstrip().endswith("PASS"), p.stdout


def test_client_twin_equals_reference_client():
    """GpuTcpClient vs the reference EfviTcpClient (tests/cpp/test_ref_client.cpp) against a scripted,
    adversarial server: SYN answered by a SYN-ACK, a wrong-ack SYN-ACK, RST|ACK, a bare RST, a bare SYN or
    silence; reconnects; adversarial data streams and FINs.  Every client frame and the handler log identical
    over 24 scripts (sequential backend)."""
    p = subprocess.run([_bin("test_ref_client"), "twin", "24"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert p.stdout.count("twin vs reference: ") == 24 and "DIFFERENT" not in p.stdout, p.stdout
    assert p.stdout.rstrip().endswith("PASS"), p.stdout


@pytest.mark.gpu
def test_gpu_client_equals_reference_client():
    """The same 8 scripts through GpuTcpClient on the GPU: per-poll classify, the release path, and the
    classify posted to the resident service (Conf::RxResident) on both paths."""
    p = subprocess.run([_bin("test_ref_client"), "gpu", "8"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert p.stdout.count("GpuTcpClient (GPU) vs reference") == 8 and "DIFFERENT" not in p.stdout, p.stdout
    assert p.stdout.count("GpuTcpClient (GPU, release path) vs reference") == 8, p.stdout
    assert p.stdout.count("GpuTcpClient (GPU, resident service) vs reference") == 8, p.stdout
    assert p.stdout.count("GpuTcpClient (GPU, resident, release path) vs reference") == 8, p.stdout
    assert p.stdout.rstrip().endswith("PASS"), p.stdout
