"""GpuTcpServer (include/pollnet_amd/tcp_server.hpp): pollnet's EfviTcpServer surface
(EfviTcp.h:177-309) over the GPU RX/TX paths, driven by the reference example's own
handler (example/tcpserver.cc:61-90, compiled unchanged; tests/cpp/test_tcp_server.cpp).

CPU: the sequential twin (oracle classification against the live table) alone — the
server logic: handshakes, echo through writeNonblock, RSTs to unknown flows and after
close, every stream echoed intact, every TX frame's checksums valid.
GPU: the same traffic through pn_classify / pn_tx_fill at several frames-per-poll; the
handler log and every TX frame must equal the twin's."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "test_tcp_server")


def _run(*args):
    if not os.path.exists(BIN):
        if not os.path.isdir("/root/reference"):
            pytest.skip("tests/cpp/test_tcp_server not built (its handler text comes from /root/reference)")
        subprocess.run(["make", "-C", ROOT, "tests/cpp/test_tcp_server"], check=True, capture_output=True)
    return subprocess.run([BIN, *args], capture_output=True, text=True, timeout=300)


@pytest.mark.parametrize("per_poll", [1, 64, 512, 5000])
def test_server_twin_example_handler(per_poll):
    p = _run("twin", str(per_poll))
    assert p.returncode == 0, p.stdout + p.stderr
    assert "200/200 echoes intact, 0 bad checksums" in p.stdout, p.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("per_poll", [1, 37, 512, 8192])
def test_gpu_server_matches_twin(per_poll):
    p = _run("gpu", str(per_poll))
    assert p.returncode == 0, p.stdout + p.stderr
    assert "gpu: handler log identical, TX frames identical" in p.stdout, p.stdout


PEER = os.path.join(ROOT, "tests", "cpp", "test_tcp_server_peer")


def _peer(mode, populations=1, env=None):
    if not os.path.exists(PEER):
        subprocess.run(["make", "-C", ROOT, "tests/cpp/test_tcp_server_peer"], check=True, capture_output=True)
    return subprocess.run([PEER, mode, str(populations)], capture_output=True, text=True, timeout=300,
                          env=None if env is None else {**os.environ, **env})


def test_server_twin_reactive_peers():
    """120 reactive in-memory TCP clients with 3 % loss each way and a 1-ms-per-poll
    clock: handshake / SYN-ACK and RTO retransmission, delayed ACKs, window-limited
    sends, receive timeouts, admission refusal, server FINs — echoes intact, idle flows
    timed out, nothing left open (sequential twin alone, no GPU); 6 populations and loss
    patterns, 4 RX modes each."""
    p = _peer("twin", 6)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "PASS" in p.stdout


@pytest.mark.gpu
def test_gpu_server_reactive_peers_match_twin():
    """The same on the GPU backend, 4 populations x 8 RX modes (every poll, latency budget,
    chunks, pipelined one and two polls deep, and the resident service every poll and pipelined one and two
    polls deep): handler log and every TX frame equal to the twin's in each run."""
    p = _peer("gpu", 4)
    assert p.returncode == 0, p.stdout + p.stderr
    assert p.stdout.count("gpu: handler log identical, TX frames identical") == 32, p.stdout


@pytest.mark.gpu
def test_gpu_server_resident_post_ids_wrap():
    """The resident-service modes with the service's post counter started 16 below 2^32 (PN_SERVICE_FIRST_POST):
    every run's posts cross the wrap (post id 0 included, which GpuRx once took for "no post outstanding"), and the
    handler log and every TX frame still equal the twin's."""
    p = _peer("gpu", 1, env={"PN_SERVICE_FIRST_POST": str(0xFFFFFFF0)})
    assert p.returncode == 0, p.stdout + p.stderr
    assert p.stdout.count("gpu: handler log identical, TX frames identical") == 8, p.stdout


@pytest.mark.gpu
def test_gpu_server_resident_host_mailbox():
    """The resident-service modes with the service's mailbox in pinned host memory (PN_SERVICE_HOST_MAILBOX: the
    path a device without a large BAR takes): handler log and every TX frame equal to the twin's."""
    p = _peer("gpu", 1, env={"PN_SERVICE_HOST_MAILBOX": "1"})
    assert p.returncode == 0, p.stdout + p.stderr
    assert p.stdout.count("gpu: handler log identical, TX frames identical") == 8, p.stdout


CLISRV = os.path.join(ROOT, "tests", "cpp", "test_tcp_client_server")


def _clisrv(mode, runs=1):
    if not os.path.exists(CLISRV):
        if not os.path.isdir("/root/reference"):
            pytest.skip("tests/cpp/test_tcp_client_server not built (its handler texts come from /root/reference)")
        subprocess.run(["make", "-C", ROOT, "tests/cpp/test_tcp_client_server"], check=True, capture_output=True)
    return subprocess.run([CLISRV, mode, str(runs)], capture_output=True, text=True, timeout=300)


def test_client_server_twin_reference_examples():
    """GpuTcpClient <-> GpuTcpServer over a lossy in-memory wire, running the reference's
    example client and server handlers (tcpclient.cc:68-95, tcpserver.cc:61-90) unchanged:
    connect, 1-s send timeouts echoed in order, close, reconnect (sequential backends);
    8 loss patterns.  Each classify-every-poll run is also run with both ends as the reference's
    own EfviTcpServer / EfviTcpClient (oracle/ref_server.hpp: efvitcp's TcpServer, TcpClient,
    TcpConn and Core compiled from /root/reference): every wire frame and both logs identical."""
    p = _clisrv("twin", 8)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "PASS" in p.stdout
    assert p.stdout.count("twin vs reference EfviTcpServer/EfviTcpClient: handler logs identical, wire frames "
                          "identical") == 8, p.stdout


@pytest.mark.gpu
def test_gpu_client_server_match_twin():
    """Both ends on the GPU backend, 4 loss patterns, classify-every-poll and pipelined RX: logs
    and wire frames equal the twin's."""
    p = _clisrv("gpu", 4)
    assert p.returncode == 0, p.stdout + p.stderr
    assert p.stdout.count("gpu: handler logs identical, wire frames identical") == 4, p.stdout
    assert p.stdout.count("gpu (pipelined): handler logs identical, wire frames identical") == 4, p.stdout


TXHOST = os.path.join(ROOT, "tests", "cpp", "test_tx_host")


def test_engine_host_tx_checksums_equal_oracle_fill():
    """The engine's host-side checksums for header-only TX batches (srv_detail::fill_tcp_checksums)
    equal the oracle's PN_TX_TCP fill — itself pinned to the reference's copyAndSum / setOptDataLen
    (tests/test_tx.py) — on 20,000 random frames, every tot_len 40..1500, frames below the headers
    untouched."""
    if not os.path.exists(TXHOST):
        subprocess.run(["make", "-C", ROOT, "tests/cpp/test_tx_host"], check=True, capture_output=True)
    p = subprocess.run([TXHOST, "20000"], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0 and "PASS" in p.stdout, p.stdout + p.stderr


SRVBENCH = os.path.join(ROOT, "bench", "bench_tcp_server")


def test_server_bench_release_pair_cpu():
    """bench_tcp_server's host-side legs (no GPU): the sequential twin on the release path, the same pipelined with
    its classify / dispatch split timed, and -- where the reference's text was present at build -- the reference's
    own server (oracle/ref_server.hpp) on the same workload, 64 events per pollNet.  Every leg must deliver every
    byte (no RST, no disconnect), and the reference leg must ACK every second segment as the engine does."""
    import json

    if not os.path.exists(SRVBENCH):
        subprocess.run(["make", "-C", ROOT, "bench/bench_tcp_server"], check=True, capture_output=True)
    p = subprocess.run([SRVBENCH, "256", "40", "release_pair"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["delivered_ok"] is True
    timed = line["cpu_rxbatch_512_pipelined_release_path_timed"]
    assert timed["ns_per_frame_dispatch"] > 0 and timed["ns_per_frame_classify"] > 0
    assert line["cpu_rxbatch_512_release_path"]["acks_per_frame"] == pytest.approx(0.5, abs=0.01)
    if os.path.exists(os.path.join(ROOT, "oracle", "_ref", "conn_efvitcpserver.inc")):
        ref = line["reference_server_release_build"]
        assert ref["mframes_per_s"] > 0 and ref["acks_per_frame"] == pytest.approx(0.5, abs=0.01)


def test_server_bench_echo_cpu_legs():
    """bench_tcp_server echo (the reference example's echo server: every delivery written back, the peers
    acknowledging it): the sequential twin and the reference's own server echo every byte they receive (no
    refused write, no RST); the GPU legs need a GPU and are skipped here (they report an error without one)."""
    import json

    if not os.path.exists(SRVBENCH):
        subprocess.run(["make", "-C", ROOT, "bench/bench_tcp_server"], check=True, capture_output=True)
    p = subprocess.run([SRVBENCH, "256", "30", "echo"], capture_output=True, text=True, timeout=300)
    line = json.loads(p.stdout.strip().splitlines()[-1])
    twin = line["cpu_echo_512_release_path"]
    assert "error" not in twin, twin
    assert twin["echo_payload_gbit_per_s"] > 0
    if os.path.exists(os.path.join(ROOT, "oracle", "_ref", "conn_efvitcpserver.inc")):
        ref = line["reference_server_echo_release_build"]
        assert "error" not in ref, ref
        assert ref["echo_payload_gbit_per_s"] > 0
