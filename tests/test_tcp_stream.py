"""TcpStream filter + reassembly (include/pollnet_amd/tcp_stream.hpp, SURVEY §8(f)
rank 3) against the reference's own TcpStream.h compiled into oracle/_ref.

CPU: StreamReassembler vs TcpStream<WaitForResend, BUFSIZE> for true/false x 1 MiB /
4 KiB — 800 random sniffed streams (SYN restarts, reordering past 5 extents,
duplicates, re-segmentation, losses, buffer overruns, message-granular handlers):
every packet's return value, handler-call size and consumed byte identical.
GPU: pn_match_streams vs TcpStream::filterPacket (first accepting filter of 8
overlapping wildcard filters over TCP/UDP/ARP/IPv6/IHL=6 traffic), and GpuTcpStreams
(copy / zero-copy, 3 chunk sizes) vs reference TcpStreams fed frame by frame."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref", "libref_tcpstream.so")


def _bin(name):
    b = os.path.join(ROOT, "tests", "cpp", name)
    if not os.path.exists(b):
        subprocess.run(["make", "-C", ROOT, f"tests/cpp/{name}"], check=True, capture_output=True)
    return b


def test_reassembler_vs_reference_tcpstream():
    if not os.path.exists(REF):
        pytest.skip("oracle/_ref/libref_tcpstream.so not built (needs /root/reference)")
    p = subprocess.run([_bin("test_tcp_stream"), REF, "200"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "800/800 streams identical" in p.stdout, p.stdout
    # GpuTcpStreams' host filter (later streams of a frame) equals the reference's filterPacket
    assert "filterPacket: 200000 frames" in p.stdout and " 0 differ from the reference" in p.stdout, p.stdout


@pytest.mark.gpu
def test_gpu_match_and_streams_vs_reference():
    assert os.path.exists(REF), "oracle/_ref/libref_tcpstream.so must travel with the repo"
    p = subprocess.run([_bin("test_gpu_tcp_stream"), REF], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "PASS" in p.stdout and " 0 ids differ" in p.stdout, p.stdout
    # both delivery modes (every accepting stream, as independent TcpStreams; first match only), 2 x 3 chunkings each
    assert p.stdout.count("8/8 streams identical") == 12, p.stdout
    assert p.stdout.count("every matching stream): 8/8") == 6, p.stdout
