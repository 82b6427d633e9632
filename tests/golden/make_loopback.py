"""Capture real kernel-generated Ethernet/IPv4/TCP frames on `lo` (AF_PACKET) for
the golden fixtures: tests/golden/loopback_frames.npz.

Why: the reference has no tests or vectors, and efvitcp/Core.h cannot be built
here (ef_vi headers absent).  Linux-generated frames give an independent pin:
  - every IPv4 header checksum is valid (Core::checksum's 20-byte IP sum,
    Core.h:451-453, must fold to 0);
  - TCP on loopback is CHECKSUM_PARTIAL: the checksum field holds the folded
    pseudo-header sum (src, dst, proto 6, tcp length) that a NIC would finish,
    which pins the pseudo-header words of Core.h:460-464;
  - SYN/ACK frames carry TCP options (doff 8/10), exercising payload_off.
Run once in the build container (needs CAP_NET_RAW); the output is committed.
"""
import os
import socket
import struct
import threading
import time

import numpy as np


def capture():
    s = socket.socket(socket.AF_PACKET, socket.SOCK_RAW, socket.htons(0x0003))
    s.bind(("lo", 0))
    s.settimeout(0.5)
    srv = socket.socket()
    srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)
    port = srv.getsockname()[1]

    def server():
        c, _ = srv.accept()
        while True:
            d = c.recv(65536)
            if not d:
                break
            c.sendall(d)
        c.close()

    threading.Thread(target=server, daemon=True).start()
    cl = socket.create_connection(("127.0.0.1", port))
    # payload sizes chosen to give odd and even TCP lengths, all < 1500 B
    for i, n in enumerate([1, 2, 3, 100, 137, 511, 512, 999, 1000, 1400, 1447, 1448]):
        cl.sendall(bytes((i * 7 + k) & 255 for k in range(n)))
        got = 0
        while got < n:
            got += len(cl.recv(65536))
    cl.close()
    time.sleep(0.3)
    frames = []
    while True:
        try:
            d, addr = s.recvfrom(70000)
        except socket.timeout:
            break
        if addr[2] == socket.PACKET_OUTGOING:
            continue
        if len(d) >= 54 and d[12:14] == b"\x08\x00" and d[23] == 6 and len(d) <= 1514:
            sp, dp = struct.unpack("!HH", d[34:38])
            if port in (sp, dp):
                frames.append(d)
    return frames


def main():
    frames = capture()
    assert frames, "no frames captured"
    stride, off = 2048, 2
    slots = np.zeros((len(frames), stride), np.uint8)
    for i, f in enumerate(frames):
        slots[i, off:off + len(f)] = np.frombuffer(f, np.uint8)
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "loopback_frames.npz")
    np.savez_compressed(out, slots=slots, lengths=np.array([len(f) for f in frames], np.uint32), stride=stride,
                        frame_off=off)
    print(f"wrote {len(frames)} frames to {out}")


if __name__ == "__main__":
    main()
