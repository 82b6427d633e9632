"""TX checksum fill: pn_tx_fill vs the reference's own incremental
checksum path, restated in oracle/pn_tx_oracle.c.

The reference never sums an outgoing frame in one pass: it folds CSum state carried by
the connection (TcpConn.h:149-186, 310-323, 422-428), the appended pieces
(copyAndSum, TcpConn.h:257-299), resendUna's in-place patch (TcpConn.h:771-785),
sumRst for RST / TIME_WAIT ACKs (Core.h:385-446), and Efvi's cached IPv4 sum
(Efvi.h:405-411, 611-621).  orc_tx_build_batch drives those restatements to build the
frames a reference sender puts on the wire; pn_tx_fill, which recomputes the checksums
from the frame bytes in one HBM pass, must reproduce them byte for byte.

The reference's own send-path byte work (TcpConn::copyAndSum, SendBuf::setOptDataLen and
CSum; Efvi's cached IPv4 sum and update_udp_pkt — compiled verbatim into
oracle/_ref/libref_core.so) builds data segments and datagrams too; the recomputation, and
pn_tx_fill on the GPU, reproduce those byte for byte.

CPU: the incremental path equals the byte recomputation (orc_tx_fill_batch) on every
frame kind; every TCP frame passes the reference's own debug self-check (Core::checksum,
Core.h:448-472, applied by Core::send :478); RFC 1071 known answer; Efvi's cache carry
defect.  GPU: pn_tx_fill vs both, all alignments, jumbo slots, ragged batches, and a
full-size C2 round trip through pn_classify.
"""
import numpy as np
import pytest

from oracle import pyoracle as orc

IP = 14  # offsets from the Ethernet header
TCP = 34
E_EMPTY = np.array([(1 << 63, 0, 0)] * 2, dtype=orc.ENTRY_DTYPE)


def scramble(slots, frame_off, mode, lens_too, seed=7):
    """Overwrite every field pn_tx_fill writes with junk (what a send buffer holds before the fold)."""
    rng = np.random.default_rng(seed)
    s = slots.copy()
    n = len(s)
    b = frame_off
    s[:, b + IP + 10:b + IP + 12] = rng.integers(0, 256, (n, 2), dtype=np.uint8)
    if mode == orc.TX_TCP:
        s[:, b + TCP + 16:b + TCP + 18] = rng.integers(0, 256, (n, 2), dtype=np.uint8)
    if lens_too:
        s[:, b + IP + 2:b + IP + 4] = rng.integers(0, 256, (n, 2), dtype=np.uint8)
        if mode != orc.TX_TCP:
            s[:, b + IP + 24:b + IP + 26] = rng.integers(0, 256, (n, 2), dtype=np.uint8)
    return s


def word_sum(b):
    b = bytes(b)
    if len(b) & 1:
        b += b"\0"
    return int(np.frombuffer(b, dtype="<u2").astype(np.uint64).sum())


def fold(s):  # CSum::fold (Core.h:94-98)
    r = (s >> 16) + (s & 0xFFFF)
    r += r >> 16
    return ~r & 0xFFFF


# ---------------------------------------------------------------- CPU (oracle) ----

@pytest.mark.parametrize("mode", [orc.TX_TCP, orc.TX_UDP_EFVI])
@pytest.mark.parametrize("lens_too", [True, False])
def test_reference_path_equals_byte_recompute(mode, lens_too):
    slots, lens, kinds = orc.tx_build_batch(0x7A11, 20000, mode=mode)
    if mode == orc.TX_TCP:
        assert set(np.unique(kinds)) == {0, 1, 2, 3, 4}, np.bincount(kinds)
    s = scramble(slots, 14, mode, lens_too)
    orc.tx_fill_batch(s, 2048, 14, len(s), lens if lens_too else None, mode)
    bad = np.nonzero((s != slots).any(1))[0]
    assert len(bad) == 0, f"{len(bad)} frames differ, kinds {np.bincount(kinds[bad], minlength=6)}"


def test_reference_frames_pass_reference_self_check():
    """Core::send runs Core::checksum on every outgoing frame in the debug build (Core.h:478)."""
    slots, lens, kinds = orc.tx_build_batch(0xC0DE, 20000)
    rec = orc.classify_batch(slots, 2048, 14, len(slots), E_EMPTY, 1, 1)
    f = rec["flags"]
    assert np.all(f & 0x0001), "IP_OK"  # CSum.add<20>(ip).fold() == 0
    assert np.all(f & 0x0800), "RFC_TCP_OK"  # pseudo-header + zero-padded segment
    tot = (slots[:, 14 + IP + 2].astype(np.int64) << 8) | slots[:, 14 + IP + 3]
    assert np.array_equal(tot - 40, lens.astype(np.int64))
    # the debug check's literal odd-length read (the byte after the segment, Core.h:113-117)
    # agrees wherever that byte is 0
    pad = slots[np.arange(len(slots)), np.minimum(14 + IP + tot, 2047)]
    zero_pad = ((tot & 1) == 0) | (pad == 0)
    assert np.all(f[zero_pad] & 0x0002)


def test_rfc1071_known_answer():
    """The classic IPv4 header 4500 0073 0000 4000 4011 [b861] c0a8 0001 c0a8 00c7."""
    hdr = bytes.fromhex("450000730000400040110000c0a80001c0a800c7")
    slot = np.zeros((1, 256), dtype=np.uint8)
    slot[0, 16:36] = np.frombuffer(hdr, dtype=np.uint8)
    slot[0, 16 + 2:16 + 4] = [0x00, 0x73]  # tot_len 115 (fits the slot)
    for mode in (orc.TX_UDP_EFVI, orc.TX_UDP):
        s = slot.copy()
        orc.tx_fill_batch(s, 256, 2, 1, None, mode)
        assert bytes(s[0, 16 + 10:16 + 12]) == bytes.fromhex("b861"), mode


def craft_udp_header(saddr_words, daddr_words, paylen):
    """Efvi's init_udp_pkt header (Efvi.h:590-636) with chosen address words (LE u16)."""
    ip = bytearray(20)
    ip[0] = 0x45
    ip[6:8] = (0x0040).to_bytes(2, "little")
    ip[8], ip[9] = 64, 17
    ip[12:16] = b"".join(int(w).to_bytes(2, "little") for w in saddr_words)
    ip[16:20] = b"".join(int(w).to_bytes(2, "little") for w in daddr_words)
    tot = 28 + paylen
    ip[2:4] = tot.to_bytes(2, "big")
    return bytes(ip)


def efvi_check(ip):
    """Efvi.h:405-411 + 615-617 restated in Python (a third formulation)."""
    words = np.frombuffer(ip, dtype="<u2").astype(np.int64)
    cache = int(words.sum()) - int(words[1]) - int(words[5])  # template: tot_len = check = 0
    cache = (cache >> 16) + (cache & 0xFFFF)
    cache += cache >> 16
    ipsum = cache + int(words[1])
    ipsum += ipsum >> 16
    return ~ipsum & 0xFFFF


def test_efvi_cache_carry_defect():
    """When the cached sum's first fold carries (c1 >= 0x10000), Efvi's `cache += cache >> 16`
    adds the carry again without clearing it: every header with that address pair gets a
    checksum one too small, which does not verify.  PN_TX_UDP_EFVI keeps it bit for bit,
    PN_TX_UDP writes CSum::fold."""
    # S = 0x1FFFF exactly: fixed words 0x0045 + 0x0040 + 0x1140 = 0x11C5; addresses make up the rest
    need = 0x1FFFF - 0x11C5
    saddr = [0xFFFF, need - 0xFFFF]
    ip = craft_udp_header(saddr, [0, 0], 100)
    words = np.frombuffer(ip, dtype="<u2").astype(np.int64)
    assert int(words.sum()) - int(words[1]) == 0x1FFFF
    slot = np.zeros((1, 256), dtype=np.uint8)
    slot[0, 16:36] = np.frombuffer(ip, dtype=np.uint8)
    got = {}
    for mode in (orc.TX_UDP_EFVI, orc.TX_UDP):
        s = slot.copy()
        orc.tx_fill_batch(s, 256, 2, 1, None, mode)
        got[mode] = int.from_bytes(bytes(s[0, 26:28]), "little")
        verify = fold(word_sum(s[0, 16:36]))
        assert (verify == 0) == (mode == orc.TX_UDP), (mode, hex(got[mode]))
    assert got[orc.TX_UDP_EFVI] == efvi_check(ip)
    assert got[orc.TX_UDP] == fold(int(words.sum()) - int(words[5]))
    assert got[orc.TX_UDP] == got[orc.TX_UDP_EFVI] + 1
    # and for headers whose first fold does not carry the two modes agree
    rng = np.random.default_rng(3)
    n_same = 0
    for _ in range(2000):
        ip = craft_udp_header(rng.integers(0, 1 << 16, 2), rng.integers(0, 1 << 16, 2), int(rng.integers(0, 1473)))
        w = np.frombuffer(ip, dtype="<u2").astype(np.int64)
        c = int(w.sum()) - int(w[1]) - int(w[5])
        if (c >> 16) + (c & 0xFFFF) < 0x10000:
            assert efvi_check(ip) == fold(int(w.sum()) - int(w[5]))
            n_same += 1
    assert n_same > 1900


def test_untouched_frames():
    """tot_len below the bare headers or past the slot: nothing written."""
    slots, lens, _ = orc.tx_build_batch(11, 64)
    s = scramble(slots, 14, orc.TX_TCP, False)
    tot = np.array([0, 39, 2034 - 14 + 1, 65535] + [60] * 60, dtype=np.uint16)
    s[:, 14 + IP + 2] = tot >> 8
    s[:, 14 + IP + 3] = tot & 0xFF
    before = s.copy()
    orc.tx_fill_batch(s, 2048, 14, 64, None, orc.TX_TCP)
    assert np.array_equal(s[:4], before[:4])
    assert not np.array_equal(s[4:], before[4:])
    # lens that wrap htons(40 + len) below 40 or beyond the slot
    s = before.copy()
    orc.tx_fill_batch(s, 2048, 14, 2, np.array([65500, 3000], dtype=np.uint16), orc.TX_TCP)
    assert np.array_equal(s[:2], before[:2])


# ---------------------------------------------------------------- GPU ----

def _gpu():
    import torch

    import pollnet_amd as pa

    assert torch.cuda.is_available()
    return torch, pa


def _fill_gpu(ctx, torch, slots, stride, frame_off, n, lens, mode):
    d = torch.from_numpy(slots.reshape(-1)).cuda()
    l = None if lens is None else torch.from_numpy(lens.astype(np.uint16).view(np.int16)).cuda()
    ctx.tx_fill(d, stride, frame_off, n, l, mode)
    torch.cuda.synchronize()
    return d.cpu().numpy().reshape(slots.shape)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("frame_off", [14, 2])
@pytest.mark.parametrize("lens_too", [True, False])
def test_gpu_fill_equals_reference_frames(mode, frame_off, lens_too):
    torch, pa = _gpu()
    ctx = pa.RxContext(0)
    build_mode = orc.TX_TCP if mode == 0 else orc.TX_UDP_EFVI
    slots, lens, kinds = orc.tx_build_batch(0xF111 + frame_off, 30000, frame_off=frame_off, mode=build_mode)
    s = scramble(slots, frame_off, build_mode, lens_too)
    got = _fill_gpu(ctx, torch, s, 2048, frame_off, len(s), lens if lens_too else None, mode)
    if mode == 2:  # CSum::fold: equal to Efvi's wherever Efvi's verifies
        exp = s.copy()
        orc.tx_fill_batch(exp, 2048, frame_off, len(s), lens if lens_too else None, orc.TX_UDP)
        assert np.array_equal(got, exp)
        efvi_ok = orc.classify_batch(slots, 2048, frame_off, len(slots), E_EMPTY, 1, 1)["flags"] & 1
        assert np.array_equal(got[efvi_ok != 0], slots[efvi_ok != 0])
    else:
        bad = np.nonzero((got != slots).any(1))[0]
        assert len(bad) == 0, f"{len(bad)} frames differ (kinds {np.bincount(kinds[bad], minlength=6)}), first {bad[:5]}"
    ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_gpu_fill_random_bytes_all_layouts(mode):
    """Arbitrary bytes (any tot_len, incl. out-of-range ones left untouched), every
    (frame_off + 14) % 16 class, every line offset of the window block, jumbo slots, ragged n,
    both launch forms (in place up to 65,536 frames, two-phase above)."""
    torch, pa = _gpu()
    ctx = pa.RxContext(0)
    rng = np.random.default_rng(mode + 100)
    for stride, frame_off, n in [(2048, 2, 4099), (2048, 14, 1000), (2048, 0, 777), (2048, 4, 65), (2048, 6, 64),
                                 (2048, 8, 63), (2048, 10, 1), (2048, 12, 300), (2064, 2, 513), (4096, 34, 200),
                                 (16384, 2, 130), (112, 2, 200), (1024, 2, 333),
                                 # window block off the line grid: stream from the next line, header in
                                 # the first line (18, 50) or across both (66, 98), block at line + 112 (114, 126)
                                 (2048, 18, 300), (2048, 50, 64), (2048, 66, 200), (2048, 98, 70), (2048, 114, 150),
                                 (2048, 126, 129),
                                 # 32 frames per wave (frames_per_wave; 64 in the full-size round trip below)
                                 (2048, 14, 40000),
                                 # the one-launch in-place form up to kTxInPlaceMaxFrames = 65,536 frames,
                                 # the two-phase form (patch records + patch launch) above it
                                 (2048, 14, 65536), (2048, 2, 70001), (2048, 0, 65537)]:
        avail = stride - frame_off
        slots = rng.integers(0, 256, (n, stride), dtype=np.uint8)
        tot = rng.integers(0, avail + 64, n)
        sane = rng.random(n) < 0.5  # half the frames with a length that fits the slot
        tot[sane] = rng.integers(40, max(41, avail - 14 + 1), int(sane.sum()))
        slots[:, frame_off + IP + 2] = (tot >> 8) & 0xFF
        slots[:, frame_off + IP + 3] = tot & 0xFF
        lens = rng.integers(0, 65536, n).astype(np.uint16)
        lens[rng.random(n) < 0.7] %= max(1, avail - 40)
        for use_lens in (False, True):
            exp = slots.copy()
            orc.tx_fill_batch(exp, stride, frame_off, n, lens if use_lens else None, mode)
            got = _fill_gpu(ctx, torch, slots, stride, frame_off, n, lens if use_lens else None, mode)
            bad = np.nonzero((got != exp).any(1))[0]
            assert len(bad) == 0, (stride, frame_off, n, use_lens, bad[:5])
    ctx.close()


@pytest.mark.gpu
def test_gpu_efvi_defect_and_jumbo_datagrams():
    torch, pa = _gpu()
    ctx = pa.RxContext(0)
    need = 0x1FFFF - 0x11C5
    stride, off = 65536, 2
    slots = np.zeros((3, stride), dtype=np.uint8)
    for i, paylen in enumerate([100, 1400, 65000]):
        ip = craft_udp_header([0xFFFF, need - 0xFFFF], [0, 0], paylen)
        slots[i, off + 14:off + 34] = np.frombuffer(ip, dtype=np.uint8)
    for mode in (1, 2):
        exp = slots.copy()
        orc.tx_fill_batch(exp, stride, off, 3, None, mode)
        got = _fill_gpu(ctx, torch, slots, stride, off, 3, None, mode)
        assert np.array_equal(got, exp)
        for i in range(3):
            ok = fold(word_sum(got[i, off + 14:off + 34])) == 0
            assert ok == (mode == 2)
    ctx.close()


@pytest.mark.gpu
def test_gpu_full_size_c2_round_trip():
    """1 Mi C2 frames (2 GiB): scramble both checksums, pn_tx_fill, then pn_classify — every
    frame verifies (IP_OK, TCP_OK), and the frames the generator built valid come back
    byte-identical (the generator flips one payload bit in every 1024th frame)."""
    torch, pa = _gpu()
    ctx = pa.RxContext(0)
    p = pa.rx.GenParams.for_config(2)
    n = 1 << 20
    host = pa.gen_frames(p, n)
    d = torch.from_numpy(host.reshape(-1)).cuda()
    ref = d.clone()
    v = d.view(n, 2048)
    v[:, 2 + IP + 10:2 + IP + 12] = 0x5A
    v[:, 2 + TCP + 16:2 + TCP + 18] = 0xA5
    ctx.tx_fill(d, 2048, 2, n)
    t = pa.gen_conn_table(p)
    ctx.set_conn_table(t)
    res = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
    ctx.classify(d, 2048, 2, n, res)
    torch.cuda.synchronize()
    flags = res.view(torch.int16).view(n, 8)[:, 6].to(torch.int32) & 0xFFFF
    assert bool(((flags & 3) == 3).all())
    same = (v == ref.view(n, 2048)).all(dim=1)
    corrupted = torch.zeros(n, dtype=torch.bool, device="cuda")
    corrupted[1023::1024] = True  # framegen.cpp: one flipped payload bit when (i & 1023) == 1023
    assert bool(same[~corrupted].all())
    assert not bool(same[corrupted].any())
    ctx.close()


@pytest.mark.gpu
def test_gpu_fill_argument_contract():
    """n = 0 is a no-op; an unknown mode, a misaligned buffer or a layout outside the contract
    (odd frame_off, stride not a 16-B multiple or too short) fails with PN_EINVAL and a message,
    before any launch: the frames are left as they were."""
    torch, pa = _gpu()
    ctx = pa.RxContext(0)
    slots, _, _ = orc.tx_build_batch(0xA11, 64, frame_off=14, mode=orc.TX_TCP)
    s = scramble(slots, 14, orc.TX_TCP, False)
    d = torch.from_numpy(s.reshape(-1).copy()).cuda()
    ctx.tx_fill(d, 2048, 14, 0)
    torch.cuda.synchronize()
    assert np.array_equal(d.cpu().numpy(), s.reshape(-1))
    bad_calls = [
        dict(frames=d, stride=2048, off=14, mode=7),          # unknown mode
        dict(frames=d[2:], stride=2048, off=14, mode=0),      # frames not 16-B aligned
        dict(frames=d, stride=2040, off=14, mode=0),          # stride not a 16-B multiple
        dict(frames=d, stride=2048, off=13, mode=0),          # odd frame_off
        dict(frames=d, stride=96, off=14, mode=0),            # stride < frame_off + 96
        dict(frames=d, stride=65552, off=14, mode=0),         # stride > 65536
    ]
    for c in bad_calls:
        with pytest.raises(pa.PollnetError, match=r"\(-?\d+\)"):
            ctx.tx_fill(c["frames"], c["stride"], c["off"], 16, None, c["mode"])
    torch.cuda.synchronize()
    assert np.array_equal(d.cpu().numpy(), s.reshape(-1))
    ctx.tx_fill(d, 2048, 14, 64)  # the ctx still works after the refused calls
    torch.cuda.synchronize()
    assert np.array_equal(d.cpu().numpy().reshape(s.shape), slots)
    ctx.close()


def _ref_built_segments(seed, n, frame_off=14, stride=2048):
    """n data segments built by the reference's own send-path code (oracle/_ref/libref_core.so:
    TcpConn::copyAndSum and SendBuf::setOptDataLen compiled verbatim, the connection's cached
    sums restated around them): random addresses, ports, seq/ack/window, payloads of 0..1460
    bytes appended in 1..4 random pieces (odd sizes put later pieces at odd addresses)."""
    ref = orc.ref_core()
    if ref is None:
        pytest.skip("oracle/_ref/libref_core.so not built (needs /root/reference)")
    rng = np.random.default_rng(seed)
    slots = np.zeros((n, stride), np.uint8)
    for i in range(n):
        e = slots[i, frame_off:]
        e[0:12] = rng.integers(0, 256, 12)
        e[12:14] = (0x08, 0x00)
        e[14:34] = rng.integers(0, 256, 20)  # IpHeader: any tos/id/frag/ttl/addresses
        e[14] = 0x45
        e[23] = 6
        e[34:54] = rng.integers(0, 256, 20)  # TcpHeader: any ports/seq/ack/flags/window
        e[46] = 0x50 | (e[46] & 0x0F)  # data_offset 5
        e[52:54] = 0  # urgent pointer
        ln = int(rng.integers(0, 1461))
        payload = rng.integers(0, 256, ln, dtype=np.uint8)
        pieces = np.array(rng.integers(1, 700, int(rng.integers(1, 5))), np.uint32)
        buf = np.ascontiguousarray(slots[i])
        ref.ref_tx_data_segment(buf.ctypes.data + frame_off, payload.ctypes.data, ln, pieces.ctypes.data, len(pieces))
        slots[i] = buf
        assert np.array_equal(slots[i, frame_off + 54:frame_off + 54 + ln], payload)
    return slots


def test_byte_recompute_equals_reference_send_path():
    """The oracle's one-pass recomputation (the GPU kernel's contract) reproduces segments the
    reference's own copyAndSum + setOptDataLen built, byte for byte, in the SendBuf layout
    (frame_off 14) and the RX-ring layout (2); every one passes the reference's Core::checksum
    when its segment is even (odd ones: the debug check reads the byte after the segment)."""
    for off in (14, 2):
        slots = _ref_built_segments(0x5E0D + off, 3000, off)
        s = scramble(slots, off, orc.TX_TCP, False)
        orc.tx_fill_batch(s, 2048, off, len(s), None, orc.TX_TCP)
        assert np.array_equal(s, slots)
        rec = orc.classify_batch(slots, 2048, off, len(slots), E_EMPTY, 1, 1)
        tot = (slots[:, off + 16].astype(int) << 8) | slots[:, off + 17]
        even = (tot & 1) == 0
        assert ((rec["flags"][even] & 3) == 3).all() and even.sum() > 1000


@pytest.mark.gpu
@pytest.mark.parametrize("frame_off", [14, 2])
def test_gpu_fill_equals_reference_send_path(frame_off):
    """pn_tx_fill on segments the reference's own copyAndSum + setOptDataLen built (checksums
    scrambled first) gives back those segments byte for byte, in both launch forms."""
    torch, pa = _gpu()
    ctx = pa.RxContext(0)
    slots = _ref_built_segments(0x6E0D + frame_off, 3000, frame_off)
    s = scramble(slots, frame_off, orc.TX_TCP, False)
    got = _fill_gpu(ctx, torch, s, 2048, frame_off, len(s), None, 0)
    assert np.array_equal(got, slots)
    big = np.tile(s, (23, 1))[:66000]  # > kTxInPlaceMaxFrames: the two-phase form
    got = _fill_gpu(ctx, torch, big, 2048, frame_off, len(big), None, 0)
    assert np.array_equal(got, np.tile(slots, (23, 1))[:66000])
    ctx.close()


def _ref_efvi_datagrams(seed, n, frame_off=2, stride=2048):
    """n UDP datagrams through Efvi's own code (oracle/_ref/libref_core.so: the cached IPv4 sum,
    Efvi.h:406-411, and update_udp_pkt, :611-621, compiled verbatim): random addresses and
    header words, random payload lengths, and every 8th header chosen so that the cache's first
    end-around step carries (the defect).  Returns (slots, paylens, defect rows)."""
    ref = orc.ref_core()
    if ref is None:
        pytest.skip("oracle/_ref/libref_core.so not built (needs /root/reference)")
    rng = np.random.default_rng(seed)
    slots = np.zeros((n, stride), np.uint8)
    paylens = rng.integers(0, stride - frame_off - 42 + 1, n).astype(np.uint16)
    defect = np.zeros(n, bool)
    need = 0x1FFFF - 0x11C5  # craft_udp_header's other words sum to 0x11C5
    for i in range(n):
        e = slots[i, frame_off:]
        e[0:12] = rng.integers(0, 256, 12)
        e[12:14] = (0x08, 0x00)
        if i % 8 == 0:
            e[14:34] = np.frombuffer(craft_udp_header([0xFFFF, need - 0xFFFF], [0, 0], 0), np.uint8)
        else:
            e[14:34] = rng.integers(0, 256, 20)
            e[14], e[23] = 0x45, 17
        e[34:42] = rng.integers(0, 256, 8)
        e[42:42 + int(paylens[i])] = rng.integers(0, 256, int(paylens[i]))
        words = e[14:34].view("<u2").astype(np.int64)
        c = int(words.sum()) - int(words[1]) - int(words[5])
        defect[i] = (c >> 16) + (c & 0xFFFF) >= 0x10000
        buf = np.ascontiguousarray(slots[i])
        ref.ref_efvi_udp_datagram(buf.ctypes.data + frame_off, int(paylens[i]))
        slots[i] = buf
    assert defect.sum() >= n // 8
    return slots, paylens, defect


def test_efvi_mode_equals_reference_update_udp_pkt():
    """PN_TX_UDP_EFVI's recomputation (with lens = paylen) reproduces Efvi's own
    update_udp_pkt output byte for byte, the carry defect included; PN_TX_UDP agrees wherever
    Efvi's checksum verifies and differs exactly on the defect rows."""
    for off in (2, 14):
        slots, paylens, defect = _ref_efvi_datagrams(0xEF1 + off, 2000, off)
        s = scramble(slots, off, orc.TX_UDP_EFVI, True)
        orc.tx_fill_batch(s, 2048, off, len(s), paylens, orc.TX_UDP_EFVI)
        assert np.array_equal(s, slots)
        u = scramble(slots, off, orc.TX_UDP_EFVI, True)
        orc.tx_fill_batch(u, 2048, off, len(u), paylens, orc.TX_UDP)
        differs = (u != slots).any(1)
        assert np.array_equal(differs, defect)


@pytest.mark.gpu
def test_gpu_efvi_mode_equals_reference_update_udp_pkt():
    torch, pa = _gpu()
    ctx = pa.RxContext(0)
    for off in (2, 14):
        slots, paylens, _ = _ref_efvi_datagrams(0xEF9 + off, 3000, off)
        s = scramble(slots, off, orc.TX_UDP_EFVI, True)
        got = _fill_gpu(ctx, torch, s, 2048, off, len(s), paylens, 1)
        assert np.array_equal(got, slots)
    ctx.close()
