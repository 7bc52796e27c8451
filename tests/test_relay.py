"""Relay wire format (include/cyaes_relay.h) against the
restatement of the reference relay in oracle/relay_oracle.py.  Host logic
only: no GPU."""
import random
import struct

import pytest

import cyclone_amd as ca
import relay_oracle as ro

SIZES = [0, 1, 15, 16, 17, 31, 1400, 1472, 4095, 0xFEFF, 0xFF00]


def test_round16_and_packet_bytes():
    lib = ca.load_library()
    for n in list(range(0, 70)) + SIZES:
        assert lib.cyaes_relay_round16(n) == ro.round16(n)
        assert ca.relay_packet_bytes(n) == 12 + ro.round16(n)


@pytest.mark.parametrize("size", SIZES)
def test_build_forward_matches_reference_packet(size):
    rng = random.Random(size)
    chunk = bytes(rng.randrange(256) for _ in range(size))
    conn = rng.randrange(-2**31, 2**31)
    assert ca.relay_build_forward(conn, chunk) == ro.seal_forward(None, conn, chunk, encrypt=False)
    pkt = ca.relay_build_forward(conn, chunk)
    lib = ca.load_library()
    buf = (ca.ctypes.c_uint8 * len(pkt)).from_buffer_copy(pkt)
    assert lib.cyaes_relay_forward_id(buf) == conn and lib.cyaes_relay_forward_size(buf) == size
    assert struct.unpack(">HH", pkt[:4]) == (8 + ro.round16(size), ro.RELAY_FORWARD)


def _check_packet(mem, size, pid, head_size, content):
    """PACKET_CHECK (cyt_unit_packet.cpp:18-23): BE u16 size and id in the
    first 4 bytes, memory size = head + packet size, content."""
    assert mem is not None
    assert bytes(mem[0:4]) == struct.pack(">HH", size, pid)
    assert len(mem) == head_size + size
    assert struct.unpack(">H", bytes(mem[2:4]))[0] == pid and struct.unpack(">H", bytes(mem[0:2]))[0] == size
    assert bytes(mem[head_size:head_size + size]) == bytes(content[:size])


def test_reference_packet_test_case():
    """The reference's own Packet TEST_CASE (test/unit/cyt_unit_packet.cpp:39-142),
    re-expressed against the framing restatement (relay_oracle.build_packet /
    take_packet) and, at the relay's head size of 4, against cyaes_relay_parse.
    The test's rand() bytes become a seeded generator; build_from_pipe
    (:108-121) is not restated: the relay reads connections through ring
    buffers (Packet::build_from_ringbuf), which is what the product parses."""
    HEAD_SIZE, PACKET_ID, RESERVED = 8, 0x1234, struct.pack("<I", 0xFACEC00D)
    rng = random.Random(0x1234)
    # build_from_memory with no content (:52-57)
    mem = ro.build_packet(HEAD_SIZE, PACKET_ID, b"")
    _check_packet(mem, 0, PACKET_ID, HEAD_SIZE, b"")
    temp = bytes(rng.randrange(256) for _ in range(1024))
    half = 512
    _check_packet(ro.build_packet(HEAD_SIZE, PACKET_ID, temp[:half]), half, PACKET_ID, HEAD_SIZE, temp)  # :70-71
    _check_packet(ro.build_packet(HEAD_SIZE, PACKET_ID, temp), 1024, PACKET_ID, HEAD_SIZE, temp)  # :77-78
    _check_packet(ro.build_packet(HEAD_SIZE, PACKET_ID, temp[:half], temp[half:]), 1024, PACKET_ID, HEAD_SIZE,
                  temp)  # two parts, :84-85
    # build_from_ringbuf (:91-103): incomplete until head + size bytes are present
    rb = bytearray()
    assert ro.take_packet(rb, HEAD_SIZE) is None
    rb += struct.pack(">HH", 1024, PACKET_ID) + RESERVED
    assert ro.take_packet(rb, HEAD_SIZE) is None
    rb += temp[:half]
    assert ro.take_packet(rb, HEAD_SIZE) is None
    rb += temp[half:]
    mem = ro.take_packet(rb, HEAD_SIZE)
    _check_packet(mem, 1024, PACKET_ID, HEAD_SIZE, temp)
    assert mem[4:8] == RESERVED  # PACKET_CHECK_WITH_RESERVED, :26-28
    # large packet, 0xFFFF bytes, whole and in two parts (:124-135)
    big = bytes(rng.randrange(256) for _ in range(0xFFFF))
    _check_packet(ro.build_packet(HEAD_SIZE, PACKET_ID, big), 0xFFFF, PACKET_ID, HEAD_SIZE, big)
    _check_packet(ro.build_packet(HEAD_SIZE, PACKET_ID, big[:0x7FFF], big[0x7FFF:]), 0xFFFF, PACKET_ID, HEAD_SIZE,
                  big)
    assert ro.build_packet(HEAD_SIZE, PACKET_ID, big, b"x") is None  # over 0xFFFF builds nothing (cye_packet.cpp:117-118)
    # The same ring-buffer sequence at the relay's head size (RELAY_PACKET_HEADSIZE = 4) through the product's parser.
    rb = bytearray()
    steps = [b"", struct.pack(">HH", 1024, PACKET_ID), temp[:half], temp[half:]]
    for i, part in enumerate(steps):
        rb += part
        got, used = ca.relay_parse(bytes(rb))
        want, wused = ro.parse_stream(bytes(rb))
        assert (got, used) == (want, wused)
        assert got == ([(0, 1024, PACKET_ID)] if i == len(steps) - 1 else [])
    mem = ro.take_packet(rb, 4)
    _check_packet(mem, 1024, PACKET_ID, 4, temp)


def test_build_forward_rejects_oversize_chunk():
    with pytest.raises(ValueError):
        ca.relay_build_forward(1, bytes(0xFF01))
    lib = ca.load_library()
    assert lib.cyaes_relay_build_forward(None, 1, None, 0) == 0


def _stream(rng, n):
    pkts = []
    for _ in range(n):
        if rng.random() < 0.2:  # other relay messages share the connection (relay_protocol.h:9-14)
            pid = rng.choice([ro.RELAY_HANDSHAKE_ID, ro.RELAY_HANDSHAKE_ID + 1, ro.RELAY_HANDSHAKE_ID + 2])
            pkts.append(bytes(ro.build_packet(4, pid, struct.pack("<i", rng.randrange(1000)))))
        else:
            size = rng.choice(SIZES + [rng.randrange(1, 3000)])
            pkts.append(ro.seal_forward(None, rng.randrange(100), bytes(rng.randrange(256) for _ in range(size)),
                                        encrypt=False))
    return pkts


def test_parse_matches_reference_incl_incomplete_tail():
    rng = random.Random(5)
    pkts = _stream(rng, 60)
    stream = b"".join(pkts)
    for cut in [len(stream), len(stream) - 1, len(stream) - len(pkts[-1]), 3, 0, 4]:
        got, used = ca.relay_parse(stream[:cut])
        want, wused = ro.parse_stream(stream[:cut])
        assert got == want and used == wused


def test_payloads_select_forward_packets():
    rng = random.Random(6)
    pkts = _stream(rng, 40)
    stream = b"".join(pkts)
    parsed, _ = ca.relay_parse(stream)
    off, ln = ca.relay_payloads(parsed, base=1000)
    want = [(1000 + o + 12, s - 8) for o, s, i in parsed if i == ro.RELAY_FORWARD and s > 8]
    assert list(zip(off, ln)) == want
    assert all(o % 4 == 0 for o in off) and all(x % 16 == 0 for x in ln)
    bad = [(0, 8 + 17, ro.RELAY_FORWARD)]  # a payload the reference encrypt path cannot produce
    with pytest.raises(ValueError):
        ca.relay_payloads(bad)


def test_relay_stride_recognises_equal_packet_streams():
    """cyaes_relay_stride: a parsed stream of equal FORWARD packets is one
    strided batch (payload at packet offset 12, stride = packet size, the
    layout cyaes_gpu_*_strided take); anything irregular is not."""
    chunks = [bytes([i % 251]) * 1472 for i in range(50)]
    stream = b"".join(ro.seal_forward(None, i, c, encrypt=False) for i, c in enumerate(chunks))
    off, ln = ca.relay_payloads(ca.relay_parse(stream)[0], base=1000)
    assert ca.relay_stride(off, ln) == (1012, ca.relay_packet_bytes(1472), 1472)
    assert ca.relay_stride(off[:1], ln[:1]) == (1012, 1472, 1472)  # one payload: stride = its size
    assert ca.relay_stride([], []) is None
    assert ca.relay_stride(off, ln[:-1] + [1456]) is None             # a shorter last payload
    assert ca.relay_stride(off[:10] + off[11:], ln[:-1]) is None      # a missing packet
    assert ca.relay_stride([0, 100], [1472, 1472]) is None            # overlapping payloads
    assert ca.relay_stride([100, 0], [16, 16]) is None                # descending offsets


def test_batcher_without_device_fails_loudly():
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("checks the no-device path")
    except ImportError:
        pass
    with pytest.raises(ca.CyaesError) as e:
        ca.Batcher(0)
    assert e.value.status == ca.CYAES_ENODEV


def test_relay_wire_format_fuzz_under_sanitizers(tmp_path):
    """tests/cpp/fuzz_relay.cpp: random FORWARD / foreign / garbage / truncated
    streams through the host parser and builder, built with ASan + UBSan."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path / "fuzz_relay")
    subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-I" + os.path.join(root, "include"), "-o", exe,
                    os.path.join(root, "tests", "cpp", "fuzz_relay.cpp"),
                    os.path.join(root, "cyclone_amd", "csrc", "cyaes_relay.cpp")], check=True)
    # verify_asan_link_order=0: tolerate libraries preloaded by the environment
    r = subprocess.run([exe, "3000"], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, ASAN_OPTIONS="verify_asan_link_order=0:detect_leaks=0"))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "3000 streams ok" in r.stdout
