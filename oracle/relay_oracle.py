"""relay_oracle.py -- TEST INFRASTRUCTURE ONLY: restatement of the reference
relay's packet path around Rijndael (thejinchao/cyclone samples/relay and
source/cyEvent/event/cye_packet.cpp), in plain Python over the AES oracle.
Only tests/ import it, as the checker for include/cyaes_relay.h and the
batcher's SEAL / OPEN requests.

Parity is pinned by this restatement of the reference code (cited line by
line), by the AES oracle's own pins, and -- for the Packet framing -- by the
reference's own Packet TEST_CASE (test/unit/cyt_unit_packet.cpp:39-142),
re-expressed in tests/test_relay.py::test_reference_packet_test_case against
build_packet / take_packet below.  The reference ships no relay byte vectors,
so the RELAY_FORWARD layout on top of the framing is restated, not
vector-pinned.
"""
import struct

from oracle import Rijndael

RELAY_PACKET_HEADSIZE = 4  # relay_protocol.h:5-7
RELAY_HANDSHAKE_ID = 100   # relay_protocol.h:9-14 (enum continues: +1, +2, +3)
RELAY_FORWARD = RELAY_HANDSHAKE_ID + 3
MAX_CHUNK = 0xFF00         # relay_local.cpp:189, relay_server.cpp:454
FILL = 0xCE                # Packet::_resize memset, cye_packet.cpp:102


def round16(size):
    """RelayLocal::_round16, relay_local.cpp:430-432."""
    return size if (size & 0xF) == 0 else (size & ~0xF) + 0x10


def build_packet(head_size, packet_id, content, content2=b""):
    """Packet::build_from_memory (cye_packet.cpp:107-138): 0xCE-filled memory
    of head_size + size bytes (:90-105), BE u16 size and id (:123-124), the
    two content parts copied back to back (:129-137).  A total above 0xFFFF
    builds nothing (:117-118): None."""
    assert head_size >= 4  # _resize's assert, cye_packet.cpp:92
    size = len(content) + len(content2)
    if size > 0xFFFF:
        return None
    mem = bytearray([FILL]) * (head_size + size)
    mem[0:2] = struct.pack(">H", size)
    mem[2:4] = struct.pack(">H", packet_id)
    mem[head_size:head_size + size] = bytes(content) + bytes(content2)
    return mem


def take_packet(buf, head_size):
    """Packet::build_from_ringbuf (cye_packet.cpp:166-181) on the bytes buf
    holds: None while fewer than 2 bytes (the size) or fewer than head_size +
    size bytes are present, else the packet's memory (head_size + size bytes,
    the head's reserved bytes included as received)."""
    if len(buf) < 2:
        return None
    size, = struct.unpack(">H", bytes(buf[0:2]))
    if len(buf) < head_size + size:
        return None
    return bytes(buf[:head_size + size])


def seal_forward(key, conn_id, chunk, encrypt=True):
    """One iteration of RelayLocal::onLocalMessage's loop (relay_local.cpp:189-206):
    packet of 8 + round16(size) content bytes, RelayForwardMsg{id, size} memcpy'd
    (host order, little-endian here), chunk copied, payload encrypted in place
    with iv = nullptr."""
    size = len(chunk)
    assert size <= MAX_CHUNK
    padded = round16(size)
    content = bytearray([FILL]) * (8 + padded)  # build_from_memory(..., nullptr): content stays 0xCE
    content[0:8] = struct.pack("<ii", conn_id, size)
    content[8:8 + size] = chunk
    pkt = build_packet(RELAY_PACKET_HEADSIZE, RELAY_FORWARD, content)
    if encrypt and padded:
        buf = bytearray(pkt[12:12 + padded])
        Rijndael(key).encrypt(buf, buf, padded)
        pkt[12:12 + padded] = buf
    return bytes(pkt)


def open_forward(key, pkt):
    """RelayServer forward handling (relay_server.cpp:329): decrypt
    packet_size - sizeof(RelayForwardMsg) bytes at content + 8, in place;
    returns (conn_id, payload of forwardMsg.size bytes, whole packet)."""
    pkt = bytearray(pkt)
    psize, = struct.unpack(">H", pkt[0:2])
    n = psize - 8
    if n:
        buf = bytearray(pkt[12:12 + n])
        Rijndael(key).decrypt(buf, buf, n)
        pkt[12:12 + n] = buf
    conn_id, size = struct.unpack("<ii", pkt[4:12])
    return conn_id, bytes(pkt[12:12 + size]), bytes(pkt)


def parse_stream(stream, head_size=RELAY_PACKET_HEADSIZE):
    """take_packet (Packet::build_from_ringbuf, cye_packet.cpp:166-181) in a
    loop, as the relay's onMessage handlers drain a connection's ring buffer:
    returns [(offset, packet_size, packet_id)] and the bytes consumed."""
    out, pos = [], 0
    while True:
        mem = take_packet(stream[pos:], head_size)
        if mem is None:
            break
        psize, pid = struct.unpack(">HH", mem[0:4])
        out.append((pos, psize, pid))
        pos += len(mem)
    return out, pos
