// cyaes_relay.cpp -- relay wire format (include/cyaes_relay.h).  Host-only.
// Reference: samples/relay/relay_protocol.h:5-42, relay_local.cpp:189-206,
// 365, 430-432; relay_server.cpp:329, 454-472; cye_packet.cpp:90-181.
#include <string.h>

#include "cyaes_relay.h"

namespace {

uint16_t be16(const uint8_t* p) { return (uint16_t)((p[0] << 8) | p[1]); }
void put_be16(uint8_t* p, uint16_t v) {
    p[0] = (uint8_t)(v >> 8);
    p[1] = (uint8_t)v;
}
int32_t get_i32(const uint8_t* p) {  // host byte order, as memcpy of the struct field
    int32_t v;
    memcpy(&v, p, 4);
    return v;
}

}  // namespace

extern "C" {

uint32_t cyaes_relay_round16(uint32_t size) { return (size & 0xFu) == 0 ? size : (size & ~0xFu) + 0x10u; }

uint32_t cyaes_relay_packet_bytes(uint32_t msg_size) {
    return CYAES_RELAY_PAYLOAD_OFFSET + cyaes_relay_round16(msg_size);
}

uint32_t cyaes_relay_build_forward(uint8_t* dst, int32_t conn_id, const uint8_t* payload, uint32_t size) {
    if (!dst || size > CYAES_RELAY_MAX_CHUNK || (size && !payload)) return 0;
    const uint32_t padded = cyaes_relay_round16(size);
    const uint32_t total = CYAES_RELAY_PAYLOAD_OFFSET + padded;
    // Packet::build_from_memory(4, RELAY_FORWARD, 8 + padded, nullptr): the
    // memory is 0xCE-filled, then size/id are stored big-endian.
    put_be16(dst, (uint16_t)(8 + padded));
    put_be16(dst + 2, (uint16_t)CYAES_RELAY_FORWARD);
    const int32_t msg[2] = {conn_id, (int32_t)size};  // RelayForwardMsg, memcpy'd (relay_local.cpp:199)
    memcpy(dst + CYAES_RELAY_HEADSIZE, msg, sizeof(msg));
    if (size) memcpy(dst + CYAES_RELAY_PAYLOAD_OFFSET, payload, size);
    memset(dst + CYAES_RELAY_PAYLOAD_OFFSET + size, CYAES_RELAY_PAD, padded - size);
    return total;
}

uint32_t cyaes_relay_parse(const uint8_t* stream, size_t len, uint64_t* offsets, uint32_t* packet_sizes,
                           uint16_t* packet_ids, uint32_t max_packets, size_t* consumed) {
    size_t pos = 0;
    uint32_t n = 0;
    while (stream && n < max_packets && len - pos >= CYAES_RELAY_HEADSIZE) {
        const uint32_t psize = be16(stream + pos);
        if (len - pos < CYAES_RELAY_HEADSIZE + (size_t)psize) break;  // incomplete (cye_packet.cpp:176)
        if (offsets) offsets[n] = pos;
        if (packet_sizes) packet_sizes[n] = psize;
        if (packet_ids) packet_ids[n] = be16(stream + pos + 2);
        n++;
        pos += CYAES_RELAY_HEADSIZE + psize;
    }
    if (consumed) *consumed = pos;
    return n;
}

int64_t cyaes_relay_payloads(const uint64_t* offsets, const uint32_t* packet_sizes, const uint16_t* packet_ids,
                             uint32_t npackets, uint64_t base, uint64_t* pay_off, uint32_t* pay_len) {
    if (npackets && (!offsets || !packet_sizes || !packet_ids || !pay_off || !pay_len)) return -1;
    int64_t j = 0;
    for (uint32_t k = 0; k < npackets; k++) {
        if (packet_ids[k] != CYAES_RELAY_FORWARD) continue;
        if (packet_sizes[k] < 8 || (packet_sizes[k] - 8) % 16) return -1;
        if (packet_sizes[k] == 8) continue;  // empty payload: decrypt(buf, buf, 0) is a no-op
        pay_off[j] = base + offsets[k] + CYAES_RELAY_PAYLOAD_OFFSET;
        pay_len[j] = packet_sizes[k] - 8;
        j++;
    }
    return j;
}

int cyaes_relay_stride(const uint64_t* pay_off, const uint32_t* pay_len, uint64_t n, uint64_t* first, uint64_t* stride,
                       uint32_t* payload_bytes) {
    if (n == 0 || !pay_off || !pay_len || !first || !stride || !payload_bytes) return 0;
    const uint64_t st = n > 1 ? pay_off[1] - pay_off[0] : pay_len[0];
    if (n > 1 && (pay_off[1] < pay_off[0] || st < pay_len[0])) return 0;
    for (uint64_t j = 0; j < n; j++)
        if (pay_len[j] != pay_len[0] || pay_off[j] != pay_off[0] + j * st) return 0;
    *first = pay_off[0];
    *stride = st;
    *payload_bytes = pay_len[0];
    return 1;
}

int32_t cyaes_relay_forward_id(const uint8_t* pkt) { return pkt ? get_i32(pkt + CYAES_RELAY_HEADSIZE) : 0; }
int32_t cyaes_relay_forward_size(const uint8_t* pkt) { return pkt ? get_i32(pkt + CYAES_RELAY_HEADSIZE + 4) : 0; }

}  // extern "C"
