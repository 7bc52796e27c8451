/*
 * cyaes_relay.h -- relay wire format around the AES path (SURVEY.md §8(f) row 2,
 * "Packet wire-format gather/scatter").  Host-side, no device calls.
 *
 * The reference relay (samples/relay) wraps every forwarded TCP chunk in a
 * cyclone::Packet (source/cyEvent/event/cye_packet.h:6-25):
 *
 *   offset 0   BE u16  packet_size   (= 8 + round16(msg_size))
 *   offset 2   BE u16  packet_id     (RELAY_FORWARD = 103)
 *   offset 4   RelayForwardMsg { int32 id; int32 size; }  (host byte order,
 *              relay_protocol.h:36-42; size = msg_size, the unpadded length)
 *   offset 12  payload: msg_size bytes, then 0xCE up to a multiple of 16
 *              (Packet::_resize fills the buffer with 0xCE, cye_packet.cpp:102)
 *
 * and encrypts the padded payload in place with Rijndael::encrypt(buf, buf,
 * round16(msg_size)) (relay_local.cpp:189-206, relay_server.cpp:454-472);
 * the receiver decrypts packet_size - 8 bytes at offset 12 in place
 * (relay_local.cpp:365, relay_server.cpp:329).  Chunks are at most 0xFF00
 * bytes (relay_local.cpp:189).
 *
 * A batch of such packets laid out back to back (the byte stream one
 * connection sends) has its payloads at offsets that are 4-byte aligned, so
 * cyaes_gpu_{encrypt,decrypt}_ragged (cyaes.h) process them where they lie:
 * cyaes_relay_parse + cyaes_relay_payloads give the offsets and sizes.
 * cyaes_batch.h's SEAL / OPEN requests do the whole gather -> GPU -> scatter.
 */
#ifndef CYAES_RELAY_H
#define CYAES_RELAY_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CYAES_RELAY_HEADSIZE 4          /* RELAY_PACKET_HEADSIZE, relay_protocol.h:5-7   */
#define CYAES_RELAY_FORWARD 103         /* RELAY_FORWARD, relay_protocol.h:9-14          */
#define CYAES_RELAY_PAYLOAD_OFFSET 12   /* head + sizeof(RelayForwardMsg)                */
#define CYAES_RELAY_MAX_CHUNK 0xFF00u   /* relay_local.cpp:189, relay_server.cpp:454     */
#define CYAES_RELAY_PAD 0xCE            /* cye_packet.cpp:102                            */

/* _round16 (relay_local.cpp:430-432). */
uint32_t cyaes_relay_round16(uint32_t size);

/* Bytes of the RELAY_FORWARD packet carrying msg_size payload bytes:
 * 12 + round16(msg_size). */
uint32_t cyaes_relay_packet_bytes(uint32_t msg_size);

/* Builds the plaintext RELAY_FORWARD packet of relay_local.cpp:189-201 into
 * dst (cyaes_relay_packet_bytes(size) bytes): header, RelayForwardMsg{conn_id,
 * size}, payload, 0xCE padding.  Returns the packet bytes, or 0 if size >
 * CYAES_RELAY_MAX_CHUNK or a pointer is NULL (payload may be NULL if size == 0). */
uint32_t cyaes_relay_build_forward(uint8_t* dst, int32_t conn_id, const uint8_t* payload, uint32_t size);

/* Walks a received byte stream the way Packet::build_from_ringbuf does
 * (cye_packet.cpp:166-181): a packet is complete when 4 + packet_size bytes
 * are present.  For up to max_packets complete packets writes offset,
 * packet_size and packet_id (any id).  Returns the number found; *consumed
 * (nullable) = bytes they span, i.e. where an incomplete tail begins. */
uint32_t cyaes_relay_parse(const uint8_t* stream, size_t len, uint64_t* offsets, uint32_t* packet_sizes,
                           uint16_t* packet_ids, uint32_t max_packets, size_t* consumed);

/* Selects the RELAY_FORWARD packets of a parsed stream and writes the
 * ragged-batch description of their encrypted payloads:
 *   pay_off[j] = base + offsets[k] + 12,  pay_len[j] = packet_sizes[k] - 8.
 * Returns j (the number of FORWARD packets with a non-empty payload), or -1
 * if one has a payload length that is not a multiple of 16 (it cannot have
 * come from the reference encrypt path). */
int64_t cyaes_relay_payloads(const uint64_t* offsets, const uint32_t* packet_sizes, const uint16_t* packet_ids,
                             uint32_t npackets, uint64_t base, uint64_t* pay_off, uint32_t* pay_len);

/* 1 if the n payloads of a ragged description are equally strided and
 * equally sized (pay_off[j] = pay_off[0] + j * stride, pay_len[j] = pay_len[0],
 * stride >= pay_len[0]): a stream of equal packets, which
 * cyaes_gpu_{en,de}crypt_strided processes without device lists; *first,
 * *stride and *payload_bytes are set then.  0 otherwise (n == 0 included). */
int cyaes_relay_stride(const uint64_t* pay_off, const uint32_t* pay_len, uint64_t n, uint64_t* first, uint64_t* stride,
                       uint32_t* payload_bytes);

/* RelayForwardMsg fields of a packet starting at pkt (host byte order). */
int32_t cyaes_relay_forward_id(const uint8_t* pkt);
int32_t cyaes_relay_forward_size(const uint8_t* pkt);

#ifdef __cplusplus
}
#endif

#endif /* CYAES_RELAY_H */
