// relay_calls.cpp -- the relay sample's cyclone::Rijndael call expressions,
// verbatim, compiled against the drop-in header (include/cyclone_amd/cyr_rijndael.h).
// INTEGRATION.md §1 claims samples/relay compiles unchanged against it; this
// file is that claim as a test.  The statements inside the marked blocks are
// copied character for character from the reference call sites:
//   relay_local.cpp:329-334   key hand-off after the DH handshake
//   relay_local.cpp:204-207   encrypt in place (relay_server.cpp:470-473 is the same)
//   relay_local.cpp:363-366   decrypt in place (relay_server.cpp:327-330 is the same)
//   relay_local.cpp:343       key wipe
// The scaffolding around them (Pipe, Packet, RelayForwardMsg) is this test's
// own minimal stand-in for the relay's types, shaped only so the expressions
// type-check the same way: m_secretKey.bytes is a uint8_t[16] like
// DH_KEY::bytes, get_packet_content() returns char*, get_packet_size() a size_t.
//
// usage: relay_calls            encrypt -> decrypt round trip of one relay chunk (needs the GPU)
//        relay_calls --compile  exit 0 (the build is the test)
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <vector>

#include "cyclone_amd/cyr_rijndael.h"

using namespace cyclone;

namespace {

struct DhKey {
    uint8_t bytes[16];
};
struct Pipe {
    DhKey m_secretKey, m_privateKey;
    Rijndael* m_encrypt = nullptr;
    Rijndael* m_decrypt = nullptr;
};
struct RelayForwardMsg {  // relay_protocol.h:36-42: {int32_t id; int32_t size;}, 8 bytes
    int32_t id;
    int32_t size;
};
class Packet {  // 4-B head + content, content 4-B aligned as in cye_packet.cpp:90-138
public:
    explicit Packet(size_t content) : m_buf(4 + content + 16), m_size(content) {}
    char* get_packet_content() { return m_buf.data() + 4; }
    size_t get_packet_size() const { return m_size; }

private:
    std::vector<char> m_buf;
    size_t m_size;
};

size_t _round16(size_t size) { return ((size & 0xF) == 0) ? size : ((size & (size_t)(~0xF)) + 0x10); }

}  // namespace

int main(int argc, char** argv) {
    if (argc > 1 && !strcmp(argv[1], "--compile")) return 0;
    Pipe p;
    Pipe* pipe = &p;
    for (int i = 0; i < 16; i++) pipe->m_secretKey.bytes[i] = (uint8_t)(0x11 * i + 3);
    for (int i = 0; i < 16; i++) pipe->m_privateKey.bytes[i] = (uint8_t)i;

    // ---- relay_local.cpp:329-334 (verbatim) ----
					pipe->m_encrypt = new Rijndael(pipe->m_secretKey.bytes);

					//create decrypter
					for (size_t i = 0; i < Rijndael::BLOCK_SIZE; i++)
						pipe->m_privateKey.bytes[i] = (uint8_t)(~(pipe->m_privateKey.bytes[i]));
					pipe->m_decrypt = new Rijndael(pipe->m_secretKey.bytes);
    // ---- end ----

    const size_t msgSize = 1000;  // a chunk that is not a multiple of 16, as relay's ring-buffer reads are
    size_t buf_round_size = _round16(msgSize);
    RelayForwardMsg forwardMsg{7, (int32_t)msgSize};
    Packet packet(sizeof(RelayForwardMsg) + buf_round_size);
    memcpy(packet.get_packet_content(), &forwardMsg, sizeof(forwardMsg));
    uint8_t* chunk = (uint8_t*)packet.get_packet_content() + sizeof(forwardMsg);
    for (size_t i = 0; i < buf_round_size; i++) chunk[i] = i < msgSize ? (uint8_t)(i * 7 + 1) : 0xCE;
    std::vector<uint8_t> plain(chunk, chunk + buf_round_size);

    // ---- relay_local.cpp:204-207 (verbatim) ----
			{
				uint8_t* buf = (uint8_t*)packet.get_packet_content() + sizeof(forwardMsg);
				pipe->m_encrypt->encrypt(buf, buf, buf_round_size);
			}
    // ---- end ----
    const bool changed = memcmp(chunk, plain.data(), buf_round_size) != 0;

    // ---- relay_local.cpp:363-366 (verbatim) ----
					{
						uint8_t* buf = (uint8_t*)packet.get_packet_content() + sizeof(RelayForwardMsg);
						pipe->m_decrypt->decrypt(buf, buf, packet.get_packet_size() - sizeof(RelayForwardMsg));
					}
    // ---- end ----
    const bool back = memcmp(chunk, plain.data(), buf_round_size) == 0;

    // ---- relay_local.cpp:343 (verbatim) ----
				memset(pipe->m_secretKey.bytes, 0, Rijndael::BLOCK_SIZE);
    // ---- end ----
    delete pipe->m_encrypt;
    delete pipe->m_decrypt;
    if (!changed || !back) {
        printf("relay_calls: FAILED (ciphertext differs from plaintext: %d, round trip: %d)\n", changed, back);
        return 1;
    }
    printf("relay_calls: ok (relay call expressions, %zu-byte chunk encrypted and decrypted in place)\n",
           buf_round_size);
    return 0;
}
