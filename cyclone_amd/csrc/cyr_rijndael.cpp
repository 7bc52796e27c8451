// cyr_rijndael.cpp -- cyclone::Rijndael drop-in over the C-ABI (cyaes.h).
#include "cyclone_amd/cyr_rijndael.h"

#include <stdio.h>
#include <stdlib.h>

namespace cyclone {

const Rijndael::BLOCK Rijndael::DefaultIV = {0x00, 0x01, 0x02, 0x03, 0x04, 0x05, 0x06, 0x07,
                                             0x08, 0x09, 0x0a, 0x0b, 0x0c, 0x0d, 0x0e, 0x0f};

Rijndael::~Rijndael() {}

// Fails closed.  The reference's scalar encrypt cannot fail, and the relay
// encrypts in place and never checks a status (relay_local.cpp:206,
// relay_server.cpp:472): a call that returned with its buffer untouched would
// send the plaintext.  So any non-OK status -- a bad argument (the
// reference's assert, cyr_rijndael.cpp:590-591,614-615) or a device error
// (no GPU, CYAES_DEVICE out of range, out of memory) -- aborts, in NDEBUG
// builds too.
[[noreturn]] static void fail(const char* what, int status) {
    fprintf(stderr, "cyclone::Rijndael::%s: %s (status %d); aborting rather than leave the buffer unprocessed\n",
            what, cyaes_strerror(status), status);
    abort();
}

// A key that cannot be expanded (NULL; the reference dereferences it,
// cyr_rijndael.cpp:526-534) would leave a schedule that encrypts with the
// wrong key: fail closed here too.
Rijndael::Rijndael(const BLOCK key) : m_status(CYAES_OK) {
    m_status = cyaes_key_expand(key, &m_key);
    if (m_status != CYAES_OK) fail("Rijndael", m_status);
}

void Rijndael::encrypt(const uint8_t* input, uint8_t* output, size_t size, BLOCK iv) {
    m_status = cyaes_cbc_encrypt(&m_key, input, output, size, iv);
    if (m_status != CYAES_OK) fail("encrypt", m_status);
}

void Rijndael::decrypt(const uint8_t* input, uint8_t* output, size_t size, BLOCK iv) {
    m_status = cyaes_cbc_decrypt(&m_key, input, output, size, iv);
    if (m_status != CYAES_OK) fail("decrypt", m_status);
}

}  // namespace cyclone
