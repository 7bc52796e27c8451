// cyr_rijndael.cpp -- cyclone::Rijndael drop-in over the C-ABI (cyaes.h).
#include "cyclone_amd/cyr_rijndael.h"

#include <assert.h>

namespace cyclone {

const Rijndael::BLOCK Rijndael::DefaultIV = {0x00, 0x01, 0x02, 0x03, 0x04, 0x05, 0x06, 0x07,
                                             0x08, 0x09, 0x0a, 0x0b, 0x0c, 0x0d, 0x0e, 0x0f};

Rijndael::Rijndael(const BLOCK key) : m_status(CYAES_OK) { m_status = cyaes_key_expand(key, &m_key); }

Rijndael::~Rijndael() {}

void Rijndael::encrypt(const uint8_t* input, uint8_t* output, size_t size, BLOCK iv) {
    m_status = cyaes_cbc_encrypt(&m_key, input, output, size, iv);
    assert(m_status == CYAES_OK);
}

void Rijndael::decrypt(const uint8_t* input, uint8_t* output, size_t size, BLOCK iv) {
    m_status = cyaes_cbc_decrypt(&m_key, input, output, size, iv);
    assert(m_status == CYAES_OK);
}

}  // namespace cyclone
