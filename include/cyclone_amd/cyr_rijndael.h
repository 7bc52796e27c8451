/*
 * cyr_rijndael.h -- drop-in for thejinchao/cyclone `cyclone::Rijndael`
 * (source/cyCrypt/crypt/cyr_rijndael.h:11-53): same class name, enum,
 * typedef, static IV, constructor and encrypt/decrypt signatures, so
 * samples/relay/relay_{local,server}.cpp compile unchanged against it.
 * The object holds the same 352-byte schedule (m_Ke/m_Kd); encrypt/decrypt
 * run on the MI355X through the C-ABI in <cyaes.h>.
 *
 * Error behaviour: fail closed.  A size that is not a multiple of 16 or a NULL
 * buffer (the reference's asserts, cyr_rijndael.cpp:590-591,614-615) and any
 * device error (no gfx950 GPU, CYAES_DEVICE out of range, out of memory)
 * abort the process, in NDEBUG builds too: the relay encrypts in place and
 * never checks a status, so a skipped call would send plaintext.
 * last_status() reports the C-ABI status of the last (successful) call.
 */
#pragma once

#include <stddef.h>
#include <stdint.h>

#include "../cyaes.h"

namespace cyclone {

class Rijndael {
public:
    enum { BLOCK_SIZE = 16 };
    typedef uint8_t BLOCK[BLOCK_SIZE];

    // Default Initial Vector (cyr_rijndael.cpp:503-504)
    static const BLOCK DefaultIV;

    // Construct, and expand a user-supplied key material into a session key.
    Rijndael(const BLOCK key);
    ~Rijndael();

    // Encrypt memory, CBC mode (cyr_rijndael.cpp:588-609)
    void encrypt(const uint8_t* input, uint8_t* output, size_t size, BLOCK iv = nullptr);
    // Decrypt memory, CBC mode (cyr_rijndael.cpp:612-635)
    void decrypt(const uint8_t* input, uint8_t* output, size_t size, BLOCK iv = nullptr);

    // Extension: C-ABI status of the last encrypt/decrypt (CYAES_OK, ...).
    int last_status() const { return m_status; }
    // Extension: the expanded schedule, reference layout.
    const cyaes_key& schedule() const { return m_key; }

private:
    cyaes_key m_key;  // m_Ke[ROUNDS+1][BC], m_Kd[ROUNDS+1][BC]
    int m_status;
};

}  // namespace cyclone
