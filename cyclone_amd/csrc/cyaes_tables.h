// cyaes_tables.h -- host-side generation of the device tables and key
// schedules.  The reference ships 12.5 KiB of literal tables
// (cyr_rijndael.cpp:25-501); here they are derived from GF(2^8) arithmetic
// once per process and laid out for the gfx950 kernels.
#pragma once

#include <stdint.h>

#include "cyaes.h"

namespace cyaes {

struct HostTables {
    uint8_t sbox[256];
    uint8_t inv_sbox[256];
    // Encrypt: TL1 (LE bytes 2s,s,s,3s), TL2/TL3/TL4 = rotl8/16/24(TL1).
    uint32_t enc[1024];
    // Decrypt: TL5 (LE bytes 14s,9s,13s,11s), TL7 = rotl16(TL5), Si * 0x01010101.
    uint32_t dec[768];
};

const HostTables& host_tables();

// Reference-layout schedule (Rijndael::Rijndael, cyr_rijndael.cpp:507-572).
void expand_key(const uint8_t key[16], cyaes_key* out);

// Device schedule: 88 little-endian words (ek[44], dk[44]).
void to_device_schedule(const cyaes_key& k, uint32_t out[88]);
void from_device_schedule(const uint32_t in[88], cyaes_key* k);

}  // namespace cyaes
