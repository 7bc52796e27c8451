// cyaes_tables.cpp -- see cyaes_tables.h.
#include "cyaes_tables.h"

#include <string.h>

#include <mutex>

namespace cyaes {
namespace {

uint8_t xtime(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0x00)); }

uint8_t mul(uint8_t a, uint8_t b) {
    uint8_t r = 0;
    for (; b; b >>= 1, a = xtime(a))
        if (b & 1) r ^= a;
    return r;
}

uint32_t le(uint8_t b0, uint8_t b1, uint8_t b2, uint8_t b3) {
    return (uint32_t)b0 | ((uint32_t)b1 << 8) | ((uint32_t)b2 << 16) | ((uint32_t)b3 << 24);
}

uint32_t rotl(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

HostTables build() {
    HostTables t;
    // S-box via log/antilog tables over generator 3, then the affine map.
    uint8_t exp3[256], log3[256];
    uint8_t x = 1;
    for (int i = 0; i < 255; i++) {
        exp3[i] = x;
        log3[x] = (uint8_t)i;
        x = (uint8_t)(x ^ xtime(x));  // x *= 3
    }
    exp3[255] = exp3[0];
    for (int v = 0; v < 256; v++) {
        uint8_t inv = v ? exp3[(255 - log3[v]) % 255] : 0;
        uint8_t s = inv;
        for (int r = 1; r <= 4; r++) s ^= (uint8_t)((inv << r) | (inv >> (8 - r)));
        s ^= 0x63;
        t.sbox[v] = s;
        t.inv_sbox[s] = (uint8_t)v;
    }
    for (int v = 0; v < 256; v++) {
        const uint8_t s = t.sbox[v], si = t.inv_sbox[v];
        const uint32_t tl1 = le(mul(s, 2), s, s, mul(s, 3));
        t.enc[v] = tl1;
        t.enc[256 + v] = rotl(tl1, 8);
        t.enc[512 + v] = rotl(tl1, 16);
        t.enc[768 + v] = rotl(tl1, 24);
        const uint32_t tl5 = le(mul(si, 14), mul(si, 9), mul(si, 13), mul(si, 11));
        t.dec[v] = tl5;
        t.dec[256 + v] = rotl(tl5, 16);
        t.dec[512 + v] = (uint32_t)si * 0x01010101u;
    }
    return t;
}

uint32_t bswap(uint32_t v) { return __builtin_bswap32(v); }

}  // namespace

const HostTables& host_tables() {
    static HostTables tables;
    static std::once_flag once;
    std::call_once(once, [] { tables = build(); });
    return tables;
}

void expand_key(const uint8_t key[16], cyaes_key* out) {
    const HostTables& t = host_tables();
    // FIPS-197 KeyExpansion on bytes: w[i] is 4 bytes, 44 words.
    uint8_t w[44][4];
    memcpy(w, key, 16);
    uint8_t rcon = 1;
    for (int i = 4; i < 44; i++) {
        uint8_t tmp[4] = {w[i - 1][0], w[i - 1][1], w[i - 1][2], w[i - 1][3]};
        if (i % 4 == 0) {
            const uint8_t first = tmp[0];
            tmp[0] = (uint8_t)(t.sbox[tmp[1]] ^ rcon);
            tmp[1] = t.sbox[tmp[2]];
            tmp[2] = t.sbox[tmp[3]];
            tmp[3] = t.sbox[first];
            rcon = xtime(rcon);
        }
        for (int b = 0; b < 4; b++) w[i][b] = (uint8_t)(w[i - 4][b] ^ tmp[b]);
    }
    // Reference packing: big-endian words, Ke[r][c] = w[4r+c] (cyr_rijndael.cpp:526-541).
    for (int r = 0; r <= CYAES_ROUNDS; r++)
        for (int c = 0; c < 4; c++) {
            const uint8_t* b = w[4 * r + c];
            out->ke[r][c] = ((uint32_t)b[0] << 24) | ((uint32_t)b[1] << 16) | ((uint32_t)b[2] << 8) | b[3];
        }
    // Equivalent inverse cipher schedule: Kd[r] = InvMixColumns(Ke[10-r]) for
    // r = 1..9, plain for r = 0 and 10 (cyr_rijndael.cpp:540,559,563-571).
    for (int r = 0; r <= CYAES_ROUNDS; r++)
        for (int c = 0; c < 4; c++) {
            const uint8_t* b = w[4 * (CYAES_ROUNDS - r) + c];
            uint8_t o[4] = {b[0], b[1], b[2], b[3]};
            if (r > 0 && r < CYAES_ROUNDS) {
                o[0] = (uint8_t)(mul(b[0], 14) ^ mul(b[1], 11) ^ mul(b[2], 13) ^ mul(b[3], 9));
                o[1] = (uint8_t)(mul(b[0], 9) ^ mul(b[1], 14) ^ mul(b[2], 11) ^ mul(b[3], 13));
                o[2] = (uint8_t)(mul(b[0], 13) ^ mul(b[1], 9) ^ mul(b[2], 14) ^ mul(b[3], 11));
                o[3] = (uint8_t)(mul(b[0], 11) ^ mul(b[1], 13) ^ mul(b[2], 9) ^ mul(b[3], 14));
            }
            out->kd[r][c] = ((uint32_t)o[0] << 24) | ((uint32_t)o[1] << 16) | ((uint32_t)o[2] << 8) | o[3];
        }
}

void to_device_schedule(const cyaes_key& k, uint32_t out[88]) {
    for (int r = 0; r <= CYAES_ROUNDS; r++)
        for (int c = 0; c < 4; c++) {
            out[4 * r + c] = bswap(k.ke[r][c]);
            out[44 + 4 * r + c] = bswap(k.kd[r][c]);
        }
}

void from_device_schedule(const uint32_t in[88], cyaes_key* k) {
    for (int r = 0; r <= CYAES_ROUNDS; r++)
        for (int c = 0; c < 4; c++) {
            k->ke[r][c] = bswap(in[4 * r + c]);
            k->kd[r][c] = bswap(in[44 + 4 * r + c]);
        }
}

}  // namespace cyaes
