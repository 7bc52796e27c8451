/*
 * gen_openssl_vectors.c -- golden-vector generator (build container only).
 *
 * Independent of both the oracle and the product: AES-128-CBC comes from
 * OpenSSL's libcrypto (EVP_aes_128_cbc, padding off), which the survey
 * measured bit-identical to the compiled reference Rijndael on 4096x1024 B,
 * 4096x1472 B and 64x65536 B batches.  The reference
 * itself cannot be built here without its cmake-generated cyclone_config.h
 * (DESIGN.md §6), so these vectors carry the reference semantics through
 * that measured equivalence plus the reference's own KAT (ref_kat.json).
 *
 * Build & run (writes tests/golden/openssl_vectors.json):
 *   gcc -O2 -pthread tests/golden/gen_openssl_vectors.c -lcrypto -o /tmp/genv
 *   /tmp/genv > tests/golden/openssl_vectors.json
 *   /tmp/genv e > tests/golden/config_e_passes.json   (config E, per pass)
 *
 * Workload definitions (DESIGN.md §5 / SURVEY.md §8d):
 *   plaintext word w of payload p = splitmix64(0x5EEDC1C1 + (p << 20) + w), LE
 *   key 00..0f (configs A,B,C,E); config D: payload p uses session key p/256,
 *   session key s = LE(splitmix64(S + 2s)) || LE(splitmix64(S + 2s + 1)),
 *   S = 0xC1C10E55D0000000.  Every payload is its own chain from DefaultIV.
 *   digest = (XOR_i h_i, SUM_i h_i), h_i = splitmix64(word_i ^ splitmix64(i)).
 */
#include <openssl/aes.h>
#include <openssl/evp.h>
#include <openssl/sha.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define PT_SEED 0x5EEDC1C1ull
#define KEY_SEED 0xC1C10E55D0000000ull

static uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static void fill(uint8_t* buf, uint64_t p, uint32_t bytes) {
    uint64_t* w = (uint64_t*)buf;
    for (uint32_t i = 0; i < bytes / 8; i++) w[i] = splitmix64(PT_SEED + (p << 20) + i);
}

static void session_key(uint64_t s, uint8_t k[16]) {
    uint64_t a = splitmix64(KEY_SEED + 2 * s), b = splitmix64(KEY_SEED + 2 * s + 1);
    memcpy(k, &a, 8);
    memcpy(k + 8, &b, 8);
}

static const uint8_t IV[16] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15};
static const uint8_t K0[16] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15};

static void cbc(int enc, const uint8_t key[16], const uint8_t iv[16], const uint8_t* in, uint8_t* out, int n) {
    EVP_CIPHER_CTX* c = EVP_CIPHER_CTX_new();
    int l1 = 0, l2 = 0;
    EVP_CipherInit_ex(c, EVP_aes_128_cbc(), NULL, key, iv, enc);
    EVP_CIPHER_CTX_set_padding(c, 0);
    if (n) EVP_CipherUpdate(c, out, &l1, in, n);
    EVP_CipherFinal_ex(c, out + l1, &l2);
    EVP_CIPHER_CTX_free(c);
}

static void hex(const uint8_t* b, size_t n, char* out) {
    for (size_t i = 0; i < n; i++) sprintf(out + 2 * i, "%02x", b[i]);
}

static int unhex(const char* s, uint8_t* out) {
    size_t n = strlen(s) / 2;
    for (size_t i = 0; i < n; i++) sscanf(s + 2 * i, "%2hhx", &out[i]);
    return (int)n;
}

/* ---- config digests, threaded ------------------------------------------ */
typedef struct job {
    uint64_t p0, pb, pe;          /* global payload index base, [pb,pe) relative */
    uint32_t bytes;
    uint32_t ppk;                 /* 0 => key 00..0f */
    uint64_t px, ps, cx, cs;      /* digests of plaintext, ciphertext */
} job;

static void* worker(void* arg) {
    job* j = (job*)arg;
    uint8_t* pt = malloc(j->bytes);
    uint8_t* ct = malloc(j->bytes);
    const uint64_t wpp = j->bytes / 8;
    for (uint64_t p = j->pb; p < j->pe; p++) {
        uint8_t key[16];
        if (j->ppk) session_key(p / j->ppk, key);
        else memcpy(key, K0, 16);
        fill(pt, j->p0 + p, j->bytes);
        cbc(1, key, IV, pt, ct, (int)j->bytes);
        const uint64_t* pw = (const uint64_t*)pt;
        const uint64_t* cw = (const uint64_t*)ct;
        for (uint64_t w = 0; w < wpp; w++) {
            const uint64_t i = p * wpp + w, si = splitmix64(i);
            const uint64_t hp = splitmix64(pw[w] ^ si), hc = splitmix64(cw[w] ^ si);
            j->px ^= hp; j->ps += hp; j->cx ^= hc; j->cs += hc;
        }
    }
    free(pt);
    free(ct);
    return NULL;
}

static void config_digest_q(const char* name, uint64_t p0, uint64_t n, uint32_t bytes, uint32_t ppk, int last,
                            int quote) {
    enum { T = 8 };
    pthread_t th[T];
    job jobs[T];
    for (int t = 0; t < T; t++) {
        memset(&jobs[t], 0, sizeof(job));
        jobs[t].p0 = p0; jobs[t].bytes = bytes; jobs[t].ppk = ppk;
        jobs[t].pb = n * t / T; jobs[t].pe = n * (t + 1) / T;
        pthread_create(&th[t], NULL, worker, &jobs[t]);
    }
    uint64_t px = 0, ps = 0, cx = 0, cs = 0;
    for (int t = 0; t < T; t++) {
        pthread_join(th[t], NULL);
        px ^= jobs[t].px; ps += jobs[t].ps; cx ^= jobs[t].cx; cs += jobs[t].cs;
    }
    printf(quote ? "  \"%s\": {\"p0\": %llu," : "  {\"pass\": %s, \"p0\": %llu, \"npayloads\": %llu, \"payload_bytes\": %u, \"payloads_per_key\": %u, "
           "\"plain_digest\": [\"%016llx\", \"%016llx\"], \"cipher_digest\": [\"%016llx\", \"%016llx\"]}%s\n",
           name, (unsigned long long)p0, (unsigned long long)n, bytes, ppk, (unsigned long long)px,
           (unsigned long long)ps, (unsigned long long)cx, (unsigned long long)cs, last ? "" : ",");
    fflush(stdout);
}

static void config_digest(const char* name, uint64_t p0, uint64_t n, uint32_t bytes, uint32_t ppk, int last) {
    config_digest_q(name, p0, n, bytes, ppk, last, 1);
}

/* Config E (BASELINE.json configs[4]): 2^23 payloads x 64 KiB in fixed passes
 * of 2^18 payloads; pass i covers payloads [i*2^18, (i+1)*2^18)
 * and GPU g of G walks passes [g*32/G, (g+1)*32/G), so these 32 digests cover
 * every shard at G = 1, 2, 4, 8.  "reduced": the same walk with passes of 4096
 * payloads (the 2-rank GPU test). */
static void config_e(void) {
    char name[16];
    printf("{\n \"generator\": \"tests/golden/gen_openssl_vectors.c e (OpenSSL %s)\",\n",
           OpenSSL_version(OPENSSL_VERSION));
    printf(" \"payload_bytes\": 65536,\n \"reduced\": {\"pass_payloads\": 4096, \"passes\": [\n");
    for (int i = 0; i < 8; i++) {
        snprintf(name, sizeof name, "%d", i);
        config_digest_q(name, 4096ull * i, 4096, 65536, 0, i == 7, 0);
    }
    printf(" ]},\n \"full\": {\"pass_payloads\": 262144, \"passes\": [\n");
    for (int i = 0; i < 32; i++) {
        snprintf(name, sizeof name, "%d", i);
        config_digest_q(name, 262144ull * i, 262144, 65536, 0, i == 31, 0);
    }
    printf(" ]}\n}\n");
}

int main(int argc, char** argv) {
    char hb[2 * 65536 + 1];
    if (argc > 1 && !strcmp(argv[1], "e")) {
        config_e();
        return 0;
    }
    uint8_t a[128], b[128];
    printf("{\n \"generator\": \"tests/golden/gen_openssl_vectors.c (OpenSSL %s)\",\n",
           OpenSSL_version(OPENSSL_VERSION));

    /* Published vectors, recomputed and checked. */
    {
        const char* fips_key = "000102030405060708090a0b0c0d0e0f";
        const char* fips_pt = "00112233445566778899aabbccddeeff";
        const char* fips_ct = "69c4e0d86a7b0430d8cdb78070b4c55a";
        uint8_t k[16], p[16], c[16], z[16] = {0};
        unhex(fips_key, k); unhex(fips_pt, p);
        cbc(1, k, z, p, c, 16);  /* one block with zero IV == ECB */
        hex(c, 16, hb);
        if (strcmp(hb, fips_ct)) { fprintf(stderr, "FIPS-197 C.1 mismatch\n"); return 1; }
        printf(" \"fips197_c1\": {\"key\": \"%s\", \"plaintext\": \"%s\", \"ciphertext\": \"%s\"},\n", fips_key, fips_pt,
               fips_ct);
    }
    {
        const char* key = "2b7e151628aed2a6abf7158809cf4f3c";
        const char* pt = "6bc1bee22e409f96e93d7e117393172aae2d8a571e03ac9c9eb76fac45af8e51"
                         "30c81c46a35ce411e5fbc1191a0a52eff69f2445df4f9b17ad2b417be66c3710";
        const char* ct = "7649abac8119b246cee98e9b12e9197d5086cb9b507219ee95db113a917678b2"
                         "73bed6b8e3c1743b7116e69e222295163ff1caa1681fac09120eca307586e1a7";
        uint8_t k[16];
        unhex(key, k); unhex(pt, a);
        cbc(1, k, IV, a, b, 64);
        hex(b, 64, hb);
        if (strcmp(hb, ct)) { fprintf(stderr, "SP800-38A F.2.1 mismatch\n"); return 1; }
        printf(" \"sp800_38a_f21\": {\"key\": \"%s\", \"iv\": \"000102030405060708090a0b0c0d0e0f\", "
               "\"plaintext\": \"%s\", \"ciphertext\": \"%s\"},\n", key, pt, ct);
    }
    /* Key schedules (OpenSSL rd_key words are the reference's BE-packed m_Ke / m_Kd). */
    printf(" \"schedules\": [\n");
    const char* keys[3] = {"000102030405060708090a0b0c0d0e0f", "2b7e151628aed2a6abf7158809cf4f3c",
                           "8e1b04a1c3d5f6a7b8c9dae0f1021324"};
    for (int ki = 0; ki < 3; ki++) {
        uint8_t k[16];
        AES_KEY e, d;
        unhex(keys[ki], k);
        AES_set_encrypt_key(k, 128, &e);
        AES_set_decrypt_key(k, 128, &d);
        /* The generic C layout packs rd_key big-endian (GETU32); the AES-NI
         * layout keeps round-key bytes in memory order.  Normalise to the
         * reference's big-endian words. */
        const uint32_t be0 = ((uint32_t)k[0] << 24) | ((uint32_t)k[1] << 16) | ((uint32_t)k[2] << 8) | k[3];
        if (e.rd_key[0] != be0)
            for (int i = 0; i < 44; i++) {
                e.rd_key[i] = __builtin_bswap32(e.rd_key[i]);
                d.rd_key[i] = __builtin_bswap32(d.rd_key[i]);
            }
        printf("  {\"key\": \"%s\", \"ke\": [", keys[ki]);
        for (int i = 0; i < 44; i++) printf("%s%u", i ? ", " : "", e.rd_key[i]);
        printf("], \"kd\": [");
        for (int i = 0; i < 44; i++) printf("%s%u", i ? ", " : "", d.rd_key[i]);
        printf("]}%s\n", ki < 2 ? "," : "");
    }
    printf(" ],\n");

    /* Per-size vectors: payloads 0 and 1, key 00..0f, DefaultIV each. */
    static uint8_t pt[65536], ct[65536];
    const uint32_t sizes[] = {16, 64, 1024, 1472, 65280, 65536};
    printf(" \"sizes\": [\n");
    for (int si = 0; si < 6; si++) {
        for (uint64_t p = 0; p < 2; p++) {
            uint8_t h[32];
            fill(pt, p, sizes[si]);
            cbc(1, K0, IV, pt, ct, (int)sizes[si]);
            SHA256(ct, sizes[si], h);
            printf("  {\"payload_bytes\": %u, \"p\": %llu, \"cipher_sha256\": \"", sizes[si], (unsigned long long)p);
            hex(h, 32, hb);
            printf("%s\", \"last_block\": \"", hb);
            hex(ct + sizes[si] - 16, 16, hb);
            printf("%s\"", hb);
            if (sizes[si] <= 1472) {
                hex(ct, sizes[si], hb);
                printf(", \"ciphertext\": \"%s\"", hb);
            }
            printf("}%s\n", (si == 5 && p == 1) ? "" : ",");
        }
    }
    printf(" ],\n");
    /* Session keys of config D (first two, for the generator check). */
    {
        uint8_t k[16];
        printf(" \"session_keys\": [");
        for (int s = 0; s < 3; s++) {
            session_key((uint64_t)s, k);
            hex(k, 16, hb);
            printf("%s\"%s\"", s ? ", " : "", hb);
        }
        printf("],\n");
    }
    printf(" \"configs\": {\n");
    config_digest("A", 0, 4096, 1024, 0, 0);
    config_digest("B", 0, 1048576, 1472, 0, 0);
    config_digest("D", 0, 4096ull * 256, 1472, 256, 0);
    config_digest("C", 0, 262144, 65536, 0, 0);
    config_digest("E_rank1", 262144, 262144, 65536, 0, 1);
    printf(" }\n}\n");
    return 0;
}
