/*
 * oracle/aes_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the reference's cyCrypt AES path
 * (thejinchao/cyclone, source/cyCrypt/crypt/cyr_rijndael.{h,cpp}).  It is the
 * parity checker for the HIP product path and the "port" CPU baseline timed
 * by bench.py.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it; the product library (cyclone_amd/libcyaes.so)
 * never links or calls it.
 *
 * Pinning: checked against the reference's own known-answer test
 * (test/unit/cyt_unit_crypt.cpp:177-186), the IV-streaming and in-place
 * properties of that test (:203-231), FIPS-197 C.1 / A.1, NIST SP 800-38A
 * F.2.1-F.2.2, SHA-256 digests of the reference's static tables
 * (tests/golden/ref_tables.json, produced by tests/golden/gen_ref_tables.py
 * from the reference source text) and OpenSSL EVP_aes_128_cbc vectors
 * (tests/golden/gen_openssl_vectors.c).  See tests/test_oracle.py.
 *
 * The reference ships its tables as literals (cyr_rijndael.cpp:25-501); here
 * they are regenerated from GF(2^8) arithmetic and the table digests pin the
 * regeneration.  Word packing, round structure, CBC chaining and the IV
 * in/out contract follow the reference line for line (citations inline).
 */
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define CYO_ROUNDS 10 /* cyr_rijndael.h:48  ROUNDS=10, BC=4, KC=4 */
#define CYO_BC 4
#define CYO_KC 4
#define CYO_BLOCK 16  /* cyr_rijndael.h:14 */

/* ---- static tables (cyr_rijndael.cpp:25-501) -------------------------- */
static uint8_t sm_S[256], sm_Si[256];
static uint32_t sm_T1[256], sm_T2[256], sm_T3[256], sm_T4[256];
static uint32_t sm_T5[256], sm_T6[256], sm_T7[256], sm_T8[256];
static uint32_t sm_U1[256], sm_U2[256], sm_U3[256], sm_U4[256];
static uint8_t sm_rcon[30];

/* DefaultIV, cyr_rijndael.cpp:503-504 */
static const uint8_t kDefaultIV[16] = {0x00, 0x01, 0x02, 0x03, 0x04, 0x05, 0x06, 0x07,
                                       0x08, 0x09, 0x0a, 0x0b, 0x0c, 0x0d, 0x0e, 0x0f};

static uint8_t gf_mul(uint8_t a, uint8_t b) {
    uint8_t r = 0;
    while (b) {
        if (b & 1) r ^= a;
        a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
        b >>= 1;
    }
    return r;
}

static uint32_t pack_be(uint8_t b3, uint8_t b2, uint8_t b1, uint8_t b0) {
    return ((uint32_t)b3 << 24) | ((uint32_t)b2 << 16) | ((uint32_t)b1 << 8) | (uint32_t)b0;
}

static void init_tables_once(void) {
    /* S-box: multiplicative inverse in GF(2^8) followed by the affine map. */
    uint8_t inv[256];
    inv[0] = 0;
    for (int x = 1; x < 256; x++)
        for (int y = 1; y < 256; y++)
            if (gf_mul((uint8_t)x, (uint8_t)y) == 1) { inv[x] = (uint8_t)y; break; }
    for (int x = 0; x < 256; x++) {
        uint8_t b = inv[x], s = 0x63;
        for (int i = 0; i < 5; i++) s ^= (uint8_t)((b << i) | (b >> ((8 - i) & 7)));
        sm_S[x] = s;
        sm_Si[s] = (uint8_t)x;
    }
    for (int x = 0; x < 256; x++) {
        uint8_t s = sm_S[x], si = sm_Si[x];
        uint8_t s2 = gf_mul(s, 2), s3 = gf_mul(s, 3);
        /* encryption T-tables: MixColumns columns (2,1,1,3) and rotations */
        sm_T1[x] = pack_be(s2, s, s, s3);
        sm_T2[x] = pack_be(s3, s2, s, s);
        sm_T3[x] = pack_be(s, s3, s2, s);
        sm_T4[x] = pack_be(s, s, s3, s2);
        /* decryption T-tables: InvMixColumns columns (14,9,13,11) and rotations */
        uint8_t e = gf_mul(si, 14), n = gf_mul(si, 9), d = gf_mul(si, 13), b = gf_mul(si, 11);
        sm_T5[x] = pack_be(e, n, d, b);
        sm_T6[x] = pack_be(b, e, n, d);
        sm_T7[x] = pack_be(d, b, e, n);
        sm_T8[x] = pack_be(n, d, b, e);
        /* key-schedule InvMixColumn tables (no S-box) */
        uint8_t xe = gf_mul((uint8_t)x, 14), xn = gf_mul((uint8_t)x, 9);
        uint8_t xd = gf_mul((uint8_t)x, 13), xb = gf_mul((uint8_t)x, 11);
        sm_U1[x] = pack_be(xe, xn, xd, xb);
        sm_U2[x] = pack_be(xb, xe, xn, xd);
        sm_U3[x] = pack_be(xd, xb, xe, xn);
        sm_U4[x] = pack_be(xn, xd, xb, xe);
    }
    uint8_t r = 1;
    for (int i = 0; i < 30; i++) { sm_rcon[i] = r; r = gf_mul(r, 2); }
}

static pthread_once_t g_once = PTHREAD_ONCE_INIT;
static void init_tables(void) { pthread_once(&g_once, init_tables_once); }

/* Exposes the regenerated tables so tests can hash them against the
 * reference digests.  which: 0=S 1=Si 2..9=T1..T8 10..13=U1..U4 14=rcon */
const void* cyo_table(int which, size_t* nbytes) {
    init_tables();
    static const void* ptrs[15];
    static const size_t sizes[15] = {256, 256, 1024, 1024, 1024, 1024, 1024, 1024, 1024,
                                     1024, 1024, 1024, 1024, 1024, 30};
    ptrs[0] = sm_S;  ptrs[1] = sm_Si;
    ptrs[2] = sm_T1; ptrs[3] = sm_T2; ptrs[4] = sm_T3; ptrs[5] = sm_T4;
    ptrs[6] = sm_T5; ptrs[7] = sm_T6; ptrs[8] = sm_T7; ptrs[9] = sm_T8;
    ptrs[10] = sm_U1; ptrs[11] = sm_U2; ptrs[12] = sm_U3; ptrs[13] = sm_U4;
    ptrs[14] = sm_rcon;
    if (which < 0 || which > 14) return NULL;
    if (nbytes) *nbytes = sizes[which];
    return ptrs[which];
}

const uint8_t* cyo_default_iv(void) { return kDefaultIV; }

/* ---- Rijndael object (cyr_rijndael.h:48-52) --------------------------- */
typedef struct cyo_key {
    uint32_t Ke[CYO_ROUNDS + 1][CYO_BC]; /* m_Ke */
    uint32_t Kd[CYO_ROUNDS + 1][CYO_BC]; /* m_Kd */
} cyo_key;

size_t cyo_key_size(void) { return sizeof(cyo_key); }

/* Rijndael::Rijndael(const BLOCK key), cyr_rijndael.cpp:507-572 */
void cyo_key_expand(const uint8_t key[16], cyo_key* k) {
    init_tables();
    memset(k, 0, sizeof(*k));                              /* :509-518 */
    const int ROUND_KEY_COUNT = (CYO_ROUNDS + 1) * CYO_BC; /* :520 */
    uint32_t tk[CYO_KC];
    for (int i = 0; i < CYO_KC; i++)                       /* :526-534 big-endian words */
        tk[i] = pack_be(key[4 * i], key[4 * i + 1], key[4 * i + 2], key[4 * i + 3]);
    int t = 0;
    for (int j = 0; j < CYO_KC && t < ROUND_KEY_COUNT; j++, t++) { /* :536-541 */
        k->Ke[t / CYO_BC][t % CYO_BC] = tk[j];
        k->Kd[CYO_ROUNDS - (t / CYO_BC)][t % CYO_BC] = tk[j];
    }
    uint32_t tt, rconpointer = 0;
    while (t < ROUND_KEY_COUNT) {                          /* :543-561 */
        tt = tk[CYO_KC - 1];
        tk[0] ^= ((uint32_t)sm_S[(tt >> 16) & 0xFF] << 24) ^ ((uint32_t)sm_S[(tt >> 8) & 0xFF] << 16) ^
                 ((uint32_t)sm_S[tt & 0xFF] << 8) ^ (uint32_t)sm_S[(tt >> 24) & 0xFF] ^
                 ((uint32_t)sm_rcon[rconpointer++] << 24);
        for (int i = 1, j = 0; i < CYO_KC;) tk[i++] ^= tk[j++];
        for (int j = 0; j < CYO_KC && t < ROUND_KEY_COUNT; j++, t++) {
            k->Ke[t / CYO_BC][t % CYO_BC] = tk[j];
            k->Kd[CYO_ROUNDS - (t / CYO_BC)][t % CYO_BC] = tk[j];
        }
    }
    for (int r = 1; r < CYO_ROUNDS; r++)                   /* :563-571 InvMixColumn */
        for (int j = 0; j < CYO_BC; j++) {
            tt = k->Kd[r][j];
            k->Kd[r][j] = sm_U1[(tt >> 24) & 0xFF] ^ sm_U2[(tt >> 16) & 0xFF] ^
                          sm_U3[(tt >> 8) & 0xFF] ^ sm_U4[tt & 0xFF];
        }
}

static uint32_t load_be(const uint8_t* p) { return pack_be(p[0], p[1], p[2], p[3]); }

/* Rijndael::_encryptBlock, cyr_rijndael.cpp:638-705 */
static void encrypt_block(const cyo_key* k, const uint8_t* in, uint8_t* result) {
    const uint32_t* Ker = k->Ke[0];
    uint32_t t0 = load_be(in) ^ Ker[0], t1 = load_be(in + 4) ^ Ker[1];
    uint32_t t2 = load_be(in + 8) ^ Ker[2], t3 = load_be(in + 12) ^ Ker[3];
    for (int r = 1; r < CYO_ROUNDS; r++) {                 /* :659-682 */
        Ker = k->Ke[r];
        uint32_t a0 = sm_T1[(t0 >> 24) & 0xFF] ^ sm_T2[(t1 >> 16) & 0xFF] ^ sm_T3[(t2 >> 8) & 0xFF] ^
                      sm_T4[t3 & 0xFF] ^ Ker[0];
        uint32_t a1 = sm_T1[(t1 >> 24) & 0xFF] ^ sm_T2[(t2 >> 16) & 0xFF] ^ sm_T3[(t3 >> 8) & 0xFF] ^
                      sm_T4[t0 & 0xFF] ^ Ker[1];
        uint32_t a2 = sm_T1[(t2 >> 24) & 0xFF] ^ sm_T2[(t3 >> 16) & 0xFF] ^ sm_T3[(t0 >> 8) & 0xFF] ^
                      sm_T4[t1 & 0xFF] ^ Ker[2];
        uint32_t a3 = sm_T1[(t3 >> 24) & 0xFF] ^ sm_T2[(t0 >> 16) & 0xFF] ^ sm_T3[(t1 >> 8) & 0xFF] ^
                      sm_T4[t2 & 0xFF] ^ Ker[3];
        t0 = a0; t1 = a1; t2 = a2; t3 = a3;
    }
    const uint32_t* K = k->Ke[CYO_ROUNDS];                 /* :684-704 last round */
    const uint32_t t[4] = {t0, t1, t2, t3};
    for (int j = 0; j < 4; j++) {
        uint32_t tt = K[j];
        result[4 * j + 0] = (uint8_t)(sm_S[(t[j] >> 24) & 0xFF] ^ (tt >> 24));
        result[4 * j + 1] = (uint8_t)(sm_S[(t[(j + 1) & 3] >> 16) & 0xFF] ^ (tt >> 16));
        result[4 * j + 2] = (uint8_t)(sm_S[(t[(j + 2) & 3] >> 8) & 0xFF] ^ (tt >> 8));
        result[4 * j + 3] = (uint8_t)(sm_S[t[(j + 3) & 3] & 0xFF] ^ tt);
    }
}

/* Rijndael::_decryptBlock, cyr_rijndael.cpp:708-774 */
static void decrypt_block(const cyo_key* k, const uint8_t* in, uint8_t* result) {
    const uint32_t* Kdr = k->Kd[0];
    uint32_t t0 = load_be(in) ^ Kdr[0], t1 = load_be(in + 4) ^ Kdr[1];
    uint32_t t2 = load_be(in + 8) ^ Kdr[2], t3 = load_be(in + 12) ^ Kdr[3];
    for (int r = 1; r < CYO_ROUNDS; r++) {                 /* :728-751 inverse rotation */
        Kdr = k->Kd[r];
        uint32_t a0 = sm_T5[(t0 >> 24) & 0xFF] ^ sm_T6[(t3 >> 16) & 0xFF] ^ sm_T7[(t2 >> 8) & 0xFF] ^
                      sm_T8[t1 & 0xFF] ^ Kdr[0];
        uint32_t a1 = sm_T5[(t1 >> 24) & 0xFF] ^ sm_T6[(t0 >> 16) & 0xFF] ^ sm_T7[(t3 >> 8) & 0xFF] ^
                      sm_T8[t2 & 0xFF] ^ Kdr[1];
        uint32_t a2 = sm_T5[(t2 >> 24) & 0xFF] ^ sm_T6[(t1 >> 16) & 0xFF] ^ sm_T7[(t0 >> 8) & 0xFF] ^
                      sm_T8[t3 & 0xFF] ^ Kdr[2];
        uint32_t a3 = sm_T5[(t3 >> 24) & 0xFF] ^ sm_T6[(t2 >> 16) & 0xFF] ^ sm_T7[(t1 >> 8) & 0xFF] ^
                      sm_T8[t0 & 0xFF] ^ Kdr[3];
        t0 = a0; t1 = a1; t2 = a2; t3 = a3;
    }
    const uint32_t* K = k->Kd[CYO_ROUNDS];                 /* :753-773 last round */
    const uint32_t t[4] = {t0, t1, t2, t3};
    for (int j = 0; j < 4; j++) {
        uint32_t tt = K[j];
        result[4 * j + 0] = (uint8_t)(sm_Si[(t[j] >> 24) & 0xFF] ^ (tt >> 24));
        result[4 * j + 1] = (uint8_t)(sm_Si[(t[(j + 3) & 3] >> 16) & 0xFF] ^ (tt >> 16));
        result[4 * j + 2] = (uint8_t)(sm_Si[(t[(j + 2) & 3] >> 8) & 0xFF] ^ (tt >> 8));
        result[4 * j + 3] = (uint8_t)(sm_Si[t[(j + 1) & 3] & 0xFF] ^ tt);
    }
}

/* Rijndael::_xor, cyr_rijndael.cpp:581-585 */
static void xor_block(uint8_t* buff, const uint8_t* chain) {
    for (int i = 0; i < CYO_BLOCK; i++) buff[i] ^= chain[i];
}

/* Rijndael::encrypt, cyr_rijndael.cpp:588-609.  Returns -1 where the
 * reference would assert (:590-591). */
int cyo_encrypt(const cyo_key* k, const uint8_t* input, uint8_t* output, size_t size, uint8_t* iv) {
    if (!input || !output || (size % CYO_BLOCK) != 0) return -1;
    uint8_t chain[CYO_BLOCK];
    memcpy(chain, iv ? iv : kDefaultIV, CYO_BLOCK);         /* :594-598 */
    for (size_t i = 0; i < size; i += CYO_BLOCK, input += CYO_BLOCK, output += CYO_BLOCK) {
        xor_block(chain, input);                           /* :600-604 */
        encrypt_block(k, chain, output);
        memcpy(chain, output, CYO_BLOCK);
    }
    if (iv) memcpy(iv, chain, CYO_BLOCK);                  /* :607-608 */
    return 0;
}

/* Rijndael::decrypt, cyr_rijndael.cpp:612-635 (in-place safe ordering :626-629) */
int cyo_decrypt(const cyo_key* k, const uint8_t* input, uint8_t* output, size_t size, uint8_t* iv) {
    if (!input || !output || (size % CYO_BLOCK) != 0) return -1;
    uint8_t chain[CYO_BLOCK], temp[CYO_BLOCK];
    memcpy(chain, iv ? iv : kDefaultIV, CYO_BLOCK);
    for (size_t i = 0; i < size; i += CYO_BLOCK, input += CYO_BLOCK, output += CYO_BLOCK) {
        decrypt_block(k, input, temp);
        xor_block(temp, chain);
        memcpy(chain, input, CYO_BLOCK);
        memcpy(output, temp, CYO_BLOCK);
    }
    if (iv) memcpy(iv, chain, CYO_BLOCK);
    return 0;
}

/* ---- synthetic workload ------------------------------ */
static uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* Plaintext: 64-bit word w of payload p = splitmix64(seed + p*2^20 + w),
 * stored little-endian, for payloads [p0, p0+n). payload_bytes % 8 == 0. */
void cyo_fill_synthetic(uint8_t* buf, uint64_t p0, uint64_t n, uint32_t payload_bytes, uint64_t seed) {
    const uint32_t words = payload_bytes / 8;
    for (uint64_t p = 0; p < n; p++) {
        uint64_t* w = (uint64_t*)(buf + p * (uint64_t)payload_bytes);
        for (uint32_t i = 0; i < words; i++) w[i] = splitmix64(seed + ((p0 + p) << 20) + i);
    }
}

/* Session key s: bytes 0-7 = LE splitmix64(seed + 2s), 8-15 = LE splitmix64(seed + 2s + 1). */
void cyo_session_key(uint64_t seed, uint64_t s, uint8_t key[16]) {
    uint64_t a = splitmix64(seed + 2 * s), b = splitmix64(seed + 2 * s + 1);
    memcpy(key, &a, 8);
    memcpy(key + 8, &b, 8);
}

/* ---- batched relay semantics: one independent chain per payload ------- */
typedef struct batch_job {
    int decrypt;
    const cyo_key* keys;        /* nkeys schedules */
    uint32_t payloads_per_key;  /* payload p uses key p / payloads_per_key (0 => key 0) */
    const uint8_t* in;
    uint8_t* out;
    uint64_t p_begin, p_end;
    uint32_t payload_bytes;
} batch_job;

static void* batch_worker(void* arg) {
    batch_job* j = (batch_job*)arg;
    for (uint64_t p = j->p_begin; p < j->p_end; p++) {
        const cyo_key* k = j->payloads_per_key ? &j->keys[p / j->payloads_per_key] : &j->keys[0];
        const uint64_t off = p * (uint64_t)j->payload_bytes;
        if (j->decrypt) cyo_decrypt(k, j->in + off, j->out + off, j->payload_bytes, NULL);
        else cyo_encrypt(k, j->in + off, j->out + off, j->payload_bytes, NULL);
    }
    return NULL;
}

/* Encrypts/decrypts npayloads contiguous payloads, each an independent CBC
 * chain from DefaultIV (relay_local.cpp:206 / relay_server.cpp:329 pass no
 * IV), on nthreads threads (one Rijndael object set per thread, as relay). */
int cyo_batch(int decrypt, const cyo_key* keys, uint32_t payloads_per_key, const uint8_t* in,
              uint8_t* out, uint64_t npayloads, uint32_t payload_bytes, int nthreads) {
    if (payload_bytes % CYO_BLOCK) return -1;
    if (nthreads < 1) nthreads = 1;
    if ((uint64_t)nthreads > npayloads) nthreads = npayloads ? (int)npayloads : 1;
    batch_job* jobs = (batch_job*)calloc((size_t)nthreads, sizeof(batch_job));
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    if (!jobs || !th) { free(jobs); free(th); return -1; }
    for (int t = 0; t < nthreads; t++) {
        jobs[t].decrypt = decrypt;
        jobs[t].keys = keys;
        jobs[t].payloads_per_key = payloads_per_key;
        jobs[t].in = in;
        jobs[t].out = out;
        jobs[t].p_begin = npayloads * (uint64_t)t / (uint64_t)nthreads;
        jobs[t].p_end = npayloads * (uint64_t)(t + 1) / (uint64_t)nthreads;
        jobs[t].payload_bytes = payload_bytes;
    }
    for (int t = 1; t < nthreads; t++) pthread_create(&th[t], NULL, batch_worker, &jobs[t]);
    batch_worker(&jobs[0]);
    for (int t = 1; t < nthreads; t++) pthread_join(th[t], NULL);
    free(jobs);
    free(th);
    return 0;
}

/* Ragged relay stream: payload p = bytes [offsets[p], offsets[p] + nbytes[p])
 * of buf (in place), one independent chain from DefaultIV per payload under
 * one key -- the relay's per-packet calls on a received / sent stream
 * (relay_server.cpp:329 decrypt(buf, buf, packet_size - 8), relay_local.cpp:206
 * encrypt(buf, buf, round16(size))), payloads split over nthreads threads. */
typedef struct ragged_job {
    int decrypt;
    const cyo_key* key;
    uint8_t* buf;
    const uint64_t* offsets;
    const uint32_t* nbytes;
    uint64_t p_begin, p_end;
    int rc;
} ragged_job;

static void* ragged_worker(void* arg) {
    ragged_job* j = (ragged_job*)arg;
    for (uint64_t p = j->p_begin; p < j->p_end; p++) {
        uint8_t* q = j->buf + j->offsets[p];
        const int rc = j->decrypt ? cyo_decrypt(j->key, q, q, j->nbytes[p], NULL)
                                  : cyo_encrypt(j->key, q, q, j->nbytes[p], NULL);
        if (rc) j->rc = rc;
    }
    return NULL;
}

int cyo_batch_ragged(int decrypt, const cyo_key* key, uint8_t* buf, const uint64_t* offsets,
                     const uint32_t* nbytes, uint64_t npayloads, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if ((uint64_t)nthreads > npayloads) nthreads = npayloads ? (int)npayloads : 1;
    ragged_job* jobs = (ragged_job*)calloc((size_t)nthreads, sizeof(ragged_job));
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    if (!jobs || !th) { free(jobs); free(th); return -1; }
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = (ragged_job){decrypt, key, buf, offsets, nbytes, npayloads * (uint64_t)t / (uint64_t)nthreads,
                               npayloads * (uint64_t)(t + 1) / (uint64_t)nthreads, 0};
    }
    for (int t = 1; t < nthreads; t++) pthread_create(&th[t], NULL, ragged_worker, &jobs[t]);
    ragged_worker(&jobs[0]);
    int rc = 0;
    for (int t = 1; t < nthreads; t++) pthread_join(th[t], NULL);
    for (int t = 0; t < nthreads; t++) if (jobs[t].rc) rc = jobs[t].rc;
    free(jobs);
    free(th);
    return rc;
}

/* ---- Adler-32 (cyr_adler32.cpp:66-133), restated step for step ----------
 * BASE 65521 (:12), NMAX 5552 (:13): sums of NMAX bytes fit 32 bits before a
 * modulo.  Edge rules: NULL or len 0 -> INITIAL_ADLER (:72-73); len 1 uses
 * two conditional subtractions (:80-87); len < 16 one subtraction for a and a
 * modulo for sum2 (:90-98). */
#define CYO_ADLER_BASE 65521u
#define CYO_ADLER_NMAX 5552u

uint32_t cyo_adler32(uint32_t adler, const uint8_t* buf, size_t len) {
    if (buf == NULL || len == 0) return 1u;
    uint32_t sum2 = (adler >> 16) & 0xffff;
    adler &= 0xffff;
    if (len == 1) {
        adler += buf[0];
        if (adler >= CYO_ADLER_BASE) adler -= CYO_ADLER_BASE;
        sum2 += adler;
        if (sum2 >= CYO_ADLER_BASE) sum2 -= CYO_ADLER_BASE;
        return adler | (sum2 << 16);
    }
    if (len < 16) {
        while (len--) {
            adler += *buf++;
            sum2 += adler;
        }
        if (adler >= CYO_ADLER_BASE) adler -= CYO_ADLER_BASE;
        sum2 %= CYO_ADLER_BASE;
        return adler | (sum2 << 16);
    }
    while (len >= CYO_ADLER_NMAX) { /* :105-114 */
        len -= CYO_ADLER_NMAX;
        for (unsigned n = 0; n < CYO_ADLER_NMAX; n++) {
            adler += *buf++;
            sum2 += adler;
        }
        adler %= CYO_ADLER_BASE;
        sum2 %= CYO_ADLER_BASE;
    }
    if (len) { /* :117-129 */
        while (len--) {
            adler += *buf++;
            sum2 += adler;
        }
        adler %= CYO_ADLER_BASE;
        sum2 %= CYO_ADLER_BASE;
    }
    return adler | (sum2 << 16);
}
