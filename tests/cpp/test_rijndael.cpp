// test_rijndael.cpp -- the reference's Rijndael TEST_CASE
// (thejinchao/cyclone test/unit/cyt_unit_crypt.cpp:173-248) re-expressed
// against the drop-in cyclone::Rijndael (include/cyclone_amd/cyr_rijndael.h),
// which runs on the MI355X.  Same five properties: known answer, IV
// streaming, in place, random-key round trips, plus size-0 no-op.
//
// usage: test_rijndael tests/golden/ref_kat.txt      (exit 0 = pass)
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "cyclone_amd/cyr_rijndael.h"

using cyclone::Rijndael;

static int g_checks = 0, g_failed = 0;
#define CHECK(cond)                                                      \
    do {                                                                 \
        ++g_checks;                                                      \
        if (!(cond)) {                                                   \
            ++g_failed;                                                  \
            fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #cond); \
        }                                                                \
    } while (0)

static std::vector<uint8_t> unhex(const std::string& s) {
    std::vector<uint8_t> out(s.size() / 2);
    for (size_t i = 0; i < out.size(); i++) out[i] = (uint8_t)strtoul(s.substr(2 * i, 2).c_str(), nullptr, 16);
    return out;
}

static bool load_kat(const char* path, std::vector<uint8_t>* key, std::vector<uint8_t>* plain,
                     std::vector<uint8_t>* cipher, std::vector<uint8_t>* iv_check) {
    FILE* f = fopen(path, "r");
    if (!f) return false;
    char line[1024];
    while (fgets(line, sizeof(line), f)) {
        std::string l(line);
        while (!l.empty() && (l.back() == '\n' || l.back() == '\r')) l.pop_back();
        const size_t eq = l.find('=');
        if (eq == std::string::npos) continue;
        const std::string k = l.substr(0, eq), v = l.substr(eq + 1);
        if (k == "key") *key = unhex(v);
        else if (k == "plaintext") *plain = unhex(v);
        else if (k == "ciphertext") *cipher = unhex(v);
        else if (k == "iv_check") *iv_check = unhex(v);
    }
    fclose(f);
    return key->size() == 16 && plain->size() == 64 && cipher->size() == 64 && iv_check->size() == 16;
}

int main(int argc, char** argv) {
    std::vector<uint8_t> key, plain, cipher, iv_check;
    if (argc < 2 || !load_kat(argv[1], &key, &plain, &cipher, &iv_check)) {
        fprintf(stderr, "usage: %s ref_kat.txt\n", argv[0]);
        return 2;
    }
    Rijndael aes(key.data());
    const size_t n = plain.size();
    CHECK(n % Rijndael::BLOCK_SIZE == 0);
    uint8_t buf1[128] = {0}, buf2[128] = {0};

    // one-shot, iv = nullptr
    aes.encrypt(plain.data(), buf1, n);
    CHECK(aes.last_status() == CYAES_OK);
    CHECK(memcmp(buf1, cipher.data(), n) == 0);
    aes.decrypt(buf1, buf2, n);
    CHECK(memcmp(buf2, plain.data(), n) == 0);

    // IV streaming, 16 bytes per call
    Rijndael::BLOCK iv_buf;
    memcpy(iv_buf, Rijndael::DefaultIV, Rijndael::BLOCK_SIZE);
    for (size_t i = 0; i < n; i += Rijndael::BLOCK_SIZE) aes.encrypt(plain.data() + i, buf1 + i, 16, iv_buf);
    CHECK(memcmp(buf1, cipher.data(), n) == 0);
    CHECK(memcmp(iv_buf, iv_check.data(), 16) == 0);
    memset(buf1, 0, n);
    memcpy(iv_buf, Rijndael::DefaultIV, Rijndael::BLOCK_SIZE);
    for (size_t i = 0; i < n; i += Rijndael::BLOCK_SIZE) aes.decrypt(cipher.data() + i, buf1 + i, 16, iv_buf);
    CHECK(memcmp(buf1, plain.data(), n) == 0);
    CHECK(memcmp(iv_buf, iv_check.data(), 16) == 0);

    // in place
    memcpy(buf1, plain.data(), n);
    aes.encrypt(buf1, buf1, n);
    CHECK(memcmp(buf1, cipher.data(), n) == 0);
    aes.decrypt(buf1, buf1, n);
    CHECK(memcmp(buf1, plain.data(), n) == 0);

    // size 0: no-op, IV untouched
    uint8_t iv_keep[16];
    memset(iv_buf, 0x5a, 16);
    memcpy(iv_keep, iv_buf, 16);
    aes.encrypt(buf1, buf2, 0, iv_buf);
    CHECK(aes.last_status() == CYAES_OK);
    CHECK(memcmp(iv_buf, iv_keep, 16) == 0);

    // random keys, 128-byte round trips (glibc rand(), as the reference)
    for (int t = 0; t < 20; t++) {
        Rijndael::BLOCK key_random;
        for (int i = 0; i < 16; i++) key_random[i] = (uint8_t)(rand() & 0xFF);
        Rijndael aes2(key_random);
        for (int i = 0; i < 128; i++) buf1[i] = (uint8_t)(rand() & 0xFF);
        aes2.encrypt(buf1, buf2, 128);
        aes2.decrypt(buf2, buf2, 128);
        CHECK(memcmp(buf1, buf2, 128) == 0);
    }

    if (g_failed) {
        printf("%d of %d checks FAILED\n", g_failed, g_checks);
        return 1;
    }
    printf("All tests passed (%d assertions)\n", g_checks);
    return 0;
}
