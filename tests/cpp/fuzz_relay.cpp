// fuzz_relay.cpp -- randomized robustness test of the relay wire-format code
// (include/cyaes_relay.h, cyclone_amd/csrc/cyaes_relay.cpp), host only, built
// with AddressSanitizer + UndefinedBehaviorSanitizer by tests/test_relay.py.
//
// Streams of well-formed RELAY_FORWARD packets (relay_local.cpp:189-201),
// other packet ids, garbage and truncated tails are parsed the way
// Packet::build_from_ringbuf walks a ring buffer (cye_packet.cpp:166-181);
// checks that every reported packet lies inside the stream, that parsing
// stops exactly at an incomplete tail, that payload ranges lie inside their
// packets, and that build -> parse round-trips.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <vector>

#include "cyaes_relay.h"

#define REQUIRE(c)                                                        \
    do {                                                                  \
        if (!(c)) {                                                       \
            fprintf(stderr, "%s:%d: REQUIRE(%s) failed\n", __FILE__, __LINE__, #c); \
            exit(1);                                                      \
        }                                                                 \
    } while (0)

static uint16_t be16(const uint8_t* p) { return (uint16_t)((p[0] << 8) | p[1]); }

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 3000;
    std::mt19937_64 rng(12345);
    auto rnd = [&](uint32_t n) { return (uint32_t)(rng() % n); };
    for (int it = 0; it < iters; it++) {
        std::vector<uint8_t> s;
        std::vector<size_t> built;  // starts of the FORWARD packets we built
        const int parts = 1 + rnd(12);
        for (int p = 0; p < parts; p++) {
            const uint32_t kind = rnd(10);
            if (kind < 6) {  // RELAY_FORWARD
                const uint32_t size = rnd(4) ? rnd(3000) : rnd(CYAES_RELAY_MAX_CHUNK + 1);
                std::vector<uint8_t> chunk(size);
                for (auto& b : chunk) b = (uint8_t)rng();
                const size_t at = s.size();
                s.resize(at + cyaes_relay_packet_bytes(size));
                const uint32_t n = cyaes_relay_build_forward(s.data() + at, (int32_t)rng(), chunk.data(), size);
                REQUIRE(n == cyaes_relay_packet_bytes(size));
                REQUIRE(cyaes_relay_forward_size(s.data() + at) == (int32_t)size);
                REQUIRE(size == 0 || memcmp(s.data() + at + CYAES_RELAY_PAYLOAD_OFFSET, chunk.data(), size) == 0);
                for (uint32_t i = size; i < cyaes_relay_round16(size); i++)
                    REQUIRE(s[at + CYAES_RELAY_PAYLOAD_OFFSET + i] == CYAES_RELAY_PAD);
                built.push_back(at);
            } else if (kind < 8) {  // another packet id, any size
                const uint32_t psize = rnd(2000);
                const size_t at = s.size();
                s.resize(at + 4 + psize);
                s[at] = (uint8_t)(psize >> 8);
                s[at + 1] = (uint8_t)psize;
                const uint16_t id = (uint16_t)rnd(0x10000);
                s[at + 2] = (uint8_t)(id >> 8);
                s[at + 3] = (uint8_t)id;
                for (uint32_t i = 0; i < psize; i++) s[at + 4 + i] = (uint8_t)rng();
            } else {  // garbage
                const uint32_t g = rnd(64);
                for (uint32_t i = 0; i < g; i++) s.push_back((uint8_t)rng());
            }
        }
        if (rnd(2)) s.resize(rnd((uint32_t)s.size() + 1));  // truncated tail
        const size_t len = s.size();
        // exact-size heap copy so ASan catches any read past the end
        uint8_t* buf = (uint8_t*)malloc(len ? len : 1);
        if (len) memcpy(buf, s.data(), len);
        const uint32_t cap = (uint32_t)(len / 4 + 1);
        std::vector<uint64_t> off(cap);
        std::vector<uint32_t> sz(cap);
        std::vector<uint16_t> id(cap);
        size_t used = 0;
        const uint32_t np = cyaes_relay_parse(buf, len, off.data(), sz.data(), id.data(), cap, &used);
        size_t pos = 0;
        for (uint32_t k = 0; k < np; k++) {
            REQUIRE(off[k] == pos);
            REQUIRE(pos + 4 + sz[k] <= len);
            REQUIRE(sz[k] == be16(buf + pos) && id[k] == be16(buf + pos + 2));
            pos += 4 + sz[k];
        }
        REQUIRE(used == pos && used <= len);
        REQUIRE(len - used < 4 || len - used < 4 + (size_t)be16(buf + used));  // stopped at an incomplete tail
        // a smaller max_packets stops early and reports the prefix it walked
        if (np > 1) {
            size_t used2 = 0;
            REQUIRE(cyaes_relay_parse(buf, len, nullptr, nullptr, nullptr, np - 1, &used2) == np - 1);
            REQUIRE(used2 == off[np - 1]);
        }
        std::vector<uint64_t> po(np + 1);
        std::vector<uint32_t> pl(np + 1);
        const int64_t j = cyaes_relay_payloads(off.data(), sz.data(), id.data(), np, 1000, po.data(), pl.data());
        if (j >= 0) {
            uint32_t fwd = 0;
            for (uint32_t k = 0; k < np; k++) fwd += id[k] == CYAES_RELAY_FORWARD && sz[k] > 8;
            REQUIRE((uint32_t)j == fwd);
            for (int64_t q = 0; q < j; q++) {
                REQUIRE(pl[q] % 16 == 0 && pl[q] > 0);
                REQUIRE(po[q] >= 1000 + CYAES_RELAY_PAYLOAD_OFFSET && po[q] - 1000 + pl[q] <= used);
            }
        }
        // a stream of FORWARD packets only (no garbage, no foreign ids) parses back exactly
        if (built.size() == (size_t)parts && !built.empty()) {
            size_t whole = 0;
            for (size_t at : built) {
                const size_t end = at + cyaes_relay_packet_bytes((uint32_t)cyaes_relay_forward_size(s.data() + at));
                if (end <= len) whole++;
            }
            REQUIRE(np == whole);
            for (uint32_t k = 0; k < np; k++) REQUIRE(off[k] == built[k] && id[k] == CYAES_RELAY_FORWARD);
        }
        free(buf);
    }
    // NULL / edge arguments
    REQUIRE(cyaes_relay_parse(nullptr, 100, nullptr, nullptr, nullptr, 10, nullptr) == 0);
    REQUIRE(cyaes_relay_build_forward(nullptr, 1, nullptr, 0) == 0);
    uint8_t pkt[16];
    REQUIRE(cyaes_relay_build_forward(pkt, 1, nullptr, 0) == 12);
    REQUIRE(cyaes_relay_payloads(nullptr, nullptr, nullptr, 0, 0, nullptr, nullptr) == 0);
    REQUIRE(cyaes_relay_payloads(nullptr, nullptr, nullptr, 1, 0, nullptr, nullptr) == -1);
    printf("fuzz_relay: %d streams ok\n", iters);
    return 0;
}
