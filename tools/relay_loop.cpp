// tools/relay_loop.cpp -- the relay's whole data path through the batching
// adapter, both ends in one process, host to host.
//
// The reference relay moves a client's bytes like this:
//   relay_local  reads a chunk (<= 0xFF00 B) from the client socket, builds a
//                RELAY_FORWARD packet (header, RelayForwardMsg{id, size}, the
//                chunk, 0xCE padding to 16), encrypts its payload in place and
//                sends the packet on the tunnel (relay_local.cpp:188-217);
//   relay_server receives the tunnel's byte stream, cuts it into packets
//                (Packet::build_from_ringbuf, cye_packet.cpp:166-181), decrypts
//                each payload in place (relay_server.cpp:329) and forwards the
//                first RelayForwardMsg::size bytes to the target.
// Here each looper thread owns P pipes (one session key per pipe, the same
// secret on both ends as relay_local.cpp:329-334 / relay_server.cpp:224-229)
// and runs rounds of: SEAL K chunks per pipe into the pipe's tunnel stream
// (packets back to back, as TCP carries them) -> copy the stream into the
// server's receive buffer (the socket copy; --recv-copy 0 opens the sent bytes
// in place) -> cyaes_relay_parse -> OPEN every packet in place -> compare each
// opened payload with the chunk it came from and the RelayForwardMsg fields
// with the pipe id and chunk size.  All packet memory is one registered pool
// per looper (zero copy: the GPU gathers and scatters the packets), and the
// loopers drain their own completion queues (CYAES_BATCHER_POLL).
//
// Output: one JSON line -- packets/s through both ends, payload GiB/s, rounds,
// packets verified and mismatches.
//
// usage: relay_loop [--threads T] [--pipes P] [--chunks K] [--size B | --size rand:MAX]
//                   [--seconds S] [--recv-copy 0|1] [--verify 0|1] [--batch-mb M] [--delay-us D]
//                   [--depth R]  (rounds in flight per looper; 1 = seal, parse, open in sequence)
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

#include "cyaes.h"
#include "cyaes_batch.h"
#include "cyaes_relay.h"

using Clock = std::chrono::steady_clock;

namespace {

uint64_t splitmix(uint64_t& x) {
    uint64_t z = (x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

struct Slot {  // one round in flight: its tunnel streams and chunk sizes
    uint64_t tx_off = 0, rx_off = 0;
    std::vector<uint32_t> size;  // per (pipe, chunk)
    std::vector<uint64_t> len;   // per pipe: stream bytes
    uint64_t round = 0;
};

struct Looper {
    int id = 0;
    cyaes_batcher* b = nullptr;
    uint32_t pipes = 0, chunks = 0, max_chunk = 0, rand_size = 0, fixed_size = 0, depth = 2;
    bool recv_copy = true, verify = true;
    uint8_t* mem = nullptr;
    uint64_t src_off = 0, pipe_stream = 0;
    std::vector<Slot> slots;
    uint32_t pool = 0;
    std::vector<uint32_t> slot;  // per pipe: session slot (one secret, both ends)
    uint64_t packets = 0, payload = 0, rounds = 0, verified = 0, mismatches = 0;
    int err = CYAES_OK;
    uint64_t rng = 0;
};

// Waits for n completions of this thread's requests (poll mode).  A thread's
// requests complete in submission order, so the n are the oldest n.
int drain(cyaes_batcher* b, uint64_t n) {
    void* users[256];
    int status[256];
    int err = CYAES_OK;
    while (n) {
        const uint32_t got = cyaes_batcher_poll(b, users, status, (uint32_t)std::min<uint64_t>(n, 256));
        for (uint32_t i = 0; i < got; i++)
            if (status[i] && err == CYAES_OK) err = status[i];
        n -= got;
        if (!got) std::this_thread::yield();
    }
    return err;
}

int submit(Looper* L, std::vector<cyaes_pool_req>& reqs) {
    std::vector<int> status(reqs.size(), 0);
    if (cyaes_batcher_submit_pooled(L->b, reqs.data(), (uint32_t)reqs.size(), status.data()) != CYAES_OK)
        return *std::find_if(status.begin(), status.end(), [](int s) { return s != 0; });
    return CYAES_OK;
}

// local end: SEAL chunk k of pipe p (source bytes at a fixed spot) into the pipe's tunnel stream
int seal(Looper* L, Slot& S) {
    const uint32_t P = L->pipes, K = L->chunks;
    std::vector<cyaes_pool_req> reqs;
    reqs.reserve(P * K);
    std::fill(S.len.begin(), S.len.end(), 0);
    for (uint32_t k = 0; k < K; k++)
        for (uint32_t p = 0; p < P; p++) {
            const uint32_t n = L->rand_size ? 1 + (uint32_t)(splitmix(L->rng) % L->rand_size) : L->fixed_size;
            S.size[p * K + k] = n;
            const uint64_t src = L->src_off + (uint64_t)(p * K + k) * L->max_chunk;
            const uint64_t dst = S.tx_off + p * L->pipe_stream + S.len[p];
            reqs.push_back({CYAES_OP_RELAY_SEAL, L->slot[p], (int32_t)(1000 * L->id + p), L->pool, src, dst, n,
                            nullptr, nullptr});
            S.len[p] += cyaes_relay_packet_bytes(n);
        }
    return submit(L, reqs);
}

// the tunnel: the server end receives the stream (a socket copy), cuts it into packets, OPENs them
int open_round(Looper* L, Slot& S) {
    const uint32_t P = L->pipes, K = L->chunks;
    if (L->verify)  // on the wire: ciphertext, not the chunk (each pipe's first packet)
        for (uint32_t p = 0; p < P; p++) {
            const uint32_t n = S.size[p * K];
            const uint8_t* pkt = L->mem + S.tx_off + p * L->pipe_stream;
            const uint8_t* chunk = L->mem + L->src_off + (uint64_t)(p * K) * L->max_chunk;
            L->mismatches += n >= 16 && memcmp(pkt + CYAES_RELAY_PAYLOAD_OFFSET, chunk, 16) == 0;
        }
    std::vector<cyaes_pool_req> reqs;
    reqs.reserve(P * K);
    std::vector<uint64_t> offs(K + 1);
    std::vector<uint32_t> psz(K + 1);
    std::vector<uint16_t> pid(K + 1);
    for (uint32_t p = 0; p < P; p++) {
        uint8_t* tx = L->mem + S.tx_off + p * L->pipe_stream;
        const uint64_t rbase = (L->recv_copy ? S.rx_off : S.tx_off) + p * L->pipe_stream;
        if (L->recv_copy) memcpy(L->mem + rbase, tx, S.len[p]);
        size_t used = 0;
        const uint32_t np = cyaes_relay_parse(L->mem + rbase, S.len[p], offs.data(), psz.data(), pid.data(), K + 1, &used);
        if (np != K || used != S.len[p]) {
            fprintf(stderr, "looper %d pipe %u: parsed %u packets over %zu of %llu bytes\n", L->id, p, np, used,
                    (unsigned long long)S.len[p]);
            return CYAES_EINVAL;
        }
        for (uint32_t k = 0; k < K; k++)
            reqs.push_back({CYAES_OP_RELAY_OPEN, L->slot[p], 0, L->pool, rbase + offs[k], 0,
                            CYAES_RELAY_HEADSIZE + psz[k], nullptr, nullptr});
    }
    return submit(L, reqs);
}

// the target: what relay_server forwards must be the client's chunk
void check_round(Looper* L, const Slot& S) {
    const uint32_t P = L->pipes, K = L->chunks;
    for (uint32_t p = 0; p < P; p++) {
        const uint64_t rbase = (L->recv_copy ? S.rx_off : S.tx_off) + p * L->pipe_stream;
        uint64_t o = 0;
        for (uint32_t k = 0; k < K; k++) {
            const uint32_t n = S.size[p * K + k];
            if (L->verify) {
                const uint8_t* pkt = L->mem + rbase + o;
                const uint8_t* chunk = L->mem + L->src_off + (uint64_t)(p * K + k) * L->max_chunk;
                bool ok = cyaes_relay_forward_id(pkt) == (int32_t)(1000 * L->id + p) &&
                          cyaes_relay_forward_size(pkt) == (int32_t)n &&
                          memcmp(pkt + CYAES_RELAY_PAYLOAD_OFFSET, chunk, n) == 0;
                for (uint32_t i = n; i < cyaes_relay_round16(n); i++)  // the 0xCE padding decrypts back too
                    ok = ok && pkt[CYAES_RELAY_PAYLOAD_OFFSET + i] == CYAES_RELAY_PAD;
                L->mismatches += !ok;
                L->verified++;
            }
            o += cyaes_relay_packet_bytes(n);
            L->payload += n;
        }
    }
    L->packets += (uint64_t)P * K;
    L->rounds++;
}

// Rounds until `until` (at least min_rounds), `depth` rounds in flight: each
// looper keeps `depth` slots, and while the GPU seals or opens one slot's
// packets the looper parses, submits or checks another's.  A looper's requests
// complete in submission order, so it drains them group by group: a sealed
// round is parsed and opened, an opened round is checked and its slot sealed
// again with the next round (depth 1: the sequential seal -> parse -> open).
void run(Looper* L, Clock::time_point until, uint64_t min_rounds) {
    struct Group {
        bool open;
        uint32_t slot;
    };
    std::vector<Group> fifo;  // groups in flight, oldest first
    size_t head = 0;
    const uint64_t n = (uint64_t)L->pipes * L->chunks;
    uint64_t next_round = 0;
    auto more = [&] { return next_round < min_rounds || Clock::now() < until; };
    for (uint32_t s = 0; s < L->depth && more(); s++) {
        L->slots[s].round = next_round++;
        if ((L->err = seal(L, L->slots[s])) != CYAES_OK) return;
        fifo.push_back({false, s});
    }
    while (head < fifo.size()) {
        const Group g = fifo[head++];
        if ((L->err = drain(L->b, n)) != CYAES_OK) return;
        Slot& S = L->slots[g.slot];
        if (!g.open) {
            if ((L->err = open_round(L, S)) != CYAES_OK) return;
            fifo.push_back({true, g.slot});
        } else {
            check_round(L, S);
            if (more()) {
                S.round = next_round++;
                if ((L->err = seal(L, S)) != CYAES_OK) return;
                fifo.push_back({false, g.slot});
            }
        }
    }
}

}  // namespace

int main(int argc, char** argv) {
    uint32_t threads = 8, pipes = 16, chunks = 256, batch_mb = 32, delay_us = 100, recv_copy = 1, verify = 1, depth = 4;
    std::string size_arg = "1472";
    double seconds = 4;
    for (int i = 1; i + 1 < argc; i += 2) {
        const std::string a = argv[i];
        if (a == "--threads") threads = atoi(argv[i + 1]);
        else if (a == "--pipes") pipes = atoi(argv[i + 1]);
        else if (a == "--chunks") chunks = atoi(argv[i + 1]);
        else if (a == "--size") size_arg = argv[i + 1];
        else if (a == "--seconds") seconds = atof(argv[i + 1]);
        else if (a == "--recv-copy") recv_copy = atoi(argv[i + 1]);
        else if (a == "--verify") verify = atoi(argv[i + 1]);
        else if (a == "--batch-mb") batch_mb = atoi(argv[i + 1]);
        else if (a == "--delay-us") delay_us = atoi(argv[i + 1]);
        else if (a == "--depth") depth = atoi(argv[i + 1]);
    }
    uint32_t rand_size = 0, fixed_size = 0;
    if (size_arg.rfind("rand:", 0) == 0) rand_size = std::min<uint32_t>(atoi(size_arg.c_str() + 5), CYAES_RELAY_MAX_CHUNK);
    else fixed_size = std::min<uint32_t>(atoi(size_arg.c_str()), CYAES_RELAY_MAX_CHUNK);
    if (!threads || threads > 16 || !pipes || !chunks || (!rand_size && !fixed_size) || !depth || depth > 8) {  // 16 shards: one queue each
        fprintf(stderr, "bad arguments\n");
        return 1;
    }
    const uint32_t max_chunk = (std::max(rand_size, fixed_size) + 63) & ~63u;
    cyaes_batcher_config cfg = {0, batch_mb << 20, delay_us, 0, 0, 0, CYAES_BATCHER_POLL};
    cyaes_batcher* b = nullptr;
    int st = cyaes_batcher_create(&cfg, &b);
    if (st) {
        fprintf(stderr, "cyaes_batcher_create: %s\n", cyaes_strerror(st));
        return 1;
    }
    std::vector<Looper> L(threads);
    for (uint32_t t = 0; t < threads; t++) {
        Looper& l = L[t];
        l.id = (int)t;
        l.b = b;
        l.pipes = pipes;
        l.chunks = chunks;
        l.max_chunk = max_chunk;
        l.rand_size = rand_size;
        l.fixed_size = fixed_size;
        l.recv_copy = recv_copy != 0;
        l.verify = verify != 0;
        l.rng = 0x5EEDC1C1ull + t;
        l.depth = depth;
        l.pipe_stream = ((uint64_t)chunks * cyaes_relay_packet_bytes(max_chunk) + 4095) & ~4095ull;
        const uint64_t src = (uint64_t)pipes * chunks * max_chunk;
        l.src_off = 0;
        uint64_t at = (src + 4095) & ~4095ull;
        l.slots.resize(depth);
        for (Slot& S : l.slots) {  // per slot: the tunnel streams (sent, received)
            S.tx_off = at;
            S.rx_off = at + pipes * l.pipe_stream;
            at = S.rx_off + pipes * l.pipe_stream;
            S.size.resize((size_t)pipes * chunks);
            S.len.resize(pipes);
        }
        const uint64_t bytes = at;
        const uint64_t tx0 = l.slots[0].tx_off;
        l.mem = static_cast<uint8_t*>(aligned_alloc(4096, bytes));
        uint64_t x = 0xC1C10000ull + t;
        for (uint64_t i = 0; i + 8 <= src; i += 8) {
            const uint64_t v = splitmix(x);
            memcpy(l.mem + i, &v, 8);
        }
        memset(l.mem + tx0, 0, bytes - tx0);
        if ((st = cyaes_batcher_register_pool(b, l.mem, bytes, &l.pool)) != CYAES_OK) {
            fprintf(stderr, "cyaes_batcher_register_pool: %s\n", cyaes_strerror(st));
            return 1;
        }
        l.slot.resize(pipes);
        for (uint32_t p = 0; p < pipes; p++) {
            uint8_t key[16];
            uint64_t kx = 0xDEC0DE00ull + 65536ull * t + p;
            const uint64_t k0 = splitmix(kx), k1 = splitmix(kx);
            memcpy(key, &k0, 8);
            memcpy(key + 8, &k1, 8);
            if ((st = cyaes_batcher_session_open(b, key, &l.slot[p])) != CYAES_OK) {
                fprintf(stderr, "cyaes_batcher_session_open: %s\n", cyaes_strerror(st));
                return 1;
            }
        }
    }
    // Each looper thread: one warm-up round (clock ramp, first touch of the
    // pools; not counted), then the timed rounds once every looper is ready.
    // The same threads do both, so each keeps its own submission shard and
    // completion queue (the batcher gives threads shards round-robin).
    std::atomic<uint32_t> ready{0};
    std::atomic<bool> go{false};
    Clock::time_point t0, until;
    std::vector<std::thread> th;
    for (auto& l : L)
        th.emplace_back([&l, &ready, &go, &until] {
            run(&l, Clock::now(), 1);
            l.packets = l.payload = l.rounds = l.verified = l.mismatches = 0;
            ready.fetch_add(1);
            while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
            run(&l, until, 0);
        });
    while (ready.load() < L.size()) std::this_thread::yield();
    t0 = Clock::now();
    until = t0 + std::chrono::microseconds((int64_t)(seconds * 1e6));
    go.store(true, std::memory_order_release);
    for (auto& t : th) t.join();
    const double s = std::chrono::duration<double>(Clock::now() - t0).count();
    uint64_t packets = 0, payload = 0, rounds = 0, verified = 0, mismatches = 0;
    int err = CYAES_OK;
    for (auto& l : L) {
        packets += l.packets;
        payload += l.payload;
        rounds += l.rounds;
        verified += l.verified;
        mismatches += l.mismatches;
        if (l.err && err == CYAES_OK) err = l.err;
    }
    const int fl = cyaes_batcher_flush(b);
    for (auto& l : L) cyaes_batcher_unregister_pool(b, l.pool);
    cyaes_batcher_destroy(b);
    for (auto& l : L) free(l.mem);
    printf("{\"metric\": \"relay packets/s through both ends (SEAL, tunnel stream, parse, OPEN), host to host\", "
           "\"size\": \"%s\", \"threads\": %u, \"pipes_per_thread\": %u, \"chunks_per_pipe_round\": %u, \"depth\": %u, "
           "\"recv_copy\": %u, \"seconds\": %.2f, \"rounds\": %llu, \"packets\": %llu, \"packets_per_s\": %.0f, "
           "\"payload_gibs\": %.3f, \"verified\": %llu, \"mismatches\": %llu, \"error\": %d}\n",
           size_arg.c_str(), threads, pipes, chunks, depth, recv_copy, s, (unsigned long long)rounds,
           (unsigned long long)packets, packets / s, payload / s / (1ull << 30), (unsigned long long)verified,
           (unsigned long long)mismatches, err ? err : fl);
    return (err || fl || mismatches) ? 2 : 0;
}
