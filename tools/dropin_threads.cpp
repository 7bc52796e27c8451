// tools/dropin_threads.cpp -- the synchronous drop-in cyclone::Rijndael
// (include/cyclone_amd/cyr_rijndael.h) called from T threads at once, the
// way the relay's looper threads call it (relay_local.cpp:206,365, one
// Rijndael pair per pipe, relay_local.cpp:475: one looper per core).  Each
// thread encrypts or decrypts its own 1,472-B chunk in place with iv = nullptr,
// as the relay does, for a fixed time.  One JSON line per thread count.
// usage: build/dropin_threads [--op enc|dec] [--size 1472] [--seconds 2] [--threads 1,2,4,8,16,32,64]
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "cyclone_amd/cyr_rijndael.h"

int main(int argc, char** argv) {
    std::string op = "enc", threads = "1,2,4,8,16,32,64";
    size_t size = 1472;
    double seconds = 2.0;
    for (int i = 1; i + 1 < argc; i += 2) {
        const std::string a = argv[i];
        if (a == "--op") op = argv[i + 1];
        else if (a == "--size") size = strtoul(argv[i + 1], nullptr, 10);
        else if (a == "--seconds") seconds = atof(argv[i + 1]);
        else if (a == "--threads") threads = argv[i + 1];
    }
    size = (size + 15) / 16 * 16;
    std::vector<int> counts;
    for (size_t p = 0; p < threads.size();) {
        size_t q = threads.find(',', p);
        if (q == std::string::npos) q = threads.size();
        counts.push_back(atoi(threads.substr(p, q - p).c_str()));
        p = q + 1;
    }
    const bool dec = op == "dec";
    for (int T : counts) {
        std::vector<cyclone::Rijndael*> pipes;
        std::vector<std::vector<uint8_t>> bufs(T, std::vector<uint8_t>(size));
        for (int t = 0; t < T; t++) {
            uint8_t key[16];
            for (int i = 0; i < 16; i++) key[i] = (uint8_t)(t * 16 + i);
            pipes.push_back(new cyclone::Rijndael(key));
            for (size_t i = 0; i < size; i++) bufs[t][i] = (uint8_t)(i * 7 + t);
            dec ? pipes[t]->decrypt(bufs[t].data(), bufs[t].data(), size) : pipes[t]->encrypt(bufs[t].data(), bufs[t].data(), size);
        }
        std::atomic<bool> stop{false};
        std::vector<uint64_t> n(T, 0);
        std::vector<int> bad(T, 0);
        std::vector<std::thread> th;
        const auto t0 = std::chrono::steady_clock::now();
        for (int t = 0; t < T; t++)
            th.emplace_back([&, t] {
                uint64_t k = 0;
                while (!stop.load(std::memory_order_relaxed)) {
                    if (dec) pipes[t]->decrypt(bufs[t].data(), bufs[t].data(), size);
                    else pipes[t]->encrypt(bufs[t].data(), bufs[t].data(), size);
                    if (pipes[t]->last_status() != CYAES_OK) bad[t]++;
                    k++;
                }
                n[t] = k;
            });
        std::this_thread::sleep_for(std::chrono::duration<double>(seconds));
        stop = true;
        for (auto& x : th) x.join();
        const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        uint64_t calls = 0;
        int errs = 0;
        for (int t = 0; t < T; t++) calls += n[t], errs += bad[t];
        printf("{\"metric\": \"drop-in %s calls/s (C++ threads)\", \"size\": %zu, \"threads\": %d, \"calls_per_s\": %.0f, "
               "\"gibs\": %.4f, \"us_per_call_per_thread\": %.1f, \"errors\": %d}\n",
               dec ? "decrypt" : "encrypt", size, T, calls / el, calls * (double)size / el / (1 << 30),
               el * 1e6 * T / (calls ? calls : 1), errs);
        fflush(stdout);
        for (auto* p : pipes) delete p;
    }
    return 0;
}
