// Host-side pipeline of ldpc_decode_bits_host (ldpc-sims_amd/csrc/host_pipeline.h) against a fake copy engine,
// built by tests/test_sanitizers.py with -fsanitize=thread and with -fsanitize=address,undefined.  TEST ONLY.
//
// The fake engine runs each slot's "H2D + decode + D2H" asynchronously on its own thread (std::async), with a
// random delay, so the host's conversion of the next chunk, the drain of the previous one and the persistent
// HostPool workers all overlap the engine as on the GPU.  "Decoding" is a deterministic function of the float32
// LLR, so the output checks that every row went through exactly its own slot and chunk.
#include <stdio.h>
#include <stdlib.h>

#include <chrono>
#include <future>
#include <random>
#include <vector>

#include "host_pipeline.h"

static uint8_t fake_bit(float x) { return (uint8_t)((x < 0.0f) ^ ((int)(x * 4.0f) & 1)); }

struct FakeEngine {
    int n;
    int64_t chunk;
    int fail_at;  // submit index that fails (-1: none)
    std::vector<float> hl[2];
    std::vector<uint8_t> hb[2];
    std::future<void> fut[2];
    std::mt19937 rng;
    int submits = 0;
    FakeEngine(int n_, int64_t chunk_, int fail_at_, unsigned seed) : n(n_), chunk(chunk_), fail_at(fail_at_), rng(seed) {
        for (int s = 0; s < 2; ++s) {
            hl[s].assign((size_t)chunk * n, 0.0f);
            hb[s].assign((size_t)chunk * n, 0xAA);
        }
    }
    ~FakeEngine() {
        for (auto& f : fut)
            if (f.valid()) f.wait();  // nothing may outlive the buffers (the real engine syncs its streams)
    }
    float* h_llr(int s) { return hl[s].data(); }
    const uint8_t* h_bits(int s) { return hb[s].data(); }
    int submit(int s, int64_t nr) {
        if (submits++ == fail_at) return -7;
        const int us = (int)(rng() % 300);
        fut[s] = std::async(std::launch::async, [this, s, nr, us] {
            std::this_thread::sleep_for(std::chrono::microseconds(us));
            for (int64_t i = 0; i < nr * n; ++i) hb[s][i] = fake_bit(hl[s][i]);
        });
        return 0;
    }
    int wait(int s) {
        if (fut[s].valid()) fut[s].get();
        return 0;
    }
};

static int run_case(int64_t rows, int n, int64_t chunk, int threads, unsigned seed, int fail_at) {
    std::mt19937 rng(seed);
    std::normal_distribution<double> nd(0.0, 3.0);
    std::vector<double> llr((size_t)(rows + 3) * n);
    for (auto& x : llr) x = nd(rng);
    std::vector<double> out((size_t)(rows + 3) * n, 7.0);
    FakeEngine eng(n, std::min(chunk, std::max<int64_t>(rows, 1)), fail_at, seed);
    const int rc = ldpc::staging_pipeline(eng, llr.data(), rows, n, eng.chunk, threads, out.data());
    if (fail_at >= 0) {
        if (rc != -7) { fprintf(stderr, "expected the injected error, got %d\n", rc); return 1; }
        return 0;
    }
    if (rc != 0) { fprintf(stderr, "rc %d\n", rc); return 1; }
    for (int64_t i = 0; i < rows * n; ++i)
        if (out[i] != (double)fake_bit((float)llr[i])) {
            fprintf(stderr, "rows %lld n %d chunk %lld threads %d: element %lld wrong\n", (long long)rows, n,
                    (long long)chunk, threads, (long long)i);
            return 1;
        }
    for (size_t i = (size_t)rows * n; i < out.size(); ++i)
        if (out[i] != 7.0) { fprintf(stderr, "write past rows\n"); return 1; }
    return 0;
}

int main() {
    int bad = 0;
    const int64_t rows_l[] = {1, 5, 96, 257, 1000};
    const int64_t chunk_l[] = {1, 7, 48, 256, 4096};
    const int thr_l[] = {1, 2, 5, 16};
    unsigned seed = 1;
    for (int64_t rows : rows_l)
        for (int64_t chunk : chunk_l)
            for (int thr : thr_l) bad += run_case(rows, 64, chunk, thr, seed++, -1);
    // error injection at every submit position of a 6-chunk job: returns the error, leaves nothing running
    for (int k = 0; k < 6; ++k) bad += run_case(600, 32, 100, 4, 100 + k, k);
    // two callers at once (separate engines, one shared HostPool: its run() serialises the jobs)
    int r1 = 0, r2 = 0;
    std::thread a([&] { for (int i = 0; i < 6; ++i) r1 += run_case(513, 40, 64, 6, 500 + i, -1); });
    std::thread b([&] { for (int i = 0; i < 6; ++i) r2 += run_case(300, 72, 33, 3, 600 + i, -1); });
    a.join();
    b.join();
    bad += r1 + r2;
    printf("host pipeline: %s\n", bad ? "FAILED" : "ok");
    return bad ? 1 : 0;
}
