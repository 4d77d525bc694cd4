// host_pipeline.h — the host side of ldpc_decode_bits_host (the drop-in for decode_bits,
// pytorch/ofdm/ofdm_functions.py:131-163), in plain C++ with no HIP dependency: the persistent worker pool
// for the staging copies and the two-slot chunk pipeline.  abi.hip instantiates the pipeline with its HIP
// engine (pinned buffers, two streams, events); tests/host/test_host_pipeline.cpp instantiates it with a
// fake copy engine (a thread per slot) and runs it under ThreadSanitizer and Address/UBSanitizer.
#pragma once
#include <stdint.h>

#include <emmintrin.h>

#include <algorithm>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace ldpc {

// Host-side work of one chunk split over worker threads (the staging copies are memory-bound).  The workers
// are created once per process and parked on a condition variable between jobs: spawning them per chunk
// cost ~30 us x threads x 2 per chunk.  One job at a time (run_mtx); the caller thread takes slice 0.
class HostPool {
  public:
    static HostPool& get() {
        static HostPool p;
        return p;
    }
    void run(int slices, const std::function<void(int)>& job) {
        std::lock_guard<std::mutex> one(run_mtx_);
        ensure(slices - 1);
        {
            std::lock_guard<std::mutex> lk(m_);
            job_ = &job;
            nslices_ = slices;
            pending_ = slices - 1;
            ++gen_;
        }
        cv_.notify_all();
        job(0);
        std::unique_lock<std::mutex> lk(m_);
        done_.wait(lk, [&] { return pending_ == 0; });
        job_ = nullptr;
    }
    ~HostPool() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : workers_) t.join();
    }

  private:
    void ensure(int n) {
        while ((int)workers_.size() < n) {
            const int id = (int)workers_.size() + 1;  // slice index served by this worker
            workers_.emplace_back([this, id] { loop(id); });
        }
    }
    void loop(int id) {
        int64_t seen = 0;
        for (;;) {
            const std::function<void(int)>* job;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                if (id >= nslices_) continue;  // not part of this job
                job = job_;
            }
            (*job)(id);
            {
                std::lock_guard<std::mutex> lk(m_);
                if (--pending_ == 0) done_.notify_one();
            }
        }
    }
    std::mutex run_mtx_, m_;
    std::condition_variable cv_, done_;
    std::vector<std::thread> workers_;
    const std::function<void(int)>* job_ = nullptr;
    int64_t gen_ = 0;
    int nslices_ = 0, pending_ = 0;
    bool stop_ = false;
};

template <class F>
void parallel_rows(int64_t rows, int threads, F&& f) {
    if (threads <= 1 || rows < 2 * threads) {
        f((int64_t)0, rows);
        return;
    }
    const int64_t per = (rows + threads - 1) / threads;
    const std::function<void(int)> job = [&](int t) {
        const int64_t a = t * per, b = std::min(rows, a + per);
        if (a < b) f(a, b);
    };
    HostPool::get().run(threads, job);
}

// The staging copies with streaming (non-temporal) stores: neither destination is read again by this core —
// the pinned float32 buffer goes to the GPU by DMA, the float64 output to the caller — and a plain store
// first reads the line it writes (read-for-ownership), a third of these copies' memory traffic.  Each
// slice ends with an sfence: streaming stores are weakly ordered, and the pool's completion handshake must not
// overtake them.
inline void cvt_f64_f32_stream(const double* s, float* d, int64_t cnt) {
    int64_t i = 0;
    for (; i < cnt && (reinterpret_cast<uintptr_t>(d + i) & 15); ++i) d[i] = (float)s[i];
    for (; i + 4 <= cnt; i += 4) {
        const __m128 lo = _mm_cvtpd_ps(_mm_loadu_pd(s + i)), hi = _mm_cvtpd_ps(_mm_loadu_pd(s + i + 2));
        _mm_stream_ps(d + i, _mm_movelh_ps(lo, hi));
    }
    for (; i < cnt; ++i) d[i] = (float)s[i];
    _mm_sfence();
}
inline void expand_u8_f64_stream(const uint8_t* s, double* d, int64_t cnt) {
    int64_t i = 0;
    for (; i < cnt && (reinterpret_cast<uintptr_t>(d + i) & 15); ++i) d[i] = (double)s[i];
    for (; i + 2 <= cnt; i += 2) _mm_stream_pd(d + i, _mm_set_pd((double)s[i + 1], (double)s[i]));
    for (; i < cnt; ++i) d[i] = (double)s[i];
    _mm_sfence();
}

// The two-slot staging pipeline.  Engine (one chunk of `chunk` rows per slot):
//   float* h_llr(int slot)                  host staging buffer, chunk x n float32
//   const uint8_t* h_bits(int slot)         host result buffer, chunk x n bytes
//   int submit(int slot, int64_t nrows)     asynchronously: copy h_llr in, decode, copy the bits out into
//                                           h_bits, then mark the slot complete; 0 or an error code
//   int wait(int slot)                      block until the slot's last submit completed; 0 or an error code
// While the engine works on chunk c in slot c & 1, the host converts chunk c + 1 (float64 -> float32, the
// reference's torch.tensor(..., dtype=torch.float), ofdm_functions.py:156) into the other slot and, before
// reusing a slot, drains the chunk it held (uint8 bits -> 0.0 / 1.0 float64 into `out`, :161).
template <class Engine>
int staging_pipeline(Engine& eng, const double* llr, int64_t rows, int n, int64_t chunk, int threads, double* out) {
    const int64_t nchunks = (rows + chunk - 1) / chunk;
    auto drain = [&](int slot, int64_t c) -> int {
        const int rc = eng.wait(slot);
        if (rc != 0) return rc;
        const int64_t r0 = c * chunk, nr = std::min(chunk, rows - r0);
        const uint8_t* hb = eng.h_bits(slot);
        parallel_rows(nr, threads, [&](int64_t a, int64_t b) {
            expand_u8_f64_stream(hb + a * n, out + (r0 + a) * n, (b - a) * n);
        });
        return 0;
    };
    int rc;
    for (int64_t c = 0; c < nchunks; ++c) {
        const int slot = (int)(c & 1);
        if (c >= 2 && (rc = drain(slot, c - 2)) != 0) return rc;
        const int64_t r0 = c * chunk, nr = std::min(chunk, rows - r0);
        float* hl = eng.h_llr(slot);
        parallel_rows(nr, threads, [&](int64_t a, int64_t b) {
            cvt_f64_f32_stream(llr + (r0 + a) * n, hl + a * n, (b - a) * n);
        });
        if ((rc = eng.submit(slot, nr)) != 0) return rc;
    }
    for (int64_t c = std::max<int64_t>(0, nchunks - 2); c < nchunks; ++c)
        if ((rc = drain((int)(c & 1), c)) != 0) return rc;
    return 0;
}

}  // namespace ldpc
