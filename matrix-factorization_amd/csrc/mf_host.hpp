// mf_host.hpp -- threading helpers of the host-side passes of libmf_hip
// (preprocessing in mf_prep.cpp, evaluation order in mf_sched.cpp).
#pragma once

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <functional>
#include <thread>
#include <vector>

namespace mf {

inline int host_threads() {
    if (const char* s = std::getenv("MF_HOST_THREADS")) {
        const int v = std::atoi(s);
        if (v > 0) return std::min(v, 256);
    }
    const unsigned hw = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(16u, hw));
}

// fn(t, lo, hi) over [0, n) cut into T contiguous chunks
inline void parallel_chunks(int64_t n, int T, const std::function<void(int, int64_t, int64_t)>& fn) {
    if (T <= 1 || n < (int64_t)1 << 16) {
        fn(0, 0, n);
        return;
    }
    std::vector<std::thread> th;
    th.reserve(T);
    for (int t = 0; t < T; ++t) {
        const int64_t lo = n * t / T, hi = n * (t + 1) / T;
        th.emplace_back(fn, t, lo, hi);
    }
    for (auto& x : th) x.join();
}

inline int bucket_bits(int64_t n) {  // 2^R buckets of <= ~16K entries
    int R = 1;
    while (R < 16 && (n >> R) > (1 << 14)) ++R;
    return R;
}

inline uint64_t mix64(uint64_t x) {  // splitmix64 finaliser
    x ^= x >> 30;
    x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27;
    x *= 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

// Stable partition of rows [0, n) into NB buckets: bucket b owns the
// destinations start[b] .. start[b+1], filled in ascending row order (chunk t
// precedes chunk t+1 and each chunk is scattered in order) by emit(dst, row).
template <class F, class E>
void partition_rows(int64_t n, int NB, int T, F bucket, std::vector<int64_t>& start, E emit) {
    const int Tused = (T <= 1 || n < (int64_t)1 << 16) ? 1 : T;
    std::vector<int64_t> count((size_t)Tused * NB, 0);
    parallel_chunks(n, Tused, [&](int t, int64_t lo, int64_t hi) {
        int64_t* c = count.data() + (size_t)t * NB;
        for (int64_t p = lo; p < hi; ++p) ++c[bucket(p)];
    });
    start.assign((size_t)NB + 1, 0);
    int64_t acc = 0;
    for (int b = 0; b < NB; ++b) {
        start[b] = acc;
        for (int t = 0; t < Tused; ++t) {
            int64_t& c = count[(size_t)t * NB + b];
            const int64_t v = c;
            c = acc;  // write cursor of chunk t in bucket b
            acc += v;
        }
    }
    start[NB] = acc;
    parallel_chunks(n, Tused, [&](int t, int64_t lo, int64_t hi) {
        int64_t* cur = count.data() + (size_t)t * NB;
        for (int64_t p = lo; p < hi; ++p) emit(cur[bucket(p)]++, p);
    });
}

// fn(b) for every bucket b, dynamically balanced over T threads; stops early
// once `stop` is set
template <class F>
void for_buckets(int NB, int T, F fn, const std::atomic<int>* stop = nullptr) {
    std::atomic<int> next{0};
    auto work = [&]() {
        for (int b; !(stop && stop->load(std::memory_order_relaxed)) &&
                    (b = next.fetch_add(1)) < NB;)
            fn(b);
    };
    std::vector<std::thread> th;
    for (int t = 1; t < std::min(T, NB); ++t) th.emplace_back(work);
    work();
    for (auto& x : th) x.join();
}

}  // namespace mf
