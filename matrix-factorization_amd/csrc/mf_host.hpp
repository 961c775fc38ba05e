// mf_host.hpp -- threading helpers of the host-side passes of libmf_hip
// (preprocessing in mf_prep.cpp, evaluation order in mf_sched.cpp).
#pragma once

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <functional>
#include <memory>
#include <exception>
#include <mutex>
#include <thread>
#include <vector>

#include <sys/mman.h>

namespace mf {

inline int host_threads() {
    if (const char* s = std::getenv("MF_HOST_THREADS")) {
        const int v = std::atoi(s);
        if (v > 0) return std::min(v, 256);
    }
    const unsigned hw = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(16u, hw));
}

// The first exception thrown on any worker thread (bad_alloc of a scratch
// vector, ...), rethrown on the calling thread after every worker joined --
// an exception escaping a std::thread would call std::terminate instead of
// reaching the C ABI's error path.
struct ThreadErr {
    std::mutex m;
    std::exception_ptr e;
    template <class F>
    void guard(F&& f) {
        try {
            f();
        } catch (...) {
            std::lock_guard<std::mutex> g(m);
            if (!e) e = std::current_exception();
        }
    }
    bool failed() {
        std::lock_guard<std::mutex> g(m);
        return (bool)e;
    }
    void rethrow() {
        if (e) std::rethrow_exception(e);
    }
};

// fn(t, lo, hi) over [0, n) cut into T contiguous chunks
inline void parallel_chunks(int64_t n, int T, const std::function<void(int, int64_t, int64_t)>& fn) {
    if (T <= 1 || n < (int64_t)1 << 16) {
        fn(0, 0, n);
        return;
    }
    ThreadErr err;
    std::vector<std::thread> th;
    th.reserve(T);
    for (int t = 0; t < T; ++t) {
        const int64_t lo = n * t / T, hi = n * (t + 1) / T;
        th.emplace_back([&, t, lo, hi]() { err.guard([&]() { fn(t, lo, hi); }); });
    }
    for (auto& x : th) x.join();
    err.rethrow();
}

// Large host scratch buffers (10^8 entries at C3): anonymous mappings with
// transparent huge pages requested, not value-initialised -- the threads that
// fill them touch their pages first, 2 MB at a time where the kernel grants
// huge pages (a fresh 4 KB-page buffer costs one page fault per 4 KB, and a
// fit() builds several GB of them).
struct MapFree {
    size_t bytes = 0;
    void operator()(void* p) const {
        if (p) munmap(p, bytes);
    }
};
template <class T>
using big_ptr = std::unique_ptr<T[], MapFree>;
template <class T>
big_ptr<T> big_alloc(int64_t n) {
    const size_t bytes = std::max<size_t>(1, (size_t)n * sizeof(T));
    void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) return big_ptr<T>(nullptr, MapFree{0});
#ifdef MADV_HUGEPAGE
    (void)madvise(p, bytes, MADV_HUGEPAGE);
#endif
    return big_ptr<T>(static_cast<T*>(p), MapFree{bytes});
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
    ThreadErr err;
    auto work = [&]() {
        err.guard([&]() {
            for (int b; !(stop && stop->load(std::memory_order_relaxed)) &&
                        (b = next.fetch_add(1)) < NB;)
                fn(b);
        });
    };
    std::vector<std::thread> th;
    for (int t = 1; t < std::min(T, NB); ++t) th.emplace_back(work);
    work();
    for (auto& x : th) x.join();
    err.rethrow();
}

}  // namespace mf
