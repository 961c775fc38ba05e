// mf_prep.cpp -- fit() preprocessing at 10^8 rows, host only.
//
// RecommenderBase._preprocess_data (recommender_base.py:120-141 of the
// reference) spends a minute of fit() at C3 scale in pandas: the duplicate
// pair check (:127), the row shuffle X.sample(frac=1) (:131) and the
// first-appearance id maps (:135-138).  The GPU epochs of the same fit take
// ~12 ms each.  These helpers give the same results faster:
//
//   mf_legacy_shuffle    NumPy's legacy RandomState.shuffle (numpy 2.2,
//                        mtrand.pyx _shuffle_raw: for i = n-1 .. 1 swap
//                        x[i], x[random_interval(i)]; distributions.c
//                        random_interval: smallest all-ones mask >= max,
//                        32-bit MT19937 draws & mask until <= max) with the
//                        swap targets drawn a window ahead and prefetched;
//                        the draws, and so the MT state afterwards, are
//                        NumPy's.
//   mf_pairs_duplicated  hash-partition of the rows by (user, item) pair
//                        into cache-sized buckets, a hash set per bucket.
//   mf_factorize         pd.factorize(sort=False): the same partition by
//                        value keeps rows ascending inside a bucket, so a
//                        per-bucket hash table sees each value's first row
//                        first; code = number of first rows before it
//                        (bitmap + prefix popcount).
//   mf_first_appearance  pd.factorize of the shuffled column from dense ids
//                        of the unshuffled one (computed while the
//                        permutation is drawn): first shuffled position per
//                        id by atomic min, ranks by bitmap + prefix popcount.
//   mf_gather            threaded, prefetched dst[p] = src[idx[p]] (64-bit
//                        indices; mf_gather_i32: 32-bit).
//   mf_ids_to_i32,       threaded narrowing of the engine's inputs (ids
//   mf_f64_to_f32        range-checked).
#include <algorithm>
#include <climits>
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <immintrin.h>
#include <memory>
#include <thread>
#include <vector>

#include "../../include/mf_hip.h"
#include "mf_host.hpp"

namespace mf {
void set_error(const char* fmt, ...);
}
using mf::bucket_bits;
using mf::for_buckets;
using mf::host_threads;
using mf::big_alloc;
using mf::big_ptr;
using mf::MapFree;
using mf::mix64;
using mf::parallel_chunks;
using mf::partition_rows;
using mf::set_error;

namespace {

// ---------------------------------------------------------------- MT19937
// The standard Mersenne Twister (Matsumoto & Nishimura 1998) as NumPy's
// legacy bit generator keeps it: key[624] + position, tempered output.
constexpr int kN = 624, kM = 397;
constexpr uint32_t kMatrixA = 0x9908b0dfu, kUpper = 0x80000000u, kLower = 0x7fffffffu;

struct MT {
    uint32_t key[kN];
    int pos;

    void regen() {
        int i = 0;
        for (; i < kN - kM; ++i) {
            const uint32_t y = (key[i] & kUpper) | (key[i + 1] & kLower);
            key[i] = key[i + kM] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA);
        }
        for (; i < kN - 1; ++i) {
            const uint32_t y = (key[i] & kUpper) | (key[i + 1] & kLower);
            key[i] = key[i + (kM - kN)] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA);
        }
        const uint32_t y = (key[kN - 1] & kUpper) | (key[0] & kLower);
        key[kN - 1] = key[kM - 1] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA);
        pos = 0;
    }
    uint32_t next() {
        if (pos == kN) regen();
        uint32_t y = key[pos++];
        y ^= y >> 11;
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= y >> 18;
        return y;
    }
    // random_interval(max) for max <= 0xffffffff
    uint32_t interval(uint32_t max) {
        if (max == 0) return 0;
        uint32_t mask = max;
        mask |= mask >> 1;
        mask |= mask >> 2;
        mask |= mask >> 4;
        mask |= mask >> 8;
        mask |= mask >> 16;
        uint32_t v;
        while ((v = next() & mask) > max) {
        }
        return v;
    }
};

}  // namespace

namespace {

inline uint32_t mt_temper(uint32_t y) {
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

// ---- AVX-512 form of the draws (x86-64 hosts that have it; runtime check)
// The twist 16 words at a time, the tempering 16 outputs at a time, and the
// rejection of 16 outputs against the CURRENT bound at once: output k of a
// chunk is really tested against bound - (accepted before it), which can
// differ from the chunk's bound only for outputs within 16 of it, so a chunk
// with such an output (or a mask change, the draws' end, or the ring's end
// inside it) is done one output at a time instead -- the same outputs
// consumed, the same targets, the same MT position as the scalar loop.
__attribute__((target("avx512f"))) static inline __m512i mt_step16(__m512i cur, __m512i nxt,
                                                                     __m512i far) {
    const __m512i y = _mm512_or_si512(_mm512_and_si512(cur, _mm512_set1_epi32((int)kUpper)),
                                      _mm512_and_si512(nxt, _mm512_set1_epi32((int)kLower)));
    const __m512i one = _mm512_set1_epi32(1);
    const __m512i mag = _mm512_maskz_mov_epi32(_mm512_test_epi32_mask(y, one),
                                               _mm512_set1_epi32((int)kMatrixA));
    return _mm512_xor_si512(_mm512_xor_si512(far, _mm512_srli_epi32(y, 1)), mag);
}

__attribute__((target("avx512f"))) static void mt_regen_512(MT& mt) {
    uint32_t* key = mt.key;
    int i = 0;
    for (; i + 16 <= kN - kM; i += 16)                   // key[i + kM] not yet rewritten
        _mm512_storeu_si512(key + i, mt_step16(_mm512_loadu_si512(key + i),
                                               _mm512_loadu_si512(key + i + 1),
                                               _mm512_loadu_si512(key + i + kM)));
    for (; i < kN - kM; ++i) {
        const uint32_t y = (key[i] & kUpper) | (key[i + 1] & kLower);
        key[i] = key[i + kM] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA);
    }
    for (; i + 16 <= kN - 1; i += 16)                    // key[i - (kN - kM)] already new
        _mm512_storeu_si512(key + i, mt_step16(_mm512_loadu_si512(key + i),
                                               _mm512_loadu_si512(key + i + 1),
                                               _mm512_loadu_si512(key + i + (kM - kN))));
    for (; i < kN - 1; ++i) {
        const uint32_t y = (key[i] & kUpper) | (key[i + 1] & kLower);
        key[i] = key[i + (kM - kN)] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA);
    }
    const uint32_t y = (key[kN - 1] & kUpper) | (key[0] & kLower);
    key[kN - 1] = key[kM - 1] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA);
    mt.pos = 0;
}

__attribute__((target("avx512f"))) static inline __m512i mt_temper16(__m512i y) {
    y = _mm512_xor_si512(y, _mm512_srli_epi32(y, 11));
    y = _mm512_xor_si512(y, _mm512_and_si512(_mm512_slli_epi32(y, 7),
                                             _mm512_set1_epi32((int)0x9d2c5680u)));
    y = _mm512_xor_si512(y, _mm512_and_si512(_mm512_slli_epi32(y, 15),
                                             _mm512_set1_epi32((int)0xefc60000u)));
    return _mm512_xor_si512(y, _mm512_srli_epi32(y, 18));
}

// the draws of one MT block from position p: targets into ring[d & (R-1)],
// each prefetched; returns with p at the block's end or d at total
template <typename E>
__attribute__((target("avx512f"))) static void mt_draws_512(MT& mt, int& p, int64_t& d,
                                                            uint32_t& maxv, int64_t total,
                                                            uint32_t* ring, int64_t R,
                                                            E* data, bool pf_draw) {
    while (p < kN && d < total) {
        if ((p & 15) == 0 && maxv >= 64 && d + 16 < total && (d & (R - 1)) + 16 <= R &&
            __builtin_clz(maxv) == __builtin_clz(maxv - 16)) {
            const uint32_t mask = 0xffffffffu >> __builtin_clz(maxv);
            const __m512i v = _mm512_and_si512(mt_temper16(_mm512_loadu_si512(mt.key + p)),
                                               _mm512_set1_epi32((int)mask));
            const __mmask16 acc = _mm512_cmple_epu32_mask(v, _mm512_set1_epi32((int)maxv));
            const __mmask16 risky =
                _mm512_mask_cmpgt_epu32_mask(acc, v, _mm512_set1_epi32((int)(maxv - 16)));
            if (!risky) {
                uint32_t* o = ring + (d & (R - 1));
                _mm512_mask_compressstoreu_epi32(o, acc, v);
                const int na = __builtin_popcount((unsigned)acc);
                if (pf_draw)
                    for (int q = 0; q < na; ++q) __builtin_prefetch(data + o[q], 1, 1);
                d += na;
                maxv -= (uint32_t)na;
                p += 16;
                continue;
            }
        }
        // one output, as the scalar loop
        const uint32_t mask = 0xffffffffu >> __builtin_clz(maxv);
        const uint32_t v = mt_temper(mt.key[p++]) & mask;
        const uint32_t a = v <= maxv ? 1u : 0u;
        ring[d & (R - 1)] = v;
        if (pf_draw) __builtin_prefetch(data + v, 1, 1);
        d += a;
        maxv -= a;
    }
}

bool use_avx512() {
    static const bool cpu = [] {
        __builtin_cpu_init();
        return __builtin_cpu_supports("avx512f") != 0;
    }();
    const char* env = std::getenv("MF_SHUFFLE_SIMD");        // 0: the scalar draws
    return cpu && !(env && env[0] == '0');
}

// NumPy's _shuffle_raw on x[0..n): for i = n-1 .. 1, swap x[i] with
// x[random_interval(i)].  The draws do not depend on the data, so they are
// made a block of MT outputs at a time, ahead of the swaps that use them
// (each target prefetched), and without a branch per output: every tempered
// output is tested against the current draw's bound and the draw index
// advances by the outcome -- the same outputs consumed, the same rejections
// as MT::interval, the same MT position afterwards.  (The one-thread draw
// loop with its ~30 % mispredicted rejection branch was 0.53 of the 0.65 s
// shuffle of 100M on the GPU box's CPU; tools/shuffle_probe.cpp.)
template <typename E>
void shuffle_raw(MT& mt, E* data, int64_t n) {
    if (n < 2) return;
    const int64_t total = n - 1;                     // draws, for i = n-1 .. 1
    constexpr int64_t kR = 2048, kAhead = 256;       // target ring; swaps this far behind
    uint32_t ring[kR];
    int64_t drawn = 0, done = 0;
    const bool simd = use_avx512();
    // AVX-512 draws come in bursts of a block: their targets are prefetched
    // by the swap loop kPf swaps ahead (MF_SHUFFLE_PF: 0 = at draw time)
    const char* epf = std::getenv("MF_SHUFFLE_PF");
    const int64_t kPf = simd ? (epf ? std::max(0, std::min(248, std::atoi(epf))) : 128) : 0;
    while (done < total) {
        if (drawn < total && simd) {                 // the rest of one MT block (AVX-512)
            if (mt.pos == kN) mt_regen_512(mt);
            int p = mt.pos;
            uint32_t maxv = (uint32_t)(total - drawn);
            int64_t d = drawn;
            mt_draws_512(mt, p, d, maxv, total, ring, kR, data, kPf == 0);
            mt.pos = p;
            drawn = d;
        } else if (drawn < total) {                  // the rest of one MT block
            if (mt.pos == kN) mt.regen();
            int p = mt.pos;
            uint32_t maxv = (uint32_t)(total - drawn);   // bound of draw `drawn`: i = n-1-drawn
            int64_t d = drawn;
            while (p < kN) {
                const uint32_t mask = 0xffffffffu >> __builtin_clz(maxv);   // maxv >= 1
                const uint32_t v = mt_temper(mt.key[p++]) & mask;
                const uint32_t acc = v <= maxv ? 1u : 0u;
                ring[d & (kR - 1)] = v;
                __builtin_prefetch(data + v, 1, 1);
                d += acc;
                maxv -= acc;
                if (d == total) break;
            }
            mt.pos = p;
            drawn = d;
        }
        const int64_t lim = drawn < total ? drawn - kAhead : total;
        for (; done < lim; ++done) {
            if (kPf && done + kPf < drawn) __builtin_prefetch(data + ring[(done + kPf) & (kR - 1)], 1, 1);
            const int64_t i = total - done;
            const int64_t j = ring[done & (kR - 1)];
            const E t = data[i];
            data[i] = data[j];
            data[j] = t;
        }
    }
}

// The same shuffle on two threads: this one draws (MT twist, temper, the
// branch-free rejection of shuffle_raw) into a ring of swap targets, a second
// one applies the swaps in order, prefetching each target kAhead swaps ahead
// in its own cache.  Same outputs consumed, same targets, the same swaps in
// the same order: the result and the MT state afterwards are shuffle_raw's.
// The two stages hand over chunks of kChunk targets through two counters.
template <typename E>
void shuffle_raw_2t(MT& mt, E* data, int64_t n) {
    if (n < 2) return;
    const int64_t total = n - 1;
    constexpr int64_t kR = 1 << 16, kChunk = 1 << 11;
    const char* ea = std::getenv("MF_SHUFFLE_AHEAD");           // probes
    const int64_t kAhead = ea ? std::max(1, std::min(8192, std::atoi(ea))) : 256;
    std::unique_ptr<uint32_t[]> ring(new uint32_t[kR]);
    alignas(64) std::atomic<int64_t> drawn{0};
    alignas(64) std::atomic<int64_t> done{0};
    std::thread swapper([&]() {
        uint32_t* rg = ring.get();
        int64_t d = 0, avail = 0;
        while (d < total) {
            while (avail <= d) {                       // wait for the next chunk
                avail = drawn.load(std::memory_order_acquire);
                if (avail <= d) std::this_thread::yield();
            }
            const int64_t lim = avail;
            for (; d < lim; ++d) {
                if (d + kAhead < lim) __builtin_prefetch(data + rg[(d + kAhead) & (kR - 1)], 1, 1);
                const int64_t i = total - d;
                const int64_t j = rg[d & (kR - 1)];
                const E t = data[i];
                data[i] = data[j];
                data[j] = t;
                if ((d & (kChunk - 1)) == kChunk - 1) done.store(d + 1, std::memory_order_release);
            }
        }
        done.store(total, std::memory_order_release);
    });
    uint32_t* rg = ring.get();
    int64_t d = 0;
    uint32_t maxv = (uint32_t)total;
    int64_t pub = 0;
    while (d < total) {
        // room for a whole MT block of targets (<= kN) in the ring
        while (d + kN - done.load(std::memory_order_acquire) > kR) std::this_thread::yield();
        if (mt.pos == kN) mt.regen();
        int p = mt.pos;
        while (p < kN) {
            const uint32_t mask = 0xffffffffu >> __builtin_clz(maxv);
            const uint32_t v = mt_temper(mt.key[p++]) & mask;
            const uint32_t acc = v <= maxv ? 1u : 0u;
            rg[d & (kR - 1)] = v;
            d += acc;
            maxv -= acc;
            if (d == total) break;
        }
        mt.pos = p;
        if (d - pub >= kChunk || d == total) {
            drawn.store(d, std::memory_order_release);
            pub = d;
        }
    }
    swapper.join();
}

// shuffle_raw, or with MF_SHUFFLE_THREADS=2 shuffle_raw_2t from this many
// elements.  One thread is the default: on the GPU box's host the two-thread
// form measured SLOWER at 100M (0.44-0.58 vs 0.32-0.38 s; 1.1 vs 1.95 s in
// the build container), profiles/r06/shuffle_time_{1thread,2threads}_r06c3.txt
constexpr int64_t kShuffle2tMin = 1 << 22;

template <typename E>
void shuffle_any(MT& mt, E* data, int64_t n) {
    const char* env = std::getenv("MF_SHUFFLE_THREADS");
    if (n >= kShuffle2tMin && env && env[0] == '2')
        shuffle_raw_2t(mt, data, n);
    else
        shuffle_raw(mt, data, n);
}

// the draws of shuffle_raw alone: the swap targets j_d (d = 0 .. total-1,
// swap d exchanging x[total - d] and x[j_d]) into tgt
void draw_targets(MT& mt, uint32_t* tgt, int64_t total) {
    const bool simd = use_avx512();
    int64_t R = 1;
    while (R < total + 16) R <<= 1;                 // tgt is indexed by d itself
    int64_t d = 0;
    uint32_t maxv = (uint32_t)total;
    while (d < total) {
        int p;
        if (simd) {
            if (mt.pos == kN) mt_regen_512(mt);
            p = mt.pos;
            mt_draws_512(mt, p, d, maxv, total, tgt, R, (int32_t*)nullptr, false);
        } else {
            if (mt.pos == kN) mt.regen();
            p = mt.pos;
            while (p < kN) {
                const uint32_t mask = 0xffffffffu >> __builtin_clz(maxv);
                const uint32_t v = mt_temper(mt.key[p++]) & mask;
                const uint32_t acc = v <= maxv ? 1u : 0u;
                tgt[d] = v;
                d += acc;
                maxv -= acc;
                if (d == total) break;
            }
        }
        mt.pos = p;
    }
}

int load_mt(MT& mt, const uint32_t* mt_key, const int32_t* mt_pos, int64_t n, const char* who) {
    if (n - 1 > (int64_t)0xffffffffLL) {
        set_error("%s: n = %lld exceeds the 32-bit draw range", who, (long long)n);
        return MF_ERR_INVALID;
    }
    if (*mt_pos < 0 || *mt_pos > kN) {
        set_error("%s: MT19937 position %d outside [0, %d]", who, *mt_pos, kN);
        return MF_ERR_INVALID;
    }
    std::memcpy(mt.key, mt_key, sizeof(mt.key));
    mt.pos = *mt_pos;
    return MF_OK;
}

}  // namespace

extern "C" int mf_legacy_shuffle(uint32_t* mt_key, int32_t* mt_pos, int64_t* data, int64_t n) {
    if (!mt_key || !mt_pos || (n > 0 && !data) || n < 0) {
        set_error("mf_legacy_shuffle: null pointer or negative n");
        return MF_ERR_INVALID;
    }
    MT mt;
    if (const int rc = load_mt(mt, mt_key, mt_pos, n, "mf_legacy_shuffle")) return rc;
    shuffle_any(mt, data, n);
    std::memcpy(mt_key, mt.key, sizeof(mt.key));
    *mt_pos = mt.pos;
    return MF_OK;
}

// The shuffle in two parts (the exact schedule's shuffle on the GPU,
// engine.ExactShuffler): the draws here, on one thread -- the RandomState
// advanced exactly as by the whole shuffle -- and the swaps wherever they
// are applied (mf_shuffle_swaps_device; mf_legacy_apply_swaps_i32 for the
// last ones, on the host).
extern "C" int mf_legacy_shuffle_draws(uint32_t* mt_key, int32_t* mt_pos, int64_t n,
                                       uint32_t* targets) {
    if (!mt_key || !mt_pos || n < 0 || (n > 1 && !targets)) {
        set_error("mf_legacy_shuffle_draws: null pointer or negative n");
        return MF_ERR_INVALID;
    }
    MT mt;
    if (const int rc = load_mt(mt, mt_key, mt_pos, n, "mf_legacy_shuffle_draws")) return rc;
    if (n > 1) draw_targets(mt, targets, n - 1);
    std::memcpy(mt_key, mt.key, sizeof(mt.key));
    *mt_pos = mt.pos;
    return MF_OK;
}

// swaps d = d_begin .. n-2 of the shuffle of data[0 .. n) whose draws are
// `targets` (swap d: data[n-1-d] <-> data[targets[d]]), in order
extern "C" int mf_legacy_apply_swaps_i32(const uint32_t* targets, int64_t n, int64_t d_begin,
                                         int32_t* data) {
    const int64_t total = n - 1;
    if (n < 0 || d_begin < 0 || (n > 1 && d_begin < total && (!targets || !data))) {
        set_error("mf_legacy_apply_swaps_i32: bad arguments");
        return MF_ERR_INVALID;
    }
    for (int64_t d = d_begin; d < total; ++d) {
        if (d + 32 < total) __builtin_prefetch(data + targets[d + 32], 1, 1);
        const int64_t i = total - d, j = targets[d];
        if (j > i) {
            set_error("mf_legacy_apply_swaps_i32: target %lld of swap %lld past %lld",
                      (long long)j, (long long)d, (long long)i);
            return MF_ERR_INVALID;
        }
        const int32_t x = data[i];
        data[i] = data[j];
        data[j] = x;
    }
    return MF_OK;
}

// np.random.shuffle of a 1-D array of 4-byte elements (the same draws and
// swaps as mf_legacy_shuffle: the swap targets depend on n only)
extern "C" int mf_legacy_shuffle_i32(uint32_t* mt_key, int32_t* mt_pos, int32_t* data, int64_t n) {
    if (!mt_key || !mt_pos || (n > 0 && !data) || n < 0) {
        set_error("mf_legacy_shuffle_i32: null pointer or negative n");
        return MF_ERR_INVALID;
    }
    MT mt;
    if (const int rc = load_mt(mt, mt_key, mt_pos, n, "mf_legacy_shuffle_i32")) return rc;
    shuffle_any(mt, data, n);
    std::memcpy(mt_key, mt.key, sizeof(mt.key));
    *mt_pos = mt.pos;
    return MF_OK;
}

// np.random.permutation(n): the shuffle of arange(n) run on 4-byte elements
// while n < 2^31 (the same draws and swaps on half the bytes), widened into
// out afterwards.
extern "C" int mf_legacy_permutation(uint32_t* mt_key, int32_t* mt_pos, int64_t* out, int64_t n) {
    if (!mt_key || !mt_pos || (n > 0 && !out) || n < 0) {
        set_error("mf_legacy_permutation: null pointer or negative n");
        return MF_ERR_INVALID;
    }
    MT mt;
    if (const int rc = load_mt(mt, mt_key, mt_pos, n, "mf_legacy_permutation")) return rc;
    const int T = host_threads();
    if (n >= ((int64_t)1 << 31)) {
        parallel_chunks(n, T, [&](int, int64_t a, int64_t b) {
            for (int64_t p = a; p < b; ++p) out[p] = p;
        });
        shuffle_any(mt, out, n);
    } else {
        big_ptr<uint32_t> tmp{nullptr, MapFree{0}};
        try {
            tmp = big_alloc<uint32_t>(n);
            if (!tmp) throw std::bad_alloc();
        } catch (const std::bad_alloc&) {
            set_error("mf_legacy_permutation: cannot allocate %lld rows", (long long)n);
            return MF_ERR_NOMEM;
        }
        parallel_chunks(n, T, [&](int, int64_t a, int64_t b) {
            for (int64_t p = a; p < b; ++p) tmp[p] = (uint32_t)p;
        });
        shuffle_any(mt, tmp.get(), n);
        parallel_chunks(n, T, [&](int, int64_t a, int64_t b) {
            for (int64_t p = a; p < b; ++p) out[p] = tmp[p];
        });
    }
    std::memcpy(mt_key, mt.key, sizeof(mt.key));
    *mt_pos = mt.pos;
    return MF_OK;
}

extern "C" int mf_pairs_duplicated(const int64_t* a, const int64_t* b, int64_t n,
                                   int32_t* has_dup) {
    if (!has_dup || n < 0 || (n > 0 && (!a || !b))) {
        set_error("mf_pairs_duplicated: bad arguments");
        return MF_ERR_INVALID;
    }
    *has_dup = 0;
    if (n < 2) return MF_OK;
    const int T = host_threads(), R = bucket_bits(n);
    auto bucket = [&](int64_t p) {
        return (int)(mix64((uint64_t)a[p] * 0x9E3779B97F4A7C15ull ^ (uint64_t)b[p]) >> (64 - R));
    };
    std::vector<int64_t> start;
    big_ptr<std::pair<int64_t, int64_t>> pr{nullptr, MapFree{0}};
    try {
        pr = big_alloc<std::pair<int64_t, int64_t>>(n);
        if (!pr) throw std::bad_alloc();
        partition_rows(n, 1 << R, T, bucket, start,
                       [&](int64_t d, int64_t p) { pr[(size_t)d] = {a[p], b[p]}; });
    } catch (const std::bad_alloc&) {
        set_error("mf_pairs_duplicated: cannot allocate %lld rows", (long long)n);
        return MF_ERR_NOMEM;
    }
    std::atomic<int> found{0};
    for_buckets(1 << R, T, [&](int k) {
        const auto* v = pr.get() + start[k];
        const int64_t m = start[k + 1] - start[k];
        size_t cap = 16;
        while (cap < (size_t)m * 2) cap <<= 1;
        struct Ent {
            int64_t a, b;
            bool used;
        };
        std::vector<Ent> table(cap, Ent{0, 0, false});
        for (int64_t q = 0; q < m; ++q) {
            size_t h = (size_t)(mix64((uint64_t)v[q].first ^ mix64((uint64_t)v[q].second)) &
                                (cap - 1));
            for (;; h = (h + 1) & (cap - 1)) {
                Ent& e = table[h];
                if (!e.used) {
                    e = Ent{v[q].first, v[q].second, true};
                    break;
                }
                if (e.a == v[q].first && e.b == v[q].second) {
                    found.store(1);
                    return;
                }
            }
        }
    }, &found);
    *has_dup = found.load();
    return MF_OK;
}

extern "C" int mf_factorize(const int64_t* vals, int64_t n, int64_t* codes, int64_t* uniques,
                            int64_t* n_uniques) {
    if (n < 0 || !n_uniques || (n > 0 && (!vals || !codes || !uniques))) {
        set_error("mf_factorize: bad arguments");
        return MF_ERR_INVALID;
    }
    *n_uniques = 0;
    if (n == 0) return MF_OK;
    const int T = host_threads(), R = bucket_bits(n), NB = 1 << R;
    auto bucket = [&](int64_t p) { return (int)(mix64((uint64_t)vals[p]) >> (64 - R)); };
    const int64_t nw = (n + 63) >> 6;
    // uninitialised (first touched by the threads that fill them)
    big_ptr<int64_t> slot{nullptr, MapFree{0}}, sval{nullptr, MapFree{0}}, lid{nullptr, MapFree{0}};
    std::vector<int64_t> start, wpre;
    std::vector<std::vector<int64_t>> first((size_t)NB);
    std::unique_ptr<std::atomic<uint64_t>[]> bits;
    try {
        slot = big_alloc<int64_t>(n);
        sval = big_alloc<int64_t>(n);
        lid = big_alloc<int64_t>(n);
        if (!slot || !sval || !lid) throw std::bad_alloc();
        partition_rows(n, 1 << R, T, bucket, start, [&](int64_t d, int64_t p) {
            slot[d] = p;
            sval[d] = vals[p];
        });
        wpre.resize((size_t)nw + 1);
        bits.reset(new std::atomic<uint64_t>[(size_t)nw]);
    } catch (const std::bad_alloc&) {
        set_error("mf_factorize: cannot allocate %lld rows", (long long)n);
        return MF_ERR_NOMEM;
    }
    parallel_chunks(nw, T, [&](int, int64_t lo, int64_t hi) {
        for (int64_t w = lo; w < hi; ++w) bits[w].store(0, std::memory_order_relaxed);
    });
    // 1. per bucket (rows ascending): local ids in first-appearance order and
    //    the row of each one's first appearance, marked in `bits`
    for_buckets(NB, T, [&](int k) {
        const int64_t m = start[k + 1] - start[k];
        const int64_t* s = slot.get() + start[k];
        const int64_t* sv = sval.get() + start[k];
        int64_t* l = lid.get() + start[k];
        size_t cap = 16;
        while (cap < (size_t)m * 2) cap <<= 1;
        struct Ent {
            int64_t val, id;  // id -1 = empty
        };
        std::vector<Ent> table(cap, Ent{0, -1});
        std::vector<int64_t>& f = first[(size_t)k];
        for (int64_t q = 0; q < m; ++q) {
            const int64_t v = sv[q];
            size_t h = (size_t)(mix64((uint64_t)v) & (cap - 1));
            for (;;) {
                Ent& e = table[h];
                if (e.id < 0) {
                    e.val = v;
                    e.id = l[q] = (int64_t)f.size();
                    f.push_back(s[q]);
                    bits[s[q] >> 6].fetch_or(1ull << (s[q] & 63), std::memory_order_relaxed);
                    break;
                }
                if (e.val == v) {
                    l[q] = e.id;
                    break;
                }
                h = (h + 1) & (cap - 1);
            }
        }
    });
    // 2. code of a value = number of first appearances before its own
    wpre[0] = 0;
    for (int64_t w = 0; w < nw; ++w)
        wpre[w + 1] = wpre[w] + __builtin_popcountll(bits[w].load(std::memory_order_relaxed));
    const int64_t U = wpre[nw];
    auto code_of_row = [&](int64_t row) {
        const uint64_t word = bits[row >> 6].load(std::memory_order_relaxed);
        return wpre[row >> 6] + __builtin_popcountll(word & ((1ull << (row & 63)) - 1));
    };
    // 3. scatter codes, write the uniques in code order
    for_buckets(NB, T, [&](int k) {
        std::vector<int64_t>& f = first[(size_t)k];
        for (int64_t& row : f) {
            const int64_t c = code_of_row(row);
            uniques[c] = vals[row];
            row = c;  // local id -> code
        }
        const int64_t m = start[k + 1] - start[k];
        const int64_t* s = slot.get() + start[k];
        const int64_t* l = lid.get() + start[k];
        for (int64_t q = 0; q < m; ++q) codes[s[q]] = f[(size_t)l[q]];
    });
    *n_uniques = U;
    return MF_OK;
}

extern "C" int mf_id_range(const int64_t* vals, int64_t n, int64_t* lo, int64_t* hi) {
    if (n < 0 || !lo || !hi || (n > 0 && !vals)) {
        set_error("mf_id_range: bad arguments");
        return MF_ERR_INVALID;
    }
    const int T = host_threads();
    std::vector<int64_t> mn((size_t)T, INT64_MAX), mx((size_t)T, INT64_MIN);
    parallel_chunks(n, T, [&](int t, int64_t a, int64_t b) {
        int64_t l = INT64_MAX, h = INT64_MIN;
        for (int64_t p = a; p < b; ++p) {
            l = std::min(l, vals[p]);
            h = std::max(h, vals[p]);
        }
        mn[(size_t)t] = l;
        mx[(size_t)t] = h;
    });
    *lo = *std::min_element(mn.begin(), mn.end());
    *hi = *std::max_element(mx.begin(), mx.end());
    return MF_OK;
}

// pd.factorize(vals[perm], sort=False) from dense ids of the UNSHUFFLED
// column (dense[p] - base in [0, n_dense): the id itself when the ids span a
// small range, else mf_factorize's codes of the unshuffled column -- either
// is ready before the permutation is drawn).  The code of a dense id is the
// rank of its first position t in the shuffled order: per id the minimum t
// (an atomic min over threads that each walk a chunk of t), a bitmap of
// those first positions, and its prefix popcounts.
extern "C" int mf_first_appearance(const int64_t* dense, int64_t base, int64_t n_dense,
                                   const int64_t* perm, int64_t n, int64_t* codes,
                                   int64_t* order, int64_t* n_uniques) {
    if (n < 0 || n_dense < 0 || n_dense > (int64_t)UINT32_MAX || !n_uniques ||
        (n > 0 && (!dense || !perm || !codes || !order || n_dense == 0))) {
        set_error("mf_first_appearance: bad arguments");
        return MF_ERR_INVALID;
    }
    *n_uniques = 0;
    if (n == 0) return MF_OK;
    const int T = host_threads();
    const int64_t nw = (n + 63) >> 6;
    big_ptr<int64_t> first{nullptr, MapFree{0}};
    big_ptr<uint32_t> g{nullptr, MapFree{0}};
    big_ptr<uint64_t> bits{nullptr, MapFree{0}};
    try {
        first = big_alloc<int64_t>(n_dense);
        g = big_alloc<uint32_t>(n);
        bits = big_alloc<uint64_t>(nw);
        if (!first || !g || !bits) throw std::bad_alloc();
    } catch (const std::bad_alloc&) {
        set_error("mf_first_appearance: cannot allocate %lld rows", (long long)n);
        return MF_ERR_NOMEM;
    }
    parallel_chunks(n_dense, T, [&](int, int64_t a, int64_t b) {
        for (int64_t d = a; d < b; ++d) first[d] = n;
    });
    parallel_chunks(nw, T, [&](int, int64_t a, int64_t b) {
        for (int64_t w = a; w < b; ++w) bits[w] = 0;
    });
    std::atomic<int> bad{0};
    // 1. dense id of every shuffled row; its first shuffled position
    parallel_chunks(n, T, [&](int, int64_t a, int64_t b) {
        constexpr int kAhead = 16;
        for (int64_t t = a; t < b; ++t) {
            if (t + kAhead < b) {
                const int64_t q = perm[t + kAhead];
                if (q >= 0 && q < n) __builtin_prefetch(dense + q, 0, 0);
            }
            const int64_t p = perm[t];
            if (p < 0 || p >= n) {
                bad.store(1);
                return;
            }
            const int64_t d = dense[p] - base;
            if (d < 0 || d >= n_dense) {
                bad.store(1);
                return;
            }
            g[t] = (uint32_t)d;
            int64_t cur = __atomic_load_n(&first[d], __ATOMIC_RELAXED);
            while (t < cur && !__atomic_compare_exchange_n(&first[d], &cur, t, true,
                                                           __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
            }
        }
    });
    if (bad.load()) {
        set_error("mf_first_appearance: permutation or dense id out of range");
        return MF_ERR_INVALID;
    }
    // 2. bitmap of first positions, prefix popcounts
    parallel_chunks(n_dense, T, [&](int, int64_t a, int64_t b) {
        for (int64_t d = a; d < b; ++d) {
            const int64_t f = first[d];
            if (f < n) __atomic_fetch_or(&bits[f >> 6], 1ull << (f & 63), __ATOMIC_RELAXED);
        }
    });
    std::vector<int64_t> wpre((size_t)nw + 1);
    wpre[0] = 0;
    for (int64_t w = 0; w < nw; ++w) wpre[w + 1] = wpre[w] + __builtin_popcountll(bits[w]);
    // 3. code of every dense id (in place of its first position), ids in code order
    parallel_chunks(n_dense, T, [&](int, int64_t a, int64_t b) {
        for (int64_t d = a; d < b; ++d) {
            const int64_t f = first[d];
            if (f >= n) continue;
            const int64_t c = wpre[f >> 6] + __builtin_popcountll(bits[f >> 6] & ((1ull << (f & 63)) - 1));
            first[d] = c;
            order[c] = d;
        }
    });
    // 4. codes of the shuffled rows
    parallel_chunks(n, T, [&](int, int64_t a, int64_t b) {
        for (int64_t t = a; t < b; ++t) codes[t] = first[g[t]];
    });
    *n_uniques = wpre[nw];
    return MF_OK;
}

namespace {
// dst[p] = src[idx[p]] on the host threads, each source element prefetched a
// few rows ahead; false when an index falls outside [0, n_src)
template <typename E, typename I>
bool gather_rows(const E* s, int64_t n_src, const I* idx, int64_t n, E* d) {
    std::atomic<int> bad{0};
    parallel_chunks(n, host_threads(), [&](int, int64_t lo, int64_t hi) {
        constexpr int kAhead = 16;
        for (int64_t p = lo; p < hi; ++p) {
            if (p + kAhead < hi) {
                const int64_t q = idx[p + kAhead];
                if (q >= 0 && q < n_src) __builtin_prefetch(s + q, 0, 0);
            }
            const int64_t q = idx[p];
            if (q < 0 || q >= n_src) {
                bad.store(1);
                return;
            }
            d[p] = s[q];
        }
    });
    return !bad.load();
}

template <typename I>
int gather_any(const char* who, const void* src, int64_t n_src, int32_t elem_bytes, const I* idx,
               int64_t n, void* dst) {
    if (n < 0 || n_src < 0 || (elem_bytes != 4 && elem_bytes != 8) ||
        (n > 0 && (!src || !idx || !dst))) {
        set_error("%s: bad arguments", who);
        return MF_ERR_INVALID;
    }
    const bool ok = elem_bytes == 4
                        ? gather_rows(static_cast<const uint32_t*>(src), n_src, idx, n,
                                      static_cast<uint32_t*>(dst))
                        : gather_rows(static_cast<const uint64_t*>(src), n_src, idx, n,
                                      static_cast<uint64_t*>(dst));
    if (!ok) {
        set_error("%s: index outside [0, %lld)", who, (long long)n_src);
        return MF_ERR_INVALID;
    }
    return MF_OK;
}
}  // namespace

extern "C" int mf_gather(const void* src, int64_t n_src, int32_t elem_bytes, const int64_t* idx,
                         int64_t n, void* dst) {
    return gather_any("mf_gather", src, n_src, elem_bytes, idx, n, dst);
}

// the same with 32-bit indices (relabelling 10^8 int32 ids through an id
// permutation: the relabelled plans' host ids)
extern "C" int mf_gather_i32(const void* src, int64_t n_src, int32_t elem_bytes,
                             const int32_t* idx, int64_t n, void* dst) {
    return gather_any("mf_gather_i32", src, n_src, elem_bytes, idx, n, dst);
}

// fit()'s id columns (int64 codes) narrowed to the engine's int32 ids, each
// checked against [0, bound), and its ratings narrowed to FP32 -- on the host
// threads, which also take the destination's first-touch page faults (the
// NumPy conversions of 10^8 rows ran on one thread on fit()'s critical path)
extern "C" int mf_ids_to_i32(const int64_t* src, int64_t n, int64_t bound, int32_t* dst) {
    if (n < 0 || bound < 0 || bound > ((int64_t)1 << 31) || (n > 0 && (!src || !dst))) {
        set_error("mf_ids_to_i32: bad arguments");
        return MF_ERR_INVALID;
    }
    std::atomic<int> bad{0};
    parallel_chunks(n, host_threads(), [&](int, int64_t lo, int64_t hi) {
        int any = 0;
        for (int64_t p = lo; p < hi; ++p) {
            const int64_t v = src[p];
            any |= (v < 0) | (v >= bound);
            dst[p] = (int32_t)v;
        }
        if (any) bad.store(1);
    });
    if (bad.load()) {
        set_error("mf_ids_to_i32: an id outside [0, %lld)", (long long)bound);
        return MF_ERR_INVALID;
    }
    return MF_OK;
}

extern "C" int mf_f64_to_f32(const double* src, int64_t n, float* dst) {
    if (n < 0 || (n > 0 && (!src || !dst))) {
        set_error("mf_f64_to_f32: bad arguments");
        return MF_ERR_INVALID;
    }
    parallel_chunks(n, host_threads(), [&](int, int64_t lo, int64_t hi) {
        for (int64_t p = lo; p < hi; ++p) dst[p] = (float)src[p];
    });
    return MF_OK;
}

// Fingerprint of a host buffer (KernelMF._predictor: are the device copies of
// P / Q / b_u / b_i still those of the NumPy attributes, in-place edits
// included?).  Chunks of 64-bit words are folded with the splitmix64
// multiply-rotate lanes on the host threads (splitmix64 finaliser per
// chunk); the chunk hashes are combined in order.  Not
// cryptographic: equal buffers give equal values, a changed word changes the
// value with overwhelming probability.
extern "C" uint64_t mf_fingerprint(const void* data, int64_t n_bytes) {
    if (!data || n_bytes <= 0) return 0x9E3779B97F4A7C15ull ^ (uint64_t)n_bytes;
    const unsigned char* b = static_cast<const unsigned char*>(data);
    const int64_t nw = n_bytes / 8;
    const int T = host_threads();
    const int C = std::max(1, std::min<int>(4 * T, (int)(nw >> 16) + 1));   // chunks
    std::vector<uint64_t> part((size_t)C, 0);
    for_buckets(C, T, [&](int c) {
        const int64_t lo = nw * c / C, hi = nw * (c + 1) / C;
        // four independent multiply-rotate lanes (memory-bound, not latency-bound)
        constexpr uint64_t K = 0x9FB21C651E98DF25ull;
        uint64_t h[4] = {0x243F6A8885A308D3ull + (uint64_t)c, 0x13198A2E03707344ull,
                         0xA4093822299F31D0ull, 0x082EFA98EC4E6C89ull};
        int64_t w = lo;
        for (; w + 3 < hi; w += 4) {
            uint64_t x[4];
            std::memcpy(x, b + 8 * w, 32);
            for (int j = 0; j < 4; ++j) {
                const uint64_t y = h[j] ^ x[j];
                h[j] = ((y << 29) | (y >> 35)) * K;
            }
        }
        for (; w < hi; ++w) {
            uint64_t x;
            std::memcpy(&x, b + 8 * w, 8);
            h[0] = mix64(h[0] ^ x);
        }
        const uint64_t h0 = mix64(h[0] ^ mix64(h[1])), h1 = mix64(h[2] ^ mix64(h[3]));
        part[(size_t)c] = mix64(h0 ^ (h1 * 0x9E3779B97F4A7C15ull));
    });
    uint64_t h = (uint64_t)n_bytes;
    for (int c = 0; c < C; ++c) h = mix64(h ^ part[(size_t)c]) + (uint64_t)c;
    for (int64_t t = nw * 8; t < n_bytes; ++t) h = mix64(h ^ b[t]);
    return h;
}
