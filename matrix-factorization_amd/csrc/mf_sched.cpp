// mf_sched.cpp -- host-side batch schedulers and error plumbing of libmf_hip.
//
// The reference's epoch is one sequential sweep over the ratings in a
// shuffled order (kernel_matrix_factorization.py:371-425).  Every update
// reads and writes one user row and one item row, so two ratings conflict
// exactly when they share a user or an item.  The GPU applies ratings in
// conflict-free BATCHES; these schedulers build them:
//
//   mf_sched_levels  exact order: level(t) = 1 + max(level of the previous
//                    rating of the same user / item in visit order).  Levels
//                    applied in order reproduce the sequential sweep exactly.
//   mf_sched_color   throughput: greedy edge colouring, every colour is a
//                    matching of the rating graph, so the colours may be
//                    applied in any order (a different valid sequential order
//                    per epoch, chosen by the caller).
#include <algorithm>
#include <climits>
#include <exception>
#include <thread>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <new>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "../../include/mf_hip.h"
#include "mf_host.hpp"

namespace mf {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

int hip_fail(hipError_t e, const char* what) {
    set_error("%s: %s (%d)", what, hipGetErrorString(e), (int)e);
    return MF_ERR_HIP;
}

}  // namespace mf

using mf::set_error;

extern "C" const char* mf_last_error(void) { return mf::g_err; }
extern "C" int mf_abi_version(void) { return MF_ABI_VERSION; }

static int check_ids(const int32_t* u, const int32_t* it, int64_t n, int32_t nu, int32_t ni) {
    for (int64_t j = 0; j < n; ++j) {
        if (u[j] < 0 || u[j] >= nu || it[j] < 0 || it[j] >= ni) {
            set_error("rating %lld has ids (%d, %d) outside [0,%d) x [0,%d)", (long long)j, u[j],
                      it[j], nu, ni);
            return MF_ERR_INVALID;
        }
    }
    return MF_OK;
}

extern "C" int mf_sched_levels(const int32_t* user_ids, const int32_t* item_ids, int64_t n,
                               const int64_t* order, int32_t n_users, int32_t n_items,
                               int32_t use_user, int32_t use_item, int32_t* sched_out,
                               int64_t* level_offsets, int64_t offsets_cap,
                               int32_t* n_levels_out) {
    if (n < 0 || n_users < 0 || n_items < 0 || !n_levels_out || (n > 0 && !sched_out) ||
        !level_offsets || offsets_cap < 1) {
        set_error("mf_sched_levels: bad arguments");
        return MF_ERR_INVALID;
    }
    if (int rc = check_ids(user_ids, item_ids, n, n_users, n_items)) return rc;
    try {
        std::vector<int32_t> lu(use_user ? (size_t)n_users : 0, 0);
        std::vector<int32_t> li(use_item ? (size_t)n_items : 0, 0);
        std::vector<int32_t> lvl((size_t)n);
        int32_t maxl = n > 0 ? 1 : 0;
        for (int64_t t = 0; t < n; ++t) {
            const int64_t j = order ? order[t] : t;
            if (j < 0 || j >= n) {
                set_error("order[%lld] = %lld out of range", (long long)t, (long long)j);
                return MF_ERR_INVALID;
            }
            int32_t L = 0;
            if (use_user) L = lu[user_ids[j]];
            if (use_item) L = std::max(L, li[item_ids[j]]);
            L += 1;
            if (use_user) lu[user_ids[j]] = L;
            if (use_item) li[item_ids[j]] = L;
            lvl[t] = L;
            maxl = std::max(maxl, L);
        }
        *n_levels_out = maxl;
        if ((int64_t)maxl + 1 > offsets_cap) {
            set_error("level_offsets capacity %lld < %d", (long long)offsets_cap, maxl + 1);
            return MF_ERR_CAPACITY;
        }
        std::fill(level_offsets, level_offsets + maxl + 1, 0);
        for (int64_t t = 0; t < n; ++t) level_offsets[lvl[t]] += 1;   // count at L
        for (int32_t L = 1; L <= maxl; ++L) level_offsets[L] += level_offsets[L - 1];
        // level L (1-based) occupies [offsets[L-1], offsets[L]); fill stably
        std::vector<int64_t> cur(level_offsets, level_offsets + maxl);
        for (int64_t t = 0; t < n; ++t) {
            const int64_t j = order ? order[t] : t;
            sched_out[cur[lvl[t] - 1]++] = (int32_t)j;
        }
    } catch (const std::bad_alloc&) {
        set_error("mf_sched_levels: out of host memory");
        return MF_ERR_NOMEM;
    }
    return MF_OK;
}

// Exact order at scale: the same conflict-free levels property, built on T
// threads.  The visit order is cut into T contiguous chunks; chunk c's levels
// are computed as if it were alone (its own last-level tables, level 1 = its
// first ratings) and placed after every level of chunks 0..c-1.  A rating's
// level is then above every earlier rating of its user and item (same chunk:
// the greedy rule; earlier chunk: a lower level range), and no two ratings of
// one level share a user or an item, so applying the levels in order is the
// sequential sweep of `order` -- bit for bit the result of mf_sched_levels'
// greedy levels, with sum over chunks of the chunk depths instead of the
// global depth (C3: ~1.4x the launches).  Chunk c's ratings fill exactly
// positions [lo_c, hi_c) of sched_out (its levels follow all earlier
// chunks'), so the stable fill by level is per chunk too.  `order` holds
// 32-bit rating indices (n < 2^31).
extern "C" int mf_sched_levels_chunked(const int32_t* user_ids, const int32_t* item_ids,
                                       int64_t n, const int32_t* order, int32_t n_users,
                                       int32_t n_items, int32_t use_user, int32_t use_item,
                                       int32_t n_chunks, int32_t* sched_out,
                                       int64_t* level_offsets, int64_t offsets_cap,
                                       int32_t* n_levels_out) {
    if (n < 0 || n >= ((int64_t)1 << 31) || n_users < 0 || n_items < 0 || !n_levels_out ||
        (n > 0 && (!sched_out || !order || !user_ids || !item_ids)) || !level_offsets ||
        offsets_cap < 1) {
        set_error("mf_sched_levels_chunked: bad arguments");
        return MF_ERR_INVALID;
    }
    int T = n_chunks > 0 ? n_chunks : (n >= ((int64_t)1 << 20) ? mf::host_threads() : 1);
    T = (int)std::max<int64_t>(1, std::min<int64_t>(T, std::max<int64_t>(n, 1)));
    try {
        std::vector<int64_t> lo(T + 1);
        for (int c = 0; c <= T; ++c) lo[c] = n * c / T;
        auto lvl = mf::big_alloc<int32_t>(n);
        if (!lvl) throw std::bad_alloc();
        std::vector<int32_t> depth(T, 0);
        std::vector<std::vector<int64_t>> cnt(T);
        std::vector<int64_t> bad(T, -1);                 // first bad order entry per chunk
        std::vector<int64_t> bad_id(T, -1);              // first rating with bad ids
        mf::ThreadErr err;
        auto pass1 = [&](int c) {
            err.guard([&]() {
                std::vector<int32_t> lu(use_user ? (size_t)n_users : 0, 0);
                std::vector<int32_t> li(use_item ? (size_t)n_items : 0, 0);
                int32_t maxl = 0;
                constexpr int64_t kAhead = 16;
                const int64_t a = lo[c], b = lo[c + 1];
                for (int64_t t = a; t < b; ++t) {
                    if (t + kAhead < b) {
                        const int64_t jp = order[t + kAhead];
                        if ((uint64_t)jp < (uint64_t)n) {
                            __builtin_prefetch(user_ids + jp, 0, 0);
                            __builtin_prefetch(item_ids + jp, 0, 0);
                        }
                    }
                    const int64_t j = order[t];
                    if ((uint64_t)j >= (uint64_t)n) {
                        bad[c] = t;
                        return;
                    }
                    const int32_t uu = user_ids[j], ii = item_ids[j];
                    if ((uint32_t)uu >= (uint32_t)n_users || (uint32_t)ii >= (uint32_t)n_items) {
                        bad_id[c] = j;
                        return;
                    }
                    int32_t L = 0;
                    if (use_user) L = lu[uu];
                    if (use_item) L = std::max(L, li[ii]);
                    L += 1;
                    if (use_user) lu[uu] = L;
                    if (use_item) li[ii] = L;
                    lvl[t] = L;
                    maxl = std::max(maxl, L);
                }
                depth[c] = maxl;
                std::vector<int64_t>& h = cnt[c];
                h.assign((size_t)maxl + 1, 0);
                for (int64_t t = a; t < b; ++t) ++h[lvl[t]];
            });
        };
        std::vector<std::thread> th;
        for (int c = 1; c < T; ++c) th.emplace_back(pass1, c);
        pass1(0);
        for (auto& x : th) x.join();
        th.clear();
        err.rethrow();
        for (int c = 0; c < T; ++c) {
            if (bad[c] >= 0) {
                set_error("order[%lld] = %lld out of range", (long long)bad[c],
                          (long long)order[bad[c]]);
                return MF_ERR_INVALID;
            }
            if (bad_id[c] >= 0) {
                const int64_t j = bad_id[c];
                set_error("rating %lld has ids (%d, %d) outside [0,%d) x [0,%d)", (long long)j,
                          user_ids[j], item_ids[j], n_users, n_items);
                return MF_ERR_INVALID;
            }
        }
        // global level offsets: chunk c's level L (1-based) is global level
        // base_c + L; its ratings sit at lo_c + (chunk-c ratings of lower level)
        std::vector<int64_t> base(T + 1, 0);
        for (int c = 0; c < T; ++c) base[c + 1] = base[c] + depth[c];
        const int64_t nl = base[T];
        if (nl > INT32_MAX) {
            set_error("mf_sched_levels_chunked: %lld levels", (long long)nl);
            return MF_ERR_INVALID;
        }
        *n_levels_out = (int32_t)nl;
        if (nl + 1 > offsets_cap) {
            set_error("level_offsets capacity %lld < %lld", (long long)offsets_cap,
                      (long long)(nl + 1));
            return MF_ERR_CAPACITY;
        }
        level_offsets[0] = 0;
        for (int c = 0; c < T; ++c) {
            int64_t acc = lo[c];
            for (int32_t L = 1; L <= depth[c]; ++L) {
                acc += cnt[c][L];
                level_offsets[base[c] + L] = acc;
            }
        }
        auto pass2 = [&](int c) {
            err.guard([&]() {
                const int32_t D = depth[c];
                std::vector<int64_t> cur((size_t)D + 1);
                int64_t acc = lo[c];
                for (int32_t L = 1; L <= D; ++L) {
                    cur[L] = acc;
                    acc += cnt[c][L];
                }
                for (int64_t t = lo[c]; t < lo[c + 1]; ++t) sched_out[cur[lvl[t]]++] = order[t];
            });
        };
        for (int c = 1; c < T; ++c) th.emplace_back(pass2, c);
        pass2(0);
        for (auto& x : th) x.join();
        err.rethrow();
    } catch (const std::bad_alloc&) {
        set_error("mf_sched_levels_chunked: out of host memory");
        return MF_ERR_NOMEM;
    } catch (const std::exception& e) {
        set_error("mf_sched_levels_chunked: %s", e.what());
        return MF_ERR_INVALID;
    }
    return MF_OK;
}

extern "C" int mf_sched_color(const int32_t* user_ids, const int32_t* item_ids, int64_t n,
                              int32_t n_users, int32_t n_items, int32_t* sched_out,
                              int64_t* color_offsets, int64_t offsets_cap,
                              int32_t* n_colors_out) {
    if (n < 0 || n_users < 0 || n_items < 0 || !n_colors_out || (n > 0 && !sched_out) ||
        !color_offsets || offsets_cap < 1) {
        set_error("mf_sched_color: bad arguments");
        return MF_ERR_INVALID;
    }
    if (int rc = check_ids(user_ids, item_ids, n, n_users, n_items)) return rc;
    *n_colors_out = 0;
    color_offsets[0] = 0;
    if (n == 0) return MF_OK;
    try {
        // CSR by item, ratings of an item in input order
        std::vector<int64_t> iptr((size_t)n_items + 1, 0);
        std::vector<int32_t> udeg((size_t)n_users, 0);
        for (int64_t j = 0; j < n; ++j) {
            iptr[item_ids[j] + 1] += 1;
            udeg[user_ids[j]] += 1;
        }
        int64_t dmax_i = 0;
        for (int32_t i = 0; i < n_items; ++i) {
            dmax_i = std::max(dmax_i, iptr[i + 1]);
            iptr[i + 1] += iptr[i];
        }
        const int64_t dmax_u = *std::max_element(udeg.begin(), udeg.end());
        const int64_t bound = dmax_u + dmax_i - 1;            // greedy never exceeds
        if (bound + 1 > offsets_cap) {
            set_error("color_offsets capacity %lld < %lld", (long long)offsets_cap,
                      (long long)(bound + 1));
            return MF_ERR_CAPACITY;
        }
        std::vector<int32_t> ilist((size_t)n);
        {
            std::vector<int64_t> cur(iptr.begin(), iptr.end() - 1);
            for (int64_t j = 0; j < n; ++j) ilist[cur[item_ids[j]]++] = (int32_t)j;
        }
        const int64_t W = (bound + 63) / 64;
        std::vector<uint64_t> ubits((size_t)n_users * (size_t)W, 0);
        std::vector<uint64_t> ibits((size_t)W, 0);
        std::vector<int32_t> color((size_t)n);
        std::vector<int64_t> ccount((size_t)bound + 1, 0);
        int32_t ncol = 0;
        constexpr int kAhead = 16;
        for (int32_t it = 0; it < n_items; ++it) {
            const int64_t b = iptr[it], e = iptr[it + 1];
            if (b == e) continue;
            std::fill(ibits.begin(), ibits.end(), 0);
            for (int64_t t = b; t < e; ++t) {
                if (t + kAhead < e)
                    __builtin_prefetch(&ubits[(size_t)user_ids[ilist[t + kAhead]] * W]);
                const int32_t j = ilist[t];
                uint64_t* ub = &ubits[(size_t)user_ids[j] * W];
                int64_t c = -1;
                for (int64_t w = 0; w < W; ++w) {
                    const uint64_t freeb = ~(ub[w] | ibits[w]);
                    if (freeb) {
                        c = w * 64 + __builtin_ctzll(freeb);
                        break;
                    }
                }
                if (c < 0 || c >= bound) {  // cannot happen: |used| <= bound - 1
                    set_error("internal: edge colouring exceeded bound %lld", (long long)bound);
                    return MF_ERR_INVALID;
                }
                ub[c >> 6] |= 1ull << (c & 63);
                ibits[c >> 6] |= 1ull << (c & 63);
                color[j] = (int32_t)c;
                ccount[c] += 1;
                ncol = std::max(ncol, (int32_t)c + 1);
            }
        }
        // stable counting sort by colour of the item-major sequence:
        // inside a colour, ratings ascend by item id.
        color_offsets[0] = 0;
        for (int32_t c = 0; c < ncol; ++c) color_offsets[c + 1] = color_offsets[c] + ccount[c];
        std::vector<int64_t> cur(color_offsets, color_offsets + ncol);
        for (int64_t t = 0; t < n; ++t) {
            const int32_t j = ilist[t];
            sched_out[cur[color[j]]++] = j;
        }
        *n_colors_out = ncol;
    } catch (const std::bad_alloc&) {
        set_error("mf_sched_color: out of host memory");
        return MF_ERR_NOMEM;
    }
    return MF_OK;
}

// Rows bucketed by key (a stable partition), then users ascending inside
// each bucket (a stable counting sort): the evaluation orders of the SSE pass.
template <typename Key>
static void sched_by_key_then_user(const int32_t* user_ids, int64_t n, int32_t n_users,
                                   int32_t n_keys, Key key, int32_t* sched_out,
                                   int64_t* offsets) {
    const int T = mf::host_threads();
    std::vector<int64_t> start;
    mf::partition_rows(
        n, n_keys, T, key, start, [&](int64_t d, int64_t p) { sched_out[d] = (int32_t)p; });
    for (int32_t x = 0; x <= n_keys; ++x) offsets[x] = start[x];
    mf::for_buckets(n_keys, T, [&](int s) {
        int32_t* q = sched_out + start[s];
        const int64_t m = start[s + 1] - start[s];
        std::vector<int64_t> cnt((size_t)n_users + 1, 0);
        for (int64_t j = 0; j < m; ++j) cnt[user_ids[q[j]] + 1] += 1;
        for (int32_t x = 0; x < n_users; ++x) cnt[x + 1] += cnt[x];
        std::vector<int32_t> tmp((size_t)m);
        for (int64_t j = 0; j < m; ++j) tmp[cnt[user_ids[q[j]]]++] = q[j];
        std::copy(tmp.begin(), tmp.end(), q);
    });
}

extern "C" int mf_sched_slices(const int32_t* user_ids, const int32_t* item_ids, int64_t n,
                               int32_t n_users, int32_t n_items, int32_t n_slices,
                               int32_t* sched_out, int64_t* slice_offsets) {
    if (n < 0 || n_users < 0 || n_items < 0 || n_slices < 1 || n_slices > 64 ||
        (n > 0 && !sched_out) || !slice_offsets) {
        set_error("mf_sched_slices: bad arguments");
        return MF_ERR_INVALID;
    }
    if (int rc = check_ids(user_ids, item_ids, n, n_users, n_items)) return rc;
    try {
        // stable sort by key = slice(item) * n_users + user: a stable
        // partition by slice, then a counting sort by user inside each slice
        auto slice_of = [&](int32_t it) {
            return (int)((int64_t)it * n_slices / (n_items > 0 ? n_items : 1));
        };
        sched_by_key_then_user(user_ids, n, n_users, n_slices,
                               [&](int64_t p) { return slice_of(item_ids[p]); }, sched_out,
                               slice_offsets);
    } catch (const std::bad_alloc&) {
        set_error("mf_sched_slices: out of host memory");
        return MF_ERR_NOMEM;
    }
    return MF_OK;
}

extern "C" int mf_sched_tiles(const int32_t* user_ids, const int32_t* item_ids, int64_t n,
                              int32_t n_users, int32_t n_items, int32_t n_chunks,
                              int32_t n_slices, int32_t* sched_out, int64_t* tile_offsets) {
    if (n < 0 || n_users < 0 || n_items < 0 || n_chunks < 1 || n_slices < 1 ||
        (int64_t)n_chunks * n_slices > 128 || (n > 0 && !sched_out) || !tile_offsets) {
        set_error("mf_sched_tiles: bad arguments (n_chunks * n_slices must be in [1, 128])");
        return MF_ERR_INVALID;
    }
    if (int rc = check_ids(user_ids, item_ids, n, n_users, n_items)) return rc;
    try {
        // user chunks: contiguous id ranges of about equal rating counts
        std::vector<int64_t> deg((size_t)n_users + 1, 0);
        for (int64_t p = 0; p < n; ++p) deg[(size_t)user_ids[p] + 1] += 1;
        for (int32_t x = 0; x < n_users; ++x) deg[x + 1] += deg[x];
        std::vector<uint8_t> chunk_of((size_t)n_users, 0);
        int32_t c = 0;
        for (int32_t x = 0; x < n_users; ++x) {
            // user x goes to the chunk its first rating's rank falls in
            while (c + 1 < n_chunks && deg[x] * n_chunks >= (int64_t)(c + 1) * n) ++c;
            chunk_of[x] = (uint8_t)c;
        }
        auto slice_of = [&](int32_t it) {
            return (int)((int64_t)it * n_slices / (n_items > 0 ? n_items : 1));
        };
        sched_by_key_then_user(
            user_ids, n, n_users, n_chunks * n_slices,
            [&](int64_t p) { return (int)chunk_of[user_ids[p]] * n_slices + slice_of(item_ids[p]); },
            sched_out, tile_offsets);
    } catch (const std::bad_alloc&) {
        set_error("mf_sched_tiles: out of host memory");
        return MF_ERR_NOMEM;
    }
    return MF_OK;
}
