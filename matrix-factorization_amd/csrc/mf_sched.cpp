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
        const int T = mf::host_threads();
        std::vector<int64_t> start;
        mf::partition_rows(
            n, n_slices, T, [&](int64_t p) { return slice_of(item_ids[p]); }, start,
            [&](int64_t d, int64_t p) { sched_out[d] = (int32_t)p; });
        for (int32_t x = 0; x <= n_slices; ++x) slice_offsets[x] = start[x];
        mf::for_buckets(n_slices, T, [&](int s) {
            int32_t* q = sched_out + start[s];
            const int64_t m = start[s + 1] - start[s];
            std::vector<int64_t> cnt((size_t)n_users + 1, 0);
            for (int64_t j = 0; j < m; ++j) cnt[user_ids[q[j]] + 1] += 1;
            for (int32_t x = 0; x < n_users; ++x) cnt[x + 1] += cnt[x];
            std::vector<int32_t> tmp((size_t)m);
            for (int64_t j = 0; j < m; ++j) tmp[cnt[user_ids[q[j]]]++] = q[j];
            std::copy(tmp.begin(), tmp.end(), q);
        });
    } catch (const std::bad_alloc&) {
        set_error("mf_sched_slices: out of host memory");
        return MF_ERR_NOMEM;
    }
    return MF_OK;
}
