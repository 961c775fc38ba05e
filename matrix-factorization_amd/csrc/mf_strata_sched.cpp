// mf_strata_sched.cpp -- plan of the stratified sweep (mf_sched_strata;
// kernel: mf_strata.hpp).
//
// Ratings are bucketed into B*B blocks (user range x item range), stored
// block-major with block (ub, ib) at stratum s = (ub - ib) mod B, slot w = ib,
// and coloured inside each block: greedy, item-major, item j starting its
// colour search at (sum of the previous items' degrees) mod D, D = the block's
// largest item / user degree, so colours come out close to D in number and
// even in size.  A user's ratings inside one block get colours >= user_gap
// apart.  Blocks are coloured on worker threads (std::thread, no OpenMP
// runtime next to torch's).
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <thread>
#include <vector>

#include "../../include/mf_hip.h"

namespace mf {
void set_error(const char* fmt, ...);
}
using mf::set_error;

namespace {

struct Scratch {
    std::vector<int32_t> idx, byitem, icount, ucount, uhead, next, colour, csize, cpos;
    std::vector<uint32_t> stamp;
    uint32_t cur = 0;
};

// Colour block [lo, hi) of `sched` in place; returns the colour offsets
// (relative to lo, n_colours + 1 entries).
std::vector<int32_t> colour_block(const int32_t* u, const int32_t* it, int32_t* sched, int64_t lo,
                                  int64_t hi, int32_t ilo, int32_t nqi, int32_t ulo, int32_t nus,
                                  int32_t gap, Scratch& S) {
    const int32_t m = (int32_t)(hi - lo);
    std::vector<int32_t> offs(1, 0);
    if (m == 0) return offs;
    S.idx.assign(sched + lo, sched + hi);
    S.icount.assign((size_t)nqi + 1, 0);
    if ((int32_t)S.ucount.size() < nus) S.ucount.resize(nus, 0);
    if ((int32_t)S.uhead.size() < nus) S.uhead.resize(nus, -1);
    int32_t dmax = 1;
    for (int32_t x = 0; x < m; ++x) {
        const int32_t j = S.idx[x];
        ++S.icount[it[j] - ilo + 1];
        dmax = std::max(dmax, ++S.ucount[u[j] - ulo]);
    }
    for (int32_t q = 0; q < nqi; ++q) {
        dmax = std::max(dmax, S.icount[q + 1]);
        S.icount[q + 1] += S.icount[q];
    }
    S.byitem.resize(m);
    for (int32_t x = 0; x < m; ++x) {                  // stable by item
        const int32_t j = S.idx[x];
        S.byitem[S.icount[it[j] - ilo]++] = j;
    }
    for (int32_t x = 0; x < m; ++x) S.ucount[u[S.idx[x]] - ulo] = 0;
    S.next.resize(m);
    S.colour.resize(m);
    const int32_t D = dmax;
    int64_t rot = 0;
    int32_t ncol = 0;
    int32_t x = 0;
    while (x < m) {
        const int32_t item = it[S.byitem[x]];
        int32_t y = x;
        while (y < m && it[S.byitem[y]] == item) ++y;
        if (++S.cur == 0) {                            // stamp wrap: reset
            std::fill(S.stamp.begin(), S.stamp.end(), 0u);
            S.cur = 1;
        }
        const int32_t start = (int32_t)(rot % D);
        rot += y - x;
        for (int32_t z = x; z < y; ++z) {
            const int32_t j = S.byitem[z];
            const int32_t ul = u[j] - ulo;
            for (int32_t t = 0;; ++t) {
                const int32_t c = t < D ? (start + t) % D : t;
                if (c < (int32_t)S.stamp.size() && S.stamp[c] == S.cur) continue;
                bool ok = true;
                for (int32_t e = S.uhead[ul]; e >= 0; e = S.next[e]) {
                    if (std::abs(S.colour[e] - c) < gap) { ok = false; break; }
                }
                if (!ok) continue;
                if (c >= (int32_t)S.stamp.size()) S.stamp.resize((size_t)c + 64, 0u);
                S.stamp[c] = S.cur;
                S.colour[z] = c;
                S.next[z] = S.uhead[ul];
                S.uhead[ul] = z;
                ncol = std::max(ncol, c + 1);
                break;
            }
        }
        x = y;
    }
    for (int32_t z = 0; z < m; ++z) S.uhead[u[S.byitem[z]] - ulo] = -1;
    // stable counting sort by colour
    S.csize.assign((size_t)ncol + 1, 0);
    for (int32_t z = 0; z < m; ++z) ++S.csize[S.colour[z] + 1];
    for (int32_t c = 0; c < ncol; ++c) S.csize[c + 1] += S.csize[c];
    offs.assign(S.csize.begin(), S.csize.end());
    S.cpos.assign(S.csize.begin(), S.csize.end() - 1);
    for (int32_t z = 0; z < m; ++z) sched[lo + S.cpos[S.colour[z]]++] = S.byitem[z];
    return offs;
}

bool bounds_ok(const int32_t* b, int32_t nb, int32_t total) {
    if (b[0] != 0 || b[nb] != total) return false;
    for (int32_t x = 0; x < nb; ++x)
        if (b[x + 1] < b[x]) return false;
    return true;
}

}  // namespace

extern "C" int mf_sched_strata(const int32_t* user_ids, const int32_t* item_ids, int64_t n,
                               int32_t n_users, int32_t n_items, int32_t n_blocks,
                               const int32_t* user_bounds, const int32_t* item_bounds,
                               int32_t user_gap, int32_t* sched_out, int64_t* block_offsets,
                               int32_t* colour_start, int32_t* colour_offsets,
                               int64_t colour_cap, int64_t* n_colour_offsets) {
    if (n < 0 || n_users < 0 || n_items < 0 || n_blocks < 1 || colour_cap < 0) {
        set_error("invalid sizes (n=%lld, n_blocks=%d)", (long long)n, n_blocks);
        return MF_ERR_INVALID;
    }
    if ((int64_t)n_blocks * n_blocks >= ((int64_t)1 << 31) || n > INT32_MAX) {
        set_error("n_blocks=%d / n=%lld too large", n_blocks, (long long)n);
        return MF_ERR_INVALID;
    }
    if (user_gap < 1 || user_gap > 2) {
        set_error("user_gap must be 1 or 2, got %d", user_gap);
        return MF_ERR_INVALID;
    }
    if (!user_bounds || !item_bounds || !block_offsets || !colour_start || !n_colour_offsets ||
        (n > 0 && (!user_ids || !item_ids || !sched_out))) {
        set_error("NULL argument");
        return MF_ERR_INVALID;
    }
    const int32_t B = n_blocks;
    if (!bounds_ok(user_bounds, B, n_users) || !bounds_ok(item_bounds, B, n_items)) {
        set_error("user/item bounds must rise from 0 to n_users/n_items over n_blocks+1 entries");
        return MF_ERR_INVALID;
    }
    std::vector<int32_t> ub_of(n_users), ib_of(n_items);
    for (int32_t b = 0; b < B; ++b) {
        for (int32_t x = user_bounds[b]; x < user_bounds[b + 1]; ++x) ub_of[x] = b;
        for (int32_t x = item_bounds[b]; x < item_bounds[b + 1]; ++x) ib_of[x] = b;
    }
    const int64_t BB = (int64_t)B * B;
    std::vector<int32_t> key(n);
    std::vector<int64_t> pos(BB + 1, 0);
    for (int64_t j = 0; j < n; ++j) {
        const int32_t uu = user_ids[j], ii = item_ids[j];
        if (uu < 0 || uu >= n_users || ii < 0 || ii >= n_items) {
            set_error("rating %lld has ids (%d, %d) outside [0,%d) x [0,%d)", (long long)j, uu, ii,
                      n_users, n_items);
            return MF_ERR_INVALID;
        }
        const int32_t w = ib_of[ii];
        const int32_t s = (ub_of[uu] - w + B) % B;
        key[j] = (int32_t)((int64_t)s * B + w);
        ++pos[key[j] + 1];
    }
    for (int64_t b = 0; b < BB; ++b) pos[b + 1] += pos[b];
    std::copy(pos.begin(), pos.end(), block_offsets);
    for (int64_t j = 0; j < n; ++j) sched_out[pos[key[j]]++] = (int32_t)j;
    std::vector<int32_t>().swap(key);

    std::vector<std::vector<int32_t>> offs(BB);
    std::atomic<int64_t> next{0};
    auto worker = [&]() {
        Scratch S;
        for (;;) {
            const int64_t b0 = next.fetch_add(64);
            if (b0 >= BB) break;
            for (int64_t b = b0; b < std::min(BB, b0 + 64); ++b) {
                const int32_t s = (int32_t)(b / B), w = (int32_t)(b % B);
                const int32_t ub = (w + s) % B;
                offs[b] = colour_block(user_ids, item_ids, sched_out, block_offsets[b],
                                       block_offsets[b + 1], item_bounds[w],
                                       item_bounds[w + 1] - item_bounds[w], user_bounds[ub],
                                       user_bounds[ub + 1] - user_bounds[ub], user_gap, S);
            }
        }
    };
    const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    const unsigned nt = (unsigned)std::min<int64_t>(hw, std::max<int64_t>(1, n / 200000));
    std::vector<std::thread> th;
    for (unsigned t = 1; t < nt; ++t) th.emplace_back(worker);
    worker();
    for (auto& t : th) t.join();

    int64_t tot = 0;
    for (int64_t b = 0; b < BB; ++b) {
        colour_start[b] = (int32_t)tot;
        tot += (int64_t)offs[b].size();
    }
    colour_start[BB] = (int32_t)tot;
    *n_colour_offsets = tot;
    if (tot > colour_cap || tot >= INT32_MAX) {
        set_error("colour_offsets needs %lld entries, colour_cap=%lld", (long long)tot,
                  (long long)colour_cap);
        return MF_ERR_INVALID;
    }
    for (int64_t b = 0; b < BB; ++b)
        std::copy(offs[b].begin(), offs[b].end(), colour_offsets + colour_start[b]);
    return MF_OK;
}
