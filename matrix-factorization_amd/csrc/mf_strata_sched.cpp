// mf_strata_sched.cpp -- plan of the slotted stratified sweep
// (mf_strata_plan_*; kernel: mf_strata.hpp).
//
// Ratings are bucketed into C*B*B blocks: C*B user ranges (C = the number of
// user-range classes, 1 by default) x B item ranges; block (ub, ib) belongs
// to stratum s = (ub - C*ib) mod C*B, slot w = ib, and is stored at s*B + w
// (C = 1: s = (ub - ib) mod B).  Stratum s holds the user ranges of class
// s mod C only, so strata of different classes share no user (the kernel's
// slack between hand-offs, mf_strata.hpp).  Inside a block:
//   1. every user of the block is OWNED by one of NS rating slots (longest
//      processing time first: users by falling degree onto the least loaded
//      slot), so all of a user's ratings in the block run on one lane group,
//      in program order -- the kernel never needs a barrier for user rows;
//   2. the ratings are the edges of a bipartite multigraph (slot, item) and
//      are edge-coloured with exactly D = max(largest slot load, largest item
//      degree) colours (Koenig: alternating-path recolouring), one colour per
//      step.  A step holds at most one rating per slot and per item.
// The block's plan is a dense D x NS grid of rating indices (-1 = idle slot).
// Blocks are planned on worker threads (std::thread, no OpenMP runtime next
// to torch's).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <queue>
#include <thread>
#include <vector>

#include "../../include/mf_hip.h"
#include "mf_host.hpp"

namespace mf {
void set_error(const char* fmt, ...);
}
using mf::set_error;

struct mf_strata_plan {
    int32_t B = 0;
    int32_t C = 1;                  // user-range classes: C*B user ranges
    int32_t NS = 0;
    std::vector<int64_t> bstep;     // C*B*B + 1 step offsets
    std::vector<int32_t> sched;     // bstep[B*B] * NS positions
};

namespace {

struct Scratch {
    std::vector<int32_t> ucnt, uslot, users, load;
    std::vector<int32_t> es, eq, ej, ecol, icnt;
    std::vector<int32_t> sc, ic, path;
};

// Plan one block: ratings idx[0..m) with item ids in [ilo, ilo+nqi) and user
// ids in [ulo, ulo+nus).  Appends D*NS entries to `grid`; returns D.
int32_t plan_block(const int32_t* u, const int32_t* it, const int32_t* idx, int32_t m,
                   int32_t ilo, int32_t nqi, int32_t ulo, int32_t nus, int32_t NS, Scratch& S,
                   std::vector<int32_t>& grid) {
    if (m == 0) return 0;
    if ((int32_t)S.ucnt.size() < nus) {
        S.ucnt.resize(nus, 0);
        S.uslot.resize(nus, -1);
    }
    S.users.clear();
    for (int32_t x = 0; x < m; ++x) {
        const int32_t ul = u[idx[x]] - ulo;
        if (S.ucnt[ul]++ == 0) S.users.push_back(ul);
    }
    // longest processing time first: users by falling degree (ties: id)
    std::sort(S.users.begin(), S.users.end(), [&](int32_t a, int32_t b) {
        return S.ucnt[a] != S.ucnt[b] ? S.ucnt[a] > S.ucnt[b] : a < b;
    });
    S.load.assign(NS, 0);
    using LS = std::pair<int32_t, int32_t>;      // (load, slot), least first
    std::priority_queue<LS, std::vector<LS>, std::greater<LS>> heap;
    for (int32_t s = 0; s < NS; ++s) heap.push({0, s});
    int32_t D = 1;
    for (int32_t ul : S.users) {
        LS top = heap.top();
        heap.pop();
        S.uslot[ul] = top.second;
        top.first += S.ucnt[ul];
        S.load[top.second] = top.first;
        D = std::max(D, top.first);
        heap.push(top);
    }
    S.icnt.assign(nqi, 0);
    S.es.resize(m);
    S.eq.resize(m);
    S.ej.resize(m);
    for (int32_t x = 0; x < m; ++x) {
        const int32_t j = idx[x];
        S.es[x] = S.uslot[u[j] - ulo];
        S.eq[x] = it[j] - ilo;
        S.ej[x] = j;
        D = std::max(D, ++S.icnt[S.eq[x]]);
    }
    for (int32_t ul : S.users) {
        S.ucnt[ul] = 0;
        S.uslot[ul] = -1;
    }
    // Koenig edge colouring with D colours
    S.sc.assign((size_t)NS * D, -1);
    S.ic.assign((size_t)nqi * D, -1);
    S.ecol.assign(m, -1);
    auto set = [&](int32_t e, int32_t c) {
        S.ecol[e] = c;
        S.sc[(size_t)S.es[e] * D + c] = e;
        S.ic[(size_t)S.eq[e] * D + c] = e;
    };
    for (int32_t e = 0; e < m; ++e) {
        const int32_t s = S.es[e], q = S.eq[e];
        const int32_t* scs = &S.sc[(size_t)s * D];
        const int32_t* ics = &S.ic[(size_t)q * D];
        int32_t a = 0, b = 0;
        while (scs[a] >= 0) ++a;                 // free at the slot (< D: load <= D)
        while (ics[b] >= 0) ++b;                 // free at the item
        if (ics[a] < 0) { set(e, a); continue; }
        if (scs[b] < 0) { set(e, b); continue; }
        // swap a <-> b along the alternating path that leaves item q by its
        // a-edge; it never reaches slot s (s has no a-edge), so afterwards a
        // is free at both ends of e
        S.path.clear();
        int32_t cur = q;
        for (;;) {
            const int32_t e1 = S.ic[(size_t)cur * D + a];
            if (e1 < 0) break;
            S.path.push_back(e1);
            const int32_t e2 = S.sc[(size_t)S.es[e1] * D + b];
            if (e2 < 0) break;
            S.path.push_back(e2);
            cur = S.eq[e2];
        }
        for (int32_t pe : S.path) {
            const int32_t c = S.ecol[pe];
            S.sc[(size_t)S.es[pe] * D + c] = -1;
            S.ic[(size_t)S.eq[pe] * D + c] = -1;
        }
        for (int32_t pe : S.path) set(pe, S.ecol[pe] == a ? b : a);
        set(e, a);
    }
    const size_t g0 = grid.size();
    grid.resize(g0 + (size_t)D * NS, -1);
    for (int32_t e = 0; e < m; ++e) grid[g0 + (size_t)S.ecol[e] * NS + S.es[e]] = S.ej[e];
    return D;
}

bool bounds_ok(const int32_t* b, int32_t nb, int32_t total) {
    if (b[0] != 0 || b[nb] != total) return false;
    for (int32_t x = 0; x < nb; ++x)
        if (b[x + 1] < b[x]) return false;
    return true;
}

}  // namespace

extern "C" int mf_strata_plan_build_classes(const int32_t* user_ids, const int32_t* item_ids,
                                            int64_t n, int32_t n_users, int32_t n_items,
                                            int32_t n_blocks, int32_t n_classes,
                                            const int32_t* user_bounds,
                                            const int32_t* item_bounds, int32_t n_slots,
                                            mf_strata_plan** plan_out) {
    if (!plan_out) {
        set_error("NULL plan_out");
        return MF_ERR_INVALID;
    }
    *plan_out = nullptr;
    if (n < 0 || n_users < 0 || n_items < 0 || n_blocks < 1 || n_slots < 1 || n_slots > 4096 ||
        n_classes < 1 || n_classes > MF_STRATA_MAX_CLASSES) {
        set_error("invalid sizes (n=%lld, n_blocks=%d, n_classes=%d, n_slots=%d)", (long long)n,
                  n_blocks, n_classes, n_slots);
        return MF_ERR_INVALID;
    }
    if ((int64_t)n_classes * n_blocks * n_blocks >= ((int64_t)1 << 31) || n > INT32_MAX) {
        set_error("n_blocks=%d / n=%lld too large", n_blocks, (long long)n);
        return MF_ERR_INVALID;
    }
    if (!user_bounds || !item_bounds || (n > 0 && (!user_ids || !item_ids))) {
        set_error("NULL argument");
        return MF_ERR_INVALID;
    }
    const int32_t B = n_blocks, C = n_classes, CB = n_classes * n_blocks;
    if (!bounds_ok(user_bounds, CB, n_users) || !bounds_ok(item_bounds, B, n_items)) {
        set_error("user/item bounds must rise from 0 to n_users/n_items over "
                  "n_classes*n_blocks+1 / n_blocks+1 entries");
        return MF_ERR_INVALID;
    }
    const bool tm = std::getenv("MF_PLAN_TIMING") != nullptr;     // diagnostics
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto t0 = now();
    auto lap = [&](const char* what) {
        if (!tm) return;
        const auto t1 = now();
        std::fprintf(stderr, "[mf_strata_plan] %s %.3f s\n", what,
                     std::chrono::duration<double>(t1 - t0).count());
        t0 = t1;
    };
    std::vector<int32_t> ub_of(n_users), ib_of(n_items);
    for (int32_t b = 0; b < CB; ++b)
        for (int32_t x = user_bounds[b]; x < user_bounds[b + 1]; ++x) ub_of[x] = b;
    for (int32_t b = 0; b < B; ++b)
        for (int32_t x = item_bounds[b]; x < item_bounds[b + 1]; ++x) ib_of[x] = b;
    const int64_t BB = (int64_t)CB * B;
    const int T = mf::host_threads();
    {   // first rating (lowest index) with an id out of range, if any
        std::atomic<int64_t> first_bad{n};
        mf::parallel_chunks(n, T, [&](int, int64_t lo, int64_t hi) {
            for (int64_t j = lo; j < hi; ++j) {
                const int32_t uu = user_ids[j], ii = item_ids[j];
                if (uu < 0 || uu >= n_users || ii < 0 || ii >= n_items) {
                    int64_t cur = first_bad.load();
                    while (j < cur && !first_bad.compare_exchange_weak(cur, j)) {
                    }
                    return;
                }
            }
        });
        const int64_t j = first_bad.load();
        if (j < n) {
            set_error("rating %lld has ids (%d, %d) outside [0,%d) x [0,%d)", (long long)j,
                      user_ids[j], item_ids[j], n_users, n_items);
            return MF_ERR_INVALID;
        }
    }
    // ratings by block (stable): block of (user range ub, item range w) is
    // stored at s*B + w with s = (ub - C*w) mod C*B
    std::vector<int32_t> bucket(n);
    std::vector<int64_t> boff;
    mf::partition_rows(
        n, (int)BB, T,
        [&](int64_t j) {
            const int32_t w = ib_of[item_ids[j]];
            const int64_t sv = (((int64_t)ub_of[user_ids[j]] - (int64_t)C * w) % CB + CB) % CB;
            return (int)(sv * B + w);
        },
        boff, [&](int64_t d, int64_t j) { bucket[d] = (int32_t)j; });
    lap("validate + partition");

    // plan the blocks in chunks of 64 on worker threads
    const int64_t CH = 64;
    const int64_t nch = (BB + CH - 1) / CH;
    std::vector<std::vector<int32_t>> grids(nch);
    std::vector<int32_t> steps(BB, 0);
    std::atomic<int64_t> next{0};
    auto worker = [&]() {
        Scratch S;
        for (;;) {
            const int64_t c = next.fetch_add(1);
            if (c >= nch) break;
            for (int64_t b = c * CH; b < std::min(BB, (c + 1) * CH); ++b) {
                const int32_t s = (int32_t)(b / B), w = (int32_t)(b % B);
                const int32_t ub = (int32_t)(((int64_t)s + (int64_t)C * w) % CB);
                steps[b] = plan_block(user_ids, item_ids, bucket.data() + boff[b],
                                      (int32_t)(boff[b + 1] - boff[b]), item_bounds[w],
                                      item_bounds[w + 1] - item_bounds[w], user_bounds[ub],
                                      user_bounds[ub + 1] - user_bounds[ub], n_slots, S, grids[c]);
            }
        }
    };
    const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    const unsigned nt = (unsigned)std::min<int64_t>(hw, std::max<int64_t>(1, n / 200000));
    std::vector<std::thread> th;
    for (unsigned t = 1; t < nt; ++t) th.emplace_back(worker);
    worker();
    for (auto& t : th) t.join();
    lap("plan blocks");

    auto* plan = new (std::nothrow) mf_strata_plan;
    if (!plan) {
        set_error("out of host memory");
        return MF_ERR_NOMEM;
    }
    plan->B = B;
    plan->C = C;
    plan->NS = n_slots;
    plan->bstep.resize(BB + 1);
    plan->bstep[0] = 0;
    for (int64_t b = 0; b < BB; ++b) plan->bstep[b + 1] = plan->bstep[b] + steps[b];
    plan->sched.reserve((size_t)plan->bstep[BB] * n_slots);
    for (auto& g : grids) {
        plan->sched.insert(plan->sched.end(), g.begin(), g.end());
        std::vector<int32_t>().swap(g);
    }
    lap("assemble");
    *plan_out = plan;
    return MF_OK;
}

extern "C" int mf_strata_plan_build(const int32_t* user_ids, const int32_t* item_ids, int64_t n,
                                    int32_t n_users, int32_t n_items, int32_t n_blocks,
                                    const int32_t* user_bounds, const int32_t* item_bounds,
                                    int32_t n_slots, mf_strata_plan** plan_out) {
    return mf_strata_plan_build_classes(user_ids, item_ids, n, n_users, n_items, n_blocks, 1,
                                        user_bounds, item_bounds, n_slots, plan_out);
}

extern "C" int64_t mf_strata_plan_positions(const mf_strata_plan* plan) {
    return plan ? (int64_t)plan->sched.size() : -1;
}

extern "C" int mf_strata_plan_fetch(const mf_strata_plan* plan, int32_t* sched_out,
                                    int64_t* block_steps) {
    if (!plan || !block_steps || (!plan->sched.empty() && !sched_out)) {
        set_error("NULL argument");
        return MF_ERR_INVALID;
    }
    std::copy(plan->sched.begin(), plan->sched.end(), sched_out);
    std::copy(plan->bstep.begin(), plan->bstep.end(), block_steps);
    return MF_OK;
}

extern "C" void mf_strata_plan_free(mf_strata_plan* plan) { delete plan; }
