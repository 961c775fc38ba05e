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
#include <memory>
#include <new>
#include <stdexcept>
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
    mf::big_ptr<int32_t> sched{nullptr, mf::MapFree{0}};   // bstep[C*B*B] * NS positions
    int64_t n_sched = 0;
};

namespace {

// diagnostics (MF_PLAN_TIMING): time per planning phase, summed over blocks
std::atomic<int64_t> g_phase_ns[4];
std::atomic<int64_t> g_paths{0}, g_path_len{0};

struct Trip { int32_t row, u, i; };               // a rating's row and ids

struct Scratch {
    std::vector<uint64_t> smask, imask, lvl, ubits;
    std::vector<int32_t> dstart, order;
    std::vector<int32_t> ucnt, uslot, users, load;
    std::vector<int32_t> es, eq, ecol, icnt;
    std::vector<int32_t> sc, ic, path;
};

// Plan one block: its m ratings (bt[]: row, user id, item id; in row order)
// with item ids in [ilo, ilo+nqi) and user ids in [ulo, ulo+nus).  Returns D
// and, with `pos`, writes each rating's position in the block's D*NS grid
// (step * NS + slot) to pos[] (without: the step count only -- D is known
// before the colouring).  es_save: each rating's slot is written there;
// es_load: the slots are taken from there (a step-count pass of the same NS)
// instead of being assigned again.
int32_t plan_block(const Trip* bt, int32_t m,
                   int32_t ilo, int32_t nqi, int32_t ulo, int32_t nus, int32_t NS, Scratch& S,
                   int32_t* pos, int32_t* es_save = nullptr, const int32_t* es_load = nullptr) {
    if (m == 0) return 0;
    using clk = std::chrono::steady_clock;
    const auto c0 = clk::now();
    auto c1 = c0;
    int32_t D = 1;
    if (es_load) {                               // slots known: loads and degrees only
        S.es.assign(es_load, es_load + m);
        S.eq.resize(m);
        S.icnt.assign(nqi, 0);
        S.load.assign(NS, 0);
        for (int32_t x = 0; x < m; ++x) {
            S.eq[x] = bt[x].i - ilo;
            D = std::max(D, ++S.icnt[S.eq[x]]);
            D = std::max(D, ++S.load[S.es[x]]);
        }
        goto colour;
    }
    {
    if ((int32_t)S.ucnt.size() < nus) {
        S.ucnt.resize(nus, 0);
        S.uslot.resize(nus, -1);
    }
    const int32_t NW = (nus + 63) >> 6;
    if ((int32_t)S.ubits.size() < NW) S.ubits.resize(NW, 0);
    S.users.clear();
    int32_t maxdeg = 0;
    for (int32_t x = 0; x < m; ++x) {
        const int32_t ul = bt[x].u - ulo;
        if (S.ucnt[ul]++ == 0) S.users.push_back(ul);
        S.ubits[ul >> 6] |= 1ull << (ul & 63);
        maxdeg = std::max(maxdeg, S.ucnt[ul]);
    }
    // longest processing time first: users by falling degree, ties by id --
    // a counting sort (degrees are small), ids ascending within a degree
    S.dstart.assign((size_t)maxdeg + 2, 0);
    for (int32_t ul : S.users) ++S.dstart[(size_t)(maxdeg - S.ucnt[ul]) + 1];
    for (int32_t d = 0; d <= maxdeg; ++d) S.dstart[d + 1] += S.dstart[d];
    S.order.resize(S.users.size());
    if ((int64_t)S.users.size() * 8 < nus) {                       // few users: sort them
        std::sort(S.users.begin(), S.users.end());                // ids ascending
        for (int32_t ul : S.users) S.order[(size_t)S.dstart[maxdeg - S.ucnt[ul]]++] = ul;
    } else {                        // else the set bits of the id range, ascending
        for (int32_t w = 0; w < NW; ++w)
            for (uint64_t b = S.ubits[w]; b; b &= b - 1) {
                const int32_t ul = w * 64 + __builtin_ctzll(b);
                S.order[(size_t)S.dstart[maxdeg - S.ucnt[ul]]++] = ul;
            }
    }
    if ((int64_t)S.users.size() * 4 < NW)
        for (int32_t ul : S.users) S.ubits[ul >> 6] = 0;
    else
        std::fill(S.ubits.begin(), S.ubits.begin() + NW, 0);
    c1 = clk::now();
    // each user onto the least loaded slot, ties to the lowest slot index
    // (the order a (load, slot) min-heap pops): one bit set of slots per load
    // level, the lowest set bit of the lowest non-empty level is the slot
    const int32_t WD = (NS + 63) / 64;
    // > any load reached: LPT puts a user on a slot loaded <= m / NS (the
    // mean), so no load exceeds m / NS + maxdeg (int64: no overflow for a
    // block of a heavy user among many)
    int64_t cap = (int64_t)m / NS + maxdeg + 2;
    S.lvl.assign((size_t)cap * WD, 0);
    for (int32_t x = 0; x < NS; ++x) S.lvl[(size_t)(x >> 6)] |= 1ull << (x & 63);
    S.load.assign(NS, 0);
    int32_t low = 0;
    if (WD == 1) {             // NS <= 64: one word per level
        uint64_t* L = S.lvl.data();
        const size_t U = S.order.size();
        for (size_t k = 0; k < U;) {
            while (!L[low]) ++low;
            if ((int64_t)low + 1 >= cap) {                        // grow (never reached)
                S.lvl.resize((size_t)low + 2, 0);
                cap = (int64_t)low + 2;
                L = S.lvl.data();
            }
            const int32_t ul0 = S.order[k];
            if (S.ucnt[ul0] == 1) {
                // degree 1 from here on (falling degree): the users take the
                // level's slots in ascending order, each to level low + 1 --
                // what one user at a time would do
                uint64_t b = L[low], moved = 0;
                for (; b && k < U; b &= b - 1) {
                    const int32_t slot = __builtin_ctzll(b), ul = S.order[k++];
                    moved |= 1ull << slot;
                    S.uslot[ul] = slot;
                    S.load[slot] = low + 1;
                }
                L[low] = b;
                L[low + 1] |= moved;
                D = std::max(D, low + 1);
                continue;
            }
            const int32_t slot = __builtin_ctzll(L[low]);
            L[low] &= L[low] - 1;
            const int32_t nl = low + S.ucnt[ul0];
            if (nl >= cap) {                                      // grow (never reached)
                S.lvl.resize((size_t)nl + 1, 0);
                cap = (int64_t)nl + 1;
                L = S.lvl.data();
            }
            L[nl] |= 1ull << slot;
            S.uslot[ul0] = slot;
            S.load[slot] = nl;
            D = std::max(D, nl);
            ++k;
        }
    } else
    for (int32_t ul : S.order) {
        while (true) {                                            // lowest non-empty level
            bool any = false;
            for (int32_t w = 0; w < WD; ++w) any |= S.lvl[(size_t)low * WD + w] != 0;
            if (any) break;
            ++low;
        }
        int32_t slot = 0;
        for (int32_t w = 0; w < WD; ++w) {
            const uint64_t b = S.lvl[(size_t)low * WD + w];
            if (b) { slot = w * 64 + __builtin_ctzll(b); break; }
        }
        S.lvl[(size_t)low * WD + (slot >> 6)] &= ~(1ull << (slot & 63));
        const int32_t nl = low + S.ucnt[ul];
        if (nl >= cap) {                                          // grow (never reached)
            S.lvl.resize((size_t)(nl + 1) * WD, 0);
            cap = (int64_t)nl + 1;
        }
        S.lvl[(size_t)nl * WD + (slot >> 6)] |= 1ull << (slot & 63);
        S.uslot[ul] = slot;
        S.load[slot] = nl;
        D = std::max(D, nl);
    }
    S.icnt.assign(nqi, 0);
    S.es.resize(m);
    S.eq.resize(m);
    for (int32_t x = 0; x < m; ++x) {
        S.es[x] = S.uslot[bt[x].u - ulo];
        S.eq[x] = bt[x].i - ilo;
        D = std::max(D, ++S.icnt[S.eq[x]]);
    }
    for (int32_t ul : S.users) {
        S.ucnt[ul] = 0;
        S.uslot[ul] = -1;
    }
    if (es_save) std::copy(S.es.begin(), S.es.begin() + m, es_save);
    }
    if (!pos) return D;                          // the step count only
colour:
    // a grid position is step * NS + slot in int32: a block whose D x NS grid
    // reaches 2^31 (one very skewed block: D can reach m) is refused
    if ((int64_t)D * NS >= ((int64_t)1 << 31))
        throw std::length_error("a strata block's grid of D x NS positions reaches 2^31");
    const auto c2 = clk::now();
    // Koenig edge colouring with D colours
    S.ecol.resize(m);
    auto set = [&](int32_t e, int32_t c) {
        S.ecol[e] = c;
        S.sc[(size_t)S.es[e] * D + c] = e;
        S.ic[(size_t)S.eq[e] * D + c] = e;
    };
    // the (slot, colour) and (item, colour) -> edge tables, for the repairs;
    // with masks they are built at the first repair, from the colours so far
    bool tables = false;
    auto build_tables = [&](int32_t upto) {
        S.sc.assign((size_t)NS * D, -1);
        S.ic.assign((size_t)nqi * D, -1);
        for (int32_t x = 0; x < upto; ++x) set(x, S.ecol[x]);
        tables = true;
    };
    // used-colour masks per slot and per item (D <= 64): a colour free at both
    // ends is found in O(1), and the alternating-path repair runs only when
    // the two ends have no free colour in common
    const bool masks = D <= 64;
    if (masks) {
        S.smask.assign(NS, 0);
        S.imask.assign(nqi, 0);
    } else {
        build_tables(0);
    }
    for (int32_t e = 0; e < m; ++e) {
        const int32_t s = S.es[e], q = S.eq[e];
        if (masks) {
            const uint64_t both = S.smask[s] | S.imask[q];
            if (~both & (D == 64 ? ~0ull : ((1ull << D) - 1))) {
                const int32_t c = __builtin_ctzll(~both);
                if (tables) set(e, c);
                else S.ecol[e] = c;
                S.smask[s] |= 1ull << c;
                S.imask[q] |= 1ull << c;
                continue;
            }
            if (!tables) build_tables(e);
        }
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
        g_paths += 1;
        g_path_len += (int64_t)S.path.size();
        if (masks) {   // colours a and b moved along the path: refresh its ends' masks
            const uint64_t ab = (1ull << a) | (1ull << b);
            auto fix_s = [&](int32_t x) {
                uint64_t mk = S.smask[x] & ~ab;
                if (S.sc[(size_t)x * D + a] >= 0) mk |= 1ull << a;
                if (S.sc[(size_t)x * D + b] >= 0) mk |= 1ull << b;
                S.smask[x] = mk;
            };
            auto fix_i = [&](int32_t x) {
                uint64_t mk = S.imask[x] & ~ab;
                if (S.ic[(size_t)x * D + a] >= 0) mk |= 1ull << a;
                if (S.ic[(size_t)x * D + b] >= 0) mk |= 1ull << b;
                S.imask[x] = mk;
            };
            fix_s(s);
            fix_i(q);
            for (int32_t pe : S.path) {
                fix_s(S.es[pe]);
                fix_i(S.eq[pe]);
            }
        }
    }
    const auto c3 = clk::now();
    for (int32_t e = 0; e < m; ++e) pos[e] = S.ecol[e] * NS + S.es[e];
    const auto c4 = clk::now();
    auto ns = [](auto a, auto b) {
        return (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(b - a).count();
    };
    g_phase_ns[0] += ns(c0, c1);
    g_phase_ns[1] += ns(c1, c2);
    g_phase_ns[2] += ns(c2, c3);
    g_phase_ns[3] += ns(c3, c4);
    return D;
}

bool bounds_ok(const int32_t* b, int32_t nb, int32_t total) {
    if (b[0] != 0 || b[nb] != total) return false;
    for (int32_t x = 0; x < nb; ++x)
        if (b[x + 1] < b[x]) return false;
    return true;
}

}  // namespace

static int plan_build(const int32_t* user_ids, const int32_t* item_ids, int64_t n,
                      int32_t n_users, int32_t n_items, int32_t n_blocks, int32_t n_classes,
                      const int32_t* user_bounds, const int32_t* item_bounds,
                      const int32_t* slot_cands, const int32_t* wave_cands, int32_t n_cands,
                      double fill_stop, int32_t* picked, mf_strata_plan** plan_out) {
    if (!plan_out) {
        set_error("NULL plan_out");
        return MF_ERR_INVALID;
    }
    *plan_out = nullptr;
    if (!slot_cands || !wave_cands || n_cands < 1 || n_cands > 8) {
        set_error("1 to 8 (slots, waves) candidates expected");
        return MF_ERR_INVALID;
    }
    for (int32_t c = 0; c < n_cands; ++c) {
        if (n < 0 || n_users < 0 || n_items < 0 || n_blocks < 1 || slot_cands[c] < 1 ||
            slot_cands[c] > 4096 || wave_cands[c] < 1 || n_classes < 1 ||
            n_classes > MF_STRATA_MAX_CLASSES) {
            set_error("invalid sizes (n=%lld, n_blocks=%d, n_classes=%d, n_slots=%d, waves=%d)",
                      (long long)n, n_blocks, n_classes, slot_cands[c], wave_cands[c]);
            return MF_ERR_INVALID;
        }
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
    lap("range tables");
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
    // stored at s*B + w with s = (ub - C*w) mod C*B.  Two passes keep every
    // scatter cache-sized: the rows by stratum s (C*B buckets, threaded over
    // row chunks), then each stratum's rows by w (B buckets, strata spread
    // over the threads); both passes are stable, so the blocks keep row order.
    // The passes carry the user and item ids along, so planning a block
    // reads its ratings sequentially.  Large buffers are not value-initialised
    // (the threads that fill them touch their pages first).
    lap("validate");
    auto buf = [](int64_t len) {
        auto b = mf::big_alloc<int32_t>(len);
        if (!b) throw std::bad_alloc();
        return b;
    };
    auto key = buf(n);
    // the stratum of every row once (the user-range lookup is a random read of
    // a 4 MB table per row; the partition reads the key twice)
    auto key_pass = [&](auto* ubt, auto* ibt) {
        mf::parallel_chunks(n, T, [&](int, int64_t lo, int64_t hi) {
            for (int64_t j = lo; j < hi; ++j) {
                // ub < C*B and C*w < C*B: one conditional add, no division
                const int32_t sv = (int32_t)ubt[user_ids[j]] - C * (int32_t)ibt[item_ids[j]];
                key[j] = sv < 0 ? sv + CB : sv;
            }
        });
    };
    if (CB < 65536) {       // 16-bit range tables: the 10^6-user table stays in cache
        std::vector<uint16_t> u16(ub_of.begin(), ub_of.end()), i16(ib_of.begin(), ib_of.end());
        key_pass(u16.data(), i16.data());
    } else {
        key_pass(ub_of.data(), ib_of.data());
    }
    lap("stratum keys");
    std::vector<int64_t> soff, boff((size_t)BB + 1, 0);
    auto strip = mf::big_alloc<Trip>(n);
    if (!strip) throw std::bad_alloc();
    mf::partition_rows(
        n, CB, T, [&](int64_t j) { return (int)key[j]; },
        soff, [&](int64_t d, int64_t j) { strip[d] = Trip{(int32_t)j, user_ids[j], item_ids[j]}; });
    key.reset();
    lap("validate + stratum pass");
    auto b_t = mf::big_alloc<Trip>(n);         // one write stream per bucket
    if (!b_t) throw std::bad_alloc();
    mf::for_buckets(CB, T, [&](int sv) {
        const int64_t lo = soff[sv], hi = soff[sv + 1];
        std::vector<int64_t> cnt((size_t)B + 1, 0);
        thread_local std::vector<int32_t> wv;     // each row's item range, looked up once
        wv.resize((size_t)(hi - lo));
        for (int64_t d = lo; d < hi; ++d) {
            const int32_t w = ib_of[strip[d].i];
            wv[(size_t)(d - lo)] = w;
            ++cnt[w + 1];
        }
        for (int32_t w = 0; w < B; ++w) cnt[w + 1] += cnt[w];
        for (int32_t w = 0; w < B; ++w) boff[(size_t)sv * B + w] = lo + cnt[w];
        for (int64_t d = lo; d < hi; ++d) b_t[lo + cnt[wv[(size_t)(d - lo)]]++] = strip[d];
    });
    boff[BB] = n;
    strip.reset();
    lap("block pass");

    // Plan the blocks in chunks of 64 on worker threads.  With several
    // (slots, waves) candidates, the step counts of each come first (the slot
    // assignment and the degrees: no colouring) and pick the one of least
    // steps * waves -- the first as soon as it fills fill_stop of its
    // positions; then the pick is planned in one pass: a block's step count
    // is known only once it is coloured, so each rating's grid position
    // (step * NS + slot, < 2^31: D <= m) is kept beside it and the grids are
    // written once the step offsets are summed.
    const int64_t CH = 64;
    const int64_t nch = (BB + CH - 1) / CH;
    std::vector<int32_t> steps(BB, 0);
    auto b_pos = buf(n);
    const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    const unsigned nt = (unsigned)std::min<int64_t>(hw, std::max<int64_t>(1, n / 200000));
    auto blocks = [&](int32_t NS, int32_t* pos, int32_t* es_save, const int32_t* es_load) {
        std::atomic<int64_t> next{0};
        mf::ThreadErr err;
        auto worker = [&]() { err.guard([&]() {
            Scratch S;
            for (;;) {
                if (err.failed()) break;               // another worker threw: stop
                const int64_t c = next.fetch_add(1);
                if (c >= nch) break;
                for (int64_t b = c * CH; b < std::min(BB, (c + 1) * CH); ++b) {
                    const int32_t sv = (int32_t)(b / B), w = (int32_t)(b % B);
                    const int32_t ub = (int32_t)(((int64_t)sv + (int64_t)C * w) % CB);
                    const int64_t o = boff[b];
                    steps[b] = plan_block(
                        b_t.get() + o, (int32_t)(boff[b + 1] - o),
                        item_bounds[w], item_bounds[w + 1] - item_bounds[w], user_bounds[ub],
                        user_bounds[ub + 1] - user_bounds[ub], NS, S, pos ? pos + o : nullptr,
                        es_save ? es_save + o : nullptr, es_load ? es_load + o : nullptr);
                }
            }
        }); };
        std::vector<std::thread> th;
        for (unsigned t = 1; t < nt; ++t) th.emplace_back(worker);
        worker();
        for (auto& t : th) t.join();
        err.rethrow();                                 // -> the C ABI's bad_alloc path
    };
    int32_t pick = 0;
    // the slots of the best candidate so far and of the current one: the
    // pick's full pass colours from them instead of assigning them again
    decltype(buf(0)) es_best, es_cur;
    if (n_cands > 1) {
        int64_t best = -1;
        es_best = buf(n);
        es_cur = buf(n);
        for (int32_t c = 0; c < n_cands; ++c) {
            blocks(slot_cands[c], nullptr, es_cur.get(), nullptr);
            int64_t total = 0;
            for (int64_t b = 0; b < BB; ++b) total += steps[b];
            const int64_t cost = total * wave_cands[c];
            if (best < 0 || cost < best) {
                best = cost;
                pick = c;
                std::swap(es_best, es_cur);
            }
            const double fill = (double)n / (double)std::max<int64_t>(total * slot_cands[c], 1);
            if (c == 0 && fill_stop > 0 && fill >= fill_stop) break;
        }
        lap("candidate steps");
    }
    const int32_t n_slots = slot_cands[pick];
    if (picked) *picked = pick;
    es_cur.reset();
    blocks(n_slots, b_pos.get(), nullptr, es_best ? es_best.get() : nullptr);
    es_best.reset();
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
    plan->sched = mf::big_alloc<int32_t>(plan->bstep[BB] * n_slots);
    if (!plan->sched) {                            // (the plan is not yet handed out)
        delete plan;
        set_error("out of host memory");
        return MF_ERR_NOMEM;
    }
    plan->n_sched = plan->bstep[BB] * n_slots;
    int32_t* sched = plan->sched.get();
    mf::for_buckets((int)nch, T, [&](int c) {
        for (int64_t b = c * CH; b < std::min(BB, (c + 1) * CH); ++b) {
            int32_t* grid = sched + plan->bstep[b] * n_slots;
            std::fill(grid, grid + (int64_t)steps[b] * n_slots, -1);
            for (int64_t e = boff[b]; e < boff[b + 1]; ++e) grid[b_pos[e]] = b_t[e].row;
        }
    });
    lap("grids");
    if (tm) {
        std::fprintf(stderr, "[mf_strata_plan]   per-block phases (thread-s): users+sort %.3f, "
                     "slots+edges %.3f, colour %.3f, grid %.3f; repairs %lld, mean path %.1f\n",
                     g_phase_ns[0] * 1e-9, g_phase_ns[1] * 1e-9, g_phase_ns[2] * 1e-9,
                     g_phase_ns[3] * 1e-9, (long long)g_paths.load(),
                     g_paths ? (double)g_path_len / (double)g_paths : 0.0);
        for (auto& x : g_phase_ns) x = 0;
        g_paths = 0;
        g_path_len = 0;
    }
    *plan_out = plan;
    return MF_OK;
}

extern "C" int mf_strata_plan_build_pick(const int32_t* user_ids, const int32_t* item_ids,
                                         int64_t n, int32_t n_users, int32_t n_items,
                                         int32_t n_blocks, int32_t n_classes,
                                         const int32_t* user_bounds, const int32_t* item_bounds,
                                         const int32_t* slot_cands, const int32_t* wave_cands,
                                         int32_t n_cands, double fill_stop, int32_t* picked,
                                         mf_strata_plan** plan_out) {
    try {
        return plan_build(user_ids, item_ids, n, n_users, n_items, n_blocks, n_classes,
                          user_bounds, item_bounds, slot_cands, wave_cands, n_cands, fill_stop,
                          picked, plan_out);
    } catch (const std::bad_alloc&) {
        if (plan_out) *plan_out = nullptr;
        set_error("out of host memory (strata plan of %lld ratings)", (long long)n);
        return MF_ERR_NOMEM;
    } catch (const std::exception& e) {
        if (plan_out) *plan_out = nullptr;
        set_error("strata planner failed: %s", e.what());
        return MF_ERR_INVALID;
    }
}

extern "C" int mf_strata_plan_build_classes(const int32_t* user_ids, const int32_t* item_ids,
                                            int64_t n, int32_t n_users, int32_t n_items,
                                            int32_t n_blocks, int32_t n_classes,
                                            const int32_t* user_bounds,
                                            const int32_t* item_bounds, int32_t n_slots,
                                            mf_strata_plan** plan_out) {
    try {
        const int32_t waves = 1;
        return plan_build(user_ids, item_ids, n, n_users, n_items, n_blocks, n_classes,
                          user_bounds, item_bounds, &n_slots, &waves, 1, 0.0, nullptr, plan_out);
    } catch (const std::bad_alloc&) {
        if (plan_out) *plan_out = nullptr;
        set_error("out of host memory (strata plan of %lld ratings)", (long long)n);
        return MF_ERR_NOMEM;
    } catch (const std::exception& e) {
        if (plan_out) *plan_out = nullptr;
        set_error("strata planner failed: %s", e.what());
        return MF_ERR_INVALID;
    }
}

extern "C" int mf_strata_plan_build(const int32_t* user_ids, const int32_t* item_ids, int64_t n,
                                    int32_t n_users, int32_t n_items, int32_t n_blocks,
                                    const int32_t* user_bounds, const int32_t* item_bounds,
                                    int32_t n_slots, mf_strata_plan** plan_out) {
    return mf_strata_plan_build_classes(user_ids, item_ids, n, n_users, n_items, n_blocks, 1,
                                        user_bounds, item_bounds, n_slots, plan_out);
}

extern "C" int64_t mf_strata_plan_positions(const mf_strata_plan* plan) {
    return plan ? plan->n_sched : -1;
}

extern "C" int mf_strata_plan_fetch(const mf_strata_plan* plan, int32_t* sched_out,
                                    int64_t* block_steps) {
    if (!plan || !block_steps || (plan->n_sched > 0 && !sched_out)) {
        set_error("NULL argument");
        return MF_ERR_INVALID;
    }
    // threaded copy (10^8 positions at C3)
    const int32_t* src = plan->sched.get();
    mf::parallel_chunks(plan->n_sched, mf::host_threads(), [&](int, int64_t lo, int64_t hi) {
        std::copy(src + lo, src + hi, sched_out + lo);
    });
    std::copy(plan->bstep.begin(), plan->bstep.end(), block_steps);
    return MF_OK;
}

extern "C" void mf_strata_plan_free(mf_strata_plan* plan) { delete plan; }
