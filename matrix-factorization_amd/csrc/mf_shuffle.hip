// mf_shuffle.hip -- the swaps of NumPy's shuffle on the GPU.
//
// The exact schedule (fit(schedule="exact")) shuffles its 10^8-row visit
// order every epoch with np.random.shuffle (kernel_matrix_factorization.py
// :371 of the reference; mtrand.pyx _shuffle_raw: for i = n-1 .. 1 swap x[i]
// with x[random_interval(i)]).  On one host thread that is ~0.24 s at C3,
// the epoch's bound.  The draws do not depend on the data: they are made on
// the host (mf_legacy_shuffle_draws, one thread, the RandomState advanced as
// by the whole shuffle) and the swaps applied here.
//
// Swap d (d = 0 .. total-1, total = n-1) exchanges x[total - d] and
// x[j_d].  Two swaps commute unless they share a position, and a swap reads
// nothing but its two positions, so a block of swaps [d0, d1) runs in
// rounds of deterministic reservations: every pending swap raises both
// positions' 64-bit reservation word to (round tag << 32 | ~local index)
// -- earlier swaps win -- and a swap holding both words is the earliest
// pending swap touching either position, every earlier swap touching them
// being done: it commits.  The rest go to the next round (a chain of L
// dependent swaps takes L rounds; what is left after kShRounds grid-wide
// rounds is finished by one workgroup, k_sh_finish).  Blocks go in order and hold at most i/32 swaps, so
// ~6 % collide.  Tags only grow, so the words are never cleared (zeroed
// once by the caller).  The last swaps (i below the caller's d_end bound)
// are left to the host (mf_legacy_apply_swaps_i32), where they are cheap.
// The result is the sequential order's, bit for bit (tests/test_gpu_shuffle.py).
#include <cstdlib>

#include "mf_common.hpp"

namespace mf {

constexpr int kShThreads = 256;
constexpr int64_t kShBlockMax = 1 << 22;        // swaps per block at most
constexpr int64_t kShBlockMin = 1 << 12;
constexpr int kShRounds = 3;               // grid-wide rounds per block
constexpr int kShGridMax = 2048;

struct ShArgs {
    const uint32_t* tgt;                          // j_d
    int64_t total, d0, len;                       // swaps d0 .. d0 + len - 1
    unsigned long long* res;                      // reservation word per position
    int32_t* data;
};

// the round's swaps: local indices list[0 .. *n_in), or 0 .. len-1 (list null)
__device__ __forceinline__ int64_t sh_count(const ShArgs& a, const uint32_t* n_in) {
    return n_in ? (int64_t)*n_in : a.len;
}

__global__ __launch_bounds__(kShThreads) void k_sh_reserve(ShArgs a, const uint32_t* list,
                                                           const uint32_t* n_in,
                                                           unsigned long long tag,
                                                           uint32_t* n_out) {
    // the count the commit kernel appends to (its list was consumed a round ago)
    if (blockIdx.x == 0 && threadIdx.x == 0) *n_out = 0u;
    const int64_t cnt = sh_count(a, n_in);
    for (int64_t x = (int64_t)blockIdx.x * kShThreads + threadIdx.x; x < cnt;
         x += (int64_t)gridDim.x * kShThreads) {
        const uint32_t k = list ? list[x] : (uint32_t)x;
        const int64_t d = a.d0 + k;
        const unsigned long long v = (tag << 32) | (unsigned long long)(0xffffffffu - k);
        atomicMax(a.res + (a.total - d), v);
        atomicMax(a.res + a.tgt[d], v);
    }
}

__global__ __launch_bounds__(kShThreads) void k_sh_commit(ShArgs a, const uint32_t* list,
                                                          const uint32_t* n_in,
                                                          unsigned long long tag, uint32_t* out,
                                                          uint32_t* n_out) {
    const int64_t cnt = sh_count(a, n_in);
    for (int64_t x = (int64_t)blockIdx.x * kShThreads + threadIdx.x; x < cnt;
         x += (int64_t)gridDim.x * kShThreads) {
        const uint32_t k = list ? list[x] : (uint32_t)x;
        const int64_t d = a.d0 + k;
        const unsigned long long v = (tag << 32) | (unsigned long long)(0xffffffffu - k);
        const int64_t i = a.total - d, j = a.tgt[d];
        if (a.res[i] == v && a.res[j] == v) {
            const int32_t t = a.data[i];
            a.data[i] = a.data[j];
            a.data[j] = t;
        } else {
            out[atomicAdd(n_out, 1u)] = k;
        }
    }
}

// what the grid-wide rounds left (swaps in dependency chains longer than
// the rounds), finished by one workgroup in more reservation rounds of its
// own (a chain of L swaps takes L rounds; the words are read with atomic
// loads, device-coherent), and, past kShFinishRounds, by one thread in
// swap order (insertion sort: nothing is left by then in practice)
constexpr int kShFinishThreads = 1024;
constexpr int kShFinishRounds = 64;

__global__ __launch_bounds__(kShFinishThreads) void k_sh_finish(ShArgs a, uint32_t* list_a,
                                                                uint32_t* list_b,
                                                                const uint32_t* n_in,
                                                                unsigned long long tag) {
    __shared__ uint32_t s_n[2];
    const int t = threadIdx.x;
    if (t == 0) { s_n[0] = *n_in; s_n[1] = 0u; }
    __syncthreads();
    uint32_t* lists[2] = {list_a, list_b};
    int cur = 0;
    for (int r = 0; r < kShFinishRounds; ++r) {
        const uint32_t n = s_n[cur];
        if (n == 0) return;                               // block-uniform
        const uint32_t* in = lists[cur];
        uint32_t* out = lists[cur ^ 1];
        const unsigned long long tg = tag + (unsigned long long)r;
        for (uint32_t x = t; x < n; x += kShFinishThreads) {
            const uint32_t k = in[x];
            const int64_t d = a.d0 + k;
            const unsigned long long v = (tg << 32) | (unsigned long long)(0xffffffffu - k);
            atomicMax(a.res + (a.total - d), v);
            atomicMax(a.res + a.tgt[d], v);
        }
        __syncthreads();
        for (uint32_t x = t; x < n; x += kShFinishThreads) {
            const uint32_t k = in[x];
            const int64_t d = a.d0 + k;
            const unsigned long long v = (tg << 32) | (unsigned long long)(0xffffffffu - k);
            const int64_t i = a.total - d, j = a.tgt[d];
            const unsigned long long ri = __hip_atomic_load(a.res + i, __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_AGENT);
            const unsigned long long rj = __hip_atomic_load(a.res + j, __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_AGENT);
            if (ri == v && rj == v) {
                const int32_t tmp = a.data[i];
                a.data[i] = a.data[j];
                a.data[j] = tmp;
            } else {
                out[atomicAdd(&s_n[cur ^ 1], 1u)] = k;
            }
        }
        __syncthreads();
        if (t == 0) s_n[cur] = 0u;
        cur ^= 1;
        __syncthreads();
    }
    if (t != 0) return;
    const uint32_t n = s_n[cur];
    uint32_t* list = lists[cur];
    for (uint32_t x = 1; x < n; ++x) {
        const uint32_t key = list[x];
        uint32_t y = x;
        for (; y > 0 && list[y - 1] > key; --y) list[y] = list[y - 1];
        list[y] = key;
    }
    for (uint32_t x = 0; x < n; ++x) {
        const int64_t d = a.d0 + list[x];
        const int64_t i = a.total - d, j = a.tgt[d];
        const int32_t tmp = a.data[i];
        a.data[i] = a.data[j];
        a.data[j] = tmp;
    }
}

}  // namespace mf

using namespace mf;

extern "C" size_t mf_shuffle_swaps_workspace_bytes(int64_t n) {
    (void)n;
    return (size_t)(2 * kShBlockMax + 64) * sizeof(uint32_t);
}

extern "C" int mf_shuffle_swaps_device(const uint32_t* targets, int64_t n, int64_t d_end,
                                       int32_t* data, unsigned long long* reservations,
                                       void* workspace, uint64_t* tag_io, void* stream) {
    const int64_t total = n - 1;
    if (n < 0 || n > ((int64_t)1 << 32) || d_end < 0 || d_end > (total > 0 ? total : 0) ||
        !tag_io || *tag_io == 0 || *tag_io >= (1ull << 31) ||
        (d_end > 0 && (!targets || !data || !reservations || !workspace))) {
        set_error("mf_shuffle_swaps_device: bad arguments");
        return MF_ERR_INVALID;
    }
    hipStream_t s = (hipStream_t)stream;
    // MF_SHUFFLE_GPU_ROUNDS (tests): fewer grid-wide rounds, so that
    // k_sh_finish takes thousands of stragglers
    int rounds = kShRounds;
    if (const char* e = std::getenv("MF_SHUFFLE_GPU_ROUNDS")) rounds = std::max(1, std::min(kShRounds, std::atoi(e)));
    uint32_t* lists[2] = {(uint32_t*)workspace, (uint32_t*)workspace + kShBlockMax};
    uint32_t* counts = (uint32_t*)workspace + 2 * kShBlockMax;     // [2], 64-word aligned
    unsigned long long tag = *tag_io;
    for (int64_t d0 = 0; d0 < d_end;) {
        const int64_t i0 = total - d0;
        const int64_t B = std::max(kShBlockMin, std::min(kShBlockMax, i0 >> 5));
        const int64_t d1 = std::min(d_end, d0 + B);
        ShArgs a{targets, total, d0, d1 - d0, reservations, data};
        const int grid = (int)std::min<int64_t>(kShGridMax, (a.len + kShThreads - 1) / kShThreads);
        for (int r = 0; r < rounds; ++r) {
            const uint32_t* in = r == 0 ? nullptr : lists[r & 1];
            const uint32_t* n_in = r == 0 ? nullptr : counts + (r & 1);
            uint32_t* out = lists[(r + 1) & 1];
            uint32_t* n_out = counts + ((r + 1) & 1);
            hipLaunchKernelGGL(k_sh_reserve, dim3(grid), dim3(kShThreads), 0, s, a, in, n_in, tag,
                               n_out);
            hipLaunchKernelGGL(k_sh_commit, dim3(grid), dim3(kShThreads), 0, s, a, in, n_in, tag,
                               out, n_out);
            ++tag;
        }
        hipLaunchKernelGGL(k_sh_finish, dim3(1), dim3(kShFinishThreads), 0, s, a,
                           lists[rounds & 1], lists[(rounds + 1) & 1], counts + (rounds & 1), tag);
        tag += kShFinishRounds;
        d0 = d1;
    }
    MF_HIP_CHECK(hipGetLastError());
    *tag_io = tag;
    return MF_OK;
}
