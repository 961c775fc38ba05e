// tools/shuffle_probe.cpp -- host timing probe: NumPy-legacy Fisher-Yates (MT19937 draws +
// prefetched swaps, as mf_prep.cpp) on one thread vs draws on a second thread
// feeding the swap thread through a ring; same permutation and MT state.
// Build: g++ -O3 -march=native -std=c++17 -pthread tools/shuffle_probe.cpp -o tools/shuffle_probe
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>
#include <algorithm>
constexpr int kN = 624, kM = 397;
constexpr uint32_t kMatrixA = 0x9908b0dfu, kUpper = 0x80000000u, kLower = 0x7fffffffu;
struct MT {
    uint32_t key[kN]; int pos;
    void seed(uint32_t s){ key[0]=s; for(int i=1;i<kN;i++) key[i]=1812433253u*(key[i-1]^(key[i-1]>>30))+i; pos=kN; }
    void regen() { int i = 0;
        for (; i < kN - kM; ++i) { const uint32_t y = (key[i] & kUpper) | (key[i + 1] & kLower); key[i] = key[i + kM] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA); }
        for (; i < kN - 1; ++i) { const uint32_t y = (key[i] & kUpper) | (key[i + 1] & kLower); key[i] = key[i + (kM - kN)] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA); }
        const uint32_t y = (key[kN - 1] & kUpper) | (key[0] & kLower); key[kN - 1] = key[kM - 1] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA); pos = 0; }
    uint32_t next() { if (pos == kN) regen(); uint32_t y = key[pos++]; y ^= y >> 11; y ^= (y << 7) & 0x9d2c5680u; y ^= (y << 15) & 0xefc60000u; y ^= y >> 18; return y; }
    uint32_t interval(uint32_t max) { if (max == 0) return 0; uint32_t mask = max; mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16; uint32_t v; while ((v = next() & mask) > max) {} return v; }
};
template <typename E> void shuffle_raw(MT& mt, E* data, int64_t n) {
    constexpr int kWin = 64; uint32_t ring[kWin]; int64_t i = n - 1, drawn = n - 1;
    const int64_t pre = std::min<int64_t>(kWin, std::max<int64_t>(n - 1, 0));
    for (int w = 0; w < pre; ++w, --drawn) { const uint32_t j = mt.interval((uint32_t)drawn); ring[drawn % kWin] = j; __builtin_prefetch(data + j, 1, 1); }
    for (; i >= 1; --i) { const int64_t j = ring[i % kWin]; if (drawn >= 1) { const uint32_t jn = mt.interval((uint32_t)drawn); ring[drawn % kWin] = jn; __builtin_prefetch(data + jn, 1, 1); --drawn; }
        const E t = data[i]; data[i] = data[j]; data[j] = t; }
}
// two threads: producer draws swap targets into a ring (blocks of kB), consumer swaps
template <typename E, int PD> void shuffle_2t(MT& mt, E* data, int64_t n) {
    if (n < 2) return;
    constexpr int64_t kB = 1 << 14, kR = 8;             // block size, blocks in the ring
    std::vector<uint32_t> ring(kB * kR);
    std::atomic<int64_t> produced{0};                   // draws produced (count)
    const int64_t total = n - 1;                        // draws for i = n-1 .. 1
    std::atomic<int64_t> consumed{0};
    std::thread prod([&] {
        int64_t d = 0;
        while (d < total) {
            const int64_t blk_end = std::min(total, d + kB);
            while (d + kB - consumed.load(std::memory_order_acquire) > kB * kR) {}  // ring full
            for (; d < blk_end; ++d) ring[d % (kB * kR)] = mt.interval((uint32_t)(n - 1 - d));
            produced.store(d, std::memory_order_release);
        }
    });
    int64_t avail = 0;
    for (int64_t d = 0; d < total; ++d) {
        const int64_t need = std::min(total, d + PD + 1);
        while (avail < need) avail = produced.load(std::memory_order_acquire);
        if (d + PD < total) __builtin_prefetch(data + ring[(d + PD) % (kB * kR)], 1, 1);
        const int64_t i = n - 1 - d;
        const int64_t j = ring[d % (kB * kR)];
        const E t = data[i]; data[i] = data[j]; data[j] = t;
        if ((d & (kB - 1)) == kB - 1) consumed.store(d + 1, std::memory_order_release);
    }
    prod.join();
}
int main() {
    const int64_t n = 100000000;
    std::vector<int32_t> a(n), b(n);
    for (int64_t i = 0; i < n; ++i) a[i] = b[i] = (int32_t)i;
    MT m1, m2; m1.seed(5); m2.seed(5);
    auto t0 = std::chrono::steady_clock::now(); shuffle_raw(m1, a.data(), n);
    auto t1 = std::chrono::steady_clock::now(); shuffle_2t<int32_t, 64>(m2, b.data(), n);
    auto t2 = std::chrono::steady_clock::now();
    printf("1t %.3f s  2t %.3f s  equal %d  mt equal %d\n", std::chrono::duration<double>(t1-t0).count(), std::chrono::duration<double>(t2-t1).count(), (int)(a==b), (int)(m1.pos==m2.pos && !memcmp(m1.key,m2.key,sizeof(m1.key))));
    // MT only time
    MT m3; m3.seed(5); auto t3 = std::chrono::steady_clock::now(); uint64_t s=0; for (int64_t d=0; d<n-1; ++d) s += m3.interval((uint32_t)(n-1-d)); auto t4 = std::chrono::steady_clock::now();
    printf("draws only %.3f s (%llu)\n", std::chrono::duration<double>(t4-t3).count(), (unsigned long long)s);
}
