// sort_bench.hip — timing experiment for the token-sort scatter passes (not
// product code).  On N synthetic records shaped like the kept token records
// at the 10 GB config (key = word id << 32 | file id0, file ids ascending,
// word ids Zipf-like over 2^20), times:
//   copy      read + write of the N records (the pass's streaming floor)
//   onesweep  one k_onesweep pass over a 7-bit digit (as the product runs it)
//   rocprim   rocprim::radix_sort_keys over the same 7 bits, and over 20 bits
// Usage: sort_bench [N]
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <type_traits>
#include <vector>

#include <rocprim/device/device_radix_sort.hpp>

#include "../csrc/ii_prims.h"
using namespace ii;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__device__ uint64_t mixk(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
__global__ void k_fill(uint64_t* k, uint64_t n, uint32_t files) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const double u = (double)(mixk(i) >> 11) * (1.0 / 9007199254740992.0);
        const uint32_t rank = (uint32_t)exp(u * log(800000.0));                  // ~1/x over [1, 8e5)
        const uint32_t wid = (uint32_t)(mixk(rank * 0x9E3779B97F4A7C15ull) & 0xFFFFFu);  // hot slot of that word
        k[i] = ((uint64_t)wid << 32) | (uint32_t)(i * files / n);
    }
}
__global__ void k_copy(const uint4* __restrict__ a, uint4* __restrict__ b, uint64_t n16) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x)
        b[i] = a[i];
}
// copy with 4 x 16 B per lane in flight, nontemporal both ways
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_copy4(const u32x4* __restrict__ a, u32x4* __restrict__ b, uint64_t n16) {
    const uint64_t stride = (uint64_t)gridDim.x * 256 * 4;
    for (uint64_t base = (uint64_t)blockIdx.x * 256 * 4 + threadIdx.x; base < n16; base += stride) {
        u32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) if (base + u * 256 < n16) v[u] = __builtin_nontemporal_load(a + base + u * 256);
#pragma unroll
        for (int u = 0; u < 4; u++) if (base + u * 256 < n16) __builtin_nontemporal_store(v[u], b + base + u * 256);
    }
}
__global__ void k_dhist(const uint64_t* __restrict__ k, uint64_t n, int shift, uint32_t dmask, uint64_t* h) {
    __shared__ uint32_t c[kRadix];
    for (int i = threadIdx.x; i < kRadix; i += blockDim.x) c[i] = 0;
    __syncthreads();
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        atomicAdd(&c[(uint32_t)(k[i] >> shift) & dmask], 1u);
    __syncthreads();
    for (int i = threadIdx.x; i < kRadix; i += blockDim.x)
        if (c[i]) atomicAdd((unsigned long long*)&h[i], (unsigned long long)c[i]);
}
__global__ void k_check_sorted(const uint64_t* __restrict__ k, uint64_t n, int shift, uint32_t dmask, unsigned long long* bad) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x + 1; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t a = (uint32_t)(k[i - 1] >> shift) & dmask, b = (uint32_t)(k[i] >> shift) & dmask;
        if (a > b || (a == b && (uint32_t)k[i - 1] > (uint32_t)k[i])) atomicAdd(bad, 1ull);
    }
}

template <int NT, int IT, int kLbPer = 2>
__global__ __launch_bounds__(NT) void k_sweep_stamp(const uint64_t* __restrict__ kin, uint64_t* __restrict__ kout,
                                                 uint64_t n, int shift, int dbits, const uint64_t* __restrict__ dbase,
                                                 uint64_t* __restrict__ status, uint32_t* __restrict__ ticket,
                                                 uint64_t epoch, unsigned long long* __restrict__ err, uint64_t* __restrict__ stamp, int abl) {
    constexpr int NW = NT / 64;
    constexpr int kTileN = NT * IT;
    constexpr int kDW = kRadix / 64;
    static_assert(NT >= kRadix && NT % 64 == 0, "one digit per thread of the first kRadix threads");
    __shared__ uint64_t s_keys[kTileN];
    __shared__ uint32_t s_wcnt[NW][kRadix];
    __shared__ uint32_t s_tstart[kRadix];
    __shared__ uint64_t s_run[kRadix];
    __shared__ uint64_t s_scan[kDW];
    __shared__ uint32_t s_tot[kRadix];
    __shared__ uint32_t s_tile;

    const int w = wave_id(), l = lane_id(), t = threadIdx.x;
    const uint32_t ndig = 1u << dbits, dmask = ndig - 1u;
    const bool digit_thread = t < (int)ndig;
    const uint64_t st0 = __builtin_amdgcn_s_memtime();
    if (t == 0) s_tile = atomicAdd(ticket, 1u);
    if (t < kRadix) {
#pragma unroll
        for (int ww = 0; ww < NW; ww++) s_wcnt[ww][t] = 0;
    }
    __syncthreads();
    const uint64_t tile = s_tile;
    const uint64_t st0b = __builtin_amdgcn_s_memtime();
    const uint64_t tb = tile * kTileN;
    const uint64_t lt = lanemask_lt();
    const uint64_t wbase = tb + (uint64_t)w * 64 * IT + l;
    uint64_t key[IT];
#pragma unroll
    for (int k = 0; k < IT; k++) {
        const uint64_t idx = wbase + (uint64_t)k * 64;
        key[k] = idx < n ? kin[idx] : ~0ull;
    }
    // ranks inside the wave: per item, the lanes sharing a digit (ballots on
    // its bits); the lowest of them adds the group's size to the wave's digit
    // counter (LDS atomic with return) and the others take the old count from
    // it — the items' atomics are independent, so they pipeline in the LDS
    // unit instead of one read-modify-write round trip per item
    uint32_t info[IT];  // rank inside the item's group | group size << 8 | leader lane << 16
#pragma unroll
    for (int k = 0; k < IT; k++) {
        const bool valid = wbase + (uint64_t)k * 64 < n;
        const uint32_t d = (uint32_t)(key[k] >> shift) & dmask;
        uint64_t m = __ballot(valid);
#pragma unroll
        for (int b = 0; b < kRadixBits; b++) {
            if (b < dbits) {
                const bool bit = (d >> b) & 1;
                const uint64_t bb = __ballot(bit);
                m &= bit ? bb : ~bb;
            }
        }
        info[k] = valid ? (uint32_t)__popcll(m & lt) | ((uint32_t)__popcll(m) << 8) | ((uint32_t)__builtin_ctzll(m) << 16)
                        : 0xFFFFFFFFu;
    }
    uint32_t before[IT];
#pragma unroll
    for (int k = 0; k < IT; k++) {
        before[k] = 0;
        if ((info[k] & 0xFFu) == 0u)  // group leader (invalid lanes carry 0xFF)
            before[k] = atomicAdd(&s_wcnt[w][(uint32_t)(key[k] >> shift) & dmask], (info[k] >> 8) & 0xFFu);
    }
    uint64_t st1 = 0;
    {
        uint64_t x = 0;
#pragma unroll
        for (int kk = 0; kk < IT; kk++) x ^= key[kk];
        if (x == 0x1234567ull) err[1] = x;
        st1 = __builtin_amdgcn_s_memtime();
    }
    uint32_t rank[IT];
#pragma unroll
    for (int k = 0; k < IT; k++)
        rank[k] = (uint32_t)__shfl((int)before[k], (int)((info[k] >> 16) & 63u), 64) + (info[k] & 0xFFu);
    __syncthreads();
    const uint64_t st2 = __builtin_amdgcn_s_memtime();
    uint32_t cw[NW];
    uint32_t tot_d = 0;
    if (t < kRadix) {
#pragma unroll
        for (int ww = 0; ww < NW; ww++) {
            cw[ww] = s_wcnt[ww][t];
            tot_d += cw[ww];
        }
    }
    // publish this tile's digit counts at once (flag A), so that later tiles
    // can pass over it while it still reorders
    const uint64_t ep = epoch << 40;
    if (digit_thread) {
        s_tot[t] = tot_d;
        __hip_atomic_store(status + tile * kRadix + t, ep | (tile == 0 ? kLbFlagP : kLbFlagA) | tot_d,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // digit t: tile start, per-wave offsets (as k_radix_scatter); the tile is
    // reordered by digit in LDS before the look-back, which it does not need
    const uint64_t inc = wave_incl_scan(tot_d);
    if (w < kDW && l == 63) s_scan[w] = inc;
    __syncthreads();
    uint64_t wb = 0, all = 0;
#pragma unroll
    for (int ww = 0; ww < kDW; ww++) {
        const uint64_t sv = s_scan[ww];
        if (ww < w) wb += sv;
        all += sv;
    }
    if (t < kRadix) {
        uint32_t run = (uint32_t)(wb + inc - tot_d);
        s_tstart[t] = run;
#pragma unroll
        for (int ww = 0; ww < NW; ww++) {
            s_wcnt[ww][t] = run;
            run += cw[ww];
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < IT; k++) {
        if (wbase + (uint64_t)k * 64 < n) {
            const uint32_t d = (uint32_t)(key[k] >> shift) & dmask;
            s_keys[s_wcnt[w][d] + rank[k]] = key[k];
        }
    }
    __syncthreads();
    const uint64_t st3 = __builtin_amdgcn_s_memtime();
    // look-back: sum the earlier tiles' counts of each digit until an
    // inclusive prefix (flag P).  Four lanes per digit, each loading the
    // entries of kLbPer different earlier tiles per round trip: a quad passes
    // over 4 * kLbPer tiles per round trip.  (At one tile per lane the walk
    // advanced about as fast as new tiles started, so every tile walked far.)
    const uint32_t gj = t & 3;  // place of this lane in its quad
    for (uint32_t gd = t >> 2; gd < ndig && !(abl & 2); gd += NT / 4) {  // the quad's digit; control flow is quad-uniform
        uint64_t excl = 0;
        for (int64_t base = (int64_t)tile - 1; base >= 0; base -= 4 * kLbPer) {
            uint64_t v[kLbPer];
#pragma unroll
            for (int u = 0; u < kLbPer; u++) {  // entry of tile base - (4 u + gj): distance 4 u + gj
                const int64_t p = base - (int64_t)(4 * u + gj);
                v[u] = p >= 0 ? __hip_atomic_load(status + (uint64_t)p * kRadix + gd, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT)
                              : ep | kLbFlagP;  // before tile 0: an inclusive prefix of 0
            }
#pragma unroll
            for (int u = 0; u < kLbPer; u++) {
                // tile p has not published yet (its workgroup is running); a wait of seconds means a
                // broken hand-off: flag it and let the launch drain rather than spin forever
                const int64_t p = base - (int64_t)(4 * u + gj);
                for (uint32_t spin = 0; (v[u] >> 40) != epoch; spin++) {
                    if (spin == (1u << 24)) {
                        atomicOr(err, kLbTimeout);
                        v[u] = ep | kLbFlagP;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                    v[u] = __hip_atomic_load(status + (uint64_t)p * kRadix + gd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            // the nearest inclusive prefix among the quad's tiles ends the walk
            uint32_t q = 0;
#pragma unroll
            for (int u = 0; u < kLbPer; u++)
                q |= ((uint32_t)(__ballot((v[u] & kLbFlagP) != 0) >> (lane_id() & ~3)) & 0xFu) << (4 * u);
            const uint32_t upto = q ? (uint32_t)__builtin_ctz(q) : 4u * kLbPer - 1u;
            uint64_t add = 0;
#pragma unroll
            for (int u = 0; u < kLbPer; u++)
                if (4u * u + gj <= upto) add += v[u] & kLbValMask;
            add += (uint64_t)__shfl_xor((long long)add, 1, 64);
            add += (uint64_t)__shfl_xor((long long)add, 2, 64);
            excl += add;
            if (q) break;
        }
        if (gj == 0) {
            if (tile != 0)
                __hip_atomic_store(status + tile * kRadix + gd, ep | kLbFlagP | (excl + s_tot[gd]), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            s_run[gd] = dbase[gd] + excl;
        }
    }
    if ((abl & 2) && t < (int)ndig) s_run[t] = dbase[t] + tile * s_tot[t];
    __syncthreads();
    const uint64_t st4 = __builtin_amdgcn_s_memtime();
    const uint32_t tile_n = (uint32_t)all;
#pragma unroll
    for (int j = 0; j < IT; j++) {
        const uint32_t p = j * NT + t;
        if (p < tile_n) {
            const uint64_t k = s_keys[p];
            const uint32_t d = (uint32_t)(k >> shift) & dmask;
            if (!(abl & 1)) kout[s_run[d] + (p - s_tstart[d])] = k;
        }
    }
    const uint64_t st5 = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    const uint64_t st6 = __builtin_amdgcn_s_memtime();
    if (t == 0) {
        uint64_t* o = stamp + tile * 8;
        o[0] = st0; o[1] = st1; o[7] = st0b; o[2] = st2; o[3] = st3; o[4] = st4; o[5] = st5; o[6] = st6;
    }
}
template <class F>
float time_best(F f, int reps = 5) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float best = 1e30f;
    for (int r = 0; r < reps; r++) {
        CK(hipEventRecord(a));
        f();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
    }
    return best;
}

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 478000000ull;
    const double gb = 16.0 * n / 1e9;  // read + write per pass
    uint64_t *a, *b, *h, *dbase, *status;
    uint32_t* ticket;
    unsigned long long* err;
    CK(hipMalloc(&a, n * 8));
    CK(hipMalloc(&b, n * 8));
    CK(hipMalloc(&h, kRadix * 8));
    CK(hipMalloc(&dbase, kRadix * 8));
    CK(hipMalloc(&err, 8));
    const uint64_t ntiles = (n + kSweepTile - 1) / kSweepTile;
    const uint64_t maxtiles = (n + 2047) / 2048;
    CK(hipMalloc(&status, maxtiles * kRadix * 8));
    CK(hipMalloc(&ticket, 4));
    CK(hipMemset(status, 0, maxtiles * kRadix * 8));
    CK(hipMemset(err, 0, 8));
    k_fill<<<4096, 256>>>(a, n, 10000);
    CK(hipDeviceSynchronize());

    const float t_copy = time_best([&] { k_copy<<<8192, 256>>>((const uint4*)a, (uint4*)b, n / 2); });
    printf("copy      %7.3f ms  %6.2f TB/s\n", t_copy, gb / t_copy);

    for (int g : {1024, 2048, 4096}) {
        const float t4 = time_best([&] { k_copy4<<<g, 256>>>((const u32x4*)a, (u32x4*)b, n / 2); });
        printf("copy4 nt grid %5d %7.3f ms  %6.2f TB/s\n", g, t4, gb / t4);
    }
    const int shift = 32, dbits = 7;
    CK(hipMemset(h, 0, kRadix * 8));
    k_dhist<<<2048, 256>>>(a, n, shift, (1u << dbits) - 1, h);
    k_digit_bases<<<1, kRadix>>>(h, dbase);
    uint64_t epoch = 0;
    const float t_sweep = time_best([&] {
        epoch++;
        CK(hipMemsetAsync(ticket, 0, 4));
        k_onesweep<kSweepThreads, kSweepItems><<<(unsigned)ntiles, kSweepThreads>>>(a, b, n, shift, dbits, dbase, status,
                                                                                     ticket, epoch, err, nullptr, nullptr);
    });
    unsigned long long* bad;
    CK(hipMalloc(&bad, 8));
    auto shape = [&](auto per) {
        constexpr int NT = kSweepThreads, IT = kSweepItems, PER = decltype(per)::value;
        const uint64_t nt_tiles = (n + NT * IT - 1) / (NT * IT);
        const float tt = time_best([&] {
            epoch++;
            CK(hipMemsetAsync(ticket, 0, 4));
            k_onesweep<NT, IT, PER><<<(unsigned)nt_tiles, NT>>>(a, b, n, shift, dbits, dbase, status, ticket, epoch, err,
                                                                 nullptr, nullptr);
        });
        printf("onesweep lookback %2d per lane %7.3f ms  %6.2f TB/s\n", PER, tt, gb / tt);
    };
    {   // reduce-then-scan scatter (the first token-sort pass): chunk histograms, host scan, scatter
        const uint32_t nchunks = kMaxChunks;
        const uint64_t tile = kScatterThreads * kScatterItems;
        const uint64_t chunk = ((n + nchunks - 1) / nchunks + tile - 1) / tile * tile;
        const uint32_t nch = (uint32_t)((n + chunk - 1) / chunk);
        uint64_t* table;
        CK(hipMalloc(&table, sizeof(uint64_t) * kRadix * nch));
        CK(hipMemset(table, 0, sizeof(uint64_t) * kRadix * nch));
        k_radix_hist<<<nch, kBlock>>>(a, n, chunk, shift, (1u << dbits) - 1, nch, table);
        std::vector<uint64_t> ht((size_t)kRadix * nch);
        CK(hipMemcpy(ht.data(), table, ht.size() * 8, hipMemcpyDeviceToHost));
        uint64_t run = 0;
        for (auto& v : ht) { const uint64_t c = v; v = run; run += c; }
        CK(hipMemcpy(table, ht.data(), ht.size() * 8, hipMemcpyHostToDevice));
        const float ts = time_best([&] {
            k_radix_scatter<false, kScatterThreads, kScatterItems><<<nch, kScatterThreads>>>(
                a, b, nullptr, nullptr, n, chunk, shift, dbits, nch, table, nullptr, nullptr, nullptr, 0, 0u);
        });
        CK(hipMemset(bad, 0, 8));
        k_check_sorted<<<4096, 256>>>(b, n, shift, (1u << dbits) - 1, bad);
        unsigned long long hb = 0;
        CK(hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost));
        printf("scatter (table) %7.3f ms  %6.2f TB/s (unsorted %llu)\n", ts, gb / ts, hb);
    }
    CK(hipMemset(bad, 0, 8));
    k_check_sorted<<<4096, 256>>>(b, n, shift, (1u << dbits) - 1, bad);
    unsigned long long hbad = 0, herr = 0;
    CK(hipMemcpy(&hbad, bad, 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&herr, err, 8, hipMemcpyDeviceToHost));
    printf("onesweep  %7.3f ms  %6.2f TB/s  (unsorted pairs %llu, err %llu)\n", t_sweep, gb / t_sweep, hbad, herr);

    for (int abl = 0; abl < 2; abl++) {
        uint64_t* stamp;
        CK(hipMalloc(&stamp, ntiles * 64));
        CK(hipMemset(stamp, 0, ntiles * 64));
        epoch++;
        CK(hipMemsetAsync(ticket, 0, 4));
        k_sweep_stamp<kSweepThreads, kSweepItems><<<(unsigned)ntiles, kSweepThreads>>>(a, b, n, shift, dbits, dbase, status,
                                                                                        ticket, epoch, err, stamp, abl);
        CK(hipDeviceSynchronize());
        uint64_t* hs = (uint64_t*)malloc(ntiles * 64);
        CK(hipMemcpy(hs, stamp, ntiles * 64, hipMemcpyDeviceToHost));
        double ph[6] = {0}, tk = 0;
        uint64_t tmin = ~0ull, tmax = 0;
        for (uint64_t i = 0; i < ntiles; i++) {
            for (int j = 0; j < 6; j++) ph[j] += (double)(hs[i * 8 + j + 1] - hs[i * 8 + j]);
            tk += (double)(hs[i * 8 + 7] - hs[i * 8]);
            if (hs[i * 8] < tmin) tmin = hs[i * 8];
            if (hs[i * 8 + 6] > tmax) tmax = hs[i * 8 + 6];
        }
        printf("stamped sweep abl %d: span %.0f ticks; per tile (ticks): load %.0f rank %.0f reorder %.0f lookback %.0f "
               "store-issue %.0f store-drain %.0f\n", abl, (double)(tmax - tmin), ph[0] / ntiles, ph[1] / ntiles, ph[2] / ntiles,
               ph[3] / ntiles, ph[4] / ntiles, ph[5] / ntiles);
        printf("  of the load phase, ticket + barrier: %.0f\n", tk / ntiles);
        // tiles per time decile, to see ramp / tail
        for (int q = 0; q < 10; q++) {
            uint64_t c = 0;
            for (uint64_t i = 0; i < ntiles; i++) {
                const double f = (double)(hs[i * 8] - tmin) / (double)(tmax - tmin);
                if (f >= q / 10.0 && f < (q + 1) / 10.0) c++;
            }
            printf("  decile %d: %llu tiles started\n", q, (unsigned long long)c);
        }
    }
    size_t tmp_bytes = 0;
    CK(rocprim::radix_sort_keys(nullptr, tmp_bytes, a, b, (size_t)n, 32, 39));
    size_t tmp2 = 0;
    CK(rocprim::radix_sort_keys(nullptr, tmp2, a, b, (size_t)n, 32, 52));
    if (tmp2 > tmp_bytes) tmp_bytes = tmp2;
    void* tmp;
    CK(hipMalloc(&tmp, tmp_bytes));
    const float t_rp7 = time_best([&] { CK(rocprim::radix_sort_keys(tmp, tmp_bytes, a, b, (size_t)n, 32, 39)); });
    printf("rocprim7  %7.3f ms  %6.2f TB/s (one 7-bit pass incl. its histogram)\n", t_rp7, gb / t_rp7);
    const float t_rp20 = time_best([&] { CK(rocprim::radix_sort_keys(tmp, tmp_bytes, a, b, (size_t)n, 32, 52)); });
    printf("rocprim20 %7.3f ms  (20-bit key)\n", t_rp20);
    return 0;
}
