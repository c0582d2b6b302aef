// k1_ablate.hip — timing experiment for the K1 emit kernel (not product code).
// Times the K1b kernel body (tok_emit_chunk, ii_kernels.h) with other probe
// policies on one synthetic Zipf corpus: the product's HotProbe; no probe (the
// slot is the home slot, no load); a probe of the same shape confined to a
// region of 2^b slots (2^b * 8 bytes: the cost of the probe instruction when
// its lines stay in L1 / L2); and k_tok_count and a read-only pass.
// Usage: k1_ablate [bytes] [files] [vocab]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include "../csrc/ii_kernels.h"
using namespace ii;

typedef struct { uint64_t total_bytes; uint32_t nfiles, vocab; uint64_t seed; double size_sigma; } iigen_params;
extern "C" int iigen_layout(const iigen_params*, uint64_t*);
extern "C" int iigen_fill(const iigen_params*, const uint64_t*, uint8_t*, int);

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

// read-only reference: the count kernel's access pattern (one wave per
// chunk, 16 B per lane, 8 loads in flight), XOR of the words
__global__ __launch_bounds__(kBlock) void k_read_only(const uint8_t* __restrict__ text, uint64_t nbytes, uint64_t nch,
                                                      uint64_t* out) {
    const uint64_t c = wave_chunk();
    const uint64_t lo = c * kChunk;
    uint32_t x = 0;
    if (c < nch && lo + kChunk <= nbytes) {
        for (int jb = 0; jb < (int)(kChunk / 1024); jb += 8) {
            uint4 v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) v[u] = *reinterpret_cast<const uint4*>(text + lo + 16 * (64ull * (jb + u) + lane_id()));
#pragma unroll
            for (int u = 0; u < 8; u++) x ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
        }
    }
    if (x == 0x12345678u) out[c] = x;
}

template <class F>
float best_of(F f) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    float best = 1e9;
    for (int it = 0; it < 5; it++) {
        CK(hipEventRecord(a)); f(); CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b)); if (ms < best) best = ms;
    }
    return best;
}

// probe of the same shape as HotProbe's first load, confined to 2^B slots; the slot is the home slot
template <int B>
struct RegionProbe {
    __device__ __forceinline__ uint32_t operator()(const Table& t, bool fast, uint64_t key, uint32_t home, uint64_t) const {
        if (!fast) return kSlotNone;
        if (B == 0) return home;
        const ulonglong2 q = *reinterpret_cast<const ulonglong2*>(t.keys + (home & ((1u << B) - 2u)));
        return q.x == key + 1 ? kSlotNone : home;  // (never equal in practice: keeps the load)
    }
};
// HotProbe with the bucket's first NP slot pairs (in probe order) loaded at once: one round trip
template <int NP>
struct WideProbe {
    __device__ __forceinline__ uint32_t operator()(const Table& t, bool fast, uint64_t key, uint32_t home,
                                                   uint64_t pos) const {
        if (!fast) return kSlotNone;
        const uint32_t bbase = home & ~(uint32_t)(kBucket - 1), start = home & (kBucket - 2);
        ulonglong2 q[NP];
#pragma unroll
        for (int j = 0; j < NP; j++)
            q[j] = *reinterpret_cast<const ulonglong2*>(t.keys + bbase + ((start + 2 * j) & (kBucket - 2)));
        uint32_t match = 0, empty = 0;
#pragma unroll
        for (int j = 0; j < NP; j++) {
            match |= ((uint32_t)(q[j].x == key) << (2 * j)) | ((uint32_t)(q[j].y == key) << (2 * j + 1));
            empty |= ((uint32_t)(q[j].x == 0ull) << (2 * j)) | ((uint32_t)(q[j].y == 0ull) << (2 * j + 1));
        }
        return bucket_resolve(t, match, empty, key, bbase, start, pos);
    }
};

// the home slot's pair only: a word found there, or claimed there (kClaim), resolves; every other
// token goes to the K1c tail (no second round trip in the rounds)
template <bool kClaim>
struct PairProbe {
    __device__ __forceinline__ uint32_t operator()(const Table& t, bool fast, uint64_t key, uint32_t home,
                                                   uint64_t pos) const {
        if (!fast) return kSlotNone;
        const uint32_t bbase = home & ~(uint32_t)(kBucket - 1), start = home & (kBucket - 2);
        const ulonglong2 q = *reinterpret_cast<const ulonglong2*>(t.keys + bbase + start);
        const uint32_t match = (uint32_t)(q.x == key) | ((uint32_t)(q.y == key) << 1);
        const uint32_t empty = (uint32_t)(q.x == 0ull) | ((uint32_t)(q.y == 0ull) << 1);
        if (!kClaim && !match) return kSlotNone;
        return bucket_resolve(t, match, empty, key, bbase, start, pos);
    }
};

// HotProbe whose claims do not wait: a word found in the two pairs resolves; a word whose pairs have
// an empty slot claims the first one with a CAS whose result nobody waits for, and goes to the K1c
// tail (table_find finds it there, or places it where the CAS lost)
struct LazyProbe {
    __device__ __forceinline__ uint32_t operator()(const Table& t, bool fast, uint64_t key, uint32_t home,
                                                   uint64_t pos) const {
        const uint32_t bbase = home & ~(uint32_t)(kBucket - 1), start = home & (kBucket - 2);
        ulonglong2 qa = make_ulonglong2(1ull, 1ull), qb = make_ulonglong2(1ull, 1ull);
        if (fast) qa = *reinterpret_cast<const ulonglong2*>(t.keys + bbase + start);
        uint32_t match = (uint32_t)(qa.x == key) | ((uint32_t)(qa.y == key) << 1);
        uint32_t empty = (uint32_t)(qa.x == 0ull) | ((uint32_t)(qa.y == 0ull) << 1);
        if (fast && !(match | empty)) {
            qb = *reinterpret_cast<const ulonglong2*>(t.keys + bbase + ((start + 2) & (kBucket - 2)));
            match |= ((uint32_t)(qb.x == key) << 2) | ((uint32_t)(qb.y == key) << 3);
            empty |= ((uint32_t)(qb.x == 0ull) << 2) | ((uint32_t)(qb.y == 0ull) << 3);
        }
        if (!fast) return kSlotNone;
        if (match) return bbase + ((start + __builtin_ctz(match)) & (kBucket - 1));
        if (empty) atomicCAS(&t.keys[bbase + ((start + __builtin_ctz(empty)) & (kBucket - 1))], 0ull,
                             (unsigned long long)key);
        return kSlotNone;
    }
};

template <class Probe>
__global__ __launch_bounds__(kBlock, 8) void k_emit_variant(const uint8_t* __restrict__ text, uint64_t nbytes, uint64_t nch,
                                                         const uint64_t* __restrict__ file_start,
                                                         uint64_t* __restrict__ chunk_off, uint64_t cap, Table tab,
                                                         uint64_t* __restrict__ rec, uint32_t* __restrict__ chunk_hist,
                                                         uint32_t* __restrict__ pend, uint32_t* __restrict__ pend_cnt,
                                                         const uint32_t* __restrict__ cf, LongTok* __restrict__ longs,
                                                         uint64_t long_per, uint32_t narrow_keys) {
    __shared__ __attribute__((aligned(16))) EmitLds s_lds[kWG];
    tok_emit_chunk<Probe>(text, nbytes, nch, file_start, chunk_off, cap, tab, rec, chunk_hist, pend, pend_cnt, cf, longs,
                          long_per, narrow_keys, s_lds);
}

template <class Probe>
float run(const uint8_t* d_text, uint64_t nb, uint64_t* fstart, uint32_t* fid, uint32_t nf, uint64_t* chunk_off,
          Table tab, uint64_t nslots, uint64_t* rec, uint32_t* chist, LongTok* longs, uint64_t lcap, uint64_t nch,
          uint32_t* pend, uint32_t* pcnt) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    uint32_t* cf;
    const uint32_t wg = (uint32_t)((nch + kWG - 1) / kWG);
    CK(hipMalloc(&cf, 12 * nch));
    k_chunk_files<<<(uint32_t)((nch + kBlock - 1) / kBlock), kBlock>>>(fstart, nf, nb, kChunk, nch, cf);
    float best = 1e9;
    for (int it = 0; it < 4; it++) {
        CK(hipMemset(tab.keys, 0, nslots * 8));
        CK(hipMemset(tab.counters, 0, 8 * C_NUM));
        CK(hipEventRecord(a));
        k_emit_variant<Probe><<<wg, kBlock>>>(d_text, nb, nch, fstart, chunk_off, 0, tab, rec, chist, pend, pcnt, cf,
                                              longs, lcap / kLongShards, (uint32_t)kNarrowKeys);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
    }
    return best;
}

int main(int argc, char** argv) {
    iigen_params p = {argc > 1 ? strtoull(argv[1], 0, 10) : 1000000000ull, argc > 2 ? (uint32_t)atoi(argv[2]) : 1000u,
                      argc > 3 ? (uint32_t)atoi(argv[3]) : 1000000u, 3, 1.0};
    std::vector<uint64_t> off(p.nfiles + 1);
    std::vector<uint8_t> text(p.total_bytes + 16);
    iigen_layout(&p, off.data());
    iigen_fill(&p, off.data(), text.data(), 16);
    const uint64_t nb = p.total_bytes, nch = (nb + kChunk - 1) / kChunk;
    uint8_t* d_text; uint64_t *fstart, *chunk, *rec, *counters; uint32_t *fid, *chist; LongTok* longs;
    unsigned long long* keys; uint64_t* rep;
    const uint64_t big = 1ull << 22, nslots = kHotSlots + big, lcap = 1ull << 24;
    CK(hipMalloc(&d_text, nb + 64)); CK(hipMemcpy(d_text, text.data(), nb, hipMemcpyHostToDevice));
    std::vector<uint32_t> ids(p.nfiles);
    for (uint32_t i = 0; i < p.nfiles; i++) ids[i] = i;
    CK(hipMalloc(&fstart, 8 * p.nfiles)); CK(hipMemcpy(fstart, off.data(), 8 * p.nfiles, hipMemcpyHostToDevice));
    CK(hipMalloc(&fid, 4 * p.nfiles)); CK(hipMemcpy(fid, ids.data(), 4 * p.nfiles, hipMemcpyHostToDevice));
    CK(hipMalloc(&chunk, 8 * (nch + 1))); CK(hipMalloc(&chist, 4 * 26 * nch)); CK(hipMalloc(&counters, 8 * C_NUM));
    CK(hipMalloc(&keys, 8 * nslots)); CK(hipMalloc(&rep, 8 * nslots)); CK(hipMalloc(&longs, sizeof(LongTok) * lcap));
    // count pass -> offsets (host scan)
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    CK(hipEventRecord(a));
    const uint32_t wg = (uint32_t)((nch + kWG - 1) / kWG);
    k_tok_count<<<wg, kBlock>>>(d_text, nb, nch, chunk);
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms_count; CK(hipEventElapsedTime(&ms_count, a, b));
    std::vector<uint64_t> cnt(nch + 1);
    CK(hipMemcpy(cnt.data(), chunk, 8 * nch, hipMemcpyDeviceToHost));
    uint64_t T = 0;
    for (uint64_t c = 0; c < nch; c++) { uint64_t x = cnt[c]; cnt[c] = T; T += x; }
    cnt[nch] = T;  // chunk_off[c + 1] bounds chunk c's pending list (dense layout)
    CK(hipMemcpy(chunk, cnt.data(), 8 * (nch + 1), hipMemcpyHostToDevice));
    CK(hipMalloc(&rec, 8 * T));
    uint32_t *pend, *pcnt;
    CK(hipMalloc(&pend, 4 * T)); CK(hipMalloc(&pcnt, 4 * nch));
    Table tab{keys, rep, big - 1, 0x51ed270b27a3f3c1ull, counters};
#define RUN(A, name) do { float e_ = run<A>(d_text, nb, fstart, fid, p.nfiles, chunk, tab, nslots, rec, chist, longs, lcap, nch, pend, pcnt); \
    unsigned long long np_ = 0; std::vector<uint32_t> pc_(nch); CK(hipMemcpy(pc_.data(), pcnt, 4 * nch, hipMemcpyDeviceToHost)); \
    for (auto x : pc_) np_ += (x & 0xFFFFu) + (x >> 16); \
    printf("emit %-22s: %.3f ms  pending %llu\n", name, e_, np_); } while (0)
    printf("bytes %llu tokens %llu count %.3f ms\n", (unsigned long long)nb, (unsigned long long)T, ms_count);
    RUN(HotProbe, "full (HotProbe)");
    RUN(LazyProbe, "claims without waiting");
    RUN(HotProbe, "full (HotProbe) again");
    RUN(LazyProbe, "claims without waiting again");
    RUN(RegionProbe<0>, "no probe");
    RUN(RegionProbe<12>, "probe 32 KB region");
    RUN(RegionProbe<17>, "probe 1 MB region");
    RUN(RegionProbe<18>, "probe 2 MB region");
    RUN(RegionProbe<20>, "probe 8 MB region");
    printf("count (best of 5): %.3f ms\n", best_of([&] { k_tok_count<<<wg, kBlock>>>(d_text, nb, nch, chunk); }));
    printf("read-only (best of 5): %.3f ms\n", best_of([&] { k_read_only<<<wg, kBlock>>>(d_text, nb, nch, chunk); }));
    return 0;
}
