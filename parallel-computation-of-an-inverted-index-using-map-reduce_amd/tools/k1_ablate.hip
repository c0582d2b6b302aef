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
#include <algorithm>
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
// (B = 0: no load at all)
template <int B>
struct RegionProbe {
    __device__ __forceinline__ ProbeState begin(const Table& t, bool fast, uint64_t, uint32_t home) const {
        ProbeState st{make_ulonglong2(0ull, 0ull), home};
        if (B && fast) st.qa = *reinterpret_cast<const ulonglong2*>(t.keys + (home & ((1u << (B ? B : 1)) - 2u)));
        return st;
    }
    __device__ __forceinline__ uint32_t finish(const Table&, const ProbeState& st, bool fast, uint64_t key,
                                              uint64_t) const {
        if (!fast) return kSlotNone;
        return st.qa.x == key + 1 ? kSlotNone : st.home;  // (never equal in practice: keeps the load)
    }
};
// A small direct-mapped cache in front of HotProbe: (key, slot) of the most frequent hot words
// (found by counting a previous run's records, tools only), 2^B entries of 16 B; a miss takes HotProbe.
// What a sampling pre-pass could buy: the share of tokens served by an L1 / L2-resident table.
__device__ const ulonglong2* g_small = nullptr;
__host__ __device__ __forceinline__ uint32_t small_hash(uint64_t key) {
    uint32_t h = (uint32_t)(key >> 32) * 0x9E3779B1u ^ (uint32_t)key * 0x85EBCA77u;
    return h ^ (h >> 15);
}
template <int B>
struct SmallProbe {
    __device__ __forceinline__ ProbeState begin(const Table& t, bool fast, uint64_t key, uint32_t home) const {
        ProbeState st{make_ulonglong2(0ull, 0ull), home};
        if (fast) st.qa = g_small[small_hash(key) & ((1u << B) - 1u)];
        return st;
    }
    __device__ __forceinline__ uint32_t finish(const Table& t, const ProbeState& st, bool fast, uint64_t key,
                                              uint64_t pos) const {
        if (fast && st.qa.x == key) return (uint32_t)st.qa.y;
        const bool miss = fast && st.qa.x != key;
        return HotProbe().finish(t, HotProbe().begin(t, miss, key, st.home), miss, key, pos);
    }
};

__global__ void k_slot_hist(const uint64_t* __restrict__ rec, uint64_t n, uint32_t* __restrict__ cnt) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t s = rec[i] >> 32;
        if (s < kHotSlots) atomicAdd(&cnt[s], 1u);
    }
}

template <class Probe>
__global__ __launch_bounds__(kBlock, 8) void k_emit_variant(const uint8_t* __restrict__ text, uint64_t nbytes, uint64_t nch,
                                                         const uint64_t* __restrict__ file_start,
                                                         uint64_t* __restrict__ chunk_off, uint64_t cap, Table tab,
                                                         uint64_t* __restrict__ rec, uint32_t* __restrict__ chunk_hist,
                                                         uint32_t* __restrict__ pend, uint32_t* __restrict__ pend_cnt,
                                                         const uint32_t* __restrict__ cf, LongTok* __restrict__ longs,
                                                         uint64_t long_per, uint32_t narrow_keys) {
    __shared__ __attribute__((aligned(16))) EmitLds s_lds[kWG];
    const uint64_t c = wave_chunk();
    if (c < nch)
        tok_emit_chunk<Probe>(text, nbytes, nch, file_start, chunk_off, cap, tab, rec, chunk_hist, pend, pend_cnt, cf,
                              longs, long_per, narrow_keys, 32u - 23u /* the 2^20 + 2^22 slots of main() */, c,
                              s_lds[c - (uint64_t)blockIdx.x * kWG]);
}

template <class Probe>
float run(const uint8_t* d_text, uint64_t nb, uint64_t* fstart, uint32_t* fid, uint32_t nf, uint64_t* chunk_off,
          Table tab, uint64_t nslots, uint64_t* rec, uint32_t* chist, LongTok* longs, uint64_t lcap, uint64_t nch,
          uint32_t* pend, uint32_t* pcnt, bool warm = false) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    uint32_t* cf;
    const uint32_t wg = (uint32_t)((nch + kWG - 1) / kWG);
    CK(hipMalloc(&cf, 12 * nch));
    k_chunk_files<<<(uint32_t)((nch + kBlock - 1) / kBlock), kBlock>>>(fstart, nf, nb, kChunk, nch, cf);
    float best = 1e9;
    for (int it = 0; it < 4; it++) {
        if (!warm) CK(hipMemset(tab.keys, 0, nslots * 8));  // warm: the words of earlier runs stay
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
    Table tab{keys, rep, big - 1, 0x51ed270b27a3f3c1ull, counters, ~0ull};
#define RUNW(A, name, warm) do { float e_ = run<A>(d_text, nb, fstart, fid, p.nfiles, chunk, tab, nslots, rec, chist, longs, lcap, nch, pend, pcnt, warm); \
    unsigned long long np_ = 0; std::vector<uint32_t> pc_(nch); CK(hipMemcpy(pc_.data(), pcnt, 4 * nch, hipMemcpyDeviceToHost)); \
    for (auto x : pc_) np_ += (x & 0xFFFFu) + (x >> 16); \
    printf("emit %-30s: %.3f ms  pending %llu\n", name, e_, np_); } while (0)
#define RUN(A, name) RUNW(A, name, false)
    printf("bytes %llu tokens %llu count %.3f ms\n", (unsigned long long)nb, (unsigned long long)T, ms_count);
    RUN(HotProbe, "full (HotProbe)");
    // small front tables of the most frequent hot words (counted from the records of a warm run)
    RUNW(HotProbe, "HotProbe, warm table", true);
    {
        uint32_t* d_cnt;
        CK(hipMalloc(&d_cnt, 4 * kHotSlots));
        CK(hipMemset(d_cnt, 0, 4 * kHotSlots));
        k_slot_hist<<<4096, 256>>>(rec, T, d_cnt);
        std::vector<uint32_t> hc(kHotSlots);
        std::vector<unsigned long long> hk(kHotSlots);
        CK(hipMemcpy(hc.data(), d_cnt, 4 * kHotSlots, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hk.data(), keys, 8 * kHotSlots, hipMemcpyDeviceToHost));
        std::vector<uint32_t> order(kHotSlots);
        for (uint32_t i = 0; i < kHotSlots; i++) order[i] = i;
        std::sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) { return hc[x] > hc[y]; });
        ulonglong2* d_small;
        CK(hipMalloc(&d_small, 16ull << 14));
        for (int B = 11; B <= 14; B++) {
            std::vector<ulonglong2> tbl(1u << B, make_ulonglong2(0ull, 0ull));
            uint64_t served = 0;
            for (uint32_t j = 0; j < (1u << B) && hc[order[j]]; j++) {  // most frequent first; a taken entry keeps its word
                const uint32_t sl = order[j];
                ulonglong2& e = tbl[small_hash(hk[sl]) & ((1u << B) - 1u)];
                if (e.x == 0ull) { e = make_ulonglong2(hk[sl], sl); served += hc[sl]; }
            }
            CK(hipMemcpy(d_small, tbl.data(), 16ull << B, hipMemcpyHostToDevice));
            CK(hipMemcpyToSymbol(HIP_SYMBOL(g_small), &d_small, sizeof(d_small)));
            printf("small table 2^%d entries (%u KB): %.1f %% of tokens\n", B, 16u << B >> 10, 100.0 * served / T);
            if (B == 11) RUNW(SmallProbe<11>, "small 2^11 + HotProbe, warm", true);
            if (B == 12) RUNW(SmallProbe<12>, "small 2^12 + HotProbe, warm", true);
            if (B == 13) RUNW(SmallProbe<13>, "small 2^13 + HotProbe, warm", true);
            if (B == 14) RUNW(SmallProbe<14>, "small 2^14 + HotProbe, warm", true);
        }
        RUNW(HotProbe, "HotProbe, warm table again", true);
    }
    RUN(RegionProbe<0>, "no probe");
    RUN(RegionProbe<12>, "probe 32 KB region");
    RUN(RegionProbe<17>, "probe 1 MB region");
    RUN(RegionProbe<18>, "probe 2 MB region");
    RUN(RegionProbe<20>, "probe 8 MB region");
    printf("count (best of 5): %.3f ms\n", best_of([&] { k_tok_count<<<wg, kBlock>>>(d_text, nb, nch, chunk); }));
    printf("read-only (best of 5): %.3f ms\n", best_of([&] { k_read_only<<<wg, kBlock>>>(d_text, nb, nch, chunk); }));
    return 0;
}
