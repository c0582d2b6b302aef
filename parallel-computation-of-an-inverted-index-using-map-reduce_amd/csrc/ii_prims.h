// ii_prims.h — device-wide primitives for the MI355X inverted-index pipeline:
// exclusive scan and a stable LSD radix sort, both written for wave64 / gfx950.
//
// Both use the "reduce-then-scan" structure with NO inter-workgroup
// communication inside a launch: every workgroup owns one contiguous chunk of
// the input, a first kernel reduces each chunk, a one-workgroup kernel scans
// the per-chunk results, and a third kernel re-reads its chunk and writes.
// Chunks are processed tile by tile in order, so the radix sort is stable.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ii {

constexpr int kBlock = 256;           // threads per workgroup (4 waves)
constexpr int kWaves = kBlock / 64;
constexpr int kMaxChunks = 2048;      // workgroups of a reduce-then-scan launch

// Streaming accesses with the non-temporal hint, where measured to help: the
// histogram reads and the first token-sort pass (records read once; the slot
// -> lexid remap it gathers from should stay in the per-XCD L2s).  The scatter
// and the tokenizer measured slower with it (writes lose L2 combining).
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint64_t ld_nt(const uint64_t* p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void st_nt(uint64_t* p, uint64_t v) { __builtin_nontemporal_store(v, p); }
__device__ __forceinline__ uint4 ld_nt16(const void* p) {
    const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }
__device__ __forceinline__ uint64_t lanemask_lt() {
    return (lane_id() == 0) ? 0ull : (~0ull >> (64 - lane_id()));
}
// set bits of the wave mask m below this lane (v_mbcnt_lo + v_mbcnt_hi)
__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Inclusive wave64 scan of a u64 value.
__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t v) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint64_t t = __shfl_up(v, o, 64);
        if (lane_id() >= o) v += t;
    }
    return v;
}
// Inclusive wave64 scan with DPP (GFX9 row_shr inside the 16-lane rows, then
// row_bcast:15 / :31 across them): six VALU adds instead of six ds_bpermute
// round trips.  A lane whose source lies outside its row (or a row that the
// row mask leaves out) adds the `old` operand, 0.
__device__ __forceinline__ uint32_t wave_incl_scan32(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
    return v;
}
__device__ __forceinline__ uint64_t wave_sum(uint64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Exclusive block scan (256 threads); returns the exclusive prefix and the block total.
__device__ __forceinline__ uint64_t block_excl_scan(uint64_t v, uint64_t* total, uint64_t* lds /*kWaves+1*/) {
    uint64_t inc = wave_incl_scan(v);
    if (lane_id() == 63) lds[wave_id()] = inc;
    __syncthreads();
    uint64_t wbase = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < kWaves; w++) {
        uint64_t s = lds[w];
        if (w < wave_id()) wbase += s;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return wbase + inc - v;
}

// ----------------------------------------------------------------------------
// Device-wide exclusive scan over n items.  Op provides
//   uint64_t value(uint64_t i)                 (the item)
//   void     emit(uint64_t i, uint64_t excl, uint64_t value)
// Items are handled per chunk; per-chunk sums land in `partial`.
// ----------------------------------------------------------------------------
// Both passes keep several items per thread in flight: the reduce sums four
// strided items per iteration (independent loads), the apply gives every
// thread kScanItems consecutive items — a serial prefix in registers and one
// block scan per 2048 items instead of one per 256 (the per-256 form ran the
// dictionary's 5.2 M-slot compaction scan at 0.5 ms, latency-bound).
constexpr int kScanItems = 8;
template <class Op>
__global__ __launch_bounds__(kBlock) void k_scan_reduce(Op op, uint64_t n, uint64_t chunk, uint64_t* partial) {
    __shared__ uint64_t lds[kWaves + 1];
    uint64_t lo = (uint64_t)blockIdx.x * chunk, hi = lo + chunk < n ? lo + chunk : n;
    uint64_t acc = 0;
    uint64_t i = lo + threadIdx.x;
    for (; i + 3 * kBlock < hi; i += 4 * kBlock) {
        const uint64_t a = op.value(i), b = op.value(i + kBlock), c = op.value(i + 2 * kBlock),
                       d = op.value(i + 3 * kBlock);
        acc += (a + b) + (c + d);
    }
    for (; i < hi; i += kBlock) acc += op.value(i);
    acc = wave_sum(acc);
    if (lane_id() == 0) lds[wave_id()] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t = 0;
        for (int w = 0; w < kWaves; w++) t += lds[w];
        partial[blockIdx.x] = t;
    }
}

// One workgroup: exclusive scan of m <= kMaxChunks values in place; total -> *total.
__global__ __launch_bounds__(kBlock) void k_scan_partials(uint64_t* partial, uint32_t m, uint64_t* total) {
    __shared__ uint64_t lds[kWaves + 1];
    constexpr int kPer = kMaxChunks / kBlock;  // 8 values per thread
    uint64_t v[kPer];
    uint64_t s = 0;
#pragma unroll
    for (int j = 0; j < kPer; j++) {
        uint32_t i = threadIdx.x * kPer + j;
        v[j] = i < m ? partial[i] : 0;
        s += v[j];
    }
    uint64_t tot;
    uint64_t ex = block_excl_scan(s, &tot, lds);
#pragma unroll
    for (int j = 0; j < kPer; j++) {
        uint32_t i = threadIdx.x * kPer + j;
        if (i < m) partial[i] = ex;
        ex += v[j];
    }
    if (threadIdx.x == 0 && total) *total = tot;
}

template <class Op>
__global__ __launch_bounds__(kBlock) void k_scan_apply(Op op, uint64_t n, uint64_t chunk, const uint64_t* partial) {
    __shared__ uint64_t lds[kWaves + 1];
    uint64_t lo = (uint64_t)blockIdx.x * chunk, hi = lo + chunk < n ? lo + chunk : n;
    uint64_t run = partial[blockIdx.x];
    for (uint64_t base = lo; base < hi; base += (uint64_t)kBlock * kScanItems) {
        const uint64_t i0 = base + (uint64_t)threadIdx.x * kScanItems;
        uint64_t v[kScanItems];
        uint64_t s = 0;
#pragma unroll
        for (int j = 0; j < kScanItems; j++) {
            v[j] = i0 + j < hi ? op.value(i0 + j) : 0;
            s += v[j];
        }
        uint64_t tot;
        uint64_t ex = run + block_excl_scan(s, &tot, lds);
#pragma unroll
        for (int j = 0; j < kScanItems; j++) {
            if (i0 + j < hi) op.emit(i0 + j, ex, v[j]);
            ex += v[j];
        }
        run += tot;
    }
}

// Small scans in ONE launch (n <= kScanSingleMax): one 1024-thread workgroup,
// 16 consecutive items per thread per round, a running base across rounds;
// *total = the sum.  The three-launch form costs ~20 us of launches and gaps
// whatever n is, which the radix passes over a few 10^5 dictionary keys (one
// table scan each) paid eight times per dictionary.
constexpr int kScanSingleThreads = 1024, kScanSingleItems = 16;
constexpr uint64_t kScanSingleMax = 2ull * kScanSingleThreads * kScanSingleItems;
template <class Op>
__global__ __launch_bounds__(kScanSingleThreads) void k_scan_single(Op op, uint64_t n, uint64_t* total) {
    constexpr int NW = kScanSingleThreads / 64;
    __shared__ uint64_t lds[NW];
    uint64_t run = 0;
    for (uint64_t base = 0; base < n; base += (uint64_t)kScanSingleThreads * kScanSingleItems) {
        const uint64_t i0 = base + (uint64_t)threadIdx.x * kScanSingleItems;
        uint64_t v[kScanSingleItems];
        uint64_t sum = 0;
#pragma unroll
        for (int j = 0; j < kScanSingleItems; j++) {
            v[j] = i0 + j < n ? op.value(i0 + j) : 0;
            sum += v[j];
        }
        const uint64_t inc = wave_incl_scan(sum);
        if (lane_id() == 63) lds[wave_id()] = inc;
        __syncthreads();
        uint64_t wb = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < NW; w++) {
            const uint64_t x = lds[w];
            if (w < wave_id()) wb += x;
            tot += x;
        }
        __syncthreads();
        uint64_t ex = run + wb + inc - sum;
#pragma unroll
        for (int j = 0; j < kScanSingleItems; j++) {
            if (i0 + j < n) op.emit(i0 + j, ex, v[j]);
            ex += v[j];
        }
        run += tot;
    }
    if (threadIdx.x == 0 && total) *total = run;
}

// ----------------------------------------------------------------------------
// Stable LSD radix sort, 8-bit digits.  Keys u64 (digit taken from bits
// [shift, shift+8)), optional u32 payload.  Each pass: histogram per chunk
// (digit-major table), exclusive scan of the table, stable scatter.
// ----------------------------------------------------------------------------
constexpr int kRadixBits = 8;
constexpr int kRadix = 1 << kRadixBits;
constexpr int kMsdMaxBits = 11;                    // the packed sort's top digit: up to 2048 buckets (tbk is u16)
constexpr int kMsdMax = 1 << kMsdMaxBits;
constexpr int kSortItems = 16;                     // keys per thread per tile
constexpr int kSortTile = kBlock * kSortItems;     // 4096 keys per tile
constexpr int kScatterThreads = 512;              // token-sort scatter: tiles of 512 x 16 keys (runs twice as long
constexpr int kScatterItems = 16;                  // as 256 x 16: 2.22 -> 1.95 ms per pass at 10 GB; 1024 x 16 and
                                                   // 512 x 24 were slower)
constexpr int kSweepThreads = 512, kSweepItems = 16;  // onesweep tiles of 8192 keys (512 x 8, 256 x 16: slower —
                                                      // more tiles for every look-back to walk over)
constexpr int kSweepTile = kSweepThreads * kSweepItems;  // keys per onesweep tile

// Per-chunk digit histogram -> table[digit * nchunks + chunk] (digit-major, so
// one exclusive scan of the table yields every chunk's scatter base).  Same
// tile grid and item mapping as the scatter.  K: u64 or u32 keys.
template <class K = uint64_t>
__global__ __launch_bounds__(kBlock) void k_radix_hist(const K* __restrict__ keys, uint64_t n, uint64_t chunk,
                                                       int shift, uint32_t dmask, uint32_t nchunks,
                                                       uint64_t* __restrict__ table) {
    __shared__ uint32_t cnt[kWaves][kRadix];
    for (int i = threadIdx.x; i < kWaves * kRadix; i += kBlock) (&cnt[0][0])[i] = 0;
    __syncthreads();
    const uint64_t lo = (uint64_t)blockIdx.x * chunk, hi = lo + chunk < n ? lo + chunk : n;
    uint32_t* mine = cnt[wave_id()];
    // the histogram ignores order: 16-B loads (kv keys per lane, 1 KiB per wave
    // instruction); lo and the tile are multiples of kv, so a load is split only at hi
    constexpr int kv = 16 / (int)sizeof(K);
    const uint64_t pofs = (uint64_t)wave_id() * 64 * kSortItems + kv * (uint64_t)lane_id();
    for (uint64_t tb = lo; tb < hi; tb += kSortTile) {
        K raw[kSortItems];
#pragma unroll
        for (int k = 0; k < kSortItems / kv; k++) {
            const uint64_t idx = tb + pofs + (uint64_t)k * 64 * kv;
            if (idx + kv - 1 < hi) {
                const uint4 v = ld_nt16(keys + idx);
                if constexpr (sizeof(K) == 8) {
                    raw[2 * k] = (uint64_t)v.x | ((uint64_t)v.y << 32);
                    raw[2 * k + 1] = (uint64_t)v.z | ((uint64_t)v.w << 32);
                } else {
                    raw[4 * k] = v.x; raw[4 * k + 1] = v.y; raw[4 * k + 2] = v.z; raw[4 * k + 3] = v.w;
                }
            } else {
#pragma unroll
                for (int u = 0; u < kv; u++) raw[kv * k + u] = idx + u < hi ? keys[idx + u] : (K)0;
            }
        }
#pragma unroll
        for (int k = 0; k < kSortItems; k++) {
            const uint64_t idx = tb + pofs + (uint64_t)(k / kv) * 64 * kv + k % kv;
            if (idx < hi) atomicAdd(&mine[(uint32_t)(raw[k] >> shift) & dmask], 1u);
        }
    }
    __syncthreads();
    for (int d = threadIdx.x; d < kRadix; d += kBlock) {
        uint32_t t = 0;
#pragma unroll
        for (int w = 0; w < kWaves; w++) t += cnt[w][d];
        table[(uint64_t)d * nchunks + blockIdx.x] = t;
    }
}

// Stable scatter.  Tile layout: thread (wave w, lane l) holds items k at
// tile_base + w*64*kSortItems + k*64 + l, so (w, k, l) order == index order.
// Ranks inside a wave come from a 64-lane match on the digit (8 ballots);
// the tile is reordered by digit in LDS and written out in runs.
// kept (optional): workgroup b reads [kept[kMaxChunks + b], + kept[b]) — the
// compacted ranges k_sort0_compact leaves — instead of [b*chunk, (b+1)*chunk).
// dbits <= kRadixBits: digit width of this pass (fewer buckets -> longer runs
// per tile -> better coalesced stores).
// NT threads per workgroup: a tile holds NT * kSortItems keys, so with
// NT = 512 every digit's output run is twice as long as with 256 (the store
// side is what bounds the pass: 6-bit passes, with twice the run length of
// 7-bit ones, run ~15 % faster).  Threads t < kRadix own one digit each.
// kPack (the MSD pass of the packed token sort, see k_onesweep_seg): the
// record (key << 32 | id) goes out as the u32 (key & pack_low) << pack_f | id
// — the digit (the key's top bits) is implied by the bucket it lands in — and
// digit d's output starts pad[d] records later (buckets padded to whole tiles).
template <bool kHasVals, int NT = kBlock, int IT = kSortItems, bool kPack = false, class K = uint64_t>
__global__ __launch_bounds__(NT) void k_radix_scatter(const K* __restrict__ kin, K* __restrict__ kout,
                                                      const uint32_t* __restrict__ vin, uint32_t* __restrict__ vout,
                                                      uint64_t n, uint64_t chunk, int shift, int dbits,
                                                      uint32_t nchunks, const uint64_t* __restrict__ table,
                                                      const uint64_t* __restrict__ kept, uint32_t* __restrict__ kout32,
                                                      const uint64_t* __restrict__ pad, int pack_f, uint32_t pack_low) {
    constexpr int NW = NT / 64;
    constexpr int kTileN = NT * IT;
    constexpr int kDW = kRadix / 64;  // waves that own digits
    static_assert(NT >= kRadix && NT % 64 == 0, "one digit per thread of the first kRadix threads");
    static_assert(!kPack || sizeof(K) == 8, "the packed MSD scatter reads u64 records");
    __shared__ K s_keys[kTileN];
    __shared__ uint32_t s_vals[kHasVals ? kTileN : 1];
    __shared__ uint32_t s_wcnt[NW][kRadix];
    __shared__ uint32_t s_tstart[kRadix];
    __shared__ uint64_t s_run[kRadix];
    __shared__ uint64_t s_scan[kDW];

    const int w = wave_id(), l = lane_id(), t = threadIdx.x;
    const bool digit_thread = t < kRadix;
    const uint32_t dmask = (1u << dbits) - 1u;
    const uint64_t lo = kept ? kept[kMaxChunks + blockIdx.x] : (uint64_t)blockIdx.x * chunk;
    const uint64_t hi = kept ? lo + kept[blockIdx.x] : (lo + chunk < n ? lo + chunk : n);
    if (digit_thread) s_run[t] = table[(uint64_t)t * nchunks + blockIdx.x] + (kPack ? pad[t] : 0ull);
    const uint64_t lt = lanemask_lt();

    // the next tile's keys are loaded while this tile is ranked and written
    K nkey[IT];
    uint32_t nval[IT];
    auto load_tile = [&](uint64_t tb) {
        const uint64_t wb = tb + (uint64_t)w * 64 * IT + l;
#pragma unroll
        for (int k = 0; k < IT; k++) {
            const uint64_t idx = wb + (uint64_t)k * 64;
            nkey[k] = idx < hi ? kin[idx] : (K)~0ull;
            if (kHasVals) nval[k] = idx < hi ? vin[idx] : 0u;
        }
    };
    if (lo < hi) load_tile(lo);
    uint32_t tot_d = 0;
    for (uint64_t tb = lo; tb < hi; tb += kTileN) {
        if (digit_thread) {
#pragma unroll
            for (int ww = 0; ww < NW; ww++) s_wcnt[ww][t] = 0;
        }
        K key[IT];
        uint32_t val[IT];
        uint32_t rank[IT];
        const uint64_t wbase = tb + (uint64_t)w * 64 * IT + l;
#pragma unroll
        for (int k = 0; k < IT; k++) {
            key[k] = nkey[k];
            if (kHasVals) val[k] = nval[k];
        }
        __syncthreads();
        // ranks inside the wave (one LDS read-modify-write per item; the
        // leader-atomic form of k_onesweep measured slower here: 2.10 -> 2.17
        // ms, its extra registers cost the prefetched tile a wave per SIMD)
#pragma unroll
        for (int k = 0; k < IT; k++) {
            const bool valid = wbase + (uint64_t)k * 64 < hi;
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
            uint32_t r = 0;
            if (valid) {
                const uint32_t before = s_wcnt[w][d];
                r = before + __popcll(m & lt);
                if ((m & lt) == 0) s_wcnt[w][d] = before + __popcll(m);
            }
            rank[k] = r;
        }
        __syncthreads();
        // digit t: totals, tile start, per-wave offsets
        uint32_t cw[NW];
        tot_d = 0;
        if (digit_thread) {
#pragma unroll
            for (int ww = 0; ww < NW; ww++) {
                cw[ww] = s_wcnt[ww][t];
                tot_d += cw[ww];
            }
        }
        const uint32_t inc = wave_incl_scan32(tot_d);  // (a tile holds at most kTileN keys)
        if (w < kDW && l == 63) s_scan[w] = inc;
        __syncthreads();
        uint32_t wb = 0, all = 0;
#pragma unroll
        for (int ww = 0; ww < kDW; ww++) {
            const uint32_t sv = (uint32_t)s_scan[ww];
            if (ww < w) wb += sv;
            all += sv;
        }
        if (digit_thread) {
            uint32_t run = wb + inc - tot_d;
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
            if (wbase + (uint64_t)k * 64 < hi) {
                const uint32_t d = (uint32_t)(key[k] >> shift) & dmask;
                const uint32_t pos = s_wcnt[w][d] + rank[k];
                s_keys[pos] = key[k];
                if (kHasVals) s_vals[pos] = val[k];
            }
        }
        __syncthreads();
        if (tb + kTileN < hi) load_tile(tb + kTileN);  // (issuing them before the ranking measured slower)
        const uint32_t tile_n = (uint32_t)all;
#pragma unroll
        for (int j = 0; j < IT; j++) {
            const uint32_t p = j * NT + t;
            if (p < tile_n) {
                const K k = s_keys[p];
                const uint32_t d = (uint32_t)(k >> shift) & dmask;
                const uint64_t dst = s_run[d] + (p - s_tstart[d]);
                if constexpr (kPack) kout32[dst] = (((uint32_t)((uint64_t)k >> 32) & pack_low) << pack_f) | (uint32_t)k;
                else kout[dst] = k;
                if (kHasVals) vout[dst] = s_vals[p];
            }
        }
        __syncthreads();
        if (digit_thread) s_run[t] += tot_d;
        // the next iteration's first __syncthreads orders this update before use
    }
}

// The packed token sort's MSD scatter in the u32 form: as
// k_radix_scatter<kPack> — workgroup b reads its kept range [kept[kMaxChunks +
// b], + kept[b]), ranks each tile by digit inside each wave (ballots, per-wave
// counts), reorders it in LDS and writes the u32 records low << pack_f | id in
// runs, digit d's run at its scanned table base + pad[d] — with R >= 2^m
// digits spread over the threads (R / NT consecutive digits each; top digits
// up to kMsdMaxBits: configs[4]'s rank-7 share needs m = 10 with 19-bit file
// indices, m = 11 with the 20-bit id0s the first pass writes there) and the tile
// held as the u32 records plus u16 digits, per-wave counts in u16 (a tile
// holds < 2^16 records): 62 / 74 KiB of LDS at R = 512 / 1024 (512 threads x
// 16 records).  R = 2048 (local_reduce: configs[4]'s rank-7 share with id0s
// in the records, m = 11) takes 256 threads x 32 records with u32 run bases
// (kRun32: every position of the padded layout < 2^32), 76 KiB and two
// workgroups per CU, else 512 x 32 with u64 bases, 148 KiB and one: 4.82
// against 5.0 ms, the step 0.4-0.6 ms shorter (profiles/r6zf_msd_scatter_
// two_workgroups_ab.txt; 16 records a thread at 100 KiB: 0.95 ms a step slower,
// non-temporal stores 0.8 ms slower, profiles/r6zb_msd_scatter_2048_ab.txt).
// (Round 4, measured and dropped: the first pass writing the records already
// split — u32 + a u8 top digit, 5 bytes read here instead of 8 — made the
// first pass 0.2 ms slower and this pass no faster at config3.)
template <int NT, int IT, int R, bool kRun32 = false>
__global__ __launch_bounds__(NT) void k_msd_scatter(const uint64_t* __restrict__ kin, uint32_t* __restrict__ kout32,
                                                    int shift, int dbits, uint32_t nchunks,
                                                    const uint64_t* __restrict__ table,
                                                    const uint64_t* __restrict__ kept,
                                                    const uint64_t* __restrict__ pad, int pack_f, uint32_t pack_low) {
    constexpr int NW = NT / 64;
    constexpr int kTileN = NT * IT;
    constexpr int DPT = R / NT > 0 ? R / NT : 1;  // digits per thread (threads t < R own one when R < NT)
    static_assert((R % NT == 0 || NT % R == 0) && kTileN < 65536 && R <= kMsdMax, "u16 tile offsets");
    __shared__ uint32_t s_keys[kTileN];
    __shared__ uint16_t s_dig[kTileN];
    __shared__ uint16_t s_wcnt[NW][R];
    __shared__ uint16_t s_tstart[R];
    using RunT = typename std::conditional<kRun32, uint32_t, uint64_t>::type;  // kRun32: the launcher checked
    __shared__ RunT s_run[R];                                                    // every position < 2^32
    __shared__ uint32_t s_scan[NW];
    const int w = wave_id(), l = lane_id(), t = threadIdx.x;
    const uint32_t ndig = 1u << dbits, dmask = ndig - 1u;
    const uint32_t d0 = (uint32_t)t * DPT;  // this thread's digits [d0, d0 + DPT) (those below ndig)
    const uint64_t lo = kept[kMaxChunks + blockIdx.x], hi = lo + kept[blockIdx.x];
#pragma unroll
    for (int i = 0; i < DPT; i++)
        if (d0 + i < ndig) s_run[d0 + i] = (RunT)(table[(uint64_t)(d0 + i) * nchunks + blockIdx.x] + pad[d0 + i]);
    const uint64_t lt = lanemask_lt();
    uint32_t nrec[IT], ndg[IT];
    auto load_tile = [&](uint64_t tb) {
        const uint64_t wb = tb + (uint64_t)w * 64 * IT + l;
#pragma unroll
        for (int k = 0; k < IT; k++) {
            const uint64_t idx = wb + (uint64_t)k * 64;
            const uint64_t x = idx < hi ? kin[idx] : 0ull;
            nrec[k] = (((uint32_t)(x >> 32) & pack_low) << pack_f) | (uint32_t)x;
            ndg[k] = (uint32_t)(x >> shift) & dmask;
        }
    };
    if (lo < hi) load_tile(lo);
    for (uint64_t tb = lo; tb < hi; tb += kTileN) {
#pragma unroll
        for (int i = 0; i < DPT; i++)
            if (d0 + i < ndig) {
#pragma unroll
                for (int ww = 0; ww < NW; ww++) s_wcnt[ww][d0 + i] = 0;
            }
        uint32_t rec[IT], dg[IT];
#pragma unroll
        for (int k = 0; k < IT; k++) {
            rec[k] = nrec[k];
            dg[k] = ndg[k];
        }
        const uint64_t wbase = tb + (uint64_t)w * 64 * IT + l;
        __syncthreads();
        uint32_t rank[IT];
#pragma unroll
        for (int k = 0; k < IT; k++) {
            const bool valid = wbase + (uint64_t)k * 64 < hi;
            const uint32_t d = dg[k];
            uint64_t m = __ballot(valid);
#pragma unroll
            for (int b = 0; b < kMsdMaxBits; b++) {
                if (b < dbits) {
                    const bool bit = (d >> b) & 1;
                    const uint64_t bb = __ballot(bit);
                    m &= bit ? bb : ~bb;
                }
            }
            uint32_t r = 0;
            if (valid) {
                const uint32_t before = s_wcnt[w][d];
                r = before + __popcll(m & lt);
                if ((m & lt) == 0) s_wcnt[w][d] = (uint16_t)(before + __popcll(m));
            }
            rank[k] = r;
        }
        __syncthreads();
        // this thread's digits: tile totals, then (after the block scan) the tile start and per-wave offsets
        uint32_t tot[DPT], mine = 0;
#pragma unroll
        for (int i = 0; i < DPT; i++) {
            tot[i] = 0;
            if (d0 + i < ndig) {
#pragma unroll
                for (int ww = 0; ww < NW; ww++) tot[i] += s_wcnt[ww][d0 + i];
            }
            mine += tot[i];
        }
        const uint32_t inc = wave_incl_scan32(mine);
        if (l == 63) s_scan[w] = inc;
        __syncthreads();
        uint32_t wb = 0, all = 0;
#pragma unroll
        for (int ww = 0; ww < NW; ww++) {
            const uint32_t sv = s_scan[ww];
            if (ww < w) wb += sv;
            all += sv;
        }
        uint32_t run = wb + inc - mine;
#pragma unroll
        for (int i = 0; i < DPT; i++)
            if (d0 + i < ndig) {
                s_tstart[d0 + i] = (uint16_t)run;
#pragma unroll
                for (int ww = 0; ww < NW; ww++) {
                    const uint32_t c = s_wcnt[ww][d0 + i];
                    s_wcnt[ww][d0 + i] = (uint16_t)run;
                    run += c;
                }
            }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < IT; k++) {
            if (wbase + (uint64_t)k * 64 < hi) {
                const uint32_t pos = s_wcnt[w][dg[k]] + rank[k];
                s_keys[pos] = rec[k];
                s_dig[pos] = (uint16_t)dg[k];
            }
        }
        __syncthreads();
        if (tb + kTileN < hi) load_tile(tb + kTileN);
#pragma unroll
        for (int j = 0; j < IT; j++) {
            const uint32_t p = j * NT + t;
            if (p < all) {
                const uint32_t d = s_dig[p];
                kout32[(uint64_t)s_run[d] + (p - s_tstart[d])] = s_keys[p];
            }
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < DPT; i++)
            if (d0 + i < ndig) s_run[d0 + i] += tot[i];
        // the next iteration's first __syncthreads orders this update before use
    }
}

// ----------------------------------------------------------------------------
// Onesweep scatter pass (decoupled look-back, no histogram pass): the global
// count of every digit is known up front (dbase[d] = exclusive prefix over
// digits, counted while an earlier pass wrote the keys), so a tile only needs
// the number of keys with digit d in all EARLIER tiles.  Tiles are claimed in
// order from a ticket counter (a tile waits only on tiles whose workgroups
// are already running: no deadlock whatever the residency); each tile
// publishes, per digit, its own count (flag A), looks back over earlier
// tiles' entries — summing A counts until it meets an inclusive prefix
// (flag P) — and publishes its inclusive prefix (P).  Every entry is one
// naturally aligned 8-byte granule written by one agent-scope store and read
// by agent-scope loads (cross-XCD visible without fences,
// MI355X_MICROARCH.md "inter-workgroup visibility"):
//   bits 63..40 epoch of the pass (entries of other passes read as "not
//   yet"; no clearing between passes), 39..38 flag, 37..0 count.
// Same tile shape and store runs as k_radix_scatter; the tile is reordered in
// LDS before the look-back, which only the global stores need.
constexpr uint64_t kLbFlagA = 1ull << 38, kLbFlagP = 2ull << 38, kLbValMask = (1ull << 38) - 1;
constexpr unsigned long long kLbTimeout = 8;  // error bit (counters[C_OVERFLOW]) of a look-back that never resolved
// kLbPer: look-back entries per lane per round trip (tools/sort_bench.hip, one
// 7-bit pass over 4.8e8 records: 1 -> 5.7 ms, 2 -> 2.07, 3 -> 2.11, 4 -> 2.18,
// 8 -> 2.50: too few and the walk falls behind, too many and the granule loads
// themselves cost).
// kVals: u32 values ride with the keys (vin -> vout), as k_radix_scatter<true>
// (the dictionary's key / index sorts, run_sort_sweep).
template <int NT, int IT, int kLbPer = 2, bool kVals = false>
__global__ __launch_bounds__(NT) void k_onesweep(const uint64_t* __restrict__ kin, uint64_t* __restrict__ kout,
                                                 uint64_t n, int shift, int dbits, const uint64_t* __restrict__ dbase,
                                                 uint64_t* __restrict__ status, uint32_t* __restrict__ ticket,
                                                 uint64_t epoch, unsigned long long* __restrict__ err,
                                                 const uint32_t* __restrict__ vin, uint32_t* __restrict__ vout) {
    constexpr int NW = NT / 64;
    constexpr int kTileN = NT * IT;
    constexpr int kDW = kRadix / 64;
    static_assert(NT >= kRadix && NT % 64 == 0, "one digit per thread of the first kRadix threads");
    __shared__ uint64_t s_keys[kTileN];
    __shared__ uint32_t s_vals[kVals ? kTileN : 1];
    __shared__ uint32_t s_wcnt[NW][kRadix];
    __shared__ uint32_t s_tstart[kRadix];
    __shared__ uint64_t s_run[kRadix];
    __shared__ uint64_t s_scan[kDW];
    __shared__ uint32_t s_tot[kRadix];
    __shared__ uint32_t s_tile;

    const int w = wave_id(), l = lane_id(), t = threadIdx.x;
    const uint32_t ndig = 1u << dbits, dmask = ndig - 1u;
    const bool digit_thread = t < (int)ndig;
    if (t == 0) s_tile = atomicAdd(ticket, 1u);
    if (t < kRadix) {
#pragma unroll
        for (int ww = 0; ww < NW; ww++) s_wcnt[ww][t] = 0;
    }
    __syncthreads();
    const uint64_t tile = s_tile;
    const uint64_t tb = tile * kTileN;
    const uint64_t lt = lanemask_lt();
    const uint64_t wbase = tb + (uint64_t)w * 64 * IT + l;
    uint64_t key[IT];
    uint32_t val[kVals ? IT : 1];
#pragma unroll
    for (int k = 0; k < IT; k++) {
        const uint64_t idx = wbase + (uint64_t)k * 64;
        key[k] = idx < n ? kin[idx] : ~0ull;
        if (kVals) val[k] = idx < n ? vin[idx] : 0u;
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
    uint32_t rank[IT];
#pragma unroll
    for (int k = 0; k < IT; k++)
        rank[k] = (uint32_t)__shfl((int)before[k], (int)((info[k] >> 16) & 63u), 64) + (info[k] & 0xFFu);
    __syncthreads();
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
            if (kVals) s_vals[s_wcnt[w][d] + rank[k]] = val[k];
        }
    }
    // look-back: sum the earlier tiles' counts of each digit until an
    // inclusive prefix (flag P).  Four lanes per digit, each loading the
    // entries of kLbPer different earlier tiles per round trip: a quad passes
    // over 4 * kLbPer tiles per round trip.  (At one tile per lane the walk
    // advanced about as fast as new tiles started, so every tile walked far.)
    const uint32_t gj = t & 3;  // place of this lane in its quad
    for (uint32_t gd = t >> 2; gd < ndig; gd += NT / 4) {  // the quad's digit; control flow is quad-uniform
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
    __syncthreads();
    const uint32_t tile_n = (uint32_t)all;
#pragma unroll
    for (int j = 0; j < IT; j++) {
        const uint32_t p = j * NT + t;
        if (p < tile_n) {
            const uint64_t k = s_keys[p];
            const uint32_t d = (uint32_t)(k >> shift) & dmask;
            kout[s_run[d] + (p - s_tstart[d])] = k;
            if (kVals) vout[s_run[d] + (p - s_tstart[d])] = s_vals[p];
        }
    }
}

// Digit counts of every LSD pass of a sort in one read of the keys: pass p's
// digit is the key's bits [lo + p * bits, min(lo + (p + 1) * bits, hi)), counts[p * kRadix + d]
// (zeroed beforehand); per-workgroup LDS counters, then one global atomic per
// non-zero counter.  (run_sort_sweep: the onesweep passes need only these.)
constexpr int kHistMaxPasses = 8;
__global__ __launch_bounds__(kBlock) void k_hist_passes(const uint64_t* __restrict__ keys, uint64_t n, int lo, int hi,
                                                        int bits, int npass, uint64_t* __restrict__ counts) {
    __shared__ uint32_t h[kHistMaxPasses][kRadix];
    for (int i = threadIdx.x; i < kHistMaxPasses * kRadix; i += kBlock) (&h[0][0])[i] = 0;
    __syncthreads();
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock) {
        const uint64_t k = keys[i];
        for (int p = 0; p < npass; p++) {  // (the last pass's digit may be narrower: hi - its shift bits)
            const int sh = lo + p * bits, db = bits < hi - sh ? bits : hi - sh;
            atomicAdd(&h[p][(uint32_t)(k >> sh) & ((1u << db) - 1u)], 1u);
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < npass * kRadix; i += kBlock) {
        const uint32_t v = (&h[0][0])[i];
        if (v) atomicAdd((unsigned long long*)&counts[i], (unsigned long long)v);
    }
}

// ----------------------------------------------------------------------------
// Packed token sort (MSD bucket, then LSD inside the buckets, u32 records).
// The token records are key << 32 | id with a key of W bits and ids of F bits;
// when W - m + F <= 32 for an m-bit top digit, the first scatter partitions
// the records by the key's top m bits (k_radix_scatter<kPack>) into buckets
// padded to whole onesweep tiles and writes each as the u32
// low << F | id (low = the key's other W - m bits): the bucket implies the top
// digit.  The remaining digits are sorted inside each bucket by onesweep passes
// over the u32 records (k_onesweep_seg): a tile lies in one bucket and looks
// back only over its bucket's tiles.  K3 (k_uniq_sweep<true>) reads the
// sorted u32 records in the same padded layout and writes the u64 pairs.
// Against three u64 passes and a u64 K3 read this moves 36 instead of 56
// bytes per record (8 + 4 scatter, 4 histogram, 4 + 4, 4 + 4, K3 read 4).
//
// Bucket geometry (one workgroup): bstart[h] = dense start of bucket h (the
// exclusive scan of the MSD scatter's digit-major table, column 0) and
// bstart[nb] = the total; btile[h] = its first tile in the padded layout
// (btile[nb] = all tiles); pad[h] = btile[h] * tile - bstart[h].
__global__ __launch_bounds__(kRadix) void k_msd_geometry(const uint64_t* __restrict__ table, uint32_t nchunks,
                                                         uint32_t nb, const uint64_t* __restrict__ total, uint32_t tile,
                                                         uint64_t* __restrict__ bstart, uint32_t* __restrict__ btile,
                                                         uint64_t* __restrict__ pad) {
    __shared__ uint64_t lds[kRadix / 64 + 1];
    const uint64_t tot = *total;
    uint64_t carry = 0;  // tiles of the buckets before this round's
    for (uint32_t hb = 0; hb < nb; hb += kRadix) {  // (nb > kRadix: the wide top digits)
        const uint32_t h = hb + threadIdx.x;
        const uint64_t s = h < nb ? table[(uint64_t)h * nchunks] : tot;
        const uint64_t e = h + 1 < nb ? table[(uint64_t)(h + 1) * nchunks] : tot;
        const uint64_t nt = h < nb ? (e - s + tile - 1) / tile : 0;
        const uint64_t inc = wave_incl_scan(nt);
        if (lane_id() == 63) lds[wave_id()] = inc;
        __syncthreads();
        uint64_t base = 0, all = 0;
        for (int w = 0; w < kRadix / 64; w++) {
            if (w < wave_id()) base += lds[w];
            all += lds[w];
        }
        const uint64_t t0 = carry + base + inc - nt;
        if (h < nb) {
            bstart[h] = s;
            btile[h] = (uint32_t)t0;
            pad[h] = t0 * tile - s;
        }
        carry += all;
        __syncthreads();  // (lds is rewritten by the next round)
    }
    if (threadIdx.x == 0) {
        bstart[nb] = tot;
        btile[nb] = (uint32_t)carry;
    }
}

// tbk[tile] = the bucket of every tile of the padded layout (one workgroup
// per bucket), so that a tile finds its bucket with one load.
__global__ __launch_bounds__(kBlock) void k_tile_buckets(const uint32_t* __restrict__ btile, uint16_t* __restrict__ tbk) {
    const uint32_t h = blockIdx.x;
    for (uint32_t i = btile[h] + threadIdx.x; i < btile[h + 1]; i += kBlock) tbk[i] = (uint16_t)h;
}

// Per-bucket counts of the two LSD digits of the packed records:
// gh[(2 h + j) * kRadix + d] += records of bucket h whose digit j is d (digit j
// = bits [s_j, s_j + b_j) of the u32).  A workgroup counts tiles
// [blockIdx.x * per, + per) of the padded layout, 16-B loads (4 records a lane),
// and adds its counts to gh whenever its tiles enter a new bucket.
template <int NT, int IT>
__global__ __launch_bounds__(NT) void k_seg_hist(const uint32_t* __restrict__ rec, const uint32_t* __restrict__ btile,
                                                 const uint64_t* __restrict__ bstart, uint32_t nb, uint32_t per, int s0,
                                                 int b0, int s1, int b1, uint64_t* __restrict__ gh) {
    constexpr uint32_t kTileN = NT * IT;
    static_assert(IT % 4 == 0, "16-B loads");
    // four copies of each histogram, lane l adds to copy l % 4 (row stride kRadix + 1: a digit's four
    // copies sit in four banks), so lanes of one wave instruction that share a digit split four ways:
    // a bucket ruled by a few frequent words (configs[4]'s rank-7 share, one record per file of its
    // most frequent words) sent most lanes to one counter, and same-address LDS atomics serialise
    // (8 conflict cycles per LDS instruction there, 3 at config3): the rank-7 sort 29.7 -> 26.5 ms,
    // config3 unchanged; grouping equal digits by ballots first (three leader rounds) instead cost
    // config3 0.7 ms and saved rank 7 1.2 (profiles/r4m_seg_hist_ab.txt)
    constexpr int kCopies = 4;
    constexpr int kStride = kRadix + 1;
    __shared__ uint32_t c0s[kCopies * kStride], c1s[kCopies * kStride];
    uint32_t* c0 = c0s;
    uint32_t* c1 = c1s;
    const uint32_t t = threadIdx.x;
    const uint32_t m0 = (1u << b0) - 1u, m1 = (1u << b1) - 1u;
    const uint32_t all = btile[nb];
    uint32_t tile = blockIdx.x * per;
    const uint32_t tend = tile + per < all ? tile + per : all;
    if (tile >= tend) return;
    for (uint32_t i = t; i < kCopies * kStride; i += NT) c0[i] = c1[i] = 0;
    const uint32_t cofs = (lane_id() & 3u) * kStride;
    // bucket of the first tile: the last h with btile[h] <= tile (empty buckets share a start)
    uint32_t lo = 0, hi = nb - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) / 2;
        if (btile[mid] <= tile) lo = mid;
        else hi = mid - 1;
    }
    uint32_t h = lo;
    auto flush = [&]() {
        __syncthreads();
        for (uint32_t d = t; d < kRadix; d += NT) {
            uint32_t a0 = 0, a1 = 0;
#pragma unroll
            for (int cp = 0; cp < kCopies; cp++) {
                a0 += c0[cp * kStride + d];
                a1 += c1[cp * kStride + d];
                c0[cp * kStride + d] = c1[cp * kStride + d] = 0;
            }
            if (a0) atomicAdd((unsigned long long*)&gh[(2ull * h) * kRadix + d], (unsigned long long)a0);
            if (a1) atomicAdd((unsigned long long*)&gh[(2ull * h + 1) * kRadix + d], (unsigned long long)a1);
        }
        __syncthreads();
    };
    __syncthreads();
    for (; tile < tend; tile++) {
        if (tile >= btile[h + 1]) {  // (workgroup-uniform) the tiles entered a later bucket
            flush();
            while (tile >= btile[h + 1]) h++;
        }
        const uint64_t tb = (uint64_t)tile * kTileN;
        const uint64_t vend = (uint64_t)btile[h] * kTileN + (bstart[h + 1] - bstart[h]);
#pragma unroll
        for (int k = 0; k < IT / 4; k++) {
            const uint64_t idx = tb + 4ull * ((uint64_t)k * NT + t);
            uint4 v = make_uint4(0u, 0u, 0u, 0u);
            if (idx < vend) v = *reinterpret_cast<const uint4*>(rec + idx);
            const uint32_t r[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int q = 0; q < 4; q++) {
                if (idx + q < vend) {
                    atomicAdd(&c0[cofs + ((r[q] >> s0) & m0)], 1u);
                    atomicAdd(&c1[cofs + ((r[q] >> s1) & m1)], 1u);
                }
            }
        }
    }
    flush();
}

// One LSD pass inside the buckets of the packed layout (k_onesweep's
// decoupled look-back, per bucket): tile = ticket; its bucket h (btile); the
// records [btile[h] * tile, + count of h) are valid; the look-back stops at
// the bucket's first tile, which publishes an inclusive prefix at once.
// Digit d of bucket h starts at the bucket's padded start + dbase[h * dstride + d].
// (kLbPer: look-back granules per lane, 8 tiles per round trip per digit; 1 or
// 4 measured no faster in round 4, at config3 or on the rank-7 share whose
// buckets span ~190 tiles.)
// (launch bound of 6 waves per SIMD: without one the compiler spent 256 VGPRs
// with spills, one workgroup per CU, 2.4x slower than k_onesweep.  Round 4,
// dropped: a workgroup claiming two tiles and loading both up front — its
// second tile publishes only after the first is written, and the look-backs
// behind it wait in a chain: 1.6 -> 115 ms per pass.)
template <int NT, int IT, int kLbPer = 2>
__global__ __launch_bounds__(NT, 6) void k_onesweep_seg(const uint32_t* __restrict__ kin, uint64_t ncap,
                                                     uint32_t* __restrict__ kout,
                                                     const uint32_t* __restrict__ btile,
                                                     const uint16_t* __restrict__ tbk,
                                                     const uint64_t* __restrict__ bstart, uint32_t nb, int shift,
                                                     int dbits, const uint64_t* __restrict__ dbase, uint32_t dstride,
                                                     uint64_t* __restrict__ status,
                                                     uint32_t* __restrict__ ticket, uint64_t epoch,
                                                     unsigned long long* __restrict__ err) {
    constexpr int NW = NT / 64;
    constexpr int kTileN = NT * IT;
    constexpr int kDW = kRadix / 64;
    static_assert(NT >= kRadix && NT % 64 == 0, "one digit per thread of the first kRadix threads");
    __shared__ uint32_t s_keys[kTileN];
    __shared__ uint32_t s_wcnt[NW][kRadix];
    __shared__ uint32_t s_tstart[kRadix];
    __shared__ uint64_t s_run[kRadix];
    __shared__ uint64_t s_scan[kDW];
    __shared__ uint32_t s_tot[kRadix];
    __shared__ uint32_t s_tile;

    const int w = wave_id(), l = lane_id(), t = threadIdx.x;
    const uint32_t ndig = 1u << dbits, dmask = ndig - 1u;
    const bool digit_thread = t < (int)ndig;
    if (t == 0) s_tile = atomicAdd(ticket, 1u);
    if (t < kRadix) {
#pragma unroll
        for (int ww = 0; ww < NW; ww++) s_wcnt[ww][t] = 0;
    }
    __syncthreads();
    // the tile read with readfirstlane: wave-uniform (scalar), so the bucket's bounds and every
    // per-item bound compare stay in SGPRs (read from LDS they spilled 256 VGPRs)
    const uint64_t tile = (uint32_t)__builtin_amdgcn_readfirstlane(s_tile);
    const uint64_t tb = tile * kTileN;
    const uint64_t lt = lanemask_lt();
    const uint64_t wbase = tb + (uint64_t)w * 64 * IT + l;
    // the keys first (their addresses do not depend on the bucket; ncap bounds the padded layout's
    // allocation), the bucket's bounds while they are in flight
    uint32_t key[IT];
#pragma unroll
    for (int k = 0; k < IT; k++) {
        const uint64_t idx = wbase + (uint64_t)k * 64;
        key[k] = idx < ncap ? kin[idx] : ~0u;
    }
    if (tile >= btile[nb]) return;  // (workgroup-uniform) a spare workgroup of the launch's upper bound
    const uint32_t h = tbk[tile];
    const uint64_t tile0 = btile[h];
    const uint64_t vend = tile0 * kTileN + (bstart[h + 1] - bstart[h]);
    // the tile's valid records [0, vrel) in 32-bit tile-relative indices
    const uint32_t vrel = vend <= tb ? 0u : vend - tb < (uint64_t)kTileN ? (uint32_t)(vend - tb) : (uint32_t)kTileN;
    const uint32_t wrel = (uint32_t)w * 64 * IT + (uint32_t)l;
#pragma unroll
    for (int k = 0; k < IT; k++)
        if (wrel + (uint32_t)k * 64 >= vrel) key[k] = ~0u;
    uint32_t info[IT];  // as k_onesweep: rank in the item's group | group size << 8 | leader lane << 16
#pragma unroll
    for (int k = 0; k < IT; k++) {
        const bool valid = wrel + (uint32_t)k * 64 < vrel;
        const uint32_t d = (key[k] >> shift) & dmask;
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
        uint32_t before = 0;
        if ((info[k] & 0xFFu) == 0u) before = atomicAdd(&s_wcnt[w][d], (info[k] >> 8) & 0xFFu);
        info[k] = (uint32_t)__shfl((int)before, (int)((info[k] >> 16) & 63u), 64) + (info[k] & 0xFFu);  // -> rank
    }
    const uint32_t* rank = info;
    __syncthreads();
    uint32_t tot_d = 0;  // (the per-wave counts are read again below: held in registers they spilled)
    if (t < kRadix) {
#pragma unroll
        for (int ww = 0; ww < NW; ww++) tot_d += s_wcnt[ww][t];
    }
    const uint64_t ep = epoch << 40;
    if (digit_thread) {
        s_tot[t] = tot_d;
        __hip_atomic_store(status + tile * kRadix + t, ep | (tile == tile0 ? kLbFlagP : kLbFlagA) | tot_d,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const uint32_t inc = wave_incl_scan32(tot_d);  // (a tile holds at most kTileN records)
    if (w < kDW && l == 63) s_scan[w] = inc;
    __syncthreads();
    uint32_t wb = 0, all = 0;
#pragma unroll
    for (int ww = 0; ww < kDW; ww++) {
        const uint32_t sv = (uint32_t)s_scan[ww];
        if (ww < w) wb += sv;
        all += sv;
    }
    if (t < kRadix) {
        uint32_t run = wb + inc - tot_d;
        s_tstart[t] = run;
#pragma unroll
        for (int ww = 0; ww < NW; ww++) {
            const uint32_t cnt = s_wcnt[ww][t];
            s_wcnt[ww][t] = run;
            run += cnt;
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < IT; k++) {
        if (wrel + (uint32_t)k * 64 < vrel) s_keys[s_wcnt[w][(key[k] >> shift) & dmask] + rank[k]] = key[k];
    }
    // look-back over the bucket's earlier tiles (k_onesweep's quads of lanes)
    const uint64_t obase = tile0 * kTileN;
    const uint32_t gj = t & 3;
    for (uint32_t gd = t >> 2; gd < ndig; gd += NT / 4) {
        uint64_t excl = 0;
        for (int64_t base = (int64_t)tile - 1; base >= (int64_t)tile0; base -= 4 * kLbPer) {
            uint64_t v[kLbPer];
#pragma unroll
            for (int u = 0; u < kLbPer; u++) {
                const int64_t p = base - (int64_t)(4 * u + gj);
                v[u] = p >= (int64_t)tile0 ? __hip_atomic_load(status + (uint64_t)p * kRadix + gd, __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_AGENT)
                                           : ep | kLbFlagP;  // before the bucket's first tile: a prefix of 0
            }
#pragma unroll
            for (int u = 0; u < kLbPer; u++) {
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
            if (tile != tile0)
                __hip_atomic_store(status + tile * kRadix + gd, ep | kLbFlagP | (excl + s_tot[gd]), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            s_run[gd] = obase + dbase[(uint64_t)h * dstride + gd] + excl;
        }
    }
    __syncthreads();
    const uint32_t tile_n = (uint32_t)all;
#pragma unroll
    for (int j = 0; j < IT; j++) {
        const uint32_t p = j * NT + t;
        if (p < tile_n) {
            const uint32_t k = s_keys[p];
            kout[s_run[(k >> shift) & dmask] + (p - s_tstart[(k >> shift) & dmask])] = k;
        }
    }
}

// dbase[r * kRadix + d] = exclusive prefix over digits of dhist[r * kRadix + d]
// (one workgroup per row).
__global__ __launch_bounds__(kRadix) void k_digit_bases(const uint64_t* __restrict__ dhist, uint64_t* __restrict__ dbase) {
    __shared__ uint64_t lds[kRadix / 64 + 1];
    const uint64_t v = dhist[blockIdx.x * kRadix + threadIdx.x];
    const uint64_t inc = wave_incl_scan(v);
    if (lane_id() == 63) lds[wave_id()] = inc;
    __syncthreads();
    uint64_t base = 0;
    for (int w = 0; w < wave_id(); w++) base += lds[w];
    dbase[blockIdx.x * kRadix + threadIdx.x] = base + inc - v;
}

}  // namespace ii
