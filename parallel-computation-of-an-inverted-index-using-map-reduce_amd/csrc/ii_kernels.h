// ii_kernels.h — the inverted-index kernels (K1..K5) for MI355X (gfx950).
//
// Reference path replaced (see DESIGN.md for the full map):
//   K1 k_tok_count/k_tok_emit  mapper() hot loop, main.c:102-118, + partial
//                      files main.c:116 (records, word table, letter counts)
//   Kd dictionary      (no reference equivalent: gives every distinct word a
//                      lexicographic id so that the reducer's strcmp order,
//                      main.c:63, becomes integer order)
//   K2 token sort      the reducer's dictionary scan main.c:170-187 (radix sort
//                      in ii_prims.h)
//   K3 k_unique_*      fileID dedup + add_number, main.c:176-184, 67-77
//   K4 final order     qsort by (df desc, word asc), main.c:55-64, 215
//   K5 k_fmt_*         writer, main.c:227-234 (IDs ascending: main.c:217-226)
#pragma once
#include <type_traits>

#include "ii_prims.h"

namespace ii {

// ---------------------------------------------------------------- constants
// bytes of text per K1 chunk (one wave each, see "K1 chunks"); 32 KiB against 16: K1b 11.68-11.74 ->
// 11.61-11.63 ms at config3 (half the chunks' fixed costs: file bounds, the K1c tail, the histogram
// write), configs[4]'s rank 7 unchanged; 8 KiB: 12.1 ms (profiles/r6zp_chunk_size_ab.txt)
constexpr uint64_t kChunk = 32768;
constexpr int kMaxWord = 299;      // MAX_WORD - 1 letters (main.c:7, 105)
constexpr int kMaxProbe = 1 << 12;  // big-table probe bound (load <= 1/2 enforced by the host): past it, C_OVERFLOW

constexpr uint32_t kSlotNone = 0xFFFFFFFFu;  // token with no letters (dropped, main.c:113)

// counters[] layout (u64)
enum : int {
    C_LONG = 0,      // long tokens appended
    C_OVERFLOW = 1,  // word table probe limit hit / long list full
    C_INSERT = 2,    // distinct keys (set from a scan of the table)
    C_COLLIDE = 3,   // long-word hash collision detected
    C_HIST = 4,      // 26 first-letter counters
    C_TIES = 30,     // dictionary entries sharing a 12-letter prefix
    C_MAXLEN = 31,   // longest tied word
    C_LONGMAX = 32,  // fullest long-token queue shard
    C_LSHARD = 40,   // kLongShards queue counters, 16 apart (one 128-B line each)
    C_NUM = 40 + 64 * 16
};
// Long tokens are queued in kLongShards shards (by chunk) so that the
// queue's atomics do not all hit one address: one word saturates at about
// 90 atomics per microsecond (MI355X_MICROARCH.md, fanin / dequeue rows).
constexpr int kLongShards = 64;

// C-locale isspace: the fscanf("%s") delimiter set (main.c:102).
__device__ __forceinline__ bool is_ws(uint32_t c) { return c == 32u || (c - 9u) < 5u; }
// letter index 0..25 for A-Z / a-z (main.c:106-110), >= 26 otherwise
__device__ __forceinline__ uint32_t letter_of(uint32_t c) { return (c | 0x20u) - 0x61u; }

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// ---------------------------------------------------------------- word table
// Word identity -> slot (the word's provisional id).  Keys are exact for
// words of <= 12 letters (5-bit letter codes, left aligned, low 4 bits 0) and
// a 60-bit hash tagged 0xF for longer words (verified after the map, see
// k_long_verify); 0 = empty.  Keys never change once set, so a stale empty
// read is corrected by the CAS.
//
// Two levels, one slot space:
//   hot table  slots [0, kHotSlots = 2^20): 8-slot buckets (one 64-B line),
//              probed inside the bucket only.  Words that arrive first — in a
//              Zipf corpus mostly the frequent ones — fill it; the probes of
//              frequent words hit L2, the rest the Infinity Cache (8 MB of
//              keys).  K1b resolves hot words itself; words that overflow to
//              the big table go to K1c (2^19 slots: 7.8 % of tokens, 2^20: less,
//              K1c 5.1 -> 3.4 ms at 10 GB).
//   big table  slots [kHotSlots, kHotSlots + cap): linear probing; words
//              whose hot bucket was already full.
// A word lives in exactly one place: a probe scans the same bucket (then the
// same big-table run) in the same order and slots only go empty -> full.
constexpr int kHotLog2 = 20;  // hot level: 2^20 slots (8 MB of keys) in 8-slot buckets (2^19: emit 14.6 -> 16.5 ms, 2^18: 18.4 ms
                              // at 10 GB with K1c fused; earlier, separate K1c: 2^19 -> 2^20: K1c 5.1 -> 3.4 ms
                              // at 10 GB, fewer words overflow to the big table)
constexpr uint64_t kHotSlots = 1ull << kHotLog2;
constexpr int kBucket = 8;

struct Table {
    unsigned long long* keys;  // [kHotSlots + big_cap]
    uint64_t* rep;             // token start of the inserting occurrence
    uint64_t big_mask;         // big_cap - 1
    uint64_t seed;
    uint64_t* counters;
    uint64_t long_mask;        // hashed keys keep these bits of the hash (~0; fewer: the II_TEST_LONG_KEY_BITS test knob)
};

// Home slot of a key in the hot table: a 32-bit multiply-xorshift hash of the
// key's two halves (cheap enough for every token).  The big table uses an
// independent 64-bit mix (big_home), only on the miss path.
__device__ __forceinline__ uint32_t hot_slot(uint64_t key, uint64_t seed) {
    uint32_t h = ((uint32_t)(key >> 32) ^ (uint32_t)seed) * 0x9E3779B1u +
                 ((uint32_t)key ^ (uint32_t)(seed >> 32)) * 0x85EBCA77u;
    h ^= h >> 15;
    h *= 0x2C1B3C6Du;
    h ^= h >> 12;
    return h & (uint32_t)(kHotSlots - 1);
}
__device__ __forceinline__ uint64_t big_home(const Table& t, uint64_t key) { return mix64(key ^ t.seed) & t.big_mask; }

// CAS-insert key at empty slot s; returns the key now stored there.
__device__ __forceinline__ unsigned long long table_claim(const Table& t, uint64_t s, uint64_t key, uint64_t pos) {
    const unsigned long long old = atomicCAS(&t.keys[s], 0ull, (unsigned long long)key);
    if (old == 0ull) {  // inserted; distinct words are counted later by a scan of the table
        t.rep[s] = pos;
        return key;
    }
    return old;
}

// Slot of key, inserting it if new.  Slow path of the probe (the home slot
// did not hold the key): the 8-slot hot bucket (one 64-B line) and the word's
// big-table home slot are loaded together, so a word living at its big-table
// home costs one round trip; the bucket is scanned with bit masks in probe
// order (from the first slot of the home slot's pair, wrapping inside the
// bucket); a full bucket sends the word to the big table (linear probing).
__device__ __forceinline__ uint32_t table_find(const Table& t, uint64_t key, uint32_t home, uint64_t pos) {
    const uint32_t h7 = home & (kBucket - 2);  // probe order: from the home slot's pair
    const uint64_t bbase = home & ~(uint32_t)(kBucket - 1);
    uint64_t h = big_home(t, key);
    const ulonglong2* bp = reinterpret_cast<const ulonglong2*>(t.keys + bbase);
    const ulonglong2 p0 = bp[0], p1 = bp[1], p2 = bp[2], p3 = bp[3];
    unsigned long long kb = t.keys[kHotSlots + h];
    const unsigned long long k[8] = {p0.x, p0.y, p1.x, p1.y, p2.x, p2.y, p3.x, p3.y};
    uint32_t match = 0, full = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        match |= (uint32_t)(k[j] == key) << j;
        full |= (uint32_t)(k[j] != 0ull) << j;
    }
    if (match) return (uint32_t)(bbase + __builtin_ctz(match));
    for (int it = 0; it < kBucket; it++) {
        const uint32_t empty = ~full & 0xFFu;
        if (!empty) break;
        const uint32_t rot = ((empty >> h7) | (empty << (8 - h7))) & 0xFFu;
        const uint32_t p = (h7 + __builtin_ctz(rot)) & (kBucket - 1);
        if (table_claim(t, bbase + p, key, pos) == key) return (uint32_t)(bbase + p);
        full |= 1u << p;
    }
    for (int probe = 0; probe < kMaxProbe; probe++) {
        const uint64_t s = kHotSlots + h;
        if (probe) kb = t.keys[s];
        if (kb == 0ull) kb = table_claim(t, s, key, pos);
        if (kb == key) return (uint32_t)s;
        h = (h + 1) & t.big_mask;
        // a table another lane found full: this attempt is void (the host regrows the table and maps
        // again), so leave at once — a full table otherwise costs every new word kMaxProbe probes
        // (3.4 s instead of 27 ms for the first map of configs[4]'s rank-7 share, 6.7·10^6 words)
        if ((probe & 15) == 15 &&
            (__hip_atomic_load(&t.counters[C_OVERFLOW], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 1ull))
            return 0;
    }
    atomicOr((unsigned long long*)&t.counters[C_OVERFLOW], 1ull);
    return 0;
}

// ---------------------------------------------------------------- K1 tokenizer
// Full cleaned word at a token start (main.c:105-111, <= 299 letters):
// length, FNV-style hash of the letter codes and the first-12 prefix.
struct LongWord {
    uint64_t hash;
    uint64_t prefix;
    uint32_t len;
};
__device__ __forceinline__ LongWord read_word(const uint8_t* __restrict__ text, uint64_t nbytes, uint64_t pos) {
    LongWord w{1469598103934665603ull, 0ull, 0u};
    for (uint64_t g = pos; g < nbytes; g++) {
        uint32_t c = text[g];
        if (c == 0u || is_ws(c)) break;
        uint32_t lc = letter_of(c);
        if (lc < 26u) {
            w.len++;
            if (w.len <= 12) w.prefix |= (uint64_t)(lc + 1) << (64 - 5 * w.len);
            w.hash = (w.hash ^ (lc + 1)) * 1099511628211ull;
            if (w.len == kMaxWord) break;
        }
    }
    return w;
}

__device__ __forceinline__ uint64_t long_key(uint64_t hash, uint32_t len, uint64_t seed, uint64_t mask) {
    return ((mix64(hash ^ seed ^ ((uint64_t)len << 48)) & mask) << 4) | 0xFull;
}

// Reader of the staged tile: tile-local byte j (j >= -16); LDS is read one
// aligned dword at a time (the walk touches ~2 dwords per token instead of
// ~7 bytes), past the halo it falls back to global memory.
struct TileReader {
    const uint8_t* s;
    const uint8_t* __restrict__ text;
    uint64_t nbytes, tile_lo;
    uint32_t lim, di, dw;  // lim = bytes staged in LDS after the 16-byte left piece
    __device__ __forceinline__ TileReader(const uint8_t* s_, const uint8_t* text_, uint64_t nb, uint64_t lo, uint32_t lim_)
        : s(s_), text(text_), nbytes(nb), tile_lo(lo), lim(lim_), di(0xFFFFFFFFu), dw(0) {}
    __device__ __forceinline__ uint32_t get(uint32_t j) {
        if (j < lim) {
            const uint32_t a = 16 + j;
            if ((a >> 2) != di) {
                di = a >> 2;
                dw = reinterpret_cast<const uint32_t*>(s)[di];
            }
            return (dw >> ((a & 3) * 8)) & 0xFFu;
        }
        const uint64_t g = tile_lo + j;
        return g < nbytes ? text[g] : 32u;
    }
};

// Word key of a token (the cleaning loop of main.c:105-111): exact 5-bit
// packing for <= 12 letters, tagged hash otherwise; its letter count (0 =
// dropped, main.c:113) and first letter.
struct TokKey {
    uint64_t key;
    uint32_t nlet;
    uint32_t first;
};

// A token is kept iff a letter comes before the first whitespace / NUL
// (main.c:105, 113).  Cheap form for the count pass.
__device__ __forceinline__ bool token_kept(TileReader& rd, uint32_t p) {
    for (uint32_t j = p;; j++) {
        const uint32_t c = rd.get(j);
        if (c == 0u || is_ws(c)) return false;
        if (letter_of(c) < 26u) return true;
    }
}

// file index of byte position pos: last f in [f_lo, f_hi] with start[f] <= pos
__device__ __forceinline__ uint32_t file_of(const uint64_t* __restrict__ start, uint32_t f_lo, uint32_t f_hi, uint64_t pos) {
    while (f_lo < f_hi) {
        uint32_t mid = f_lo + (f_hi - f_lo + 1) / 2;
        if (start[mid] <= pos) f_lo = mid;
        else f_hi = mid - 1;
    }
    return f_lo;
}

// Per K1 chunk c: {first file, last file, first file again} — one binary
// search per chunk for the whole grid, instead of a serial search by one
// thread at the start of every K1b / K1c workgroup (~28 dependent loads in
// each workgroup's critical path).
// File numbers in the K1 records are SHARD-LOCAL: the index of the file in the
// mapped file table (0 .. nfiles - 1), dense and, since files are mapped in
// ascending id0 order, monotone in id0.  The id bits of the token sort then
// depend on the shard's file count, not on the global list (a rank of an
// ii_partition share whose ids span [0, 10^6) sorts 17-bit indices, not 20-bit
// ids); K3 maps an index back to its id0 (k_uniq_sweep, fmap) when it writes
// the pairs.
__global__ __launch_bounds__(kBlock) void k_chunk_files(const uint64_t* __restrict__ file_start, uint32_t nfiles,
                                                        uint64_t nbytes, uint64_t chunk, uint64_t nch,
                                                        uint32_t* __restrict__ cf) {
    const uint64_t c = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (c >= nch) return;
    const uint64_t lo = c * chunk, hi = lo + chunk < nbytes ? lo + chunk : nbytes;
    const uint32_t f0 = file_of(file_start, 0, nfiles - 1, lo);
    const uint32_t f1 = file_of(file_start, f0, nfiles - 1, hi - 1);
    cf[3 * c] = f0;
    cf[3 * c + 1] = f1;
    cf[3 * c + 2] = f0;
}

// The 16 bytes at g, a multiple of 16 (the text is 16-byte aligned); bytes
// outside [0, nbytes) read as ' '.  An aligned 16-B block never straddles a
// page, so once its first byte is text the whole load is safe; the bytes past
// the end are replaced (no per-byte path: it would cost every caller's
// registers).
__device__ __forceinline__ uint32_t keep_bytes(uint32_t w, int64_t left) {
    if (left >= 4) return w;
    if (left <= 0) return 0x20202020u;
    const uint32_t m = (1u << (8 * (uint32_t)left)) - 1u;
    return (w & m) | (0x20202020u & ~m);
}
__device__ __forceinline__ uint4 load16(const uint8_t* __restrict__ text, uint64_t nbytes, int64_t g) {
    if (g < 0 || (uint64_t)g >= nbytes) return make_uint4(0x20202020u, 0x20202020u, 0x20202020u, 0x20202020u);
    uint4 v = *reinterpret_cast<const uint4*>(text + g);
    const int64_t left = (int64_t)(nbytes - (uint64_t)g);
    if (left < 16) {
        v.x = keep_bytes(v.x, left);
        v.y = keep_bytes(v.y, left - 4);
        v.z = keep_bytes(v.z, left - 8);
        v.w = keep_bytes(v.w, left - 12);
    }
    return v;
}

// ---- SWAR byte classes, 4 bytes per u32 (exact, no inter-byte carries)
// bit 7 of each byte set where the byte is zero
__device__ __forceinline__ uint32_t zero_bytes(uint32_t x) {
    return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
}
struct Classes {
    uint32_t ws, letter, nul;  // 16-bit masks over the lane's window
};
// class flags of 4 bytes: bit 7 of each byte (nothing else) set where the byte is of the class
__device__ __forceinline__ void classify_flags4(uint32_t x, uint32_t& ws, uint32_t& let, uint32_t& nul) {
    const uint32_t hb = x & 0x80808080u;
    const uint32_t y = x & 0x7F7F7F7Fu;
    const uint32_t sp = zero_bytes(x ^ 0x20202020u);                                  // ' '
    const uint32_t ctl = (y + 0x77777777u) & ~(y + 0x72727272u) & ~hb & 0x80808080u;   // 9..13
    ws = sp | ctl;                                        // C-locale isspace (main.c:102)
    const uint32_t z = (x | 0x20202020u) & 0x7F7F7F7Fu;
    let = (z + 0x1F1F1F1Fu) & ~(z + 0x05050505u) & ~hb & 0x80808080u;  // A-Z / a-z (main.c:106-110)
    nul = zero_bytes(x);
}
// The bit-7 flags of 16 bytes (f0 = bytes 0..3, ...) -> a 16-bit mask: each
// flag byte (0x80 or 0) times its bit's weight, summed by v_dot4_u32_u8 (two
// per 8 bits, weights 1..128 / 128 each) instead of shifting every flag into place.
__device__ __forceinline__ uint32_t flags16(uint32_t f0, uint32_t f1, uint32_t f2, uint32_t f3) {
    const uint32_t lo = __builtin_amdgcn_udot4(f1, 0x80402010u, __builtin_amdgcn_udot4(f0, 0x08040201u, 0u, false), false);
    const uint32_t hi = __builtin_amdgcn_udot4(f3, 0x80402010u, __builtin_amdgcn_udot4(f2, 0x08040201u, 0u, false), false);
    return (lo >> 7) | ((hi >> 7) << 8);
}
__device__ __forceinline__ Classes classify16(const uint4& v) {
    uint32_t ws[4], let[4], nul[4];
    classify_flags4(v.x, ws[0], let[0], nul[0]);
    classify_flags4(v.y, ws[1], let[1], nul[1]);
    classify_flags4(v.z, ws[2], let[2], nul[2]);
    classify_flags4(v.w, ws[3], let[3], nul[3]);
    return Classes{flags16(ws[0], ws[1], ws[2], ws[3]), flags16(let[0], let[1], let[2], let[3]),
                   flags16(nul[0], nul[1], nul[2], nul[3])};
}

// Kept tokens among the starts (a letter before the first whitespace / NUL,
// main.c:105, 113); decided from the masks, walking LDS only when the window
// ends before the token shows a letter, space or NUL.
__device__ __forceinline__ uint32_t kept_starts(uint32_t starts, const Classes& cl, const uint8_t* s_text,
                                                const uint8_t* __restrict__ text, uint64_t nbytes, uint64_t tile_lo,
                                                uint32_t wlo, uint32_t lim) {
    const uint32_t ev = cl.letter | cl.ws | cl.nul;
    uint32_t kept = 0;
    for (uint32_t m = starts & ~cl.letter; m; m &= m - 1) {  // starts that are not letters themselves
        const uint32_t i = __builtin_ctz(m);
        const uint32_t e = ev >> i;
        bool k;
        if (e) k = (cl.letter >> (i + __builtin_ctz(e))) & 1u;
        else {
            TileReader rd(s_text, text, nbytes, tile_lo, lim);
            k = token_kept(rd, wlo + 16);
        }
        kept |= (uint32_t)k << i;
    }
    return kept | (starts & cl.letter);
}

// First 16 bytes of the token starting at window offset i (0..15), taken
// from the lane's 32-byte view w[0..7] = own window + next lane's window.
__device__ __forceinline__ uint32_t sel4(uint32_t k, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    const uint32_t lo = (k & 1u) ? b : a;  // two-level select: v_cndmask, no branches
    const uint32_t hi = (k & 1u) ? d : c;
    return (k & 2u) ? hi : lo;
}
__device__ __forceinline__ uint4 token_bytes(const uint32_t (&w)[8], uint32_t i) {
    const uint32_t wo = i >> 2, bo = i & 3;
    uint32_t x[5];
#pragma unroll
    for (int j = 0; j < 5; j++) x[j] = sel4(wo, w[j], w[j + 1], w[j + 2], w[j + 3]);
    return make_uint4(__builtin_amdgcn_alignbyte(x[1], x[0], bo), __builtin_amdgcn_alignbyte(x[2], x[1], bo),
                      __builtin_amdgcn_alignbyte(x[3], x[2], bo), __builtin_amdgcn_alignbyte(x[4], x[3], bo));
}

// 16 bytes of the text at any position g, from two aligned 16-B loads.
__device__ __forceinline__ uint4 global_block16(const uint8_t* __restrict__ text, uint64_t nbytes, uint64_t g) {
    const int64_t a = (int64_t)(g & ~15ull);
    const uint4 lo = load16(text, nbytes, a), hi = load16(text, nbytes, a + 16);
    const uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    return token_bytes(w, (uint32_t)(g & 15u));
}

// 16 bytes of the staged tile at tile-local position p (any alignment):
// two aligned LDS reads + byte shift; past the staged halo, global memory.
__device__ __forceinline__ uint4 tile_block16(const uint8_t* s_text, const uint8_t* __restrict__ text, uint64_t nbytes,
                                              uint64_t tile_lo, uint32_t p, uint32_t lim) {
    const uint32_t a = 16 + p;
    const uint32_t base = a & ~15u;
    if (base + 32 <= 16 + lim) {
        const uint4 lo = *reinterpret_cast<const uint4*>(s_text + base);
        const uint4 hi = *reinterpret_cast<const uint4*>(s_text + base + 16);
        const uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        return token_bytes(w, a & 15u);
    }
    return global_block16(text, nbytes, tile_lo + p);
}

__device__ __forceinline__ uint32_t byte_dyn(const uint4& b, uint32_t j) {
    return (sel4(j >> 2, b.x, b.y, b.z, b.w) >> (8 * (j & 3u))) & 0xFFu;
}

// ---------------------------------------------------------------- K1 chunks
// The text is cut into chunks of kChunk bytes, ONE WAVE per chunk (kWG
// chunks per workgroup): a wave walks its chunk alone, with wave-level
// ballots / scans and wave-private LDS, and never waits at a workgroup
// barrier — the waves of a CU drift apart and overlap each other's memory
// latency instead of meeting at a barrier every round.
constexpr int kWG = kBlock / 64;  // chunks (waves) per workgroup

// This wave's chunk, as a wave-uniform (scalar) value: the compiler cannot
// prove threadIdx.x / 64 uniform, and everything derived from it would
// otherwise live in vector registers.
__device__ __forceinline__ uint64_t wave_chunk() {
    return (uint64_t)blockIdx.x * kWG + (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
}

// Orders this wave's earlier LDS accesses before its later ones (LDS
// instructions of one wave execute in program order; this keeps the compiler
// from moving them across).  Not a workgroup barrier.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ uint32_t wave_sum32(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o, 64);
    return v;
}

// K1a: kept tokens per chunk -> chunk_cnt[c] (dense record layout only),
// straight from HBM: lane l classifies windows 64 j + l of the chunk with
// 16-B loads; the byte before a window comes from the neighbour lane, or a
// 1-byte load for lane 0; the rare start whose keep decision lies past its
// window walks the text in HBM (kept_starts with nothing staged).
__device__ __forceinline__ uint32_t window_kept(const uint4& v, uint64_t g, const uint8_t* __restrict__ text,
                                                uint64_t nbytes) {
    const Classes cl = classify16(v);
    uint32_t prev = (uint32_t)__shfl_up((int)v.w, 1, 64) >> 24;
    if (lane_id() == 0) prev = (g > 0 && g - 1 < nbytes) ? text[g - 1] : 32u;
    const uint32_t starts = ~cl.ws & ((cl.ws << 1) | (is_ws(prev) ? 1u : 0u)) & 0xFFFFu;
    return __popc(kept_starts(starts, cl, nullptr, text, nbytes, g, 0, 0));
}

__global__ __launch_bounds__(kBlock) void k_tok_count(const uint8_t* __restrict__ text, uint64_t nbytes, uint64_t nch,
                                                      uint64_t* __restrict__ chunk_cnt) {
    constexpr int kWinsPerLane = (int)(kChunk / 16 / 64);
    constexpr int kInFlight = 8;
    const uint64_t c = wave_chunk();
    if (c >= nch) return;
    const uint64_t chunk_lo = c * kChunk;
    const int l = lane_id();
    uint32_t kept = 0;
    if (chunk_lo + kChunk + 16 <= nbytes) {  // interior chunk: plain 16-B loads, 8 in flight per lane
        for (int jb = 0; jb < kWinsPerLane; jb += kInFlight) {
            uint4 v[kInFlight];
#pragma unroll
            for (int u = 0; u < kInFlight; u++)
                v[u] = *reinterpret_cast<const uint4*>(text + chunk_lo + 16 * (64ull * (jb + u) + l));
#pragma unroll
            for (int u = 0; u < kInFlight; u++) kept += window_kept(v[u], chunk_lo + 16 * (64ull * (jb + u) + l), text, nbytes);
        }
    } else {
        for (int j = 0; j < kWinsPerLane; j++) {
            const uint64_t g = chunk_lo + 16 * (64ull * j + l);
            kept += window_kept(load16(text, nbytes, (int64_t)g), g, text, nbytes);
        }
    }
    kept = wave_sum32(kept);
    if (l == 0) chunk_cnt[c] = kept;
}

// Long token queued for the exactness check (k_long_verify).
struct LongTok {
    uint64_t pos;   // token start
    uint64_t slot;  // word-table slot it was given
};

// Record layout of K1b / K1c.  Dense (cap == 0): chunk c's records start at
// chunk_off[c], the exclusive scan of k_tok_count's counts.  Fixed capacity
// (cap == kChunkCap): chunk c owns rec[c * cap, (c + 1) * cap) and pend
// likewise, no counting pass; K1b leaves the chunk's token count in
// chunk_off[c] and the first sort pass gathers the used prefixes.
// Inside its slot, chunk c's records start at a per-chunk rotation and wrap:
// a Zipf chunk fills ~30 % of its slot, so unrotated prefixes would all sit
// at the same low offsets of every slot and load only the HBM channels those
// offsets interleave to.
constexpr uint64_t kChunkCap = kChunk / 2;  // a token start follows a whitespace byte
static_assert((kChunkCap & (kChunkCap - 1)) == 0, "slot rotation wraps with a mask");
__device__ __forceinline__ uint32_t chunk_rot(uint64_t c) {
    return (uint32_t)((((uint32_t)c * 2654435761u) >> 22) << 5) & (uint32_t)(kChunkCap - 1);  // 256-B steps
}
__device__ __forceinline__ uint64_t chunk_base(const uint64_t* chunk_off, uint64_t cap, uint64_t c) {
    return cap ? c * cap : chunk_off[c];
}
// Narrow records: in the fixed-capacity layout, a chunk that lies inside one
// file (k_chunk_files: first file == last file, ~98 % of config3's chunks)
// stores its records as u32 word slots in the first half of its slot (the
// file id is the chunk's, restored by the first sort pass), which halves the
// record bytes K1b writes and the first sort pass reads.  Its fast-path misses
// keep their keys in the second half (kNarrowKeys u64 entries, in miss order);
// a chunk with more misses than that (narrow_keys, kNarrowKeys unless a test
// lowers it with II_NARROW_KEYS) sends the rest down the general path.
// Round 6: a chunk over several files is narrow too when their number fits the low lbits of
// a u32 record: slot << lbits | (file - the chunk's first file), lbits = 32 - the bits of the
// map's slots (rec_lbits; 10 at config3, 7 for configs[4]'s shares); a one-file chunk's record
// stays its slot.  configs[4]'s rank-7
// share (440 000 files of ~28 KB: most chunks span two or three) wrote 8-B records for nearly
// every token before.
constexpr uint32_t kNarrowKeys = (uint32_t)(kChunkCap / 2);
__device__ __forceinline__ bool chunk_narrow(uint64_t cap, const uint32_t* cf, uint64_t c, uint32_t lbits) {
    return cap && cf[3 * c + 1] - cf[3 * c] < (1u << lbits);  // (lbits = 0: one-file chunks only)
}
// host: the low record bits left beside a slot, or 0 (one-file narrow chunks only) for inputs of
// large files, where few chunks span several files (config3: 2 %; the decode cost the first pass
// 0.12 ms there and saved nothing)
inline uint32_t rec_lbits(uint64_t nslots, uint64_t nbytes, uint64_t nfiles) {
    if (nfiles == 0 || nbytes / nfiles >= (256u << 10)) return 0;
    uint32_t b = 0;
    while (b < 32 && (1ull << b) < nslots) b++;
    return 32 - b;
}
// the chunk's j-th record sits at cbase (chunk_base) + ((j + rot) & wrap), (rot,
// wrap) = (chunk_rot(c), kChunkCap - 1) in the fixed-capacity layout (u32
// units for a narrow chunk), (0, ~0) in the dense one
__device__ __forceinline__ uint32_t rec_wrap(uint64_t cap) { return cap ? (uint32_t)(kChunkCap - 1) : ~0u; }
__device__ __forceinline__ uint32_t rec_rot(uint64_t cap, uint64_t c) { return cap ? chunk_rot(c) : 0u; }


// ---------------------------------------------------------------- K1b emit
// One wave per chunk (see "K1 chunks"), in rounds of kRound bytes: 2 windows
// of 16 B per lane, window w = 64 j + lane, so each load instruction reads
// 1 KiB contiguous; the next round is loaded while this one is worked on.
// Per round, all in wave-private LDS:
//   1. SWAR classes per window -> kept token starts (main.c:102-113) and the
//      window's terminator / letter bit masks;
//   2. one wave scan of 2 packed 16-bit counts -> the token index of every
//      kept start in text order; the starts are listed;
//   3. 64 tokens at a time, one per lane: the register key path (masks + 12
//      bytes from LDS, 5-bit packing, main.c:105-111) and the hot-table
//      probe (two lanes load the 32 B that begin a key's probe order); a hit
//      stores its record straight to HBM (consecutive lanes, consecutive
//      records); probe misses and general-path tokens (inner punctuation,
//      > 12 letters, > 16 bytes) are listed for K1c.
// Records rec[i] = slot << 32 | file id0, in text order (the partial files'
// "word id" lines, main.c:116).  First letters are counted per chunk
// (chunk_hist = the partial_<letter>.txt line counts).
constexpr int kWin = 2;                          // 16-B windows per lane per round
constexpr int kRound = kWin * 16 * 64;           // 2 KiB of text per wave round
constexpr int kRoundWins = kRound / 16;          // windows per round
constexpr int kRoundHalo = 64;                   // bytes staged past the round (a fast key reads <= 16)
constexpr int kHaloPieces = kRoundHalo / 16;
constexpr int kRoundStaged = kRound + kRoundHalo;  // bytes staged in LDS after the left piece
constexpr int kMaxRoundTok = kRound / 2;         // a token start needs a space before it
static_assert(kChunk % kRound == 0, "a chunk is a whole number of rounds");
static_assert(kWin * 16 <= 32, "2 packed 16-bit window counts per lane");

// wave-private LDS of K1b
struct EmitLds {
    uint8_t text[16 + kRoundStaged];  // [0, 16): the 16 bytes before the round
    uint32_t mask[kRoundWins + 1];    // per window: terminator (ws | NUL) bits | letter bits << 16
    uint16_t off[kMaxRoundTok];       // round-local start of every kept token, text order
    uint32_t hist[32];                // the chunk's first-letter counts
};

struct RoundRegs {
    uint4 v[kWin];  // lane's windows
    uint4 h;        // left piece (lane 0) / halo pieces (lanes 1..kHaloPieces)
};
// A round's loads are plain 16-B loads of aligned blocks with no branch
// between an interior and an edge form (two forms merge into one set of
// registers only by waiting for the loads): a block that starts past the
// text's last block is loaded from that block, and one before the text from
// block 0; store_round replaces what lies outside [0, nbytes) by spaces.  So
// the next round's loads stay in flight while this round is worked on.
__device__ __forceinline__ int64_t piece_pos(uint64_t lo, int l) {  // left piece (lane 0) / halo pieces
    return (int64_t)lo + 16 * (l == 0 ? -1 : kRoundWins + l - 1);
}
__device__ __forceinline__ void fetch_round(RoundRegs& r, const uint8_t* __restrict__ text, uint64_t nbytes, uint64_t lo) {
    const int l = lane_id();
    const uint64_t last = (nbytes - 1) & ~15ull;
#pragma unroll
    for (int j = 0; j < kWin; j++) {
        const uint64_t g = lo + 16 * (64 * j + l);
        r.v[j] = *reinterpret_cast<const uint4*>(text + (g < last ? g : last));
    }
    r.h = make_uint4(0, 0, 0, 0);
    if (l <= kHaloPieces) {
        const int64_t g = piece_pos(lo, l);
        r.h = *reinterpret_cast<const uint4*>(text + (g < 0 ? 0 : (uint64_t)g < last ? (uint64_t)g : last));
    }
}
__device__ __forceinline__ uint4 outside_spaces(uint4 v, int64_t g, uint64_t nbytes) {
    if (g < 0 || (uint64_t)g >= nbytes) return make_uint4(0x20202020u, 0x20202020u, 0x20202020u, 0x20202020u);
    const int64_t left = (int64_t)(nbytes - (uint64_t)g);
    if (left < 16) {
        v.x = keep_bytes(v.x, left);
        v.y = keep_bytes(v.y, left - 4);
        v.z = keep_bytes(v.z, left - 8);
        v.w = keep_bytes(v.w, left - 12);
    }
    return v;
}
__device__ __forceinline__ void store_round(uint8_t* s_text, RoundRegs r, uint64_t nbytes, uint64_t lo) {
    const int l = lane_id();
    if (lo < 16 || lo + kRoundStaged > nbytes) {  // (wave-uniform) a piece may lie outside the text
#pragma unroll
        for (int j = 0; j < kWin; j++) r.v[j] = outside_spaces(r.v[j], (int64_t)(lo + 16 * (64 * j + l)), nbytes);
        r.h = outside_spaces(r.h, piece_pos(lo, l), nbytes);
    }
#pragma unroll
    for (int j = 0; j < kWin; j++) *reinterpret_cast<uint4*>(s_text + 16 + 16 * (64 * j + l)) = r.v[j];
    if (l <= kHaloPieces) *reinterpret_cast<uint4*>(s_text + 16 + 16 * (l == 0 ? -1 : kRoundWins + l - 1)) = r.h;
}

// 4 letters (bytes, first in the low byte) -> their 5-bit codes, first letter
// in the high bits (20 bits).  x & 0x1F is the letter code for A-Z and a-z.
// Two v_dot4_u32_u8 of the codes: 32 c0 + c1 and 32 c2 + c3.
__device__ __forceinline__ uint32_t pack4(uint32_t x) {
    const uint32_t c = x & 0x1F1F1F1Fu;
    return (__builtin_amdgcn_udot4(c, 0x00000120u, 0u, false) << 10) | __builtin_amdgcn_udot4(c, 0x01200000u, 0u, false);
}

// Byte g (0..15) of the 16-byte value lo | hi << 64 removed: the bytes above
// it move down one place (three 64-bit shifts and two masked merges).
__device__ __forceinline__ void drop_byte(uint64_t& lo, uint64_t& hi, uint32_t g) {
    const uint64_t ml = g >= 8 ? ~0ull : (1ull << (8 * g)) - 1ull;         // bytes of lo that stay
    const uint64_t mh = g < 8 ? 0ull : (1ull << (8 * (g - 8))) - 1ull;     // bytes of hi that stay
    lo = (lo & ml) | (((lo >> 8) | (hi << 56)) & ~ml);
    hi = (hi & mh) | ((hi >> 8) & ~mh);
}

// Register key path of the cleaning loop (main.c:105-111): the token ends
// (whitespace / NUL) within reach of the round's masks and keeps 1..12
// letters; letters in one run from its first byte (plain or capitalised
// words, trailing punctuation), or — within its first 16 bytes — with up to
// three other bytes among them (a leading bracket, an apostrophe, a 2-byte
// UTF-8 letter: main.c:105-111 drops them), which are removed from the 16
// bytes read from LDS before the 5-bit packing.  Returns false for every
// other token (general path, K1c).
__device__ __forceinline__ bool round_fast_key(const uint8_t* s_text, const uint32_t* s_mask, uint32_t p, TokKey& k) {
    const uint32_t w0 = p >> 4, sh = p & 15u;
    const uint32_t m0 = s_mask[w0], m1 = s_mask[w0 + 1];
    const uint32_t term = ((m0 & 0xFFFFu) | (m1 << 16)) >> sh;
    const uint32_t let = ((m0 >> 16) | (m1 & 0xFFFF0000u)) >> sh;
    if (term == 0) return false;
    const uint32_t e = __builtin_ctz(term);
    const uint32_t lm = let & ((1u << e) - 1u);
    const uint32_t n = __popc(lm);
    if (n == 0 || n > 12) return false;
    const uint32_t a = 16u + p, al = a & 3u;
    const uint32_t* s32 = reinterpret_cast<const uint32_t*>(s_text) + (a >> 2);
    const uint32_t d0 = s32[0], d1 = s32[1], d2 = s32[2], d3 = s32[3];
    uint32_t x[3] = {__builtin_amdgcn_alignbyte(d1, d0, al), __builtin_amdgcn_alignbyte(d2, d1, al),
                     __builtin_amdgcn_alignbyte(d3, d2, al)};
    if (lm != (1u << n) - 1u) {  // other bytes before or among the letters
        if (e > 16) return false;
        uint32_t gaps = ~lm & ((2u << (31 - __builtin_clz(lm))) - 1u);  // below the last letter
        if (__popc(gaps) > 3) return false;
        const uint32_t d4 = s32[4];
        uint64_t lo = ((uint64_t)x[1] << 32) | x[0];
        uint64_t hi = ((uint64_t)__builtin_amdgcn_alignbyte(d4, d3, al) << 32) | x[2];
        while (gaps) {  // from the highest down: the lower positions stay put
            const uint32_t g = 31 - __builtin_clz(gaps);
            drop_byte(lo, hi, g);
            gaps &= ~(1u << g);
        }
        x[0] = (uint32_t)lo;
        x[1] = (uint32_t)(lo >> 32);
        x[2] = (uint32_t)hi;
    }
    const uint64_t key = ((uint64_t)pack4(x[0]) << 44) | ((uint64_t)pack4(x[1]) << 24) | ((uint64_t)pack4(x[2]) << 4);
    k.key = key & (~0ull << (64 - 5 * n));
    k.nlet = n;
    k.first = (x[0] & 31u) - 1u;
    return true;
}

// Hot-table probe of K1b: a lane loads the two 16-B slot pairs that begin
// its key's probe order in the 8-slot bucket (home's pair and the next, one
// 64-B line; the probe order of a bucket starts at the home slot's pair, see
// table_find).  A frequent word sits in its home pair or the next one (it
// was inserted while its bucket was still empty), so the short window decides
// almost every token; the rest go to K1c.  (Two lanes sharing one token's
// loads, so that an instruction touches half as many lines, measured 0.35 ms
// slower at 10 GB: the shuffles that route keys and results cost more VALU.)
// match / empty: 4-bit masks over the seen probe positions 0..3.  A match is
// the slot; otherwise the first empty position is claimed (table_find's rule,
// so a word still lives in exactly one place); no empty slot, or a raced
// claim, leaves the word to K1c.
__device__ __forceinline__ uint32_t bucket_resolve(const Table& t, uint32_t match, uint32_t empty, uint64_t key,
                                                   uint32_t bbase, uint32_t start, uint64_t pos) {
    const uint32_t m = match ? match : empty;
    if (!m) return kSlotNone;
    const uint32_t s = bbase + ((start + __builtin_ctz(m)) & (kBucket - 1));
    if (match) return s;
    return table_claim(t, s, key, pos) == key ? s : kSlotNone;
}

// Unresolved token of a chunk (K1b -> K1c), one u32: chunk-relative start
// (16 bits) | chunk-relative token index << 16.  A chunk's list holds its
// fast-path misses (the key left in the record slot) from the front of its
// region and its general-path tokens from the back; pend_cnt[c] = the two
// counts (low / high 16 bits).  The region is the chunk's record range, and
// there are at most as many pending tokens as tokens.
static_assert(kChunk <= 65536 && kChunkCap <= 32768, "pending-token fields");
__device__ __forceinline__ uint64_t pend_limit(const uint64_t* chunk_off, uint64_t cap, uint64_t cbase, uint64_t c) {
    return cap ? cbase + cap : chunk_off[c + 1];  // dense: chunk_off is the exclusive scan of the counts
}

// General form of the cleaning loop (main.c:105-111) for the token at text
// position pos, one aligned 16-byte block per step (SWAR classes; the bytes
// of the first block before pos are ignored).  The cleaned word's letters
// form a stream of codes (1..26, one byte each) that is hashed one dword (4
// letters) at a time; the first three dwords are the first 12 letters (the
// exact key of a word of <= 12 letters).  A block whose letters form one run
// (a plain or capitalised word, trailing punctuation) is appended as a whole;
// other blocks letter by letter.  Stops at whitespace, NUL or the 299th letter.
struct LetterStream {
    uint64_t hash;
    uint32_t pend, pc;  // codes not yet folded: pc bytes (0..3)
    uint32_t nd, n;     // dwords folded, letters
    uint32_t d0, d1, d2;
    __device__ __forceinline__ void fold(uint32_t w) {
        d0 = nd == 0 ? w : d0;
        d1 = nd == 1 ? w : d1;
        d2 = nd == 2 ? w : d2;
        hash = (hash ^ w) * 1099511628211ull;
        nd++;
    }
};
__device__ __forceinline__ TokKey general_key(const uint8_t* __restrict__ text, uint64_t nbytes, uint64_t pos,
                                              uint64_t seed, uint64_t long_mask) {
    LetterStream st{1469598103934665603ull ^ seed, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
    uint64_t g = pos & ~15ull;
    uint32_t below = (1u << (pos & 15u)) - 1u;  // first block: bytes before the token
    for (;;) {
        const uint4 b = load16(text, nbytes, (int64_t)g);
        const Classes cl = classify16(b);
        const uint32_t term = (cl.ws | cl.nul) & ~below;
        const uint32_t e = term ? __builtin_ctz(term) : 16u;
        const uint32_t lm = cl.letter & ~below & ((1u << e) - 1u);
        below = 0;
        const uint32_t k = __popc(lm);
        if (lm && (lm & (lm + (lm & (0u - lm)))) == 0 && st.n + k <= (uint32_t)kMaxWord) {
            // one run of k letters from byte s: shift it to byte 0, letter codes, bytes >= k cleared
            const uint32_t s = __builtin_ctz(lm);
            uint64_t lo = ((uint64_t)b.y << 32) | b.x, hi = ((uint64_t)b.w << 32) | b.z;
            if (s >= 8) {
                lo = hi >> (8 * (s - 8));
                hi = 0;
            } else if (s) {
                lo = (lo >> (8 * s)) | (hi << (64 - 8 * s));
                hi >>= 8 * s;
            }
            lo &= (k >= 8 ? ~0ull : (1ull << (8 * k)) - 1ull) & 0x1F1F1F1F1F1F1F1Full;
            hi &= (k <= 8 ? 0ull : k >= 16 ? ~0ull : (1ull << (8 * (k - 8))) - 1ull) & 0x1F1F1F1F1F1F1F1Full;
            // behind the pending codes: 5 dwords, the first (pc + k) / 4 of them complete
            const uint32_t sh = 8 * st.pc;
            const uint32_t w[5] = {st.pend | ((uint32_t)lo << sh), (uint32_t)(lo >> (32 - sh)),
                                   (uint32_t)(((hi << 32) | (lo >> 32)) >> (32 - sh)), (uint32_t)(hi >> (32 - sh)),
                                   (uint32_t)((hi >> 32) >> (32 - sh))};
            const uint32_t t = st.pc + k, full = t >> 2;
#pragma unroll
            for (int i = 0; i < 4; i++)
                if ((uint32_t)i < full) st.fold(w[i]);
            st.pend = sel4(full & 3u, w[0], w[1], w[2], w[3]);
            st.pend = full == 4 ? w[4] : st.pend;
            st.pc = t & 3u;
            st.n += k;
        } else {
            for (uint32_t m = lm; m && st.n < (uint32_t)kMaxWord; m &= m - 1) {
                st.pend |= (byte_dyn(b, __builtin_ctz(m)) & 0x1Fu) << (8 * st.pc);
                st.n++;
                if (++st.pc == 4) {
                    st.fold(st.pend);
                    st.pend = 0;
                    st.pc = 0;
                }
            }
        }
        if (term || st.n == (uint32_t)kMaxWord) break;
        g += 16;
    }
    if (st.pc) st.fold(st.pend);
    const uint64_t key = st.n <= 12 ? ((uint64_t)pack4(st.d0) << 44) | ((uint64_t)pack4(st.d1) << 24) |
                                          ((uint64_t)pack4(st.d2) << 4)
                                    : long_key(st.hash, st.n, seed, long_mask);
    return TokKey{key, st.n, st.n ? (st.d0 & 31u) - 1u : 0u};
}

// K1c, the chunk's pending tokens (K1b's list), one per lane, run by the
// chunk's own wave once its rounds are done: general-path tokens
// (main.c:105-111 with inner punctuation, > 12 letters or > 16 bytes: key
// from the text) or fast-path misses (full hot bucket, raced claim: key left
// in the record slot) — full table lookup / insert (table_find), record.
// Their dependent loads overlap the other waves' rounds (K1b is VALU-bound,
// this is latency-bound), instead of a kernel of its own.  Tokens of more
// than 12 letters (hashed keys) are queued for k_long_verify.
template <bool kSlow>
__device__ __forceinline__ void resolve_pending(const uint8_t* __restrict__ text, uint64_t nbytes, uint64_t c,
                                                const uint64_t* __restrict__ file_start, uint32_t f_lo, uint32_t f_hi,
                                                uint64_t cbase, uint32_t wrap, uint32_t rot,
                                                bool narrow, uint32_t lbits, uint64_t pend_end, const uint32_t* __restrict__ pend, uint32_t n,
                                                const Table& tab, uint64_t* __restrict__ rec, uint32_t* hist,
                                                LongTok* __restrict__ longs, uint64_t long_per) {
    const int l = lane_id();
    const uint64_t chunk_lo = c * kChunk;
    for (uint32_t i0 = 0; i0 < n; i0 += 64) {
        const uint32_t i = i0 + l;
        bool is_long = false;
        uint64_t pos = 0, slot = 0;
        if (i < n) {
            const uint32_t e = kSlow ? pend[pend_end - 1 - i] : pend[cbase + i];
            pos = chunk_lo + (e & 0xFFFFu);
            const uint32_t jr = ((e >> 16) + rot) & wrap;  // the token's record in the chunk's slot
            uint64_t key;
            if (kSlow) {
                const TokKey k = general_key(text, nbytes, pos, tab.seed, tab.long_mask);
                atomicAdd(&hist[k.first], 1u);
                key = k.key;
                is_long = k.nlet > 12;
            } else {
                key = rec[cbase + (narrow ? kNarrowKeys + i : jr)];
            }
            slot = table_find(tab, key, hot_slot(key, tab.seed), pos);
            const uint32_t f = f_lo == f_hi ? f_lo : file_of(file_start, f_lo, f_hi, pos);
            if (narrow)
                reinterpret_cast<uint32_t*>(rec + cbase)[jr] = f_lo == f_hi ? (uint32_t)slot : ((uint32_t)slot << lbits) | (f - f_lo);
            else rec[cbase + jr] = (slot << 32) | f;
        }
        if (!kSlow) continue;
        // hashed keys: queue for the exactness check, one atomic per wave on the chunk's shard
        const uint64_t lm = __ballot(is_long);
        if (lm) {
            const uint32_t shard = (uint32_t)(c & (kLongShards - 1));
            const int leader = __builtin_ctzll(lm);
            unsigned long long base = 0;
            if (l == leader)
                base = atomicAdd((unsigned long long*)&tab.counters[C_LSHARD + 16 * shard], (unsigned long long)__popcll(lm));
            base = (unsigned long long)__shfl((long long)base, leader, 64);
            if (is_long) {
                const uint64_t g = base + lanes_below(lm);
                if (g < long_per) longs[shard * long_per + g] = LongTok{pos, slot};
                else atomicOr((unsigned long long*)&tab.counters[C_OVERFLOW], 2ull);
            }
        }
    }
}

// The fast path's hot-table probe (K1b step 3): the slot of a token's word
// from the two 16-B slot pairs that begin its probe order, kSlotNone when the
// word is left to K1c.  The home slot's pair first (begin: its load is issued,
// and K1b builds the next batch's keys while it is in flight); only a lane
// whose home pair is full without its key loads the next pair (finish): the
// vector L1 handles a probe lane by lane (random lines), so the lanes left out
// of an instruction are what it saves.  (A policy type: tools/k1_ablate.hip
// times the same kernel body with other probes, e.g. none.)
struct ProbeState {
    ulonglong2 qa;
    uint32_t home;
};
struct HotProbe {
    __device__ __forceinline__ ProbeState begin(const Table& t, bool fast, uint64_t key, uint32_t home) const {
        ProbeState st{make_ulonglong2(1ull, 1ull), home};
        if (fast) st.qa = *reinterpret_cast<const ulonglong2*>(t.keys + (home & ~1u));
        return st;
    }
    __device__ __forceinline__ uint32_t finish(const Table& t, const ProbeState& st, bool fast, uint64_t key,
                                              uint64_t pos) const {
        const uint32_t bbase = st.home & ~(uint32_t)(kBucket - 1), start = st.home & (kBucket - 2);
        uint32_t match = (uint32_t)(st.qa.x == key) | ((uint32_t)(st.qa.y == key) << 1);
        uint32_t empty = (uint32_t)(st.qa.x == 0ull) | ((uint32_t)(st.qa.y == 0ull) << 1);
        if (fast && !(match | empty)) {
            const ulonglong2 qb = *reinterpret_cast<const ulonglong2*>(t.keys + bbase + ((start + 2) & (kBucket - 2)));
            match |= ((uint32_t)(qb.x == key) << 2) | ((uint32_t)(qb.y == key) << 3);
            empty |= ((uint32_t)(qb.x == 0ull) << 2) | ((uint32_t)(qb.y == 0ull) << 3);
        }
        return fast ? bucket_resolve(t, match, empty, key, bbase, start, pos) : kSlotNone;
    }
};

// The probe for vocabularies larger than the hot level (DeepProbe, chosen by
// the host when most of the previous map's distinct words lived in the big
// table — configs[4]'s vocabulary of 10^7 against 2^20 hot slots): a lane
// whose home pair is full without its key loads the bucket's other three
// pairs and its big-table home slot in one more round trip, so a word
// resolved at its big home (found, or claimed there: table_find's rule, whose
// linear probe starts at the home) no longer goes to the K1c tail; only words
// past their big home do.  (With a vocabulary that fits the hot level the
// extra round trip costs more than the few K1c tokens it saves: emit +0.2 ms
// at 10 GB.  Round 5: the second pair in the same round trip as the rest of
// the bucket instead of one of its own, emit 22.47 -> 21.83 ms on the rank-7
// share of configs[4]: nearly every batch has a lane past its home pair.)
struct DeepProbe {
    __device__ __forceinline__ ProbeState begin(const Table& t, bool fast, uint64_t key, uint32_t home) const {
        return HotProbe().begin(t, fast, key, home);
    }
    __device__ __forceinline__ uint32_t finish(const Table& t, const ProbeState& st, bool fast, uint64_t key,
                                              uint64_t pos) const {
        const uint32_t bbase = st.home & ~(uint32_t)(kBucket - 1), start = st.home & (kBucket - 2);
        uint32_t match = (uint32_t)(st.qa.x == key) | ((uint32_t)(st.qa.y == key) << 1);
        uint32_t empty = (uint32_t)(st.qa.x == 0ull) | ((uint32_t)(st.qa.y == 0ull) << 1);
        if (fast && !(match | empty)) {  // the bucket's other three pairs and the big-table home, one round trip
            const uint64_t h = big_home(t, key);
            const ulonglong2 qb = *reinterpret_cast<const ulonglong2*>(t.keys + bbase + ((start + 2) & (kBucket - 2)));
            const ulonglong2 qc = *reinterpret_cast<const ulonglong2*>(t.keys + bbase + ((start + 4) & (kBucket - 2)));
            const ulonglong2 qd = *reinterpret_cast<const ulonglong2*>(t.keys + bbase + ((start + 6) & (kBucket - 2)));
            const unsigned long long kb = t.keys[kHotSlots + h];
            match |= ((uint32_t)(qb.x == key) << 2) | ((uint32_t)(qb.y == key) << 3);
            empty |= ((uint32_t)(qb.x == 0ull) << 2) | ((uint32_t)(qb.y == 0ull) << 3);
            match |= ((uint32_t)(qc.x == key) << 4) | ((uint32_t)(qc.y == key) << 5) | ((uint32_t)(qd.x == key) << 6) |
                     ((uint32_t)(qd.y == key) << 7);
            empty |= ((uint32_t)(qc.x == 0ull) << 4) | ((uint32_t)(qc.y == 0ull) << 5) | ((uint32_t)(qd.x == 0ull) << 6) |
                     ((uint32_t)(qd.y == 0ull) << 7);
            if (!(match | empty)) {  // a full bucket: the word lives in the big table
                const uint64_t s = kHotSlots + h;
                if (kb == key) return (uint32_t)s;
                return kb == 0ull && table_claim(t, s, key, pos) == key ? (uint32_t)s : kSlotNone;
            }
        }
        return fast ? bucket_resolve(t, match, empty, key, bbase, start, pos) : kSlotNone;
    }
};

// K1b for the chunk of this wave (the kernel body; Probe: HotProbe or DeepProbe in the product).
template <class Probe>
__device__ __forceinline__ void tok_emit_chunk(const uint8_t* __restrict__ text, uint64_t nbytes, uint64_t nch,
                                               const uint64_t* __restrict__ file_start,
                                               uint64_t* __restrict__ chunk_off, uint64_t cap, const Table& tab,
                                               uint64_t* __restrict__ rec, uint32_t* __restrict__ chunk_hist,
                                               uint32_t* __restrict__ pend, uint32_t* __restrict__ pend_cnt,
                                               const uint32_t* __restrict__ cf, LongTok* __restrict__ longs,
                                               uint64_t long_per, uint32_t narrow_keys, uint32_t lbits, uint64_t c,
                                               EmitLds& W) {
    const int l = lane_id();
    const uint64_t chunk_lo = c * kChunk;
    const uint64_t chunk_hi = chunk_lo + kChunk < nbytes ? chunk_lo + kChunk : nbytes;
    // the chunk's files (k_chunk_files), wave-uniform
    const uint32_t f_lo = cf[3 * c], f_hi = cf[3 * c + 1];
    const bool fsame = f_lo == f_hi;
    const bool narrow = chunk_narrow(cap, cf, c, lbits);
    // a chunk over a few files (configs[4]'s small-file shares): the starts of its files after the first,
    // wave-uniform, so that a token's file is a few compares instead of a dependent load per batch
    constexpr uint32_t kFb = 3;
    const bool fsmall = f_hi - f_lo <= kFb;
    uint64_t fb[kFb];
#pragma unroll
    for (uint32_t k = 0; k < kFb; k++) fb[k] = !fsame && f_lo + 1 + k <= f_hi ? file_start[f_lo + 1 + k] : ~0ull;
    const uint64_t cbase = chunk_base(chunk_off, cap, c);
    uint32_t* const rec32 = reinterpret_cast<uint32_t*>(rec + cbase);
    const uint32_t rot = rec_rot(cap, c), wrap = rec_wrap(cap);
    uint32_t out = 0;               // records emitted so far (wave-uniform)
    uint32_t npf = 0, nps = 0;      // tokens left to K1c: fast-path misses, general-path tokens
    const uint64_t pend_end = pend_limit(chunk_off, cap, cbase, c);
    const uint32_t nk_lim = narrow ? narrow_keys : ~0u;  // (a bound held in a register, not a kernel argument re-read per batch)
    if (l < 32) W.hist[l] = 0;
    RoundRegs nxt;
    fetch_round(nxt, text, nbytes, chunk_lo);
    for (uint64_t lo = chunk_lo; lo < chunk_hi; lo += kRound) {
        wave_sync();  // the previous round's readers of W are done
        store_round(W.text, nxt, nbytes, lo);
        // the next round (the last round re-loads its own blocks, cache hits: a
        // conditional fetch would merge registers and wait for the loads here)
        fetch_round(nxt, text, nbytes, lo + kRound < chunk_hi ? lo + kRound : lo);
        wave_sync();
        // 1. kept starts and window masks (windows re-read from LDS: the next
        //    round's bytes are in flight in the registers)
        uint32_t kept[kWin];
        uint32_t cnt = 0;
#pragma unroll
        for (int j = 0; j < kWin; j++) {
            const uint32_t w = 64 * j + l;
            const uint4 v = *reinterpret_cast<const uint4*>(W.text + 16 + 16 * w);
            const Classes cl = classify16(v);
            W.mask[w] = (cl.ws | cl.nul) | (cl.letter << 16);
            const uint32_t prev = W.text[16 + 16 * w - 1];  // byte before the window
            const uint32_t starts = ~cl.ws & ((cl.ws << 1) | (is_ws(prev) ? 1u : 0u)) & 0xFFFFu;
            kept[j] = kept_starts(starts, cl, W.text, text, nbytes, lo, 16 * w, kRoundStaged);
            cnt |= (uint32_t)__popc(kept[j]) << (16 * j);
        }
        if (l == 0) {  // first halo window: masks past the round's last byte
            const Classes ch = classify16(*reinterpret_cast<const uint4*>(W.text + 16 + kRound));
            W.mask[kRoundWins] = (ch.ws | ch.nul) | (ch.letter << 16);
        }
        // 2. token index of every kept start (window j of all lanes before j + 1)
        const uint32_t inc = wave_incl_scan32(cnt);
        const uint32_t ex = inc - cnt;
        const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
        const uint32_t ntok = (tot & 0xFFFFu) + (tot >> 16);
        {
            uint32_t o = ex & 0xFFFFu;
            for (uint32_t m = kept[0]; m; m &= m - 1) W.off[o++] = (uint16_t)(16 * l + __builtin_ctz(m));
            o = (tot & 0xFFFFu) + (ex >> 16);
            for (uint32_t m = kept[1]; m; m &= m - 1) W.off[o++] = (uint16_t)(16 * (64 + l) + __builtin_ctz(m));
        }
        wave_sync();
        const uint32_t pbase = (uint32_t)(lo - chunk_lo);
        // 3. keys + hot-bucket probes, one token per lane, 64 tokens a batch; the
        //    next batch's keys are built (LDS + VALU) while this batch's probe
        //    load is in flight.  (Issuing the next batch's PROBES before
        //    resolving this one measured slower: 13.4 -> 14.6 ms at 10 GB, the
        //    extra registers cost a wave per SIMD.)
        uint32_t p_n = l < ntok ? W.off[l] : 0u;
        TokKey tk_n{0ull, 0u, 0u};
        bool fast_n = l < ntok && round_fast_key(W.text, W.mask, p_n, tk_n);
        for (uint32_t b0 = 0; b0 < ntok; b0 += 64) {
            const uint32_t q = b0 + l;
            const bool valid = q < ntok;
            const uint32_t p = p_n;
            const TokKey tk = tk_n;
            const bool fast = fast_n;
            if (fast) atomicAdd(&W.hist[tk.first], 1u);  // LDS: same-letter lanes serialize in the LDS unit, not in VALU
            const ProbeState pst = Probe().begin(tab, fast, tk.key, hot_slot(tk.key, tab.seed));
            if (b0 + 64 < ntok) {  // (wave-uniform) the next batch's keys
                const uint32_t qn = q + 64;
                p_n = qn < ntok ? W.off[qn] : 0u;
                tk_n = TokKey{0ull, 0u, 0u};
                fast_n = qn < ntok && round_fast_key(W.text, W.mask, p_n, tk_n);
            }
            const uint32_t slot = Probe().finish(tab, pst, fast, tk.key, lo + p);
            const bool resolved = fast && slot != kSlotNone;
            bool pf = fast && !resolved, ps = valid && !fast;
            uint64_t mf = __ballot(pf);
            if (npf + (uint32_t)__popcll(mf) > nk_lim) {  // (wave-uniform, adversarial) no room for
                if (pf) atomicSub(&W.hist[tk.first], 1u);                     // more keys: K1c re-reads them from the
                ps = ps || pf;                                                // text (and counts their letters)
                pf = false;
                mf = 0;
            }
            const uint32_t jr = (out + q + rot) & wrap;  // this token's record in the chunk's slot
            if (resolved) {
                if (narrow && fsame) {  // (wave-uniform) a one-file chunk: the slot
                    rec32[jr] = slot;
                } else {
                    uint32_t f = f_lo;
                    if (fsmall) {
#pragma unroll
                        for (uint32_t k = 0; k < kFb; k++) f += lo + p >= fb[k];
                    } else {
                        f = file_of(file_start, f_lo, f_hi, lo + p);
                    }
                    if (narrow) rec32[jr] = (slot << lbits) | (f - f_lo);
                    else rec[cbase + jr] = ((uint64_t)slot << 32) | f;
                }
            } else if (pf) {
                rec[cbase + (narrow ? kNarrowKeys + npf + lanes_below(mf) : jr)] = tk.key;
            }
            // pending: fast-path misses from the front of the chunk's list, general-path tokens
            // from its back, so that K1c runs each kind without divergence
            const uint64_t ms = __ballot(ps);
            const uint32_t e = (pbase + p) | ((out + q) << 16);
            if (pf) pend[cbase + npf + lanes_below(mf)] = e;
            if (ps) pend[pend_end - 1 - (nps + lanes_below(ms))] = e;
            npf += (uint32_t)__popcll(mf);
            nps += (uint32_t)__popcll(ms);
        }
        out += ntok;
    }
    // 4. K1c: the chunk's pending tokens.  The lanes read entries other lanes
    //    of this wave stored: the stores are complete (vmcnt) before the loads.
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    resolve_pending<false>(text, nbytes, c, file_start, f_lo, f_hi, cbase, wrap, rot, narrow, lbits, pend_end, pend, npf,
                           tab, rec, W.hist, longs, long_per);
    resolve_pending<true>(text, nbytes, c, file_start, f_lo, f_hi, cbase, wrap, rot, narrow, lbits, pend_end, pend, nps,
                          tab, rec, W.hist, longs, long_per);
    wave_sync();
    if (l < 26) chunk_hist[c * 26 + l] = W.hist[l];
    if (l == 0) {
        pend_cnt[c] = npf | (nps << 16);
        if (cap) chunk_off[c] = out;  // fixed-capacity layout: the chunk's token count
    }
}

// K1b.  Launch bound of 8 waves per SIMD: it caps the SGPRs at 78 (52 spilled
// to VGPR lanes); at the compiler's own 106 SGPRs the SGPR file held 7 waves
// per SIMD and the pass ran 12.35 ms instead of 11.70 at 10 GB.
// kKeysArg: the narrow chunks' key capacity comes from the argument (the
// II_NARROW_KEYS test knob); otherwise it is the constant kNarrowKeys (the
// SGPR-capped kernel re-read the argument from memory once per batch).
template <bool kKeysArg, bool kDeep>
__global__ __launch_bounds__(kBlock, 8) void k_tok_emit(const uint8_t* __restrict__ text, uint64_t nbytes, uint64_t nch,
                                                     const uint64_t* __restrict__ file_start,
                                                     uint64_t* __restrict__ chunk_off, uint64_t cap, Table tab,
                                                     uint64_t* __restrict__ rec, uint32_t* __restrict__ chunk_hist,
                                                     uint32_t* __restrict__ pend, uint32_t* __restrict__ pend_cnt,
                                                     const uint32_t* __restrict__ cf, LongTok* __restrict__ longs,
                                                     uint64_t long_per, uint32_t narrow_keys, uint32_t lbits) {
    __shared__ __attribute__((aligned(16))) EmitLds s_lds[kWG];
    const uint32_t w = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // one chunk per wave (waves that loop over chunks, a grid of the resident workgroups: emit 11.46 -> 12.98 ms
    // at 10 GB, same-box A/B)
    const uint64_t c = (uint64_t)blockIdx.x * kWG + w;
    if (c < nch)
        tok_emit_chunk<typename std::conditional<kDeep, DeepProbe, HotProbe>::type>(
            text, nbytes, nch, file_start, chunk_off, cap, tab, rec, chunk_hist, pend, pend_cnt, cf, longs, long_per,
            kKeysArg ? narrow_keys : kNarrowKeys, lbits, c, s_lds[w]);
}

// counters[C_HIST + l] = sum over chunks of chunk_hist[chunk][l]: the
// per-letter totals of the per-chunk letter counts (chunk_hist[c * 26 + l]).
// The grid is a multiple of 13 blocks (256 · 13 threads = 26 · 128), so every
// thread strides over one letter's column (coalesced across the grid), four
// loads in flight; then one LDS and one global add per letter and workgroup;
// counters[C_HIST ..] must be zero on entry.  (416 blocks with one load in
// flight: 64 us for the 63 MB of configs[2]'s 6·10^5 chunks, on the map's
// critical path.)
constexpr uint32_t kHistBlocksMax = 13 * 128;
inline uint32_t hist_blocks(uint64_t nch) {
    const uint64_t want = (nch * 26 + 16 * kBlock - 1) / (16 * kBlock);  // ~16 loads per thread
    const uint64_t b = (want + 12) / 13 * 13;
    return (uint32_t)(b < 13 ? 13 : b > kHistBlocksMax ? kHistBlocksMax : b);
}
__global__ __launch_bounds__(kBlock) void k_hist_reduce(const uint32_t* __restrict__ chunk_hist, uint64_t nch,
                                                        uint64_t* __restrict__ counters) {
    __shared__ unsigned long long s[26];
    if (threadIdx.x < 26) s[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * kBlock, n = nch * 26;
    const uint64_t g = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    uint64_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    uint64_t e = g;
    for (; e + 3 * stride < n; e += 4 * stride) {
        a0 += chunk_hist[e];
        a1 += chunk_hist[e + stride];
        a2 += chunk_hist[e + 2 * stride];
        a3 += chunk_hist[e + 3 * stride];
    }
    for (; e < n; e += stride) a0 += chunk_hist[e];
    atomicAdd(&s[g % 26], (unsigned long long)(a0 + a1 + a2 + a3));
    __syncthreads();
    if (threadIdx.x < 26) atomicAdd((unsigned long long*)&counters[C_HIST + threadIdx.x], s[threadIdx.x]);
}

// number of occupied word-table slots
struct OpOccupied {
    const unsigned long long* keys;
    __device__ uint64_t value(uint64_t i) const { return keys[i] != 0ull; }
    __device__ void emit(uint64_t, uint64_t, uint64_t) const {}
};

// Letter walk of a cleaned word (main.c:105-111) over cached aligned 16-byte
// blocks: one load per block instead of a dependent byte load per letter; the
// block's letter / terminator masks find the next letter without a byte loop.
struct LetterCursor {
    uint64_t g;      // next byte to look at
    uint64_t base;   // cached block (~0: none)
    uint32_t let, term;
    uint4 blk;
    uint32_t n;      // letters returned
    // next letter (0..25), or 26 once the word has ended (whitespace, NUL, end
    // of text — load16 reads it as spaces — or 299 letters)
    __device__ __forceinline__ uint32_t next(const uint8_t* __restrict__ text, uint64_t nbytes) {
        if (n >= (uint32_t)kMaxWord) return 26u;
        for (;;) {
            const uint64_t b = g & ~15ull;
            if (b != base) {
                base = b;
                blk = load16(text, nbytes, (int64_t)b);
                const Classes cl = classify16(blk);
                let = cl.letter;
                term = cl.ws | cl.nul;
            }
            const uint32_t j = (uint32_t)(g & 15u);
            const uint32_t ev = ((let | term) >> j) & 0xFFFFu;
            if (!ev) {
                g = b + 16;
                continue;
            }
            const uint32_t i = j + __builtin_ctz(ev);
            if ((term >> i) & 1u) return 26u;  // ended: g stays at the terminator
            g = b + i + 1;
            n++;
            return letter_of(byte_dyn(blk, i));
        }
    }
};

// byte mask (0xFF per selected byte) of the low 4 bits of m, one bit per byte
__device__ __forceinline__ uint32_t byte_mask4(uint32_t m) { return ((m & 0xFu) * 0x00204081u & 0x01010101u) * 0xFFu; }

// Two tokens whose raw bytes agree up to their last letter (letters compared
// case-insensitively; what follows the last letter is dropped by the cleaning
// loop, main.c:105-111, so trailing punctuation may differ) clean to the same
// word.  Returns 1 = same word, 0 = undecided (the letter walk decides): a
// token that ends in a block where the other does not, or bytes that differ
// before the last letter.  (Comparing up to the first whitespace sent every
// occurrence with a trailing '.', ',' ... — 5 % of the corpus's tokens — to
// the letter walk, which held whole waves.)
__device__ __forceinline__ int same_raw_token(const uint8_t* __restrict__ text, uint64_t nbytes, uint64_t a, uint64_t b) {
    for (uint32_t off = 0; off < 4 * (uint32_t)kMaxWord; off += 16) {
        const uint4 A = global_block16(text, nbytes, a + off), B = global_block16(text, nbytes, b + off);
        const Classes ca = classify16(A), cb = classify16(B);
        const uint32_t ta = ca.ws | ca.nul, tb = cb.ws | cb.nul;
        const uint32_t ea = ta ? __builtin_ctz(ta) : 16u, eb = tb ? __builtin_ctz(tb) : 16u;
        if ((ea == 16u) != (eb == 16u)) return 0;
        uint32_t m = 0xFFFFu;  // bytes that must agree
        const uint32_t la = ca.letter & ((1u << ea) - 1u), lb = cb.letter & ((1u << eb) - 1u);
        if (ea < 16u) {  // both end here: compare up to the last letter (none: the earlier blocks decided)
            const int za = la ? 31 - __builtin_clz(la) : -1, zb = lb ? 31 - __builtin_clz(lb) : -1;
            if (za != zb) return 0;
            m = za < 0 ? 0u : (2u << za) - 1u;
        }
        if ((la ^ lb) & m) return 0;
        const uint32_t wa[4] = {A.x, A.y, A.z, A.w}, wb[4] = {B.x, B.y, B.z, B.w};
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t lowa = wa[k] | (byte_mask4(ca.letter >> (4 * k)) & 0x20202020u);
            const uint32_t lowb = wb[k] | (byte_mask4(cb.letter >> (4 * k)) & 0x20202020u);
            if ((lowa ^ lowb) & byte_mask4(m >> (4 * k))) return 0;
        }
        if (ea < 16u) return 1;
    }
    return 0;
}

constexpr uint32_t kLvBlocks = 128;  // k_long_verify workgroups per queue shard (launched before the counts are known)
static_assert(C_HIST + 26 <= C_LONGMAX, "map_core reads counters [0, C_LONGMAX]");

// Exactness check for hashed keys: every long token must spell the same word
// as its slot's representative occurrence.  Most occurrences repeat the
// representative's bytes (same_raw_token); the rest are walked letter by letter.
// Grid (kLongShards, y): blockIdx.x = the queue shard.
__global__ __launch_bounds__(kBlock) void k_long_verify(const uint8_t* __restrict__ text, uint64_t nbytes,
                                                        const LongTok* __restrict__ longs, uint64_t long_per,
                                                        const uint64_t* __restrict__ rep, uint64_t* counters) {
    // (the shard's count, at most its capacity: the queue may have overflowed, C_OVERFLOW bit 2, and the
    // map retries then; the kernel is launched before the host has looked)
    const uint64_t n = min((unsigned long long)counters[C_LSHARD + 16 * blockIdx.x], (unsigned long long)long_per);
    const LongTok* q = longs + blockIdx.x * long_per;
    for (uint64_t i = (uint64_t)blockIdx.y * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.y * kBlock) {
        LongTok lt = q[i];
        uint64_t a = lt.pos, b = rep[lt.slot];
        if (a == b || same_raw_token(text, nbytes, a, b)) continue;
        LetterCursor ca{a, ~0ull, 0u, 0u, make_uint4(0, 0, 0, 0), 0u}, cb{b, ~0ull, 0u, 0u, make_uint4(0, 0, 0, 0), 0u};
        for (;;) {
            const uint32_t la = ca.next(text, nbytes);
            const uint32_t lb = cb.next(text, nbytes);
            if (la != lb) {
                atomicOr((unsigned long long*)&counters[C_COLLIDE], 1ull);
                break;
            }
            if (la == 26u) break;
        }
    }
}

// Totals of the long-token queue shards: counters[C_LONG] = all queued,
// counters[C_LONGMAX] = the fullest shard.  One wave.
__global__ void k_long_totals(uint64_t* counters) {
    const uint64_t n = counters[C_LSHARD + 16 * lane_id()];
    uint64_t m = n, t = n;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t x = (uint64_t)__shfl_xor((long long)m, o, 64);
        m = x > m ? x : m;
        t += (uint64_t)__shfl_xor((long long)t, o, 64);
    }
    if (lane_id() == 0) {
        counters[C_LONG] = t;
        counters[C_LONGMAX] = m;
    }
}
static_assert(kLongShards == 64, "k_long_totals: one lane per shard");

// Separator contract of ii_map_device: the byte before every file start is
// whitespace (*bad != 0 otherwise).
__global__ void k_check_layout(const uint8_t* __restrict__ text, const uint64_t* __restrict__ file_start, uint32_t nfiles,
                               uint64_t* bad) {
    uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f == 0 || f >= nfiles) return;
    uint64_t s = file_start[f];
    if (s > 0 && !is_ws(text[s - 1])) atomicOr((unsigned long long*)bad, 1ull);
}

// ---------------------------------------------------------------- dictionary
// Scan op: compact occupied table slots into dict_slot[].
// dict_slot[d] = the d-th occupied slot (ascending); rank_hot (optional):
// rank_hot[s] = d for the occupied hot slots (the compact pairs' formatter
// turns a group's first word id into its dense index with it)
struct OpCompactSlots {
    const unsigned long long* keys;
    uint32_t* dict_slot;
    uint32_t* rank_hot;
    __device__ uint64_t value(uint64_t i) const { return keys[i] != 0ull; }
    __device__ void emit(uint64_t i, uint64_t ex, uint64_t v) const {
        if (v) {
            dict_slot[ex] = (uint32_t)i;
            if (rank_hot && i < kHotSlots) rank_hot[i] = (uint32_t)ex;
        }
    }
};

// Lexicographic sort key of each distinct word: first 12 letters packed
// (strcmp order, main.c:63) | 1 if the word is longer than 12 letters.
__global__ __launch_bounds__(kBlock) void k_dict_keys(const uint8_t* __restrict__ text, uint64_t nbytes,
                                                      const unsigned long long* __restrict__ keys,
                                                      const uint64_t* __restrict__ rep,
                                                      const uint32_t* __restrict__ dict_slot, uint32_t V,
                                                      uint64_t* __restrict__ sortkey, uint32_t* __restrict__ idx) {
    uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= V) return;
    uint32_t s = dict_slot[i];
    uint64_t k = keys[s];
    if ((k & 0xFull) == 0) sortkey[i] = k;
    else sortkey[i] = read_word(text, nbytes, rep[s]).prefix | 1ull;
    idx[i] = i;
}

// Letters [12c, 12c+12) of a word, packed like the prefix (0-padded).
__device__ __forceinline__ uint64_t word_chunk(const uint8_t* __restrict__ text, uint64_t nbytes, uint64_t pos, uint32_t c) {
    uint64_t packed = 0;
    uint32_t n = 0;
    const uint32_t lo = 12 * c, hi = lo + 12;
    for (uint64_t g = pos; g < nbytes; g++) {
        uint32_t ch = text[g];
        if (ch == 0u || is_ws(ch)) break;
        uint32_t lc = letter_of(ch);
        if (lc < 26u) {
            if (n >= lo && n < hi) packed |= (uint64_t)(lc + 1) << (64 - 5 * (n - lo + 1));
            n++;
            if (n >= hi || n == (uint32_t)kMaxWord) break;
        }
    }
    return packed;
}

// Tie detection after the prefix sort: words sharing a 12-letter prefix and
// both longer than 12 letters.  run_start[j] = first position of j's run.
__global__ __launch_bounds__(kBlock) void k_tie_mark(const uint64_t* __restrict__ sk, uint32_t V,
                                                     uint32_t* __restrict__ tied, uint64_t* counters) {
    uint32_t j = blockIdx.x * kBlock + threadIdx.x;
    if (j >= V) return;
    bool t = (j > 0 && sk[j] == sk[j - 1]) || (j + 1 < V && sk[j] == sk[j + 1]);
    tied[j] = t;
    if (t) atomicAdd((unsigned long long*)&counters[C_TIES], 1ull);
}

struct OpCompactTied {
    const uint32_t* tied;
    uint32_t* tpos;  // positions of tied entries, ascending
    __device__ uint64_t value(uint64_t i) const { return tied[i]; }
    __device__ void emit(uint64_t i, uint64_t ex, uint64_t v) const {
        if (v) tpos[ex] = (uint32_t)i;
    }
};

// Runs of equal prefix keys inside the tied subset: rid[i] = run of subset
// element i, rfirst[run] = subset index of the run's first element.
struct OpTieRuns {
    const uint32_t* tpos;
    const uint64_t* sk;
    uint32_t* rid;
    uint32_t* rfirst;
    __device__ uint64_t value(uint64_t i) const { return i == 0 || sk[tpos[i]] != sk[tpos[i - 1]]; }
    __device__ void emit(uint64_t i, uint64_t ex, uint64_t v) const {
        rid[i] = (uint32_t)(ex + v - 1);
        if (v) rfirst[ex] = (uint32_t)i;
    }
};

// Subset element i0 (original subset order): its dictionary index and length.
__global__ __launch_bounds__(kBlock) void k_tie_init(const uint8_t* __restrict__ text, uint64_t nbytes,
                                                     const uint32_t* __restrict__ tpos, uint32_t nt,
                                                     const uint32_t* __restrict__ dict_idx,
                                                     const uint32_t* __restrict__ dict_slot, const uint64_t* __restrict__ rep,
                                                     uint32_t* __restrict__ tdict, uint32_t* __restrict__ tval,
                                                     uint64_t* counters) {
    uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= nt) return;
    uint32_t d = dict_idx[tpos[i]];
    tdict[i] = d;
    tval[i] = i;
    uint32_t len = read_word(text, nbytes, rep[dict_slot[d]]).len;
    atomicMax((unsigned long long*)&counters[C_MAXLEN], (unsigned long long)len);
}

// Sort key of the current subset order: letters [12c, 12c+12) (c >= 1), or,
// with c == 0, the subset index of the element's run start.
__global__ __launch_bounds__(kBlock) void k_tie_keys(const uint8_t* __restrict__ text, uint64_t nbytes,
                                                     const uint32_t* __restrict__ tval, uint32_t nt,
                                                     const uint32_t* __restrict__ tdict,
                                                     const uint32_t* __restrict__ dict_slot, const uint64_t* __restrict__ rep,
                                                     const uint32_t* __restrict__ rid, const uint32_t* __restrict__ rfirst,
                                                     uint32_t c, uint64_t* __restrict__ tkey) {
    uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= nt) return;
    uint32_t i0 = tval[i];
    if (c == 0) tkey[i] = rfirst[rid[i0]];
    else tkey[i] = word_chunk(text, nbytes, rep[dict_slot[tdict[i0]]], c);
}

// Subset sorted by (run, chunks 1..K): run r (first subset index s) occupies
// final positions tpos[s] + (i - s).
__global__ __launch_bounds__(kBlock) void k_tie_place(const uint64_t* __restrict__ tkey, const uint32_t* __restrict__ tval,
                                                      uint32_t nt, const uint32_t* __restrict__ tpos,
                                                      const uint32_t* __restrict__ tdict, uint32_t* __restrict__ dict_idx) {
    uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= nt) return;
    uint32_t s = (uint32_t)tkey[i];
    dict_idx[tpos[s] + (i - s)] = tdict[tval[i]];
}

// Per lexicographic id j: remap[slot] = j, the word's key / occurrence / length.
// Word ids for the single-GPU token sort ("wid" keys).  The token sort only
// has to GROUP each word's records (ids ascending); lexicographic order is
// needed per word, not per record.  So records are sorted by a word id that
// costs no gather for hot-table words: wid = the hot slot itself, and for a
// big-table word kHotSlots + its rank among the occupied big slots.  K3 maps
// wid -> lexid once per distinct pair, where consecutive records share the
// word (a coalesced broadcast), instead of sort0 gathering remap[slot] for
// every kept record in text order (random, one L2 request per lane).
// nhot = number of occupied hot slots (dict_slot ascends): *nhot must be 0 on entry.
__global__ __launch_bounds__(kBlock) void k_count_hot(const uint32_t* __restrict__ dict_slot, uint32_t V,
                                                      uint32_t* __restrict__ nhot) {
    const uint32_t d = blockIdx.x * kBlock + threadIdx.x;
    if (d < V && dict_slot[d] < kHotSlots && (d + 1 == V || dict_slot[d + 1] >= kHotSlots)) *nhot = d + 1;
}
// wmap[slot] = wid for the big-table slots: kHotSlots + the slot's rank among
// the occupied big slots (dict_slot ascends; the token sort needs only this)
__global__ __launch_bounds__(kBlock) void k_wid_map(const uint32_t* __restrict__ dict_slot, uint32_t V,
                                                    const uint32_t* __restrict__ nhot, uint32_t* __restrict__ wmap) {
    const uint32_t d = blockIdx.x * kBlock + threadIdx.x;
    if (d >= V) return;
    const uint32_t s = dict_slot[d];
    if (s >= kHotSlots) wmap[s] = (uint32_t)kHotSlots + (d - *nhot);
}
// per lexid j: wid(j) (as k_wid_map); lexw[wid] = j, widl[j] = wid
__global__ __launch_bounds__(kBlock) void k_wid_finish(const uint32_t* __restrict__ dict_idx,
                                                       const uint32_t* __restrict__ dict_slot, uint32_t V,
                                                       const uint32_t* __restrict__ nhot, uint32_t* __restrict__ lexw,
                                                       uint32_t* __restrict__ widl) {
    const uint32_t j = blockIdx.x * kBlock + threadIdx.x;
    if (j >= V) return;
    const uint32_t d = dict_idx[j], s = dict_slot[d];
    const uint32_t wid = s < kHotSlots ? s : (uint32_t)kHotSlots + (d - *nhot);
    lexw[wid] = j;
    widl[j] = wid;
}

__global__ __launch_bounds__(kBlock) void k_lex_finish(const uint8_t* __restrict__ text, uint64_t nbytes,
                                                       const uint32_t* __restrict__ dict_idx,
                                                       const uint32_t* __restrict__ dict_slot,
                                                       const unsigned long long* __restrict__ keys,
                                                       const uint64_t* __restrict__ rep, uint32_t V,
                                                       uint32_t* __restrict__ remap, uint64_t* __restrict__ lex_key,
                                                       uint64_t* __restrict__ lex_rep, uint32_t* __restrict__ lex_len) {
    uint32_t j = blockIdx.x * kBlock + threadIdx.x;
    if (j >= V) return;
    uint32_t s = dict_slot[dict_idx[j]];
    remap[s] = j;
    uint64_t k = keys[s];
    lex_key[j] = k;
    lex_rep[j] = rep[s];
    uint32_t len;
    if ((k & 0xFull) == 0) {
        len = 0;
        while (len < 12 && ((k >> (59 - 5 * len)) & 31ull)) len++;
    } else {
        len = read_word(text, nbytes, rep[s]).len;
    }
    lex_len[j] = len;
}

// letter_start[l] = first lexicographic id whose word starts with letter l.
__global__ __launch_bounds__(kBlock) void k_letter_start(const uint64_t* __restrict__ sk, uint32_t V,
                                                         uint32_t* __restrict__ letter_start) {
    uint32_t j = blockIdx.x * kBlock + threadIdx.x;
    if (j > V) return;
    int lj = j < V ? (int)(sk[j] >> 59) - 1 : 26;
    int lp = j > 0 ? (int)(sk[j - 1] >> 59) - 1 : -1;
    for (int l = lp + 1; l <= lj; l++) letter_start[l] = j;
}

// ---------------------------------------------------------------- K2 first pass
// First pass of the token sort over the records in text order
// (slot << 32 | shard-local file index), one workgroup per contiguous range, tiles of
// kCTile records with the scatter's item mapping:
//  * drops repeated (hot word, file) records: a record whose slot is a
//    hot-table slot and whose file is the tile's epoch file is dropped when
//    the same slot was already kept in this epoch (LDS bitmap, cleared when
//    the epoch changes; the epoch of a tile is the file of the previous
//    tile's last record — what every thread knows after that tile's barrier,
//    so a tile costs one barrier, and two when the file changes).  Only exact
//    duplicates go, and which copy survives does not matter, so K3 still sees
//    every distinct (word, file) pair;
//  * replaces the slot by the word's sort key (remap: lexicographic id, or
//    with kWid the word id — the hot slot itself, remap only for big-table
//    words);
//  * writes the kept records, in order, to kout[lo ...) and counts their
//    pass-0 digit (digit-major table, as k_radix_hist).
// Workgroup b takes the K1b chunks [b * group, (b + 1) * group): virtual
// record indices voff[c0] .. voff[c1] (voff = exclusive scan of the chunk
// token counts), stored at c * cap + (i - voff[c]) in the fixed-capacity
// layout or at i in the dense one (cap == 0).  Its kept records go to
// kout[voff[c0] ...): kept[b] = their number, kept[kMaxChunks + b] =
// voff[c0], the range pass 0's scatter reads back.
// The dedup bitmap covers the whole hot level (1 bit per slot in LDS, 128
// KiB: one 1024-thread workgroup per CU; covering only half of it doubled
// the sort time, and a 64 KiB direct-mapped cache of kept records — two
// workgroups per CU — kept 0.50 T records instead of 0.34 T: the frequent
// words' entries were evicted by the rare ones; round 4: two 512-thread
// workgroups per CU, each reading the range and deduplicating one half of the
// hot slots with a 64 KiB bitmap, 3.9 -> 8.0 ms; the kept records written as
// u32 + top digit instead of u64, 3.9 -> 4.1 ms and the MSD scatter no faster).  The kept records' later
// radix digits are counted here too (dhist, global atomics per workgroup):
// the onesweep passes that follow need only those global counts.
constexpr uint32_t kDedupWords = (uint32_t)(kHotSlots / 32);
constexpr int kCBlock = 1024;                   // 16 waves share one 128 KiB dedup bitmap
constexpr int kS0Items = 8;                     // records per thread per tile (12, 16: spills)
constexpr int kCWaves = kCBlock / 64;
constexpr int kCTile = kS0Items * kCBlock;      // records per tile
constexpr uint32_t kCMaxGroup = 1024;           // K1b chunks per workgroup (LDS offsets)
constexpr int kLaterDigits = 2;                 // digits counted for the onesweep passes
// LDS: 16 KiB counts + 128 KiB bitmap + 4 KiB offsets + 2 KiB later digits: one workgroup per CU

// kWideD: top digits of up to kMsdMaxBits bits (the packed sort's wide MSD
// split, k_msd_scatter): one count row of kMsdMax digits shared by the waves
// (16 per-wave rows would not fit beside the bitmap); rows d <= dmask.
// kHashD (small files: a file's records span fewer than two tiles, so the
// epoch bitmap deduplicated only the records of one file per tile and was
// cleared on nearly every tile): the same 128 KiB hold an open-addressed set
// of kHsSlots u32 entries (file mod 128) << 25 | slot, any slot below 2^25 - 1,
// not only hot ones.  The set is cleared when the epoch has moved 64 files
// past the last clear (ec), so every entry's file lies in [ec, ec + 128) and
// its 7 bits name it; an entry whose file is below the tile's epoch belongs to
// a finished file (files ascend through a range) and is taken over by the next
// record that probes it.  Records outside [epoch, epoch + 64) or with larger
// slots are kept unprobed.  A record is dropped only when its own entry is
// found, i.e. a copy was inserted, and so kept; a full probe sequence keeps the
// record (K3 drops what the first pass keeps twice).  (u64 entries of whole
// records, half as many: 14.1 ms against the bitmap's 8.3 on configs[4]'s
// rank-7 share, most first probes meeting a live entry.)
constexpr uint32_t kHsSlots = kDedupWords;  // u32 entries in the bitmap's LDS
constexpr int kHsProbe = 8;
constexpr int kHsRounds = 2;  // probe rounds batched over a thread's items (the rest: one item at a time)
constexpr uint32_t kHsEmpty = ~0u;
constexpr uint32_t kHsSlotLimit = (1u << 25) - 1u;  // slots below it are probed
constexpr uint32_t kHsFileWin = 64;                 // files past the epoch that are probed
// A narrow chunk's u32 record as slot << 32 | file.  cfid: the chunk's first file f0, bit 31 set
// when the chunk spans several files (record = slot << lbits | file - f0; else the slot).
constexpr uint32_t kCfMulti = 0x80000000u;
__device__ __forceinline__ uint64_t narrow_rec(uint32_t x, uint32_t cfid, uint32_t lbits) {
    const uint32_t lb = (cfid & kCfMulti) ? lbits : 0u;
    return ((uint64_t)(x >> lb) << 32) | ((cfid & ~kCfMulti) + (x & ((1u << lb) - 1u)));
}
// kMulti: the map wrote multi-file narrow chunks (rec_lbits != 0)
template <bool kWid, bool kWideD = false, bool kHashD = false, bool kMulti = false>
__global__ __launch_bounds__(kCBlock, 4) void k_sort0_compact(const uint64_t* __restrict__ keys,
                                                           const uint64_t* __restrict__ voff, uint32_t nch_in,
                                                           uint32_t group, uint64_t cap, int shift, uint32_t dmask,
                                                           uint32_t nchunks, uint64_t* __restrict__ table,
                                                           const uint32_t* __restrict__ remap,
                                                           uint64_t* __restrict__ kout, uint64_t* __restrict__ kept,
                                                           int shift1, int shift2, uint64_t* __restrict__ dhist,
                                                           const uint32_t* __restrict__ cf,
                                                           unsigned long long* __restrict__ narrow_recs, uint32_t lbits,
                                                           const uint32_t* __restrict__ fmap) {
    constexpr int NT = kCBlock, NWv = kCWaves;
    constexpr int kTile = kCTile;
    constexpr uint32_t kBmWords = kDedupWords;
    constexpr int kCntRows = kWideD ? 1 : NWv;
    constexpr int kCntD = kWideD ? kMsdMax : kRadix;
    __shared__ uint32_t cnt[kCntRows][kCntD];
    __shared__ uint32_t bm[kBmWords];  // the bitmap, or (kHashD) the set
    __shared__ uint32_t s_voff[kCMaxGroup + 1];  // voff[c0 + i] - voff[c0] (< group * kChunkCap)
    __shared__ uint32_t s_cfid[kCMaxGroup];      // narrow chunk: its first file (| kCfMulti: several); ~0: u64 records
    __shared__ uint32_t s_later[kLaterDigits][kRadix];
    __shared__ uint32_t s_wtot[2][NWv];          // per tile parity: one barrier per tile
    __shared__ uint32_t s_last[2];               // per tile parity: file of the tile's last record
    const int w = wave_id(), l = lane_id();
    const uint32_t c0 = blockIdx.x * group, ng = c0 + group < nch_in ? group : nch_in - c0;
    for (int i = threadIdx.x; i < kCntRows * kCntD; i += NT) (&cnt[0][0])[i] = 0;
    for (int i = threadIdx.x; i < kLaterDigits * kRadix; i += NT) (&s_later[0][0])[i] = 0;
    for (uint32_t i = threadIdx.x; i < kBmWords; i += NT) bm[i] = kHashD ? kHsEmpty : 0u;
    const uint64_t lo = voff[c0], hi = voff[c0 + ng];
    for (uint32_t i = threadIdx.x; i <= ng; i += NT) s_voff[i] = (uint32_t)(voff[c0 + i] - lo);
    for (uint32_t i = threadIdx.x; i < ng; i += NT)
        s_cfid[i] = chunk_narrow(cap, cf, c0 + i, lbits)
                        ? cf[3 * (c0 + i) + 2] | (kMulti && cf[3 * (c0 + i) + 1] != cf[3 * (c0 + i)] ? kCfMulti : 0u)
                        : ~0u;
    __syncthreads();
    if (narrow_recs && w == 0) {  // records of this range read as u32 (narrow chunks): the pass's honest read bytes
        uint32_t nr = 0;
        for (uint32_t i = l; i < ng; i += 64) nr += s_cfid[i] != ~0u ? s_voff[i + 1] - s_voff[i] : 0u;
        nr = wave_sum32(nr);
        if (l == 0 && nr) atomicAdd(narrow_recs, (unsigned long long)nr);
    }
    const uint64_t tofs = (uint64_t)w * 64 * kS0Items + l;
    const uint64_t lt = lanemask_lt();
    // this lane's chunk cursor (its indices only grow), all in registers so a
    // record's address needs no LDS round trip unless it enters a new chunk
    uint32_t g = 0;
    uint32_t gnext = s_voff[1];                      // first WG-relative index past chunk g
    uint32_t gadj = chunk_rot(c0);                   // rot(chunk) - chunk start
    uint64_t gbase = (uint64_t)c0 * cap;
    uint32_t gfid = ng ? s_cfid[0] : ~0u;            // narrow chunk's file (~0: u64 records)
    uint64_t o = lo;  // next output position
    // The next tile's records are loaded while this one is written: issued
    // after this tile's remap gathers have been consumed (vmcnt is in order, so
    // a prefetch issued before them would make the gathers wait for it).
    // A narrow chunk's record is the u32 half (nodd bit) of the u64 loaded, its
    // file the chunk's (nfid); one load form for both kinds, so the loads stay
    // in flight (a branch between two load forms would wait for them).
    uint64_t nraw[kS0Items];
    uint32_t nfid[kS0Items];  // narrow item: its chunk's file id; ~0: a u64 record
    uint32_t nodd = 0;
    auto load_tile = [&](uint64_t tb) {
        nodd = 0;
#pragma unroll
        for (int k = 0; k < kS0Items; k++) {
            const uint64_t idx = tb + tofs + (uint64_t)k * 64;
            uint64_t src = idx;
            nfid[k] = ~0u;
            if (cap && idx < hi) {
                const uint32_t ri = (uint32_t)(idx - lo);
                if (ri >= gnext) {
                    uint32_t gs;
                    do {
                        gs = gnext;
                        gnext = s_voff[++g + 1];
                    } while (ri >= gnext);
                    gadj = chunk_rot(c0 + g) - gs;
                    gbase = (uint64_t)(c0 + g) * cap;
                    gfid = s_cfid[g];
                }
                const uint32_t j = (ri + gadj) & (uint32_t)(kChunkCap - 1);
                nfid[k] = gfid;
                const bool nw = gfid != ~0u;
                nodd |= (uint32_t)(nw && (j & 1u)) << k;
                src = gbase + (nw ? j >> 1 : j);
            }
            nraw[k] = idx < hi ? ld_nt(keys + src) : 0ull;
        }
    };
    if (lo < hi) load_tile(lo);
    // the first tile's epoch: the file of the range's first record (every lane loads it)
    uint32_t epoch = lo >= hi ? 0u
                   : s_cfid[0] != ~0u
                       ? (uint32_t)narrow_rec(reinterpret_cast<const uint32_t*>(keys + (uint64_t)c0 * cap)[chunk_rot(c0)],
                                              s_cfid[0], lbits)
                       : (uint32_t)keys[cap ? (uint64_t)c0 * cap + chunk_rot(c0) : lo];
    uint32_t par = 0;
    uint32_t ec = epoch;  // kHashD: the epoch of the set's last clear
    for (uint64_t tb = lo; tb < hi; tb += kTile, par ^= 1u) {
        uint64_t raw[kS0Items];
#pragma unroll
        for (int k = 0; k < kS0Items; k++)
            raw[k] = nfid[k] == ~0u ? nraw[k]
                     : kMulti       ? narrow_rec((uint32_t)(nraw[k] >> (32 * ((nodd >> k) & 1u))), nfid[k], lbits)
                                    : ((nraw[k] >> (32 * ((nodd >> k) & 1u))) << 32) | nfid[k];
        if (tb != lo && s_last[par ^ 1u] != epoch) {  // (workgroup-uniform) a new file: clear the bitmap
            epoch = s_last[par ^ 1u];
            if (!kHashD || epoch - ec >= kHsFileWin) {  // (kHashD: every 64 files)
                for (uint32_t i = threadIdx.x; i < kBmWords; i += NT) bm[i] = kHashD ? kHsEmpty : 0u;
                ec = epoch;
                __syncthreads();
            }
        }
        uint32_t hkeep = 0;  // kHashD: the items the set keeps
        if (kHashD) {
            // first probes of all items at once (one LDS round trip for the loads, one for the
            // CASes); the rest of a probe sequence, per item, only where another record took the entry
            // (the entry index is recomputed where it is used: holding it spilled)
            auto hs_of = [](uint32_t q) { return (q * 0x9E3779B1u) >> (32 - 15); };
            static_assert(kHsSlots == 1u << 15, "hs_of yields 15 bits");
            // an entry is free, or a finished file's: its file (ec + its 7 bits mod 128) below the epoch
            auto hs_free = [&](uint32_t x) { return x == kHsEmpty || ec + (((x >> 25) - ec) & 127u) < epoch; };
            uint32_t q[kS0Items], live = 0, slow = 0;
            uint32_t e[kS0Items];
#pragma unroll
            for (int k = 0; k < kS0Items; k++) {
                const uint32_t f = (uint32_t)raw[k], sl = (uint32_t)(raw[k] >> 32);
                q[k] = ((f & 127u) << 25) | sl;
                e[k] = kHsEmpty;
                if (tb + tofs + (uint64_t)k * 64 < hi) {
                    if (sl < kHsSlotLimit && f - epoch < kHsFileWin) {
                        live |= 1u << k;
                        e[k] = __hip_atomic_load(&bm[hs_of(q[k])], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    } else {
                        hkeep |= 1u << k;  // not probed: kept
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < kS0Items; k++) {
                if (!((live >> k) & 1u) || e[k] == q[k]) continue;  // a copy was inserted (and kept)
                if (hs_free(e[k])) {
                    const uint32_t o = atomicCAS(&bm[hs_of(q[k])], e[k], q[k]);
                    if (o == e[k]) hkeep |= 1u << k;      // inserted: keep
                    else if (o != q[k]) slow |= 1u << k;  // another record took it: probe on
                } else {
                    slow |= 1u << k;
                }
            }
            if (slow) {  // second round, batched like the first: the next entry of every item passed on
                uint32_t s2 = 0;
#pragma unroll
                for (int k = 0; k < kS0Items; k++)
                    if ((slow >> k) & 1u)
                        e[k] = __hip_atomic_load(&bm[(hs_of(q[k]) + 1u) & (kHsSlots - 1)], __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
                for (int k = 0; k < kS0Items; k++) {
                    if (!((slow >> k) & 1u) || e[k] == q[k]) continue;
                    if (hs_free(e[k])) {
                        const uint32_t o = atomicCAS(&bm[(hs_of(q[k]) + 1u) & (kHsSlots - 1)], e[k], q[k]);
                        if (o == e[k]) hkeep |= 1u << k;
                        else if (o != q[k]) s2 |= 1u << k;
                    } else {
                        s2 |= 1u << k;
                    }
                }
                slow = s2;
            }
            while (slow) {  // (one item at a time from entry + kHsRounds, selected without indexing the arrays)
                const int k = __builtin_ctz(slow);
                slow &= slow - 1u;
                uint32_t qk = q[0];
#pragma unroll
                for (int j = 1; j < kS0Items; j++) qk = j == k ? q[j] : qk;
                uint32_t hh = (hs_of(qk) + (uint32_t)kHsRounds) & (kHsSlots - 1);
                bool keepk = true;  // a full probe sequence keeps the record
                for (int p = kHsRounds; p < kHsProbe; p++) {
                    const uint32_t x = __hip_atomic_load(&bm[hh], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (x == qk) {
                        keepk = false;
                        break;
                    }
                    if (hs_free(x)) {
                        const uint32_t o = atomicCAS(&bm[hh], x, qk);
                        if (o == x) break;
                        if (o == qk) {
                            keepk = false;
                            break;
                        }
                        continue;  // taken meanwhile: look at it again
                    }
                    hh = (hh + 1) & (kHsSlots - 1);
                }
                hkeep |= (uint32_t)keepk << k;
            }
        }
        uint32_t keep = 0, wcount = 0;
        uint32_t pos[kS0Items];
#pragma unroll
        for (int k = 0; k < kS0Items; k++) {
            bool ok = tb + tofs + (uint64_t)k * 64 < hi;
            const uint64_t slot = raw[k] >> 32;
            if (kHashD) {
                ok = ok && ((hkeep >> k) & 1u);
            } else if (ok && slot < kHotSlots && (uint32_t)raw[k] == epoch) {
                const uint32_t bit = 1u << (slot & 31);
                ok = !(atomicOr(&bm[slot >> 5], bit) & bit);
            }
            const uint64_t b = __ballot(ok);
            pos[k] = wcount + (uint32_t)__popcll(b & lt);
            wcount += (uint32_t)__popcll(b);
            keep |= (uint32_t)ok << k;
        }
        // the tile's last record (thread NT - 1, item kS0Items - 1; or the range's last)
        const uint64_t last = tb + kTile < hi ? tb + kTile - 1 : hi - 1;
#pragma unroll
        for (int k = 0; k < kS0Items; k++)
            if (tb + tofs + (uint64_t)k * 64 == last) s_last[par] = (uint32_t)raw[k];  // (the low half is the file)
        // slot -> sort key, in place; with fmap the shard-local file index -> id0 too (a tile's
        // records come from a few neighbouring files, so these gathers hit the same lines, where
        // K3's, in word order, missed L1 on nearly every pair; the record-set form only)
        if (kHashD && fmap) {
#pragma unroll
            for (int k = 0; k < kS0Items; k++)
                if ((keep >> k) & 1u) {
                    const uint32_t slot = (uint32_t)(raw[k] >> 32);
                    const uint32_t key = (kWid && slot < kHotSlots) ? slot : remap[slot];
                    raw[k] = ((uint64_t)key << 32) | fmap[(uint32_t)raw[k]];
                }
        } else {
#pragma unroll
            for (int k = 0; k < kS0Items; k++)
                if ((keep >> k) & 1u) {
                    const uint32_t slot = (uint32_t)(raw[k] >> 32);
                    // wid keys: only big-table words need the map (remap = wmap)
                    const uint32_t key = (kWid && slot < kHotSlots) ? slot : remap[slot];
                    raw[k] = ((uint64_t)key << 32) | (raw[k] & 0xFFFFFFFFull);
                }
        }
        if (l == 0) s_wtot[par][w] = wcount;
        // the record set (small files): the next tile's loads go out before the barrier, in flight while
        // the wave waits there (rank 7 of configs[4]: first pass 8.84 -> 8.19 ms, 214.0 -> 217.0 GB/s;
        // the bitmap form at config3 got slower, 3.83 -> 4.18 ms, and issues them after it)
        if (kHashD && tb + kTile < hi) load_tile(tb + kTile);
        __syncthreads();  // (s_wtot[par] and s_last[par] are rewritten two tiles later, after the next barrier)
        uint32_t wbase = 0, ttot = 0;
#pragma unroll
        for (int ww = 0; ww < NWv; ww++) {
            const uint32_t c = s_wtot[par][ww];
            if (ww < w) wbase += c;
            ttot += c;
        }
        if (!kHashD && tb + kTile < hi) load_tile(tb + kTile);
#pragma unroll
        for (int k = 0; k < kS0Items; k++) {
            if ((keep >> k) & 1u) {
                const uint64_t r = raw[k];
                st_nt(kout + o + wbase + pos[k], r);
                atomicAdd(&cnt[kWideD ? 0 : w][(uint32_t)(r >> shift) & dmask], 1u);
                if (dhist) {
                    atomicAdd(&s_later[0][(uint32_t)(r >> shift1) & dmask], 1u);
                    atomicAdd(&s_later[1][(uint32_t)(r >> shift2) & dmask], 1u);
                }
            }
        }
        o += ttot;
    }
    __syncthreads();
    for (int d = threadIdx.x; d < (kWideD ? (int)dmask + 1 : kRadix); d += NT) {
        uint32_t tt = 0;
#pragma unroll
        for (int ww = 0; ww < kCntRows; ww++) tt += cnt[ww][d];
        table[(uint64_t)d * nchunks + blockIdx.x] = tt;
        if (kWideD) continue;  // (no later digits: the packed sort only)
        if (dhist) {
            if (s_later[0][d]) atomicAdd((unsigned long long*)&dhist[d], (unsigned long long)s_later[0][d]);
            if (s_later[1][d]) atomicAdd((unsigned long long*)&dhist[kRadix + d], (unsigned long long)s_later[1][d]);
        }
    }
    if (threadIdx.x == 0) {
        kept[blockIdx.x] = o - lo;
        kept[kMaxChunks + blockIdx.x] = lo;
    }
}

// ---------------------------------------------------------------- K2 support
// slot -> lexicographic id in the record's high word.
__global__ __launch_bounds__(kBlock) void k_remap(uint64_t* __restrict__ rec, uint64_t n, const uint32_t* __restrict__ remap) {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock) {
        uint64_t r = rec[i];
        rec[i] = ((uint64_t)remap[r >> 32] << 32) | (r & 0xFFFFFFFFull);
    }
}

// ---------------------------------------------------------------- K3 unique + posting bytes
// Records sorted by (lexid, file): the first of each equal run is a distinct
// (word, file) pair (main.c:176-184, add_number main.c:67-77); its posting
// "id0+1" takes its digits + 1 bytes (the following ' ' or ']',
// main.c:228-234).  One reduce-then-scan yields both prefixes: uniq[u] = the
// pair, P[u] = byte offset of its posting (P[p] - P[post_start[w]] is the
// offset inside word w's list; written only at word starts and u % 64 == 0,
// the entries k_fmt_words / k_fmt_posts read) and post_start[lexid] = the
// word's first pair.
constexpr int kUniqItems = 4;                        // records per thread per tile
constexpr int kUniqTile = kUniqItems * kBlock;       // item q of thread t: tile base + q * kBlock + t (coalesced)
static_assert(kUniqItems == 4, "per-item prefixes travel as 8-bit (flags) and 16-bit (bytes) fields");

// id0 of a record's file: the records of a map carry shard-local file indices
// (k_chunk_files); fmap = the mapped files' id0s, or null when index == id0
// (the file table is 0, 1, 2, ...; the owners' merged pairs carry id0s).
// K3 (k_uniq_sweep<kPacked, kFmap>) gathers fmap[f] only in its kFmap instance;
// many small files with scattered ids (configs[4]'s rank-7 share) skip it: their
// first pass already wrote id0s (k_sort0_compact's fmap, local_reduce).

// digits of v = id0 + 1 <= 2^32 (1..10), branch-free
__device__ __forceinline__ uint32_t id_digits(uint64_t v) {
    return 1u + (v >= 10ull) + (v >= 100ull) + (v >= 1000ull) + (v >= 10000ull) + (v >= 100000ull) +
           (v >= 1000000ull) + (v >= 10000000ull) + (v >= 100000000ull) + (v >= 1000000000ull);
}
// Posting bytes of a pair by its shard-local file index f (ids ascend with f):
// t[k - 1] = the first index whose id0 + 1 has more than k digits, so the bytes
// (separator + digits of id0 + 1) follow from nine compares instead of a
// gather of fmap[f] — K3 publishes its tile aggregate without waiting for
// the gathers (configs[4]'s rank-7 share: 4.4·10^5 files, a 1.8 MB fmap that
// misses L1 on every pair).
struct IdDigitsTh {
    uint32_t t[9];
};
__device__ __forceinline__ uint32_t pair_bytes(const uint32_t* __restrict__ fmap, const IdDigitsTh& th, uint32_t f) {
    if (!fmap) return id_digits((uint64_t)f + 1) + 1;
    uint32_t d = 2;
#pragma unroll
    for (int k = 0; k < 9; k++) d += f >= th.t[k];
    return d;
}

// 8-bit fields -> 16-bit fields of a u64
__device__ __forceinline__ uint64_t field8_spread(uint32_t x) {
    return (uint64_t)(x & 0xFFu) | (uint64_t)((x >> 8) & 0xFFu) << 16 | (uint64_t)((x >> 16) & 0xFFu) << 32 |
           (uint64_t)(x >> 24) << 48;
}

// K3's block exclusive scan of a thread's pair flags (c8: one 8-bit field per
// item, a wave sums at most 64 in a field) and posting bytes (bl / bh: 16-bit
// fields of items 0-1 / 2-3, at most 64 * 11 per wave): three DPP wave scans
// (ii_prims.h wave_incl_scan32) instead of two u64 shuffle scans, then the
// waves' totals through LDS.  Returns 16-bit fields (no carries: a block field
// sums at most kBlock * 11) and the block totals.
__device__ __forceinline__ void uniq_block_scan(uint32_t c8, uint32_t bl, uint32_t bh, uint64_t& ec, uint64_t& eb,
                                                uint64_t& tc, uint64_t& tb, uint64_t* lds /*2*kWaves*/) {
    const uint64_t ic = field8_spread(wave_incl_scan32(c8));
    const uint64_t ib = (uint64_t)wave_incl_scan32(bl) | (uint64_t)wave_incl_scan32(bh) << 32;
    if (lane_id() == 63) {
        lds[wave_id()] = ic;
        lds[kWaves + wave_id()] = ib;
    }
    __syncthreads();
    uint64_t wa = 0, wb = 0;
    tc = tb = 0;
#pragma unroll
    for (int w = 0; w < kWaves; w++) {
        const uint64_t sa = lds[w], sb = lds[kWaves + w];
        if (w < wave_id()) {
            wa += sa;
            wb += sb;
        }
        tc += sa;
        tb += sb;
    }
    __syncthreads();
    ec = wa + ic - field8_spread(c8);
    eb = wb + ib - ((uint64_t)bl | (uint64_t)bh << 32);
}

// Compact pairs (uniq32 != null; the index is formatted, not exported): K3
// writes each pair as the u32 id0 | kPairFirst when it starts its word, and
// g64[u / 64] = the word key of pair u at every multiple of 64 — half the
// bytes of the u64 pairs for K3 to write and the formatter to read.  The
// words come in key order and every word has a pair, so a pair's word is its
// group's first word plus the word starts between them (k_fmt_posts<true>).
constexpr uint32_t kPairFirst = 0x80000000u;

// K3 in one pass (decoupled look-back, as k_onesweep): a workgroup takes a
// tile of kUniqSub sub-tiles (kUniqTile records each) from a ticket, scans
// them, publishes the tile's distinct
// pairs and posting bytes (two 8-byte granules: epoch << 40 | flag | value),
// walks back over the earlier tiles' granules for its starting pair index
// and byte offset, and writes uniq / P / post_start / post_end.  The records
// are read once instead of twice.  The last tile also writes the totals:
// *U_out = distinct pairs, *B_out = posting bytes.
constexpr int kUniqSub = 4;  // 1, 2, 8 sub-tiles: 5.65, 3.51, 4.83 ms against 2.94 at 10 GB (ticket rate, occupancy)
constexpr int kUniqSweepTile = kUniqSub * kUniqTile;  // 4096 records
// kPacked: the records come from the packed token sort (k_onesweep_seg, u32
// low << pack_f | id in tile-padded buckets, ii_prims.h): K3 tile `tile` lies
// in sort tile tile / 2, so in one bucket h; its valid records end at the
// bucket's count, the word id is h << lowbits | low, and the first record of a
// bucket has no predecessor (a bucket's words differ from every other
// bucket's).  The last record of each bucket closes its word (post_end),
// which the dense form leaves to the next word's start and k_post_last.
static_assert(kSweepTile == 2 * kUniqSweepTile, "K3 tile = half a packed-sort tile");
// kFmap: the records carry shard-local file indices (fmap != null; the
// launcher picks kFmap = false only for fmap == null, index == id0): their id0s
// are gathered for all sub-tiles at once, before the look-back (the gathers
// miss L1 for a share of 4·10^5 files and were one dependent round trip per
// sub-tile in the write phase).
template <bool kPacked, bool kFmap = false>
__global__ __launch_bounds__(kBlock, kPacked ? 8 : 4) void k_uniq_sweep(const uint64_t* __restrict__ rec, uint64_t n,
                                                       const uint32_t* __restrict__ rec32, uint64_t ncap,
                                                       const uint32_t* __restrict__ btile,
                                                       const uint16_t* __restrict__ tbk,
                                                       const uint64_t* __restrict__ bstart, uint32_t nb, int pack_f,
                                                       int lowbits, uint64_t* __restrict__ uniq, uint64_t* __restrict__ P,
                                                       uint64_t* __restrict__ post_start, uint64_t* __restrict__ post_end,
                                                       uint64_t* __restrict__ status, uint32_t* __restrict__ ticket,
                                                       uint64_t epoch, uint64_t* __restrict__ U_out,
                                                       uint64_t* __restrict__ B_out, unsigned long long* __restrict__ err,
                                                       const uint32_t* __restrict__ fmap, uint32_t* __restrict__ uniq32,
                                                       uint32_t* __restrict__ g64, IdDigitsTh dth, uint32_t fid_off) {
    // the tile staged in LDS (scanned, then written after the look-back): u64
    // records from [1] with the record before the tile at [0], or in the packed
    // form the raw u32 records (16 KiB, 8 workgroups per CU instead of 3) and
    // the record before the tile apart
    __shared__ uint64_t s_rec[kPacked ? 1 : kUniqSweepTile + 1];
    __shared__ uint32_t s_raw[kPacked ? kUniqSweepTile : 1];
    __shared__ uint64_t s_prev;
    __shared__ uint64_t lds[2 * kWaves];
    __shared__ uint64_t s_tot[kUniqSub][2];  // per sub-tile: pair / byte totals (16-bit fields)
    __shared__ uint64_t s_base[2];
    __shared__ uint32_t s_tile;
    constexpr int kPer = kUniqSweepTile / kBlock;
    const int t = threadIdx.x;
    // a sort pass before this one that flagged kLbTimeout left records out of place (their keys may
    // lie past the word range): every workgroup leaves before its ticket, and the host, which reads
    // the flags with U, returns II_ERR_INTERNAL.  (The flag's load is in flight with the ticket.)
    if (t == 0) {
        const unsigned long long e0 = *err;
        const uint32_t tk = atomicAdd(ticket, 1u);
        s_tile = (e0 & kLbTimeout) ? ~0u : tk;
    }
    __syncthreads();
    if (s_tile == ~0u) return;
    const uint64_t tile = (uint32_t)__builtin_amdgcn_readfirstlane(s_tile);
    const uint64_t lo = tile * kUniqSweepTile;
    uint64_t ntiles, hi, first = 0, vend = 0;
    uint32_t h = 0;
    const uint32_t idmask = kPacked ? (1u << pack_f) - 1u : 0u;
    auto unpack = [&](uint32_t x) -> uint64_t {
        return ((uint64_t)((h << lowbits) | (x >> pack_f)) << 32) | (x & idmask);
    };
    if (kPacked) {
        // the loads first (their addresses do not depend on the bucket; ncap bounds the padded layout's
        // allocation), the bucket's bounds while they are in flight: a chain of loads before them made
        // the tiles publish late and K3 ran 1.6x longer
        uint32_t raw[kPer];
#pragma unroll
        for (int j = 0; j < kPer; j++) {
            const uint64_t i = lo + (uint64_t)j * kBlock + t;
            raw[j] = i < ncap ? rec32[i] : 0u;
        }
        const uint32_t rprev = (t == 0 && lo > 0 && lo <= ncap) ? rec32[lo - 1] : 0u;
        ntiles = 2ull * btile[nb];
        if (tile >= ntiles) return;  // (workgroup-uniform) a spare workgroup of the launch's upper bound
        h = (uint32_t)__builtin_amdgcn_readfirstlane(tbk[tile / 2]);
        first = (uint64_t)btile[h] * kSweepTile;
        vend = first + (bstart[h + 1] - bstart[h]);
        hi = lo + kUniqSweepTile < vend ? lo + kUniqSweepTile : vend;
        hi = hi < lo ? lo : hi;
#pragma unroll
        for (int j = 0; j < kPer; j++) s_raw[j * kBlock + t] = raw[j];
        if (t == 0) s_prev = (lo > first && lo < vend) ? unpack(rprev) : ~0ull;
    } else {
        ntiles = (n + kUniqSweepTile - 1) / kUniqSweepTile;
        hi = lo + kUniqSweepTile < n ? lo + kUniqSweepTile : n;
        uint64_t v[kPer];
#pragma unroll
        for (int j = 0; j < kPer; j++) {
            const uint64_t i = lo + (uint64_t)j * kBlock + t;
            v[j] = i < hi ? rec[i] : ~0ull;
        }
#pragma unroll
        for (int j = 0; j < kPer; j++) s_rec[1 + j * kBlock + t] = v[j];
        if (t == 0) s_rec[0] = lo > 0 ? rec[lo - 1] : ~0ull;
    }
    __syncthreads();
    // item (k, q) of this thread: tile index k * kUniqTile + q * kBlock + t
    // (coalesced); pv = the record before it (~0: none).  Past hi the packed
    // form's values are padding, never flagged (the i < hi tests below).
    auto item = [&](int k, int q, uint64_t& r, uint64_t& pv) {
        const uint32_t x = (uint32_t)(k * kUniqTile + q * kBlock + t);
        if (kPacked) {
            r = unpack(s_raw[x]);
            pv = x == 0 ? s_prev : unpack(s_raw[x - 1]);
        } else {
            r = s_rec[1 + x];
            pv = s_rec[x];
        }
    };
    // 1. every item's flag and posting bytes (per sub-tile: 8-bit flag fields, 16-bit byte
    //    fields), kept in registers selected by the (uniform) sub-tile index — the loops
    //    stay rolled, so the LDS reads of all sub-tiles are not hoisted together
    static_assert(kUniqSub == 4, "four register slots");
    uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0, l0 = 0, l1 = 0, l2 = 0, l3 = 0, h0 = 0, h1 = 0, h2 = 0, h3 = 0;
    uint32_t tcount = 0, tbytes = 0;  // this thread's pairs / posting bytes
#pragma unroll 1
    for (int k = 0; k < kUniqSub; k++) {
        uint32_t c8 = 0, bl = 0, bh = 0;
#pragma unroll
        for (int q = 0; q < kUniqItems; q++) {
            uint64_t r, pv;
            item(k, q, r, pv);
            const uint64_t i = lo + (uint64_t)k * kUniqTile + (uint64_t)q * kBlock + t;
            if (i < hi && r != pv) {  // (pv = ~0 before the first record: never a record)
                c8 |= 1u << (8 * q);
                const uint32_t d = pair_bytes(kFmap ? fmap : nullptr, dth, (uint32_t)r + (kFmap ? 0u : fid_off));
                if (q < 2) bl += d << (16 * q);
                else bh += d << (16 * (q - 2));
                tcount++;
                tbytes += d;
            }
        }
        c0 = k == 0 ? c8 : c0; c1 = k == 1 ? c8 : c1; c2 = k == 2 ? c8 : c2; c3 = k == 3 ? c8 : c3;
        l0 = k == 0 ? bl : l0; l1 = k == 1 ? bl : l1; l2 = k == 2 ? bl : l2; l3 = k == 3 ? bl : l3;
        h0 = k == 0 ? bh : h0; h1 = k == 1 ? bh : h1; h2 = k == 2 ? bh : h2; h3 = k == 3 ? bh : h3;
    }
    // 2. the tile's totals (one block reduction) and its aggregate published at once, before
    //    the sub-tile scans: later tiles' look-backs sum it instead of waiting for them
    {
        const uint32_t wc = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan32(tcount), 63);
        const uint32_t wb = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan32(tbytes), 63);
        if (lane_id() == 0) {
            lds[wave_id()] = wc;
            lds[kWaves + wave_id()] = wb;
        }
    }
    __syncthreads();
    uint64_t C = 0, B = 0;
#pragma unroll
    for (int w = 0; w < kWaves; w++) {
        C += lds[w];
        B += lds[kWaves + w];
    }
    const uint64_t ep = epoch << 40;
    if (t == 0 || t == 32)
        __hip_atomic_store(status + 2 * tile + (t >> 5), ep | (tile == 0 ? kLbFlagP : kLbFlagA) | (t == 0 ? C : B),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();  // (lds is reused by the scans)
    // 3. per sub-tile: this thread's exclusive pair / byte offsets (16-bit fields)
    uint64_t exc0 = 0, exc1 = 0, exc2 = 0, exc3 = 0, exb0 = 0, exb1 = 0, exb2 = 0, exb3 = 0;
#pragma unroll 1
    for (int k = 0; k < kUniqSub; k++) {
        const uint32_t c8 = k == 0 ? c0 : k == 1 ? c1 : k == 2 ? c2 : c3;
        const uint32_t bl = k == 0 ? l0 : k == 1 ? l1 : k == 2 ? l2 : l3;
        const uint32_t bh = k == 0 ? h0 : k == 1 ? h1 : k == 2 ? h2 : h3;
        uint64_t ec, eb, tc, tb;
        uniq_block_scan(c8, bl, bh, ec, eb, tc, tb, lds);
        const uint64_t fc = ec | field8_spread(c8) << 15;  // the item's own flag rides in bit 15 of its field
        exc0 = k == 0 ? fc : exc0;
        exc1 = k == 1 ? fc : exc1;
        exc2 = k == 2 ? fc : exc2;
        exc3 = k == 3 ? fc : exc3;
        exb0 = k == 0 ? eb : exb0;
        exb1 = k == 1 ? eb : exb1;
        exb2 = k == 2 ? eb : exb2;
        exb3 = k == 3 ? eb : exb3;
        if (t == 0) {
            s_tot[k][0] = tc;
            s_tot[k][1] = tb;
        }
    }
    uint32_t gid[kUniqSub * kUniqItems];  // kFmap: every flagged item's id0 (in flight during the look-back)
#pragma unroll
    for (int k = 0; k < kUniqSub; k++) {
        const uint64_t ec = k == 0 ? exc0 : k == 1 ? exc1 : k == 2 ? exc2 : exc3;
#pragma unroll
        for (int q = 0; q < kUniqItems; q++) {
            gid[k * kUniqItems + q] = 0u;
            if (kFmap && ((ec >> (16 * q)) & 0x8000ull)) {
                uint64_t r, pv;
                item(k, q, r, pv);
                gid[k * kUniqItems + q] = fmap[(uint32_t)r];
            }
        }
    }
    // look-back, wave 0: lanes 0..31 walk the pair counts, lanes 32..63 the
    // byte counts, each half loading the granules of 32 earlier tiles per
    // round trip (walking one tile per round trip, the walk fell behind the
    // rate at which tiles start, so every tile walked far; 128 per round trip,
    // four granules a lane, measured slower in round 4: K3 1.55 -> 1.71 ms)
    if (t < 64) {
        const uint32_t f = (uint32_t)t >> 5, j = (uint32_t)t & 31u;  // field, distance - 1 of the tile this lane loads
        const uint64_t v0 = f == 0 ? C : B;  // (the aggregate is published above)
        uint64_t excl = 0;
        bool done = tile == 0;
        for (int64_t base = (int64_t)tile - 1; __ballot(!done) != 0; base -= 32) {
            uint64_t v = ep | kLbFlagP;  // before tile 0: an inclusive prefix of 0
            const int64_t p = base - (int64_t)j;
            if (!done && p >= 0) {
                const uint64_t* e = status + 2 * (uint64_t)p + f;
                v = __hip_atomic_load(e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                for (uint32_t spin = 0; (v >> 40) != epoch; spin++) {  // tile p's workgroup is running it
                    if (spin == (1u << 24)) {
                        atomicOr(err, kLbTimeout);
                        v = ep | kLbFlagP;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                    v = __hip_atomic_load(e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            // this half's nearest inclusive prefix ends its walk
            const uint32_t q = (uint32_t)(__ballot((v & kLbFlagP) != 0) >> (32 * f));
            const uint32_t upto = q ? (uint32_t)__builtin_ctz(q) : 31u;
            uint64_t add = (!done && j <= upto) ? (v & kLbValMask) : 0;
#pragma unroll
            for (int o = 1; o < 32; o <<= 1) add += (uint64_t)__shfl_xor((long long)add, o, 64);
            excl += add;
            done = done || q != 0;
        }
        if (j == 0) {
            if (tile != 0)
                __hip_atomic_store(status + 2 * tile + f, ep | kLbFlagP | (excl + v0), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            s_base[f] = excl;
            if (tile == ntiles - 1) {
                if (f == 0) *U_out = excl + v0;
                else *B_out = excl + v0;
            }
        }
    }
    __syncthreads();
    uint64_t rc = s_base[0], rb = s_base[1];
#pragma unroll 1
    for (int k = 0; k < kUniqSub; k++) {
        const uint64_t ec = k == 0 ? exc0 : k == 1 ? exc1 : k == 2 ? exc2 : exc3;
        const uint64_t eb = k == 0 ? exb0 : k == 1 ? exb1 : k == 2 ? exb2 : exb3;
        const uint64_t tc = s_tot[k][0], tb = s_tot[k][1];
#pragma unroll
        for (int q = 0; q < kUniqItems; q++) {
            const uint64_t f = (ec >> (16 * q)) & 0xFFFFull;
            const uint64_t i = lo + (uint64_t)k * kUniqTile + (uint64_t)q * kBlock + t;
            if (f & 0x8000ull) {
                uint64_t r, pv;
                item(k, q, r, pv);
                const uint64_t uu = rc + (f & 0x7FFFull);
                const uint32_t key = (uint32_t)(r >> 32), pkey = (uint32_t)(pv >> 32);
                const bool wstart = pv == ~0ull || key != pkey;
                const uint32_t id0 = !kFmap ? (uint32_t)r + fid_off
                                   : k == 0 ? gid[q] : k == 1 ? gid[kUniqItems + q]
                                   : k == 2 ? gid[2 * kUniqItems + q] : gid[3 * kUniqItems + q];
                if (uniq32) {  // (uniform)
                    uniq32[uu] = id0 | (wstart ? kPairFirst : 0u);
                    if ((uu & 63u) == 0) g64[uu >> 6] = key;
                } else {
                    uniq[uu] = (r & ~0xFFFFFFFFull) | id0;
                }
                // P is read at word starts (k_fmt_words, OpLineOff) and at the
                // first posting of every 64 (k_fmt_posts) only
                if (wstart || (uu & 63u) == 0) P[uu] = rb + ((eb >> (16 * q)) & 0xFFFFull);
                if (wstart) {
                    post_start[key] = uu;
                    if (pv != ~0ull) post_end[pkey] = uu;
                }
            }
            if (kPacked && i + 1 == vend) {  // the bucket's last record: its word ends after the pairs so far
                uint64_t r, pv;
                item(k, q, r, pv);
                post_end[(uint32_t)(r >> 32)] = rc + (f & 0x7FFFull) + ((f >> 15) & 1u);
            }
            rc += (tc >> (16 * q)) & 0xFFFFull;
            rb += (tb >> (16 * q)) & 0xFFFFull;
        }
    }
}

// post_end of the last word = U (= post_start[V], written by the scan)
__global__ void k_post_last(const uint64_t* __restrict__ rec, uint64_t n, const uint64_t* __restrict__ U,
                            uint64_t* __restrict__ post_end) {
    if (threadIdx.x == 0 && n) post_end[(uint32_t)(rec[n - 1] >> 32)] = *U;
}
// wid-keyed word starts / ends -> lexid-indexed ones (V threads)
__global__ __launch_bounds__(kBlock) void k_wid_post(const uint32_t* __restrict__ widl, uint32_t V,
                                                     const uint64_t* __restrict__ ps_w, const uint64_t* __restrict__ pe_w,
                                                     uint64_t* __restrict__ ps, uint64_t* __restrict__ pe) {
    const uint32_t j = blockIdx.x * kBlock + threadIdx.x;
    if (j >= V) return;
    const uint32_t w = widl[j];
    ps[j] = ps_w[w];
    pe[j] = pe_w[w];
}

// ---------------------------------------------------------------- K4 order
// key = letter << dbits | (dmax - df): ascending == (letter, df desc); the
// stable sort keeps lexicographic order among equal df (main.c:55-64).
// Also each word's line bytes "word:[" + postings + "\n" -> linelen[j] (by
// lexid), the value OpLineOff scans in final order: one gather per line
// there instead of five dependent ones.
__global__ __launch_bounds__(kBlock) void k_order_keys(const uint64_t* __restrict__ sk, const uint64_t* __restrict__ post_start,
                                                       const uint64_t* __restrict__ post_end,
                                                       uint32_t V, int dbits, uint64_t* __restrict__ okey,
                                                       uint32_t* __restrict__ oval, const uint32_t* __restrict__ lex_len,
                                                       const uint64_t* __restrict__ P, uint64_t* __restrict__ linelen) {
    uint32_t j = blockIdx.x * kBlock + threadIdx.x;
    if (j >= V) return;
    const uint64_t s = post_start[j], e = post_end[j];
    uint64_t df = e - s;
    uint64_t dmax = (1ull << dbits) - 1;
    uint64_t letter = (sk[j] >> 59) - 1;
    okey[j] = (letter << dbits) | (dmax - df);
    oval[j] = j;
    linelen[j] = (uint64_t)lex_len[j] + 3 + (P[e] - P[s]);
}

// ---------------------------------------------------------------- K5 format
// A word's len letters at o.  <= 12 letters: from the packed key (5-bit codes,
// first letter highest), the bytes built in two registers and stored with two
// overlapping stores (one byte store per letter before).  Longer words: the
// cleaned letters of the inserting occurrence in the text (main.c:105-111),
// read one aligned 16-byte block per load (a byte load per text byte before:
// each letter waited a load round trip, since a load after a store waits for it).
__device__ __forceinline__ void write_word(const uint8_t* __restrict__ text, uint64_t nbytes, uint64_t key, uint64_t rep,
                                           uint32_t len, uint8_t* __restrict__ o) {
    if ((key & 0xFull) == 0) {
        uint64_t b0 = 0, b1 = 0;  // bytes 0..7, 8..11 (past len: 0x60, never stored)
#pragma unroll
        for (int i = 0; i < 12; i++) {
            const uint64_t ch = 0x60ull + ((key >> (59 - 5 * i)) & 31ull);
            if (i < 8) b0 |= ch << (8 * i);
            else b1 |= ch << (8 * (i - 8));
        }
        if (len >= 8u) {
            const uint32_t k = len - 8u;  // the last 8 bytes: [k, len) of b0 | b1 << 64
            const uint64_t t = k ? (b0 >> (8 * k)) | (b1 << (64 - 8 * k)) : b0;
            __builtin_memcpy(o, &b0, 8);
            __builtin_memcpy(o + k, &t, 8);
        } else if (len >= 4u) {
            const uint32_t a = (uint32_t)b0, t = (uint32_t)(b0 >> (8 * (len - 4u)));
            __builtin_memcpy(o, &a, 4);
            __builtin_memcpy(o + (len - 4u), &t, 4);
        } else if (len >= 2u) {
            const uint16_t a = (uint16_t)b0, t = (uint16_t)(b0 >> (8 * (len - 2u)));
            __builtin_memcpy(o, &a, 2);
            __builtin_memcpy(o + (len - 2u), &t, 2);
        } else if (len == 1u) {
            o[0] = (uint8_t)b0;
        }
    } else {
        uint32_t n = 0;
        for (uint64_t g = rep & ~15ull; g < nbytes && n < len; g += 16) {
            const uint4 v = load16(text, nbytes, (int64_t)g);
            for (uint32_t j = g < rep ? (uint32_t)(rep - g) : 0u; j < 16u && n < len; j++) {
                const uint32_t lc = letter_of(byte_dyn(v, j));
                if (lc < 26u) o[n++] = (uint8_t)('a' + lc);
            }
        }
    }
}

// line byte offsets in final order: loff[w] holds word w's line bytes
// (k_order_keys) and receives the line's offset (each item is read and then
// written by the same thread of k_scan_apply, after k_scan_reduce has read all)
struct OpLineOff {
    const uint32_t* ord;
    uint64_t* loff;  // by lexid
    __device__ uint64_t value(uint64_t i) const { return loff[ord[i]]; }
    __device__ void emit(uint64_t i, uint64_t ex, uint64_t) const { loff[ord[i]] = ex; }
};

constexpr int kFmtWordItems = 4;  // words per thread of k_fmt_words
__global__ __launch_bounds__(kBlock) void k_fmt_words(const uint8_t* __restrict__ text, uint64_t nbytes,
                                                      const uint64_t* __restrict__ lex_key, const uint64_t* __restrict__ lex_rep,
                                                      const uint32_t* __restrict__ lex_len,
                                                      const uint64_t* __restrict__ post_start,
                                                      const uint64_t* __restrict__ post_end, const uint64_t* __restrict__ P,
                                                      const uint64_t* __restrict__ loff, uint32_t V, uint8_t* __restrict__ out,
                                                      const uint32_t* __restrict__ widl, uint64_t* __restrict__ fbase) {
    // kFmtWordItems words per thread, strided by the grid, every load of all of them issued before the
    // first store (a load issued after a store waits for it too: vmcnt counts both)
    const uint32_t stride = gridDim.x * kBlock;
    const uint32_t j0 = blockIdx.x * kBlock + threadIdx.x;
    uint64_t o[kFmtWordItems], ps[kFmtWordItems], pe[kFmtWordItems], key[kFmtWordItems], rep[kFmtWordItems];
    uint32_t len[kFmtWordItems], wl[kFmtWordItems];
#pragma unroll
    for (int q = 0; q < kFmtWordItems; q++) {
        const uint32_t j = j0 + q * stride;
        const bool ok = j < V;
        o[q] = ok ? loff[j] : 0ull;
        len[q] = ok ? lex_len[j] : 0u;
        // posting p of word j starts at fbase[key(j)] + P[p] (key = wid or lexid):
        // one gather per posting in k_fmt_posts instead of four
        ps[q] = ok ? P[post_start[j]] : 0ull;
        pe[q] = ok ? P[post_end[j]] : 0ull;
        key[q] = ok ? lex_key[j] : 0ull;
        rep[q] = ok ? lex_rep[j] : 0ull;
        wl[q] = ok ? (widl ? widl[j] : j) : 0u;
    }
#pragma unroll
    for (int q = 0; q < kFmtWordItems; q++) {
        if (j0 + q * stride >= V) continue;
        fbase[wl[q]] = o[q] + len[q] + 2 - ps[q];
        out[o[q] + len[q] + 3 + (pe[q] - ps[q]) - 1] = '\n';
        write_word(text, nbytes, key[q], rep[q], len[q], out + o[q]);
        const uint16_t open = (uint16_t)(':' | ('[' << 8));
        __builtin_memcpy(out + o[q] + len[q], &open, 2);
    }
}

// uniq keys are wids or lexids, fbase is indexed the same way (k_fmt_words).
// A wave formats kFmtItems groups of 64 consecutive postings per iteration,
// with every group's loads (pairs, then the fbase gathers) issued before any
// digits are written: one dependent load chain per group left the pass
// latency-bound.  A group reads the posting byte offset of its first posting
// only (P is written at multiples of 64 and at word starts, k_uniq_sweep) and
// places the rest by a wave scan of their byte counts, so the pass reads
// 8 bytes per posting instead of 16.
// g64[g] (a word id, compact pairs of a word-id sort) -> the word's dense
// index (its rank among the occupied slots): one pass over U / 64 entries, so
// that the formatter's chain stays group key -> fbase (a rank gather in it
// made the pass 1.64 -> 1.9 ms, one more dependent load per group)
__global__ __launch_bounds__(kBlock) void k_g64_dense(uint32_t* __restrict__ g64, uint64_t n,
                                                      const uint32_t* __restrict__ rank_hot,
                                                      const uint32_t* __restrict__ nhot) {
    const uint64_t g = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (g >= n) return;
    const uint32_t w = g64[g];
    g64[g] = w < (uint32_t)kHotSlots ? rank_hot[w] : *nhot + (w - (uint32_t)kHotSlots);
}

constexpr int kFmtItems = 4;  // groups per wave (2 or 8: slower)
// k32: the compact pairs (uniq32 / g64, k_uniq_sweep): g64 holds each
// group's first word as a dense index d (k_g64_dense; lexid keys are dense
// already), the word of lane i = d + the word starts in lanes 1..i, and fbase
// is indexed by d.
template <bool k32>
__global__ __launch_bounds__(kBlock, 8) void k_fmt_posts(const uint64_t* __restrict__ uniq,
                                                      const uint32_t* __restrict__ uniq32,
                                                      const uint32_t* __restrict__ g64, uint64_t U,
                                                      const uint64_t* __restrict__ fbase, const uint64_t* __restrict__ P,
                                                      uint8_t* __restrict__ out) {
    constexpr uint64_t kSpan = 64ull * kFmtItems;  // postings of one wave per iteration
    const uint64_t nwaves = (uint64_t)gridDim.x * kWaves;
    const int l = lane_id();
    const uint64_t le = ~0ull >> (63 - l);  // lanes 0..l
    for (uint64_t g0 = ((uint64_t)blockIdx.x * kWaves + (uint64_t)wave_id()) * kSpan; g0 < U; g0 += nwaves * kSpan) {
        uint64_t r[kFmtItems], pb[kFmtItems], fb[kFmtItems];
        uint32_t wn[kFmtItems];  // k32: 1 if the posting after this one starts a word; else its word
        uint32_t x[kFmtItems], wd[kFmtItems];
#pragma unroll
        for (int k = 0; k < kFmtItems; k++) {
            const uint64_t p = g0 + (uint64_t)k * 64 + (uint64_t)l;
            if (k32) {
                x[k] = p < U ? uniq32[p] : kPairFirst;
                wd[k] = g0 + (uint64_t)k * 64 < U ? g64[(g0 >> 6) + k] : 0u;
            } else {
                r[k] = p < U ? uniq[p] : 0ull;
            }
            pb[k] = g0 + (uint64_t)k * 64 < U ? P[g0 + (uint64_t)k * 64] : 0ull;
        }
        // the posting after each group's lane 63 (the next group's lane 0)
        const uint64_t pn = g0 + kSpan;
        uint32_t xtail = kPairFirst, wtail = 0u;
        if (l == 63 && pn < U) {
            if (k32) xtail = uniq32[pn];
            else wtail = (uint32_t)(uniq[pn] >> 32);
        }
        if (k32) {
#pragma unroll
            for (int k = 0; k < kFmtItems; k++) {
                const uint32_t d0 = wd[k];
                const uint64_t fm = __ballot((x[k] & kPairFirst) != 0u);
                const uint32_t d = d0 + (uint32_t)__popcll(fm & le & ~1ull);
                const uint64_t p = g0 + (uint64_t)k * 64 + (uint64_t)l;
                fb[k] = p < U ? fbase[d] : 0ull;
                const uint32_t nx = k + 1 < kFmtItems ? (uint32_t)__shfl((int)x[k + 1 < kFmtItems ? k + 1 : k], 0, 64) : xtail;
                wn[k] = l == 63 ? (nx >> 31) : (uint32_t)(fm >> (l + 1)) & 1u;
            }
        } else {
#pragma unroll
            for (int k = 0; k < kFmtItems; k++) {
                const uint64_t p = g0 + (uint64_t)k * 64 + (uint64_t)l;
                fb[k] = p < U ? fbase[(uint32_t)(r[k] >> 32)] : 0ull;
            }
#pragma unroll
            for (int k = 0; k < kFmtItems; k++) {
                const uint32_t w = (uint32_t)(r[k] >> 32);
                uint32_t d = __shfl_down(w, 1, 64);
                const uint32_t first_next = k + 1 < kFmtItems ? __shfl((uint32_t)(r[k + 1 < kFmtItems ? k + 1 : k] >> 32), 0, 64)
                                                              : wtail;
                wn[k] = l == 63 ? first_next : d;
            }
        }
#pragma unroll
        for (int k = 0; k < kFmtItems; k++) {
            const uint64_t p = g0 + (uint64_t)k * 64 + (uint64_t)l;
            const bool live = p < U;
            const uint64_t id = k32 ? (uint64_t)(x[k] & ~kPairFirst) + 1 : (r[k] & 0xFFFFFFFFull) + 1;
            const uint32_t nd = id_digits(id);
            const uint32_t len = live ? nd + 1u : 0u;
            const uint32_t inc = wave_incl_scan32(len);  // inclusive wave scan (64 postings x <= 11 bytes)
            if (!live) continue;
            // last posting of the word: the next pair belongs to another word (runs are contiguous)
            const bool last = p + 1 == U || (k32 ? wn[k] != 0u : wn[k] != (uint32_t)(r[k] >> 32));
            const uint64_t o = fb[k] + pb[k] + (inc - len);
            if (nd <= 7u) {
                // digits + separator (<= 8 bytes) built in one register, then stored with two
                // unaligned stores (native on gfx950): one byte store per digit made the pass
                // issue-bound.
                // The 8 decimal digits of id (< 10^7 here, leading zeros) by SWAR: two 4-digit
                // halves, each split into 2-digit 16-bit lanes, each lane into a tens / ones byte
                // (multiply-shift divisions exact below 10^4 and 10^2), then the leading zeros shifted
                // out — straight-line VALU instead of a loop of nd divisions by 10
                const uint32_t v = (uint32_t)id, vh = v / 10000u, vl = v - vh * 10000u;
                const uint32_t hh = (vh * 10486u) >> 20, lh = (vl * 10486u) >> 20;
                uint32_t A = hh | ((vh - hh * 100u) << 16), B = lh | ((vl - lh * 100u) << 16);
                const uint32_t Az = ((A * 103u) >> 10) & 0x000F000Fu, Bz = ((B * 103u) >> 10) & 0x000F000Fu;
                A = Az | ((A - Az * 10u) << 8);
                B = Bz | ((B - Bz * 10u) << 8);
                const uint64_t dig = (((uint64_t)B << 32) | A) | 0x3030303030303030ull;
                const uint64_t s = (dig >> (8 * (8 - nd))) | ((uint64_t)(last ? ']' : ' ') << (8 * nd));
                // two stores per posting, the second ending at its last byte: they overlap for
                // len < 8 (the same bytes twice, from one lane), so a wave whose postings all take
                // 4..8 bytes issues exactly two dword stores (three sized stores before: dword /
                // short / byte; 7-byte postings, rank 7's 6-digit ids, needed all three)
                uint8_t* d = out + o;
                if (len >= 4u) {
                    const uint32_t a = (uint32_t)s, b = (uint32_t)(s >> (8 * (len - 4u)));
                    __builtin_memcpy(d, &a, 4);
                    __builtin_memcpy(d + (len - 4u), &b, 4);
                } else {  // 2 or 3 bytes (one digit + separator, or two)
                    const uint16_t a = (uint16_t)s, b = (uint16_t)(s >> (8 * (len - 2u)));
                    __builtin_memcpy(d, &a, 2);
                    __builtin_memcpy(d + (len - 2u), &b, 2);
                }
            } else {  // ids >= 10^7: one byte per digit
                uint64_t v = id;
                for (int i = (int)nd - 1; i >= 0; i--) {
                    out[o + i] = (uint8_t)('0' + v % 10u);
                    v /= 10u;
                }
                out[o + nd] = last ? ']' : ' ';
            }
        }
    }
}

__global__ void k_letter_off(const uint32_t* __restrict__ letter_start, const uint32_t* __restrict__ ord,
                             const uint64_t* __restrict__ loff, uint32_t V, uint64_t total, uint64_t* __restrict__ letter_off) {
    int l = threadIdx.x;
    if (l > 26) return;
    uint32_t i = letter_start[l];
    letter_off[l] = i < V ? loff[ord[i]] : total;
}

// ---------------------------------------------------------------- exchange
// Segment sent to the owner of a letter range, 8-byte aligned:
//   u64 header[8] = {kSegMagic, nwords, npairs, arena_bytes, letter_lo, letter_hi, 0, 0}
//   u64 pairs[npairs]   (word index within the segment) << 32 | id0
//   u8  arena[]         the segment's words in lexicographic order, each + ' '
constexpr uint64_t kSegMagic = 0x3147455349495849ull;  // "IXIISEG1"

// word arena offsets: letters + one separator per word
struct OpWordArena {
    const uint32_t* llen;
    uint64_t* woff;
    __device__ uint64_t value(uint64_t j) const { return (uint64_t)llen[j] + 1; }
    __device__ void emit(uint64_t j, uint64_t ex, uint64_t) const { woff[j] = ex; }
};

// Exchange after a word-id reduce: in lexicographic word order (the order
// export segments carry) pair s (grouped by word id) of word j = lexw[wid] is
// the (psx[j] + s - ps[j])-th, psx = exclusive scan of the words' pair counts
// in lexid order (k_export_pairs_wid) — instead of sorting the tokens by lexid
// (whose first pass gathers a map entry for every word).
struct OpRunLen {
    const uint64_t* ps;
    const uint64_t* pe;
    uint64_t* psx;
    __device__ uint64_t value(uint64_t j) const { return pe[j] - ps[j]; }
    __device__ void emit(uint64_t j, uint64_t ex, uint64_t) const { psx[j] = ex; }
};

// per letter l: first word, first pair, first arena byte
__global__ void k_letter_points(const uint32_t* __restrict__ letter_start, const uint64_t* __restrict__ post_start,
                                const uint64_t* __restrict__ woff, uint64_t* __restrict__ pts) {
    int l = threadIdx.x;
    if (l > 26) return;
    uint32_t j = letter_start[l];
    pts[3 * l] = j;
    pts[3 * l + 1] = post_start[j];
    pts[3 * l + 2] = woff[j];
}

__global__ __launch_bounds__(kBlock) void k_export_words(const uint8_t* __restrict__ text, uint64_t nbytes,
                                                         const uint64_t* __restrict__ lex_key,
                                                         const uint64_t* __restrict__ lex_rep,
                                                         const uint32_t* __restrict__ lex_len,
                                                         const uint64_t* __restrict__ woff, uint32_t j0, uint32_t j1,
                                                         uint8_t* __restrict__ arena) {
    uint32_t j = j0 + blockIdx.x * kBlock + threadIdx.x;
    if (j >= j1) return;
    uint8_t* o = arena + (woff[j] - woff[j0]);
    uint32_t len = lex_len[j];
    write_word(text, nbytes, lex_key[j], lex_rep[j], len, o);
    o[len] = ' ';
}

// Export of a word-id reduce's pairs straight from their word-id order (no
// lexid-ordered copy first): pair i of word w (lexid j = lexw[w]) is the
// (psx[j] + i - ps[j])-th pair in lexid order; the part whose lexid range
// holds j (parts in LDS, a binary search over <= II_MAX_PARTS starts) gets it
// as (j - j0) << 32 | id0 at dst + that index - the part's first pair.  (The
// copy, k_pairs_by_lexid, wrote and re-read 16 bytes a pair more.)
constexpr int kExportMaxParts = 64;  // II_MAX_PARTS
constexpr int kExportItems = 4;      // pairs per thread per step of k_export_pairs_wid
struct ExportParts {
    uint32_t n;
    uint32_t j0[kExportMaxParts + 1];  // first lexid of part r (j0[n] = V)
    uint64_t p0[kExportMaxParts];      // its first pair in lexid order
    uint64_t* dst[kExportMaxParts];    // its segment's pair array
};
__global__ __launch_bounds__(kBlock) void k_export_pairs_wid(const uint64_t* __restrict__ uniq, uint64_t U,
                                                             const uint32_t* __restrict__ lexw,
                                                             const uint64_t* __restrict__ ps,
                                                             const uint64_t* __restrict__ psx, ExportParts parts) {
    __shared__ uint32_t s_j0[kExportMaxParts + 1];
    __shared__ uint64_t s_p0[kExportMaxParts];
    __shared__ uint64_t* s_dst[kExportMaxParts];
    for (uint32_t r = threadIdx.x; r <= parts.n; r += kBlock) {
        s_j0[r] = parts.j0[r];
        if (r < parts.n) {
            s_p0[r] = parts.p0[r];
            s_dst[r] = parts.dst[r];
        }
    }
    __syncthreads();
    // kExportItems pairs per thread per step, each of the three dependent loads
    // (pair, word's lexid, its offsets) issued for all of them before the next:
    // one chain of three round trips per kExportItems pairs instead of per pair
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    for (uint64_t i0 = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i0 < U; i0 += kExportItems * stride) {
        uint64_t rr[kExportItems], px[kExportItems], pw[kExportItems];
        uint32_t j[kExportItems];
#pragma unroll
        for (int q = 0; q < kExportItems; q++) {
            const uint64_t i = i0 + q * stride;
            rr[q] = i < U ? uniq[i] : 0ull;
        }
#pragma unroll
        for (int q = 0; q < kExportItems; q++) j[q] = i0 + q * stride < U ? lexw[rr[q] >> 32] : 0u;
#pragma unroll
        for (int q = 0; q < kExportItems; q++) {
            const bool ok = i0 + q * stride < U;
            px[q] = ok ? psx[j[q]] : 0ull;
            pw[q] = ok ? ps[j[q]] : 0ull;
        }
#pragma unroll
        for (int q = 0; q < kExportItems; q++) {
            const uint64_t i = i0 + q * stride;
            if (i >= U) continue;
            uint32_t lo = 0, hi = parts.n - 1;  // the last part with j0 <= j
            while (lo < hi) {
                const uint32_t mid = (lo + hi + 1) / 2;
                if (s_j0[mid] <= j[q]) lo = mid;
                else hi = mid - 1;
            }
            s_dst[lo][px[q] + (i - pw[q]) - s_p0[lo]] = ((uint64_t)(j[q] - s_j0[lo]) << 32) | (rr[q] & 0xFFFFFFFFull);
        }
    }
}

__global__ __launch_bounds__(kBlock) void k_export_pairs(const uint64_t* __restrict__ uniq, uint64_t p0, uint64_t p1,
                                                         uint32_t j0, uint64_t* __restrict__ out) {
    for (uint64_t p = p0 + (uint64_t)blockIdx.x * kBlock + threadIdx.x; p < p1; p += (uint64_t)gridDim.x * kBlock) {
        uint64_t r = uniq[p];
        out[p - p0] = (((r >> 32) - j0) << 32) | (r & 0xFFFFFFFFull);
    }
}

// h[6], h[7] = 1 + the smallest / largest id0 of the exporting context's
// files (0 = unknown): lets the owner skip its id sort when the sources' id
// ranges ascend without overlap (ii_import)
__global__ void k_export_header(uint64_t* __restrict__ h, uint64_t nwords, uint64_t npairs, uint64_t arena, uint64_t llo,
                                uint64_t lhi, uint64_t id_lo1, uint64_t id_hi1) {
    if (threadIdx.x == 0) {
        h[0] = kSegMagic; h[1] = nwords; h[2] = npairs; h[3] = arena; h[4] = llo; h[5] = lhi; h[6] = id_lo1;
        h[7] = id_hi1;
    }
}

// received pair -> (global lexid, id0): word k of the merged word text was
// tokenised into wrec[k] = slot << 32; remap gives the owner's lexicographic id.
// k32: the u32 record lexid << f32 | id0 instead (the owner's sort keys fit 32 bits).
// All sources in one launch: source s's np pairs at p[s] go to out[pbase[s] ...)
// and get workgroups [bstart[s], bstart[s + 1]) of kImportPer pairs each, so a
// workgroup reads ONE source (its index found by a uniform binary search;
// per-source launches cost their launch gaps and tails, and an earlier
// one-launch form that looked the source up per element was slower still).
constexpr int kImportMaxSrc = 64;  // II_MAX_PARTS
constexpr uint32_t kImportPer = kBlock * 8;
struct ImportSrc {
    uint32_t n;
    uint32_t bstart[kImportMaxSrc + 1];
    const uint64_t* p[kImportMaxSrc];
    uint64_t np[kImportMaxSrc], wbase[kImportMaxSrc], pbase[kImportMaxSrc];
};
template <bool k32>
__global__ __launch_bounds__(kBlock) void k_import_pairs(ImportSrc src, const uint64_t* __restrict__ wrec,
                                                         const uint32_t* __restrict__ remap, void* __restrict__ out,
                                                         int f32) {
    const uint32_t b = blockIdx.x;
    if (b >= src.bstart[src.n]) return;
    uint32_t lo = 0, hi = src.n - 1;  // the last source whose first workgroup is <= b
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) / 2;
        if (src.bstart[mid] <= b) lo = mid;
        else hi = mid - 1;
    }
    const uint32_t s = __builtin_amdgcn_readfirstlane(lo);
    const uint64_t* __restrict__ pairs = src.p[s];
    const uint64_t np = src.np[s], wbase = src.wbase[s], pbase = src.pbase[s];
    const uint64_t i0 = (uint64_t)(b - src.bstart[s]) * kImportPer;
    const uint64_t i1 = i0 + kImportPer < np ? i0 + kImportPer : np;
    // three rounds of loads in flight (pairs, word records, remap), not one chain per pair
    constexpr int kQ = kImportPer / kBlock;
    uint64_t r[kQ], slot[kQ];
#pragma unroll
    for (int q = 0; q < kQ; q++) {
        const uint64_t i = i0 + (uint64_t)q * kBlock + threadIdx.x;
        r[q] = i < i1 ? pairs[i] : 0ull;
    }
#pragma unroll
    for (int q = 0; q < kQ; q++) {
        const uint64_t i = i0 + (uint64_t)q * kBlock + threadIdx.x;
        slot[q] = i < i1 ? wrec[wbase + (r[q] >> 32)] >> 32 : 0ull;
    }
#pragma unroll
    for (int q = 0; q < kQ; q++) {
        const uint64_t i = i0 + (uint64_t)q * kBlock + threadIdx.x;
        if (i < i1) {
            const uint32_t lex = remap[slot[q]];
            if (k32) static_cast<uint32_t*>(out)[pbase + i] = (lex << f32) | (uint32_t)r[q];
            else static_cast<uint64_t*>(out)[pbase + i] = ((uint64_t)lex << 32) | (r[q] & 0xFFFFFFFFull);
        }
    }
}
// The packed layout's geometry for ONE bucket of n u32 records from index 0
// (the owner's merged u32 pairs, read by k_uniq_sweep<true> as bucket 0:
// lexid = record >> F, as the packed sort's bucket-0 words)
__global__ void k_one_bucket(uint64_t* __restrict__ bstart, uint32_t* __restrict__ btile, uint64_t n, uint32_t ntb) {
    bstart[0] = 0;
    bstart[1] = n;
    btile[0] = 0;
    btile[1] = ntb;
}
// u32 records lexid << f | id0 -> the u64 records lexid << 32 | id0 K3 reads
__global__ __launch_bounds__(kBlock) void k_unpack32(const uint32_t* __restrict__ in, uint64_t n, int f,
                                                     uint64_t* __restrict__ out) {
    const uint32_t m = (1u << f) - 1u;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock) {
        const uint32_t x = in[i];
        out[i] = ((uint64_t)(x >> f) << 32) | (x & m);
    }
}

// Owner-side merge of the received segments when their id ranges ascend
// (ii_import): every segment is sorted by (lexid, id0), so the merged order
// (lexid, source) is (lexid, id0).  Per (word w, source g): the run of the
// word's pairs in segment g -> its place in the merged array (one scan over
// V x G run lengths), then one scatter of coalesced runs instead of three
// radix passes.
__global__ __launch_bounds__(kBlock) void k_merge_runs(const uint64_t* __restrict__ r, uint64_t pb, uint64_t np,
                                                       uint32_t G, uint32_t g, uint64_t* __restrict__ rstart,
                                                       uint64_t* __restrict__ rend) {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < np; i += (uint64_t)gridDim.x * kBlock) {
        const uint32_t w = (uint32_t)(r[pb + i] >> 32);
        const uint64_t k = (uint64_t)w * G + g;
        if (i == 0 || (uint32_t)(r[pb + i - 1] >> 32) != w) rstart[k] = pb + i;
        if (i + 1 == np || (uint32_t)(r[pb + i + 1] >> 32) != w) rend[k] = pb + i + 1;
    }
}
// run lengths (rend = 0: no run) -> exclusive offsets, in place in rend
struct OpMergeRuns {
    const uint64_t* rstart;
    uint64_t* rend;
    __device__ uint64_t value(uint64_t i) const { return rend[i] ? rend[i] - rstart[i] : 0; }
    __device__ void emit(uint64_t i, uint64_t ex, uint64_t) const { rend[i] = ex; }
};
__global__ __launch_bounds__(kBlock) void k_merge_scatter(const uint64_t* __restrict__ r, uint64_t pb, uint64_t np,
                                                          uint32_t G, uint32_t g, const uint64_t* __restrict__ rstart,
                                                          const uint64_t* __restrict__ roff, uint64_t* __restrict__ out) {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < np; i += (uint64_t)gridDim.x * kBlock) {
        const uint64_t v = r[pb + i];
        const uint64_t k = (uint64_t)(uint32_t)(v >> 32) * G + g;
        out[roff[k] + (pb + i - rstart[k])] = v;
    }
}

// Owner-side merge of interleaved sources (ii_import; main.c:129-130 owner,
// 170-213 its reduce): every source's pairs arrive sorted by the owner's
// (lexid, id0) — the source's words in lexicographic order map to ascending
// owner lexids, each word's ids ascending — so the owner merges G sorted runs
// instead of sorting them: ceil(log2 G) rounds of pairwise merge-path merges,
// each one coalesced read and one write of every record.  A round's pairs
// (run 2p, run 2p + 1) are described on the host (MergeRound, passed by
// value); the partition kernel finds, for every tile boundary of every pair,
// how many of the first k outputs come from the left run (binary search of the
// merge path, left run first on ties), and each tile workgroup then merges its
// two slices through LDS.  K: u64 records lexid << 32 | id0, or u32 records
// lexid << F | id0 when both fit.
constexpr int kMergeMaxPairs = 32;            // runs per round: II_MAX_PARTS / 2
constexpr int kMergeNT = 256, kMergeIT = 8;   // a tile = 2048 outputs
constexpr int kMergeTile = kMergeNT * kMergeIT;
struct MergeRound {
    uint32_t npairs;
    uint64_t a[kMergeMaxPairs];     // left run start (= the pair's output start)
    uint64_t na[kMergeMaxPairs], nb[kMergeMaxPairs];  // run lengths (the right run starts at a + na)
    uint32_t tile0[kMergeMaxPairs + 1];  // the pair's first tile; tile0[npairs] = all tiles
};

__device__ __forceinline__ uint32_t merge_pair_of(const MergeRound& mr, uint32_t tile) {
    uint32_t p = 0;
    while (p + 1 < mr.npairs && tile >= mr.tile0[p + 1]) p++;
    return p;
}

// the merge path: of the first k outputs of merging A (na) and B (nb), how many come from A
template <class K>
__device__ __forceinline__ uint64_t merge_corank(const K* __restrict__ A, uint64_t na, const K* __restrict__ B,
                                                 uint64_t nb, uint64_t k) {
    uint64_t lo = k > nb ? k - nb : 0, hi = k < na ? k : na;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (A[mid] <= B[k - 1 - mid]) lo = mid + 1;  // (A first on ties: stable)
        else hi = mid;
    }
    return lo;
}

// split[tile] = A-elements before the tile's first output, one thread per tile
// boundary (a wave per boundary searching 64 points per round trip was not
// faster in the run that measured it)
template <class K>
__global__ __launch_bounds__(kBlock) void k_merge_partition(const K* __restrict__ src, MergeRound mr,
                                                            uint64_t* __restrict__ split) {
    const uint32_t tile = blockIdx.x * kBlock + threadIdx.x;
    if (tile > mr.tile0[mr.npairs]) return;
    if (tile == mr.tile0[mr.npairs]) {  // (the end of the last pair)
        split[tile] = mr.na[mr.npairs - 1];
        return;
    }
    const uint32_t p = merge_pair_of(mr, tile);
    const uint64_t k = (uint64_t)(tile - mr.tile0[p]) * kMergeTile;
    const K* A = src + mr.a[p];
    split[tile] = merge_corank(A, mr.na[p], A + mr.na[p], mr.nb[p], k);
}

// Persistent tile loop: workgroup b takes tiles b, b + grid, ...; the next
// tile's two slices are loaded into registers while this one is merged in LDS
// (a workgroup with one short-lived tile waited out every load: 0.31 ms per
// round of 5·10^7 u64 records, 2.7 TB/s).
template <class K>
__global__ __launch_bounds__(kMergeNT) void k_merge_tiles(const K* __restrict__ src, K* __restrict__ dst, MergeRound mr,
                                                          const uint64_t* __restrict__ split) {
    __shared__ K s_in[kMergeTile];
    __shared__ K s_out[kMergeTile];
    const uint32_t ntiles = mr.tile0[mr.npairs];
    struct Slice {
        uint32_t p, la, lb, n;
        uint64_t k0;
    };
    auto slice_of = [&](uint32_t tile) {
        Slice sl;
        sl.p = merge_pair_of(mr, tile);
        const uint64_t na = mr.na[sl.p], nb = mr.nb[sl.p];
        sl.k0 = (uint64_t)(tile - mr.tile0[sl.p]) * kMergeTile;
        const uint64_t k1 = sl.k0 + kMergeTile < na + nb ? sl.k0 + kMergeTile : na + nb;
        const uint64_t i0 = split[tile];
        const uint64_t i1 = tile + 1 == mr.tile0[sl.p + 1] ? na : split[tile + 1];  // (the pair's last tile ends at na)
        sl.la = (uint32_t)(i1 - i0);
        sl.lb = (uint32_t)((k1 - i1) - (sl.k0 - i0));
        sl.n = sl.la + sl.lb;
        return sl;
    };
    // this thread's elements x = q * kMergeNT + t of a tile: its left slice, then its right slice
    K pre[kMergeIT];
    auto load = [&](uint32_t tile, const Slice& sl) {
        const K* A = src + mr.a[sl.p];
        const K* B = A + mr.na[sl.p];
        const uint64_t i0 = split[tile], j0 = sl.k0 - i0;
#pragma unroll
        for (int q = 0; q < kMergeIT; q++) {
            const uint32_t x = q * kMergeNT + threadIdx.x;
            pre[q] = x < sl.la ? A[i0 + x] : x < sl.n ? B[j0 + (x - sl.la)] : (K)0;
        }
    };
    uint32_t tile = blockIdx.x;
    if (tile >= ntiles) return;
    Slice sl = slice_of(tile);
    load(tile, sl);
    for (;;) {
#pragma unroll
        for (int q = 0; q < kMergeIT; q++) s_in[q * kMergeNT + threadIdx.x] = pre[q];
        __syncthreads();  // (also: every thread has stored the last tile's s_out)
        const uint32_t next = tile + gridDim.x;
        Slice nsl{};
        if (next < ntiles) {
            nsl = slice_of(next);
            load(next, nsl);
        }
        // this thread's outputs [q0, q0 + IT): its own merge path inside the tile, then a sequential merge
        const uint32_t la = sl.la, lb = sl.lb, n = sl.n;
        const uint32_t q0 = threadIdx.x * kMergeIT;
        if (q0 < n) {
            uint32_t lo = q0 > lb ? q0 - lb : 0, hi = q0 < la ? q0 : la;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (s_in[mid] <= s_in[la + q0 - 1 - mid]) lo = mid + 1;
                else hi = mid;
            }
            uint32_t ia = lo, ib = q0 - lo;
#pragma unroll
            for (int q = 0; q < kMergeIT; q++) {
                if (q0 + q >= n) break;
                const bool takeA = ib >= lb || (ia < la && s_in[ia] <= s_in[la + ib]);
                s_out[q0 + q] = takeA ? s_in[ia] : s_in[la + ib];
                ia += takeA;
                ib += !takeA;
            }
        }
        __syncthreads();
        K* out = dst + mr.a[sl.p] + sl.k0;
        for (uint32_t x = threadIdx.x; x < n; x += kMergeNT) out[x] = s_out[x];
        if (next >= ntiles) return;  // (workgroup-uniform)
        tile = next;
        sl = nsl;
    }
}

}  // namespace ii
