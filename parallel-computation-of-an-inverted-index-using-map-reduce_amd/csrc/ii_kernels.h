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
#include "ii_prims.h"

namespace ii {

// ---------------------------------------------------------------- constants
constexpr int kTile = 4096;        // bytes staged per tokenizer step (256 lanes x 16 B)
constexpr int kHalo = 512;         // right halo staged with each tile
constexpr int kChunkTiles = 16;    // tiles per tokenizer workgroup
constexpr uint64_t kChunk = (uint64_t)kTile * kChunkTiles;  // 64 KiB of text per workgroup
constexpr int kMaxWord = 299;      // MAX_WORD - 1 letters (main.c:7, 105)
constexpr int kMaxProbe = 1 << 14;

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
    C_NUM = 32
};

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
//   hot table  slots [0, 2^17): 8-slot buckets (one 64-B line), probed inside
//              the bucket only.  Words that arrive first — in a Zipf corpus
//              mostly the frequent ones — fill it; 1 MB of keys stays in every
//              XCD's 4 MB L2, so most probes never leave L2.
//   big table  slots [2^17, 2^17 + cap): linear probing; words whose hot
//              bucket was already full.
// A word lives in exactly one place: a probe scans the same bucket (then the
// same big-table run) in the same order and slots only go empty -> full.
constexpr int kHotLog2 = 17;
constexpr uint64_t kHotSlots = 1ull << kHotLog2;
constexpr int kBucket = 8;

struct Table {
    unsigned long long* keys;  // [kHotSlots + big_cap]
    uint64_t* rep;             // token start of the inserting occurrence
    uint64_t big_mask;         // big_cap - 1
    uint64_t seed;
    uint64_t* counters;
};

__device__ __forceinline__ uint64_t table_hash(const Table& t, uint64_t key) { return mix64(key ^ t.seed); }
__device__ __forceinline__ uint64_t hot_home(uint64_t hh) { return hh & (kHotSlots - 1); }

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
// order (home, home+1, ... within the bucket); a full bucket sends the word
// to the big table (linear probing).
__device__ __forceinline__ uint32_t table_find(const Table& t, uint64_t key, uint64_t hh, uint64_t pos) {
    const uint64_t home = hot_home(hh);
    const uint32_t h7 = (uint32_t)(home & (kBucket - 1));
    const uint64_t bbase = home - h7;
    uint64_t h = (hh >> 20) & t.big_mask;
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

__device__ __forceinline__ uint64_t long_key(uint64_t hash, uint32_t len, uint64_t seed) {
    return (mix64(hash ^ seed ^ ((uint64_t)len << 48)) << 4) | 0xFull;
}

// Reader of the staged tile: tile-local byte j (j >= -16); LDS is read one
// aligned dword at a time (the walk touches ~2 dwords per token instead of
// ~7 bytes), past the halo it falls back to global memory.
struct TileReader {
    const uint8_t* s;
    const uint8_t* __restrict__ text;
    uint64_t nbytes, tile_lo;
    uint32_t di, dw;
    __device__ __forceinline__ TileReader(const uint8_t* s_, const uint8_t* text_, uint64_t nb, uint64_t lo)
        : s(s_), text(text_), nbytes(nb), tile_lo(lo), di(0xFFFFFFFFu), dw(0) {}
    __device__ __forceinline__ uint32_t get(uint32_t j) {
        if (j < (uint32_t)(kTile + kHalo)) {
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

// Cleaning loop of main.c:105-111 from tile-local byte p: stops at whitespace,
// NUL or the 299th letter.  Returns the word key (exact 5-bit packing for
// <= 12 letters, tagged hash otherwise) and its letter count (0 = dropped).
struct TokKey {
    uint64_t key;
    uint32_t nlet;
    uint32_t first;
};
__device__ __forceinline__ TokKey token_key(TileReader& rd, uint32_t p, uint64_t seed) {
    uint64_t packed = 0, hash = 1469598103934665603ull;
    uint32_t n = 0, first = 0;
    for (uint32_t j = p;; j++) {
        const uint32_t c = rd.get(j);
        if (c == 0u || is_ws(c)) break;
        const uint32_t lc = letter_of(c);
        if (lc < 26u) {
            if (n == 0) first = lc;
            n++;
            if (n <= 12) packed |= (uint64_t)(lc + 1) << (64 - 5 * n);
            hash = (hash ^ (lc + 1)) * 1099511628211ull;
            if (n == (uint32_t)kMaxWord) break;
        }
    }
    return TokKey{n <= 12 ? packed : long_key(hash, n, seed), n, first};
}

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

__device__ __forceinline__ uint4 load16(const uint8_t* __restrict__ text, uint64_t nbytes, int64_t g) {
    if (g >= 0 && (uint64_t)g + 16 <= nbytes) return *reinterpret_cast<const uint4*>(text + g);
    uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 16; i++) {
        const int64_t gi = g + i;
        const uint32_t b = (gi >= 0 && (uint64_t)gi < nbytes) ? text[gi] : 32u;
        w[i >> 2] |= b << ((i & 3) * 8);
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// Tile staging, software-pipelined: fetch_tile() loads the text of
// [tile_lo - 16, tile_lo + kTile + kHalo) into registers (16 B per lane; lane
// t's own window [tile_lo + 16t, +16) in .v, the left piece and the halo in
// .h of lanes 0..32) one tile ahead; store_tile() writes them to LDS.  Bytes
// outside the text read as ' ' (so position 0 starts a token).
struct TileRegs {
    uint4 v, h;
};
constexpr int kExtraPieces = 1 + kHalo / 16;  // left piece + halo pieces
__device__ __forceinline__ TileRegs fetch_tile(const uint8_t* __restrict__ text, uint64_t nbytes, uint64_t tile_lo) {
    const int t = threadIdx.x;
    TileRegs r;
    r.v = load16(text, nbytes, (int64_t)tile_lo + 16 * t);
    r.h = make_uint4(0, 0, 0, 0);
    if (t < kExtraPieces) {
        const int q = t == 0 ? -1 : kTile / 16 + t - 1;
        r.h = load16(text, nbytes, (int64_t)tile_lo + 16 * q);
    }
    return r;
}
__device__ __forceinline__ void store_tile(uint8_t* s_text, const TileRegs& r) {
    const int t = threadIdx.x;
    *reinterpret_cast<uint4*>(s_text + 16 + 16 * t) = r.v;
    if (t < kExtraPieces) {
        const int q = t == 0 ? -1 : kTile / 16 + t - 1;
        *reinterpret_cast<uint4*>(s_text + 16 + 16 * q) = r.h;
    }
}

__device__ __forceinline__ uint32_t byte_of(const uint4& v, int i) {
    const uint32_t w = i < 4 ? v.x : i < 8 ? v.y : i < 12 ? v.z : v.w;
    return (w >> ((i & 3) * 8)) & 0xFFu;
}

// ---- SWAR byte classes, 4 bytes per u32 (exact, no inter-byte carries)
// bit 7 of each byte set where the byte is zero
__device__ __forceinline__ uint32_t zero_bytes(uint32_t x) {
    return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
}
// the four bit-7 flags -> a 4-bit mask
__device__ __forceinline__ uint32_t hb4(uint32_t m) {
    return ((m >> 7) & 1u) | ((m >> 14) & 2u) | ((m >> 21) & 4u) | ((m >> 28) & 8u);
}
struct Classes {
    uint32_t ws, letter, nul;  // 16-bit masks over the lane's window
};
__device__ __forceinline__ void classify4(uint32_t x, uint32_t& ws, uint32_t& let, uint32_t& nul) {
    const uint32_t hb = x & 0x80808080u;
    const uint32_t y = x & 0x7F7F7F7Fu;
    const uint32_t sp = zero_bytes(x ^ 0x20202020u);                                  // ' '
    const uint32_t ctl = (y + 0x77777777u) & ~(y + 0x72727272u) & ~hb & 0x80808080u;   // 9..13
    ws = hb4(sp | ctl);                                   // C-locale isspace (main.c:102)
    const uint32_t z = (x | 0x20202020u) & 0x7F7F7F7Fu;
    let = hb4((z + 0x1F1F1F1Fu) & ~(z + 0x05050505u) & ~hb & 0x80808080u);  // A-Z / a-z (main.c:106-110)
    nul = hb4(zero_bytes(x));
}
__device__ __forceinline__ Classes classify16(const uint4& v) {
    Classes c{0, 0, 0};
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; k++) {
        uint32_t a, b, n;
        classify4(w[k], a, b, n);
        c.ws |= a << (4 * k);
        c.letter |= b << (4 * k);
        c.nul |= n << (4 * k);
    }
    return c;
}

// Token starts of the lane's window (non-space after space, main.c:102).  The
// byte before the window comes from the neighbour lane (LDS for lane 0 of a
// wave).  Call after the staging barrier.
__device__ __forceinline__ uint32_t lane_starts(const uint4& v, const Classes& cl, const uint8_t* s_text) {
    const int t = threadIdx.x;
    uint32_t prev = __shfl_up(v.w, 1, 64) >> 24;
    if ((t & 63) == 0) prev = s_text[16 + 16 * t - 1];
    const uint32_t prev_ws = is_ws(prev) ? 1u : 0u;
    return ~cl.ws & ((cl.ws << 1) | prev_ws) & 0xFFFFu;
}

// Kept tokens among the starts (a letter before the first whitespace / NUL,
// main.c:105, 113); decided from the masks, walking LDS only when the window
// ends before the token shows a letter, space or NUL.
__device__ __forceinline__ uint32_t kept_starts(uint32_t starts, const Classes& cl, const uint8_t* s_text,
                                                const uint8_t* __restrict__ text, uint64_t nbytes, uint64_t tile_lo,
                                                uint32_t wlo) {
    const uint32_t ev = cl.letter | cl.ws | cl.nul;
    uint32_t kept = 0;
    for (uint32_t m = starts & ~cl.letter; m; m &= m - 1) {  // starts that are not letters themselves
        const uint32_t i = __builtin_ctz(m);
        const uint32_t e = ev >> i;
        bool k;
        if (e) k = (cl.letter >> (i + __builtin_ctz(e))) & 1u;
        else {
            TileReader rd(s_text, text, nbytes, tile_lo);
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

// Register fast path of the cleaning loop (main.c:105-111) for the common
// token: it ends (whitespace / NUL) inside its first 16 bytes and its letters
// form one run from its first byte (plain or capitalised words, trailing
// punctuation) with at most 12 letters.  Returns false otherwise.
__device__ __forceinline__ bool fast_key(const uint4& tb, TokKey& out) {
    const Classes c = classify16(tb);
    const uint32_t term = c.ws | c.nul;
    if (term == 0) return false;
    const uint32_t e = __builtin_ctz(term);
    const uint32_t lm = c.letter & ((1u << e) - 1u);
    const uint32_t n = __popc(lm);
    if (n == 0 || n > 12 || lm != (1u << n) - 1u) return false;
    const uint32_t w[3] = {(tb.x | 0x20202020u) & 0x1F1F1F1Fu, (tb.y | 0x20202020u) & 0x1F1F1F1Fu,
                           (tb.z | 0x20202020u) & 0x1F1F1F1Fu};
    uint64_t packed = 0;
#pragma unroll
    for (int k = 0; k < 12; k++) packed |= (uint64_t)((w[k >> 2] >> (8 * (k & 3))) & 31u) << (59 - 5 * k);
    out.key = packed & (~0ull << (64 - 5 * n));
    out.nlet = n;
    out.first = (w[0] & 31u) - 1u;
    return true;
}

// 16 bytes of the staged tile at tile-local position p (any alignment):
// two aligned LDS reads + byte shift; past the staged halo, global memory.
__device__ __forceinline__ uint4 tile_block16(const uint8_t* s_text, const uint8_t* __restrict__ text, uint64_t nbytes,
                                              uint64_t tile_lo, uint32_t p) {
    const uint32_t a = 16 + p;
    const uint32_t base = a & ~15u;
    if (base + 32 <= (uint32_t)(16 + kTile + kHalo)) {
        const uint4 lo = *reinterpret_cast<const uint4*>(s_text + base);
        const uint4 hi = *reinterpret_cast<const uint4*>(s_text + base + 16);
        const uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        return token_bytes(w, a & 15u);
    }
    return load16(text, nbytes, (int64_t)tile_lo + p);
}

__device__ __forceinline__ uint32_t byte_dyn(const uint4& b, uint32_t j) {
    return (sel4(j >> 2, b.x, b.y, b.z, b.w) >> (8 * (j & 3u))) & 0xFFu;
}

// General form of the cleaning loop (main.c:105-111): 16 bytes per step,
// SWAR classes, then only the letter bytes are visited.  Stops at whitespace,
// NUL or the 299th letter.  first16 = the token's first 16 bytes.
__device__ __forceinline__ TokKey general_key(uint4 b, const uint8_t* s_text, const uint8_t* __restrict__ text,
                                              uint64_t nbytes, uint64_t tile_lo, uint32_t p, uint64_t seed) {
    uint64_t packed = 0, hash = 1469598103934665603ull;
    uint32_t n = 0, first = 0;
    for (;;) {
        const Classes cl = classify16(b);
        const uint32_t term = cl.ws | cl.nul;
        const uint32_t e = term ? __builtin_ctz(term) : 16u;
        bool done = term != 0;
        for (uint32_t m = cl.letter & ((1u << e) - 1u); m; m &= m - 1) {
            const uint32_t lc = (byte_dyn(b, __builtin_ctz(m)) | 0x20u) - 0x61u;
            if (n == 0) first = lc;
            n++;
            if (n <= 12) packed |= (uint64_t)(lc + 1) << (64 - 5 * n);
            hash = (hash ^ (lc + 1)) * 1099511628211ull;
            if (n == (uint32_t)kMaxWord) {
                done = true;
                break;
            }
        }
        if (done) break;
        p += 16;
        b = tile_block16(s_text, text, nbytes, tile_lo, p);
    }
    return TokKey{n <= 12 ? packed : long_key(hash, n, seed), n, first};
}

// K1a: kept tokens per 64 KiB chunk -> chunk_cnt[blockIdx.x].
__global__ __launch_bounds__(kBlock) void k_tok_count(const uint8_t* __restrict__ text, uint64_t nbytes,
                                                      uint64_t* __restrict__ chunk_cnt) {
    __shared__ __attribute__((aligned(16))) uint8_t s_text[16 + kTile + kHalo];
    __shared__ uint64_t s_scan[kWaves + 1];
    const uint64_t chunk_lo = (uint64_t)blockIdx.x * kChunk;
    const uint64_t chunk_hi = chunk_lo + kChunk < nbytes ? chunk_lo + kChunk : nbytes;
    const uint32_t wlo = (uint32_t)threadIdx.x * 16;
    uint64_t kept = 0;
    TileRegs nxt = fetch_tile(text, nbytes, chunk_lo);
    for (uint64_t tile_lo = chunk_lo; tile_lo < chunk_hi; tile_lo += kTile) {
        __syncthreads();
        store_tile(s_text, nxt);
        const uint4 v = nxt.v;
        if (tile_lo + kTile < chunk_hi) nxt = fetch_tile(text, nbytes, tile_lo + kTile);
        __syncthreads();
        const Classes cl = classify16(v);
        kept += __popc(kept_starts(lane_starts(v, cl, s_text), cl, s_text, text, nbytes, tile_lo, wlo));
    }
    uint64_t tot;
    (void)block_excl_scan(kept, &tot, s_scan);
    if (threadIdx.x == 0) chunk_cnt[blockIdx.x] = tot;
}

// Long token queued for the exactness check (k_long_verify).
struct LongTok {
    uint64_t pos;   // token start
    uint64_t slot;  // word-table slot it was given
};
constexpr int kLongBuf = 128;  // per-workgroup LDS buffer of long tokens

// Queue a long token for k_long_verify: into the workgroup's LDS buffer, or
// straight to global memory when the tile alone overflows the buffer.
__device__ __forceinline__ void queue_long(bool direct, LongTok* s_long, uint32_t* s_lcount, uint64_t lbase,
                                           LongTok* __restrict__ longs, uint64_t long_cap, const Table& tab, uint64_t pos,
                                           uint32_t slot) {
    if (direct) {
        const uint64_t li = lbase + atomicAdd(s_lcount, 1u);
        if (li < long_cap) longs[li] = LongTok{pos, slot};
        else atomicOr((unsigned long long*)&tab.counters[C_OVERFLOW], 2ull);
    } else {
        s_long[atomicAdd(s_lcount, 1u)] = LongTok{pos, slot};
    }
}

// K1b: chunk_off holds exclusive record offsets.  Per 4 KiB tile:
//   1. masks -> kept token starts, block scan -> token index per lane
//   2. each lane walks its kept tokens (LDS) -> word key into s_key[index]
//   3. the tile's tokens are spread evenly over the 256 threads, which probe
//      the word table with up to 4 independent loads in flight each
//   4. records rec[i] = slot << 32 | file id0 leave through LDS, coalesced.
// First letters are counted per chunk (chunk_hist[chunk][26] = the
// partial_<letter>.txt line counts); tokens of > 12 letters are queued for the
// hash-collision check.  No global atomics on a shared word per token.
// kAblate (timing experiments only, tools/k1_ablate.hip; the product uses 0):
// bit 0 = skip the table probe, bit 1 = skip the token walk, bit 2 = skip the
// letter histogram, bit 3 = no long-token queue, bit 4 = fast path only.
template <int kAblate = 0>
__global__ __launch_bounds__(kBlock) void k_tok_emit(const uint8_t* __restrict__ text, uint64_t nbytes,
                                                     const uint64_t* __restrict__ file_start,
                                                     const uint32_t* __restrict__ file_id, uint32_t nfiles,
                                                     const uint64_t* __restrict__ chunk_off, Table tab,
                                                     uint64_t* __restrict__ rec, uint32_t* __restrict__ chunk_hist,
                                                     LongTok* __restrict__ longs, uint64_t long_cap) {
    constexpr int kMaxTok = kTile / 2 + 1;
    __shared__ __attribute__((aligned(16))) uint8_t s_text[16 + kTile + kHalo];
    __shared__ uint64_t s_key[kMaxTok];   // word key, then the record
    __shared__ uint16_t s_off[kMaxTok];   // tile offset | 0x8000 if long
    __shared__ uint16_t s_slow[kMaxTok];  // tokens for the general key path
    __shared__ uint32_t s_nslow, s_nmiss;
    __shared__ LongTok s_long[kLongBuf];
    __shared__ uint64_t s_scan[kWaves + 1];
    __shared__ uint32_t s_hist[32];
    __shared__ uint32_t s_f[2];
    __shared__ uint32_t s_lcount;
    __shared__ uint64_t s_lbase;

    const uint64_t chunk_lo = (uint64_t)blockIdx.x * kChunk;
    const uint64_t chunk_hi = chunk_lo + kChunk < nbytes ? chunk_lo + kChunk : nbytes;
    const int t = threadIdx.x;
    if (t < 32) s_hist[t] = 0;
    if (t == 0) {
        s_f[0] = file_of(file_start, 0, nfiles - 1, chunk_lo);
        s_f[1] = file_of(file_start, s_f[0], nfiles - 1, chunk_hi - 1);
        s_lcount = 0;
    }
    uint64_t out = chunk_off[blockIdx.x];
    const uint32_t wlo = (uint32_t)t * 16;

    TileRegs nxt = fetch_tile(text, nbytes, chunk_lo);
    for (uint64_t tile_lo = chunk_lo; tile_lo < chunk_hi; tile_lo += kTile) {
        __syncthreads();
        store_tile(s_text, nxt);
        const uint4 v = nxt.v;
        if (tile_lo + kTile < chunk_hi) nxt = fetch_tile(text, nbytes, tile_lo + kTile);
        __syncthreads();
        // 1. kept starts
        if (t == 0) s_nslow = s_nmiss = 0;
        const Classes cl = classify16(v);
        const uint32_t kept = kept_starts(lane_starts(v, cl, s_text), cl, s_text, text, nbytes, tile_lo, wlo);
        uint64_t tot;
        uint32_t o = (uint32_t)block_excl_scan(__popc(kept), &tot, s_scan);
        // 2a. word keys, register fast path; the rest go to a compact list
        uint32_t nlong = 0;
        {
            const uint4 nx = *reinterpret_cast<const uint4*>(s_text + 16 + wlo + 16);  // next lane's window
            const uint32_t w8[8] = {v.x, v.y, v.z, v.w, nx.x, nx.y, nx.z, nx.w};
            for (uint32_t m = kept; m; m &= m - 1) {
                const uint32_t i = __builtin_ctz(m);
                TokKey k;
                bool ok;
                if (kAblate & 2) {
                    k = TokKey{(uint64_t)(wlo + i + 1) << 8, 3u, i % 26u};
                    ok = true;
                } else {
                    ok = fast_key(token_bytes(w8, i), k);
                }
                s_off[o] = (uint16_t)(wlo + i);
                if (ok) {
                    if (!(kAblate & 4)) atomicAdd(&s_hist[k.first], 1u);
                    s_key[o] = k.key;
                } else {
                    s_slow[atomicAdd(&s_nslow, 1u)] = (uint16_t)o;
                }
                o++;
            }
        }
        __syncthreads();
        // 2b. general path (inner punctuation, > 12 letters, > 16 bytes), one token per thread
        for (uint32_t q = t; q < s_nslow; q += kBlock) {
            const uint32_t j = s_slow[q];
            const uint32_t p = s_off[j];
            TokKey k = (kAblate & 16) ? TokKey{(uint64_t)(p + 1) << 8, 3u, p % 26u}
                                      : general_key(tile_block16(s_text, text, nbytes, tile_lo, p), s_text, text, nbytes,
                                                    tile_lo, p, tab.seed);
            if (kAblate & 8) k.nlet = k.nlet > 12 ? 12 : k.nlet;
            if (!(kAblate & 4)) atomicAdd(&s_hist[k.first], 1u);
            s_key[j] = k.key;
            if (k.nlet > 12) {
                s_off[j] = (uint16_t)(p | 0x8000u);
                nlong++;
            }
        }
        uint64_t ltot;
        (void)block_excl_scan(nlong, &ltot, s_scan);  // also the barrier before phase 3
        // long-token queue: LDS buffer, one global atomic per flush
        const bool direct = ltot > (uint64_t)kLongBuf;
        if (ltot && (direct || s_lcount + ltot > (uint64_t)kLongBuf)) {
            if (t == 0) s_lbase = atomicAdd((unsigned long long*)&tab.counters[C_LONG], (unsigned long long)s_lcount);
            __syncthreads();
            for (uint32_t q = t; q < s_lcount; q += kBlock) {
                if (s_lbase + q < long_cap) longs[s_lbase + q] = s_long[q];
                else atomicOr((unsigned long long*)&tab.counters[C_OVERFLOW], 2ull);
            }
            __syncthreads();
            if (t == 0) {
                s_lcount = 0;
                if (direct) s_lbase = atomicAdd((unsigned long long*)&tab.counters[C_LONG], (unsigned long long)ltot);
            }
            __syncthreads();
        }
        // 3a. probe the hot-table home slot: token q = t + u*kBlock, four
        //     loads in flight per thread; misses go to a compact list
        const uint32_t ntok = (uint32_t)tot;
        const uint32_t fsame = s_f[0] == s_f[1];
        for (uint32_t base = t; base < ntok; base += 4 * kBlock) {
            uint64_t key[4], h[4];
            unsigned long long kk[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint32_t q = base + u * kBlock;
                key[u] = q < ntok ? s_key[q] : 0ull;
                h[u] = table_hash(tab, key[u]);
            }
#pragma unroll
            for (int u = 0; u < 4; u++)
                kk[u] = (kAblate & 1) ? key[u] : (base + u * kBlock < ntok) ? tab.keys[hot_home(h[u])] : 0ull;
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const uint32_t q = base + u * kBlock;
                if (q >= ntok) continue;
                if (kk[u] != key[u]) {
                    s_slow[atomicAdd(&s_nmiss, 1u)] = (uint16_t)q;
                    continue;
                }
                const uint32_t off = s_off[q];
                const uint64_t pos = tile_lo + (off & 0x7FFFu);
                const uint32_t slot = (uint32_t)hot_home(h[u]);
                const uint32_t f = fsame ? s_f[0] : file_of(file_start, s_f[0], s_f[1], pos);
                s_key[q] = ((uint64_t)slot << 32) | file_id[f];
                if (off & 0x8000u) queue_long(direct, s_long, &s_lcount, s_lbase, longs, long_cap, tab, pos, slot);
            }
        }
        __syncthreads();
        // 3b. misses, one per thread: bucket line + big-table home in one round trip
        for (uint32_t r = t; r < s_nmiss; r += kBlock) {
            const uint32_t q = s_slow[r];
            const uint64_t key = s_key[q];
            const uint32_t off = s_off[q];
            const uint64_t pos = tile_lo + (off & 0x7FFFu);
            const uint32_t slot = table_find(tab, key, table_hash(tab, key), pos);
            const uint32_t f = fsame ? s_f[0] : file_of(file_start, s_f[0], s_f[1], pos);
            s_key[q] = ((uint64_t)slot << 32) | file_id[f];
            if (off & 0x8000u) queue_long(direct, s_long, &s_lcount, s_lbase, longs, long_cap, tab, pos, slot);
        }
        __syncthreads();
        if (direct && t == 0) s_lcount = 0;
        // 4. coalesced record store
        for (uint32_t q = t; q < ntok; q += kBlock) rec[out + q] = s_key[q];
        out += tot;
    }
    __syncthreads();
    if (s_lcount) {
        if (t == 0) s_lbase = atomicAdd((unsigned long long*)&tab.counters[C_LONG], (unsigned long long)s_lcount);
        __syncthreads();
        for (uint32_t q = t; q < s_lcount; q += kBlock) {
            if (s_lbase + q < long_cap) longs[s_lbase + q] = s_long[q];
            else atomicOr((unsigned long long*)&tab.counters[C_OVERFLOW], 2ull);
        }
    }
    if (t < 26) chunk_hist[(uint64_t)blockIdx.x * 26 + t] = s_hist[t];
}

// counters[C_HIST + l] = sum over chunks of chunk_hist[chunk][l] (one block per letter)
__global__ __launch_bounds__(kBlock) void k_hist_reduce(const uint32_t* __restrict__ chunk_hist, uint64_t nch,
                                                        uint64_t* __restrict__ counters) {
    __shared__ uint64_t s_scan[kWaves + 1];
    uint64_t acc = 0;
    for (uint64_t c = threadIdx.x; c < nch; c += kBlock) acc += chunk_hist[c * 26 + blockIdx.x];
    uint64_t tot;
    (void)block_excl_scan(acc, &tot, s_scan);
    if (threadIdx.x == 0) counters[C_HIST + blockIdx.x] = tot;
}

// number of occupied word-table slots
struct OpOccupied {
    const unsigned long long* keys;
    __device__ uint64_t value(uint64_t i) const { return keys[i] != 0ull; }
    __device__ void emit(uint64_t, uint64_t, uint64_t) const {}
};

// Next letter (0..25) of a cleaned word at *g, or 26 once the word has ended
// (whitespace, NUL, end of text, or 299 letters).
__device__ __forceinline__ uint32_t next_letter(const uint8_t* __restrict__ text, uint64_t nbytes, uint64_t* g,
                                                uint32_t* n) {
    if (*n >= (uint32_t)kMaxWord) return 26u;
    while (*g < nbytes) {
        uint32_t c = text[*g];
        if (c == 0u || is_ws(c)) break;
        (*g)++;
        uint32_t lc = letter_of(c);
        if (lc < 26u) {
            (*n)++;
            return lc;
        }
    }
    *g = nbytes;
    return 26u;
}

// Exactness check for hashed keys: every long token must spell the same word
// as its slot's representative occurrence.
__global__ __launch_bounds__(kBlock) void k_long_verify(const uint8_t* __restrict__ text, uint64_t nbytes,
                                                        const LongTok* __restrict__ longs, uint64_t nlong,
                                                        const uint64_t* __restrict__ rep, uint64_t* counters) {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < nlong; i += (uint64_t)gridDim.x * kBlock) {
        LongTok lt = longs[i];
        uint64_t a = lt.pos, b = rep[lt.slot];
        if (a == b) continue;
        uint32_t na = 0, nb = 0;
        for (;;) {
            uint32_t la = next_letter(text, nbytes, &a, &na);
            uint32_t lb = next_letter(text, nbytes, &b, &nb);
            if (la != lb) {
                atomicOr((unsigned long long*)&counters[C_COLLIDE], 1ull);
                break;
            }
            if (la == 26u) break;
        }
    }
}

// Separator contract of ii_map_device: the byte before every file start is whitespace.
__global__ void k_check_layout(const uint8_t* __restrict__ text, const uint64_t* __restrict__ file_start, uint32_t nfiles,
                               uint64_t* counters) {
    uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f == 0 || f >= nfiles) return;
    uint64_t s = file_start[f];
    if (s > 0 && !is_ws(text[s - 1])) atomicOr((unsigned long long*)&counters[C_OVERFLOW], 4ull);
}

// ---------------------------------------------------------------- dictionary
// Scan op: compact occupied table slots into dict_slot[].
struct OpCompactSlots {
    const unsigned long long* keys;
    uint32_t* dict_slot;
    __device__ uint64_t value(uint64_t i) const { return keys[i] != 0ull; }
    __device__ void emit(uint64_t i, uint64_t ex, uint64_t v) const {
        if (v) dict_slot[ex] = (uint32_t)i;
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

// ---------------------------------------------------------------- K2 support
// slot -> lexicographic id in the record's high word.
__global__ __launch_bounds__(kBlock) void k_remap(uint64_t* __restrict__ rec, uint64_t n, const uint32_t* __restrict__ remap) {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock) {
        uint64_t r = rec[i];
        rec[i] = ((uint64_t)remap[r >> 32] << 32) | (r & 0xFFFFFFFFull);
    }
}

// ---------------------------------------------------------------- K3 unique
// Records sorted by (lexid, fid): keep the first of each equal run (distinct
// fileIDs per word, main.c:176-184); post_start[lexid] = first unique index.
struct OpUnique {
    const uint64_t* rec;
    uint64_t* uniq;
    uint64_t* post_start;
    __device__ uint64_t value(uint64_t i) const { return i == 0 || rec[i] != rec[i - 1]; }
    __device__ void emit(uint64_t i, uint64_t ex, uint64_t v) const {
        if (!v) return;
        uint64_t r = rec[i];
        uniq[ex] = r;
        if (i == 0 || (r >> 32) != (rec[i - 1] >> 32)) post_start[r >> 32] = ex;
    }
};

// ---------------------------------------------------------------- K4 order
// key = letter << dbits | (dmax - df): ascending == (letter, df desc); the
// stable sort keeps lexicographic order among equal df (main.c:55-64).
__global__ __launch_bounds__(kBlock) void k_order_keys(const uint64_t* __restrict__ sk, const uint64_t* __restrict__ post_start,
                                                       uint32_t V, int dbits, uint64_t* __restrict__ okey,
                                                       uint32_t* __restrict__ oval) {
    uint32_t j = blockIdx.x * kBlock + threadIdx.x;
    if (j >= V) return;
    uint64_t df = post_start[j + 1] - post_start[j];
    uint64_t dmax = (1ull << dbits) - 1;
    uint64_t letter = (sk[j] >> 59) - 1;
    okey[j] = (letter << dbits) | (dmax - df);
    oval[j] = j;
}

// ---------------------------------------------------------------- K5 format
__device__ __forceinline__ uint32_t ndigits(uint64_t v) {
    uint32_t d = 1;
    while (v >= 10) { v /= 10; d++; }
    return d;
}

__device__ __forceinline__ void write_word(const uint8_t* __restrict__ text, uint64_t nbytes, uint64_t key, uint64_t rep,
                                           uint32_t len, uint8_t* __restrict__ o) {
    if ((key & 0xFull) == 0) {
        for (uint32_t i = 0; i < len; i++) o[i] = (uint8_t)('a' - 1 + ((key >> (59 - 5 * i)) & 31ull));
    } else {
        uint32_t n = 0;
        for (uint64_t g = rep; g < nbytes && n < len; g++) {
            uint32_t lc = letter_of(text[g]);
            if (lc < 26u) o[n++] = (uint8_t)('a' + lc);
        }
    }
}

// bytes of one posting: digits of id0+1 plus the following ' ' or ']'
struct OpPostBytes {
    const uint64_t* uniq;
    uint64_t* P;
    __device__ uint64_t value(uint64_t i) const { return ndigits((uniq[i] & 0xFFFFFFFFull) + 1) + 1; }
    __device__ void emit(uint64_t i, uint64_t ex, uint64_t) const { P[i] = ex; }
};

// line bytes in final order: "word:[" + postings + "\n"
struct OpLineOff {
    const uint32_t* ord;
    const uint32_t* lex_len;
    const uint64_t* post_start;
    const uint64_t* P;
    uint64_t* loff;  // by lexid
    __device__ uint64_t value(uint64_t i) const {
        uint32_t w = ord[i];
        return (uint64_t)lex_len[w] + 3 + (P[post_start[w + 1]] - P[post_start[w]]);
    }
    __device__ void emit(uint64_t i, uint64_t ex, uint64_t) const { loff[ord[i]] = ex; }
};

__global__ __launch_bounds__(kBlock) void k_fmt_words(const uint8_t* __restrict__ text, uint64_t nbytes,
                                                      const uint64_t* __restrict__ lex_key, const uint64_t* __restrict__ lex_rep,
                                                      const uint32_t* __restrict__ lex_len,
                                                      const uint64_t* __restrict__ post_start, const uint64_t* __restrict__ P,
                                                      const uint64_t* __restrict__ loff, uint32_t V, uint8_t* __restrict__ out) {
    uint32_t j = blockIdx.x * kBlock + threadIdx.x;
    if (j >= V) return;
    uint64_t o = loff[j];
    uint32_t len = lex_len[j];
    write_word(text, nbytes, lex_key[j], lex_rep[j], len, out + o);
    out[o + len] = ':';
    out[o + len + 1] = '[';
    out[o + len + 3 + (P[post_start[j + 1]] - P[post_start[j]]) - 1] = '\n';
}

__global__ __launch_bounds__(kBlock) void k_fmt_posts(const uint64_t* __restrict__ uniq, uint64_t U,
                                                      const uint32_t* __restrict__ lex_len,
                                                      const uint64_t* __restrict__ post_start, const uint64_t* __restrict__ P,
                                                      const uint64_t* __restrict__ loff, uint8_t* __restrict__ out) {
    for (uint64_t p = (uint64_t)blockIdx.x * kBlock + threadIdx.x; p < U; p += (uint64_t)gridDim.x * kBlock) {
        uint64_t r = uniq[p];
        uint32_t w = (uint32_t)(r >> 32);
        uint64_t id = (r & 0xFFFFFFFFull) + 1;
        uint64_t ps = post_start[w];
        uint64_t o = loff[w] + lex_len[w] + 2 + (P[p] - P[ps]);
        uint32_t nd = ndigits(id);
        for (int i = (int)nd - 1; i >= 0; i--) { out[o + i] = (uint8_t)('0' + id % 10); id /= 10; }
        out[o + nd] = (p + 1 == post_start[w + 1]) ? ']' : ' ';
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

__global__ __launch_bounds__(kBlock) void k_export_pairs(const uint64_t* __restrict__ uniq, uint64_t p0, uint64_t p1,
                                                         uint32_t j0, uint64_t* __restrict__ out) {
    for (uint64_t p = p0 + (uint64_t)blockIdx.x * kBlock + threadIdx.x; p < p1; p += (uint64_t)gridDim.x * kBlock) {
        uint64_t r = uniq[p];
        out[p - p0] = (((r >> 32) - j0) << 32) | (r & 0xFFFFFFFFull);
    }
}

__global__ void k_export_header(uint64_t* __restrict__ h, uint64_t nwords, uint64_t npairs, uint64_t arena, uint64_t llo,
                                uint64_t lhi) {
    if (threadIdx.x == 0) {
        h[0] = kSegMagic; h[1] = nwords; h[2] = npairs; h[3] = arena; h[4] = llo; h[5] = lhi; h[6] = 0; h[7] = 0;
    }
}

// received pair -> (global lexid, id0): word k of the merged word text was
// tokenised into wrec[k] = slot << 32; remap gives the owner's lexicographic id
__global__ __launch_bounds__(kBlock) void k_import_pairs(const uint64_t* __restrict__ pairs, uint64_t np, uint64_t wbase,
                                                         const uint64_t* __restrict__ wrec,
                                                         const uint32_t* __restrict__ remap, uint64_t* __restrict__ out) {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < np; i += (uint64_t)gridDim.x * kBlock) {
        uint64_t r = pairs[i];
        uint64_t slot = wrec[wbase + (r >> 32)] >> 32;
        out[i] = ((uint64_t)remap[slot] << 32) | (r & 0xFFFFFFFFull);
    }
}

}  // namespace ii
