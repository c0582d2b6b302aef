// ii_kernels.h — the inverted-index kernels (K1..K5) for MI355X (gfx950).
//
// Reference path replaced (see DESIGN.md for the full map):
//   K1 k_tokenize      mapper() hot loop, main.c:102-118, + partial files main.c:116
//   K1 k_long_tokens   same, for words longer than 12 letters
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
constexpr uint32_t kSlotLong = 0xFFFFFFFEu;  // > 12 letters: finished by k_long_tokens

// counters[] layout (u64)
enum : int {
    C_LONG = 0,      // long tokens appended
    C_OVERFLOW = 1,  // word table probe limit hit / long list full
    C_INSERT = 2,    // distinct keys inserted
    C_COLLIDE = 3,   // long-word hash collision detected
    C_HIST = 4,      // 26 first-letter counters
    C_TIES = 30,     // dictionary entries sharing a 12-letter prefix
    C_MAXLEN = 31,   // longest tied word
    C_NUM = 32
};

struct LongTok {
    uint64_t pos;   // token start in text
    uint64_t rec;   // record index
    uint64_t fid;   // file id (u32)
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
// Open addressing, linear probing, 64-bit keys, 0 = empty.  Keys are exact for
// words of <= 12 letters (5-bit letter codes, left aligned, low 4 bits 0) and a
// 60-bit hash tagged 0xF for longer words (verified after the map, see
// k_long_verify).  Keys never change once set, so a stale empty read is fixed
// by the CAS.  The slot index is the word's provisional id.
struct Table {
    unsigned long long* keys;
    uint64_t* rep;      // token start of the inserting occurrence
    uint64_t mask;
    uint64_t seed;
    uint64_t* counters;
};

__device__ __forceinline__ uint32_t table_insert(const Table& t, uint64_t key, uint64_t pos) {
    uint64_t h = mix64(key ^ t.seed) & t.mask;
    for (int probe = 0; probe < kMaxProbe; probe++) {
        unsigned long long k = t.keys[h];
        if (k == key) return (uint32_t)h;
        if (k == 0ull) {
            unsigned long long old = atomicCAS(&t.keys[h], 0ull, (unsigned long long)key);
            if (old == 0ull) {
                t.rep[h] = pos;
                atomicAdd((unsigned long long*)&t.counters[C_INSERT], 1ull);
                return (uint32_t)h;
            }
            if (old == key) return (uint32_t)h;
        }
        h = (h + 1) & t.mask;
    }
    atomicOr((unsigned long long*)&t.counters[C_OVERFLOW], 1ull);
    return 0;
}

// ---------------------------------------------------------------- K1 tokenizer
struct Walk {
    uint64_t packed;  // first 12 letter codes (1..26), left aligned
    uint32_t nlet;    // letters seen, stops counting at 13
    uint32_t first;   // first letter index
};

// Walk a token from tile-local byte p: cleaning loop of main.c:105-111 (stops at
// NUL, whitespace, or once a 13th letter shows the word is "long").
__device__ __forceinline__ Walk walk_token(const uint8_t* s, const uint8_t* __restrict__ text, uint64_t nbytes,
                                           uint64_t tile_lo, uint32_t p) {
    Walk w{0ull, 0u, 0u};
    for (uint32_t j = p;; j++) {
        uint32_t c;
        if (j < (uint32_t)(kTile + kHalo)) c = s[16 + j];
        else {
            uint64_t g = tile_lo + j;
            c = g < nbytes ? text[g] : 32u;
        }
        if (c == 0u || is_ws(c)) break;
        uint32_t lc = letter_of(c);
        if (lc < 26u) {
            if (w.nlet == 0) w.first = lc;
            w.nlet++;
            if (w.nlet > 12) break;
            w.packed |= (uint64_t)(lc + 1) << (64 - 5 * w.nlet);
        }
    }
    return w;
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

// kEmit = false: count kept tokens per chunk -> chunk_cnt[blockIdx.x].
// kEmit = true : chunk_cnt holds exclusive offsets; write records
//                rec[i] = slot << 32 | fid in text order, insert words into the
//                table, count first letters, and queue long tokens.
template <bool kEmit>
__global__ __launch_bounds__(kBlock) void k_tokenize(const uint8_t* __restrict__ text, uint64_t nbytes,
                                                     const uint64_t* __restrict__ file_start,
                                                     const uint32_t* __restrict__ file_id, uint32_t nfiles,
                                                     uint64_t* __restrict__ chunk_cnt, Table tab,
                                                     uint64_t* __restrict__ rec, LongTok* __restrict__ longs,
                                                     uint64_t long_cap) {
    __shared__ __attribute__((aligned(16))) uint8_t s_text[16 + kTile + kHalo];
    __shared__ uint32_t s_slot[kEmit ? kTile : 1];
    __shared__ uint64_t s_scan[kWaves + 1];
    __shared__ uint32_t s_hist[32];
    __shared__ uint32_t s_f[2];

    const uint64_t chunk_lo = (uint64_t)blockIdx.x * kChunk;
    const uint64_t chunk_hi = chunk_lo + kChunk < nbytes ? chunk_lo + kChunk : nbytes;
    const int t = threadIdx.x;
    if (t < 32) s_hist[t] = 0;
    if (kEmit && t == 0) {
        s_f[0] = file_of(file_start, 0, nfiles - 1, chunk_lo);
        s_f[1] = file_of(file_start, s_f[0], nfiles - 1, chunk_hi - 1);
    }
    uint64_t out = kEmit ? chunk_cnt[blockIdx.x] : 0;
    uint64_t kept_all = 0;

    for (uint64_t tile_lo = chunk_lo; tile_lo < chunk_hi; tile_lo += kTile) {
        __syncthreads();
        // stage [tile_lo - 16, tile_lo + kTile + kHalo) in 16-byte pieces; bytes
        // outside the text read as ' ' (so position 0 starts a token).
        for (int q = t; q < (16 + kTile + kHalo) / 16; q += kBlock) {
            const int64_t g = (int64_t)tile_lo - 16 + (int64_t)q * 16;
            uint4 v;
            if (g >= 0 && (uint64_t)g + 16 <= nbytes) {
                v = *reinterpret_cast<const uint4*>(text + g);
            } else {
                uint8_t b[16];
#pragma unroll
                for (int i = 0; i < 16; i++) {
                    int64_t gi = g + i;
                    b[i] = (gi >= 0 && (uint64_t)gi < nbytes) ? text[gi] : (uint8_t)32;
                }
                v = *reinterpret_cast<uint4*>(b);
            }
            *reinterpret_cast<uint4*>(s_text + q * 16) = v;
        }
        __syncthreads();

        const uint32_t wlo = (uint32_t)t * 16;
        // token starts in this lane's 16 bytes: non-space after space (main.c:102)
        uint32_t starts = 0;
        {
            uint32_t prev = s_text[16 + wlo - 1];
#pragma unroll
            for (int i = 0; i < 16; i++) {
                uint32_t c = s_text[16 + wlo + i];
                if (!is_ws(c) && is_ws(prev)) starts |= 1u << i;
                prev = c;
            }
        }
        uint32_t kept = 0;
        for (uint32_t m = starts; m; m &= m - 1) {
            const uint32_t i = __builtin_ctz(m);
            Walk w = walk_token(s_text, text, nbytes, tile_lo, wlo + i);
            if (w.nlet == 0) {
                if (kEmit) s_slot[wlo + i] = kSlotNone;
                continue;
            }
            kept++;
            if (kEmit) {
                atomicAdd(&s_hist[w.first], 1u);
                s_slot[wlo + i] = w.nlet <= 12 ? table_insert(tab, w.packed, tile_lo + wlo + i) : kSlotLong;
            }
        }
        if (!kEmit) {
            kept_all += kept;
            continue;
        }
        uint64_t tot;
        uint64_t o = out + block_excl_scan(kept, &tot, s_scan);
        out += tot;
        if (kept) {
            const uint64_t gpos = tile_lo + wlo;
            uint32_t f = file_of(file_start, s_f[0], s_f[1], gpos);
            for (uint32_t m = starts; m; m &= m - 1) {
                const uint32_t i = __builtin_ctz(m);
                const uint32_t slot = s_slot[wlo + i];
                if (slot == kSlotNone) continue;
                const uint64_t pos = gpos + i;
                while (f < s_f[1] && file_start[f + 1] <= pos) f++;
                const uint32_t fid = file_id[f];
                if (slot == kSlotLong) {
                    uint64_t li = atomicAdd((unsigned long long*)&tab.counters[C_LONG], 1ull);
                    if (li < long_cap) longs[li] = LongTok{pos, o, fid};
                    else atomicOr((unsigned long long*)&tab.counters[C_OVERFLOW], 2ull);
                    rec[o] = fid;
                } else {
                    rec[o] = ((uint64_t)slot << 32) | fid;
                }
                o++;
            }
        }
    }
    if (!kEmit) {
        uint64_t tot;
        (void)block_excl_scan(kept_all, &tot, s_scan);
        if (t == 0) chunk_cnt[blockIdx.x] = tot;
    } else {
        __syncthreads();
        if (t < 26 && s_hist[t]) atomicAdd((unsigned long long*)&tab.counters[C_HIST + t], (unsigned long long)s_hist[t]);
    }
}

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

__device__ __forceinline__ uint64_t long_key(const LongWord& w, uint64_t seed) {
    return (mix64(w.hash ^ seed ^ ((uint64_t)w.len << 48)) << 4) | 0xFull;
}

__global__ __launch_bounds__(kBlock) void k_long_tokens(const uint8_t* __restrict__ text, uint64_t nbytes,
                                                        const LongTok* __restrict__ longs, uint64_t nlong, Table tab,
                                                        uint64_t* __restrict__ rec) {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < nlong; i += (uint64_t)gridDim.x * kBlock) {
        LongTok lt = longs[i];
        LongWord w = read_word(text, nbytes, lt.pos);
        uint32_t slot = table_insert(tab, long_key(w, tab.seed), lt.pos);
        rec[lt.rec] = ((uint64_t)slot << 32) | lt.fid;
    }
}

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
                                                        const uint64_t* __restrict__ rec, const uint64_t* __restrict__ rep,
                                                        uint64_t* counters) {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < nlong; i += (uint64_t)gridDim.x * kBlock) {
        LongTok lt = longs[i];
        uint64_t a = lt.pos, b = rep[rec[lt.rec] >> 32];
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
