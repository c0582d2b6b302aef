// ii_partial.h — partial-file emitter.
//
// The reference's mappers write every kept token as the line
// "<clean word> <id0+1>\n" to partial_<first letter>.txt (main.c:113-118,
// format at main.c:116; files created at main.c:332-341).  The index itself
// never needs these files (K1 keeps the records in HBM), so this is an
// optional compatibility / debugging output, built on the device from the
// resident text alone (no word table, no records):
//
//   pieces   the host cuts every file, in the caller's emission order, into
//            pieces of at most kPartPiece bytes (a piece lies inside one file)
//   count    one workgroup per piece: bytes each letter's lines take
//            -> cnt[letter][piece] (letter-major)
//   scan     one exclusive scan over the flattened [26][npieces] array gives
//            every (letter, piece) its offset in the 26 texts laid back to back
//   write    one workgroup per piece: per-thread per-letter byte counts, 26
//            block scans, then every thread writes its lines in text order
//
// A line's bytes: cleaned letters (<= 299, main.c:105) + ' ' + digits of
// id0+1 + '\n'.  Inside a piece tokens keep their text order, pieces keep the
// caller's order, so with the order of one mapper's files (main.c:93, files
// sorted by size, main.c:300) the text is byte-identical to the reference's
// partial_<l>.txt for M = 1.  With M > 1 the reference's line order depends
// on thread timing (all mappers share each FILE*, main.c:116); the order
// given here (mapper 0's files, then mapper 1's, ...) is one of its outcomes.
#pragma once
#include "ii_kernels.h"

namespace ii {

struct PartPiece {
    uint64_t lo, hi;  // byte range of the piece (inside one file)
    uint32_t id0, pad;
};
constexpr int kPartSeg = 256;                           // bytes of a piece per thread
constexpr uint64_t kPartPiece = (uint64_t)kPartSeg * kBlock;  // 64 KiB

// The token starting at p: its first kept letter (26 if it keeps none) and
// the number of letters kept (scanning stops at whitespace, at a NUL or
// after 299 letters: main.c:102-111).
__device__ __forceinline__ uint32_t part_token(const uint8_t* __restrict__ text, uint64_t nbytes, uint64_t p,
                                               uint32_t& len) {
    uint32_t first = 26, n = 0;
    for (uint64_t q = p; q < nbytes && n < (uint32_t)kMaxWord; q++) {
        const uint32_t ch = text[q];
        if (ch == 0 || is_ws(ch)) break;
        const uint32_t l = letter_of(ch);
        if (l < 26) {
            if (n == 0) first = l;
            n++;
        }
    }
    len = n;
    return first;
}

// Visits the tokens that start in this thread's segment of the piece.
template <class F>
__device__ __forceinline__ void part_tokens(const uint8_t* __restrict__ text, uint64_t nbytes, const PartPiece& pp,
                                            F&& f) {
    const uint64_t s0 = pp.lo + (uint64_t)threadIdx.x * kPartSeg;
    const uint64_t s1 = s0 + kPartSeg < pp.hi ? s0 + kPartSeg : pp.hi;
    if (s0 >= s1) return;
    uint32_t prev = s0 > 0 ? text[s0 - 1] : 32u;  // a file start follows a whitespace byte (separator contract)
    for (uint64_t p = s0; p < s1; p++) {
        const uint32_t ch = text[p];
        if (!is_ws(ch) && is_ws(prev)) {
            uint32_t len;
            const uint32_t l = part_token(text, nbytes, p, len);
            if (l < 26) f(p, l, len);
        }
        prev = ch;
    }
}

__global__ __launch_bounds__(kBlock) void k_part_count(const uint8_t* __restrict__ text, uint64_t nbytes,
                                                       const PartPiece* __restrict__ pieces, uint32_t np,
                                                       uint64_t* __restrict__ cnt) {
    __shared__ uint32_t s[26];
    if (threadIdx.x < 26) s[threadIdx.x] = 0;
    __syncthreads();
    const PartPiece pp = pieces[blockIdx.x];
    const uint32_t extra = id_digits(pp.id0 + 1ull) + 2;  // ' ' + digits + '\n'
    part_tokens(text, nbytes, pp, [&](uint64_t, uint32_t l, uint32_t len) { atomicAdd(&s[l], len + extra); });
    __syncthreads();
    if (threadIdx.x < 26) cnt[(uint64_t)threadIdx.x * np + blockIdx.x] = s[threadIdx.x];
}

__global__ __launch_bounds__(kBlock) void k_part_write(const uint8_t* __restrict__ text, uint64_t nbytes,
                                                       const PartPiece* __restrict__ pieces, uint32_t np,
                                                       const uint64_t* __restrict__ off, uint8_t* __restrict__ out) {
    __shared__ uint32_t s[26][kBlock];
    __shared__ uint64_t sc[kWaves + 1];
    const uint32_t t = threadIdx.x;
    for (int l = 0; l < 26; l++) s[l][t] = 0;
    const PartPiece pp = pieces[blockIdx.x];
    const uint64_t id = pp.id0 + 1ull;
    const uint32_t nd = id_digits(id);
    part_tokens(text, nbytes, pp, [&](uint64_t, uint32_t l, uint32_t len) { s[l][t] += len + nd + 2; });
    for (int l = 0; l < 26; l++) {  // thread t's first byte inside (letter, piece)
        uint64_t tot;
        s[l][t] = (uint32_t)block_excl_scan(s[l][t], &tot, sc);
    }
    char digits[10];
    uint64_t v = id;
    for (int i = (int)nd - 1; i >= 0; i--) {
        digits[i] = (char)('0' + v % 10);
        v /= 10;
    }
    part_tokens(text, nbytes, pp, [&](uint64_t p, uint32_t l, uint32_t len) {
        uint8_t* o = out + off[(uint64_t)l * np + blockIdx.x] + s[l][t];
        uint32_t n = 0;
        for (uint64_t q = p; n < len; q++) {
            const uint32_t ch = text[q];
            if (letter_of(ch) < 26) o[n++] = (uint8_t)(ch | 0x20u);  // A-Z + 32 (main.c:106-107)
        }
        o[n++] = ' ';
        for (uint32_t i = 0; i < nd; i++) o[n++] = (uint8_t)digits[i];
        o[n++] = '\n';
        s[l][t] += n;
    });
}

// letter_off[l] = offset of letter l's text (off[l * np]), letter_off[26] = total
__global__ void k_part_letter_off(const uint64_t* __restrict__ off, uint32_t np, const uint64_t* __restrict__ total,
                                  uint64_t* __restrict__ letter_off) {
    const uint32_t l = threadIdx.x;
    if (l < 26) letter_off[l] = np ? off[(uint64_t)l * np] : 0;
    if (l == 26) letter_off[26] = np ? *total : 0;
}

}  // namespace ii
