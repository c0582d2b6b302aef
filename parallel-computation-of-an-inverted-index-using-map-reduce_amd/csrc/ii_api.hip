// ii_api.hip — C ABI (include/ii.h) and host orchestration of the MI355X
// inverted-index pipeline.  One context = one GPU = one HIP stream; every
// buffer is device-resident and reused across calls (grown on demand, never
// freed inside the pipeline), sized for HBM3E rather than for a CPU page cache.
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <fcntl.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <vector>

#include "../../include/ii.h"
#include "ii_kernels.h"
#include "ii_partial.h"
#include "ii_reader.h"


using namespace ii;

namespace {

struct DBuf {
    void* p = nullptr;
    size_t cap = 0;
};

constexpr int kMaxTimedPasses = 16;

}  // namespace

struct ii_ctx {
    int dev = 0;
    hipStream_t st = nullptr;
    hipStream_t st2 = nullptr;  // side stream: the exactness check of hashed keys (k_long_verify) beside the reduce
    bool lv_pending = false;    // a k_long_verify on st2 whose verdict the host has not read yet (ev_res[1])
    bool test_collide = false;  // test knob II_TEST_COLLIDE=1: the first check of the context reports a collision
    uint32_t collide_retries = 0;
    int test_long_bits = 64;    // test knob II_TEST_LONG_KEY_BITS=b: the first map of a context hashes long words to b bits
    uint64_t* hbuf = nullptr;   // pinned host words for readbacks queued before a later sync (kHbufWords):
                                // [0] collide verdict, [1] V check, [2, 4) K3, [4, 8) MSD, [16, 64) map, [64, ) read_u64
    hipEvent_t ev_rd = nullptr;  // after a readback queued ahead of further work (read_wait)

    // input
    DBuf text_own;  // text copied in by ii_map_host / ii_map_files
    const uint8_t* text = nullptr;
    uint64_t nbytes = 0;
    uint32_t nfiles = 0;
    uint32_t id_bound = 0;  // 1 + largest file id0 (bounds df)
    // the mapped files' id0s are fid_off, fid_off + 1, ... (a caller's id range; ii_partition's size-sorted
    // shares are not): K3 adds fid_off to K1's shard-local file index instead of gathering fid[index]
    bool fid_affine = true;
    // the packed token sort's first pass maps shard-local file indices to id0s (local_reduce):
    // the sorted records then carry id0s, and K3 gathers nothing
    const uint32_t* s0_fmap = nullptr;
    uint32_t fid_off = 0;
    IdDigitsTh dth{};       // K3's posting bytes by file index (pair_bytes)
    DBuf fstart, fid;
    std::vector<uint64_t> h_fstart;  // host copies of the mapped files' starts / ids
    std::vector<uint32_t> h_fid;

    // scratch
    DBuf partial, totals, counters, chunk_cnt, chunk_hist, rtable, kept;
    DBuf partial2, rtable2, kept2;  // the same scratch for work queued on st2 (SideScope)
    // K1
    DBuf rec, rec2, longs, pend, pend_cnt, chunk_files;
    DBuf tkeys, trep;
    uint64_t big_cap = 1ull << 22;  // big word table; total slots = kHotSlots + big_cap
    uint64_t big_next = 0;          // big_cap for the next map, from the last local reduce's V (0: keep)
    bool big_fixed = false;         // II_TABLE_LOG2 set the capacity (a test knob): never shrunk
    uint64_t long_cap = 0;
    uint64_t seed = 0x51ed270b27a3f3c1ull;
    // dictionary
    DBuf dslot, dkey, dkey2, didx, didx2, remap, lkey, lrep, llen, lstart;
    DBuf tied, tpos, rid, rfirst, tdict, tk, tk2, tv, tv2;
    // reduce / order / format
    DBuf uniq, pstart, pstop, pstart_w, pstop_w, okey, okey2, oval, oval2, P, loff, out, letter_off;
    DBuf pstart_x;  // exchange after a word-id reduce: each word's first pair in lexid order (letter_points)
    DBuf mstart, mend;      // ii_import merge: per (word, source) run start / end -> merged offset
    DBuf moff;              // ii_import merge-path rounds: the left run's share before every tile (k_merge_partition)
    DBuf wmap, lexw, widl;  // wid keys (single-GPU reduce): big slot -> wid, wid -> lexid, lexid -> wid
    DBuf drank, g64;        // compact pairs: hot slot -> dense word index; word key of every 64th pair
    bool pairs32 = false;   // uniq holds compact u32 pairs (k_uniq_sweep uniq32): formatted, never exported
    DBuf fbase;             // per word key: output byte of its first posting minus P[first pair]
    DBuf dhist, lbstat, ticket;  // onesweep token-sort passes: digit counts / bases, look-back entries, tile ticket
    DBuf shist;                  // run_sort_sweep: every pass's digit counts, then bases
    bool on_side = false;        // inside a SideScope (c->st is st2): the look-back buffers belong to the main stream
    DBuf msd;                    // packed token sort: bucket geometry, per-bucket digit counts and bases
    DBuf tbk;                    // packed token sort: bucket of every tile (u16)
    uint64_t lb_cap = 0;         // look-back entries allocated (and cleared)
    uint64_t lb_epoch = 0;       // epoch of the last onesweep pass
    bool wid_pairs = false; // the partial index came from a wid-keyed sort (no letter-contiguous pairs)
    bool xpairs = false;    // pstart_x holds this partial index's lexid-order word starts
    uint64_t NW = 0;        // wid range
    // partial-file emitter (ii_partials)
    DBuf ppieces, pcnt, pout, ploff;
    std::vector<char> part_host;
    uint64_t h_part_off[II_ALPHABET + 1] = {0};
    bool part_valid = false;
    bool text_is_input = false;  // c->text holds mapped input files (not an imported word arena)
    // exchange
    DBuf woff, pts;
    uint64_t h_pts[3 * (II_ALPHABET + 1)] = {0};
    int planned_parts = 0;
    int part_lo[II_MAX_PARTS] = {0}, part_hi[II_MAX_PARTS] = {0};  // letter range of every export part

    uint64_t T = 0, V = 0, U = 0, nlong = 0, out_bytes = 0;
    int test_lb_timeout = 0;  // test knob II_TEST_LB_TIMEOUT: the look-back timeout flag raised after K3 (1),
                              // after the token sort (sort: K3 must skip its work), after a key + value sort
                              // by onesweep passes (sweep) or after the final-order sort (order); the reduce
                              // (or the owner's import) must fail
    uint32_t retries = 0;
    bool mapped = false, have_pairs = false, reduced = false;
    uint64_t* rec_sorted = nullptr;
    uint32_t* ord = nullptr;
    uint64_t hist[II_ALPHABET] = {0};
    uint64_t h_letter_off[II_ALPHABET + 1] = {0};
    std::vector<char> host_text;
    bool host_valid = false;

    hipEvent_t ev[8] = {};
    hipEvent_t ev_emit[2] = {};  // around the last (successful) k_tok_emit launch
    hipEvent_t ev_res[2] = {};   // around the last k_long_verify launch (none: no long tokens)
    hipEvent_t ev_sc[2 * kMaxTimedPasses] = {};
    uint64_t sc_bytes[kMaxTimedPasses] = {0};  // algorithmic bytes of each timed scatter launch
    int n_sc = 0;
    uint64_t T_sorted = 0;  // records left after the pass-0 dedup
    hipEvent_t ev_c0[2] = {};  // around k_sort0_compact
    hipEvent_t ev_dict[2] = {};  // the dictionary's lexicographic part on st2: may start / done
    uint64_t c0_bytes = 0;     // its algorithmic bytes (records read + kept records written)
    bool sort_packed = false;  // the last token sort ran in the packed form (run_sort_packed)
    int sort_W = 0, sort_F = 0;  // its key / file-index bits
    uint64_t sort_hist_bytes = 0;  // its bucket-histogram reads
    // packed form: the sorted u32 records' layout (bucket geometry in msd, bits), for K3
    uint32_t pk_nb = 0, pk_ntb = 0;
    uint64_t pk_ncap = 0;  // u32 records K3 may load (the padded layout's extent)
    int ncu = 256;         // compute units (persistent launches)
    int pk_F = 0, pk_L = 0;
    uint64_t n_pending = 0; // tokens K1b left to K1c
    bool deep_probe = false; // K1b's DeepProbe: most distinct words of the context's last reduce lived in the big table
    uint32_t rec_lbits = 0;  // the last map's narrow records: slot << rec_lbits | file - the chunk's first file
    bool map_deep = false;   // the last map ran K1b with DeepProbe
    uint64_t rec_cap = 0;   // K1 record layout: kChunkCap per chunk, or 0 = dense (counted)
    uint64_t nch_map = 0;   // K1b chunks of the last map
    // pipelined file reader (ii_map_files): per thread a stream and two pinned windows
    std::vector<hipStream_t> io_st;
    std::vector<uint8_t*> io_buf;
    std::vector<hipEvent_t> io_ev;
    double io_ms = 0;       // host wall time of the last ii_map_files read + upload
    uint64_t io_bytes = 0;
    ii_stats stats;
};

// A sticky device error (a kernel's illegal memory access, an abort, a lost
// device) leaves every queue of the process unusable: after it, a wait on an
// event or a stream of ANY context may never return (round 3: a CLI with
// eight contexts on one device sat in such waits after the first context's
// copy reported the fault).  The first sticky error poisons the library: every
// later entry point returns II_ERR_HIP at once, with no HIP call, and
// ii_close releases nothing on the device (the process is expected to exit).
static volatile int g_poisoned = 0;
static void note_hip_error(hipError_t e) {
    switch (e) {
        case hipErrorIllegalAddress:
        case hipErrorLaunchFailure:
        case hipErrorAssert:
        case hipErrorLaunchTimeOut:
        case hipErrorECCNotCorrectable:
        case hipErrorNoDevice:
        case hipErrorContextIsDestroyed:
            __atomic_store_n(&g_poisoned, 1, __ATOMIC_SEQ_CST);
            break;
        default:
            break;
    }
}
static inline bool poisoned() { return __atomic_load_n(&g_poisoned, __ATOMIC_SEQ_CST) != 0; }
// A HIP result checked by hand (reader threads, timers, memory queries): true on
// success; a failure is recorded like HIPCK's, so a sticky fault first seen
// there still poisons the library.
static inline bool hip_ok(hipError_t e) {
    if (e == hipSuccess) return true;
    note_hip_error(e);
    return false;
}

#define HIPCK(x)                                                                               \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            note_hip_error(e_);                                                                \
            fprintf(stderr, "libii: %s failed: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, \
                    __LINE__);                                                                 \
            return II_ERR_HIP;                                                                 \
        }                                                                                      \
    } while (0)

// entry-point guard: no HIP call after a sticky error
#define LIVE_OR_FAIL()                   \
    do {                                 \
        if (poisoned()) return II_ERR_HIP; \
    } while (0)

#define CK(x)                   \
    do {                        \
        int r_ = (x);           \
        if (r_ != II_OK) return r_; \
    } while (0)

static int grow(DBuf& b, size_t bytes) {
    if (bytes <= b.cap && b.p) return II_OK;
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.cap = 0;
    size_t want = std::max<size_t>(bytes + bytes / 8, 256);
    if (!hip_ok(hipMalloc(&b.p, want))) {
        (void)hipGetLastError();
        if (!hip_ok(hipMalloc(&b.p, std::max<size_t>(bytes, 256)))) {
            (void)hipGetLastError();
            b.p = nullptr;
            return II_ERR_NOMEM;
        }
        want = std::max<size_t>(bytes, 256);
    }
    b.cap = want;
    return II_OK;
}

template <class T>
static T* P_(DBuf& b) {
    return reinterpret_cast<T*>(b.p);
}

static inline uint32_t grid_for(uint64_t n) { return (uint32_t)std::max<uint64_t>(1, (n + kBlock - 1) / kBlock); }
static inline double now_ms() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}
static inline int bitlen(uint64_t v) { return v ? 64 - __builtin_clzll(v) : 0; }
// bytes the packed token sort's u32 layout of n records may take (every bucket padded to whole tiles)
// (n + (kMsdMax + 1) tiles: every bucket's last tile padded, plus the launch's whole tiles, k_onesweep_seg ncap)
static inline size_t packed_bytes(uint64_t n) { return sizeof(uint32_t) * (n + (uint64_t)(kMsdMax + 1) * kSweepTile); }

// ----------------------------------------------------------------- scan / sort
// Readbacks go through the pinned words c->hbuf: a copy into pageable memory is a synchronisation of its
// own (two in a row cost two host round trips of GPU idle time).
constexpr size_t kHbufWords = 128, kHbufRead = 64;
constexpr size_t kHbufLbFlag = 12;  // counters[C_OVERFLOW] read with the dictionary's and K4's readbacks
static int read_u64(ii_ctx* c, const void* dptr, uint64_t* out, size_t n = 1) {
    if (n > kHbufWords - kHbufRead) {  // (larger tables: straight into the caller's memory)
        HIPCK(hipMemcpyAsync(out, dptr, n * sizeof(uint64_t), hipMemcpyDeviceToHost, c->st));
        HIPCK(hipStreamSynchronize(c->st));
        return II_OK;
    }
    HIPCK(hipMemcpyAsync(c->hbuf + kHbufRead, dptr, n * sizeof(uint64_t), hipMemcpyDeviceToHost, c->st));
    HIPCK(hipStreamSynchronize(c->st));
    memcpy(out, c->hbuf + kHbufRead, n * sizeof(uint64_t));
    return II_OK;
}
// A readback queued ahead of more work (read_queue ... launches ... read_wait): the host wakes while the
// later kernels run, and what it launches next is queued behind them, so the GPU does not idle for the
// round trip.  (hbuf words [at, at + n), at + n <= kHbufRead.)
static int read_queue(ii_ctx* c, const void* dptr, size_t at, size_t n) {
    HIPCK(hipMemcpyAsync(c->hbuf + at, dptr, n * sizeof(uint64_t), hipMemcpyDeviceToHost, c->st));
    HIPCK(hipEventRecord(c->ev_rd, c->st));
    return II_OK;
}
static int read_wait(ii_ctx* c, uint64_t* out, size_t at, size_t n) {
    HIPCK(hipEventSynchronize(c->ev_rd));
    memcpy(out, c->hbuf + at, n * sizeof(uint64_t));
    return II_OK;
}

template <class Op>
static int run_scan(ii_ctx* c, Op op, uint64_t n, uint64_t* d_total) {
    if (n == 0) {
        if (d_total) HIPCK(hipMemsetAsync(d_total, 0, sizeof(uint64_t), c->st));
        return II_OK;
    }
    if (n <= kScanSingleMax) {  // (one launch)
        k_scan_single<Op><<<1, kScanSingleThreads, 0, c->st>>>(op, n, d_total);
        HIPCK(hipGetLastError());
        return II_OK;
    }
    uint64_t nch = std::min<uint64_t>(kMaxChunks, (n + kBlock - 1) / kBlock);
    uint64_t chunk = ((n + nch - 1) / nch + kBlock - 1) / kBlock * kBlock;
    nch = (n + chunk - 1) / chunk;
    uint64_t* part = P_<uint64_t>(c->partial);
    k_scan_reduce<Op><<<(uint32_t)nch, kBlock, 0, c->st>>>(op, n, chunk, part);
    k_scan_partials<<<1, kBlock, 0, c->st>>>(part, (uint32_t)nch, d_total);
    k_scan_apply<Op><<<(uint32_t)nch, kBlock, 0, c->st>>>(op, n, chunk, part);
    HIPCK(hipGetLastError());
    return II_OK;
}

// Sum of op.value over [0, n) -> *d_total (reduce + partials only).
template <class Op>
static int run_reduce(ii_ctx* c, Op op, uint64_t n, uint64_t* d_total) {
    if (n == 0) {
        HIPCK(hipMemsetAsync(d_total, 0, sizeof(uint64_t), c->st));
        return II_OK;
    }
    uint64_t nch = std::min<uint64_t>(kMaxChunks, (n + kBlock - 1) / kBlock);
    uint64_t chunk = ((n + nch - 1) / nch + kBlock - 1) / kBlock * kBlock;
    nch = (n + chunk - 1) / chunk;
    uint64_t* part = P_<uint64_t>(c->partial);
    k_scan_reduce<Op><<<(uint32_t)nch, kBlock, 0, c->st>>>(op, n, chunk, part);
    k_scan_partials<<<1, kBlock, 0, c->st>>>(part, (uint32_t)nch, d_total);
    HIPCK(hipGetLastError());
    return II_OK;
}

// pending tokens of a chunk: two 16-bit counts (k_tok_emit)
struct OpPendCount {
    const uint32_t* a;
    __device__ uint64_t value(uint64_t i) const { return (a[i] & 0xFFFFu) + (a[i] >> 16); }
    __device__ void emit(uint64_t, uint64_t, uint64_t) const {}
};

struct OpInPlace {
    uint64_t* a;
    __device__ uint64_t value(uint64_t i) const { return a[i]; }
    __device__ void emit(uint64_t i, uint64_t ex, uint64_t) const { a[i] = ex; }
};

// Look-back state for one decoupled-look-back launch with `entries` 8-byte
// granules: a new epoch (entries of earlier launches then read as "not yet
// published", so nothing is cleared between launches; cleared once when the
// buffer grows or the 24-bit epoch wraps) and a zeroed tile ticket.
static int lookback_pass(ii_ctx* c, uint64_t entries) {
    CK(grow(c->ticket, sizeof(uint32_t) * 4));
    if (c->lb_cap < entries) {
        CK(grow(c->lbstat, sizeof(uint64_t) * entries));
        c->lb_cap = c->lbstat.cap / sizeof(uint64_t);
        HIPCK(hipMemsetAsync(c->lbstat.p, 0, c->lbstat.cap, c->st));  // epoch 0 = never published
        c->lb_epoch = 0;
    }
    if (++c->lb_epoch >= (1u << 24)) {
        HIPCK(hipMemsetAsync(c->lbstat.p, 0, c->lbstat.cap, c->st));
        c->lb_epoch = 1;
    }
    HIPCK(hipMemsetAsync(c->ticket.p, 0, sizeof(uint32_t), c->st));
    return II_OK;
}

// The first pass of a token sort (k_sort0_compact) over the K1 records *k into
// *k2: one workgroup per `group` K1b chunks (at most kMaxChunks workgroups),
// one table column each.
struct S0Geom {
    uint64_t group, ncol;  // ncol: workgroups = table columns = the scatter's workgroups
};
static int s0_geometry(ii_ctx* c, S0Geom* g) {
    const uint64_t nch_in = c->nch_map;
    g->group = (nch_in + kMaxChunks - 1) / kMaxChunks;
    if (nch_in == 0 || g->group > kCMaxGroup) return II_ERR_NOMEM;
    g->ncol = (nch_in + g->group - 1) / g->group;
    return II_OK;
}
// The first pass's algorithmic bytes: 4 B per record of a narrow chunk (K1b
// wrote u32 word slots there; two lanes share each 8-B load), 8 B per other
// record, 8 B per kept record written.
static uint64_t s0_bytes(uint64_t n_in, uint64_t n_narrow, uint64_t n_kept) {
    n_narrow = std::min(n_narrow, n_in);
    return 4 * n_narrow + 8 * (n_in - n_narrow) + 8 * n_kept;
}
template <bool kWid, bool kWideD, bool kHashD = false>
static void sort0_inst(ii_ctx* c, const S0Geom& g, const uint64_t* k, uint64_t* k2, int shift, uint32_t dmask,
                       uint64_t* table, const uint32_t* remap, uint64_t* kept, int shift1, int shift2, uint64_t* dhist) {
    (c->rec_lbits ? k_sort0_compact<kWid, kWideD, kHashD, true> : k_sort0_compact<kWid, kWideD, kHashD, false>)
        <<<(uint32_t)g.ncol, kCBlock, 0, c->st>>>(
        k, P_<uint64_t>(c->chunk_cnt), (uint32_t)c->nch_map, (uint32_t)g.group, c->rec_cap, shift, dmask,
        (uint32_t)g.ncol, table, remap, k2, kept, shift1, shift2, dhist, P_<uint32_t>(c->chunk_files),
        P_<unsigned long long>(c->totals) + 8, c->rec_lbits, c->s0_fmap);
}
static void launch_sort0(ii_ctx* c, const S0Geom& g, bool wid, const uint64_t* k, uint64_t* k2, int shift,
                         uint32_t dmask, uint64_t* table, const uint32_t* remap, uint64_t* kept, int shift1, int shift2,
                         uint64_t* dhist, bool wide = false, bool hashd = false) {
    if (hashd) {  // (the packed sort only: no later-digit counts)
        if (wid && wide) sort0_inst<true, true, true>(c, g, k, k2, shift, dmask, table, remap, kept, 0, 0, nullptr);
        else if (wid) sort0_inst<true, false, true>(c, g, k, k2, shift, dmask, table, remap, kept, 0, 0, nullptr);
        else if (wide) sort0_inst<false, true, true>(c, g, k, k2, shift, dmask, table, remap, kept, 0, 0, nullptr);
        else sort0_inst<false, false, true>(c, g, k, k2, shift, dmask, table, remap, kept, 0, 0, nullptr);
        return;
    }
    if (wid && wide) sort0_inst<true, true>(c, g, k, k2, shift, dmask, table, remap, kept, shift1, shift2, dhist);
    else if (wid) sort0_inst<true, false>(c, g, k, k2, shift, dmask, table, remap, kept, shift1, shift2, dhist);
    else if (wide) sort0_inst<false, true>(c, g, k, k2, shift, dmask, table, remap, kept, shift1, shift2, dhist);
    else sort0_inst<false, false>(c, g, k, k2, shift, dmask, table, remap, kept, shift1, shift2, dhist);
}

// test knobs: raise error bits on the device (stream-ordered)
__global__ void k_set_bits(uint64_t* p, unsigned long long bits) { atomicOr((unsigned long long*)p, bits); }

// Stable LSD radix sort of n u64 keys (optionally with u32 values) on bits
// [lo, hi).  On return *k / *v point at the sorted arrays (buffers swap).
// With remap0 (token sort only, no values) the first pass is k_sort0_compact:
// it drops repeated (hot word, file) records, maps slots to lexicographic ids
// and compacts each workgroup's range into *k2; that pass's scatter reads the
// kept ranges back into *k, and the remaining passes run over the kept
// records only.  *n_out receives the number of records kept.
// The same sort without a first pass, by onesweep passes: one read of the
// keys counts every pass's digits (k_hist_passes), then one launch per pass
// (decoupled look-back: no per-pass histogram, table scan or scan launches).
// The dictionary's key / index sorts of the exchange path and the owner's
// import ran 8 x (histogram + scan + scatter) small launches before.  Main
// stream only: the look-back entries and the tile ticket are the token sort's.
static int run_sort_sweep(ii_ctx* c, uint64_t** k, uint64_t** k2, uint32_t** v, uint32_t** v2, uint64_t n, int lo,
                          int hi, int* passes) {
    const int npass = (hi - lo + kRadixBits - 1) / kRadixBits;
    const int bits = (hi - lo + npass - 1) / npass;
    if (npass > kHistMaxPasses) return II_ERR_INTERNAL;
    CK(grow(c->shist, sizeof(uint64_t) * 2 * kHistMaxPasses * kRadix));
    uint64_t* counts = P_<uint64_t>(c->shist);
    uint64_t* bases = counts + kHistMaxPasses * kRadix;
    HIPCK(hipMemsetAsync(counts, 0, sizeof(uint64_t) * npass * kRadix, c->st));
    k_hist_passes<<<(uint32_t)std::min<uint64_t>(4 * (uint64_t)c->ncu, grid_for(n)), kBlock, 0, c->st>>>(
        *k, n, lo, hi, bits, npass, counts);
    k_digit_bases<<<npass, kRadix, 0, c->st>>>(counts, bases);
    HIPCK(hipGetLastError());
    const uint64_t ntiles = (n + kSweepTile - 1) / kSweepTile;
    for (int p = 0; p < npass; p++) {
        const int shift = lo + p * bits, db = std::min(bits, hi - shift);
        CK(lookback_pass(c, ntiles * kRadix));
        if (v)
            k_onesweep<kSweepThreads, kSweepItems, 2, true><<<(uint32_t)ntiles, kSweepThreads, 0, c->st>>>(
                *k, *k2, n, shift, db, bases + (uint64_t)p * kRadix, P_<uint64_t>(c->lbstat), P_<uint32_t>(c->ticket),
                c->lb_epoch, P_<unsigned long long>(c->counters) + C_OVERFLOW, *v, *v2);
        else
            k_onesweep<kSweepThreads, kSweepItems><<<(uint32_t)ntiles, kSweepThreads, 0, c->st>>>(
                *k, *k2, n, shift, db, bases + (uint64_t)p * kRadix, P_<uint64_t>(c->lbstat), P_<uint32_t>(c->ticket),
                c->lb_epoch, P_<unsigned long long>(c->counters) + C_OVERFLOW, nullptr, nullptr);
        HIPCK(hipGetLastError());
        std::swap(*k, *k2);
        if (v) std::swap(*v, *v2);
        if (passes) (*passes)++;
    }
    if (c->test_lb_timeout == 3 && v) k_set_bits<<<1, 1, 0, c->st>>>(P_<uint64_t>(c->counters) + C_OVERFLOW, kLbTimeout);
    return II_OK;
}

// sweep_ok = false keeps the histogram + scan + scatter passes, which cannot time out: for sorts whose
// values later kernels use as indices before the host can read the look-back flag (a onesweep pass that
// flagged kLbTimeout leaves slots of its output unwritten — stale values, out-of-range indices).
static int run_sort(ii_ctx* c, uint64_t** k, uint64_t** k2, uint32_t** v, uint32_t** v2, uint64_t n, int lo, int hi,
                    bool timed, int* passes, const uint32_t* remap0 = nullptr, uint64_t* n_out = nullptr,
                    bool wid = false, bool sweep_ok = true) {
    if (passes) *passes = 0;
    if (n_out) *n_out = n;
    if (hi <= lo || (n <= 1 && !remap0)) return II_OK;
    if (remap0 && v) return II_ERR_INTERNAL;
    if (!remap0 && sweep_ok && !c->on_side && !timed && !getenv("II_SORT_NO_SWEEP")) return run_sort_sweep(c, k, k2, v, v2, n, lo, hi, passes);
    // first pass over K1's records: one workgroup (or pair) per `group` K1b chunks
    S0Geom s0{};
    if (remap0) CK(s0_geometry(c, &s0));
    uint64_t nch = 0, chunk = 0;
    auto regrid = [&](uint64_t m, uint64_t tile) {
        nch = std::min<uint64_t>(kMaxChunks, (m + tile - 1) / tile);
        chunk = ((m + nch - 1) / nch + tile - 1) / tile * tile;
        nch = (m + chunk - 1) / chunk;
    };
    if (remap0) {
        nch = s0.ncol;
        chunk = 0;
    } else {
        regrid(n, kSortTile);
    }
    CK(grow(c->rtable, sizeof(uint64_t) * kRadix * kMaxChunks));
    CK(grow(c->kept, sizeof(uint64_t) * 2 * kMaxChunks));
    uint64_t* table = P_<uint64_t>(c->rtable);
    uint64_t* kept = P_<uint64_t>(c->kept);
    const bool kv = v != nullptr;
    uint64_t* totals = P_<uint64_t>(c->totals);
    // even digit widths: the fewest passes of <= kRadixBits bits, each as narrow
    // as that allows (fewer buckets -> longer output runs per tile)
    const int npass = (hi - lo + kRadixBits - 1) / kRadixBits;
    const int bits = (hi - lo + npass - 1) / npass;
    // token sort: the passes after the first are onesweep passes (decoupled
    // look-back) when their digits fit the histograms k_sort0_compact keeps
    const bool sweep = remap0 && npass - 1 <= kLaterDigits;
    uint64_t* dhist = nullptr;
    if (sweep) {
        CK(grow(c->dhist, sizeof(uint64_t) * 2 * kLaterDigits * kRadix));
        dhist = P_<uint64_t>(c->dhist);
        HIPCK(hipMemsetAsync(dhist, 0, sizeof(uint64_t) * kLaterDigits * kRadix, c->st));
    }
    for (int shift = lo, pass = 0; shift < hi; shift += bits, pass++) {
        const int db = std::min(bits, hi - shift);
        const uint32_t dmask = (1u << db) - 1u;
        const bool first0 = remap0 && shift == lo;
        const bool ev = timed && c->n_sc < kMaxTimedPasses;
        const uint64_t* src = first0 ? *k2 : *k;
        uint64_t* dst = first0 ? *k : *k2;
        if (first0) {
            if (timed) HIPCK(hipEventRecord(c->ev_c0[0], c->st));
            launch_sort0(c, s0, wid, *k, *k2, shift, dmask, table, remap0, kept, lo + bits, lo + 2 * bits, dhist);
            if (timed) HIPCK(hipEventRecord(c->ev_c0[1], c->st));
            CK(run_scan(c, OpInPlace{table}, (uint64_t)kRadix * nch, totals + 4));
            if (sweep) k_digit_bases<<<kLaterDigits, kRadix, 0, c->st>>>(dhist, dhist + kLaterDigits * kRadix);
        } else if (sweep) {
            // onesweep: one launch per pass, no histogram pass, no table scan
            const uint64_t ntiles = (n + kSweepTile - 1) / kSweepTile;
            CK(lookback_pass(c, ntiles * kRadix));
            if (ev) HIPCK(hipEventRecord(c->ev_sc[2 * c->n_sc], c->st));
            k_onesweep<kSweepThreads, kSweepItems><<<(uint32_t)ntiles, kSweepThreads, 0, c->st>>>(
                src, dst, n, shift, db, dhist + kLaterDigits * kRadix + (uint64_t)(pass - 1) * kRadix,
                P_<uint64_t>(c->lbstat), P_<uint32_t>(c->ticket), c->lb_epoch,
                P_<unsigned long long>(c->counters) + C_OVERFLOW, nullptr, nullptr);
            if (ev) {
                HIPCK(hipEventRecord(c->ev_sc[2 * c->n_sc + 1], c->st));
                c->sc_bytes[c->n_sc] = 16 * n;
                c->n_sc++;
            }
            HIPCK(hipGetLastError());
            if (passes) (*passes)++;
            std::swap(*k, *k2);
            continue;
        } else {
            k_radix_hist<<<(uint32_t)nch, kBlock, 0, c->st>>>(*k, n, chunk, shift, dmask, (uint32_t)nch, table);
            CK(run_scan(c, OpInPlace{table}, (uint64_t)kRadix * nch, nullptr));
        }
        if (ev) HIPCK(hipEventRecord(c->ev_sc[2 * c->n_sc], c->st));
        if (kv)
            k_radix_scatter<true><<<(uint32_t)nch, kBlock, 0, c->st>>>(src, dst, *v, *v2, n, chunk, shift, db,
                                                                      (uint32_t)nch, table, nullptr, nullptr, nullptr,
                                                                      0, 0u);
        else
            k_radix_scatter<false, kScatterThreads, kScatterItems><<<(uint32_t)nch, kScatterThreads, 0, c->st>>>(
                src, dst, nullptr, nullptr, n, chunk, shift, db, (uint32_t)nch, table, first0 ? kept : nullptr, nullptr,
                nullptr, 0, 0u);
        if (ev) {
            HIPCK(hipEventRecord(c->ev_sc[2 * c->n_sc + 1], c->st));
            c->n_sc++;
        }
        HIPCK(hipGetLastError());
        if (passes) (*passes)++;
        if (first0) {  // sorted by the first digit, in *k: the rest runs over the kept records
            const uint64_t n_in = n;
            uint64_t t47[5];
            CK(read_u64(c, totals + 4, t47, 5));
            n = t47[0];
            if (wid) {  // exact wid range (k_count_hot wrote the occupied hot slots to totals[7])
                c->NW = kHotSlots + (c->V - (t47[3] & 0xFFFFFFFFull));
                hi = std::min(hi, lo + std::max(1, bitlen(c->NW - 1)));
            }
            c->c0_bytes = s0_bytes(n_in, t47[4], n);
            if (ev) c->sc_bytes[c->n_sc - 1] = 16 * n;
            if (n_out) *n_out = n;
            if (n <= 1) break;
            regrid(n, kSortTile);
        } else {
            std::swap(*k, *k2);
            if (kv) std::swap(*v, *v2);
            if (ev) c->sc_bytes[c->n_sc - 1] = 16 * n + (kv ? 8 * n : 0);
        }
    }
    return II_OK;
}

// *p |= bits (one thread; the II_TEST_LB_TIMEOUT test knob)

// Stable LSD radix sort of n u32 keys on bits [0, bits): *k / *k2 ping-pong,
// on return *k holds the sorted keys (the owner's merged pairs when lexid and
// id0 fit one u32, ii_import).
static int run_sort32(ii_ctx* c, uint32_t** k, uint32_t** k2, uint64_t n, int bits, int* passes) {
    *passes = 0;
    if (n <= 1 || bits <= 0) return II_OK;
    CK(grow(c->rtable, sizeof(uint64_t) * kRadix * kMaxChunks));
    uint64_t* table = P_<uint64_t>(c->rtable);
    uint64_t nch = std::min<uint64_t>(kMaxChunks, (n + kSortTile - 1) / kSortTile);
    const uint64_t chunk = ((n + nch - 1) / nch + kSortTile - 1) / kSortTile * kSortTile;
    nch = (n + chunk - 1) / chunk;
    const int npass = (bits + kRadixBits - 1) / kRadixBits, db = (bits + npass - 1) / npass;
    for (int shift = 0; shift < bits; shift += db) {
        const int w = std::min(db, bits - shift);
        const uint32_t dmask = (1u << w) - 1u;
        k_radix_hist<uint32_t><<<(uint32_t)nch, kBlock, 0, c->st>>>(*k, n, chunk, shift, dmask, (uint32_t)nch, table);
        CK(run_scan(c, OpInPlace{table}, (uint64_t)kRadix * nch, nullptr));
        k_radix_scatter<false, kScatterThreads, kScatterItems, false, uint32_t>
            <<<(uint32_t)nch, kScatterThreads, 0, c->st>>>(*k, *k2, nullptr, nullptr, n, chunk, shift, w, (uint32_t)nch,
                                                           table, nullptr, nullptr, nullptr, 0, 0u);
        HIPCK(hipGetLastError());
        std::swap(*k, *k2);
        (*passes)++;
    }
    return II_OK;
}

// Packed token sort (ii_prims.h, "Packed token sort"): the top digit m of a
// W-bit key when the other W - m key bits and the F id bits fit a u32 and
// leave two LSD passes of <= kRadixBits bits; 0 = not packable.  Top digits
// of up to kMsdMaxBits bits (k_msd_scatter_wide past kRadixBits).
// II_PACKED_M=<m> (test knob): at least m top bits, so that small inputs reach
// the wide split.
static int packed_top_bits(int W, int F) {
    if (getenv("II_PACKED_SORT") && !strcmp(getenv("II_PACKED_SORT"), "0")) return 0;
    const char* fm = getenv("II_PACKED_M");
    const int m = std::max({7, W + F - 32, fm ? atoi(fm) : 0});
    const int L = W - m;
    return (m <= kMsdMaxBits && L >= 2 && L <= 2 * kRadixBits) ? m : 0;
}

// The first pass's dedup for the packed sort: the record set (kHashD) when the
// files average fewer than kHashDedupTokens tokens (configs[4]'s small-file
// shares: 3.9·10^3), the epoch bitmap otherwise (config3: 1.4·10^5 per file,
// more distinct pairs per file than the set holds).  II_S0_DEDUP=set|bitmap
// (test and A/B knob) forces one.
constexpr uint64_t kHashDedupTokens = 16384;
// files at which the first pass maps file indices to id0s (local_reduce; a 256 KiB fmap)
constexpr uint32_t kS0FmapFiles = 65536;
static bool dedup_by_set(const ii_ctx* c, uint64_t n) {
    const char* e = getenv("II_S0_DEDUP");
    if (e && !strcmp(e, "set")) return true;
    if (e && !strcmp(e, "bitmap")) return false;
    return c->nfiles && n < kHashDedupTokens * (uint64_t)c->nfiles;
}

// The packed sort's bucket geometry and LSD digit counts in c->msd (sized for
// kMsdMax buckets): bstart[kMsdMax + 1] | pad[kMsdMax] | btile (u32)[kMsdMax + 1]
// | gh[2 kMsdMax kRadix] | gbase[2 kMsdMax kRadix]
struct MsdLayout {
    uint64_t *bstart, *pad, *gh, *gbase;
    uint32_t* btile;
};
static MsdLayout msd_layout(ii_ctx* c) {
    constexpr size_t kGeo = 3 * (size_t)kMsdMax + 2;
    MsdLayout g;
    g.bstart = P_<uint64_t>(c->msd);
    g.pad = g.bstart + kMsdMax + 1;
    g.btile = reinterpret_cast<uint32_t*>(g.pad + kMsdMax);
    g.gh = g.bstart + kGeo;
    g.gbase = g.gh + 2 * (size_t)kMsdMax * kRadix;
    return g;
}
static constexpr size_t kMsdBytes = sizeof(uint64_t) * (3 * (size_t)kMsdMax + 2 + 4 * (size_t)kMsdMax * kRadix);

// The token sort of local_reduce in the packed form: k_sort0_compact (dedup,
// key remap, compaction, counts of the top digit per workgroup) into *k2, the
// MSD scatter into buckets of u32 records (*k, padded), per-bucket digit
// counts, two bucket-local onesweep passes (*k -> *k2 -> *k, both writing u32
// records in the padded buckets; K3 reads that layout).  Keys sit at bits
// [lo, lo + W) of the records, ids below 2^F.  On return *k holds the *n_out
// sorted records.
static int run_sort_packed(ii_ctx* c, uint64_t** k, uint64_t** k2, uint64_t n, int lo, int W, int F, int m,
                           const uint32_t* remap0, uint64_t* n_out, bool wid, int* passes) {
    *passes = 0;
    *n_out = n;
    const uint32_t nb = 1u << m;
    const int L = W - m, b0 = L - L / 2, b1 = L / 2;
    const bool wide = m > kRadixBits;  // (k_sort0_compact<.., kWideD>, k_msd_scatter_wide)
    const uint32_t rows = wide ? nb : kRadix;  // digit rows of the table
    S0Geom s0{};
    CK(s0_geometry(c, &s0));
    const uint64_t nch = s0.ncol;
    CK(grow(c->rtable, sizeof(uint64_t) * rows * kMaxChunks));
    CK(grow(c->kept, sizeof(uint64_t) * 2 * kMaxChunks));
    CK(grow(c->msd, kMsdBytes));
    const MsdLayout g = msd_layout(c);
    uint64_t* bstart = g.bstart;
    uint64_t* pad = g.pad;
    uint32_t* btile = g.btile;
    uint64_t* gh = g.gh;
    uint64_t* gbase = g.gbase;
    uint64_t* table = P_<uint64_t>(c->rtable);
    uint64_t* kept = P_<uint64_t>(c->kept);
    uint64_t* totals = P_<uint64_t>(c->totals);
    unsigned long long* err = P_<unsigned long long>(c->counters) + C_OVERFLOW;
    const int shift = lo + L;  // the top digit of the key
    const uint32_t dmask = nb - 1u;

    HIPCK(hipEventRecord(c->ev_c0[0], c->st));
    launch_sort0(c, s0, wid, *k, *k2, shift, dmask, table, remap0, kept, 0, 0, nullptr, wide, dedup_by_set(c, n));
    HIPCK(hipEventRecord(c->ev_c0[1], c->st));
    CK(run_scan(c, OpInPlace{table}, (uint64_t)rows * nch, totals + 4));
    k_msd_geometry<<<1, kRadix, 0, c->st>>>(table, (uint32_t)nch, nb, totals + 4, kSweepTile, bstart, btile, pad);
    HIPCK(hipMemsetAsync(gh, 0, sizeof(uint64_t) * 2 * nb * kRadix, c->st));
    HIPCK(hipGetLastError());
    CK(read_queue(c, totals + 4, 4, 5));  // (kept count, wid range, narrow records: read while the scatter runs)
    // MSD scatter: u64 records -> u32 records in padded buckets
    const bool ev = c->n_sc + 3 <= kMaxTimedPasses;
    if (ev) HIPCK(hipEventRecord(c->ev_sc[2 * c->n_sc], c->st));
    uint32_t* out32 = reinterpret_cast<uint32_t*>(*k);
    constexpr int NTs = kScatterThreads, ITs = kScatterItems;
    // (for 8-bit top digits k_msd_scatter<.., 256> measured 0.1 ms slower than k_radix_scatter<kPack>, also
    // with 8- or 12-record tiles at 6 waves per SIMD, 3 workgroups per CU)
    if (wide) {
        // 2048 digits: 256 threads x 32 records and u32 run bases when every position of the padded
        // layout fits (76 KiB of LDS, two workgroups per CU), else 512 x 32 with u64 bases (148 KiB)
        const bool run32 = n + (uint64_t)nb * kSweepTile < (1ull << 32);
        if (m > 10 && run32)
            k_msd_scatter<NTs / 2, 2 * ITs, kMsdMax, true><<<(uint32_t)nch, NTs / 2, 0, c->st>>>(
                *k2, out32, shift, m, (uint32_t)nch, table, kept, pad, F, (1u << L) - 1u);
        else
            (m <= 9 ? k_msd_scatter<NTs, ITs, 512> : m <= 10 ? k_msd_scatter<NTs, ITs, 1024>
                    : k_msd_scatter<NTs, 2 * ITs, kMsdMax>)<<<(uint32_t)nch, NTs, 0, c->st>>>(
                *k2, out32, shift, m, (uint32_t)nch, table, kept, pad, F, (1u << L) - 1u);
    } else {
        k_radix_scatter<false, kScatterThreads, kScatterItems, true><<<(uint32_t)nch, kScatterThreads, 0, c->st>>>(
            *k2, (uint64_t*)nullptr, nullptr, nullptr, n, 0, shift, m, (uint32_t)nch, table, kept,
            reinterpret_cast<uint32_t*>(*k), pad, F, (1u << L) - 1u);
    }
    if (ev) HIPCK(hipEventRecord(c->ev_sc[2 * c->n_sc + 1], c->st));
    HIPCK(hipGetLastError());
    uint64_t t47[5];
    CK(read_wait(c, t47, 4, 5));
    const uint64_t n_in = n;
    n = t47[0];
    if (wid) c->NW = kHotSlots + (c->V - (t47[3] & 0xFFFFFFFFull));  // exact wid range (k_count_hot)
    c->c0_bytes = s0_bytes(n_in, t47[4], n);
    *n_out = n;
    if (ev) c->sc_bytes[c->n_sc++] = 12 * n;
    *passes = 1;
    if (n == 0) return II_OK;
    // per-bucket digit counts of the two LSD passes -> bases
    c->sort_packed = true;
    c->sort_hist_bytes = 4 * n;
    c->pk_nb = nb;
    c->pk_F = F;
    c->pk_L = L;
    const uint64_t ntb = (n + kSweepTile - 1) / kSweepTile + nb;  // tiles of the padded layout, at most
    const uint32_t hg = (uint32_t)std::min<uint64_t>(kMaxChunks, ntb);
    const uint32_t per = (uint32_t)((ntb + hg - 1) / hg);
    c->pk_ntb = (uint32_t)ntb;
    c->pk_ncap = ntb * kSweepTile;
    CK(grow(c->tbk, sizeof(uint16_t) * ntb));
    uint16_t* tbk = P_<uint16_t>(c->tbk);
    k_tile_buckets<<<nb, kBlock, 0, c->st>>>(btile, tbk);
    k_seg_hist<kSweepThreads, kSweepItems><<<hg, kSweepThreads, 0, c->st>>>(
        reinterpret_cast<const uint32_t*>(*k), btile, bstart, nb, per, F, b0, F + b0, b1, gh);
    k_digit_bases<<<2 * nb, kRadix, 0, c->st>>>(gh, gbase);
    HIPCK(hipGetLastError());
    // two bucket-local onesweep passes, both u32 -> u32 in the padded buckets (K3 reads that layout)
    for (int p = 0; p < 2; p++) {
        CK(lookback_pass(c, ntb * kRadix));
        const bool evp = c->n_sc < kMaxTimedPasses;
        if (evp) HIPCK(hipEventRecord(c->ev_sc[2 * c->n_sc], c->st));
        k_onesweep_seg<kSweepThreads, kSweepItems><<<(uint32_t)ntb, kSweepThreads, 0, c->st>>>(
            reinterpret_cast<const uint32_t*>(p == 0 ? *k : *k2), ntb * kSweepTile,
            reinterpret_cast<uint32_t*>(p == 0 ? *k2 : *k), btile,
            tbk, bstart, nb, p == 0 ? F : F + b0, p == 0 ? b0 : b1, gbase + p * kRadix, 2 * kRadix, P_<uint64_t>(c->lbstat),
            P_<uint32_t>(c->ticket), c->lb_epoch, err);
        if (evp) {
            HIPCK(hipEventRecord(c->ev_sc[2 * c->n_sc + 1], c->st));
            c->sc_bytes[c->n_sc++] = 8 * n;
        }
        HIPCK(hipGetLastError());
        (*passes)++;
    }
    return II_OK;
}

// K3: distinct (lexid, id0) pairs of the sorted records r[0, n), their
// posting byte offsets (P[U] = all posting bytes) and each word's first pair
// (post_start[V] = U).  Sets c->U.  fmap: id0 of every shard-local file index
// the records carry (null: the records carry id0 - fid_off).
static int run_unique(ii_ctx* c, const uint64_t* r, uint64_t n, bool wid, bool packed, const uint32_t* fmap,
                      bool compact, uint32_t fid_off = 0) {
    c->xpairs = false;
    if (compact && c->id_bound > kPairFirst) compact = false;  // (the top bit marks a word's first pair: u64 pairs)
    c->pairs32 = compact;
    CK(grow(c->uniq, sizeof(uint64_t) * std::max<uint64_t>(n, 1)));
    CK(grow(c->P, sizeof(uint64_t) * (n + 1)));
    CK(grow(c->pstart, sizeof(uint64_t) * (c->V + 1)));
    CK(grow(c->pstop, sizeof(uint64_t) * (c->V + 1)));
    uint64_t* pe = P_<uint64_t>(c->pstop);
    uint64_t* uniq = P_<uint64_t>(c->uniq);
    uint64_t* Pp = P_<uint64_t>(c->P);
    uint64_t* ps = P_<uint64_t>(c->pstart);
    uint64_t* totals = P_<uint64_t>(c->totals);
    uint32_t* u32 = nullptr;
    uint32_t* g64 = nullptr;
    if (compact) {  // (file ids below 2^31: the top bit marks a word's first pair)
        CK(grow(c->g64, sizeof(uint32_t) * (n / 64 + 2)));
        u32 = P_<uint32_t>(c->uniq);
        g64 = P_<uint32_t>(c->g64);
    }
    if (n == 0) {
        HIPCK(hipMemsetAsync(ps + c->V, 0, sizeof(uint64_t), c->st));
        HIPCK(hipMemsetAsync(Pp, 0, sizeof(uint64_t), c->st));
        // (the callers read host words queued on the stream before this call — local_reduce's
        // collision verdict — after run_unique returns: the other path's read_wait covers them)
        HIPCK(hipStreamSynchronize(c->st));
        c->U = 0;
        return II_OK;
    }
    uint64_t* ps_k = ps;  // starts / ends by record key
    uint64_t* pe_k = pe;
    if (wid) {
        CK(grow(c->pstart_w, sizeof(uint64_t) * (c->NW + 1)));
        CK(grow(c->pstop_w, sizeof(uint64_t) * (c->NW + 1)));
        ps_k = P_<uint64_t>(c->pstart_w);
        pe_k = P_<uint64_t>(c->pstop_w);
    }
    // one pass with decoupled look-back (k_uniq_sweep): U -> post_start[V], posting bytes -> totals[6]
    if (packed) {  // r: the packed sort's u32 records in their padded buckets (k_uniq_sweep<true>)
        const MsdLayout g = msd_layout(c);
        const uint64_t* bstart = g.bstart;
        const uint32_t* btile = g.btile;
        const uint64_t ntiles = 2ull * c->pk_ntb;  // at most: the spare ones leave at once
        CK(lookback_pass(c, 2 * ntiles));
        (fmap ? k_uniq_sweep<true, true> : k_uniq_sweep<true, false>)<<<(uint32_t)ntiles, kBlock, 0, c->st>>>(
            nullptr, n, reinterpret_cast<const uint32_t*>(r), c->pk_ncap, btile, P_<uint16_t>(c->tbk), bstart, c->pk_nb, c->pk_F, c->pk_L, uniq, Pp, ps_k,
            pe_k, P_<uint64_t>(c->lbstat), P_<uint32_t>(c->ticket), c->lb_epoch, ps + c->V, totals + 6,
            P_<unsigned long long>(c->counters) + C_OVERFLOW, fmap, u32, g64, c->dth, fid_off);
    } else {
        const uint64_t ntiles = (n + kUniqSweepTile - 1) / kUniqSweepTile;
        CK(lookback_pass(c, 2 * ntiles));
        (fmap ? k_uniq_sweep<false, true> : k_uniq_sweep<false, false>)<<<(uint32_t)ntiles, kBlock, 0, c->st>>>(
            r, n, nullptr, 0, nullptr, nullptr, nullptr, 0, 0, 0, uniq, Pp, ps_k, pe_k, P_<uint64_t>(c->lbstat),
            P_<uint32_t>(c->ticket), c->lb_epoch, ps + c->V, totals + 6, P_<unsigned long long>(c->counters) + C_OVERFLOW,
            fmap, u32, g64, c->dth, fid_off);
        k_post_last<<<1, 64, 0, c->st>>>(r, n, ps + c->V, pe_k);
    }
    // K3's look-back flags kLbTimeout instead of hanging (a predecessor tile that never
    // published reads as a prefix of 0): the pairs and offsets are then wrong — an error.
    // The flags and U are read back while k_wid_post runs.
    uint64_t* ovf = P_<uint64_t>(c->counters) + C_OVERFLOW;
    if (c->test_lb_timeout == 1) k_set_bits<<<1, 1, 0, c->st>>>(ovf, kLbTimeout);
    HIPCK(hipMemcpyAsync(c->hbuf + 2, ovf, sizeof(uint64_t), hipMemcpyDeviceToHost, c->st));
    CK(read_queue(c, ps + c->V, 3, 1));
    if (wid)
        k_wid_post<<<grid_for(c->V), kBlock, 0, c->st>>>(P_<uint32_t>(c->widl), (uint32_t)c->V, ps_k, pe_k, ps, pe);
    HIPCK(hipGetLastError());
    uint64_t fu[2];
    CK(read_wait(c, fu, 2, 2));
    c->U = fu[1];
    if (fu[0] & kLbTimeout) return II_ERR_INTERNAL;
    HIPCK(hipMemcpyAsync(Pp + c->U, totals + 6, sizeof(uint64_t), hipMemcpyDeviceToDevice, c->st));
    return II_OK;
}

// ----------------------------------------------------------------- lifecycle
extern "C" int ii_open(ii_ctx** out, int device) {
    if (!out) return II_ERR_ARG;
    *out = nullptr;
    LIVE_OR_FAIL();
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
        (void)hipGetLastError();
        return II_ERR_NODEV;
    }
    if (device < 0 || device >= n) return II_ERR_ARG;
    ii_ctx* c = new ii_ctx();
    c->dev = device;
    HIPCK(hipSetDevice(device));
    HIPCK(hipDeviceGetAttribute(&c->ncu, hipDeviceAttributeMultiprocessorCount, device));
    HIPCK(hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking));
    HIPCK(hipStreamCreateWithFlags(&c->st2, hipStreamNonBlocking));
    for (auto& e : c->ev) HIPCK(hipEventCreate(&e));
    for (auto& e : c->ev_sc) HIPCK(hipEventCreate(&e));
    for (auto& e : c->ev_emit) HIPCK(hipEventCreate(&e));
    for (auto& e : c->ev_res) HIPCK(hipEventCreate(&e));
    for (auto& e : c->ev_c0) HIPCK(hipEventCreate(&e));
    for (auto& e : c->ev_dict) HIPCK(hipEventCreate(&e));
    HIPCK(hipHostMalloc((void**)&c->hbuf, kHbufWords * sizeof(uint64_t), hipHostMallocDefault));
    HIPCK(hipEventCreateWithFlags(&c->ev_rd, hipEventDisableTiming));
    if (grow(c->partial, sizeof(uint64_t) * (2 * kMaxChunks + 1)) ||
        grow(c->partial2, sizeof(uint64_t) * (2 * kMaxChunks + 1)) || grow(c->totals, sizeof(uint64_t) * 16) ||
        grow(c->counters, sizeof(uint64_t) * C_NUM)) {
        ii_close(c);
        return II_ERR_NOMEM;
    }
    if (const char* e = getenv("II_TEST_LB_TIMEOUT")) c->test_lb_timeout = !strcmp(e, "1")       ? 1
                                                                : !strcmp(e, "sort")  ? 2
                                                                : !strcmp(e, "sweep") ? 3
                                                                : !strcmp(e, "order") ? 4
                                                                                      : 0;
    c->test_collide = getenv("II_TEST_COLLIDE") && !strcmp(getenv("II_TEST_COLLIDE"), "1");
    if (getenv("II_TEST_LONG_KEY_BITS")) c->test_long_bits = std::min(64, std::max(0, atoi(getenv("II_TEST_LONG_KEY_BITS"))));
    const char* s = getenv("II_TABLE_LOG2");
    if (s && atoi(s) >= 10 && atoi(s) <= 30) {
        c->big_cap = 1ull << atoi(s);
        c->big_fixed = true;
    }
    memset(&c->stats, 0, sizeof(c->stats));
    *out = c;
    return II_OK;
}

extern "C" void ii_close(ii_ctx* c) {
    if (!c) return;
    if (poisoned()) {  // (a wait or free on a faulted device may never return: leave it to process exit)
        delete c;
        return;
    }
    (void)hipSetDevice(c->dev);
    if (c->st) (void)hipStreamSynchronize(c->st);
    if (c->st2) (void)hipStreamSynchronize(c->st2);  // (work on st2 reads the buffers freed below)
    DBuf* all[] = {&c->text_own, &c->fstart, &c->fid,   &c->partial, &c->totals, &c->counters, &c->chunk_cnt, &c->chunk_hist,
                   &c->rtable,   &c->rec,    &c->rec2,  &c->longs,   &c->tkeys,  &c->trep,     &c->dslot,
                   &c->dkey,     &c->dkey2,  &c->didx,  &c->didx2,   &c->remap,  &c->lkey,     &c->lrep,
                   &c->llen,     &c->lstart, &c->tied,  &c->tpos,    &c->rid,    &c->rfirst,   &c->tdict,
                   &c->tk,       &c->tk2,    &c->tv,    &c->tv2,     &c->uniq,   &c->pstart,   &c->okey,
                   &c->okey2,    &c->oval,   &c->oval2, &c->P,       &c->loff,   &c->out,      &c->letter_off,
                   &c->woff,     &c->pts,    &c->pend,  &c->pend_cnt, &c->kept,
                   &c->ppieces,  &c->pcnt,   &c->pout,  &c->ploff, &c->chunk_files, &c->pstop, &c->wmap,
                   &c->lexw,     &c->widl,   &c->fbase, &c->pstart_w, &c->pstop_w, &c->mstart, &c->mend,
                   &c->dhist,    &c->lbstat, &c->ticket, &c->pstart_x, &c->msd, &c->tbk, &c->moff,
                   &c->partial2, &c->rtable2, &c->kept2, &c->drank, &c->g64, &c->shist};
    for (DBuf* b : all)
        if (b->p) (void)hipFree(b->p);
    for (auto& e : c->ev)
        if (e) (void)hipEventDestroy(e);
    for (auto& e : c->ev_sc)
        if (e) (void)hipEventDestroy(e);
    for (auto& e : c->ev_emit)
        if (e) (void)hipEventDestroy(e);
    for (auto& e : c->ev_res)
        if (e) (void)hipEventDestroy(e);
    for (auto& e : c->ev_c0)
        if (e) (void)hipEventDestroy(e);
    for (auto& e : c->ev_dict)
        if (e) (void)hipEventDestroy(e);
    if (c->ev_rd) (void)hipEventDestroy(c->ev_rd);
    if (c->st2) (void)hipStreamSynchronize(c->st2);
    if (c->st2) (void)hipStreamDestroy(c->st2);
    if (c->hbuf) (void)hipHostFree(c->hbuf);
    for (auto s : c->io_st) (void)hipStreamSynchronize(s);
    for (auto s : c->io_st) (void)hipStreamDestroy(s);
    for (auto e : c->io_ev) (void)hipEventDestroy(e);
    for (auto b : c->io_buf) (void)hipHostFree(b);
    if (c->st) (void)hipStreamDestroy(c->st);
    delete c;
}

extern "C" const char* ii_strerror(int code) {
    switch (code) {
        case II_OK: return "ok";
        case II_ERR_ARG: return "invalid argument";
        case II_ERR_HIP: return "HIP runtime error";
        case II_ERR_NOMEM: return "out of memory";
        case II_ERR_IO: return "I/O error";
        case II_ERR_STATE: return "call out of order";
        case II_ERR_LAYOUT: return "device text violates the file separator contract";
        case II_ERR_INTERNAL: return "internal consistency check failed";
        case II_ERR_NODEV: return "no HIP device";
        default: return "unknown error";
    }
}

// ----------------------------------------------------------------- map (K1)
// K1 record layout: the fixed-capacity one (no counting pass) unless
// II_REC_LAYOUT=dense or its buffers (12 B per K1b token slot, 6 B per text
// byte) would take more than 40% of the device memory left.
static bool use_fixed_capacity(ii_ctx* c, uint64_t nch, bool dense) {
    if (dense) return false;
    const char* e = getenv("II_REC_LAYOUT");
    if (e && !strcmp(e, "dense")) return false;
    if (e && !strcmp(e, "fixed")) return true;
    size_t fr = 0, tot = 0;
    if (!hip_ok(hipMemGetInfo(&fr, &tot))) {
        (void)hipGetLastError();
        return false;
    }
    const double held = (double)c->rec.cap + (double)c->pend.cap;
    return 12.0 * (double)nch * (double)kChunkCap <= 0.4 * ((double)fr + held);
}

// Room for fast-path miss keys in a narrow chunk (kNarrowKeys); tests lower it
// with II_NARROW_KEYS to drive the overflow path on ordinary corpora.
static uint32_t narrow_keys() {
    const char* e = getenv("II_NARROW_KEYS");
    if (!e || !*e) return (uint32_t)kNarrowKeys;
    const unsigned long v = strtoul(e, nullptr, 10);
    return v < kNarrowKeys ? (uint32_t)v : (uint32_t)kNarrowKeys;
}

// dense: records of token k at rec[k] (the import path indexes them so).
// The main map (not dense) leaves the exactness check of its hashed keys
// (k_long_verify) running on the side stream while the reduce proceeds on the
// main one; local_reduce reads its verdict after K3 (check_long_words) and
// re-runs map + reduce with a new seed on a collision.  The import's word
// map checks at once.
static int map_core(ii_ctx* c, uint64_t hist_out[II_ALPHABET], bool dense = false) {
    // a check of an earlier map still reads the table, the long queue and the counters
    if (c->lv_pending) HIPCK(hipStreamWaitEvent(c->st, c->ev_res[1], 0));
    c->lv_pending = false;
    c->mapped = c->have_pairs = c->reduced = false;
    c->wid_pairs = false;
    c->planned_parts = 0;
    c->host_valid = false;
    c->n_sc = 0;
    c->c0_bytes = 0;
    c->retries = 0;
    memset(&c->stats, 0, sizeof(c->stats));
    uint64_t* counters = P_<uint64_t>(c->counters);
    uint64_t* totals = P_<uint64_t>(c->totals);
    HIPCK(hipEventRecord(c->ev[0], c->st));
    HIPCK(hipMemsetAsync(counters, 0, sizeof(uint64_t) * C_NUM, c->st));
    c->T = c->V = c->U = c->nlong = c->T_sorted = 0;
    if (c->nbytes == 0 || c->nfiles == 0) {
        memset(c->hist, 0, sizeof(c->hist));
        if (hist_out) memset(hist_out, 0, sizeof(uint64_t) * II_ALPHABET);
        HIPCK(hipEventRecord(c->ev[1], c->st));
        HIPCK(hipEventRecord(c->ev[2], c->st));
        c->mapped = true;
        return II_OK;
    }
    // a big table sized by the last local reduce's vocabulary (shrink only): the map's memset, its
    // occupancy count and the dictionary's slot compaction read every slot (2^22 of them: 32 MB for
    // the 4·10^4 big-table words of configs[2])
    if (!dense && c->big_next && c->big_next < c->big_cap && !c->big_fixed) c->big_cap = c->big_next;
    // a context with no reduce to size it by (the CLI's only map): the big table from the input's size
    // — about one slot per 768 bytes, 2^22 .. 2^26 slots (16 B each: keys + occurrences).  With the
    // 2^22 of round 5 the first map of configs[4]'s rank-7 share (6.7e6 words in 12.5 GB) filled the
    // table, and K1b ran a void attempt before the regrow: 58.6 ms of map instead of ~26.
    if (!dense && !c->big_next && !c->big_fixed && c->text_is_input) {
        uint64_t want = 1ull << 22;
        while (want < (1ull << 26) && want < c->nbytes / 768) want <<= 1;
        c->big_cap = std::max(c->big_cap, want);
    }
    const uint64_t nch = (c->nbytes + kChunk - 1) / kChunk;
    const uint32_t wg_chunks = (uint32_t)((nch + kWG - 1) / kWG);  // K1 kernels: one wave per chunk
    c->nch_map = nch;
    CK(grow(c->chunk_cnt, sizeof(uint64_t) * (nch + 1)));
    CK(grow(c->chunk_hist, sizeof(uint32_t) * 26 * nch));
    uint64_t* chunk_cnt = P_<uint64_t>(c->chunk_cnt);
    const uint64_t* fstart = P_<uint64_t>(c->fstart);

    // the separator contract, checked on the device (totals[9]); the host looks once, with the map's
    // other results
    // (totals[8]: the first sort pass's count of records in narrow chunks, zeroed with it)
    HIPCK(hipMemsetAsync(totals + 8, 0, 2 * sizeof(uint64_t), c->st));
    k_check_layout<<<grid_for(c->nfiles), kBlock, 0, c->st>>>(c->text, fstart, c->nfiles, totals + 9);
    HIPCK(hipMemsetAsync(chunk_cnt + nch, 0, sizeof(uint64_t), c->st));  // voff[nch] = T after the scan
    c->rec_cap = use_fixed_capacity(c, nch, dense) ? kChunkCap : 0;
    if (c->rec_cap) {
        CK(grow(c->rec, std::max(sizeof(uint64_t) * nch * kChunkCap, packed_bytes(nch * kChunkCap))));
        CK(grow(c->pend, sizeof(uint32_t) * nch * kChunkCap));
        c->T = 0;
    } else {
        uint64_t hv[2];
        k_tok_count<<<wg_chunks, kBlock, 0, c->st>>>(c->text, c->nbytes, nch, chunk_cnt);
        CK(run_scan(c, OpInPlace{chunk_cnt}, nch + 1, totals));
        CK(read_u64(c, totals, &hv[0]));
        CK(read_u64(c, totals + 9, &hv[1]));
        if (hv[1]) return II_ERR_LAYOUT;
        c->T = hv[0];
        CK(grow(c->rec, std::max(sizeof(uint64_t) * std::max<uint64_t>(c->T, 1), packed_bytes(c->T))));
        CK(grow(c->rec2, std::max(sizeof(uint64_t) * std::max<uint64_t>(c->T, 1), packed_bytes(c->T))));
        CK(grow(c->pend, sizeof(uint32_t) * std::max<uint64_t>(c->T, 1)));
    }
    CK(grow(c->pend_cnt, sizeof(uint32_t) * nch));
    CK(grow(c->chunk_files, sizeof(uint32_t) * 3 * nch));
    k_chunk_files<<<grid_for(nch), kBlock, 0, c->st>>>(fstart, c->nfiles, c->nbytes, kChunk, nch,
                                                      P_<uint32_t>(c->chunk_files));
    // the long queue grows on overflow (a retry of the map); at least one chunk of nothing but long
    // tokens (13 letters + a separator each) per queue shard, so that inputs of up to kLongShards
    // chunks never retry for it
    const uint64_t t_est = c->rec_cap ? c->nbytes / 4 : c->T;
    const uint64_t lmin = std::max<uint64_t>((uint64_t)kLongShards * (kChunk / 14 + 1), t_est / 64);
    if (c->long_cap < lmin) c->long_cap = lmin;

    // K1b, its counts, the exactness check of hashed keys, the token count scan
    // and the letter histogram are all queued before the host looks: one host
    // round trip per attempt (a retry redoes them all)
    for (int attempt = 0;; attempt++) {
        if (attempt > 12) return II_ERR_INTERNAL;
        if (c->big_cap > (1ull << 30)) return II_ERR_NOMEM;  // slots must fit 31 bits
        const uint64_t nslots = kHotSlots + c->big_cap;
        CK(grow(c->tkeys, sizeof(uint64_t) * nslots));
        CK(grow(c->trep, sizeof(uint64_t) * nslots));
        CK(grow(c->longs, sizeof(LongTok) * c->long_cap));
        HIPCK(hipMemsetAsync(c->tkeys.p, 0, sizeof(uint64_t) * nslots, c->st));
        HIPCK(hipMemsetAsync(counters, 0, sizeof(uint64_t) * C_NUM, c->st));
        // (the test knob: real collisions between different long words, until the first retry)
        const uint64_t long_mask = c->test_long_bits < 64 && c->collide_retries == 0 ? (1ull << c->test_long_bits) - 1ull : ~0ull;
        Table tab{P_<unsigned long long>(c->tkeys), P_<uint64_t>(c->trep), c->big_cap - 1, c->seed, counters, long_mask};
        HIPCK(hipEventRecord(c->ev_emit[0], c->st));
        const uint32_t nkeys = narrow_keys();
        c->map_deep = c->deep_probe;
        auto* emit = nkeys == kNarrowKeys ? (c->deep_probe ? k_tok_emit<false, true> : k_tok_emit<false, false>)
                                          : (c->deep_probe ? k_tok_emit<true, true> : k_tok_emit<true, false>);
        c->rec_lbits = rec_lbits(nslots, c->nbytes, c->nfiles);
        emit<<<wg_chunks, kBlock, 0, c->st>>>(
            c->text, c->nbytes, nch, fstart, chunk_cnt, c->rec_cap, tab, P_<uint64_t>(c->rec),
            P_<uint32_t>(c->chunk_hist), P_<uint32_t>(c->pend), P_<uint32_t>(c->pend_cnt), P_<uint32_t>(c->chunk_files),
            P_<LongTok>(c->longs), c->long_cap / kLongShards, nkeys, c->rec_lbits);
        HIPCK(hipEventRecord(c->ev_emit[1], c->st));
        k_long_totals<<<1, 64, 0, c->st>>>(counters);
        CK(run_reduce(c, OpPendCount{P_<uint32_t>(c->pend_cnt)}, nch, totals + 5));
        HIPCK(hipGetLastError());
        CK(run_reduce(c, OpOccupied{P_<unsigned long long>(c->tkeys)}, nslots, counters + C_INSERT));
        if (dense) {
            HIPCK(hipEventRecord(c->ev_res[0], c->st));
            k_long_verify<<<dim3(kLongShards, kLvBlocks), kBlock, 0, c->st>>>(
                c->text, c->nbytes, P_<LongTok>(c->longs), c->long_cap / kLongShards, P_<uint64_t>(c->trep), counters);
            HIPCK(hipEventRecord(c->ev_res[1], c->st));
        }
        if (c->rec_cap) CK(run_scan(c, OpInPlace{chunk_cnt}, nch + 1, totals));  // chunk token counts -> voff
        k_hist_reduce<<<hist_blocks(nch), kBlock, 0, c->st>>>(P_<uint32_t>(c->chunk_hist), nch, counters);
        HIPCK(hipGetLastError());
        uint64_t cnt[C_LONGMAX + 1], tot[10];  // (C_HIST .. C_HIST + 25 lie inside)
        static_assert(16 + C_LONGMAX + 1 <= kHbufRead, "map readback words");
        HIPCK(hipMemcpyAsync(c->hbuf + 16, counters, sizeof(cnt), hipMemcpyDeviceToHost, c->st));
        CK(read_u64(c, totals, tot, 10));  // (one synchronisation for both)
        memcpy(cnt, c->hbuf + 16, sizeof(cnt));
        if (tot[9]) return II_ERR_LAYOUT;
        if ((cnt[C_OVERFLOW] & 1) || cnt[C_INSERT] > kHotSlots / 2 + c->big_cap / 2) {
            c->big_cap *= 4;
            c->retries++;
            // more words than the hot level and a 2^22-slot big table hold: most of them live in the
            // big table, so the retry probes the bucket and the big home at once (DeepProbe; a context
            // with history chose it from its last reduce already)
            if (c->big_cap >= (1ull << 24) && c->text_is_input) c->deep_probe = true;
            continue;
        }
        if (cnt[C_OVERFLOW] & 2) {
            c->long_cap = (uint64_t)kLongShards * (cnt[C_LONGMAX] + cnt[C_LONGMAX] / 4 + 1024);
            c->retries++;
            continue;
        }
        if (cnt[C_COLLIDE]) {  // two long words hashed alike: new seed, redo (Las Vegas)
            if (++c->collide_retries > 12) return II_ERR_INTERNAL;
            c->seed = c->seed * 0x9e3779b97f4a7c15ull + 0x632be59bd9b4e019ull;
            c->retries++;
            continue;
        }
        c->nlong = cnt[C_LONG];
        c->V = cnt[C_INSERT];
        c->n_pending = tot[5];
        if (c->rec_cap) {
            c->T = tot[0];
            CK(grow(c->rec2, std::max(sizeof(uint64_t) * std::max<uint64_t>(c->T, 1), packed_bytes(c->T))));
        }
        memcpy(c->hist, cnt + C_HIST, sizeof(c->hist));
        break;
    }
    if (hist_out) memcpy(hist_out, c->hist, sizeof(c->hist));
    HIPCK(hipEventRecord(c->ev[1], c->st));
    if (!dense) {  // the exactness check on the side stream, after K1b (ev[1])
        uint64_t* counters_d = P_<uint64_t>(c->counters);
        HIPCK(hipStreamWaitEvent(c->st2, c->ev[1], 0));
        HIPCK(hipEventRecord(c->ev_res[0], c->st2));
        k_long_verify<<<dim3(kLongShards, kLvBlocks), kBlock, 0, c->st2>>>(
            c->text, c->nbytes, P_<LongTok>(c->longs), c->long_cap / kLongShards, P_<uint64_t>(c->trep), counters_d);
        if (c->test_collide) k_set_bits<<<1, 1, 0, c->st2>>>(counters_d + C_COLLIDE, 1ull);
        c->test_collide = false;
        HIPCK(hipEventRecord(c->ev_res[1], c->st2));
        HIPCK(hipGetLastError());
        c->lv_pending = true;
    }
    c->mapped = true;
    return II_OK;
}

// A map's exactness check (k_long_verify on st2) still reads c->text, the
// word table and the long queue until the reduce reads its verdict.  A new
// map before that reduce must not overwrite the text under it (ii_map_host /
// ii_map_files / ii_import write text_own from the host or the io streams
// before map_core orders c->st behind the check): wait for it on the host.
static int settle_side(ii_ctx* c) {
    if (c->lv_pending) HIPCK(hipEventSynchronize(c->ev_res[1]));
    return II_OK;
}

static int set_files(ii_ctx* c, const uint64_t* file_start, const uint32_t* file_id0, uint32_t nfiles) {
    for (uint32_t f = 1; f < nfiles; f++)
        if (file_id0[f] <= file_id0[f - 1] || file_start[f] < file_start[f - 1]) return II_ERR_ARG;
    if (nfiles && file_start[nfiles - 1] > c->nbytes) return II_ERR_ARG;
    // the same file table as the last call (a benchmark or a re-index of the
    // same layout): the device copy is current, skip the upload and its sync
    const bool same = nfiles && nfiles == c->nfiles && c->h_fstart.size() == nfiles &&
                      !memcmp(c->h_fstart.data(), file_start, sizeof(uint64_t) * nfiles) &&
                      !memcmp(c->h_fid.data(), file_id0, sizeof(uint32_t) * nfiles);
    CK(grow(c->fstart, sizeof(uint64_t) * (nfiles + 1)));
    CK(grow(c->fid, sizeof(uint32_t) * (nfiles + 1)));
    if (nfiles && !same) {
        HIPCK(hipMemcpyAsync(c->fstart.p, file_start, sizeof(uint64_t) * nfiles, hipMemcpyHostToDevice, c->st));
        HIPCK(hipMemcpyAsync(c->fid.p, file_id0, sizeof(uint32_t) * nfiles, hipMemcpyHostToDevice, c->st));
        HIPCK(hipStreamSynchronize(c->st));  // caller's host arrays may go away after return
    }
    c->nfiles = nfiles;
    c->id_bound = nfiles ? file_id0[nfiles - 1] + 1 : 0;
    // ascending ids: the last is first + nfiles - 1 iff they are consecutive
    c->fid_affine = !nfiles || file_id0[nfiles - 1] - file_id0[0] == nfiles - 1;
    c->fid_off = nfiles ? file_id0[0] : 0u;
    c->h_fstart.assign(file_start, file_start + nfiles);
    c->h_fid.assign(file_id0, file_id0 + nfiles);
    for (int k = 0; k < 9; k++) {  // the first file index whose id0 + 1 >= 10^(k + 1)
        uint64_t p10 = 10;
        for (int j = 0; j < k; j++) p10 *= 10;
        c->dth.t[k] = (uint32_t)(std::lower_bound(c->h_fid.begin(), c->h_fid.end(), (uint32_t)std::min<uint64_t>(p10 - 1, ~0u)) -
                                 c->h_fid.begin());
    }
    c->part_valid = false;
    c->text_is_input = true;
    c->collide_retries = 0;
    return II_OK;
}

extern "C" int ii_map_device(ii_ctx* c, const uint8_t* d_text, uint64_t nbytes, const uint64_t* file_start,
                             const uint32_t* file_id0, uint32_t nfiles, uint64_t hist_out[II_ALPHABET]) {
    if (!c || (nfiles && (!file_start || !file_id0)) || (nbytes && !d_text)) return II_ERR_ARG;
    if (((uintptr_t)d_text & 15u) != 0) return II_ERR_ARG;  // 16-byte staging loads
    LIVE_OR_FAIL();
    HIPCK(hipSetDevice(c->dev));
    CK(settle_side(c));
    c->text = d_text;
    c->nbytes = nbytes;
    CK(set_files(c, file_start, file_id0, nfiles));
    return map_core(c, hist_out);
}

static bool host_ws(uint8_t ch) { return ch == ' ' || (ch >= 9 && ch <= 13); }

// Lay files out back to back, inserting '\n' after a file whose last byte is
// not whitespace (separator contract), then one H2D copy.
extern "C" int ii_map_host(ii_ctx* c, const uint8_t* text, const uint64_t* file_off, const uint32_t* file_id0,
                           uint32_t nfiles, uint64_t hist_out[II_ALPHABET]) {
    if (!c || (nfiles && (!file_off || !file_id0 || !text))) return II_ERR_ARG;
    LIVE_OR_FAIL();
    HIPCK(hipSetDevice(c->dev));
    CK(settle_side(c));
    c->io_ms = 0;
    c->io_bytes = 0;
    for (uint32_t f = 0; f < nfiles; f++)
        if (file_off[f + 1] < file_off[f]) return II_ERR_ARG;
    uint64_t total = nfiles ? file_off[nfiles] - file_off[0] + nfiles : 0;
    std::vector<uint8_t> stage(total + 1);
    std::vector<uint64_t> fs(nfiles);
    uint64_t o = 0;
    for (uint32_t f = 0; f < nfiles; f++) {
        fs[f] = o;
        uint64_t n = file_off[f + 1] - file_off[f];
        if (n) memcpy(stage.data() + o, text + file_off[f], n);
        o += n;
        if (f + 1 < nfiles && (n == 0 || !host_ws(stage[o - 1]))) stage[o++] = '\n';
    }
    CK(grow(c->text_own, std::max<uint64_t>(o, 16)));
    if (o) HIPCK(hipMemcpyAsync(c->text_own.p, stage.data(), o, hipMemcpyHostToDevice, c->st));
    HIPCK(hipStreamSynchronize(c->st));
    c->text = P_<uint8_t>(c->text_own);
    c->nbytes = o;
    CK(set_files(c, fs.data(), file_id0, nfiles));
    return map_core(c, hist_out);
}

// ----------------------------------------------------------------- file reader (§8 f2)
// ii_map_files replaces the mappers' fopen/fscanf (main.c:93-102) with a
// pipelined reader: the device layout is known from the stat sizes (file f at
// off[f], one '\n' separator after every file), the layout is cut into
// windows of kIoWin bytes, and each of up to kIoThreads host threads reads
// its windows (pread straight into one of its two pinned buffers) and hands
// each one to its own stream as an async H2D copy, so reading window k+1
// overlaps copying window k.  A file shorter than its stat size is padded
// with spaces (no tokens); a file that turns out longer than its stat size
// (grown, or a size the caller did not know) makes the call fall back to
// whole-file reads (read_all_then_map).
namespace {
constexpr uint64_t kIoWin = 8ull << 20;
constexpr int kIoThreads = 16;

struct IoJob {
    ii_ctx* c;
    IoLayout lay;  // the device layout and its host-only reader (ii_reader.h)
    uint8_t* d_text;
    uint64_t total, nwin;
    int nt;
    int err;      // first error (II_*), 0 = ok
};
struct IoArg {
    IoJob* j;
    int t;
};

static void* io_worker(void* p) {
    IoArg* a = (IoArg*)p;
    IoJob* j = a->j;
    ii_ctx* c = j->c;
    int err = II_OK;
    if (!hip_ok(hipSetDevice(c->dev))) err = II_ERR_HIP;
    int k = 0;
    for (uint64_t w = (uint64_t)a->t; err == II_OK && w < j->nwin; w += (uint64_t)j->nt, k ^= 1) {
        const int b = 2 * a->t + k;
        if (!hip_ok(hipEventSynchronize(c->io_ev[b]))) { err = II_ERR_HIP; break; }  // buffer free again
        const uint64_t lo = w * kIoWin, hi = std::min(j->total, lo + kIoWin);
        io_fill(&j->lay, lo, hi, c->io_buf[b]);
        if (!hip_ok(hipMemcpyAsync(j->d_text + lo, c->io_buf[b], hi - lo, hipMemcpyHostToDevice, c->io_st[a->t])) ||
            !hip_ok(hipEventRecord(c->io_ev[b], c->io_st[a->t])))
            err = II_ERR_HIP;
    }
    if (err == II_OK && !hip_ok(hipStreamSynchronize(c->io_st[a->t]))) err = II_ERR_HIP;
    if (err != II_OK) {
        pthread_mutex_lock(&j->lay.mu);
        if (!j->err) j->err = err;
        pthread_mutex_unlock(&j->lay.mu);
    }
    return nullptr;
}

static int io_setup(ii_ctx* c, int nt) {
    while ((int)c->io_st.size() < nt) {
        hipStream_t s;
        HIPCK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        c->io_st.push_back(s);
        for (int k = 0; k < 2; k++) {
            void* h = nullptr;
            hipEvent_t e;
            HIPCK(hipHostMalloc(&h, kIoWin, hipHostMallocDefault));
            HIPCK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            HIPCK(hipEventRecord(e, s));  // the first wait on it returns at once
            c->io_buf.push_back((uint8_t*)h);
            c->io_ev.push_back(e);
        }
    }
    return II_OK;
}

// Whole-file reads, then one copy (files whose size was not known up front).
// The pipelined pass that found a grown file has already reported the
// missing ones (main.c:98), so this pass skips them quietly.
struct ReadJob {
    const ii_file* files;
    uint32_t n;
    std::vector<std::vector<uint8_t>>* data;
    uint32_t next;
    pthread_mutex_t mu;
};
void* read_worker(void* arg) {
    ReadJob* j = (ReadJob*)arg;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        uint32_t f = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (f >= j->n) break;
        FILE* fp = fopen(j->files[f].path, "rb");
        if (!fp) continue;  // reported by io_fill
        std::vector<uint8_t>& d = (*j->data)[f];
        d.resize(j->files[f].size ? j->files[f].size + 1 : 4096);
        size_t len = 0, r;
        while ((r = fread(d.data() + len, 1, d.size() - len, fp)) > 0) {
            len += r;
            if (len == d.size()) d.resize(d.size() * 2);
        }
        d.resize(len);
        fclose(fp);
    }
    return nullptr;
}
}  // namespace

static int read_all_then_map(ii_ctx* c, const ii_file* files, uint32_t nfiles, int nthreads,
                             uint64_t hist_out[II_ALPHABET]) {
    std::vector<std::vector<uint8_t>> data(nfiles);
    ReadJob job{files, nfiles, &data, 0, PTHREAD_MUTEX_INITIALIZER};
    int nt = std::max(1, std::min(nthreads, 64));
    std::vector<pthread_t> th(nt);
    for (int t = 0; t < nt; t++) pthread_create(&th[t], nullptr, read_worker, &job);
    for (int t = 0; t < nt; t++) pthread_join(th[t], nullptr);
    std::vector<uint64_t> off(nfiles + 1, 0);
    std::vector<uint32_t> ids(nfiles);
    for (uint32_t f = 0; f < nfiles; f++) {
        off[f + 1] = off[f] + data[f].size();
        ids[f] = files[f].id0;
    }
    std::vector<uint8_t> text(off[nfiles] + 1);
    for (uint32_t f = 0; f < nfiles; f++)
        if (!data[f].empty()) memcpy(text.data() + off[f], data[f].data(), data[f].size());
    data.clear();
    return ii_map_host(c, text.data(), off.data(), ids.data(), nfiles, hist_out);
}

extern "C" int ii_map_files(ii_ctx* c, const ii_file* files, uint32_t nfiles, int nthreads,
                            uint64_t hist_out[II_ALPHABET]) {
    if (!c || (nfiles && !files)) return II_ERR_ARG;
    for (uint32_t f = 0; f < nfiles; f++)
        if (!files[f].path || (f && files[f].id0 <= files[f - 1].id0)) return II_ERR_ARG;
    LIVE_OR_FAIL();
    HIPCK(hipSetDevice(c->dev));
    CK(settle_side(c));
    const double t0 = now_ms();
    std::vector<uint64_t> off(nfiles + 1, 0);
    for (uint32_t f = 0; f < nfiles; f++) off[f + 1] = off[f] + files[f].size + 1;
    const uint64_t total = off[nfiles];
    CK(grow(c->text_own, std::max<uint64_t>(total, 16)));
    const int nt = (int)std::max<uint64_t>(1, std::min<uint64_t>({(uint64_t)std::max(nthreads, 1), (uint64_t)kIoThreads,
                                                                    (total + kIoWin - 1) / kIoWin}));
    CK(io_setup(c, nt));
    IoJob job{c, IoLayout{files, nfiles, off.data(), 0, PTHREAD_MUTEX_INITIALIZER}, P_<uint8_t>(c->text_own), total,
              (total + kIoWin - 1) / kIoWin, nt, 0};
    std::vector<pthread_t> th(nt);
    std::vector<IoArg> args(nt);
    for (int t = 0; t < nt; t++) {
        args[t] = IoArg{&job, t};
        pthread_create(&th[t], nullptr, io_worker, &args[t]);
    }
    for (int t = 0; t < nt; t++) pthread_join(th[t], nullptr);
    if (job.err) return job.err;
    if (job.lay.grown) return read_all_then_map(c, files, nfiles, nthreads, hist_out);
    c->io_ms = now_ms() - t0;
    c->io_bytes = total;
    c->text = P_<uint8_t>(c->text_own);
    c->nbytes = total;
    std::vector<uint32_t> ids(nfiles);
    for (uint32_t f = 0; f < nfiles; f++) ids[f] = files[f].id0;
    CK(set_files(c, off.data(), ids.data(), nfiles));
    return map_core(c, hist_out);
}

// ----------------------------------------------------------------- reduce
// Work queued on the side stream st2 with scratch of its own: run_sort and
// run_scan take c->st, c->rtable, c->partial and c->kept, so for the life of
// the object those name st2's copies.  (A host-side swap: kernels capture
// their pointers at launch, so work queued earlier keeps its buffers.)
struct SideScope {
    ii_ctx* c;
    explicit SideScope(ii_ctx* c_) : c(c_) { swap(); }
    ~SideScope() { swap(); }
    void swap() {
        std::swap(c->st, c->st2);
        std::swap(c->partial, c->partial2);
        std::swap(c->rtable, c->rtable2);
        std::swap(c->kept, c->kept2);
        c->on_side = !c->on_side;
    }
};

// Dictionary, part 1 — all the token sort needs: every dictionary buffer
// grown, the occupied slots compacted (dslot, ascending: V of them; the count
// is copied to hbuf[1] for a check after a later synchronisation) and, for
// word-id keys, the hot-slot count and the big-table words' ids (wmap).
static int dict_slots(ii_ctx* c, bool wid) {
    uint64_t* totals = P_<uint64_t>(c->totals);
    const uint32_t V = (uint32_t)c->V;
    CK(grow(c->dslot, sizeof(uint32_t) * (V + 1)));
    CK(grow(c->dkey, sizeof(uint64_t) * (V + 1)));
    CK(grow(c->dkey2, sizeof(uint64_t) * (V + 1)));
    CK(grow(c->didx, sizeof(uint32_t) * (V + 1)));
    CK(grow(c->didx2, sizeof(uint32_t) * (V + 1)));
    const uint64_t nslots = kHotSlots + c->big_cap;
    CK(grow(c->remap, sizeof(uint32_t) * nslots));
    CK(grow(c->lkey, sizeof(uint64_t) * (V + 1)));
    CK(grow(c->lrep, sizeof(uint64_t) * (V + 1)));
    CK(grow(c->llen, sizeof(uint32_t) * (V + 1)));
    CK(grow(c->lstart, sizeof(uint32_t) * (II_ALPHABET + 1)));
    CK(grow(c->tied, sizeof(uint32_t) * (V + 1)));
    CK(grow(c->rtable2, sizeof(uint64_t) * kRadix * kMaxChunks));  // st2's sort scratch, grown here (never
    CK(grow(c->kept2, sizeof(uint64_t) * 2 * kMaxChunks));           // reallocated while st2 runs)
    uint32_t* dslot = P_<uint32_t>(c->dslot);
    if (wid) CK(grow(c->drank, sizeof(uint32_t) * kHotSlots));
    CK(run_scan(c, OpCompactSlots{P_<unsigned long long>(c->tkeys), dslot, wid ? P_<uint32_t>(c->drank) : nullptr},
                nslots, totals + 1));
    HIPCK(hipMemcpyAsync(c->hbuf + 1, totals + 1, sizeof(uint64_t), hipMemcpyDeviceToHost, c->st));
    if (wid) {  // word ids of the single-GPU token sort (k_wid_map; k_wid_finish after the lexicographic sort)
        CK(grow(c->wmap, sizeof(uint32_t) * nslots));
        CK(grow(c->lexw, sizeof(uint32_t) * (kHotSlots + V)));
        CK(grow(c->widl, sizeof(uint32_t) * (V + 1)));
        uint32_t* nhot = reinterpret_cast<uint32_t*>(totals + 7);
        HIPCK(hipMemsetAsync(totals + 7, 0, sizeof(uint64_t), c->st));
        k_count_hot<<<grid_for(V), kBlock, 0, c->st>>>(dslot, V, nhot);
        k_wid_map<<<grid_for(V), kBlock, 0, c->st>>>(dslot, V, nhot, P_<uint32_t>(c->wmap));
        HIPCK(hipGetLastError());
        c->NW = kHotSlots + V;  // bound; run_sort refines it from totals[7] after its first pass (no extra sync)
    }
    return II_OK;
}

// Dictionary, part 2: the lexicographic order of the V words (prefix-key
// sort, ties of longer words), remap / lkey / lrep / llen / lstart, and for
// word-id keys wid <-> lexid (lexw, widl).  Needs dict_slots' results.
static int dict_lex(ii_ctx* c, bool wid) {
    uint64_t* counters = P_<uint64_t>(c->counters);
    uint64_t* totals = P_<uint64_t>(c->totals);
    const uint32_t V = (uint32_t)c->V;
    const unsigned long long* keys = P_<unsigned long long>(c->tkeys);
    const uint64_t* rep = P_<uint64_t>(c->trep);
    uint32_t* dslot = P_<uint32_t>(c->dslot);
    uint64_t* sk = P_<uint64_t>(c->dkey);
    uint64_t* sk2 = P_<uint64_t>(c->dkey2);
    uint32_t* di = P_<uint32_t>(c->didx);
    uint32_t* di2 = P_<uint32_t>(c->didx2);
    k_dict_keys<<<grid_for(V), kBlock, 0, c->st>>>(c->text, c->nbytes, keys, rep, dslot, V, sk, di);
    CK(run_sort(c, &sk, &sk2, &di, &di2, V, 0, 64, false, nullptr));

    // words sharing a 12-letter prefix (both longer than 12): order them by
    // their remaining letters (LSD over 12-letter chunks on the tied subset)
    HIPCK(hipMemsetAsync(counters + C_TIES, 0, 2 * sizeof(uint64_t), c->st));
    k_tie_mark<<<grid_for(V), kBlock, 0, c->st>>>(sk, V, P_<uint32_t>(c->tied), counters);
    uint64_t nt;
    // the key sort may have run as onesweep passes: its look-back flag comes back with the tie count
    // (one synchronisation), before any kernel uses its values (di) as indices
    HIPCK(hipMemcpyAsync(c->hbuf + kHbufLbFlag, counters + C_OVERFLOW, sizeof(uint64_t), hipMemcpyDeviceToHost, c->st));
    CK(read_u64(c, counters + C_TIES, &nt));
    if (c->hbuf[kHbufLbFlag] & kLbTimeout) return II_ERR_INTERNAL;
    if (nt) {
        CK(grow(c->tpos, sizeof(uint32_t) * nt));
        CK(grow(c->rid, sizeof(uint32_t) * nt));
        CK(grow(c->rfirst, sizeof(uint32_t) * nt));
        CK(grow(c->tdict, sizeof(uint32_t) * nt));
        CK(grow(c->tk, sizeof(uint64_t) * nt));
        CK(grow(c->tk2, sizeof(uint64_t) * nt));
        CK(grow(c->tv, sizeof(uint32_t) * nt));
        CK(grow(c->tv2, sizeof(uint32_t) * nt));
        uint32_t* tpos = P_<uint32_t>(c->tpos);
        uint32_t* rid = P_<uint32_t>(c->rid);
        uint32_t* rfirst = P_<uint32_t>(c->rfirst);
        uint32_t* tdict = P_<uint32_t>(c->tdict);
        CK(run_scan(c, OpCompactTied{P_<uint32_t>(c->tied), tpos}, V, nullptr));
        CK(run_scan(c, OpTieRuns{tpos, sk, rid, rfirst}, nt, nullptr));
        uint32_t* tv = P_<uint32_t>(c->tv);
        uint32_t* tv2 = P_<uint32_t>(c->tv2);
        uint64_t* tk = P_<uint64_t>(c->tk);
        uint64_t* tk2 = P_<uint64_t>(c->tk2);
        k_tie_init<<<grid_for(nt), kBlock, 0, c->st>>>(c->text, c->nbytes, tpos, (uint32_t)nt, di, dslot, rep, tdict, tv,
                                                      counters);
        uint64_t maxlen;
        CK(read_u64(c, counters + C_MAXLEN, &maxlen));
        const uint32_t kmax = (uint32_t)((maxlen + 11) / 12) - 1;  // chunks 1..kmax beyond the prefix
        for (uint32_t ch = kmax; ch >= 1; ch--) {
            k_tie_keys<<<grid_for(nt), kBlock, 0, c->st>>>(c->text, c->nbytes, tv, (uint32_t)nt, tdict, dslot, rep, rid,
                                                          rfirst, ch, tk);
            CK(run_sort(c, &tk, &tk2, &tv, &tv2, nt, 0, 64, false, nullptr, nullptr, nullptr, false, false));
        }
        k_tie_keys<<<grid_for(nt), kBlock, 0, c->st>>>(c->text, c->nbytes, tv, (uint32_t)nt, tdict, dslot, rep, rid, rfirst,
                                                      0, tk);
        CK(run_sort(c, &tk, &tk2, &tv, &tv2, nt, 0, std::max(1, bitlen(nt)), false, nullptr, nullptr, nullptr, false,
                    false));
        k_tie_place<<<grid_for(nt), kBlock, 0, c->st>>>(tk, tv, (uint32_t)nt, tpos, tdict, di);
        HIPCK(hipGetLastError());
    }
    k_lex_finish<<<grid_for(V), kBlock, 0, c->st>>>(c->text, c->nbytes, di, dslot, keys, rep, V, P_<uint32_t>(c->remap),
                                                   P_<uint64_t>(c->lkey), P_<uint64_t>(c->lrep), P_<uint32_t>(c->llen));
    k_letter_start<<<grid_for(V + 1), kBlock, 0, c->st>>>(sk, V, P_<uint32_t>(c->lstart));
    if (wid)
        k_wid_finish<<<grid_for(V), kBlock, 0, c->st>>>(di, dslot, V, reinterpret_cast<const uint32_t*>(totals + 7),
                                                       P_<uint32_t>(c->lexw), P_<uint32_t>(c->widl));
    HIPCK(hipGetLastError());
    // keep the sorted prefix keys in dkey for the order step, their dictionary
    // indices in didx (the compact pairs' formatter)
    if (sk != P_<uint64_t>(c->dkey)) std::swap(c->dkey, c->dkey2);
    if (di != P_<uint32_t>(c->didx)) std::swap(c->didx, c->didx2);
    return II_OK;
}

// The whole dictionary in stream order (the owner's import; lexid-keyed sorts).
static int build_dictionary(ii_ctx* c, bool wid = false) {
    CK(dict_slots(c, wid));
    uint64_t vchk;
    CK(read_u64(c, P_<uint64_t>(c->totals) + 1, &vchk));
    if (vchk != c->V) return II_ERR_INTERNAL;
    return dict_lex(c, wid);
}

// Local reduce: dictionary (lexicographic ids), K2 token sort, K3 unique
// pairs.  After it the context holds a partial index: uniq (lexid, id0)
// pairs grouped by word, post_start, and the per-word dictionary arrays.
// wid: sort by word id (single-GPU reduce, k_wid_finish) instead of lexid;
// the exchange path needs letter-contiguous pairs and sorts by lexid.
static int local_reduce(ii_ctx* c, bool wid, bool compact) {
    uint64_t* totals = P_<uint64_t>(c->totals);
    (void)totals;
    c->n_sc = 0;
    const uint64_t T = c->T, V = c->V;
    int sort_passes = 0;
    if (T == 0) {
        c->U = 0;
        c->have_pairs = true;
        for (int e = 2; e < 5; e++) HIPCK(hipEventRecord(c->ev[e], c->st));
        return II_OK;
    }
    // ---- dictionary: lexicographic ids
    if (getenv("II_SORT_KEYS") && !strcmp(getenv("II_SORT_KEYS"), "lexid")) wid = false;
    // word-id keys: the token sort needs only the slot part of the dictionary;
    // its lexicographic part (a sort of the V prefix keys, ~0.5 ms of small
    // launches and host round trips) runs on st2 beside the sort, queued once
    // the sort is; K3's word-id -> lexid step waits for it
    const bool dict_side = wid && !(getenv("II_DICT_SIDE") && !strcmp(getenv("II_DICT_SIDE"), "0"));  // (same-box A/B: 394.0-394.5 GB/s with the dictionary in stream order, 395.6-396.3 beside the sort)
    if (dict_side) {
        CK(dict_slots(c, true));
        HIPCK(hipEventRecord(c->ev_dict[0], c->st));
    } else if (wid) {
        CK(build_dictionary(c, true));
    } else {
        CK(build_dictionary(c, false));
    }
    HIPCK(hipEventRecord(c->ev[2], c->st));

    // ---- K2: sort records by (lexid, fid); fid order is kept by stability
    uint64_t* r = P_<uint64_t>(c->rec);
    uint64_t* r2 = P_<uint64_t>(c->rec2);
    const int lb = std::max(1, bitlen((wid ? c->NW : V) - 1));
    uint64_t Tk = T;
    // the records carry shard-local file indices (k_chunk_files): F bits for this map's files
    int F = std::max(1, bitlen(c->nfiles ? c->nfiles - 1 : 0));
    // many small files with non-consecutive ids (a size-sorted ii_partition share): the first pass
    // (its record-set form) writes id0s (F = their bits) when the packed form still holds them —
    // K3's gather of fmap[index], in word order, missed L1 on nearly every pair (II_S0_FMAP=0|1:
    // A/B and test knob)
    bool s0map = false;
    if (!c->fid_affine && c->id_bound && dedup_by_set(c, T)) {
        const int Fg = std::max(1, bitlen(c->id_bound - 1));
        const char* e = getenv("II_S0_FMAP");
        if ((e ? strcmp(e, "0") != 0 : c->nfiles >= kS0FmapFiles) && packed_top_bits(lb, Fg)) {
            F = Fg;
            s0map = true;
        }
    }
    c->sort_packed = false;
    c->sort_W = lb;
    c->sort_F = F;
    const int m = packed_top_bits(lb, F);
    if (m) {
        c->s0_fmap = s0map ? P_<uint32_t>(c->fid) : nullptr;
        const int rc = run_sort_packed(c, &r, &r2, T, 32, lb, F, m, P_<uint32_t>(wid ? c->wmap : c->remap), &Tk, wid,
                                       &sort_passes);
        c->s0_fmap = nullptr;
        CK(rc);
    } else
        CK(run_sort(c, &r, &r2, nullptr, nullptr, T, 32, 32 + lb, true, &sort_passes,
                    P_<uint32_t>(wid ? c->wmap : c->remap), &Tk, wid));
    c->rec_sorted = r;
    c->T_sorted = Tk;
    // the next map's probe depth: DeepProbe when most distinct words live in the big table (NW = the
    // hot slots + the big-table words; wid keys only: lexid keys leave the choice as it was)
    if (wid) c->deep_probe = 2 * (c->NW - kHotSlots) > V;
    // the next map's big table: map_core regrows it when V > kHotSlots / 2 + big_cap / 2, so leave
    // room for 1.5 V, and keep the big table's load under 1/4 (a power of two, at least 2^16)
    // (input maps only: an import's vocabulary is one letter range of the shard's)
    if (c->text_is_input) {
        const uint64_t in_big = wid ? c->NW - kHotSlots : V;
        uint64_t want = 1ull << 16;
        while (kHotSlots / 2 + want / 2 < 3 * V / 2 || want < 4 * in_big) want <<= 1;
        c->big_next = want;
    }
    HIPCK(hipEventRecord(c->ev[3], c->st));
    if (dict_side) {
        HIPCK(hipEventSynchronize(c->ev_dict[0]));  // (the sort's own synchronisation is past it already)
        if (c->hbuf[1] != V) return II_ERR_INTERNAL;
        {
            SideScope side(c);  // c->st is st2 in here
            HIPCK(hipStreamWaitEvent(c->st, c->ev_dict[0], 0));
            CK(dict_lex(c, true));
            HIPCK(hipEventRecord(c->ev_dict[1], c->st));
        }
        HIPCK(hipStreamWaitEvent(c->st, c->ev_dict[1], 0));
    }
    // (a onesweep look-back that never resolved flags kLbTimeout: K3 then does nothing and run_unique,
    // which reads the flags with U, returns II_ERR_INTERNAL)
    if (c->test_lb_timeout == 2) k_set_bits<<<1, 1, 0, c->st>>>(P_<uint64_t>(c->counters) + C_OVERFLOW, kLbTimeout);

    // ---- K3: unique (word, file) pairs, posting byte offsets, posting starts.  The verdict of
    // the map's exactness check (k_long_verify on the side stream, map_core) is read with K3's
    // results (one host round trip); two long words with one hashed key: new seed, map + reduce again
    const bool check = c->lv_pending;
    if (check) {
        HIPCK(hipStreamWaitEvent(c->st, c->ev_res[1], 0));
        HIPCK(hipMemcpyAsync(c->hbuf, P_<uint64_t>(c->counters) + C_COLLIDE, sizeof(uint64_t), hipMemcpyDeviceToHost,
                             c->st));
    }
    CK(run_unique(c, r, Tk, wid, c->sort_packed, c->fid_affine || s0map ? nullptr : P_<uint32_t>(c->fid), compact,
                  c->fid_affine ? c->fid_off : 0u));
    if (check) {
        c->lv_pending = false;
        if (c->hbuf[0]) {  // (Las Vegas: the output never depends on the seed)
            if (++c->collide_retries > 12) return II_ERR_INTERNAL;
            c->seed = c->seed * 0x9e3779b97f4a7c15ull + 0x632be59bd9b4e019ull;
            const uint32_t r0 = c->retries;
            CK(map_core(c, nullptr));
            c->retries += r0 + 1;
            return local_reduce(c, wid, compact);
        }
    }
    c->wid_pairs = wid;
    HIPCK(hipEventRecord(c->ev[4], c->st));
    c->stats.sort_passes = (uint32_t)sort_passes;
    c->have_pairs = true;
    return II_OK;
}

// K4 final order + K5 formatting of the partial index held by the context.
static int order_and_format(ii_ctx* c, int copy_text) {
    uint64_t* totals = P_<uint64_t>(c->totals);
    const uint64_t V = c->V;
    if (c->U == 0 || V == 0) {
        c->out_bytes = 0;
        memset(c->h_letter_off, 0, sizeof(c->h_letter_off));
        for (int e = 5; e < 8; e++) HIPCK(hipEventRecord(c->ev[e], c->st));
        HIPCK(hipStreamSynchronize(c->st));
        c->host_text.clear();
        c->host_valid = copy_text != 0;
        c->reduced = true;
        return II_OK;
    }
    uint64_t* uniq = P_<uint64_t>(c->uniq);
    uint64_t* ps = P_<uint64_t>(c->pstart);
    // ---- K4: final order (letter, df desc, word asc)
    CK(grow(c->okey, sizeof(uint64_t) * V));
    CK(grow(c->okey2, sizeof(uint64_t) * V));
    CK(grow(c->oval, sizeof(uint32_t) * V));
    CK(grow(c->oval2, sizeof(uint32_t) * V));
    uint64_t* ok = P_<uint64_t>(c->okey);
    uint64_t* ok2 = P_<uint64_t>(c->okey2);
    uint32_t* ov = P_<uint32_t>(c->oval);
    uint32_t* ov2 = P_<uint32_t>(c->oval2);
    const int dbits = std::max(1, bitlen(c->id_bound));
    uint64_t* pe = P_<uint64_t>(c->pstop);
    uint64_t* Pp = P_<uint64_t>(c->P);
    CK(grow(c->loff, sizeof(uint64_t) * (V + 1)));
    uint64_t* loff = P_<uint64_t>(c->loff);
    k_order_keys<<<grid_for(V), kBlock, 0, c->st>>>(P_<uint64_t>(c->dkey), ps, pe, (uint32_t)V, dbits, ok, ov,
                                                    P_<uint32_t>(c->llen), Pp, loff);
    // (histogram passes: ov indexes loff / the formatter's tables before the host reads any flag)
    CK(run_sort(c, &ok, &ok2, &ov, &ov2, V, 0, dbits + 5, false, nullptr, nullptr, nullptr, false, false));
    if (c->test_lb_timeout == 4) k_set_bits<<<1, 1, 0, c->st>>>(P_<uint64_t>(c->counters) + C_OVERFLOW, kLbTimeout);
    c->ord = ov;
    HIPCK(hipEventRecord(c->ev[5], c->st));

    // ---- K5: format "word:[ids]\n" lines
    CK(grow(c->letter_off, sizeof(uint64_t) * (II_ALPHABET + 1)));
    CK(run_scan(c, OpLineOff{ov, loff}, V, totals + 2));
    CK(read_u64(c, totals + 2, &c->out_bytes));
    CK(grow(c->out, std::max<uint64_t>(c->out_bytes, 16)));
    uint8_t* out = P_<uint8_t>(c->out);
    // fbase by the pairs' word key (wid or lexid), or with compact pairs by the
    // dense word index (dict_idx of a lexid; lexid keys are dense already)
    const bool dense_wid = c->pairs32 && c->wid_pairs;
    CK(grow(c->fbase, sizeof(uint64_t) * (c->wid_pairs && !c->pairs32 ? c->NW : V)));
    uint64_t* fb = P_<uint64_t>(c->fbase);
    const uint32_t* fkey = dense_wid ? P_<uint32_t>(c->didx) : c->wid_pairs && !c->pairs32 ? P_<uint32_t>(c->widl) : nullptr;
    k_fmt_words<<<grid_for((V + kFmtWordItems - 1) / kFmtWordItems), kBlock, 0, c->st>>>(c->text, c->nbytes, P_<uint64_t>(c->lkey), P_<uint64_t>(c->lrep),
                                                  P_<uint32_t>(c->llen), ps, pe, Pp, loff, (uint32_t)V, out, fkey, fb);
    const uint32_t gfmt = (uint32_t)std::min<uint64_t>(16384, grid_for(c->U));
    if (c->pairs32) {
        const uint64_t ng = (c->U + 63) / 64;
        if (dense_wid)
            k_g64_dense<<<grid_for(ng), kBlock, 0, c->st>>>(P_<uint32_t>(c->g64), ng, P_<uint32_t>(c->drank),
                                                           reinterpret_cast<const uint32_t*>(totals + 7));
        k_fmt_posts<true><<<gfmt, kBlock, 0, c->st>>>(nullptr, P_<uint32_t>(c->uniq), P_<uint32_t>(c->g64), c->U, fb,
                                                      Pp, out);
    } else {
        k_fmt_posts<false><<<gfmt, kBlock, 0, c->st>>>(uniq, nullptr, nullptr, c->U, fb, Pp, out);
    }
    k_letter_off<<<1, 64, 0, c->st>>>(P_<uint32_t>(c->lstart), ov, loff, (uint32_t)V, c->out_bytes,
                                      P_<uint64_t>(c->letter_off));
    HIPCK(hipGetLastError());
    HIPCK(hipEventRecord(c->ev[6], c->st));
    // every sort of this reduce has run: a look-back flag raised by any of them (K3 and the dictionary
    // check theirs earlier) fails the reduce with the letter offsets' readback
    HIPCK(hipMemcpyAsync(c->hbuf + kHbufLbFlag, P_<uint64_t>(c->counters) + C_OVERFLOW, sizeof(uint64_t),
                         hipMemcpyDeviceToHost, c->st));
    CK(read_u64(c, c->letter_off.p, c->h_letter_off, II_ALPHABET + 1));
    if (c->hbuf[kHbufLbFlag] & kLbTimeout) return II_ERR_INTERNAL;
    if (copy_text) {
        c->host_text.resize(c->out_bytes + 1);
        if (c->out_bytes)
            HIPCK(hipMemcpyAsync(c->host_text.data(), out, c->out_bytes, hipMemcpyDeviceToHost, c->st));
    }
    HIPCK(hipEventRecord(c->ev[7], c->st));
    HIPCK(hipStreamSynchronize(c->st));
    c->host_valid = copy_text != 0;
    c->reduced = true;
    return II_OK;
}

// The exchange needs the u64 (word, id0) pairs of a word-id reduce.  A
// formatted-only reduce (ii_reduce) wrote compact pairs and its token sort
// consumed the K1 records in place (the packed passes write u32 records into
// rec), so an export after it maps the same input again before the local
// reduce (the input is the context's own copy, or the caller's d_text, which
// the context keeps until the next map call).  An owner's merged pairs
// (ii_import) are not exported again.
static int exportable_pairs(ii_ctx* c) {
    if (c->pairs32 && !c->text_is_input) return II_ERR_STATE;
    if (c->have_pairs && !c->pairs32) return II_OK;
    if (c->have_pairs && c->pairs32) CK(map_core(c, nullptr));  // records consumed: map again
    return local_reduce(c, true, false);
}

extern "C" int ii_reduce_local(ii_ctx* c) {
    if (!c) return II_ERR_ARG;
    if (!c->mapped) return II_ERR_STATE;
    LIVE_OR_FAIL();
    HIPCK(hipSetDevice(c->dev));
    return exportable_pairs(c);
}

extern "C" int ii_reduce(ii_ctx* c, int copy_text) {
    if (!c) return II_ERR_ARG;
    if (!c->mapped) return II_ERR_STATE;
    LIVE_OR_FAIL();
    HIPCK(hipSetDevice(c->dev));
    if (!c->have_pairs) CK(local_reduce(c, true, true));  // formatted only: compact pairs
    return order_and_format(c, copy_text);
}

// ----------------------------------------------------------------- exchange
// Per-letter points of the partial index (first word / pair / arena byte).
// After a word-id reduce the words' lexid-order pair starts (pstart_x) are
// scanned once per reduce; ii_export places the pairs by them.
// (a word-id reduce's pairs are exported from their word-id order by k_export_pairs_wid)
static int letter_points(ii_ctx* c) {
    const uint64_t V = c->V;
    if (V == 0 || c->T == 0) {
        memset(c->h_pts, 0, sizeof(c->h_pts));
        return II_OK;
    }
    const uint64_t* ps = P_<uint64_t>(c->pstart);
    if (c->wid_pairs) {  // the pairs' lexid-order starts (the export places each pair by them)
        CK(grow(c->pstart_x, sizeof(uint64_t) * (V + 1)));
        uint64_t* psx = P_<uint64_t>(c->pstart_x);
        if (!c->xpairs) {
            CK(run_scan(c, OpRunLen{ps, P_<uint64_t>(c->pstop), psx}, V, psx + V));
            c->xpairs = true;
        }
        ps = psx;
    }
    CK(grow(c->woff, sizeof(uint64_t) * (V + 1)));
    CK(grow(c->pts, sizeof(uint64_t) * 3 * (II_ALPHABET + 1)));
    uint64_t* woff = P_<uint64_t>(c->woff);
    CK(run_scan(c, OpWordArena{P_<uint32_t>(c->llen), woff}, V, woff + V));
    k_letter_points<<<1, 64, 0, c->st>>>(P_<uint32_t>(c->lstart), ps, woff, P_<uint64_t>(c->pts));
    HIPCK(hipGetLastError());
    CK(read_u64(c, c->pts.p, c->h_pts, 3 * (II_ALPHABET + 1)));
    return II_OK;
}

static inline uint64_t seg_bytes(uint64_t nw, uint64_t np, uint64_t arena) {
    (void)nw;
    return 64 + 8 * np + ((arena + 7) & ~7ull);
}

static int plan_core(ii_ctx* c, int nparts, const int* lo_in, const int* hi_in, uint64_t* bytes_out) {
    if (!c || nparts < 1 || nparts > II_MAX_PARTS || !bytes_out) return II_ERR_ARG;
    if (!c->mapped) return II_ERR_STATE;
    for (int r = 0; r < nparts; r++) {
        int lo, hi;
        if (lo_in) {
            lo = lo_in[r];
            hi = hi_in[r];
            // contiguous, in order, covering [0, 26)
            if (lo < 0 || hi < lo || hi > II_ALPHABET || lo != (r ? c->part_hi[r - 1] : 0)) return II_ERR_ARG;
        } else {
            ii_reducer_letters(r, nparts, &lo, &hi);
        }
        c->part_lo[r] = lo;
        c->part_hi[r] = hi;
    }
    if (c->part_hi[nparts - 1] != II_ALPHABET) return II_ERR_ARG;
    LIVE_OR_FAIL();
    HIPCK(hipSetDevice(c->dev));
    CK(exportable_pairs(c));
    CK(letter_points(c));
    for (int r = 0; r < nparts; r++) {
        const uint64_t* a = c->h_pts + 3 * c->part_lo[r];
        const uint64_t* b = c->h_pts + 3 * c->part_hi[r];
        bytes_out[r] = seg_bytes(b[0] - a[0], b[1] - a[1], b[2] - a[2]);
    }
    c->planned_parts = nparts;
    return II_OK;
}

extern "C" int ii_export_plan(ii_ctx* c, int nparts, uint64_t* bytes_out) {
    return plan_core(c, nparts, nullptr, nullptr, bytes_out);
}

extern "C" int ii_export_plan_ranges(ii_ctx* c, int nparts, const int* letter_lo, const int* letter_hi,
                                     uint64_t* bytes_out) {
    if (!letter_lo || !letter_hi) return II_ERR_ARG;
    return plan_core(c, nparts, letter_lo, letter_hi, bytes_out);
}

extern "C" int ii_letter_load(ii_ctx* c, uint64_t pairs[II_ALPHABET]) {
    if (!c || !pairs) return II_ERR_ARG;
    if (!c->mapped) return II_ERR_STATE;
    LIVE_OR_FAIL();
    HIPCK(hipSetDevice(c->dev));
    CK(exportable_pairs(c));
    CK(letter_points(c));
    for (int l = 0; l < II_ALPHABET; l++) pairs[l] = c->h_pts[3 * (l + 1) + 1] - c->h_pts[3 * l + 1];
    return II_OK;
}

extern "C" int ii_export(ii_ctx* c, int nparts, void* d_send, const uint64_t* send_off) {
    if (!c || nparts < 1 || !d_send || !send_off) return II_ERR_ARG;
    if (c->planned_parts != nparts) return II_ERR_STATE;
    LIVE_OR_FAIL();
    HIPCK(hipSetDevice(c->dev));
    static_assert(kExportMaxParts >= II_MAX_PARTS, "one export launch for every part");
    ExportParts xp;
    memset(&xp, 0, sizeof(xp));
    xp.n = (uint32_t)nparts;
    for (int r = 0; r < nparts; r++) {
        if (send_off[r] & 7) return II_ERR_ARG;
        const int lo = c->part_lo[r], hi = c->part_hi[r];
        const uint64_t* a = c->h_pts + 3 * lo;
        const uint64_t* b = c->h_pts + 3 * hi;
        const uint64_t nw = b[0] - a[0], np = b[1] - a[1], ab = b[2] - a[2];
        uint8_t* seg = (uint8_t*)d_send + send_off[r];
        uint64_t* pairs = (uint64_t*)(seg + 64);
        uint8_t* arena = seg + 64 + 8 * np;
        const uint64_t id_lo1 = c->h_fid.empty() ? 0 : 1ull + c->h_fid.front();
        const uint64_t id_hi1 = c->h_fid.empty() ? 0 : 1ull + c->h_fid.back();
        xp.j0[r] = (uint32_t)a[0];
        xp.j0[r + 1] = (uint32_t)b[0];
        xp.p0[r] = a[1];
        xp.dst[r] = pairs;
        k_export_header<<<1, 64, 0, c->st>>>((uint64_t*)seg, nw, np, ab, lo, hi, id_lo1, id_hi1);
        if (np && !c->wid_pairs)
            k_export_pairs<<<(uint32_t)std::min<uint64_t>(8192, grid_for(np)), kBlock, 0, c->st>>>(
                P_<uint64_t>(c->uniq), a[1], b[1], (uint32_t)a[0], pairs);
        if (nw)
            k_export_words<<<grid_for(nw), kBlock, 0, c->st>>>(c->text, c->nbytes, P_<uint64_t>(c->lkey),
                                                              P_<uint64_t>(c->lrep), P_<uint32_t>(c->llen),
                                                              P_<uint64_t>(c->woff), (uint32_t)a[0], (uint32_t)b[0],
                                                              arena);
        HIPCK(hipGetLastError());
    }
    if (c->wid_pairs && c->U) {  // every part's pairs in one pass over the word-id order
        k_export_pairs_wid<<<(uint32_t)std::min<uint64_t>(16384, grid_for((c->U + kExportItems - 1) / kExportItems)), kBlock, 0, c->st>>>(
            P_<uint64_t>(c->uniq), c->U, P_<uint32_t>(c->lexw), P_<uint64_t>(c->pstart), P_<uint64_t>(c->pstart_x), xp);
        HIPCK(hipGetLastError());
    }
    HIPCK(hipStreamSynchronize(c->st));
    return II_OK;
}

// The owner's merge of G sorted runs (back to back in *src, lengths len):
// ceil(log2 G) rounds of pairwise merge-path merges (ii_kernels.h
// k_merge_partition / k_merge_tiles), *src / *dst ping-pong; on return *src
// holds the merged records.  *rounds = the rounds run.
template <class K>
static int merge_sources(ii_ctx* c, K** src, K** dst, std::vector<uint64_t> len, int* rounds) {
    *rounds = 0;
    while (len.size() > 1) {
        MergeRound mr;
        memset(&mr, 0, sizeof(mr));
        mr.npairs = (uint32_t)((len.size() + 1) / 2);
        if (mr.npairs > (uint32_t)kMergeMaxPairs) return II_ERR_ARG;
        std::vector<uint64_t> next;
        uint64_t a = 0, tiles = 0;
        for (uint32_t p = 0; p < mr.npairs; p++) {
            const uint64_t na = len[2 * p], nb = 2 * p + 1 < len.size() ? len[2 * p + 1] : 0;
            mr.a[p] = a;
            mr.na[p] = na;
            mr.nb[p] = nb;
            mr.tile0[p] = (uint32_t)tiles;
            tiles += (na + nb + kMergeTile - 1) / kMergeTile;
            a += na + nb;
            next.push_back(na + nb);
        }
        if (tiles >= (1ull << 31)) return II_ERR_NOMEM;
        mr.tile0[mr.npairs] = (uint32_t)tiles;
        if (tiles) {
            CK(grow(c->moff, sizeof(uint64_t) * (tiles + 1)));
            uint64_t* split = P_<uint64_t>(c->moff);
            k_merge_partition<K><<<grid_for(tiles + 1), kBlock, 0, c->st>>>(*src, mr, split);
            // persistent workgroups: a few per CU (LDS: 2 tiles of K)
            const uint64_t grid = std::min<uint64_t>(tiles, (uint64_t)c->ncu * (sizeof(K) == 8 ? 4 : 8));
            k_merge_tiles<K><<<(uint32_t)grid, kMergeNT, 0, c->st>>>(*src, *dst, mr, split);
            HIPCK(hipGetLastError());
        }
        std::swap(*src, *dst);
        len.swap(next);
        (*rounds)++;
    }
    return II_OK;
}

extern "C" int ii_import(ii_ctx* c, int nparts, const void* d_recv, const uint64_t* recv_off, uint32_t id_bound) {
    if (!c || nparts < 1 || nparts > II_MAX_PARTS || !recv_off || (!d_recv && nparts)) return II_ERR_ARG;
    LIVE_OR_FAIL();
    HIPCK(hipSetDevice(c->dev));
    CK(settle_side(c));
    std::vector<uint64_t> hdr(8 * (size_t)nparts);
    for (int s = 0; s < nparts; s++) {
        if (recv_off[s] & 7) return II_ERR_ARG;
        HIPCK(hipMemcpyAsync(&hdr[8 * s], (const uint8_t*)d_recv + recv_off[s], 64, hipMemcpyDeviceToHost, c->st));
    }
    HIPCK(hipStreamSynchronize(c->st));
    uint64_t W = 0, NP = 0, A = 0;
    for (int s = 0; s < nparts; s++) {
        if (hdr[8 * s] != kSegMagic) return II_ERR_ARG;
        W += hdr[8 * s + 1];
        NP += hdr[8 * s + 2];
        A += hdr[8 * s + 3];
    }
    // merged word text: every source's words, in source order
    CK(grow(c->text_own, std::max<uint64_t>(A, 16)));
    uint64_t o = 0;
    for (int s = 0; s < nparts; s++) {
        const uint64_t np = hdr[8 * s + 2], ab = hdr[8 * s + 3];
        if (ab)
            HIPCK(hipMemcpyAsync((uint8_t*)c->text_own.p + o, (const uint8_t*)d_recv + recv_off[s] + 64 + 8 * np, ab,
                                 hipMemcpyDeviceToDevice, c->st));
        o += ab;
    }
    CK(grow(c->rec, sizeof(uint64_t) * std::max<uint64_t>({W, NP, 1})));
    CK(grow(c->rec2, sizeof(uint64_t) * std::max<uint64_t>({W, NP, 1}) + 16));  // + the u32 form's alignment pad
    c->text = P_<uint8_t>(c->text_own);
    c->nbytes = A;
    const uint64_t fs0 = 0;
    const uint32_t id0 = 0;
    CK(set_files(c, &fs0, &id0, A ? 1 : 0));
    c->text_is_input = false;
    CK(map_core(c, nullptr, true));  // tokenises the words: word k -> rec[k] = slot << 32
    if (c->T != W) return II_ERR_INTERNAL;
    c->id_bound = id_bound;
    if (W == 0) {
        c->T = 0;
        c->U = 0;
        c->have_pairs = true;
        return II_OK;
    }
    CK(build_dictionary(c));
    HIPCK(hipEventRecord(c->ev[2], c->st));
    uint64_t* wrec = P_<uint64_t>(c->rec);
    uint64_t* r = P_<uint64_t>(c->rec2);
    uint64_t* r2 = P_<uint64_t>(c->rec);
    // how the owner orders the received pairs by (lexid, id0): sources whose id ranges ascend without
    // overlap (ranks owning contiguous file ranges) merge as whole (word, source) runs in one scatter;
    // interleaved ones (ii_partition's size-sorted shards) by pairwise merge-path rounds, u32 records
    // lexid << F | id0 when both fit.  II_IMPORT_ID_SORT=1 (test knob) radix-sorts instead, =64 in the
    // u64 form.
    bool ordered = true;
    uint64_t prev_hi1 = 0;
    for (int s = 0; s < nparts && ordered; s++) {
        if (hdr[8 * s + 2] == 0) continue;
        const uint64_t lo1 = hdr[8 * s + 6], hi1 = hdr[8 * s + 7];
        if (lo1 == 0 || hi1 < lo1 || lo1 <= prev_hi1) ordered = false;
        prev_hi1 = hi1;
    }
    const char* ids_env = getenv("II_IMPORT_ID_SORT");
    const bool id_sort = ids_env != nullptr;
    const bool scatter_runs = !id_sort && ordered;
    const int Fid = std::max(1, bitlen(id_bound ? id_bound - 1 : 0)), Lw = std::max(1, bitlen(c->V - 1));
    const bool use32 = !scatter_runs && Lw + Fid <= 32 && !(id_sort && !strcmp(ids_env, "64"));
    // The pairs go to r (rec2) in every form: r2 is rec, which holds the word
    // records wrec every source's pairs are mapped through (writing records
    // there would overwrite word records later sources still read).
    static_assert(kImportMaxSrc >= II_MAX_PARTS, "one import launch for every source");
    ImportSrc isrc;
    memset(&isrc, 0, sizeof(isrc));
    isrc.n = (uint32_t)nparts;
    std::vector<uint64_t> runs;
    uint64_t wbase = 0, pbase = 0, blocks = 0;
    for (int s = 0; s < nparts; s++) {
        const uint64_t nw = hdr[8 * s + 1], np = hdr[8 * s + 2];
        isrc.p[s] = (const uint64_t*)((const uint8_t*)d_recv + recv_off[s] + 64);
        isrc.np[s] = np;
        isrc.wbase[s] = wbase;
        isrc.pbase[s] = pbase;
        isrc.bstart[s] = (uint32_t)blocks;
        blocks += (np + kImportPer - 1) / kImportPer;
        wbase += nw;
        pbase += np;
        runs.push_back(np);
    }
    if (blocks >= (1ull << 31)) return II_ERR_NOMEM;
    isrc.bstart[nparts] = (uint32_t)blocks;
    if (blocks) {
        if (use32)
            k_import_pairs<true><<<(uint32_t)blocks, kBlock, 0, c->st>>>(isrc, wrec, P_<uint32_t>(c->remap), r, Fid);
        else
            k_import_pairs<false><<<(uint32_t)blocks, kBlock, 0, c->st>>>(isrc, wrec, P_<uint32_t>(c->remap), r, 0);
    }
    HIPCK(hipGetLastError());
    int p1 = 0, p2 = 0;
    c->n_sc = 0;
    if (scatter_runs) {
        // Per (word, source) runs (k_merge_runs): with ascending id ranges the merged order is
        // (word, source), so k_merge_scatter moves whole runs
        const uint64_t nk = c->V * (uint64_t)nparts;
        CK(grow(c->mstart, sizeof(uint64_t) * std::max<uint64_t>(nk, 1)));
        CK(grow(c->mend, sizeof(uint64_t) * std::max<uint64_t>(nk, 1)));
        uint64_t* ms = P_<uint64_t>(c->mstart);
        uint64_t* me = P_<uint64_t>(c->mend);
        HIPCK(hipMemsetAsync(me, 0, sizeof(uint64_t) * nk, c->st));
        uint64_t pb = 0;
        for (int s = 0; s < nparts; s++) {
            const uint64_t np = hdr[8 * s + 2];
            if (np)
                k_merge_runs<<<(uint32_t)std::min<uint64_t>(16384, grid_for(np)), kBlock, 0, c->st>>>(
                    r, pb, np, (uint32_t)nparts, (uint32_t)s, ms, me);
            pb += np;
        }
        CK(run_scan(c, OpMergeRuns{ms, me}, nk, nullptr));
        pb = 0;
        for (int s = 0; s < nparts; s++) {
            const uint64_t np = hdr[8 * s + 2];
            if (np)
                k_merge_scatter<<<(uint32_t)std::min<uint64_t>(16384, grid_for(np)), kBlock, 0, c->st>>>(
                    r, pb, np, (uint32_t)nparts, (uint32_t)s, ms, me, r2);
            pb += np;
        }
        HIPCK(hipGetLastError());
        std::swap(r, r2);
    } else if (id_sort && use32) {  // (test knob) r holds the u32 records (its second half is the ping-pong buffer)
        uint32_t* a = reinterpret_cast<uint32_t*>(r);
        uint32_t* b = a + ((NP + 3) & ~3ull);  // 16-B aligned: k_radix_hist reads 16 B at a time
        CK(run_sort32(c, &a, &b, NP, Lw + Fid, &p1));
        // the word records are no longer read: the u64 records go to r2 (rec)
        k_unpack32<<<(uint32_t)std::min<uint64_t>(16384, grid_for(NP)), kBlock, 0, c->st>>>(a, NP, Fid, r2);
        HIPCK(hipGetLastError());
        std::swap(r, r2);
    } else if (id_sort) {  // (test knob) LSD over the id bits, then the word bits of the u64 records
        CK(run_sort(c, &r, &r2, nullptr, nullptr, NP, 0, Fid, false, &p1));
        CK(run_sort(c, &r, &r2, nullptr, nullptr, NP, 32, 32 + Lw, true, &p2));
    } else if (use32) {  // merge-path rounds over u32 records; K3 reads them as one bucket of the packed form
        uint32_t* a = reinterpret_cast<uint32_t*>(r);
        uint32_t* b = reinterpret_cast<uint32_t*>(r2);  // (rec: the word records are dead once mapped)
        CK(merge_sources(c, &a, &b, runs, &p1));
        const uint64_t ntb = (NP + kSweepTile - 1) / kSweepTile;
        CK(grow(c->msd, kMsdBytes));
        CK(grow(c->tbk, sizeof(uint16_t) * ntb));
        const MsdLayout g = msd_layout(c);
        HIPCK(hipMemsetAsync(c->tbk.p, 0, sizeof(uint16_t) * ntb, c->st));
        k_one_bucket<<<1, 1, 0, c->st>>>(g.bstart, g.btile, NP, (uint32_t)ntb);
        HIPCK(hipGetLastError());
        c->pk_nb = 1;
        c->pk_ntb = (uint32_t)ntb;
        c->pk_ncap = NP;
        c->pk_F = Fid;
        c->pk_L = Lw;
        HIPCK(hipEventRecord(c->ev[3], c->st));
        c->T = NP;
        CK(run_unique(c, reinterpret_cast<const uint64_t*>(a), NP, false, true, nullptr, true));
        HIPCK(hipEventRecord(c->ev[4], c->st));
        c->stats.sort_passes = (uint32_t)p1;
        c->have_pairs = true;
        return II_OK;
    } else {  // merge-path rounds over u64 records
        CK(merge_sources(c, &r, &r2, runs, &p1));
    }
    HIPCK(hipEventRecord(c->ev[3], c->st));
    c->T = NP;
    CK(run_unique(c, r, NP, false, false, nullptr, true));  // the owner's merged pairs: dense u64 records of id0s
    HIPCK(hipEventRecord(c->ev[4], c->st));
    c->stats.sort_passes = (uint32_t)(p1 + p2);
    c->have_pairs = true;
    return II_OK;
}

extern "C" int ii_letter_text(ii_ctx* c, int letter, const char** buf, size_t* len) {
    if (!c || letter < 0 || letter >= II_ALPHABET || !buf || !len) return II_ERR_ARG;
    if (!c->reduced || !c->host_valid) return II_ERR_STATE;
    static const char empty[1] = {0};
    uint64_t a = c->h_letter_off[letter], b = c->h_letter_off[letter + 1];
    *buf = c->host_text.empty() ? empty : c->host_text.data() + a;
    *len = (size_t)(b - a);
    return II_OK;
}

// ----------------------------------------------------------------- partial files (§8 f3)
extern "C" int ii_partials(ii_ctx* c, const uint32_t* order, uint32_t n) {
    if (!c || (n && !order)) return II_ERR_ARG;
    if (!c->mapped || !c->text_is_input) return II_ERR_STATE;
    LIVE_OR_FAIL();
    HIPCK(hipSetDevice(c->dev));
    c->part_valid = false;
    std::vector<PartPiece> pieces;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t f = order[i];
        if (f >= c->nfiles) return II_ERR_ARG;
        const uint64_t lo = c->h_fstart[f], hi = f + 1 < c->nfiles ? c->h_fstart[f + 1] : c->nbytes;
        for (uint64_t a = lo; a < hi; a += kPartPiece)
            pieces.push_back(PartPiece{a, std::min(hi, a + kPartPiece), c->h_fid[f], 0});
    }
    const uint64_t np = pieces.size();
    if (np > 0xFFFFFFFFull) return II_ERR_ARG;
    uint64_t* totals = P_<uint64_t>(c->totals);
    CK(grow(c->ploff, sizeof(uint64_t) * (II_ALPHABET + 1)));
    uint64_t* ploff = P_<uint64_t>(c->ploff);
    uint64_t total = 0;
    if (np) {
        CK(grow(c->ppieces, sizeof(PartPiece) * np));
        CK(grow(c->pcnt, sizeof(uint64_t) * 26 * np));
        HIPCK(hipMemcpyAsync(c->ppieces.p, pieces.data(), sizeof(PartPiece) * np, hipMemcpyHostToDevice, c->st));
        const PartPiece* dp = P_<PartPiece>(c->ppieces);
        uint64_t* cnt = P_<uint64_t>(c->pcnt);
        k_part_count<<<(uint32_t)np, kBlock, 0, c->st>>>(c->text, c->nbytes, dp, (uint32_t)np, cnt);
        CK(run_scan(c, OpInPlace{cnt}, 26 * np, totals));
        CK(read_u64(c, totals, &total));
        CK(grow(c->pout, std::max<uint64_t>(total, 16)));
        k_part_write<<<(uint32_t)np, kBlock, 0, c->st>>>(c->text, c->nbytes, dp, (uint32_t)np, cnt,
                                                       P_<uint8_t>(c->pout));
        k_part_letter_off<<<1, 64, 0, c->st>>>(cnt, (uint32_t)np, totals, ploff);
        HIPCK(hipGetLastError());
        CK(read_u64(c, ploff, c->h_part_off, II_ALPHABET + 1));
    } else {
        memset(c->h_part_off, 0, sizeof(c->h_part_off));
    }
    c->part_host.resize(total + 1);
    if (total) HIPCK(hipMemcpyAsync(c->part_host.data(), c->pout.p, total, hipMemcpyDeviceToHost, c->st));
    HIPCK(hipStreamSynchronize(c->st));
    c->part_valid = true;
    return II_OK;
}

extern "C" int ii_partial_text(ii_ctx* c, int letter, const char** buf, size_t* len) {
    if (!c || letter < 0 || letter >= II_ALPHABET || !buf || !len) return II_ERR_ARG;
    if (!c->part_valid) return II_ERR_STATE;
    const uint64_t a = c->h_part_off[letter], b = c->h_part_off[letter + 1];
    *buf = c->part_host.data() + a;
    *len = (size_t)(b - a);
    return II_OK;
}

extern "C" int ii_device_text(ii_ctx* c, const uint8_t** d_text, uint64_t letter_off[II_ALPHABET + 1]) {
    if (!c || !d_text) return II_ERR_ARG;
    if (!c->reduced) return II_ERR_STATE;
    *d_text = P_<uint8_t>(c->out);
    if (letter_off) memcpy(letter_off, c->h_letter_off, sizeof(c->h_letter_off));
    return II_OK;
}

static double ev_ms(hipEvent_t a, hipEvent_t b) {
    float ms = 0;
    if (!hip_ok(hipEventElapsedTime(&ms, a, b))) {
        (void)hipGetLastError();
        return 0;
    }
    return ms;
}

extern "C" int ii_get_stats(ii_ctx* c, ii_stats* o) {
    if (!c || !o) return II_ERR_ARG;
    if (!c->mapped) return II_ERR_STATE;
    LIVE_OR_FAIL();
    ii_stats s;
    memset(&s, 0, sizeof(s));
    s.bytes = c->nbytes;
    s.tokens = c->T;
    s.words = c->V;
    s.long_tokens = c->nlong;
    s.table_cap = kHotSlots + c->big_cap;
    s.retries = c->retries;
    memcpy(s.letter_tokens, c->hist, sizeof(c->hist));
    s.ms_map = ev_ms(c->ev[0], c->ev[1]);
    if (c->T) {
        s.emit_ms = ev_ms(c->ev_emit[0], c->ev_emit[1]);
        s.resolve_ms = c->nlong ? ev_ms(c->ev_res[0], c->ev_res[1]) : 0.0;
        s.resolved_tokens = c->n_pending;
        s.emit_bytes = c->nbytes + 8 * c->T;  // tokenize = B + r*T, r = 8-byte record
    }
    s.deep_probe = c->map_deep ? 1u : 0u;
    if (c->reduced || c->have_pairs) {  // (a local reduce, ii_reduce_local / the export, has these too)
        s.pairs = c->U;
        s.sort_passes = c->stats.sort_passes;
        s.ms_dict = ev_ms(c->ev[1], c->ev[2]);
        s.ms_sort = ev_ms(c->ev[2], c->ev[3]);
        s.ms_reduce = ev_ms(c->ev[3], c->ev[4]);
        if (c->reduced) {
            s.out_bytes = c->out_bytes;
            s.ms_order = ev_ms(c->ev[4], c->ev[5]);
            s.ms_format = ev_ms(c->ev[5], c->ev[6]);
            s.ms_total = ev_ms(c->ev[0], c->ev[6]);
        }
        double sum = 0;
        uint64_t bytes = 0;
        for (int i = 0; i < c->n_sc; i++) {
            sum += ev_ms(c->ev_sc[2 * i], c->ev_sc[2 * i + 1]);
            bytes += c->sc_bytes[i];
        }
        s.scatter_launches = (uint32_t)c->n_sc;
        s.scatter_ms_avg = c->n_sc ? sum / c->n_sc : 0;
        s.scatter_bytes = c->n_sc ? bytes / c->n_sc : 0;  // per launch: bytes read + written
        s.sort_bytes = bytes + (c->sort_packed ? c->sort_hist_bytes : 0);
        s.sort_packed = c->sort_packed ? 1u : 0u;
        s.pair_bytes = c->pairs32 ? 4u : 8u;
        s.sort_key_bits = (uint32_t)c->sort_W;
        s.sort_id_bits = (uint32_t)c->sort_F;
        s.sorted_records = c->T_sorted;
        if (c->c0_bytes) {
            s.sort0_ms = ev_ms(c->ev_c0[0], c->ev_c0[1]);
            s.sort0_bytes = c->c0_bytes;
        }
    }
    s.io_ms = c->io_ms;
    s.io_bytes = c->io_bytes;
    *o = s;
    return II_OK;
}

// ----------------------------------------------------------------- host helpers
extern "C" int ii_reducer_letters(int r, int R, int* lo, int* hi) {
    if (R < 1 || r < 0 || r >= R || !lo || !hi) return II_ERR_ARG;
    *lo = (II_ALPHABET / R) * r;                                       // main.c:129
    *hi = (r == R - 1) ? II_ALPHABET : (II_ALPHABET / R) * (r + 1);    // main.c:130
    return II_OK;
}

// Contiguous letter ranges for nparts owners minimising the largest summed
// weight (linear partition: DP for the optimum, then a greedy fill to it, so
// earlier parts take as much as the optimum allows).  Pure host arithmetic.
extern "C" int ii_balanced_letters(const uint64_t* w, int nparts, int* lo, int* hi) {
    if (!w || nparts < 1 || nparts > II_MAX_PARTS || !lo || !hi) return II_ERR_ARG;
    const int L = II_ALPHABET;
    uint64_t pre[II_ALPHABET + 1] = {0};
    for (int l = 0; l < L; l++) pre[l + 1] = pre[l] + w[l];
    // best[k][i]: the smallest possible largest part when letters [0, i) go to k parts
    std::vector<std::vector<uint64_t>> best(nparts + 1, std::vector<uint64_t>(L + 1, UINT64_MAX));
    best[0][0] = 0;
    for (int k = 1; k <= nparts; k++)
        for (int i = 0; i <= L; i++)
            for (int j = 0; j <= i; j++)
                if (best[k - 1][j] != UINT64_MAX)
                    best[k][i] = std::min(best[k][i], std::max(best[k - 1][j], pre[i] - pre[j]));
    const uint64_t opt = best[nparts][L];
    int r = 0;
    uint64_t sum = 0;
    lo[0] = 0;
    for (int l = 0; l < L; l++) {
        if (sum + w[l] > opt && r < nparts - 1) {
            hi[r] = l;
            lo[++r] = l;
            sum = 0;
        }
        sum += w[l];
    }
    hi[r] = L;
    for (int k = r + 1; k < nparts; k++) lo[k] = hi[k] = L;
    return II_OK;
}

extern "C" int ii_partition(const uint64_t* sizes, uint32_t nfiles, int M, uint32_t* order, uint32_t* shard_begin,
                            uint32_t* shard_end) {
    if (M < 1 || (nfiles && (!sizes || !order)) || !shard_begin || !shard_end) return II_ERR_ARG;
    for (uint32_t i = 0; i < nfiles; i++) order[i] = i;
    // size descending (main.c:21-25, 300); ties by list position (stable)
    std::stable_sort(order, order + nfiles, [&](uint32_t a, uint32_t b) { return sizes[a] > sizes[b]; });
    uint64_t total = 0;
    for (uint32_t i = 0; i < nfiles; i++) total += sizes[i];
    const uint64_t per = total / (uint64_t)M;  // main.c:307
    for (int m = 0; m < M; m++) shard_begin[m] = shard_end[m] = nfiles;
    int cur = 0;
    uint64_t cum = 0;
    shard_begin[0] = 0;
    for (uint32_t i = 0; i < nfiles; i++) {  // main.c:315-322
        cum += sizes[order[i]];
        if (cum >= per && cur < M - 1) {
            shard_end[cur] = i + 1;
            shard_begin[++cur] = i + 1;
            cum = 0;
        }
    }
    shard_end[cur] = nfiles;  // main.c:323
    for (int m = cur + 1; m < M; m++) shard_begin[m] = shard_end[m] = nfiles;  // defined: empty shards
    return II_OK;
}
