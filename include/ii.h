/*
 * ii.h — C ABI of the MI355X inverted-index builder (libii.so).
 *
 * Drop-in boundary for the reference's mapper/reducer path
 * (/root/reference/main.c).  The reference has no library API: its path sits
 * behind the CLI `tema1 <M> <R> <list>` (main.c:246-255) and the pthread
 * entry points mapper()/reducer() (main.c:85, main.c:126) joined by the
 * partial_<letter>.txt files (main.c:332-341).  Each entry point below names
 * the reference code it replaces.  All signatures use plain C types and
 * pointers only.
 *
 * Ownership: the caller owns the file list, paths and input buffers; the
 * context owns every device and host buffer it allocates, including the
 * text returned by ii_letter_text (valid until the next ii_map_* / ii_reduce
 * call, an export plan or letter load that follows ii_reduce — see
 * ii_export_plan — or ii_close).
 * Errors: 0 = OK, negative = error code (ii_strerror).  Calls on one context
 * are not re-entrant; use one context per GPU.
 */
#ifndef II_H
#define II_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define II_ALPHABET 26 /* main.c:9 ALPHABET_SIZE */
#define II_MAX_WORD 300 /* main.c:7 MAX_WORD: cleaned words keep <= 299 letters */

enum {
    II_OK = 0,
    II_ERR_ARG = -1,        /* bad argument (NULL, out-of-range, unsorted IDs) */
    II_ERR_HIP = -2,        /* a HIP runtime call failed */
    II_ERR_NOMEM = -3,      /* device or host allocation failed */
    II_ERR_IO = -4,         /* list file unreadable / malformed (main.c:257-285) */
    II_ERR_STATE = -5,      /* call out of order (e.g. ii_reduce before any map) */
    II_ERR_LAYOUT = -6,     /* device text violates the separator contract */
    II_ERR_INTERNAL = -7,   /* internal consistency check failed */
    II_ERR_NODEV = -8       /* no HIP device */
};

typedef struct ii_ctx ii_ctx;

/* One input file of a shard.  Replaces FileInfo (main.c:14-18).  id0 is the
 * 0-based position in the list file (main.c:275) and is printed as id0+1
 * (main.c:116).  mapper is the reference mapper whose shard holds the file
 * (ii_partition, main.c:300-323): only printed, in the missing-file message
 * "Mapper <mapper>: Error opening file <path>" (main.c:98); 0 if unknown. */
typedef struct {
    const char *path;
    uint64_t size;
    uint32_t id0;
    int32_t mapper;
} ii_file;

/* Per-run counters (no reference equivalent; the reference only prints). */
typedef struct {
    uint64_t bytes;        /* input bytes indexed (B) */
    uint64_t tokens;       /* kept tokens T (= lines the reference writes to partial files) */
    uint64_t pairs;        /* unique (word, file) pairs U */
    uint64_t words;        /* distinct words V */
    uint64_t long_tokens;  /* tokens with more than 12 letters */
    uint64_t out_bytes;    /* bytes of the 26 letter texts */
    uint64_t table_cap;    /* word-table capacity (slots) */
    uint32_t retries;      /* word-table regrows / rehashes in the last map */
    uint32_t sort_passes;  /* radix passes of the token sort */
    uint64_t letter_tokens[II_ALPHABET]; /* tokens per first letter (partial_<l>.txt line counts) */
    /* device time per phase, milliseconds (hipEvent, stream-ordered) */
    double ms_map;         /* tokenize + word table (K1) */
    double ms_dict;        /* dictionary / lexicographic ids */
    double ms_sort;        /* token sort (K2) */
    double ms_reduce;      /* unique + postings (K3) */
    double ms_order;       /* final order (K4) */
    double ms_format;      /* text formatting (K5) */
    double ms_total;
    /* dominant kernel: the radix scatter of the token sort */
    double scatter_ms_avg; /* average duration of one token-sort scatter launch */
    uint64_t scatter_bytes;/* average algorithmic bytes of one token-sort scatter launch */
    uint32_t scatter_launches;
    uint64_t sorted_records; /* records left after the sort's first-pass (hot word, file) dedup */
    /* tokenizer kernel (K1b k_tok_emit), the dominant kernel */
    double emit_ms;        /* duration of the last k_tok_emit launch */
    uint64_t emit_bytes;   /* its algorithmic bytes: B text read + 8 B per record written */
    double resolve_ms;     /* k_long_verify, the exactness pass of hashed (> 12-letter) keys */
    uint64_t resolved_tokens; /* tokens K1b's fast path left to its K1c tail (general path, full hot bucket, raced claim) */
    double sort0_ms;       /* first token-sort pass: dedup + lexid remap + compaction (k_sort0_compact) */
    uint64_t sort0_bytes;  /* its algorithmic bytes: the records read (4 B each from narrow chunks, whose u32
                              word slots K1b wrote, 8 B from the others) + 8 B per kept record written */
    /* ii_map_files only (0 otherwise): host wall time of reading the files and
     * uploading them (pipelined pread -> pinned windows -> async H2D), and
     * the bytes uploaded */
    double io_ms;
    uint64_t io_bytes;
    /* bytes the token sort's passes after the first move (reads + writes of
     * every scatter / onesweep launch and the packed form's bucket histogram) */
    uint64_t sort_bytes;
    uint32_t sort_packed;  /* 1: the packed form (u32 records in buckets, ii_prims.h) ran */
    uint32_t sort_key_bits;  /* W: bits of the token sort's word keys */
    uint32_t sort_id_bits;   /* F: bits of the sorted records' file fields: shard-local indices, or id0s when the first pass maps them (packed form: W + F - 32 <= 11) */
    uint32_t pair_bytes;     /* bytes per distinct pair K3 wrote: 4 (compact, formatted only) or 8 (exportable) */
    uint32_t deep_probe;     /* 1: the last map's K1b probed the whole bucket and the big-table home (large vocabulary) */
} ii_stats;

/* Open a context on HIP device `device`. */
int ii_open(ii_ctx **out, int device);
void ii_close(ii_ctx *ctx);
const char *ii_strerror(int code);

/*
 * Map phase.  Replaces mapper() (main.c:85-124) for a whole shard plus the
 * partial-file shuffle (main.c:332-341, 116, 371-373): tokens become
 * device-resident (word, file) records; hist_out (may be NULL) receives the
 * number of tokens per first letter, i.e. the line counts the reference
 * would have written to partial_<letter>.txt.
 *
 * Files must be given in ascending id0 order.  Missing / unreadable files are
 * reported once on stderr in the reference's wording (main.c:98, with
 * ii_file.mapper) and contribute nothing; they are not an error.  `nthreads` host reader threads (the
 * reference's M, at most 16) read the files: files[f].size (the stat size)
 * fixes each file's place on the device, the threads pread 8 MiB windows
 * into pinned buffers and upload each with an async copy on their own stream
 * while reading the next.  A file found longer than its
 * size makes the call fall back to whole-file reads.
 */
int ii_map_files(ii_ctx *ctx, const ii_file *files, uint32_t nfiles, int nthreads,
                 uint64_t hist_out[II_ALPHABET]);

/* Map phase over host memory: file f is text[file_off[f] .. file_off[f+1]),
 * with IDs file_id0[f] (ascending). */
int ii_map_host(ii_ctx *ctx, const uint8_t *text, const uint64_t *file_off, const uint32_t *file_id0,
                uint32_t nfiles, uint64_t hist_out[II_ALPHABET]);

/* Map phase over device-resident text (no host copy of the text).
 * d_text holds nbytes bytes; host arrays file_start (nfiles entries) and
 * file_id0 (ascending) describe the files: file f starts at file_start[f] and
 * ends where the next begins (or at nbytes).  Separator contract: for every
 * f > 0 with file_start[f] > 0, d_text[file_start[f] - 1] must be C-locale
 * whitespace, so no token can span two files (checked: II_ERR_LAYOUT).
 * d_text must be 16-byte aligned (II_ERR_ARG otherwise).
 * The context keeps a pointer to d_text until the next map call. */
int ii_map_device(ii_ctx *ctx, const uint8_t *d_text, uint64_t nbytes, const uint64_t *file_start,
                  const uint32_t *file_id0, uint32_t nfiles, uint64_t hist_out[II_ALPHABET]);

/*
 * Reduce phase.  Replaces reducer() (main.c:126-242) for all 26 letters:
 * group by word, distinct file IDs (main.c:170-213), order by (df desc,
 * word asc) with ascending IDs (main.c:55-64, 215-226), and format every
 * line "word:[id id ...]\n" (main.c:227-234) — all on the device.
 * With copy_text != 0 the text is also copied to host memory for
 * ii_letter_text; with 0 it stays device-resident (benchmarking).
 */
int ii_reduce(ii_ctx *ctx, int copy_text);

/* First half of ii_reduce: distinct (word, file) pairs grouped by word — the
 * state the reducers reach after main.c:170-213, for this context's files.
 * Needed explicitly only before ii_export_plan (ii_reduce runs it itself). */
int ii_reduce_local(ii_ctx *ctx);

/*
 * Multi-GPU exchange.  The reference assigns first-letter
 * ranges to reducers (main.c:129-130); with G GPUs, GPU r owns the letters
 * ii_reducer_letters(r, G).  Each GPU maps its shard of files, then:
 *   ii_export_plan  -> bytes of the segment for every owner (host array)
 *   ii_export       -> writes the segments into a device send buffer at the
 *                      caller's (8-byte aligned) offsets
 *   (caller moves segment r of every GPU to GPU r: RCCL all-to-allv)
 *   ii_import       -> merges the G received segments (one per source, in
 *                      source order) into this context's partial index
 *   ii_reduce       -> orders and formats the owner's letters
 * Segment layout (little-endian, 8-byte aligned):
 *   u64 header[8] = {magic "IXIISEG1", nwords, npairs, arena_bytes,
 *                    letter_lo, letter_hi, 1 + smallest id0, 1 + largest id0}
 *                   (the exporter's file ids; 0, 0 = unknown)
 *   u64 pairs[npairs] = (word index in segment) << 32 | id0
 *   u8  arena[arena_bytes rounded up to 8] = words in lexicographic order,
 *                    each followed by ' '
 * id_bound = 1 + the largest id0 of all files of all GPUs.
 * Called after ii_reduce (whose token sort consumed the mapped records),
 * ii_export_plan, ii_export_plan_ranges and ii_letter_load index the mapped
 * input again: the text of the last ii_map_* call must still be valid (for
 * ii_map_device, d_text), and the ii_letter_text results of that ii_reduce
 * are invalidated (II_ERR_STATE until the next ii_reduce).
 */
int ii_export_plan(ii_ctx *ctx, int nparts, uint64_t *seg_bytes);

/* Histogram-balanced letter ownership.  The reference's
 * 26/G split (main.c:129-130) gives owners 4 % to 24 % of the work at G = 8;
 * instead, part r may own the contiguous letters [letter_lo[r], letter_hi[r])
 * chosen from a per-letter load:
 *   ii_letter_load       -> distinct (word, file) pairs per first letter of
 *                           this context's partial index (sum it over GPUs)
 *   ii_balanced_letters  -> contiguous ranges minimising the largest part's
 *                           load (pure host arithmetic; parts may be empty)
 *   ii_export_plan_ranges-> ii_export_plan with those ranges (every GPU must
 *                           pass the same ranges) */
#define II_MAX_PARTS 64
int ii_letter_load(ii_ctx *ctx, uint64_t pairs[II_ALPHABET]);
int ii_balanced_letters(const uint64_t weight[II_ALPHABET], int nparts, int *letter_lo, int *letter_hi);
int ii_export_plan_ranges(ii_ctx *ctx, int nparts, const int *letter_lo, const int *letter_hi, uint64_t *seg_bytes);
int ii_export(ii_ctx *ctx, int nparts, void *d_send, const uint64_t *send_off);
/* ii_import: segment s comes from source s (0 .. nparts-1, any order of file
 * ids across sources), and every file id belongs to ONE source — files are
 * sharded, not replicated (main.c:300-323 gives each file one mapper).
 * 1 <= nparts <= II_MAX_PARTS, else II_ERR_ARG. */
int ii_import(ii_ctx *ctx, int nparts, const void *d_recv, const uint64_t *recv_off, uint32_t id_bound);

/* Text of <letter>.txt (letter 0..25 = 'a'..'z'), valid until the next call. */
int ii_letter_text(ii_ctx *ctx, int letter, const char **buf, size_t *len);

/*
 * Partial files.  The reference's mappers write every kept
 * token as "<clean word> <id0+1>\n" to partial_<first letter>.txt
 * (main.c:113-118; files created at main.c:332-341).  The index does not need
 * them; this builds their text on the device from the mapped input (valid
 * after any ii_map_* call, until the next one; not after ii_import).
 * order[0..n) lists indices of the mapped files (0 = first file of the map
 * call) in emission order; tokens keep their text order inside each file.
 * With the size order of ii_partition and M = 1 the text is byte-identical to
 * the reference's; with M > 1 the reference interleaves mappers by thread
 * timing, and the order given here (mapper 0's files, then mapper 1's, ...)
 * is one of its outcomes.
 */
int ii_partials(ii_ctx *ctx, const uint32_t *order, uint32_t n);
/* Text of partial_<letter>.txt after ii_partials, valid until the next map or
 * ii_partials call. */
int ii_partial_text(ii_ctx *ctx, int letter, const char **buf, size_t *len);

/* Counters and phase timings of the last map + reduce. */
int ii_get_stats(ii_ctx *ctx, ii_stats *out);

/* Device pointer + byte offsets of the formatted index (device-resident
 * output, letter l = [letter_off[l], letter_off[l+1])). */
int ii_device_text(ii_ctx *ctx, const uint8_t **d_text, uint64_t letter_off[II_ALPHABET + 1]);

/* Reducer letter range (main.c:129-130): reducer r of R owns
 * [(26/R)*r, r == R-1 ? 26 : (26/R)*(r+1)).  Pure host arithmetic. */
int ii_reducer_letters(int r, int R, int *lo, int *hi);

/* Size-sorted greedy shard partition (main.c:21-25, 300-323), defined for
 * every M >= 1 (empty shards where the reference is undefined):
 * order[] receives the file indices sorted by (size desc, index asc);
 * shard_begin/shard_end (M entries each) receive [begin, end) ranges into
 * order[].  Pure host arithmetic. */
int ii_partition(const uint64_t *sizes, uint32_t nfiles, int M, uint32_t *order, uint32_t *shard_begin,
                 uint32_t *shard_end);

#ifdef __cplusplus
}
#endif
#endif /* II_H */
