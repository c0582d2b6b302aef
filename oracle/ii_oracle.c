/*
 * ii_oracle.c — CPU restatement of the reference inverted-index semantics.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity CHECKER for the MI355X
 * product path; it is never linked into, called by, or shipped with the
 * product (libii.so / ii_index).  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may use it.
 *
 * Parity is PINNED: outputs of this restatement are checked byte-for-byte
 * against outputs of the reference binary itself (oracle/_ref/tema1, built
 * from /root/reference/main.c by oracle/Makefile) on every fixture under
 * tests/golden/ (configs 1 and 2, the edge corpus, seeded random corpora).
 *
 * What it restates (reference = /root/reference/main.c):
 *   - file list: count, then `count` whitespace-delimited names; ID = list
 *     position (main.c:263-285, id at main.c:275, printed id+1 at main.c:116)
 *   - tokenizer: fscanf("%s") whitespace tokens, C-locale isspace set
 *     (main.c:102)
 *   - cleaning: keep A-Z (+32) and a-z, stop at the first NUL, at most
 *     MAX_WORD-1 = 299 letters, drop tokens with no letters (main.c:103-113)
 *   - bucketing by first letter (main.c:114-116)
 *   - reducer: distinct file IDs per word (main.c:170-213, add_number
 *     main.c:67-77)
 *   - order: df descending, then strcmp ascending (compare_word_entries
 *     main.c:55-64, qsort main.c:215); IDs ascending (main.c:217-226)
 *   - writer: "word:[id id ...]\n" into <letter>.txt (main.c:227-234)
 * Reference UB is defined as SURVEY.md §9.11 says: raw tokens longer than 299
 * bytes keep their first 299 letters; any number of files.
 *
 * The restatement groups with a hash map instead of the reference's linear
 * scan (main.c:172-173) — same result, O(T) instead of O(T*V).
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#define OR_MAX_WORD 300 /* main.c:7 */
#define OR_ALPHA 26     /* main.c:9 */

/* C-locale isspace (fscanf %s delimiter set, main.c:102). */
static inline int or_isspace(unsigned char c) {
    return c == ' ' || (c >= 0x09 && c <= 0x0d);
}

typedef struct {
    char *word;     /* cleaned word, NUL-terminated */
    uint32_t len;
    uint64_t hash;
    uint32_t *ids;  /* distinct 1-based file IDs, ascending (files are visited in ID order) */
    uint32_t n, cap;
} or_entry;

typedef struct {
    or_entry *e;
    uint32_t n, cap;     /* entries */
    uint32_t *slot;      /* open-addressing table of entry index + 1 */
    uint64_t mask;
} or_dict;

static uint64_t or_hash(const char *s, uint32_t n) {
    uint64_t h = 1469598103934665603ull;
    for (uint32_t i = 0; i < n; i++) { h ^= (unsigned char)s[i]; h *= 1099511628211ull; }
    return h ^ (h >> 29);
}

static void or_dict_grow(or_dict *d) {
    uint64_t ncap = d->mask ? (d->mask + 1) * 2 : 1024;
    uint32_t *ns = calloc(ncap, sizeof(uint32_t));
    if (!ns) { fprintf(stderr, "oracle: out of memory\n"); exit(EXIT_FAILURE); }
    for (uint32_t i = 0; i < d->n; i++) {
        uint64_t s = d->e[i].hash & (ncap - 1);
        while (ns[s]) s = (s + 1) & (ncap - 1);
        ns[s] = i + 1;
    }
    free(d->slot);
    d->slot = ns;
    d->mask = ncap - 1;
}

/* Record (word, id1) — the reducer's "find word, add id if new" step
 * (main.c:170-213).  Because files are visited in ascending ID order, a
 * duplicate ID is always the last one appended. */
static void or_dict_add(or_dict *d, const char *w, uint32_t n, uint32_t id1) {
    if ((uint64_t)(d->n + 1) * 2 > d->mask + 1) or_dict_grow(d);
    uint64_t h = or_hash(w, n);
    uint64_t s = h & d->mask;
    for (;;) {
        uint32_t x = d->slot[s];
        if (!x) break;
        or_entry *e = &d->e[x - 1];
        if (e->hash == h && e->len == n && memcmp(e->word, w, n) == 0) {
            if (e->ids[e->n - 1] != id1) {
                if (e->n == e->cap) {
                    e->cap *= 2;
                    e->ids = realloc(e->ids, e->cap * sizeof(uint32_t));
                    if (!e->ids) { fprintf(stderr, "oracle: out of memory\n"); exit(EXIT_FAILURE); }
                }
                e->ids[e->n++] = id1;
            }
            return;
        }
        s = (s + 1) & d->mask;
    }
    if (d->n == d->cap) {
        d->cap = d->cap ? d->cap * 2 : 1024;
        d->e = realloc(d->e, d->cap * sizeof(or_entry));
        if (!d->e) { fprintf(stderr, "oracle: out of memory\n"); exit(EXIT_FAILURE); }
    }
    or_entry *e = &d->e[d->n];
    e->word = malloc(n + 1);
    memcpy(e->word, w, n);
    e->word[n] = 0;
    e->len = n;
    e->hash = h;
    e->cap = 4;
    e->ids = malloc(e->cap * sizeof(uint32_t));
    e->ids[0] = id1;
    e->n = 1;
    d->slot[s] = ++d->n;
}

/* Tokenize one file's bytes (mapper hot loop, main.c:102-118): emit(ctx,
 * clean word, letters) for every token that keeps a letter. */
typedef void (*or_emit_fn)(void *ctx, const char *w, uint32_t n, uint32_t id1);
static void or_tokens(const unsigned char *p, uint64_t len, uint32_t id1, or_emit_fn emit, void *ctx) {
    char clean[OR_MAX_WORD];
    uint64_t i = 0;
    while (i < len) {
        while (i < len && or_isspace(p[i])) i++;
        if (i >= len) break;
        /* token = maximal run of non-space bytes (NUL is not a delimiter) */
        uint32_t j = 0;
        int stopped = 0; /* cleaning loop ended: NUL seen or 299 letters (main.c:105) */
        while (i < len && !or_isspace(p[i])) {
            unsigned char c = p[i++];
            if (stopped) continue;
            if (c == 0) { stopped = 1; continue; }
            if (c >= 'A' && c <= 'Z') clean[j++] = (char)(c + 32);
            else if (c >= 'a' && c <= 'z') clean[j++] = (char)c;
            if (j >= OR_MAX_WORD - 1) stopped = 1;
        }
        if (j > 0) emit(ctx, clean, j, id1); /* main.c:113 */
    }
}

static void or_emit_dict(void *ctx, const char *w, uint32_t n, uint32_t id1) {
    or_dict *dicts = ctx;
    or_dict_add(&dicts[w[0] - 'a'], w, n, id1); /* bucket by first letter, main.c:114-116 */
}

static void or_map_bytes(or_dict dicts[OR_ALPHA], const unsigned char *p, uint64_t len, uint32_t id1) {
    or_tokens(p, len, id1, or_emit_dict, dicts);
}

static int or_cmp(const void *a, const void *b) {
    const or_entry *x = a, *y = b;
    if (x->n != y->n) return x->n > y->n ? -1 : 1; /* df descending, main.c:59-61 */
    return strcmp(x->word, y->word);                /* word ascending, main.c:63 */
}

static uint32_t or_digits(uint32_t v) {
    uint32_t d = 1;
    while (v >= 10) { v /= 10; d++; }
    return d;
}

/* Format one letter's entries (writer, main.c:227-234). Returns malloc'd text. */
static char *or_reduce_letter(or_dict *d, uint64_t *out_len) {
    if (d->n) qsort(d->e, d->n, sizeof(or_entry), or_cmp); /* (qsort of a null array is UB, even of 0 items: UBSan) */
    uint64_t total = 0;
    for (uint32_t i = 0; i < d->n; i++) {
        total += d->e[i].len + 4; /* ":[" "]\n" */
        for (uint32_t k = 0; k < d->e[i].n; k++) total += or_digits(d->e[i].ids[k]) + (k ? 1 : 0);
    }
    char *buf = malloc(total + 1);
    char *o = buf;
    for (uint32_t i = 0; i < d->n; i++) {
        or_entry *e = &d->e[i];
        memcpy(o, e->word, e->len); o += e->len;
        *o++ = ':'; *o++ = '[';
        for (uint32_t k = 0; k < e->n; k++) {
            if (k) *o++ = ' ';
            o += sprintf(o, "%u", e->ids[k]);
        }
        *o++ = ']'; *o++ = '\n';
    }
    *out_len = (uint64_t)(o - buf);
    return buf;
}

static void or_dict_free(or_dict *d) {
    for (uint32_t i = 0; i < d->n; i++) { free(d->e[i].word); free(d->e[i].ids); }
    free(d->e); free(d->slot);
    memset(d, 0, sizeof(*d));
}

/*
 * In-memory entry point (used by tests and bench.py's cpu_baseline):
 *   text      concatenated file bytes
 *   file_off  nfiles+1 offsets into text; file f = [file_off[f], file_off[f+1])
 *   file_id0  0-based file IDs (printed as id0+1); must be ascending
 *   out       receives a malloc'd buffer holding the 26 letter texts back to back
 *   letter_off receives 27 offsets into *out
 * Returns 0.  Free *out with ii_oracle_free.
 */
int ii_oracle_index(const unsigned char *text, const uint64_t *file_off, const uint32_t *file_id0,
                    uint32_t nfiles, char **out, uint64_t letter_off[OR_ALPHA + 1]) {
    for (uint32_t f = 1; f < nfiles; f++)
        if (file_id0[f] <= file_id0[f - 1]) return -1; /* IDs must ascend */
    or_dict dicts[OR_ALPHA];
    memset(dicts, 0, sizeof(dicts));
    for (uint32_t f = 0; f < nfiles; f++)
        or_map_bytes(dicts, text + file_off[f], file_off[f + 1] - file_off[f], file_id0[f] + 1);
    char *parts[OR_ALPHA];
    uint64_t lens[OR_ALPHA], total = 0;
    for (int l = 0; l < OR_ALPHA; l++) {
        parts[l] = or_reduce_letter(&dicts[l], &lens[l]);
        total += lens[l];
        or_dict_free(&dicts[l]);
    }
    char *buf = malloc(total + 1);
    uint64_t o = 0;
    for (int l = 0; l < OR_ALPHA; l++) {
        letter_off[l] = o;
        memcpy(buf + o, parts[l], lens[l]);
        o += lens[l];
        free(parts[l]);
    }
    letter_off[OR_ALPHA] = o;
    *out = buf;
    return 0;
}

void ii_oracle_free(void *p) { free(p); }

/*
 * Multithreaded form of ii_oracle_index (the CPU baseline of bench.py at full
 * size, and the generator of tests/golden/bench_hashes.json).  Same result,
 * same rules; the reference's two phases with `nthreads` workers each:
 *   map    (mapper(), main.c:85-124): thread k tokenizes a contiguous run of
 *          files (ascending IDs) into its own 26 per-letter dictionaries;
 *   reduce (reducer(), main.c:126-242): letters are taken from a shared
 *          counter; a letter's thread-local dictionaries are merged in thread
 *          order — thread k's IDs all exceed thread k-1's, so appending keeps
 *          every posting list ascending with no dedup across threads — then
 *          ordered and formatted as in or_reduce_letter.
 */
typedef struct {
    const unsigned char *text;
    const uint64_t *file_off;
    const uint32_t *file_id0;
    uint32_t f_lo, f_hi;
    or_dict dicts[OR_ALPHA];
} or_map_job;

static void *or_map_worker(void *p) {
    or_map_job *j = p;
    for (uint32_t f = j->f_lo; f < j->f_hi; f++)
        or_map_bytes(j->dicts, j->text + j->file_off[f], j->file_off[f + 1] - j->file_off[f], j->file_id0[f] + 1);
    return NULL;
}

/* Append src's postings of one word to dst (src's IDs all exceed dst's). */
static void or_dict_merge_entry(or_dict *d, or_entry *src) {
    if ((uint64_t)(d->n + 1) * 2 > d->mask + 1) or_dict_grow(d);
    uint64_t s = src->hash & d->mask;
    for (;;) {
        uint32_t x = d->slot[s];
        if (!x) break;
        or_entry *e = &d->e[x - 1];
        if (e->hash == src->hash && e->len == src->len && memcmp(e->word, src->word, src->len) == 0) {
            if (e->n + src->n > e->cap) {
                while (e->n + src->n > e->cap) e->cap *= 2;
                e->ids = realloc(e->ids, e->cap * sizeof(uint32_t));
                if (!e->ids) { fprintf(stderr, "oracle: out of memory\n"); exit(EXIT_FAILURE); }
            }
            memcpy(e->ids + e->n, src->ids, src->n * sizeof(uint32_t));
            e->n += src->n;
            free(src->ids);
            free(src->word);
            return;
        }
        s = (s + 1) & d->mask;
    }
    if (d->n == d->cap) {
        d->cap = d->cap ? d->cap * 2 : 1024;
        d->e = realloc(d->e, d->cap * sizeof(or_entry));
        if (!d->e) { fprintf(stderr, "oracle: out of memory\n"); exit(EXIT_FAILURE); }
    }
    d->e[d->n] = *src; /* takes ownership of word and ids */
    d->slot[s] = ++d->n;
}

typedef struct {
    or_map_job *maps;
    int nmaps;
    char *parts[OR_ALPHA];
    uint64_t lens[OR_ALPHA];
    int next;
    pthread_mutex_t mu;
} or_reduce_job;

static void *or_reduce_worker(void *p) {
    or_reduce_job *j = p;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        int l = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (l >= OR_ALPHA) break;
        or_dict acc;
        memset(&acc, 0, sizeof(acc));
        for (int k = 0; k < j->nmaps; k++) {
            or_dict *src = &j->maps[k].dicts[l];
            for (uint32_t i = 0; i < src->n; i++) or_dict_merge_entry(&acc, &src->e[i]);
            free(src->e);
            free(src->slot);
            memset(src, 0, sizeof(*src));
        }
        j->parts[l] = or_reduce_letter(&acc, &j->lens[l]);
        or_dict_free(&acc);
    }
    return NULL;
}

int ii_oracle_index_mt(const unsigned char *text, const uint64_t *file_off, const uint32_t *file_id0,
                       uint32_t nfiles, int nthreads, char **out, uint64_t letter_off[OR_ALPHA + 1]) {
    for (uint32_t f = 1; f < nfiles; f++)
        if (file_id0[f] <= file_id0[f - 1]) return -1; /* IDs must ascend */
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    /* contiguous file runs of about equal bytes */
    or_map_job *maps = calloc((size_t)nthreads, sizeof(or_map_job));
    const uint64_t total = nfiles ? file_off[nfiles] - file_off[0] : 0;
    uint32_t f = 0;
    for (int k = 0; k < nthreads; k++) {
        maps[k].text = text;
        maps[k].file_off = file_off;
        maps[k].file_id0 = file_id0;
        maps[k].f_lo = f;
        const uint64_t goal = nfiles ? file_off[0] + total * (uint64_t)(k + 1) / (uint64_t)nthreads : 0;
        while (f < nfiles && (k == nthreads - 1 || file_off[f + 1] <= goal)) f++;
        maps[k].f_hi = f;
    }
    pthread_t th[256];
    for (int k = 0; k < nthreads; k++) pthread_create(&th[k], NULL, or_map_worker, &maps[k]);
    for (int k = 0; k < nthreads; k++) pthread_join(th[k], NULL);
    or_reduce_job rj;
    memset(&rj, 0, sizeof(rj));
    rj.maps = maps;
    rj.nmaps = nthreads;
    pthread_mutex_init(&rj.mu, NULL);
    const int nr = nthreads < OR_ALPHA ? nthreads : OR_ALPHA;
    for (int k = 0; k < nr; k++) pthread_create(&th[k], NULL, or_reduce_worker, &rj);
    for (int k = 0; k < nr; k++) pthread_join(th[k], NULL);
    pthread_mutex_destroy(&rj.mu);
    free(maps);
    uint64_t sum = 0;
    for (int l = 0; l < OR_ALPHA; l++) sum += rj.lens[l];
    char *buf = malloc(sum + 1);
    uint64_t o = 0;
    for (int l = 0; l < OR_ALPHA; l++) {
        letter_off[l] = o;
        memcpy(buf + o, rj.parts[l], rj.lens[l]);
        o += rj.lens[l];
        free(rj.parts[l]);
    }
    letter_off[OR_ALPHA] = o;
    *out = buf;
    return 0;
}

/* Partial files (main.c:113-118, format "%s %d\n" at main.c:116): one growing
 * buffer per letter. */
typedef struct { char *b; uint64_t n, cap; } or_buf;
static void or_emit_partial(void *ctx, const char *w, uint32_t n, uint32_t id1) {
    or_buf *pb = &((or_buf *)ctx)[w[0] - 'a'];
    if (pb->n + n + 16 > pb->cap) {
        pb->cap = (pb->cap + n + 16) * 2;
        pb->b = realloc(pb->b, pb->cap);
    }
    memcpy(pb->b + pb->n, w, n);
    pb->n += n;
    pb->n += (uint64_t)sprintf(pb->b + pb->n, " %u\n", id1);
}

/*
 * Text of the 26 partial_<letter>.txt files when one mapper reads the files
 * order[0..norder) one after another (main.c:93-124): lines in token order.
 * Same buffer convention as ii_oracle_index.
 */
int ii_oracle_partials(const unsigned char *text, const uint64_t *file_off, const uint32_t *file_id0,
                       uint32_t nfiles, const uint32_t *order, uint32_t norder, char **out,
                       uint64_t letter_off[OR_ALPHA + 1]) {
    or_buf bufs[OR_ALPHA];
    memset(bufs, 0, sizeof(bufs));
    for (uint32_t i = 0; i < norder; i++) {
        uint32_t f = order[i];
        if (f >= nfiles) return -1;
        or_tokens(text + file_off[f], file_off[f + 1] - file_off[f], file_id0[f] + 1, or_emit_partial, bufs);
    }
    uint64_t total = 0;
    for (int l = 0; l < OR_ALPHA; l++) total += bufs[l].n;
    char *buf = malloc(total + 1);
    uint64_t o = 0;
    for (int l = 0; l < OR_ALPHA; l++) {
        letter_off[l] = o;
        if (bufs[l].n) memcpy(buf + o, bufs[l].b, bufs[l].n);
        o += bufs[l].n;
        free(bufs[l].b);
    }
    letter_off[OR_ALPHA] = o;
    *out = buf;
    return 0;
}

/*
 * Streaming, letter-range form (the oracle of BASELINE configs[4] at its full
 * 100 GB / 10^6 files, which no single in-memory call holds): the same map and
 * reduce rules, over batches of files given in ascending id order, keeping
 * only words whose first letter lies in [lo, hi) (main.c:114-116 buckets by
 * it; a reducer owns a letter range, main.c:129-130).  Every batch's files are
 * mapped by nthreads workers into private dictionaries (contiguous file runs,
 * as ii_oracle_index_mt) and merged, letter by letter, into the stream's
 * dictionaries — a batch's ids all exceed the earlier batches', so appending
 * keeps every posting list ascending.  ii_oracle_stream_letter then orders and
 * formats one letter (or_reduce_letter) and releases its dictionary.
 */
typedef struct {
    or_dict dicts[OR_ALPHA];
    int lo, hi;
    uint32_t last_id1; /* largest id + 1 added so far */
} or_stream;

typedef struct {
    const unsigned char *text;
    const uint64_t *file_off;
    const uint32_t *file_id0;
    uint32_t f_lo, f_hi;
    int lo, hi;
    or_dict dicts[OR_ALPHA];
} or_stream_job;

static void or_emit_range(void *ctx, const char *w, uint32_t n, uint32_t id1) {
    or_stream_job *j = ctx;
    const int l = w[0] - 'a';
    if (l >= j->lo && l < j->hi) or_dict_add(&j->dicts[l], w, n, id1);
}

static void *or_stream_map_worker(void *p) {
    or_stream_job *j = p;
    for (uint32_t f = j->f_lo; f < j->f_hi; f++)
        or_tokens(j->text + j->file_off[f], j->file_off[f + 1] - j->file_off[f], j->file_id0[f] + 1, or_emit_range, j);
    return NULL;
}

typedef struct {
    or_stream *st;
    or_stream_job *jobs;
    int njobs, next;
    pthread_mutex_t mu;
} or_stream_merge;

static void *or_stream_merge_worker(void *p) {
    or_stream_merge *m = p;
    for (;;) {
        pthread_mutex_lock(&m->mu);
        const int l = m->st->lo + m->next++;
        pthread_mutex_unlock(&m->mu);
        if (l >= m->st->hi) break;
        for (int k = 0; k < m->njobs; k++) {
            or_dict *src = &m->jobs[k].dicts[l];
            for (uint32_t i = 0; i < src->n; i++) or_dict_merge_entry(&m->st->dicts[l], &src->e[i]);
            free(src->e);
            free(src->slot);
            memset(src, 0, sizeof(*src));
        }
    }
    return NULL;
}

void *ii_oracle_stream_open(int lo, int hi) {
    if (lo < 0 || hi > OR_ALPHA || lo > hi) return NULL;
    or_stream *st = calloc(1, sizeof(or_stream));
    if (st) { st->lo = lo; st->hi = hi; }
    return st;
}

/* Add a batch: file f = text[file_off[f] .. file_off[f+1]) with id file_id0[f],
 * ids ascending and above every id added before.  Returns 0, or -1. */
int ii_oracle_stream_add(void *h, const unsigned char *text, const uint64_t *file_off, const uint32_t *file_id0,
                         uint32_t nfiles, int nthreads) {
    or_stream *st = h;
    if (!st) return -1;
    for (uint32_t f = 0; f < nfiles; f++) {
        if (file_id0[f] + 1 <= st->last_id1) return -1; /* IDs must ascend across batches */
        st->last_id1 = file_id0[f] + 1;
    }
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    or_stream_job *jobs = calloc((size_t)nthreads, sizeof(or_stream_job));
    if (!jobs) return -1;
    const uint64_t total = nfiles ? file_off[nfiles] - file_off[0] : 0;
    uint32_t f = 0;
    for (int k = 0; k < nthreads; k++) {
        jobs[k].text = text;
        jobs[k].file_off = file_off;
        jobs[k].file_id0 = file_id0;
        jobs[k].lo = st->lo;
        jobs[k].hi = st->hi;
        jobs[k].f_lo = f;
        const uint64_t goal = nfiles ? file_off[0] + total * (uint64_t)(k + 1) / (uint64_t)nthreads : 0;
        while (f < nfiles && (k == nthreads - 1 || file_off[f + 1] <= goal)) f++;
        jobs[k].f_hi = f;
    }
    pthread_t th[256];
    for (int k = 0; k < nthreads; k++) pthread_create(&th[k], NULL, or_stream_map_worker, &jobs[k]);
    for (int k = 0; k < nthreads; k++) pthread_join(th[k], NULL);
    or_stream_merge m;
    memset(&m, 0, sizeof(m));
    m.st = st;
    m.jobs = jobs;
    m.njobs = nthreads;
    pthread_mutex_init(&m.mu, NULL);
    const int nm = nthreads < st->hi - st->lo ? nthreads : st->hi - st->lo;
    for (int k = 0; k < nm; k++) pthread_create(&th[k], NULL, or_stream_merge_worker, &m);
    for (int k = 0; k < nm; k++) pthread_join(th[k], NULL);
    pthread_mutex_destroy(&m.mu);
    free(jobs);
    return 0;
}

/* Order and format letter l (lo <= l < hi): *out (free with ii_oracle_free),
 * *len bytes, *words lines; the letter's dictionary is released. */
int ii_oracle_stream_letter(void *h, int l, char **out, uint64_t *len, uint64_t *words) {
    or_stream *st = h;
    if (!st || l < st->lo || l >= st->hi) return -1;
    *words = st->dicts[l].n;
    *out = or_reduce_letter(&st->dicts[l], len);
    or_dict_free(&st->dicts[l]);
    return 0;
}

void ii_oracle_stream_close(void *h) {
    or_stream *st = h;
    if (!st) return;
    for (int l = 0; l < OR_ALPHA; l++) or_dict_free(&st->dicts[l]);
    free(st);
}

#ifdef II_ORACLE_MAIN
/* Same CLI as the reference: <num_mappers> <num_reducers> <input_file_list>
 * (main.c:246-260); outputs a.txt..z.txt in the CWD. */
static unsigned char *or_read_file(const char *path, uint64_t *len) {
    FILE *f = fopen(path, "rb");
    if (!f) return NULL;
    uint64_t cap = 1 << 16, n = 0;
    unsigned char *b = malloc(cap);
    size_t r;
    while ((r = fread(b + n, 1, cap - n, f)) > 0) {
        n += r;
        if (n == cap) { cap *= 2; b = realloc(b, cap); }
    }
    fclose(f);
    *len = n;
    return b;
}

int main(int argc, char **argv) {
    if (argc < 4) {
        fprintf(stderr, "Usage: %s <num_mappers> <num_reducers> <input_file_list>\n", argv[0]);
        return -1;
    }
    int num_reducers = atoi(argv[2]);
    FILE *fl = fopen(argv[3], "r");
    if (!fl) { fprintf(stderr, "Error opening input file list: %s\n", argv[3]); return -1; }
    int count;
    if (fscanf(fl, "%d", &count) != 1) {
        fprintf(stderr, "Error reading the number of files from input file list\n");
        fclose(fl);
        return -1;
    }
    if (count < 0) count = 0;
    char **names = calloc((size_t)count + 1, sizeof(char *));
    for (int i = 0; i < count; i++) {
        names[i] = malloc(4096);
        if (fscanf(fl, "%4095s", names[i]) != 1) {
            fprintf(stderr, "Error reading file name from input file list\n");
            fclose(fl);
            for (int k = 0; k <= i; k++) free(names[k]);
            free(names);
            return -1;
        }
    }
    fclose(fl);
    unsigned char *text = NULL;
    uint64_t tlen = 0, tcap = 0;
    uint64_t *off = malloc(((size_t)count + 1) * sizeof(uint64_t));
    uint32_t *ids = malloc(((size_t)count + 1) * sizeof(uint32_t));
    for (int i = 0; i < count; i++) {
        struct stat st;
        if (stat(names[i], &st) != 0) fprintf(stderr, "Error getting size of file: %s\n", names[i]);
        off[i] = tlen;
        ids[i] = (uint32_t)i;
        uint64_t n = 0;
        unsigned char *b = or_read_file(names[i], &n);
        if (!b) { fprintf(stderr, "Mapper %d: Error opening file %s\n", 0, names[i]); continue; }
        if (tlen + n > tcap) { tcap = (tlen + n) * 2 + 1024; text = realloc(text, tcap); }
        memcpy(text + tlen, b, n);
        tlen += n;
        free(b);
    }
    off[count] = tlen;
    char *out;
    uint64_t loff[OR_ALPHA + 1];
    ii_oracle_index(text ? text : (unsigned char *)"", off, ids, (uint32_t)count, &out, loff);
    int rc = 0;
    if (num_reducers > 0) {
        for (int l = 0; l < OR_ALPHA && rc == 0; l++) {
            char fn[16];
            snprintf(fn, sizeof(fn), "%c.txt", 'a' + l);
            FILE *o = fopen(fn, "w");
            if (!o) { fprintf(stderr, "Error creating output file: %s\n", fn); rc = -1; break; }
            fwrite(out + loff[l], 1, loff[l + 1] - loff[l], o);
            fclose(o);
        }
    }
    ii_oracle_free(out);
    for (int i = 0; i < count; i++) free(names[i]);
    free(names);
    free(text);
    free(off);
    free(ids);
    return rc;
}
#endif
