/*
 * iigen.c — seeded synthetic Zipf corpus generator.
 *
 * Produces the benchmark corpora of BASELINE.json configs 3-5: N files whose
 * sizes are lognormal (sigma = 1) scaled to an exact byte total, filled with
 * English-like tokens drawn from a vocabulary with a Zipf (s ~= 1) rank
 * distribution.  Output is a single buffer of concatenated files plus the
 * N+1 file offsets — the same layout the device pipeline consumes.
 *
 * Vocabulary word r (r = 0 is the most frequent):
 *   length 1 + Poisson(5) clipped to 1..24; 0.1 % of words 25..64 letters;
 *   letters drawn with English letter frequencies.
 * Token decorations: 10 % capitalised, 5 % trailing .,;:!?, 2 % apostrophe,
 * 1 % digit-only tokens, 0.5 % a 2-byte UTF-8 letter inside the word.
 * Separators: ' ', '\n' about every 12 tokens, occasional '\t' and "\r\n".
 * Raw tokens stay <= 70 bytes (well under the reference's 299-byte limit).
 *
 * Determinism: every file is generated from its own splitmix64 stream
 * (seed, file index), so output does not depend on the thread count.
 * Rank sampling uses the continuous inverse CDF of 1/x, r = (V+1)^u - 1
 * (a Zipf s = 1 approximation).
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct {
    uint64_t total_bytes; /* exact corpus size */
    uint32_t nfiles;
    uint32_t vocab;       /* vocabulary size V */
    uint64_t seed;
    double size_sigma;    /* lognormal sigma of file sizes (1.0) */
} iigen_params;

static inline uint64_t sm64(uint64_t *s) {
    uint64_t z = (*s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
static inline double u01(uint64_t *s) { return (double)(sm64(s) >> 11) * (1.0 / 9007199254740992.0); }
/* uniform integer in [0, n) */
static inline uint32_t below(uint64_t *s, uint32_t n) { return (uint32_t)(((sm64(s) >> 32) * (uint64_t)n) >> 32); }

/* English letter frequencies, per 100000 */
static const uint32_t kFreq[26] = {8167, 1492, 2782, 4253, 12702, 2228, 2015, 6094, 6966, 153, 772, 4025, 2406,
                                   6749, 7507, 1929, 95, 5987, 6327, 9056, 2758, 978, 2360, 150, 1974, 74};

typedef struct {
    const iigen_params *p;
    char *words;       /* vocabulary text */
    uint64_t *woff;    /* V+1 offsets */
    uint32_t cdf[26];
    uint32_t cdf_total;
    double logv;
    const uint64_t *file_off;
    uint8_t *out;
    const uint32_t *sel;     /* iigen_fill_files: the files to make (NULL = all) */
    const uint64_t *sel_off; /* their places in out */
    uint32_t nwork;          /* files to make */
    uint32_t next_file;
    pthread_mutex_t mu;
} gen_ctx;

static char pick_letter(const gen_ctx *g, uint64_t *s) {
    uint32_t x = below(s, g->cdf_total);
    int l = 0;
    while (l < 25 && x >= g->cdf[l]) l++;
    return (char)('a' + l);
}

static uint32_t poisson5(uint64_t *s) {
    /* inverse transform, lambda = 5 */
    double u = u01(s), p = exp(-5.0), c = p;
    uint32_t k = 0;
    while (u > c && k < 40) { k++; p *= 5.0 / k; c += p; }
    return k;
}

static int build_vocab(gen_ctx *g) {
    uint32_t V = g->p->vocab;
    g->woff = malloc(((size_t)V + 1) * sizeof(uint64_t));
    uint32_t *len = malloc((size_t)V * sizeof(uint32_t));
    if (!g->woff || !len) return -1;
    uint64_t tot = 0;
    for (uint32_t r = 0; r < V; r++) {
        uint64_t s = g->p->seed * 0x632be59bd9b4e019ull ^ ((uint64_t)r * 0x9e3779b97f4a7c15ull) ^ 0x5bd1e995ull;
        uint32_t L;
        if (below(&s, 1000) == 0) L = 25 + below(&s, 40);
        else { L = 1 + poisson5(&s); if (L > 24) L = 24; }
        len[r] = L;
        g->woff[r] = tot;
        tot += L;
    }
    g->woff[V] = tot;
    g->words = malloc(tot + 1);
    if (!g->words) return -1;
    for (uint32_t r = 0; r < V; r++) {
        uint64_t s = g->p->seed * 0x2545f4914f6cdd1dull ^ ((uint64_t)r * 0xd6e8feb86659fd93ull) ^ 0x27d4eb2full;
        for (uint32_t i = 0; i < len[r]; i++) g->words[g->woff[r] + i] = pick_letter(g, &s);
    }
    free(len);
    return 0;
}

/* Fill one file of exactly n bytes. */
static void gen_file(const gen_ctx *g, uint32_t f, uint8_t *o, uint64_t n) {
    uint64_t s = g->p->seed ^ ((uint64_t)(f + 1) * 0xa0761d6478bd642full);
    sm64(&s);
    uint64_t i = 0;
    uint32_t since_nl = 0, nl_at = 8 + below(&s, 9);
    char tok[96];
    while (i < n) {
        uint32_t tl = 0;
        uint32_t kind = below(&s, 1000);
        if (kind < 10) { /* 1 %: digit-only token */
            uint32_t nd = 1 + below(&s, 4);
            for (uint32_t k = 0; k < nd; k++) tok[tl++] = (char)('0' + below(&s, 10));
        } else {
            double u = u01(&s);
            uint32_t r = (uint32_t)(exp(u * g->logv) - 1.0);
            if (r >= g->p->vocab) r = g->p->vocab - 1;
            uint32_t L = (uint32_t)(g->woff[r + 1] - g->woff[r]);
            memcpy(tok, g->words + g->woff[r], L);
            tl = L;
            if (below(&s, 100) < 10) tok[0] = (char)(tok[0] - 32);           /* capitalised */
            if (below(&s, 1000) < 5 && tl >= 2) {                             /* 2-byte UTF-8 */
                uint32_t at = 1 + below(&s, tl - 1);
                memmove(tok + at + 2, tok + at, tl - at);
                tok[at] = (char)0xC3; tok[at + 1] = (char)(0xA0 + below(&s, 0x1F));
                tl += 2;
            }
            if (below(&s, 100) < 2 && tl >= 2) {                              /* apostrophe */
                uint32_t at = 1 + below(&s, tl - 1);
                memmove(tok + at + 1, tok + at, tl - at);
                tok[at] = '\'';
                tl += 1;
            }
            if (below(&s, 100) < 5) tok[tl++] = ".,;:!?"[below(&s, 6)];        /* trailing punct */
        }
        /* separator */
        char sep[2];
        uint32_t sl = 1;
        sep[0] = ' ';
        if (++since_nl >= nl_at) {
            since_nl = 0;
            nl_at = 8 + below(&s, 9);
            if (below(&s, 50) == 0) { sep[0] = '\r'; sep[1] = '\n'; sl = 2; }
            else sep[0] = '\n';
        } else if (below(&s, 200) == 0) sep[0] = '\t';
        if (i + tl + sl > n) { /* pad the tail of the file with spaces / newline */
            while (i < n) { o[i] = (i + 1 == n) ? '\n' : ' '; i++; }
            break;
        }
        memcpy(o + i, tok, tl); i += tl;
        memcpy(o + i, sep, sl); i += sl;
    }
}

static void *worker(void *arg) {
    gen_ctx *g = arg;
    for (;;) {
        pthread_mutex_lock(&g->mu);
        uint32_t k = g->next_file;
        if (k < g->nwork) g->next_file++;
        pthread_mutex_unlock(&g->mu);
        if (k >= g->nwork) break;
        const uint32_t f = g->sel ? g->sel[k] : k;
        gen_file(g, f, g->out + (g->sel ? g->sel_off[k] : g->file_off[f]), g->file_off[f + 1] - g->file_off[f]);
    }
    return NULL;
}

/* File sizes: lognormal(sigma) weights scaled to total_bytes exactly. */
int iigen_layout(const iigen_params *p, uint64_t *file_off) {
    if (!p || !file_off || p->nfiles == 0) return -1;
    double *w = malloc(sizeof(double) * p->nfiles);
    if (!w) return -1;
    uint64_t s = p->seed ^ 0x8ebc6af09c88c6e3ull;
    double sum = 0;
    for (uint32_t f = 0; f < p->nfiles; f++) {
        double u1 = u01(&s), u2 = u01(&s);
        if (u1 < 1e-300) u1 = 1e-300;
        double z = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
        w[f] = exp(p->size_sigma * z);
        sum += w[f];
    }
    uint64_t acc = 0;
    double cum = 0;
    file_off[0] = 0;
    for (uint32_t f = 0; f < p->nfiles; f++) {
        cum += w[f];
        uint64_t end = (f + 1 == p->nfiles) ? p->total_bytes : (uint64_t)((cum / sum) * (double)p->total_bytes);
        if (end < acc) end = acc;
        if (end > p->total_bytes) end = p->total_bytes;
        file_off[f + 1] = end;
        acc = end;
    }
    free(w);
    return 0;
}

static int fill_core(const iigen_params *p, const uint64_t *file_off, const uint32_t *sel, const uint64_t *sel_off,
                     uint32_t nsel, uint8_t *out, int nthreads) {
    if (!p || !file_off || !out || p->vocab == 0) return -1;
    gen_ctx g;
    memset(&g, 0, sizeof(g));
    g.p = p;
    g.sel = sel;
    g.sel_off = sel_off;
    g.nwork = sel ? nsel : p->nfiles;
    uint32_t acc = 0;
    for (int l = 0; l < 26; l++) { acc += kFreq[l]; g.cdf[l] = acc; }
    g.cdf_total = acc;
    g.logv = log((double)p->vocab + 1.0);
    g.file_off = file_off;
    g.out = out;
    pthread_mutex_init(&g.mu, NULL);
    if (build_vocab(&g)) return -1;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, worker, &g);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    pthread_mutex_destroy(&g.mu);
    free(g.words);
    free(g.woff);
    return 0;
}

int iigen_fill(const iigen_params *p, const uint64_t *file_off, uint8_t *out, int nthreads) {
    return fill_core(p, file_off, NULL, NULL, 0, out, nthreads);
}

/* A subset of the corpus (a GPU's shard): files sel[0..nsel) (any order; each
 * file's bytes are exactly those iigen_fill gives it, since every file has its
 * own random stream) back to back in out, file sel[k] at out_off[k]
 * (out_off[0] = 0, out_off[k + 1] = out_off[k] + its size; nsel + 1 entries
 * written). */
int iigen_fill_files(const iigen_params *p, const uint64_t *file_off, const uint32_t *sel, uint32_t nsel,
                     uint64_t *out_off, uint8_t *out, int nthreads) {
    if (!p || !file_off || (nsel && !sel) || !out_off) return -1;
    out_off[0] = 0;
    for (uint32_t k = 0; k < nsel; k++) {
        if (sel[k] >= p->nfiles) return -1;
        out_off[k + 1] = out_off[k] + (file_off[sel[k] + 1] - file_off[sel[k]]);
    }
    if (nsel == 0) return 0;
    return fill_core(p, file_off, sel, out_off, nsel, out, nthreads);
}

#ifdef IIGEN_MAIN
/* iigen <outdir> <total_bytes> <nfiles> <vocab> <seed> [threads]
 * writes <outdir>/f<i>.txt and <outdir>/list.txt (reference list format). */
int main(int argc, char **argv) {
    if (argc < 6) {
        fprintf(stderr, "usage: %s <outdir> <total_bytes> <nfiles> <vocab> <seed> [threads]\n", argv[0]);
        return 2;
    }
    iigen_params p = {strtoull(argv[2], 0, 10), (uint32_t)atoi(argv[3]), (uint32_t)atoi(argv[4]),
                      strtoull(argv[5], 0, 10), 1.0};
    int th = argc > 6 ? atoi(argv[6]) : 8;
    uint64_t *off = malloc(sizeof(uint64_t) * (p.nfiles + 1));
    uint8_t *buf = malloc(p.total_bytes + 1);
    if (iigen_layout(&p, off) || iigen_fill(&p, off, buf, th)) return 1;
    char path[4096];
    snprintf(path, sizeof(path), "%s/list.txt", argv[1]);
    FILE *lf = fopen(path, "w");
    if (!lf) return 1;
    fprintf(lf, "%u\n", p.nfiles);
    for (uint32_t f = 0; f < p.nfiles; f++) {
        snprintf(path, sizeof(path), "%s/f%u.txt", argv[1], f);
        FILE *o = fopen(path, "wb");
        if (!o) return 1;
        fwrite(buf + off[f], 1, off[f + 1] - off[f], o);
        fclose(o);
        fprintf(lf, "%s\n", path);
    }
    fclose(lf);
    return 0;
}
#endif
