/*
 * ii_check.c — property checker of one formatted letter file <letter>.txt.
 *
 * TEST INFRASTRUCTURE ONLY (like ii_oracle.c: never linked into or called by
 * the product).  Where no oracle output exists for a corpus — BASELINE
 * configs[4] at its full 100 GB / 10^6 files — the GPU index is checked by the
 * properties the reference's writer guarantees for every input
 * (/root/reference/main.c):
 *   - every line is  word ":[" id (" " id)* "]\n"  (main.c:227-234), the word
 *     1..299 letters a-z (main.c:105-111) starting with the file's letter
 *     (main.c:114-116), each id a decimal without leading zeros in [1, id_max]
 *     (1-based file ids, main.c:116, 275);
 *   - ids strictly ascending inside a line (distinct ids, main.c:176-184,
 *     sorted at main.c:217-226);
 *   - lines ordered by (df desc, strcmp asc), strictly (words are distinct,
 *     main.c:55-64, 215).
 * The text is split into nthreads pieces at line starts; each thread checks
 * its lines and the order against the line before its first one.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define CK_MAX_WORD 299

typedef struct {
    const char *t;
    uint64_t len, a, b; /* lines starting in [a, b) */
    int letter;
    uint64_t id_max;
    uint64_t lines, sum_df, max_df;
    uint64_t bad_at; /* first violation (offset), or UINT64_MAX */
    int bad;         /* its kind (negative), 0 = none */
} ck_job;

/* Parse the line at p; returns its end (one past '\n') or 0 with *err set.
 * *w / *wl: the word, *df: its id count. */
static uint64_t ck_line(const ck_job *j, uint64_t p, uint64_t *wl, uint64_t *df, int *err) {
    const char *t = j->t;
    const uint64_t n = j->len;
    uint64_t q = p;
    while (q < n && t[q] >= 'a' && t[q] <= 'z') q++;
    *wl = q - p;
    if (*wl == 0 || *wl > CK_MAX_WORD) { *err = -1; return 0; }           /* word: 1..299 letters */
    if (t[p] != 'a' + j->letter) { *err = -2; return 0; }                   /* first letter = file's */
    if (q + 2 > n || t[q] != ':' || t[q + 1] != '[') { *err = -3; return 0; }
    q += 2;
    uint64_t prev = 0, cnt = 0;
    for (;;) {
        if (q >= n || t[q] < '1' || t[q] > '9') { *err = -4; return 0; }     /* id: no leading zero */
        uint64_t v = 0;
        int nd = 0;
        while (q < n && t[q] >= '0' && t[q] <= '9') {
            if (++nd > 19) { *err = -4; return 0; }
            v = v * 10 + (uint64_t)(t[q++] - '0');
        }
        if (v > j->id_max) { *err = -5; return 0; }                          /* id in [1, id_max] */
        if (cnt && v <= prev) { *err = -6; return 0; }                       /* ascending, distinct */
        prev = v;
        cnt++;
        if (q < n && t[q] == ' ') { q++; continue; }
        if (q + 2 <= n && t[q] == ']' && t[q + 1] == '\n') { q += 2; break; }
        *err = -3;
        return 0;
    }
    *df = cnt;
    return q;
}

/* order of consecutive lines (word a, df da) then (word b, df db): df desc, then strcmp asc */
static int ck_before(const char *a, uint64_t al, uint64_t da, const char *b, uint64_t bl, uint64_t db) {
    if (da != db) return da > db;
    const uint64_t m = al < bl ? al : bl;
    const int c = memcmp(a, b, m);
    return c < 0 || (c == 0 && al < bl);
}

static void *ck_worker(void *arg) {
    ck_job *j = arg;
    j->bad_at = UINT64_MAX;
    uint64_t pw = 0, pwl = 0, pdf = 0;
    int have_prev = 0;
    if (j->a > 0) { /* the line before this piece's first one */
        uint64_t s = j->a - 1;
        while (s > 0 && j->t[s - 1] != '\n') s--;
        int err = 0;
        if (ck_line(j, s, &pwl, &pdf, &err)) { pw = s; have_prev = 1; }
    }
    for (uint64_t p = j->a; p < j->b;) {
        uint64_t wl, df;
        int err = 0;
        const uint64_t e = ck_line(j, p, &wl, &df, &err);
        if (!e) { j->bad = err; j->bad_at = p; return NULL; }
        if (have_prev && !ck_before(j->t + pw, pwl, pdf, j->t + p, wl, df)) { j->bad = -7; j->bad_at = p; return NULL; }
        j->lines++;
        j->sum_df += df;
        if (df > j->max_df) j->max_df = df;
        pw = p; pwl = wl; pdf = df; have_prev = 1;
        p = e;
    }
    return NULL;
}

/*
 * Check text[0 .. len) as <'a' + letter>.txt.  out[0] = lines, out[1] = sum of
 * df (= distinct (word, file) pairs), out[2] = largest df, out[3] = offset of
 * the first violation (or UINT64_MAX).  Returns 0, or the violation's kind:
 * -1 word length, -2 first letter, -3 line syntax, -4 id syntax, -5 id out of
 * range, -6 ids not strictly ascending, -7 lines out of order, -8 text does
 * not end with a line end, -9 bad argument.
 */
int ii_check_letter(const char *text, uint64_t len, int letter, uint64_t id_max, int nthreads, uint64_t out[4]) {
    memset(out, 0, 4 * sizeof(uint64_t));
    out[3] = UINT64_MAX;
    if (letter < 0 || letter > 25 || (len && !text)) return -9;
    if (len == 0) return 0;
    if (text[len - 1] != '\n') { out[3] = len - 1; return -8; }
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 64) nthreads = 64;
    if ((uint64_t)nthreads > len / 4096 + 1) nthreads = (int)(len / 4096 + 1);
    ck_job jobs[64];
    uint64_t cut[65];
    cut[0] = 0;
    for (int k = 1; k < nthreads; k++) { /* piece k starts at the first line start at or after len * k / n */
        uint64_t s = len * (uint64_t)k / (uint64_t)nthreads;
        if (s < cut[k - 1]) s = cut[k - 1];
        while (s < len && s > 0 && text[s - 1] != '\n') s++;
        cut[k] = s;
    }
    cut[nthreads] = len;
    pthread_t th[64];
    for (int k = 0; k < nthreads; k++) {
        memset(&jobs[k], 0, sizeof(ck_job));
        jobs[k].t = text;
        jobs[k].len = len;
        jobs[k].a = cut[k];
        jobs[k].b = cut[k + 1];
        jobs[k].letter = letter;
        jobs[k].id_max = id_max;
        pthread_create(&th[k], NULL, ck_worker, &jobs[k]);
    }
    int rc = 0;
    for (int k = 0; k < nthreads; k++) {
        pthread_join(th[k], NULL);
        if (jobs[k].bad && !rc) { rc = jobs[k].bad; out[3] = jobs[k].bad_at; }
        out[0] += jobs[k].lines;
        out[1] += jobs[k].sum_df;
        if (jobs[k].max_df > out[2]) out[2] = jobs[k].max_df;
    }
    return rc;
}
