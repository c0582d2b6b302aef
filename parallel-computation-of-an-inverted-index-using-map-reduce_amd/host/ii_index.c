/*
 * ii_index.c — C host CLI, drop-in for the reference's `tema1`:
 *
 *     ii_index <num_mappers> <num_reducers> <input_file_list>
 *
 * Same argument handling, list format, file-ID numbering and outputs
 * (a.txt .. z.txt in the current directory) as /root/reference/main.c:246-390.
 * The map and reduce phases (main.c:326-384) run on MI355X GPUs through
 * libii.so (include/ii.h); M sizes the host reader threads and R the writer
 * threads, neither changes the output.
 *
 * GPUs: II_GPUS=G (a number, or "all" = every visible device; default 1).
 * With G > 1 the files are sharded over G contexts by the reference's own
 * size heuristic (ii_partition, main.c:300-323), one host pthread per context
 * maps and locally reduces its shard, the G contexts exchange letter ranges —
 * the reference's reducer map with R = G (main.c:129-130), or histogram-
 * balanced ranges with II_LETTER_SPLIT=balanced — and each
 * owner merges, orders and formats its letters.  The exchange moves the
 * export segments with ONE grouped RCCL ncclSend / ncclRecv round over xGMI
 * when the G contexts sit on G distinct devices; when fewer devices are
 * visible the contexts share them ("G logical shards") and the
 * segments move by device copies.  Output is identical for every G.
 * Test knob II_TEST_MULTI=1: G = 1 takes the multi-context path too — one
 * context that exports its segment, exchanges it with itself through a real
 * one-rank RCCL communicator (ncclCommInitRank + grouped ncclSend / ncclRecv to
 * self) and imports it: the RCCL branch runs on a one-GPU box.
 *
 * With II_PARTIAL_FILES=1 in the environment the CLI also leaves the
 * reference's partial_<letter>.txt files in the current directory
 * (main.c:332-341, lines "<word> <id>\n" written at main.c:116), mapper m's
 * files (size order, main.c:300-323) after mapper m-1's: byte-identical to
 * the reference's for M = 1.  Off by default: the index
 * does not need them.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include "ii.h"

#define MAXG II_MAX_PARTS

struct shard;
/* What every context of a multi-GPU run shares: the letter owners (lo/hi,
 * known before the map with the reference's split, after it with the
 * balanced one), the exchange mode and, over RCCL, the communicator's id. */
typedef struct {
    struct shard *sh;
    int G, distinct, ranges_known;
    int lo[MAXG], hi[MAXG];
    ncclUniqueId nccl_id;
} multi_run;

/* One GPU context of the multi-GPU CLI and its shard of files. */
typedef struct shard {
    int g, dev, nparts;
    ii_ctx *ctx;
    ii_file *files;   /* the shard's files, ascending id0 */
    uint32_t n;
    uint32_t *local;  /* list index -> index in this shard (UINT32_MAX: another shard) */
    int nthreads;
    int rc;
    multi_run *run;
    uint64_t load[II_ALPHABET];  /* balanced split: distinct pairs per first letter of this shard */
    /* exchange: segment bytes for every owner, send / receive offsets */
    uint64_t seg[MAXG], send_off[MAXG + 1], recv_off[MAXG + 1];
    void *d_send, *d_recv;
    uint32_t id_bound;
} shard;

/* ---- phases: one pthread per context, joined by run_phase.
 * A failed context ends the phase at once: run_phase returns its error
 * without waiting for the other contexts, because after a device fault their
 * threads may sit in HIP waits that never return (round 3: eight contexts on
 * one device, the first one's copy reported an illegal memory access, and the
 * CLI waited for the others until it was killed).  main() then prints the
 * error and leaves with _exit, making no further HIP call.
 * Test knob II_TEST_FAIL=<phase>:<g> (phase map or merge): context g returns
 * II_ERR_INTERNAL at the start of that phase and every other context of the
 * phase blocks for good, as behind a faulted device. */
typedef struct {
    pthread_mutex_t mu;
    pthread_cond_t cv;
    int done, err;
} phase_sync;

typedef struct {
    shard *s;
    int g, G;
    phase_sync *ps;
    void (*body)(shard *);
    const char *name;
} phase_arg;

/* the context II_TEST_FAIL names for this phase, or -1 (also for an index
 * outside 0 .. G-1: a stray value must not block the CLI) */
static int test_fail_ctx(const char *phase, int G) {
    const char *e = getenv("II_TEST_FAIL");
    size_t n = strlen(phase);
    if (!e || strncmp(e, phase, n) || e[n] != ':') return -1;
    char *end;
    const long g = strtol(e + n + 1, &end, 10);
    return end != e + n + 1 && *end == 0 && g >= 0 && g < G ? (int)g : -1;
}

static void *phase_thread(void *p) {
    phase_arg *a = p;
    const int fail = test_fail_ctx(a->name, a->G);
    if (fail == a->g) {
        a->s->rc = II_ERR_INTERNAL;
    } else if (fail >= 0) {
        for (;;) pause(); /* the simulated stuck context */
    } else {
        a->body(a->s);
    }
    pthread_mutex_lock(&a->ps->mu);
    a->ps->done++;
    if (a->s->rc != II_OK && a->ps->err == II_OK) a->ps->err = a->s->rc;
    pthread_cond_signal(&a->ps->cv);
    pthread_mutex_unlock(&a->ps->mu);
    return NULL;
}

/* Run body on every context; II_OK once all succeeded (threads joined), or the
 * first error as soon as it is reported (the other threads are left alone). */
static int run_phase(shard *sh, int G, void (*body)(shard *), const char *name) {
    /* static: threads left behind by a failed phase still hold them (main() then exits); a phase
     * starts only after the previous one joined all of its threads */
    static phase_sync ps = {PTHREAD_MUTEX_INITIALIZER, PTHREAD_COND_INITIALIZER, 0, 0};
    static phase_arg args[MAXG];
    pthread_t th[MAXG];
    ps.done = 0;
    ps.err = II_OK;
    int started = 0;
    for (int g = 0; g < G; g++) {
        args[g] = (phase_arg){&sh[g], g, G, &ps, body, name};
        if (pthread_create(&th[g], NULL, phase_thread, &args[g]) != 0) {
            sh[g].rc = II_ERR_NOMEM;
            break;
        }
        started++;
    }
    pthread_mutex_lock(&ps.mu);
    while (ps.done < started && ps.err == II_OK) pthread_cond_wait(&ps.cv, &ps.mu);
    int rc = ps.err;
    pthread_mutex_unlock(&ps.mu);
    if (rc == II_OK && started < G) rc = II_ERR_NOMEM;
    if (rc != II_OK) return rc; /* (threads still running are not joined) */
    for (int g = 0; g < started; g++) pthread_join(th[g], NULL);
    return II_OK;
}

/* Export of one context: its segment for every owner into a device buffer of
 * its own (ii_export waits for its copies: in this context's thread, so the G
 * exports overlap). */
static void export_body(shard *s) {
    const multi_run *m = s->run;
    s->rc = ii_export_plan_ranges(s->ctx, m->G, m->lo, m->hi, s->seg);
    if (s->rc != II_OK) return;
    s->send_off[0] = 0;
    for (int r = 0; r < m->G; r++) s->send_off[r + 1] = s->send_off[r] + s->seg[r];
    if (hipSetDevice(s->dev) != hipSuccess || hipMalloc(&s->d_send, s->send_off[m->G] + 8) != hipSuccess) {
        s->d_send = NULL;
        s->rc = II_ERR_NOMEM;
        return;
    }
    s->rc = ii_export(s->ctx, m->G, s->d_send, s->send_off);
}
/* Map phase of one context: map + local reduce of its shard, then — when the
 * letter owners are known up front (the reference's split) — its export; with
 * the balanced split, its per-letter load instead. */
static void map_body(shard *s) {
    s->rc = ii_open(&s->ctx, s->dev);
    if (s->rc == II_OK) s->rc = ii_map_files(s->ctx, s->files, s->n, s->nthreads, NULL);
    if (s->rc == II_OK) s->rc = ii_reduce_local(s->ctx); /* distinct (word, file) pairs of the shard */
    if (s->rc != II_OK) return;
    if (s->run->ranges_known) export_body(s);
    else s->rc = ii_letter_load(s->ctx, s->load);
}
/* Receive of owner g: segment g of every source into d_recv at recv_off[source].
 * Over RCCL (a device per context) every context runs its own rank of one
 * grouped ncclSend / ncclRecv round (point-to-point over xGMI: it sends its
 * segments and receives its own); with shared devices the owner copies its
 * segments from the sources' send buffers (device copies, all owners at once). */
static int receive(shard *s) {
    multi_run *m = s->run;
    shard *sh = m->sh;
    const int G = m->G, g = s->g;
    if (hipSetDevice(s->dev) != hipSuccess) return II_ERR_HIP;
    if (hipMalloc(&s->d_recv, s->recv_off[G] + 8) != hipSuccess) {
        s->d_recv = NULL;
        return II_ERR_NOMEM;
    }
    hipStream_t st;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return II_ERR_HIP;
    int bad = 0;
    if (m->distinct) {
        ncclComm_t comm;
        if (ncclCommInitRank(&comm, G, m->nccl_id, g) != ncclSuccess) {
            (void)hipStreamDestroy(st);
            return II_ERR_HIP;
        }
        bad |= ncclGroupStart() != ncclSuccess;
        for (int r = 0; r < G && !bad; r++) {
            if (s->seg[r]) /* my segment for owner r */
                bad |= ncclSend((const char *)s->d_send + s->send_off[r], s->seg[r], ncclUint8, r, comm, st) !=
                       ncclSuccess;
            if (sh[r].seg[g]) /* source r's segment for me */
                bad |= ncclRecv((char *)s->d_recv + s->recv_off[r], sh[r].seg[g], ncclUint8, r, comm, st) !=
                       ncclSuccess;
        }
        bad |= ncclGroupEnd() != ncclSuccess;
        bad |= hipStreamSynchronize(st) != hipSuccess;
        ncclCommDestroy(comm);
    } else {
        for (int r = 0; r < G && !bad; r++) {
            const uint64_t n = sh[r].seg[g];
            if (n)
                bad |= hipMemcpyPeerAsync((char *)s->d_recv + s->recv_off[r], s->dev,
                                          (const char *)sh[r].d_send + sh[r].send_off[g], sh[r].dev, n, st) !=
                       hipSuccess;
        }
        bad |= hipStreamSynchronize(st) != hipSuccess;
    }
    (void)hipStreamDestroy(st);
    return bad ? II_ERR_HIP : II_OK;
}
static void merge_body(shard *s) {
    s->rc = receive(s);
    if (s->rc == II_OK) s->rc = ii_import(s->ctx, s->nparts, s->d_recv, s->recv_off, s->id_bound);
    if (s->rc == II_OK) s->rc = ii_reduce(s->ctx, 1);
}

typedef struct {
    ii_ctx **owner;  /* context holding each letter's text */
    int r, R;
    int err;
} writer_arg;

/* Reducer r of R writes its letter range (main.c:129-130, 143-155). */
static void *writer(void *p) {
    writer_arg *w = p;
    int lo, hi;
    printf("REDUCER\n"); /* main.c:141 */
    if (ii_reducer_letters(w->r, w->R, &lo, &hi) != II_OK) return NULL;
    for (int l = lo; l < hi; l++) {
        const char *buf;
        size_t len;
        char name[16];
        snprintf(name, sizeof(name), "%c.txt", 'a' + l);
        if (ii_letter_text(w->owner[l], l, &buf, &len) != II_OK) { w->err = 1; continue; }
        FILE *o = fopen(name, "w");
        if (!o) { printf("eroare la fisierul final\n"); w->err = 1; continue; } /* main.c:151-154 */
        if (len && fwrite(buf, 1, len, o) != len) w->err = 1;
        fclose(o);
    }
    return NULL;
}

static int gpus_requested(void) {
    const char *e = getenv("II_GPUS");
    if (!e || !*e) return 1;
    if (!strcmp(e, "all")) {
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n < 1) return 1;
        return n > MAXG ? MAXG : n;
    }
    int g = atoi(e);
    return g < 1 ? 1 : g > MAXG ? MAXG : g;
}

/* Multi-context index (G > 1), first half: shard the files, then, one
 * pthread per context, map + local reduce every shard and (reference split)
 * export its segments.  The letter owners: the reference's reducer map with
 * R = G (main.c:129-130), or with II_LETTER_SPLIT=balanced ranges balanced on
 * the summed per-letter loads, known only after the maps. */
static int multi_map(const ii_file *files, const uint64_t *sizes, uint32_t count, int M, int G, shard *sh,
                     multi_run *run) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) {
        if (test_fail_ctx("map", G) < 0) return II_ERR_NODEV;
        ndev = 1; /* (the test knob's map phase opens no device: it runs without one) */
    }
    run->sh = sh;
    run->G = G;
    run->distinct = ndev >= G;
    const char *split = getenv("II_LETTER_SPLIT");
    run->ranges_known = !(split && !strcmp(split, "balanced"));
    if (run->ranges_known)
        for (int r = 0; r < G; r++) ii_reducer_letters(r, G, &run->lo[r], &run->hi[r]); /* main.c:129-130 */
    uint32_t *order = calloc((size_t)count + 1, sizeof(uint32_t));
    uint32_t *shard_of = calloc((size_t)count + 1, sizeof(uint32_t));
    uint32_t sb[MAXG], se[MAXG];
    ii_partition(sizes, count, G, order, sb, se); /* main.c:300-323 with M = G */
    for (int g = 0; g < G; g++)
        for (uint32_t j = sb[g]; j < se[g]; j++) shard_of[order[j]] = (uint32_t)g;
    for (int g = 0; g < G; g++) {
        sh[g].g = g;
        sh[g].run = run;
        sh[g].dev = g % ndev;
        sh[g].nparts = G;
        sh[g].n = 0;
        sh[g].files = calloc((size_t)(se[g] - sb[g]) + 1, sizeof(ii_file));
        sh[g].local = malloc(((size_t)count + 1) * sizeof(uint32_t));
        sh[g].nthreads = M / G > 0 ? M / G : 1;
        sh[g].id_bound = count;
    }
    /* every shard in ascending id0 = list order (ii_map_files requires it; postings come out ascending) */
    for (uint32_t i = 0; i < count; i++)
        for (int g = 0; g < G; g++) {
            if (shard_of[i] == (uint32_t)g) {
                sh[g].local[i] = sh[g].n;
                sh[g].files[sh[g].n++] = files[i];
            } else {
                sh[g].local[i] = UINT32_MAX;
            }
        }
    free(order);
    free(shard_of);
    return run_phase(sh, G, map_body, "map");
}

/* Second half: (balanced split) letter owners and the exports, then one
 * phase in which every context receives its segments (RCCL, or device copies
 * when contexts share devices), merges them, orders and formats its letters.
 * owner[l] receives the context holding letter l.  The exchange buffers are
 * freed by the caller (multi_exchange), on every return. */
static int multi_exchange_body(int G, shard *sh, multi_run *run, ii_ctx **owner) {
    int rc = II_OK;
    if (!run->ranges_known) {
        uint64_t load[II_ALPHABET] = {0};
        for (int g = 0; g < G; g++)
            for (int l = 0; l < II_ALPHABET; l++) load[l] += sh[g].load[l];
        if ((rc = ii_balanced_letters(load, G, run->lo, run->hi)) != II_OK) return rc;
        if ((rc = run_phase(sh, G, export_body, "export")) != II_OK) return rc;
    }
    for (int r = 0; r < G; r++)
        for (int l = run->lo[r]; l < run->hi[r]; l++) owner[l] = sh[r].ctx;
    for (int r = 0; r < G; r++) {
        sh[r].recv_off[0] = 0;
        for (int g = 0; g < G; g++) sh[r].recv_off[g + 1] = sh[r].recv_off[g] + sh[g].seg[r];
    }
    if (run->distinct && ncclGetUniqueId(&run->nccl_id) != ncclSuccess) return II_ERR_HIP;
    return run_phase(sh, G, merge_body, "merge");
}

static int multi_exchange(int G, shard *sh, multi_run *run, ii_ctx **owner) {
    const int rc = multi_exchange_body(G, sh, run, owner);
    if (rc != II_OK) return rc; /* (no HIP call after a failure: main() exits) */
    for (int g = 0; g < G; g++) {
        (void)hipSetDevice(sh[g].dev);
        if (sh[g].d_send) (void)hipFree(sh[g].d_send);
        if (sh[g].d_recv) (void)hipFree(sh[g].d_recv);
        sh[g].d_send = sh[g].d_recv = NULL;
    }
    return rc;
}

/* partial_<letter>.txt (main.c:332-341): emit[] lists the files in the
 * reference's emission order (mapper 0's, then mapper 1's, ...); with G
 * contexts every run of consecutive files held by one context is appended in
 * turn. */
static int write_partials(shard *sh, int G, ii_ctx *single, const uint32_t *emit, uint32_t n) {
    FILE *out[II_ALPHABET];
    for (int l = 0; l < II_ALPHABET; l++) {
        char name[32];
        snprintf(name, sizeof(name), "partial_%c.txt", 'a' + l);
        out[l] = fopen(name, "w+");
        if (!out[l]) {
            fprintf(stderr, "Error creating partial file: %s\n", name); /* main.c:336 */
            for (int k = 0; k < l; k++) fclose(out[k]);
            return II_ERR_IO;
        }
    }
    int rc = II_OK;
    uint32_t *run = malloc(((size_t)n + 1) * sizeof(uint32_t));
    for (uint32_t i = 0; i < n && rc == II_OK;) {
        ii_ctx *ctx = single;
        uint32_t k = 0, j = i;
        if (single) {
            for (; j < n; j++) run[k++] = emit[j];
        } else {
            int g = 0;
            while (sh[g].local[emit[i]] == UINT32_MAX) g++;
            ctx = sh[g].ctx;
            for (; j < n && sh[g].local[emit[j]] != UINT32_MAX; j++) run[k++] = sh[g].local[emit[j]];
        }
        i = j;
        rc = ii_partials(ctx, run, k);
        for (int l = 0; rc == II_OK && l < II_ALPHABET; l++) {
            const char *buf;
            size_t len;
            rc = ii_partial_text(ctx, l, &buf, &len);
            if (rc == II_OK && len && fwrite(buf, 1, len, out[l]) != len) rc = II_ERR_IO;
        }
    }
    free(run);
    for (int l = 0; l < II_ALPHABET; l++) fclose(out[l]);
    return rc;
}

/* Everything main() allocates, released on every return path (the ASan/UBSan
 * build of tests/test_sanitizers.py runs the list-parsing errors too). */
typedef struct {
    ii_file *files;
    uint64_t *sizes;
    char **names;
    int nnames;
    uint32_t *order, *sb, *se;
} cli_state;

static void cli_free(cli_state *c) {
    for (int i = 0; i < c->nnames; i++) free(c->names[i]);
    free(c->names);
    free(c->files);
    free(c->sizes);
    free(c->order);
    free(c->sb);
    free(c->se);
}

/* II_METRICS=path (or "-" for stderr): one JSON line per run — input, wall
 * time, counts and device phase times of the contexts that hold the output
 * (a per-run metrics record; the reference only prints). */
static double wall_ms(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}
static void write_metrics(const char *dest, double t0, int M, int R, int G, uint32_t nfiles, const uint64_t *sizes,
                          ii_ctx *single, shard *sh, int err) {
    uint64_t bytes = 0, pairs = 0, words = 0, out = 0, tokens = 0;
    double ms_map = 0, ms_reduce = 0;
    for (uint32_t i = 0; i < nfiles; i++) bytes += sizes[i];
    for (int g = 0; g < (single ? 1 : sh ? G : 0); g++) {
        ii_ctx *c = single ? single : sh[g].ctx;
        ii_stats st;
        if (!c || ii_get_stats(c, &st) != II_OK) continue;
        pairs += st.pairs; /* owners hold disjoint letters: their pairs, words and texts add up */
        words += st.words;
        out += st.out_bytes;
        if (single) {
            tokens = st.tokens;
            ms_map = st.ms_map;
            ms_reduce = st.ms_total - st.ms_map;
        }
    }
    const double wall = wall_ms() - t0;
    FILE *f = strcmp(dest, "-") ? fopen(dest, "a") : stderr;
    if (!f) return;
    fprintf(f,
            "{\"tool\": \"ii_index\", \"ok\": %s, \"mappers\": %d, \"reducers\": %d, \"gpus\": %d, \"files\": %u, "
            "\"bytes\": %llu, \"wall_ms\": %.3f, \"GBps_wall\": %.4f, \"pairs\": %llu, \"words\": %llu, "
            "\"out_bytes\": %llu",
            err ? "false" : "true", M, R, G, nfiles, (unsigned long long)bytes, wall, wall > 0 ? bytes / (wall * 1e6) : 0.0,
            (unsigned long long)pairs, (unsigned long long)words, (unsigned long long)out);
    if (single)
        fprintf(f, ", \"tokens\": %llu, \"device_ms_map\": %.3f, \"device_ms_reduce\": %.3f",
                (unsigned long long)tokens, ms_map, ms_reduce);
    fprintf(f, "}\n");
    if (f != stderr) fclose(f);
}

int main(int argc, char **argv) {
    const double t0 = wall_ms();
    if (argc < 4) {
        fprintf(stderr, "Usage: %s <num_mappers> <num_reducers> <input_file_list>\n", argv[0]); /* main.c:249 */
        return -1;
    }
    int M = atoi(argv[1]);
    int R = atoi(argv[2]);
    if (M < 1) M = 1; /* reference: SIGFPE at main.c:307; defined here */
    FILE *fl = fopen(argv[3], "r");
    if (!fl) {
        fprintf(stderr, "Error opening input file list: %s\n", argv[3]);
        return -1;
    }
    int count;
    if (fscanf(fl, "%d", &count) != 1) {
        fprintf(stderr, "Error reading the number of files from input file list\n");
        fclose(fl);
        return -1;
    }
    if (count < 0) count = 0;
    /* any number of files (the reference overflows files[MAX_FILES] past 360, main.c:8, 270) */
    cli_state cs = {0};
    cs.files = calloc((size_t)count + 1, sizeof(ii_file));
    cs.sizes = calloc((size_t)count + 1, sizeof(uint64_t));
    cs.names = calloc((size_t)count + 1, sizeof(char *));
    if (!cs.files || !cs.sizes || !cs.names) {
        fprintf(stderr, "Memory allocation failed for file name\n");
        fclose(fl);
        cli_free(&cs);
        return -1;
    }
    ii_file *files = cs.files;
    uint64_t *sizes = cs.sizes;
    for (int i = 0; i < count; i++) {
        cs.names[i] = malloc(4096);
        if (!cs.names[i]) {
            fprintf(stderr, "Memory allocation failed for file name\n");
            fclose(fl);
            cli_free(&cs);
            return -1;
        }
        cs.nnames = i + 1;
        if (fscanf(fl, "%4095s", cs.names[i]) != 1) {
            fprintf(stderr, "Error reading file name from input file list\n");
            fclose(fl);
            cli_free(&cs);
            return -1;
        }
        struct stat st;
        if (stat(cs.names[i], &st) == 0) sizes[i] = (uint64_t)st.st_size;
        else fprintf(stderr, "Error getting size of file: %s\n", cs.names[i]); /* main.c:294 */
        files[i].path = cs.names[i];
        files[i].size = sizes[i];
        files[i].id0 = (uint32_t)i; /* main.c:275 */
    }
    fclose(fl);

    /* size-balanced shards (main.c:300-328); printed like the reference */
    cs.order = calloc((size_t)count + 1, sizeof(uint32_t));
    cs.sb = calloc((size_t)M, sizeof(uint32_t));
    cs.se = calloc((size_t)M, sizeof(uint32_t));
    if (!cs.order || !cs.sb || !cs.se) {
        cli_free(&cs);
        return 1;
    }
    uint32_t *order = cs.order, *sb = cs.sb, *se = cs.se;
    ii_partition(sizes, (uint32_t)count, M, order, sb, se);
    for (int m = 0; m < M; m++) {
        printf("Mapper %d: Files %u to %u\n", m, sb[m], se[m]);
        for (uint32_t i = sb[m]; i < se[m]; i++) files[order[i]].mapper = m; /* main.c:98 names it */
    }
    /* the reference's emission order of the partial files: mapper 0's files, then mapper 1's, ... */
    uint32_t nemit = 0;
    for (int m = 0; m < M; m++)
        for (uint32_t i = sb[m]; i < se[m]; i++) order[nemit++] = order[i];
    const char *pe = getenv("II_PARTIAL_FILES");
    const int partials = pe && atoi(pe) == 1;

    const int G = gpus_requested();
    ii_ctx *owner[II_ALPHABET];
    ii_ctx *single = NULL;
    shard sh[MAXG];
    memset(sh, 0, sizeof(sh));
    multi_run run;
    memset(&run, 0, sizeof(run));
    int rc, reported = 0;
    const char *tm = getenv("II_TEST_MULTI");
    if (G == 1 && !(tm && !strcmp(tm, "1"))) {
        rc = ii_open(&single, 0);
        if (rc == II_OK) {
            /* files in list (= ID) order: postings come out ascending (main.c:217-226) */
            rc = ii_map_files(single, files, (uint32_t)count, M, NULL);
            if (rc == II_OK && partials) rc = write_partials(NULL, 0, single, order, nemit);
            if (rc == II_OK) rc = ii_reduce(single, 1);
            for (int l = 0; l < II_ALPHABET; l++) owner[l] = single;
        } else {
            fprintf(stderr, "ii_index: cannot open device: %s\n", ii_strerror(rc));
            reported = 1;
        }
    } else {
        rc = multi_map(files, sizes, (uint32_t)count, M, G, sh, &run);
        /* partial files while the contexts still hold their input files (before the exchange) */
        if (rc == II_OK && partials) rc = write_partials(sh, G, NULL, order, nemit);
        if (rc == II_OK) rc = multi_exchange(G, sh, &run, owner);
    }
    int err = 0;
    if (rc != II_OK) {
        /* a failed phase: report and leave at once — other contexts' threads may still sit in HIP
         * calls on a faulted device, so no join, no ii_close, no device statistics */
        if (!reported) fprintf(stderr, "ii_index: %s\n", ii_strerror(rc));
        const char *metrics = getenv("II_METRICS");
        if (metrics && *metrics) write_metrics(metrics, t0, M, R, G, (uint32_t)count, sizes, NULL, NULL, 1);
        fflush(stdout);
        fflush(stderr);
        _exit(1);
    } else if (R > 0) {
        pthread_t *th = calloc((size_t)R, sizeof(pthread_t));
        writer_arg *wa = calloc((size_t)R, sizeof(writer_arg));
        for (int r = 0; r < R; r++) {
            wa[r] = (writer_arg){owner, r, R, 0};
            pthread_create(&th[r], NULL, writer, &wa[r]);
        }
        for (int r = 0; r < R; r++) {
            pthread_join(th[r], NULL);
            err |= wa[r].err;
        }
        free(th);
        free(wa);
    }
    const char *metrics = getenv("II_METRICS");
    if (metrics && *metrics) write_metrics(metrics, t0, M, R, G, (uint32_t)count, sizes, single, sh, err);
    if (single) ii_close(single);
    for (int g = 0; g < G; g++) {
        if (sh[g].ctx) ii_close(sh[g].ctx);
        free(sh[g].files);
        free(sh[g].local);
    }
    cli_free(&cs);
    return err ? 1 : 0;
}
