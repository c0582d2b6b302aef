/*
 * ii_index.c — C host CLI, drop-in for the reference's `tema1`:
 *
 *     ii_index <num_mappers> <num_reducers> <input_file_list>
 *
 * Same argument handling, list format, file-ID numbering and outputs
 * (a.txt .. z.txt in the current directory) as /root/reference/main.c:246-390.
 * The map and reduce phases (main.c:326-384) run on the MI355X through
 * libii.so (include/ii.h); M sizes the host reader threads and R the writer
 * threads, neither changes the output.
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

#include "ii.h"

typedef struct {
    ii_ctx *ctx;
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
        if (ii_letter_text(w->ctx, l, &buf, &len) != II_OK) { w->err = 1; continue; }
        FILE *o = fopen(name, "w");
        if (!o) { printf("eroare la fisierul final\n"); w->err = 1; continue; } /* main.c:151-154 */
        if (len && fwrite(buf, 1, len, o) != len) w->err = 1;
        fclose(o);
    }
    return NULL;
}

int main(int argc, char **argv) {
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
    ii_file *files = calloc((size_t)count + 1, sizeof(ii_file));
    uint64_t *sizes = calloc((size_t)count + 1, sizeof(uint64_t));
    char **names = calloc((size_t)count + 1, sizeof(char *));
    for (int i = 0; i < count; i++) {
        names[i] = malloc(4096);
        if (!names[i]) {
            fprintf(stderr, "Memory allocation failed for file name\n");
            fclose(fl);
            return -1;
        }
        if (fscanf(fl, "%4095s", names[i]) != 1) {
            fprintf(stderr, "Error reading file name from input file list\n");
            fclose(fl);
            return -1;
        }
        struct stat st;
        if (stat(names[i], &st) == 0) sizes[i] = (uint64_t)st.st_size;
        else fprintf(stderr, "Error getting size of file: %s\n", names[i]); /* main.c:294 */
        files[i].path = names[i];
        files[i].size = sizes[i];
        files[i].id0 = (uint32_t)i; /* main.c:275 */
    }
    fclose(fl);

    /* size-balanced shards (main.c:300-328); printed like the reference */
    uint32_t *order = calloc((size_t)count + 1, sizeof(uint32_t));
    uint32_t *sb = calloc((size_t)M, sizeof(uint32_t)), *se = calloc((size_t)M, sizeof(uint32_t));
    ii_partition(sizes, (uint32_t)count, M, order, sb, se);
    for (int m = 0; m < M; m++) {
        printf("Mapper %d: Files %u to %u\n", m, sb[m], se[m]);
        for (uint32_t i = sb[m]; i < se[m]; i++) files[order[i]].mapper = m; /* main.c:98 names it */
    }

    ii_ctx *ctx = NULL;
    int rc = ii_open(&ctx, 0);
    if (rc != II_OK) {
        fprintf(stderr, "ii_index: cannot open device: %s\n", ii_strerror(rc));
        return 1;
    }
    /* files in list (= ID) order: postings come out ascending (main.c:217-226) */
    rc = ii_map_files(ctx, files, (uint32_t)count, M, NULL);
    const char *pe = getenv("II_PARTIAL_FILES");
    if (rc == II_OK && pe && atoi(pe) == 1) {
        /* mapper m reads order[sb[m] .. se[m]) (main.c:93); mappers one after another */
        uint32_t n = 0;
        for (int m = 0; m < M; m++)
            for (uint32_t i = sb[m]; i < se[m]; i++) order[n++] = order[i];
        rc = ii_partials(ctx, order, n);
        for (int l = 0; rc == II_OK && l < 26; l++) {
            const char *buf;
            size_t len;
            char name[32];
            snprintf(name, sizeof(name), "partial_%c.txt", 'a' + l);
            rc = ii_partial_text(ctx, l, &buf, &len);
            if (rc != II_OK) break;
            FILE *o = fopen(name, "w+");
            if (!o) {
                fprintf(stderr, "Error creating partial file: %s\n", name); /* main.c:336 */
                rc = II_ERR_IO;
                break;
            }
            if (len && fwrite(buf, 1, len, o) != len) rc = II_ERR_IO;
            fclose(o);
        }
    }
    if (rc == II_OK) rc = ii_reduce(ctx, 1);
    if (rc != II_OK) {
        fprintf(stderr, "ii_index: %s\n", ii_strerror(rc));
        ii_close(ctx);
        return 1;
    }
    int err = 0;
    if (R > 0) {
        pthread_t *th = calloc((size_t)R, sizeof(pthread_t));
        writer_arg *wa = calloc((size_t)R, sizeof(writer_arg));
        for (int r = 0; r < R; r++) {
            wa[r] = (writer_arg){ctx, r, R, 0};
            pthread_create(&th[r], NULL, writer, &wa[r]);
        }
        for (int r = 0; r < R; r++) {
            pthread_join(th[r], NULL);
            err |= wa[r].err;
        }
        free(th);
        free(wa);
    }
    ii_close(ctx);
    for (int i = 0; i < count; i++) free(names[i]);
    free(names);
    free(files);
    free(sizes);
    free(order);
    free(sb);
    free(se);
    return err ? 1 : 0;
}
