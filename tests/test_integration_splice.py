"""CPU: the function-seam splice of INTEGRATION.md §2, compiled verbatim.

The reference's partition (main.c:300-323) leaves INCLUSIVE shard ends:
file_end[m] is the last file of mapper m (main.c:318, 323), and the mapper
walks [start_file, end_file) with end_file = file_end + 1 (main.c:355).  The
splice must therefore loop k <= file_end[m], or it skips the last file of
every mapper and hands ii_map_files uninitialised entries.

The harness fills files[] (size-sorted, main.c:300), file_start[] and
file_end[] the way main.c:307-323 does — a restatement of those lines, checked
against libii's ii_partition — and runs the C block of INTEGRATION.md §2 as
the body of a function.  The ii_* entry points it calls are stubs (no GPU):
ii_map_files checks that every in[id0] was written with its own path, size,
id0 and owning mapper (the buffer is poisoned before the block fills it).
"""
import os
import re
import subprocess

import pytest

from conftest import PKG, REPO

HARNESS = r"""
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "ii.h"

typedef struct FileInfo { char *file_name; long file_size; int id; } FileInfo;  /* main.c:14-18 */

static FileInfo *g_orig;       /* list order: g_orig[i].id == i */
static int *g_owner;           /* mapper that owns list file i */
static int g_n, g_mapped, g_bad;

/* poisoned allocation: an entry the splice does not write fails the check */
static void *poison_malloc(size_t n) { void *p = malloc(n ? n : 1); memset(p, 0xA5, n); return p; }

struct ii_ctx { int dummy; };
static struct ii_ctx g_ctx;
int ii_open(ii_ctx **out, int device) { (void)device; *out = &g_ctx; return II_OK; }
void ii_close(ii_ctx *ctx) { (void)ctx; }
int ii_reduce(ii_ctx *ctx, int copy_text) { (void)ctx; (void)copy_text; return II_OK; }
int ii_letter_text(ii_ctx *ctx, int letter, const char **buf, size_t *len) {
    (void)ctx; (void)letter; *buf = ""; *len = 0; return II_OK;
}
static int (*real_reducer_letters)(int, int, int *, int *);
int ii_reducer_letters(int r, int R, int *lo, int *hi) { return real_reducer_letters(r, R, lo, hi); }
int ii_map_files(ii_ctx *ctx, const ii_file *f, uint32_t n, int nthreads, uint64_t *hist) {
    (void)ctx; (void)nthreads; (void)hist;
    g_mapped = 1;
    if ((int)n != g_n) { printf("nfiles %u != %d\n", n, g_n); g_bad++; return II_ERR_ARG; }
    for (int i = 0; i < g_n; i++) {
        if (f[i].id0 != (uint32_t)i || f[i].path != g_orig[i].file_name ||
            f[i].size != (uint64_t)g_orig[i].file_size || f[i].mapper != g_owner[i]) {
            printf("in[%d] not set: id0 %u mapper %d (want %d)\n", i, f[i].id0, f[i].mapper, g_owner[i]);
            g_bad++;
        }
    }
    return g_bad ? II_ERR_ARG : II_OK;
}

/* the block of INTEGRATION.md section 2, verbatim, as a function body */
static int splice(FileInfo *files, int file_count, int num_mappers, int num_reducers,
                  int *file_start, int *file_end) {
#define malloc(n) poison_malloc(n)
#include "splice.inc"
#undef malloc
    return 0;
}

static int cmp_size(const void *a, const void *b) {  /* main.c:21-25, ties by list position */
    const FileInfo *x = a, *y = b;
    if (x->file_size != y->file_size) return x->file_size < y->file_size ? 1 : -1;
    return x->id - y->id;
}

int main(int argc, char **argv) {
    void *lib = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
    if (!lib) { printf("dlopen: %s\n", dlerror()); return 2; }
    int (*part)(const uint64_t *, uint32_t, int, uint32_t *, uint32_t *, uint32_t *) =
        (int (*)(const uint64_t *, uint32_t, int, uint32_t *, uint32_t *, uint32_t *))dlsym(lib, "ii_partition");
    real_reducer_letters = (int (*)(int, int, int *, int *))dlsym(lib, "ii_reducer_letters");
    if (!part || !real_reducer_letters) return 2;
    const int ns[] = {1, 3, 355}, Ms[] = {1, 2, 3, 8};
    int cases = 0;
    for (int a = 0; a < 3; a++) for (int b = 0; b < 4; b++) {
        const int n = ns[a], M = Ms[b];
        g_n = n;
        g_orig = calloc(n, sizeof(FileInfo));
        g_owner = calloc(n, sizeof(int));
        uint64_t *sizes = calloc(n, sizeof(uint64_t));
        unsigned s = 12345u + 77u * n;
        for (int i = 0; i < n; i++) {      /* ragged sizes with ties and empty files */
            s = s * 1103515245u + 12345u;
            long sz = (long)((s >> 8) % 97000u);
            if (i % 7 == 3) sz = 0;
            if (i % 11 == 5 && i) sz = g_orig[i - 1].file_size;
            g_orig[i].file_name = malloc(16);
            snprintf(g_orig[i].file_name, 16, "f%03d", i);
            g_orig[i].file_size = sz;
            g_orig[i].id = i;
            sizes[i] = (uint64_t)sz;
        }
        FileInfo *files = malloc(n * sizeof(FileInfo));
        memcpy(files, g_orig, n * sizeof(FileInfo));
        qsort(files, n, sizeof(FileInfo), cmp_size);                     /* main.c:300 */
        long total = 0;
        for (int i = 0; i < n; i++) total += files[i].file_size;
        long size_per_mapper = total / M;                                  /* main.c:307 */
        int *file_start = malloc(M * sizeof(int)), *file_end = malloc(M * sizeof(int));
        for (int m = 0; m < M; m++) { file_start[m] = n; file_end[m] = n - 1; }  /* unset in main.c: empty */
        long cum = 0;
        int cur = 0;
        file_start[0] = 0;
        for (int i = 0; i < n; ++i) {                                      /* main.c:315-322 */
            cum += files[i].file_size;
            if (cum >= size_per_mapper && cur < M - 1) {
                file_end[cur] = i;
                file_start[++cur] = i + 1;
                cum = 0;
            }
        }
        file_end[cur] = n - 1;                                             /* main.c:323 */
        uint32_t *order = malloc(n * sizeof(uint32_t)), *sb = malloc(M * 4), *se = malloc(M * 4);
        if (part(sizes, n, M, order, sb, se)) return 3;
        for (int m = 0; m < M; m++) {
            if ((int)sb[m] != file_start[m] || (int)se[m] != file_end[m] + 1) {
                printf("n=%d M=%d mapper %d: main.c [%d, %d] vs ii_partition [%u, %u)\n", n, M, m,
                       file_start[m], file_end[m], sb[m], se[m]);
                return 4;
            }
            for (uint32_t k = sb[m]; k < se[m]; k++) {
                if (files[k].id != (int)order[k]) return 5;
                g_owner[order[k]] = m;
            }
        }
        g_mapped = 0;
        g_bad = 0;
        int rc = splice(files, n, M, 26, file_start, file_end);
        if (rc || !g_mapped || g_bad) { printf("n=%d M=%d: rc %d mapped %d bad %d\n", n, M, rc, g_mapped, g_bad); return 1; }
        cases++;
        for (int i = 0; i < n; i++) free(g_orig[i].file_name);
        free(g_orig); free(g_owner); free(sizes); free(files); free(file_start); free(file_end);
        free(order); free(sb); free(se);
    }
    printf("ok %d cases\n", cases);
    return 0;
}
"""


def splice_block():
    doc = open(os.path.join(REPO, "INTEGRATION.md")).read()
    sec = doc.split("## 2. The function seam", 1)[1].split("\n## ", 1)[0]
    blocks = re.findall(r"```c\n(.*?)```", sec, flags=re.S)
    assert blocks, "no C block in INTEGRATION.md section 2"
    return blocks[0]


def build_and_run(tmp_path, block):
    (tmp_path / "splice.inc").write_text(block)
    (tmp_path / "harness.c").write_text(HARNESS)
    exe = tmp_path / "harness"
    subprocess.run(["gcc", "-O1", "-g", "-Wall", "-Wno-unused-variable", "-fsanitize=address,undefined",
                    "-I", os.path.join(REPO, "include"), "-I", str(tmp_path), "-o", str(exe),
                    str(tmp_path / "harness.c"), "-ldl"], check=True, capture_output=True, text=True)
    out_dir = tmp_path / "out"   # the block writes a.txt ... z.txt into the CWD
    out_dir.mkdir()
    return subprocess.run([str(exe), os.path.join(PKG, "libii.so")], cwd=out_dir, capture_output=True,
                          text=True, timeout=120, env=dict(os.environ, ASAN_OPTIONS="detect_leaks=0"))


def test_integration_splice_sets_every_file_once(tmp_path):
    r = build_and_run(tmp_path, splice_block())
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok 12 cases" in r.stdout
    assert sorted(os.listdir(tmp_path / "out")) == sorted("%c.txt" % (97 + l) for l in range(26))


def test_harness_catches_the_exclusive_end_bug(tmp_path):
    """The round-4 splice (k < file_end[m]) must fail the same harness."""
    block = splice_block().replace("k <= file_end[m]", "k < file_end[m]")
    assert "k < file_end[m]" in block
    r = build_and_run(tmp_path, block)
    assert r.returncode != 0 and "not set" in r.stdout, r.stdout + r.stderr
