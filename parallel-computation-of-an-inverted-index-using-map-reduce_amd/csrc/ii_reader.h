// ii_reader.h — the host side of ii_map_files' pipelined reader (SURVEY §8 f2;
// replaces the mappers' fopen / fscanf, main.c:93-102): the device layout of
// the files (file f at off[f], one '\n' separator after every file) is cut
// into windows, and io_fill reads one window with pread.  Plain C++ and POSIX
// only — no HIP — so tests/test_sanitizers.py builds it into a host program
// (tools/reader_san.cpp) under ASan / UBSan; libii.so's reader threads call
// the same function.
#pragma once
#include <fcntl.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>

#include "../../include/ii.h"

struct IoLayout {
    const ii_file* files;
    uint32_t nfiles;
    const uint64_t* off;  // nfiles + 1: device offset of every file (+1 separator each)
    int grown;            // some file had more bytes than its stat size
    pthread_mutex_t mu;
};

// Fill window [lo, hi) of the device layout into buf.
static inline void io_fill(IoLayout* j, uint64_t lo, uint64_t hi, uint8_t* buf) {
    uint32_t f = (uint32_t)(std::upper_bound(j->off, j->off + j->nfiles + 1, lo) - j->off) - 1;
    for (; f < j->nfiles && j->off[f] < hi; f++) {
        const uint64_t fsz = j->off[f + 1] - j->off[f] - 1;  // bytes of file f (separator excluded)
        const uint64_t a = std::max(lo, j->off[f]), b = std::min(hi, j->off[f] + fsz);
        if (b > a || (fsz == 0 && j->off[f] >= lo)) {
            // every window that holds file bytes (or the separator of an empty file) opens it;
            // only the window holding the file's first byte reports a failure (main.c:98)
            const int fd = open(j->files[f].path, O_RDONLY);
            const bool first = j->off[f] >= lo;
            if (fd < 0) {
                if (first) fprintf(stderr, "Mapper %d: Error opening file %s\n", j->files[f].mapper, j->files[f].path);
                if (b > a) memset(buf + (a - lo), ' ', b - a);
            } else {
                uint64_t done = 0;
                while (a + done < b) {
                    const ssize_t r = pread(fd, buf + (a + done - lo), b - a - done, (off_t)(a + done - j->off[f]));
                    if (r <= 0) break;
                    done += (uint64_t)r;
                }
                if (a + done < b) memset(buf + (a + done - lo), ' ', b - a - done);  // shorter than stat: spaces
                if (j->off[f] + fsz <= hi) {  // this window holds the file's end: is there more?
                    uint8_t extra;
                    if (pread(fd, &extra, 1, (off_t)fsz) == 1) {
                        pthread_mutex_lock(&j->mu);
                        j->grown = 1;
                        pthread_mutex_unlock(&j->mu);
                    }
                }
                close(fd);
            }
        }
        const uint64_t sep = j->off[f] + fsz;  // separator byte of file f
        if (sep >= lo && sep < hi) buf[sep - lo] = '\n';
    }
}

