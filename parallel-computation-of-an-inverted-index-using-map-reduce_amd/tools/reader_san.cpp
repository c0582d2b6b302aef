// reader_san.cpp — host-only driver of ii_map_files' reader (csrc/ii_reader.h)
// for the ASan / UBSan build of tests/test_sanitizers.py: the
// listed files are laid out as the device would hold them (file f at off[f],
// a '\n' after each, sizes from the list — the stat sizes ii_map_files gets),
// read window by window with io_fill by several threads into host memory
// (libii.so's reader threads do the same into pinned buffers), and the image is
// written to stdout together with the "grown" verdict.
//   reader_san WINDOW THREADS size0 path0 [size1 path1 ...]
#include <stdlib.h>

#include <vector>

#include "../csrc/ii_reader.h"

struct Arg {
    IoLayout* lay;
    uint8_t* img;
    uint64_t total, win;
    int t, nt;
};

static void* worker(void* p) {
    Arg* a = (Arg*)p;
    for (uint64_t lo = (uint64_t)a->t * a->win; lo < a->total; lo += (uint64_t)a->nt * a->win) {
        const uint64_t hi = lo + a->win < a->total ? lo + a->win : a->total;
        std::vector<uint8_t> buf(hi - lo, 0xEE);  // a window buffer of its own (the pinned windows)
        io_fill(a->lay, lo, hi, buf.data());
        memcpy(a->img + lo, buf.data(), hi - lo);
    }
    return nullptr;
}

int main(int argc, char** argv) {
    if (argc < 3 || (argc - 3) % 2) {
        fprintf(stderr, "usage: %s WINDOW THREADS size0 path0 ...\n", argv[0]);
        return 2;
    }
    const uint64_t win = strtoull(argv[1], nullptr, 10);
    const int nt = atoi(argv[2]);
    const uint32_t n = (uint32_t)(argc - 3) / 2;
    std::vector<ii_file> files(n);
    std::vector<uint64_t> off(n + 1, 0);
    for (uint32_t f = 0; f < n; f++) {
        files[f].size = strtoull(argv[3 + 2 * f], nullptr, 10);
        files[f].path = argv[4 + 2 * f];
        files[f].id0 = f;
        files[f].mapper = (int32_t)(f % 3);
        off[f + 1] = off[f] + files[f].size + 1;
    }
    const uint64_t total = off[n];
    std::vector<uint8_t> img(total + 1, 0);
    IoLayout lay{files.data(), n, off.data(), 0, PTHREAD_MUTEX_INITIALIZER};
    std::vector<pthread_t> th(nt);
    std::vector<Arg> args(nt);
    for (int t = 0; t < nt; t++) {
        args[t] = Arg{&lay, img.data(), total, win ? win : 1, t, nt};
        pthread_create(&th[t], nullptr, worker, &args[t]);
    }
    for (int t = 0; t < nt; t++) pthread_join(th[t], nullptr);
    printf("grown=%d\n", lay.grown);
    fflush(stdout);
    if (total && fwrite(img.data(), 1, total, stdout) != total) return 1;
    return 0;
}
