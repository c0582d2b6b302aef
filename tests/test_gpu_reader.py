"""GPU: the pipelined file reader behind ii_map_files (SURVEY.md §8 f2:
pread into pinned 8 MiB windows, async H2D per reader thread) gives the same
index as the oracle on files that straddle windows, with missing, empty,
shrunk and grown files."""
import os
import tempfile

import pytest

import ii_ctypes
from oracle_py import oracle_index
from test_gpu_parity import assert_same, rand_corpus

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def idx():
    ix = ii_ctypes.Index(0)
    yield ix
    ix.close()


def write_files(td, text, off):
    paths = []
    for f in range(len(off) - 1):
        p = os.path.join(td, "f%04d.txt" % f)
        with open(p, "wb") as fh:
            fh.write(text[off[f]:off[f + 1]])
        paths.append(p)
    return paths


@pytest.mark.parametrize("nthreads", [1, 3, 16])
def test_reader_windows_vs_oracle(idx, nthreads):
    # ~30 MB over 120 files: several 8 MiB windows, files straddling window edges
    t, off = ii_ctypes.zipf_corpus(30_000_000, 120, 200_000, 11, threads=8)
    off = off.tolist()
    with tempfile.TemporaryDirectory() as td:
        paths = write_files(td, bytes(t), off)
        idx.map_files(paths, nthreads=nthreads)
        idx.reduce()
        st = idx.stats()
        assert st.io_bytes == off[-1] + len(paths) and st.io_ms > 0
    assert_same(idx.letters(), oracle_index(t, off, list(range(120))), "reader")


def test_reader_missing_empty_shrunk_grown(idx, capfd):
    text, off, ids = rand_corpus(5, 30, 40000)
    with tempfile.TemporaryDirectory() as td:
        paths = write_files(td, text, off)
        paths[3] = os.path.join(td, "missing.txt")
        sizes = [off[f + 1] - off[f] for f in range(30)]
        sizes[3] = 0
        exp_text, exp_off = bytearray(), [0]
        for f in range(30):
            if f != 3:
                exp_text += text[off[f]:off[f + 1]]
            exp_off.append(len(exp_text))
        exp = oracle_index(bytes(exp_text), exp_off, ids)
        mappers = [(f * 7) % 5 for f in range(30)]  # file 3 belongs to mapper 1
        # exact sizes
        idx.map_files(paths, nthreads=4, sizes=sizes, mappers=mappers)
        idx.reduce()
        assert_same(idx.letters(), exp, "exact")
        # the owning mapper's id, as main.c:98 prints it
        assert "Mapper 1: Error opening file %s\n" % paths[3] in capfd.readouterr().err
        # sizes larger than the files: the reader pads with spaces
        idx.map_files(paths, nthreads=4, sizes=[s + 5000 for s in sizes])
        idx.reduce()
        assert_same(idx.letters(), exp, "padded")
        # a size smaller than its file: the reader falls back to whole-file reads
        small = list(sizes)
        small[7] = max(0, small[7] // 2)
        small[8] = 0
        capfd.readouterr()
        idx.map_files(paths, nthreads=4, sizes=small, mappers=mappers)
        idx.reduce()
        assert_same(idx.letters(), exp, "grown")
        # reported once, although the fallback re-reads every file
        assert capfd.readouterr().err.count("Error opening file %s" % paths[3]) == 1
