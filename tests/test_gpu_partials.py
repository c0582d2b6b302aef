"""GPU parity of the partial-file emitter (ii_partials):
against the reference binary's own partial_<letter>.txt files (one mapper,
tests/golden/partials.json) and against the oracle's restatement on seeded
corpora with arbitrary file orders."""
import hashlib
import os
import random
import subprocess
import tempfile

import pytest

import ii_ctypes
from conftest import CASES, PKG, case_arrays, materialize, partials_meta, size_order
from oracle_py import oracle_partials
from test_gpu_parity import LETTERS, assert_same, rand_corpus

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def idx():
    ix = ii_ctypes.Index(0)
    yield ix
    ix.close()


def assert_hashes(got, meta, ctx):
    for l in LETTERS:
        assert hashlib.sha256(got[l]).hexdigest() == meta[l]["sha256"], "%s partial_%s.txt differs" % (ctx, l)


@pytest.mark.parametrize("case", CASES)
def test_partials_match_reference(idx, case):
    text, off, ids, _ = case_arrays(case)
    idx.map_host(text, off, ids)
    assert_hashes(idx.partials(size_order(case)), partials_meta()[case], case)


@pytest.mark.parametrize("case", ["config1", "edge", "zipf_small"])
def test_cli_partial_files(case):
    with tempfile.TemporaryDirectory() as td:
        _, _, expected = materialize(case, td)
        env = dict(os.environ, II_PARTIAL_FILES="1")
        r = subprocess.run([os.path.join(PKG, "ii_index"), "1", "3", "list.txt"], cwd=td, capture_output=True,
                           timeout=120, env=env)
        assert r.returncode == 0, r.stderr.decode()
        got = {l: open(os.path.join(td, "partial_%s.txt" % l), "rb").read() for l in LETTERS}
        assert_hashes(got, partials_meta()[case], case)
        assert_same({l: open(os.path.join(td, l + ".txt"), "rb").read() for l in LETTERS}, expected, case)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_partials_random_orders_vs_oracle(idx, seed):
    # long tokens (250..700 bytes), NULs, every delimiter; files of up to 200 KB
    # span several 64 KiB pieces; orders repeat and skip files
    text, off, ids = rand_corpus(seed, [6, 60, 300][seed - 1], [200000, 20000, 2000][seed - 1])
    idx.map_host(text, off, ids)
    rng = random.Random(seed)
    for order in [list(range(len(ids))), rng.sample(range(len(ids)), len(ids)),
                  [rng.randrange(len(ids)) for _ in range(len(ids) // 2 + 1)], []]:
        assert_same(idx.partials(order), oracle_partials(text, off, ids, order), "seed %d" % seed)


def test_partials_after_reduce_and_zipf(idx):
    t, off = ii_ctypes.zipf_corpus(8_000_000, 90, 100_000, 7, threads=8)
    ids = [2 * i + 1 for i in range(90)]
    offl = off.tolist()
    idx.map_host(t, offl, ids)
    idx.reduce()  # the text stays resident: partials may follow the reduce
    order = sorted(range(90), key=lambda i: (-(offl[i + 1] - offl[i]), i))
    assert_same(idx.partials(order), oracle_partials(t, off, ids, order), "zipf")


def test_partials_state_and_args(idx):
    ix = ii_ctypes.Index(0)
    try:
        with pytest.raises(ii_ctypes.IIError):
            ix.partials([0])  # nothing mapped
    finally:
        ix.close()
    idx.map_host(b"Abc de", [0, 6], [0])
    with pytest.raises(ii_ctypes.IIError):
        idx.partials([1])  # file index out of range
    got = idx.partials([0])
    assert got["a"] == b"abc 1\n" and got["d"] == b"de 1\n"
