"""GPU parity: the MI355X path (libii.so through the C ABI and the ii_index
CLI) against the reference's golden outputs and the oracle, bit-exact."""
import os
import random
import subprocess
import tempfile

import numpy as np
import pytest

import ii_ctypes
from conftest import CASES, PKG, case_arrays, materialize
from oracle_py import oracle_index

pytestmark = pytest.mark.gpu
LETTERS = "abcdefghijklmnopqrstuvwxyz"


@pytest.fixture(scope="module")
def idx():
    ix = ii_ctypes.Index(0)
    yield ix
    ix.close()


def assert_same(got, expected, ctx=""):
    for l in LETTERS:
        if got[l] != expected[l]:
            a, b = got[l], expected[l]
            i = next((k for k in range(min(len(a), len(b))) if a[k] != b[k]), min(len(a), len(b)))
            raise AssertionError("%s letter %s differs at byte %d: got %r expected %r" %
                                 (ctx, l, i, a[max(0, i - 40):i + 40], b[max(0, i - 40):i + 40]))


@pytest.mark.parametrize("case", CASES)
def test_cli_matches_reference(case):
    with tempfile.TemporaryDirectory() as td:
        _, _, expected = materialize(case, td)
        r = subprocess.run([os.path.join(PKG, "ii_index"), "3", "5", "list.txt"], cwd=td, capture_output=True,
                           timeout=120)
        assert r.returncode == 0, r.stderr.decode()
        got = {l: open(os.path.join(td, l + ".txt"), "rb").read() for l in LETTERS}
        assert_same(got, expected, case)
        # missing files: reported once each, by the mapper whose shard holds them (main.c:98, 290-296)
        toks = open(os.path.join(td, "list.txt")).read().split()
        paths = toks[1:1 + int(toks[0])]
        sizes = [os.path.getsize(os.path.join(td, p)) if os.path.exists(os.path.join(td, p)) else 0 for p in paths]
        order, sb, se = ii_ctypes.partition(sizes, 3)
        err = r.stderr.decode()
        for m in range(3):
            for i in order[sb[m]:se[m]]:
                if not os.path.exists(os.path.join(td, paths[i])):
                    assert err.count("Mapper %d: Error opening file %s\n" % (m, paths[i])) == 1, err
                    assert "Error getting size of file: %s\n" % paths[i] in err


@pytest.mark.parametrize("case", CASES)
def test_map_host_matches_reference(idx, case):
    text, off, ids, expected = case_arrays(case)
    hist = idx.map_host(text, off, ids)
    idx.reduce()
    assert_same(idx.letters(), expected, case)
    st = idx.stats()
    assert sum(hist) == st.tokens
    lines = {l: expected[l].count(b"\n") for l in LETTERS}
    for i, l in enumerate(LETTERS):
        assert (hist[i] == 0) == (lines[l] == 0)
    assert st.words == sum(lines.values())
    assert st.out_bytes == sum(len(v) for v in expected.values())


def test_map_device_torch_buffer(idx):
    import torch
    text, off, ids, expected = case_arrays("config2")
    # build the device layout: separator after each file (contract of ii_map_device)
    buf = bytearray()
    starts = []
    for f in range(len(ids)):
        starts.append(len(buf))
        buf += text[off[f]:off[f + 1]] + b"\n"
    d = torch.tensor(np.frombuffer(bytes(buf), dtype=np.uint8), device="cuda")
    torch.cuda.synchronize()
    idx.map_device(d.data_ptr(), len(buf), starts, ids)
    idx.reduce()
    assert_same(idx.letters(), expected, "device")


def test_map_device_layout_violation(idx):
    import torch
    d = torch.tensor(np.frombuffer(b"abc def", dtype=np.uint8), device="cuda")
    torch.cuda.synchronize()
    with pytest.raises(ii_ctypes.IIError) as e:
        idx.map_device(d.data_ptr(), 7, [0, 2], [0, 1])  # file 1 starts mid-token
    assert e.value.code == -6


def test_empty_inputs(idx):
    for text, off, ids in [(b"", [0], []), (b"", [0, 0, 0], [0, 1]), (b"123 ,,, \n\t 456", [0, 15], [0]),
                           (b" \x00abc ", [0, 6], [0])]:
        idx.map_host(text, off, ids)
        idx.reduce()
        got = idx.letters()
        assert all(v == b"" for v in got.values())


def rand_corpus(seed, nfiles, max_bytes):
    rng = random.Random(seed)
    letters = b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ"
    other = b"0123456789.,'-_\x00\x80\xc3\xa9\xff\x1c\x85\xa0"
    spaces = b" \t\n\x0b\x0c\r"
    vocab = [bytes(rng.choice(letters) for _ in range(rng.choice([1, 2, 3, 5, 8, 12, 13, 15, 24, 25, 40])))
             for _ in range(300)]
    text = bytearray()
    off = [0]
    for _ in range(nfiles):
        n = rng.randint(0, max_bytes)
        f = bytearray()
        while len(f) < n:
            t = bytearray(rng.choice(vocab))
            for _ in range(rng.choice([0, 0, 1, 2])):
                t.insert(rng.randint(0, len(t)), rng.choice(other))
            if rng.random() < 0.002:
                t = bytearray(rng.choice(letters) for _ in range(rng.randint(250, 700)))  # beyond 299: defined UB
            f += t + bytes([rng.choice(spaces)])
        if rng.random() < 0.5:
            f = f.rstrip(spaces)
        text += f
        off.append(len(text))
    return bytes(text), off, list(range(nfiles))


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_random_corpora_vs_oracle(idx, seed):
    text, off, ids = rand_corpus(seed, [5, 50, 200, 900][seed - 1], [200000, 30000, 3000, 400][seed - 1])
    idx.map_host(text, off, ids)
    idx.reduce()
    assert_same(idx.letters(), oracle_index(text, off, ids), "seed %d" % seed)


def test_noncontiguous_ids(idx):
    # a shard: files with gaps in their IDs (multi-GPU shards, missing files)
    text, off, _ = rand_corpus(9, 40, 5000)
    ids = [3 * i + 7 for i in range(40)]
    idx.map_host(text, off, ids)
    idx.reduce()
    assert_same(idx.letters(), oracle_index(text, off, ids), "ids")


@pytest.mark.parametrize("first", [1, 95, 9999980, 4294967200])
def test_offset_contiguous_ids(idx, first):
    # an ii_partition share: consecutive ids from `first` (K3 adds the offset to the shard-local
    # file index instead of gathering the id), across digit-count boundaries and past 2^31
    # (u64 pairs instead of the compact form)
    text, off, _ = rand_corpus(11, 40, 5000)
    ids = [first + i for i in range(40)]
    idx.map_host(text, off, ids)
    idx.reduce()
    assert_same(idx.letters(), oracle_index(text, off, ids), "first %d" % first)


def long_variant_corpus(seed, nfiles=60, per_file=3000):
    """Long words (13-120 letters) written many ways: case changes, digits,
    punctuation, high bytes and NULs inside, so that most occurrences differ
    in their raw bytes from the word's representative and k_long_verify walks
    them letter by letter (across several 16-byte blocks)."""
    rng = random.Random(seed)
    base = [bytes(rng.choice(LETTERS.encode()) for _ in range(rng.choice([13, 14, 17, 29, 31, 33, 64, 120])))
            for _ in range(150)]
    # words that agree on a long raw prefix and differ late
    base += [b[:-1] + bytes([(b[-1] - 97 + 1) % 26 + 97]) for b in base[:40]]
    other = b"0123456789.,'-_\x80\xc3\xa9\xff\x1c"
    text = bytearray()
    off = [0]
    for _ in range(nfiles):
        f = bytearray()
        for _ in range(per_file // 40):
            t = bytearray(rng.choice(base))
            for i in range(len(t)):
                if rng.random() < 0.2:
                    t[i] ^= 0x20
            for _ in range(rng.choice([0, 0, 1, 3, 8])):
                t.insert(rng.randint(0, len(t)), rng.choice(other))
            f += t + rng.choice([b" ", b"\n", b"\t"])
        text += f
        off.append(len(text))
    return bytes(text), off, list(range(nfiles))


@pytest.mark.parametrize("seed", [31, 32])
def test_long_word_variants_vs_oracle(idx, seed):
    text, off, ids = long_variant_corpus(seed)
    idx.map_host(text, off, ids)
    idx.reduce()
    assert_same(idx.letters(), oracle_index(text, off, ids), "long variants %d" % seed)
    # every variant verified as its word: no (false) hash collision forced a re-map
    assert idx.stats().retries == 0


def test_table_regrow_and_reuse():
    os.environ["II_TABLE_LOG2"] = "10"  # 1024-slot big table: forces several regrows
    try:
        ix = ii_ctypes.Index(0)
    finally:
        del os.environ["II_TABLE_LOG2"]
    t, off = ii_ctypes.zipf_corpus(24_000_000, 300, 400_000, 5, threads=8)
    ids = list(range(300))
    exp = oracle_index(t, off, ids)
    for _ in range(2):
        ix.map_host(t, off.tolist(), ids)
        ix.reduce()
        assert_same(ix.letters(), exp, "regrow")
    st = ix.stats()
    assert st.words > 131072 and st.table_cap >= 2 * st.words
    ix.close()


def test_zipf_medium_vs_oracle(idx):
    t, off = ii_ctypes.zipf_corpus(48_000_000, 700, 300_000, 21, threads=8)
    ids = list(range(700))
    idx.map_host(t, off.tolist(), ids)
    idx.reduce()
    assert_same(idx.letters(), oracle_index(t, off, ids), "zipf48M")


def dense_sparse_corpus():
    """Empty K1b chunks (whitespace only), chunks at the fixed capacity (one
    letter per two bytes: kChunk / 2 tokens) and ordinary text across files."""
    rng = random.Random(5)
    parts = [b" " * 200_000, b"".join(rng.choice([b"a ", b"B\t", b"c\n"]) for _ in range(70_000)),
             b"\n" * 150_000]
    t2, off2, _ = rand_corpus(11, 30, 20_000)
    text = bytearray()
    off = [0]
    for p in parts + [t2[off2[i]:off2[i + 1]] for i in range(30)] + [b"x " * 40_000]:
        text += p
        off.append(len(text))
    return bytes(text), off, list(range(len(off) - 1))


def test_record_layouts_vs_oracle():
    """K1's dense (counted) and fixed-capacity record layouts give the same index."""
    text, off, ids = dense_sparse_corpus()
    exp = oracle_index(text, off, ids)
    counts = {}
    for layout in ["dense", "fixed"]:
        os.environ["II_REC_LAYOUT"] = layout
        try:
            ix = ii_ctypes.Index(0)
            for case in ["config2", "edge"]:
                t, o, i, e = case_arrays(case)
                ix.map_host(t, o, i)
                ix.reduce()
                assert_same(ix.letters(), e, layout + " " + case)
            ix.map_host(text, off, ids)
            ix.reduce()
            assert_same(ix.letters(), exp, layout)
            st = ix.stats()
            counts[layout] = (st.tokens, st.pairs, st.words)
            ix.close()
        finally:
            del os.environ["II_REC_LAYOUT"]
    assert counts["dense"] == counts["fixed"]


def test_narrow_key_overflow_vs_oracle():
    """Narrow (u32) records: a single-file chunk keeps its fast-path misses'
    keys in a bounded area; II_NARROW_KEYS lowers that bound so that the
    overflow path (the rest go down K1c's general path, letter counts
    corrected) runs on an ordinary corpus whose vocabulary overflows the hot
    table (many misses per chunk)."""
    t, off = ii_ctypes.zipf_corpus(24_000_000, 40, 3_000_000, 29, threads=8)
    ids = list(range(40))
    exp = oracle_index(t, off, ids)
    for cap in ["0", "5", "64"]:
        os.environ["II_NARROW_KEYS"] = cap
        try:
            ix = ii_ctypes.Index(0)
            ix.map_host(t, off.tolist(), ids)
            ix.reduce()
            assert_same(ix.letters(), exp, "narrow keys " + cap)
            assert ix.stats().resolved_tokens > 0
            ix.close()
        finally:
            del os.environ["II_NARROW_KEYS"]


# ---------------------------------------------------------------- multi-GPU exchange logic
def shard_and_merge(text, off, G, id_bound=None, balanced=False, contiguous=False, pre_reduce=False, id_stride=1):
    """G logical shards on one device: files split by the reference's size
    heuristic (ii_partition), each shard mapped in its own context, letter
    ranges exchanged (ii_export / ii_import) and formatted by their owner.
    pre_reduce: every shard first indexes its own files alone (ii_reduce:
    compact pairs, the token sort consumes the K1 records in place), checked
    against the oracle, and only then exports (which must map again)."""
    import ii_dist
    n = len(off) - 1
    sizes = [off[i + 1] - off[i] for i in range(n)]
    order, sb, se = ii_ctypes.partition(sizes, G)
    if contiguous:  # rank g owns files [g*n/G, (g+1)*n/G) (the bench's layout): ordered id ranges
        order = list(range(n))
        sb = [g * n // G for g in range(G)]
        se = [(g + 1) * n // G for g in range(G)]
    idxs = []
    try:
        for g in range(G):
            fids = sorted(order[sb[g]:se[g]])
            t = bytearray()
            o = [0]
            for f in fids:
                t += text[off[f]:off[f + 1]]
                o.append(len(t))
            ix = ii_ctypes.Index(0)
            idxs.append(ix)
            ix.map_host(bytes(t), o, [f * id_stride for f in fids])
            if pre_reduce:
                ix.reduce()
                assert_same(ix.letters(), oracle_index(bytes(t), o, [f * id_stride for f in fids]),
                            "shard %d alone" % g)
        los, his = ii_dist.logical_shards_reduce(idxs, id_bound if id_bound is not None else (n - 1) * id_stride + 1,
                                                 balanced=balanced)
        merged = {}
        for g, ix in enumerate(idxs):
            lo, hi = los[g], his[g]
            if not balanced:
                assert (lo, hi) == ii_ctypes.reducer_letters(g, G)
            got = ix.letters()
            for l in range(26):
                ch = chr(97 + l)
                if lo <= l < hi:
                    merged[ch] = got[ch]
                else:
                    assert got[ch] == b"", "rank %d holds letter %s it does not own" % (g, ch)
        return merged
    finally:
        for ix in idxs:
            ix.close()


@pytest.mark.parametrize("case,G", [("config2", 2), ("config2", 3), ("zipf_small", 4), ("edge", 5), ("rand_1", 8),
                                    ("tiny360", 2)])
def test_logical_shards_match_reference(case, G):
    text, off, ids, expected = case_arrays(case)
    assert_same(shard_and_merge(text, off, G), expected, "%s G=%d" % (case, G))


@pytest.mark.parametrize("case,G", [("config2", 3), ("zipf_small", 8), ("edge", 4), ("tiny360", 5)])
def test_logical_shards_contiguous_ids(case, G):
    # contiguous id ranges per shard: the owners skip their id sort (ii_import)
    text, off, ids, expected = case_arrays(case)
    assert_same(shard_and_merge(text, off, G, contiguous=True), expected, "%s G=%d contiguous" % (case, G))
    assert_same(shard_and_merge(text, off, G, contiguous=True, balanced=True), expected,
                "%s G=%d contiguous balanced" % (case, G))


def test_logical_shards_zipf_vs_oracle():
    t, off = ii_ctypes.zipf_corpus(24_000_000, 300, 200_000, 33, threads=8)
    off = off.tolist()
    text = t.tobytes()
    exp = oracle_index(text, off, list(range(300)))
    assert_same(shard_and_merge(text, off, 4), exp, "zipf G=4")
    assert_same(shard_and_merge(text, off, 4, contiguous=True), exp, "zipf G=4 contiguous")
    # 7 owners merging 7 interleaved sources (3 merge-path rounds, the odd run carried), and ids spread
    # to 2^27: lexid + id bits exceed 32, so the owners merge u64 records
    assert_same(shard_and_merge(text, off, 7), exp, "zipf G=7")
    stride = 449_000
    exp_s = oracle_index(text, off, [f * stride for f in range(300)])
    assert_same(shard_and_merge(text, off, 7, id_stride=stride), exp_s, "zipf G=7, ids spread to 2^27")


def test_generic_sort_forms_vs_oracle():
    # the owners' dictionary and id sorts run as onesweep passes (run_sort_sweep); II_SORT_NO_SWEEP=1
    # keeps the histogram + scan + scatter passes: both forms must give the oracle's index
    t, off = ii_ctypes.zipf_corpus(6_000_000, 120, 60_000, 17, threads=8)
    off = off.tolist()
    text = t.tobytes()
    exp = oracle_index(text, off, list(range(120)))
    assert_same(shard_and_merge(text, off, 5), exp, "zipf G=5 onesweep sorts")
    os.environ["II_SORT_NO_SWEEP"] = "1"
    try:
        assert_same(shard_and_merge(text, off, 5), exp, "zipf G=5 histogram sorts")
    finally:
        del os.environ["II_SORT_NO_SWEEP"]


@pytest.mark.parametrize("case,G,balanced", [("config2", 3, False), ("zipf_small", 4, True)])
def test_export_after_reduce(case, G, balanced):
    # ii_reduce's compact token sort consumes the K1 records; an export plan / letter
    # load after it must index the shard again instead of re-sorting the consumed records
    text, off, ids, expected = case_arrays(case)
    assert_same(shard_and_merge(text, off, G, balanced=balanced, pre_reduce=True), expected,
                "%s G=%d export after reduce" % (case, G))


@pytest.mark.parametrize("case,G", [("config2", 3), ("zipf_small", 8), ("edge", 4)])
def test_logical_shards_balanced_letters(case, G):
    # histogram-balanced owners: same output, other ownership
    text, off, ids, expected = case_arrays(case)
    assert_same(shard_and_merge(text, off, G, balanced=True), expected, "%s G=%d balanced" % (case, G))


@pytest.mark.parametrize("nf", [100_000, 300_000])
def test_config5_shape_vs_oracle(nf):
    # BASELINE configs[4]'s shape at a size the oracle finishes in seconds: 10^5 / 3*10^5 files (far
    # beyond the reference's 360, main.c:8), vocabulary 10^7 (most words overflow the hot level), 1-3 KB
    # files.  The packed sort runs when W + F - 32 <= 11 (W word-id bits, F file-index bits): 17-bit
    # indices pack with the 22-bit word ids of this vocabulary under an 8-bit top digit, 19-bit ones
    # (configs[4]'s last rank) under a 9-bit one (k_msd_scatter_wide)
    t, off = ii_ctypes.zipf_corpus(300_000_000, nf, 10_000_000, 5, threads=16)
    ids = list(range(nf))
    exp = oracle_index(t, off, ids, threads=16)
    os.environ["II_TABLE_LOG2"] = "24"  # (a big table that holds the vocabulary: no regrow)
    try:
        with ii_ctypes.Index(0) as ix:
            # most words overflow the hot level: the first map probes two pairs (K1c resolves the
            # big-table words), and the next map of the context knows it and takes DeepProbe (bucket +
            # big home)
            for deep in (0, 1):
                ix.map_host(t, off.tolist(), ids)
                ix.reduce()
                assert_same(ix.letters(), exp, "300 MB, %d files, vocab 1e7, deep probe %d" % (nf, deep))
                st = ix.stats()
                assert st.deep_probe == deep and st.retries == 0
    finally:
        del os.environ["II_TABLE_LOG2"]
    with ii_ctypes.Index(0) as ix2:
        # a cold context sizes its big table by the input (2^22 slots for 300 MB): the vocabulary
        # overflows it, the map regrows the table and its retry takes DeepProbe
        ix2.map_host(t, off.tolist(), ids)
        ix2.reduce()
        assert_same(ix2.letters(), exp, "300 MB, %d files, vocab 1e7, cold context" % nf)
        assert ix2.stats().retries >= 1 and ix2.stats().deep_probe == 1
    assert st.words == sum(v.count(b"\n") for v in exp.values()) and st.words > 3_000_000
    assert st.sort_packed == 1 and st.sort_key_bits + st.sort_id_bits - 32 <= 11
    assert st.sort_id_bits == (nf - 1).bit_length()


def test_table_sized_by_last_vocabulary():
    # a context's next map sizes its big table by the last local reduce's vocabulary (shrink only,
    # ii_api.hip map_core): the second map of a small-vocabulary corpus takes a smaller table with no
    # regrow, and a larger vocabulary after it regrows (retries) and stays exact
    small = ii_ctypes.zipf_corpus(20_000_000, 64, 50_000, 3, threads=8)
    large = ii_ctypes.zipf_corpus(60_000_000, 64, 4_000_000, 4, threads=8)
    with ii_ctypes.Index(0) as ix:
        caps = []
        for t, off in (small, small, large):
            ids = list(range(len(off) - 1))
            ix.map_host(t, off.tolist(), ids)
            ix.reduce()
            assert_same(ix.letters(), oracle_index(t, off, ids), "table sizing, cap %d" % ix.stats().table_cap)
            caps.append((ix.stats().table_cap, ix.stats().retries))
    assert caps[1][0] < caps[0][0] and caps[1][1] == 0, caps
    assert caps[2][1] >= 1, caps


def test_large_vocab_vs_oracle_both_key_modes():
    # V ~ 2.2M distinct words (> 2^21): lexids need 22 bits, many words overflow
    # the hot level, so the word-id keys mix hot slots and big-table ranks;
    # the same corpus through lexid keys (the exchange path's sort) as well
    t, off = ii_ctypes.zipf_corpus(200_000_000, 500, 5_000_000, 17, threads=8)
    ids = list(range(500))
    exp = oracle_index(t, off, ids)
    ix = ii_ctypes.Index(0)
    try:
        for keys in ["wid", "lexid"]:
            os.environ["II_SORT_KEYS"] = keys
            ix.map_host(t, off.tolist(), ids)
            ix.reduce()
            assert_same(ix.letters(), exp, "vocab 5e6, %s keys" % keys)
        st = ix.stats()
        assert st.words > (1 << 21)
    finally:
        os.environ.pop("II_SORT_KEYS", None)
        ix.close()


def test_packed_sort_forms_vs_oracle():
    """The token sort's packed form (ii_prims.h "Packed token sort": MSD buckets
    of u32 records, two bucket-local onesweep passes) against the u64 form
    (II_PACKED_SORT=0) and the oracle, for dense ids and for ids spread to 19
    and 22 bits: the records carry shard-local file indices (10 bits for 700
    files, k_chunk_files), so every shape packs and K3 maps the indices back
    to the ids (k_uniq_sweep fmap) in both forms."""
    t, off = ii_ctypes.zipf_corpus(48_000_000, 700, 300_000, 23, threads=8)
    off = off.tolist()
    for ids, packed in [(list(range(700)), 1), ([700 * i for i in range(700)], 1), ([6007 * i for i in range(700)], 1)]:
        exp = oracle_index(t, off, ids)
        for env in [None, "0"]:
            if env is not None:
                os.environ["II_PACKED_SORT"] = env
            try:
                with ii_ctypes.Index(0) as ix:
                    ix.map_host(t, off, ids)
                    ix.reduce()
                    assert_same(ix.letters(), exp, "ids up to %d, II_PACKED_SORT=%s" % (ids[-1], env))
                    st = ix.stats()
                    assert st.sort_packed == (packed if env is None else 0)
                    assert st.sort_bytes > 0
            finally:
                os.environ.pop("II_PACKED_SORT", None)


@pytest.mark.parametrize("env", [{"II_PACKED_M": "9"}, {"II_PACKED_M": "10"}, {"II_PACKED_M": "11"},
                                 {"II_PACKED_M": "10", "II_SORT_KEYS": "lexid"}])
def test_wide_top_digit_vs_oracle(env):
    """The token sort's wide top digit (II_PACKED_M forces m top bits: the
    wide MSD split k_msd_scatter and k_sort0_compact's wide count row, the form
    configs[4]'s F = 19 share takes) with both key kinds, against the oracle;
    ids spread to 22 bits and 700 files of very different sizes."""
    t, off = ii_ctypes.zipf_corpus(48_000_000, 700, 3_000_000, 29, threads=8)
    off = off.tolist()
    ids = [6007 * i for i in range(700)]
    exp = oracle_index(t, off, ids)
    try:
        os.environ.update(env)
        with ii_ctypes.Index(0) as ix:
            for rep in range(2):  # (the second map reuses the grown buffers)
                ix.map_host(t, off, ids)
                ix.reduce()
                assert_same(ix.letters(), exp, "%s rep %d" % (env, rep))
            st = ix.stats()
            assert st.sort_packed == 1
            assert st.sort_bytes > 0
    finally:
        for k in env:
            os.environ.pop(k, None)


@pytest.mark.parametrize("env", [{}, {"II_PACKED_M": "10"}, {"II_PACKED_M": "11"}, {"II_SORT_KEYS": "lexid"}])
def test_first_pass_record_set_vs_oracle(env):
    """The first pass's record-set dedup (k_sort0_compact<.., kHashD>), the
    form small-file shares take (configs[4]'s rank 7: 3.9·10^3 tokens per
    file): 9000 files of ~3 KB against the oracle, the set chosen by itself
    and forced (II_S0_DEDUP=set) on 40 files of 1 MB, where live pairs
    outnumber the set's entries and full probe sequences keep records, and on
    the small files with 0-100 empty files after each (4.6·10^5 files: file
    indices jump past the set's 64-file window and its 128-file names).  On
    small files it must keep fewer records than the epoch bitmap."""
    small = ii_ctypes.zipf_corpus(27_000_000, 9000, 1_000_000, 53, threads=8)
    large = ii_ctypes.zipf_corpus(40_000_000, 40, 1_000_000, 59, threads=8)
    rng = random.Random(53)
    gappy = [0]
    for o in small[1].tolist()[1:]:
        gappy += [gappy[-1]] * rng.randint(0, 100) + [o]
    try:
        os.environ.update(env)
        for (t, off), force in ((small, None), (small, "bitmap"), (large, "set"), ((small[0], gappy), None)):
            off = off.tolist() if hasattr(off, "tolist") else off
            ids = list(range(len(off) - 1))
            exp = oracle_index(t, off, ids)
            if force:
                os.environ["II_S0_DEDUP"] = force
            try:
                with ii_ctypes.Index(0) as ix:
                    ix.map_host(t, off, ids)
                    ix.reduce()
                    assert_same(ix.letters(), exp, "%s II_S0_DEDUP=%s" % (env, force))
                    st = ix.stats()
                    assert st.sort_packed == 1
                    kept = st.sorted_records
            finally:
                os.environ.pop("II_S0_DEDUP", None)
            if force is None and off is gappy:
                continue
            if force is None:
                kept_set, pairs = kept, st.pairs
                assert kept_set <= 1.05 * pairs, (kept_set, pairs)
            elif force == "bitmap":
                assert kept_set < 0.9 * kept, (kept_set, kept)
    finally:
        for k in env:
            os.environ.pop(k, None)


def test_global_ids_of_a_share_stay_packed():
    """A rank's ii_partition share (main.c:300-323): 2000 files whose global ids
    span [0, 10^6) — the shape of a configs[4] rank.  The records carry 11-bit
    shard-local indices, so the packed sort runs; postings print the global ids."""
    t, off = ii_ctypes.zipf_corpus(40_000_000, 2000, 1_000_000, 41, threads=8)
    rng = random.Random(41)
    ids = sorted(rng.sample(range(1_000_000), 2000))
    exp = oracle_index(t, off, ids)
    with ii_ctypes.Index(0) as ix:
        ix.map_host(t, off.tolist(), ids)
        ix.reduce()
        assert_same(ix.letters(), exp, "global ids of a share")
        assert ix.stats().sort_packed == 1


@pytest.mark.parametrize("fm", ["1", "0"])
def test_first_pass_file_id_map_vs_oracle(fm):
    """The first pass maps shard-local file indices to id0s (k_sort0_compact's
    fmap, the record-set form; local_reduce takes it by itself from 65536
    files, the shape of configs[4]'s rank-7 share), so the sorted records
    carry 20-bit id0s and K3 gathers nothing.  II_S0_FMAP=1 forces it on 9000
    small files with sparse global ids in [0, 10^6), on the same files with
    0-100 empty files after each, on ids up to 2^31 (too many bits for the
    packed form: the local indices stay), and on the tiny shapes; =0 keeps the
    gather in K3.  All against the oracle."""
    t, off = ii_ctypes.zipf_corpus(27_000_000, 9000, 1_000_000, 67, threads=8)
    off = off.tolist()
    rng = random.Random(67)
    gappy = [0]
    for o in off[1:]:
        gappy += [gappy[-1]] * rng.randint(0, 100) + [o]
    cases = [(t, off, sorted(rng.sample(range(1_000_000), 9000)), 20),
             (t, gappy, sorted(rng.sample(range(1_000_000), len(gappy) - 1)), 20),
             (t, off, sorted(rng.sample(range(1 << 31), 9000)), None)]
    for files, ids in TINY:
        if ids[-1] - ids[0] + 1 != len(ids):  # (consecutive ids take the affine path)
            text = b"\n".join(files)
            o = [0]
            for i, f in enumerate(files):
                o.append(o[-1] + len(f) + (1 if i + 1 < len(files) else 0))
            cases.append((text, o, ids, None))
    os.environ["II_S0_FMAP"] = fm
    try:
        for n, (text, o, ids, bits) in enumerate(cases):
            with ii_ctypes.Index(0) as ix:
                ix.map_host(text, o, ids)
                ix.reduce()
                assert_same(ix.letters(), oracle_index(text, o, ids), "II_S0_FMAP=%s case %d" % (fm, n))
                st = ix.stats()
                if bits:
                    assert st.sort_packed == 1
                    want = bits if fm == "1" else max(1, (len(o) - 2).bit_length())
                    assert st.sort_id_bits == want, (n, st.sort_id_bits, want)
    finally:
        os.environ.pop("II_S0_FMAP", None)


def test_dictionary_in_stream_order_vs_oracle():
    """II_DICT_SIDE=0: the dictionary's lexicographic part in stream order
    instead of beside the token sort (its side-stream placement is what every
    other test runs) — the reference's golden cases and a Zipf corpus."""
    os.environ["II_DICT_SIDE"] = "0"
    try:
        with ii_ctypes.Index(0) as ix:
            for case in CASES:
                text, off, ids, expected = case_arrays(case)
                ix.map_host(text, off, ids)
                ix.reduce()
                assert_same(ix.letters(), expected, "II_DICT_SIDE=0 " + case)
            t, off = ii_ctypes.zipf_corpus(20_000_000, 300, 1_000_000, 71, threads=8)
            off = off.tolist()
            ids = list(range(len(off) - 1))
            ix.map_host(t, off, ids)
            ix.reduce()
            assert_same(ix.letters(), oracle_index(t, off, ids), "II_DICT_SIDE=0 zipf")
    finally:
        os.environ.pop("II_DICT_SIDE", None)


TINY = [
    ([b"a"], [0]),
    ([b"a b"], [4]),
    ([b"b a c"], [0]),
    ([b"", b"x"], [0, 1]),
    ([b"", b"", b""], [0, 1, 2]),
    ([b"zz zz zz"], [9]),
    ([b"", b"q", b""], [1, 5, 6]),
    ([b"y", b"y", b"y"], [0, 2, 3]),
    ([b"a", b"", b"b"], [0, 1, 2]),
]


@pytest.mark.parametrize("k", range(len(TINY)))
def test_tiny_shapes_vs_oracle(idx, k):
    """1-3 records, empty files, buckets left empty: the packed sort's geometry
    and K3 on the smallest inputs (the round-2 fault on 1-file / empty shards)."""
    files, ids = TINY[k]
    text = b"\n".join(files)
    off = [0]
    for i, f in enumerate(files):
        off.append(off[-1] + len(f) + (1 if i + 1 < len(files) else 0))
    idx.map_host(text, off, ids)
    idx.reduce()
    assert_same(idx.letters(), oracle_index(text, off, ids), "tiny %d" % k)


@pytest.mark.parametrize("k", [0, 2, 4, 6, 8])
def test_tiny_shapes_logical_shards(k):
    # the same through the exchange: shards of one file, of one empty file, and empty shards
    files, ids = TINY[k]
    text = b"\n".join(files)
    off = [0]
    for i, f in enumerate(files):
        off.append(off[-1] + len(f) + (1 if i + 1 < len(files) else 0))
    exp = oracle_index(text, off, list(range(len(files))))  # (shard_and_merge numbers files by list position)
    assert_same(shard_and_merge(text, off, 3), exp, "tiny %d G=3" % k)


@pytest.mark.parametrize("where", ["1", "sort", "sweep", "order"])
def test_k3_lookback_timeout_is_an_error(where):
    """K3 and the onesweep passes flag a look-back that never resolved
    (kLbTimeout) instead of hanging; the host must turn the flag into
    II_ERR_INTERNAL, not return the wrong pairs (II_TEST_LB_TIMEOUT=1 raises
    the flag after K3; =sort after the token sort, where K3 must skip its work:
    the records are out of place and their keys may lie past the word range;
    =sweep after a key + value sort that ran as onesweep passes — the owners'
    dictionary sort on the main stream, whose flag is read with the tie count
    before any kernel indexes by its values; =order after the final-order sort,
    checked with the letter offsets' readback)."""
    text, off, ids, _ = case_arrays("config2")
    os.environ["II_TEST_LB_TIMEOUT"] = where
    try:
        if where != "sweep":  # (one GPU: the dictionary sorts on the side stream, by histogram passes)
            with ii_ctypes.Index(0) as ix:
                ix.map_host(text, off, ids)
                with pytest.raises(ii_ctypes.IIError) as e:
                    ix.reduce()
                assert e.value.code == -7
        # through the exchange: the owners' dictionary sorts run as onesweep passes on the main stream
        # (run_sort_sweep), the owners' final order as histogram passes
        if where in ("sweep", "order"):
            with pytest.raises(ii_ctypes.IIError) as e:
                shard_and_merge(text, off, 3)
            assert e.value.code == -7
    finally:
        os.environ.pop("II_TEST_LB_TIMEOUT", None)


def test_long_word_collision_retry():
    """The exactness check of hashed (> 12-letter) keys runs on a side stream
    beside the reduce; its verdict is read with K3's results, and a collision
    re-runs map + reduce with a new seed.  II_TEST_COLLIDE=1 makes the first
    check of a context report one: same output, one more retry."""
    text, off, ids = long_variant_corpus(33)
    exp = oracle_index(text, off, ids)
    os.environ["II_TEST_COLLIDE"] = "1"
    try:
        with ii_ctypes.Index(0) as ix:
            ix.map_host(text, off, ids)
            ix.reduce()
            assert_same(ix.letters(), exp, "collision retry")
            assert ix.stats().retries >= 1
    finally:
        os.environ.pop("II_TEST_COLLIDE", None)


# ---------------------------------------------------------------- exactness of hashed (> 12-letter) keys
# II_TEST_LONG_KEY_BITS=0 makes the first map of a context hash every long
# word to ONE key, so two different long words really collide: the check
# (k_long_verify: raw bytes up to the last letter, else the letter walk) must
# flag it — a retry with full keys — and must not flag raw forms of one word
# (case, trailing punctuation, inner apostrophes, a leading bracket).
ONE_WORD = [b"internationalization", b"Internationalization.", b"INTERNATIONALIZATION,", b"(internationalization",
            b"inter'nationalization", b"internationalization!?", b"InTeRnAtIoNaLiZaTiOn;"]
COLLIDE_CASES = {
    "one_word": (ONE_WORD, False),
    "two_words": (ONE_WORD + [b"characterizations"], True),
    "plural": (ONE_WORD + [b"internationalizations."], True),   # one more letter after the shared ones
    "after_punct": (ONE_WORD + [b"internationalization.x"], True),  # a letter after trailing punctuation
}


def collide_corpus(forms, nfiles=24, seed=7):
    rng = random.Random(seed)
    short = [b"the", b"of", b"and", b"Word", b"a", b"zebra", b"it's"]
    text = bytearray()
    off = [0]
    for f in range(nfiles):
        toks = [rng.choice(forms) if rng.random() < 0.3 else rng.choice(short) for _ in range(400 + 37 * f)]
        toks[f % len(toks)] = forms[f % len(forms)]  # every form occurs
        text += b" ".join(toks) + b"\n"
        off.append(len(text))
    return bytes(text), off, list(range(nfiles))


@pytest.mark.parametrize("case", sorted(COLLIDE_CASES))
def test_long_key_collisions_detected(case):
    forms, collide = COLLIDE_CASES[case]
    text, off, ids = collide_corpus(forms)
    exp = oracle_index(text, off, ids)
    os.environ["II_TEST_LONG_KEY_BITS"] = "0"
    try:
        with ii_ctypes.Index(0) as ix:
            ix.map_host(text, off, ids)
            ix.reduce()
            assert_same(ix.letters(), exp, "long-key collisions %s" % case)
            retries = ix.stats().retries
        assert (retries >= 1) == collide, "%s: %d map retries" % (case, retries)
        # the same through G = 3 logical shards: the owners' import maps the received words densely
        got = shard_and_merge(text, off, 3)
        assert_same(got, exp, "long-key collisions %s, 3 shards" % case)
    finally:
        os.environ.pop("II_TEST_LONG_KEY_BITS", None)
