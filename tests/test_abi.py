"""CPU: the C-ABI library loads, exports every entry point include/ii.h
declares, and its pure-host helpers match the reference's arithmetic."""
import ctypes
import os
import re

import pytest

import ii_ctypes
from conftest import PKG, REPO


def declared_functions():
    src = open(os.path.join(REPO, "include", "ii.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ii_[a-z_]+)\s*\(", src)))


def test_header_declares_expected_entry_points():
    fns = declared_functions()
    for f in ["ii_open", "ii_close", "ii_strerror", "ii_map_files", "ii_map_host", "ii_map_device", "ii_reduce",
              "ii_letter_text", "ii_get_stats", "ii_device_text", "ii_reducer_letters", "ii_partition"]:
        assert f in fns


def test_library_exports_every_declared_symbol():
    L = ctypes.CDLL(os.path.join(PKG, "libii.so"))
    missing = [f for f in declared_functions() if not hasattr(L, f)]
    assert not missing, missing


def test_strerror():
    L = ii_ctypes.lib()
    assert L.ii_strerror(0) == b"ok"
    assert L.ii_strerror(-6).startswith(b"device text")


def test_reducer_letters_matches_main_c_129_130():
    for R in range(1, 40):
        covered = []
        for r in range(R):
            lo, hi = ii_ctypes.reducer_letters(r, R)
            exp_lo = (26 // R) * r
            exp_hi = 26 if r == R - 1 else (26 // R) * (r + 1)
            assert (lo, hi) == (exp_lo, exp_hi)
            covered += list(range(lo, hi))
        assert sorted(covered) == list(range(26))
    with pytest.raises(ii_ctypes.IIError):
        ii_ctypes.reducer_letters(0, 0)


def ref_partition(sizes, M):
    """main.c:300-323 restated (stable size-desc order)."""
    order = sorted(range(len(sizes)), key=lambda i: (-sizes[i], i))
    per = sum(sizes) // M
    start, end = [None] * M, [None] * M
    cur, cum = 0, 0
    start[0] = 0
    for i in range(len(sizes)):
        cum += sizes[order[i]]
        if cum >= per and cur < M - 1:
            end[cur] = i
            cur += 1
            start[cur] = i + 1
            cum = 0
    end[cur] = len(sizes) - 1
    return order, start, end, cur


def test_partition_matches_reference_config2():
    # config 2, M=8 -> [0,11) [11,27) [27,47) [47,71) [71,100) [100,137) [137,191) [191,355)
    from conftest import case_arrays
    _, off, _, _ = case_arrays("config2")
    sizes = [off[i + 1] - off[i] for i in range(len(off) - 1)]
    order, sb, se = ii_ctypes.partition(sizes, 8)
    assert list(zip(sb, se)) == [(0, 11), (11, 27), (27, 47), (47, 71), (71, 100), (100, 137), (137, 191),
                                 (191, 355)]
    assert order == sorted(range(len(sizes)), key=lambda i: (-sizes[i], i))


@pytest.mark.parametrize("M", [1, 2, 3, 5, 8, 13, 64])
def test_partition_random(M):
    import random
    rng = random.Random(M)
    for _ in range(20):
        n = rng.randint(0, 50)
        sizes = [rng.choice([0, 1, 10, 100, 1000, rng.randint(0, 5000)]) for _ in range(n)]
        order, sb, se = ii_ctypes.partition(sizes, M)
        rorder, rs, re_, cur = ref_partition(sizes, M)
        assert order == rorder
        for m in range(cur + 1):
            assert sb[m] == rs[m] and se[m] == re_[m] + 1
        for m in range(cur + 1, M):  # undefined in the reference: empty here
            assert sb[m] == se[m]
        covered = [order[i] for m in range(M) for i in range(sb[m], se[m])]
        assert sorted(covered) == list(range(n))


def test_open_without_gpu_reports_nodev():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(ii_ctypes.IIError) as e:
        ii_ctypes.Index(0)
    assert e.value.code == -8


def _brute_best(w, parts):
    """Smallest possible largest part of a contiguous split of w into parts."""
    import functools

    @functools.lru_cache(None)
    def f(i, k):
        if i == len(w):
            return 0
        if k == 1:
            return sum(w[i:])
        return min(max(sum(w[i:j]), f(j, k - 1)) for j in range(i, len(w) + 1))
    return f(0, parts)


@pytest.mark.parametrize("parts", [1, 2, 3, 5, 8])
def test_balanced_letters_optimal_and_contiguous(parts):
    import random
    rng = random.Random(parts)
    for trial in range(12):
        w = [rng.choice([0, 0, 1, 5, 100, rng.randint(0, 10 ** 6)]) for _ in range(26)]
        lo, hi = ii_ctypes.balanced_letters(w, parts)
        assert lo[0] == 0 and hi[-1] == 26
        for r in range(parts):
            assert lo[r] <= hi[r]
            if r:
                assert lo[r] == hi[r - 1]
        largest = max(sum(w[lo[r]:hi[r]]) for r in range(parts))
        if parts <= 3:
            assert largest == _brute_best(tuple(w), parts)
        # never worse than the reference's 26/parts split (main.c:129-130)
        ref = max(sum(w[a:b]) for a, b in (ii_ctypes.reducer_letters(r, parts) for r in range(parts)))
        assert largest <= ref
