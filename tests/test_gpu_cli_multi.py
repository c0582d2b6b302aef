"""GPU: the drop-in CLI over several GPU contexts (II_GPUS=G):
files sharded by the reference's size heuristic (main.c:300-323), one host
pthread per context, letter ranges exchanged (the reference's reducer map
with R = G, main.c:129-130, or II_LETTER_SPLIT=balanced) — against every
reference golden.  With one visible device the G contexts share it and the
segments move by device copies; on a node with >= G devices the same code
path moves them with grouped RCCL send / recv."""
import hashlib
import os
import subprocess
import tempfile

import pytest

from conftest import CASES, PKG, materialize, partials_meta
from test_gpu_parity import LETTERS, assert_same

pytestmark = pytest.mark.gpu


def run_cli(case, M, R, env_extra):
    with tempfile.TemporaryDirectory() as td:
        _, _, expected = materialize(case, td)
        env = dict(os.environ, **env_extra)
        r = subprocess.run([os.path.join(PKG, "ii_index"), str(M), str(R), "list.txt"], cwd=td, capture_output=True,
                           timeout=180, env=env)
        assert r.returncode == 0, r.stderr.decode()
        got = {l: open(os.path.join(td, l + ".txt"), "rb").read() for l in LETTERS}
        parts = {l: open(os.path.join(td, "partial_%s.txt" % l), "rb").read() for l in LETTERS} \
            if env_extra.get("II_PARTIAL_FILES") == "1" else None
        return got, expected, parts, r


@pytest.mark.parametrize("case", CASES)
def test_cli_three_gpus_matches_reference(case):
    got, expected, _, r = run_cli(case, 4, 5, {"II_GPUS": "3"})
    assert_same(got, expected, "%s II_GPUS=3" % case)
    assert r.stdout.decode().count("REDUCER\n") == 5


@pytest.mark.parametrize("case,G,split", [("config2", 2, "reference"), ("config2", 8, "balanced"),
                                          ("zipf_small", 5, "balanced"), ("edge", 7, "reference"),
                                          ("tiny360", 4, "balanced"), ("rand_2", 26, "reference")])
def test_cli_gpu_counts_and_letter_splits(case, G, split):
    got, expected, _, _ = run_cli(case, 3, 26, {"II_GPUS": str(G), "II_LETTER_SPLIT": split})
    assert_same(got, expected, "%s II_GPUS=%d %s" % (case, G, split))


@pytest.mark.parametrize("case", ["config1", "edge", "zipf_small"])
def test_cli_multi_gpu_partial_files(case):
    # M = 1: the reference's own partial files, byte for byte, although the files live on 3 contexts
    got, expected, parts, _ = run_cli(case, 1, 2, {"II_GPUS": "3", "II_PARTIAL_FILES": "1"})
    assert_same(got, expected, case)
    meta = partials_meta()[case]
    for l in LETTERS:
        assert hashlib.sha256(parts[l]).hexdigest() == meta[l]["sha256"], "%s partial_%s.txt differs" % (case, l)


@pytest.mark.parametrize("case,G", [("config2", 3), ("zipf_small", 4), ("edge", 5)])
@pytest.mark.parametrize("env", [{}, {"II_IMPORT_ID_SORT": "1"}, {"II_IMPORT_ID_SORT": "64"}])
def test_cli_owner_sort_forms(case, G, env):
    # the owners' merge of the received pairs: interleaved ids from the size heuristic take pairwise
    # merge-path rounds (k_merge_partition / k_merge_tiles; 2 rounds at G = 3, 3 at G = 5);
    # II_IMPORT_ID_SORT=1 radix-sorts instead (u32 records), =64 sorts the u64 records — byte-identical
    got, expected, _, _ = run_cli(case, 3, 26, dict({"II_GPUS": str(G), "II_LETTER_SPLIT": "balanced"}, **env))
    assert_same(got, expected, "%s II_GPUS=%d %s" % (case, G, env))


@pytest.mark.parametrize("G", [1, 3])
def test_cli_metrics_line(G):
    """II_METRICS=path: the CLI appends one JSON line per run whose
    counts agree with the output it wrote."""
    import json
    with tempfile.TemporaryDirectory() as md:
        path = os.path.join(md, "m.jsonl")
        got, expected, _, _ = run_cli("config2", 4, 26, {"II_GPUS": str(G), "II_METRICS": path})
        assert_same(got, expected, "metrics run G=%d" % G)
        lines = open(path).read().splitlines()
    assert len(lines) == 1
    m = json.loads(lines[0])
    assert m["ok"] is True and m["gpus"] == G and m["files"] == 355 and m["bytes"] == 5756194
    assert m["words"] == sum(v.count(b"\n") for v in expected.values())
    assert m["pairs"] == sum(v.count(b" ") + v.count(b"\n") for v in expected.values())
    assert m["out_bytes"] == sum(len(v) for v in expected.values())
    assert m["wall_ms"] > 0


@pytest.mark.parametrize("case,split", [(c, "reference") for c in CASES] + [("config2", "balanced")])
def test_cli_rccl_one_rank_matches_reference(case, split):
    """The CLI's RCCL branch (host/ii_index.c receive(): ncclCommInitRank from
    one ncclGetUniqueId, one grouped ncclSend / ncclRecv round) on a one-GPU
    box: II_TEST_MULTI=1 sends G = 1 down the multi-context path, so the one
    context exports its letter segment, moves it to itself through a real
    one-rank communicator and imports it (main.c:129-130 with R = 1) —
    byte-identical to the reference's goldens."""
    got, expected, _, r = run_cli(case, 2, 26, {"II_GPUS": "1", "II_TEST_MULTI": "1", "II_LETTER_SPLIT": split})
    assert_same(got, expected, "%s RCCL one rank %s" % (case, split))
    assert r.stdout.decode().count("REDUCER\n") == 26


def test_cli_failed_owner_exits_promptly():
    """II_TEST_FAIL=merge:3 with II_GPUS=5: owner 3's import fails and the other
    owners' threads block, as behind a faulted device (round 3's post-fault
    hang): the CLI must report the error and exit non-zero within
    15 s, making no further HIP call."""
    import time
    with tempfile.TemporaryDirectory() as td:
        materialize("config2", td)
        env = dict(os.environ, II_GPUS="5", II_TEST_FAIL="merge:3")
        t0 = time.time()
        r = subprocess.run([os.path.join(PKG, "ii_index"), "3", "26", "list.txt"], cwd=td, capture_output=True,
                           timeout=120, env=env)
        dt = time.time() - t0
    err = r.stderr.decode(errors="replace")
    assert r.returncode == 1, err
    assert "internal consistency check failed" in err, err
    assert dt < 15.0, dt
