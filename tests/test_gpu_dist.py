"""GPU, world size 2 with gloo, both ranks on cuda:0 (and world size 1 over
RCCL): the N > 1 product path end to end — files sharded by the reference's size heuristic (ii_partition,
main.c:300-323), map + local reduce per rank, ii_dist.exchange_and_reduce
(export -> all-to-allv -> import -> order + format), and the owners' letters
merged — against the reference goldens; and bench.py --gpus 2 itself."""
import hashlib
import json
import os
import socket
import subprocess
import sys

import pytest
import torch.multiprocessing as mp

from conftest import REPO, case_arrays

pytestmark = pytest.mark.gpu
LETTERS = "abcdefghijklmnopqrstuvwxyz"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, cases, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    import ii_ctypes
    import ii_dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = []
    try:
        ix = ii_ctypes.Index(0)
        for case, balanced in cases:
            text, off, _, _ = case_arrays(case)
            n = len(off) - 1
            order, sb, se = ii_ctypes.partition([off[i + 1] - off[i] for i in range(n)], world)
            fids = sorted(order[sb[rank]:se[rank]])
            t = b"".join(text[off[f]:off[f + 1]] for f in fids)
            o = [0]
            for f in fids:
                o.append(o[-1] + off[f + 1] - off[f])
            for rep in range(2):  # twice: the second exchange reuses the first one's freed buffers
                ix.map_host(t, o, fids)
                _, (lo, hi) = ii_dist.exchange_and_reduce(ix, n, copy_text=True, balanced=balanced)
                got = ix.letters()
                out.append((case, balanced, rep, lo[rank], hi[rank], got))
        ix.close()
        q.put((rank, out, None))
    except Exception as e:  # noqa: BLE001
        q.put((rank, out, repr(e)))
    finally:
        dist.destroy_process_group()


def test_exchange_and_reduce_gloo_world2():
    cases = [(c, b) for c in ["config2", "zipf_small", "edge"] for b in (False, True)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, cases, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (o, err)) for r, o, err in (q.get(timeout=240) for _ in range(2)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(2):
        assert res[r][1] is None, res[r][1]
    for i, (case, balanced) in enumerate(cases):
        _, _, _, expected = case_arrays(case)
        for rep in range(2):
            merged = {}
            for r in range(2):
                c, b, rp, lo, hi, got = res[r][0][2 * i + rep]
                assert (c, b, rp) == (case, balanced, rep)
                for l in range(26):
                    if lo <= l < hi:
                        merged[LETTERS[l]] = got[LETTERS[l]]
                    else:
                        assert got[LETTERS[l]] == b"", "rank %d holds letter %s it does not own" % (r, LETTERS[l])
            for l in LETTERS:
                assert merged[l] == expected[l], "%s balanced=%s rep %d: letter %s differs" % (case, balanced, rep, l)


def _rank_nccl(port, cases, q):
    """World size 1 under backend "nccl" (RCCL): ii_dist's count exchange and
    payload all_to_all_single run as real RCCL collectives on device tensors."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    import ii_ctypes
    import ii_dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    out = []
    try:
        assert dist.get_backend() == "nccl" and not ii_dist._host_staged(None)
        with ii_ctypes.Index(0) as ix:
            for case, balanced in cases:
                text, off, ids, _ = case_arrays(case)
                ix.map_host(text, off, ids)
                recv_sizes, (lo, hi) = ii_dist.exchange_and_reduce(ix, len(ids), copy_text=True, balanced=balanced)
                out.append((case, balanced, lo[0], hi[0], recv_sizes, ix.letters()))
        q.put((out, None))
    except Exception as e:  # noqa: BLE001
        q.put((out, repr(e)))
    finally:
        dist.destroy_process_group()


def test_exchange_and_reduce_nccl_world1():
    """ii_dist.exchange_and_reduce over RCCL on the one-GPU box: one rank owns
    all 26 letters (main.c:129-130 with R = 1), its segment goes through RCCL's
    all_to_all_single to itself, and the imported index must equal the
    reference's goldens."""
    cases = [(c, b) for c in ["config1", "config2", "edge", "zipf_small"] for b in (False, True)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rank_nccl, args=(_free_port(), cases, q))
    p.start()
    out, err = q.get(timeout=240)
    p.join(timeout=60)
    assert err is None, err
    assert p.exitcode == 0
    assert len(out) == len(cases)
    for (case, balanced), (c, b, lo, hi, recv_sizes, got) in zip(cases, out):
        _, _, _, expected = case_arrays(case)
        assert (c, b, lo, hi) == (case, balanced, 0, 26)
        assert len(recv_sizes) == 1 and recv_sizes[0] > 0
        for l in LETTERS:
            assert got[l] == expected[l], "%s balanced=%s over RCCL: letter %s differs" % (case, balanced, l)


def test_bench_two_ranks_gloo_strong_scaling():
    # bench.py --gpus 2 launches its own ranks (torch.distributed.run), shards ONE corpus by ii_partition
    # and reports n_gpus 2; its per-letter hashes must equal the oracle's on the same corpus
    import ii_ctypes
    from oracle_py import oracle_index
    nb, nf, vocab, seed = 60_000_000, 400, 200_000, 3
    env = dict(os.environ, II_DIST_BACKEND="gloo")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                        "--bytes", str(nb), "--files", str(nf), "--vocab", str(vocab), "--seed", str(seed),
                        "--no-cpu-baseline", "--io-bytes", "0"], cwd=REPO, env=env, capture_output=True, timeout=300)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    line = json.loads([x for x in r.stdout.decode().splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["scaling"] == "strong"
    # the N > 1 line reports rank 0's own map + local reduce (a 4-rank line once printed zeros)
    assert line["counts"]["pairs"] > 0 and line["counts"]["sort_passes"] > 0, line["counts"]
    assert line["roofline_sort_phase"]["frac"] > 0, line["roofline_sort_phase"]
    assert line["roofline"]["frac"] > 0, line["roofline"]
    t, off = ii_ctypes.zipf_corpus(nb, nf, vocab, seed, threads=8)
    exp = oracle_index(t, off, list(range(nf)), threads=8)
    assert line["output_letter_sha256"] == {l: hashlib.sha256(exp[l]).hexdigest() for l in LETTERS}
