"""CPU, world_size 2 (gloo): the N>1 exchange path's collective layer —
count exchange + all-to-allv of byte segments, as bench.py runs it over
RCCL on device tensors."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import ii_dist


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(100 + rank)
        results = []
        for trial in range(4):
            # segment for destination d from rank r: bytes (r, d, trial, i) pattern
            sizes = [int(torch.randint(0, 40, (1,), generator=g)) * 8 if trial != 1 else 0 for _ in range(world)]
            parts = [torch.tensor([(rank * 31 + d * 7 + trial + i) % 251 for i in range(sizes[d])], dtype=torch.uint8)
                     for d in range(world)]
            send = torch.cat(parts) if sum(sizes) else torch.empty(0, dtype=torch.uint8)
            recv, rsizes = ii_dist.alltoallv_bytes(send, sizes)
            off = 0
            ok = True
            for s in range(world):
                seg = recv[off:off + rsizes[s]].tolist()
                exp = [(s * 31 + rank * 7 + trial + i) % 251 for i in range(rsizes[s])]
                ok &= seg == exp
                off += rsizes[s]
            results.append((ok, rsizes))
        q.put((rank, results))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_alltoallv_bytes_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # sizes seen by rank d from rank s equal what s sent to d
    for d in range(world):
        for ok, _ in out[d]:
            assert ok
    for t in range(4):
        for d in range(world):
            for s in range(world):
                assert out[d][t][1][s] % 8 == 0


def test_prefix():
    assert ii_dist.prefix([3, 0, 5]) == ([0, 3, 3], 8)


def _balanced_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import ii_ctypes
        g = torch.Generator().manual_seed(7 + rank)
        load = torch.randint(0, 10 ** 6, (26,), generator=g, dtype=torch.int64)
        total = load.clone()
        dist.all_reduce(total)
        q.put((rank, ii_ctypes.balanced_letters([int(x) for x in total.tolist()], world),
               [int(x) for x in total.tolist()]))
    finally:
        dist.destroy_process_group()


def test_balanced_owner_ranges_agree_gloo():
    # every rank derives the same histogram-balanced owner ranges from the
    # all-reduced letter loads (the N>1 exchange of bench.py --gpus N)
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_balanced_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict((r, (rng, tot)) for r, rng, tot in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert out[0] == out[1]
    (lo, hi), tot = out[0]
    assert lo[0] == 0 and hi[-1] == 26 and lo[1] == hi[0]
