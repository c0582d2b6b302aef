"""Multi-GPU exchange of the inverted-index builder.

One process per GPU (torch.distributed; backend "nccl" is RCCL on ROCm).
Every rank maps its own shard of files, reduces it locally to distinct
(word, file) pairs, then ONE all-to-allv routes each first-letter range to the
rank that owns it — the reference's reducer-to-letter assignment
(main.c:129-130) with R = world size — and the owner merges and formats.

The byte movement is backend-agnostic (RCCL for device tensors, gloo for CPU
tensors in the CPU tests); segment packing / merging is libii.so's
ii_export / ii_import.
"""
import torch
import torch.distributed as dist


def prefix(sizes):
    off, acc = [], 0
    for s in sizes:
        off.append(acc)
        acc += s
    return off, acc


def _host_staged(group):
    """gloo moves host tensors only: device buffers are staged through host
    memory (CPU tests and N>1 rehearsals on fewer GPUs, never measurements)."""
    return dist.get_backend(group) == "gloo"


def alltoallv_bytes(send, send_sizes, group=None):
    """Exchange variable-size byte segments: send[off_r : off_r + send_sizes[r]]
    goes to rank r.  Returns (recv, recv_sizes) with the segments from ranks
    0..world-1 back to back.  One count exchange + one all_to_all_single."""
    world = dist.get_world_size(group)
    out_dev = send.device
    if _host_staged(group) and send.is_cuda:
        send = send.cpu()
    dev = send.device
    cnt = torch.tensor(send_sizes, dtype=torch.int64, device=dev)
    rcnt = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_to_all_single(rcnt, cnt, group=group)
    recv_sizes = [int(x) for x in rcnt.tolist()]
    recv = torch.empty(sum(recv_sizes), dtype=torch.uint8, device=dev)
    dist.all_to_all_single(recv, send, output_split_sizes=recv_sizes, input_split_sizes=list(send_sizes),
                           group=group)
    return recv.to(out_dev), recv_sizes


def owner_ranges(idx_loads, world):
    """Histogram-balanced letter ranges from the per-letter
    pair counts summed over all shards."""
    import ii_ctypes
    total = [sum(col) for col in zip(*idx_loads)]
    return ii_ctypes.balanced_letters(total, world)


def exchange_and_reduce(idx, id_bound, group=None, copy_text=False, balanced=False, on_local=None):
    """Local reduce -> export -> all-to-allv -> import -> order + format.
    After it, idx holds the final text of this rank's letters — the
    reference's reducer map ii_reducer_letters(rank, world) (main.c:129-130),
    or with balanced=True the histogram-balanced ranges every rank derives from
    the same all-reduced letter loads; the other letters are empty.  Returns
    (recv_sizes, (letter_lo, letter_hi)).  on_local(idx), if given, runs once the
    local map + reduce + export are done (before the import maps the received
    words in the same context)."""
    import ii_ctypes
    world = dist.get_world_size(group)
    if balanced:
        load = torch.tensor(idx.letter_load(), dtype=torch.int64, device="cpu" if _host_staged(group) else "cuda")
        dist.all_reduce(load, group=group)
        lo, hi = ii_ctypes.balanced_letters([int(x) for x in load.tolist()], world)
    else:
        lo, hi = zip(*[ii_ctypes.reducer_letters(r, world) for r in range(world)])
        lo, hi = list(lo), list(hi)
    sizes = idx.export_plan_ranges(lo, hi)
    send_off, total = prefix(sizes)
    send = torch.empty(max(total, 8), dtype=torch.uint8, device="cuda")
    idx.export(world, send.data_ptr(), send_off)
    if on_local is not None:
        on_local(idx)
    recv, recv_sizes = alltoallv_bytes(send[:total], sizes, group)
    recv_off, _ = prefix(recv_sizes)
    if recv.numel() == 0:
        recv = torch.empty(8, dtype=torch.uint8, device="cuda")
    # the collective (or gloo's host -> device copy) was queued on torch's
    # current stream; libii reads recv on its own stream, so the bytes must
    # have landed before ii_import starts
    torch.cuda.current_stream().synchronize()
    idx.import_(world, recv.data_ptr(), recv_off, id_bound)
    idx.reduce(copy_text=copy_text)
    return recv_sizes, (lo, hi)


def logical_shards_reduce(idxs, id_bound, copy_text=True, balanced=False):
    """The same exchange among G contexts on ONE device (no collective): the
    "G logical shards on 1 device" mode of SURVEY.md §4 that exercises the
    export/import logic when fewer GPUs are present.  Returns the owners'
    (letter_lo, letter_hi)."""
    import ii_ctypes
    G = len(idxs)
    if balanced:
        lo, hi = owner_ranges([ix.letter_load() for ix in idxs], G)
    else:
        lo, hi = zip(*[ii_ctypes.reducer_letters(r, G) for r in range(G)])
        lo, hi = list(lo), list(hi)
    sends = []
    for ix in idxs:
        sizes = ix.export_plan_ranges(lo, hi)
        off, total = prefix(sizes)
        buf = torch.empty(max(total, 8), dtype=torch.uint8, device="cuda")
        ix.export(G, buf.data_ptr(), off)
        sends.append((buf, sizes, off))
    for d, ix in enumerate(idxs):
        parts = [s[0][s[2][d]:s[2][d] + s[1][d]] for s in sends]
        recv_sizes = [s[1][d] for s in sends]
        recv = torch.cat(parts) if sum(recv_sizes) else torch.empty(8, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        ix.import_(G, recv.data_ptr(), prefix(recv_sizes)[0], id_bound)
        ix.reduce(copy_text=copy_text)
    return lo, hi
