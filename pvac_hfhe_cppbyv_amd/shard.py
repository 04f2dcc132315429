"""Host-side sharding of independent cipher pairs over ranks (one process per GPU).

The hot path has no exchange step: every pair is independent, so rank r owns the
contiguous global pair range shard_range(N, world, r) and generates / processes it alone. Inputs
and nonces are keyed by the GLOBAL pair index (Engine.gen_fresh(first_index=...),
Engine.fill_nonces(first_index=...)), so the union of the shards equals a single-GPU run. The only
collective is the all_gather of per-rank output-edge totals, which places each shard in the global
(sharded) CSR of the result — BASELINE cfg 5's "gather-only". Works on any torch.distributed backend
(RCCL "nccl" on the GPU node, "gloo" in CPU tests).

Self-check of a sharded run (bench.py): every rank folds its per-pair output digests into one
order-independent, index-keyed sum (shard_digest), so the sum over ranks equals the digest of one
single-GPU run of the whole global batch; ranks all_gather those sums and the digests of a window of
their pairs, which rank 0 recomputes from the global pair indices (all_gather_u64).
"""
from __future__ import annotations


def shard_range(n_total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous balanced split of [0, n_total): (start, count) of `rank`."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(n_total, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def exclusive_offsets(counts):
    out, run = [], 0
    for c in counts:
        out.append(run)
        run += int(c)
    return out, run


def global_edge_offsets(local_total: int, device=None):
    """All ranks' output-edge totals (one all_gather of 8 bytes per rank) -> (this rank's offset in
    the global edge CSR, grand total, per-rank totals). No process group: (0, local_total, [local]).
    A one-rank group still issues the collective (bench.py PVAC_BENCH_DIST=1: RCCL on one GPU)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return 0, int(local_total), [int(local_total)]
    world, rank = dist.get_world_size(), dist.get_rank()
    if dist.get_backend() == "gloo":
        device = "cpu"
    mine = torch.tensor([int(local_total)], dtype=torch.int64, device=device)
    allt = torch.zeros(world, dtype=torch.int64, device=device)
    dist.all_gather_into_tensor(allt, mine)
    per = [int(x) for x in allt.cpu().tolist()]
    offs, total = exclusive_offsets(per)
    return offs[rank], total, per


def max_over_ranks(value: float, device=None) -> float:
    """Timing reduction of the driver contract (max over ranks)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return float(value)
    if dist.get_backend() == "gloo":
        device = "cpu"
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


_M64 = (1 << 64) - 1


def shard_digest(pair_digests, first_index: int) -> int:
    """sum_i mix(d_i, first_index + i) mod 2^64 over a shard's per-pair digests (numpy u64): keyed by
    the GLOBAL pair index and additive over disjoint shards."""
    import numpy as np
    d = np.ascontiguousarray(pair_digests, dtype=np.uint64)
    with np.errstate(over="ignore"):
        g = np.arange(first_index, first_index + len(d), dtype=np.uint64)
        z = d + g * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
        return int(z.sum(dtype=np.uint64))


def combine_digests(ds) -> int:
    return sum(int(x) for x in ds) & _M64


def all_gather_u64(values, device=None):
    """all_gather of an equal-length u64 vector from every rank -> list (per rank) of numpy u64.
    No process group: [values]."""
    import numpy as np
    import torch
    import torch.distributed as dist
    v = np.ascontiguousarray(values, dtype=np.uint64)
    if not (dist.is_available() and dist.is_initialized()):
        return [v.copy()]
    world = dist.get_world_size()
    if dist.get_backend() == "gloo":
        device = "cpu"
    mine = torch.from_numpy(v.view(np.int64).copy()).to(device)
    allt = torch.zeros(world * len(v), dtype=torch.int64, device=device)
    dist.all_gather_into_tensor(allt, mine)
    a = allt.cpu().numpy().view(np.uint64)
    return [a[r * len(v):(r + 1) * len(v)].copy() for r in range(world)]


def compact_rows(X, n=None):
    """The used rows of a (capacity-padded) DeviceBatch as flat int64 tensors on its device:
    (l_cnt, e_cnt, layers [sum l_cnt, 5], meta, w_lo, w_hi, sigma or None), ciphers in order."""
    import torch
    n = X.n if n is None else n

    def rows(off, cnt):
        cnt = cnt[:n].to(torch.int64)
        start = torch.repeat_interleave(off[:n].to(torch.int64) - (torch.cumsum(cnt, 0) - cnt), cnt)
        return start + torch.arange(start.numel(), device=start.device)

    li, ei = rows(X.l_off, X.l_cnt), rows(X.e_off, X.e_cnt)
    sig = None if X.sigma is None else X.sigma[ei]
    return (X.l_cnt[:n].to(torch.int64), X.e_cnt[:n].to(torch.int64), X.layers[li], X.meta[ei], X.w_lo[ei], X.w_hi[ei],
            sig)


def gather_batch(X, n=None, device=None):
    """Result concat of a sharded run for SMALL batches (BASELINE cfg 5's optional gather over xGMI):
    every rank's ciphers (compacted, in rank order = global pair order) on every rank, as one
    DeviceBatch with a compact CSR. Two collectives: an all_gather of the per-rank row counts, then
    one all_gather_into_tensor of each rank's payload padded to the largest (RCCL on device
    tensors; gloo on CPU copies). No process group: the compacted X itself. At cfg 5's sizes
    (~490 GB of output) this is not meant to run: results stay sharded (global_edge_offsets)."""
    import torch
    import torch.distributed as dist
    from . import DeviceBatch
    lc, ec, lay, meta, wlo, whi, sig = compact_rows(X, n)
    on = dist.is_available() and dist.is_initialized()
    dev = lc.device
    if on and dist.get_backend() == "gloo":
        dev = torch.device("cpu")
    elif device is not None:
        dev = torch.device(device)
    sw = 0 if sig is None else int(sig.shape[1])
    parts = [lc, ec, lay.reshape(-1), meta, wlo, whi] + ([sig.reshape(-1)] if sw else [])
    payload = torch.cat([p.to(dev).reshape(-1) for p in parts])
    head = torch.tensor([lc.numel(), int(lay.shape[0]), int(meta.numel()), payload.numel()], dtype=torch.int64,
                        device=dev)
    if on:
        world = dist.get_world_size()
        heads = torch.zeros(world * 4, dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(heads, head)
        heads = heads.reshape(world, 4).cpu().tolist()
        width = max(h[3] for h in heads)
        buf = torch.zeros(width, dtype=torch.int64, device=dev)
        buf[:payload.numel()] = payload
        allp = torch.zeros(world * width, dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(allp, buf)
        chunks = [allp[r * width:r * width + heads[r][3]] for r in range(world)]
    else:
        heads, chunks = [head.cpu().tolist()], [payload]
    fields = [[] for _ in range(7)]
    for (nc, nl, ne, _), p in zip(heads, chunks):
        sizes = [nc, nc, 5 * nl, ne, ne, ne] + ([ne * sw] if sw else [])
        segs = torch.split(p, sizes)
        for k, t in enumerate(segs):
            fields[k].append(t)
    cat = [torch.cat(f) if f else None for f in fields]
    l_cnt, e_cnt = cat[0], cat[1]
    l_off = torch.cumsum(l_cnt, 0) - l_cnt
    e_off = torch.cumsum(e_cnt, 0) - e_cnt
    out_dev = lc.device if device is None else torch.device(device)
    mv = lambda t: None if t is None else t.to(out_dev)
    return DeviceBatch(int(l_cnt.numel()), mv(l_off), mv(l_cnt), mv(cat[2].reshape(-1, 5)), mv(e_off), mv(e_cnt),
                       mv(cat[3]), mv(cat[4]), mv(cat[5]), mv(cat[6].reshape(-1, sw)) if sw else None)
