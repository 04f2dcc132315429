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
