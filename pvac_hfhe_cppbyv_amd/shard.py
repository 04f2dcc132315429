"""Host-side sharding of independent cipher pairs over ranks (one process per GPU).

The hot path has no exchange step: every pair is independent, so rank r owns the
contiguous global pair range shard_range(N, world, r) and generates / processes it alone. Inputs
and nonces are keyed by the GLOBAL pair index (Engine.gen_fresh(first_index=...),
Engine.fill_nonces(first_index=...)), so the union of the shards equals a single-GPU run. The only
collective is the all_gather of per-rank output-edge totals, which places each shard in the global
(sharded) CSR of the result — BASELINE cfg 5's "gather-only". Works on any torch.distributed backend
(RCCL "nccl" on the GPU node, "gloo" in CPU tests).
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
    the global edge CSR, grand total, per-rank totals). Single process: (0, local_total, [local])."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
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
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    if dist.get_backend() == "gloo":
        device = "cpu"
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
