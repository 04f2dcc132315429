"""Multi-process sharding logic (pvac_hfhe_cppbyv_amd/shard.py) on world size 2 with gloo, CPU only.
The GPU path uses the same code over RCCL (bench.py); shard invariance of the engine's results is
checked on the GPU in tests/test_gpu_shard.py."""
import os
import socket

import pytest

from pvac_hfhe_cppbyv_amd.shard import exclusive_offsets, shard_range


def test_shard_range_partitions():
    for n in (0, 1, 7, 1000, 1 << 20):
        for w in (1, 2, 3, 8):
            got = [shard_range(n, w, r) for r in range(w)]
            assert sum(c for _, c in got) == n
            pos = 0
            for s, c in got:
                assert s == pos
                pos += c
            assert max(c for _, c in got) - min(c for _, c in got) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_total, q):
    import torch
    import torch.distributed as dist
    from pvac_hfhe_cppbyv_amd.shard import global_edge_offsets, max_over_ranks, shard_range
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    start, count = shard_range(n_total, world, rank)
    # stand-in per-pair output sizes keyed by the global pair index (what the engine returns)
    sizes = [1190 + (g * 7919) % 53 for g in range(start, start + count)]
    off, total, per = global_edge_offsets(sum(sizes))
    slow = max_over_ranks(0.5 + rank)
    from pvac_hfhe_cppbyv_amd.shard import all_gather_u64, shard_digest
    import numpy as np
    dig = np.array([(g * 0x9E3779B97F4A7C15) & (2**64 - 1) for g in range(start, start + count)], np.uint64)
    heads = all_gather_u64([shard_digest(dig, start), count, 2**64 - 1 - rank])
    q.put((rank, start, count, off, total, per, slow, [list(map(int, h)) for h in heads]))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_global_offsets():
    import torch.multiprocessing as mp
    n_total = 1001
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_total, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full = [1190 + (g * 7919) % 53 for g in range(n_total)]
    offs, total = exclusive_offsets([sum(full[s:s + c]) for _, s, c, *_ in res])
    import numpy as np
    from pvac_hfhe_cppbyv_amd.shard import combine_digests, shard_digest
    dig_all = np.array([(g * 0x9E3779B97F4A7C15) & (2**64 - 1) for g in range(n_total)], np.uint64)
    for (rank, s, c, off, tot, per, slow, heads), want in zip(res, offs):
        assert off == want                 # this shard's place in the global edge CSR
        assert tot == total == sum(full)   # grand total agrees on every rank
        assert slow == 1.5                 # max over ranks
        # u64 all_gather (full 64-bit range) and the index-keyed shard digests add up to the whole
        assert [h[2] for h in heads] == [2**64 - 1, 2**64 - 2] and [h[1] for h in heads] == [res[0][2], res[1][2]]
        assert combine_digests(h[0] for h in heads) == shard_digest(dig_all, 0)
    assert res[0][1] == 0 and res[1][1] == res[0][2]


def _gather_worker(rank, world, port, q):
    import numpy as np
    import torch
    import torch.distributed as dist
    from pvac_hfhe_cppbyv_amd import DeviceBatch, HostCipher, LAYER_DT
    from pvac_hfhe_cppbyv_amd.shard import gather_batch
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(100 + rank)
    cs = []
    for i in range(3 + rank):   # ragged shards: 3 and 4 ciphers, one of them empty
        ne = 0 if (rank, i) == (1, 2) else int(rng.integers(1, 60))
        L = np.zeros(int(rng.integers(1, 5)), LAYER_DT)
        L["ztag"] = rng.integers(0, 2**63, len(L), dtype=np.uint64)
        cs.append(HostCipher(L, rng.integers(0, 2**63, ne, dtype=np.uint64), rng.integers(0, 2**63, ne, dtype=np.uint64),
                             rng.integers(0, 2**63, ne, dtype=np.uint64)))
    X = DeviceBatch.from_host(cs, "cpu")
    # capacity padding as engine outputs have it: 3 unused rows after every cipher's rows
    gap = lambda cnt: torch.cumsum(cnt, 0) - cnt + 3 * torch.arange(X.n, dtype=torch.int64)

    def spread(a, off_old, off_new, cnt, width=None):
        out = torch.full((int(off_new[-1] + cnt[-1]) + 3,) + tuple(a.shape[1:]), -1, dtype=a.dtype)
        for i in range(X.n):
            out[int(off_new[i]):int(off_new[i] + cnt[i])] = a[int(off_old[i]):int(off_old[i] + cnt[i])]
        return out

    lo2, eo2 = gap(X.l_cnt), gap(X.e_cnt)
    X = DeviceBatch(X.n, lo2, X.l_cnt, spread(X.layers, X.l_off, lo2, X.l_cnt), eo2, X.e_cnt,
                    spread(X.meta, X.e_off, eo2, X.e_cnt), spread(X.w_lo, X.e_off, eo2, X.e_cnt),
                    spread(X.w_hi, X.e_off, eo2, X.e_cnt))
    G = gather_batch(X)
    got = G.to_host()
    q.put((rank, [(c.layers.tobytes(), c.meta.tobytes(), c.w_lo.tobytes(), c.w_hi.tobytes()) for c in got],
           [(c.layers.tobytes(), c.meta.tobytes(), c.w_lo.tobytes(), c.w_hi.tobytes()) for c in cs]))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_gather_batch():
    """shard.gather_batch (the optional result concat of cfg 5) on world size 2 over gloo: every rank
    receives both shards' ciphers in rank order, byte-identical, ragged shards and an empty cipher."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = res[0][2] + res[1][2]
    assert len(want) == 7
    for _, got, _ in res:
        assert got == want
