"""Shard invariance on the GPU: the union of two shards (generated and multiplied with global
pair indices, as bench.py's ranks do) equals one single-GPU batch, pair for pair."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_two_shards_equal_one_batch():
    from pvac_hfhe_cppbyv_amd import Engine
    eng = Engine(device=0, canon_tag=0x5EED0005)
    n = 1024

    def run(first, count):
        A = eng.gen_fresh(count, 0x51, 20, first_index=first)
        B = eng.gen_fresh(count, 0x52, 20, first_index=first)
        Cb, plan = eng.ct_mul_plan(A, B)
        nonces = eng.fill_nonces(A, B, Cb, plan, 0x53, first_index=first)
        out = eng.ct_mul(A, B, nonces=nonces, C_=Cb, plan=plan)
        dig = eng.digest(out).cpu().numpy().view(np.uint64)
        lay = out.to_host()
        return dig, [(c.nE, c.layers["ztag"].tobytes()) for c in lay]

    d_all, l_all = run(0, n)
    d0, l0 = run(0, n // 2)
    d1, l1 = run(n // 2, n - n // 2)
    assert np.array_equal(np.concatenate([d0, d1]), d_all)
    assert l0 + l1 == l_all


def _bench_run(args, world, port=None, backend="gloo", launcher=False, shared=False):
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PVAC_BENCH_BACKEND=backend)
    env.pop("PVAC_BENCH_ALLOW_SHARED", None)
    if shared:   # the one-GPU rehearsal: ranks share cuda:0
        env["PVAC_BENCH_ALLOW_SHARED"] = "1"
    if launcher:   # torch.distributed.run even for one rank: the process group and its collectives run
        env["PVAC_BENCH_DIST"] = "1"
    if not launcher:   # bench.py itself (at --gpus N > 1 it starts the N ranks)
        cmd = [sys.executable, os.path.join(root, "bench.py")] + args
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(root, "bench.py")] + args
    return subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=root)


def _bench_json(args, world, port=None, backend="gloo", launcher=False, shared=False):
    import json
    p = _bench_run(args, world, port, backend, launcher, shared)
    assert p.returncode == 0, p.stderr[-3000:]
    js = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(js) == 1, p.stdout[-3000:]
    return json.loads(js[0])


def test_bench_world2_shard_digests_equal_one_gpu():
    """bench.py's N>1 path on one GPU: `bench.py --gpus 2` starts the two ranks itself (gloo for the
    gathers, both on cuda:0 in the shared-device rehearsal); each runs its shard of the global
    batch, rank 0 recomputes both ranks' pair windows from the global indices, the gsum invariant
    holds on every pair, and the gathered digest equals a one-rank run of the same 2 x 4096 pairs.
    The line counts ONE GPU for the two ranks."""
    common = ["--steps", "1", "--warmup", "0", "--no-cpu", "--no-extras", "--check-window", "512"]
    two = _bench_json(["--gpus", "2", "--pairs", "4096"] + common, 2, shared=True)
    one = _bench_json(["--gpus", "1", "--pairs", "8192"] + common, 1)
    c2, c1 = two["checks"], one["checks"]
    assert two["n_gpus"] == 1 and two["ranks"] == 2 and two["dist"] == {"world_size": 2, "backend": "gloo"}
    assert one["n_gpus"] == 1 and one["ranks"] == 1
    assert c2["shard_digests_ok"] and c2["shard_windows"]["ranks"] == 2
    assert c2["result_gather"]["match"] and c2["result_gather"]["ciphers"] == 16
    assert c2["gsum_invariant"]["ok"] and c2["gsum_invariant"]["pairs"] == 8192
    assert c1["shard_digests_ok"] and c1["gsum_invariant"]["pairs"] == 8192
    assert c2["global_digest"] == c1["global_digest"]
    assert c2["global_output_edges"] == c1["global_output_edges"]


def test_bench_rccl_one_rank_collectives():
    """bench.py's distributed flow over RCCL ("nccl" backend on ROCm) with one rank on cuda:0
    (torch.distributed.run, PVAC_BENCH_DIST=1): the process group, the device-tensor all_gathers of
    edge totals / shard digests / pair windows and the all_reduce of the step time go through RCCL,
    and the result equals a run without any process group. (The 1-GPU pool cannot host two RCCL
    ranks on one device; the world-2 flow is covered over gloo above.)"""
    from test_shard_dist import _free_port
    common = ["--gpus", "1", "--pairs", "4096", "--steps", "1", "--warmup", "0", "--no-cpu", "--no-extras",
              "--check-window", "512"]
    rccl = _bench_json(common, 1, _free_port(), backend="nccl", launcher=True)
    plain = _bench_json(common, 1)
    c, c0 = rccl["checks"], plain["checks"]
    assert c["collective_backend"] == "nccl" and c0["collective_backend"] is None
    assert c["shard_digests_ok"] and c["gsum_invariant"]["ok"] and c["gsum_invariant"]["pairs"] == 4096
    assert c["result_gather"]["match"]   # shard.gather_batch over RCCL (one rank)
    assert c["global_digest"] == c0["global_digest"]
    assert c["global_output_edges"] == c0["global_output_edges"]


def test_bench_gpus2_on_one_gpu_fails_loudly():
    """Without the rehearsal switch, `bench.py --gpus N` with fewer than N GPUs stops before any
    GPU work with a clear message instead of reporting N GPUs."""
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("more than one GPU visible")
    p = _bench_run(["--gpus", "2", "--pairs", "4096", "--steps", "1", "--warmup", "0", "--no-cpu", "--no-extras"], 2)
    assert p.returncode == 2, p.stderr[-2000:]
    assert "distinct visible GPUs" in p.stderr
    assert not [l for l in p.stdout.splitlines() if l.startswith("{")]
