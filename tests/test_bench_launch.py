"""bench.py's multi-rank launch on the CPU: `--gpus N` with no launcher environment starts N ranks
itself (torch.distributed.run, 127.0.0.1) before touching the GPU, rank 0's line comes back as
the one JSON line, and the ranks refuse to share a device unless the one-GPU rehearsal asks for it.
`--topology-only` runs the launch, the process group and the device census without GPU work."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra, launcher_world=None):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "PVAC_BENCH_ALLOW_SHARED"):
        env.pop(k, None)
    env.update(env_extra)
    if launcher_world:
        from test_shard_dist import _free_port
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={launcher_world}",
               "--master-addr=127.0.0.1", f"--master-port={_free_port()}", BENCH] + args
    else:
        cmd = [sys.executable, BENCH] + args
    return subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)


def test_spawn_world2_gloo_merged_line():
    p = _run(["--gpus", "2", "--topology-only"], {"PVAC_BENCH_BACKEND": "gloo", "PVAC_BENCH_ALLOW_SHARED": "1"})
    assert p.returncode == 0, p.stderr[-3000:]
    js = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(js) == 1, p.stdout
    r = json.loads(js[0])
    assert r["topology_only"] and r["ranks"] == 2
    assert r["dist"] == {"world_size": 2, "backend": "gloo"}
    assert sorted(d["rank"] for d in r["devices"]) == [0, 1]
    # both ranks on this host's CPU: one distinct device, so n_gpus never counts ranks
    assert r["n_gpus"] == len({d["id"] for d in r["devices"]}) == 1


def test_spawn_refuses_more_gpus_than_visible():
    import torch
    n = max(2, torch.cuda.device_count() + 1)
    p = _run(["--gpus", str(n), "--topology-only"], {"PVAC_BENCH_BACKEND": "gloo"})
    assert p.returncode == 2
    assert "distinct visible GPUs" in p.stderr
    assert not [l for l in p.stdout.splitlines() if l.startswith("{")]


def test_launcher_ranks_sharing_a_device_fail():
    """Under an external launcher, two ranks that land on the same device stop with an error
    instead of reporting two GPUs."""
    p = _run(["--gpus", "2", "--topology-only"], {"PVAC_BENCH_BACKEND": "gloo"}, launcher_world=2)
    assert p.returncode != 0
    assert "distinct devices" in p.stderr


def test_launcher_gpus_flag_must_match_world():
    p = _run(["--gpus", "3", "--topology-only"], {"PVAC_BENCH_BACKEND": "gloo", "PVAC_BENCH_ALLOW_SHARED": "1"},
             launcher_world=2)
    assert p.returncode != 0
    assert "launcher started 2 ranks" in p.stderr
