#!/usr/bin/env python3
"""bench.py — headline benchmark of the MI355X pvac-hfhe engine (driver contract).

Workload (BASELINE.json cfg 3): batched weights-only ct_mul over fresh-shaped Cipher pairs
(2 BASE layers x 20 distinct (idx, ch) edges per layer, default Params B=337), 2^20 pairs on
one GPU, inputs resident in HBM. One step = plan (sizing) + exec over the whole batch.
Multi-GPU (cfg 5): one process per GPU, 2^21 pairs per rank (2^24 at N=8); each rank owns an
independent shard (weak scaling); the only collective is the gather of per-rank output totals
(global CSR offsets), over RCCL. `python bench.py --gpus N` (N > 1, no launcher environment) starts
N ranks itself through torch.distributed.run before this process touches the GPU; under a launcher
(WORLD_SIZE set) each rank takes its own GPU (LOCAL_RANK) and the ranks check that their devices
are distinct. The line reports the devices and the world size / backend torch.distributed saw.

Also reported (side fields, rank 0): cfg 2 element-wise Fp127 add/mul at 2^24, full ct_mul WITH
sigma (the reference's complete ct_mul) on a smaller batch, cfg 4 (GPU enc_value + depth-8
chains over 2^16 inputs) and batched enc_value, each with its CPU baseline where one exists.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

METRIC = "ct_mul/sec (batched Cipher) + achieved HBM GB/s vs peak, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (one rank each). N > 1 without a launcher: bench.py starts N ranks itself")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--pairs", type=int, default=None,
                    help="pairs per GPU (default 2^20 = cfg 3 at N=1; 2^21 at N>1, so N=8 is cfg 5's 2^24 pairs)")
    ap.add_argument("--epl", type=int, default=20, help="edges per BASE layer")
    ap.add_argument("--shard-rank", type=int, default=None,
                    help="one GPU runs rank R's shard of a cfg-5 job: pairs [R n, (R + 1) n) of the global batch "
                         "(n = --pairs, default 2^21): the per-GPU shape of the 8-GPU run, checked end to end")
    ap.add_argument("--cpu-pairs", type=int, default=1 << 17)
    ap.add_argument("--cpu-threads", type=int, default=1)
    ap.add_argument("--cpu-share-threads", type=int, default=16, help="second CPU baseline: the box's CPU share")
    ap.add_argument("--sigma-pairs", type=int, default=1 << 12)
    ap.add_argument("--chain-inputs", type=int, default=1 << 16, help="cfg 4 chain inputs (enc_value outputs)")
    ap.add_argument("--chain-chunk", type=int, default=1 << 10,
                    help="cfg 4: inputs per chunk (4 streams x 1024 reserve the HBM that 1 x 4096 does)")
    ap.add_argument("--chain-depth", type=int, default=8)
    ap.add_argument("--chain-check", type=int, default=16,
                    help="cfg 4: chains (first inputs of the first chunk) whose final outputs are digest-compared "
                         "with the pinned CPU port, which is also timed on them (cpu_baseline)")
    ap.add_argument("--chain-ref", type=int, default=2, help="cfg 4: reference chains (oracle/_ref) timed, depth 4")
    ap.add_argument("--chain-streams", type=int, default=6,
                    help="cfg 4: worker streams of the engine's chain call (pvac_hip_ct_mul_chain): one chunk's "
                         "host planning and dependent launches overlap the other chunks' kernels (6: +1.5%% over 4, "
                         "profiles/r05/rows/chain_streams2.log)")
    ap.add_argument("--chain-no-check", action="store_true",
                    help="cfg 4: skip the checked second pass and the CPU sample (kernel-trace profiling)")
    ap.add_argument("--chain-compare-streams", action="store_true",
                    help="cfg 4: also time the chain call with 1 worker stream on a subset (side field)")
    ap.add_argument("--enc-values", type=int, default=1 << 14, help="enc_value batch (f2)")
    ap.add_argument("--only", choices=["chain", "sigma", "fp", "enc", "add"], default=None,
                    help="run one side measurement alone (profiling) and print its JSON")
    ap.add_argument("--check-window", type=int, default=4096,
                    help="pairs per rank whose digests rank 0 recomputes from global indices (shard check)")
    ap.add_argument("--topology-only", action="store_true",
                    help="launcher check: every rank reports its device and the process group, no GPU work")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extras", action="store_true")
    return ap.parse_args()


def _shared_ok():
    """PVAC_BENCH_ALLOW_SHARED=1: ranks may share a GPU (the one-GPU rehearsal of the N > 1 flow;
    gloo collectives). Never set by the driver: there every rank must own a distinct GPU."""
    return os.environ.get("PVAC_BENCH_ALLOW_SHARED") == "1"


def spawn(args):
    """`--gpus N` (N > 1) with no launcher: start N ranks (torch.distributed.run, one process per
    GPU, 127.0.0.1 rendezvous) and forward rank 0's JSON line. This process never initialises the
    GPU (torch.cuda.device_count() does not on this ROCm image), so nothing is re-executed after a
    HIP call. Returns the children's exit status."""
    import socket
    import subprocess
    import torch
    n = args.gpus
    vis = torch.cuda.device_count()
    if n > vis and not _shared_ok():
        print(f"bench.py: --gpus {n} needs {n} distinct visible GPUs (one rank each); this host shows {vis}",
              file=sys.stderr, flush=True)
        return 2
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, bufsize=1)
    lines = []
    for line in proc.stdout:   # progress is forwarded as it comes (to stderr); the JSON line last
        if line.startswith("{"):
            lines.append(line.strip())
        else:
            sys.stderr.write(line)
            sys.stderr.flush()
    rc = proc.wait()
    if rc != 0:
        print(f"bench.py: ranks exited with status {rc}", file=sys.stderr, flush=True)
        return rc
    if len(lines) != 1:
        print(f"bench.py: expected one JSON line from rank 0, got {len(lines)}", file=sys.stderr, flush=True)
        return 3
    print(lines[0], flush=True)
    return 0


def _device_id(torch, gpu):
    """Identity of a rank's GPU: the device uuid (distinct per physical GPU, whatever each rank's
    visible-device numbering), else host + ordinal; "cpu" for a device-less launcher check."""
    import socket
    if gpu is None:
        return f"{socket.gethostname()}:cpu"
    try:
        pr = torch.cuda.get_device_properties(gpu)
        return f"{pr.uuid}" if str(pr.uuid) else f"{socket.gethostname()}:{pr.pci_domain_id}:{pr.pci_bus_id}"
    except Exception:
        return f"{socket.gethostname()}:cuda:{gpu}"


def topology(torch, dist, dist_on, world, rank, gpu):
    """Every rank's device and what torch.distributed saw; raises unless the ranks own distinct
    devices (or sharing was asked for)."""
    me = {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")), "device": gpu,
          "id": _device_id(torch, gpu)}
    if dist_on:
        allv = [None] * dist.get_world_size()
        dist.all_gather_object(allv, me)
        seen = {"world_size": dist.get_world_size(), "backend": str(dist.get_backend())}
    else:
        allv = [me]
        seen = {"world_size": 1, "backend": None}
    distinct = len({d["id"] for d in allv})
    if distinct < len(allv) and not _shared_ok():
        raise RuntimeError(f"bench.py: {len(allv)} ranks on {distinct} distinct devices ({allv}); one rank per "
                           "GPU is required (PVAC_BENCH_ALLOW_SHARED=1 only for the one-GPU rehearsal)")
    if seen["world_size"] != world:
        raise RuntimeError(f"bench.py: WORLD_SIZE {world} but the process group has {seen['world_size']} ranks")
    return {"n_gpus": distinct, "ranks": len(allv), "devices": allv, "dist": seen,
            "shared_devices": distinct < len(allv)}


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        sys.exit(spawn(args))
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started {world} ranks")
    # one process per GPU over RCCL; PVAC_BENCH_BACKEND=gloo + PVAC_BENCH_ALLOW_SHARED=1 rehearse
    # the multi-rank flow with ranks sharing the visible GPUs (local rank modulo the device count)
    backend = os.environ.get("PVAC_BENCH_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if args.topology_only:
        gpu = None if ndev == 0 else local % ndev
    elif local < ndev:
        gpu = local
    elif _shared_ok() and ndev:
        gpu = local % ndev
    else:
        raise SystemExit(f"bench.py: rank {rank} (local {local}) has no GPU of its own ({ndev} visible)")
    # PVAC_BENCH_DIST=1 runs the distributed flow (process group, gathers, self-checks) at world 1
    # too: under torch.distributed.run with one rank it puts the collectives on RCCL on a 1-GPU box
    dist_on = world > 1 or os.environ.get("PVAC_BENCH_DIST") == "1"
    if dist_on:
        if gpu is not None:
            torch.cuda.set_device(gpu)
        if backend == "nccl" and gpu is not None:
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group("gloo")
    topo = topology(torch, dist, dist_on, world, rank, gpu)
    if args.topology_only:
        if rank == 0:
            print(json.dumps({"metric": METRIC, "value": None, "unit": "ct_mul/s", "topology_only": True,
                              "n_gpus": topo["n_gpus"], "ranks": topo["ranks"], "devices": topo["devices"],
                              "dist": topo["dist"]}), flush=True)
        if dist_on:
            dist.barrier()
            dist.destroy_process_group()
        return
    from pvac_hfhe_cppbyv_amd import Engine

    eng = Engine(device=gpu, canon_tag=0x5EED0003)
    dev = eng.device
    if args.only == "chain":
        print(json.dumps(chain_bench(eng, args)), flush=True)
        return
    if args.only == "sigma":
        print(json.dumps(sigma_bench(eng, args, False)), flush=True)
        return
    if args.only == "enc":
        print(json.dumps(enc_bench(eng, args, False)), flush=True)
        return
    if args.only == "add":
        print(json.dumps(add_bench(eng, args)), flush=True)
        return
    from pvac_hfhe_cppbyv_amd.shard import global_edge_offsets, max_over_ranks
    shard_rank = args.shard_rank if world == 1 else None
    n = args.pairs if args.pairs else (1 << 20 if world == 1 and shard_rank is None else 1 << 21)
    # weak scaling: rank r owns global pairs [r*n, (r+1)*n); inputs and nonces are keyed by the
    # global pair index, so the N-GPU result is the 1-GPU result of the same global batch, sharded.
    # --shard-rank R at world 1 runs rank R's shard alone (global pair indices up to (R + 1) n)
    first = (shard_rank if shard_rank is not None else rank) * n
    seed = 0x5EED0003
    A = eng.gen_fresh(n, seed, args.epl, first_index=first)
    B = eng.gen_fresh(n, seed + 1, args.epl, first_index=first)
    nonces = None
    placement = {}
    outbuf = []

    def step():
        # one step = plan + exec of the whole batch (pvac_hip_ct_mul: one call, no host round trip
        # between them) into output arrays sized on the first step and reused, then the totals gather
        nonlocal nonces
        if not outbuf:
            Cb, plan = eng.ct_mul_plan(A, B)
            nonces = eng.fill_nonces(A, B, Cb, plan, seed + 2, first_index=first)
            out = eng.ct_mul(A, B, nonces=nonces, C_=Cb, plan=plan)
            outbuf.extend([out, eng.ct_mul_step(A, B, out, nonces)])
        else:
            out = outbuf[0]
            plan = outbuf[1]()
        # gather-only (cfg 5): per-rank output totals -> this shard's offset in the global edge CSR
        off, total, _ = global_edge_offsets(plan.total_edge_slots, device=dev)
        placement.update(offset=off, total_edge_slots=total)
        return out, plan

    out = plan = None
    for _ in range(args.warmup):
        out, plan = step()
    torch.cuda.synchronize(dev)
    if dist_on:
        dist.barrier()
    eng.timing_reset()
    eng.timing(True)
    redo0 = eng.ct_mul_redo_count()
    torch.cuda.synchronize(dev)
    if dist_on:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out, plan = step()
    torch.cuda.synchronize(dev)
    if dist_on:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    eng.timing(False)
    kern_ms, kern_launches = eng.timing_get("ct_mul_fresh")
    lay_ms, lay_launches = eng.timing_get("mul_layers_fresh")
    elapsed = max_over_ranks(elapsed, device=dev)
    ms_per_step = 1000.0 * elapsed / args.steps
    value = world * n / (elapsed / args.steps)

    # ---- algorithmic bytes of the dominant kernel k_ct_mul_fresh: per pair
    #   24 B x (|A.E| + |B.E| + |C.E|)  edge records (meta 8 + w 16) read / written
    # + 16 B x (|A.L| + |B.L|)          rule/pa/pb of the input layers (compact_layers parents)
    # + 104 B                           offsets / counts / class / status of A, B, C
    # (the product-layer records, 40 B x |C.L| + 16 B nonces x |A.L||B.L|, are written by
    #  k_mul_layers_fresh and reported as step bytes below)
    e_cnt = out.e_cnt[:n].to(torch.float64)
    l_cnt = out.l_cnt[:n].to(torch.float64)
    la, lb = A.l_cnt[:n].to(torch.float64), B.l_cnt[:n].to(torch.float64)
    na, nb = A.e_cnt[:n].to(torch.float64), B.e_cnt[:n].to(torch.float64)
    alg_bytes = float((24 * (na + nb + e_cnt) + 16 * (la + lb) + 104).sum().item())
    step_bytes = alg_bytes + float((40 * (la + lb + l_cnt) + 16 * la * lb).sum().item())
    avg_kernel_ms = kern_ms / max(kern_launches, 1)
    achieved = alg_bytes / (avg_kernel_ms / 1000.0) / 1e9 if avg_kernel_ms > 0 else None
    out_edges = float(e_cnt.sum().item())

    result = {
        "metric": METRIC,
        "value": value,
        "unit": "ct_mul/s",
        "n_gpus": topo["n_gpus"],
        "ranks": topo["ranks"],
        "devices": [d["id"] for d in topo["devices"]],
        "dist": topo["dist"],
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic (device splitmix64 generator, cfg-3 fresh-shaped ciphers)",
        "config": {
            "workload": ("cfg3" if world == 1 and shard_rank is None else "cfg5") +
                        (f" (rank {shard_rank}'s shard alone: global pairs [{first}, {first + n}))"
                         if shard_rank is not None else "") +
                        f": {n} fresh-shaped Cipher pairs per GPU, batched ct_mul, weights-only (weights + "
                        "layers + the reference's emit order; no sigma in the timed region), default Params B=337",
            "pairs_per_gpu": n,
            "edges_per_layer": args.epl,
            "global_pairs": world * n,
            "output_edges_per_pair": out_edges / n,
            "parallelism": f"dp{world} (independent pair shards, gather of totals over "
                           f"{topo['dist']['backend'] or 'no process group'})",
            "shard": {"first_pair": first, "edge_slot_offset": placement.get("offset"),
                      "global_edge_slots": placement.get("total_edge_slots")},
        },
        "roofline": {
            # the kernel is VALU-issue-bound (roofline.valu.frac, PMC), not HBM-bound; achieved / peak /
            # frac are its HBM figures (algorithmic bytes over the HIP-event time), the contract's metric
            "bound": "valu",
            "frac_basis": "hbm (algorithmic bytes / kernel time / 8 TB/s); the binding roof is roofline.valu",
            "kernel": FRESH_KERNEL,
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
            "traffic": None,
            "alg_bytes_per_launch": alg_bytes,
            "avg_kernel_ms": avg_kernel_ms,
            "kernel_launches": kern_launches,
            "step_alg_bytes": step_bytes,
            "layers_kernel_avg_ms": lay_ms / max(lay_launches, 1),
            "step_GBs": step_bytes / (ms_per_step / 1000.0) / 1e9,
        },
        "cpu_baseline": None,
    }
    # HBM traffic and the VALU counters of the same kernel from the committed PMC record
    # (tools/pmc_target.sh -> profiles/pmc/headline.json), quoted only when the record was taken on
    # THIS library binary (sha256 of libpvac_hip.so) and this batch shape; null plus the reason else
    pm, why = pmc_record("headline", {"pairs": n, "epl": args.epl})
    result["roofline"]["traffic"] = pm.get("traffic") if pm else None
    result["roofline"]["traffic_source"] = PMC_SOURCE if pm else why
    result["roofline"]["valu"] = valu_roofline(eng, pm, why, avg_kernel_ms, n, "pair")

    # fresh-kernel pairs re-run on the general path during the timed steps (a key sum of 0 mod p:
    # never for these uniform nonzero weights, so any redo here is a kernel defect costing time)
    redo = eng.ct_mul_redo_count() - redo0
    result["checks"] = self_checks(eng, args, A, B, out, nonces, n, first, seed, world, rank)
    result["checks"]["fresh_redo"] = {"pairs_per_step": redo / args.steps, "ok": redo == 0}
    result["checks"]["collective_backend"] = dist.get_backend() if dist_on else None
    if rank == 0 and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline(eng, A, B, out, n, args)
    # the cfg-3 batch (~35 GB of inputs, outputs and nonces) is done with: release it so the side
    # measurements (chains size their sub-batches from free HBM) run on an empty device
    A = B = out = nonces = plan = None
    placement.clear()
    torch.cuda.synchronize(dev)
    torch.cuda.empty_cache()
    if rank == 0 and not args.no_extras:
        try:
            result["extras"] = extras(eng, args, world == 1 and not args.no_cpu)
        except Exception as ex:   # side measurements must not hide the headline
            result["extras"] = {"error": repr(ex)}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist_on:
        dist.barrier()
        dist.destroy_process_group()


FRESH_KERNEL = "k_ct_mul_fresh3"   # the fresh-pair kernel launch_ct_mul_fresh runs (k_mul_fresh.hip)
PMC_SOURCE = ("rocprofv3 --pmc, one counter group per run, mean per full-size dispatch; traffic = 2 x FETCH_SIZE "
              "(wide-read correction) + WRITE_SIZE (tools/pmc_target.sh, tools/pmc_stamp.py)")
_LIB_SHA = None


def lib_sha256():
    """sha256 of the libpvac_hip.so this process loaded (the PMC records are stamped with it)."""
    global _LIB_SHA
    if _LIB_SHA is None:
        import hashlib
        from pvac_hfhe_cppbyv_amd import _LIB_PATH
        h = hashlib.sha256()
        with open(_LIB_PATH, "rb") as f:
            for blk in iter(lambda: f.read(1 << 20), b""):
                h.update(blk)
        _LIB_SHA = h.hexdigest()
    return _LIB_SHA


def pmc_record(target, workload):
    """profiles/pmc/<target>.json when it was taken on this library binary and this workload:
    (record, None); else ({}, the reason)."""
    path = os.path.join(ROOT, "profiles", "pmc", target + ".json")
    if not os.path.exists(path):
        return {}, f"no PMC record profiles/pmc/{target}.json"
    try:
        with open(path) as f:
            rec = json.load(f)
    except Exception as ex:
        return {}, f"unreadable PMC record: {ex!r}"
    if rec.get("lib_sha256") != lib_sha256():
        return {}, (f"profiles/pmc/{target}.json was taken on libpvac_hip.so sha256 {str(rec.get('lib_sha256'))[:12]}, "
                    f"this run loaded {lib_sha256()[:12]}: counters of another binary are not quoted")
    got = rec.get("workload") or {}
    for k, v in workload.items():
        if got.get(k) != v:
            return {}, f"PMC record workload {got} differs from this run's {workload}"
    return rec, None


def valu_roofline(eng, rec, why, kernel_ms, units, unit_name):
    """The VALU side of a kernel's roofline from its PMC record: frac = the counter-measured VALU-busy
    fraction, 4 x SQ_ACTIVE_INST_VALU (quad-cycles) / (kernel cycles x 1,024 SIMDs), <= 1 by
    construction; beside it the VALU instruction rate against two ceilings measured now on this GPU
    (pvac_hip_alu_ceiling 4: a 32-bit mix, 0: the v_mad_u64_u32 mix; the per-opcode issue costs are
    in profiles/r05/issue_probe.json)."""
    try:
        ceil32, ceilmad = eng.alu_ceiling(4), eng.alu_ceiling(0)
    except Exception:
        ceil32 = ceilmad = None
    out = {"unit": "fraction of SIMD cycles issuing VALU (SQ_ACTIVE_INST_VALU)", "frac": None,
           "mix32_ceiling_inst_per_s": ceil32, "madmix_ceiling_inst_per_s": ceilmad}
    if not rec:
        out["note"] = why
        return out
    vi = rec.get("valu_insts")
    out.update({"frac": rec.get("valu_busy"), "achieved": rec.get("valu_busy"), "peak": 1.0,
                f"insts_per_{unit_name}": vi / units if vi else None,
                "lds_active_frac": rec.get("lds_active_frac"),
                "lds_bank_conflict_frac": rec.get("lds_bank_conflict_frac"), "wait_frac": rec.get("wait_frac"),
                "clock_hz_pmc_run": rec.get("clock_hz_est"), "source": PMC_SOURCE,
                "lib_sha256": rec.get("lib_sha256")})
    if vi and kernel_ms > 0:
        rate = vi / (kernel_ms / 1000.0)
        out["inst_per_s"] = rate
        if ceil32:
            out["rate_vs_mix32_ceiling"] = rate / ceil32
    return out


def self_checks(eng, args, A, B, out, nonces, n, first, seed, world, rank):
    """Outside the timed region, on the last step's output of every rank:
    * the reference's gsum invariant check_mul_gsum_all (utils/metrics.hpp:88-113) on EVERY pair;
    * shard digests: each rank's index-keyed digest sum (their sum over ranks is the digest of a
      one-GPU run of the whole global batch) and the per-pair digests of its last `check_window`
      pairs, all_gathered; rank 0 recomputes every rank's window from the global pair indices and
      compares (inputs and nonces are keyed by the global index, so a sharded run must match)."""
    import numpy as np
    import torch
    from pvac_hfhe_cppbyv_amd import powg_table
    from pvac_hfhe_cppbyv_amd.shard import all_gather_u64, combine_digests, shard_digest
    dev = eng.device
    eng.set_powg(powg_table(eng.params.B))
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    bad = eng.check_mul_gsum(A, B, out, nonces)
    inv_ms = 1000.0 * (time.perf_counter() - t0)
    dig = eng.digest(out)[:n].cpu().numpy().view(np.uint64).copy()
    K = max(1, min(args.check_window, n))
    edges = int(out.e_cnt[:n].sum().item())
    head = all_gather_u64([shard_digest(dig, first), bad, edges, first, n], device=dev)
    wins = all_gather_u64(dig[n - K:], device=dev)
    failed = int(sum(int(h[1]) for h in head))
    res = {"gsum_invariant": {"check": "check_mul_gsum_all (reference utils/metrics.hpp:88-113), every pair of "
                                       "every rank, on the device (k_check.hip)",
                              "pairs": int(sum(int(h[4]) for h in head)), "failed": failed, "ok": failed == 0,
                              "ms_rank0": inv_ms},
           "global_digest": "%016x" % combine_digests(h[0] for h in head),
           "global_output_edges": int(sum(int(h[2]) for h in head))}
    if rank == 0:
        match = True
        for r, h in enumerate(head):
            g0 = int(h[3]) + int(h[4]) - K
            Aw = eng.gen_fresh(K, seed, args.epl, first_index=g0)
            Bw = eng.gen_fresh(K, seed + 1, args.epl, first_index=g0)
            Cw, pw = eng.ct_mul_plan(Aw, Bw)
            nw = eng.fill_nonces(Aw, Bw, Cw, pw, seed + 2, first_index=g0)
            ow = eng.ct_mul(Aw, Bw, nonces=nw, C_=Cw, plan=pw)
            dw = eng.digest(ow)[:K].cpu().numpy().view(np.uint64)
            match = match and bool(np.array_equal(dw, wins[r]))
            del Aw, Bw, Cw, ow, nw
        res["shard_windows"] = {"pairs_per_rank": K, "ranks": world, "recomputed_on": "rank 0", "match": match}
        res["shard_digests_ok"] = bool(match and failed == 0)
    # the optional result concat (shard.gather_batch: RCCL all_gather of compacted shards) on each
    # rank's last 8 pairs: the gathered ciphers' digests equal the window digests every rank sent
    from pvac_hfhe_cppbyv_amd import DeviceBatch
    from pvac_hfhe_cppbyv_amd.shard import gather_batch
    k8 = min(8, K)
    tail = DeviceBatch(k8, out.l_off[n - k8:n], out.l_cnt[n - k8:n], out.layers, out.e_off[n - k8:n],
                       out.e_cnt[n - k8:n], out.meta, out.w_lo, out.w_hi)
    G = gather_batch(tail)
    gd = eng.digest(G).cpu().numpy().view(np.uint64)
    want = np.concatenate([w[len(w) - k8:] for w in wins])
    res["result_gather"] = {"pairs_per_rank": k8, "ranks": world, "ciphers": int(G.n),
                            "match": bool(G.n == k8 * world and np.array_equal(gd, want))}
    return res


def cpu_baseline(eng, A, B, out, n, args):
    """The pinned CPU port (oracle/pvac_oracle.cpp: same algorithm as the reference's
    ct_mul minus sigma, std::unordered_map aggregation) on a bounded sample of the SAME
    device-resident inputs; digests are cross-checked against the GPU output."""
    import numpy as np
    from helpers import Oracle, default_params
    orc = Oracle.load()
    k = min(args.cpu_pairs, n)
    u = lambda t: t.cpu().numpy().view(np.uint64)
    al, a_lay, ae, am, awl, awh = _pack_host(A, k)
    bl, b_lay, be, bm, bwl, bwh = _pack_host(B, k)
    counts = np.zeros(k, np.uint64)
    digests = np.zeros(k, np.uint64)
    prm = default_params(0x5EED0003)
    import ctypes as C
    P = lambda x: x.ctypes.data_as(C.c_void_p)
    secs = orc.lib.orc_ct_mul_batch_timed(C.byref(prm), k, P(al), P(a_lay), P(ae), P(am), P(awl), P(awh),
                                          P(bl), P(b_lay), P(be), P(bm), P(bwl), P(bwh), args.cpu_threads,
                                          P(counts), P(digests))
    gpu_dig = u(eng.digest(out)[:k])
    gpu_cnt = u(out.e_cnt[:k])
    # the same port on the GPU box's CPU share (16 threads, independent pairs), for scale
    mt = max(1, args.cpu_share_threads)
    secs_mt = orc.lib.orc_ct_mul_batch_timed(C.byref(prm), k, P(al), P(a_lay), P(ae), P(am), P(awl), P(awh),
                                             P(bl), P(b_lay), P(be), P(bm), P(bwl), P(bwh), mt, P(counts), P(digests))
    return {
        "multi_thread": {"value": k / secs_mt, "cores": mt, "seconds": secs_mt},
        "value": k / secs,
        "unit": "ct_mul/s",
        "cores": args.cpu_threads,
        "kind": "port",
        "sample": f"{k} of the {n} device-resident pairs (first k), weights-only ct_mul incl. layer ztags, "
                  f"{secs:.2f} s",
        "impl": "oracle/pvac_oracle.cpp (pinned to the reference by tests/test_oracle.py)",
        "cpu_model": _cpu_model(),
        "gpu_output_matches": bool(np.array_equal(gpu_dig, digests) and np.array_equal(gpu_cnt, counts)),
    }


def _pack_host(X, k):
    """The first k ciphers of a device batch (capacity-padded CSR allowed) as host arrays in the
    oracle's packed layout: offsets with k + 1 entries (u64), layer records, meta, w_lo, w_hi."""
    import numpy as np
    import torch
    u = lambda t: t.cpu().numpy().view(np.uint64)

    def rows(off, cnt):   # the used slots of every cipher, in order
        cnt = cnt.to(torch.int64)
        excl = torch.cumsum(cnt, 0) - cnt
        idx = torch.repeat_interleave(off.to(torch.int64) - excl, cnt)
        packed = torch.zeros(k + 1, dtype=torch.int64, device=cnt.device)
        packed[1:] = torch.cumsum(cnt, 0)
        return idx + torch.arange(idx.numel(), device=idx.device), packed

    li, lo = rows(X.l_off[:k], X.l_cnt[:k])
    ei, eo = rows(X.e_off[:k], X.e_cnt[:k])
    cs = np.ascontiguousarray
    return (cs(u(lo)), cs(X.layers[li].cpu().numpy()), cs(u(eo)), cs(u(X.meta[ei])), cs(u(X.w_lo[ei])),
            cs(u(X.w_hi[ei])))


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return None


def extras(eng, args, with_cpu):
    """cfg 2 (2^24 Fp127 add/mul) and full ct_mul WITH sigma on a smaller batch."""
    import numpy as np
    import torch
    from pvac_hfhe_cppbyv_amd import FP_ADD, FP_MUL, MUL_WITH_SIGMA
    dev = eng.device
    res = {}
    # ---- cfg 2: element-wise Fp127
    nfp = 1 << 24
    bufs = [torch.empty(nfp, dtype=torch.int64, device=dev) for _ in range(6)]
    for i, t in enumerate(bufs[:4]):
        eng.fill_random(t, 0x5EED0002 + i)
    bufs[1] &= (1 << 63) - 1
    bufs[3] &= (1 << 63) - 1
    fp = {}
    for name, op in (("add", FP_ADD), ("mul", FP_MUL)):
        for _ in range(3):
            eng.fp_binop(op, *bufs[:4], out=(bufs[4], bufs[5]))
        eng.timing_reset()
        eng.timing(True)
        for _ in range(20):
            eng.fp_binop(op, *bufs[:4], out=(bufs[4], bufs[5]))
        eng.timing(False)
        ms, cnt = eng.timing_get("fp_binop")
        avg = ms / max(cnt, 1)
        gbs = 48.0 * nfp / (avg / 1000.0) / 1e9
        fp[name] = {"elements": nfp, "avg_kernel_ms": avg, "Gop_s": nfp / (avg / 1000.0) / 1e9,
                    "achieved_GBs": gbs, "frac_of_hbm_peak": gbs / HBM_PEAK_GBS}
        if with_cpu:
            from helpers import Oracle
            orc = Oracle.load()
            m = 1 << 22
            h = [t[:m].cpu().numpy().view(np.uint64).copy() for t in bufs[:4]]
            olo, ohi = np.zeros(m, np.uint64), np.zeros(m, np.uint64)
            import ctypes as C
            P = lambda x: x.ctypes.data_as(C.c_void_p)
            secs = orc.lib.orc_fp_binop_timed(0 if name == "add" else 2, *(P(x) for x in h), P(olo), P(ohi), m, 1)
            fp[name]["cpu_baseline"] = {"value": m / secs / 1e9, "unit": "Gop/s", "cores": 1, "kind": "port",
                                        "sample": f"{m} elements"}
            glo = bufs[4][:m].cpu().numpy().view(np.uint64)
            fp[name]["gpu_output_matches"] = bool(np.array_equal(glo, olo))
    res["fp127_cfg2"] = fp
    del bufs
    res["ct_add_sub_cfg3"] = add_bench(eng, args, with_cpu)
    res["ct_mul_with_sigma"] = sigma_bench(eng, args, with_cpu)
    res["cfg4_chain"] = chain_bench(eng, args)
    res["enc_value"] = enc_bench(eng, args, with_cpu)
    res["ct_mul_host_roundtrip"] = _host_roundtrip()
    res["ct_mul_single"] = _single_call()
    return res


def _single_call(calls=100):
    """Latency of ONE by-value drop-in call, as the reference's callers make them
    (tests/test_main.cpp:178-188, :291-292): pvac_hip::ct_mul(pk, A, B) with sigma, host Cipher in
    and out, on fresh x fresh and on chain-step-3 x fresh (tests/cpp/test_adapter --time-single).
    Reported next to the reference binary's 108.6 ms per ct_mul; never the headline."""
    import subprocess
    exe = os.path.join(ROOT, "tests", "cpp", "build", "test_adapter")
    if not os.path.exists(exe):
        return None
    try:
        outp = subprocess.run([exe, "--time-single", str(calls)], capture_output=True, text=True, timeout=300)
        r = json.loads([l for l in outp.stdout.splitlines() if l.startswith("{")][-1])
        r["path"] = "pvac_hip::ct_mul(pk, A, B) with sigma, one call at a time, tests/cpp/test_adapter --time-single"
        r["reference_ms_per_call"] = 108.6   # BASELINE.md, fresh x fresh with sigma, 1 core
        return r
    except Exception as ex:
        return {"error": repr(ex)}


def _host_roundtrip(pairs=1 << 15):
    """PCIe-inclusive rate through the C++ drop-in adapter (include/pvac_hip.hpp): host AoS
    ciphers in and out (AoS -> SoA, H2D, plan + exec, D2H, SoA -> AoS), weights only. Never the
    headline value; reported so the device-resident value can be read against it."""
    import subprocess
    exe = os.path.join(ROOT, "tests", "cpp", "build", "test_adapter")
    if not os.path.exists(exe):
        return None
    try:
        outp = subprocess.run([exe, "--time", str(pairs)], capture_output=True, text=True, timeout=300)
        r = json.loads([l for l in outp.stdout.splitlines() if l.startswith("{")][-1])
        r["path"] = "pvac_hip::ct_mul_batch (host Cipher vectors), tests/cpp/test_adapter --time"
        return r
    except Exception as ex:
        return {"error": repr(ex)}


def _add_cpu_prep(A, B, k):
    return k, _pack_host(A, k), _pack_host(B, k)


def _add_cpu(eng, cpu, C_, neg, args):
    """The pinned port's ct_add / ct_sub on the first k pairs of the same batch (1 thread and the
    box's CPU share), edge digests compared with the GPU output."""
    import ctypes as C
    import numpy as np
    from helpers import Oracle, default_params
    orc = Oracle.load()
    prm = default_params(0x5EED0003)
    k, a, b = cpu
    P = lambda x: x.ctypes.data_as(C.c_void_p)
    out = {}
    for th in (1, max(1, args.cpu_share_threads)):
        cnt, dig = np.zeros(k, np.uint64), np.zeros(k, np.uint64)
        secs = orc.lib.orc_ct_add_batch_timed(C.byref(prm), k, *(P(x) for x in a), *(P(x) for x in b), int(neg), th,
                                              P(cnt), P(dig))
        out[th] = (secs, cnt, dig)
    secs, cnt, dig = out[1]
    u = lambda t: t.cpu().numpy().view(np.uint64)
    mt = max(1, args.cpu_share_threads)
    return {"value": k / secs, "unit": "ops/s", "cores": 1, "kind": "port",
            "sample": f"the first {k} pairs of the batch, weights-only, {secs:.2f} s",
            "multi_thread": {"value": k / out[mt][0], "cores": mt, "seconds": out[mt][0]},
            "gpu_output_matches": bool(np.array_equal(u(eng.digest(_head(C_, k))), dig) and
                                       np.array_equal(u(C_.e_cnt[:k]), cnt))}


def add_bench(eng, args, with_cpu=False):
    """Batched ct_add / ct_sub / ct_scale (A13 / A6) on the cfg-3 batch shape (2^20 fresh-shaped pairs,
    weights only): the k_ct_add stream kernel against the HBM roofline. Algorithmic bytes per
    pair: every input edge read and written once (2 x 24 B x (|A.E| + |B.E|)), every layer record
    read and written (2 x 40 B x (|A.L| + |B.L|)), plus 5 x 8 B of counts / offsets per cipher."""
    import torch
    dev = eng.device
    n = args.pairs if args.pairs else 1 << 20
    A = eng.gen_fresh(n, 0x5EED0A01, args.epl)
    B = eng.gen_fresh(n, 0x5EED0A02, args.epl)
    res = {"pairs": n}
    cpu = _add_cpu_prep(A, B, min(args.cpu_pairs, n)) if with_cpu else None
    for name, neg in (("add", False), ("sub", True)):
        C_ = eng.ct_add(A, B, negate=neg)   # warm-up
        if cpu is not None:
            res.setdefault("cpu_baseline", {})[name] = _add_cpu(eng, cpu, C_, neg, args)
        del C_
        torch.cuda.synchronize(dev)
        eng.timing_reset()
        eng.timing(True)
        reps = 5
        t0 = time.perf_counter()
        for _ in range(reps):
            C_ = None
            C_ = eng.ct_add(A, B, negate=neg)
        torch.cuda.synchronize(dev)
        el = (time.perf_counter() - t0) / reps
        eng.timing(False)
        ms, cnt = eng.timing_get("ct_add")
        avg = ms / max(cnt, 1)
        ne = float((A.e_cnt[:n] + B.e_cnt[:n]).sum().item())
        nl = float((A.l_cnt[:n] + B.l_cnt[:n]).sum().item())
        alg = 48.0 * ne + 80.0 * nl + 5 * 8.0 * 3 * n
        res[name] = {"ops_per_s": n / el, "ms_per_batch": el * 1000, "avg_kernel_ms": avg,
                     "achieved_GBs": alg / (avg / 1000.0) / 1e9 if avg > 0 else None,
                     "frac_of_hbm_peak": alg / (avg / 1000.0) / 1e9 / HBM_PEAK_GBS if avg > 0 else None,
                     "output_edges": int(C_.e_cnt[:n].sum().item())}
        del C_
    # ct_scale (A6), in place on A: each edge's weight read and written (2 x 16 B) plus its count/offset
    s = (1 << 100) + 12345
    for _ in range(2):
        eng.ct_scale(A, s)
    torch.cuda.synchronize(dev)
    eng.timing_reset()
    eng.timing(True)
    for _ in range(5):
        eng.ct_scale(A, s)
    torch.cuda.synchronize(dev)
    eng.timing(False)
    ms, cnt = eng.timing_get("ct_scale")
    avg = ms / max(cnt, 1)
    ne_a = float(A.e_cnt[:n].sum().item())
    alg = 32.0 * ne_a + 16.0 * n
    res["scale"] = {"avg_kernel_ms": avg, "ops_per_s": n / (avg / 1000.0) if avg > 0 else None,
                    "achieved_GBs": alg / (avg / 1000.0) / 1e9 if avg > 0 else None,
                    "frac_of_hbm_peak": alg / (avg / 1000.0) / 1e9 / HBM_PEAK_GBS if avg > 0 else None}
    del A, B
    torch.cuda.empty_cache()
    return res


def sigma_bench(eng, args, with_cpu):
    """Full ct_mul WITH sigma (reference-complete ct_mul, f1) on a smaller batch."""
    import torch
    from pvac_hfhe_cppbyv_amd import MUL_WITH_SIGMA
    dev = eng.device
    ns = args.sigma_pairs
    eng.gen_H()
    A = eng.gen_fresh(ns, 0x51, args.epl)
    B = eng.gen_fresh(ns, 0x52, args.epl)
    Cb, plan = eng.ct_mul_plan(A, B)
    nonces = torch.empty(2 * plan.total_layer_slots, dtype=torch.int64, device=dev)
    salts = torch.empty(plan.total_edge_slots, dtype=torch.int64, device=dev)
    eng.fill_random(nonces, 0x53)
    eng.fill_random(salts, 0x54)
    eng.ct_mul(A, B, nonces=nonces, salts=salts, flags=MUL_WITH_SIGMA, C_=Cb, plan=plan)
    torch.cuda.synchronize(dev)
    eng.timing_reset()
    eng.timing(True)
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        Cb, plan = eng.ct_mul_plan(A, B)
        Cs = eng.ct_mul(A, B, nonces=nonces, salts=salts, flags=MUL_WITH_SIGMA, C_=Cb, plan=plan)
    torch.cuda.synchronize(dev)
    el = (time.perf_counter() - t0) / reps
    eng.timing(False)
    sms, scnt = eng.timing_get("sigma")
    edges = float(Cs.e_cnt[:ns].sum().item())
    sig_avg = sms / max(scnt, 1)
    sig_bytes = edges * 1024.0 + edges * (8 + 8) + edges * 8   # sigma written + meta/salt read
    full = {"pairs": ns, "ct_mul_per_s": ns / el, "ms_per_batch": el * 1000,
            "sigma_kernel_ms": sig_avg, "sigma_GBs": sig_bytes / (sig_avg / 1000.0) / 1e9,
            "edges": edges}
    # self-check (untimed): the same batch through two other column expansions of k_sigma (u16 rows,
    # the generic guarded loop: different tables and decoders, same selection) gives the same bytes
    # for every sigma of the batch (PVAC_SIGMA_PATH, read per launch)
    if os.environ.get("PVAC_SIGMA_PATH") is None:
        agree = {}
        cnt = Cs.e_cnt[:ns].long()
        start = torch.repeat_interleave(Cs.e_off[:ns].long() - (torch.cumsum(cnt, 0) - cnt), cnt)
        rows = start + torch.arange(int(cnt.sum().item()), device=dev)   # the written edge slots
        ref = Cs.sigma[rows].clone()
        for path in ("u16", "generic"):
            os.environ["PVAC_SIGMA_PATH"] = path
            try:
                Cb2, plan2 = eng.ct_mul_plan(A, B)
                C2 = eng.ct_mul(A, B, nonces=nonces, salts=salts, flags=MUL_WITH_SIGMA, C_=Cb2, plan=plan2)
                torch.cuda.synchronize(dev)
                agree[path] = bool(torch.equal(C2.sigma[rows], ref))
            finally:
                del os.environ["PVAC_SIGMA_PATH"]
            del C2, Cb2
        full["checks"] = {"sigma_paths_agree": all(agree.values()), "paths": ["delta"] + list(agree)}
    # k_sigma is not HBM-bound (1 KiB written per edge): VALU issue (SHA-256) and the LDS pipe (its
    # atomic-XOR flips) bound it; the counters come from profiles/pmc/sigma.json when it was taken on
    # this library binary and this batch
    rec, why = pmc_record("sigma", {"pairs": ns, "edges": edges})
    full["roofline"] = {"bound": "valu+lds", "valu": valu_roofline(eng, rec, why, sig_avg, edges, "edge"),
                        "traffic": rec.get("traffic") if rec else None,
                        "lds_active_frac": rec.get("lds_active_frac") if rec else None}
    if with_cpu:
        full["cpu_baseline"] = _ref_full_baseline()
    return full


ENC_STRIDE = 256   # random words per enc_value (the reference draws ~170; status 1 if short)


def _enc_keys(eng):
    """Synthetic key material for enc_value: random prf_k / LPN secret, H from canon_tag,
    powg_B = powers of an element of order B, as keygen makes it (so the gsum invariant holds)."""
    import numpy as np
    P = (1 << 127) - 1
    rng = np.random.default_rng(0xE1C)
    eng.gen_H()
    eng.set_secret(rng.integers(0, 2**64, 4, dtype=np.uint64), rng.integers(0, 2**64, 64, dtype=np.uint64))
    from pvac_hfhe_cppbyv_amd import powg_table
    eng.set_powg(powg_table(eng.params.B, int(rng.integers(2, 2**62))))


def enc_bench(eng, args, with_cpu):
    """f2: batched enc_value (LPN PRF + signal/noise equations + sigma), synthetic key material
    (random prf_k / LPN secret, powg_B = powers of a random element), draws from a device stream."""
    import numpy as np
    import torch
    dev = eng.device
    _enc_keys(eng)
    n, stride = args.enc_values, ENC_STRIDE
    vals = torch.empty(n, dtype=torch.int64, device=dev)
    rnd = torch.empty(n * stride, dtype=torch.int64, device=dev)
    eng.fill_random(vals, 0xE1)
    eng.fill_random(rnd, 0xE2)
    res = {"values": n}
    for sig in (False, True):
        C_, st = eng.enc_value(vals, rnd, sigma=sig)   # warm-up
        torch.cuda.synchronize(dev)
        eng.timing_reset()
        eng.timing(True)
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            C_, st = eng.enc_value(vals, rnd, sigma=sig)
        torch.cuda.synchronize(dev)
        el = (time.perf_counter() - t0) / reps
        eng.timing(False)
        ms, cnt = eng.timing_get("enc_value")
        key = "with_sigma" if sig else "weights_only"
        res[key] = {"enc_per_s": n / el, "ms_per_batch": el * 1000, "avg_call_ms": ms / max(cnt, 1),
                    "edges": int(C_.e_cnt[:n].sum().item()), "status_nonzero": int((st != 0).sum())}
    if with_cpu:
        res["cpu_baseline"] = _ref_enc_baseline()
    return res


def _ref_enc_baseline():
    """The UNMODIFIED reference enc_value (full, incl. sigma and the 16384-row LPN) on one core."""
    import subprocess
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    if not os.path.exists(exe):
        return None
    try:
        outp = subprocess.run([exe, "time_enc", "64"], capture_output=True, text=True, timeout=120)
        line = [l for l in outp.stdout.splitlines() if l.startswith("{")][-1]
        r = json.loads(line)
        return {"value": r["enc_per_s"], "unit": "enc_value/s", "cores": 1, "kind": "reference",
                "sample": f"{r['calls']} enc_value calls (reference pvac-hfhe 0.1.0), {r['seconds']:.2f} s"}
    except Exception as ex:
        return {"error": repr(ex)}


def chain_bench(eng, args):
    """cfg 4 (SURVEY 8(d) restatement of test_depth): x_i = enc_value(v_i) on the GPU for all 2^16
    inputs (timed on its own), then c_0 = x_i, c_k = ct_mul(c_{k-1}, x_i) to depth 8
    (tests/test_main.cpp:289-295). One library call (pvac_hip_ct_mul_chain) runs every chain: the
    engine cuts the inputs into chunks and runs them on `--chain-streams` internal worker streams,
    each step plan + exec on the general path. The timed pass does nothing else: no checks, no
    read-backs, wall clock from the call to its return. A second, untimed pass with the same nonces
    runs the reference's gsum invariant on every pair of every step and digests every final chain;
    its digests must equal the timed pass's (first chains) and the pinned CPU port's."""
    import numpy as np
    import torch
    from pvac_hfhe_cppbyv_amd import DeviceBatch, powg_table
    dev = eng.device
    n, chunk, depth = args.chain_inputs, min(args.chain_chunk, args.chain_inputs), args.chain_depth
    n_chk = max(0, min(args.chain_check, n))
    S = max(1, args.chain_streams)
    seed = 0x5EED0040
    # the earlier side legs' cached blocks go back to the driver first (the chain's workers size
    # their scratch from the free HBM)
    torch.cuda.synchronize(dev)
    torch.cuda.empty_cache()
    torch.cuda.reset_peak_memory_stats(dev)
    _enc_keys(eng)
    eng.set_powg(powg_table(eng.params.B))
    vals = torch.empty(n, dtype=torch.int64, device=dev)
    rnd = torch.empty(n * ENC_STRIDE, dtype=torch.int64, device=dev)
    eng.fill_random(vals, 0x5EED0004)
    eng.fill_random(rnd, 0x5EED1004)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    X_all, st = eng.enc_value(vals, rnd)   # status read back = synchronised
    enc_s = time.perf_counter() - t0
    del rnd
    bad = int((st != 0).sum())
    in_edges = float(X_all.e_cnt[:n].sum().item())

    def view(c0, k):   # chunk of the producer's batch (offsets are absolute: no copy)
        return DeviceBatch(k, X_all.l_off[c0:c0 + k], X_all.l_cnt[c0:c0 + k], X_all.layers, X_all.e_off[c0:c0 + k],
                           X_all.e_cnt[c0:c0 + k], X_all.meta, X_all.w_lo, X_all.w_hi)

    # warm-up (untimed): one chunk per worker through every depth sizes each worker's arena and
    # output buffers (a first allocation of tens of GB waits for the driver to clear the VRAM)
    eng.ct_mul_chain(view(0, min(n, S * chunk)), depth, nonce_seed=seed ^ 0xFFFF, streams=S, chunk=chunk)
    torch.cuda.synchronize(dev)
    # timed pass: the chains and nothing else (the monotonic-clock window lets a kernel trace of the
    # same command pick out this pass's dispatches: tools/chain_window.py)
    w0 = time.monotonic_ns()
    t1 = time.perf_counter()
    # (final edge counts of every chain: copies; position-keyed sum digests of the first chunk of each
    # worker, S x chunk inputs: a sum digest reads the whole c_depth, ~1.4 ms of HBM per 1024 depth-8
    # chains, so all of them would add ~6% to the chain's kernel time; the serial FNV-1a digests come
    # from the check pass, which must reproduce every count and these sum digests)
    n_sd = min(n, 4 * chunk)   # a fixed prefix: the timed pass digests 4 chunks whatever the stream count
    r = eng.ct_mul_chain(X_all, depth, nonce_seed=seed, streams=S, chunk=chunk, count_n=n, sumdigest=n_sd)
    torch.cuda.synchronize(dev)
    chain_s = time.perf_counter() - t1
    w1 = time.monotonic_ns()
    peak = torch.cuda.max_memory_reserved(dev) / 1e9
    if args.chain_no_check:   # profiling runs: the warm-up and the timed pass only
        del X_all, vals
        return {"inputs": n, "depth": depth, "chunk": chunk, "streams": S, "chain_seconds": chain_s,
                "ct_mul_per_s": n * depth / chain_s, "timed_window_monotonic_ns": [w0, w1],
                "edges_per_input_by_step": [e / n for e in r["edges"]], "products": float(sum(r["products"])),
                "redo_pairs": r["redo"], "image_pair_steps": r["image_steps"], "peak_hbm_reserved_gb": peak}
    # check pass (untimed): same nonces, gsum invariant on every pair-step, every final digest
    t2 = time.perf_counter()
    rc = eng.ct_mul_chain(X_all, depth, nonce_seed=seed, streams=S, chunk=chunk, check_gsum=True, digest_n=n_chk,
                          count_n=n, sumdigest=n_sd)
    check_s = time.perf_counter() - t2
    same = bool(np.array_equal(rc["counts"], r["counts"]))
    same_dig = bool(np.array_equal(rc["sumdigests"], r["sumdigests"]))
    x_host = _pack_host(X_all, n_chk) if n_chk else None   # the sampled chains' inputs
    del X_all, vals
    products = float(sum(r["products"]))
    out = {"inputs": n, "depth": depth, "chunk": chunk, "streams": S, "producer": "GPU enc_value (weights-only)",
           "engine_call": "pvac_hip_ct_mul_chain (one caller thread; the engine's own worker streams)",
           "seconds": enc_s + chain_s, "enc_seconds": enc_s, "chain_seconds": chain_s,
           "library_seconds": r["seconds"],
           "chains_per_s": n / (enc_s + chain_s), "ct_mul_per_s": n * depth / chain_s,
           "ct_mul_per_s_incl_enc": n * depth / (enc_s + chain_s),
           "timing": "wall clock of the timed call alone (synchronised on both sides); no checks or read-backs "
                     "inside it; the invariant and digests come from a second, untimed pass",
           "enc_status_nonzero": bad, "input_edges_per_value": in_edges / n,
           "products": products, "Gfp_mul_per_s": products / chain_s / 1e9,
           "edges_per_input_by_step": [e / n for e in r["edges"]],
           "redo_pairs": r["redo"], "peak_hbm_reserved_gb": peak, "timed_window_monotonic_ns": [w0, w1],
           "image_pair_steps": r["image_steps"],
           "intermediate_layout": "dense images between steps 3..depth-1 (include/pvac_hip.h): the timed pass; "
                                  "the check pass (gsum on every step) keeps records throughout, and its final "
                                  "counts and sum digests must equal the timed pass's"}
    gf, gp = rc["gsum_failed"], rc["gsum_pairs"]
    out["invariant"] = {"check": "check_mul_gsum_all (reference utils/metrics.hpp:88-113) on every pair of every "
                                 "step, on the device (second, untimed pass with the same nonces)", "pair_steps": gp,
                        "failed": gf, "invariant_ok": gf == 0 and gp == n * depth, "check_pass_seconds": check_s,
                        "timed_pass_counts_equal": same,
                        "timed_pass_sumdigests_equal": same_dig, "sumdigest_inputs": n_sd,
                        "edges_equal": rc["edges"] == r["edges"]}
    # Roofline of the products: per second against the matrix-core ceiling measured on this GPU
    # (k_ubench.hip k_probe_mfma8: back-to-back v_mfma_i32_32x32x32_i8, 64 dense-mode products
    # each); the round-2 column-accumulator (col26_mac) and round-1 fp_mul_fold1 VALU ceilings
    # beside it. The chain step is bound by memory latency and traffic, not by either.
    try:
        ceil = eng.alu_ceiling(5)
        out["roofline"] = {"bound": "mfma", "achieved": products / chain_s, "peak": ceil, "unit": "products/s",
                           "frac": products / chain_s / ceil,
                           "peak_source": "pvac_hip_alu_ceiling(5): back-to-back v_mfma_i32_32x32x32_i8 x 64 "
                                          "products, 8 waves/SIMD",
                           "col26_ceiling": eng.alu_ceiling(3), "fold1_ceiling": eng.alu_ceiling(1)}
    except Exception as ex:
        out["roofline"] = {"error": repr(ex)}
    # chain PMC record (profiles/pmc/chain.json, tools/pmc_target.sh chain): HBM traffic and VALU /
    # MFMA counts per input chain of the same depth / chunk / streams, when taken on this binary
    crec, cwhy = pmc_record("chain", {"depth": depth, "chunk": chunk, "streams": S})
    if crec:
        ni = max(1, (crec.get("workload") or {}).get("inputs") or 1)
        tot = crec.get("total") or {}
        out["pmc_per_input"] = {
            "hbm_write_bytes": tot.get("hbm_write_bytes", 0) / ni, "hbm_read_bytes": tot.get("hbm_read_bytes_corrected", 0) / ni,
            "kernels": {k: {f: v / ni for f, v in d.items() if f in ("traffic", "valu_insts")}
                        for k, d in (crec.get("kernels") or {}).items()},
            "inputs_profiled": ni, "lib_sha256": crec.get("lib_sha256"), "source": PMC_SOURCE}
    else:
        out["pmc_per_input"] = {"note": cwhy}
    if args.chain_compare_streams:
        # the same call with S worker streams and with ONE on 4 chunks per worker of new inputs
        try:
            out["streams_compare"] = _chain_streams_compare(eng, args, min(n, 4 * S * chunk), depth, chunk, S, seed)
        except Exception as ex:
            out["streams_compare"] = {"error": repr(ex)}
    if n_chk and x_host is not None:
        out.update(_chain_cpu(args, x_host, n_chk, depth, rc["digests"][:n_chk], rc["counts"][:n_chk],
                              n * depth / chain_s))
    return out


def _chain_streams_compare(eng, args, k, depth, chunk, S, seed):
    """ct_mul/s of the chain call on k fresh enc_value inputs with S worker streams and with 1."""
    import torch
    vals = torch.empty(k, dtype=torch.int64, device=eng.device)
    rnd = torch.empty(k * ENC_STRIDE, dtype=torch.int64, device=eng.device)
    eng.fill_random(vals, 0x5EED2004)
    eng.fill_random(rnd, 0x5EED3004)
    X, _ = eng.enc_value(vals, rnd)
    res = {"inputs": k}
    for s in (S, 1):
        eng.ct_mul_chain(X, depth, nonce_seed=seed, streams=s, chunk=chunk)   # warm
        torch.cuda.synchronize(eng.device)
        t = time.perf_counter()
        eng.ct_mul_chain(X, depth, nonce_seed=seed, streams=s, chunk=chunk)
        torch.cuda.synchronize(eng.device)
        res[f"streams_{s}_ct_mul_per_s"] = k * depth / (time.perf_counter() - t)
    return res


def _head(X, k):
    """View of the first k ciphers of a batch (absolute offsets: no copy)."""
    from pvac_hfhe_cppbyv_amd import DeviceBatch
    return DeviceBatch(k, X.l_off[:k], X.l_cnt[:k], X.layers, X.e_off[:k], X.e_cnt[:k], X.meta, X.w_lo, X.w_hi)


def _chain_cpu(args, x_host, k, depth, gpu_dig, gpu_cnt, gpu_rate):
    """cfg 4's CPU side on the bench's own first k chains (same enc_value inputs): the pinned port
    (oracle/pvac_oracle.cpp, the reference's unordered_map aggregation) runs c_j = ct_mul(c_{j-1}, x)
    to the same depth on 1 thread and on the box's CPU share, and its final edge digests must equal
    the GPU's; the unmodified reference (oracle/_ref, full ct_mul with sigma) is timed on a short chain."""
    import ctypes as C
    import numpy as np
    from helpers import Oracle, default_params
    orc = Oracle.load()
    prm = default_params(0x5EED0003)
    lo, lay, eo, meta, wl, wh = x_host
    P = lambda x: x.ctypes.data_as(C.c_void_p)
    res = {}
    runs = {}
    for th in (1, max(1, args.cpu_share_threads)):
        cnt, dig, se = np.zeros(k, np.uint64), np.zeros(k, np.uint64), np.zeros(depth, np.uint64)
        secs = orc.lib.orc_ct_mul_chain_timed(C.byref(prm), k, P(lo), P(lay), P(eo), P(meta), P(wl), P(wh), depth, th,
                                              P(cnt), P(dig), P(se))
        runs[th] = (secs, cnt, dig, se)
    secs, cnt, dig, se = runs[1]
    ok = gpu_dig is not None and bool(np.array_equal(dig, gpu_dig) and np.array_equal(cnt, gpu_cnt))
    res["oracle_sample_ok"] = ok
    res["oracle_sample"] = {"chains": k, "depth": depth, "check": "final c_depth edge digests (meta, w) and edge "
                            "counts of the bench's first chains vs the pinned CPU port on the same enc_value inputs",
                            "edges_per_input_by_step": [float(x) / k for x in se]}
    mt = max(1, args.cpu_share_threads)
    res["cpu_baseline"] = {
        "value": k * depth / secs, "unit": "ct_mul/s", "cores": 1, "kind": "port",
        "sample": f"{k} chains to depth {depth} (the bench's first {k} enc_value inputs), weights-only, {secs:.2f} s",
        "multi_thread": {"value": k * depth / runs[mt][0], "cores": mt, "seconds": runs[mt][0]},
        "impl": "oracle/pvac_oracle.cpp orc_ct_mul_chain_timed (pinned to the reference by tests/test_oracle.py)",
        "gpu_over_cpu_1core": gpu_rate / (k * depth / secs)}
    ref = _ref_chain_baseline(args.chain_ref)
    if ref:
        res["cpu_baseline"]["reference"] = ref
    return res


def _ref_chain_baseline(ninputs, depth=4):
    """The UNMODIFIED reference's chain (full ct_mul WITH sigma, tests/test_main.cpp:289-295 shape):
    depth 4 on a few inputs, since its sigma stage costs ~104 us per output edge (depth 8 would take
    ~80 s per chain)."""
    import subprocess
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    if not os.path.exists(exe) or ninputs <= 0:
        return None
    try:
        outp = subprocess.run([exe, "time_chain", str(ninputs), str(depth)], capture_output=True, text=True,
                              timeout=240)
        r = json.loads([l for l in outp.stdout.splitlines() if l.startswith("{")][-1])
        return {"value": r["ct_mul_per_s"], "unit": "ct_mul/s", "cores": 1, "kind": "reference",
                "sample": f"{r['inputs']} chains to depth {r['depth']} (reference pvac-hfhe 0.1.0, enc_value inputs, "
                          f"full ct_mul with sigma), {r['seconds']:.2f} s",
                "edges_by_step": r["edges_by_step"]}
    except Exception as ex:
        return {"error": repr(ex)}


def _ref_full_baseline():
    """The UNMODIFIED reference ct_mul (with sigma) when oracle/_ref was built here and shipped;
    otherwise None."""
    import subprocess
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    if not os.path.exists(exe):
        return None
    try:
        outp = subprocess.run([exe, "time_mul", "96", "1"], capture_output=True, text=True, timeout=120)
        line = [l for l in outp.stdout.splitlines() if l.startswith("{")][-1]
        r = json.loads(line)
        return {"value": r["ct_mul_per_s"], "unit": "ct_mul/s", "cores": 1, "kind": "reference",
                "sample": f"{r['pairs']} fresh x fresh ct_mul (reference pvac-hfhe 0.1.0, with sigma), "
                          f"{r['seconds']:.2f} s"}
    except Exception as ex:
        return {"error": repr(ex)}


if __name__ == "__main__":
    main()
