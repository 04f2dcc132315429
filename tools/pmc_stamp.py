#!/usr/bin/env python3
"""One PMC record per bench target (tools/pmc_target.sh), stamped with the library it profiled.

The record carries the sha256 of pvac_hfhe_cppbyv_amd/lib/libpvac_hip.so as it was on the GPU box,
the workload the bench ran (parsed from the bench's own JSON line in the pass logs) and, per launch
of the target kernel (headline, sigma: mean over the full-size dispatches) or per timed chain (chain:
totals over the dispatches inside the bench's monotonic window):

* HBM traffic: 2 x FETCH_SIZE (the guide's wide-read correction) + WRITE_SIZE, in bytes;
* VALU: SQ_INSTS_VALU, and the counter-measured VALU-busy fraction
  valu_busy = 4 x SQ_ACTIVE_INST_VALU / (kernel cycles x SIMDs): SQ_ACTIVE_INST_* count quad-cycles
  (MI355X_MICROARCH.md, 's_memtime tick vs SQ PMC units'); kernel cycles = GRBM_GUI_ACTIVE / 8 XCDs;
  1,024 SIMDs (256 CUs x 4). The same fraction with SQ_BUSY_CYCLES as the clock is given beside it;
* LDS: SQ_LDS_IDX_ACTIVE and SQ_LDS_BANK_CONFLICT over CU cycles; wait fraction SQ_WAIT_ANY /
  SQ_WAVE_CYCLES; the shader clock the kernel ran at (kernel cycles / its duration).

bench.py quotes `traffic` / `valu` from a record only when its lib_sha256 equals the sha256 of the
library bench.py itself loaded, and writes null plus the reason otherwise."""
import argparse
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
LIB = os.path.join(ROOT, "pvac_hfhe_cppbyv_amd", "lib", "libpvac_hip.so")
N_SIMD = 1024
N_CU = 256
KERNEL = {"headline": "k_ct_mul_fresh3", "sigma": "k_sigma"}


def lib_sha256(path=LIB):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()


def bench_line(d):
    """The bench's JSON line from the first pass log that has one."""
    for i in range(1, 9):
        p = os.path.join(d, f"p{i}.log")
        if not os.path.exists(p):
            continue
        for line in open(p, errors="replace").read().splitlines():
            if line.startswith("{"):
                try:
                    return json.loads(line)
                except ValueError:
                    pass
    return {}


def derived(m, launches=1):
    """Per-record derived figures from summed (per launch or per window) counters."""
    r = {}
    cyc = m.get("GRBM_GUI_ACTIVE", 0) / 8.0 / max(launches, 1)
    if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
        r["hbm_read_bytes"] = 2 * m["FETCH_SIZE"] * 1024
        r["hbm_write_bytes"] = m["WRITE_SIZE"] * 1024
        r["traffic"] = r["hbm_read_bytes"] + r["hbm_write_bytes"]
    if "SQ_INSTS_VALU" in m:
        r["valu_insts"] = m["SQ_INSTS_VALU"]
    if cyc and "SQ_ACTIVE_INST_VALU" in m:
        r["kernel_cycles"] = cyc
        r["valu_busy"] = 4.0 * m["SQ_ACTIVE_INST_VALU"] / max(launches, 1) / (cyc * N_SIMD)
    if m.get("SQ_BUSY_CYCLES") and "SQ_ACTIVE_INST_VALU" in m and cyc:
        sq_units = m["SQ_BUSY_CYCLES"] / max(launches, 1) / cyc   # SQ_BUSY_CYCLES sums the SQs' clocks
        r["sq_units"] = sq_units
        r["valu_busy_sq_clock"] = 4.0 * m["SQ_ACTIVE_INST_VALU"] / (m["SQ_BUSY_CYCLES"] * N_SIMD / sq_units)
    if cyc and "SQ_LDS_IDX_ACTIVE" in m:
        r["lds_active_frac"] = m["SQ_LDS_IDX_ACTIVE"] / max(launches, 1) / (N_CU * cyc)
    if cyc and "SQ_LDS_BANK_CONFLICT" in m:
        r["lds_bank_conflict_frac"] = m["SQ_LDS_BANK_CONFLICT"] / max(launches, 1) / (N_CU * cyc)
    if m.get("SQ_WAVE_CYCLES") and "SQ_WAIT_ANY" in m:
        r["wait_frac"] = m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"]
    if m.get("SQ_INSTS_VALU") and "SQ_INSTS_VALU_INT32" in m:
        r["int32_frac"] = m["SQ_INSTS_VALU_INT32"] / m["SQ_INSTS_VALU"]
        r["int64_frac"] = m.get("SQ_INSTS_VALU_INT64", 0) / m["SQ_INSTS_VALU"]
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--target", required=True, choices=["headline", "sigma", "chain"])
    ap.add_argument("--dir", required=True)
    ap.add_argument("bench_args", nargs="*")
    a = ap.parse_args()
    line = bench_line(a.dir)
    rec = {"target": a.target, "lib_sha256": lib_sha256(), "bench_args": a.bench_args,
           "source": "rocprofv3 --pmc, one counter group per run (tools/pmc_target.sh); derived figures: "
                     "tools/pmc_stamp.py"}
    if a.target in KERNEL:
        import pmc_summary
        summ = pmc_summary.summarize(a.dir)
        k = summ.get(KERNEL[a.target], {})
        rec["kernel"] = KERNEL[a.target]
        rec["counters_per_launch"] = {n: v for n, v in k.items() if n.isupper() or n.startswith(("SQ_", "GRBM_"))}
        rec["dispatches"] = k.get("dispatches")
        rec.update(derived(k))
        if a.target == "headline":
            cfg = line.get("config", {})
            rec["workload"] = {"pairs": cfg.get("pairs_per_gpu"), "epl": cfg.get("edges_per_layer")}
            rec["alg_bytes_per_launch"] = line.get("roofline", {}).get("alg_bytes_per_launch")
            rec["kernel_ms_bench"] = line.get("roofline", {}).get("avg_kernel_ms")
        else:
            rec["workload"] = {"pairs": line.get("pairs"), "edges": line.get("edges")}
            rec["kernel_ms_bench"] = line.get("sigma_kernel_ms")
        if rec.get("kernel_cycles") and rec.get("kernel_ms_bench"):
            rec["clock_hz_est"] = rec["kernel_cycles"] / (rec["kernel_ms_bench"] * 1e-3)
    else:
        import pmc_chain_summary
        summ = pmc_chain_summary.summarize(a.dir)
        rec["workload"] = {"inputs": line.get("inputs"), "depth": line.get("depth"), "chunk": line.get("chunk"),
                           "streams": line.get("streams")}
        kern = {}
        for name, m in summ.items():
            if name.startswith("_"):
                continue
            d = derived(m, launches=1)
            d["dispatches"] = m.get("dispatches")
            d["ms_by_pass"] = m.get("ms_by_pass")
            d.pop("kernel_cycles", None)   # window totals: GRBM sums every dispatch, per-kernel cycles overlap
            d.pop("valu_busy", None)
            d.pop("valu_busy_sq_clock", None)
            d.pop("lds_active_frac", None)
            d.pop("lds_bank_conflict_frac", None)
            kern[name] = d
        rec["kernels"] = kern
        rec["total"] = summ.get("_total")
        rec["timed_window_monotonic_ns"] = line.get("timed_window_monotonic_ns")
    json.dump(rec, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main()
