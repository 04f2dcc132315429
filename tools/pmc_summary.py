#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs (tools/prof_pmc.sh) per kernel: mean per dispatch.

FETCH_SIZE/WRITE_SIZE are reported in KB by rocprofv3; HBM bytes per launch follow the
MI355X guide's correction: FETCH_SIZE counts 64 B per 128-B request for wide streaming reads,
so the read side is doubled (MI355X_MICROARCH.md, HBM section); WRITE_SIZE is taken as is.
No cycles-per-instruction constant: the VALU roofline divides SQ_INSTS_VALU per launch by the kernel
time and by the ceiling measured on the device (pvac_hip_alu_ceiling, bench.py roofline.valu).
lds_bank_conflict_frac = SQ_LDS_BANK_CONFLICT / (256 CUs x kernel cycles), wait_frac =
SQ_WAIT_ANY / SQ_WAVE_CYCLES.

Full-size dispatches only: a bench run launches the headline kernel on the whole batch (warm-up +
timed steps) and once more on the self-check window (4,096 pairs) with the SAME persistent grid, so
the grid size cannot tell them apart. Each pass keeps the dispatches whose duration is at least half
of that pass's longest one (the round-2 summaries averaged all four dispatches equally, which
scaled every per-launch figure by ~3/4). `dispatches` records how many were kept and dropped."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def summarize(root):
    acc = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(dict)   # (kernel, pass file) -> {dispatch: ns}
    for path in glob.glob(os.path.join(root, "**", "*counter_collection*.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                k = row.get("Kernel_Name", "?")
                short = k.replace("(anonymous namespace)", "anon").split("(")[0].split("<")[0].split("::")[-1]
                name = row.get("Counter_Name")
                try:
                    v = float(row.get("Counter_Value", "nan"))
                    ns = float(row.get("End_Timestamp", 0)) - float(row.get("Start_Timestamp", 0))
                except ValueError:
                    continue
                disp = (path, row.get("Dispatch_Id"))
                acc[short][(name, disp)].append(v)
                dur[(short, path)][disp] = ns
    out = {}
    for kern, d in acc.items():
        keep, dropped = set(), 0
        for (k2, _path), dd in dur.items():
            if k2 != kern or not dd:
                continue
            top = max(dd.values())
            for disp, ns in dd.items():
                if ns >= 0.5 * top:
                    keep.add(disp)
                else:
                    dropped += 1
        per = defaultdict(list)
        for (name, disp), vals in d.items():
            if disp in keep:
                per[name].append(sum(vals))   # sum over XCD/SE dimensions of one dispatch
        out[kern] = {n: sum(v) / len(v) for n, v in per.items()}
        m = out[kern]
        m["dispatches"] = {"kept_per_pass": max((len(v) for v in per.values()), default=0),
                           "dropped_short": dropped}
        if "FETCH_SIZE" in m:
            m["hbm_read_bytes_corrected"] = 2 * m["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in m:
            m["hbm_write_bytes"] = m["WRITE_SIZE"] * 1024
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            m["hbm_bytes_per_launch"] = m["hbm_read_bytes_corrected"] + m["hbm_write_bytes"]
        if m.get("GRBM_GUI_ACTIVE"):
            # GRBM_GUI_ACTIVE sums the 8 XCDs' clocks: kernel cycles = GRBM_GUI_ACTIVE / 8
            cyc = m["GRBM_GUI_ACTIVE"] / 8.0
            m["kernel_cycles"] = cyc
            if "SQ_LDS_BANK_CONFLICT" in m:
                m["lds_bank_conflict_frac"] = m["SQ_LDS_BANK_CONFLICT"] / (256.0 * cyc)
        if m.get("SQ_WAVE_CYCLES") and "SQ_WAIT_ANY" in m:
            m["wait_frac"] = m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"]
    return out


def main(root):
    json.dump(summarize(root), sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
