#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter CSVs (tools/prof_pmc.sh) per kernel: mean per dispatch.

FETCH_SIZE/WRITE_SIZE are reported in KB by rocprofv3; HBM bytes per launch follow the
MI355X guide's correction: FETCH_SIZE counts 64 B per 128-B request for wide streaming reads,
so the read side is doubled (MI355X_MICROARCH.md, HBM section); WRITE_SIZE is taken as is.
valu_busy_frac = SQ_INSTS_VALU x 4 cycles / (1024 SIMDs x kernel cycles): the integer-ALU roofline."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main(root):
    acc = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(os.path.join(root, "**", "*counter_collection*.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                k = row.get("Kernel_Name", "?")
                short = k.replace("(anonymous namespace)", "anon").split("(")[0].split("<")[0].split("::")[-1]
                name = row.get("Counter_Name")
                try:
                    v = float(row.get("Counter_Value", "nan"))
                except ValueError:
                    continue
                acc[short][(name, row.get("Dispatch_Id"))].append(v)
    out = {}
    for kern, d in acc.items():
        per = defaultdict(list)
        for (name, _disp), vals in d.items():
            per[name].append(sum(vals))   # sum over XCD/SE dimensions of one dispatch
        out[kern] = {n: sum(v) / len(v) for n, v in per.items()}
        m = out[kern]
        if "FETCH_SIZE" in m:
            m["hbm_read_bytes_corrected"] = 2 * m["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in m:
            m["hbm_write_bytes"] = m["WRITE_SIZE"] * 1024
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            m["hbm_bytes_per_launch"] = m["hbm_read_bytes_corrected"] + m["hbm_write_bytes"]
        if "SQ_INSTS_VALU" in m and m.get("GRBM_GUI_ACTIVE"):
            # a wave64 VALU instruction holds its 16-lane SIMD for 4 cycles; GRBM_GUI_ACTIVE sums the
            # 8 XCDs' clocks; 256 CUs x 4 SIMDs
            m["valu_busy_frac"] = m["SQ_INSTS_VALU"] * 4.0 / (1024.0 * m["GRBM_GUI_ACTIVE"] / 8.0)
    json.dump(out, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
