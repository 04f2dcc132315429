#!/usr/bin/env python3
"""Per-opcode VALU issue rates on this GPU (pvac_hip_issue_probe) with the shader clock measured in
the same launch, and the two older mixed probes (pvac_hip_alu_ceiling kinds 0 and 4) beside them.

cycles per wave64 instruction per SIMD = SIMDs x clock / (instructions per second), SIMDs = CUs x 4.
Prints one JSON object (GPU box): python3 tools/issue_probe.py > gpurun_out/issue_probe.json"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from pvac_hfhe_cppbyv_amd import Engine
    eng = Engine(device=0)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    simds = 4 * cus
    res = {"cus": cus, "simds": simds, "ops": {}}
    for wps in (1, 2, 4, 8):
        for op in Engine.ISSUE_OPS:
            per_s, hz = eng.issue_probe(op, wps)
            res["ops"].setdefault(op, {})[f"wps{wps}"] = {
                "inst_per_s": per_s, "clock_hz": hz,
                "cycles_per_inst": simds * hz / per_s if per_s else None}
    for kind, name in ((4, "mix32_kind4"), (0, "madmix_kind0")):
        per_s = eng.alu_ceiling(kind)
        hz = res["ops"]["v_add_u32"]["wps8"]["clock_hz"]
        res[name] = {"inst_per_s": per_s, "cycles_per_inst_at_add_clock": simds * hz / per_s if per_s else None}
    json.dump(res, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
