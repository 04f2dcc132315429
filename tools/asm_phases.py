"""Static instruction mix of k_ct_mul_fresh per phase: compiles csrc/k_mul_fresh.hip with
-DPVAC_ASM_MARKS (the PHASE_STAMP sites become asm comments) and counts VALU / SALU / LDS /
VMEM instructions between consecutive marks. Diagnostic only (CPU, no GPU).
Usage: python tools/asm_phases.py [extra hipcc flags]"""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "pvac_hfhe_cppbyv_amd", "csrc", "k_mul_fresh.hip")
OUT = "/tmp/k_mul_fresh_marks.s"


def main():
    cmd = ["/opt/rocm/bin/hipcc", "-std=c++17", "-O3", "--offload-arch=gfx950", "-x", "hip", "--cuda-device-only",
           "-S", "-DPVAC_ASM_MARKS", *sys.argv[1:], SRC, "-o", OUT]
    subprocess.check_call(cmd, stderr=subprocess.DEVNULL)
    lines = open(OUT).read().splitlines()
    kern = os.environ.get("KERNEL", "k_ct_mul_fresh3")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + kern + r"I\S*:", l))
    end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
    cur = "entry"
    cnt = collections.OrderedDict()
    for l in lines[start:end]:
        m = re.search(r"PVAC_MARK (\d+)", l)
        if m:
            cur = m.group(1)
            continue
        t = l.strip().split()
        if not t or t[0].startswith((";", ".")) or t[0].endswith(":"):
            continue
        op = t[0]
        cls = ("valu" if op.startswith("v_") else "salu" if op.startswith("s_") and not op.startswith(("s_waitcnt", "s_barrier", "s_cbranch", "s_branch", "s_load", "s_buffer")) else
               "lds" if op.startswith("ds_") else "vmem" if op.startswith(("global_", "buffer_", "flat_")) else
               "smem" if op.startswith(("s_load", "s_buffer")) else "ctl")
        d = cnt.setdefault(cur, collections.Counter())
        d[cls] += 1
    tot = collections.Counter()
    for k, d in cnt.items():
        tot.update(d)
        print(f"after mark {k:>5}: " + " ".join(f"{c}={d[c]}" for c in ("valu", "salu", "lds", "vmem", "smem", "ctl")))
    print("total:          " + " ".join(f"{c}={tot[c]}" for c in ("valu", "salu", "lds", "vmem", "smem", "ctl")))


if __name__ == "__main__":
    main()
