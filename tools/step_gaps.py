"""Timeline of one bench step from a rocprofv3 kernel trace: every dispatch between two
consecutive launches of an anchor kernel (default k_ct_mul_fresh3), with the idle gaps.
Usage: python3 tools/step_gaps.py <kernel_trace.csv> [anchor] [steps]"""
import csv
import re
import sys


def main():
    path = sys.argv[1]
    anchor = sys.argv[2] if len(sys.argv) > 2 else "k_ct_mul_fresh3"
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ev = []
    for r in rows:
        m = re.search(r"(k_\w+)", r["Kernel_Name"])
        ev.append((m.group(1) if m else r["Kernel_Name"][:40], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    idx = [k for k, e in enumerate(ev) if e[0] == anchor]
    for a, b in list(zip(idx, idx[1:]))[-steps:]:
        t0 = ev[a][1]
        busy = 0
        last_end = t0
        print(f"--- step: {anchor} at {t0}, next at +{(ev[b][1] - t0) / 1e3:.1f} us")
        for name, s, e in ev[a:b + 1]:
            gap = (s - last_end) / 1e3
            print(f"  {(s - t0) / 1e3:10.1f} us  +gap {gap:8.1f}  {name:40s} {(e - s) / 1e3:10.1f} us")
            busy += e - s
            last_end = max(last_end, e)
        span = ev[b][1] - t0
        print(f"  span {span / 1e3:.1f} us, busy {busy / 1e3:.1f} us, idle {(span - busy) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
