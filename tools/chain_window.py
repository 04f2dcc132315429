"""Per-kernel totals of the cfg-4 timed pass from a rocprofv3 kernel trace of `bench.py --only chain`:
keeps the dispatches that start inside the bench line's timed_window_monotonic_ns (rocprofv3
timestamps are CLOCK_MONOTONIC ns, like time.monotonic_ns()), sums their durations per kernel, and
checks them against the wall clock: the summed kernel time of S streams must not exceed S x the
window. Diagnostic only.
Usage: python tools/chain_window.py <kernel_trace.csv> <bench line json file> [out.json]"""
import collections
import csv
import json
import sys


def main():
    trace, line = sys.argv[1], sys.argv[2]
    d = json.loads([l for l in open(line).read().splitlines() if l.startswith("{")][-1])
    c = d.get("extras", {}).get("cfg4_chain", d)
    w0, w1 = c["timed_window_monotonic_ns"]
    tot = collections.Counter()
    cnt = collections.Counter()
    first, last = None, None
    with open(trace) as f:
        for row in csv.DictReader(f):
            s, e = int(row["Start_Timestamp"]), int(row["End_Timestamp"])
            if s < w0 or s > w1:
                continue
            k = row["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
            k = k.split("(")[0].split("<")[0].split("::")[-1].strip()
            tot[k] += e - s
            cnt[k] += 1
            first = s if first is None else min(first, s)
            last = e if last is None else max(last, e)
    wall = (w1 - w0) / 1e9
    ksum = sum(tot.values()) / 1e9
    out = {"window_s": wall, "kernel_seconds_sum": ksum, "streams": c.get("streams"),
           "sum_le_streams_x_window": ksum <= (c.get("streams") or 1) * wall,
           "busy_span_s": (last - first) / 1e9 if first else None,
           "ct_mul_per_s_bench": c.get("ct_mul_per_s"),
           "kernels": {k: {"ms": v / 1e6, "dispatches": cnt[k]} for k, v in tot.most_common()}}
    js = json.dumps(out, indent=1)
    print(js)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(js + "\n")


if __name__ == "__main__":
    main()
