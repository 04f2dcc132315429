"""Timing experiments on k_sigma (GPU box): full ct_mul with sigma on 4096 fresh pairs through each
library given; prints the sigma kernel's average time. The experiment libraries (make exp) remove
one piece of work, so their sigmas are WRONG; the point is the marginal cost of that piece.
Usage: python tools/exp_sigma.py lib1.so [lib2.so ...]"""
import json
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from pvac_hfhe_cppbyv_amd import Engine, load_library  # noqa: E402


def main():
    res = {}
    args = types.SimpleNamespace(sigma_pairs=1 << 12, epl=20)
    for path in sys.argv[1:]:
        eng = Engine(device=0, canon_tag=0x5EED0003, lib=load_library(path))
        r = bench.sigma_bench(eng, args, False)
        res[os.path.basename(path)] = round(r["sigma_kernel_ms"], 3)
        res[os.path.basename(path) + ":checks"] = r.get("checks")
        print(os.path.basename(path), res[os.path.basename(path)], r.get("checks"), flush=True)
        del eng
        torch.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
