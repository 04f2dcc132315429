"""A/B timing of k_ct.hip variants (GPU box): bench.py's ct_add / ct_sub / ct_scale leg on the cfg-3
batch through each library given (make variant-ct); prints the kernel averages.
Usage: python tools/exp_add.py lib1.so [lib2.so ...]"""
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
    args = types.SimpleNamespace(pairs=0, epl=20)
    for path in sys.argv[1:]:
        eng = Engine(device=0, canon_tag=0x5EED0003, lib=load_library(path))
        r = bench.add_bench(eng, args)
        key = os.path.basename(path)
        res[key] = {k: round(v["avg_kernel_ms"], 4) for k, v in r.items() if isinstance(v, dict) and "avg_kernel_ms" in v}
        print(key, res[key], flush=True)
        del eng
        torch.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
