"""A/B timing of k_fp.hip variants (GPU box): cfg-2 element-wise Fp127 add / mul on 2^24 elements
through each library given (make variant-f VFILE=k_fp); prints the kernel averages in ms.
Usage: python tools/exp_fp.py lib1.so [lib2.so ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from pvac_hfhe_cppbyv_amd import FP_ADD, FP_MUL, Engine, load_library  # noqa: E402


def main():
    res = {}
    n = 1 << 24
    for path in sys.argv[1:]:
        eng = Engine(device=0, canon_tag=0x5EED0002, lib=load_library(path))
        bufs = [torch.empty(n, dtype=torch.int64, device=eng.device) for _ in range(6)]
        for i, t in enumerate(bufs[:4]):
            eng.fill_random(t, 0x5EED0002 + i)
        bufs[1] &= (1 << 63) - 1
        bufs[3] &= (1 << 63) - 1
        r = {}
        for name, op in (("add", FP_ADD), ("mul", FP_MUL)):
            for _ in range(3):
                eng.fp_binop(op, *bufs[:4], out=(bufs[4], bufs[5]))
            eng.timing_reset()
            eng.timing(True)
            for _ in range(20):
                eng.fp_binop(op, *bufs[:4], out=(bufs[4], bufs[5]))
            eng.timing(False)
            ms, cnt = eng.timing_get("fp_binop")
            r[name] = round(ms / max(cnt, 1), 4)
        res[os.path.basename(path)] = r
        print(os.path.basename(path), r, flush=True)
        del eng, bufs
        torch.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
