"""A/B of the element-wise Fp kernels (GPU box): BASELINE cfg 2's 2^24-element add and mul through
each library given, average kernel time over 20 launches (HIP events), alternating libraries.
Outputs are compared with the first library's. Usage: python tools/fp_ab.py lib1.so [lib2.so ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from pvac_hfhe_cppbyv_amd import FP_ADD, FP_MUL, Engine, load_library  # noqa: E402


def main():
    n = 1 << 24
    g = torch.Generator(device="cuda").manual_seed(7)
    a = [torch.randint(-2**62, 2**62, (n,), dtype=torch.int64, device="cuda", generator=g) for _ in range(4)]
    a[1] &= (1 << 62) - 1
    a[3] &= (1 << 62) - 1
    res, ref = {}, {}
    for path in sys.argv[1:]:
        lib = load_library(path)
        eng = Engine(device=0, lib=lib)
        name = os.path.basename(path)
        for opn, op in (("add", FP_ADD), ("mul", FP_MUL)):
            out = eng.fp_binop(op, a[0], a[1], a[2], a[3])
            torch.cuda.synchronize()
            eng.timing_reset()
            eng.timing(True)
            for _ in range(20):
                eng.fp_binop(op, a[0], a[1], a[2], a[3], out=out)
            torch.cuda.synchronize()
            eng.timing(False)
            ms, k = eng.timing_get("fp_binop")
            key = f"{name}:{opn}"
            res[key] = round(ms / max(k, 1), 4)
            dig = (out[0].sum().item(), out[1].sum().item())
            same = ref.setdefault(opn, dig) == dig
            print(key, res[key], "ms", round(48 * n / (res[key] * 1e-3) / 1e9), "GB/s", "same" if same else "DIFFERENT",
                  flush=True)
        # ct_scale over cfg 3's 2^20 fresh ciphers (41.9 M weights, read and written in place)
        X = eng.gen_fresh(1 << 20, 0x5EED0003, 20)
        ne = int(X.e_cnt.sum().item())
        eng.ct_scale(X, 3)
        torch.cuda.synchronize()
        eng.timing_reset()
        eng.timing(True)
        for _ in range(20):
            eng.ct_scale(X, 3)
        torch.cuda.synchronize()
        eng.timing(False)
        ms, k = eng.timing_get("ct_scale")
        key = f"{name}:scale"
        res[key] = round(ms / max(k, 1), 4)
        dig = eng.digest(X).sum().item()
        same = ref.setdefault("scale", dig) == dig
        print(key, res[key], "ms", round(32 * ne / (res[key] * 1e-3) / 1e9), "GB/s", "same" if same else "DIFFERENT",
              flush=True)
        del X, eng
    print(json.dumps(res))


if __name__ == "__main__":
    main()
