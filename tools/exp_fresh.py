"""Timing experiments on k_ct_mul_fresh (GPU box): cfg-3 batch through each library given, average
kernel time of the fresh kernel over 5 launches. The experiment libraries (make exp) each remove one
piece of work, so their outputs are wrong; the point is the marginal cost of that piece.
Usage: python tools/exp_fresh.py lib1.so [lib2.so ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from pvac_hfhe_cppbyv_amd import Engine, load_library  # noqa: E402


def main():
    n = 1 << 20
    res = {}
    ref = None
    for path in sys.argv[1:]:
        lib = load_library(path)
        eng = Engine(device=0, canon_tag=0x5EED0003, lib=lib)
        A = eng.gen_fresh(n, 0x5EED0003, 20)
        B = eng.gen_fresh(n, 0x5EED0004, 20)
        Cb, plan = eng.ct_mul_plan(A, B)
        nonces = eng.fill_nonces(A, B, Cb, plan, 1)
        eng.ct_mul(A, B, nonces=nonces, C_=Cb, plan=plan)
        torch.cuda.synchronize()
        eng.timing_reset()
        eng.timing(True)
        for _ in range(5):
            eng.ct_mul(A, B, nonces=nonces, C_=Cb, plan=plan)
        torch.cuda.synchronize()
        eng.timing(False)
        ms, k = eng.timing_get("ct_mul_fresh")
        res[os.path.basename(path)] = round(ms / max(k, 1), 3)
        lms, lk = eng.timing_get("mul_layers_fresh")
        res[os.path.basename(path) + ":layers_ms"] = round(lms / max(lk, 1), 4)
        # outputs vs the first library's (the product): a variant must be bit-exact
        out = eng.ct_mul(A, B, nonces=nonces, C_=Cb, plan=plan)
        dig = eng.digest(out).cpu()
        if ref is None:
            ref = dig
        same = bool(torch.equal(dig, ref))
        res[os.path.basename(path) + ":same_as_first"] = same
        res[os.path.basename(path) + ":redo"] = eng.ct_mul_redo_count()
        print(os.path.basename(path), res[os.path.basename(path)], "layers", res[os.path.basename(path) + ":layers_ms"],
              "same" if same else "DIFFERENT", flush=True)
        del out, dig
        del A, B, Cb, plan, nonces, eng
        torch.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
