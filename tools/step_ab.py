"""Whole-step A/B (GPU box): the bench's cfg-3 step (ct_mul_plan + ct_mul over 2^20 fresh pairs, the
nonces filled once) through each library given, wall clock per step over 10 steps after 2 warm-up
steps; outputs compared with the first library's. Catches host-side costs (read-backs, waits,
launch gaps) that a kernel timer does not see. Usage: python tools/step_ab.py lib1.so [lib2.so ...]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from pvac_hfhe_cppbyv_amd import Engine, load_library  # noqa: E402


def main():
    n, steps = 1 << 20, 10
    res, ref = {}, None
    for path in sys.argv[1:]:
        eng = Engine(device=0, canon_tag=0x5EED0003, lib=load_library(path))
        A = eng.gen_fresh(n, 0x5EED0003, 20)
        B = eng.gen_fresh(n, 0x5EED0004, 20)
        Cb, plan = eng.ct_mul_plan(A, B)
        nonces = eng.fill_nonces(A, B, Cb, plan, 0x5EED0005)
        out = None
        for _ in range(2):
            out = None
            Cb, plan = eng.ct_mul_plan(A, B)
            out = eng.ct_mul(A, B, nonces=nonces, C_=Cb, plan=plan)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            out = None
            Cb, plan = eng.ct_mul_plan(A, B)
            out = eng.ct_mul(A, B, nonces=nonces, C_=Cb, plan=plan)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / steps
        dig = eng.digest(out).cpu()
        lay = out.layers[:plan.total_layer_slots].cpu()   # the layer records (ztags) too
        same = ref is None or (bool(torch.equal(dig, ref[0])) and bool(torch.equal(lay, ref[1])))
        if ref is None:
            ref = (dig, lay)
        name = os.path.basename(path)
        res[name] = round(ms, 4)
        print(name, round(ms, 4), "ms/step", "same" if same else "DIFFERENT", flush=True)
        del out, dig, lay, A, B, Cb, plan, nonces, eng
        torch.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
