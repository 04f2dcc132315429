"""cfg-4 chain A/B (GPU box): the chain call (pvac_hip_ct_mul_chain) on the same GPU enc_value inputs through
each library given, alternating, with 1 and with 4 worker streams; final digests must agree between
libraries. Usage: python tools/chain_ab.py [--inputs N] [--streams 1,4] [--chunks 1024] lib1.so [lib2.so ...]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from pvac_hfhe_cppbyv_amd import Engine, load_library  # noqa: E402


def main():
    argv = sys.argv[1:]
    n = 16384
    streams = (1, 4)
    chunks = (1024,)
    while argv and argv[0] in ("--inputs", "--streams", "--chunks"):
        if argv[0] == "--inputs":
            n = int(argv[1])
        elif argv[0] == "--chunks":
            chunks = tuple(int(x) for x in argv[1].split(","))
        else:
            streams = tuple(int(x) for x in argv[1].split(","))
        argv = argv[2:]
    res = {}
    ref = None
    for path in argv:
        eng = Engine(device=0, canon_tag=0x5EED0003, lib=load_library(path))
        bench._enc_keys(eng)
        vals = torch.empty(n, dtype=torch.int64, device=eng.device)
        rnd = torch.empty(n * bench.ENC_STRIDE, dtype=torch.int64, device=eng.device)
        eng.fill_random(vals, 0x5EED0004)
        eng.fill_random(rnd, 0x5EED1004)
        X, st = eng.enc_value(vals, rnd)
        del rnd
        name = os.path.basename(path)
        for s, c in [(s, c) for s in streams for c in chunks]:
            eng.ct_mul_chain(X, 8, streams=s, chunk=c)   # warm: arenas, buffers
            torch.cuda.synchronize()
            t = time.perf_counter()
            r = eng.ct_mul_chain(X, 8, streams=s, chunk=c, digest_n=64)
            torch.cuda.synchronize()
            el = time.perf_counter() - t
            k = f"{name}:s{s}" + (f":c{c}" if len(chunks) > 1 else "")
            res[k] = round(n * 8 / el)
            same = ref is None or bool(np.array_equal(ref, r["digests"]))
            if ref is None:
                ref = r["digests"]
            print(k, res[k], "ct_mul/s", "same" if same else "DIFFERENT", "redo", r["redo"], "image_steps",
                  r.get("image_steps"), flush=True)
        del X, eng
        torch.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
