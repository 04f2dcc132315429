"""A/B of enc_value (GPU box): bench.py's enc_bench (16,384 values, weights only and with sigma)
through each library given; prints values/s and the enc_value launches' average time. Outputs are compared
by a digest of the weights-only batch. Usage: python tools/enc_ab.py lib1.so [lib2.so ...]"""
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
    res, ref = {}, None
    args = types.SimpleNamespace(enc_values=1 << 14)
    for path in sys.argv[1:]:
        eng = Engine(device=0, canon_tag=0x5EED0003, lib=load_library(path))
        eng.timing_reset()
        eng.timing(True)
        r = bench.enc_bench(eng, args, False)
        eng.timing(False)
        ms, k = eng.timing_get("enc_value")
        name = os.path.basename(path)
        # outputs: one more weights-only batch from a fixed stream, digested
        n, stride = 4096, bench.ENC_STRIDE
        vals = torch.empty(n, dtype=torch.int64, device=eng.device)
        rnd = torch.empty(n * stride, dtype=torch.int64, device=eng.device)
        eng.fill_random(vals, 0xA1)
        eng.fill_random(rnd, 0xA2)
        X, st = eng.enc_value(vals, rnd)
        dig = int(eng.digest(X).sum().item())
        ref = dig if ref is None else ref
        res[name] = {"enc_per_s": round(r["weights_only"]["enc_per_s"]), "with_sigma": round(r["with_sigma"]["enc_per_s"]),
                     "enc_kernel_ms": round(ms / max(k, 1), 3), "same": dig == ref}
        print(name, json.dumps(res[name]), flush=True)
        del eng, X, vals, rnd
        torch.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
