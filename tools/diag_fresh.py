"""Per-phase wall time of k_ct_mul_fresh from the DIAGNOSTIC build (lib/libpvac_hip_diag.so,
s_memtime stamps of wave 0 per workgroup). Diagnostic only: never used by tests or bench.py.
Usage (GPU box): python tools/diag_fresh.py [pairs]"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from pvac_hfhe_cppbyv_amd import Engine, load_library  # noqa: E402

# k_ct_mul_fresh3 (default kernel): work phases end with an lgkmcnt(0) stamp, then the barrier wait
PHASES = ["loop top (header, rebuild)", "P1 key times", "  B1 wait", "P2 order", "  B2 wait", "P3 closure (wave 0)",
          "  B3 wait (scan)", "P4 positions", "  B4 wait", "P5 products", "  B5 wait", "P6 writer", "P6 reset+stage",
          "  B6 wait", "-", "-", "-", "-"]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    lib = load_library(os.path.join(ROOT, "pvac_hfhe_cppbyv_amd", "lib", "libpvac_hip_diag.so"))
    lib.pvac_hip_diag_fresh_stamps.argtypes = [C.c_void_p, C.c_size_t]
    eng = Engine(device=0, canon_tag=0x5EED0003, lib=lib)
    A = eng.gen_fresh(n, 0x5EED0003, 20)
    B = eng.gen_fresh(n, 0x5EED0004, 20)
    for _ in range(2):
        Cb, plan = eng.ct_mul_plan(A, B)
        nonces = eng.fill_nonces(A, B, Cb, plan, 1)
        eng.ct_mul(A, B, nonces=nonces, C_=Cb, plan=plan)
    torch.cuda.synchronize()
    st = np.zeros(4096 * 18, np.uint64)
    assert lib.pvac_hip_diag_fresh_stamps(st.ctypes.data_as(C.c_void_p), st.size) == 0
    st = st.reshape(4096, 18)
    used = st[st.sum(axis=1) > 0]
    tot = used.sum(axis=0).astype(np.float64)
    frac = tot / tot.sum()
    per_pair = tot / used.shape[0] / (n / used.shape[0])  # ticks per pair per workgroup
    print(json.dumps({"workgroups": int(used.shape[0]), "pairs": n,
                      "ticks_per_pair_per_wg": float(tot.sum() / n),
                      "phases": {PHASES[i]: {"frac": round(float(frac[i]), 4), "ticks_per_pair": round(float(per_pair[i]), 1)}
                                 for i in range(len(PHASES))}}, indent=1))


if __name__ == "__main__":
    main()
