"""Workgroup residency of the fresh ct_mul kernel from the CENSUS build (lib/libpvac_hip_census.so):
per-workgroup start / end times and CU ids. Diagnostic only: never used by tests or bench.py.
Usage (GPU box): python tools/census_fresh.py [pairs]"""
import ctypes as C
import collections
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from pvac_hfhe_cppbyv_amd import Engine, load_library  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    lib = load_library(os.path.join(ROOT, "pvac_hfhe_cppbyv_amd", "lib", "libpvac_hip_census.so"))
    lib.pvac_hip_diag_census.argtypes = [C.c_void_p, C.c_size_t]
    eng = Engine(device=0, canon_tag=0x5EED0003, lib=lib)
    A = eng.gen_fresh(n, 0x5EED0003, 20)
    B = eng.gen_fresh(n, 0x5EED0004, 20)
    for _ in range(2):
        Cb, plan = eng.ct_mul_plan(A, B)
        nonces = eng.fill_nonces(A, B, Cb, plan, 1)
        eng.ct_mul(A, B, nonces=nonces, C_=Cb, plan=plan)
    torch.cuda.synchronize()
    st = np.zeros(4096 * 4, np.uint64)
    assert lib.pvac_hip_diag_census(st.ctypes.data_as(C.c_void_p), st.size) == 0
    st = st.reshape(4096, 4)
    used = st[st[:, 1] > 0]
    t0 = used[:, 0].min()
    start = (used[:, 0] - t0) / 100.0   # us (100 MHz)
    end = (used[:, 1] - t0) / 100.0
    print("workgroups", len(used), "kernel span us %.1f" % end.max())
    print("start us: min %.1f p50 %.1f p90 %.1f max %.1f" % tuple(np.percentile(start, [0, 50, 90, 100])))
    print("end   us: min %.1f p50 %.1f p90 %.1f max %.1f" % tuple(np.percentile(end, [0, 50, 90, 100])))
    print("pairs per wg: min %d max %d" % (used[:, 2].min(), used[:, 2].max()))
    hw = used[:, 3].astype(np.int64)
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 0x7
    key = list(zip(se, sh, cu))
    cnt = collections.Counter(key)
    late = start > 0.25 * end.max()
    print("distinct (se, sh, cu) ids", len(cnt), "max wg per id", max(cnt.values()), "late starters", int(late.sum()))


if __name__ == "__main__":
    main()
