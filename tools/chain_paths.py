"""Which ct_mul path each chain step takes (GPU box): runs chains step by step through the engine and
prints, per step, the path counters (fresh kernel, general path, its iblk order, direct mode), the
pairs' layer and edge counts, and the dense-image condition of each pair (every cell of every product
layer with edges filled). Usage: python tools/chain_paths.py [--four [--epl E]] [--B B] [--n N] [--depth D]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from pvac_hfhe_cppbyv_amd import Engine  # noqa: E402


def main():
    argv = sys.argv[1:]
    four = "--four" in argv
    n = int(argv[argv.index("--n") + 1]) if "--n" in argv else 3
    depth = int(argv[argv.index("--depth") + 1]) if "--depth" in argv else 4
    Bm = int(argv[argv.index("--B") + 1]) if "--B" in argv else 337
    eng = Engine(device=0, canon_tag=0xF0A4, B=Bm)
    if four:
        epl = int(argv[argv.index("--epl") + 1]) if "--epl" in argv else 15
        X = eng.ct_add(eng.gen_fresh(n, 0xF0A6, epl), eng.gen_fresh(n, 0xF0A7, epl))
    else:
        X = eng.gen_fresh(n, 0xF0A6, 20)
    lib = eng.lib
    lib.pvac_hip_bucket_count.restype = C.c_uint64
    cnt = (C.c_uint64 * 4)()
    cur = X
    for d in range(depth):
        lib.pvac_hip_ct_mul_path_count(eng.ctx, cnt)
        before = list(cnt)
        Cb, plan = eng.ct_mul_plan(cur, X)
        nonces = torch.empty(2 * max(plan.total_layer_slots, 1), dtype=torch.int64, device=eng.device)
        eng.fill_random(nonces, 0xF0A5 + d)
        nxt = eng.ct_mul(cur, X, nonces=nonces, C_=Cb, plan=plan)
        lib.pvac_hip_ct_mul_path_count(eng.ctx, cnt)
        delta = [a - b for a, b in zip(cnt, before)]
        la = cur.l_cnt[:n].cpu().tolist()
        na = cur.e_cnt[:n].cpu().tolist()
        nb = [int(lib.pvac_hip_bucket_count(C.c_uint64(a * int(X.e_cnt[i].item())))) for i, a in enumerate(na)]
        print(f"step {d + 1}: paths fresh/general/iblk/direct {delta}  |A.L| {la}  |A.E| {na}  buckets {nb}  "
              f"|C.E| {nxt.e_cnt[:n].cpu().tolist()}", flush=True)
        cur = nxt


if __name__ == "__main__":
    main()
