"""Phase split of k_large_products_direct (GPU box, diagnostic build only): runs the cfg-4 chain on
one worker stream through lib/exp/libpvac_hip_dirst.so (make variant-f VFILE=k_mul_large VNAME=dirst
VFLAGS=-DPVAC_DIR_STAMPS) and prints wave 0's s_memtime cycles per phase summed over workgroups:
0 setup / loop, 1 dense staging (A-layer gather), 2 matrix-core rows, 3 range writer; per A layer;
the same for k_large_count_la (setup, stage_tt, key records, iblk counts + writer list).
Usage: python tools/diag_direct.py [inputs]"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from pvac_hfhe_cppbyv_amd import Engine, load_library  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    lib = load_library(os.path.join(ROOT, "pvac_hfhe_cppbyv_amd", "lib", "exp", "libpvac_hip_dirst.so"))
    eng = Engine(device=0, canon_tag=0x5EED0003, lib=lib)
    bench._enc_keys(eng)
    vals = torch.empty(n, dtype=torch.int64, device=eng.device)
    rnd = torch.empty(n * bench.ENC_STRIDE, dtype=torch.int64, device=eng.device)
    eng.fill_random(vals, 0x5EED0004)
    eng.fill_random(rnd, 0x5EED1004)
    X, st = eng.enc_value(vals, rnd)
    eng.ct_mul_chain(X, 8, streams=1, chunk=1024)
    torch.cuda.synchronize()
    buf = (C.c_ulonglong * 24)()
    lib.pvac_hip_diag_dir_stamps(buf, 1)
    eng.ct_mul_chain(X, 8, streams=1, chunk=1024)
    torch.cuda.synchronize()
    assert lib.pvac_hip_diag_dir_stamps(buf, 1) == 0
    v = list(buf)
    tot = sum(v[:4]) + sum(v[16:21])
    names = ["setup", "stage_dense", "mfma_rows", "writer"]
    out = {"a_layers": v[4], "workgroups": v[5], "cycles_total": tot}
    for i, nm in enumerate(names):
        out[nm] = {"frac": round(v[i] / max(tot, 1), 4), "cycles_per_a_layer": round(v[i] / max(v[4], 1))}
    # the writer's parts (phase 3 above is the record writer's output loop plus the layer's last wait):
    # image steps (intermediate): entries + offsets, key expansion into the LDS position table, the
    # coalesced cell pass; record steps (final): entries + offsets + scan, key expansion
    for i, nm in enumerate(["img_entries", "img_expand", "rec_entries", "rec_expand", "img_cells"]):
        out["writer_" + nm] = {"frac": round(v[16 + i] / max(tot, 1), 4), "cycles_per_a_layer": round(v[16 + i] / max(v[4], 1))}
    tc = sum(v[8:12])
    out["count_la"] = {"a_layers": v[12], "cycles_total": tc, "list_entries_per_a_layer": round(v[13] / max(v[12], 1), 1)}
    for i, nm in enumerate(["setup", "stage_tt", "keys", "iblk_list"]):
        out["count_la"][nm] = {"frac": round(v[8 + i] / max(tc, 1), 4), "cycles_per_a_layer": round(v[8 + i] / max(v[12], 1))}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
