"""Debug helper (GPU box): runs chain steps 1-2 of the golden fixtures through the engine and
saves the outputs under gpurun_out/ for a host-side diff against the oracle."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import REF, Cipher, read_ct, read_layers_u64, read_u64  # noqa: E402
from test_gpu_large import _run_mul  # noqa: E402
import json  # noqa: E402

from pvac_hfhe_cppbyv_amd import Engine  # noqa: E402

man = json.load(open(os.path.join(REF, "manifest.json")))
eng = Engine(device=0, canon_tag=man["canon_tag"])
c1 = Cipher(read_layers_u64("chain1_layers.u64"), *[getattr(read_ct(os.path.join(REF, "chain1.ct"))[0], f)
                                                     for f in ("meta", "w_lo", "w_hi")])
x = read_ct(os.path.join(REF, "chain2_x.ct"))[0]
out, plan, _ = _run_mul(eng, [c1], [x], [read_u64("chain2_stream.u64")])
o = out[0]
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", "dbg_chain2.npz"), meta=o.meta, lo=o.w_lo, hi=o.w_hi,
         layers=o.layers.view(np.uint8))
print("saved", o.nE, plan.n_large)
