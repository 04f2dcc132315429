"""Shard invariance on the GPU: the union of two shards (generated and multiplied with global
pair indices, as bench.py's ranks do) equals one single-GPU batch, pair for pair."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_two_shards_equal_one_batch():
    from pvac_hfhe_cppbyv_amd import Engine
    eng = Engine(device=0, canon_tag=0x5EED0005)
    n = 1024

    def run(first, count):
        A = eng.gen_fresh(count, 0x51, 20, first_index=first)
        B = eng.gen_fresh(count, 0x52, 20, first_index=first)
        Cb, plan = eng.ct_mul_plan(A, B)
        nonces = eng.fill_nonces(A, B, Cb, plan, 0x53, first_index=first)
        out = eng.ct_mul(A, B, nonces=nonces, C_=Cb, plan=plan)
        dig = eng.digest(out).cpu().numpy().view(np.uint64)
        lay = out.to_host()
        return dig, [(c.nE, c.layers["ztag"].tobytes()) for c in lay]

    d_all, l_all = run(0, n)
    d0, l0 = run(0, n // 2)
    d1, l1 = run(n // 2, n - n // 2)
    assert np.array_equal(np.concatenate([d0, d1]), d_all)
    assert l0 + l1 == l_all
