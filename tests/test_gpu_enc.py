"""GPU LPN PRF and enc_value (k_prf.hip, k_enc.hip; reference crypto/lpn.hpp:159-275,
ops/encrypt.hpp:114-291) against the reference's own outputs (oracle/ref_harness.cpp cmd_enc:
prf_R_core over 12 seeds x 6 domains, prf_R, prf_R_noise, prf_noise_delta; complete enc_value
outputs with their getrandom streams) and the pinned oracle on random seeds."""
import os

import numpy as np
import pytest

from helpers import REF, fixture_secret, read_ct, read_u64

pytestmark = pytest.mark.gpu


def _eng(H="gen"):
    from pvac_hfhe_cppbyv_amd import Engine
    sk, man, em = fixture_secret()
    eng = Engine(device=0, canon_tag=man["canon_tag"])
    assert eng.gen_H().hex() == man["H_digest"]
    eng.set_secret(read_u64("sk_prf_k.u64"), read_u64("sk_lpn_s.u64"), em["lpn_n"], em["lpn_t"], em["lpn_tau_num"],
                   em["lpn_tau_den"])
    eng.set_powg(read_u64("powg_B.u64"))
    return eng, sk, man, em


def _pairs(a):
    return [int(a[i, 0]) | (int(a[i, 1]) << 64) for i in range(len(a))]


def test_prf_fixtures():
    eng, _, _, _ = _eng()
    seeds = read_u64("prf_seeds.u64").reshape(-1, 3)
    outs = read_u64("prf_out.u64").reshape(len(seeds), -1, 2)
    for kind in range(8):
        assert eng.prf(kind, seeds) == _pairs(outs[:, kind]), kind


def test_prf_random_vs_oracle(oracle):
    eng, sk, man, _ = _eng()
    rng = np.random.default_rng(77)
    seeds = rng.integers(0, 2**64, (300, 3), dtype=np.uint64)
    got = eng.prf(4, seeds)
    for i in range(0, 300, 7):
        lo, hi = oracle.prf_core(sk, man["canon_tag"], seeds[i], 4)
        assert got[i] == lo | (hi << 64)
    got6 = eng.prf(6, seeds[:16])
    for i in range(16):
        lo, hi = oracle.prf_R(sk, man["canon_tag"], seeds[i])
        assert got6[i] == lo | (hi << 64)


def test_prf_digest_from_dense_H(oracle):
    """set_H (dense host matrix) derives the same H_digest the PRF keys depend on."""
    from pvac_hfhe_cppbyv_amd import Engine
    sk, man, em = fixture_secret()
    eng = Engine(device=0, canon_tag=man["canon_tag"])
    H, d = oracle.gen_H(man["canon_tag"])
    eng.set_H(H)
    eng.set_secret(read_u64("sk_prf_k.u64"), read_u64("sk_lpn_s.u64"))
    seeds = read_u64("prf_seeds.u64").reshape(-1, 3)
    outs = read_u64("prf_out.u64").reshape(len(seeds), -1, 2)
    assert eng.prf(6, seeds) == _pairs(outs[:, 6])
