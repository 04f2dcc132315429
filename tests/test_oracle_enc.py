"""Pins the oracle's LPN PRF and enc_value restatement (oracle/pvac_oracle.cpp) to the reference's
own outputs minted by oracle/ref_harness.cpp (cmd_enc): prf_R_core over 12 seeds x 6 domains,
prf_R, prf_R_noise and prf_noise_delta, and 12 complete enc_value outputs with the getrandom
streams they consumed. Also checks the 127-row truncation of prf_R_core against the reference's
full 16384-row loop, restated (full_rows=1). CPU only."""
import os

import numpy as np
import pytest

from helpers import REF, fixture_secret, read_ct, read_u64, write_ct


@pytest.fixture(scope="module")
def key():
    return fixture_secret()


def _seeds_outs():
    seeds = read_u64("prf_seeds.u64").reshape(-1, 3)
    return seeds, read_u64("prf_out.u64").reshape(len(seeds), -1, 2)


def test_prf_core_fixtures(oracle, key):
    sk, man, _ = key
    seeds, outs = _seeds_outs()
    for k, sd in enumerate(seeds):
        for d in range(6):
            assert oracle.prf_core(sk, man["canon_tag"], sd, d) == tuple(int(x) for x in outs[k, d]), (k, d)
        assert oracle.prf_R(sk, man["canon_tag"], sd) == tuple(int(x) for x in outs[k, 6])
        assert oracle.prf_R(sk, man["canon_tag"], sd, noise=True) == tuple(int(x) for x in outs[k, 7])
        for kind in range(2):
            for g in range(5):
                got = oracle.prf_noise_delta(sk, man["canon_tag"], sd, g, kind)
                assert got == tuple(int(x) for x in outs[k, 8 + 5 * kind + g]), (k, kind, g)


def test_prf_core_truncation_is_exact(oracle, key):
    """toep_127 only reads LPN rows 0..126: the full loop gives the same value."""
    sk, man, _ = key
    seeds, outs = _seeds_outs()
    sd = seeds[3]
    assert oracle.prf_core(sk, man["canon_tag"], sd, 2, full=True) == oracle.prf_core(sk, man["canon_tag"], sd, 2)
    assert oracle.prf_core(sk, man["canon_tag"], sd, 2, full=True) == tuple(int(x) for x in outs[3, 2])


def test_enc_value_fixtures_weights(oracle, key):
    sk, man, em = key
    powg = read_u64("powg_B.u64")
    for i, rec in enumerate(em["enc"]):
        ref = read_ct(os.path.join(REF, f"enc{i}.ct"))[0]
        st = read_u64(f"enc{i}_stream.u64")
        c, used = oracle.enc_value(sk, rec["v"], st, powg, canon_tag=man["canon_tag"])
        assert used == len(st) == rec["stream"]
        assert c.nE == ref.nE == rec["edges"] and c.nL == ref.nL == rec["layers"]
        for f in ("rule", "ztag", "nonce_lo", "nonce_hi"):
            assert np.array_equal(c.layers[f], ref.layers[f]), f
        assert np.array_equal(c.meta, ref.meta)
        assert np.array_equal(c.w_lo, ref.w_lo) and np.array_equal(c.w_hi, ref.w_hi)


def test_enc_value_fixture_with_sigma_bytes(oracle, key):
    """One complete enc_value including every sigma: the .ct bytes equal the reference's file."""
    sk, man, em = key
    H, digest = oracle.gen_H(man["canon_tag"])
    assert digest.hex() == man["H_digest"]
    powg = read_u64("powg_B.u64")
    i = 3
    st = read_u64(f"enc{i}_stream.u64")
    c, _ = oracle.enc_value(sk, em["enc"][i]["v"], st, powg, H=H, canon_tag=man["canon_tag"])
    with open(os.path.join(REF, f"enc{i}.ct"), "rb") as f:
        assert write_ct([c]) == f.read()


def test_enc_value_depth_and_zero_fixtures(oracle, key):
    """enc_value_depth (depth hints 1, 3, 8, 15) and enc_zero_depth (0, 5): the oracle reproduces the
    reference's .ct bytes, sigmas included, from the streams it consumed (ref_harness encdepth)."""
    import json
    sk, man, _ = key
    H, _ = oracle.gen_H(man["canon_tag"])
    powg = read_u64("powg_B.u64")
    with open(os.path.join(REF, "encd_manifest.json")) as f:
        fm = json.load(f)
    for i, c in enumerate(fm["cases"]):
        st = read_u64(f"encd{i}_stream.u64")
        got, used = oracle.enc_value(sk, c["v"], st, powg, H=H, canon_tag=man["canon_tag"], depth=c["depth"])
        assert used == len(st) == c["stream"] and got.nE == c["edges"], i
        with open(os.path.join(REF, f"encd{i}.ct"), "rb") as f:
            assert write_ct([got]) == f.read(), i


def test_enc_deep_depth_and_noise_params_fixtures(oracle, key):
    """enc_value_depth / enc_zero_depth past depth hint 15 (16, 31, 60, 100) and with non-default noise
    Params (noise_entropy_bits, tuple2_fraction, depth_slope_bits), including a plan with no noise group
    and one bumped from one group to two (plan_noise, ops/encrypt.hpp:16-27): the oracle reproduces the
    reference's .ct bytes from the streams it consumed (ref_harness encdeep)."""
    import json
    sk, man, _ = key
    H, _ = oracle.gen_H(man["canon_tag"])
    powg = read_u64("powg_B.u64")
    with open(os.path.join(REF, "encx_manifest.json")) as f:
        fm = json.load(f)
    try:
        for i, c in enumerate(fm["cases"]):
            oracle.set_noise(c["noise_entropy_bits"], c["tuple2_fraction"], c["depth_slope_bits"])
            st = read_u64(f"encx{i}_stream.u64")
            got, used = oracle.enc_value(sk, c["v"], st, powg, H=H, canon_tag=man["canon_tag"], depth=c["depth"])
            assert used == len(st) == c["stream"] and got.nE == c["edges"], i
            with open(os.path.join(REF, f"encx{i}.ct"), "rb") as f:
                assert write_ct([got]) == f.read(), i
    finally:
        oracle.set_noise()
