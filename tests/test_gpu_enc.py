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


def _streams(em, stride):
    rnd = np.zeros((len(em["enc"]), stride), np.uint64)
    for i in range(len(em["enc"])):
        s = read_u64(f"enc{i}_stream.u64")
        rnd[i, :len(s)] = s
    return rnd


@pytest.mark.parametrize("sigma", [False, True])
def test_enc_value_fixtures(sigma):
    """The reference's getrandom streams reproduce its enc_value outputs (with sigma: byte-exact .ct)."""
    from helpers import write_ct
    eng, _, man, em = _eng()
    vals = np.array([r["v"] for r in em["enc"]], np.uint64)
    C_, st = eng.enc_value(vals, _streams(em, 256), sigma=sigma)
    assert not st.any()
    out = C_.to_host()
    for i in range(len(vals)):
        ref = read_ct(os.path.join(REF, f"enc{i}.ct"))[0]
        c = out[i]
        assert c.nE == ref.nE and c.nL == ref.nL
        assert np.array_equal(c.meta, ref.meta)
        assert np.array_equal(c.w_lo, ref.w_lo) and np.array_equal(c.w_hi, ref.w_hi)
        for f in ("rule", "ztag", "nonce_lo", "nonce_hi"):
            assert np.array_equal(c.layers[f], ref.layers[f]), f
        if sigma:
            from helpers import Cipher
            with open(os.path.join(REF, f"enc{i}.ct"), "rb") as f:
                assert write_ct([Cipher(c.layers, c.meta, c.w_lo, c.w_hi, c.sigma)]) == f.read()


def test_enc_value_random_vs_oracle(oracle):
    eng, sk, man, em = _eng()
    rng = np.random.default_rng(91)
    n, stride = 64, 256
    vals = rng.integers(0, 2**64, n, dtype=np.uint64)
    rnd = rng.integers(0, 2**64, (n, stride), dtype=np.uint64)
    C_, st = eng.enc_value(vals, rnd)
    assert not st.any()
    out = C_.to_host()
    powg = read_u64("powg_B.u64")
    for i in range(0, n, 5):
        ref, used = oracle.enc_value(sk, int(vals[i]), rnd[i], powg, canon_tag=man["canon_tag"])
        c = out[i]
        assert c.nE == ref.nE
        assert np.array_equal(c.meta, ref.meta)
        assert np.array_equal(c.w_lo, ref.w_lo) and np.array_equal(c.w_hi, ref.w_hi)
        assert np.array_equal(c.layers["ztag"], ref.layers["ztag"])


def test_enc_short_stream_status():
    eng, _, _, em = _eng()
    C_, st = eng.enc_value(np.array([5, 6], np.uint64), np.ones((2, 100), np.uint64))
    assert list(st) == [1, 1]


def test_enc_dec_roundtrip_with_gpu_prf():
    """dec(enc(v)) = v entirely on the GPU: enc_value, base_R (prf_R of BASE layers), dec_value."""
    eng, _, man, em = _eng()
    rng = np.random.default_rng(92)
    n = 256
    vals = rng.integers(0, 2**64, n, dtype=np.uint64)
    vals[:4] = [0, 1, 2**64 - 1, 12345]
    C_, st = eng.enc_value(vals, rng.integers(0, 2**64, (n, 256), dtype=np.uint64))
    assert not st.any()
    got, st2 = eng.dec_value(C_, eng.base_R(C_))
    assert not st2.any()
    assert got == [int(v) for v in vals]


@pytest.mark.parametrize("sigma", [False, True])
def test_enc_value_depth_and_zero_fixtures(sigma):
    """enc_value_depth (hints 1, 3, 8, 15) and enc_zero_depth (0, 5) on the GPU from the reference's
    streams: byte-exact .ct output (with sigma), every case decrypting to its value."""
    import json
    from helpers import write_ct
    eng, _, man, _ = _eng()
    with open(os.path.join(REF, "encd_manifest.json")) as f:
        fm = json.load(f)
    for i, c in enumerate(fm["cases"]):
        st = read_u64(f"encd{i}_stream.u64")
        _, ep, dh = eng.enc_caps(c["depth"])
        assert len(st) <= dh and c["edges"] <= ep
        rnd = np.zeros((1, dh), np.uint64)
        rnd[0, :len(st)] = st
        C_, status = eng.enc_value(np.array([c["v"]], np.uint64), rnd, sigma=sigma, depth=c["depth"])
        assert not status.any(), i
        got = C_.to_host()[0]
        ref = read_ct(os.path.join(REF, f"encd{i}.ct"))[0]
        assert np.array_equal(got.meta, ref.meta) and np.array_equal(got.w_lo, ref.w_lo), i
        assert np.array_equal(got.w_hi, ref.w_hi), i
        if sigma:
            from helpers import Cipher
            L = got.layers
            with open(os.path.join(REF, f"encd{i}.ct"), "rb") as f:
                assert write_ct([Cipher(L, got.meta, got.w_lo, got.w_hi, got.sigma)]) == f.read(), i
        R = eng.base_R(C_)
        vals, dst = eng.dec_value(C_, R)
        assert vals[0] == c["v"] and not dst.any(), i


@pytest.mark.parametrize("sigma", [False, True])
def test_enc_deep_depth_and_noise_params_fixtures(sigma):
    """enc_value_depth / enc_zero_depth past depth hint 15 (16, 31, 60, 100: the large plan-record
    class, up to 210 pre-merge edges per half) and with non-default noise Params set through
    pvac_hip_ctx_set_noise (a plan with no noise group, one bumped from one group to two): byte-exact
    .ct output against the reference's (ref_harness encdeep), sigmas included, and every case
    decrypting to its value."""
    import json
    from helpers import Cipher, write_ct
    eng, _, man, _ = _eng()
    with open(os.path.join(REF, "encx_manifest.json")) as f:
        fm = json.load(f)
    for i, c in enumerate(fm["cases"]):
        eng.set_noise(c["noise_entropy_bits"], c["tuple2_fraction"], c["depth_slope_bits"])
        st = read_u64(f"encx{i}_stream.u64")
        _, ep, dh = eng.enc_caps(c["depth"])
        assert len(st) <= dh and c["edges"] <= ep, i
        rnd = np.zeros((1, dh), np.uint64)
        rnd[0, :len(st)] = st
        C_, status = eng.enc_value(np.array([c["v"]], np.uint64), rnd, sigma=sigma, depth=c["depth"])
        assert not status.any(), i
        got = C_.to_host()[0]
        ref = read_ct(os.path.join(REF, f"encx{i}.ct"))[0]
        assert np.array_equal(got.meta, ref.meta) and np.array_equal(got.w_lo, ref.w_lo), i
        assert np.array_equal(got.w_hi, ref.w_hi), i
        if sigma:
            with open(os.path.join(REF, f"encx{i}.ct"), "rb") as f:
                assert write_ct([Cipher(got.layers, got.meta, got.w_lo, got.w_hi, got.sigma)]) == f.read(), i
        vals, dst = eng.dec_value(C_, eng.base_R(C_))
        assert vals[0] == c["v"] and not dst.any(), i


def test_enc_depth_beyond_supported_plan_is_refused():
    """Plans above 256 pre-merge edges per half (depth hint > 124 with the default Params) are
    PVAC_ENOSYS; bad noise Params are PVAC_EINVAL."""
    from pvac_hfhe_cppbyv_amd import PvacError
    eng, _, _, _ = _eng()
    assert eng.enc_caps(124)[1] <= 2 * 256
    with pytest.raises(PvacError):
        eng.enc_caps(125)
    for bad in ((-1.0, 0.55, 16.0), (120.0, 1.5, 16.0), (120.0, 0.55, -2.0), (float("nan"), 0.55, 16.0)):
        with pytest.raises(PvacError):
            eng.set_noise(*bad)
