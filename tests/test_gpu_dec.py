"""GPU dec_value (k_dec.hip; reference ops/decrypt.hpp:12-89) with fixture BASE-layer R values:
fp_inv golden vectors, fresh ciphers decrypt to the plaintexts the reference encrypted, GPU
ct_add / ct_sub / ct_mul outputs decrypt to x + y, x - y, x * y, the reference's chain and square
steps decrypt to the values the reference recorded, random layer DAGs match the oracle, and bad
layer graphs / edge references are reported per cipher."""
import os

import numpy as np
import pytest

from helpers import P, REF, Cipher, LAYER_DT, R_for, read_ct, read_layers_u64, read_u64

pytestmark = pytest.mark.gpu


def _dev_batch(engine, ciphers):
    from pvac_hfhe_cppbyv_amd import DeviceBatch, HostCipher
    hc = [HostCipher(c.layers, c.meta, c.w_lo, c.w_hi, None) for c in ciphers]
    return DeviceBatch.from_host(hc, engine.device)


def _eng(manifest):
    from pvac_hfhe_cppbyv_amd import Engine
    eng = Engine(device=0, canon_tag=manifest["canon_tag"])
    eng.set_powg(read_u64("powg_B.u64"))
    return eng


def test_fp_inv_golden(engine):
    from pvac_hfhe_cppbyv_amd import FP_INV
    import torch
    t = lambda a: torch.from_numpy(a.view(np.int64)).to(engine.device)
    lo, hi = engine.fp_binop(FP_INV, t(read_u64("fp_inv_in_lo.u64")), t(read_u64("fp_inv_in_hi.u64")))
    assert np.array_equal(lo.cpu().numpy().view(np.uint64), read_u64("fp_inv_lo.u64"))
    assert np.array_equal(hi.cpu().numpy().view(np.uint64), read_u64("fp_inv_hi.u64"))


def test_dec_fresh_and_op_outputs(manifest):
    eng = _eng(manifest)
    xs = [read_ct(os.path.join(REF, f"pair{p}_x.ct"))[0] for p in range(8)]
    ys = [read_ct(os.path.join(REF, f"pair{p}_y.ct"))[0] for p in range(8)]
    Rx = [read_u64(f"pair{p}_x_R.u64") for p in range(8)]
    Ry = [read_u64(f"pair{p}_y_R.u64") for p in range(8)]
    # fresh ciphers: one batch of 16
    vals, st = eng.dec_value(_dev_batch(eng, xs + ys), np.concatenate(Rx + Ry))
    assert not st.any()
    assert vals == [manifest["pairs"][p]["x"] for p in range(8)] + [manifest["pairs"][p]["y"] for p in range(8)]
    A, B = _dev_batch(eng, xs), _dev_batch(eng, ys)
    outs = {"add": eng.ct_add(A, B).to_host(), "sub": eng.ct_add(A, B, negate=True).to_host(),
            "mul": [eng.ct_mul(_dev_batch(eng, [x]), _dev_batch(eng, [y]), nonce_seed=p).to_host()[0]
                    for p, (x, y) in enumerate(zip(xs, ys))]}
    for op, fn in (("add", lambda a, b: a + b), ("sub", lambda a, b: a - b), ("mul", lambda a, b: a * b)):
        cs = [Cipher(o.layers, o.meta, o.w_lo, o.w_hi) for o in outs[op]]
        R = np.concatenate([R_for(c, [(x, rx), (y, ry)]) for c, x, y, rx, ry in zip(cs, xs, ys, Rx, Ry)])
        vals, st = eng.dec_value(_dev_batch(eng, cs), R)
        assert not st.any()
        exp = [fn(manifest["pairs"][p]["x"], manifest["pairs"][p]["y"]) % P for p in range(8)]
        assert vals == exp, op


@pytest.mark.parametrize("kind,steps", [("chain", 3), ("sq", 2)])
def test_dec_reference_chains(manifest, kind, steps):
    """The reference's own ct_mul chain / square outputs (fixtures) decrypt to its recorded values."""
    eng = _eng(manifest)
    c0 = read_ct(os.path.join(REF, f"{kind}0.ct"))[0]
    Rin = [(c0, read_u64(f"{kind}0_R.u64"))]
    cs, Rs, exp = [], [], []
    for k in range(1, steps + 1):
        if kind == "chain":
            x = read_ct(os.path.join(REF, f"chain{k}_x.ct"))[0]
            Rin.append((x, read_u64(f"chain{k}_x_R.u64")))
        full = read_layers_u64(f"{kind}{k}_layers.u64")
        c = read_ct(os.path.join(REF, f"{kind}{k}.ct"))[0]
        c = Cipher(full, c.meta, c.w_lo, c.w_hi)
        cs.append(c)
        Rs.append(R_for(c, Rin))
        rec = manifest["chain" if kind == "chain" else "square"][k - 1]
        exp.append(rec["dec"][0] | (rec["dec"][1] << 64))
    vals, st = eng.dec_value(_dev_batch(eng, cs), np.concatenate(Rs))
    assert not st.any()
    assert vals == exp


def _rand_cipher(rng, nl, ne, B=337):
    L = np.zeros(nl, LAYER_DT)
    for l in range(nl):
        if l < 2 or rng.random() < 0.3:
            L["rule"][l] = 0
        else:   # PROD over any earlier layers (and some later ones: the sweeps handle any DAG)
            L["rule"][l] = 1
            L["pa"][l], L["pb"][l] = rng.integers(0, l), rng.integers(0, l)
    lay = rng.integers(0, max(nl, 1), ne).astype(np.uint64)
    meta = lay | (rng.integers(0, B, ne).astype(np.uint64) << np.uint64(32)) | \
        (rng.integers(0, 3, ne).astype(np.uint64) << np.uint64(48))
    lo = rng.integers(0, 2**64, ne, dtype=np.uint64)
    hi = rng.integers(0, 2**64, ne, dtype=np.uint64)   # non-canonical weights too: fp_mul is exact
    return Cipher(L, meta, lo, hi)


def test_dec_random_dags_vs_oracle(manifest, oracle):
    eng = _eng(manifest)
    rng = np.random.default_rng(17)
    cs, Rs = [], []
    for k in range(24):
        c = _rand_cipher(rng, int(rng.integers(1, 40)), int(rng.integers(0, 300)))
        # reverse some layer orders: children before parents (not produced by ct ops, legal DAG)
        if k % 3 == 0 and c.nL > 3:
            perm = np.arange(c.nL)[::-1]
            inv = np.argsort(perm)
            L = c.layers[perm].copy()
            prod = L["rule"] == 1
            L["pa"][prod] = inv[L["pa"][prod]]
            L["pb"][prod] = inv[L["pb"][prod]]
            lid = (c.meta & np.uint64(0xFFFFFFFF)).astype(np.int64)
            meta = (c.meta & ~np.uint64(0xFFFFFFFF)) | inv[lid].astype(np.uint64)
            c = Cipher(L, meta, c.w_lo, c.w_hi)
        R = rng.integers(0, 2**63, 2 * c.nL, dtype=np.uint64)
        R[(k % 5 == 1) * 2: (k % 5 == 1) * 4] = 0   # a zero R (inv(0) = 0) in some ciphers
        cs.append(c)
        Rs.append(R)
    vals, st = eng.dec_value(_dev_batch(eng, cs), np.concatenate(Rs))
    assert not st.any()
    powg = read_u64("powg_B.u64")
    for c, R, v in zip(cs, Rs, vals):
        lo, hi = oracle.dec(c, powg, R)
        assert v == lo | (hi << 64)


def test_dec_status(manifest):
    eng = _eng(manifest)
    rng = np.random.default_rng(5)
    good = _rand_cipher(rng, 6, 50)
    cyc = _rand_cipher(rng, 6, 50)
    cyc.layers["rule"][3], cyc.layers["pa"][3], cyc.layers["pb"][3] = 1, 4, 0
    cyc.layers["rule"][4], cyc.layers["pa"][4], cyc.layers["pb"][4] = 1, 3, 0   # 3 <-> 4
    oor = _rand_cipher(rng, 6, 50)
    oor.layers["rule"][5], oor.layers["pa"][5], oor.layers["pb"][5] = 1, 9, 0    # parent out of range
    bad_idx = _rand_cipher(rng, 6, 50)
    bad_idx.meta[7] = (bad_idx.meta[7] & np.uint64(0xFFFFFFFF)) | (np.uint64(400) << np.uint64(32))   # idx >= B
    bad_lid = _rand_cipher(rng, 6, 50)
    bad_lid.meta[3] = (bad_lid.meta[3] & ~np.uint64(0xFFFFFFFF)) | np.uint64(6)                      # layer >= |L|
    cs = [good, cyc, oor, bad_idx, bad_lid]
    R = np.concatenate([rng.integers(1, 2**63, 2 * c.nL, dtype=np.uint64) for c in cs])
    _, st = eng.dec_value(_dev_batch(eng, cs), R)
    assert list(st) == [0, 1, 1, 2, 2]
