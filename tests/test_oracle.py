"""Pin the CPU oracle (oracle/pvac_oracle.cpp) against golden vectors minted by the UNMODIFIED
reference (oracle/ref_harness.cpp, tests/golden/ref) and the reference's own shipped data
(tests/golden/bounty). CPU-only."""
import numpy as np
import pytest

from helpers import (GOLD, REF, Cipher, read_ct, read_layers_u64, read_u64, write_ct, R_for, to_int, P)
import os


# ----------------------------------------------------------------------------- Fp (core/field.hpp)
@pytest.mark.parametrize("op", ["add", "sub", "mul"])
def test_fp_binop_golden(oracle, op):
    a_lo, a_hi, b_lo, b_hi = (read_u64(f"fp_{n}.u64") for n in ("a_lo", "a_hi", "b_lo", "b_hi"))
    lo, hi = oracle.fp(op, a_lo, a_hi, b_lo, b_hi)
    assert np.array_equal(lo, read_u64(f"fp_{op}_lo.u64"))
    assert np.array_equal(hi, read_u64(f"fp_{op}_hi.u64"))


def test_fp_neg_fromwords_inv_pow_golden(oracle):
    a_lo, a_hi = read_u64("fp_a_lo.u64"), read_u64("fp_a_hi.u64")
    lo, hi = oracle.fp("neg", a_lo, a_hi)
    assert np.array_equal(lo, read_u64("fp_neg_lo.u64")) and np.array_equal(hi, read_u64("fp_neg_hi.u64"))
    lo, hi = oracle.fp("from_words", a_lo, a_hi)
    assert np.array_equal(lo, read_u64("fp_fromw_lo.u64")) and np.array_equal(hi, read_u64("fp_fromw_hi.u64"))
    lo, hi = oracle.fp("inv", read_u64("fp_inv_in_lo.u64"), read_u64("fp_inv_in_hi.u64"))
    assert np.array_equal(lo, read_u64("fp_inv_lo.u64")) and np.array_equal(hi, read_u64("fp_inv_hi.u64"))
    lo, hi = oracle.fp("pow", read_u64("fp_pow_a_lo.u64"), read_u64("fp_pow_a_hi.u64"), read_u64("fp_pow_e.u64"))
    assert np.array_equal(lo, read_u64("fp_pow_r_lo.u64")) and np.array_equal(hi, read_u64("fp_pow_r_hi.u64"))


def test_fp_canonical_matches_bigint(oracle):
    """Canonical inputs: add/sub/mul equal exact integer arithmetic mod p (test_fp_core.cpp spirit)."""
    rng = np.random.default_rng(7)
    n = 2000
    a = [int(x) % P for x in rng.integers(0, 2**63, n, dtype=np.uint64).astype(object) * (2**64) +
         rng.integers(0, 2**63, n, dtype=np.uint64).astype(object)]
    b = [int(x) % P for x in rng.integers(0, 2**63, n, dtype=np.uint64).astype(object) * (2**64) +
         rng.integers(0, 2**63, n, dtype=np.uint64).astype(object)]
    alo = np.array([x & (2**64 - 1) for x in a], np.uint64)
    ahi = np.array([x >> 64 for x in a], np.uint64)
    blo = np.array([x & (2**64 - 1) for x in b], np.uint64)
    bhi = np.array([x >> 64 for x in b], np.uint64)
    for op, f in (("add", lambda x, y: (x + y) % P), ("sub", lambda x, y: (x - y) % P),
                  ("mul", lambda x, y: (x * y) % P)):
        lo, hi = oracle.fp(op, alo, ahi, blo, bhi)
        got = [to_int(l, h) for l, h in zip(lo, hi)]
        assert got == [f(x, y) for x, y in zip(a, b)], op


# ----------------------------------------------------------------------------- hashing / PRG
def test_sha256_abc_kat(oracle):
    """Known answer from the reference's own test (tests/test_prf.cpp:11-25)."""
    assert oracle.sha256(b"abc").hex() == "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"


def test_gen_H_digest_and_columns(oracle, manifest, H_dense):
    ref_cols = read_u64("H_cols0_63.u64").reshape(64, 128)
    assert np.array_equal(H_dense[:64], ref_cols)
    # every column has exactly h_col_wt = 192 bits
    pc = np.unpackbits(H_dense[:256].view(np.uint8), axis=1).sum(axis=1)
    assert (pc == 192).all()


def test_bucket_count_matches_survey(oracle):
    # bucket_count(1560) = 1613, bucket_count(48800) = 49201 (libstdc++ GCC 11)
    assert oracle.bucket_count(1560) == 1613
    assert oracle.bucket_count(48800) == 49201


# ----------------------------------------------------------------------------- ciphertext ops
def _pair(p):
    x = read_ct(os.path.join(REF, f"pair{p}_x.ct"))[0]
    y = read_ct(os.path.join(REF, f"pair{p}_y.ct"))[0]
    return x, y


def _same(a: Cipher, b: Cipher, layers=True, weights=True, sigma=False):
    if layers:
        for f in ("rule", "pa", "pb", "ztag", "nonce_lo", "nonce_hi"):
            assert np.array_equal(a.layers[f], b.layers[f]), f
    assert np.array_equal(a.meta, b.meta)
    if weights:
        assert np.array_equal(a.w_lo, b.w_lo) and np.array_equal(a.w_hi, b.w_hi)
    if sigma:
        assert np.array_equal(a.sigma, b.sigma)


def _ct_layers_view(c: Cipher):
    """.ct drops seeds of PROD layers and pa/pb of BASE layers; project accordingly."""
    L = c.layers.copy()
    prod = L["rule"] == 1
    L["ztag"][prod] = 0
    L["nonce_lo"][prod] = 0
    L["nonce_hi"][prod] = 0
    L["pa"][~prod] = 0
    L["pb"][~prod] = 0
    return Cipher(L, c.meta, c.w_lo, c.w_hi, c.sigma)


@pytest.mark.parametrize("p", range(8))
def test_ct_add_sub_golden(oracle, manifest, p):
    x, y = _pair(p)
    for op, neg in (("add", False), ("sub", True)):
        got = oracle.ct_add(x, y, negate=neg)
        ref = read_ct(os.path.join(REF, f"pair{p}_{op}.ct"))[0]
        _same(_ct_layers_view(got), ref, sigma=True)
        H_digest = bytes.fromhex(manifest["H_digest"])
        assert oracle.commit(got, manifest["canon_tag"], H_digest).hex() == manifest["pairs"][p][f"commit_{op}"]


def _fr_manifest():
    import json
    with open(os.path.join(REF, "fr_manifest.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("k", range(5))
def test_ct_mul_full_range_golden(oracle, k):
    """ct_mul on weights anywhere in [0, 2^128) (fp_mul takes any operand, core/field.hpp:113-213):
    full-range random words, the special values p, p-1, 2^127, 2^128-1, 0, 1, a cancelling key pair
    (w, p - w on one key) and a general-path shape; the oracle equals the reference's own output
    (oracle/ref_harness.cpp fullrange)."""
    fm = _fr_manifest()
    x = read_ct(os.path.join(REF, f"fr{k}_x.ct"))[0]
    y = read_ct(os.path.join(REF, f"fr{k}_y.ct"))[0]
    stream = read_u64(f"fr{k}_mul_stream.u64")
    nn = 2 * x.nL * y.nL
    got = oracle.ct_mul(x, y, stream[:nn], stream[nn:], canon_tag=fm["canon_tag"])
    ref = read_ct(os.path.join(REF, f"fr{k}_mul_w.ct"))[0]
    _same(_ct_layers_view(got), ref)
    full_layers = read_layers_u64(f"fr{k}_mul_layers.u64")
    for f in ("rule", "pa", "pb", "ztag", "nonce_lo", "nonce_hi"):
        assert np.array_equal(got.layers[f], full_layers[f]), f
    assert len(stream) == nn + got.nE
    if k <= 1:   # full-range inputs: lo top bits and hi >= 2^63 both occur
        assert (x.w_hi >= np.uint64(1 << 63)).any() and (x.w_lo >= np.uint64(1 << 63)).any()


@pytest.mark.parametrize("p", range(8))
def test_ct_mul_weights_golden(oracle, manifest, p):
    x, y = _pair(p)
    stream = read_u64(f"pair{p}_mul_stream.u64")
    nn = 2 * x.nL * y.nL
    got = oracle.ct_mul(x, y, stream[:nn], stream[nn:], canon_tag=manifest["canon_tag"])
    ref = read_ct(os.path.join(REF, f"pair{p}_mul_w.ct"))[0]
    _same(_ct_layers_view(got), ref)
    full_layers = read_layers_u64(f"pair{p}_mul_layers.u64")
    for f in ("rule", "ztag", "nonce_lo", "nonce_hi"):
        assert np.array_equal(got.layers[f], full_layers[f]), f
    assert len(stream) == nn + got.nE            # one salt per emitted edge (arithmetic.hpp:90-94)
    # decryption round trip with fixture R values (ops/decrypt.hpp)
    powg = read_u64("powg_B.u64")
    R = R_for(got, [(x, read_u64(f"pair{p}_x_R.u64")), (y, read_u64(f"pair{p}_y_R.u64"))])
    assert list(oracle.dec(got, powg, R)) == manifest["pairs"][p]["dec_mul"]
    m = manifest["pairs"][p]
    assert oracle.dec(got, powg, R)[0] == (m["x"] * m["y"]) % P


@pytest.mark.parametrize("p", [0, 3])
def test_ct_mul_sigma_golden(oracle, manifest, H_dense, p):
    x, y = _pair(p)
    stream = read_u64(f"pair{p}_mul_stream.u64")
    nn = 2 * x.nL * y.nL
    got = oracle.ct_mul(x, y, stream[:nn], stream[nn:], H=H_dense, canon_tag=manifest["canon_tag"])
    H_digest = bytes.fromhex(manifest["H_digest"])
    assert oracle.commit(got, manifest["canon_tag"], H_digest).hex() == manifest["pairs"][p]["commit_mul"]
    if p == 0:
        ref = read_ct(os.path.join(REF, "pair0_mul.ct"))[0]
        _same(_ct_layers_view(got), ref, sigma=True)


def _chain_inputs():
    c0 = read_ct(os.path.join(REF, "chain0.ct"))[0]
    return c0


@pytest.mark.parametrize("kind,steps", [("chain", 3), ("sq", 2)])
def test_chain_and_square_golden(oracle, manifest, kind, steps):
    c = read_ct(os.path.join(REF, f"{kind}0.ct"))[0]
    Rin = [(c, read_u64(f"{kind}0_R.u64"))]
    cur = c
    for k in range(1, steps + 1):
        if kind == "chain":
            x = read_ct(os.path.join(REF, f"chain{k}_x.ct"))[0]
            Rin.append((x, read_u64(f"chain{k}_x_R.u64")))
        else:
            x = cur
        stream = read_u64(f"{kind}{k}_stream.u64")
        nn = 2 * cur.nL * x.nL
        got = oracle.ct_mul(cur, x, stream[:nn], stream[nn:], canon_tag=manifest["canon_tag"])
        ref = read_ct(os.path.join(REF, f"{kind}{k}.ct"))[0]
        _same(_ct_layers_view(got), ref)
        full = read_layers_u64(f"{kind}{k}_layers.u64")
        assert np.array_equal(got.layers["ztag"], full["ztag"])
        rec = manifest["chain" if kind == "chain" else "square"][k - 1]
        assert got.nE == rec["edges"] and got.nL == rec["layers"]
        R = R_for(got, Rin)
        assert list(oracle.dec(got, read_u64("powg_B.u64"), R)) == rec["dec"]
        # the next step multiplies the full (layer-seeded) product
        cur = Cipher(full, got.meta, got.w_lo, got.w_hi)


def test_guard_compact_edges_golden(oracle, manifest):
    """guard_budget -> compact_edges (encrypt.hpp:39-71,106-111) with duplicates + non-canonical w."""
    x = read_ct(os.path.join(REF, "guard_x.ct"))[0]
    y = read_ct(os.path.join(REF, "guard_y.ct"))[0]
    got = oracle.ct_add(x, y, edge_budget=16)
    ref = read_ct(os.path.join(REF, "guard_add.ct"))[0]
    _same(_ct_layers_view(got), ref, sigma=True)
    H_digest = bytes.fromhex(manifest["H_digest"])
    assert oracle.commit(got, manifest["canon_tag"], H_digest).hex() == manifest["guard"]["commit"]


def test_bounty2_sum_is_ct_add_bytewise(oracle):
    """The reference ships sum.ct = combine_ciphers(a.ct, b.ct) (tests/add.cpp:220-228)."""
    a = read_ct(os.path.join(GOLD, "bounty", "a.ct"))[0]
    b = read_ct(os.path.join(GOLD, "bounty", "b.ct"))[0]
    s = oracle.ct_add(a, b)
    with open(os.path.join(GOLD, "bounty", "sum.ct"), "rb") as f:
        assert write_ct([_ct_layers_view(s)]) == f.read()


def test_ct_reader_roundtrip_seed3():
    path = os.path.join(GOLD, "bounty", "seed3.ct")
    cts = read_ct(path)
    assert len(cts) == 9
    with open(path, "rb") as f:
        assert write_ct(cts) == f.read()


def _pack(cs):
    lc = np.array([c.nL for c in cs], np.uint64)
    ec = np.array([c.nE for c in cs], np.uint64)
    lo = np.concatenate([[0], np.cumsum(lc)]).astype(np.uint64)
    eo = np.concatenate([[0], np.cumsum(ec)]).astype(np.uint64)
    cat = lambda f: np.ascontiguousarray(np.concatenate([getattr(c, f) for c in cs]).astype(np.uint64))
    return lo, np.ascontiguousarray(np.concatenate([c.layers for c in cs])), eo, cat("meta"), cat("w_lo"), cat("w_hi")


def _fnv(c):
    h = 0xcbf29ce484222325
    for m, lo, hi in zip(c.meta, c.w_lo, c.w_hi):
        for x in (int(m), int(lo), int(hi)):
            for i in range(8):
                h = ((h ^ ((x >> (8 * i)) & 0xFF)) * 0x100000001b3) & (2**64 - 1)
    return h


def test_chain_timed_equals_stepwise_ct_mul(oracle):
    """The cfg-4 CPU baseline (orc_ct_mul_chain_timed, bench.py extras.cfg4_chain.cpu_baseline) is
    the same chain as ct_mul step by step on the reference's own enc_value outputs, on 1 and 3
    threads: final edge digests and per-step edge totals."""
    import ctypes as C
    from helpers import default_params
    xs = [read_ct(os.path.join(REF, f"enc{i}.ct"))[0] for i in range(3)]
    depth = 3
    ref_d, ref_steps = [], np.zeros(depth, np.uint64)
    for x in xs:
        c = x
        for d in range(depth):
            c = oracle.ct_mul(c, x, np.zeros(2 * c.nL * x.nL, np.uint64), canon_tag=0x5EED0003)
            ref_steps[d] += c.nE
        ref_d.append(_fnv(c))
    P_ = lambda a: a.ctypes.data_as(C.c_void_p)
    packed = _pack(xs)
    prm = default_params(0x5EED0003)
    for th in (1, 3):
        cnt, dig, se = np.zeros(3, np.uint64), np.zeros(3, np.uint64), np.zeros(depth, np.uint64)
        oracle.lib.orc_ct_mul_chain_timed(C.byref(prm), 3, *(P_(a) for a in packed), depth, th, P_(cnt), P_(dig), P_(se))
        assert [int(v) for v in dig] == ref_d
        assert np.array_equal(se, ref_steps)


def test_add_batch_timed_equals_ct_add(oracle):
    """bench.py's ct_add / ct_sub CPU baseline (orc_ct_add_batch_timed) reproduces the reference's
    own ct_add / ct_sub outputs of the eight fixture pairs (edge digests and counts)."""
    import ctypes as C
    from helpers import default_params
    xs = [read_ct(os.path.join(REF, f"pair{p}_x.ct"))[0] for p in range(8)]
    ys = [read_ct(os.path.join(REF, f"pair{p}_y.ct"))[0] for p in range(8)]
    P_ = lambda a: a.ctypes.data_as(C.c_void_p)
    a, b = _pack(xs), _pack(ys)
    prm = default_params(0)
    for neg, name in ((0, "add"), (1, "sub")):
        refs = [read_ct(os.path.join(REF, f"pair{p}_{name}.ct"))[0] for p in range(8)]
        cnt, dig = np.zeros(8, np.uint64), np.zeros(8, np.uint64)
        oracle.lib.orc_ct_add_batch_timed(C.byref(prm), 8, *(P_(x) for x in a), *(P_(x) for x in b), neg, 2,
                                          P_(cnt), P_(dig))
        assert [int(v) for v in cnt] == [r.nE for r in refs]
        assert [int(v) for v in dig] == [_fnv(r) for r in refs]


def test_chainx_fixture_replay(oracle, manifest, H_dense):
    """The chain entry point's fixture (ref_harness chainx): x = enc_value(2), c_k = ct_mul(c_{k-1}, x),
    k = 1..4, one getrandom stream. The oracle replays it step by step (each step's nonces, then its
    salts: skipped for steps 1..3, used for step 4's sigmas), reproducing every step's edge / layer /
    stream counts, c_4's weights-only .ct bytes, its full layer table, every sigma digest, and its
    decryption (x^5 = 32)."""
    import hashlib
    import json
    with open(os.path.join(REF, "chainx_manifest.json")) as f:
        man = json.load(f)
    x = read_ct(os.path.join(REF, "chainx_x.ct"))[0]
    xw = Cipher(x.layers, x.meta, x.w_lo, x.w_hi)
    stream = read_u64("chainx_stream.u64")
    pos, c = 0, xw
    depth = man["depth"]
    for k in range(depth):
        nn = 2 * c.nL * x.nL
        nz = stream[pos:pos + nn]
        w = oracle.ct_mul(c, xw, nz, canon_tag=man["canon_tag"])   # weights: the salt count
        rec = man["steps"][k]
        assert w.nE == rec["edges"] and w.nL == rec["layers"] and nn + w.nE == rec["stream"]
        if k + 1 == depth:
            c = oracle.ct_mul(c, xw, nz, salts=stream[pos + nn:pos + nn + w.nE], H=H_dense, canon_tag=man["canon_tag"])
        else:
            c = w
        pos += nn + w.nE
    assert pos == len(stream) == man["stream"]
    with open(os.path.join(REF, "chainx_final.ct"), "rb") as f:
        assert write_ct([Cipher(c.layers, c.meta, c.w_lo, c.w_hi)]) == f.read()
    full = read_layers_u64("chainx_final_layers.u64")
    for fld in ("rule", "ztag", "nonce_lo", "nonce_hi"):
        assert np.array_equal(c.layers[fld], full[fld])
    dig = read_u64("chainx_final_sigdig.u64")
    got = np.array([int.from_bytes(hashlib.sha256(s.astype("<u8").tobytes()).digest()[:8], "little")
                    for s in c.sigma], np.uint64)
    assert np.array_equal(got, dig)
    R = R_for(c, [(x, read_u64("chainx_x_R.u64"))])
    assert list(oracle.dec(c, read_u64("powg_B.u64"), R)) == man["dec"] == [32, 0]


def _chainf(name):
    import json
    with open(os.path.join(REF, f"{name}_manifest.json")) as f:
        return json.load(f)


def _weights(c):
    return Cipher(c.layers, c.meta, c.w_lo, c.w_hi)


def _chainf_replay(oracle, man, H, sk, powg, sigma_steps):
    """The port replaying ref_harness chainf / chainf8 (the reference's own loop, tests/test_main.cpp:
    289-293: x = enc_value(2), c_k = ct_mul(c_{k-1}, enc_value(2))): every operand encrypted from its
    stretch of the regenerated getrandom stream, every step's nonces from the head of its mul stretch.
    Checks |E|, |L| and the sigma-less commit_ct of every step, and the commit with sigmas (salts from
    the rest of the stretch) for the steps in sigma_steps. Returns (x, operands, c_depth weights-only,
    c_depth with sigmas or None)."""
    from helpers import splitmix_stream
    S, tag = man["seed"], man["canon_tag"]
    Hd = bytes.fromhex(_man_H_digest())
    j0, n = man["x_stream"]
    x, used = oracle.enc_value(sk, 2, splitmix_stream(S, j0, n), powg, canon_tag=tag)
    assert used == n
    c, ys, full = _weights(x), [], None
    for k, rec in enumerate(man["steps"], start=1):
        e0, en = rec["enc_stream"]
        y, used = oracle.enc_value(sk, 2, splitmix_stream(S, e0, en), powg, canon_tag=tag)
        assert used == en
        y = _weights(y)
        ys.append(y)
        m0, mn = rec["mul_stream"]
        nn = rec["nonce_words"]
        assert nn == 2 * c.nL * y.nL
        words = splitmix_stream(S, m0, mn)
        if k in sigma_steps:
            full = oracle.ct_mul(c, y, words[:nn], salts=words[nn:], H=H, canon_tag=tag)
            assert oracle.commit(full, tag, Hd).hex() == rec["commit"], k
        c = oracle.ct_mul(c, y, words[:nn], canon_tag=tag)
        assert c.nE == rec["edges"] and c.nL == rec["layers"] and nn + c.nE == mn, k
        assert oracle.commit(c, tag, Hd).hex() == rec["commit_weights"], k
    return x, ys, c, full


def _man_H_digest():
    import json
    with open(os.path.join(REF, "manifest.json")) as f:
        return json.load(f)["H_digest"]


def test_chainf_fixture_replay(oracle, H_dense):
    """ref_harness chainf: the reference's own chain loop with a FRESH enc_value(2) operand per step
    (tests/test_main.cpp:291-292), depth 4, one interleaved getrandom stream (enc, mul, enc, ...).
    The stream regenerated from its seed equals the committed stream; the port's enc_value reproduces
    x and every operand from their stretches; every step's commit_ct with and without sigmas; c_4's
    weights-only .ct bytes, layer table, sigma digests and decryption (2^5 = 32)."""
    import hashlib
    from helpers import R_for, fixture_secret, splitmix_stream
    man = _chainf("chainf")
    sk, _, _ = fixture_secret()
    powg = read_u64("powg_B.u64")
    stream = read_u64("chainf_stream.u64")
    assert len(stream) == man["stream"] and np.array_equal(splitmix_stream(man["seed"], 0, len(stream)), stream)
    x, ys, c, full = _chainf_replay(oracle, man, H_dense, sk, powg, sigma_steps=range(1, 5))
    for name, got in [("x", x)] + [(f"y{k}", y) for k, y in enumerate(ys, start=1)]:
        with open(os.path.join(REF, f"chainf_{name}.ct"), "rb") as f:
            assert write_ct([got]) == f.read(), name
    with open(os.path.join(REF, "chainf_final.ct"), "rb") as f:
        assert write_ct([c]) == f.read()
    lay = read_layers_u64("chainf_final_layers.u64")
    for fld in ("rule", "ztag", "nonce_lo", "nonce_hi"):
        assert np.array_equal(full.layers[fld], lay[fld])
    dig = np.array([int.from_bytes(hashlib.sha256(s.astype("<u8").tobytes()).digest()[:8], "little")
                    for s in full.sigma], np.uint64)
    assert np.array_equal(dig, read_u64("chainf_final_sigdig.u64"))
    R = _base_R(oracle, sk, man["canon_tag"], c)
    assert list(oracle.dec(c, powg, R)) == man["dec"] == [32, 0]


def _base_R(oracle, sk, tag, c):
    """prf_R of every BASE layer of c (2 words per layer slot, 0 for PROD layers)."""
    R = np.zeros(2 * c.nL, np.uint64)
    for i, L in enumerate(c.layers):
        if L["rule"] == 0:
            R[2 * i:2 * i + 2] = oracle.prf_R(sk, tag, (L["ztag"], L["nonce_lo"], L["nonce_hi"]))
    return R


def test_chainf8_fixture_digests(oracle, H_dense):
    """ref_harness chainf8: the same loop to depth 8 (steps 5-8: dense layers, the direct-mode regime,
    c_8 with 345,088 edges), pinned by the reference's per-step commit_ct digests. The port reproduces
    every step's sigma-less commit (weights, layers incl. nonces / ztags, emit order) and the commit
    with sigmas of steps 1-5, and c_8 decrypts to 2^9."""
    from helpers import fixture_secret
    man = _chainf("chainf8")
    sk, _, _ = fixture_secret()
    powg = read_u64("powg_B.u64")
    assert man["depth"] == 8
    _, _, c, _ = _chainf_replay(oracle, man, H_dense, sk, powg, sigma_steps=range(1, 6))
    assert c.nE == 345088
    R = _base_R(oracle, sk, man["canon_tag"], c)
    assert list(oracle.dec(c, powg, R)) == man["dec"] == [512, 0]
