"""GPU parity: the MI355X engine (libpvac_hip.so, via its C ABI) against the reference's golden
vectors and the pinned CPU oracle. Bit-exact everywhere (integer/byte work)."""
import os

import numpy as np
import pytest

from helpers import (REF, Cipher, read_ct, read_layers_u64, read_u64, R_for, P)

pytestmark = pytest.mark.gpu


def _dev_batch(engine, ciphers, sigma=False):
    from pvac_hfhe_cppbyv_amd import DeviceBatch, HostCipher
    hc = [HostCipher(c.layers, c.meta, c.w_lo, c.w_hi, c.sigma) for c in ciphers]
    return DeviceBatch.from_host(hc, engine.device, sigma=sigma)


def _i64(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64))


# ------------------------------------------------------------------ element-wise Fp (cfg 2)
@pytest.mark.parametrize("op", ["add", "sub", "mul", "neg"])
def test_fp_binop_golden(engine, op):
    from pvac_hfhe_cppbyv_amd import FP_ADD, FP_SUB, FP_MUL, FP_NEG
    code = {"add": FP_ADD, "sub": FP_SUB, "mul": FP_MUL, "neg": FP_NEG}[op]
    d = engine.device
    a_lo, a_hi, b_lo, b_hi = (_i64(read_u64(f"fp_{n}.u64")).to(d) for n in ("a_lo", "a_hi", "b_lo", "b_hi"))
    lo, hi = engine.fp_binop(code, a_lo, a_hi, b_lo, b_hi)
    assert np.array_equal(lo.cpu().numpy().view(np.uint64), read_u64(f"fp_{op}_lo.u64"))
    assert np.array_equal(hi.cpu().numpy().view(np.uint64), read_u64(f"fp_{op}_hi.u64"))


@pytest.mark.parametrize("n", [1, 2, 3, 4095, 65537])
def test_fp_binop_ragged_and_unaligned(engine, oracle, n):
    """Odd sizes take the scalar tail; 8-byte-misaligned views take the scalar kernel."""
    from pvac_hfhe_cppbyv_amd import FP_MUL, FP_ADD, FP_SUB
    rng = np.random.default_rng(n + 1)
    buf = [rng.integers(0, 2**63, n + 1, dtype=np.uint64) * np.uint64(2) + np.uint64(1) for _ in range(4)]
    t = [_i64(b).to(engine.device) for b in buf]
    for off in (0, 1):
        views = [x[off:off + n] for x in t]
        for code, name in ((FP_MUL, "mul"), (FP_ADD, "add"), (FP_SUB, "sub")):
            lo, hi = engine.fp_binop(code, *views)
            ref_lo, ref_hi = oracle.fp(name, *(b[off:off + n] for b in buf))
            assert np.array_equal(lo.cpu().numpy().view(np.uint64), ref_lo)
            assert np.array_equal(hi.cpu().numpy().view(np.uint64), ref_hi)


def test_fp_scale_broadcast(engine, oracle):
    from pvac_hfhe_cppbyv_amd import FP_SCALE
    rng = np.random.default_rng(3)
    n = 10001
    a_lo = rng.integers(0, 2**63, n, dtype=np.uint64) * np.uint64(2)
    a_hi = rng.integers(0, 2**63, n, dtype=np.uint64)
    s_lo, s_hi = np.array([12345678901234567], np.uint64), np.array([987654321], np.uint64)
    d = engine.device
    lo, hi = engine.fp_binop(FP_SCALE, _i64(a_lo).to(d), _i64(a_hi).to(d), _i64(s_lo).to(d), _i64(s_hi).to(d))
    r_lo, r_hi = oracle.fp("mul", a_lo, a_hi, np.repeat(s_lo, n), np.repeat(s_hi, n))
    assert np.array_equal(lo.cpu().numpy().view(np.uint64), r_lo)
    assert np.array_equal(hi.cpu().numpy().view(np.uint64), r_hi)


def test_fp_full_size_properties(engine, oracle):
    """cfg 2 size (2^24): sample vs oracle + size-independent identities on every element:
    (a + b) - b == a and a * 1 == a for canonical inputs."""
    import torch
    from pvac_hfhe_cppbyv_amd import FP_ADD, FP_SUB, FP_MUL
    n = 1 << 24
    d = engine.device
    a_lo = torch.empty(n, dtype=torch.int64, device=d)
    a_hi = torch.empty(n, dtype=torch.int64, device=d)
    b_lo = torch.empty(n, dtype=torch.int64, device=d)
    b_hi = torch.empty(n, dtype=torch.int64, device=d)
    for t, s in ((a_lo, 1), (a_hi, 2), (b_lo, 3), (b_hi, 4)):
        engine.fill_random(t, 0x5EED0002 + s)
    a_hi &= (1 << 62) - 1   # canonical (< 2^126)
    b_hi &= (1 << 62) - 1
    s_lo, s_hi = engine.fp_binop(FP_ADD, a_lo, a_hi, b_lo, b_hi)
    r_lo, r_hi = engine.fp_binop(FP_SUB, s_lo, s_hi, b_lo, b_hi)
    assert torch.equal(r_lo, a_lo) and torch.equal(r_hi, a_hi)
    one_lo = torch.ones(n, dtype=torch.int64, device=d)
    one_hi = torch.zeros(n, dtype=torch.int64, device=d)
    m_lo, m_hi = engine.fp_binop(FP_MUL, a_lo, a_hi, one_lo, one_hi)
    assert torch.equal(m_lo, a_lo) and torch.equal(m_hi, a_hi)
    p_lo, p_hi = engine.fp_binop(FP_MUL, a_lo, a_hi, b_lo, b_hi)
    idx = torch.randint(0, n, (20000,), device=d)
    u = lambda t: t[idx].cpu().numpy().view(np.uint64)
    o_lo, o_hi = oracle.fp("mul", u(a_lo), u(a_hi), u(b_lo), u(b_hi))
    assert np.array_equal(u(p_lo), o_lo) and np.array_equal(u(p_hi), o_hi)


# ------------------------------------------------------------------ ct_add / ct_sub
def _ct_layers_view(c):
    L = c.layers.copy()
    prod = L["rule"] == 1
    for f in ("ztag", "nonce_lo", "nonce_hi"):
        L[f][prod] = 0
    L["pa"][~prod] = 0
    L["pb"][~prod] = 0
    return L


def _assert_same(got, ref, sigma=False, layers_view=True):
    L = _ct_layers_view(got) if layers_view else got.layers
    for f in ("rule", "pa", "pb", "ztag", "nonce_lo", "nonce_hi"):
        assert np.array_equal(L[f], ref.layers[f]), f
    assert np.array_equal(got.meta, ref.meta)
    assert np.array_equal(got.w_lo, ref.w_lo) and np.array_equal(got.w_hi, ref.w_hi)
    if sigma:
        assert np.array_equal(got.sigma, ref.sigma)


def test_ct_add_sub_golden_batched(engine):
    xs = [read_ct(os.path.join(REF, f"pair{p}_x.ct"))[0] for p in range(8)]
    ys = [read_ct(os.path.join(REF, f"pair{p}_y.ct"))[0] for p in range(8)]
    A, B = _dev_batch(engine, xs, sigma=True), _dev_batch(engine, ys, sigma=True)
    for op, neg in (("add", False), ("sub", True)):
        out = engine.ct_add(A, B, negate=neg, sigma=True).to_host()
        for p in range(8):
            _assert_same(out[p], read_ct(os.path.join(REF, f"pair{p}_{op}.ct"))[0], sigma=True)


def test_bounty2_sum_gpu(engine):
    from helpers import GOLD, write_ct
    a = read_ct(os.path.join(GOLD, "bounty", "a.ct"))[0]
    b = read_ct(os.path.join(GOLD, "bounty", "b.ct"))[0]
    s = engine.ct_add(_dev_batch(engine, [a], True), _dev_batch(engine, [b], True), sigma=True).to_host()[0]
    c = Cipher(_ct_layers_view(s), s.meta, s.w_lo, s.w_hi, s.sigma)
    with open(os.path.join(GOLD, "bounty", "sum.ct"), "rb") as f:
        assert write_ct([c]) == f.read()


# ------------------------------------------------------------------ ct_mul (fresh pairs)
def _nonce_buffer(engine, Cb, x_list, y_list, streams):
    """Place each pair's reference nonce stream at its product-layer slots."""
    loff = Cb.l_off.cpu().numpy().view(np.uint64)
    total = int(loff[-1]) + x_list[-1].nL + y_list[-1].nL + x_list[-1].nL * y_list[-1].nL
    buf = np.zeros(2 * total, np.uint64)
    for p, (x, y, st) in enumerate(zip(x_list, y_list, streams)):
        base = int(loff[p]) + x.nL + y.nL
        nn = 2 * x.nL * y.nL
        buf[2 * base:2 * base + nn] = st[:nn]
    return _i64(buf).to(engine.device)


def test_ct_mul_weights_golden_batched(engine, manifest):
    from pvac_hfhe_cppbyv_amd import Engine
    eng = Engine(device=0, canon_tag=manifest["canon_tag"])
    xs = [read_ct(os.path.join(REF, f"pair{p}_x.ct"))[0] for p in range(8)]
    ys = [read_ct(os.path.join(REF, f"pair{p}_y.ct"))[0] for p in range(8)]
    streams = [read_u64(f"pair{p}_mul_stream.u64") for p in range(8)]
    A, B = _dev_batch(eng, xs), _dev_batch(eng, ys)
    Cb, plan = eng.ct_mul_plan(A, B)
    assert plan.n_small == 8 and plan.n_large == 0
    nonces = _nonce_buffer(eng, Cb, xs, ys, streams)
    out = eng.ct_mul(A, B, nonces=nonces, C_=Cb, plan=plan).to_host()
    powg = read_u64("powg_B.u64")
    for p in range(8):
        ref = read_ct(os.path.join(REF, f"pair{p}_mul_w.ct"))[0]
        _assert_same(out[p], ref)
        full = read_layers_u64(f"pair{p}_mul_layers.u64")
        for f in ("rule", "ztag", "nonce_lo", "nonce_hi"):
            assert np.array_equal(out[p].layers[f], full[f]), f
        assert len(streams[p]) == 2 * xs[p].nL * ys[p].nL + out[p].nE


def test_ct_mul_sigma_golden(engine, manifest, oracle):
    """WITH_SIGMA: device gen_H must reproduce H_digest, and every product sigma must match the
    reference (pair 0 byte-for-byte, pairs 0..7 through commit_ct)."""
    from pvac_hfhe_cppbyv_amd import Engine, MUL_WITH_SIGMA
    eng = Engine(device=0, canon_tag=manifest["canon_tag"])
    assert eng.gen_H().hex() == manifest["H_digest"]
    xs = [read_ct(os.path.join(REF, f"pair{p}_x.ct"))[0] for p in range(8)]
    ys = [read_ct(os.path.join(REF, f"pair{p}_y.ct"))[0] for p in range(8)]
    streams = [read_u64(f"pair{p}_mul_stream.u64") for p in range(8)]
    A, B = _dev_batch(eng, xs), _dev_batch(eng, ys)
    Cb, plan = eng.ct_mul_plan(A, B)
    nonces = _nonce_buffer(eng, Cb, xs, ys, streams)
    eoff = Cb.e_off.cpu().numpy().view(np.uint64)
    salts = np.zeros(plan.total_edge_slots, np.uint64)
    for p in range(8):
        nn = 2 * xs[p].nL * ys[p].nL
        s = streams[p][nn:]
        salts[int(eoff[p]):int(eoff[p]) + len(s)] = s
    Cr = eng.ct_mul(A, B, nonces=nonces, salts=_i64(salts).to(eng.device), flags=MUL_WITH_SIGMA, C_=Cb,
                    plan=plan)
    out = Cr.to_host()
    ref0 = read_ct(os.path.join(REF, "pair0_mul.ct"))[0]
    _assert_same(out[0], ref0, sigma=True)
    # pvac_hip_batch_pack (what the C++ adapter copies to the host): dense offsets, the same rows
    P = eng.pack(Cr)
    lc = P.l_cnt.cpu().numpy().astype(np.uint64)
    ec = P.e_cnt.cpu().numpy().astype(np.uint64)
    assert np.array_equal(P.l_off.cpu().numpy().astype(np.uint64), np.cumsum(lc) - lc)
    assert np.array_equal(P.e_off.cpu().numpy().astype(np.uint64), np.cumsum(ec) - ec)
    assert P.layers.shape[0] == int(lc.sum()) and P.meta.shape[0] == int(ec.sum()) == P.sigma.shape[0]
    assert int(ec.sum()) < plan.total_edge_slots
    for p, c in enumerate(P.to_host()):
        _assert_same(c, out[p], sigma=True, layers_view=False)
    Hd = bytes.fromhex(manifest["H_digest"])
    for p in range(8):
        c = out[p]
        got = Cipher(c.layers, c.meta, c.w_lo, c.w_hi, c.sigma)
        assert oracle.commit(got, manifest["canon_tag"], Hd).hex() == manifest["pairs"][p]["commit_mul"], p


def test_ct_mul_synthetic_vs_oracle(engine, oracle):
    """4096 synthetic fresh-shaped pairs (cfg-3 generator, also 19/21-edge layers): every pair
    bit-exact vs the oracle, including emit order."""
    from pvac_hfhe_cppbyv_amd import Engine
    eng = Engine(device=0, canon_tag=0x1234)
    for epl in (20, 19, 21, 1):
        n = 4096 if epl == 20 else 256
        A = eng.gen_fresh(n, 0xA000 + epl, epl)
        B = eng.gen_fresh(n, 0xB000 + epl, epl)
        Cb, plan = eng.ct_mul_plan(A, B)
        nonces = eng.torch.empty(2 * plan.total_layer_slots, dtype=eng.torch.int64, device=eng.device)
        eng.fill_random(nonces, 77)
        r0 = eng.ct_mul_redo_count()
        out = eng.ct_mul(A, B, nonces=nonces, C_=Cb, plan=plan).to_host()
        if epl != 1:   # (1 edge per layer: 1,348 key slots in 5 buckets, beyond the member list)
            assert eng.ct_mul_redo_count() == r0, "ordinary fresh pairs fell back to the general path"
        ha, hb = A.to_host(), B.to_host()
        nz = nonces.cpu().numpy().view(np.uint64)
        loff = Cb.l_off.cpu().numpy().view(np.uint64)
        for p in range(n):
            x, y = ha[p], hb[p]
            base = int(loff[p]) + x.nL + y.nL
            nn = 2 * x.nL * y.nL
            ref = oracle.ct_mul(Cipher(x.layers, x.meta, x.w_lo, x.w_hi), Cipher(y.layers, y.meta, y.w_lo, y.w_hi),
                                nz[2 * base:2 * base + nn], canon_tag=0x1234)
            _assert_same(out[p], ref, layers_view=False)


def test_ct_mul_one_call_equals_plan_exec(engine):
    """pvac_hip_ct_mul (plan + exec in one call into caller-sized outputs, the bench's step) gives
    the bytes of plan then exec, call after call into the same arrays, and refuses outputs smaller
    than the plan's totals with PVAC_ENOMEM before launching anything."""
    from pvac_hfhe_cppbyv_amd import DeviceBatch, Engine, PvacError
    eng = Engine(device=0, canon_tag=0x1234)
    n = 4096
    A = eng.gen_fresh(n, 0xA001, 20)
    B = eng.gen_fresh(n, 0xB001, 20)
    Cb, plan = eng.ct_mul_plan(A, B)
    nonces = eng.torch.empty(2 * plan.total_layer_slots, dtype=eng.torch.int64, device=eng.device)
    eng.fill_random(nonces, 91)
    ref = eng.ct_mul(A, B, nonces=nonces, C_=Cb, plan=plan).to_host()
    D = eng.ct_mul(A, B, nonces=nonces)   # arrays sized by its own plan
    for fill in (0x5A5A5A5A5A5A5A5A, -1):
        for t in (D.meta, D.w_lo, D.w_hi, D.layers, D.e_cnt, D.l_cnt):
            t.fill_(fill)
        p2 = eng.ct_mul_into(A, B, D, nonces)
        assert (p2.total_layer_slots, p2.total_edge_slots) == (plan.total_layer_slots, plan.total_edge_slots)
        got = D.to_host()
        for p in range(n):
            _assert_same(got[p], ref[p], layers_view=False)
    run = eng.ct_mul_step(A, B, D, nonces)   # the bench's prepared form of the same call
    for t in (D.meta, D.w_lo, D.w_hi, D.layers):
        t.fill_(7)
    assert run().total_edge_slots == plan.total_edge_slots
    got = D.to_host()
    for p in range(n):
        _assert_same(got[p], ref[p], layers_view=False)
    small = DeviceBatch.empty(n, plan.total_layer_slots, plan.total_edge_slots - 1, eng.device)
    with pytest.raises(PvacError):
        eng.ct_mul_into(A, B, small, nonces)
    # the context stays usable and the refused plan is not exec-able
    again = eng.ct_mul_into(A, B, D, nonces)
    assert again.total_edge_slots == plan.total_edge_slots


def test_ct_mul_full_range_golden(engine):
    """The reference's own ct_mul outputs on weights anywhere in [0, 2^128) (oracle/ref_harness.cpp
    fullrange): full-range words, p, p-1, 2^127, 2^128-1, 0, a cancelling key pair (fresh kernel ->
    redo on the general path) and a general-path shape, all in one batch, byte-exact."""
    import json
    from pvac_hfhe_cppbyv_amd import Engine
    with open(os.path.join(REF, "fr_manifest.json")) as f:
        fm = json.load(f)
    eng = Engine(device=0, canon_tag=fm["canon_tag"])
    ks = range(len(fm["cases"]))
    xs = [read_ct(os.path.join(REF, f"fr{k}_x.ct"))[0] for k in ks]
    ys = [read_ct(os.path.join(REF, f"fr{k}_y.ct"))[0] for k in ks]
    streams = [read_u64(f"fr{k}_mul_stream.u64") for k in ks]
    A, B = _dev_batch(eng, xs), _dev_batch(eng, ys)
    Cb, plan = eng.ct_mul_plan(A, B)
    assert plan.n_small == 4 and plan.n_large == 1
    nonces = _nonce_buffer(eng, Cb, xs, ys, streams)
    redo0 = eng.ct_mul_redo_count()
    out = eng.ct_mul(A, B, nonces=nonces, C_=Cb, plan=plan).to_host()
    assert eng.ct_mul_redo_count() - redo0 == 2   # exactly cases 2 (zero weights) and 3 (cancelling keys)
    for k in ks:
        _assert_same(out[k], read_ct(os.path.join(REF, f"fr{k}_mul_w.ct"))[0])
        full = read_layers_u64(f"fr{k}_mul_layers.u64")
        for f in ("rule", "pa", "pb", "ztag", "nonce_lo", "nonce_hi"):
            assert np.array_equal(out[k].layers[f], full[f]), (k, f)
    # the reference's gsum invariant (utils/metrics.hpp:88-113) on the device, with the fixture
    # key's powg_B; then one corrupted output weight must be caught at its pair
    eng.set_powg(read_u64("powg_B.u64"))
    assert eng.check_mul_gsum(A, B, Cb, nonces) == 0
    eo = int(Cb.e_off[3].item())
    Cb.w_lo[eo + 7] ^= 1
    bad, st = eng.check_mul_gsum(A, B, Cb, nonces, status=True)
    assert bad == 1 and list(st) == [0, 0, 0, 1, 0]


_SPECIAL_W = [(2**64 - 1, 2**63 - 1), (2**64 - 2, 2**63 - 1), (0, 2**63), (2**64 - 1, 2**64 - 1), (0, 0), (1, 0),
              (1, 2**63), (2**64 - 1, 2**63), (2**63, 2**62), (5, 2**64 - 16)]


def _full_range_cipher(rng, nl, ne, special_frac=0.15, dup_frac=0.1):
    """A random cipher whose weights cover [0, 2^128): both words uniform, a share replaced by the
    special values, and a share of edges that repeat an earlier edge's (layer, idx, ch) with the
    negated weight (keys whose sums cancel)."""
    from helpers import LAYER_DT
    L = np.zeros(nl, LAYER_DT)
    L["ztag"] = rng.integers(0, 2**63, nl, dtype=np.uint64)
    L["nonce_lo"] = rng.integers(0, 2**63, nl, dtype=np.uint64)
    lay = rng.integers(0, nl, ne).astype(np.uint64)
    idx = rng.integers(0, 337, ne).astype(np.uint64)
    ch = rng.integers(0, 2, ne).astype(np.uint64)
    lo = rng.integers(0, 2**64, ne, dtype=np.uint64)
    hi = rng.integers(0, 2**64, ne, dtype=np.uint64)
    for e in np.flatnonzero(rng.random(ne) < special_frac):
        lo[e], hi[e] = _SPECIAL_W[rng.integers(0, len(_SPECIAL_W))]
    for e in np.flatnonzero(rng.random(ne) < dup_frac):
        if e == 0:
            continue
        s = int(rng.integers(0, e))
        lay[e], idx[e], ch[e] = lay[s], idx[s], ch[s]
        w = ((int(hi[s]) << 64) | int(lo[s])) % P
        nw = (P - w) % P
        lo[e], hi[e] = nw & (2**64 - 1), nw >> 64
    meta = lay | (idx << np.uint64(32)) | (ch << np.uint64(48))
    return Cipher(L, meta, lo, hi)


@pytest.mark.parametrize("shape", ["fresh", "general"])
def test_ct_mul_full_range_vs_oracle(engine, oracle, shape):
    """Synthetic full-range weights (lo and hi uniform over u64, the special values p, p-1, 2^127,
    2^128-1, 0, 1 and cancelling duplicates) through the fresh kernel (2 x 20-edge layers) and the
    general path (3 x 60 by 2 x 70 edges) vs the oracle, bit-exact incl. emit order."""
    from pvac_hfhe_cppbyv_amd import Engine
    rng = np.random.default_rng(0xF011 if shape == "fresh" else 0xF012)
    eng = Engine(device=0, canon_tag=0x77)
    if shape == "fresh":
        n, sa, sb = 1024, (2, 40), (2, 40)
    else:
        n, sa, sb = 24, (3, 60), (2, 70)
    xs = [_full_range_cipher(rng, *sa) for _ in range(n)]
    ys = [_full_range_cipher(rng, *sb) for _ in range(n)]
    A, B = _dev_batch(eng, xs), _dev_batch(eng, ys)
    Cb, plan = eng.ct_mul_plan(A, B)
    assert (plan.n_small, plan.n_large) == ((n, 0) if shape == "fresh" else (0, n))
    nonces = eng.torch.empty(2 * plan.total_layer_slots, dtype=eng.torch.int64, device=eng.device)
    eng.fill_random(nonces, 0xF00)
    out = eng.ct_mul(A, B, nonces=nonces, C_=Cb, plan=plan).to_host()
    nz = nonces.cpu().numpy().view(np.uint64)
    loff = Cb.l_off.cpu().numpy().view(np.uint64)
    for p, (x, y) in enumerate(zip(xs, ys)):
        base = int(loff[p]) + x.nL + y.nL
        ref = oracle.ct_mul(x, y, nz[2 * base:2 * base + 2 * x.nL * y.nL], canon_tag=0x77)
        _assert_same(out[p], ref, layers_view=False)


def test_ct_mul_rejects_out_of_contract_edges(engine, oracle):
    """Edges outside the Cipher contract (layer_id >= |X.L|, idx >= B, ch > 1) reject their pair on
    both paths: status 2 and an empty output (include/pvac_hip.h, pvac_hip_ct_mul_status); the
    valid pairs of the same batch are unaffected and bit-exact vs the oracle."""
    from pvac_hfhe_cppbyv_amd import Engine
    rng = np.random.default_rng(0xBAD)
    eng = Engine(device=0, canon_tag=0x99)
    shapes = [((2, 40), (2, 40))] * 4 + [((3, 60), (2, 70))] * 3
    xs = [_full_range_cipher(rng, *a, dup_frac=0) for a, _ in shapes]
    ys = [_full_range_cipher(rng, *b, dup_frac=0) for _, b in shapes]
    u = np.uint64
    xs[1].meta[5] = (xs[1].meta[5] & ~(u(0xFFFF) << u(32))) | (u(337) << u(32))   # idx == B
    ys[2].meta[7] = (ys[2].meta[7] & ~(u(0xFF) << u(48))) | (u(2) << u(48))        # ch == 2
    xs[3].meta[0] = (xs[3].meta[0] & ~u(0xFFFFFFFF)) | u(2)                           # layer_id == |A.L|
    ys[5].meta[3] = (ys[5].meta[3] & ~(u(0xFFFF) << u(32))) | (u(4000) << u(32))  # idx >> B (general path)
    A, B = _dev_batch(eng, xs), _dev_batch(eng, ys)
    Cb, plan = eng.ct_mul_plan(A, B)
    assert (plan.n_small, plan.n_large) == (4, 3)
    nonces = eng.torch.empty(2 * plan.total_layer_slots, dtype=eng.torch.int64, device=eng.device)
    eng.fill_random(nonces, 0xBAD)
    out = eng.ct_mul(A, B, nonces=nonces, C_=Cb, plan=plan)
    st = eng.ct_mul_status(len(shapes))
    assert list(st) == [0, 2, 2, 2, 0, 2, 0]
    host = out.to_host()
    nz = nonces.cpu().numpy().view(np.uint64)
    loff = Cb.l_off.cpu().numpy().view(np.uint64)
    for p, (x, y) in enumerate(zip(xs, ys)):
        if st[p] == 2:
            assert host[p].nE == 0 and host[p].nL == 0
            continue
        base = int(loff[p]) + x.nL + y.nL
        ref = oracle.ct_mul(x, y, nz[2 * base:2 * base + 2 * x.nL * y.nL], canon_tag=0x99)
        _assert_same(host[p], ref, layers_view=False)


def test_ct_mul_edge_cases(engine, oracle):
    """Empty ciphers, single-edge ciphers, 1-layer ciphers, and a tiny edge_budget that triggers
    guard_budget -> compact_edges ordering (encrypt.hpp:106-111)."""
    from pvac_hfhe_cppbyv_amd import Engine, HostCipher, LAYER_DT
    rng = np.random.default_rng(11)

    def mk(nl, ne):
        L = np.zeros(nl, LAYER_DT)
        L["ztag"] = rng.integers(0, 2**63, nl, dtype=np.uint64)
        L["nonce_lo"] = rng.integers(0, 2**63, nl, dtype=np.uint64)
        if nl == 0:
            ne = 0
        lay = rng.integers(0, max(nl, 1), ne).astype(np.uint64)
        idx = rng.integers(0, 337, ne).astype(np.uint64)
        ch = rng.integers(0, 2, ne).astype(np.uint64)
        meta = lay | (idx << np.uint64(32)) | (ch << np.uint64(48))
        lo = rng.integers(0, 2**63, ne, dtype=np.uint64)
        hi = rng.integers(0, 2**62, ne, dtype=np.uint64)
        return Cipher(L, meta, lo, hi)

    shapes = [((2, 40), (2, 0)), ((2, 0), (2, 40)), ((0, 0), (2, 40)), ((1, 1), (1, 1)), ((1, 30), (2, 40)),
              ((2, 64), (2, 64)), ((1, 100), (1, 40)), ((3, 60), (1, 60)), ((2, 40), (2, 40))]
    for budget in (1200000, 500):
        eng = Engine(device=0, canon_tag=99, edge_budget=budget)
        xs = [mk(*a) for a, _ in shapes]
        ys = [mk(*b) for _, b in shapes]
        A, B = _dev_batch(eng, xs), _dev_batch(eng, ys)
        Cb, plan = eng.ct_mul_plan(A, B)
        nonces = eng.torch.empty(2 * max(plan.total_layer_slots, 1), dtype=eng.torch.int64, device=eng.device)
        eng.fill_random(nonces, 5)
        out = eng.ct_mul(A, B, nonces=nonces, C_=Cb, plan=plan).to_host()
        nz = nonces.cpu().numpy().view(np.uint64)
        loff = Cb.l_off.cpu().numpy().view(np.uint64)
        for p, (x, y) in enumerate(zip(xs, ys)):
            base = int(loff[p]) + x.nL + y.nL
            ref = oracle.ct_mul(x, y, nz[2 * base:2 * base + 2 * x.nL * y.nL], canon_tag=99, edge_budget=budget)
            _assert_same(out[p], ref, layers_view=False)


def test_ct_mul_roundtrip_decrypt(engine, manifest, oracle):
    """dec(ct_mul(enc x, enc y)) == x*y with fixture R values (reference test_main.cpp:178-188)."""
    from pvac_hfhe_cppbyv_amd import Engine
    eng = Engine(device=0, canon_tag=manifest["canon_tag"])
    powg = read_u64("powg_B.u64")
    for p in range(8):
        x = read_ct(os.path.join(REF, f"pair{p}_x.ct"))[0]
        y = read_ct(os.path.join(REF, f"pair{p}_y.ct"))[0]
        out = eng.ct_mul(_dev_batch(eng, [x]), _dev_batch(eng, [y]), nonce_seed=p).to_host()[0]
        c = Cipher(out.layers, out.meta, out.w_lo, out.w_hi)
        R = R_for(c, [(x, read_u64(f"pair{p}_x_R.u64")), (y, read_u64(f"pair{p}_y_R.u64"))])
        m = manifest["pairs"][p]
        assert oracle.dec(c, powg, R)[0] == (m["x"] * m["y"]) % P


def test_sigma_batch_matches_oracle(engine, oracle):
    """pvac_hip_sigma_batch on arbitrary (layer, idx, ch, salt) edges vs the oracle's sigma_from_H,
    with H uploaded from a host dense matrix (set_H)."""
    from pvac_hfhe_cppbyv_amd import Engine
    eng = Engine(device=0, canon_tag=4242)
    H, _ = oracle.gen_H(4242)
    eng.set_H(H)
    X = eng.gen_fresh(6, 31, 20)
    X.sigma = eng.torch.zeros((X.meta.numel(), 128), dtype=eng.torch.int64, device=eng.device)
    salts = eng.torch.empty(X.meta.numel(), dtype=eng.torch.int64, device=eng.device)
    eng.fill_random(salts, 9)
    eng.sigma(X, salts)
    hs = X.to_host()
    sl = salts.cpu().numpy().view(np.uint64)
    k = 0
    for c in hs:
        for e in range(c.nE):
            L = c.layers[int(c.meta[e]) & 0xFFFFFFFF]
            ref = oracle.sigma(4242, H, int(L["ztag"]), int(L["nonce_lo"]), int(L["nonce_hi"]),
                               (int(c.meta[e]) >> 32) & 0xFFFF, (int(c.meta[e]) >> 48) & 0xFF, int(sl[k]))
            assert np.array_equal(c.sigma[e], ref), (k,)
            k += 1


@pytest.mark.parametrize("path", ["delta", "u16", "copies", "generic"])
def test_sigma_expansion_paths(engine, oracle, monkeypatch, path):
    """Every column-expansion path of k_sigma (PVAC_SIGMA_PATH: byte-delta tables, u16 rows with
    per-wave images, per-lane-group copies, the generic guarded loop) gives the oracle's
    sigma_from_H on a sample, and the same bytes as the default path on 2,600 edges."""
    from pvac_hfhe_cppbyv_amd import Engine
    eng = Engine(device=0, canon_tag=77)
    H, _ = oracle.gen_H(77)
    eng.set_H(H)
    X = eng.gen_fresh(65, 41, 20)
    ne = X.meta.numel()
    salts = eng.torch.empty(ne, dtype=eng.torch.int64, device=eng.device)
    eng.fill_random(salts, 12)
    X.sigma = eng.torch.zeros((ne, 128), dtype=eng.torch.int64, device=eng.device)
    monkeypatch.delenv("PVAC_SIGMA_PATH", raising=False)
    eng.sigma(X, salts)
    ref_all = X.sigma.clone()
    X.sigma.fill_(-1)
    monkeypatch.setenv("PVAC_SIGMA_PATH", path)
    eng.sigma(X, salts)
    eng.torch.cuda.synchronize()
    assert eng.torch.equal(X.sigma, ref_all)
    hs = X.to_host()
    sl = salts.cpu().numpy().view(np.uint64)
    k = 0
    for c in hs[:3]:
        for e in range(c.nE):
            L = c.layers[int(c.meta[e]) & 0xFFFFFFFF]
            ref = oracle.sigma(77, H, int(L["ztag"]), int(L["nonce_lo"]), int(L["nonce_hi"]),
                               (int(c.meta[e]) >> 32) & 0xFFFF, (int(c.meta[e]) >> 48) & 0xFF, int(sl[k]))
            assert np.array_equal(c.sigma[e], ref), (path, k)
            k += 1


def _pair_host(X, p):
    """Cipher p of a device batch, copied alone (no full-batch transfer)."""
    from helpers import LAYER_DT
    u = lambda t: t.cpu().numpy().view(np.uint64)
    lo, lc = int(X.l_off[p].item()), int(X.l_cnt[p].item())
    eo, ec = int(X.e_off[p].item()), int(X.e_cnt[p].item())
    layers = X.layers[lo:lo + lc].cpu().numpy().reshape(-1).view(LAYER_DT).copy()
    return Cipher(layers, u(X.meta[eo:eo + ec]).copy(), u(X.w_lo[eo:eo + ec]).copy(), u(X.w_hi[eo:eo + ec]).copy())


def _full_batch_vs_oracle(oracle, n, first, n_picks, rerun):
    """One full batch of the bench's generator at global pair indices [first, first + n): every
    reported output slot written by this launch (sentinel-filled outputs), every pair's edges equal to
    the pinned CPU port's (per-pair digests), the reference's gsum invariant on every pair, n_picks
    pairs spread over the batch bit-exact vs the oracle (weights, emit order, layers incl. ztags),
    every pair within its planned capacity with status 0, and (rerun) a second run identical."""
    from pvac_hfhe_cppbyv_amd import Engine
    eng = Engine(device=0, canon_tag=0x5EED0003)
    A = eng.gen_fresh(n, 0x5EED0003, 20, first_index=first)
    B = eng.gen_fresh(n, 0x5EED0004, 20, first_index=first)
    Cb, plan = eng.ct_mul_plan(A, B)
    nonces = eng.fill_nonces(A, B, Cb, plan, 0x5EED0005, first_index=first)
    # outputs pre-filled with a sentinel no record can hold (meta ch byte, w_hi top bit): every
    # reported edge and layer slot must have been written by this launch, not left from an earlier one
    torch = eng.torch
    es, ls = plan.total_edge_slots, plan.total_layer_slots
    Cb.layers = torch.full((ls, 5), -1, dtype=torch.int64, device=eng.device)
    Cb.meta, Cb.w_lo, Cb.w_hi = (torch.full((es,), -1, dtype=torch.int64, device=eng.device) for _ in range(3))
    out = eng.ct_mul(A, B, nonces=nonces, C_=Cb, plan=plan)
    assert eng.ct_mul_redo_count() == 0
    assert not eng.ct_mul_status(n).any()   # every pair in the reference's hash order
    tot_e, tot_l = int(out.e_cnt[:n].sum().item()), int(out.l_cnt[:n].sum().item())
    for t in (out.meta, out.w_lo, out.w_hi):
        assert int((t != -1).sum().item()) == tot_e
    assert int((out.layers[:, 1] != -1).sum().item()) == tot_l
    u = lambda t: t.cpu().numpy().view(np.uint64)
    ecnt, eoff = u(out.e_cnt[:n]), u(out.e_off[:n])
    cap = np.diff(np.append(eoff, np.uint64(plan.total_edge_slots)))
    assert (ecnt <= cap).all() and ecnt.min() > 0
    dig1 = u(eng.digest(out)[:n]).copy()
    # EVERY pair's edges (meta, w in emit order) against the pinned CPU port, by per-pair FNV-1a
    # digest: the oracle runs the reference's unordered_map aggregation on 16 threads
    import ctypes as C
    from helpers import default_params, pack_device_batch
    P_ = lambda x: x.ctypes.data_as(C.c_void_p)
    pa, pb = pack_device_batch(A, n), pack_device_batch(B, n)
    cnt, dig = np.zeros(n, np.uint64), np.zeros(n, np.uint64)
    oracle.lib.orc_ct_mul_batch_timed(C.byref(default_params(0x5EED0003)), n, *(P_(x) for x in pa), *(P_(x) for x in pb),
                                      16, P_(cnt), P_(dig))
    assert np.array_equal(cnt, ecnt)
    bad = np.nonzero(dig != dig1)[0]
    assert bad.size == 0, f"{bad.size} pairs differ from the oracle, first {bad[:8]}"
    del pa, pb
    # the reference's gsum invariant (utils/metrics.hpp:88-113) on every pair
    eng.set_powg(read_u64("powg_B.u64"))
    assert eng.check_mul_gsum(A, B, out, nonces) == 0
    rng = np.random.default_rng(3)
    picks = np.unique(np.concatenate([[0, n - 1], rng.integers(0, n, n_picks - 2)]))
    nz = nonces.cpu().numpy().view(np.uint64)
    loff = u(Cb.l_off[:n])
    for p in picks:
        x, y = _pair_host(A, int(p)), _pair_host(B, int(p))
        base = int(loff[p]) + x.nL + y.nL
        ref = oracle.ct_mul(x, y, nz[2 * base:2 * base + 2 * x.nL * y.nL], canon_tag=0x5EED0003)
        _assert_same(_pair_host(out, int(p)), ref, layers_view=False)
    if not rerun:
        return dig1
    del out, Cb   # two 2^20-pair outputs together are ~140 GB
    eng.torch.cuda.empty_cache()
    Cb2, plan2 = eng.ct_mul_plan(A, B)
    out2 = eng.ct_mul(A, B, nonces=nonces, C_=Cb2, plan=plan2)
    assert np.array_equal(u(eng.digest(out2)[:n]), dig1)
    return dig1


def test_cfg3_full_batch_sampled_vs_oracle(oracle):
    """BASELINE cfg 3 at its full size (2^20 fresh-shaped pairs, the bench's batch and generator):
    the full-batch checks of _full_batch_vs_oracle, 512 pairs bit-exact, a rerun identical."""
    _full_batch_vs_oracle(oracle, 1 << 20, 0, 512, rerun=True)


def test_cfg5_rank7_shard_vs_oracle(oracle):
    """BASELINE cfg 5's per-GPU work: the last rank's shard of the 8-GPU job, alone on this GPU —
    2^21 pairs at global indices [7 * 2^21, 2^24) from the bench's generator and nonces (bench.py at
    --gpus 8 hands rank 7 exactly this), ~136 GB of output capacity: every slot written, every pair's
    digest equal to the pinned port's, the gsum invariant on every pair, 256 pairs bit-exact vs the
    oracle, status and capacities. Its digests also equal the same global pairs cut from a batch that
    starts at another offset (the shard is keyed by global index only)."""
    n, first = 1 << 21, 7 << 21
    dig = _full_batch_vs_oracle(oracle, n, first, 256, rerun=False)
    from pvac_hfhe_cppbyv_amd import Engine
    eng = Engine(device=0, canon_tag=0x5EED0003)
    k, off = 4096, (7 << 21) + (1 << 20)   # 4,096 pairs from the middle of the shard, generated alone
    A = eng.gen_fresh(k, 0x5EED0003, 20, first_index=off)
    B = eng.gen_fresh(k, 0x5EED0004, 20, first_index=off)
    Cb, plan = eng.ct_mul_plan(A, B)
    nz = eng.fill_nonces(A, B, Cb, plan, 0x5EED0005, first_index=off)
    o = eng.ct_mul(A, B, nonces=nz, C_=Cb, plan=plan)
    assert np.array_equal(eng.digest(o)[:k].cpu().numpy().view(np.uint64), dig[off - first:off - first + k])


@pytest.mark.parametrize("s", [2, P - 1, (0x0123456789ABCDEF << 64) | 0xFEDCBA9876543210])
def test_ct_scale_ragged(engine, oracle, s):
    """ct_scale (ops/arithmetic.hpp:33-37) in place, per-edge fp_mul by s, on ciphers whose edge
    counts straddle k_ct_scale's register-held first 64 weights (0, 1, 31..33, 63..65, 97, a
    fresh cipher and the full chain-step-3 cipher); layers and edge metadata pass through."""
    chain = read_ct(os.path.join(REF, "chain3.ct"))[0]
    fresh = read_ct(os.path.join(REF, "pair0_x.ct"))[0]
    cs = [Cipher(chain.layers, chain.meta[:k], chain.w_lo[:k], chain.w_hi[:k]) for k in (0, 1, 31, 32, 33, 63, 64, 65, 97)]
    cs += [fresh, chain]
    X = _dev_batch(engine, cs)
    engine.ct_scale(X, s)
    out = X.to_host()
    s_lo, s_hi = np.uint64(s & ((1 << 64) - 1)), np.uint64(s >> 64)
    for c, o in zip(cs, out):
        n = len(c.w_lo)
        want_lo, want_hi = oracle.fp("mul", c.w_lo, c.w_hi, np.full(n, s_lo, np.uint64), np.full(n, s_hi, np.uint64))
        assert np.array_equal(o.w_lo, want_lo) and np.array_equal(o.w_hi, want_hi)
        assert np.array_equal(o.meta, c.meta) and o.layers.tobytes() == c.layers.tobytes()


def test_ct_neg_and_div_const(engine, oracle):
    """ct_neg (ops/arithmetic.hpp:39-41) = ct_scale by p - 1 and ct_div_const (:108-110) = ct_scale
    by fp_inv(k) (core/field.hpp:229-273), against the oracle's fp_mul / fp_inv; k = 0 scales by
    fp_inv(0) = 0 as the reference does."""
    chain = read_ct(os.path.join(REF, "chain3.ct"))[0]
    fresh = read_ct(os.path.join(REF, "pair0_x.ct"))[0]
    cs = [fresh, chain]
    one = lambda v: (np.array([v & ((1 << 64) - 1)], np.uint64), np.array([v >> 64], np.uint64))
    X = _dev_batch(engine, cs)
    engine.ct_neg(X)
    for c, o in zip(cs, X.to_host()):
        n = len(c.w_lo)
        want = oracle.fp("mul", c.w_lo, c.w_hi, np.full(n, ~np.uint64(1), np.uint64),
                         np.full(n, np.uint64(0x7FFFFFFFFFFFFFFF), np.uint64))
        assert np.array_equal(o.w_lo, want[0]) and np.array_equal(o.w_hi, want[1])
        assert np.array_equal(o.meta, c.meta) and o.layers.tobytes() == c.layers.tobytes()
    for k in (2, 0, 1, P - 1, (0x0123456789ABCDEF << 64) | 0xFEDCBA9876543210, (1 << 128) - 1):
        ilo, ihi = oracle.fp("inv", *one(k))
        assert engine.fp_inv(k) == int(ilo[0]) | (int(ihi[0]) << 64)
        X = _dev_batch(engine, cs)
        engine.ct_div_const(X, k)
        for c, o in zip(cs, X.to_host()):
            n = len(c.w_lo)
            want = oracle.fp("mul", c.w_lo, c.w_hi, np.full(n, ilo[0], np.uint64), np.full(n, ihi[0], np.uint64))
            assert np.array_equal(o.w_lo, want[0]) and np.array_equal(o.w_hi, want[1])
    assert engine.fp_inv(2) == 1 << 126


def test_ct_mul_api_errors_leave_context_usable(oracle):
    """Errors fail loudly (PvacError with the ABI's message) and leave the context usable:
    |A| != |B| at plan time, exec with a plan a later plan made stale, and a pair whose product
    layers exceed the general path's table (|A.L| + |B.L| + |A.L||B.L| > 16,384: PVAC_ENOSYS,
    where the reference would run it). A normal batch on the same context is then bit-exact."""
    from pvac_hfhe_cppbyv_amd import Engine, PvacError
    eng = Engine(device=0, canon_tag=0x55)
    rng = np.random.default_rng(0x55)
    xs = [_full_range_cipher(rng, 2, 40, dup_frac=0) for _ in range(3)]
    ys = [_full_range_cipher(rng, 2, 40, dup_frac=0) for _ in range(3)]
    A, B = _dev_batch(eng, xs), _dev_batch(eng, ys)
    with pytest.raises(PvacError):
        eng.ct_mul_plan(A, _dev_batch(eng, ys[:2]))
    Cb, plan = eng.ct_mul_plan(A, B)
    nonces = eng.torch.empty(2 * plan.total_layer_slots, dtype=eng.torch.int64, device=eng.device)
    eng.fill_random(nonces, 0x55)
    Cb2, plan2 = eng.ct_mul_plan(A, B)   # `plan` is stale from here on
    with pytest.raises(PvacError, match="latest"):
        eng.ct_mul(A, B, nonces=nonces, C_=Cb, plan=plan)
    big_a, big_b = _full_range_cipher(rng, 200, 64, dup_frac=0), _full_range_cipher(rng, 90, 64, dup_frac=0)
    with pytest.raises(PvacError, match="layers"):
        eng.ct_mul_plan(_dev_batch(eng, [big_a]), _dev_batch(eng, [big_b]))
    Cb, plan = eng.ct_mul_plan(A, B)
    out = eng.ct_mul(A, B, nonces=nonces, C_=Cb, plan=plan).to_host()
    assert list(eng.ct_mul_status(3)) == [0, 0, 0]
    nz = nonces.cpu().numpy().view(np.uint64)
    loff = Cb.l_off.cpu().numpy().view(np.uint64)
    for p, (x, y) in enumerate(zip(xs, ys)):
        base = int(loff[p]) + x.nL + y.nL
        ref = oracle.ct_mul(x, y, nz[2 * base:2 * base + 2 * x.nL * y.nL], canon_tag=0x55)
        _assert_same(out[p], ref, layers_view=False)


def test_sumdigest_matches_numpy_restatement():
    """pvac_hip_batch_sumdigest (the parallel position-keyed digest the chain's timed pass uses) equals
    its numpy restatement on ragged ciphers (0, 1, 255, 256, 257 and thousands of edges)."""
    from pvac_hfhe_cppbyv_amd import DeviceBatch, Engine, HostCipher
    from helpers import LAYER_DT, sumdigest
    eng = Engine(device=0)
    rng = np.random.default_rng(0x5D16)
    cs = []
    for ne in (0, 1, 255, 256, 257, 4099):
        L = np.zeros(2, LAYER_DT)
        cs.append(HostCipher(L, rng.integers(0, 2**63, ne, dtype=np.uint64), rng.integers(0, 2**64, ne, dtype=np.uint64),
                             rng.integers(0, 2**64, ne, dtype=np.uint64)))
    got = eng.sumdigest(DeviceBatch.from_host(cs, eng.device)).cpu().numpy().view(np.uint64)
    assert [int(g) for g in got] == [sumdigest(c) for c in cs]
