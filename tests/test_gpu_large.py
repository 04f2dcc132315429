"""GPU parity of the general ct_mul path (k_mul_large.hip): chains c_k = c_{k-1} * x_k
(reference tests/test_main.cpp:289-295), squares c <- c * c (tests/test_depth.cpp:46), pairs the
fresh kernel cannot hold, mixed batches, duplicate edges, guard_budget ordering. Bit-exact
against the reference's golden fixtures and the pinned CPU oracle."""
import hashlib
import os

import numpy as np
import pytest

from helpers import REF, Cipher, LAYER_DT, read_ct, read_layers_u64, read_u64, R_for

pytestmark = pytest.mark.gpu


def _dev_batch(engine, ciphers, sigma=False):
    from pvac_hfhe_cppbyv_amd import DeviceBatch, HostCipher
    hc = [HostCipher(c.layers, c.meta, c.w_lo, c.w_hi, c.sigma) for c in ciphers]
    return DeviceBatch.from_host(hc, engine.device, sigma=sigma)


def _i64(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64))


def _layers_view(L):
    L = L.copy()
    prod = L["rule"] == 1
    for f in ("ztag", "nonce_lo", "nonce_hi"):
        L[f][prod] = 0
    L["pa"][~prod] = 0
    L["pb"][~prod] = 0
    return L


def _same(got, ref, view=True, sigma=False):
    L = _layers_view(got.layers) if view else got.layers
    for f in ("rule", "pa", "pb", "ztag", "nonce_lo", "nonce_hi"):
        assert np.array_equal(L[f], ref.layers[f]), f
    assert got.nE == ref.nE
    assert np.array_equal(got.meta, ref.meta)
    assert np.array_equal(got.w_lo, ref.w_lo) and np.array_equal(got.w_hi, ref.w_hi)
    if sigma:
        assert np.array_equal(got.sigma, ref.sigma)


def _run_mul(eng, xs, ys, streams=None, seed=1, flags=0, with_salts=False):
    """Batched ct_mul; per-pair reference streams (nonces, then salts) placed at their slots."""
    A, B = _dev_batch(eng, xs), _dev_batch(eng, ys)
    Cb, plan = eng.ct_mul_plan(A, B)
    loff = Cb.l_off.cpu().numpy().view(np.uint64)
    eoff = Cb.e_off.cpu().numpy().view(np.uint64)
    rng = np.random.default_rng(seed)
    nonces = rng.integers(0, 2**63, 2 * max(plan.total_layer_slots, 1), dtype=np.uint64)
    salts = np.zeros(max(plan.total_edge_slots, 1), np.uint64)
    per = []
    for p, (x, y) in enumerate(zip(xs, ys)):
        base = int(loff[p]) + x.nL + y.nL
        nn = 2 * x.nL * y.nL
        if streams is not None:
            nonces[2 * base:2 * base + nn] = streams[p][:nn]
            s = streams[p][nn:]
            salts[int(eoff[p]):int(eoff[p]) + len(s)] = s
        per.append(nonces[2 * base:2 * base + nn].copy())
    kw = {}
    if with_salts:
        kw["salts"] = _i64(salts).to(eng.device)
    out = eng.ct_mul(A, B, nonces=_i64(nonces).to(eng.device), C_=Cb, plan=plan, flags=flags, **kw)
    return out.to_host(), plan, per


def _sigdig(sig):
    """Per-edge digest of the harness: first 8 bytes (LE) of SHA-256 over the LE sigma words."""
    return np.array([int.from_bytes(hashlib.sha256(row.astype("<u8").tobytes()).digest()[:8], "little")
                     for row in sig], np.uint64)


# ------------------------------------------------------------------ reference golden chains
@pytest.mark.parametrize("kind,steps", [("chain", 3), ("sq", 2)])
def test_chain_and_square_golden_gpu(manifest, kind, steps):
    """Each step as a batch of one through the engine: layers (incl. ztags), edge order and
    weights identical to the reference's .ct; edges/layers/dec values from the manifest."""
    from pvac_hfhe_cppbyv_amd import Engine
    from helpers import Oracle
    orc = Oracle.load()
    eng = Engine(device=0, canon_tag=manifest["canon_tag"])
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
        out, plan, _ = _run_mul(eng, [cur], [x], [stream])
        if k >= 2:
            assert plan.n_large == 1, "step >= 2 must take the general path"
        got = out[0]
        _same(got, read_ct(os.path.join(REF, f"{kind}{k}.ct"))[0])
        full = read_layers_u64(f"{kind}{k}_layers.u64")
        assert np.array_equal(got.layers["ztag"], full["ztag"])
        rec = manifest["chain" if kind == "chain" else "square"][k - 1]
        assert got.nE == rec["edges"] and got.nL == rec["layers"]
        gc = Cipher(got.layers, got.meta, got.w_lo, got.w_hi)
        assert list(orc.dec(gc, read_u64("powg_B.u64"), R_for(gc, Rin))) == rec["dec"]
        cur = Cipher(full, got.meta, got.w_lo, got.w_hi)


def test_chain_sigma_golden_gpu(manifest):
    """WITH_SIGMA on chain step 2 (general path): every output sigma's digest equals the
    reference's (crypto/matrix.hpp:267-303 with the reference's salts)."""
    from pvac_hfhe_cppbyv_amd import Engine, MUL_WITH_SIGMA
    eng = Engine(device=0, canon_tag=manifest["canon_tag"])
    assert eng.gen_H().hex() == manifest["H_digest"]
    c1 = Cipher(read_layers_u64("chain1_layers.u64"), *[getattr(read_ct(os.path.join(REF, "chain1.ct"))[0], f)
                                                         for f in ("meta", "w_lo", "w_hi")])
    x = read_ct(os.path.join(REF, "chain2_x.ct"))[0]
    out, plan, _ = _run_mul(eng, [c1], [x], [read_u64("chain2_stream.u64")], flags=MUL_WITH_SIGMA,
                            with_salts=True)
    assert plan.n_large == 1
    assert np.array_equal(_sigdig(out[0].sigma), read_u64("chain2_sigdig.u64"))


# ------------------------------------------------------------------ synthetic vs oracle
def _mk(rng, nl, ne, dup_ok=True, B=337):
    L = np.zeros(nl, LAYER_DT)
    L["ztag"] = rng.integers(0, 2**63, nl, dtype=np.uint64)
    L["nonce_lo"] = rng.integers(0, 2**63, nl, dtype=np.uint64)
    if nl == 0:
        ne = 0
    if dup_ok:
        lay = rng.integers(0, max(nl, 1), ne).astype(np.uint64)
        idx = rng.integers(0, B, ne).astype(np.uint64)
        ch = rng.integers(0, 2, ne).astype(np.uint64)
    else:   # distinct (layer, idx, ch), shuffled
        pick = rng.choice(max(nl, 1) * 2 * B, size=ne, replace=False).astype(np.uint64)
        lay, rest = pick // np.uint64(2 * B), pick % np.uint64(2 * B)
        idx, ch = rest >> np.uint64(1), rest & np.uint64(1)
    meta = lay | (idx << np.uint64(32)) | (ch << np.uint64(48))
    lo = rng.integers(0, 2**63, ne, dtype=np.uint64)
    hi = rng.integers(0, 2**62, ne, dtype=np.uint64)
    return Cipher(L, meta, lo, hi)


def _check_vs_oracle(oracle, eng_kw, xs, ys, seed):
    from pvac_hfhe_cppbyv_amd import Engine
    eng = Engine(device=0, **eng_kw)
    out, plan, per = _run_mul(eng, xs, ys, seed=seed)
    for p, (x, y) in enumerate(zip(xs, ys)):
        ref = oracle.ct_mul(x, y, per[p], canon_tag=eng_kw.get("canon_tag", 0),
                            edge_budget=eng_kw.get("edge_budget", 1200000))
        _same(out[p], ref, view=False)
    return plan


def test_large_dense_chain_like_vs_oracle(oracle):
    """Dense-owner mode: 3-6 layer ciphers with 200-674 distinct edges per layer times fresh-like
    ciphers, plus their transposes (dense side = B)."""
    rng = np.random.default_rng(5)
    xs, ys = [], []
    for k in range(12):
        nl = 3 + k % 4
        x = _mk(rng, nl, int(nl * rng.integers(200, 674)), dup_ok=False)
        y = _mk(rng, 2, 40, dup_ok=False)
        xs.append(x); ys.append(y)
        xs.append(y); ys.append(x)
    plan = _check_vs_oracle(oracle, {"canon_tag": 7}, xs, ys, 11)
    assert plan.n_large == len(xs)


def test_large_column_bounds_vs_oracle(oracle):
    """Column accumulators of the dense loop (fp127.hpp col26_*) at their limits: both sides
    saturated (every (idx, ch) cell of a layer, so the sparse side is 674 edges = 6 chunks of 128),
    weights at and near the top of the canonical range (p - 1 = all 26-bit limbs full, values that
    canonicalise to it, 2^127 - 2^k) mixed with random full-range words; squares and a 2-layer x
    1-layer shape, vs the oracle bit-exact."""
    rng = np.random.default_rng(0xC0126)
    B = 337
    p = (1 << 127) - 1
    top = [p - 1, p - 2, (1 << 127) - (1 << 26) - 1, (1 << 126), p + (p - 1), (1 << 128) - 2]

    def sat(nl, top_frac):
        n = nl * 2 * B
        pick = rng.permutation(n).astype(np.uint64)   # every (layer, idx, ch) once, shuffled
        lay, rest = pick // np.uint64(2 * B), pick % np.uint64(2 * B)
        meta = lay | ((rest >> np.uint64(1)) << np.uint64(32)) | ((rest & np.uint64(1)) << np.uint64(48))
        lo = rng.integers(0, 2**64 - 1, n, dtype=np.uint64, endpoint=True)
        hi = rng.integers(0, 2**64 - 1, n, dtype=np.uint64, endpoint=True)
        sel = rng.random(n) < top_frac
        for k in np.nonzero(sel)[0]:
            v = top[int(rng.integers(0, len(top)))]
            lo[k], hi[k] = v & (2**64 - 1), v >> 64
        L = np.zeros(nl, LAYER_DT)
        L["ztag"] = rng.integers(0, 2**63, nl, dtype=np.uint64)
        L["nonce_lo"] = rng.integers(0, 2**63, nl, dtype=np.uint64)
        return Cipher(L, meta, lo, hi)

    xs, ys = [], []
    for k in range(6):
        x = sat(1 + k % 2, 1.0 if k < 2 else 0.5)
        y = x if k % 3 == 0 else sat(1, 1.0 if k < 2 else 0.5)
        xs.append(x)
        ys.append(y)
    plan = _check_vs_oracle(oracle, {"canon_tag": 0xC0}, xs, ys, 0xC1)
    assert plan.n_large == len(xs)


@pytest.mark.parametrize("Bm", [97, 1031])
def test_ct_mul_other_B_vs_oracle(oracle, Bm):
    """Params.B other than 337 (the reference takes B from Params, core/types.hpp): a small B
    (dense tables of 194 cells) and B = 1031 (three output rows per products lane, 97 KB of LDS per
    workgroup), fresh-shaped and dense chain-like pairs, vs the oracle with the same B."""
    from pvac_hfhe_cppbyv_amd import Engine
    rng = np.random.default_rng(Bm)
    xs, ys = [], []
    for k in range(6):
        xs.append(_mk(rng, 2, 20 + k, dup_ok=False, B=Bm))
        ys.append(_mk(rng, 2, 20, dup_ok=False, B=Bm))
    for k in range(6):
        nl = 2 + k % 3
        x = _mk(rng, nl, int(nl * rng.integers(Bm // 2, 2 * Bm)), dup_ok=False, B=Bm)
        y = _mk(rng, 2, 40, dup_ok=False, B=Bm)
        xs.append(x); ys.append(y)
        xs.append(y); ys.append(x)
    xs.append(_mk(rng, 3, 60, dup_ok=True, B=Bm))   # duplicates: scatter mode
    ys.append(_mk(rng, 2, 50, dup_ok=True, B=Bm))
    eng = Engine(device=0, B=Bm, canon_tag=0xB0)
    out, plan, per = _run_mul(eng, xs, ys, seed=Bm)
    for p, (x, y) in enumerate(zip(xs, ys)):
        ref = oracle.ct_mul(x, y, per[p], canon_tag=0xB0, Bm=Bm)
        _same(out[p], ref, view=False)


def test_large_scatter_and_duplicates_vs_oracle(oracle):
    """Scatter mode (sparse x sparse tasks) and duplicate (layer, idx, ch) edges in the dense side,
    empty layers, empty ciphers, single edges."""
    rng = np.random.default_rng(6)
    shapes = [((5, 30), (4, 30)), ((3, 700), (3, 5)), ((8, 8), (8, 8)), ((2, 0), (9, 10)), ((0, 0), (7, 1)),
              ((6, 1), (6, 1)), ((4, 400), (2, 60)), ((12, 90), (3, 40))]
    xs = [_mk(rng, *a) for a, _ in shapes]
    ys = [_mk(rng, *b) for _, b in shapes]
    _check_vs_oracle(oracle, {"canon_tag": 8}, xs, ys, 12)


def test_large_guard_budget_vs_oracle(oracle):
    """guard_budget -> compact_edges order for pairs above edge_budget (encrypt.hpp:106-111)."""
    rng = np.random.default_rng(7)
    xs = [_mk(rng, 4, 600, dup_ok=False) for _ in range(3)]
    ys = [_mk(rng, 2, 40, dup_ok=False) for _ in range(3)]
    _check_vs_oracle(oracle, {"canon_tag": 9, "edge_budget": 2000}, xs, ys, 13)


def test_mixed_batch_small_and_large_vs_oracle(oracle):
    """Fresh-shape and general pairs interleaved in one batch share one output CSR."""
    from pvac_hfhe_cppbyv_amd import Engine
    rng = np.random.default_rng(8)
    xs, ys = [], []
    for k in range(40):
        if k % 3 == 0:
            xs.append(_mk(rng, 4, 900, dup_ok=False)); ys.append(_mk(rng, 2, 40, dup_ok=False))
        else:
            xs.append(_mk(rng, 2, 40, dup_ok=False)); ys.append(_mk(rng, 2, 40, dup_ok=False))
    plan = _check_vs_oracle(oracle, {"canon_tag": 10}, xs, ys, 14)
    assert plan.n_small > 0 and plan.n_large > 0


def test_engine_chain_depth5_vs_oracle(oracle):
    """Engine-driven chains c_k = c_{k-1} * x_k for 16 inputs to depth 5, each step checked against
    the oracle on the engine's own previous output (cfg-4 shape at reduced depth)."""
    from pvac_hfhe_cppbyv_amd import Engine
    eng = Engine(device=0, canon_tag=0xC4)
    n = 16
    X = eng.gen_fresh(n, 0x4000, 20).to_host()
    cur = [Cipher(c.layers, c.meta, c.w_lo, c.w_hi) for c in X]
    for k in range(1, 6):
        xk = [Cipher(c.layers, c.meta, c.w_lo, c.w_hi) for c in eng.gen_fresh(n, 0x4000 + k, 20).to_host()]
        out, plan, per = _run_mul(eng, cur, xk, seed=100 + k)
        for p in range(n):
            ref = oracle.ct_mul(cur[p], xk[p], per[p], canon_tag=0xC4)
            _same(out[p], ref, view=False)
        cur = [Cipher(o.layers, o.meta, o.w_lo, o.w_hi) for o in out]
    assert cur[0].nE > 10000


def _max_bucket_edges(oracle, x, y, B=337):
    """Edges of the fullest libstdc++ bucket of ct_mul(x, y)'s keys (channels with products; random
    weights make every such sum nonzero), and whether the pair takes the static-group path."""
    G = 0x9E3779B97F4A7C15
    LB = len(y.layers)
    la, ia, ca = (x.meta & 0xFFFFFFFF).astype(np.int64), ((x.meta >> np.uint64(32)) & 0xFFFF).astype(np.int64), (x.meta >> np.uint64(48)).astype(np.int64)
    lb, ib, cb = (y.meta & 0xFFFFFFFF).astype(np.int64), ((y.meta >> np.uint64(32)) & 0xFFFF).astype(np.int64), (y.meta >> np.uint64(48)).astype(np.int64)
    lp = (la[:, None] * LB + lb[None, :]).ravel()
    r = ((ia[:, None] + ib[None, :]) % B).ravel()
    ch = (ca[:, None] ^ cb[None, :]).ravel()
    keych = np.unique(lp * (2 * B) + r * 2 + ch)
    keys, E = np.unique(keych // 2, return_counts=True)
    n = x.nE * y.nE
    nbk = oracle.bucket_count(n)
    bk = np.array([(((int(k) // B) << 32 | (int(k) % B)) * G % 2**64) % nbk for k in keys], dtype=np.uint64)
    _, inv = np.unique(bk, return_inverse=True)
    per = np.bincount(inv, weights=E)
    S = len(x.layers) * LB * B
    return int(per.max()), nbk >= 2 * S


def test_static_bucket_groups_and_escape_codes_vs_oracle(oracle):
    """General-path ordering structures: static bucket groups (bucket count >= 2 S: saturated
    4-layer ciphers x sparse 8-layer ciphers, whose colliding buckets hold 3+ edges, the escape code
    of the 16-time leader blocks) next to dynamic bucket chains (sparse pairs) in one batch."""
    rng = np.random.default_rng(9)
    xs, ys = [], []
    for k in range(6):
        xs.append(_mk(rng, 4, 4 * 2 * 337, dup_ok=False)); ys.append(_mk(rng, 8, 16, dup_ok=False))
        xs.append(_mk(rng, 4, 30, dup_ok=False)); ys.append(_mk(rng, 2, 40, dup_ok=False))
    kinds = [_max_bucket_edges(oracle, x, y) for x, y in zip(xs, ys)]
    assert any(st and mx >= 3 for mx, st in kinds), kinds   # static groups with escape codes
    assert any(not st for _, st in kinds), kinds             # dynamic chains
    plan = _check_vs_oracle(oracle, {"canon_tag": 11}, xs, ys, 15)
    assert plan.n_large == len(xs)


def _mk_layers(rng, counts, dup_layers=(), B=337):
    """A cipher with exactly counts[l] edges in layer l (distinct (idx, ch) cells, in shuffled
    order), except layers in dup_layers, which repeat some of their cells."""
    nl = len(counts)
    L = np.zeros(nl, LAYER_DT)
    L["ztag"] = rng.integers(0, 2**63, nl, dtype=np.uint64)
    L["nonce_lo"] = rng.integers(0, 2**63, nl, dtype=np.uint64)
    metas = []
    for l, c in enumerate(counts):
        cells = rng.choice(2 * B, size=c, replace=l in dup_layers).astype(np.uint64)
        metas.append(np.uint64(l) | ((cells >> np.uint64(1)) << np.uint64(32)) | ((cells & np.uint64(1)) << np.uint64(48)))
    meta = np.concatenate(metas) if metas else np.zeros(0, np.uint64)
    meta = meta[rng.permutation(len(meta))]
    ne = len(meta)
    lo = rng.integers(0, 2**64 - 1, ne, dtype=np.uint64, endpoint=True)
    hi = rng.integers(0, 2**64 - 1, ne, dtype=np.uint64, endpoint=True)
    return Cipher(L, meta, lo, hi)


@pytest.mark.parametrize("all_iblk", [False, True])
def test_iblk_order_and_fallbacks_vs_oracle(oracle, all_iblk):
    """Per-A-edge emit order (k_mul_large.hip iblk_layer / order): chain-step shapes (dense A layers
    x B layers of <= 20 edges, |B.E| up to 63, keys sharing libstdc++ buckets) bit-exact vs the
    oracle, next to the pairs that must fall back to the block marks inside the same batch: a B
    layer of 21+ edges, an A layer with duplicate (idx, ch) cells, an A layer below the dense
    threshold (48 edges), and |B.E| = 64; and small-|B.E| pairs whose keys share buckets. A batch of
    iblk pairs only runs rank / order / write on 1/16 of the workgroups."""
    rng = np.random.default_rng(0x1B1C)
    xs, ys = [], []
    full = [674, 674, 674, 674]
    for k in range(4):   # iblk: saturated and partly filled A layers x fresh-like B
        xs.append(_mk_layers(rng, full if k % 2 == 0 else [500, 674, 300, 650]))
        ys.append(_mk_layers(rng, [20, 20] if k < 2 else [19, 17]))
    xs.append(_mk_layers(rng, [600, 674, 674])); ys.append(_mk_layers(rng, [15, 15, 15]))   # 3 B layers
    xs.append(_mk_layers(rng, [674, 674])); ys.append(_mk_layers(rng, [16, 16, 16, 15]))     # |B.E| = 63
    if not all_iblk:   # with a pair that is not iblk the batch runs the per-slot passes on full grids
        xs.append(_mk_layers(rng, full)); ys.append(_mk_layers(rng, [16, 16, 16, 16]))        # 64: not iblk
    xs.append(_mk_layers(rng, full)); ys.append(_mk_layers(rng, [25, 15]))                    # B layer > 20
    xs.append(_mk_layers(rng, [674, 600, 674], dup_layers=(1,))); ys.append(_mk_layers(rng, [20, 20]))   # duplicates
    xs.append(_mk_layers(rng, [674, 30, 674])); ys.append(_mk_layers(rng, [20, 20]))          # A layer < 48
    xs.append(_mk_layers(rng, [674, 674, 0, 674])); ys.append(_mk_layers(rng, [20, 0, 20]))   # empty layers
    shared = [_max_bucket_edges(oracle, x, y) for x, y in zip(xs, ys)]
    assert all(st for _, st in shared), shared   # static bucket groups everywhere
    # iblk pairs whose keys share libstdc++ buckets (up to 4 keys per bucket): chain-step shapes
    # have none (the multiplicative hash spreads their keys), small |B.E| puts the bucket count near
    # 2 S. `rank` moves edges between A edge counts; `order` probes the flagged ranges
    for a, b in [([674, 674], [1, 1]), ([674] * 4, [2, 1]), ([674, 674], [3, 2]), ([674] * 3, [2, 2, 1]),
                 ([400, 674], [2, 2])]:
        xs.append(_mk_layers(rng, a)); ys.append(_mk_layers(rng, b))
        mx, st = _max_bucket_edges(oracle, xs[-1], ys[-1])
        assert st and mx >= 4, (a, b, mx, st)
    plan = _check_vs_oracle(oracle, {"canon_tag": 0x1B}, xs, ys, 0x1B2)
    assert plan.n_large == len(xs)


def test_iblk_guard_budget_vs_oracle(oracle):
    """iblk pairs above edge_budget take the canonical (layer, idx, P<M) order with hash-order salt
    positions (k_large_order on the reduced grid of an all-iblk batch), next to iblk pairs below it."""
    rng = np.random.default_rng(0x1B3)
    xs = [_mk_layers(rng, [674, 674, 500]) for _ in range(3)] + [_mk_layers(rng, [300, 200])]
    ys = [_mk_layers(rng, [20, 20]) for _ in range(4)]
    _check_vs_oracle(oracle, {"canon_tag": 0x1C, "edge_budget": 30000}, xs, ys, 0x1B4)


def test_engine_chain_depth8_vs_oracle(oracle):
    """BASELINE cfg 4 at its full depth: c_k = c_{k-1} * x for two fresh inputs to depth 8
    (345,088 edges, 6.8 M products per pair at step 8, static bucket groups and 16-time leader
    blocks in use), every step bit-exact vs the oracle on the engine's previous output."""
    from pvac_hfhe_cppbyv_amd import Engine
    eng = Engine(device=0, canon_tag=0xC8)
    n = 2
    X = [Cipher(c.layers, c.meta, c.w_lo, c.w_hi) for c in eng.gen_fresh(n, 0x8000, 20).to_host()]
    cur = X
    for k in range(1, 9):
        out, plan, per = _run_mul(eng, cur, X, seed=200 + k)
        for p in range(n):
            ref = oracle.ct_mul(cur[p], X[p], per[p], canon_tag=0xC8)
            _same(out[p], ref, view=False)
        cur = [Cipher(o.layers, o.meta, o.w_lo, o.w_hi) for o in out]
    assert min(c.nE for c in cur) == 345088


def test_enc_value_chain_depth8_vs_oracle(oracle):
    """cfg 4 with its real producer: x_i = GPU enc_value(v_i) (38-40 edges, compact_edges-merged and
    Fisher-Yates shuffled within each layer, ops/encrypt.hpp:162-291), then c_k = ct_mul(c_{k-1}, x_i)
    to depth 8 with every step's input the engine's own DEVICE output (no host round trip, as in
    bench.py), each step bit-exact vs the oracle (tests/test_main.cpp:289-295 restated)."""
    import torch
    from helpers import fixture_secret
    from pvac_hfhe_cppbyv_amd import Engine
    sk, man, em = fixture_secret()
    eng = Engine(device=0, canon_tag=man["canon_tag"])
    assert eng.gen_H().hex() == man["H_digest"]
    eng.set_secret(read_u64("sk_prf_k.u64"), read_u64("sk_lpn_s.u64"), em["lpn_n"], em["lpn_t"], em["lpn_tau_num"],
                   em["lpn_tau_den"])
    eng.set_powg(read_u64("powg_B.u64"))
    rng = np.random.default_rng(0xC4A1)
    n = 3
    vals = rng.integers(0, 2**64, n, dtype=np.uint64)
    X, st = eng.enc_value(vals, rng.integers(0, 2**64, (n, 256), dtype=np.uint64))
    assert not st.any()
    xh = [Cipher(c.layers, c.meta, c.w_lo, c.w_hi) for c in X.to_host()]
    assert all(38 <= c.nE <= 40 for c in xh)
    cur_d, cur_h = X, xh
    for k in range(1, 9):
        Cb, plan = eng.ct_mul_plan(cur_d, X)
        nonces = torch.empty(2 * max(plan.total_layer_slots, 1), dtype=torch.int64, device=eng.device)
        eng.fill_random(nonces, 0xC4A0 + k)
        out = eng.ct_mul(cur_d, X, nonces=nonces, C_=Cb, plan=plan)
        assert eng.check_mul_gsum(cur_d, X, out, nonces) == 0
        oh = out.to_host()
        nz = nonces.cpu().numpy().view(np.uint64)
        loff = Cb.l_off.cpu().numpy().view(np.uint64)
        for p in range(n):
            base = int(loff[p]) + cur_h[p].nL + xh[p].nL
            per = nz[2 * base:2 * base + 2 * cur_h[p].nL * xh[p].nL]
            ref = oracle.ct_mul(cur_h[p], xh[p], per, canon_tag=man["canon_tag"])
            _same(oh[p], ref, view=False)
        cur_d, cur_h = out, [Cipher(o.layers, o.meta, o.w_lo, o.w_hi) for o in oh]
    assert min(c.nE for c in cur_h) > 300000


def _bucket_census(x, y, nbk, B=337):
    """Per libstdc++ bucket of ct_mul(x, y)'s key slots: (slots of the key space in the bucket, keys
    with products). Returns the largest number of emitting keys among buckets of 4+ slots."""
    G = 0x9E3779B97F4A7C15
    LA, LB = len(x.layers), len(y.layers)
    slots = np.arange(LA * LB * B, dtype=np.uint64)
    keys = ((slots // np.uint64(B)) << np.uint64(32)) | (slots % np.uint64(B))
    bk = (keys * np.uint64(G)) % np.uint64(nbk)   # u64 wrap-around multiply, as size_t
    size = np.bincount(bk.astype(np.int64), minlength=nbk)
    la = (x.meta & np.uint64(0xFFFFFFFF)).astype(np.int64)
    ia = ((x.meta >> np.uint64(32)) & np.uint64(0xFFFF)).astype(np.int64)
    lb = (y.meta & np.uint64(0xFFFFFFFF)).astype(np.int64)
    ib = ((y.meta >> np.uint64(32)) & np.uint64(0xFFFF)).astype(np.int64)
    present = np.unique(((la[:, None] * LB + lb[None, :]) * B + (ia[:, None] + ib[None, :]) % B).ravel())
    pk = np.bincount(bk[present].astype(np.int64), minlength=nbk)
    big = size >= 4
    return int(pk[big].max()) if big.any() else 0


def test_fresh_big_buckets_no_redo_vs_oracle(oracle):
    """Buckets of 4+ key slots (the fresh kernel's member list, k_mul_fresh.hip P4) with several
    emitting keys: every rank comes from unmodified first-insert times, so the fresh kernel emits
    the reference order itself (no pair falls back to the general path) and matches the oracle.
    The default fresh shape (20 edges per layer: 1,613 buckets) has no bucket of more than 3 slots;
    16 x 20 edges per layer (32 x 40 edges) gives 1,280 products, 1,289 buckets and 92 key slots
    in buckets of 4 (all held in the kernel's member list)."""
    import torch
    from pvac_hfhe_cppbyv_amd import Engine
    eng = Engine(device=0, canon_tag=0xB16)
    n = 2048
    A, B = eng.gen_fresh(n, 0xB160, 16), eng.gen_fresh(n, 0xB161, 20)
    Cb, plan = eng.ct_mul_plan(A, B)
    assert plan.n_large == 0
    nonces = torch.empty(2 * plan.total_layer_slots, dtype=torch.int64, device=eng.device)
    eng.fill_random(nonces, 0xB162)
    r0 = eng.ct_mul_redo_count()
    out = eng.ct_mul(A, B, nonces=nonces, C_=Cb, plan=plan).to_host()
    assert eng.ct_mul_redo_count() == r0
    ha, hb = A.to_host(), B.to_host()
    nz = nonces.cpu().numpy().view(np.uint64)
    loff = Cb.l_off.cpu().numpy().view(np.uint64)
    hit = 0
    for p in range(0, n, 16):
        x = Cipher(ha[p].layers, ha[p].meta, ha[p].w_lo, ha[p].w_hi)
        y = Cipher(hb[p].layers, hb[p].meta, hb[p].w_lo, hb[p].w_hi)
        hit += _bucket_census(x, y, oracle.bucket_count(x.nE * y.nE)) >= 2
        base = int(loff[p]) + x.nL + y.nL
        ref = oracle.ct_mul(x, y, nz[2 * base:2 * base + 2 * x.nL * y.nL], canon_tag=0xB16)
        _same(out[p], ref, view=False)
    assert hit >= 8   # the sampled pairs do exercise big buckets with several emitting keys


def test_enc_value_chains_depth8_digests_vs_oracle(oracle):
    """cfg 4's workload on 64 GPU enc_value inputs at once: c_k = ct_mul(c_{k-1}, x) to depth 8 on
    the device, every final chain's edges (per-chain FNV-1a digest over meta and w) and edge count
    equal to the pinned CPU port's chain on the same inputs (orc_ct_mul_chain_timed, 16 threads)."""
    import ctypes as C
    import torch
    from helpers import default_params, fixture_secret, pack_device_batch
    from pvac_hfhe_cppbyv_amd import Engine
    sk, man, em = fixture_secret()
    eng = Engine(device=0, canon_tag=man["canon_tag"])
    assert eng.gen_H().hex() == man["H_digest"]
    eng.set_secret(read_u64("sk_prf_k.u64"), read_u64("sk_lpn_s.u64"), em["lpn_n"], em["lpn_t"], em["lpn_tau_num"],
                   em["lpn_tau_den"])
    eng.set_powg(read_u64("powg_B.u64"))
    rng = np.random.default_rng(0xC4A2)
    n, depth = 64, 8
    X, st = eng.enc_value(rng.integers(0, 2**64, n, dtype=np.uint64), rng.integers(0, 2**64, (n, 256), dtype=np.uint64))
    assert not st.any()
    cur = X
    for k in range(depth):
        Cb, plan = eng.ct_mul_plan(cur, X)
        nonces = torch.empty(2 * max(plan.total_layer_slots, 1), dtype=torch.int64, device=eng.device)
        eng.fill_random(nonces, 0xC4B0 + k)
        cur = eng.ct_mul(cur, X, nonces=nonces, C_=Cb, plan=plan)
    gdig = eng.digest(cur).cpu().numpy().view(np.uint64)
    gcnt = cur.e_cnt[:n].cpu().numpy().view(np.uint64)
    P_ = lambda a: a.ctypes.data_as(C.c_void_p)
    px = pack_device_batch(X, n)
    cnt, dig, se = np.zeros(n, np.uint64), np.zeros(n, np.uint64), np.zeros(depth, np.uint64)
    oracle.lib.orc_ct_mul_chain_timed(C.byref(default_params(man["canon_tag"])), n, *(P_(a) for a in px), depth, 16,
                                      P_(cnt), P_(dig), P_(se))
    assert np.array_equal(cnt, gcnt)
    assert np.array_equal(dig, gdig)
    assert int(se[-1]) == int(gcnt.sum()) and gcnt.min() > 300000


def test_direct_cancelling_key_redo_vs_oracle(oracle):
    """Chain-step pairs take the direct mode (large_desc::direct: emit positions counted from key
    presence, C's records written from the products' epilogue). A P cell whose products cancel
    (sum 0 mod p, arithmetic.hpp:96-101 drops its edge) breaks the presence assumption: the pair
    must be handed to the redo on the exact path and come out bit-exact. Here one A weight is
    solved so that the P sum of key (0, 0, r) is 0; the other pairs of the batch stay direct."""
    from pvac_hfhe_cppbyv_amd import Engine
    B = 337
    rng = np.random.default_rng(0xCA2C)
    xs = [_mk_layers(rng, [674] * 4) for _ in range(4)]   # 4 A layers: no two key slots share a bucket
    ys = [_mk_layers(rng, [20, 20]) for _ in range(4)]
    x, y = xs[1], ys[1]
    lid = lambda m: int(m & 0xFFFFFFFF)
    idx = lambda m: int((m >> 32) & 0xFFFF)
    ch = lambda m: int((m >> 48) & 0xFF)
    w = lambda c, k: (int(c.w_lo[k]) | (int(c.w_hi[k]) << 64)) % ((1 << 127) - 1)
    P_ = (1 << 127) - 1
    r = 5
    a_at = {(idx(m), ch(m)): k for k, m in enumerate(x.meta) if lid(m) == 0}
    terms = []   # (A edge, B edge) of every product in key (0, 0, r)'s P cell
    for j, m in enumerate(y.meta):
        if lid(m) == 0:
            terms.append((a_at[((r - idx(m)) % B, ch(m))], j))
    assert len(terms) == 20
    (k0, j0), rest = terms[0], terms[1:]
    s = sum(w(x, k) * w(y, j) for k, j in rest) % P_
    v = (-s * pow(w(y, j0), P_ - 2, P_)) % P_
    x.w_lo[k0], x.w_hi[k0] = np.uint64(v & ((1 << 64) - 1)), np.uint64(v >> 64)
    assert (sum(w(x, k) * w(y, j) for k, j in terms)) % P_ == 0
    eng = Engine(device=0, canon_tag=0xCA2D)
    r0 = eng.ct_mul_redo_count()
    out, plan, per = _run_mul(eng, xs, ys, seed=0xCA2E)
    assert plan.n_large == 4
    assert eng.ct_mul_redo_count() - r0 == 1   # only the cancelling pair left the direct mode
    for p in range(4):
        ref = oracle.ct_mul(xs[p], ys[p], per[p], canon_tag=0xCA2D)
        _same(out[p], ref, view=False)
    assert out[0].nE == 8 * 337 * 2 and out[1].nE == 8 * 337 * 2 - 1   # saturated: every cell emits but one


@pytest.mark.parametrize("Bm", [97, 337, 1024])
def test_direct_mode_shapes_vs_oracle(oracle, Bm):
    """The direct mode (k_large_count_la / scan_direct / products_direct) across B: saturated and
    partly filled dense A layers (48 .. 2B distinct cells) times 1-4 B layers of <= 20 edges, 4 or 8
    A layers. B = 1024 puts 2 B = 2,048 dense cells on a 256-thread workgroup, past the cells
    count_la holds in registers (kPendCells x 256), so its direct-store path runs too. Every pair
    bit-exact vs the oracle; the path counters show the direct mode ran and nothing was redone.
    Then the same shapes with an edge_budget below their output: scan_direct hands each pair to the
    redo (canonical order), again bit-exact."""
    from pvac_hfhe_cppbyv_amd import Engine
    rng = np.random.default_rng(0xD1 + Bm)
    xs, ys = [], []
    for k in range(6):
        nla = 4 if k % 2 == 0 else 8
        counts = [2 * Bm if (k + l) % 3 else int(rng.integers(48, 2 * Bm)) for l in range(nla)]
        xs.append(_mk_layers(rng, counts, B=Bm))
        ys.append(_mk_layers(rng, [20, 20, 13, 7][: 1 + k % 4], B=Bm))
    eng = Engine(device=0, B=Bm, canon_tag=0xD2)
    p0, r0 = eng.ct_mul_path_counts(), eng.ct_mul_redo_count()
    out, plan, per = _run_mul(eng, xs, ys, seed=0xD3)
    p1 = eng.ct_mul_path_counts()
    assert plan.n_large == len(xs)
    nd = p1["direct"] - p0["direct"]   # pairs whose key slots share no libstdc++ bucket
    assert nd >= 2 and eng.ct_mul_redo_count() == r0
    for p in range(len(xs)):
        _same(out[p], oracle.ct_mul(xs[p], ys[p], per[p], canon_tag=0xD2, Bm=Bm), view=False)
    budget = min(o.nE for o in out) - 1
    eng2 = Engine(device=0, B=Bm, canon_tag=0xD2, edge_budget=budget)
    out2, plan2, per2 = _run_mul(eng2, xs, ys, seed=0xD3)
    pc = eng2.ct_mul_path_counts()
    assert pc["direct"] == nd and eng2.ct_mul_redo_count() == nd   # every direct pair is over budget
    for p in range(len(xs)):
        _same(out2[p], oracle.ct_mul(xs[p], ys[p], per2[p], canon_tag=0xD2, Bm=Bm, edge_budget=budget), view=False)


def test_direct_pairs_canonical_flag_no_redo(oracle):
    """PVAC_MUL_ORDER_CANONICAL on a batch of direct-eligible chain-step pairs: exec
    rebuilds their descriptors for the exact path before launching, so no pair runs the direct
    kernels only to be redone. Output is the canonical (layer, idx, P<M) order, which the oracle
    produces for any pair over edge_budget (here 0: every pair), bit-exact; the path counters show
    no direct pair and the redo count stays put. The same engine then runs the same batch without
    the flag, and the direct mode comes back (the plan's descriptors are rebuilt per exec)."""
    from pvac_hfhe_cppbyv_amd import Engine, MUL_ORDER_CANONICAL
    rng = np.random.default_rng(0xCA70)
    xs = [_mk_layers(rng, [674] * 4) for _ in range(3)]
    ys = [_mk_layers(rng, [20, 20]) for _ in range(3)]
    eng = Engine(device=0, canon_tag=0xCA71)
    p0, r0 = eng.ct_mul_path_counts(), eng.ct_mul_redo_count()
    out, plan, per = _run_mul(eng, xs, ys, seed=0xCA72, flags=MUL_ORDER_CANONICAL)
    p1 = eng.ct_mul_path_counts()
    assert plan.n_large == 3
    assert p1["direct"] == p0["direct"] and eng.ct_mul_redo_count() == r0
    for p in range(3):
        _same(out[p], oracle.ct_mul(xs[p], ys[p], per[p], canon_tag=0xCA71, edge_budget=0), view=False)
    out2, _, per2 = _run_mul(eng, xs, ys, seed=0xCA72)
    assert eng.ct_mul_path_counts()["direct"] - p1["direct"] == 3 and eng.ct_mul_redo_count() == r0
    for p in range(3):
        _same(out2[p], oracle.ct_mul(xs[p], ys[p], per2[p], canon_tag=0xCA71), view=False)
