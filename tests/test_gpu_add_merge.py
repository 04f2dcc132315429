"""GPU parity of ct_add / ct_sub above edge_budget (k_add_merge.hip): guard_budget ->
compact_edges -> compact_layers (reference ops/arithmetic.hpp:12-31, ops/encrypt.hpp:39-111).
Pinned to the reference's own guard fixture (guard_x + guard_y at edge_budget 16, sigmas
included) and to the CPU oracle on synthetic batches that mix pairs under and over the budget,
duplicate keys, exact cancellations (A - A), doubled edges (A + A) and non-canonical weights
(fp_add's truncation quirk makes the merge order-dependent)."""
import os

import numpy as np
import pytest

from helpers import REF, Cipher, LAYER_DT, read_ct

pytestmark = pytest.mark.gpu


def _dev_batch(engine, ciphers, sigma=False):
    from pvac_hfhe_cppbyv_amd import DeviceBatch, HostCipher
    hc = [HostCipher(c.layers, c.meta, c.w_lo, c.w_hi, c.sigma) for c in ciphers]
    return DeviceBatch.from_host(hc, engine.device, sigma=sigma)


def _layers_view(L):
    L = L.copy()
    prod = L["rule"] == 1
    for f in ("ztag", "nonce_lo", "nonce_hi"):
        L[f][prod] = 0
    L["pa"][~prod] = 0
    L["pb"][~prod] = 0
    return L


def _same(got, ref, sigma=False, view=False):
    L = _layers_view(got.layers) if view else got.layers
    for f in ("rule", "pa", "pb", "ztag", "nonce_lo", "nonce_hi"):
        assert np.array_equal(L[f], ref.layers[f]), f
    assert got.nE == ref.nE
    assert np.array_equal(got.meta, ref.meta)
    assert np.array_equal(got.w_lo, ref.w_lo) and np.array_equal(got.w_hi, ref.w_hi)
    if sigma:
        assert np.array_equal(got.sigma, ref.sigma)


def _mk(rng, nl, ne, B=337, idx_range=None, sigma=False, noncanon=0.0):
    L = np.zeros(nl, LAYER_DT)
    L["ztag"] = rng.integers(0, 2**63, nl, dtype=np.uint64)
    L["nonce_lo"] = rng.integers(0, 2**63, nl, dtype=np.uint64)
    if nl == 0:
        ne = 0
    lay = rng.integers(0, max(nl, 1), ne).astype(np.uint64)
    idx = rng.integers(0, idx_range or B, ne).astype(np.uint64)
    ch = rng.integers(0, 2, ne).astype(np.uint64)
    meta = lay | (idx << np.uint64(32)) | (ch << np.uint64(48))
    lo = rng.integers(0, 2**63, ne, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, ne, dtype=np.uint64)
    hi = rng.integers(0, 2**63 - 1, ne, dtype=np.uint64)
    bad = rng.random(ne) < noncanon   # hi >= 2^63: non-canonical inputs (fp_add truncation quirk)
    hi[bad] |= np.uint64(1 << 63)
    sig = rng.integers(0, 2**63, (ne, 128), dtype=np.uint64) if sigma else None
    return Cipher(L, meta, lo, hi, sig)


def test_guard_fixture_gpu():
    """The reference's own guard_budget case: ct_add(guard_x, guard_y) at edge_budget 16."""
    from pvac_hfhe_cppbyv_amd import Engine
    x = read_ct(os.path.join(REF, "guard_x.ct"))[0]
    y = read_ct(os.path.join(REF, "guard_y.ct"))[0]
    ref = read_ct(os.path.join(REF, "guard_add.ct"))[0]
    eng = Engine(device=0, edge_budget=16)
    out = eng.ct_add(_dev_batch(eng, [x], True), _dev_batch(eng, [y], True), sigma=True).to_host()[0]
    _same(out, ref, sigma=True, view=True)


@pytest.mark.parametrize("negate", [False, True])
@pytest.mark.parametrize("sigma", [False, True])
def test_merge_vs_oracle(oracle, negate, sigma):
    from pvac_hfhe_cppbyv_amd import Engine
    budget = 120
    rng = np.random.default_rng(31 + 2 * negate + sigma)
    xs, ys = [], []
    for k in range(14):
        nl_a, nl_b = 1 + k % 4, 1 + (k * 3) % 5
        kind = k % 7
        if kind == 0:     # under budget: plain concatenation in the same batch
            x, y = _mk(rng, nl_a, 40, sigma=sigma), _mk(rng, nl_b, 40, sigma=sigma)
        elif kind == 1:   # A op A: cancellations (sub) / doubling (add)
            x = _mk(rng, nl_a, 150, idx_range=40, sigma=sigma)
            y = x
        elif kind == 2:   # heavy duplicates in a narrow idx range
            x, y = _mk(rng, nl_a, 300, idx_range=8, sigma=sigma), _mk(rng, nl_b, 200, idx_range=8, sigma=sigma)
        elif kind == 3:   # non-canonical weights in the merged groups
            x = _mk(rng, nl_a, 260, idx_range=20, sigma=sigma, noncanon=0.5)
            y = _mk(rng, nl_b, 90, idx_range=20, sigma=sigma, noncanon=0.5)
        elif kind == 4:   # one side empty
            x, y = _mk(rng, nl_a, 0, sigma=sigma), _mk(rng, nl_b, 200, sigma=sigma)
        elif kind == 5:   # PROD layers referencing BASE layers (compact_layers closure after the merge)
            x, y = _mk(rng, 4, 180, idx_range=30, sigma=sigma), _mk(rng, 3, 100, idx_range=30, sigma=sigma)
            for c in (x, y):
                c.layers["rule"][-1] = 1
                c.layers["pa"][-1] = 0
                c.layers["pb"][-1] = 1
        else:             # sparse, mostly distinct keys
            x, y = _mk(rng, nl_a, 400, sigma=sigma), _mk(rng, nl_b, 300, sigma=sigma)
        xs.append(x)
        ys.append(y)
    eng = Engine(device=0, edge_budget=budget)
    A, B = _dev_batch(eng, xs, sigma), _dev_batch(eng, ys, sigma)
    out = eng.ct_add(A, B, negate=negate, sigma=sigma).to_host()
    n_over = 0
    for p, (x, y) in enumerate(zip(xs, ys)):
        n_over += x.nE + y.nE > budget
        ref = oracle.ct_add(x, y, negate=negate, edge_budget=budget)
        _same(out[p], ref, sigma=sigma)
    assert n_over >= 10


def test_exact_cancellations_drop_groups_and_layers(oracle):
    """A holds every edge twice with weights w and p - w (same key, same sigma): each group sums
    to 0 with a zero sigma XOR and is dropped, and A's layers become unused (compact_layers);
    only B's edges and layer survive."""
    from pvac_hfhe_cppbyv_amd import Engine
    rng = np.random.default_rng(44)
    half = _mk(rng, 3, 150, sigma=True)
    p_lo, p_hi = np.uint64(2**64 - 1), np.uint64(2**63 - 1)
    keep = (half.w_lo != 0) | (half.w_hi != 0)
    half = Cipher(half.layers, half.meta[keep], half.w_lo[keep], half.w_hi[keep], half.sigma[keep])
    neg_lo = p_lo - half.w_lo                       # p - w for canonical w != 0 (no borrow: p_lo is all ones)
    neg_hi = p_hi - half.w_hi
    x = Cipher(half.layers, np.concatenate([half.meta, half.meta]), np.concatenate([half.w_lo, neg_lo]),
               np.concatenate([half.w_hi, neg_hi]), np.concatenate([half.sigma, half.sigma]))
    y = _mk(rng, 1, 10, sigma=True)
    y = Cipher(y.layers, (np.arange(10, dtype=np.uint64) << np.uint64(32)), y.w_lo, y.w_hi, y.sigma)
    eng = Engine(device=0, edge_budget=100)
    out = eng.ct_add(_dev_batch(eng, [x], True), _dev_batch(eng, [y], True), sigma=True).to_host()[0]
    assert out.nE == 10 and out.nL == 1
    _same(out, oracle.ct_add(x, y, edge_budget=100), sigma=True)


def test_codec_interop_gpu():
    """File -> native codec -> device -> ct_add / ct_sub -> native codec -> file, byte-identical
    to the reference's own outputs (pair fixtures batched through one multi-cipher image, and
    bounty2 a.ct + b.ct -> sum.ct)."""
    from pvac_hfhe_cppbyv_amd import Engine, codec
    from helpers import GOLD
    eng = Engine(device=0)
    xs = [codec.read_ct(os.path.join(REF, f"pair{p}_x.ct"))[0] for p in range(8)]
    ys = [codec.read_ct(os.path.join(REF, f"pair{p}_y.ct"))[0] for p in range(8)]
    A = codec.load_ct(codec.write_ct(xs), eng.device)
    B = codec.load_ct(codec.write_ct(ys), eng.device)
    for op, neg in (("add", False), ("sub", True)):
        out = eng.ct_add(A, B, negate=neg, sigma=True)
        for p, c in enumerate(out.to_host()):
            with open(os.path.join(REF, f"pair{p}_{op}.ct"), "rb") as f:
                assert codec.write_ct([c]) == f.read(), (op, p)
    a = codec.load_ct(os.path.join(GOLD, "bounty", "a.ct"), eng.device)
    b = codec.load_ct(os.path.join(GOLD, "bounty", "b.ct"), eng.device)
    s = eng.ct_add(a, b, sigma=True)
    with open(os.path.join(GOLD, "bounty", "sum.ct"), "rb") as f:
        assert codec.write_ct(s.to_host()) == f.read()


@pytest.mark.parametrize("nl_total", [6, 30, 40, 62, 90])
@pytest.mark.parametrize("negate", [False, True])
def test_add_layer_widths_vs_oracle(oracle, nl_total, negate):
    """ct_add / ct_sub below edge_budget for every kernel width: 32-lane groups (<= 32 layers),
    64-lane groups (<= 64) and the workgroup kernel (> 64). PROD layers with parents, layers no edge
    references (compact_layers drops them unless a kept PROD layer needs them), batch tails that
    leave half-empty lane groups, sigma carried."""
    from pvac_hfhe_cppbyv_amd import Engine
    rng = np.random.default_rng(nl_total * 7 + negate)
    xs, ys = [], []
    for k in range(13):   # odd count: the last 32-lane group of the last wave has no pair
        la = max(1, nl_total // 2 - k % 3)
        lb = max(1, nl_total - la)
        x, y = _mk(rng, la, 30 + k, sigma=True), _mk(rng, lb, 25, sigma=True)
        for c in (x, y):
            n = len(c.layers)
            # edges only on even layers; odd layers >= 2 are PROD of two earlier layers
            c.meta = (c.meta & ~np.uint64(0xFFFFFFFF)) | ((c.meta & np.uint64(0xFFFFFFFF)) & ~np.uint64(1))
            for l in range(3, n, 4):
                c.layers["rule"][l] = 1
                c.layers["pa"][l] = l - 1
                c.layers["pb"][l] = l - 3
        xs.append(x)
        ys.append(y)
    eng = Engine(device=0)
    A, B = _dev_batch(eng, xs, True), _dev_batch(eng, ys, True)
    out = eng.ct_add(A, B, negate=negate, sigma=True).to_host()
    for p, (x, y) in enumerate(zip(xs, ys)):
        ref = oracle.ct_add(x, y, negate=negate)
        _same(out[p], ref, sigma=True)
