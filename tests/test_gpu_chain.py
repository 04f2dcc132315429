"""pvac_hip_ct_mul_chain (include/pvac_hip.h): the reference's chain workload c_k = ct_mul(c_{k-1}, x)
(tests/test_main.cpp:289-295) over a batch of inputs, run by the library on internal worker streams.
Every chain's final c_depth must equal the same chain driven step by step through ct_mul_plan /
ct_mul_exec on one stream, and the pinned CPU port's chain (orc_ct_mul_chain_timed)."""
import ctypes as C

import numpy as np
import pytest

from helpers import Cipher, default_params, fixture_secret, pack_device_batch, read_u64

pytestmark = pytest.mark.gpu


def _stepwise(eng, X, depth, seed, chunk):
    """The same chains step by step on the caller's stream, chunk by chunk with the library's nonce
    seeds (nonce_seed + 97 * first_input + step): final digests, counts and per-step edge sums."""
    import torch
    from pvac_hfhe_cppbyv_amd import DeviceBatch
    dig, cnt, edges = [], [], [0] * depth
    for c0 in range(0, X.n, chunk):
        k = min(chunk, X.n - c0)
        Xv = DeviceBatch(k, X.l_off[c0:c0 + k], X.l_cnt[c0:c0 + k], X.layers, X.e_off[c0:c0 + k],
                         X.e_cnt[c0:c0 + k], X.meta, X.w_lo, X.w_hi)
        cur = Xv
        for d in range(depth):
            Cb, plan = eng.ct_mul_plan(cur, Xv)
            nonces = torch.empty(2 * max(plan.total_layer_slots, 1), dtype=torch.int64, device=eng.device)
            eng.fill_random(nonces, seed + 97 * c0 + d)
            cur = eng.ct_mul(cur, Xv, nonces=nonces, C_=Cb, plan=plan)
            edges[d] += int(cur.e_cnt[:k].sum().item())
        dig.append(eng.digest(cur).cpu().numpy().view(np.uint64).copy())
        cnt.append(cur.e_cnt[:k].cpu().numpy().view(np.uint64).copy())
    return np.concatenate(dig), np.concatenate(cnt), edges


def test_chain_api_equals_stepwise_and_oracle(oracle):
    """enc_value inputs (the cfg-4 producer), depth 5, 3 worker streams over chunks of 7 (a ragged
    last chunk): digests and edge counts of every chain equal the step-by-step engine run and the
    CPU port; the gsum invariant holds on every pair-step; the statistics add up."""
    from pvac_hfhe_cppbyv_amd import Engine
    sk, man, em = fixture_secret()
    eng = Engine(device=0, canon_tag=man["canon_tag"])
    assert eng.gen_H().hex() == man["H_digest"]
    eng.set_secret(read_u64("sk_prf_k.u64"), read_u64("sk_lpn_s.u64"), em["lpn_n"], em["lpn_t"], em["lpn_tau_num"],
                   em["lpn_tau_den"])
    eng.set_powg(read_u64("powg_B.u64"))
    rng = np.random.default_rng(0xC4A5)
    n, depth, chunk, seed = 40, 5, 7, 0x7E57
    X, st = eng.enc_value(rng.integers(0, 2**64, n, dtype=np.uint64), rng.integers(0, 2**64, (n, 256), dtype=np.uint64))
    assert not st.any()
    r = eng.ct_mul_chain(X, depth, nonce_seed=seed, streams=3, chunk=chunk, check_gsum=True, digest_n=n)
    assert r["chunks"] == (n + chunk - 1) // chunk and r["pair_steps"] == n * depth
    assert r["gsum_pairs"] == n * depth and r["gsum_failed"] == 0 and r["redo"] == 0
    dig, cnt, edges = _stepwise(eng, X, depth, seed, chunk)
    assert np.array_equal(r["digests"], dig) and np.array_equal(r["counts"], cnt)
    assert r["edges"] == edges and r["edges"][-1] == int(cnt.sum())
    xe = X.e_cnt[:n].cpu().numpy().astype(np.int64)
    assert r["products"][0] == int((xe * xe).sum())
    # the CPU port's chains on the same inputs
    px = pack_device_batch(X, n)
    P_ = lambda a: a.ctypes.data_as(C.c_void_p)
    ocnt, odig, se = np.zeros(n, np.uint64), np.zeros(n, np.uint64), np.zeros(depth, np.uint64)
    oracle.lib.orc_ct_mul_chain_timed(C.byref(default_params(man["canon_tag"])), n, *(P_(a) for a in px), depth, 8,
                                      P_(ocnt), P_(odig), P_(se))
    assert np.array_equal(ocnt, cnt) and np.array_equal(odig, dig)
    # a second call reuses the worker contexts and buffers: same result
    r2 = eng.ct_mul_chain(X, depth, nonce_seed=seed, streams=3, chunk=chunk, digest_n=n)
    assert np.array_equal(r2["digests"], dig) and r2["gsum_pairs"] == 0


def test_chain_depth8_vs_oracle(oracle):
    """cfg 4's full depth on a few chains: steps 3-8 run the direct mode, and from step 7 on the A
    operand holds more edges than k_large_lists keeps in registers (its later rounds re-read the
    metas) and spans many 32-edge count groups; final digests and counts equal the CPU port's."""
    from pvac_hfhe_cppbyv_amd import Engine
    sk, man, em = fixture_secret()
    eng = Engine(device=0, canon_tag=man["canon_tag"])
    assert eng.gen_H().hex() == man["H_digest"]
    eng.set_secret(read_u64("sk_prf_k.u64"), read_u64("sk_lpn_s.u64"), em["lpn_n"], em["lpn_t"], em["lpn_tau_num"],
                   em["lpn_tau_den"])
    eng.set_powg(read_u64("powg_B.u64"))
    rng = np.random.default_rng(0xD8)
    n, depth = 3, 8
    X, st = eng.enc_value(rng.integers(0, 2**64, n, dtype=np.uint64), rng.integers(0, 2**64, (n, 256), dtype=np.uint64))
    assert not st.any()
    r = eng.ct_mul_chain(X, depth, nonce_seed=0xD8, streams=2, chunk=2, check_gsum=True, digest_n=n)
    assert r["gsum_pairs"] == n * depth and r["gsum_failed"] == 0 and r["redo"] == 0
    assert r["edges"][5] > n * 4 * 8192   # step 7's A operands: > 32 K edges each
    px = pack_device_batch(X, n)
    P_ = lambda a: a.ctypes.data_as(C.c_void_p)
    ocnt, odig, se = np.zeros(n, np.uint64), np.zeros(n, np.uint64), np.zeros(depth, np.uint64)
    oracle.lib.orc_ct_mul_chain_timed(C.byref(default_params(man["canon_tag"])), n, *(P_(a) for a in px), depth, 8,
                                      P_(ocnt), P_(odig), P_(se))
    assert np.array_equal(ocnt, r["counts"]) and np.array_equal(odig, r["digests"])


def test_chain_api_callbacks_and_errors():
    """fill_nonces / on_chunk callbacks from the worker threads: every chunk arrives once with its
    first input and size, the nonces come from the callback (different nonces, same edges: a digest
    covers (meta, w) only, and layer ztags change), and a failing callback stops the chain with
    PVAC_EINVAL. Bad options are refused."""
    import threading
    import torch
    from pvac_hfhe_cppbyv_amd import FILL_NONCES_CB, ON_CHUNK_CB, Engine, PvacError
    eng = Engine(device=0, canon_tag=0xCA11)
    n, depth, chunk = 24, 3, 5
    X = eng.gen_fresh(n, 0xCA12, 20)
    base = eng.ct_mul_chain(X, depth, streams=2, chunk=chunk, digest_n=n)
    lock = threading.Lock()
    seen, fills = [], []
    fill_lib = eng.lib

    def fill(user, step, first, nwords, dev, stream):
        # splitmix words through a context of this thread's own (one thread per context)
        with lock:
            fills.append((step, first, nwords))
        return 0 if fill_lib.pvac_hip_fill_random(ctxs[threading.get_ident()], 0xF111 + step, dev, nwords) == 0 else 1

    def chunk_cb(user, first, cb, stream):
        b = cb.contents
        with lock:
            seen.append((first, b.n))
        return 0

    # per-thread helper contexts for the fill callback (created lazily on the worker threads)
    ctxs = {}
    from pvac_hfhe_cppbyv_amd import Params

    def fill_wrap(user, step, first, nwords, dev, stream):
        tid = threading.get_ident()
        if tid not in ctxs:
            c = C.c_void_p()
            prm = Params(B=337, m_bits=8192, n_bits=16384, h_col_wt=192, x_col_wt=128, err_wt=128,
                         edge_budget=1200000, canon_tag=0xCA11)
            assert eng.lib.pvac_hip_ctx_create(0, C.byref(prm), C.byref(c)) == 0
            assert eng.lib.pvac_hip_ctx_set_stream(c, C.c_void_p(stream)) == 0
            ctxs[tid] = c
        return fill(user, step, first, nwords, dev, stream)

    fcb, ccb = FILL_NONCES_CB(fill_wrap), ON_CHUNK_CB(chunk_cb)
    r = eng.ct_mul_chain(X, depth, streams=2, chunk=chunk, digest_n=n, fill_nonces=fcb, on_chunk=ccb)
    for c in ctxs.values():
        eng.lib.pvac_hip_ctx_destroy(c)
    assert sorted(seen) == [(c0, min(chunk, n - c0)) for c0 in range(0, n, chunk)]
    assert len(fills) == depth * len(seen) and all(w >= 2 for _, _, w in fills)
    assert np.array_equal(r["digests"], base["digests"])

    def bad_chunk(user, first, cb, stream):
        return 1

    with pytest.raises(PvacError):
        eng.ct_mul_chain(X, depth, streams=2, chunk=chunk, on_chunk=ON_CHUNK_CB(bad_chunk))
    with pytest.raises(PvacError):
        eng.ct_mul_chain(X, 0)
    with pytest.raises(PvacError):   # no powg on this context
        eng.ct_mul_chain(X, 2, check_gsum=True)
    # the context is still usable after the errors
    r3 = eng.ct_mul_chain(X, depth, streams=2, chunk=chunk, digest_n=n)
    assert np.array_equal(r3["digests"], base["digests"])
    torch.cuda.synchronize()


def test_reference_chain_2_pow_10_on_gpu(oracle):
    """The reference's own end-to-end chain check, as its loop is written (tests/test_main.cpp:289-293:
    chain = enc_value(2), then nine times chain = ct_mul(chain, enc_value(2)), dec_value == 2^10), all
    on the GPU through the chain entry point: x and a FRESH enc_value(2) operand per step (GPU PRF, ten
    independent encryptions per chain) passed as per-step operands (pvac_chain_opts.operands), nine
    steps through pvac_hip_ct_mul_chain with its dense-image intermediate steps (step 9's A operands hold
    ~345 K edges, its outputs ~690 K), the final ciphers taken from the on_chunk callback, then base_R
    (prf_R of the BASE layers) and dec_value: every chain decrypts to 2^10. The depth-9 digests and edge
    counts equal the CPU port's chains over the same operands (orc_ct_mul_chain_ops_timed)."""
    import threading
    from pvac_hfhe_cppbyv_amd import ON_CHUNK_CB, DeviceBatch, Engine, HostCipher
    from helpers import hip_batch_to_host
    sk, man, em = fixture_secret()
    eng = Engine(device=0, canon_tag=man["canon_tag"])
    assert eng.gen_H().hex() == man["H_digest"]
    eng.set_secret(read_u64("sk_prf_k.u64"), read_u64("sk_lpn_s.u64"), em["lpn_n"], em["lpn_t"], em["lpn_tau_num"],
                   em["lpn_tau_den"])
    eng.set_powg(read_u64("powg_B.u64"))
    rng = np.random.default_rng(0x2A10)
    n, depth = 4, 9
    X, st = eng.enc_value(np.full(n, 2, np.uint64), rng.integers(0, 2**64, (n, 256), dtype=np.uint64))
    assert not st.any()
    ops = []
    for _ in range(depth):
        Y, st = eng.enc_value(np.full(n, 2, np.uint64), rng.integers(0, 2**64, (n, 256), dtype=np.uint64))
        assert not st.any()
        ops.append(Y)
    lock = threading.Lock()
    finals = {}

    def keep(user, first, cb, stream):
        cs = hip_batch_to_host(cb.contents, stream)
        with lock:
            for i, c in enumerate(cs):
                finals[first + i] = c
        return 0

    r = eng.ct_mul_chain(X, depth, nonce_seed=0x2A11, streams=2, chunk=2, digest_n=n, operands=ops,
                         on_chunk=ON_CHUNK_CB(keep))
    assert r["image_steps"] > 0 and r["redo"] == 0   # the image fast path holds with fresh operands
    # the reference's gsum invariant on every pair-step, depth 9 included (step 9's layer tables exceed
    # a workgroup's LDS: k_check_gsum runs over global slabs), records throughout: the same chains
    chk = eng.ct_mul_chain(X, depth, nonce_seed=0x2A11, streams=2, chunk=2, digest_n=n, operands=ops,
                           check_gsum=True)
    assert chk["gsum_pairs"] == n * depth and chk["gsum_failed"] == 0 and chk["image_steps"] == 0
    assert np.array_equal(chk["digests"], r["digests"]) and np.array_equal(chk["counts"], r["counts"])
    assert sorted(finals) == list(range(n))
    assert min(c.nE for c in finals.values()) > 600000   # step 9 on the GPU: ~690 K-edge ciphers
    cs = [finals[i] for i in range(n)]
    F = DeviceBatch.from_host([HostCipher(c.layers, c.meta, c.w_lo, c.w_hi, None) for c in cs], eng.device)
    vals, dst = eng.dec_value(F, eng.base_R(F))
    assert not dst.any()
    assert vals == [1 << 10] * n
    px = pack_device_batch(X, n)
    po = [pack_device_batch(Y, n) for Y in ops]
    cat = lambda k: np.ascontiguousarray(np.concatenate([p[k] for p in po]))
    eoff = lambda k: np.ascontiguousarray(np.concatenate([[0]] + [p[k][1:] + sum(int(q[k][-1]) for q in po[:j])
                                                                  for j, p in enumerate(po)]).astype(np.uint64))
    oops = (eoff(0), cat(1), eoff(2), cat(3), cat(4), cat(5))
    P_ = lambda a: a.ctypes.data_as(C.c_void_p)
    ocnt, odig, se = np.zeros(n, np.uint64), np.zeros(n, np.uint64), np.zeros(depth, np.uint64)
    oracle.lib.orc_ct_mul_chain_ops_timed(C.byref(default_params(man["canon_tag"])), n, *(P_(a) for a in px), depth,
                                          depth, *(P_(a) for a in oops), 8, P_(ocnt), P_(odig), P_(se))
    assert np.array_equal(ocnt, r["counts"]) and np.array_equal(odig, r["digests"])
    assert np.array_equal(ocnt, np.array([c.nE for c in cs], np.uint64))
    assert [int(v) for v in se] == r["edges"]


def test_chain_two_device_ranges_equal_one_device():
    """The in-library multi-device path on one GPU: devices = [0, 0] splits the inputs into two ranges
    of whole chunks, each run by its own worker contexts; with PVAC_CHAIN_STAGE_INPUTS the second
    range copies every chunk into worker-local buffers first (the path a worker on another GPU
    takes, there with peer reads). Digests, counts, per-step statistics and chunk count equal the
    one-device call; the partition is pvac_hip_chain_partition's."""
    import ctypes
    from pvac_hfhe_cppbyv_amd import Engine
    eng = Engine(device=0, canon_tag=0xD0D0)
    n, depth, chunk = 37, 4, 5
    X = eng.gen_fresh(n, 0xD0D1, 20)
    one = eng.ct_mul_chain(X, depth, streams=2, chunk=chunk, digest_n=n, nonce_seed=0xD0D2, sumdigest=True)
    two = eng.ct_mul_chain(X, depth, streams=2, chunk=chunk, digest_n=n, nonce_seed=0xD0D2, devices=[0, 0],
                           stage_inputs=True, sumdigest=23)
    assert np.array_equal(one["digests"], two["digests"]) and np.array_equal(one["counts"], two["counts"])
    assert len(one["sumdigests"]) == n and np.array_equal(one["sumdigests"][:23], two["sumdigests"])
    assert one["edges"] == two["edges"] and one["products"] == two["products"]
    assert two["chunks"] == one["chunks"] == (n + chunk - 1) // chunk
    three = eng.ct_mul_chain(X, depth, streams=1, chunk=chunk, digest_n=n, nonce_seed=0xD0D2, devices=[0, 0, 0])
    assert np.array_equal(one["digests"], three["digests"])
    f = (ctypes.c_uint64 * 4)()
    assert eng.lib.pvac_hip_chain_partition(n, chunk, 3, f) == 0
    assert list(f) == [0, 10, 25, 37]   # 8 chunks dealt 2 / 3 / 3


def test_chain_layout_changes_release_worker_memory():
    """Calls with different (streams, chunk) layouts on one context: a layout change returns the
    workers' grown output buffers and scratch arenas before the new HBM shares are taken (without it
    a larger-chunk call followed by more streams ran out of memory on the 2^16-input bench shape).
    Every layout gives the same digests and counts; the device's free memory after a small-chunk call
    is not below what it was after the large-chunk call."""
    import torch
    from pvac_hfhe_cppbyv_amd import Engine
    eng = Engine(device=0, canon_tag=0xD0D5)
    n, depth = 41, 4
    X = eng.gen_fresh(n, 0xD0D6, 20)
    base = eng.ct_mul_chain(X, depth, streams=2, chunk=5, digest_n=n, nonce_seed=0xD0D7)
    big = eng.ct_mul_chain(X, depth, streams=1, chunk=41, digest_n=n, nonce_seed=0xD0D7)
    torch.cuda.synchronize()
    free_big = torch.cuda.mem_get_info()[0]
    for streams, chunk in ((3, 2), (4, 7), (2, 5)):
        r = eng.ct_mul_chain(X, depth, streams=streams, chunk=chunk, digest_n=n, nonce_seed=0xD0D7)
        assert np.array_equal(base["digests"], r["digests"]) and np.array_equal(base["counts"], r["counts"])
        assert r["chunks"] == (n + chunk - 1) // chunk
    assert np.array_equal(base["digests"], big["digests"])
    torch.cuda.synchronize()
    assert torch.cuda.mem_get_info()[0] + (64 << 20) >= free_big


def test_chain_final_step_sigma_vs_oracle(oracle, manifest, H_dense):
    """PVAC_MUL_WITH_SIGMA on the chain entry point: the final step's edges get sigma_from_H with
    the salts the salts_at hook writes (hash-order position per edge), intermediate steps stay
    weights-only. Nonces come from the nonces_at hook (host numpy words, recorded). The last step is
    recomputed by the oracle from c_{depth-1} (captured by after_step) with the same nonces, salts
    and H: layers, weights and every sigma byte-exact."""
    import threading
    from pvac_hfhe_cppbyv_amd import ON_CHUNK_CB, STEP_CB, Engine
    from helpers import Cipher, hip_batch_to_host, hip_d2h_u64, hip_h2d
    eng = Engine(device=0, canon_tag=manifest["canon_tag"])
    assert eng.gen_H().hex() == manifest["H_digest"]
    n, depth, chunk = 6, 3, 4
    X = eng.gen_fresh(n, 0x516A, 20)
    xs = X.to_host()
    lock = threading.Lock()
    rng = np.random.default_rng(0x516B)
    rec = {}

    def nonces_at(user, step, first, A, Xb, Cb, words, nw, stream):
        w = rng.integers(0, 2**64, int(nw), dtype=np.uint64)
        with lock:
            rec[("n", step, first)] = (w, hip_d2h_u64(Cb.contents.l_off, Cb.contents.n, stream))
        hip_h2d(words, w, stream)
        return 0

    def after_step(user, step, first, A, Xb, Cb, words, nw, stream):
        if step == depth - 2:
            with lock:
                rec[("prev", first)] = hip_batch_to_host(Cb.contents, stream)
        return 0

    def salts_at(user, step, first, A, Xb, Cb, words, nw, stream):
        assert step == depth - 1
        w = rng.integers(0, 2**64, int(nw), dtype=np.uint64)
        with lock:
            rec[("s", first)] = (w, hip_d2h_u64(Cb.contents.e_off, Cb.contents.n, stream))
        hip_h2d(words, w, stream)
        return 0

    def keep(user, first, cb, stream):
        with lock:
            rec[("out", first)] = hip_batch_to_host(cb.contents, stream, sigma_words=128)
        return 0

    hooks = dict(nonces_at=STEP_CB(nonces_at), after_step=STEP_CB(after_step), salts_at=STEP_CB(salts_at),
                 on_chunk=ON_CHUNK_CB(keep))
    eng.ct_mul_chain(X, depth, streams=2, chunk=chunk, sigma=True, **hooks)
    for c0 in range(0, n, chunk):
        words, loff = rec[("n", depth - 1, c0)]
        salts, eoff = rec[("s", c0)]
        for i, (prev, out) in enumerate(zip(rec[("prev", c0)], rec[("out", c0)])):
            x = xs[c0 + i]
            s0 = int(loff[i]) + prev.nL + x.nL
            nz = words[2 * s0:2 * s0 + 2 * prev.nL * x.nL]
            ref = oracle.ct_mul(prev, Cipher(x.layers, x.meta, x.w_lo, x.w_hi), nz,
                                salts=salts[int(eoff[i]):int(eoff[i]) + out.nE], H=H_dense,
                                canon_tag=manifest["canon_tag"])
            assert out.nE == ref.nE and np.array_equal(out.meta, ref.meta)
            assert np.array_equal(out.w_lo, ref.w_lo) and np.array_equal(out.w_hi, ref.w_hi)
            assert np.array_equal(out.layers["ztag"], ref.layers["ztag"])
            assert np.array_equal(out.sigma, ref.sigma)


def _enc_inputs(eng, n, seed):
    sk, man, em = fixture_secret()
    assert eng.gen_H().hex() == man["H_digest"]
    eng.set_secret(read_u64("sk_prf_k.u64"), read_u64("sk_lpn_s.u64"), em["lpn_n"], em["lpn_t"], em["lpn_tau_num"],
                   em["lpn_tau_den"])
    eng.set_powg(read_u64("powg_B.u64"))
    rng = np.random.default_rng(seed)
    X, st = eng.enc_value(rng.integers(0, 2**64, n, dtype=np.uint64), rng.integers(0, 2**64, (n, 256), dtype=np.uint64))
    assert not st.any()
    return X, man


def _oracle_chain(oracle, X, n, depth, canon_tag, edge_budget=1200000, B=337):
    px = pack_device_batch(X, n)
    P_ = lambda a: a.ctypes.data_as(C.c_void_p)
    ocnt, odig, se = np.zeros(n, np.uint64), np.zeros(n, np.uint64), np.zeros(depth, np.uint64)
    oracle.lib.orc_ct_mul_chain_timed(C.byref(default_params(canon_tag, edge_budget=edge_budget, B=B)), n,
                                      *(P_(a) for a in px), depth, 8, P_(ocnt), P_(odig), P_(se))
    return ocnt, odig


def test_chain_dense_images_equal_records(oracle):
    """Intermediate chain steps hand their C to the next step as dense images (k_large_products_direct's
    image writer: cell c of product layer lp at slot lp 2B + c with its hash-order position; the next
    step's k_large_lists takes the slabs as its A lists and the dense staging reads the weights in
    slab order). enc_value inputs to depth 7 without hooks (steps 3-6 write images) give the same final
    digests, edge counts and per-step edge sums as the same chains with an after_step hook (records
    at every step), as the step-by-step engine run and as the CPU port."""
    from pvac_hfhe_cppbyv_amd import STEP_CB, Engine
    eng = Engine(device=0, canon_tag=fixture_secret()[1]["canon_tag"])
    n, depth, chunk, seed = 5, 7, 3, 0x1A6E
    X, man = _enc_inputs(eng, n, 0x1A6D)
    img = eng.ct_mul_chain(X, depth, nonce_seed=seed, streams=2, chunk=chunk, digest_n=n)

    def after(user, step, first, A, Xb, Cb, words, nw, stream):
        return 0

    rec = eng.ct_mul_chain(X, depth, nonce_seed=seed, streams=2, chunk=chunk, digest_n=n, after_step=STEP_CB(after))
    assert img["redo"] == 0 and rec["redo"] == 0
    assert img["image_steps"] == 4 * n and rec["image_steps"] == 0   # steps 3-6 handed on as images
    assert np.array_equal(img["digests"], rec["digests"]) and np.array_equal(img["counts"], rec["counts"])
    assert img["edges"] == rec["edges"] and img["edges"][5] == n * 128 * 674   # step 6: 128 dense product layers
    dig, cnt, edges = _stepwise(eng, X, depth, seed, chunk)
    assert np.array_equal(img["digests"], dig) and np.array_equal(img["counts"], cnt) and img["edges"] == edges
    ocnt, odig = _oracle_chain(oracle, X, n, depth, man["canon_tag"])
    assert np.array_equal(ocnt, cnt) and np.array_equal(odig, dig)


def test_chain_image_inputs_redone_on_records(oracle):
    """edge_budget between step 4's and step 5's output sizes (21,568 and 43,136 edges): step 4 writes
    its C as dense images, and every step-5 pair exceeds the budget, so guard_budget's canonical order
    sends it to the redo, which first turns its image input back into hash-order records
    (k_img_copy / k_img_scatter). Final digests and counts equal the record-only run (after_step hook)
    and the CPU port's chain with the same edge_budget."""
    from pvac_hfhe_cppbyv_amd import STEP_CB, Engine
    man = fixture_secret()[1]
    eng = Engine(device=0, canon_tag=man["canon_tag"], edge_budget=30000)
    n, depth, chunk, seed = 4, 6, 2, 0x1A6F
    X, _ = _enc_inputs(eng, n, 0x1A70)
    img = eng.ct_mul_chain(X, depth, nonce_seed=seed, streams=2, chunk=chunk, digest_n=n)
    assert img["redo"] >= 2 * n and img["image_steps"] == 2 * n   # images: steps 3, 4; redone: steps 5, 6

    def after(user, step, first, A, Xb, Cb, words, nw, stream):
        return 0

    rec = eng.ct_mul_chain(X, depth, nonce_seed=seed, streams=2, chunk=chunk, digest_n=n, after_step=STEP_CB(after))
    assert np.array_equal(img["digests"], rec["digests"]) and np.array_equal(img["counts"], rec["counts"])
    ocnt, odig = _oracle_chain(oracle, X, n, depth, man["canon_tag"], edge_budget=30000)
    assert np.array_equal(ocnt, img["counts"]) and np.array_equal(odig, img["digests"])


def test_chain_images_with_four_b_layers(oracle):
    """Inputs with four edge layers (ct_add of two fresh batches, 15 edges per layer: 60 <= 63 B edges,
    the direct mode's per-A-edge masks) and B = 131 (262 cells per product layer, so the product
    layers fill after two steps): every chain step multiplies by four B layers, so the image writer
    takes its scattered-store path (more than two B layers), and the intermediate steps whose product
    layers are all filled hand C on as dense images. Final digests and counts equal the record-only
    run (after_step hook), the step-by-step engine run and the CPU port's chain."""
    from pvac_hfhe_cppbyv_amd import STEP_CB, Engine
    tag, Bm = 0xF0A4, 131
    eng = Engine(device=0, canon_tag=tag, B=Bm)
    n, depth, chunk, seed = 3, 4, 2, 0xF0A5
    X = eng.ct_add(eng.gen_fresh(n, 0xF0A6, 15), eng.gen_fresh(n, 0xF0A7, 15))
    assert X.l_cnt[:n].cpu().tolist() == [4] * n and X.e_cnt[:n].cpu().tolist() == [60] * n
    img = eng.ct_mul_chain(X, depth, nonce_seed=seed, streams=2, chunk=chunk, digest_n=n)

    def after(user, step, first, A, Xb, Cb, words, nw, stream):
        return 0

    rec = eng.ct_mul_chain(X, depth, nonce_seed=seed, streams=2, chunk=chunk, digest_n=n, after_step=STEP_CB(after))
    assert img["redo"] == 0 and rec["redo"] == 0
    # step 3's C (256 product layers x 262 cells) is full: one image per chain; step 2's is not
    assert img["image_steps"] == n and rec["image_steps"] == 0
    assert img["edges"][2] == n * 256 * 2 * Bm
    assert np.array_equal(img["digests"], rec["digests"]) and np.array_equal(img["counts"], rec["counts"])
    assert img["edges"] == rec["edges"]
    dig, cnt, edges = _stepwise(eng, X, depth, seed, chunk)
    assert np.array_equal(img["digests"], dig) and np.array_equal(img["counts"], cnt) and img["edges"] == edges
    ocnt, odig = _oracle_chain(oracle, X, n, depth, tag, B=Bm)
    assert np.array_equal(ocnt, cnt) and np.array_equal(odig, dig)


def _chainf_on_gpu(eng, man, depth, n, powg, images=True):
    """ref_harness chainf / chainf8 on the GPU through the chain entry point: x and every operand
    encrypted by the GPU enc_value from their stretches of the regenerated stream (device splitmix,
    pvac_hip_fill_random at the stretch's offset), the operands passed per step, each step's nonces from
    the head of its mul stretch (nonces_at) and the final step's salts from the rest (salts_at), sigmas
    on the final step. n copies of the chain run in one call (2 streams, chunks of 1). Returns the
    final ciphers (with sigmas) and the call's statistics."""
    import threading
    import torch
    from pvac_hfhe_cppbyv_amd import ON_CHUNK_CB, STEP_CB
    from helpers import hip_batch_to_host, hip_d2h_u64, hip_h2d, splitmix_stream, stream_seed
    S = man["seed"]
    stride = eng.enc_caps()[2]

    def enc_stretch(j0, ln):
        assert ln <= stride
        rnd = torch.empty(stride, dtype=torch.int64, device=eng.device)
        eng.fill_random(rnd, stream_seed(S, j0))   # the device generator at the stretch's offset
        assert np.array_equal(rnd.cpu().numpy().view(np.uint64), splitmix_stream(S, j0, stride))
        Y, st = eng.enc_value(np.full(n, 2, np.uint64), rnd.repeat(n).reshape(n, stride))
        assert not st.any()
        return Y

    X = enc_stretch(*man["x_stream"])
    ops = [enc_stretch(*rec["enc_stream"]) for rec in man["steps"][:depth]]
    lock = threading.Lock()
    finals = {}

    def nonces_at(user, step, first, A, Xb, Cb, words, nw, stream):
        rec = man["steps"][step]
        m0, nn = rec["mul_stream"][0], rec["nonce_words"]
        k = Cb.contents.n
        la, lx = hip_d2h_u64(A.contents.l_cnt, k, stream), hip_d2h_u64(Xb.contents.l_cnt, k, stream)
        lo = hip_d2h_u64(Cb.contents.l_off, k, stream)
        w = np.zeros(int(nw), np.uint64)
        for i in range(k):
            assert 2 * int(la[i]) * int(lx[i]) == nn
            s0 = 2 * int(lo[i] + la[i] + lx[i])
            w[s0:s0 + nn] = splitmix_stream(S, m0, nn)
        hip_h2d(words, w, stream)
        return 0

    def salts_at(user, step, first, A, Xb, Cb, words, nw, stream):
        rec = man["steps"][step]
        m0, nn = rec["mul_stream"][0], rec["nonce_words"]
        k = Cb.contents.n
        ec, eo = hip_d2h_u64(Cb.contents.e_cnt, k, stream), hip_d2h_u64(Cb.contents.e_off, k, stream)
        w = np.zeros(int(nw), np.uint64)
        for i in range(k):
            assert int(ec[i]) == rec["edges"]
            w[int(eo[i]):int(eo[i]) + int(ec[i])] = splitmix_stream(S, m0 + nn, int(ec[i]))
        hip_h2d(words, w, stream)
        return 0

    def keep(user, first, cb, stream):
        cs = hip_batch_to_host(cb.contents, stream, sigma_words=128)
        with lock:
            for i, c in enumerate(cs):
                finals[first + i] = c
        return 0

    hooks = dict(nonces_at=STEP_CB(nonces_at), salts_at=STEP_CB(salts_at), on_chunk=ON_CHUNK_CB(keep))
    if not images:
        hooks["after_step"] = STEP_CB(lambda *a: 0)
    r = eng.ct_mul_chain(X, depth, streams=2, chunk=1, sigma=True, operands=ops, digest_n=n, **hooks)
    return [finals[i] for i in range(n)], r


def _chainf_check(oracle, eng, man, depth, cs, powg):
    """c_depth against the fixture: edges, layers, commit_ct with sigmas and of the weights only."""
    from helpers import Cipher as HC
    import json
    import os
    from helpers import REF
    with open(os.path.join(REF, "manifest.json")) as f:
        Hd = bytes.fromhex(json.load(f)["H_digest"])
    rec = man["steps"][depth - 1]
    for c in cs:
        assert c.nE == rec["edges"] and c.nL == rec["layers"]
        assert oracle.commit(c, man["canon_tag"], Hd).hex() == rec["commit"], depth
        assert oracle.commit(HC(c.layers, c.meta, c.w_lo, c.w_hi), man["canon_tag"], Hd).hex() == rec["commit_weights"]


def _chainf_engine(name):
    import json
    import os
    from pvac_hfhe_cppbyv_amd import Engine
    from helpers import REF
    with open(os.path.join(REF, f"{name}_manifest.json")) as f:
        man = json.load(f)
    sk, m0, em = fixture_secret()
    eng = Engine(device=0, canon_tag=man["canon_tag"])
    assert eng.gen_H().hex() == m0["H_digest"]
    eng.set_secret(read_u64("sk_prf_k.u64"), read_u64("sk_lpn_s.u64"), em["lpn_n"], em["lpn_t"], em["lpn_tau_num"],
                   em["lpn_tau_den"])
    powg = read_u64("powg_B.u64")
    eng.set_powg(powg)
    return eng, man, powg


def test_chainf_reference_loop_replay_on_gpu(oracle):
    """The reference's own chain loop with a fresh enc_value(2) per step (tests/test_main.cpp:289-293,
    ref_harness chainf, depth 4, full stream) through the chain entry point's per-step operands: for
    every depth k = 1..4 a chain call of depth k gives c_k whose commit_ct (with sigmas, and of the
    weights alone) equals the reference's; c_4's weights-only .ct bytes, layer table and per-edge sigma
    digests equal the fixture files, and it decrypts to 2^5 on the GPU. Two copies per call."""
    import hashlib
    import os
    from pvac_hfhe_cppbyv_amd import DeviceBatch, HostCipher
    from helpers import REF, Cipher as HC, read_layers_u64
    from helpers import write_ct
    eng, man, powg = _chainf_engine("chainf")
    for k in range(1, man["depth"] + 1):
        cs, r = _chainf_on_gpu(eng, man, k, 2, powg)
        assert r["redo"] == 0
        _chainf_check(oracle, eng, man, k, cs, powg)
    c = cs[0]
    with open(os.path.join(REF, "chainf_final.ct"), "rb") as f:
        assert write_ct([HC(c.layers, c.meta, c.w_lo, c.w_hi)]) == f.read()
    lay = read_layers_u64("chainf_final_layers.u64")
    for fld in ("rule", "ztag", "nonce_lo", "nonce_hi"):
        assert np.array_equal(c.layers[fld], lay[fld])
    dig = np.array([int.from_bytes(hashlib.sha256(s.astype("<u8").tobytes()).digest()[:8], "little")
                    for s in c.sigma], np.uint64)
    assert np.array_equal(dig, read_u64("chainf_final_sigdig.u64"))
    F = DeviceBatch.from_host([HostCipher(c.layers, c.meta, c.w_lo, c.w_hi, None)], eng.device)
    vals, st = eng.dec_value(F, eng.base_R(F))
    assert not st.any() and vals == [32]


def test_chainf8_reference_loop_depth8_on_gpu(oracle):
    """The same loop to depth 8 (ref_harness chainf8: steps 5-8 are the dense / direct-mode / image
    regime, c_8 holds 345,088 edges), pinned to the reference's own per-step commit_ct digests: a chain
    call of depth k for every k = 1..8 through the per-step operands, with the dense images between
    steps 3 .. k-1, gives c_k whose commit (with sigmas, and of the weights alone) equals the
    reference's; the depth-8 call with records throughout (an after_step hook) gives the same c_8; c_8
    decrypts to 2^9 on the GPU."""
    from pvac_hfhe_cppbyv_amd import DeviceBatch, HostCipher
    eng, man, powg = _chainf_engine("chainf8")
    assert man["depth"] == 8
    for k in range(1, 9):
        cs, r = _chainf_on_gpu(eng, man, k, 1, powg)
        assert r["redo"] == 0
        if k >= 4:
            assert r["image_steps"] == k - 3   # steps 3 .. k - 1 handed on as images
        _chainf_check(oracle, eng, man, k, cs, powg)
    rec_cs, r = _chainf_on_gpu(eng, man, 8, 1, powg, images=False)
    assert r["image_steps"] == 0
    _chainf_check(oracle, eng, man, 8, rec_cs, powg)
    c = cs[0]
    F = DeviceBatch.from_host([HostCipher(c.layers, c.meta, c.w_lo, c.w_hi, None)], eng.device)
    vals, st = eng.dec_value(F, eng.base_R(F))
    assert not st.any() and vals == [512]


def _three_layer_ciphers(rng, k, epl=20, B=337):
    """k host ciphers of 3 BASE layers x epl distinct (idx, ch) cells (3 epl <= 63 edges: the direct
    mode's per-A-edge masks), weights canonical and nonzero."""
    from pvac_hfhe_cppbyv_amd import HostCipher
    from helpers import LAYER_DT
    out = []
    for _ in range(k):
        L = np.zeros(3, LAYER_DT)
        L["ztag"], L["nonce_lo"], L["nonce_hi"] = (rng.integers(0, 2**63, 3, dtype=np.uint64) for _ in range(3))
        meta = []
        for l in range(3):
            for c in rng.choice(2 * B, epl, replace=False):
                meta.append(l | (int(c % B) << 32) | (int(c // B) << 48))
        ne = len(meta)
        out.append(HostCipher(L, np.array(meta, np.uint64), rng.integers(1, 2**64, ne, dtype=np.uint64),
                              rng.integers(0, 2**62, ne, dtype=np.uint64)))
    return out


def test_chain_image_redo_of_mixed_sizes(oracle):
    """ADVICE r5 (k_img_copy / k_img_scatter batching): image inputs of DIFFERENT sizes turned back into
    records in one exec, in launches of two pairs (PVAC_CHAIN_IMG_BATCH2). Four chains in one chunk:
    pairs 0, 1 multiply by 2-layer operands at step 1, pairs 2, 3 by 3-layer ones, later steps by x, so
    from step 3 on the second pair group's dense images hold more product layers. edge_budget sits
    between every step-4 and every step-5 output: steps 3 and 4 hand C on as images, and at step 5 all
    four pairs leave the direct mode, so their images (small, small, large, large) are converted in two
    launches. Digests and counts equal the record-only run (after_step hook), the call without the
    small launches, and the CPU port's chains with the same operands and budget."""
    import ctypes
    from pvac_hfhe_cppbyv_amd import STEP_CB, DeviceBatch, Engine
    rng = np.random.default_rng(0x1A6B)
    tag = 0x1A6B
    n, depth = 4, 6
    probe = Engine(device=0, canon_tag=tag)
    X = probe.gen_fresh(n, 0x1A6C, 20)
    xs = X.to_host()
    y3 = _three_layer_ciphers(rng, 2)
    ops_h = [xs[0], xs[1], y3[0], y3[1]]
    # step sizes of both groups from the CPU port: the budget goes between steps 4 and 5
    sizes = []
    for i in (0, 2):
        c = Cipher(xs[i].layers, xs[i].meta, xs[i].w_lo, xs[i].w_hi)
        row = []
        for d in range(depth):
            y = ops_h[i] if d == 0 else xs[i]
            y = Cipher(y.layers, y.meta, y.w_lo, y.w_hi)
            c = oracle.ct_mul(c, y, np.zeros(2 * c.nL * y.nL, np.uint64), canon_tag=tag)
            row.append(c.nE)
        sizes.append(row)
    budget = max(sizes[0][3], sizes[1][3])
    assert min(sizes[0][4], sizes[1][4]) > budget and sizes[1][2] != sizes[0][2]
    eng = Engine(device=0, canon_tag=tag, edge_budget=budget)
    X = DeviceBatch.from_host(xs, eng.device)
    Y = DeviceBatch.from_host(ops_h, eng.device)
    kw = dict(nonce_seed=0x1A6D, streams=1, chunk=n, digest_n=n, operands=[Y])
    img2 = eng.ct_mul_chain(X, depth, img_batch2=True, **kw)
    assert img2["image_steps"] == 2 * n and img2["redo"] >= 2 * n   # images: steps 3, 4; redone: 5, 6
    img = eng.ct_mul_chain(X, depth, **kw)
    rec = eng.ct_mul_chain(X, depth, after_step=STEP_CB(lambda *a: 0), **kw)
    assert rec["image_steps"] == 0
    for r in (img, rec):
        assert np.array_equal(img2["digests"], r["digests"]) and np.array_equal(img2["counts"], r["counts"])
    assert [int(v) for v in img2["counts"]] == [sizes[0][-1]] * 2 + [sizes[1][-1]] * 2
    px, po = pack_device_batch(X, n), pack_device_batch(Y, n)
    P_ = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    ocnt, odig, se = np.zeros(n, np.uint64), np.zeros(n, np.uint64), np.zeros(depth, np.uint64)
    oracle.lib.orc_ct_mul_chain_ops_timed(ctypes.byref(default_params(tag, edge_budget=budget)), n, *(P_(a) for a in px),
                                          depth, 1, *(P_(a) for a in po), 4, P_(ocnt), P_(odig), P_(se))
    assert np.array_equal(ocnt, img2["counts"]) and np.array_equal(odig, img2["digests"])
