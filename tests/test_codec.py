"""The native .ct codec (csrc/ct_codec.cpp; reference tests/add.cpp:22-155 saveCts/loadCts):
every fixture the reference wrote parses to the same records as the independent Python reader in
helpers.py and serializes back to the identical bytes; malformed images are rejected; thread
count does not change results. CPU only (the codec is host code); the GPU interop check is in
test_gpu_codec_interop."""
import glob
import os
import struct

import numpy as np
import pytest

from helpers import CT_MAGIC, GOLD, LAYER_DT, Cipher, read_ct

FIXTURES = sorted(glob.glob(os.path.join(GOLD, "**", "*.ct"), recursive=True))


@pytest.fixture(scope="module")
def codec():
    from pvac_hfhe_cppbyv_amd import codec as c
    return c


def _same_records(a, b):
    assert a.nL == b.nL and a.nE == b.nE
    for f in ("rule", "pa", "pb", "ztag", "nonce_lo", "nonce_hi"):
        assert np.array_equal(a.layers[f], b.layers[f]), f
    assert np.array_equal(a.meta, b.meta)
    assert np.array_equal(a.w_lo, b.w_lo) and np.array_equal(a.w_hi, b.w_hi)
    if b.sigma is None:
        assert a.sigma is None or a.nE == 0
    else:
        assert np.array_equal(a.sigma, b.sigma)


@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.relpath(p, GOLD) for p in FIXTURES])
def test_fixture_roundtrip(codec, path):
    raw = open(path, "rb").read()
    mine, ref = codec.read_ct(path), read_ct(path)
    assert len(mine) == len(ref)
    for a, b in zip(mine, ref):
        _same_records(a, b)
    bits = codec.scan(raw).sigma_bits
    assert codec.write_ct(mine, sigma_bits=bits or 8192) == raw


def test_fixture_count(codec):
    assert len(FIXTURES) >= 50   # the oracle harness' ct fixtures + bounty2/3 data


def _synthetic(rng, n, sigma):
    out = []
    for k in range(n):
        nl, ne = int(rng.integers(0, 6)), int(rng.integers(0, 50))
        L = np.zeros(nl, LAYER_DT)
        L["rule"] = rng.integers(0, 3, nl)           # BASE, PROD, and an unknown rule
        base = L["rule"] == 0
        L["ztag"][base] = rng.integers(0, 2**63, base.sum(), dtype=np.uint64)
        L["nonce_lo"][base] = rng.integers(0, 2**63, base.sum(), dtype=np.uint64)
        L["nonce_hi"][base] = rng.integers(0, 2**63, base.sum(), dtype=np.uint64)
        prod = L["rule"] == 1
        L["pa"][prod] = rng.integers(0, 2**32, prod.sum(), dtype=np.uint64)
        L["pb"][prod] = rng.integers(0, 2**32, prod.sum(), dtype=np.uint64)
        meta = (rng.integers(0, 2**32, ne, dtype=np.uint64) | (rng.integers(0, 2**16, ne, dtype=np.uint64) << np.uint64(32))
                | (rng.integers(0, 256, ne, dtype=np.uint64) << np.uint64(48)))
        sg = rng.integers(0, 2**63, (ne, 128), dtype=np.uint64) if sigma else None
        out.append(Cipher(L, meta, rng.integers(0, 2**63, ne, dtype=np.uint64),
                          rng.integers(0, 2**63, ne, dtype=np.uint64), sg))
    return out


@pytest.mark.parametrize("sigma", [False, True])
def test_synthetic_roundtrip_and_threads(codec, sigma):
    rng = np.random.default_rng(3 + sigma)
    cs = _synthetic(rng, 40, sigma)
    from pvac_hfhe_cppbyv_amd import HostCipher
    hc = [HostCipher(c.layers, c.meta, c.w_lo, c.w_hi, c.sigma) for c in cs]
    raw = codec.write_ct(hc, sigma_bits=8192 if sigma else 0, threads=1)
    assert raw == codec.write_ct(hc, sigma_bits=8192 if sigma else 0, threads=7)
    info = codec.scan(raw)
    assert info.n_ciphers == 40 and info.total_edges == sum(c.nE for c in cs)
    assert info.sigma_bits == (8192 if sigma else 0)
    for threads in (1, 5):
        back = codec.read_ct(raw, threads=threads)
        for a, c in zip(back, cs):
            exp = c.layers.copy()
            unk = exp["rule"] > 1   # unknown rules keep only the rule byte
            for f in ("pa", "pb", "ztag", "nonce_lo", "nonce_hi"):
                exp[f][unk] = 0
            exp["ztag"][exp["rule"] == 1] = 0
            exp["nonce_lo"][exp["rule"] == 1] = 0
            exp["nonce_hi"][exp["rule"] == 1] = 0
            exp["pa"][exp["rule"] == 0] = 0
            exp["pb"][exp["rule"] == 0] = 0
            _same_records(a, Cipher(exp, c.meta, c.w_lo, c.w_hi, c.sigma))
        assert codec.write_ct(back, sigma_bits=8192 if sigma else 0) == raw


def test_empty_file(codec):
    raw = struct.pack("<IIQ", CT_MAGIC, 1, 0)
    assert codec.read_ct(raw) == []
    assert codec.write_ct([]) == raw


def test_malformed_rejected(codec):
    from pvac_hfhe_cppbyv_amd import PvacError
    raw = open(os.path.join(GOLD, "bounty", "a.ct"), "rb").read()
    bad = [raw[:-1], raw + b"\0", b"\0" * 4 + raw[4:], raw[:4] + struct.pack("<I", 2) + raw[8:], raw[:16],
           raw[:8] + struct.pack("<Q", 1 << 60) + raw[16:]]
    for b in bad:
        with pytest.raises(PvacError):
            codec.read_ct(b)


def test_mixed_sigma_bits_rejected(codec):
    from pvac_hfhe_cppbyv_amd import PvacError
    # one edge with an 8192-bit sigma, one with none
    e1 = struct.pack("<IHBBQQI", 0, 1, 0, 0, 5, 6, 8192) + b"\1" * 1024
    e2 = struct.pack("<IHBBQQI", 0, 2, 1, 0, 7, 8, 0)
    lay = struct.pack("<BQQQ", 0, 1, 2, 3)
    raw = struct.pack("<IIQ", CT_MAGIC, 1, 1) + struct.pack("<II", 1, 2) + lay + e1 + e2
    info = codec.scan(raw)
    assert info.flags & codec.CT_MIXED_SIGMA
    with pytest.raises(PvacError):
        codec.read_ct(raw)
