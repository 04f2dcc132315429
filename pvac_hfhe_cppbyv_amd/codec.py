"""The reference's .ct ciphertext file format (tests/add.cpp:22-155: saveCts / loadCts) through the
native codec (csrc/ct_codec.cpp, C ABI pvac_ct_scan / pvac_ct_parse / pvac_ct_write).

  read_ct(src)            -> list[HostCipher]            (src: path, bytes or memoryview)
  read_ct_soa(src)        -> dict of SoA numpy arrays    (dense CSR, one copy, no per-cipher split)
  write_ct(ciphers)       -> bytes                       (list[HostCipher] or an SoA dict)
  load_ct(src, device)    -> DeviceBatch                 (parse on the host, one H2D copy per array)
  save_ct(batch, path)                                   (DeviceBatch -> file)

PROD layers carry no seed on disk (the reference's putLayer writes pa/pb only), so parsed PROD
layers have ztag = nonce = 0; sigmas round-trip bit-exactly.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import LAYER_DT, CtBatch, DeviceBatch, HostCipher, PvacError, load_library

CT_MIXED_SIGMA = 0x1
_LIB = None


class CtFileInfo(C.Structure):
    _fields_ = [("n_ciphers", C.c_uint64), ("total_layers", C.c_uint64), ("total_edges", C.c_uint64),
                ("sigma_bits", C.c_uint32), ("sigma_words", C.c_uint32), ("flags", C.c_uint32),
                ("pad", C.c_uint32)]


def _lib():
    global _LIB
    if _LIB is None:
        _LIB = load_library()
    return _LIB


def _bytes(src) -> np.ndarray:
    if isinstance(src, (str, os.PathLike)):
        return np.fromfile(src, dtype=np.uint8)
    return np.frombuffer(src, dtype=np.uint8)


def _ptr(a):
    return None if a is None else C.c_void_p(a.ctypes.data)


def _check(rc, what):
    if rc != 0:
        raise PvacError(f"{what}: status {rc}")


def scan(src) -> CtFileInfo:
    buf = _bytes(src)
    info = CtFileInfo()
    _check(_lib().pvac_ct_scan(_ptr(buf), buf.size, C.byref(info)), "pvac_ct_scan")
    return info


def read_ct_soa(src, threads: int = 0) -> dict:
    buf = _bytes(src)
    info = CtFileInfo()
    lib = _lib()
    _check(lib.pvac_ct_scan(_ptr(buf), buf.size, C.byref(info)), "pvac_ct_scan")
    n, nl, ne, sw = int(info.n_ciphers), int(info.total_layers), int(info.total_edges), int(info.sigma_words)
    soa = {
        "l_off": np.zeros(max(n, 1), np.uint64), "l_cnt": np.zeros(max(n, 1), np.uint64),
        "e_off": np.zeros(max(n, 1), np.uint64), "e_cnt": np.zeros(max(n, 1), np.uint64),
        "layers": np.zeros(max(nl, 1), LAYER_DT),
        "meta": np.zeros(max(ne, 1), np.uint64), "w_lo": np.zeros(max(ne, 1), np.uint64),
        "w_hi": np.zeros(max(ne, 1), np.uint64),
        "sigma": np.zeros((max(ne, 1), sw), np.uint64) if sw else None,
    }
    X = CtBatch(n=n, l_off=_ptr(soa["l_off"]), l_cnt=_ptr(soa["l_cnt"]), layers=_ptr(soa["layers"]),
                e_off=_ptr(soa["e_off"]), e_cnt=_ptr(soa["e_cnt"]), meta=_ptr(soa["meta"]), w_lo=_ptr(soa["w_lo"]),
                w_hi=_ptr(soa["w_hi"]), sigma=_ptr(soa["sigma"]), sigma_words=sw)
    _check(lib.pvac_ct_parse(_ptr(buf), buf.size, C.byref(X), int(threads)), "pvac_ct_parse")
    soa["n"], soa["total_layers"], soa["total_edges"] = n, nl, ne
    soa["sigma_bits"] = int(info.sigma_bits)
    return soa


def read_ct(src, threads: int = 0) -> list:
    s = read_ct_soa(src, threads)
    out = []
    for i in range(s["n"]):
        a, b = int(s["l_off"][i]), int(s["l_off"][i] + s["l_cnt"][i])
        c, d = int(s["e_off"][i]), int(s["e_off"][i] + s["e_cnt"][i])
        out.append(HostCipher(s["layers"][a:b].copy(), s["meta"][c:d].copy(), s["w_lo"][c:d].copy(),
                              s["w_hi"][c:d].copy(), None if s["sigma"] is None else s["sigma"][c:d].copy()))
    return out


def _soa_from_ciphers(ciphers) -> dict:
    n = len(ciphers)
    lc = np.array([c.nL for c in ciphers], np.uint64)
    ec = np.array([c.nE for c in ciphers], np.uint64)
    has_sig = n > 0 and all(c.sigma is not None for c in ciphers)
    cat = lambda f, dt: (np.concatenate([getattr(c, f) for c in ciphers]).astype(dt) if n else np.zeros(0, dt))
    return {
        "n": n, "l_cnt": lc, "e_cnt": ec,
        "l_off": (np.concatenate([[0], np.cumsum(lc)[:-1]]) if n else lc).astype(np.uint64),
        "e_off": (np.concatenate([[0], np.cumsum(ec)[:-1]]) if n else ec).astype(np.uint64),
        "layers": cat("layers", LAYER_DT), "meta": cat("meta", np.uint64), "w_lo": cat("w_lo", np.uint64),
        "w_hi": cat("w_hi", np.uint64),
        "sigma": np.concatenate([c.sigma for c in ciphers]).astype(np.uint64) if has_sig else None,
    }


def write_ct(ciphers, sigma_bits: int = 8192, threads: int = 0) -> bytes:
    s = ciphers if isinstance(ciphers, dict) else _soa_from_ciphers(list(ciphers))
    keep = {k: (np.ascontiguousarray(v) if isinstance(v, np.ndarray) else v) for k, v in s.items()}
    sig = keep.get("sigma")
    sw = int(sig.shape[1]) if sig is not None and sig.ndim == 2 else 0
    X = CtBatch(n=keep["n"], l_off=_ptr(keep["l_off"]), l_cnt=_ptr(keep["l_cnt"]), layers=_ptr(keep["layers"]),
                e_off=_ptr(keep["e_off"]), e_cnt=_ptr(keep["e_cnt"]), meta=_ptr(keep["meta"]),
                w_lo=_ptr(keep["w_lo"]), w_hi=_ptr(keep["w_hi"]), sigma=_ptr(sig) if sw else None,
                sigma_words=sw)
    lib = _lib()
    size = C.c_uint64()
    _check(lib.pvac_ct_serialized_size(C.byref(X), sigma_bits, C.byref(size)), "pvac_ct_serialized_size")
    out = np.zeros(int(size.value), np.uint8)
    wrote = C.c_uint64()
    _check(lib.pvac_ct_write(C.byref(X), sigma_bits, _ptr(out), out.size, C.byref(wrote), int(threads)),
           "pvac_ct_write")
    return out[: int(wrote.value)].tobytes()


def load_ct(src, device, sigma: bool = True, threads: int = 0) -> DeviceBatch:
    """Parse on the host into dense SoA arrays, then one host-to-device copy per array."""
    import torch
    s = read_ct_soa(src, threads)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(device)
    lay = torch.from_numpy(np.ascontiguousarray(s["layers"]).view(np.int64).reshape(-1, 5)).to(device)
    sg = None
    if sigma and s["sigma"] is not None:
        sg = torch.from_numpy(np.ascontiguousarray(s["sigma"]).view(np.int64)).to(device)
    return DeviceBatch(s["n"], t(s["l_off"]), t(s["l_cnt"]), lay, t(s["e_off"]), t(s["e_cnt"]), t(s["meta"]),
                       t(s["w_lo"]), t(s["w_hi"]), sg)


def save_ct(batch: DeviceBatch, path, sigma_bits: int = 8192, threads: int = 0) -> int:
    data = write_ct(batch.to_host(), sigma_bits, threads)
    with open(path, "wb") as f:
        f.write(data)
    return len(data)
