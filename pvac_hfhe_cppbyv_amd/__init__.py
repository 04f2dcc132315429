"""pvac_hfhe_cppbyv_amd — MI355X batched ciphertext-arithmetic engine for pvac-hfhe.

Python view of the C ABI in include/pvac_hip.h (libpvac_hip.so). PyTorch is used only for
device memory and streams; every operation runs in the hand-written HIP kernels of
csrc/. There is NO CPU fallback: if the native library is missing this module raises.

Host-side cipher representation mirrors pvac::Cipher (reference core/types.hpp:96-119):
  layers : numpy structured array LAYER_DT (rule, pa, pb, pad, ztag, nonce_lo, nonce_hi)
  meta   : u64 = layer_id | idx << 32 | ch << 48   (the .ct edge header)
  w_lo/hi: u64 limbs of the Fp weight
  sigma  : (nE, 128) u64 or None
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "lib", "libpvac_hip.so")

LAYER_DT = np.dtype([("rule", "<u4"), ("pa", "<u4"), ("pb", "<u4"), ("pad", "<u4"),
                     ("ztag", "<u8"), ("nonce_lo", "<u8"), ("nonce_hi", "<u8")])

FP_ADD, FP_SUB, FP_MUL, FP_NEG, FP_SCALE, FP_INV = 0, 1, 2, 3, 4, 5
MUL_WITH_SIGMA, MUL_ORDER_CANONICAL = 0x1, 0x2
CHAIN_CHECK_GSUM = 0x100
CHAIN_STAGE_INPUTS = 0x200
CHAIN_IMG_BATCH2 = 0x400
CHAIN_MAX_DEPTH = 32
ENC_WITH_SIGMA = 0x1

P = (1 << 127) - 1


class PvacError(RuntimeError):
    pass


def powg_table(B: int = 337, h: int = 3):
    """powg_B of a key as keygen builds it (crypto/keygen.hpp:67-95): g = h^((p-1)/B) for the first
    h >= `h` with g != 1, powg[i] = g^i, as B (lo, hi) u64 pairs. g^B == 1, which the gsum invariant
    (check_mul_gsum) relies on."""
    if (P - 1) % B:
        raise ValueError("B must divide p - 1")
    while True:
        g = pow(h, (P - 1) // B, P)
        if g != 1:
            break
        h += 1
    out = np.zeros(2 * B, np.uint64)
    x = 1
    for i in range(B):
        out[2 * i], out[2 * i + 1] = x & (2**64 - 1), x >> 64
        x = x * g % P
    return out


class Params(C.Structure):
    _fields_ = [("B", C.c_uint32), ("m_bits", C.c_uint32), ("n_bits", C.c_uint32), ("h_col_wt", C.c_uint32),
                ("x_col_wt", C.c_uint32), ("err_wt", C.c_uint32), ("edge_budget", C.c_uint64),
                ("canon_tag", C.c_uint64)]


class CtBatch(C.Structure):
    _fields_ = [("n", C.c_uint64), ("l_off", C.c_void_p), ("l_cnt", C.c_void_p), ("layers", C.c_void_p),
                ("e_off", C.c_void_p), ("e_cnt", C.c_void_p), ("meta", C.c_void_p), ("w_lo", C.c_void_p),
                ("w_hi", C.c_void_p), ("sigma", C.c_void_p), ("sigma_words", C.c_uint32), ("pad", C.c_uint32)]


class Plan(C.Structure):
    _fields_ = [("total_layer_slots", C.c_uint64), ("total_edge_slots", C.c_uint64), ("n_pairs", C.c_uint64),
                ("n_small", C.c_uint64), ("n_large", C.c_uint64), ("n_invalid", C.c_uint64),
                ("max_keys", C.c_uint32), ("max_prod", C.c_uint32), ("max_na", C.c_uint32),
                ("max_nb", C.c_uint32), ("max_buckets", C.c_uint32), ("max_layers", C.c_uint32),
                ("kind", C.c_uint32), ("reserved", C.c_uint32 * 5)]


FILL_NONCES_CB = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_uint32, C.c_uint64, C.c_uint64, C.c_void_p, C.c_void_p)
ON_CHUNK_CB = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_uint64, C.POINTER(CtBatch), C.c_void_p)
# pvac_chain_step_fn(user, step, first_input, A, X, C, dev_words, n_words, stream): nonces_at / after_step / salts_at
STEP_CB = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_uint32, C.c_uint64, C.POINTER(CtBatch), C.POINTER(CtBatch),
                      C.POINTER(CtBatch), C.c_void_p, C.c_uint64, C.c_void_p)


class ChainOpts(C.Structure):
    _fields_ = [("depth", C.c_uint32), ("streams", C.c_uint32), ("chunk", C.c_uint64), ("nonce_seed", C.c_uint64),
                ("flags", C.c_uint32), ("pad", C.c_uint32), ("digest_n", C.c_uint64), ("digest_out", C.c_void_p),
                ("count_n", C.c_uint64), ("count_out", C.c_void_p), ("fill_nonces", FILL_NONCES_CB),
                ("on_chunk", ON_CHUNK_CB),
                ("user", C.c_void_p), ("nonces_at", STEP_CB), ("after_step", STEP_CB), ("salts_at", STEP_CB),
                ("devices", C.c_void_p), ("n_devices", C.c_uint32), ("pad2", C.c_uint32),
                ("sumdigest_out", C.c_void_p), ("sumdigest_n", C.c_uint64),
                ("operands", C.c_void_p), ("n_operands", C.c_uint32), ("pad3", C.c_uint32)]


class ChainStats(C.Structure):
    _fields_ = [("pair_steps", C.c_uint64), ("edges", C.c_uint64 * CHAIN_MAX_DEPTH),
                ("products", C.c_uint64 * CHAIN_MAX_DEPTH), ("gsum_pairs", C.c_uint64), ("gsum_failed", C.c_uint64),
                ("redo", C.c_uint64), ("chunks", C.c_uint64), ("seconds", C.c_double),
                ("image_steps", C.c_uint64)]


def load_library(path: str = _LIB_PATH) -> C.CDLL:
    if not os.path.exists(path):
        raise PvacError(f"native engine not built: {path} missing (run __graft_entry__.build())")
    lib = C.CDLL(path)
    vp, u64, u32, i32 = C.c_void_p, C.c_uint64, C.c_uint32, C.c_int
    sig = {
        "pvac_hip_abi_version": ([], i32),
        "pvac_hip_ctx_create": ([i32, C.POINTER(Params), C.POINTER(vp)], i32),
        "pvac_hip_ctx_destroy": ([vp], i32),
        "pvac_hip_ctx_set_stream": ([vp, vp], i32),
        "pvac_hip_ctx_stream": ([vp], vp),
        "pvac_hip_ctx_synchronize": ([vp], i32),
        "pvac_hip_last_error": ([vp], C.c_char_p),
        "pvac_hip_ctx_set_H": ([vp, vp, u32, u32], i32),
        "pvac_hip_ctx_gen_H": ([vp, vp], i32),
        "pvac_hip_timing_enable": ([vp, i32], i32),
        "pvac_hip_timing_get": ([vp, C.c_char_p, C.POINTER(C.c_double), C.POINTER(u64)], i32),
        "pvac_hip_timing_reset": ([vp], i32),
        "pvac_hip_fp_binop": ([vp, i32, vp, vp, vp, vp, vp, vp, C.c_size_t], i32),
        "pvac_hip_ct_mul_plan": ([vp, C.POINTER(CtBatch), C.POINTER(CtBatch), C.POINTER(CtBatch),
                                  C.POINTER(Plan)], i32),
        "pvac_hip_ct_mul_exec": ([vp, C.POINTER(Plan), C.POINTER(CtBatch), C.POINTER(CtBatch), vp, vp,
                                  C.POINTER(CtBatch), u32], i32),
        "pvac_hip_ct_mul": ([vp, C.POINTER(CtBatch), C.POINTER(CtBatch), C.POINTER(CtBatch), u64, u64, vp, vp, u32,
                             C.POINTER(Plan)], i32),
        "pvac_hip_ct_mul_redo_count": ([vp, C.POINTER(u64)], i32),
        "pvac_hip_ct_mul_path_count": ([vp, C.POINTER(u64)], i32),
        "pvac_hip_ctx_set_noise": ([vp, C.c_double, C.c_double, C.c_double], i32),
        "pvac_hip_ct_mul_status": ([vp, vp, C.c_size_t], i32),
        "pvac_hip_ct_mul_chain": ([vp, C.POINTER(CtBatch), C.POINTER(ChainOpts), C.POINTER(ChainStats)], i32),
        "pvac_hip_alu_ceiling": ([vp, i32, C.POINTER(C.c_double)], i32),
        "pvac_hip_issue_probe": ([vp, i32, i32, C.POINTER(C.c_double), C.POINTER(C.c_double)], i32),
        "pvac_hip_check_mul_gsum": ([vp, C.POINTER(CtBatch), C.POINTER(CtBatch), C.POINTER(CtBatch), vp, vp,
                                     C.POINTER(u64)], i32),
        "pvac_hip_ct_add_plan": ([vp, C.POINTER(CtBatch), C.POINTER(CtBatch), C.POINTER(CtBatch),
                                  C.POINTER(Plan)], i32),
        "pvac_hip_ct_add_exec": ([vp, C.POINTER(Plan), C.POINTER(CtBatch), C.POINTER(CtBatch), i32,
                                  C.POINTER(CtBatch)], i32),
        "pvac_hip_ct_scale": ([vp, C.POINTER(CtBatch), u64, u64], i32),
        "pvac_hip_sigma_batch": ([vp, C.POINTER(CtBatch), vp], i32),
        "pvac_hip_gen_fresh_batch": ([vp, u64, u32, C.POINTER(CtBatch)], i32),
        "pvac_hip_gen_fresh_batch_at": ([vp, u64, u64, u32, C.POINTER(CtBatch)], i32),
        "pvac_hip_fill_nonces": ([vp, u64, u64, C.POINTER(CtBatch), C.POINTER(CtBatch), C.POINTER(CtBatch), vp], i32),
        "pvac_hip_fill_random": ([vp, u64, vp, C.c_size_t], i32),
        "pvac_hip_batch_digest": ([vp, C.POINTER(CtBatch), vp], i32),
        "pvac_hip_batch_sumdigest": ([vp, C.POINTER(CtBatch), vp], i32),
        "pvac_hip_batch_pack": ([vp, C.POINTER(CtBatch), C.POINTER(CtBatch), C.POINTER(u64)], i32),
        "pvac_hip_bucket_count": ([u64], u64),
        "pvac_hip_chain_partition": ([u64, u64, u32, vp], i32),
        "pvac_hip_memcpy": ([vp, vp, C.c_size_t, vp], i32),
        "pvac_hip_ctx_set_powg": ([vp, vp, u32], i32),
        "pvac_hip_ctx_set_secret": ([vp, vp, vp, u32, u32, u32, u32], i32),
        "pvac_hip_ctx_set_H_digest": ([vp, vp], i32),
        "pvac_hip_prf": ([vp, i32, C.c_size_t, vp, vp], i32),
        "pvac_hip_enc_caps": ([vp, C.POINTER(u32), C.POINTER(u32), C.POINTER(u32)], i32),
        "pvac_hip_enc_value": ([vp, C.c_size_t, vp, vp, u32, C.POINTER(CtBatch), u32, vp], i32),
        "pvac_hip_enc_caps_depth": ([vp, i32, C.POINTER(u32), C.POINTER(u32), C.POINTER(u32)], i32),
        "pvac_hip_enc_value_depth": ([vp, C.c_size_t, vp, vp, u32, i32, C.POINTER(CtBatch), u32, vp], i32),
        "pvac_hip_base_R": ([vp, C.POINTER(CtBatch), vp], i32),
        "pvac_hip_dec_value": ([vp, C.POINTER(CtBatch), vp, vp, vp], i32),
        "pvac_ct_scan": ([vp, C.c_size_t, vp], i32),
        "pvac_ct_parse": ([vp, C.c_size_t, C.POINTER(CtBatch), i32], i32),
        "pvac_ct_serialized_size": ([C.POINTER(CtBatch), u32, C.POINTER(u64)], i32),
        "pvac_ct_write": ([C.POINTER(CtBatch), u32, vp, C.c_size_t, C.POINTER(u64), i32], i32),
    }
    for name, (args, res) in sig.items():
        f = getattr(lib, name)
        f.argtypes = args
        f.restype = res
    return lib


# ------------------------------------------------------------------------------ host ciphers
@dataclass
class HostCipher:
    layers: np.ndarray
    meta: np.ndarray
    w_lo: np.ndarray
    w_hi: np.ndarray
    sigma: np.ndarray | None = None

    @property
    def nL(self):
        return len(self.layers)

    @property
    def nE(self):
        return len(self.meta)


def _t(x):
    import torch
    return torch.from_numpy(np.ascontiguousarray(x).view(np.int64))


class DeviceBatch:
    """A pvac_ct_batch whose arrays are torch CUDA tensors (int64 storage of u64 data)."""

    def __init__(self, n, l_off, l_cnt, layers, e_off, e_cnt, meta, w_lo, w_hi, sigma=None):
        self.n = n
        self.l_off, self.l_cnt, self.layers = l_off, l_cnt, layers
        self.e_off, self.e_cnt = e_off, e_cnt
        self.meta, self.w_lo, self.w_hi, self.sigma = meta, w_lo, w_hi, sigma

    def struct(self) -> CtBatch:
        # positional integer addresses (0 = NULL): built on every call, so kept cheap
        p = lambda t: 0 if t is None else t.data_ptr()
        return CtBatch(self.n, p(self.l_off), p(self.l_cnt), p(self.layers), p(self.e_off), p(self.e_cnt),
                       p(self.meta), p(self.w_lo), p(self.w_hi), p(self.sigma), 128, 0)

    @staticmethod
    def empty(n, layer_slots, edge_slots, device, sigma=False):
        import torch
        z = lambda k: torch.zeros(max(int(k), 1), dtype=torch.int64, device=device)
        return DeviceBatch(n, z(n), z(n), torch.zeros((max(int(layer_slots), 1), 5), dtype=torch.int64,
                                                       device=device),
                           z(n), z(n), z(edge_slots), z(edge_slots), z(edge_slots),
                           torch.zeros((max(int(edge_slots), 1), 128), dtype=torch.int64, device=device)
                           if sigma else None)

    @staticmethod
    def from_host(ciphers, device, sigma=False):
        import torch
        n = len(ciphers)
        lc = np.array([c.nL for c in ciphers], np.uint64)
        ec = np.array([c.nE for c in ciphers], np.uint64)
        lo = np.concatenate([[0], np.cumsum(lc)[:-1]]).astype(np.uint64) if n else lc
        eo = np.concatenate([[0], np.cumsum(ec)[:-1]]).astype(np.uint64) if n else ec
        layers = np.concatenate([c.layers for c in ciphers]) if n else np.zeros(0, LAYER_DT)
        cat = lambda f: np.concatenate([getattr(c, f) for c in ciphers]).astype(np.uint64) if n else \
            np.zeros(0, np.uint64)
        meta, wlo, whi = cat("meta"), cat("w_lo"), cat("w_hi")
        sg = None
        if sigma:
            sg = np.concatenate([c.sigma if c.sigma is not None else np.zeros((c.nE, 128), np.uint64)
                                 for c in ciphers]).astype(np.uint64)
        dev = lambda a: _t(a if len(a) else np.zeros(1, np.uint64)).to(device)
        lay = torch.from_numpy(np.ascontiguousarray(layers).view(np.int64).reshape(-1, 5) if len(layers)
                               else np.zeros((1, 5), np.int64)).to(device)
        return DeviceBatch(n, dev(lo), dev(lc), lay, dev(eo), dev(ec), dev(meta), dev(wlo), dev(whi),
                           None if sg is None else torch.from_numpy(sg.view(np.int64) if len(sg) else
                                                                    np.zeros((1, 128), np.int64)).to(device))

    def to_host(self):
        u = lambda t: t.cpu().numpy().view(np.uint64)
        lo, lc, eo, ec = u(self.l_off), u(self.l_cnt), u(self.e_off), u(self.e_cnt)
        layers = self.layers.cpu().numpy().reshape(-1).view(LAYER_DT)
        meta, wlo, whi = u(self.meta), u(self.w_lo), u(self.w_hi)
        sg = None if self.sigma is None else self.sigma.cpu().numpy().view(np.uint64)
        out = []
        for i in range(self.n):
            a, b = int(lo[i]), int(lo[i] + lc[i])
            c, d = int(eo[i]), int(eo[i] + ec[i])
            out.append(HostCipher(layers[a:b].copy(), meta[c:d].copy(), wlo[c:d].copy(), whi[c:d].copy(),
                                  None if sg is None else sg[c:d].copy()))
        return out


# ------------------------------------------------------------------------------ engine
class Engine:
    """One pvac_hip_ctx on one GPU, bound to torch's current stream on that device."""

    def __init__(self, device=0, B=337, m_bits=8192, n_bits=16384, h_col_wt=192, x_col_wt=128, err_wt=128,
                 edge_budget=1200000, canon_tag=0, lib: C.CDLL | None = None):
        import torch
        self.torch = torch
        self.lib = lib or load_library()
        self.device = torch.device("cuda", device)
        self.params = Params(B=B, m_bits=m_bits, n_bits=n_bits, h_col_wt=h_col_wt, x_col_wt=x_col_wt,
                             err_wt=err_wt, edge_budget=edge_budget, canon_tag=canon_tag)
        ctx = C.c_void_p()
        self._check(self.lib.pvac_hip_ctx_create(device, C.byref(self.params), C.byref(ctx)), None)
        self.ctx = ctx
        with torch.cuda.device(self.device):
            stream = torch.cuda.current_stream(self.device)
        self._check(self.lib.pvac_hip_ctx_set_stream(self.ctx, C.c_void_p(stream.cuda_stream)))

    def __del__(self):
        try:
            if getattr(self, "ctx", None):
                self.lib.pvac_hip_ctx_destroy(self.ctx)
                self.ctx = None
        except Exception:
            pass

    def _check(self, rc, ctx="self"):
        if rc != 0:
            msg = ""
            if ctx == "self" and getattr(self, "ctx", None):
                msg = self.lib.pvac_hip_last_error(self.ctx).decode(errors="replace")
            raise PvacError(f"pvac_hip error {rc}: {msg}")

    def sync(self):
        self._check(self.lib.pvac_hip_ctx_synchronize(self.ctx))

    # ---- field
    def fp_binop(self, op, a_lo, a_hi, b_lo=None, b_hi=None, out=None):
        torch = self.torch
        n = a_lo.numel()
        c_lo, c_hi = out if out is not None else (torch.empty_like(a_lo), torch.empty_like(a_hi))
        p = lambda t: None if t is None else C.c_void_p(t.data_ptr())
        self._check(self.lib.pvac_hip_fp_binop(self.ctx, op, p(a_lo), p(a_hi), p(b_lo), p(b_hi), p(c_lo), p(c_hi),
                                               n))
        return c_lo, c_hi

    # ---- LPN PRF (crypto/lpn.hpp)
    def set_secret(self, prf_k, lpn_s, lpn_n=4096, lpn_t=16384, tau_num=1, tau_den=8):
        k = np.ascontiguousarray(np.asarray(prf_k, dtype=np.uint64).reshape(4))
        s = np.ascontiguousarray(np.asarray(lpn_s, dtype=np.uint64))
        self._check(self.lib.pvac_hip_ctx_set_secret(self.ctx, C.c_void_p(k.ctypes.data), C.c_void_p(s.ctypes.data),
                                                     lpn_n, lpn_t, tau_num, tau_den))

    def set_H_digest(self, digest: bytes):
        b = C.create_string_buffer(bytes(digest), 32)
        self._check(self.lib.pvac_hip_ctx_set_H_digest(self.ctx, b))

    def prf(self, kind, seeds):
        """seeds: (n, 3) u64 {ztag, nonce_lo, nonce_hi}; kind 0..5 core(dom), 6 prf_R, 7 prf_R_noise.
        Returns a list of ints."""
        torch = self.torch
        a = np.ascontiguousarray(np.asarray(seeds, dtype=np.uint64).reshape(-1, 3))
        n = len(a)
        sd = _t(a.reshape(-1) if n else np.zeros(3, np.uint64)).to(self.device)
        out = torch.zeros(2 * max(n, 1), dtype=torch.int64, device=self.device)
        self._check(self.lib.pvac_hip_prf(self.ctx, kind, n, C.c_void_p(sd.data_ptr()), C.c_void_p(out.data_ptr())))
        o = out.cpu().numpy().view(np.uint64)
        return [int(o[2 * i]) | (int(o[2 * i + 1]) << 64) for i in range(n)]

    # ---- encryption (ops/encrypt.hpp:281-287)
    def enc_caps(self, depth=0):
        lp, ep, dh = C.c_uint32(), C.c_uint32(), C.c_uint32()
        self._check(self.lib.pvac_hip_enc_caps_depth(self.ctx, int(depth), C.byref(lp), C.byref(ep), C.byref(dh)))
        return lp.value, ep.value, dh.value

    def enc_value(self, values, rnd, sigma=False, depth=0):
        """values: n u64 (host array or device tensor); rnd: (n, stride) u64 draws per value (the
        reference's csprng_u64 stream). depth > 0: enc_value_depth (ops/encrypt.hpp:281-287); a value
        of 0 is enc_zero_depth (:293-298). Returns (DeviceBatch, status numpy u32)."""
        torch = self.torch
        if isinstance(values, np.ndarray) or isinstance(values, list):
            values = _t(np.ascontiguousarray(np.asarray(values, dtype=np.uint64))).to(self.device)
        if isinstance(rnd, np.ndarray):
            rnd = _t(np.ascontiguousarray(rnd, np.uint64)).to(self.device)
        n = values.numel()
        stride = rnd.numel() // max(n, 1)
        lp, ep, _ = self.enc_caps(depth)
        z = lambda k: torch.zeros(max(k, 1), dtype=torch.int64, device=self.device)
        C_ = DeviceBatch(n, z(n), z(n), torch.zeros((max(lp * n, 1), 5), dtype=torch.int64, device=self.device), z(n),
                         z(n), z(ep * n), z(ep * n), z(ep * n),
                         torch.zeros((max(ep * n, 1), 128), dtype=torch.int64, device=self.device) if sigma else None)
        status = torch.zeros(max(n, 1), dtype=torch.int32, device=self.device)
        sc = C_.struct()
        self._check(self.lib.pvac_hip_enc_value_depth(self.ctx, n, C.c_void_p(values.data_ptr()),
                                                      C.c_void_p(rnd.data_ptr()), stride, int(depth), C.byref(sc),
                                                      ENC_WITH_SIGMA if sigma else 0, C.c_void_p(status.data_ptr())))
        return C_, status.cpu().numpy().view(np.uint32)[:n]

    def base_R(self, X: DeviceBatch):
        """prf_R of every BASE layer slot of X (device tensor, 2 int64 words per slot)."""
        torch = self.torch
        slots = int((X.l_off + X.l_cnt).max().item()) if X.n else 0
        R = torch.zeros(2 * max(slots, 1), dtype=torch.int64, device=self.device)
        sx = X.struct()
        self._check(self.lib.pvac_hip_base_R(self.ctx, C.byref(sx), C.c_void_p(R.data_ptr())))
        return R

    # ---- decryption (ops/decrypt.hpp:12-89)
    def set_powg(self, powg):
        """pk.powg_B: u64 array of B (lo, hi) pairs (host)."""
        a = np.ascontiguousarray(np.asarray(powg, dtype=np.uint64).reshape(-1))
        self._check(self.lib.pvac_hip_ctx_set_powg(self.ctx, C.c_void_p(a.ctypes.data), len(a) // 2))

    def dec_value(self, X: DeviceBatch, R_base):
        """R_base: 2 u64 per layer slot of X (host array or device tensor; BASE entries used).
        Returns (values: list[int], status: numpy u32 per cipher)."""
        torch = self.torch
        if isinstance(R_base, np.ndarray):
            R_base = _t(np.ascontiguousarray(R_base, np.uint64)).to(self.device)
        out = torch.zeros(2 * max(X.n, 1), dtype=torch.int64, device=self.device)
        status = torch.zeros(max(X.n, 1), dtype=torch.int32, device=self.device)
        sx = X.struct()
        self._check(self.lib.pvac_hip_dec_value(self.ctx, C.byref(sx), C.c_void_p(R_base.data_ptr()),
                                                C.c_void_p(out.data_ptr()), C.c_void_p(status.data_ptr())))
        o = out.cpu().numpy().view(np.uint64)
        vals = [int(o[2 * i]) | (int(o[2 * i + 1]) << 64) for i in range(X.n)]
        return vals, status.cpu().numpy().view(np.uint32)[: X.n]

    # ---- ciphertext ops
    def ct_mul_plan(self, A: DeviceBatch, B: DeviceBatch):
        torch = self.torch
        m = max(A.n, 1)
        # l_off, l_cnt, e_off, e_cnt: the plan kernel writes all four (capacities, zero counts)
        cnt = torch.empty(4 * m, dtype=torch.int64, device=self.device)
        C_ = DeviceBatch(A.n, cnt[:m], cnt[m:2 * m], None, cnt[2 * m:3 * m], cnt[3 * m:], None, None, None)
        plan = Plan()
        sa, sb, sc = A.struct(), B.struct(), C_.struct()
        self._check(self.lib.pvac_hip_ct_mul_plan(self.ctx, C.byref(sa), C.byref(sb), C.byref(sc), C.byref(plan)))
        return C_, plan

    def ct_mul(self, A: DeviceBatch, B: DeviceBatch, nonces=None, salts=None, flags=0, C_=None, plan=None,
               nonce_seed=None):
        """Batched ct_mul. nonces: device int64 tensor parallel to output layer slots (2 words each);
        if None, filled from a splitmix stream (nonce_seed) on the device."""
        torch = self.torch
        if C_ is None or plan is None:
            C_, plan = self.ct_mul_plan(A, B)
        if C_.layers is None:
            C_.layers = torch.empty((max(plan.total_layer_slots, 1), 5), dtype=torch.int64, device=self.device)
            e = max(plan.total_edge_slots, 1)
            C_.meta = torch.empty(e, dtype=torch.int64, device=self.device)
            C_.w_lo = torch.empty(e, dtype=torch.int64, device=self.device)
            C_.w_hi = torch.empty(e, dtype=torch.int64, device=self.device)
            if flags & MUL_WITH_SIGMA:
                C_.sigma = torch.empty((e, 128), dtype=torch.int64, device=self.device)
        if nonces is None:
            nonces = torch.empty(2 * max(plan.total_layer_slots, 1), dtype=torch.int64, device=self.device)
            self.fill_random(nonces, 0x5EED0003 if nonce_seed is None else nonce_seed)
        p = lambda t: None if t is None else C.c_void_p(t.data_ptr())
        sa, sb, sc = A.struct(), B.struct(), C_.struct()
        self._check(self.lib.pvac_hip_ct_mul_exec(self.ctx, C.byref(plan), C.byref(sa), C.byref(sb), p(nonces),
                                                  p(salts), C.byref(sc), flags))
        return C_

    def ct_mul_into(self, A: DeviceBatch, B: DeviceBatch, C_: DeviceBatch, nonces, salts=None, flags=0):
        """plan + exec in one call (pvac_hip_ct_mul) into C_, whose arrays were sized once (e.g. by
        ct_mul on a batch of the same shape); returns the plan."""
        cap_l = C_.layers.shape[0]
        cap_e = C_.meta.shape[0]
        p = lambda t: None if t is None else C.c_void_p(t.data_ptr())
        plan = Plan()
        sa, sb, sc = A.struct(), B.struct(), C_.struct()
        self._check(self.lib.pvac_hip_ct_mul(self.ctx, C.byref(sa), C.byref(sb), C.byref(sc), cap_l, cap_e,
                                             p(nonces), p(salts), flags, C.byref(plan)))
        return plan

    def ct_mul_step(self, A: DeviceBatch, B: DeviceBatch, C_: DeviceBatch, nonces, salts=None, flags=0):
        """ct_mul_into over fixed batches, its ctypes arguments built once: the returned function
        runs plan + exec (pvac_hip_ct_mul) per call and returns the plan (one object, refreshed by
        every call)."""
        p = lambda t: None if t is None else C.c_void_p(t.data_ptr())
        plan = Plan()
        sa, sb, sc = A.struct(), B.struct(), C_.struct()
        args = (self.ctx, C.byref(sa), C.byref(sb), C.byref(sc), C_.layers.shape[0], C_.meta.shape[0], p(nonces),
                p(salts), flags, C.byref(plan))
        fn, check = self.lib.pvac_hip_ct_mul, self._check
        keep = (sa, sb, sc, A, B, C_, nonces, salts)

        def run():
            rc = fn(*args)
            if rc:
                check(rc)
            return plan

        run.keep = keep
        return run

    def ct_mul_chain(self, X: DeviceBatch, depth, nonce_seed=0x5EED0040, streams=4, chunk=1024, check_gsum=False,
                     digest_n=0, canonical=False, fill_nonces=None, on_chunk=None, count_n=None, sigma=False,
                     devices=None, stage_inputs=False, nonces_at=None, after_step=None, salts_at=None,
                     sumdigest=False, operands=None, img_batch2=False):
        """c_0 = x, c_k = ct_mul(c_{k-1}, x) to `depth` for every input x of X (tests/test_main.cpp:289-295)
        on `streams` internal worker streams in chunks of `chunk` inputs (pvac_hip_ct_mul_chain).
        Returns a dict of the call's statistics; with digest_n > 0 also the final digests / edge
        counts of inputs [0, digest_n) (numpy u64). fill_nonces / on_chunk: optional ctypes callbacks
        (FILL_NONCES_CB / ON_CHUNK_CB), called from the library's worker threads. count_n: inputs whose
        final edge counts are returned (default digest_n; the FNV-1a digest walks a cipher's edges
        serially, a count is a copy). sigma: the final step with sigmas (needs H). devices: GPU
        ordinals, one contiguous range of whole chunks each (stage_inputs: ranges after the first copy
        their chunks to worker buffers even on this device). nonces_at / after_step / salts_at: STEP_CB
        hooks (include/pvac_hip.h). sumdigest: True (every input) or the number of leading inputs
        whose pvac_hip_batch_sumdigest is returned. operands: DeviceBatches of |X| ciphers, step d
        multiplying by operands[d] (the reference's loop with a fresh enc_value per step,
        tests/test_main.cpp:291-292), later steps by X. img_batch2: image conversions in launches of
        two pairs (tests)."""
        torch = self.torch
        dn = min(int(digest_n), X.n)
        cn = dn if count_n is None else min(int(count_n), X.n)
        dig = torch.zeros(max(dn, 1), dtype=torch.int64, device=self.device)
        cnt = torch.zeros(max(cn, 1), dtype=torch.int64, device=self.device)
        sn = min(X.n if sumdigest is True else int(sumdigest or 0), X.n)   # True: every input
        sdg = torch.zeros(max(sn, 1), dtype=torch.int64, device=self.device) if sn else None
        devs = (C.c_int * len(devices))(*devices) if devices else None
        ops = list(operands or [])
        for Y in ops:
            if Y.n != X.n:
                raise PvacError("ct_mul_chain: every operand batch needs |X| ciphers")
        op_structs = (CtBatch * len(ops))(*[Y.struct() for Y in ops]) if ops else None
        o = ChainOpts(depth=depth, streams=streams, chunk=chunk, nonce_seed=nonce_seed,
                      flags=(CHAIN_CHECK_GSUM if check_gsum else 0) | (MUL_ORDER_CANONICAL if canonical else 0) |
                      (MUL_WITH_SIGMA if sigma else 0) | (CHAIN_STAGE_INPUTS if stage_inputs else 0) |
                      (CHAIN_IMG_BATCH2 if img_batch2 else 0),
                      pad=0, digest_n=dn, digest_out=C.c_void_p(dig.data_ptr()) if dn else None,
                      count_n=cn, count_out=C.c_void_p(cnt.data_ptr()) if cn else None,
                      fill_nonces=fill_nonces or FILL_NONCES_CB(), on_chunk=on_chunk or ON_CHUNK_CB(), user=None,
                      nonces_at=nonces_at or STEP_CB(), after_step=after_step or STEP_CB(),
                      salts_at=salts_at or STEP_CB(), devices=C.cast(devs, C.c_void_p) if devs else None,
                      n_devices=len(devices) if devices else 0, pad2=0,
                      sumdigest_out=C.c_void_p(sdg.data_ptr()) if sdg is not None else None, sumdigest_n=sn,
                      operands=C.cast(op_structs, C.c_void_p) if ops else None, n_operands=len(ops), pad3=0)
        st = ChainStats()
        sx = X.struct()
        self._check(self.lib.pvac_hip_ct_mul_chain(self.ctx, C.byref(sx), C.byref(o), C.byref(st)))
        res = {"pair_steps": st.pair_steps, "edges": [st.edges[d] for d in range(depth)],
               "products": [st.products[d] for d in range(depth)], "gsum_pairs": st.gsum_pairs,
               "gsum_failed": st.gsum_failed, "redo": st.redo, "chunks": st.chunks, "seconds": st.seconds,
               "image_steps": st.image_steps}
        if dn:
            res["digests"] = dig[:dn].cpu().numpy().view(np.uint64).copy()
        if cn:
            res["counts"] = cnt[:cn].cpu().numpy().view(np.uint64).copy()
        if sdg is not None:
            res["sumdigests"] = sdg[:sn].cpu().numpy().view(np.uint64).copy()
        return res

    def ct_mul_redo_count(self):
        """Fresh-shape pairs re-run on the general path because a key sum was 0 mod p."""
        v = C.c_uint64(0)
        self._check(self.lib.pvac_hip_ct_mul_redo_count(self.ctx, C.byref(v)))
        return v.value

    def set_noise(self, noise_entropy_bits=120.0, tuple2_fraction=0.55, depth_slope_bits=16.0):
        """The reference Params' noise fields for enc_value's plan_noise (ops/encrypt.hpp:16-27)."""
        self._check(self.lib.pvac_hip_ctx_set_noise(self.ctx, float(noise_entropy_bits), float(tuple2_fraction),
                                                    float(depth_slope_bits)))

    def ct_mul_path_counts(self):
        """Pair launches by path since the context was created: {fresh, general, iblk, direct}."""
        v = (C.c_uint64 * 4)()
        self._check(self.lib.pvac_hip_ct_mul_path_count(self.ctx, v))
        return dict(zip(("fresh", "general", "iblk", "direct"), (int(x) for x in v)))

    def ct_mul_status(self, n):
        """Per-pair outcome of the last ct_mul (0 hash order, 1 canonical order, 2 rejected)."""
        out = self.torch.zeros(max(n, 1), dtype=self.torch.int32, device=self.device)
        self._check(self.lib.pvac_hip_ct_mul_status(self.ctx, C.c_void_p(out.data_ptr()), n))
        return out.cpu().numpy().view(np.uint32)[:n]

    def alu_ceiling(self, kind):
        """Measured ops/s: 0 wave64 integer VALU instructions, 1 fp_mul_fold1, 2 fp_mul products."""
        v = C.c_double(0)
        self._check(self.lib.pvac_hip_alu_ceiling(self.ctx, kind, C.byref(v)))
        return v.value

    ISSUE_OPS = ("v_add_u32", "v_xor_b32", "v_alignbit_b32", "v_lshlrev_b32", "v_min_u32", "v_add3_u32",
                 "v_pk_add_u16", "v_fma_f32", "v_mul_lo_u32", "v_mul_hi_u32", "v_cndmask_b32", "v_bfe_u32",
                 "v_add_co_u32", "v_and_or_b32", "v_pk_min_u16", "v_bitop3_b32", "v_mad_u64_u32",
                 "v_cndmask_b32_e64", "v_lshl_add_u32", "v_mov_b32_dpp", "v_perm_b32", "v_mul_u32_u24", "v_sub_u32",
                 "v_max3_u32", "v_cmp+v_cndmask_vcc", "v_cndmask_b32_e64_vcc", "v_addc_co_u32_vcc",
                 "v_addc_co_u32_e64_sgpr", "v_cmp_e64+v_cndmask_e64", "v_min_u32_e64", "v_add_u32_e64", "v_and_b32",
                 "v_or_b32", "v_lshrrev_b32", "v_mov_b32", "v_max_u32", "v_add_u32_sdwa", "v_lshlrev_b32_sdwa_src1",
                 "v_lshlrev_b32_sdwa_src0", "v_xor_b32_e64", "v_mad_u32_u24")

    def issue_probe(self, op, waves_per_simd=8):
        """Per-opcode VALU issue rate (pvac_hip_issue_probe): (wave64 inst/s chip-wide, shader clock Hz
        measured in the same launch). `op` is an index or a name of ISSUE_OPS."""
        if isinstance(op, str):
            op = self.ISSUE_OPS.index(op)
        v, hz = C.c_double(0), C.c_double(0)
        self._check(self.lib.pvac_hip_issue_probe(self.ctx, op, waves_per_simd, C.byref(v), C.byref(hz)))
        return v.value, hz.value

    def check_mul_gsum(self, A: DeviceBatch, B: DeviceBatch, C_: DeviceBatch, nonces, status=False):
        """The reference's gsum invariant (utils/metrics.hpp:88-113) on every pair of a ct_mul
        batch; needs set_powg. Returns the number of failing pairs (and per-pair status)."""
        torch = self.torch
        st = torch.zeros(max(A.n, 1), dtype=torch.int32, device=self.device) if status else None
        bad = C.c_uint64(0)
        sa, sb, sc = A.struct(), B.struct(), C_.struct()
        self._check(self.lib.pvac_hip_check_mul_gsum(self.ctx, C.byref(sa), C.byref(sb), C.byref(sc),
                                                     C.c_void_p(nonces.data_ptr()),
                                                     C.c_void_p(st.data_ptr()) if status else None, C.byref(bad)))
        if status:
            return bad.value, st.cpu().numpy().view(np.uint32)[:A.n]
        return bad.value

    def ct_add(self, A: DeviceBatch, B: DeviceBatch, negate=False, sigma=False):
        torch = self.torch
        n = A.n
        z = lambda: torch.zeros(max(n, 1), dtype=torch.int64, device=self.device)
        C_ = DeviceBatch(n, z(), z(), None, z(), z(), None, None, None)
        plan = Plan()
        sa, sb, sc = A.struct(), B.struct(), C_.struct()
        self._check(self.lib.pvac_hip_ct_add_plan(self.ctx, C.byref(sa), C.byref(sb), C.byref(sc), C.byref(plan)))
        e = max(plan.total_edge_slots, 1)
        C_.layers = torch.empty((max(plan.total_layer_slots, 1), 5), dtype=torch.int64, device=self.device)
        C_.meta = torch.empty(e, dtype=torch.int64, device=self.device)
        C_.w_lo = torch.empty(e, dtype=torch.int64, device=self.device)
        C_.w_hi = torch.empty(e, dtype=torch.int64, device=self.device)
        if sigma:
            C_.sigma = torch.empty((e, 128), dtype=torch.int64, device=self.device)
        sc = C_.struct()
        self._check(self.lib.pvac_hip_ct_add_exec(self.ctx, C.byref(plan), C.byref(sa), C.byref(sb), int(negate),
                                                  C.byref(sc)))
        return C_

    def ct_scale(self, X: DeviceBatch, s: int):
        sx = X.struct()
        self._check(self.lib.pvac_hip_ct_scale(self.ctx, C.byref(sx), s & ((1 << 64) - 1), s >> 64))
        return X

    def ct_neg(self, X: DeviceBatch):
        """ct_neg (ops/arithmetic.hpp:39-41): ct_scale by fp_neg(1) = p - 1, in place."""
        return self.ct_scale(X, (1 << 127) - 2)

    def fp_inv(self, k: int) -> int:
        """fp_inv (core/field.hpp:229-273) of one element on the device (PVAC_FP_INV); inv(0) = 0."""
        a = _t(np.array([k & ((1 << 64) - 1), (k >> 64) & ((1 << 64) - 1)], np.uint64)).to(self.device)
        lo, hi = self.fp_binop(FP_INV, a[0:1], a[1:2])
        o = np.concatenate([lo.cpu().numpy(), hi.cpu().numpy()]).view(np.uint64)
        return int(o[0]) | (int(o[1]) << 64)

    def ct_div_const(self, X: DeviceBatch, k: int):
        """ct_div_const (ops/arithmetic.hpp:108-110): ct_scale by fp_inv(k), in place."""
        return self.ct_scale(X, self.fp_inv(k))

    def sigma(self, X: DeviceBatch, salts):
        sx = X.struct()
        self._check(self.lib.pvac_hip_sigma_batch(self.ctx, C.byref(sx), C.c_void_p(salts.data_ptr())))
        return X

    def set_H(self, H_dense: np.ndarray):
        H = np.ascontiguousarray(H_dense, np.uint64)
        self._check(self.lib.pvac_hip_ctx_set_H(self.ctx, H.ctypes.data_as(C.c_void_p), H.shape[0], H.shape[1]))

    def gen_H(self) -> bytes:
        d = C.create_string_buffer(32)
        self._check(self.lib.pvac_hip_ctx_gen_H(self.ctx, d))
        return d.raw

    # ---- synthetic inputs / checks
    def fill_random(self, t, seed):
        self._check(self.lib.pvac_hip_fill_random(self.ctx, seed, C.c_void_p(t.data_ptr()), t.numel()))
        return t

    def gen_fresh(self, n, seed, edges_per_layer=20, first_index=0):
        """cfg-3 synthetic fresh-shaped ciphers; cipher i is keyed by global index first_index + i."""
        X = DeviceBatch.empty(n, 2 * n, 2 * edges_per_layer * n, self.device)
        sx = X.struct()
        self._check(self.lib.pvac_hip_gen_fresh_batch_at(self.ctx, seed, first_index, edges_per_layer, C.byref(sx)))
        return X

    def fill_nonces(self, A, B, C_, plan, seed, first_index=0):
        """Product-layer nonces keyed by (seed, global pair index, product layer) for a planned ct_mul."""
        out = self.torch.zeros(2 * max(plan.total_layer_slots, 1), dtype=self.torch.int64, device=self.device)
        sa, sb, sc = A.struct(), B.struct(), C_.struct()
        self._check(self.lib.pvac_hip_fill_nonces(self.ctx, seed, first_index, C.byref(sa), C.byref(sb), C.byref(sc),
                                                  C.c_void_p(out.data_ptr())))
        return out

    def digest(self, X: DeviceBatch):
        out = self.torch.empty(max(X.n, 1), dtype=self.torch.int64, device=self.device)
        sx = X.struct()
        self._check(self.lib.pvac_hip_batch_digest(self.ctx, C.byref(sx), C.c_void_p(out.data_ptr())))
        return out[:X.n]

    def sumdigest(self, X: DeviceBatch):
        """Position-keyed parallel digest per cipher (pvac_hip_batch_sumdigest)."""
        out = self.torch.empty(max(X.n, 1), dtype=self.torch.int64, device=self.device)
        sx = X.struct()
        self._check(self.lib.pvac_hip_batch_sumdigest(self.ctx, C.byref(sx), C.c_void_p(out.data_ptr())))
        return out[:X.n]

    def pack(self, X: DeviceBatch) -> DeviceBatch:
        """X's used rows back to back (pvac_hip_batch_pack): dense offsets, arrays of exactly the
        packed sizes (sigma kept when X has it)."""
        t = self.torch
        rows = lambda a: a.shape[0] if a is not None else 0
        sig = X.sigma is not None
        D = DeviceBatch.empty(X.n, rows(X.layers), rows(X.meta), self.device)
        if sig:
            D.sigma = t.empty_like(X.sigma)
        sx, sd = X.struct(), D.struct()
        tot = (C.c_uint64 * 2)()
        self._check(self.lib.pvac_hip_batch_pack(self.ctx, C.byref(sx), C.byref(sd), tot))
        nl, ne = int(tot[0]), int(tot[1])
        return DeviceBatch(X.n, D.l_off, D.l_cnt, D.layers[:nl], D.e_off, D.e_cnt, D.meta[:ne], D.w_lo[:ne],
                           D.w_hi[:ne], D.sigma[:ne] if sig else None)

    # ---- timing
    def timing(self, on=True):
        self._check(self.lib.pvac_hip_timing_enable(self.ctx, int(on)))

    def timing_get(self, name):
        ms, n = C.c_double(), C.c_uint64()
        self._check(self.lib.pvac_hip_timing_get(self.ctx, name.encode(), C.byref(ms), C.byref(n)))
        return ms.value, n.value

    def timing_reset(self):
        self._check(self.lib.pvac_hip_timing_reset(self.ctx))


__all__ = ["Engine", "DeviceBatch", "HostCipher", "PvacError", "LAYER_DT", "load_library", "FP_ADD", "FP_SUB",
           "FP_MUL", "FP_NEG", "FP_SCALE", "FP_INV", "MUL_WITH_SIGMA", "MUL_ORDER_CANONICAL", "CHAIN_CHECK_GSUM", "CHAIN_STAGE_INPUTS", "STEP_CB",
           "ChainOpts", "ChainStats", "FILL_NONCES_CB", "ON_CHUNK_CB"]
