"""TEST INFRASTRUCTURE ONLY -- ctypes view of the CPU checker (rse_oracle.c) and of
the reference's own compiled SIMD kernel (oracle/_ref/librse_ref.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module.  The shipped library never does (reed-solomon-erasure_amd/ has no path to
it), and a product call that reached this code would void every parity claim.

All shard arguments are numpy uint8 arrays.  GF(2^16) shards are uint8 arrays of
shape (n, 2): element j is bytes [2j] = coefficient of x, [2j+1] = constant
(galois_16.rs:49-51).  Lengths passed to the C side are in field elements.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None
_REF = None

_u8p = ctypes.POINTER(ctypes.c_uint8)
_szp = ctypes.POINTER(ctypes.c_size_t)


def build():
    """Compile liboracle.so (and _ref/librse_ref.so when /root/reference exists)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        L.oracle_gf8_mul.restype = ctypes.c_uint8
        L.oracle_gf8_mul.argtypes = [ctypes.c_uint8, ctypes.c_uint8]
        L.oracle_gf8_div.restype = ctypes.c_uint8
        L.oracle_gf8_div.argtypes = [ctypes.c_uint8, ctypes.c_uint8]
        L.oracle_gf8_exp.restype = ctypes.c_uint8
        L.oracle_gf8_exp.argtypes = [ctypes.c_uint8, ctypes.c_size_t]
        L.oracle_gf8_mul_slice.argtypes = [ctypes.c_uint8, _u8p, _u8p, ctypes.c_size_t]
        L.oracle_gf8_mul_slice_xor.argtypes = [ctypes.c_uint8, _u8p, _u8p, ctypes.c_size_t]
        L.oracle_gf16_mul.argtypes = [_u8p, _u8p, _u8p]
        L.oracle_gf16_add.argtypes = [_u8p, _u8p, _u8p]
        L.oracle_gf16_inverse.argtypes = [_u8p, _u8p]
        L.oracle_gf16_div.argtypes = [_u8p, _u8p, _u8p]
        L.oracle_gf16_exp.argtypes = [_u8p, ctypes.c_size_t, _u8p]
        L.oracle_matrix_invert.argtypes = [ctypes.c_int, _u8p, ctypes.c_size_t, _u8p]
        L.oracle_matrix_multiply.argtypes = [ctypes.c_int, _u8p, ctypes.c_size_t,
                                             ctypes.c_size_t, _u8p, ctypes.c_size_t, _u8p]
        L.oracle_codec_new.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_size_t,
                                       ctypes.POINTER(ctypes.c_void_p)]
        L.oracle_codec_free.argtypes = [ctypes.c_void_p]
        L.oracle_codec_matrix.restype = _u8p
        L.oracle_codec_matrix.argtypes = [ctypes.c_void_p]
        L.oracle_code_some_slices.argtypes = [ctypes.c_int, _u8p, ctypes.c_size_t,
                                              ctypes.c_size_t, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_size_t]
        for name in ("oracle_encode",):
            getattr(L, name).argtypes = [ctypes.c_void_p, ctypes.c_void_p, _szp, ctypes.c_size_t]
        L.oracle_encode_sep.argtypes = [ctypes.c_void_p, ctypes.c_void_p, _szp, ctypes.c_size_t,
                                        ctypes.c_void_p, _szp, ctypes.c_size_t]
        L.oracle_encode_single.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                           _szp, ctypes.c_size_t]
        L.oracle_encode_single_sep.argtypes = [ctypes.c_void_p, ctypes.c_size_t, _u8p,
                                               ctypes.c_size_t, ctypes.c_void_p, _szp,
                                               ctypes.c_size_t]
        L.oracle_verify.argtypes = [ctypes.c_void_p, ctypes.c_void_p, _szp, ctypes.c_size_t,
                                    ctypes.POINTER(ctypes.c_int)]
        L.oracle_verify_with_buffer.argtypes = [ctypes.c_void_p, ctypes.c_void_p, _szp,
                                                ctypes.c_size_t, ctypes.c_void_p, _szp,
                                                ctypes.c_size_t, ctypes.POINTER(ctypes.c_int)]
        L.oracle_reconstruct.argtypes = [ctypes.c_void_p, ctypes.c_void_p, _szp, _u8p,
                                         ctypes.c_size_t, ctypes.c_int]
        _LIB = L
    return _LIB


def ref_available():
    return os.path.exists(os.path.join(HERE, "_ref", "librse_ref.so"))


def ref():
    """The reference's compiled simd_c kernel + core.rs loop-order driver."""
    global _REF
    if _REF is None:
        L = ctypes.CDLL(os.path.join(HERE, "_ref", "librse_ref.so"))
        L.ref_gf8_mul_slice.argtypes = [ctypes.c_uint8, _u8p, _u8p, ctypes.c_size_t]
        L.ref_gf8_mul_slice_xor.argtypes = [ctypes.c_uint8, _u8p, _u8p, ctypes.c_size_t]
        L.ref_gf8_simd_bytes.restype = ctypes.c_size_t
        L.ref_gf8_simd_bytes.argtypes = [ctypes.c_size_t]
        L.ref_gf8_code_some_slices.argtypes = [_u8p, ctypes.c_size_t, ctypes.c_size_t,
                                               ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_size_t]
        if hasattr(L, "ref_gf8_code_repeat"):
            L.ref_gf8_code_repeat.argtypes = [_u8p, ctypes.c_size_t, ctypes.c_size_t,
                                              ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_size_t, ctypes.c_size_t]
        _REF = L
    return _REF


def _p(a: np.ndarray):
    assert a.dtype == np.uint8 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_u8p)


def _ptrs(arrs):
    return (ctypes.c_void_p * max(1, len(arrs)))(*[a.ctypes.data for a in arrs])


def _lens(arrs, field):
    es = 2 if field == 16 else 1
    return (ctypes.c_size_t * max(1, len(arrs)))(*[a.size // es for a in arrs])


# ------------------------------------------------------------------ scalars
def gf8_tables():
    log = np.zeros(256, np.uint8)
    exp = np.zeros(510, np.uint8)
    mul = np.zeros(256 * 256, np.uint8)
    low = np.zeros(256 * 16, np.uint8)
    high = np.zeros(256 * 16, np.uint8)
    lib().oracle_gf8_tables(_p(log), _p(exp), _p(mul), _p(low), _p(high))
    return log, exp, mul.reshape(256, 256), low.reshape(256, 16), high.reshape(256, 16)


def gf8_mul(a, b):
    return lib().oracle_gf8_mul(a, b)


def gf8_div(a, b):
    return lib().oracle_gf8_div(a, b)


def gf8_exp(a, n):
    return lib().oracle_gf8_exp(a, n)


def gf8_mul_slice(c, inp, out=None, xor=False):
    inp = np.ascontiguousarray(inp, np.uint8)
    out = np.zeros_like(inp) if out is None else out
    f = lib().oracle_gf8_mul_slice_xor if xor else lib().oracle_gf8_mul_slice
    f(c, _p(inp), _p(out), inp.size)
    return out


def _e(x):
    return np.array(x, np.uint8)


def gf16_mul(a, b):
    o = np.zeros(2, np.uint8)
    lib().oracle_gf16_mul(_p(_e(a)), _p(_e(b)), _p(o))
    return tuple(int(v) for v in o)


def gf16_add(a, b):
    o = np.zeros(2, np.uint8)
    lib().oracle_gf16_add(_p(_e(a)), _p(_e(b)), _p(o))
    return tuple(int(v) for v in o)


def gf16_inverse(a):
    o = np.zeros(2, np.uint8)
    rc = lib().oracle_gf16_inverse(_p(_e(a)), _p(o))
    if rc:
        raise ZeroDivisionError("Cannot invert 0")
    return tuple(int(v) for v in o)


def gf16_div(a, b):
    o = np.zeros(2, np.uint8)
    if lib().oracle_gf16_div(_p(_e(a)), _p(_e(b)), _p(o)):
        raise ZeroDivisionError("divide by 0")
    return tuple(int(v) for v in o)


def gf16_exp(a, n):
    o = np.zeros(2, np.uint8)
    lib().oracle_gf16_exp(_p(_e(a)), n, _p(o))
    return tuple(int(v) for v in o)


def matrix_invert(field, m):
    m = np.ascontiguousarray(m, np.uint8)
    n = m.shape[0]
    out = np.zeros_like(m)
    rc = lib().oracle_matrix_invert(field, _p(m), n, _p(out))
    if rc:
        raise ValueError("SingularMatrix")
    return out


def matrix_multiply(field, a, b):
    """matrix.rs:119-139.  GF(2^8): 2-D arrays; GF(2^16): (rows, cols, 2) arrays."""
    a = np.ascontiguousarray(a, np.uint8)
    b = np.ascontiguousarray(b, np.uint8)
    ar, ac, bc = a.shape[0], a.shape[1], b.shape[1]
    out = np.zeros((ar, bc, 2) if field == 16 else (ar, bc), np.uint8)
    lib().oracle_matrix_multiply(field, _p(a), ar, ac, _p(b), bc, _p(out))
    return out


def code_some_slices(field, rows, inputs, outputs):
    """core.rs:481-509 -- outputs[r] = sum_i rows[r][i] * inputs[i] (in place)."""
    rows = np.ascontiguousarray(rows, np.uint8)
    es = 2 if field == 16 else 1
    n_len = inputs[0].size // es
    lib().oracle_code_some_slices(field, _p(rows), len(outputs), len(inputs),
                                  _ptrs(inputs), _ptrs(outputs), n_len)
    return outputs


# ------------------------------------------------------------------- codec
class OracleError(Exception):
    def __init__(self, code):
        super().__init__(code)
        self.code = code


def _check(rc):
    if rc:
        raise OracleError(rc)


_SHARED = {}


class Codec:
    """Checker-side ReedSolomon<F> (core.rs:343-923), numpy shards in, in place."""

    def __init__(self, field, data_shards, parity_shards):
        self.field = field
        self.k, self.p = data_shards, parity_shards
        h = ctypes.c_void_p()
        _check(lib().oracle_codec_new(field, data_shards, parity_shards, ctypes.byref(h)))
        self._h = h

    @classmethod
    def shared(cls, field, data_shards, parity_shards):
        """One checker codec per shape per process: GF(2^16) past 256 shards
        inverts a ~1000 x 1000 matrix in scalar C (about a minute)."""
        key = (field, data_shards, parity_shards)
        c = _SHARED.get(key)
        if c is None:
            c = _SHARED[key] = cls(field, data_shards, parity_shards)
        return c

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and _LIB is not None:
            _LIB.oracle_codec_free(h)
            self._h = None

    @property
    def es(self):
        return 2 if self.field == 16 else 1

    def matrix(self):
        n = (self.k + self.p) * self.k * self.es
        buf = ctypes.string_at(lib().oracle_codec_matrix(self._h), n)
        m = np.frombuffer(buf, np.uint8).copy()
        if self.field == 16:
            return m.reshape(self.k + self.p, self.k, 2)
        return m.reshape(self.k + self.p, self.k)

    def encode(self, shards):
        _check(lib().oracle_encode(self._h, _ptrs(shards), _lens(shards, self.field), len(shards)))

    def encode_sep(self, data, parity):
        _check(lib().oracle_encode_sep(self._h, _ptrs(data), _lens(data, self.field), len(data),
                                       _ptrs(parity), _lens(parity, self.field), len(parity)))

    def encode_single(self, i, shards):
        _check(lib().oracle_encode_single(self._h, i, _ptrs(shards),
                                          _lens(shards, self.field), len(shards)))

    def encode_single_sep(self, i, single, parity):
        _check(lib().oracle_encode_single_sep(self._h, i, _p(single), single.size // self.es,
                                              _ptrs(parity), _lens(parity, self.field),
                                              len(parity)))

    def verify(self, shards):
        ok = ctypes.c_int(0)
        _check(lib().oracle_verify(self._h, _ptrs(shards), _lens(shards, self.field),
                                   len(shards), ctypes.byref(ok)))
        return bool(ok.value)

    def verify_with_buffer(self, shards, buffer):
        ok = ctypes.c_int(0)
        _check(lib().oracle_verify_with_buffer(self._h, _ptrs(shards), _lens(shards, self.field),
                                               len(shards), _ptrs(buffer),
                                               _lens(buffer, self.field), len(buffer),
                                               ctypes.byref(ok)))
        return bool(ok.value)

    def reconstruct(self, shards, present, data_only=False):
        pres = np.array([1 if x else 0 for x in present], np.uint8)
        _check(lib().oracle_reconstruct(self._h, _ptrs(shards), _lens(shards, self.field),
                                        _p(pres), len(shards), 1 if data_only else 0))


# ---------------------------------------------------------- synthetic data
_SM_GAMMA = np.uint64(0x9E3779B97F4A7C15)


def splitmix_bytes(seed: int, shard: int, nbytes: int) -> np.ndarray:
    """Deterministic shard bytes; identical to the device fill kernel
    (rse_util_fill_splitmix in the HIP library): 64-bit word w of shard s is
    mix(seed + s * 2^40 + w)  with mix = splitmix64's finaliser applied to
    (z + gamma), little-endian."""
    nwords = (nbytes + 7) // 8
    with np.errstate(over="ignore"):
        z = (np.uint64(seed) + np.uint64(shard) * np.uint64(1 << 40)
             + np.arange(nwords, dtype=np.uint64)) + _SM_GAMMA
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.view(np.uint8)[:nbytes].copy()
