"""GF(2^16) backend (galois_16.rs): the codec over GF((2^8)^2).

Shards are uint8 tensors of shape (n, 2): element j = [coefficient of x,
constant] (galois_16.rs:49-51)."""
import ctypes

from .core import ReedSolomon as _RS, ShardByShard as _SBS, _any_elems, _any_ptr, _any_stream, _lib, _raise

FIELD = 16
ORDER = 65536


class ReedSolomon(_RS):
    """``galois_16::ReedSolomon`` (galois_16.rs:54-55)."""

    FIELD = 16

    def __init__(self, data_shards: int, parity_shards: int):
        super().__init__(data_shards, parity_shards, field=16)


ShardByShard = _SBS


def mul_slice(c, input, out) -> None:
    """Field::mul_slice for galois_16 (the trait default, lib.rs:99-108):
    out = c * input; c = (coefficient of x, constant) or (c1 << 8) | c0.
    Device tensors or host memory (CPU tensors, numpy arrays), as galois_8.mul_slice."""
    _mul(c, input, out, 0)


def mul_slice_add(c, input, out) -> None:
    """Field::mul_slice_add (lib.rs:110-118): out += c * input."""
    _mul(c, input, out, 1)


def _mul(c, input, out, add):
    if isinstance(c, int):
        c = (c >> 8, c & 0xFF)
    n = _any_elems(input, 16)
    if n != _any_elems(out, 16):  # lib.rs:100 assert_eq!
        raise ValueError("input and out must have the same length")
    cb = (ctypes.c_uint8 * 2)(c[0] & 0xFF, c[1] & 0xFF)
    _raise(_lib.rse_gf16_mul_slice(cb, _any_ptr(input), _any_ptr(out), n, add,
                                   _any_stream(input, out)))
