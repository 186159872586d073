"""GF(2^8) backend (galois_8.rs): type aliases of the codec over the 8-bit field."""
from .core import ReedSolomon as _RS, ShardByShard as _SBS, _any_elems, _any_ptr, _any_stream, _lib, _raise

FIELD = 8
ORDER = 256


class ReedSolomon(_RS):
    """``galois_8::ReedSolomon`` (galois_8.rs:50-51)."""

    FIELD = 8

    def __init__(self, data_shards: int, parity_shards: int):
        super().__init__(data_shards, parity_shards, field=8)


ShardByShard = _SBS


def mul_slice(c: int, input, out) -> None:
    """galois_8::mul_slice (galois_8.rs:291-308): out = c * input.

    input/out may be device tensors (asynchronous on torch's current stream)
    or host memory -- CPU tensors or numpy arrays, as the reference's callers
    pass -- which go through the host pipeline and are done on return."""
    _mul(c, input, out, 0)


def mul_slice_xor(c: int, input, out) -> None:
    """galois_8::mul_slice_xor (galois_8.rs:310-327): out ^= c * input."""
    _mul(c, input, out, 1)


def _mul(c, input, out, xor):
    n = _any_elems(input, 8)
    if n != _any_elems(out, 8):  # lib.rs:100 assert_eq!
        raise ValueError("input and out must have the same length")
    _raise(_lib.rse_gf8_mul_slice(c & 0xFF, _any_ptr(input), _any_ptr(out), n, xor,
                                  _any_stream(input, out)))
