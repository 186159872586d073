"""GF(2^16) backend (galois_16.rs): the codec over GF((2^8)^2).

Shards are uint8 tensors of shape (n, 2): element j = [coefficient of x,
constant] (galois_16.rs:49-51)."""
from .core import ReedSolomon as _RS, ShardByShard as _SBS

FIELD = 16
ORDER = 65536


class ReedSolomon(_RS):
    """``galois_16::ReedSolomon`` (galois_16.rs:54-55)."""

    FIELD = 16

    def __init__(self, data_shards: int, parity_shards: int):
        super().__init__(data_shards, parity_shards, field=16)


ShardByShard = _SBS
