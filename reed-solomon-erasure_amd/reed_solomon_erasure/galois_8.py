"""GF(2^8) backend (galois_8.rs): type aliases of the codec over the 8-bit field."""
from .core import ReedSolomon as _RS, ShardByShard as _SBS

FIELD = 8
ORDER = 256


class ReedSolomon(_RS):
    """``galois_8::ReedSolomon`` (galois_8.rs:50-51)."""

    FIELD = 8

    def __init__(self, data_shards: int, parity_shards: int):
        super().__init__(data_shards, parity_shards, field=8)


ShardByShard = _SBS
