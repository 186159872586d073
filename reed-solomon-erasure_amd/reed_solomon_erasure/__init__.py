"""MI355X-native drop-in for the hot path of rust-rse/reed-solomon-erasure v6.

Mirrors the crate's public surface (src/lib.rs:36-45):

    from reed_solomon_erasure.galois_8 import ReedSolomon, ShardByShard
    from reed_solomon_erasure.galois_16 import ReedSolomon as ReedSolomon16
    from reed_solomon_erasure import Error, RSError, SBSError

Shards are torch CUDA (HIP) uint8 tensors resident in HBM; GF(2^16) shards have
shape (n, 2) ([u8;2] elements).  All arithmetic runs in librse_hip.so.
"""
from ._lib import load as _load
from .errors import DeviceError, Error, RSError, SBSError, SBSErrorKind

_load()  # fail at import time, loudly, if the HIP library is missing

from .core import ReedSolomon, ShardByShard  # noqa: E402
from . import galois_8, galois_16  # noqa: E402

__all__ = ["ReedSolomon", "ShardByShard", "Error", "RSError", "SBSError", "SBSErrorKind",
           "DeviceError", "galois_8", "galois_16"]
