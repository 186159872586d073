"""Error types of the reference (errors.rs:3-81), raised instead of returned.

Rust `Result<_, Error>` becomes a raised :class:`RSError` whose ``.error`` is an
:class:`Error` member; the numeric values are the C ABI codes (errors.rs:4-18
declaration order, as wasm/src/lib.rs:11-24 numbers them)."""
from __future__ import annotations

import enum


class Error(enum.IntEnum):
    TooFewShards = 1
    TooManyShards = 2
    TooFewDataShards = 3
    TooManyDataShards = 4
    TooFewParityShards = 5
    TooManyParityShards = 6
    TooFewBufferShards = 7
    TooManyBufferShards = 8
    IncorrectShardSize = 9
    TooFewShardsPresent = 10
    EmptyShard = 11
    InvalidShardFlags = 12
    InvalidIndex = 13

    def __str__(self):  # errors.rs:20-38
        return _MESSAGES[self]


_MESSAGES = {
    Error.TooFewShards: "The number of provided shards is smaller than the one in codec",
    Error.TooManyShards: "The number of provided shards is greater than the one in codec",
    Error.TooFewDataShards: "The number of provided data shards is smaller than the one in codec",
    Error.TooManyDataShards: "The number of provided data shards is greater than the one in codec",
    Error.TooFewParityShards: "The number of provided parity shards is smaller than the one in codec",
    Error.TooManyParityShards: "The number of provided parity shards is greater than the one in codec",
    Error.TooFewBufferShards: "The number of provided buffer shards is smaller than the number of parity shards in codec",
    Error.TooManyBufferShards: "The number of provided buffer shards is greater than the number of parity shards in codec",
    Error.IncorrectShardSize: "At least one of the provided shards is not of the correct size",
    Error.TooFewShardsPresent: "The number of shards present is smaller than number of parity shards, cannot reconstruct missing shards",
    Error.EmptyShard: "The first shard provided is of zero length",
    Error.InvalidShardFlags: "The number of flags does not match the total number of shards",
    Error.InvalidIndex: "The data shard index provided is greater or equal to the number of data shards in codec",
}


class SBSErrorKind(enum.Enum):  # errors.rs:53-68
    TooManyCalls = "Too many calls"
    LeftoverShards = "Leftover shards"
    RSError = "RSError"


class RSError(Exception):
    """A reference ``Error`` (errors.rs:4-18)."""

    def __init__(self, error: Error):
        super().__init__(str(error))
        self.error = error

    def __eq__(self, other):
        if isinstance(other, RSError):
            return self.error == other.error
        return self.error == other

    def __hash__(self):
        return hash(self.error)


class SBSError(Exception):
    """ShardByShard error (errors.rs:53-68): TooManyCalls, LeftoverShards or
    RSError(Error)."""

    def __init__(self, kind: SBSErrorKind, error: Error | None = None):
        super().__init__(str(error) if error is not None else kind.value)
        self.kind = kind
        self.error = error


class DeviceError(RuntimeError):
    """A library status >= 100 (HIP runtime failure, bad argument, OOM)."""

    def __init__(self, status: int, message: str, hip_error: int = 0):
        super().__init__(f"{message} (status {status}, hipError {hip_error})")
        self.status = status
        self.hip_error = hip_error
