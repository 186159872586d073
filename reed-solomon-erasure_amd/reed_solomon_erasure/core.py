"""``ReedSolomon<F>`` and ``ShardByShard`` (core.rs:49-924) over librse_hip.so.

Same method names, argument meaning and error behaviour as the reference, with
Rust ``Result`` errors raised as :class:`RSError`.  Shards are torch tensors in
HBM (``device='cuda'``); work is enqueued on torch's current stream, so results
are ordered with surrounding torch work exactly like any torch op.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from ._lib import load
from .errors import DeviceError, Error, RSError, SBSError, SBSErrorKind

_lib = load()

ShardList = Sequence[torch.Tensor]


def _raise(status: int):
    if status == 0:
        return
    if 1 <= status <= 13:
        raise RSError(Error(status))
    msg = _lib.rse_strerror(status).decode()
    raise DeviceError(status, msg, _lib.rse_last_device_error())


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _stream(t: Optional[torch.Tensor] = None):
    """torch's current stream on t's device (the current device for None or a
    host tensor), as the address the C ABI takes."""
    idx = t.get_device() if t is not None else -1
    if idx < 0:
        idx = torch.cuda.current_device()
    if _raw_stream is not None:  # ~0.3 us against ~2 for a torch.cuda.Stream object
        return _raw_stream(idx)
    return torch.cuda.current_stream(idx).cuda_stream


def _elems(t: torch.Tensor, field: int) -> int:
    """Rust slice length of a shard: bytes (GF(2^8)) or [u8;2] elements."""
    if t.dtype != torch.uint8:
        raise TypeError(f"shards must be uint8 tensors, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError("shards must be contiguous")
    if field == 8:
        return t.numel()
    if t.dim() >= 2 and t.shape[-1] == 2:
        return t.numel() // 2
    if t.dim() == 1 and t.numel() % 2 == 0:
        return t.numel() // 2
    raise ValueError("GF(2^16) shards are uint8 tensors of shape (n, 2)")


def _dev(t: torch.Tensor) -> int:
    if not t.is_cuda:
        raise ValueError("shards must be device (HBM) tensors; use encode_host() for host memory")
    return t.data_ptr()


def _settle(t: Optional[torch.Tensor]) -> None:
    """Waits for torch's current stream on t's device (the *_now entries are
    not stream-ordered: the shards' writers must have finished)."""
    idx = t.get_device() if t is not None else -1
    st = torch.cuda.current_stream(idx if idx >= 0 else None)
    if not st.query():
        st.synchronize()


def _check_flat(stripes: torch.Tensor, shard_len: int, n_stripes: int, total: int,
                field: int) -> None:
    """The flat calls take a base pointer: refuse a buffer the stripes overrun."""
    if stripes.dtype != torch.uint8 or not stripes.is_contiguous():
        raise ValueError("stripes must be a contiguous uint8 tensor")
    need = n_stripes * total * shard_len * (field // 8)
    if stripes.numel() < need:
        raise ValueError(f"stripes holds {stripes.numel()} bytes, {need} needed")


_U8 = torch.uint8


def _arrays(shards, field):
    """The shards' device addresses and Rust slice lengths as C arrays.  One
    pass over plain 1-D GF(2^8) device shards (the per-call cost of a
    synchronous verify); anything else, including every invalid shard, goes
    through _dev / _elems, whose errors are the API's."""
    n = len(shards)
    if field == 8:
        ptrs, lens = [], []
        for s in shards:
            if s.dtype is not _U8 or not s.is_cuda or not s.is_contiguous():
                break
            ptrs.append(s.data_ptr())
            lens.append(s.numel())
        else:
            return (ctypes.c_void_p * max(1, n))(*ptrs), (ctypes.c_size_t * max(1, n))(*lens)
    ptrs = (ctypes.c_void_p * max(1, n))(*[_dev(s) for s in shards])
    lens = (ctypes.c_size_t * max(1, n))(*[_elems(s, field) for s in shards])
    return ptrs, lens


class ReedSolomon:
    """Reed-Solomon erasure code encoder/decoder (core.rs:343-350).

    ``field`` is 8 (galois_8) or 16 (galois_16); prefer the aliases
    ``galois_8.ReedSolomon`` / ``galois_16.ReedSolomon``.
    """

    def __init__(self, data_shards: int, parity_shards: int, field: int = 8):
        if field not in (8, 16):
            raise ValueError("field must be 8 or 16")
        h = ctypes.c_void_p()
        _raise(_lib.rse_codec_new(field, data_shards, parity_shards, ctypes.byref(h)))
        self._h = h
        self.field = field
        self._k, self._p = data_shards, parity_shards

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            _lib.rse_codec_free(h)
            self._h = None

    # core.rs:352-364
    def clone(self) -> "ReedSolomon":
        other = ReedSolomon(self._k, self._p, self.field)
        other.__class__ = type(self)
        return other

    def __eq__(self, rhs) -> bool:
        return (isinstance(rhs, ReedSolomon) and self.field == rhs.field
                and self._k == rhs._k and self._p == rhs._p)

    def __repr__(self):
        return f"ReedSolomon<GF(2^{self.field})>({self._k}, {self._p})"

    # core.rs:469-479
    def data_shard_count(self) -> int:
        return self._k

    def parity_shard_count(self) -> int:
        return self._p

    def total_shard_count(self) -> int:
        return self._k + self._p

    # rse_codec_kernel_kind values (include/rse_hip.h); no reference counterpart
    KERNELS = {0: "table", 1: "bitslice-compiled", 2: "bitslice-specialised",
               3: "specialising", 4: "specialise-failed", 5: "fft-compiled"}

    def kernel_kind(self, wait: bool = False) -> str:
        """Which kernels code this codec (results are identical either way):
        bit-sliced kernels compiled into the library, bit-sliced kernels
        specialised for this codec at run time (hiprtc; the build starts at the
        first call that codes a whole 4 KiB chunk, or here with ``wait``, which
        blocks until it has finished), or the table kernels."""
        return self.KERNELS[_lib.rse_codec_kernel_kind(self._h, 1 if wait else 0)]

    def matrix(self) -> "list":
        """The (k+p) x k systematic encoding matrix (core.rs:430-436) as nested
        lists of ints (GF(2^16): (coef_of_x << 8) | constant)."""
        es = 2 if self.field == 16 else 1
        n = (self._k + self._p) * self._k * es
        buf = (ctypes.c_uint8 * n)()
        _raise(_lib.rse_codec_matrix(self._h, buf, n))
        b = bytes(buf)
        rows = []
        for r in range(self._k + self._p):
            row = []
            for c in range(self._k):
                o = (r * self._k + c) * es
                row.append(b[o] << 8 | b[o + 1] if es == 2 else b[o])
            rows.append(row)
        return rows

    # ------------------------------------------------------------- encode
    def encode(self, shards: ShardList) -> None:
        """core.rs:597-611: overwrite shards[k:] with the parity of shards[:k]."""
        ptrs, lens = _arrays(shards, self.field)
        _raise(_lib.rse_encode(self._h, ptrs, lens, len(shards), _stream(_first(shards))))

    def encode_sep(self, data: ShardList, parity: ShardList) -> None:
        """core.rs:617-632."""
        dp, dl = _arrays(data, self.field)
        pp, pl = _arrays(parity, self.field)
        _raise(_lib.rse_encode_sep(self._h, dp, dl, len(data), pp, pl, len(parity),
                                   _stream(_first(data))))

    def encode_single(self, i_data: int, shards: ShardList) -> None:
        """core.rs:545-562 (i_data == 0 overwrites parity, later ones accumulate)."""
        if i_data < 0:
            raise RSError(Error.InvalidIndex)
        ptrs, lens = _arrays(shards, self.field)
        _raise(_lib.rse_encode_single(self._h, i_data, ptrs, lens, len(shards),
                                      _stream(_first(shards))))

    def encode_single_sep(self, i_data: int, single_data: torch.Tensor,
                          parity: ShardList) -> None:
        """core.rs:576-592."""
        if i_data < 0:
            raise RSError(Error.InvalidIndex)
        pp, pl = _arrays(parity, self.field)
        _raise(_lib.rse_encode_single_sep(self._h, i_data, _dev(single_data),
                                          _elems(single_data, self.field), pp, pl, len(parity),
                                          _stream(single_data)))

    # ------------------------------------------------------------- verify
    def verify(self, shards: ShardList) -> bool:
        """core.rs:637-651."""
        ptrs, lens = _arrays(shards, self.field)
        ok = ctypes.c_int(0)
        _raise(_lib.rse_verify(self._h, ptrs, lens, len(shards), ctypes.byref(ok),
                               _stream(_first(shards))))
        return bool(ok.value)

    def verify_with_buffer(self, shards: ShardList, buffer: ShardList) -> bool:
        """core.rs:654-669: on success `buffer` holds the correct parity."""
        ptrs, lens = _arrays(shards, self.field)
        bp, bl = _arrays(buffer, self.field)
        ok = ctypes.c_int(0)
        _raise(_lib.rse_verify_with_buffer(self._h, ptrs, lens, len(shards), bp, bl, len(buffer),
                                           ctypes.byref(ok), _stream(_first(shards))))
        return bool(ok.value)

    # -------------------------------------------------------- reconstruct
    def reconstruct(self, shards: list) -> None:
        """core.rs:680-682.  `shards` is either a list of Optional[tensor]
        (Option<T>, lib.rs:126-166: None = missing, filled in place with a new
        tensor) or a list of (tensor, present) tuples ((T, bool), lib.rs:168-200:
        missing buffers are overwritten)."""
        self._reconstruct(shards, data_only=False)

    def reconstruct_data(self, shards: list) -> None:
        """core.rs:693-695: only the data shards are rebuilt."""
        self._reconstruct(shards, data_only=True)

    def _reconstruct(self, shards: list, data_only: bool, now: bool = False) -> None:
        if len(shards) < self.total_shard_count():
            raise RSError(Error.TooFewShards)
        if len(shards) > self.total_shard_count():
            raise RSError(Error.TooManyShards)
        flagged = len(shards) > 0 and all(isinstance(s, tuple) for s in shards)
        if flagged:
            bufs = [s[0] for s in shards]
            present = [bool(s[1]) for s in shards]
        else:
            bufs = list(shards)
            present = [s is not None for s in shards]
            # Option<T> semantics: run the checks of core.rs:744-772 before
            # allocating anything, then allocate zeroed missing shards
            # (lib.rs:151-165; parity only when not data_only, core.rs:805-806).
            shard_len, n_present, like = None, 0, None
            for s in bufs:
                if s is None:
                    continue
                n = _elems(s, self.field)
                if n == 0:
                    raise RSError(Error.EmptyShard)
                n_present += 1
                if shard_len is not None and n != shard_len:
                    raise RSError(Error.IncorrectShardSize)
                shard_len, like = n, s
            if n_present == self.total_shard_count():
                return
            if n_present < self._k:
                raise RSError(Error.TooFewShardsPresent)
            for i, s in enumerate(bufs):
                if s is None and (i < self._k or not data_only):
                    shape = (shard_len,) if self.field == 8 else (shard_len, 2)
                    bufs[i] = torch.zeros(shape, dtype=torch.uint8, device=like.device)
        n = len(bufs)
        ptrs = (ctypes.c_void_p * max(1, n))(
            *[(_dev(b) if b is not None else None) for b in bufs])
        lens = (ctypes.c_size_t * max(1, n))(
            *[(_elems(b, self.field) if b is not None else 0) for b in bufs])
        pres = (ctypes.c_uint8 * max(1, n))(*[1 if p else 0 for p in present])
        like = next((b for b in bufs if b is not None), None)
        if now:
            _settle(like)
            fn = _lib.rse_reconstruct_data_now if data_only else _lib.rse_reconstruct_now
            _raise(fn(self._h, ptrs, lens, pres, n))
        else:
            fn = _lib.rse_reconstruct_data if data_only else _lib.rse_reconstruct
            _raise(fn(self._h, ptrs, lens, pres, n, _stream(like)))
        if not flagged:
            for i in range(n):
                shards[i] = bufs[i]

    # ------------------------------------------------- synchronous forms
    # The reference's methods return when done (core.rs:597-695); these do
    # too: torch's current stream is waited for (the shards' writers), then
    # the *_now entry codes the stripe -- small stripes on the resident
    # dispatcher, no kernel launch -- and returns with the result in place.
    def encode_now(self, shards: ShardList) -> None:
        """encode() (core.rs:597-611), returning when the parity is written.

        The *_now calls on small shards run on a resident kernel that stays
        up RSE_OPT_DISPATCH_IDLE_US (200 us) after the last call: streams are
        not held up by it, but a device-wide synchronisation right after a
        call (torch.cuda.synchronize()) waits until it idles out; call
        ``reed_solomon_erasure.core.dispatcher_stop()`` first to end it at once."""
        ptrs, lens = _arrays(shards, self.field)
        _settle(_first(shards))
        _raise(_lib.rse_encode_now(self._h, ptrs, lens, len(shards)))

    def verify_now(self, shards: ShardList) -> bool:
        """verify() (core.rs:637-651) through rse_verify_now."""
        ptrs, lens = _arrays(shards, self.field)
        ok = ctypes.c_int(0)
        _settle(_first(shards))
        _raise(_lib.rse_verify_now(self._h, ptrs, lens, len(shards), ctypes.byref(ok)))
        return bool(ok.value)

    def reconstruct_now(self, shards: list) -> None:
        """reconstruct() (core.rs:680-682), returning when the shards are rebuilt."""
        self._reconstruct(shards, data_only=False, now=True)

    def reconstruct_data_now(self, shards: list) -> None:
        """reconstruct_data() (core.rs:693-695), returning when the data is rebuilt."""
        self._reconstruct(shards, data_only=True, now=True)

    # ------------------------------------------------ beyond the reference
    def encode_flat(self, stripes: torch.Tensor, shard_len: int, n_stripes: int = 1) -> None:
        """Encode `n_stripes` consecutive stripes of k+p shards of `shard_len`
        elements each, laid out as wasm/src/lib.rs:45-55's flat buffer."""
        _check_flat(stripes, shard_len, n_stripes, self.total_shard_count(), self.field)
        _raise(_lib.rse_encode_flat(self._h, _dev(stripes), shard_len, n_stripes,
                                    _stream(stripes)))

    def verify_flat(self, stripes: torch.Tensor, shard_len: int, n_stripes: int = 1) -> np.ndarray:
        """verify() (core.rs:637-651) of every stripe of the flat layout in one
        pass; returns one bool per stripe.  Synchronous, like verify()."""
        _check_flat(stripes, shard_len, n_stripes, self.total_shard_count(), self.field)
        ok = np.zeros(max(1, n_stripes), np.uint8)
        _raise(_lib.rse_verify_flat(self._h, _dev(stripes), shard_len, n_stripes,
                                    ok.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)),
                                    _stream(stripes)))
        return ok[:n_stripes].astype(bool)

    def reconstruct_data_flat(self, stripes: torch.Tensor, shard_len: int, n_stripes: int,
                              present: Sequence[bool]) -> None:
        """wasm/src/lib.rs:57-73 over many stripes sharing one erasure pattern."""
        pres = (ctypes.c_uint8 * len(present))(*[1 if p else 0 for p in present])
        if len(present) != self.total_shard_count():
            raise RSError(Error.InvalidShardFlags)
        _check_flat(stripes, shard_len, n_stripes, self.total_shard_count(), self.field)
        _raise(_lib.rse_reconstruct_data_flat(self._h, _dev(stripes), shard_len, n_stripes,
                                              pres, _stream(stripes)))

    def reconstruct_batch(self, stripes: torch.Tensor, shard_len: int, n_stripes: int,
                          present, data_only: bool = False) -> None:
        """reconstruct (or reconstruct_data) of `n_stripes` flat stripes, each
        with its OWN erasure pattern: `present` is n_stripes x (k+p) flags.
        Per-stripe planning (core.rs:733-923) runs as a HIP kernel.  A
        contiguous bool / uint8 device tensor of flags is read in place."""
        T = self.total_shard_count()
        if isinstance(present, torch.Tensor) and present.is_cuda:
            if (tuple(present.shape) != (n_stripes, T) or not present.is_contiguous()
                    or present.dtype not in (torch.bool, torch.uint8)
                    or present.device != stripes.device):  # read in place, on that device
                raise RSError(Error.InvalidShardFlags)
            _check_flat(stripes, shard_len, n_stripes, T, self.field)
            _raise(_lib.rse_reconstruct_batch(
                self._h, _dev(stripes), shard_len, n_stripes,
                ctypes.cast(present.data_ptr(), ctypes.POINTER(ctypes.c_uint8)),
                1 if data_only else 0, _stream(stripes)))
            return
        flags = np.ascontiguousarray(np.asarray(
            present.cpu() if isinstance(present, torch.Tensor) else present, dtype=bool))
        if flags.shape != (n_stripes, T):
            raise RSError(Error.InvalidShardFlags)
        _check_flat(stripes, shard_len, n_stripes, T, self.field)
        pres = flags.view(np.uint8)  # bool is one byte, 0 or 1: no copy
        _raise(_lib.rse_reconstruct_batch(
            self._h, _dev(stripes), shard_len, n_stripes,
            pres.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), 1 if data_only else 0,
            _stream(stripes)))

    # ---------------------------------------------- host memory (end to end)
    # The reference's own form: shards are slices in HOST memory (numpy arrays
    # or CPU tensors; pinned memory gives overlapped DMA).  Each call pipelines
    # chunks through the GPU and returns with the results in host memory.
    def encode_host(self, shards: Sequence) -> None:
        """encode() (core.rs:597-611) of host shards."""
        pa, la = _host_arrays(shards, self.field)
        _raise(_lib.rse_encode_host(self._h, pa, la, len(shards), _stream()))

    def encode_sep_host(self, data: Sequence, parity: Sequence) -> None:
        """encode_sep() (core.rs:617-632) of host shards."""
        dp, dl = _host_arrays(data, self.field)
        pp, pl = _host_arrays(parity, self.field)
        _raise(_lib.rse_encode_sep_host(self._h, dp, dl, len(data), pp, pl, len(parity), _stream()))

    def encode_single_host(self, i_data: int, shards: Sequence) -> None:
        """encode_single() (core.rs:545-562) of host shards."""
        if i_data < 0:
            raise RSError(Error.InvalidIndex)
        pa, la = _host_arrays(shards, self.field)
        _raise(_lib.rse_encode_single_host(self._h, i_data, pa, la, len(shards), _stream()))

    def encode_single_sep_host(self, i_data: int, single, parity: Sequence) -> None:
        """encode_single_sep() (core.rs:576-592) of host shards."""
        if i_data < 0:
            raise RSError(Error.InvalidIndex)
        pp, pl = _host_arrays(parity, self.field)
        _raise(_lib.rse_encode_single_sep_host(self._h, i_data, _host_ptr(single),
                                               _host_elems(single, self.field), pp, pl,
                                               len(parity), _stream()))

    def verify_host(self, shards: Sequence) -> bool:
        """verify() (core.rs:637-651) of host shards."""
        pa, la = _host_arrays(shards, self.field)
        ok = ctypes.c_int(0)
        _raise(_lib.rse_verify_host(self._h, pa, la, len(shards), ctypes.byref(ok), _stream()))
        return bool(ok.value)

    def verify_with_buffer_host(self, shards: Sequence, buffer: Sequence) -> bool:
        """verify_with_buffer() (core.rs:654-669) of host shards into a host buffer."""
        pa, la = _host_arrays(shards, self.field)
        ba, bl = _host_arrays(buffer, self.field)
        ok = ctypes.c_int(0)
        _raise(_lib.rse_verify_with_buffer_host(self._h, pa, la, len(shards), ba, bl, len(buffer),
                                                ctypes.byref(ok), _stream()))
        return bool(ok.value)

    def reconstruct_host(self, shards: list) -> None:
        """reconstruct() (core.rs:680-682) of host shards: Option (None =
        missing, filled with a new host array) or (array, present) tuples."""
        self._reconstruct_host(shards, data_only=False)

    def reconstruct_data_host(self, shards: list) -> None:
        """reconstruct_data() (core.rs:693-695) of host shards."""
        self._reconstruct_host(shards, data_only=True)

    def _reconstruct_host(self, shards: list, data_only: bool) -> None:
        T = self.total_shard_count()
        if len(shards) < T:
            raise RSError(Error.TooFewShards)
        if len(shards) > T:
            raise RSError(Error.TooManyShards)
        flagged = len(shards) > 0 and all(isinstance(s, tuple) for s in shards)
        if flagged:
            bufs = [s[0] for s in shards]
            present = [bool(s[1]) for s in shards]
        else:
            bufs = list(shards)
            present = [s is not None for s in shards]
            lens = [_host_elems(s, self.field) for s in bufs if s is not None]
            # core.rs:744-772 before allocating (lib.rs:151-165)
            for n in lens:
                if n == 0:
                    raise RSError(Error.EmptyShard)
                if n != lens[0]:
                    raise RSError(Error.IncorrectShardSize)
            if len(lens) == T:
                return
            if len(lens) < self._k:
                raise RSError(Error.TooFewShardsPresent)
            like = next(s for s in bufs if s is not None)
            for i, s in enumerate(bufs):
                if s is None and (i < self._k or not data_only):
                    bufs[i] = (np.zeros(like.shape, np.uint8) if isinstance(like, np.ndarray)
                               else torch.zeros(like.shape, dtype=torch.uint8))
        n = len(bufs)
        ptrs = (ctypes.c_void_p * max(1, n))(*[_host_ptr(b) if b is not None else None for b in bufs])
        lens = (ctypes.c_size_t * max(1, n))(
            *[_host_elems(b, self.field) if b is not None else 0 for b in bufs])
        pres = (ctypes.c_uint8 * max(1, n))(*[1 if p else 0 for p in present])
        fn = _lib.rse_reconstruct_data_host if data_only else _lib.rse_reconstruct_host
        _raise(fn(self._h, ptrs, lens, pres, n, _stream()))
        if not flagged:
            for i in range(n):
                shards[i] = bufs[i]

    def encode_host_flat(self, stripes, shard_len: int, n_stripes: int) -> None:
        """encode_flat() for a HOST buffer: one H2D / kernel / D2H pipeline
        across all stripes."""
        _check_host_flat(stripes, shard_len, n_stripes, self.total_shard_count(), self.field)
        _raise(_lib.rse_encode_host_flat(self._h, _host_ptr(stripes), shard_len, n_stripes,
                                         _stream()))

    def verify_host_flat(self, stripes, shard_len: int, n_stripes: int) -> np.ndarray:
        """verify_flat() of a HOST buffer; one bool per stripe."""
        _check_host_flat(stripes, shard_len, n_stripes, self.total_shard_count(), self.field)
        ok = np.zeros(max(1, n_stripes), np.uint8)
        _raise(_lib.rse_verify_host_flat(self._h, _host_ptr(stripes), shard_len, n_stripes,
                                         ok.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)),
                                         _stream()))
        return ok[:n_stripes].astype(bool)

    def reconstruct_host_batch(self, stripes, shard_len: int, n_stripes: int, present,
                               data_only: bool = False) -> None:
        """reconstruct_batch() of a HOST buffer: every stripe its own pattern."""
        T = self.total_shard_count()
        flags = np.ascontiguousarray(np.asarray(
            present.cpu() if isinstance(present, torch.Tensor) else present, dtype=bool))
        if flags.shape != (n_stripes, T):
            raise RSError(Error.InvalidShardFlags)
        _check_host_flat(stripes, shard_len, n_stripes, T, self.field)
        pres = flags.view(np.uint8)  # bool is one byte, 0 or 1: no copy
        _raise(_lib.rse_reconstruct_host_batch(
            self._h, _host_ptr(stripes), shard_len, n_stripes,
            pres.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), 1 if data_only else 0, _stream()))


def _first(shards):
    return shards[0] if len(shards) else None


def _host_ptr(s) -> int:
    """Address of a host shard: a CPU tensor or a contiguous uint8 numpy array."""
    if isinstance(s, torch.Tensor):
        if s.is_cuda:
            raise ValueError("the *_host calls take host memory")
        if s.dtype != torch.uint8 or not s.is_contiguous():
            raise ValueError("host shards must be contiguous uint8")
        return s.data_ptr()
    if s.dtype.itemsize != 1 or not s.flags["C_CONTIGUOUS"]:
        raise ValueError("host shards must be contiguous uint8 arrays")
    return s.ctypes.data


def _host_elems(s, field: int) -> int:
    if isinstance(s, torch.Tensor):
        _host_ptr(s)
        return _elems(s, field)
    n = s.size
    return n if field == 8 else n // 2


def _any_ptr(s) -> int:
    """Address of a shard wherever it lives: a device tensor, a CPU tensor or a
    numpy array (the Field/FFI slice hooks route by memory type)."""
    if isinstance(s, torch.Tensor) and s.is_cuda:
        _elems(s, 8)
        return s.data_ptr()
    return _host_ptr(s)


def _any_elems(s, field: int) -> int:
    if isinstance(s, torch.Tensor) and s.is_cuda:
        return _elems(s, field)
    return _host_elems(s, field)


def _any_stream(*bufs):
    """torch's current stream of the first device buffer, else of the current device."""
    for b in bufs:
        if isinstance(b, torch.Tensor) and b.is_cuda:
            return _stream(b)
    return _stream()


def _host_arrays(shards, field):
    n = len(shards)
    pa = (ctypes.c_void_p * max(1, n))(*[_host_ptr(s) for s in shards])
    la = (ctypes.c_size_t * max(1, n))(*[_host_elems(s, field) for s in shards])
    return pa, la


def _check_host_flat(stripes, shard_len: int, n_stripes: int, total: int, field: int) -> None:
    _host_ptr(stripes)
    size = stripes.numel() if isinstance(stripes, torch.Tensor) else stripes.size
    need = n_stripes * total * shard_len * (field // 8)
    if size < need:
        raise ValueError(f"stripes holds {size} bytes, {need} needed")


class ShardByShard:
    """Bookkeeper for shard-by-shard encoding (core.rs:49-231)."""

    def __init__(self, codec: ReedSolomon):
        self.codec = codec
        self.cur_input = 0

    def parity_ready(self) -> bool:  # core.rs:117-119
        return self.cur_input == self.codec.data_shard_count()

    def reset(self) -> None:  # core.rs:128-136
        if self.cur_input > 0 and not self.parity_ready():
            raise SBSError(SBSErrorKind.LeftoverShards)
        self.cur_input = 0

    def reset_force(self) -> None:  # core.rs:139-141
        self.cur_input = 0

    def cur_input_index(self) -> int:  # core.rs:144-146
        return self.cur_input

    def _checks(self, fn):
        if self.parity_ready():
            raise SBSError(SBSErrorKind.TooManyCalls)
        try:
            fn()
        except RSError as e:
            raise SBSError(SBSErrorKind.RSError, e.error) from None

    def encode(self, shards: ShardList) -> None:  # core.rs:201-212
        c = self.codec

        def checks():
            n = len(shards)
            if n < c.total_shard_count():
                raise RSError(Error.TooFewShards)
            if n > c.total_shard_count():
                raise RSError(Error.TooManyShards)
            _check_multi([_elems(s, c.field) for s in shards])

        self._checks(checks)
        c.encode_single(self.cur_input, shards)
        self.cur_input += 1

    def encode_sep(self, data: ShardList, parity: ShardList) -> None:  # core.rs:218-230
        c = self.codec

        def checks():
            if len(data) < c.data_shard_count():
                raise RSError(Error.TooFewDataShards)
            if len(data) > c.data_shard_count():
                raise RSError(Error.TooManyDataShards)
            if len(parity) < c.parity_shard_count():
                raise RSError(Error.TooFewParityShards)
            if len(parity) > c.parity_shard_count():
                raise RSError(Error.TooManyParityShards)
            dl = [_elems(s, c.field) for s in data]
            pl = [_elems(s, c.field) for s in parity]
            _check_multi(dl)
            _check_multi(pl)
            if dl[0] != pl[0]:
                raise RSError(Error.IncorrectShardSize)

        self._checks(checks)
        c.encode_single_sep(self.cur_input, data[self.cur_input], parity)
        self.cur_input += 1


def _check_multi(lens: List[int]) -> None:  # macros.rs:144-155
    if lens[0] == 0:
        raise RSError(Error.EmptyShard)
    for n in lens:
        if n != lens[0]:
            raise RSError(Error.IncorrectShardSize)


def _row_bytes(field: int, rows, n_out: int, n_in: int) -> List[int]:
    flat = []
    for r in range(n_out):
        for i in range(n_in):
            v = int(rows[r][i])
            flat += [v >> 8, v & 0xFF] if field == 16 else [v & 0xFF]
    return flat


def _same_len(lens: List[int]) -> int:
    """The C entry takes one length for every input and output: refuse a
    shorter buffer before the library reads or writes past its end (the
    reference's mul_slice asserts equal lengths, lib.rs:100)."""
    if not lens:
        return 0
    if any(n != lens[0] for n in lens):
        raise RSError(Error.IncorrectShardSize)
    return lens[0]


def code_shards(field: int, rows, inputs: ShardList, outputs: ShardList,
                accumulate: bool = False) -> None:
    """The fused kernel itself: outputs[r] (+)= sum_i rows[r][i] * inputs[i]
    (core.rs:481-509 code_some_slices when accumulate is False)."""
    n_out, n_in = len(outputs), len(inputs)
    flat = _row_bytes(field, rows, n_out, n_in)
    rb = (ctypes.c_uint8 * max(1, len(flat)))(*flat)
    ip = (ctypes.c_void_p * max(1, n_in))(*[_dev(t) for t in inputs])
    op = (ctypes.c_void_p * max(1, n_out))(*[_dev(t) for t in outputs])
    n = _same_len([_elems(t, field) for t in list(inputs) + list(outputs)])
    _raise(_lib.rse_code_shards(field, rb, n_out, n_in, ip, op, n, 1 if accumulate else 0,
                                _stream(inputs[0] if n_in else None)))


def code_shards_host(field: int, rows, inputs: Sequence, outputs: Sequence,
                     accumulate: bool = False) -> None:
    """code_shards() on HOST inputs/outputs (the code_some_slices hook,
    core.rs:481-490): pipelined through the GPU, synchronous."""
    n_out, n_in = len(outputs), len(inputs)
    flat = _row_bytes(field, rows, n_out, n_in)
    rb = (ctypes.c_uint8 * max(1, len(flat)))(*flat)
    ip = (ctypes.c_void_p * max(1, n_in))(*[_host_ptr(t) for t in inputs])
    op = (ctypes.c_void_p * max(1, n_out))(*[_host_ptr(t) for t in outputs])
    n = _same_len([_host_elems(t, field) for t in list(inputs) + list(outputs)])
    _raise(_lib.rse_code_shards_host(field, rb, n_out, n_in, ip, op, n, 1 if accumulate else 0,
                                     _stream()))


def dispatcher_stop() -> None:
    """End the resident dispatcher of the *_now calls now (it ends by itself
    RSE_OPT_DISPATCH_IDLE_US after the last call): a device-wide
    synchronisation after it does not wait for the idle time.  The next
    *_now call starts it again.  No reference counterpart."""
    _lib.rse_dispatcher_stop()


def last_kernel() -> str:
    """The last coding kernel this thread launched (rse_last_kernel)."""
    return _lib.rse_last_kernel().decode()


def fill_splitmix(t: torch.Tensor, seed: int, shard_id: int) -> None:
    """Fill a device tensor with the synthetic byte stream of (seed, shard_id)."""
    _raise(_lib.rse_fill_splitmix(_dev(t), t.numel() * t.element_size(), seed, shard_id,
                                  _stream(t)))
