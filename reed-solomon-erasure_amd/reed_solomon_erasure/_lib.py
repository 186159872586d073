"""ctypes binding of librse_hip.so (include/rse_hip.h).

The HIP library is the product: there is no CPU fallback.  If the shared object
is missing or fails to load, importing this package raises immediately.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# RSE_LIB_PATH: another build of the same library (the sanitizer builds of
# tools/sanitize.sh); the default is the in-tree librse_hip.so.
LIB_PATH = os.environ.get("RSE_LIB_PATH") or os.path.join(HERE, "librse_hip.so")

# Every entry point of include/rse_hip.h (checked by tests/test_capi.py).
EXPORTS = (
    "rse_strerror", "rse_last_device_error", "rse_version",
    "rse_codec_new", "rse_codec_free", "rse_codec_field",
    "rse_codec_data_shard_count", "rse_codec_parity_shard_count",
    "rse_codec_total_shard_count", "rse_codec_matrix", "rse_codec_kernel_kind",
    "rse_encode", "rse_encode_sep", "rse_encode_single", "rse_encode_single_sep",
    "rse_verify", "rse_verify_with_buffer", "rse_reconstruct", "rse_reconstruct_data",
    "rse_encode_flat", "rse_verify_flat", "rse_reconstruct_data_flat", "rse_reconstruct_batch",
    "rse_code_shards",
    "rse_code_shards_host", "rse_gf8_mul_slice", "rse_gal_mul", "rse_gal_mul_xor",
    "rse_gf16_mul_slice", "rse_gf8_invert_batch", "rse_gf16_invert_batch",
    "rse_encode_host", "rse_encode_host_flat", "rse_encode_sep_host", "rse_encode_single_host",
    "rse_encode_single_sep_host", "rse_verify_host", "rse_verify_with_buffer_host",
    "rse_verify_host_flat", "rse_reconstruct_host", "rse_reconstruct_data_host",
    "rse_reconstruct_host_batch", "rse_fill_splitmix",
    "rse_encode_now", "rse_verify_now", "rse_reconstruct_now", "rse_reconstruct_data_now",
    "rse_dispatcher_stop",
    "rse_set_option", "rse_get_option", "rse_last_kernel",
)

_c = ctypes
_vp = _c.c_void_p
_sz = _c.c_size_t
_szp = _c.POINTER(_c.c_size_t)
_u8p = _c.POINTER(_c.c_uint8)
_ip = _c.POINTER(_c.c_int)

_SIGS = {
    "rse_strerror": (_c.c_char_p, [_c.c_int]),
    "rse_last_device_error": (_c.c_int, []),
    "rse_version": (_c.c_char_p, []),
    "rse_codec_new": (_c.c_int, [_c.c_int, _sz, _sz, _c.POINTER(_vp)]),
    "rse_codec_free": (None, [_vp]),
    "rse_codec_field": (_c.c_int, [_vp]),
    "rse_codec_data_shard_count": (_sz, [_vp]),
    "rse_codec_parity_shard_count": (_sz, [_vp]),
    "rse_codec_total_shard_count": (_sz, [_vp]),
    "rse_codec_matrix": (_c.c_int, [_vp, _u8p, _sz]),
    "rse_codec_kernel_kind": (_c.c_int, [_vp, _c.c_int]),
    "rse_encode": (_c.c_int, [_vp, _vp, _szp, _sz, _vp]),
    "rse_encode_sep": (_c.c_int, [_vp, _vp, _szp, _sz, _vp, _szp, _sz, _vp]),
    "rse_encode_single": (_c.c_int, [_vp, _sz, _vp, _szp, _sz, _vp]),
    "rse_encode_single_sep": (_c.c_int, [_vp, _sz, _vp, _sz, _vp, _szp, _sz, _vp]),
    "rse_verify": (_c.c_int, [_vp, _vp, _szp, _sz, _ip, _vp]),
    "rse_verify_with_buffer": (_c.c_int, [_vp, _vp, _szp, _sz, _vp, _szp, _sz, _ip, _vp]),
    "rse_reconstruct": (_c.c_int, [_vp, _vp, _szp, _u8p, _sz, _vp]),
    "rse_reconstruct_data": (_c.c_int, [_vp, _vp, _szp, _u8p, _sz, _vp]),
    "rse_encode_flat": (_c.c_int, [_vp, _vp, _sz, _sz, _vp]),
    "rse_verify_flat": (_c.c_int, [_vp, _vp, _sz, _sz, _u8p, _vp]),
    "rse_reconstruct_data_flat": (_c.c_int, [_vp, _vp, _sz, _sz, _u8p, _vp]),
    "rse_reconstruct_batch": (_c.c_int, [_vp, _vp, _sz, _sz, _u8p, _c.c_int, _vp]),
    "rse_encode_host_flat": (_c.c_int, [_vp, _vp, _sz, _sz, _vp]),
    "rse_code_shards": (_c.c_int, [_c.c_int, _u8p, _sz, _sz, _vp, _vp, _sz, _c.c_int, _vp]),
    "rse_gf8_mul_slice": (_c.c_int, [_c.c_uint8, _vp, _vp, _sz, _c.c_int, _vp]),
    "rse_gf8_invert_batch": (_c.c_int, [_vp, _vp, _vp, _sz, _sz, _vp]),
    "rse_gf16_invert_batch": (_c.c_int, [_vp, _vp, _vp, _sz, _sz, _vp]),
    "rse_encode_host": (_c.c_int, [_vp, _vp, _szp, _sz, _vp]),
    "rse_verify_host": (_c.c_int, [_vp, _vp, _szp, _sz, _ip, _vp]),
    "rse_encode_sep_host": (_c.c_int, [_vp, _vp, _szp, _sz, _vp, _szp, _sz, _vp]),
    "rse_encode_single_host": (_c.c_int, [_vp, _sz, _vp, _szp, _sz, _vp]),
    "rse_encode_single_sep_host": (_c.c_int, [_vp, _sz, _vp, _sz, _vp, _szp, _sz, _vp]),
    "rse_verify_with_buffer_host": (_c.c_int, [_vp, _vp, _szp, _sz, _vp, _szp, _sz, _ip, _vp]),
    "rse_verify_host_flat": (_c.c_int, [_vp, _vp, _sz, _sz, _u8p, _vp]),
    "rse_reconstruct_host": (_c.c_int, [_vp, _vp, _szp, _u8p, _sz, _vp]),
    "rse_reconstruct_data_host": (_c.c_int, [_vp, _vp, _szp, _u8p, _sz, _vp]),
    "rse_reconstruct_host_batch": (_c.c_int, [_vp, _vp, _sz, _sz, _u8p, _c.c_int, _vp]),
    "rse_code_shards_host": (_c.c_int, [_c.c_int, _u8p, _sz, _sz, _vp, _vp, _sz, _c.c_int, _vp]),
    "rse_gal_mul": (_sz, [_u8p, _u8p, _vp, _vp, _sz]),
    "rse_gal_mul_xor": (_sz, [_u8p, _u8p, _vp, _vp, _sz]),
    "rse_gf16_mul_slice": (_c.c_int, [_u8p, _vp, _vp, _sz, _c.c_int, _vp]),
    "rse_last_kernel": (_c.c_char_p, []),
    "rse_fill_splitmix": (_c.c_int, [_vp, _sz, _c.c_uint64, _c.c_uint64, _vp]),
    "rse_encode_now": (_c.c_int, [_vp, _vp, _szp, _sz]),
    "rse_verify_now": (_c.c_int, [_vp, _vp, _szp, _sz, _ip]),
    "rse_reconstruct_now": (_c.c_int, [_vp, _vp, _szp, _u8p, _sz]),
    "rse_reconstruct_data_now": (_c.c_int, [_vp, _vp, _szp, _u8p, _sz]),
    "rse_dispatcher_stop": (None, []),
    "rse_set_option": (_c.c_int, [_c.c_int, _c.c_int64]),
    "rse_get_option": (_c.c_int64, [_c.c_int]),
}

_LIB = None


def load():
    """Load librse_hip.so.  torch is imported first so that the HIP runtime torch
    ships (SONAME libamdhip64.so.7) is the one the library binds to: one runtime,
    shared streams and device pointers."""
    global _LIB
    if _LIB is not None:
        return _LIB
    try:
        import torch  # noqa: F401  (must precede the dlopen, see docstring)
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `make -C reed-solomon-erasure_amd` "
            "(or __graft_entry__.build()).  There is no CPU fallback.")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _LIB = lib
    return lib
