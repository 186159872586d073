"""CPU-side checks of the C ABI (no device work): the library loads, exports
every entry point include/rse_hip.h declares, builds the same matrices as the
oracle, and reproduces the reference's validation errors before touching a GPU.
"""
import ctypes
import os
import re

import numpy as np
import pytest

from oracle import oracle as O
import reed_solomon_erasure as R
from reed_solomon_erasure import Error, RSError
from reed_solomon_erasure._lib import EXPORTS, load

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L = load()


def header_functions():
    text = open(os.path.join(ROOT, "include", "rse_hip.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rse_[a-z0-9_]+)\s*\(", text)))


def test_exports_every_declared_symbol():
    declared = header_functions()
    assert len(declared) >= 20
    for name in declared:
        assert hasattr(L, name), name
    assert sorted(declared) == sorted(EXPORTS)


def test_error_strings_match_errors_rs():  # errors.rs:20-38
    for e in Error:
        assert L.rse_strerror(int(e)).decode() == str(e)
    assert L.rse_strerror(0).decode() == "Ok"


def test_codec_new_errors():  # core.rs:445-454, tests/mod.rs:97-116
    for args, err in [((0, 1), Error.TooFewDataShards), ((1, 0), Error.TooFewParityShards),
                      ((129, 128), Error.TooManyShards)]:
        with pytest.raises(RSError) as ei:
            R.galois_8.ReedSolomon(*args)
        assert ei.value.error == err
    R.galois_8.ReedSolomon(128, 128)
    with pytest.raises(RSError):  # tests/galois_16.rs:24-34
        R.galois_16.ReedSolomon(65536, 1)
    with pytest.raises(RSError):
        R.galois_16.ReedSolomon(1, 65536)
    # tests/galois_16.rs:33: the widest GF(2^16) codecs are Ok
    r = R.galois_16.ReedSolomon(1, 65535)
    assert r.total_shard_count() == 65536


def test_shard_counts_and_clone():  # tests/mod.rs:118-141
    rng = np.random.default_rng(3)
    for _ in range(10):
        k, p = int(rng.integers(1, 128)), int(rng.integers(1, 128))
        r = R.galois_8.ReedSolomon(k, p)
        assert (r.data_shard_count(), r.parity_shard_count(), r.total_shard_count()) == (k, p, k + p)
    r1 = R.galois_8.ReedSolomon(10, 3)
    assert r1.clone() == r1


@pytest.mark.parametrize("field,k,p", [(8, 1, 1), (8, 3, 2), (8, 10, 4), (8, 17, 3), (8, 128, 128),
                                       (8, 200, 56), (16, 1, 1), (16, 20, 8), (16, 40, 24)])
def test_matrix_matches_oracle(field, k, p):
    r = R.core.ReedSolomon(k, p, field)
    m = np.array(r.matrix(), dtype=np.int64)
    om = O.Codec(field, k, p).matrix().astype(np.int64)
    if field == 16:
        om = om[..., 0] * 256 + om[..., 1]
    assert (m == om).all()


def test_matrix_matches_golden():
    import json
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))["generated"]
    for name, hexstr in g["encoding_matrices"].items():
        field, k, p = (int(x) for x in name[2:].split("_"))
        r = R.core.ReedSolomon(k, p, field)
        es = 2 if field == 16 else 1
        buf = (ctypes.c_uint8 * ((k + p) * k * es))()
        assert L.rse_codec_matrix(r._h, buf, len(buf)) == 0
        assert bytes(buf).hex() == hexstr


# ------- validation through the raw ABI with fake device pointers: every call
# below fails its checks before any device access, exactly as the reference
# returns Err before touching a slice.
FAKE = 0x1000


def ptrs(n):
    return (ctypes.c_void_p * max(1, n))(*([FAKE] * n))


def lens(xs):
    return (ctypes.c_size_t * max(1, len(xs)))(*xs)


def test_encode_verify_reconstruct_validation():  # tests/mod.rs:1058-1163
    r = R.galois_8.ReedSolomon(3, 2)
    ok = ctypes.c_int()
    pres = (ctypes.c_uint8 * 6)(*([1] * 6))
    for n, err in [(4, Error.TooFewShards), (6, Error.TooManyShards)]:
        assert L.rse_encode(r._h, ptrs(n), lens([10] * n), n, None) == err
        assert L.rse_verify(r._h, ptrs(n), lens([10] * n), n, ctypes.byref(ok), None) == err
        assert L.rse_reconstruct(r._h, ptrs(n), lens([10] * n), pres, n, None) == err
    r2 = R.galois_8.ReedSolomon(2, 2)
    pres4 = (ctypes.c_uint8 * 4)(1, 1, 1, 1)
    for ls, err in [([3, 2, 3, 3], Error.IncorrectShardSize), ([2, 2, 3, 3], Error.IncorrectShardSize),
                    ([2, 3, 3, 3], Error.IncorrectShardSize), ([0, 3, 3, 3], Error.EmptyShard)]:
        assert L.rse_encode(r2._h, ptrs(4), lens(ls), 4, None) == err
        assert L.rse_verify(r2._h, ptrs(4), lens(ls), 4, ctypes.byref(ok), None) == err
        assert L.rse_reconstruct(r2._h, ptrs(4), lens(ls), pres4, 4, None) == err
    none = (ctypes.c_uint8 * 4)(0, 0, 0, 0)
    assert L.rse_reconstruct(r2._h, ptrs(4), lens([3] * 4), none, 4, None) == Error.TooFewShardsPresent
    # a missing shard's buffer must have the common size ((T,bool), lib.rs:185-199)
    miss = (ctypes.c_uint8 * 4)(0, 1, 1, 1)
    assert L.rse_reconstruct(r2._h, ptrs(4), lens([2, 3, 3, 3]), miss, 4, None) == \
        Error.IncorrectShardSize
    # all present: Ok with nothing to do (core.rs:763-767) -- no device access
    assert L.rse_reconstruct(r2._h, ptrs(4), lens([3] * 4), pres4, 4, None) == 0


def test_reconstruct_batch_validation():  # core.rs:747-772 per stripe, before any device work
    r = R.galois_8.ReedSolomon(3, 2)
    pres = (ctypes.c_uint8 * 10)(1, 1, 1, 1, 1, 0, 0, 1, 1, 0)  # stripe 1: 2 present
    assert L.rse_reconstruct_batch(r._h, FAKE, 10, 2, pres, 0, None) == Error.TooFewShardsPresent
    assert L.rse_reconstruct_batch(r._h, FAKE, 10, 2, pres, 1, None) == Error.TooFewShardsPresent
    ok = (ctypes.c_uint8 * 10)(*([1] * 10))
    assert L.rse_reconstruct_batch(r._h, FAKE, 0, 2, ok, 0, None) == Error.EmptyShard
    assert L.rse_reconstruct_batch(r._h, FAKE, 10, 0, ok, 0, None) == 0
    assert L.rse_reconstruct_batch(None, FAKE, 10, 2, ok, 0, None) == 100
    with pytest.raises(R.RSError):  # shape of the flags
        r.reconstruct_batch(None, 10, 2, [[True] * 5])


def test_verify_flat_validation():  # before any device access
    r = R.galois_8.ReedSolomon(3, 2)
    ok = (ctypes.c_uint8 * 4)()
    assert L.rse_verify_flat(r._h, FAKE, 0, 4, ok, None) == Error.EmptyShard
    assert L.rse_verify_flat(r._h, FAKE, 10, 0, ok, None) == 0
    assert L.rse_verify_flat(None, FAKE, 10, 4, ok, None) == 100
    assert L.rse_verify_flat(r._h, FAKE, 10, 4, None, None) == 100


def test_buffer_and_sep_validation():  # tests/mod.rs:905-964, 2304-2619
    r = R.galois_8.ReedSolomon(3, 2)
    ok = ctypes.c_int()
    s5 = lens([100] * 5)
    assert L.rse_verify_with_buffer(r._h, ptrs(5), s5, 5, ptrs(1), lens([100]), 1,
                                    ctypes.byref(ok), None) == Error.TooFewBufferShards
    assert L.rse_verify_with_buffer(r._h, ptrs(5), s5, 5, ptrs(3), lens([100] * 3), 3,
                                    ctypes.byref(ok), None) == Error.TooManyBufferShards
    assert L.rse_verify_with_buffer(r._h, ptrs(5), s5, 5, ptrs(2), lens([0, 100]), 2,
                                    ctypes.byref(ok), None) == Error.EmptyShard
    assert L.rse_verify_with_buffer(r._h, ptrs(5), s5, 5, ptrs(2), lens([100, 99]), 2,
                                    ctypes.byref(ok), None) == Error.IncorrectShardSize
    assert L.rse_verify_with_buffer(r._h, ptrs(5), s5, 5, ptrs(2), lens([99, 99]), 2,
                                    ctypes.byref(ok), None) == Error.IncorrectShardSize
    assert L.rse_encode_sep(r._h, ptrs(2), lens([9] * 2), 2, ptrs(2), lens([9] * 2), 2,
                            None) == Error.TooFewDataShards
    assert L.rse_encode_sep(r._h, ptrs(4), lens([9] * 4), 4, ptrs(2), lens([9] * 2), 2,
                            None) == Error.TooManyDataShards
    assert L.rse_encode_sep(r._h, ptrs(3), lens([9] * 3), 3, ptrs(1), lens([9]), 1,
                            None) == Error.TooFewParityShards
    assert L.rse_encode_sep(r._h, ptrs(3), lens([9] * 3), 3, ptrs(3), lens([9] * 3), 3,
                            None) == Error.TooManyParityShards
    assert L.rse_encode_sep(r._h, ptrs(3), lens([9] * 3), 3, ptrs(2), lens([8] * 2), 2,
                            None) == Error.IncorrectShardSize
    assert L.rse_encode_single(r._h, 3, ptrs(5), s5, 5, None) == Error.InvalidIndex
    assert L.rse_encode_single(r._h, 0, ptrs(4), s5, 4, None) == Error.TooFewShards
    assert L.rse_encode_single_sep(r._h, 3, FAKE, 100, ptrs(2), lens([100] * 2), 2,
                                   None) == Error.InvalidIndex
    assert L.rse_encode_single_sep(r._h, 0, FAKE, 100, ptrs(1), lens([100]), 1,
                                   None) == Error.TooFewParityShards
    assert L.rse_encode_single_sep(r._h, 0, FAKE, 99, ptrs(2), lens([100] * 2), 2,
                                   None) == Error.IncorrectShardSize


def test_null_arguments_are_rejected():
    assert L.rse_codec_new(7, 1, 1, ctypes.byref(ctypes.c_void_p())) == 100
    assert L.rse_encode(None, ptrs(2), lens([1, 1]), 2, None) == 100
    assert L.rse_code_shards(8, None, 1, 1, ptrs(1), ptrs(1), 1, 0, None) == 100
    assert L.rse_gf8_invert_batch(None, None, None, 3, 1, None) == 100


def test_run_time_specialisation_builds_on_cpu():
    """Codecs that are not compiled in (p <= 8, k <= 32) get bit-sliced kernels
    built by hiprtc at run time, requested by the first chunk-sized call or by
    kernel_kind(wait=True); the build is host-only, so it runs here without a
    GPU.  Compiled-in codecs and ineligible ones report so."""
    assert R.galois_8.ReedSolomon(10, 4).kernel_kind() == "bitslice-compiled"
    assert R.galois_16.ReedSolomon(20, 8).kernel_kind() == "bitslice-compiled"
    assert R.galois_8.ReedSolomon(50, 20).kernel_kind() == "table"   # p > 8
    assert R.galois_8.ReedSolomon(33, 4).kernel_kind() == "table"    # k > 32
    got = L.rse_get_option(10) + L.rse_get_option(16)  # built + cached (conftest's prebuilt)
    r = R.galois_8.ReedSolomon(12, 4)
    assert r.kernel_kind(wait=True) == "bitslice-specialised"
    assert L.rse_get_option(10) + L.rse_get_option(16) >= got + 2  # encode + reconstruct modules
    assert R.galois_8.ReedSolomon(12, 4).kernel_kind() == "bitslice-specialised"  # cached
    old = L.rse_get_option(9)
    try:
        assert L.rse_set_option(9, 0) == 0  # off: new codecs stay on the table kernels
        assert R.galois_8.ReedSolomon(7, 2).kernel_kind(wait=True) == "table"
    finally:
        L.rse_set_option(9, old)


def test_wide_codec_modules_build_on_cpu():
    """Wide codecs (k > 32 or p > 8) get one module each (every wave of a
    workgroup codes its share of <= 8 outputs over all inputs); past 64
    outputs, one module per balanced group of <= 64 outputs (round 6; one
    per 8 x 32 block of the parity rows before), and with
    RSE_OPT_WIDE_BLOCK_INPUTS 0 the 8 x 32 blocks again."""
    built = L.rse_get_option(10)
    assert R.galois_8.ReedSolomon(6, 10).kernel_kind(wait=True) == "bitslice-specialised"
    assert L.rse_get_option(10) == built + 1
    built = L.rse_get_option(10)
    assert R.galois_8.ReedSolomon(34, 1).kernel_kind(wait=True) == "bitslice-specialised"
    assert L.rse_get_option(10) == built + 1
    built = L.rse_get_option(10)
    assert R.galois_8.ReedSolomon(2, 65).kernel_kind(wait=True) == "bitslice-specialised"
    assert L.rse_get_option(10) == built + 2  # output groups of 33 and 32
    built = L.rse_get_option(10)
    old = L.rse_get_option(46)
    try:
        assert L.rse_set_option(46, 0) == 0
        assert R.galois_8.ReedSolomon(3, 65).kernel_kind(wait=True) == "bitslice-specialised"
        assert L.rse_get_option(10) == built + 9  # 9 output blocks of <= 8
    finally:
        L.rse_set_option(46, old)


def _py(code, env, timeout=600):
    import subprocess
    import sys
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                          env=env, timeout=timeout, cwd=ROOT)


PRELUDE = ("import sys; sys.path.insert(0, 'reed-solomon-erasure_amd'); "
           "import reed_solomon_erasure as R; L = R._lib.load(); ")


def test_jit_disk_cache_across_processes(tmp_path):
    """A module built by one process is loaded from the on-disk cache by the
    next: no compile (RSE_OPT_JIT_MODULES stays 0, RSE_OPT_JIT_CACHE_HITS
    counts it).  Keys cover the source, so another codec misses."""
    env = dict(os.environ, RSE_JIT_CACHE_DIR=str(tmp_path))
    code = PRELUDE + ("print(R.galois_8.ReedSolomon(9, 5).kernel_kind(wait=True), "
                      "L.rse_get_option(10), L.rse_get_option(16))")
    first = _py(code, env)
    assert first.returncode == 0, first.stderr[-2000:]
    assert first.stdout.split() == ["bitslice-specialised", "2", "0"]  # encode + reconstruct
    assert len(list(tmp_path.glob("*.co"))) == 2 and not list(tmp_path.glob("*.hip"))
    second = _py(code, env)
    assert second.returncode == 0, second.stderr[-2000:]
    assert second.stdout.split() == ["bitslice-specialised", "0", "2"]
    other = _py(code.replace("(9, 5)", "(9, 4)"), env)
    assert other.stdout.split() == ["bitslice-specialised", "2", "0"]
    off = _py(PRELUDE + "L.rse_set_option(15, 0); " + code.split("; ", 3)[-1], env)
    assert off.stdout.split() == ["bitslice-specialised", "2", "0"]  # cache off: compiled


def test_exit_not_blocked_by_a_build(tmp_path):
    """A process that exits while a long build (GF(2^8) 50+20: minutes of
    hiprtc here) is in flight exits at once: the rse_jitc helper is stopped,
    nothing is left behind in the cache directory.  comgr's own compile cache
    is off, or an earlier build of the same source would finish at once."""
    import time
    env = dict(os.environ, RSE_JIT_CACHE_DIR=str(tmp_path), AMD_COMGR_CACHE="0")
    code = PRELUDE + ("import threading, time; r = R.galois_8.ReedSolomon(50, 20); "
                      "threading.Thread(target=lambda: r.kernel_kind(wait=True), daemon=True).start(); "
                      "time.sleep(2); print('bye')")
    t0 = time.time()
    out = _py(code, env, timeout=120)
    assert out.returncode == 0 and out.stdout.strip() == "bye", out.stderr[-2000:]
    assert time.time() - t0 < 60
    assert list(tmp_path.iterdir()) == []


def test_code_shards_refuses_unequal_lengths():
    """rse_code_shards(_host) take ONE length for every input and output: the
    Python mirror refuses a shorter buffer before the library could read or
    write past its end (lib.rs:100 asserts equal lengths)."""
    a = np.zeros(64, np.uint8)
    b = np.zeros(63, np.uint8)
    for ins, outs in [([a, b], [a]), ([a], [b]), ([a], [a, b]), ([b, a], [a, a])]:
        with pytest.raises(RSError) as ei:
            R.core.code_shards_host(8, [[1] * len(ins)] * len(outs), ins, outs)
        assert ei.value.error == Error.IncorrectShardSize


def header_options(name):
    import re
    hdr = open(os.path.join(ROOT, "include", name)).read()
    return {m.group(1): int(m.group(2))
            for m in re.finditer(r"#define (RSE_OPT_[A-Z0-9_]+) (\d+)", hdr)}


def test_tuning_switches_need_rse_tune():
    """include/rse_hip.h holds only the options a caller of the drop-in needs;
    the tuning / A-B switches (include/rse_hip_tune.h) are refused unless the
    environment has RSE_TUNE=1, and the two headers share no key.  Without
    it, a caller option is still taken and the tuning value stays put."""
    caller, tune = header_options("rse_hip.h"), header_options("rse_hip_tune.h")
    assert not set(caller.values()) & set(tune.values())
    assert len(caller) <= 20 and "RSE_OPT_FFT" in tune and "RSE_OPT_JIT" in caller
    env = {k_: v for k_, v in os.environ.items() if k_ != "RSE_TUNE"}
    code = PRELUDE + ("print(L.rse_set_option(51, 0), L.rse_get_option(51), "
                      "L.rse_set_option(9, 2), L.rse_get_option(9), L.rse_set_option(2, 64))")
    out = _py(code, env)
    assert out.returncode == 0, out.stderr[-2000:]
    bad = str(L.rse_set_option(99, 1))
    assert out.stdout.split() == [bad, "1", "0", "2", bad]
    out = _py(code, dict(env, RSE_TUNE="1"))
    assert out.stdout.split() == ["0", "0", "0", "2", "0"]


def test_every_header_option_is_readable():
    """Every RSE_OPT_* key include/rse_hip.h and rse_hip_tune.h declare answers rse_get_option
    (-1 is the answer for an unknown key), and the round-3 switches start at
    their documented defaults: wave-pair reconstruct and paired wide networks
    on, the event wait off, the verify completion word on."""
    keys = header_options("rse_hip.h")
    keys.update(header_options("rse_hip_tune.h"))
    assert len(keys) >= 30
    for name, key in keys.items():  # KERNEL_VARIANT's default is -1 ("the default variant")
        assert L.rse_get_option(key) != -1 or name == "RSE_OPT_KERNEL_VARIANT", name
    assert L.rse_get_option(99) == -1
    assert L.rse_set_option(99, 1) != 0
    want = {"RSE_OPT_RECON_PAIRS": 8, "RSE_OPT_WIDE_PAIRS": 1, "RSE_OPT_SYNC_EVENT": 0,
            "RSE_OPT_SPIN_WAIT": 1, "RSE_OPT_HOST_DIRECT": 1, "RSE_OPT_WIDE_BLOCK_INPUTS": 128,
            "RSE_OPT_DISPATCH_MAX_BYTES": 65536, "RSE_OPT_SUB_DEPTH": 4}
    for name, v in want.items():
        assert L.rse_get_option(keys[name]) == v, name
    old = L.rse_get_option(keys["RSE_OPT_SPIN_WAIT"])
    try:
        assert L.rse_set_option(keys["RSE_OPT_SPIN_WAIT"], 0) == 0
        assert L.rse_get_option(keys["RSE_OPT_SPIN_WAIT"]) == 0
    finally:
        L.rse_set_option(keys["RSE_OPT_SPIN_WAIT"], old)


def test_wrong_byte_timing_splits_are_refused():
    """RSE_OPT_RECON_PAIRS 4 / 5 select timing splits that skip the Horner
    steps or the data networks and so write wrong bytes; the release library
    refuses them (reconstruct must always return core.rs:680-695's bytes) and
    keeps its setting, while the real variants are still accepted.  Only
    `make tune` (-DRSE_TUNE_SPLITS, build-tune/) carries the splits."""
    RECON_PAIRS = 28
    INVALID_ARGUMENT = L.rse_set_option(99, 1)
    assert INVALID_ARGUMENT != 0
    old = L.rse_get_option(RECON_PAIRS)
    try:
        for bad in (4, 5):
            assert L.rse_set_option(RECON_PAIRS, bad) == INVALID_ARGUMENT, bad
            assert L.rse_get_option(RECON_PAIRS) == old
        for good in (0, 1, 2, 3, 6, 7, 8):
            assert L.rse_set_option(RECON_PAIRS, good) == 0, good
            assert L.rse_get_option(RECON_PAIRS) == good
    finally:
        L.rse_set_option(RECON_PAIRS, old)


def test_now_entries_validate_like_the_stream_entries():
    """rse_encode_now / rse_verify_now / rse_reconstruct(_data)_now (the
    synchronous forms, core.rs:597-695's contract) return the same errors as
    rse_encode / rse_verify / rse_reconstruct, in the same precedence, before
    any device work (tests/mod.rs:1058-1163)."""
    r = R.galois_8.ReedSolomon(3, 2)
    ok = ctypes.c_int()
    pres = (ctypes.c_uint8 * 6)(*([1] * 6))
    for n, err in [(4, Error.TooFewShards), (6, Error.TooManyShards)]:
        assert L.rse_encode_now(r._h, ptrs(n), lens([10] * n), n) == err
        assert L.rse_verify_now(r._h, ptrs(n), lens([10] * n), n, ctypes.byref(ok)) == err
        assert L.rse_reconstruct_now(r._h, ptrs(n), lens([10] * n), pres, n) == err
        assert L.rse_reconstruct_data_now(r._h, ptrs(n), lens([10] * n), pres, n) == err
    r2 = R.galois_8.ReedSolomon(2, 2)
    pres4 = (ctypes.c_uint8 * 4)(1, 1, 1, 1)
    for ls, err in [([3, 2, 3, 3], Error.IncorrectShardSize), ([2, 2, 3, 3], Error.IncorrectShardSize),
                    ([2, 3, 3, 3], Error.IncorrectShardSize), ([0, 3, 3, 3], Error.EmptyShard)]:
        assert L.rse_encode_now(r2._h, ptrs(4), lens(ls), 4) == err
        assert L.rse_encode(r2._h, ptrs(4), lens(ls), 4, None) == err
        assert L.rse_verify_now(r2._h, ptrs(4), lens(ls), 4, ctypes.byref(ok)) == err
        assert L.rse_reconstruct_now(r2._h, ptrs(4), lens(ls), pres4, 4) == err
    none = (ctypes.c_uint8 * 4)(0, 0, 0, 0)
    assert L.rse_reconstruct_now(r2._h, ptrs(4), lens([3] * 4), none, 4) == \
        Error.TooFewShardsPresent
    assert L.rse_reconstruct_now(r2._h, ptrs(4), lens([3] * 4), pres4, 4) == 0  # nothing to do
    assert L.rse_encode_now(None, ptrs(4), lens([3] * 4), 4) == 100
    assert L.rse_verify_now(r2._h, ptrs(4), lens([3] * 4), 4, None) == 100
    L.rse_dispatcher_stop()  # nothing started: a no-op
