"""The C-ABI library builds, loads and exports exactly what include/oxen_hash.h declares.

No compute calls here: on a host without a GPU the library must refuse (no CPU fallback).
"""
import ctypes
import subprocess

import pytest

from oxen_amd import _capi


def test_header_declares_the_bound_symbols(built_lib):
    declared = _capi.header_symbols()
    assert declared == sorted(_capi.SIGNATURES), (set(declared) ^ set(_capi.SIGNATURES))


def test_library_exports_every_declared_symbol(built_lib):
    out = subprocess.run(["nm", "-D", "--defined-only", built_lib], capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = [s for s in _capi.header_symbols() if s not in exported]
    assert not missing, missing
    L = _capi.lib()
    for s in _capi.header_symbols():
        assert getattr(L, s) is not None


def test_built_for_gfx950(built_lib):
    data = open(built_lib, "rb").read()
    assert b".hip_fatbin" in data
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_abi_version_and_format(built_lib):
    L = _capi.lib()
    assert L.oxh_abi_version() == 5
    buf = ctypes.create_string_buffer(40)
    # unpadded lowercase hex (merkle_hash.rs:73-77)
    n = L.oxh_format_hex(0x688558138047f8a, 0x2da4b9c5a75caad3 >> 4, buf)
    v = (0x2da4b9c5a75caad3 >> 4 << 64) | 0x688558138047f8a
    assert buf.value.decode() == format(v, "x") and n == len(format(v, "x"))
    for v in [0, 1, 15, 16, (1 << 128) - 1, 1 << 64, 0x393ba5849f5590fc5985c4bbcec0003f]:
        L.oxh_format_hex(v & (2**64 - 1), v >> 64, buf)
        assert buf.value.decode() == format(v, "x")
        L.oxh_format_dec(v & (2**64 - 1), v >> 64, buf)
        assert buf.value.decode() == str(v)  # dedup chunk names (fixedsize.rs:78)


def test_no_cpu_fallback_without_device(built_lib):
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(_capi.OxenError) as e:
        _capi.Context(0)
    assert e.value.code in (_capi.OXH_ERR_NODEVICE, _capi.OXH_ERR_HIP)
    from oxen_amd import hasher

    with pytest.raises(_capi.OxenError):
        hasher.hash_buffer(b"hello")


def test_staging_limit_is_rejected_before_any_device_work(built_lib):
    """staging_bytes above OXH_MAX_STAGING_BYTES would overflow a slot's packed fill word (31-bit byte
    offset, 19-bit item count): ctx_create refuses it with OXH_ERR_INVALID, GPU or not."""
    assert _capi.OXH_MAX_STAGING_BYTES == (1 << 31) - 256
    assert _capi.OXH_MAX_STAGING_BYTES // 4096 < (1 << 19)
    for bad in [_capi.OXH_MAX_STAGING_BYTES + 1, 1 << 31, 1 << 40]:
        with pytest.raises(_capi.OxenError) as e:
            _capi.Context(0, staging_bytes=bad)
        assert e.value.code == _capi.OXH_ERR_INVALID, e.value


def test_python_constants_match_the_header():
    """Every OXH_* integer #define in include/oxen_hash.h has the same value in oxen_amd._capi."""
    import os
    import re

    hdr = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "oxen_hash.h")).read()
    defines = {m.group(1): int(m.group(2), 0) for m in re.finditer(r"^#define\s+(OXH_[A-Z0-9_]+)\s+(-?(?:0x)?[0-9A-Fa-f]+)\b",
                                                                  hdr, re.M)}
    assert "OXH_MODE_WAVE_PACKED" in defines
    bound = {k: v for k, v in vars(_capi).items() if k.startswith("OXH_") and isinstance(v, int)}
    mismatched = {k: (v, bound[k]) for k, v in defines.items() if k in bound and bound[k] != v}
    assert not mismatched, mismatched
    modes = {k for k in defines if k.startswith("OXH_MODE_")}
    assert modes <= set(bound), modes - set(bound)


def test_comm_argument_checks_without_device(built_lib):
    """The digest-gather ABI (oxh_comm_*): argument errors are OXH_ERR_INVALID before any device or
    RCCL work; without a GPU, creating a communicator fails with OXH_ERR_NODEVICE (no CPU fallback)."""
    import torch

    L = _capi.lib()
    assert L.oxh_comm_unique_id(None) == _capi.OXH_ERR_INVALID
    h = ctypes.c_void_p()
    uid = b"\0" * _capi.OXH_COMM_ID_BYTES
    assert L.oxh_comm_create(None, 0, 1, 0, ctypes.byref(h)) == _capi.OXH_ERR_INVALID
    assert L.oxh_comm_create(uid, 1, 1, 0, ctypes.byref(h)) == _capi.OXH_ERR_INVALID
    assert L.oxh_comm_create(uid, 0, 0, 0, ctypes.byref(h)) == _capi.OXH_ERR_INVALID
    assert L.oxh_gather_digests(None, None, None, None, -1, None) == _capi.OXH_ERR_INVALID
    assert L.oxh_comm_info(None, None, None, None) == _capi.OXH_ERR_INVALID
    assert L.oxh_comm_destroy(None) == _capi.OXH_OK
    if not torch.cuda.is_available():
        assert L.oxh_comm_create(uid, 0, 1, 0, ctypes.byref(h)) == _capi.OXH_ERR_NODEVICE
        assert not h.value
        assert L.oxh_comm_check(0) == _capi.OXH_ERR_NODEVICE  # checked before anything is joined


def test_header_compiles_standalone_as_c_and_cpp(tmp_path):
    """include/oxen_hash.h is what a cgo / bindgen / plain-C caller includes: it must stand alone as C99
    (no C++ or HIP types) and as C++17, warning-free."""
    import os

    hdr = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "oxen_hash.h")
    for lang, std in (("c", "-std=c99"), ("c++", "-std=c++17")):
        r = subprocess.run(["gcc" if lang == "c" else "g++", std, "-Wall", "-Wextra", "-pedantic", "-Werror",
                            "-fsyntax-only", "-x", lang, hdr], capture_output=True, text=True)
        assert r.returncode == 0, (lang, r.stderr)


def _c_consumer(*args):
    from oxen_amd import build

    build.build_host()
    return subprocess.run([build.C_CONSUMER, *args], capture_output=True, text=True, timeout=120)


def test_plain_c_consumer_without_device(built_lib):
    """tests/native/abi_c_consumer.c: the ABI from plain C99 (gcc -std=c99 -pedantic -Werror), as a cgo /
    bindgen caller uses it -- version, formatting, argument errors, and OXH_ERR_NODEVICE from context
    creation and the comm check when no GPU is visible (no CPU fallback)."""
    import torch

    if torch.cuda.is_available():
        pytest.skip("the no-device branch needs a host without a GPU")
    r = _c_consumer()
    assert r.returncode == 0, r.stderr
    assert "all checks passed (no device)" in r.stdout


@pytest.mark.gpu
def test_plain_c_consumer_on_gpu(cuda):
    """The same C99 program on the GPU box: the reference's known answer and the SURVEY §8c vectors
    through oxh_hash_buffers and oxh_hash_streams, formatted as MerkleHash Display does."""
    r = _c_consumer("gpu")
    assert r.returncode == 0, r.stderr
    assert "all checks passed (gpu)" in r.stdout
