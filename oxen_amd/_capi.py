"""ctypes binding of the C ABI in include/oxen_hash.h (oxen_amd/liboxen_hash.so).

Loading never falls back to anything: if the library is missing the import of a hashing entry
point raises, and on a host without a gfx950 device `Context()` raises `OxenError`.
"""
from __future__ import annotations

import ctypes
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboxen_hash.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "oxen_hash.h")

OXH_OK = 0
OXH_ERR_INVALID = 1
OXH_ERR_HIP = 2
OXH_ERR_IO = 3
OXH_ERR_NOMEM = 4
OXH_ERR_NODEVICE = 5
OXH_ERR_META = 6
OXH_ERR_OPEN = 7
OXH_META_NONE = 0
OXH_META_GIVEN = 1
OXH_META_TEXT = 2
OXH_META_ERROR = 3
OXH_MODE_AUTO = 0
OXH_MODE_WAVE = 1
OXH_MODE_LANE = 2
OXH_MODE_WAVE_SHORT = 3
OXH_MODE_WAVE_PACKED = 4
OXH_MAX_STAGING_BYTES = 2147483392  # 2 GiB - 256 (include/oxen_hash.h)
OXH_COMM_ID_BYTES = 128

_u64 = ctypes.c_uint64
_u32 = ctypes.c_uint32
_u64p = ctypes.POINTER(ctypes.c_uint64)
_i32p = ctypes.POINTER(ctypes.c_int32)
_vp = ctypes.c_void_p
_int = ctypes.c_int

# name -> (restype, argtypes); must mirror include/oxen_hash.h exactly (tests/test_capi.py checks).
SIGNATURES = {
    "oxh_abi_version": (_int, []),
    "oxh_last_error": (ctypes.c_char_p, []),
    "oxh_device_count": (_int, [ctypes.POINTER(_int)]),
    "oxh_ctx_create": (_int, [_int, _u64, ctypes.POINTER(_vp)]),
    "oxh_ctx_destroy": (_int, [_vp]),
    "oxh_ctx_stream": (_vp, [_vp]),
    "oxh_xxh3_128_batch_device": (_int, [_vp, _vp, _vp, _u64, _vp, _int, _vp]),
    "oxh_chunk_digests_device": (_int, [_vp, _u64, _u64, _vp, _vp]),
    "oxh_xxh3_128_large_device": (_int, [_vp, _vp, _u64, _vp, _vp]),
    "oxh_xxh3_128_large_batch_device": (_int, [ctypes.POINTER(_vp), _u64p, _u64, _vp, _vp]),
    "oxh_hash_buffers": (_int, [_vp, ctypes.POINTER(ctypes.c_char_p), _u64p, _u64, _u64p]),
    "oxh_hash_files": (_int, [_vp, ctypes.POINTER(ctypes.c_char_p), _u64, _u64p, _u64p, _i32p]),
    "oxh_hash_files_meta": (_int, [_vp, ctypes.POINTER(ctypes.c_char_p), _u64p, _u64, _u64p, _u64p, _i32p]),
    "oxh_hash_files_ex": (_int, [_vp, ctypes.POINTER(ctypes.c_char_p), _u64p, _u64, _u64p, _u64p, _i32p, _i32p, _u64p,
                                 _i32p]),
    "oxh_add_files": (_int, [_vp, ctypes.POINTER(ctypes.c_char_p), _u64, ctypes.c_char_p, _u64p, _u64p, _i32p, _i32p]),
    "oxh_add_files_ex": (_int, [_vp, ctypes.POINTER(ctypes.c_char_p), _u64, ctypes.c_char_p, _u64p, _u64p, _i32p, _i32p,
                                _i32p]),
    "oxh_clean_corrupted_versions": (_int, [_vp, ctypes.c_char_p, _int, _u64p]),
    "oxh_hash_files_text": (_int, [_vp, ctypes.POINTER(ctypes.c_char_p), _u64, _u64p, _u64p, _i32p, _u64p]),
    "oxh_xxh3_128_text_batch_device": (_int, [_vp, _vp, _vp, _u64, _vp, _vp, _vp]),
    "oxh_hash_files_text_utf8": (_int, [_vp, ctypes.POINTER(ctypes.c_char_p), _u64, _u64p, _u64p, _i32p, _u64p, _i32p]),
    "oxh_files_modified": (_int, [_vp, ctypes.POINTER(ctypes.c_char_p), _u64p, _u64p, _vp, _u64p, _vp, _vp, _vp, _vp,
                                  _u64, _vp, _i32p, _u64p]),
    "oxh_files_modified_ex": (_int, [_vp, ctypes.POINTER(ctypes.c_char_p), _u64p, _u64p, _vp, _u64p, _vp, _vp, _vp, _vp,
                                     _u64, _vp, _i32p, _i32p, _u64p]),
    "oxh_pool_create": (_int, [_vp, _int, _int, _int, _u64, ctypes.POINTER(_vp)]),
    "oxh_pool_hash_files": (_int, [_vp, ctypes.POINTER(ctypes.c_char_p), _vp, _u64, _u64p, _u64p, _i32p]),
    "oxh_pool_hash_files_ex": (_int, [_vp, ctypes.POINTER(ctypes.c_char_p), _vp, _u64, _u64p, _u64p, _i32p, _i32p]),
    "oxh_pool_size": (_int, [_vp, ctypes.POINTER(_int), _vp]),
    "oxh_pool_destroy": (_int, [_vp]),
    "oxh_utf8_prefix_device": (_int, [_vp, _vp, _vp, _u64, _vp, _vp]),
    "oxh_combined_hash_device": (_int, [_vp, _vp, _u64, _vp, _vp]),
    "oxh_hash_streams": (_int, [_vp, _vp, _u64p, _u64p, _u64, _u64p]),
    "oxh_format_hex": (_int, [_u64, _u64, ctypes.c_char_p]),
    "oxh_format_dec": (_int, [_u64, _u64, ctypes.c_char_p]),
    "oxh_fill_splitmix": (_int, [_vp, _u64, _u64, _vp]),
    "oxh_set_kernel_variant": (_int, [_int]),
    "oxh_xxh3_stream_create": (_int, [_vp, ctypes.POINTER(_vp)]),
    "oxh_xxh3_stream_update": (_int, [_vp, _vp, _u64]),
    "oxh_xxh3_stream_digest": (_int, [_vp, _u64p]),
    "oxh_xxh3_stream_reset": (_int, [_vp]),
    "oxh_xxh3_stream_destroy": (_int, [_vp]),
    "oxh_fastcdc_device": (_int, [_vp, _u64p, _u64p, _u64, _u32, _u32, _u32, _u32, _vp, _vp, _vp, _u64, _u64p, _vp]),
    "oxh_fastcdc_max_chunks": (_u64, [_u64p, _u64, _u32]),
    "oxh_fastcdc_files": (_int, [_vp, ctypes.POINTER(ctypes.c_char_p), _u64, _u32, _u32, _u32, _u32, _u64p, _u64p, _u64p,
                                 _u64, _u64p, _u64p, _i32p, _i32p]),
    "oxh_fastcdc_host": (_int, [_vp, ctypes.POINTER(ctypes.c_char_p), _u64p, _u64, _u32, _u32, _u32, _u32, _u64p, _u64p,
                                _u64p, _u64, _u64p]),
    "oxh_chunk_digests_files": (_int, [_vp, ctypes.POINTER(ctypes.c_char_p), _u64, _u64, _u64p, _u64, _u64p, _u64p, _i32p,
                                       _i32p]),
    "oxh_chunk_digests_host": (_int, [_vp, ctypes.POINTER(ctypes.c_char_p), _u64p, _u64, _u64, _u64p, _u64, _u64p]),
    "oxh_fastcdc_files_multi": (_int, [ctypes.POINTER(_vp), _int, ctypes.POINTER(ctypes.c_char_p), _u64, _u32, _u32, _u32,
                                       _u32, _u64p, _u64p, _u64p, _u64, _u64p, _u64p, _i32p, _i32p]),
    "oxh_chunk_digests_files_multi": (_int, [ctypes.POINTER(_vp), _int, ctypes.POINTER(ctypes.c_char_p), _u64, _u64, _u64p,
                                             _u64, _u64p, _u64p, _i32p, _i32p]),
    "oxh_fastcdc_host_multi": (_int, [ctypes.POINTER(_vp), _int, ctypes.POINTER(ctypes.c_char_p), _u64p, _u64, _u32, _u32,
                                      _u32, _u32, _u64p, _u64p, _u64p, _u64, _u64p]),
    "oxh_chunk_digests_host_multi": (_int, [ctypes.POINTER(_vp), _int, ctypes.POINTER(ctypes.c_char_p), _u64p, _u64, _u64,
                                            _u64p, _u64, _u64p]),
    "oxh_fastcdc_gear": (_int, [_u64p]),
    "oxh_fastcdc_masks": (_int, [_u32, _u32, _u64p, _u64p]),
    "oxh_comm_check": (_int, [_int]),
    "oxh_ctx_counters": (_int, [_vp, _u64p, _int]),
    "oxh_comm_unique_id": (_int, [ctypes.c_char_p]),
    "oxh_comm_create": (_int, [ctypes.c_char_p, _int, _int, _int, ctypes.POINTER(_vp)]),
    "oxh_comm_info": (_int, [_vp, ctypes.POINTER(_int), ctypes.POINTER(_int), ctypes.POINTER(_int)]),
    "oxh_gather_digests": (_int, [_vp, _vp, _u64p, _vp, _int, _vp]),
    "oxh_comm_destroy": (_int, [_vp]),
}

_lib = None


class OxenError(Exception):
    """Mirror of liboxen's OxenError for this path (error/mod.rs); carries the C status code."""

    def __init__(self, msg: str, code: int = OXH_ERR_INVALID):
        super().__init__(msg)
        self.code = code


def header_symbols() -> list[str]:
    """Every function the public header declares."""
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:[\w\*\s]+?)\b(oxh_\w+)\s*\(", text, flags=re.M)))


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OxenError(f"{LIB_PATH} is missing: run `python -m oxen_amd.build` (no CPU fallback exists)",
                            OXH_ERR_NODEVICE)
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc: int, what: str) -> None:
    if rc != OXH_OK:
        msg = lib().oxh_last_error().decode(errors="replace")
        raise OxenError(f"{what} failed (status {rc}): {msg}", rc)


def device_count() -> int:
    n = _int(0)
    check(lib().oxh_device_count(ctypes.byref(n)), "oxh_device_count")
    return n.value


class Context:
    """An oxh_ctx: streams + pinned staging on one device."""

    def __init__(self, device: int = 0, staging_bytes: int = 0):
        h = _vp()
        check(lib().oxh_ctx_create(int(device), int(staging_bytes), ctypes.byref(h)), "oxh_ctx_create")
        self.handle = h
        self.device = device

    @property
    def stream(self) -> int:
        return lib().oxh_ctx_stream(self.handle) or 0

    def counters(self) -> dict:
        """oxh_ctx_counters: large-file piece-buffer allocations and their current bytes, file requests
        served on the caller's thread, file-engine runs."""
        out = (ctypes.c_uint64 * 4)()
        check(lib().oxh_ctx_counters(self.handle, out, 4), "oxh_ctx_counters")
        return {"big_allocs": int(out[0]), "big_bytes": int(out[1]), "direct_requests": int(out[2]),
                "engine_runs": int(out[3])}

    def close(self) -> None:
        if getattr(self, "handle", None):
            lib().oxh_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
