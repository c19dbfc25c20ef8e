"""Device-resident entry points over torch-allocated HBM buffers.

PyTorch is plumbing here (device memory, the current HIP stream, torch.distributed); the hashing is
the C ABI (include/oxen_hash.h). Digest tables are int64 tensors of shape (n, 2) holding the raw
u64 words (lo, hi); `to_u128_list` turns them into Python ints.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from . import _capi
from .workloads import packed_layout


def _stream(stream) -> int:
    if stream is None:
        return torch.cuda.current_stream().cuda_stream
    return int(getattr(stream, "cuda_stream", stream))


def _require_cuda(*ts: torch.Tensor) -> None:
    for t in ts:
        if not t.is_cuda:
            raise _capi.OxenError("device entry points take device-resident tensors", _capi.OXH_ERR_INVALID)


def xxh3_128_batch_device(arena: torch.Tensor, offsets: torch.Tensor, lens: torch.Tensor,
                          out: Optional[torch.Tensor] = None, mode: int = _capi.OXH_MODE_AUTO,
                          stream=None) -> torch.Tensor:
    """K1/K1s over arena[offsets[i] : offsets[i] + lens[i]] (all on the device)."""
    _require_cuda(arena, offsets, lens)
    n = lens.numel()
    if offsets.numel() != n or offsets.element_size() != 8 or lens.element_size() != 8:
        raise _capi.OxenError("offsets/lens must be 64-bit and the same length", _capi.OXH_ERR_INVALID)
    if out is None:
        out = torch.empty((n, 2), dtype=torch.int64, device=arena.device)
    _capi.check(_capi.lib().oxh_xxh3_128_batch_device(arena.data_ptr(), offsets.data_ptr(), lens.data_ptr(), n,
                                                      out.data_ptr(), int(mode), _stream(stream)),
                "oxh_xxh3_128_batch_device")
    return out


def xxh3_128_text_batch_device(arena: torch.Tensor, offsets: torch.Tensor, lens: torch.Tensor,
                               out: Optional[torch.Tensor] = None, counts: Optional[torch.Tensor] = None,
                               stream=None):
    """K1T: digests + (num_lines, num_chars) per item in one HBM pass."""
    _require_cuda(arena, offsets, lens)
    n = lens.numel()
    if out is None:
        out = torch.empty((n, 2), dtype=torch.int64, device=arena.device)
    if counts is None:
        counts = torch.empty((n, 2), dtype=torch.int64, device=arena.device)
    _capi.check(_capi.lib().oxh_xxh3_128_text_batch_device(arena.data_ptr(), offsets.data_ptr(), lens.data_ptr(), n,
                                                           out.data_ptr(), counts.data_ptr(), _stream(stream)),
                "oxh_xxh3_128_text_batch_device")
    return out, counts


def chunk_digests_device(buf: torch.Tensor, chunk: int, nbytes: Optional[int] = None,
                         out: Optional[torch.Tensor] = None, stream=None) -> torch.Tensor:
    _require_cuda(buf)
    nbytes = buf.numel() * buf.element_size() if nbytes is None else nbytes
    n = (nbytes + chunk - 1) // chunk
    if out is None:
        out = torch.empty((n, 2), dtype=torch.int64, device=buf.device)
    _capi.check(_capi.lib().oxh_chunk_digests_device(buf.data_ptr(), nbytes, chunk, out.data_ptr(), _stream(stream)),
                "oxh_chunk_digests_device")
    return out


def large_digest_device(ctx: _capi.Context, buf: torch.Tensor, nbytes: Optional[int] = None,
                        out: Optional[torch.Tensor] = None, stream=None) -> torch.Tensor:
    _require_cuda(buf)
    nbytes = buf.numel() * buf.element_size() if nbytes is None else nbytes
    if out is None:
        out = torch.empty(2, dtype=torch.int64, device=buf.device)
    _capi.check(_capi.lib().oxh_xxh3_128_large_device(ctx.handle, buf.data_ptr(), nbytes, out.data_ptr(),
                                                      _stream(stream)), "oxh_xxh3_128_large_device")
    return out


def large_digests_device(bufs: list, nbytes: Optional[list] = None, out: Optional[torch.Tensor] = None,
                         stream=None) -> torch.Tensor:
    """K1L whole-buffer digests of several large device buffers (chains run concurrently)."""
    import ctypes

    _require_cuda(*bufs)
    n = len(bufs)
    nbytes = [b.numel() * b.element_size() for b in bufs] if nbytes is None else list(nbytes)
    if out is None:
        out = torch.empty((n, 2), dtype=torch.int64, device=bufs[0].device)
    ptrs = (ctypes.c_void_p * n)(*[b.data_ptr() for b in bufs])
    lens = np.array(nbytes, dtype=np.uint64)
    _capi.check(_capi.lib().oxh_xxh3_128_large_batch_device(ptrs, lens.ctypes.data_as(_capi._u64p), n, out.data_ptr(),
                                                            _stream(stream)), "oxh_xxh3_128_large_batch_device")
    return out


def combined_hash_device(content: torch.Tensor, metadata: torch.Tensor, out: Optional[torch.Tensor] = None,
                         stream=None) -> torch.Tensor:
    _require_cuda(content, metadata)
    n = content.shape[0]
    if out is None:
        out = torch.empty((n, 2), dtype=torch.int64, device=content.device)
    _capi.check(_capi.lib().oxh_combined_hash_device(content.data_ptr(), metadata.data_ptr(), n, out.data_ptr(),
                                                     _stream(stream)), "oxh_combined_hash_device")
    return out


def fill_splitmix(buf: torch.Tensor, seed: int, nbytes: Optional[int] = None, stream=None) -> None:
    _require_cuda(buf)
    nbytes = buf.numel() * buf.element_size() if nbytes is None else nbytes
    _capi.check(_capi.lib().oxh_fill_splitmix(buf.data_ptr(), nbytes, int(seed), _stream(stream)), "oxh_fill_splitmix")


def fastcdc_device(arena: torch.Tensor, offsets, lens, min_size: int, avg_size: int, max_size: int,
                   level: int = 1, digests: bool = True, stream=None, out=None):
    """FastCDC v2020 chunks (+ XXH3-128 of every chunk) of device-resident files
    arena[offsets[i] : offsets[i] + lens[i]] (offsets/lens are host sequences).
    Returns (chunk_offsets, chunk_lens, chunk_digests or None) as int64 device tensors and
    first_chunk (numpy uint64, n+1): file i's chunks are rows first_chunk[i] .. first_chunk[i+1].
    `out` = (c_off, c_len, dig) from fastcdc_outputs() reuses preallocated chunk tables."""
    _require_cuda(arena)
    offs = np.ascontiguousarray(offsets, dtype=np.uint64)
    ln = np.ascontiguousarray(lens, dtype=np.uint64)
    n = len(ln)
    if len(offs) != n:
        raise _capi.OxenError("offsets/lens must be the same length", _capi.OXH_ERR_INVALID)
    if n and int((offs + ln).max()) > arena.numel() * arena.element_size():
        raise _capi.OxenError("a file extends past the arena", _capi.OXH_ERR_INVALID)
    L = _capi.lib()
    if out is None:
        out = fastcdc_outputs(arena, ln, min_size, digests)
    c_off, c_len, dig = out
    if not digests:
        dig = None
    cap = c_off.numel()
    need = max(1, int(L.oxh_fastcdc_max_chunks(ln.ctypes.data_as(_capi._u64p), n, max(1, int(min_size)))))
    if cap < need or c_len.numel() < need or (dig is not None and dig.shape[0] < need):
        raise _capi.OxenError(f"chunk tables hold {cap} rows, need {need}", _capi.OXH_ERR_INVALID)
    first = np.zeros(n + 1, dtype=np.uint64)
    _capi.check(L.oxh_fastcdc_device(arena.data_ptr(), offs.ctypes.data_as(_capi._u64p), ln.ctypes.data_as(_capi._u64p),
                                     n, int(min_size), int(avg_size), int(max_size), int(level), c_off.data_ptr(),
                                     c_len.data_ptr(), dig.data_ptr() if dig is not None else None, cap,
                                     first.ctypes.data_as(_capi._u64p), _stream(stream)), "oxh_fastcdc_device")
    total = int(first[n])
    return c_off[:total], c_len[:total], (dig[:total] if dig is not None else None), first


def fastcdc_outputs(arena: torch.Tensor, lens, min_size: int, digests: bool = True):
    """Chunk tables sized for fastcdc_device over files of these lengths: (c_off, c_len, dig)."""
    ln = np.ascontiguousarray(lens, dtype=np.uint64)
    cap = max(1, int(_capi.lib().oxh_fastcdc_max_chunks(ln.ctypes.data_as(_capi._u64p), len(ln), max(1, int(min_size)))))
    c_off = torch.empty(cap, dtype=torch.int64, device=arena.device)
    c_len = torch.empty(cap, dtype=torch.int64, device=arena.device)
    dig = torch.empty((cap, 2), dtype=torch.int64, device=arena.device) if digests else None
    return c_off, c_len, dig


def to_numpy_u64(t: torch.Tensor) -> np.ndarray:
    return t.detach().cpu().numpy().view(np.uint64)


def to_u128_list(t: torch.Tensor) -> list[int]:
    a = to_numpy_u64(t).reshape(-1, 2)
    return [(int(hi) << 64) | int(lo) for lo, hi in a]


@dataclass
class DeviceArena:
    """A packed, device-resident batch of synthetic buffers (one HBM allocation + descriptors)."""

    arena: torch.Tensor
    offsets: torch.Tensor
    lens: torch.Tensor
    offsets_host: np.ndarray
    lens_host: np.ndarray
    seed: int

    @property
    def n(self) -> int:
        return len(self.lens_host)

    @property
    def payload_bytes(self) -> int:
        return int(self.lens_host.sum())

    @classmethod
    def splitmix(cls, lens, seed: int = 0, device="cuda", align: int = 256, pad: int = 0) -> "DeviceArena":
        """Items packed back to back at `align`-byte boundaries (plus `pad` spare bytes after each)."""
        lens_h = np.asarray(lens, dtype=np.uint64)
        offs_h, total = packed_layout(lens_h + np.uint64(pad), align)
        alloc = max(8, (total + 7) // 8 * 8)
        arena = torch.empty(alloc, dtype=torch.uint8, device=device)
        fill_splitmix(arena, seed, alloc)
        offs = torch.from_numpy(offs_h.view(np.int64)).to(device)
        ln = torch.from_numpy(lens_h.view(np.int64)).to(device)
        return cls(arena, offs, ln, offs_h, lens_h, seed)

    def hash(self, out: Optional[torch.Tensor] = None, mode: int = _capi.OXH_MODE_AUTO, stream=None) -> torch.Tensor:
        return xxh3_128_batch_device(self.arena, self.offsets, self.lens, out, mode, stream)
