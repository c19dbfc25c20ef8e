"""Block-level dedup chunkers on the GPU.

Mirrors experiments/block-level-dedup/src/chunker/fastcdchunker.rs (`FastCDChunker`): the file is
chunked with FastCDC v2020 (min 4096, avg = chunk_size, max = 2 * chunk_size, :55-57, :83-88) and
every chunk is written to `output_dir/<decimal xxh3_128 of the chunk>` (:96-107); the chunk names go
to `metadata.bin` as bincode 1.x of `ChunkMetadata {original_file_name: String, original_file_size:
u64, chunks: Vec<String>}` (:11-16, :110-121). Boundaries and digests both come from the GPU
(`oxh_fastcdc_device`: FastCDC candidate scan + speculative walks + K1 over the chunk table).
"""
from __future__ import annotations

import os
import struct
from typing import Optional

import numpy as np
import torch

from . import _capi
from .device import fastcdc_device, to_numpy_u64

METADATA_FILE_NAME = "metadata.bin"  # fastcdchunker.rs:18
MIN_CHUNK_SIZE = 4096                # fastcdchunker.rs:55


def chunk_name(lo: int, hi: int) -> str:
    """u128::to_string() of the chunk digest (fastcdchunker.rs:98)."""
    return str((int(hi) << 64) | int(lo))


def _bincode_string(s: str) -> bytes:
    b = s.encode("utf-8")
    return struct.pack("<Q", len(b)) + b


def encode_metadata(original_file_name: str, original_file_size: int, chunks: list[str]) -> bytes:
    """bincode 1.x default (fixint, little-endian, u64 lengths) of ChunkMetadata."""
    out = [_bincode_string(original_file_name), struct.pack("<Q", original_file_size), struct.pack("<Q", len(chunks))]
    out += [_bincode_string(c) for c in chunks]
    return b"".join(out)


def decode_metadata(buf: bytes) -> tuple[str, int, list[str]]:
    pos = 0

    def take(n):
        nonlocal pos
        if pos + n > len(buf):
            raise _capi.OxenError("Bincode error: unexpected end of metadata", _capi.OXH_ERR_IO)
        v = buf[pos:pos + n]
        pos += n
        return v

    def string():
        (n,) = struct.unpack("<Q", take(8))
        return take(n).decode("utf-8")

    name = string()
    (size,) = struct.unpack("<Q", take(8))
    (count,) = struct.unpack("<Q", take(8))
    return name, size, [string() for _ in range(count)]


class FastCDChunker:
    """fastcdchunker.rs:30-66 + the Chunker trait (chunker.rs): name / pack / unpack / get_chunk_hashes."""

    def __init__(self, chunk_size: int, concurrency: int = 1, device: Optional[str] = None):
        if chunk_size == 0:
            raise ValueError("Chunk size cannot be zero")
        if concurrency == 0:
            raise ValueError("Concurrency must be greater than zero")
        self.min_chunk_size = MIN_CHUNK_SIZE
        self.avg_chunk_size = int(chunk_size)
        self.max_chunk_size = int(chunk_size) * 2
        self.device = device or "cuda"

    def name(self) -> str:
        return "fastcdc-chunker"

    def chunk_buffer(self, data: torch.Tensor):
        """(offsets, lengths, digests) of one device-resident buffer, as numpy uint64 arrays."""
        c_off, c_len, dig, _ = fastcdc_device(data, [0], [data.numel()], self.min_chunk_size, self.avg_chunk_size,
                                              self.max_chunk_size)
        return to_numpy_u64(c_off), to_numpy_u64(c_len), to_numpy_u64(dig).reshape(-1, 2)

    def pack(self, input_file: str, output_dir: str) -> str:
        os.makedirs(output_dir, exist_ok=True)
        with open(input_file, "rb") as fh:
            content = fh.read()
        size = os.stat(input_file).st_size
        host = torch.frombuffer(bytearray(content), dtype=torch.uint8) if content else torch.empty(0, dtype=torch.uint8)
        dev = host.to(self.device)
        offs, lens, digs = self.chunk_buffer(dev)
        names = []
        for o, l, (lo, hi) in zip(offs, lens, digs):
            name = chunk_name(lo, hi)
            names.append(name)
            with open(os.path.join(output_dir, name), "wb") as out:
                out.write(content[int(o):int(o) + int(l)])
        base = os.path.basename(os.path.normpath(input_file)) or "unknown_file"
        with open(os.path.join(output_dir, METADATA_FILE_NAME), "wb") as meta:
            meta.write(encode_metadata(base, size, names))
        return output_dir

    def unpack(self, input_dir: str, output_path: str) -> str:
        """The reference leaves this unimplemented (fastcdchunker.rs:124-127); here: concatenate the
        chunks listed in metadata.bin."""
        _, _, chunks = decode_metadata(open(os.path.join(input_dir, METADATA_FILE_NAME), "rb").read())
        with open(output_path, "wb") as out:
            for c in chunks:
                with open(os.path.join(input_dir, c), "rb") as fh:
                    out.write(fh.read())
        return output_path

    def get_chunk_hashes(self, input_dir: str) -> list[str]:
        return decode_metadata(open(os.path.join(input_dir, METADATA_FILE_NAME), "rb").read())[2]


def fastcdc_gear() -> list[int]:
    """The GEAR table compiled into the library (host call, no GPU needed)."""
    out = np.zeros(256, dtype=np.uint64)
    _capi.check(_capi.lib().oxh_fastcdc_gear(out.ctypes.data_as(_capi._u64p)), "oxh_fastcdc_gear")
    return [int(v) for v in out]


def fastcdc_masks(avg_size: int, level: int = 1) -> tuple[int, int]:
    s = np.zeros(1, dtype=np.uint64)
    l = np.zeros(1, dtype=np.uint64)
    _capi.check(_capi.lib().oxh_fastcdc_masks(int(avg_size), int(level), s.ctypes.data_as(_capi._u64p),
                                              l.ctypes.data_as(_capi._u64p)), "oxh_fastcdc_masks")
    return int(s[0]), int(l[0])
