"""CPU restatement of the block-level dedup's fixed-size chunk loops -- TEST INFRASTRUCTURE ONLY (the
checker for tests/, never called by the product path).

fixedsize.rs:67-91 (FixedSizeChunker::process_file):

    let mut input = BufReader::new(File::open(file_path)?);
    loop { let n = input.read(&mut buffer /* chunk_size */)?; if n == 0 { break }
           hash buffer[..n]; ...; if n < chunk_size { break } }

Rust's BufReader (std::io::BufReader, DEFAULT_BUF_SIZE 8 KiB) serves `read` from its buffer, filling
it with ONE read of the inner File when it is empty, except that an empty buffer and a request of at
least its capacity bypass it and read the File directly. A read(2) of a regular file on Linux returns
min(request, bytes left, MAX_RW_COUNT = 0x7ffff000). `reads()` below steps that state machine read by
read; the chunk extents it yields are what the reference hashes.

fixedsize_multithreaded.rs:78-110 (FixedSizeMultiChunker::split_file): chunk i = [i*chunk,
min((i+1)*chunk, size)), each read with seek + read_exact: `extents()`.

Parity pinned by stepping std's documented BufReader::read rule; the reference's Rust is not built
here (no toolchain), so no run of it backs these extents.
"""
from __future__ import annotations

BUF_CAPACITY = 8192          # std::sys::io::DEFAULT_BUF_SIZE
MAX_RW_COUNT = 0x7FFFF000    # Linux: INT_MAX & PAGE_MASK


def _file_read(pos: int, size: int, want: int) -> int:
    return max(0, min(want, size - pos, MAX_RW_COUNT))


def reads(size: int, chunk: int) -> list[tuple[int, int]]:
    """(offset, length) of every chunk fixedsize.rs's loop hashes for a `size`-byte regular file."""
    assert chunk > 0
    out = []
    pos = 0               # file position of the inner File
    buf_lo = buf_hi = 0   # buffered bytes = file [buf_lo, buf_hi); consumed up to `cur`
    cur = 0
    while True:
        if cur == buf_hi and chunk >= BUF_CAPACITY:  # bypass: buffer empty, large request
            n = _file_read(pos, size, chunk)
            off = pos
            pos += n
            cur = buf_lo = buf_hi = pos
        else:
            if cur == buf_hi:  # fill_buf: one read of up to the capacity
                k = _file_read(pos, size, BUF_CAPACITY)
                buf_lo, buf_hi = pos, pos + k
                pos += k
                cur = buf_lo
            n = min(chunk, buf_hi - cur)
            off = cur
            cur += n
        if n == 0:
            break
        out.append((off, n))
        if n < chunk:
            break
    return out


def extents(size: int, chunk: int) -> list[tuple[int, int]]:
    """fixedsize_multithreaded.rs:78-85: every chunk of the file."""
    return [(lo, min(chunk, size - lo)) for lo in range(0, size, chunk)]
