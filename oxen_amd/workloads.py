"""Deterministic synthetic workloads for the BASELINE.json configs.

* `splitmix_bytes` is the host twin of `oxh_fill_splitmix` (byte j = byte j%8 LE of
  splitmix64(seed + (j//8 + 1) * 0x9E3779B97F4A7C15)); any item of a device-resident arena can be
  regenerated on the host without copying it back.
* `write_text_repo` restates benchmark/generate_text_repo.py:5-33 (C1).
* `write_image_repo` restates benchmark/generate_image_repo.py:8-90 (C3) with a seed (the
  reference is unseeded): uint8 noise images saved as TIFF by PIL, in `images/split_{i % dirs}`.
"""
from __future__ import annotations

import os

import numpy as np

GAMMA = np.uint64(0x9E3779B97F4A7C15)
C1 = np.uint64(0xBF58476D1CE4E5B9)
C2 = np.uint64(0x94D049BB133111EB)

# BASELINE.json configs (device-resident shapes)
C2_N, C2_LEN = 100_000, 65_536          # configs[1]
C4_N, C4_LEN = 1_000_000, 262_144       # configs[3] (125 000 per GPU at 8 GPUs)
C5_FILES, C5_LEN = 16, 8 << 30          # configs[4]
C3_IMAGES, C3_DIRS, C3_SIZE = 200_000, 1_000, (128, 128)  # configs[2]


def splitmix_words(seed: int, first_word: int, nwords: int) -> np.ndarray:
    with np.errstate(over="ignore"):
        idx = np.arange(first_word + 1, first_word + 1 + nwords, dtype=np.uint64)
        z = np.uint64(seed) + idx * GAMMA
        z = (z ^ (z >> np.uint64(30))) * C1
        z = (z ^ (z >> np.uint64(27))) * C2
        return z ^ (z >> np.uint64(31))


def splitmix_bytes(seed: int, start: int, nbytes: int) -> np.ndarray:
    """Bytes [start, start + nbytes) of the splitmix64 stream of `seed`."""
    if nbytes <= 0:
        return np.zeros(0, dtype=np.uint8)
    w0 = start // 8
    w1 = (start + nbytes + 7) // 8
    b = splitmix_words(seed, w0, w1 - w0).view(np.uint8)
    s = start - w0 * 8
    return b[s:s + nbytes].copy()


def packed_layout(lens, align: int = 256):
    """Offsets of items packed back to back at `align`-byte boundaries; returns (offsets, total)."""
    lens = np.asarray(lens, dtype=np.uint64)
    padded = (lens + np.uint64(align - 1)) // np.uint64(align) * np.uint64(align)
    offs = np.zeros(len(lens), dtype=np.uint64)
    if len(lens) > 1:
        offs[1:] = np.cumsum(padded[:-1])
    total = int(offs[-1] + lens[-1]) if len(lens) else 0
    return offs, total


def text_repo_files(num_files: int = 1000, output_dir: str = "text_files") -> dict[str, bytes]:
    """generate_text_repo.py:15-33: texts/file_{i}.txt = f"File content {i}" and README.md."""
    files = {os.path.join("texts", f"file_{i}.txt"): f"File content {i}".encode() for i in range(num_files)}
    files["README.md"] = f"# Sample Repo\n\nGenerated {num_files} text files in {output_dir}".encode()
    return files


def write_text_repo(root: str, num_files: int = 1000, output_dir: str = "text_files") -> list[str]:
    paths = []
    for rel, data in text_repo_files(num_files, output_dir).items():
        p = os.path.join(root, rel)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "wb") as f:
            f.write(data)
        paths.append(p)
    return paths


def image_bytes(i: int, seed: int = 0, size=(128, 128)) -> bytes:
    """One noise image of the C3 repo as TIFF bytes (PIL), seeded per index."""
    import io

    from PIL import Image

    rng = np.random.Generator(np.random.PCG64([seed, i]))
    noise = rng.integers(0, 256, (size[0], size[1], 3), dtype=np.uint8)
    buf = io.BytesIO()
    Image.fromarray(noise).save(buf, format="TIFF")
    return buf.getvalue()


_TIFF_HEADER = {}


def tiff_header(size=(128, 128)) -> bytes:
    """The 140-byte header + IFD PIL writes for an uncompressed RGB TIFF of this size (pixels follow)."""
    if size not in _TIFF_HEADER:
        import io

        from PIL import Image

        buf = io.BytesIO()
        Image.fromarray(np.zeros((size[0], size[1], 3), dtype=np.uint8)).save(buf, format="TIFF")
        b = buf.getvalue()
        _TIFF_HEADER[size] = b[: len(b) - size[0] * size[1] * 3]
    return _TIFF_HEADER[size]


def image_bytes_fast(i: int, seed: int = 0, size=(128, 128)) -> bytes:
    """C3 image i: PIL's TIFF header + splitmix64 noise pixels (bytes [i*P, (i+1)*P) of the stream)."""
    p = size[0] * size[1] * 3
    return tiff_header(size) + splitmix_bytes(seed, i * p, p).tobytes()


def write_image_repo_fast(root: str, num_images: int, num_dirs: int = 1000, seed: int = 0, size=(128, 128),
                          threads: int = 16) -> list[str]:
    """Config 3 at full scale in seconds: the same directory layout as generate_image_repo.py with
    TIFF files whose pixel bytes come from the splitmix64 stream (valid TIFFs, see tests)."""
    from concurrent.futures import ThreadPoolExecutor

    images = os.path.join(root, "images")
    for d in range(min(num_dirs, max(num_images, 1))):
        os.makedirs(os.path.join(images, f"split_{d}"), exist_ok=True)
    hdr = tiff_header(size)
    p = size[0] * size[1] * 3
    paths = [os.path.join(images, f"split_{i % num_dirs}", f"noise_image_{i}.tiff") for i in range(num_images)]
    chunk = 2000

    def work(c0):
        c1 = min(num_images, c0 + chunk)
        px = splitmix_bytes(seed, c0 * p, (c1 - c0) * p)
        for i in range(c0, c1):
            with open(paths[i], "wb") as f:
                f.write(hdr)
                f.write(px[(i - c0) * p:(i - c0 + 1) * p].tobytes())

    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(work, range(0, num_images, chunk)))
    labels = np.random.Generator(np.random.PCG64(seed)).choice(["cat", "dog"], size=num_images)
    with open(os.path.join(root, "images.csv"), "w") as f:
        f.write("images,labels\n")
        for path, lab in zip(paths, labels):
            f.write(f"{os.path.relpath(path, root)},{lab}\n")
    with open(os.path.join(root, "README.md"), "w") as f:
        f.write(f"# Sample Repo\n\nGenerated {num_images} images with {num_dirs} directories in {root}")
    return paths + [os.path.join(root, "images.csv"), os.path.join(root, "README.md")]


def write_image_repo(root: str, num_images: int, num_dirs: int = 1000, seed: int = 0, size=(128, 128)) -> list[str]:
    """generate_image_repo.py: images/split_{i % num_dirs}/noise_image_{i}.tiff (+ images.csv, README.md)."""
    images = os.path.join(root, "images")
    for d in range(min(num_dirs, max(num_images, 1))):
        os.makedirs(os.path.join(images, f"split_{d}"), exist_ok=True)
    paths = []
    for i in range(num_images):
        p = os.path.join(images, f"split_{i % num_dirs}", f"noise_image_{i}.tiff")
        with open(p, "wb") as f:
            f.write(image_bytes(i, seed, size))
        paths.append(p)
    labels = np.random.Generator(np.random.PCG64(seed)).choice(["cat", "dog"], size=num_images)
    with open(os.path.join(root, "images.csv"), "w") as f:
        f.write("images,labels\n")
        for p, lab in zip(paths, labels):
            f.write(f"{os.path.relpath(p, root)},{lab}\n")
    with open(os.path.join(root, "README.md"), "w") as f:
        f.write(f"# Sample Repo\n\nGenerated {num_images} images with {num_dirs} directories in {root}")
    return paths + [os.path.join(root, "images.csv"), os.path.join(root, "README.md")]
