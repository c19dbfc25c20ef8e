"""A small version store with known corruption, for the `oxen fsck` (clean_corrupted_versions) tests."""
import os

import numpy as np


def make_version_store(root, digest_hex):
    """Build {root}/{hex[:2]}/{hex[2:]}/data blobs (digest_hex: bytes -> unpadded hex) and damage some.

    40 good blobs (incl. an empty one and a 2 MiB one), 3 blobs whose bytes no longer match their name,
    one suffix dir without `data`, one whose `data` is a directory, a stray file at the root (an error)
    and a stray file inside a prefix dir (skipped). Returns the expected results of a dry run, a real
    run and a second real run."""
    rng = np.random.default_rng(7)
    sizes = [0, 1, 15, 16, 17, 128, 129, 240, 241, 1024, 4096, 65536, 2 << 20]
    sizes += [int(s) for s in rng.integers(0, 200_000, 40 - len(sizes))]
    names = []
    for s in sizes:
        data = rng.integers(0, 256, s, dtype=np.uint8).tobytes()
        h = digest_hex(data)
        d = os.path.join(root, h[:2], h[2:])
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "data"), "wb") as f:
            f.write(data)
        names.append(h)
    for i in range(3):  # bit rot under an existing name
        data = rng.integers(0, 256, 3000 + i, dtype=np.uint8).tobytes()
        h = digest_hex(data)
        d = os.path.join(root, h[:2], h[2:])
        os.makedirs(d, exist_ok=True)
        bad = bytearray(data)
        bad[i * 7] ^= 0x40
        with open(os.path.join(d, "data"), "wb") as f:
            f.write(bytes(bad))
    os.makedirs(os.path.join(root, "ab", "cdef0000000000000000000000000001"))  # no data
    os.makedirs(os.path.join(root, "ab", "cdef0000000000000000000000000002", "data"))  # data is a dir
    with open(os.path.join(root, "README"), "w") as f:
        f.write("not a prefix dir\n")
    with open(os.path.join(root, names[5][:2], "stray.txt"), "w") as f:
        f.write("skipped\n")
    dry = {"scanned": 43, "corrupted": 3, "cleaned": 0, "errors": 3}
    real = {"scanned": 43, "corrupted": 3, "cleaned": 5, "errors": 3}
    again = {"scanned": 40, "corrupted": 0, "cleaned": 0, "errors": 1}
    return dry, real, again
