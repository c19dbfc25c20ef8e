"""Stress the streaming engine with the path edge-case mix (duplicates, empty files, directories,
symlinks, tiny staging) many times in one process; a stalled request prints the engine state after
OXH_WAIT_LIMIT_S seconds (set it low here). Prints one line per iteration."""
import os
import pathlib
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    from oxen_amd import _capi, hasher
    from oxen_amd.workloads import splitmix_bytes

    d = pathlib.Path(os.environ.get("TMPDIR", "/tmp")) / "oxh_stress" / "dir with space"
    d.mkdir(parents=True, exist_ok=True)
    files = []
    for k, name in enumerate(["a.bin", "ünïcödé ✓.txt", "x y z", "empty"]):
        p = d / name
        p.write_bytes(b"" if name == "empty" else splitmix_bytes(60 + k, 0, 70_000 + k).tobytes())
        files.append(str(p))
    if not (d / "link").exists():
        (d / "link").symlink_to(files[0])
        (d / "dlink").symlink_to(d)
    paths = files * 50 + [str(d / "link"), str(d / "dlink"), str(d)]
    ref = None
    for it in range(iters):
        t0 = time.perf_counter()
        with _capi.Context(0, staging_bytes=1 << 20) as c:
            for _ in range(5):
                dg, sz, st = hasher.hash_files_128bit(paths, c)
                if ref is None:
                    ref = (dg, st)
                assert (dg, st) == ref
        print(f"iter {it} ok {time.perf_counter() - t0:.3f}s", flush=True)


if __name__ == "__main__":
    main()
