"""Debug probe: hash_files over path edge cases through the engine, each case in its own process
with a time limit (which one hangs?)."""
import os
import pathlib
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CASE = r'''
import os, sys, pathlib
sys.path.insert(0, %r)
from oxen_amd import _capi, hasher
from oxen_amd.workloads import splitmix_bytes
d = pathlib.Path(%r)
files = [str(d / n) for n in ["a.bin", "\u00fcn\u00efc\u00f6d\u00e9 \u2713.txt", "x y z", "empty"]]
case = %r
if case.endswith("_oracle"):
    from oracle import oracle
    case = case[:-len("_oracle")]
paths = {"dup": files * 50, "dup_small": files * 2, "empty_only": [files[3]] * 20, "link": [str(d / "link")],
         "dirs": [str(d / "dlink"), str(d)], "all": files * 50 + [str(d / "link"), str(d / "dlink"), str(d)],
         "one_dir": [str(d)], "file_then_dir": [files[0], str(d)]}[case]
if "oracle" in dir():
    oracle.hash_files(paths, threads=8)
    print("oracle done", flush=True)
with _capi.Context(0, staging_bytes=1 << 20) as c:
    dg, sz, st = hasher.hash_files_128bit(paths, c)
print(case, "ok", st[-3:], flush=True)
'''


def main():
    from oxen_amd.workloads import splitmix_bytes

    d = pathlib.Path("/tmp/edge/dir with space")
    d.mkdir(parents=True, exist_ok=True)
    for k, name in enumerate(["a.bin", "\u00fcn\u00efc\u00f6d\u00e9 \u2713.txt", "x y z", "empty"]):
        (d / name).write_bytes(b"" if name == "empty" else splitmix_bytes(60 + k, 0, 70_000 + k).tobytes())
    if not (d / "link").exists():
        (d / "link").symlink_to(d / "a.bin")
        (d / "dlink").symlink_to(d)
    for case in sys.argv[1:]:
        try:
            r = subprocess.run([sys.executable, "-c", CASE % (ROOT, str(d), case)], timeout=25, capture_output=True, text=True,
                               env=dict(os.environ, OXH_TRACE="1"))
            print(case, "rc", r.returncode, r.stdout.strip()[-200:], r.stderr.strip()[-300:], flush=True)
        except subprocess.TimeoutExpired as e:
            print(case, "TIMEOUT", (e.stderr or b"")[-300:], flush=True)


if __name__ == "__main__":
    main()
