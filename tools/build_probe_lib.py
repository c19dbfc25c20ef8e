"""Probe build of the library: every K1 variant the A/Bs of DESIGN.md §4 measured, not only the shipped
ones. The product library (oxen_amd/liboxen_hash.so) instantiates 0 / 8 / 72 / 104 / 264; this build
adds 1 2 4 12 40 64 74 256 260 768 772 776 (-DOXH_PROBE_VARIANTS) and FastCDC's folded walk W2 + K1F
(-DOXH_PROBE_FOLD, selected by OXH_CDC_FOLD=1; DESIGN §4 "W2") into tools/probe/liboxen_hash.so.
Use it through tools/with_lib.py:
    python tools/build_probe_lib.py
    python tools/with_lib.py tools/probe/liboxen_hash.so tools/k1_small_probe.py ...
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oxen_amd import build as b  # noqa: E402

OUT = os.path.join(ROOT, "tools", "probe", "liboxen_hash.so")

if __name__ == "__main__":
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    print(b.compile_lib(OUT, defines=("OXH_PROBE_VARIANTS", "OXH_PROBE_FOLD"), verbose="-v" in sys.argv))
