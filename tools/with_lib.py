"""Run a tools/ script against another build of the library (diagnostic A/B builds):
    python tools/with_lib.py LIB.so tools/bench_fastcdc.py [args...]"""
import runpy
import sys

import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oxen_amd import _capi  # noqa: E402

_capi.LIB_PATH = os.path.abspath(sys.argv[1])
sys.argv = sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
