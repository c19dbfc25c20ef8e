#!/bin/bash
# r04n: the extended smoke (FastCDC + K1R), K1R with default-policy loads (variant 266) against nt (264)
# on packed / aligned chunk-like items, and C5 8 KiB with each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r04n}
step() {  # name, limit, command...
  local name=$1 lim=$2
  shift 2
  echo "== $name"
  timeout -k 10 "$lim" "$@" > "gpurun_out/${T}_$name.out" 2> "gpurun_out/${T}_$name.err" || {
    echo "$name failed"; tail -30 "gpurun_out/${T}_$name.err"; tail -30 "gpurun_out/${T}_$name.out"; exit 1; }
  tail -c 400 "gpurun_out/${T}_$name.out"; echo
}
step smoke 240 python -c "import __graft_entry__ as g; g.smoke()"
step parity 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -k "every_length and 266"
step probe 400 env PROBE_CASES=cdc_packed,cdc_256,fixed_8k PROBE_WG=2,4 python tools/k1_small_probe.py 264 266
step c5_8k_266 400 env OXH_K1_PACKED_VARIANT=266 python tools/bench_fastcdc.py --chunk 8192 --reps 7
step c5_8k_264 400 env OXH_K1_PACKED_VARIANT=264 python tools/bench_fastcdc.py --chunk 8192 --reps 7
