#!/bin/bash
# r04c: X rewritten (4 KiB cut steps, grid-stride pass, sparse retry). FastCDC tests, C5 at 8 KiB with
# every chunk checked, the kernel split, and a warm-up sweep.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r04c}
step() {  # name, limit, command...
  local name=$1 lim=$2
  shift 2
  echo "== $name"
  timeout -k 10 "$lim" "$@" > "gpurun_out/${T}_$name.out" 2> "gpurun_out/${T}_$name.err" || {
    echo "$name failed"; tail -30 "gpurun_out/${T}_$name.err"; tail -30 "gpurun_out/${T}_$name.out"; exit 1; }
  tail -c 900 "gpurun_out/${T}_$name.out"; echo
}
step cdc_tests 600 python -u -m pytest tests/test_fastcdc.py -m gpu -x -q --timeout 240 --timeout-method thread
step c5_8k_walk 400 env OXH_TRACE=1 python tools/bench_fastcdc.py --chunk 8192 --reps 5 --check-all
step c5_8k_prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}_c5 -o run --output-format csv -- python tools/bench_fastcdc.py --chunk 8192 --reps 3
cp "$(find gpurun_out/prof_${T}_c5 -name '*kernel_stats.csv' | head -1)" gpurun_out/${T}_c5_8k_kernel_stats.csv
for wu in 0 16384 49152 65536; do
  step c5_8k_wu$wu 300 env OXH_CDC_WARMUP_BYTES=$wu python tools/bench_fastcdc.py --chunk 8192 --reps 5
done
step c5_8k_late 300 env OXH_CDC_WALK_LATE=1 python tools/bench_fastcdc.py --chunk 8192 --reps 5
step c5_8k_scan 300 env OXH_CDC_WALK=0 python tools/bench_fastcdc.py --chunk 8192 --reps 5
