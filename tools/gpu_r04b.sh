#!/bin/bash
# r04: the FastCDC walk (W + X) first -- its parity tests alone, then C5 at 8 KiB (walk vs scan, every
# chunk checked) and the rocprofv3 split of the walk call -- then the whole GPU suite and the
# configs[3] roofline record. Every step time-limited; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r04b}
step() {  # name, limit, command...
  local name=$1 lim=$2
  shift 2
  echo "== $name"
  timeout -k 10 "$lim" "$@" > "gpurun_out/${T}_$name.out" 2> "gpurun_out/${T}_$name.err" || {
    echo "$name failed"; tail -30 "gpurun_out/${T}_$name.err"; tail -30 "gpurun_out/${T}_$name.out"; exit 1; }
  tail -c 1500 "gpurun_out/${T}_$name.out"; echo
}
step cdc_tests 600 python -u -m pytest tests/test_fastcdc.py -m gpu -x -v --timeout 240 --timeout-method thread
step c5_8k_walk 400 env OXH_TRACE=1 python tools/bench_fastcdc.py --chunk 8192 --reps 5 --check-all
step c5_8k_scan 400 env OXH_CDC_WALK=0 python tools/bench_fastcdc.py --chunk 8192 --reps 5
step c5_8k_prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}_c5 -o run --output-format csv -- python tools/bench_fastcdc.py --chunk 8192 --reps 3
cp "$(find gpurun_out/prof_${T}_c5 -name '*kernel_stats.csv' | head -1)" gpurun_out/${T}_c5_8k_kernel_stats.csv
step pytest_all 900 python -u -m pytest tests -m gpu -v --maxfail 10 --timeout 300 --timeout-method thread
TAG=r04 WORKLOAD=c4 PMC=1 bash tools/gpu_profile_driver.sh
