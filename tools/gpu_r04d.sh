#!/bin/bash
# r04d: X's bulk list copy; FastCDC tests, C5 8 KiB walk (checked) + kernel split; then the
# concurrent device / engine soak with forced piece-buffer regrowth.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r04d}
step() {  # name, limit, command...
  local name=$1 lim=$2
  shift 2
  echo "== $name"
  timeout -k 10 "$lim" "$@" > "gpurun_out/${T}_$name.out" 2> "gpurun_out/${T}_$name.err" || {
    echo "$name failed"; tail -30 "gpurun_out/${T}_$name.err"; tail -30 "gpurun_out/${T}_$name.out"; exit 1; }
  tail -c 700 "gpurun_out/${T}_$name.out"; echo
}
step cdc_tests 600 python -u -m pytest tests/test_fastcdc.py tests/test_gpu_publish.py -m gpu -x -q --timeout 240 --timeout-method thread
step c5_8k_walk 400 env OXH_TRACE=1 python tools/bench_fastcdc.py --chunk 8192 --reps 7 --check-all
step c5_8k_prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}_c5 -o run --output-format csv -- python tools/bench_fastcdc.py --chunk 8192 --reps 3
cp "$(find gpurun_out/prof_${T}_c5 -name '*kernel_stats.csv' | head -1)" gpurun_out/${T}_c5_8k_kernel_stats.csv
echo "== soak"
TAG=$T bash tools/gpu_soak_r04.sh
