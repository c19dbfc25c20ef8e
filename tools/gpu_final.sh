#!/bin/bash
# End-of-round sweep on one GPU box: the GPU suite, smoke, the C2 headline bench, the C4 per-GPU shard,
# and C5 (FastCDC at 64 / 8 KiB chunks, fixed-size chunks and whole-file digests). Every step has its
# own time limit and the chain stops at the first failure. Outputs under gpurun_out/${TAG}_*.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-final}
mkdir -p gpurun_out
step() {  # name, limit, command...
  local name=$1 lim=$2
  shift 2
  echo "== $name"
  timeout -k 10 "$lim" "$@" > "gpurun_out/${TAG}_$name.out" 2> "gpurun_out/${TAG}_$name.err" || {
    echo "$name failed"; tail -20 "gpurun_out/${TAG}_$name.err"; tail -5 "gpurun_out/${TAG}_$name.out"; exit 1; }
  tail -c 600 "gpurun_out/${TAG}_$name.out"; echo
}
step pytest 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_c2 300 python bench.py --steps 20 --warmup 3
step bench_c4 300 python bench.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline
step fastcdc_64k 300 python tools/bench_fastcdc.py --chunk 65536 --reps 5
step fastcdc_8k 300 python tools/bench_fastcdc.py --chunk 8192 --reps 5
step c5 600 python tools/bench_c5.py --reps 3
