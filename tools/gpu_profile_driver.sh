#!/bin/bash
# The driver's own bench command, profiled: one plain run, then the SAME command under
# rocprofv3 --kernel-trace --stats, summarised by tools/prof_summary.py into profiles/<TAG>_profile_c2.json
# (bench.py reports that file's average beside its HIP-event kernel time). Every GPU step has its own
# time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r03}
CMD="bench.py --gpus 1 --steps 20 --warmup 5"
mkdir -p gpurun_out
echo "== bench" && timeout -k 10 300 python3 $CMD > gpurun_out/${TAG}_bench_c2.json 2> gpurun_out/${TAG}_bench_c2.err || { tail -20 gpurun_out/${TAG}_bench_c2.err; exit 1; }
cat gpurun_out/${TAG}_bench_c2.json
echo "== rocprofv3 kernel trace of the same command"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python3 $CMD \
  > gpurun_out/${TAG}_prof_bench_c2.json 2> gpurun_out/${TAG}_prof_bench_c2.err || { tail -20 gpurun_out/${TAG}_prof_bench_c2.err; exit 1; }
STATS=$(find gpurun_out/prof_${TAG} -name '*kernel_stats.csv' | head -1)
cp "$STATS" gpurun_out/${TAG}_c2_kernel_stats.csv
python3 tools/prof_summary.py --stats gpurun_out/${TAG}_c2_kernel_stats.csv --bench gpurun_out/${TAG}_prof_bench_c2.json \
  --command "python3 $CMD" --workload c2 --out gpurun_out/${TAG}_profile_c2.json \
  --trace "$(find gpurun_out/prof_${TAG} -name '*kernel_trace.csv' | head -1)" --warmup 5 --steps 20
