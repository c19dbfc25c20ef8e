#!/bin/bash
# The driver's own bench command, profiled: one plain run, then the SAME command under
# rocprofv3 --kernel-trace --stats, summarised by tools/prof_summary.py into
# profiles/<TAG>_profile_<WORKLOAD>.json (bench.py reports that file's average beside its HIP-event
# kernel time). With PMC=1 two more passes of a short run of the workload collect FETCH_SIZE and
# WRITE_SIZE (separate passes: they do not fit one TCC pass) and tools/pmc_traffic.py turns them into
# <TAG>_traffic_<WORKLOAD>.json. Every GPU step has its own time limit; the chain stops at the first
# failure.
#   TAG=r04 WORKLOAD=c4 PMC=1 tools/gpu_profile_driver.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r04}
W=${WORKLOAD:-c2}
case $W in
  c2) ALG=6553600000 ;;     # 100 000 x 65 536 B per launch
  c4) ALG=32768000000 ;;    # 125 000 x 262 144 B per launch (one rank's shard of configs[3])
  *) echo "unknown workload $W"; exit 2 ;;
esac
CMD="bench.py --gpus 1 --steps 20 --warmup 5"
[ "$W" != c2 ] && CMD="$CMD --workload $W"
mkdir -p gpurun_out
echo "== bench $W"
timeout -k 10 300 python3 $CMD > gpurun_out/${TAG}_bench_$W.json 2> gpurun_out/${TAG}_bench_$W.err || { tail -20 gpurun_out/${TAG}_bench_$W.err; exit 1; }
cat gpurun_out/${TAG}_bench_$W.json
echo "== rocprofv3 kernel trace of the same command"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_$W -o run --output-format csv -- python3 $CMD \
  > gpurun_out/${TAG}_prof_bench_$W.json 2> gpurun_out/${TAG}_prof_bench_$W.err || { tail -20 gpurun_out/${TAG}_prof_bench_$W.err; exit 1; }
STATS=$(find gpurun_out/prof_${TAG}_$W -name '*kernel_stats.csv' | head -1)
cp "$STATS" gpurun_out/${TAG}_${W}_kernel_stats.csv
python3 tools/prof_summary.py --stats gpurun_out/${TAG}_${W}_kernel_stats.csv --bench gpurun_out/${TAG}_prof_bench_$W.json \
  --command "python3 $CMD" --workload $W --out gpurun_out/${TAG}_profile_$W.json \
  --trace "$(find gpurun_out/prof_${TAG}_$W -name '*kernel_trace.csv' | head -1)" --warmup 5 --steps 20 || exit 1
if [ "${PMC:-0}" = 1 ]; then
  SHORT="bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline"
  [ "$W" != c2 ] && SHORT="$SHORT --workload $W"
  for C in FETCH_SIZE WRITE_SIZE; do
    echo "== rocprofv3 --pmc $C"
    timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/pmc_${TAG}_${W}_$C -o run --output-format csv -- python3 $SHORT \
      > gpurun_out/${TAG}_pmc_${W}_$C.out 2> gpurun_out/${TAG}_pmc_${W}_$C.err || { tail -20 gpurun_out/${TAG}_pmc_${W}_$C.err; exit 1; }
  done
  python3 tools/pmc_traffic.py --fetch gpurun_out/pmc_${TAG}_${W}_FETCH_SIZE --write gpurun_out/pmc_${TAG}_${W}_WRITE_SIZE \
    --workload $W --algorithmic-bytes $ALG --out gpurun_out/${TAG}_traffic_$W.json || exit 1
fi
