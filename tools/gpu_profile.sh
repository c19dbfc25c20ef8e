#!/bin/bash
# Profiling session: read-bandwidth microbench, PMC traffic passes and kernel-trace stats of bench.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r01c}
WL=${WL:-c2}
mkdir -p gpurun_out
BENCH="python3 bench.py --workload $WL --steps 10 --warmup 2 --no-cpu-baseline"
echo "== readbw" && timeout -k 10 300 python3 tools/readbw.py > gpurun_out/readbw.json 2> gpurun_out/readbw.err || { tail gpurun_out/readbw.err; exit 1; }
cat gpurun_out/readbw.json
echo "== kernel trace" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- $BENCH > gpurun_out/prof_$TAG.json 2> gpurun_out/prof_$TAG.err || { tail gpurun_out/prof_$TAG.err; exit 1; }
echo "== pmc FETCH_SIZE" && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch_$TAG -o run --output-format csv -- $BENCH > /dev/null 2> gpurun_out/pmc_fetch.err || { tail gpurun_out/pmc_fetch.err; exit 1; }
echo "== pmc WRITE_SIZE" && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write_$TAG -o run --output-format csv -- $BENCH > /dev/null 2> gpurun_out/pmc_write.err || { tail gpurun_out/pmc_write.err; exit 1; }
python3 tools/pmc_traffic.py --fetch gpurun_out/pmc_fetch_$TAG --write gpurun_out/pmc_write_$TAG --workload $WL \
   --algorithmic-bytes $(python3 -c "import bench; n,l,_=bench.WORKLOADS['$WL']; print(n*l)") --out gpurun_out/${TAG}_traffic_$WL.json
echo "== bench" && timeout -k 10 600 python3 bench.py --workload $WL > gpurun_out/bench_$WL.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench_$WL.json
