#!/bin/bash
# r06 A/B: the runtime split into translation units (oxen_amd/liboxen_hash.so) against the same code as
# one translation unit (tools/ab/presplit/liboxen_hash.so, built from the pre-split oxen_hash_capi.hip
# with the product flags), alternating on one box: bench.py's C2 step (K1 unchanged: xxh3_kernels.hip
# is the same object) and the rocprofv3 kernel average of each. Every step has its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
CMD="bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
for rep in 1 2 3; do
  for v in split presplit; do
    if [ $v = split ]; then RUN="python3 $CMD"; else RUN="python3 tools/with_lib.py tools/ab/presplit/liboxen_hash.so $CMD"; fi
    timeout -k 10 240 $RUN > gpurun_out/r06f_ab_${v}_$rep.json 2> gpurun_out/r06f_ab_${v}_$rep.err || { tail -20 gpurun_out/r06f_ab_${v}_$rep.err; exit 1; }
    echo "$v $rep $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], d['roofline']['kernel_ms'])" gpurun_out/r06f_ab_${v}_$rep.json)"
  done
done
for v in split presplit; do
  if [ $v = split ]; then RUN="python3 $CMD"; else RUN="python3 tools/with_lib.py tools/ab/presplit/liboxen_hash.so $CMD"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r06f_$v -o run --output-format csv -- $RUN \
    > gpurun_out/r06f_prof_$v.json 2> gpurun_out/r06f_prof_$v.err || { tail -20 gpurun_out/r06f_prof_$v.err; exit 1; }
  STATS=$(find gpurun_out/prof_r06f_$v -name '*kernel_stats.csv' | head -1)
  cp "$STATS" gpurun_out/r06f_${v}_kernel_stats.csv
  python3 tools/prof_summary.py --stats gpurun_out/r06f_${v}_kernel_stats.csv --bench gpurun_out/r06f_prof_$v.json \
    --command "$RUN" --workload c2 --out gpurun_out/r06f_profile_$v.json \
    --trace "$(find gpurun_out/prof_r06f_$v -name '*kernel_trace.csv' | head -1)" --warmup 5 --steps 20 || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'rocprof avg', d['avg_ms'], 'timed region', d['timed_region']['avg_ms'], d['timed_region']['frac'])" gpurun_out/r06f_profile_$v.json $v
done
