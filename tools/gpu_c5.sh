#!/bin/bash
# C5 session (BASELINE configs[4]: 16 x 8 GiB, FastCDC chunk table + chunk digests): wall time per chunk
# size, then a rocprofv3 kernel trace of the same command. Every GPU step has its own limit; the chain
# stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r02e}
CHUNKS=${CHUNKS:-"65536 8192"}
mkdir -p gpurun_out
for c in $CHUNKS; do
  echo "== fastcdc chunk=$c"
  timeout -k 10 300 python3 tools/bench_fastcdc.py --chunk $c --reps 5 > gpurun_out/${TAG}_fastcdc_$c.json 2> gpurun_out/fastcdc_$c.err \
    || { tail -20 gpurun_out/fastcdc_$c.err; exit 1; }
  cat gpurun_out/${TAG}_fastcdc_$c.json
  if [ -n "$PROFILE" ]; then
    echo "== rocprofv3 chunk=$c"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5_$c -o run --output-format csv -- \
      python3 tools/bench_fastcdc.py --chunk $c --reps 5 > /dev/null 2> gpurun_out/prof_c5_$c.err \
      || { tail -20 gpurun_out/prof_c5_$c.err; exit 1; }
    find gpurun_out/prof_c5_$c -name '*kernel_stats.csv' -exec cp {} gpurun_out/${TAG}_fastcdc_${c}_kernel_stats.csv \;
  fi
done
