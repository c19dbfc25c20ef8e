#!/bin/bash
# Alternating bench.py runs of two K1 variants (C2), one JSON line each: VARIANTS="8 4" REPS=4
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in $(seq 1 ${REPS:-4}); do
  for v in ${VARIANTS:-8 4}; do
    timeout -k 10 120 python3 bench.py --steps 100 --warmup 5 --no-cpu-baseline --variant $v 2>/dev/null | \
      python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'variant': $v, 'value': d['value'], 'kernel_ms': d['roofline']['kernel_ms'], 'TBs': d['roofline']['achieved']}))" || exit 1
  done
done
