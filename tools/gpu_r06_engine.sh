#!/bin/bash
# One session for the r06 engine changes (small requests on the caller's thread, K1L for a staged batch's
# large items, large files read in parts): the engine soak with --split --mutate --regrow, then C1 and C3
# end to end and the per-call latency probe, each against the oracle. Every step has its own limit and
# the chain stops at the first failure; outputs under gpurun_out/${TAG}_*.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r06z2}
S=${SECS:-240}
mkdir -p gpurun_out
step() {  # name, limit, command...
  local name=$1 lim=$2
  shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$lim" "$@" > "gpurun_out/${TAG}_$name.json" 2> "gpurun_out/${TAG}_$name.err" || {
    echo "$name failed"; tail -20 "gpurun_out/${TAG}_$name.err"; exit 1; }
  tail -c 900 "gpurun_out/${TAG}_$name.json"; echo
}
step engine_soak $(( S + 150 )) python3 -u tools/engine_soak.py --seconds $S --split --mutate --regrow --seed 62
step c1 240 python3 tools/bench_c1.py --reps 5
step c3 600 python3 tools/bench_e2e.py --staging-mib 256 --procs 2
step latency 150 python3 tools/latency_probe.py --calls 400
