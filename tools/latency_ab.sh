#!/bin/bash
# r06 latency A/B, one box, alternating: the runtime threads' timer slack (OXH_TIMER_SLACK_NS, default
# 1000 ns, 0 = the kernel's 50 us) and the staged-batch spin (OXH_SPIN_US, default 200, 0 = the r05
# form), on tools/latency_probe.py; then C3 end to end under both (throughput must not suffer).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for v in new old; do
    if [ $v = old ]; then E="OXH_TIMER_SLACK_NS=0 OXH_SPIN_US=0"; else E="OXH_NONE=0"; fi
    timeout -k 10 200 env $E python3 tools/latency_probe.py --calls 400 > gpurun_out/r06r_lat_${v}_$rep.json 2> gpurun_out/r06r_lat_${v}_$rep.err || { tail -5 gpurun_out/r06r_lat_${v}_$rep.err; exit 1; }
    echo "$v $rep $(cat gpurun_out/r06r_lat_${v}_$rep.json)"
  done
done
for v in new old; do
  if [ $v = old ]; then E="OXH_TIMER_SLACK_NS=0 OXH_SPIN_US=0"; else E="OXH_NONE=0"; fi
  timeout -k 10 400 env $E python3 tools/bench_e2e.py --staging-mib 256 --procs 2 --only-procs > gpurun_out/r06r_c3_$v.json 2> gpurun_out/r06r_c3_$v.err || { tail -5 gpurun_out/r06r_c3_$v.err; exit 1; }
  echo "$v c3 $(python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print({k: d[k] for k in d if 'warm' in k or 'cold' in k})" gpurun_out/r06r_c3_$v.json)"
done
