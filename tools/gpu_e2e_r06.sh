#!/bin/bash
# End-to-end configs on the final r06 tree (one box): C1 (`oxen add .` on the 1 001-file text repo), C3
# (200 002 files on disk -> digests, add, fsck), C5 device-resident (FastCDC 64 / 8 KiB), and C5 end to
# end from the page cache (16 x 8 GiB in /dev/shm, FastCDC 8 KiB and fixed-size 64 KiB). Every step has
# its own limit and the chain stops at the first failure; outputs under gpurun_out/${TAG}_*.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r06e2e}
mkdir -p gpurun_out
step() {  # name, limit, command...
  local name=$1 lim=$2
  shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 "$lim" "$@" > "gpurun_out/${TAG}_$name.json" 2> "gpurun_out/${TAG}_$name.err" || {
    echo "$name failed"; tail -20 "gpurun_out/${TAG}_$name.err"; exit 1; }
  tail -c 900 "gpurun_out/${TAG}_$name.json"; echo
}
step c1 240 python3 tools/bench_c1.py --reps 5
step c3 600 python3 tools/bench_e2e.py --staging-mib 256 --procs 2
step c5dev_64k 300 python3 tools/bench_fastcdc.py --chunk 65536 --reps 5
step c5dev_8k 300 python3 tools/bench_fastcdc.py --chunk 8192 --reps 5
step c5e2e_8k 600 python3 tools/bench_fastcdc_e2e.py --dir /dev/shm/oxh_c5 --chunk 8192 --reps 2 --keep
step c5e2e_fixed64k 600 python3 tools/bench_fastcdc_e2e.py --dir /dev/shm/oxh_c5 --chunk 65536 --reps 2 --fixed
rm -rf /dev/shm/oxh_c5
