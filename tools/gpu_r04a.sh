#!/bin/bash
# r04 first GPU call: the GPU suite on the current tree, then the configs[3] (C4 shard) roofline record
# (kernel trace of the driver-shaped command + FETCH / WRITE PMC passes). Each step time-limited;
# the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail 10 --timeout 300 --timeout-method thread \
  > gpurun_out/r04a_pytest_gpu.log 2>&1
rc=$?
tail -30 gpurun_out/r04a_pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
TAG=r04 WORKLOAD=c4 PMC=1 bash tools/gpu_profile_driver.sh
