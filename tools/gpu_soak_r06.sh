#!/bin/bash
# One soak of the r06 tree (the runtime split into translation units, large-file buffers sized once per
# context, the host chunk entries' descriptor budget): the engine soak with --regrow --mutate and a
# device soak in a second process beside it, then the host chunk soak. Every step has its own limit;
# outputs under gpurun_out/${TAG}_*.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r06s}
S=${SECS:-300}
timeout -k 10 $(( S + 150 )) python -u tools/device_soak.py --seconds $(( S + 30 )) --seed 61 \
  > gpurun_out/${T}_device_soak.json 2> gpurun_out/${T}_device_soak.err &
DP=$!
timeout -k 10 $(( S + 120 )) python -u tools/engine_soak.py --seconds $S --regrow --mutate --seed 61 \
  > gpurun_out/${T}_engine_soak.json 2> gpurun_out/${T}_engine_soak.err
rc=$?
echo "engine_soak rc=$rc"; tail -c 700 gpurun_out/${T}_engine_soak.json; echo
wait $DP; drc=$?
echo "device_soak rc=$drc"; tail -c 400 gpurun_out/${T}_device_soak.json; echo
[ $rc = 0 ] && [ $drc = 0 ] || exit 1
timeout -k 10 $(( ${CDC_SECS:-180} + 120 )) python -u tools/cdc_host_soak.py --seconds ${CDC_SECS:-180} --seed 61 \
  > gpurun_out/${T}_host_chunk_soak.json 2> gpurun_out/${T}_host_chunk_soak.err
rc=$?
echo "host_chunk_soak rc=$rc"; tail -c 500 gpurun_out/${T}_host_chunk_soak.json; echo
exit $rc
