#!/bin/bash
# One engine soak (--regrow, default 1 GiB large-file pieces) under the env given in $VARIANT_ENV, with
# DEV=1 a device soak in a second process beside it (the r05n shape), for chasing the r05 stall
# (profiles/r05/INDEX.md). Output under gpurun_out/${TAG}_*.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r05s}
echo "== soak env: ${VARIANT_ENV:-none} dev=${DEV:-0} $(date +%T)"
if [ "${DEV:-0}" = 1 ]; then
  timeout -k 10 $(( ${SECS:-60} + 120 )) python -u tools/device_soak.py --seconds $(( ${SECS:-60} + 30 )) \
    > gpurun_out/${T}_device_soak.json 2> gpurun_out/${T}_device_soak.err &
  DP=$!
fi
timeout -k 10 ${LIMIT:-150} env ${VARIANT_ENV:-OXH_NONE=0} python -u tools/engine_soak.py --seconds ${SECS:-60} --regrow ${MUTATE:+--mutate} ${SEED:+--seed $SEED} \
  > gpurun_out/${T}_engine_soak.json 2> gpurun_out/${T}_engine_soak.err
rc=$?
echo "engine_soak rc=$rc"
tail -c 700 gpurun_out/${T}_engine_soak.json; echo
grep -c "stalled" gpurun_out/${T}_engine_soak.err
grep -m6 "ctx 0x" gpurun_out/${T}_engine_soak.err
if [ -n "${DP:-}" ]; then wait $DP; echo "device_soak rc=$?"; tail -c 300 gpurun_out/${T}_device_soak.json; echo; fi
exit $rc
