#!/bin/bash
# the device entry points (tools/device_soak.py, its own process, 300 s) and the file
# engine with forced piece-buffer regrowth (tools/engine_soak.py --regrow: 150 s with 1 MiB pieces, then
# 150 s with the default 1 GiB pieces) run at the same time on one GPU. Both check every answer.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r04}
timeout -k 10 420 python -u tools/device_soak.py --seconds 300 > gpurun_out/${T}_device_soak.json 2> gpurun_out/${T}_device_soak.err &
DEV=$!
OXH_BIG_PIECE_MIB=1 timeout -k 10 240 python -u tools/engine_soak.py --seconds 150 --regrow > gpurun_out/${T}_engine_soak_regrow_1mib.json 2> gpurun_out/${T}_engine_soak_regrow_1mib.err
E1=$?
if [ $E1 -eq 0 ]; then
  timeout -k 10 240 python -u tools/engine_soak.py --seconds 150 --regrow --seed 8 > gpurun_out/${T}_engine_soak_regrow_1gib.json 2> gpurun_out/${T}_engine_soak_regrow_1gib.err
  E2=$?
else
  E2=99
fi
wait $DEV
D=$?
echo "device_soak rc=$D engine_soak(1 MiB) rc=$E1 engine_soak(1 GiB) rc=$E2"
for f in gpurun_out/${T}_device_soak.json gpurun_out/${T}_engine_soak_regrow_1mib.json gpurun_out/${T}_engine_soak_regrow_1gib.json; do tail -n 2 "$f"; done
[ $D -eq 0 ] && [ $E1 -eq 0 ] && [ $E2 -eq 0 ]
