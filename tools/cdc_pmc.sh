#!/bin/bash
# PMC passes over the FastCDC pipeline (tools/bench_fastcdc.py); one counter group per run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/cdcpmc
mkdir -p $OUT
ARGS=${ARGS:---chunk 8192 --reps 1 --files 4}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE --kernel-trace -d $OUT/p1 -o run --output-format csv -- python3 tools/bench_fastcdc.py $ARGS > $OUT/p1.txt 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_WAVES SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace -d $OUT/p2 -o run --output-format csv -- python3 tools/bench_fastcdc.py $ARGS > $OUT/p2.txt 2>&1
rc=$?
tail -1 $OUT/p1.txt
exit $rc
