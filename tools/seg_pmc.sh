#!/bin/bash
# PMC passes over the F1 redesign probe (tools/cdc_segment_probe.hip); one counter group per run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/segpmc
V=${V:-dma_w8_slots1}
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/segpmc/p1 -o run --output-format csv -- ./tools/cdc_segment_probe 4 $V > gpurun_out/segpmc/p1.txt 2>&1 && \
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/segpmc/p2 -o run --output-format csv -- ./tools/cdc_segment_probe 4 $V > gpurun_out/segpmc/p2.txt 2>&1
rc=$?
cat gpurun_out/segpmc/p1.txt | grep variant
exit $rc
