#!/bin/bash
# PMC passes over K1 on packed FastCDC-like items (tools/k1_small_probe.py, case cdc_packed and
# cdc_256) for the variants given in VARIANTS; one counter group per run, each under its own limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/k1pmc
mkdir -p $OUT
V=${VARIANTS:-104 264 776}
export PROBE_CASES=${PROBE_CASES:-cdc_packed,cdc_256} PROBE_WG=2
run() {  # name, counters...
  local name=$1
  shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-trace -d $OUT/$name -o run --output-format csv -- python3 tools/k1_small_probe.py $V > $OUT/$name.txt 2>&1
}
run p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE && \
run p2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_WAVES SQ_INSTS_VMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE && \
run p3 TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE
rc=$?
tail -2 $OUT/p1.txt | cut -c1-300
exit $rc
