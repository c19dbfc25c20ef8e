#!/bin/bash
# r04s: K1R ring depth (264: 2 iterations in flight, 260: 3, 256: 4) and waves per workgroup (1 / 2 / 4)
# in the C5 8 KiB pipeline, alternating, medians of 7.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r04s}
run() {  # name, env...
  local name=$1
  shift
  timeout -k 10 300 env "$@" python tools/bench_fastcdc.py --chunk 8192 --reps 7 > gpurun_out/${T}_$name.json 2> gpurun_out/${T}_$name.err || { tail -5 gpurun_out/${T}_$name.err; exit 1; }
  echo "$name $(grep -o '"s_median": [0-9.]*' gpurun_out/${T}_$name.json)"
}
for r in 1 2; do
  run v264_r$r OXH_K1_PACKED_VARIANT=264
  run v260_r$r OXH_K1_PACKED_VARIANT=260
  run v256_r$r OXH_K1_PACKED_VARIANT=256
  run v264_wg1_r$r OXH_K1_PACKED_VARIANT=264 OXH_K1_WG_WAVES=1
  run v264_wg4_r$r OXH_K1_PACKED_VARIANT=264 OXH_K1_WG_WAVES=4
done
