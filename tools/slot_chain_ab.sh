#!/bin/bash
# Same-box A/B of the engine's large-item forms on mid-size files from the page cache through
# oxh_hash_files (tools/big_file_probe.py): "old" = every item on one K1 wave and one pread per file
# (OXH_SLOT_CHAINS=0 OXH_SPLIT_READS=0, the r01-r06 form), "chain" = K1L for a batch's items of 1 MiB and
# more (staging.hip submit_slot), "split" = that plus 4 MiB parts read by several readers for files of
# 8 MiB and more (engine.hip run_part). Alternated twice; every step time-limited; stops at the first
# failure. Output: gpurun_out/slot_ab/*.json
set -e
mkdir -p gpurun_out/slot_ab
run() {  # form files gib dir tag
  local form=$1; shift
  case $form in
    old) env="OXH_SLOT_CHAINS=0 OXH_SPLIT_READS=0" ;;
    chain) env="OXH_SLOT_CHAINS=1 OXH_SPLIT_READS=0" ;;
    split) env="OXH_SLOT_CHAINS=1 OXH_SPLIT_READS=1" ;;
  esac
  env $env timeout -k 10 200 python tools/big_file_probe.py --files $1 --gib $2 --reps 3 --dir $3 \
    > gpurun_out/slot_ab/$4_${form}_r${rep}.json
}
for rep in 1 2; do
  for form in old chain split; do
    run $form 16 0.1953125 /tmp/oxh_mid200 mid200
    run $form 64 0.0234375 /tmp/oxh_mid24 mid24
    run $form 256 0.00390625 /tmp/oxh_mid4 mid4
  done
done
