#!/bin/bash
# A/B of the FastCDC chunk pass's K1 workgroup width on C5 at 8 KiB chunks (GPU box): the FastCDC GPU
# tests, then tools/bench_fastcdc.py alternating the library's choice (2 chunks per workgroup below a
# 16 KiB mean) with OXH_K1_WG_WAVES=4, twice each; outputs gpurun_out/cdc_ab_{dflt,4}_{1,2}.json.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fastcdc.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/fastcdc_tests.log 2>&1 || { tail -20 gpurun_out/fastcdc_tests.log; exit 1; }
tail -2 gpurun_out/fastcdc_tests.log
for r in 1 2; do
  for w in dflt 4; do
    if [ $w = dflt ]; then E=""; else E="OXH_K1_WG_WAVES=4"; fi
    env $E timeout -k 10 300 python tools/bench_fastcdc.py --chunk 8192 --reps 5 --check-mib 16 > gpurun_out/cdc_ab_${w}_$r.json 2> gpurun_out/cdc_ab_${w}_$r.err || { tail -5 gpurun_out/cdc_ab_${w}_$r.err; exit 1; }
    echo "$w $r $(cat gpurun_out/cdc_ab_${w}_$r.json | head -c 400)"
  done
done
