#!/bin/bash
# r04e: K1R (a 16-lane row per chunk, four chunks per wave) -- parity of every K1R variant, the small-
# item probe K1 (104) vs K1R (264 / 260), and C5 8 KiB with FastCDC's K1 pass on each (checked), plus
# the kernel split under rocprofv3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r04m}
step() {  # name, limit, command...
  local name=$1 lim=$2
  shift 2
  echo "== $name"
  timeout -k 10 "$lim" "$@" > "gpurun_out/${T}_$name.out" 2> "gpurun_out/${T}_$name.err" || {
    echo "$name failed"; tail -30 "gpurun_out/${T}_$name.err"; tail -30 "gpurun_out/${T}_$name.out"; exit 1; }
  tail -c 900 "gpurun_out/${T}_$name.out"; echo
}
step k1r_parity 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -k "k1r or every_length or chunk_digests or ragged"
step probe 600 env PROBE_CASES=cdc_packed,cdc_256,cdc64_packed,fixed_8k,fixed_64k PROBE_WG=2,4 python tools/k1_small_probe.py 104 264 776 772 768
step c5_8k_776 400 env OXH_K1_PACKED_VARIANT=776 python tools/bench_fastcdc.py --chunk 8192 --reps 7 --check-all
step c5_8k_264 400 env OXH_K1_PACKED_VARIANT=264 python tools/bench_fastcdc.py --chunk 8192 --reps 7
step c5_8k_772 400 env OXH_K1_PACKED_VARIANT=772 python tools/bench_fastcdc.py --chunk 8192 --reps 7
step c5_64k_776 400 env OXH_K1_PACKED_VARIANT=776 python tools/bench_fastcdc.py --chunk 65536 --reps 5
export OXH_K1_PACKED_VARIANT=776
step c5_8k_prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}_c5 -o run --output-format csv -- python tools/bench_fastcdc.py --chunk 8192 --reps 3
cp "$(find gpurun_out/prof_${T}_c5 -name '*kernel_stats.csv' | head -1)" gpurun_out/${T}_c5_8k_kernel_stats.csv
