#!/bin/bash
# r05 GPU steps: STEPS picks them (comma list). Each step has its own time limit; a test failure is
# reported and the script goes on, a timeout / abort / signal stops it (nothing more on the GPU).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r05a}
step() {  # name, limit, command...
  local name=$1 lim=$2
  shift 2
  case ",${STEPS:-all}," in *",$name,"*|*",all,"*) ;; *) return 0;; esac
  echo "== $name $(date +%T)"
  timeout -k 10 "$lim" "$@" > "gpurun_out/${T}_$name.out" 2> "gpurun_out/${T}_$name.err"
  local rc=$?
  tail -c 1500 "gpurun_out/${T}_$name.out"; echo
  if [ $rc -ne 0 ]; then
    echo "$name rc=$rc"; tail -20 "gpurun_out/${T}_$name.err"
    if [ $rc -ge 124 ]; then exit $rc; fi
  fi
}
step box 30 bash -c 'nproc; free -g; df -h /tmp /dev/shm .; cat /sys/fs/cgroup/memory.max /sys/fs/cgroup/cpu.max 2>/dev/null; ulimit -n'
step newtests 900 python -u -m pytest tests/test_fastcdc.py tests/test_bench_launch.py tests/test_gpu_file_errors.py -m gpu -q --timeout 300 --timeout-method thread -k "files or host or lds or gather or reference_messages or status_and_errno"
step pytest 1200 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 300 --timeout-method thread
step bench 240 python bench.py --gpus 1 --steps 20 --warmup 5
step c1 300 python tools/bench_c1.py --reps 5
step bench_dist_torch 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 1 --dist --gather torch --steps 20 --warmup 5 --no-cpu-baseline
step bench_dist 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --dist --steps 20 --warmup 5 --no-cpu-baseline
step c5e2e_small 600 python tools/bench_fastcdc_e2e.py --dir /tmp/oxh_c5s --files 16 --gib 1 --chunk 8192 --reps 3 --cold
step probe 120 tools/fold_probe
step foldtests 900 python -u -m pytest tests/test_fastcdc.py -m gpu -q --timeout 300 --timeout-method thread -k "fold or files or host"
step c5_8k_fold 400 env OXH_CDC_FOLD=1 python tools/bench_fastcdc.py --chunk 8192 --reps 5 --check-all
step c5_8k_base 400 python tools/bench_fastcdc.py --chunk 8192 --reps 5
step c5_8k_fold_prof 400 env OXH_CDC_FOLD=1 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}_fold -o run --output-format csv -- python tools/bench_fastcdc.py --chunk 8192 --reps 3
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step e2e_nb4 600 env OXH_TRACE=1 OXH_CDC_NBOUNCE=4 python tools/bench_fastcdc_e2e.py --dir /tmp/oxh_c5s --files 16 --gib 1 --chunk 8192 --reps 3 --keep
step e2e_nb8 600 env OXH_TRACE=1 OXH_CDC_NBOUNCE=8 python tools/bench_fastcdc_e2e.py --dir /tmp/oxh_c5s --files 16 --gib 1 --chunk 8192 --reps 3
step e2e_shm_8k 900 env OXH_TRACE=1 OXH_CDC_NBOUNCE=${NB:-8} python tools/bench_fastcdc_e2e.py --dir /dev/shm/oxh_c5 --files 16 --gib 8 --chunk 8192 --reps 3 --keep
step e2e_shm_64k 900 env OXH_TRACE=1 OXH_CDC_NBOUNCE=${NB:-8} python tools/bench_fastcdc_e2e.py --dir /dev/shm/oxh_c5 --files 16 --gib 8 --chunk 65536 --reps 3
step e2e_disk_8k 900 env OXH_TRACE=1 OXH_CDC_NBOUNCE=${NB:-8} python tools/bench_fastcdc_e2e.py --dir /tmp/oxh_c5d --files 8 --gib 8 --chunk 8192 --reps 2 --cold
step profile_c2 900 env TAG=${T} WORKLOAD=c2 PMC=1 bash tools/gpu_profile_driver.sh
step c5_64k_prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}_c5_64k -o run --output-format csv -- python tools/bench_fastcdc.py --chunk 65536 --reps 3
step c5_8k_prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}_c5_8k -o run --output-format csv -- python tools/bench_fastcdc.py --chunk 8192 --reps 3
step e2e_cs1 600 env OXH_TRACE=1 OXH_CDC_COPY_STREAMS=1 python tools/bench_fastcdc_e2e.py --dir /tmp/oxh_c5s --files 16 --gib 1 --chunk 8192 --reps 5 --keep --cpu none
step e2e_cs2 600 env OXH_TRACE=1 OXH_CDC_COPY_STREAMS=2 python tools/bench_fastcdc_e2e.py --dir /tmp/oxh_c5s --files 16 --gib 1 --chunk 8192 --reps 5 --keep --cpu none
step e2e_cs1b 600 env OXH_TRACE=1 OXH_CDC_COPY_STREAMS=1 python tools/bench_fastcdc_e2e.py --dir /tmp/oxh_c5s --files 16 --gib 1 --chunk 8192 --reps 5 --cpu none
step c5_64k_walk 400 env OXH_CDC_WALK=1 python tools/bench_fastcdc.py --chunk 65536 --reps 3
step c5_64k_fold 400 env OXH_CDC_WALK=1 OXH_CDC_FOLD=1 python tools/with_lib.py tools/probe/liboxen_hash.so tools/bench_fastcdc.py --chunk 65536 --reps 3
step native 300 python -u -m pytest tests/test_native_mirror.py -m gpu -q --timeout 240 --timeout-method thread
step shm_cs1 900 env OXH_TRACE=1 OXH_CDC_COPY_STREAMS=1 python tools/bench_fastcdc_e2e.py --dir /dev/shm/oxh_c5 --files 16 --gib 8 --chunk 8192 --reps 3 --keep --cpu none
step shm_cs2 900 env OXH_TRACE=1 OXH_CDC_COPY_STREAMS=2 python tools/bench_fastcdc_e2e.py --dir /dev/shm/oxh_c5 --files 16 --gib 8 --chunk 8192 --reps 3 --keep --cpu none
step shm_cs1b 900 env OXH_TRACE=1 OXH_CDC_COPY_STREAMS=1 python tools/bench_fastcdc_e2e.py --dir /dev/shm/oxh_c5 --files 16 --gib 8 --chunk 8192 --reps 3 --keep --cpu none
step shm_cs2b 900 env OXH_TRACE=1 OXH_CDC_COPY_STREAMS=2 python tools/bench_fastcdc_e2e.py --dir /dev/shm/oxh_c5 --files 16 --gib 8 --chunk 8192 --reps 3 --cpu none
step largetests 600 python -u -m pytest tests/test_gpu_large_items.py tests/test_gpu_publish.py tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -k "large or big or publish or nomem or oversize or piece"
step big_w7 600 python tools/big_file_probe.py --files 2 --gib 4 --dir /tmp/oxh_big --reps 3
step big_w1 600 env OXH_BIG_WINDOWS=1 python tools/big_file_probe.py --files 2 --gib 4 --dir /tmp/oxh_big --reps 3
step big_w7b 600 python tools/big_file_probe.py --files 2 --gib 4 --dir /tmp/oxh_big --reps 3
step big_w1b 600 env OXH_BIG_WINDOWS=1 python tools/big_file_probe.py --files 2 --gib 4 --dir /tmp/oxh_big --reps 3
step concurrent 600 python -u -m pytest tests/test_fastcdc.py -m gpu -q --timeout 500 --timeout-method thread -k concurrent
step comm2 240 env NCCL_DEBUG=WARN python tools/comm_two_ranks.py --world 2
step levels 600 python -u -m pytest tests/test_fastcdc.py -m gpu -q --timeout 300 --timeout-method thread -k "levels or many_small"
step cdcsoak 400 python tools/cdc_host_soak.py --seconds 240
step fixed 600 python -u -m pytest tests/test_dedup_fixed.py tests/test_native_mirror.py -m gpu -v --timeout 300 --timeout-method thread
step fixed_e2e_small 600 env OXH_TRACE=1 python tools/bench_fastcdc_e2e.py --fixed --dir /tmp/oxh_fx --files 16 --gib 1 --chunk 65536 --reps 3
step fixed_e2e_shm 900 env OXH_TRACE=1 python tools/bench_fastcdc_e2e.py --fixed --dir /dev/shm/oxh_c5 --files 16 --gib 8 --chunk 65536 --reps 3 --keep
step multi 600 python -u -m pytest tests/test_fastcdc.py tests/test_native_mirror.py -m gpu -v --timeout 300 --timeout-method thread -k "multi or native"
step multi_e2e_2 900 env OXH_TRACE=1 python tools/bench_fastcdc_e2e.py --dir /dev/shm/oxh_c5 --files 16 --gib 8 --chunk 8192 --reps 3 --keep --cpu none --devices 0,0
step multi_e2e_1 900 env OXH_TRACE=1 python tools/bench_fastcdc_e2e.py --dir /dev/shm/oxh_c5 --files 16 --gib 8 --chunk 8192 --reps 3 --keep --cpu none
step restore 300 python -u -m pytest tests/test_restore.py -m gpu -v --timeout 200 --timeout-method thread
step fixed_e2e_shm4k 900 env OXH_TRACE=1 python tools/bench_fastcdc_e2e.py --fixed --dir /dev/shm/oxh_c5 --files 16 --gib 8 --chunk 4096 --reps 3 --keep
step fixedtests 600 python -u -m pytest tests/test_dedup_fixed.py tests/test_fastcdc.py tests/test_native_mirror.py -m gpu -q --timeout 300 --timeout-method thread -k "fixed or chunk_digests or multi or native"
FX="python tools/bench_fastcdc_e2e.py --fixed --dir /dev/shm/oxh_c5 --files 16 --gib 8 --reps 3 --keep"
step fx_imp4k 900 env OXH_TRACE=1 $FX --chunk 4096
step fx_desc4k 900 env OXH_TRACE=1 OXH_FIXED_IMPLICIT_SEGS=0 $FX --chunk 4096 --cpu none
step fx_imp4k_b 900 env OXH_TRACE=1 $FX --chunk 4096 --cpu none
step fx_desc4k_b 900 env OXH_TRACE=1 OXH_FIXED_IMPLICIT_SEGS=0 $FX --chunk 4096 --cpu none
step fx_imp64k 900 env OXH_TRACE=1 $FX --chunk 65536
step fx_desc64k 900 env OXH_TRACE=1 OXH_FIXED_IMPLICIT_SEGS=0 $FX --chunk 65536 --cpu none
E8="python tools/bench_fastcdc_e2e.py --dir /dev/shm/oxh_c5 --files 16 --gib 8 --chunk 8192 --reps 3 --keep --cpu none"
step bw64 900 env OXH_TRACE=1 $E8
step bw128 900 env OXH_TRACE=1 OXH_CDC_BOUNCE_MIB=128 $E8
step bw256 900 env OXH_TRACE=1 OXH_CDC_BOUNCE_MIB=256 OXH_CDC_NBOUNCE=6 python tools/bench_fastcdc_e2e.py --dir /dev/shm/oxh_c5 --files 16 --gib 8 --chunk 8192 --reps 3 --keep
step bw32 900 env OXH_TRACE=1 OXH_CDC_BOUNCE_MIB=32 OXH_CDC_NBOUNCE=16 $E8
step bw64b 900 env OXH_TRACE=1 $E8
step bw128b 900 env OXH_TRACE=1 OXH_CDC_BOUNCE_MIB=128 $E8
step nb8 900 env OXH_TRACE=1 OXH_CDC_NBOUNCE=8 $E8
step nb12 900 env OXH_TRACE=1 OXH_CDC_NBOUNCE=12 $E8
step nb16 900 env OXH_TRACE=1 OXH_CDC_NBOUNCE=16 $E8
step nb8b 900 env OXH_TRACE=1 OXH_CDC_NBOUNCE=8 $E8
step nb12b 900 env OXH_TRACE=1 OXH_CDC_NBOUNCE=12 $E8
step nb16b 900 env OXH_TRACE=1 OXH_CDC_NBOUNCE=16 $E8
rm -rf /dev/shm/oxh_c5 /tmp/oxh_c5s /tmp/oxh_c5d /tmp/oxh_big /tmp/oxh_fx
echo "== done $(date +%T)"
