#!/bin/bash
# Same-box A/B of the small-request submit (staging.hip submit_packed: the descriptors after the bytes,
# one H2D on the compute stream; OXH_DIRECT_PACKED=0 = submit_slot's three H2D on the copy stream):
# per-call latency (tools/latency_probe.py), alternated twice. Every step time-limited; stops at the
# first failure. Output: gpurun_out/packed_ab/*.json
set -e
mkdir -p gpurun_out/packed_ab
for rep in 1 2; do
  for on in 0 1; do
    OXH_DIRECT_PACKED=$on timeout -k 10 150 python tools/latency_probe.py --calls 400 > gpurun_out/packed_ab/lat_on${on}_r${rep}.json
  done
done
