#!/bin/bash
# Config 4 ring: cap the on-device generator's grid so the fold of chunk k can be co-resident
# with the generation of chunk k+1 (PGH_SYNTH_WGS; 0 = one grid row per client row).
set -o pipefail
OUT=gpurun_out/c4_synth
mkdir -p $OUT
for w in ${WGS:-0 4096 8192 16384 32768}; do
  PGH_SYNTH_WGS=$w timeout -k 10 200 python -u bench.py --workload c4-stream --steps 4 --warmup 1 --no-cpu-baseline \
      > $OUT/wgs_$w.json 2>>$OUT/err.log || exit 1
  python3 -c "import json; d=json.load(open('$OUT/wgs_$w.json')); print($w, d['value'], d['ms_per_step'], d['fold_kernel_client_diff_GBps_aggregated'])"
done
