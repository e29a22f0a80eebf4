#!/bin/bash
# Config 4: generator grid cap x ring size (chunk = ring / 2).
set -o pipefail
OUT=gpurun_out/c4_ring
mkdir -p $OUT
for r in 500 1000 2000; do for w in 6144 8192 12288; do
  PGH_SYNTH_WGS=$w timeout -k 10 200 python -u bench.py --workload c4-stream --ring $r --steps 4 --warmup 1 --no-cpu-baseline \
      > $OUT/r${r}_w$w.json 2>>$OUT/err.log || exit 1
  python3 -c "import json; d=json.load(open('$OUT/r${r}_w$w.json')); print($r, $w, d['value'], d['ms_per_step'], d['fold_kernel_client_diff_GBps_aggregated'])"
done; done
