#!/bin/bash
# Kernel GB/s vs parameter count at fixed diff bytes (occupancy limits of the param-parallel fold).
set -o pipefail
OUT=gpurun_out/small_p
mkdir -p $OUT
for cfg in "311650 10000" "1000000 3000" "100000 30000" "3000000 1000"; do
  set -- $cfg
  timeout -k 10 200 python tools/ab_variants.py --workload fedavg --params $1 --clients $2 --rounds 3 --variants 0,6,10,1 > $OUT/fedavg_p$1.json 2>>$OUT/err.log || exit 1
done
timeout -k 10 200 python tools/ab_variants.py --workload secagg --params 311650 --clients 2500 --rounds 3 --variants 0,6,10,1 > $OUT/secagg_p311650.json 2>>$OUT/err.log || exit 1
cat $OUT/*.json
