#!/bin/bash
# K1/K2 (auto variant) across shard sizes and client counts on the final kernels: does the roofline
# fraction hold away from ResNet-18 x 1,000?  One process per point (each reserves its own slab).
set -o pipefail
OUT=gpurun_out/${1:-r02an}
mkdir -p $OUT
for wl in fedavg iterative; do
  for pn in 311650:3000 1461248:1000 4000000:1000 11689512:1000 12500000:1000 25000000:400 125000000:64; do
    P=${pn%%:*}; N=${pn##*:}
    timeout -k 10 200 python3 tools/ab_variants.py --workload $wl --params $P --clients $N --variants -1 --rounds 4 \
      > $OUT/${wl}_${P}_${N}.json 2> $OUT/${wl}_${P}_${N}.err || { tail -3 $OUT/${wl}_${P}_${N}.err; exit 1; }
    echo "$wl P=$P N=$N $(tail -1 $OUT/${wl}_${P}_${N}.json | cut -c1-200)"
  done
done
