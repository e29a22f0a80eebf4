#!/bin/bash
# A/B of PGH_D2H_PIECE_MB with the parallel pre-fault on: does the D2H of piece i + 1 beside the
# copy-out of piece i pay now that the copy-out no longer takes page faults?
set -o pipefail
OUT=gpurun_out/r01ak
mkdir -p $OUT
for r in 1 2; do
  for mb in 0 8 16; do
    PGH_D2H_PIECE_MB=$mb timeout -k 10 200 python tools/time_resnet_state.py > $OUT/phases_mb${mb}_r$r.log 2>&1 || exit $?
    PGH_D2H_PIECE_MB=$mb timeout -k 10 300 python bench.py --workload resnet18-report --steps 3 --warmup 1 --no-cpu-baseline > $OUT/report_mb${mb}_r$r.json 2> $OUT/report_mb${mb}_r$r.err || exit $?
    echo "mb=$mb r=$r: $(tail -1 $OUT/phases_mb${mb}_r$r.log)"
  done
done
echo done
