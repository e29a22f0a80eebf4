#!/bin/bash
# A/B of the shares-from-the-wire close (bench.py --workload resnet18-secagg-state): the library in
# tools/_variantA (a snapshot of the tree before a change) against the tree, interleaved on one lease.
#   bash tools/ab_wire.sh <tag> [rounds]
# Snapshot A first (mtimes kept, so the copy is not rebuilt):
#   mkdir -p tools/_variantA && cp -rp bench.py pygrid_amd oracle include tools/_variantA/
set -o pipefail
OUT=gpurun_out/${1:-ab_wire}
mkdir -p $OUT
ARGS="--workload resnet18-secagg-state --steps 5 --warmup 1 --no-cpu-baseline --no-live-traffic --no-group-line --no-config-lines"
for r in $(seq 1 ${2:-3}); do
  timeout -k 10 200 python3 tools/_variantA/bench.py $ARGS > $OUT/A_$r.json 2>> $OUT/err.log || exit 1
  timeout -k 10 200 python3 bench.py $ARGS > $OUT/B_$r.json 2>> $OUT/err.log || exit 1
  echo "round $r: A $(python3 -c "import json,sys; d=json.load(open('$OUT/A_$r.json')); print(d['value'], d['ms_per_step'], d.get('wire_GBps'))") B $(python3 -c "import json,sys; d=json.load(open('$OUT/B_$r.json')); print(d['value'], d['ms_per_step'], d.get('wire_GBps'))")"
done
