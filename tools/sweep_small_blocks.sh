#!/bin/bash
# Narrow column blocks for small shards with many clients: PGH_BLOCK_BYTES (bytes of one row per
# block) 256 / 1 KiB / 4 KiB / 16 KiB vs the default (256 KiB: small shards are one row-major
# block).  Per setting one process, kernel variants interleaved inside it.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/small_blocks
mkdir -p $OUT
for case in "iterative 50000 60000" "iterative 100000 30000" "fedavg 100000 30000" "iterative 311650 10000" "fedavg 311650 10000"; do
  set -- $case
  for bb in 262144 256 1024 4096 16384; do
    PGH_BLOCK_BYTES=$bb timeout -k 10 200 python tools/ab_variants.py --workload $1 --params $2 --clients $3 --variants=-1,11,12,14,17 --rounds 4 --reps 2 > $OUT/${1}_${2}_bb$bb.json 2> $OUT/${1}_${2}_bb$bb.err || exit $?
    python -c "import json;r=json.loads(open('$OUT/${1}_${2}_bb$bb.json').read().strip().splitlines()[-1]);print('$1 P=$2 N=$3 bb=$bb', {k:v['GBps_median'] for k,v in r['variants'].items()})"
  done
done
echo done
