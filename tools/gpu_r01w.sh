#!/bin/bash
# Pipelined fold variants 21/22: parity on every fixture/mode, then interleaved A/B against v0/v6.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r01w
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "variant and (21 or 22)" > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
tail -2 $OUT/parity.log
for w in fedavg iterative weighted; do
  timeout -k 10 300 python tools/ab_variants.py --workload $w --variants 0,6,21,22 --rounds 8 > $OUT/ab_resnet_$w.json 2>&1 || exit $?
  cat $OUT/ab_resnet_$w.json
done
timeout -k 10 300 python tools/ab_variants.py --workload fedavg --params 1000000 --clients 3000 --variants 0,6,21,22 --rounds 8 > $OUT/ab_1m_fedavg.json 2>&1 || exit $?
cat $OUT/ab_1m_fedavg.json
timeout -k 10 300 python tools/ab_variants.py --workload fedavg --params 12500000 --clients 1000 --variants 0,21,22 --rounds 6 > $OUT/ab_c4shard_fedavg.json 2>&1 || exit $?
cat $OUT/ab_c4shard_fedavg.json
echo done
