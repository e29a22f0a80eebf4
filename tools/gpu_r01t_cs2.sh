#!/bin/bash
set -o pipefail
OUT=gpurun_out/r01t_cs2
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "secagg or rccl or stats" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -u bench.py --workload secagg-clients --steps 10 --warmup 2 > $OUT/n1.json 2> $OUT/n1.err || { tail $OUT/n1.err; exit 1; }
cat $OUT/n1.json
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/n1_default.json 2> $OUT/n1_default.err || { tail $OUT/n1_default.err; exit 1; }
cat $OUT/n1_default.json
PGH_BENCH_DEVICE=0 PGH_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29514 bench.py --gpus 2 --steps 4 --warmup 1 > $OUT/n2.json 2> $OUT/n2.err
rc=$?; echo "n2 rc=$rc"; cat $OUT/n2.json
