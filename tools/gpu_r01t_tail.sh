#!/bin/bash
set -o pipefail
OUT=gpurun_out/r01t_tail
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "rccl or range or shards" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
PGH_BENCH_DEVICE=0 PGH_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29515 bench.py --gpus 2 --steps 3 --warmup 1 > $OUT/n2.json 2> $OUT/n2.err || { tail $OUT/n2.err; exit 1; }
cat $OUT/n2.json
PGH_BENCH_DEVICE=0 PGH_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29516 bench.py --gpus 2 --steps 2 --warmup 1 --workload secagg-clients --clients 100 > $OUT/n2_cs.json 2> $OUT/n2_cs.err || { tail $OUT/n2_cs.err; exit 1; }
cat $OUT/n2_cs.json
