#!/bin/bash
# Rehearse bench.py's N > 1 path with 2 ranks on ONE GPU over gloo (RCCL needs one GPU per rank).
set -o pipefail
OUT=gpurun_out/rehearse
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "range or shards" > $OUT/gpu_tests.log 2>&1 || { tail -20 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
PGH_BENCH_DEVICE=0 PGH_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 4 --warmup 1 > $OUT/n2.json 2> $OUT/n2.err
rc=$?; echo "n2 rc=$rc"; tail -5 $OUT/n2.err; cat $OUT/n2.json
PGH_BENCH_DEVICE=0 PGH_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 2 --warmup 1 --workload resnet18-secagg --clients 200 > $OUT/n2_secagg.json 2> $OUT/n2_secagg.err
rc=$?; echo "n2 secagg rc=$rc"; tail -3 $OUT/n2_secagg.err; cat $OUT/n2_secagg.json
