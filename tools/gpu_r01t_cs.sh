#!/bin/bash
# Client-sharded secagg: GPU tests, N=1 bench line, 2-rank rehearsal on one GPU over gloo.
set -o pipefail
OUT=gpurun_out/r01t_cs
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "secagg or rccl" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -u bench.py --workload secagg-clients --steps 10 --warmup 2 > $OUT/n1.json 2> $OUT/n1.err || { tail $OUT/n1.err; exit 1; }
cat $OUT/n1.json
timeout -k 10 300 python -u bench.py --workload resnet18-secagg --steps 10 --warmup 2 --no-cpu-baseline > $OUT/n1_param.json 2> $OUT/n1_param.err || { tail $OUT/n1_param.err; exit 1; }
cat $OUT/n1_param.json
PGH_BENCH_DEVICE=0 PGH_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 2 --warmup 1 --workload secagg-clients --clients 200 > $OUT/n2.json 2> $OUT/n2.err
rc=$?; echo "n2 rc=$rc"; tail -5 $OUT/n2.err; cat $OUT/n2.json
