#!/bin/bash
# default bench (kernel line + e2e close), group bench at 1 GPU (RCCL) and a 2-child
# group rehearsal on GPU 0, the spawned 2-rank bench rehearsal (gloo on GPU 0).
set -o pipefail
mkdir -p gpurun_out/${1:-multi}
O=gpurun_out/${1:-multi}
run() { local name=$1; shift; echo "== $name"; timeout -k 10 400 "$@" > $O/$name.log 2>&1; local rc=$?; tail -1 $O/$name.log | cut -c1-2000; return $rc; }
run default python -u bench.py --no-cpu-baseline || exit 1
run group1 python -u bench.py --group --gpus 1 --no-cpu-baseline --steps 10 || exit 1
PGH_BENCH_DEVICES=0,0 run group2_dev0 python -u bench.py --group --gpus 2 --no-cpu-baseline --steps 10 --no-e2e || exit 1
PGH_BENCH_DEVICES=0 run group1_secagg_clients python -u bench.py --group --gpus 1 --workload secagg-clients --steps 5 || exit 1
PGH_DIST_BACKEND=gloo PGH_BENCH_DEVICE=0 run spawn2 python -u bench.py --gpus 2 --no-cpu-baseline --steps 5 --clients 500 || exit 1
