#!/bin/bash
# Multi-GPU rehearsal on one GPU, into gpurun_out/${1:-multi}/: the group bench at 1 GPU (RCCL),
# a 2-child group on GPU 0, the client-sharded secagg group; then the driver's N = 2 launch
# (torch.distributed.run, 2 ranks on GPU 0 over gloo) with every child line -- configs 1, 3, 4, 5
# (clients cut to --config-clients so two ranks fit one GPU) and the 2-child group -- under the
# run's deadline; then the same at N = 4 (4 ranks on GPU 0).  Each step time-limited; the first
# failure ends the script.  (N = 8 is the driver's to run.)
set -o pipefail
O=gpurun_out/${1:-multi}
mkdir -p "$O"
run() { local name=$1; shift; echo "== $name"; timeout -k 10 600 "$@" > "$O/$name.log" 2>&1; local rc=$?; tail -1 "$O/$name.log" | cut -c1-3000; return $rc; }
run group1 python -u bench.py --group --gpus 1 --no-cpu-baseline --steps 10 --no-e2e || exit 1
PGH_BENCH_DEVICES=0,0 run group2_dev0 python -u bench.py --group --gpus 2 --no-cpu-baseline --steps 10 --no-e2e || exit 1
PGH_BENCH_DEVICES=0 run group1_secagg_clients python -u bench.py --group --gpus 1 --workload secagg-clients --steps 5 || exit 1
PGH_DIST_BACKEND=gloo PGH_BENCH_DEVICE=0 PGH_BENCH_DEVICES=0,0 run torchrun2 python -u -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 5 \
    --warmup 2 --clients 300 --config-clients 100 || exit 1
PGH_DIST_BACKEND=gloo PGH_BENCH_DEVICE=0 PGH_BENCH_DEVICES=0,0,0,0 run torchrun4 python -u -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29543 bench.py --gpus 4 --steps 5 \
    --warmup 2 --clients 300 --config-clients 100 || exit 1
