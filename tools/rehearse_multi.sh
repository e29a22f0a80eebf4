#!/bin/bash
# Multi-GPU rehearsal on one GPU, into gpurun_out/${1:-multi}/.  Steps (STEPS="..." picks some; default all):
#   group1 group2_dev0 group1_secagg_clients   the one-process group at 1 GPU (RCCL), a 2-child group on
#                                              GPU 0, the client-sharded secagg group
#   torchrun2 torchrun4 torchrun8              the driver's launch (torch.distributed.run, N ranks on GPU 0
#                                              over gloo) with every child line -- configs 1, 3, 4, 5, the
#                                              N-child group, the live PMC passes and the CPU baseline --
#                                              under the run's 540 s deadline
#   spawn8                                     the same N = 8 run started as plain `bench.py --gpus 8` (the
#                                              parent forms the 8 ranks itself)
# Clients are cut so N ranks fit one GPU's 288 GB (the headline's 300 clients x 46.8 MB = 14 GB per
# rank; --config-clients for configs 3-5; config 4's ring follows its client count).  Each step is
# time-limited; the first failure ends the script.
set -o pipefail
O=gpurun_out/${1:-multi}
STEPS=${STEPS:-"group1 group2_dev0 group1_secagg_clients torchrun2 torchrun4 torchrun8 spawn8"}
mkdir -p "$O"
want() { [[ " $STEPS " == *" $1 "* ]]; }
run() { local name=$1; shift; echo "== $name"; timeout -k 10 600 "$@" > "$O/$name.log" 2>&1; local rc=$?; tail -1 "$O/$name.log" | cut -c1-3000; return $rc; }
devs() { local d=0; for ((i = 1; i < $1; i++)); do d="$d,0"; done; echo "$d"; }
ranks() {  # ranks() N port config_clients: the driver's torchrun launch with N ranks on GPU 0
    PGH_DIST_BACKEND=gloo PGH_BENCH_DEVICE=0 PGH_BENCH_DEVICES=$(devs "$1") run "torchrun$1" python -u -m torch.distributed.run \
        --nnodes=1 --nproc-per-node "$1" --master-addr 127.0.0.1 --master-port "$2" bench.py --gpus "$1" --steps 5 \
        --warmup 2 --clients 300 --config-clients "$3"
}
if want group1; then run group1 python -u bench.py --group --gpus 1 --no-cpu-baseline --steps 10 --no-e2e || exit 1; fi
if want group2_dev0; then
    PGH_BENCH_DEVICES=0,0 run group2_dev0 python -u bench.py --group --gpus 2 --no-cpu-baseline --steps 10 --no-e2e || exit 1
fi
if want group1_secagg_clients; then
    PGH_BENCH_DEVICES=0 run group1_secagg_clients python -u bench.py --group --gpus 1 --workload secagg-clients --steps 5 || exit 1
fi
if want torchrun2; then ranks 2 29541 100 || exit 1; fi
if want torchrun4; then ranks 4 29543 100 || exit 1; fi
if want torchrun8; then ranks 8 29545 64 || exit 1; fi
if want spawn8; then
    PGH_DIST_BACKEND=gloo PGH_BENCH_DEVICE=0 PGH_BENCH_DEVICES=$(devs 8) run spawn8 python -u bench.py --gpus 8 --steps 5 \
        --warmup 2 --clients 300 --config-clients 64 || exit 1
fi
