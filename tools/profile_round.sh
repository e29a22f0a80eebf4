#!/bin/bash
# Evidence pass on one MI355X, in two parts (each fits one gpurun call):
#   bash tools/profile_round.sh <tag> tests   -m gpu suite, smoke, every bench workload (per-rank and
#                                             one-process group at 1 GPU, 2-child group on GPU 0)
#   bash tools/profile_round.sh <tag> prof    rocprofv3 --kernel-trace --stats of the driver's default
#                                             command and of the iterative / secagg / report lines, and
#                                             the HBM PMC passes (FETCH_SIZE, WRITE_SIZE: separate runs)
# Output: gpurun_out/<tag>/ (copy to profiles/<tag>/; python tools/pmc_summarize.py gpurun_out/<tag>
# profiles/<tag> refreshes profiles/pmc_traffic.json).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-round}
PART=${2:-tests}
mkdir -p $OUT
b() { local name=$1 t=$2; shift 2; timeout -k 10 $t python -u bench.py "$@" > $OUT/bench_$name.json 2> $OUT/bench_$name.err || { echo "bench $name failed"; tail -5 $OUT/bench_$name.err; exit 1; }; echo "bench $name ok"; }
if [ "$PART" = tests ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
  b resnet18-fedavg 300 --steps 20 --warmup 5
  for w in resnet18-iterative resnet18-weighted resnet18-secagg mnist-state secagg-clients; do b $w 200 --workload $w --steps 10 --warmup 2; done
  b resnet18-state 300 --workload resnet18-state --steps 3 --warmup 1
  b resnet18-report 300 --workload resnet18-report --steps 5 --warmup 2
  b resnet18-secagg-state 400 --workload resnet18-secagg-state --steps 3 --warmup 1
  b c4-stream 300 --workload c4-stream --steps 4 --warmup 1
  b c5-ingest 300 --workload c5-ingest --steps 3 --warmup 1
  b group1-fedavg 300 --group --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline
  b group1-secagg-clients 300 --group --gpus 1 --workload secagg-clients --steps 5 --warmup 2 --no-cpu-baseline
  PGH_BENCH_DEVICES=0,0 b group2dev0-fedavg 300 --group --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e
  timeout -k 10 200 python tools/bench_b64.py > $OUT/b64.log 2>&1 || exit $?
else
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_trace_default.json 2> $OUT/bench_trace_default.err || exit $?
  for w in resnet18-iterative resnet18-secagg resnet18-report; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_$w -o run --output-format csv -- python3 bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_trace_$w.json 2> $OUT/bench_trace_$w.err || exit $?
  done
  for w in resnet18-fedavg resnet18-iterative resnet18-weighted resnet18-secagg resnet18-report; do
    for c in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 200 rocprofv3 --pmc $c -d $OUT/pmc_${w}_$c -o run --output-format csv -- python3 bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-live-traffic > $OUT/pmc_${w}_$c.log 2>&1 || exit $?
    done
  done
fi
echo done
