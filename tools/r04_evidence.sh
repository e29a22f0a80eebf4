#!/bin/bash
# Round-4 evidence pass on one MI355X (one gpurun call): the -m gpu suite, smoke, the default bench
# line, the installed SQL node end to end (tools/node_sim.py), the host ceilings of the close-time
# ingest (tools/host_budget.cpp), and the report-path kernels under rocprofv3 (trace + two PMC passes).
#   bash tools/r04_evidence.sh <tag> [skip-tests]
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04}
mkdir -p $OUT
if [ "$2" != skip-tests ]; then
  bash tools/gpu_check.sh || exit 1
  cp gpurun_out/pytest_gpu.log gpurun_out/smoke.log gpurun_out/bench.log $OUT/
fi
timeout -k 10 420 python -u tools/node_sim.py 3 > $OUT/node_sim.json 2> $OUT/node_sim.err || { tail -5 $OUT/node_sim.err; exit 1; }
echo "node_sim ok"
timeout -k 10 300 tools/_host_budget 4 > $OUT/host_budget.json 2> $OUT/host_budget.err || { tail -5 $OUT/host_budget.err; exit 1; }
echo "host_budget ok"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/rp/trace -o run --output-format csv -- python3 tools/prof_report_path.py run 2 40 > $OUT/rp_trace.log 2>&1 || { tail -5 $OUT/rp_trace.log; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $c -d $OUT/rp/pmc_$c -o run --output-format csv -- python3 tools/prof_report_path.py run 1 40 > $OUT/rp_$c.log 2>&1 || { tail -5 $OUT/rp_$c.log; exit 1; }
done
echo "report-path profile ok"
if [ "$3" = trace ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-config-lines > $OUT/bench_trace_default.json 2> $OUT/bench_trace_default.err || { tail -5 $OUT/bench_trace_default.err; exit 1; }
  echo "default bench trace ok"
fi
