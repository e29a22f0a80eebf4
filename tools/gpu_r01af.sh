#!/bin/bash
# Fast on-device generator (kind 1) for config 4: parity first, then c4-stream with each generator.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r01af
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $OUT/gpu_tests.log | head; exit $rc; }
for rep in 1 2; do
  for g in fast irwin-hall; do
    timeout -k 10 300 python bench.py --workload c4-stream --steps 4 --warmup 1 --synth $g --no-cpu-baseline > $OUT/c4_${g}_r$rep.json 2> $OUT/c4_${g}_r$rep.err || exit $?
    python -c "import json;r=json.loads(open('$OUT/c4_${g}_r$rep.json').read());print('$g', r['value'], r['ms_per_step'], r['fold_kernel_client_diff_GBps_aggregated'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_c4 -o run --output-format csv -- python3 bench.py --workload c4-stream --steps 2 --warmup 1 --no-cpu-baseline > $OUT/c4_trace.json 2> $OUT/c4_trace.err || exit $?
echo done
