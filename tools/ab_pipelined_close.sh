#!/bin/bash
# Pipelined close (PGH_FINAL_RANGES, default 4) vs one FINAL launch: GPU tests, then the report-time
# close and the MNIST / ResNet-18 bytes->bytes closes, interleaved.   usage: bash tools/ab_pipelined_close.sh <tag>
set -o pipefail
O=gpurun_out/${1:-piped}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipelined_close.py tests/test_gpu_incremental.py tests/test_gpu_parity.py tests/test_gpu_group.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc = 0 ] || exit 1
for r in 1 2; do
  for k in 1 4; do
    PGH_FINAL_RANGES=$k timeout -k 10 300 python -u bench.py --workload resnet18-report --steps 8 --warmup 2 --no-cpu-baseline > $O/report_r${k}_$r.json 2>&1 || exit 1
    PGH_FINAL_RANGES=$k timeout -k 10 300 python -u bench.py --workload resnet18-state --steps 3 --warmup 1 --no-cpu-baseline > $O/state_r${k}_$r.json 2>&1 || exit 1
  done
done
python - "$O" <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    r = json.loads([l for l in open(f) if l.startswith("{")][-1])
    print(f.split("/")[-1], r.get("cycle_close_ms"), r.get("close_ms_after_last_report"), r.get("close_ms_after_last_report_all"))
PY
