#!/bin/bash
# A/B of the report-time close (tools/close_phases.py) with one knob flipped by environment:
# A = ${A_ENV}, B = ${B_ENV} (default: ranged report ingest off / on), 3 alternating rounds, after
# the GPU tests named in ${TESTS} (default: the ranged-ingest and report-time ones); output into
# gpurun_out/${TAG:-ab}/.  Each step time-limited; the first failure ends the script.
set -o pipefail
O=gpurun_out/${TAG:-ab}
mkdir -p $O
A_ENV=${A_ENV:-PGH_INGEST_RANGES=0}
B_ENV=${B_ENV:-PGH_INGEST_RANGES=1}
TESTS=${TESTS:-tests/test_gpu_ranged_ingest.py tests/test_gpu_pipelined_close.py tests/test_gpu_incremental.py tests/test_gpu_pinned_report.py}
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for r in 1 2 3; do
  env $A_ENV timeout -k 10 120 python3 -u tools/close_phases.py 8 > $O/A_$r.jsonl 2>> $O/err.log || exit 1
  env $B_ENV timeout -k 10 120 python3 -u tools/close_phases.py 8 > $O/B_$r.jsonl 2>> $O/err.log || exit 1
  echo "round $r A $(tail -1 $O/A_$r.jsonl | cut -c1-220)"
  echo "round $r B $(tail -1 $O/B_$r.jsonl | cut -c1-220)"
done
