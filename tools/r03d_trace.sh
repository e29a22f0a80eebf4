#!/bin/bash
# Speculative report-time close under paced reports: pending GPU work at close vs the close itself,
# and a kernel trace of the same run.
set -o pipefail
out=${1:-gpurun_out/r03d}; mkdir -p $out
for arm in "spec5:--report-gap-ms 5" "nospec5:--no-speculate --report-gap-ms 5"; do
  name=${arm%%:*}; flags=${arm#*:}
  timeout -k 10 200 python -u bench.py --workload resnet18-report --steps 6 --warmup 2 --no-cpu-baseline --sync-before-close $flags \
      > $out/report_$name.json 2> $out/report_$name.err || exit 1
  python -c "import json,sys; d=json.loads(open('$out/report_$name.json').read().splitlines()[-1]); print('$name', d['close_ms_after_last_report_all'], d['pending_gpu_ms_at_close'])"
done
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run -- python3 bench.py --workload resnet18-report --steps 3 --warmup 1 --no-cpu-baseline --report-gap-ms 5 > $out/trace.log 2>&1 || { tail -5 $out/trace.log; exit 1; }
find $out/trace -name "*kernel_stats.csv" | head -3
