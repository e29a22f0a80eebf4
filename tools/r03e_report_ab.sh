#!/bin/bash
# Report-time close A/B (speculative folds on/off; back to back and paced 5 ms) with the close's
# pending GPU work timed apart.  Usage: bash tools/r03e_report_ab.sh <outdir> [steps]
set -o pipefail
out=${1:-gpurun_out/r03e}; steps=${2:-8}; mkdir -p $out
for arm in "spec:" "eager:--eager-speculate" "nospec:--no-speculate" "spec5:--report-gap-ms 5" "nospec5:--no-speculate --report-gap-ms 5"; do
  name=${arm%%:*}; flags=${arm#*:}
  timeout -k 10 200 python -u bench.py --workload resnet18-report --steps $steps --warmup 2 --no-cpu-baseline --sync-before-close $flags \
      > $out/report_$name.json 2> $out/report_$name.err || exit 1
  python -c "import json,sys; d=json.loads(open('$out/report_$name.json').read().splitlines()[-1]); print('$name', d['close_ms_after_last_report'], d['close_ms_after_last_report_all'], d['pending_gpu_ms_at_close'], d.get('rewinds_per_cycle'), d['value'])"
done
