#!/bin/bash
# Round-3 GPU pass: the speculative-fold and page-locked-ingest tests, the report-time close with and
# without speculative folds (back to back and paced), node_sim with pageable / page-locked reports.
set -o pipefail
out=${1:-gpurun_out/r03c}; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_incremental.py tests/test_gpu_group.py tests/test_gpu_report_semantics.py \
    tests/test_gpu_pinned_report.py -x -q --timeout 300 --timeout-method thread > $out/pytest_new.log 2>&1
rc=$?; tail -3 $out/pytest_new.log; [ $rc = 0 ] || exit 1
for arm in "spec:" "nospec:--no-speculate" "spec5:--report-gap-ms 5" "nospec5:--no-speculate --report-gap-ms 5"; do
  name=${arm%%:*}; flags=${arm#*:}
  timeout -k 10 200 python -u bench.py --workload resnet18-report --steps 8 --warmup 2 --no-cpu-baseline $flags \
      > $out/report_$name.json 2> $out/report_$name.err || exit 1
  python -c "import json,sys; d=json.loads(open('$out/report_$name.json').read().splitlines()[-1]); print('$name', d['close_ms_after_last_report'], d['close_ms_after_last_report_all'], d.get('rows_folded_at_close'), d.get('rewinds_per_cycle'), d['value'])"
done
for arm in "" "--pinned"; do
  name=node_sim$(echo "$arm" | tr -d ' -' | sed 's/^/_/;s/^_$//')
  timeout -k 10 300 python -u tools/node_sim.py 4 $arm > "$out/$name.json" 2> "$out/$name.err" || { tail -20 "$out/$name.err"; exit 1; }
  python - "$out/$name.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().splitlines()[-1])
print(sys.argv[1].rsplit("/", 1)[-1], "handler p50", d["report_handler_ms"]["p50"], "ingest p50", d["report_ingest_ms"]["p50"],
      "staged/report", d["host_staging_bytes_per_report"]["mean"], "closes", d["close_ms"])
PY
done
