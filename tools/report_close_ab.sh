#!/bin/bash
# Report-time close A/Bs (round 3: speculative folds, page-locked ingest, the close's output pages).
#   bash tools/report_close_ab.sh <outdir> bench [steps]  bench.py --workload resnet18-report: speculative
#                                                         (lazy) / eager / certain-only, back to back and
#                                                         5 ms apart, back to back with the close 20 ms
#                                                         later; --sync-before-close splits the queued
#                                                         GPU work from the close call
#   bash tools/report_close_ab.sh <outdir> node           tools/node_sim.py: speculative / certain-only, the
#                                                         close at once / 50 ms after the last report
#   bash tools/report_close_ab.sh <outdir> phases         node_sim --phases: engine calls inside the close
#   bash tools/report_close_ab.sh <outdir> trace          rocprofv3 kernel trace of the paced report bench
#   bash tools/report_close_ab.sh <outdir> trace_burst    kernel + memory-copy trace, close after a burst
#   bash tools/report_close_ab.sh <outdir> tests          the speculation / page-locked ingest GPU tests
# Every step under its own time limit; stops at the first failure.
set -o pipefail
out=${1:?outdir}; mode=${2:-bench}; steps=${3:-8}; mkdir -p "$out"
node_line() {
  python - "$1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().splitlines()[-1])
cc = sorted(p["close_call"] for p in d["close_phases_ms"])
print(sys.argv[1].rsplit("/", 1)[-1], "close_call median", cc[len(cc) // 2], cc, "folded before",
      [p["folded_before_close"] for p in d["close_phases_ms"]], "handler p50", d["report_handler_ms"]["p50"])
PY
}
case $mode in
tests)
  timeout -k 10 600 python -u -m pytest tests/test_gpu_incremental.py tests/test_gpu_group.py tests/test_gpu_report_semantics.py \
      tests/test_gpu_pinned_report.py tests/test_gpu_speculative_close.py -x -q --timeout 300 --timeout-method thread > "$out/pytest_new.log" 2>&1
  rc=$?; tail -3 "$out/pytest_new.log"; exit $rc ;;
bench)
  # speculative folds are opt-in since round 4 (--speculate); certain-only is the default
  for arm in "spec:--speculate" "eager:--speculate --eager-speculate" "nospec:" "spec5:--speculate --report-gap-ms 5" \
      "nospec5:--report-gap-ms 5" "spec_end20:--speculate --close-gap-ms 20" "nospec_end20:--close-gap-ms 20"; do
    name=${arm%%:*}; flags=${arm#*:}
    timeout -k 10 200 python -u bench.py --workload resnet18-report --steps "$steps" --warmup 2 --no-cpu-baseline \
        --sync-before-close $flags > "$out/report_$name.json" 2> "$out/report_$name.err" || exit 1
    python -c "import json; d=json.loads(open('$out/report_$name.json').read().splitlines()[-1]); print('$name', d['close_ms_after_last_report'], d['close_ms_after_last_report_all'], d['pending_gpu_ms_at_close'], d.get('rewinds_per_cycle'), d['value'])"
  done ;;
node)
  # round 3's node_sim flags; since round 4 tools/node_sim.py takes --arms=paced_default,... instead
  for arm in "spec0:--close-gap-ms=0" "nospec0:--no-speculate --close-gap-ms=0" "spec50:" "nospec50:--no-speculate"; do
    name=${arm%%:*}; flags=${arm#*:}
    timeout -k 10 300 python -u tools/node_sim.py 8 $flags > "$out/node_$name.json" 2> "$out/node_$name.err" || { tail -5 "$out/node_$name.err"; exit 1; }
    node_line "$out/node_$name.json"
  done ;;
phases)
  for arm in "spec50:--phases" "nospec50:--no-speculate --phases"; do
    name=${arm%%:*}; flags=${arm#*:}
    timeout -k 10 300 python -u tools/node_sim.py 6 $flags > "$out/node_$name.json" 2> "$out/node_$name.err" || { tail -5 "$out/node_$name.err"; exit 1; }
    node_line "$out/node_$name.json"
  done ;;
trace)
  export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/trace" -o run --output-format csv -- python3 bench.py \
      --workload resnet18-report --steps 3 --warmup 1 --no-cpu-baseline --report-gap-ms 5 > "$out/trace.log" 2>&1 || { tail -5 "$out/trace.log"; exit 1; } ;;
trace_burst)
  # the close right after a back-to-back burst: its fold, the FINAL ranges and the D2H behind them
  export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$out/trace_burst" -o run --output-format csv \
      -- python3 bench.py --workload resnet18-report --steps 3 --warmup 1 --no-cpu-baseline --no-speculate \
      > "$out/trace_burst.log" 2>&1 || { tail -5 "$out/trace_burst.log"; exit 1; } ;;
*) echo "unknown mode $mode"; exit 2 ;;
esac
