#!/bin/bash
# One GPU pass for a round's evidence directory: the -m gpu suite, smoke, node_sim arms
# (pageable / pinned report decode, with and without pygrid_amd.tune_process()), each step
# time-limited; stops at the first failure.  Usage: bash tools/round_check.sh <outdir> [--no-tests]
set -o pipefail
out=${1:?outdir}; shift
mkdir -p "$out"
if [ "$1" != "--no-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
      > "$out/pytest_gpu.log" 2>&1 || { tail -30 "$out/pytest_gpu.log"; exit 1; }
  tail -2 "$out/pytest_gpu.log"
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 \
      || { cat "$out/smoke.log"; exit 1; }
fi
for arm in "" "--pinned" "--tune" "--pinned --tune"; do
  name=node_sim$(echo "$arm" | tr -d ' -' | sed 's/^/_/;s/^_$//')
  timeout -k 10 300 python -u tools/node_sim.py 4 $arm > "$out/$name.json" 2> "$out/$name.err" \
      || { tail -20 "$out/$name.err"; exit 1; }
  python - "$out/$name.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().splitlines()[-1])
print(sys.argv[1].rsplit("/", 1)[-1], "handler p50", d["report_handler_ms"]["p50"], "ingest p50", d["report_ingest_ms"]["p50"],
      "staged/report", d["host_staging_bytes_per_report"]["mean"], "closes", d["close_ms"])
PY
done
