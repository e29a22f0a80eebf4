#!/bin/bash
# node_sim: speculative vs certain-only folds, close at once vs 50 ms after the last report.
set -o pipefail
out=${1:-gpurun_out/r03j}; mkdir -p $out
for arm in "spec0:--close-gap-ms=0" "nospec0:--no-speculate --close-gap-ms=0" "spec50:" "nospec50:--no-speculate"; do
  name=${arm%%:*}; flags=${arm#*:}
  timeout -k 10 300 python -u tools/node_sim.py 8 $flags > $out/node_$name.json 2> $out/node_$name.err || { tail -5 $out/node_$name.err; exit 1; }
  python - "$out/node_$name.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().splitlines()[-1])
cc = sorted(p["close_call"] for p in d["close_phases_ms"])
print(sys.argv[1].rsplit("/", 1)[-1], "close_call median", cc[len(cc) // 2], cc, "folded before", [p["folded_before_close"] for p in d["close_phases_ms"]], "handler p50", d["report_handler_ms"]["p50"])
PY
done
