#!/bin/bash
set -o pipefail
out=${1:-gpurun_out/r03k}; mkdir -p $out
for arm in "spec50:--phases" "nospec50:--no-speculate --phases"; do
  name=${arm%%:*}; flags=${arm#*:}
  timeout -k 10 300 python -u tools/node_sim.py 6 $flags > $out/node_$name.json 2> $out/node_$name.err || { tail -5 $out/node_$name.err; exit 1; }
  python - "$out/node_$name.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().splitlines()[-1])
for p in d["close_phases_ms"]:
    print(sys.argv[1].rsplit("/", 1)[-1], p)
PY
done
