#!/bin/bash
# Does a longer untimed warm-up change the default bench line? (clock / power-state ramp)
# Interleaved: --warmup 5 vs --warmup 60, two rounds, no CPU baseline / e2e / live PMC.
set -o pipefail
mkdir -p gpurun_out/${1:-r02ab}
for r in 1 2; do for w in 5 60; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup $w --no-cpu-baseline --no-e2e --no-live-traffic \
    > gpurun_out/${1:-r02ab}/w${w}_$r.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['kernel_ms'])" gpurun_out/${1:-r02ab}/w${w}_$r.json
done; done
