#!/bin/bash
# r03i: where the report decode writes (fresh bytes / page-locked block / reused pageable), and the
# wider-tile fold variants 24-26 against v0 at ResNet-18 x 1,000 (interleaved, one process).
set -o pipefail
out=${1:-gpurun_out/r03i}; mkdir -p $out
timeout -k 10 300 python -u tools/b64_into.py --reps 20 > $out/b64_into.json 2> $out/b64_into.err || exit 1
cat $out/b64_into.json
for wl in fedavg iterative; do
  timeout -k 10 300 python -u tools/ab_variants.py --workload $wl --rounds 6 --variants 0,24,25,26,8 > $out/ab_$wl.json 2> $out/ab_$wl.err || exit 1
  python -c "import json; d=json.loads(open('$out/ab_$wl.json').read().splitlines()[-1]); print('$wl', {k: v.get('GBps_median') for k, v in d['variants'].items()})"
done
