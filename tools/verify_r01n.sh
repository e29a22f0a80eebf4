set -o pipefail
OUT=gpurun_out/r01n
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread --durations=8 > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -14 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for cfg in "100000 30000" "50000 60000" "311650 10000"; do
  set -- $cfg
  timeout -k 10 200 python tools/ab_variants.py --workload iterative --params $1 --clients $2 --rounds 3 --variants 12,14,16,17,18,11 > $OUT/iterative_p$1.json 2>>$OUT/err.log || exit 1
done
python3 -c "
import json,glob
for f in sorted(glob.glob('$OUT/*.json')):
    d=json.load(open(f)); print(d['workload'], d['P'], d['N'], {k:v['GBps_median'] for k,v in d['variants'].items()})
"
