set -o pipefail
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "iter or edge or kat or mnist or stream or incremental or resnet18 or variants" > gpurun_out/gt.log 2>&1; rc=$?; tail -3 gpurun_out/gt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab_variants.py --workload iterative --rounds 4 --variants 0,6,15,11,14 || exit 1
for cfg in "100000 30000" "50000 60000" "311650 10000" "1000000 3000"; do set -- $cfg; timeout -k 10 200 python tools/ab_variants.py --workload iterative --params $1 --clients $2 --rounds 3 --variants 0,11,12,14,17 || exit 1; done
