set -o pipefail
OUT=gpurun_out/r01m
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload resnet18-report --steps 3 --warmup 1 > $OUT/bench_resnet18-report.json 2> $OUT/report.err || exit $?
cat $OUT/bench_resnet18-report.json
timeout -k 10 300 python bench.py --workload resnet18-state --steps 3 --warmup 1 > $OUT/bench_resnet18-state.json 2> $OUT/state.err || exit $?
timeout -k 10 100 python bench.py --workload mnist-state --steps 20 --warmup 3 > $OUT/bench_mnist-state.json 2> $OUT/mnist.err || exit $?
for f in $OUT/bench_*.json; do python3 -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
print('$f', d['value'], d['ms_per_step'], d.get('close_ms_after_last_report'), d.get('h2d_GBps'))"; done
