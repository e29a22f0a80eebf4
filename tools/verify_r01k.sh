set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r01k
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit $?
cat $OUT/bench.json
timeout -k 10 200 python bench.py --workload resnet18-secagg --steps 10 --warmup 2 > $OUT/bench_secagg.json 2> $OUT/bench_secagg.err || exit $?
cat $OUT/bench_secagg.json
for w in fedavg iterative weighted; do
  timeout -k 10 300 python tools/ab_variants.py --workload $w --rounds 5 --variants 14,11,6,12 > $OUT/ab_$w.json 2>>$OUT/ab_err.log || exit 1
  cat $OUT/ab_$w.json
done
