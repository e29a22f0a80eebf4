#!/bin/bash
# One GPU pass into gpurun_out/${TAG:-check}/: the -m gpu suite, smoke, then the default bench line
# (each step time-limited, stopping at the first failure).  STEPS picks a subset, e.g.
# STEPS="tests smoke" or STEPS="bench"; BENCH_ARGS is passed to bench.py.
set -o pipefail
out=gpurun_out/${TAG:-check}
mkdir -p "$out"
steps=${STEPS:-tests smoke bench}
for s in $steps; do
    case $s in
    tests)
        timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
            > "$out/pytest_gpu.log" 2>&1 || { tail -30 "$out/pytest_gpu.log"; exit 1; }
        tail -3 "$out/pytest_gpu.log" ;;
    smoke)
        timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 \
            || { cat "$out/smoke.log"; exit 1; }
        tail -2 "$out/smoke.log" ;;
    bench)
        timeout -k 10 620 python -u bench.py ${BENCH_ARGS:-} > "$out/bench.json" 2> "$out/bench.log" \
            || { tail -20 "$out/bench.log"; exit 1; }
        tail -c 600 "$out/bench.json" ;;
    esac
done
