#!/bin/bash
# GPU suite, host base64 of a ResNet-18 diff, and the end-to-end close on a 2-child group sharing GPU 0.
set -o pipefail
O=gpurun_out/${1:-check}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?; tail -2 $O/gpu_tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 200 python tools/bench_b64.py > $O/b64.log 2>&1 || exit 1; cat $O/b64.log
PGH_BENCH_DEVICES=0,0 timeout -k 10 400 python -u bench.py --group --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > $O/group2dev0_e2e.json 2>&1 || exit 1
python -c "import json; r=json.loads([l for l in open('$O/group2dev0_e2e.json') if l.startswith('{')][-1]); print(r['value'], r['cycle_close_e2e'])"
