set -o pipefail
O=gpurun_out/r02e; mkdir -p $O
timeout -k 10 200 python -u tools/time_report_close.py 10 > $O/close_default.log 2>&1 || exit 1
MALLOC_MMAP_THRESHOLD_=1073741824 MALLOC_TRIM_THRESHOLD_=4294967296 timeout -k 10 200 python -u tools/time_report_close.py 10 > $O/close_heap.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload resnet18-report --steps 8 --warmup 2 --no-cpu-baseline > $O/rep_default.json 2>&1 || exit 1
MALLOC_MMAP_THRESHOLD_=1073741824 MALLOC_TRIM_THRESHOLD_=4294967296 timeout -k 10 300 python -u bench.py --workload resnet18-report --steps 8 --warmup 2 --no-cpu-baseline > $O/rep_heap.json 2>&1 || exit 1
for f in $O/close_*.log; do echo == $f; grep -v amdgpu $f | cut -c1-200; done
for f in $O/rep_*.json; do echo == $f; python -c "import json,sys; r=json.loads([l for l in open('$f') if l.startswith('{')][-1]); print(r['close_ms_after_last_report_all'], r['cycle_close_ms'])"; done
