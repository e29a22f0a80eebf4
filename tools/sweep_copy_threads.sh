#!/bin/bash
# Host -> HBM ingest of pageable State bytes: copy-pool threads and staging size.
set -o pipefail
OUT=gpurun_out/copy_threads
mkdir -p $OUT
nproc > $OUT/nproc.txt; python3 -c "import os; print(len(os.sched_getaffinity(0)))" >> $OUT/nproc.txt
cat /sys/fs/cgroup/cpu.max >> $OUT/nproc.txt 2>/dev/null
for t in 4 8 16 24; do
  PGH_COPY_THREADS=$t timeout -k 10 200 python -u bench.py --workload resnet18-state --steps 5 --warmup 1 --no-cpu-baseline \
      > $OUT/t$t.json 2>>$OUT/err.log || exit 1
  python3 -c "import json; d=json.load(open('$OUT/t$t.json')); print($t, d['value'], d['ms_per_step'], d['h2d_GBps'])"
done
cat $OUT/nproc.txt
