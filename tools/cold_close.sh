#!/bin/bash
# Cold cycle closes (a node closes a cycle every few minutes): per-phase times of the first closes
# under glibc / prefault variants, and closes after idle gaps.   usage: bash tools/cold_close.sh <tag>
set -o pipefail
mkdir -p gpurun_out/${1:-cold}
O=gpurun_out/${1:-cold}
timeout -k 10 120 python -u tools/time_mnist_second.py 8 > $O/second_default.log 2>&1 || exit 1
MALLOC_MMAP_THRESHOLD_=131072 timeout -k 10 120 python -u tools/time_mnist_second.py 8 > $O/second_mmap_fixed.log 2>&1 || exit 1
PGH_PREFAULT=0 timeout -k 10 120 python -u tools/time_mnist_second.py 8 > $O/second_noprefault.log 2>&1 || exit 1
MALLOC_TOP_PAD_=67108864 timeout -k 10 120 python -u tools/time_mnist_second.py 8 > $O/second_toppad.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/time_mnist_cold.py > $O/mnist_cold.log 2>&1 || exit 1
for f in $O/*.log; do echo "== $f"; grep -v amdgpu.ids $f | head -12; done
