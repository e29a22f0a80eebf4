#!/bin/bash
# A/B of NUMA-local staging (PGH_NUMA: copy-pool threads bound to the GPU's socket, pinned ring
# allocated there) on the host-bound paths: the end-to-end config-2 close, State bytes -> bytes at
# ResNet-18 x 100, config 5's pinned ingest.   usage: bash tools/ab_numa.sh <tag>
set -o pipefail
O=gpurun_out/${1:-numa}; mkdir -p $O
python -c "
import torch; p = torch.cuda.get_device_properties(0)
bus = '%04x:%02x:%02x.0' % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id)
print('gpu', bus, 'numa', open('/sys/bus/pci/devices/%s/numa_node' % bus).read().strip())" > $O/gpu.txt 2>&1 || true
cat $O/gpu.txt
for r in 1 2; do
  for n in 0 1; do
    PGH_NUMA=$n timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 3 --warmup 1 > $O/default_numa${n}_$r.json 2>&1 || exit 1
    PGH_NUMA=$n timeout -k 10 300 python -u bench.py --workload resnet18-state --no-cpu-baseline --steps 3 --warmup 1 > $O/state_numa${n}_$r.json 2>&1 || exit 1
    PGH_NUMA=$n timeout -k 10 300 python -u bench.py --workload c5-ingest --no-cpu-baseline --steps 2 --warmup 1 > $O/c5_numa${n}_$r.json 2>&1 || exit 1
  done
done
python - "$O" <<'PY'
import json, sys, glob
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    r = json.loads([l for l in open(f) if l.startswith("{")][-1])
    e = r.get("cycle_close_e2e") or {}
    print(f.split("/")[-1], r["value"], r.get("cycle_close_ms") or r.get("kernel_ms"), e.get("cycle_close_ms"), e.get("client_diff_GBps"), r.get("h2d_GBps"), r.get("ingest_GBps_per_gpu"))
PY
