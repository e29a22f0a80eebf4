set -o pipefail
mkdir -p gpurun_out/r04k
for r in 8 1 2 3 4 6 8 12; do
  PGH_SLOT_FINAL_RANGES=$r timeout -k 10 120 python tools/probe_spec_close.py 4 --certain > gpurun_out/r04k/ranges_$r.jsonl 2>> gpurun_out/r04k/err.log || exit 1
done
echo done
