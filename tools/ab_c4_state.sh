set -o pipefail
OUT=gpurun_out/c4ab
mkdir -p $OUT
for v in "" "--variant 14" "--variant 6" "--variant 11"; do
  timeout -k 10 120 python bench.py --workload c4-stream --steps 3 --warmup 1 $v > $OUT/blk_$(echo $v | tr -d ' -').json 2>>$OUT/err.log || exit 1
  PGH_BLOCK_BYTES=0 timeout -k 10 120 python bench.py --workload c4-stream --steps 3 --warmup 1 $v > $OUT/rm_$(echo $v | tr -d ' -').json 2>>$OUT/err.log || exit 1
done
PGH_BLOCK_BYTES=0 timeout -k 10 200 python bench.py --workload resnet18-state --steps 3 --warmup 1 > $OUT/rm_state.json 2>>$OUT/err.log || exit 1
timeout -k 10 200 python bench.py --workload resnet18-state --steps 3 --warmup 1 > $OUT/blk_state.json 2>>$OUT/err.log || exit 1
for f in $OUT/*.json; do python3 -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1])
print('$f', d['value'], d['ms_per_step'], d['roofline']['achieved'], d.get('fold_kernel_client_diff_GBps_aggregated'), d.get('h2d_GBps'))"; done
