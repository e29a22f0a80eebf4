set -o pipefail
O=gpurun_out/r02l; mkdir -p $O
for r in 1 2 3; do
  for k in 1 4; do
    PGH_FINAL_RANGES=$k timeout -k 10 200 python -u tools/time_report_close.py 12 > $O/close_r${k}_$r.log 2>&1 || exit 1
  done
done
for f in $O/*.log; do python - "$f" <<'PY'
import sys, statistics
v = [float(l.split()[1]) for l in open(sys.argv[1]) if l[:1].isdigit()]
print(sys.argv[1].split("/")[-1], "median", round(statistics.median(v[2:]), 3), "min", round(min(v[2:]), 3), [round(x, 2) for x in v])
PY
done
