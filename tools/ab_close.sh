set -o pipefail
O=gpurun_out/r05f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for r in 1 2 3; do
  timeout -k 10 120 python3 -u tools/_variantA/tools/close_phases.py 8 > $O/A_$r.jsonl 2>> $O/err.log || exit 1
  timeout -k 10 120 python3 -u tools/close_phases.py 8 > $O/B_$r.jsonl 2>> $O/err.log || exit 1
  echo "round $r A $(tail -1 $O/A_$r.jsonl | cut -c1-200)"
  echo "round $r B $(tail -1 $O/B_$r.jsonl | cut -c1-200)"
done
timeout -k 10 620 python -u bench.py > $O/bench.json 2> $O/bench.log || { tail -20 $O/bench.log; exit 1; }
tail -c 400 $O/bench.json
