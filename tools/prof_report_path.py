#!/usr/bin/env python3
"""The kernels of the installed node's report path, profiled:

* K5 ``k_gather_f32``: a report decoded into a page-locked block (``report.PinnedPool``) is DMA'd
  whole and gathered into its slab row -- algorithmic bytes per launch 8 * P (the float payloads
  read once from the DMA'd message, written once into the row);
* the one-row fold ``k_fedavg_rows`` (workers report in assignment order, so each report's
  position is certain at once; ``fold_batch=1`` folds it alone): reads the row and the running
  state, writes the state -- 12 * P per launch (the first row: 8 * P; the close's FINAL pass reads
  the state + checkpoint and writes P floats: also 12 * P).
K5 is profiled on whole reports (``PGH_INGEST_RANGES=0``): with ranged report ingest (r05) each
report's gather runs as one launch per 8 MiB chunk instead.

    python tools/prof_report_path.py run [cycles] [reports]       the workload (run it under rocprofv3)
    python tools/prof_report_path.py summarize <gpurun dir> <profiles dir>

``run``: ResNet-18, per cycle `reports` workers report 5 ms apart (one-row folds, the regime a node
with paced reports sees), each diff base64-decoded into a pinned block and ingested through K5.
``summarize`` expects <dir>/trace (``--kernel-trace --stats``) and <dir>/pmc_FETCH_SIZE,
<dir>/pmc_WRITE_SIZE (separate ``--pmc`` passes) and writes <profiles dir>/report_path.json, and
adds rows for both kernels to profiles/pmc_traffic.json (tied to the kernel sources' sha256).
"""
import base64
import csv
import glob
import json
import sys
import time
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

P = 11_689_512
HBM_PEAK = 8000.0
KERNELS = {"k_gather_f32": 8 * P, "k_fedavg_rows<": 12 * P}


def run(cycles: int, reports: int):
    import os

    import numpy as np

    from pygrid_amd import Engine
    from pygrid_amd.incremental import IncrementalCycle
    from pygrid_amd.report import PinnedPool, b64decode
    from pygrid_amd.state_schema import build_state_fast
    from pygrid_amd.workloads import RESNET18_SHAPES

    rng = np.random.default_rng(5)
    numel = [int(np.prod(s)) for s in RESNET18_SHAPES]
    assert sum(numel) == P
    ck = build_state_fast([rng.standard_normal(s, dtype=np.float32) * np.float32(0.05) for s in RESNET18_SHAPES])
    texts = [base64.b64encode(build_state_fast([rng.standard_normal(s, dtype=np.float32) * np.float32(1e-2)
                                                for s in RESNET18_SHAPES])).decode() for _ in range(4)]
    pool = PinnedPool(max_blocks=8)
    with Engine(0) as eng:
        for cyc in range(cycles):
            os.environ.setdefault("PGH_INGEST_RANGES", "0")  # one K5 launch per report (docstring)
            inc = IncrementalCycle(eng, numel, slots=reports + 2, fold_batch=1, checkpoint=ck)
            for w in range(reports):
                inc.assigned(w)
            for w in range(reports):
                diff = b64decode(texts[w % 4], into=pool)
                inc.reported(w, diff)
                del diff
                time.sleep(0.005)
            ck = inc.close(ck)
            print(f"cycle {cyc}: {inc.last_close}", file=sys.stderr, flush=True)
        st = eng.stats()
    pool.close()
    print(json.dumps({"cycles": cycles, "reports_per_cycle": reports, "pinned_hits": pool.hits,
                      "h2d_bytes_total": st["h2d_bytes_total"]}))


def kernel_stats(tree: Path):
    out = {}
    for f in glob.glob(str(tree / "**" / "*kernel_stats.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                for k in KERNELS:
                    if k in row["Name"]:
                        e = out.setdefault(k, {"calls": 0, "total_ns": 0.0, "name": row["Name"]})
                        e["calls"] += int(row["Calls"])
                        e["total_ns"] += float(row["TotalDurationNs"])
    return out


def per_launch(tree: Path, counter: str):
    vals = {k: defaultdict(float) for k in KERNELS}
    for f in glob.glob(str(tree / "**" / "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                for k in KERNELS:
                    if k in row.get("Kernel_Name", ""):
                        vals[k][(f, row.get("Dispatch_Id"))] += float(row["Counter_Value"])
    return {k: (sum(v.values()) / len(v), len(v)) for k, v in vals.items() if v}


def summarize(src: Path, dst: Path):
    from pmc_summarize import kernels_sha256

    dst.mkdir(parents=True, exist_ok=True)
    ks = kernel_stats(src / "trace")
    fetch = per_launch(src / "pmc_FETCH_SIZE", "FETCH_SIZE")
    write = per_launch(src / "pmc_WRITE_SIZE", "WRITE_SIZE")
    sha = kernels_sha256()
    out = {}
    for k, alg in KERNELS.items():
        if k not in ks:
            continue
        avg_ms = ks[k]["total_ns"] / ks[k]["calls"] / 1e6
        achieved = alg / (avg_ms / 1e3) / 1e9
        e = {"kernel": ks[k]["name"], "launches": ks[k]["calls"], "avg_ms": round(avg_ms, 4),
             "alg_bytes_per_launch": alg, "achieved_GBps": round(achieved, 1), "frac": round(achieved / HBM_PEAK, 4),
             "alg_formula": "8 * P (payload read once + row written)" if "gather" in k
             else "12 * P (row + saved state read, state written)", "P": P}
        if k in fetch and k in write:
            hbm = (2 * fetch[k][0] + write[k][0]) * 1024
            e.update(hbm_bytes_per_launch=hbm, ratio=round(hbm / alg, 6), fetch_size_kb=fetch[k][0],
                     write_size_kb=write[k][0], pmc_launches=fetch[k][1], formula="(2*FETCH_SIZE + WRITE_SIZE)*1024")
        e["kernels_sha256"] = sha
        out[k.rstrip("<")] = e
    (dst / "report_path.json").write_text(json.dumps(out, indent=1) + "\n")
    tf = ROOT / "profiles" / "pmc_traffic.json"
    traffic = json.loads(tf.read_text())
    for k, e in out.items():
        if "hbm_bytes_per_launch" in e:
            traffic[f"report-path/{k}"] = {"per-launch": {
                kk: e[kk] for kk in ("hbm_bytes_per_launch", "alg_bytes_per_launch", "ratio", "kernel", "avg_ms",
                                     "achieved_GBps", "frac", "kernels_sha256")} | {
                "source": f"{dst}/report_path.json (tools/prof_report_path.py: rocprofv3 --kernel-trace --stats, "
                          "--pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes)"}}
    tf.write_text(json.dumps(traffic, indent=1) + "\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 2, int(sys.argv[3]) if len(sys.argv) > 3 else 40)
    else:
        sys.path.insert(0, str(ROOT / "tools"))
        summarize(Path(sys.argv[2]), Path(sys.argv[3]))
