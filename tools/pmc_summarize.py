#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes into per-launch HBM bytes (profiles/<run>/pmc_summary.json) and
refresh profiles/pmc_traffic.json, which bench.py reads for roofline.traffic.

    python tools/pmc_summarize.py gpurun_out/r01l profiles/r01l

Expects <dir>/pmc_<workload>_FETCH_SIZE/ and _WRITE_SIZE/ trees of rocprofv3 CSV output and the
matching bench line <dir>/pmc_<workload>_FETCH_SIZE.log (for the variant and algorithmic bytes).
HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: on gfx950 FETCH_SIZE counts half
the bytes of wide streaming reads (MI355X_MICROARCH.md, HBM section).
"""
import csv
import glob
import json
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
KERNEL = {"resnet18-fedavg": "k_fedavg", "resnet18-iterative": "k_fedavg", "resnet18-weighted": "k_fedavg",
          "resnet18-secagg": "k_secagg", "resnet18-report": "k_fedavg_rows"}


def kernels_sha256() -> str:
    """Hash of the kernel sources the counters were measured on (bench.py refuses to quote stale
    traffic once they change)."""
    import hashlib

    h = hashlib.sha256()
    for f in ("pygrid_amd/csrc/pgh_kernels.hip", "pygrid_amd/csrc/pgh_kernels.h"):
        h.update((ROOT / f).read_bytes())
    return h.hexdigest()


def per_launch(tree: Path, counter: str, kernel: str):
    vals = defaultdict(float)
    name = None
    for f in glob.glob(str(tree / "**" / "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                # "k_secagg<" / "k_fedavg<": not k_secagg_decode (pgh_create's warm-up) or k_fedavg_rows
                if row.get("Counter_Name") != counter or (kernel + "<") not in row.get("Kernel_Name", ""):
                    continue
                vals[(f, row.get("Dispatch_Id"))] += float(row["Counter_Value"])
                name = row["Kernel_Name"]
    if not vals:
        raise SystemExit(f"no {counter} rows for {kernel} under {tree}")
    return sum(vals.values()) / len(vals), len(vals), name


def bench_line(log: Path):
    for line in log.read_text().splitlines():
        if line.startswith("{"):
            return json.loads(line)
    raise SystemExit(f"no bench line in {log}")


def main():
    src, dst = Path(sys.argv[1]), Path(sys.argv[2])
    dst.mkdir(parents=True, exist_ok=True)
    summary = {}
    for w, k in KERNEL.items():
        if not (src / f"pmc_{w}_FETCH_SIZE").exists():
            continue
        fetch, n, name = per_launch(src / f"pmc_{w}_FETCH_SIZE", "FETCH_SIZE", k)
        write, _, _ = per_launch(src / f"pmc_{w}_WRITE_SIZE", "WRITE_SIZE", k)
        b = bench_line(src / f"pmc_{w}_FETCH_SIZE.log")
        alg = b["roofline"]["alg_bytes_per_launch"]
        hbm = (2 * fetch + write) * 1024
        summary[w] = {"variant": b["config"]["kernel_variant"], "hbm_bytes_per_launch": hbm,
                      "alg_bytes_per_launch": alg, "ratio": hbm / alg, "fetch_size_kb": fetch,
                      "write_size_kb": write, "launches_per_pass": n, "kernel": name,
                      "layout": "column-blocked slab (256 KiB blocks)",
                      "formula": "(2*FETCH_SIZE + WRITE_SIZE)*1024",
                      "source": f"{dst}/pmc_summary.json (rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE, "
                                f"separate passes)"}
    if not summary:  # no PMC passes under src: keep the committed traffic file as it is
        raise SystemExit(f"no pmc_<workload>_FETCH_SIZE passes under {src}; nothing written")
    sha = kernels_sha256()
    for e in summary.values():
        e["kernels_sha256"] = sha
    (dst / "pmc_summary.json").write_text(json.dumps(summary, indent=1) + "\n")
    path = ROOT / "profiles" / "pmc_traffic.json"
    traffic = json.loads(path.read_text()) if path.exists() else {}  # other tools' rows (report-path/*) stay
    traffic.update({w: {str(e["variant"]): {kk: e[kk] for kk in ("hbm_bytes_per_launch", "alg_bytes_per_launch",
                                                                "ratio", "kernel", "layout", "source",
                                                                "kernels_sha256")}}
                    for w, e in summary.items()})
    path.write_text(json.dumps(traffic, indent=1) + "\n")
    for w, e in summary.items():
        print(w, e["variant"], f"ratio {e['ratio']:.6f}")


if __name__ == "__main__":
    main()
