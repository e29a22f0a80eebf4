"""Mean per-dispatch value of every counter in a directory of rocprofv3 --pmc CSV passes, per
kernel (names shortened): `python tools/pmc_table.py gpurun_out/pmcv`."""
import collections
import csv
import re
import sys
from pathlib import Path


def main(root):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(Path(root).glob("**/*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            hit = re.search(r"\b(k_\w+)", r["Kernel_Name"])
            name = hit.group(1) if hit else r["Kernel_Name"][:40]
            acc[name][r["Counter_Name"]].append((r["Dispatch_Id"], float(r["Counter_Value"])))
    for name, ctrs in acc.items():
        print(name)
        for c, vals in sorted(ctrs.items()):
            per = collections.defaultdict(float)
            for d, v in vals:
                per[d] += v  # a counter may come per XCD / SE: sum per dispatch
            m = sum(per.values()) / max(len(per), 1)
            print(f"  {c:26s} {m:16.0f}  ({len(per)} dispatches)")


if __name__ == "__main__":
    main(sys.argv[1])
