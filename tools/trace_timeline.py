#!/usr/bin/env python3
"""One report-time close on a common clock: kernels, host <-> HBM copies and (when the trace has
them) HIP API calls per host thread, relative to the close's first FINAL range.

    rocprofv3 --kernel-trace --memory-copy-trace [--hip-runtime-trace] -d DIR -o run \
        --output-format csv -- python3 -u tools/close_phases.py 4 --gap-ms 0
    python tools/trace_timeline.py DIR [close index, default -2] [µs before the close, default 1200]

A close is a run of `k_fedavg_rows` launches less than 5 ms apart.  Copies rocprofv3 files as
DEVICE_TO_DEVICE are the staged report H2Ds (the pinned staging slots count as device-accessible);
consecutive identical API calls of one thread are folded into one row "xN".  Columns: start, end,
duration (µs), kind, stream or thread, name.  (Evidence: profiles/r06b/, r06d/.)
"""
import csv
import re
import sys
from pathlib import Path


def main():
    d = Path(sys.argv[1])
    which = int(sys.argv[2]) if len(sys.argv) > 2 else -2
    before = float(sys.argv[3]) * 1e3 if len(sys.argv) > 3 else 1.2e6
    ev = []
    for r in csv.DictReader(open(d / "run_memory_copy_trace.csv")):
        kind = "D2H" if "DEVICE_TO_HOST" in r["Direction"] else "H2D"
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind, "s" + r["Stream_Id"], ""))
    for r in csv.DictReader(open(d / "run_kernel_trace.csv")):
        m = re.search(r"(k_\w+|__amd_rocclr_\w+)", r["Kernel_Name"])
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K", "s" + r["Stream_Id"],
                   m.group(1) if m else r["Kernel_Name"][:40]))
    api = d / "run_hip_api_trace.csv"
    if api.exists():
        tids = {}
        for r in csv.DictReader(open(api)):
            if r["Function"] in ("hipGetLastError", "hipPeekAtLastError"):
                continue
            t = tids.setdefault(r["Thread_Id"], "T%d" % len(tids))
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "API", t, r["Function"]))
    ev.sort()
    closes, cur = [], []
    for e in ev:
        if e[2] != "K" or "fedavg_rows" not in e[4]:
            continue
        if cur and e[0] - cur[-1][1] > 5e6:
            closes.append(cur)
            cur = []
        cur.append(e)
    closes.append(cur)
    t0 = closes[which][0][0]
    rows, prev, n = [], None, 0
    for e in ev:
        if not (t0 - before < e[0] < t0 + 2.6e6):
            continue
        if prev and e[2] == "API" == prev[2] and e[3] == prev[3] and e[4] == prev[4]:
            prev, n = (prev[0], e[1], prev[2], prev[3], prev[4]), n + 1
            continue
        if prev:
            rows.append((prev, n))
        prev, n = e, 1
    if prev:
        rows.append((prev, n))
    for e, k in rows:
        print(f"{(e[0] - t0) / 1e3:9.1f} {(e[1] - t0) / 1e3:9.1f} {(e[1] - e[0]) / 1e3:7.1f} {e[2]:4} {e[3]:4} {e[4]}"
              + (f" x{k}" if k > 1 else ""))


if __name__ == "__main__":
    main()
