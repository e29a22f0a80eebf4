#!/usr/bin/env python3
"""Interleaved A/B of one command under several environment settings (cdna_hip_programming.md
rule 24: alternate the arms in one lease, never compare runs from different boxes).

    python tools/ab_env.py --tag r02l --rounds 3 --arm PGH_FINAL_RANGES=1 --arm PGH_FINAL_RANGES=4 \
        -- python3 -u bench.py --workload resnet18-report --steps 5 --no-cpu-baseline

Each --arm is a space-separated list of VAR=VALUE ("" = the defaults).  Every run is its own child
process under `timeout -k 10 <--timeout>`; the first failure ends the A/B (no retries).  Output:
gpurun_out/<tag>/<arm-label>_<round>.log, then one summary line per run: for a bench JSON line its
headline fields, for `time_*.py` logs (lines "<iter> <ms> ...") the median / min after 2 warm-up
iterations.  This parent never touches the GPU.

Round-2 A/Bs run with it (profiles/README.md): PGH_NUMA=0/1 (r02j), PGH_FINAL_RANGES=1/4 (r02k,
r02l), MALLOC_MMAP_THRESHOLD_ / MALLOC_TRIM_THRESHOLD_ heap outputs (r02e), PGH_PREFAULT and
MALLOC_TOP_PAD_ cold closes (r02b), PGH_BLOCK_BYTES slab blocks (r01l).
"""
import argparse
import json
import os
import re
import statistics
import subprocess
import sys
from pathlib import Path

HEADLINE = ("value", "kernel_ms", "cycle_close_ms", "close_ms_after_last_report", "ms_per_step")


def parse_arm(spec: str) -> dict:
    env = {}
    for tok in spec.split():
        k, sep, v = tok.partition("=")
        if not sep or not re.fullmatch(r"[A-Za-z_][A-Za-z0-9_]*", k):
            raise SystemExit(f"ab_env: bad arm setting {tok!r} (want VAR=VALUE)")
        env[k] = v
    return env


def label_of(env: dict) -> str:
    return "_".join(f"{k}-{v}" for k, v in env.items()) or "default"


def summarize(text: str) -> str:
    js = [ln for ln in text.splitlines() if ln.startswith("{")]
    if js:
        try:
            r = json.loads(js[-1])
        except json.JSONDecodeError:
            r = None
        if isinstance(r, dict):
            out = {k: r[k] for k in HEADLINE if k in r}
            e2e = r.get("cycle_close_e2e")
            if isinstance(e2e, dict):
                out["e2e_close_ms"] = e2e.get("cycle_close_ms")
            if r.get("variants"):  # tools/ab_variants.py
                out = {v: d.get("GBps_median") for v, d in r["variants"].items()}
            return json.dumps(out)
    ms = []
    for ln in text.splitlines():
        f = ln.split()
        if len(f) >= 2 and f[0].isdigit():
            try:
                ms.append(float(f[1]))
            except ValueError:
                pass
    if len(ms) > 2:
        return f"median {statistics.median(ms[2:]):.3f} min {min(ms[2:]):.3f} all {[round(x, 2) for x in ms]}"
    return (text.strip().splitlines() or ["(no output)"])[-1][:300]


def main():
    argv = sys.argv[1:]
    if "--" not in argv:
        raise SystemExit("usage: ab_env.py --tag T [--rounds R] --arm 'A=1' --arm 'A=2' -- command ...")
    cut = argv.index("--")
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--arm", action="append", default=[])
    ap.add_argument("--timeout", type=int, default=300)
    a = ap.parse_args(argv[:cut])
    cmd = argv[cut + 1:]
    if not cmd or len(a.arm) < 1:
        raise SystemExit("ab_env: need a command and at least one --arm")
    arms = [parse_arm(s) for s in a.arm]
    out = Path("gpurun_out") / a.tag
    out.mkdir(parents=True, exist_ok=True)
    for rnd in range(1, a.rounds + 1):
        for env in arms:
            log = out / f"{label_of(env)}_{rnd}.log"
            with open(log, "w") as f:
                rc = subprocess.run(["timeout", "-k", "10", str(a.timeout)] + cmd, stdout=f, stderr=subprocess.STDOUT,
                                    env={**os.environ, **env}).returncode
            text = log.read_text(errors="replace")
            print(f"{log.name}: rc={rc} {summarize(text)}", flush=True)
            if rc != 0:
                raise SystemExit(rc)


if __name__ == "__main__":
    main()
