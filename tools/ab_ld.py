#!/usr/bin/env python3
"""A/B of the slab row pitch skew (PGH_LD_MOD) x kernel variant, interleaved in one process."""
import json
import os
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    import torch

    from pygrid_amd import Engine

    shapes = [(311_650, 10_000), (100_000, 30_000), (3_000_000, 1_000), (11_689_512, 1_000)]
    mods = [1, 2, 8]
    variants = [6, 10]
    res = {}
    for P, N in shapes:
        engines = {}
        for m in mods:
            os.environ["PGH_LD_MOD"] = str(m)
            e = Engine(0)
            e.set_layout([P])
            e.reserve(N)
            e.synth_fill(1, N)
            engines[m] = e
        ck = torch.empty(P, dtype=torch.float32, device="cuda")
        out = torch.empty_like(ck)
        engines[1].synth_ckpt_device(1, ck.data_ptr())
        times = {(m, v): [] for m in mods for v in variants}
        for rnd in range(4):
            for m in mods:
                for v in variants:
                    e = engines[m]
                    e.set_variant(v)
                    e.reset_stats()
                    for _ in range(3):
                        e.fedavg_device(0, ck.data_ptr(), out.data_ptr())
                    st = e.stats()
                    if rnd:
                        times[(m, v)].append(st["kernel_ms_total"] / st["kernel_launches"])
        alg = 4 * N * P + 8 * P
        res[f"P{P}_N{N}"] = {f"mod{m}_v{v}": {"ld": engines[m].slab()[1], "median_ms": round(statistics.median(t), 4),
                                               "GBps": round(alg / statistics.median(t) / 1e6, 1)}
                             for (m, v), t in times.items()}
        for e in engines.values():
            e.close()
        torch.cuda.synchronize()
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
