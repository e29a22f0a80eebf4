#!/usr/bin/env python3
"""The bench's N > 1 step (sharding.OverlappedGather: range folds over two streams, async RCCL
all-gather per range, per-range placement) at world size 1 over RCCL, against one whole fold:
what the multi-GPU step costs a rank besides the xGMI transfer itself.

    python tools/ab_overlap_world1.py [chunks:tail ...]     (default 2:0 4:0 6:0 8:0 8:3 4:2)
"""
import json
import os
import socket
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    import torch
    import torch.distributed as dist

    from pygrid_amd import Engine
    from pygrid_amd.sharding import OverlappedGather

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    P, N = 11_689_512, 1000
    eng = Engine(0)
    eng.set_layout([P])
    eng.reserve(N)
    eng.synth_fill(1, N)
    sp = torch.cuda.current_stream().cuda_stream
    ck = torch.empty(P, dtype=torch.float32, device="cuda")
    out = torch.empty_like(ck)
    eng.synth_ckpt_device(1, ck.data_ptr(), sp)
    res = {}
    plans = [tuple(int(x) for x in a.split(":")) for a in sys.argv[1:]] or [(2, 0), (4, 0), (6, 0), (8, 0), (8, 3), (4, 2)]
    ogs = {pl: OverlappedGather(P, 1, 0, chunks=pl[0], tail=pl[1]) for pl in plans}

    def whole():
        eng.fedavg_device(0, ck.data_ptr(), out.data_ptr(), sp)

    def overlapped(pl, coll):
        og = ogs[pl]
        lp = og.local.data_ptr()
        og.run(lambda off, n, st: eng.fedavg_device_range(0, off, n, ck.data_ptr(), lp, st), force_collective=coll)
        og.assemble()

    cases = {"whole": whole}
    for pl in plans:
        cases[f"ranges{pl[0]}t{pl[1]}_rccl"] = (lambda pl=pl: overlapped(pl, True))
        cases[f"ranges{pl[0]}t{pl[1]}_copy"] = (lambda pl=pl: overlapped(pl, False))
    for f in cases.values():
        f()
    torch.cuda.synchronize()
    for _ in range(6):
        for name, f in cases.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                f()
            torch.cuda.synchronize()
            res.setdefault(name, []).append((time.perf_counter() - t0) / 5 * 1e3)
    print(json.dumps({k: round(statistics.median(v), 4) for k, v in res.items()}))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
