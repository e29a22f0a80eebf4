"""Host allocator settings for a node that moves 47 MB buffers per report and per close.

Every ResNet-18 diff a report decodes, and every new checkpoint a close returns, is a fresh ~47 MB
``bytes`` object.  glibc serves allocations that big with their own ``mmap`` and returns them with
``munmap`` when freed: the pages are faulted in again for every new buffer, and freeing one that
16 copy threads filled costs TLB shootdowns on all of them.  In a node that is on the close's path
-- the previous checkpoint is dropped when ``_average_plan_diffs`` returns -- and measured 3-6 ms
per close against 1.8-2.1 ms for the close itself (``tools/node_sim.py``, ``profiles/r02bk/``).

``tune()`` raises glibc's mmap threshold to 256 MiB and its trim threshold to 1 GiB
(``mallopt``), so such buffers come from the heap and their pages are reused.  The cost is that up
to 1 GiB of freed heap stays mapped in the process.  This changes the allocator of the WHOLE host
process (the reference node's own torch loop included), so it is never applied on import: a host
application opts in with ``pygrid_amd.tune_process()``.  ``PGH_MALLOC_TUNE=0`` makes ``tune`` a
no-op.  Returns whether it applied the settings.
"""
from __future__ import annotations

import ctypes as C
import os

M_TRIM_THRESHOLD = -1  # glibc malloc.h
M_MMAP_THRESHOLD = -3
MMAP_THRESHOLD = 256 << 20
TRIM_THRESHOLD = 1 << 30  # mallopt takes an int: 2 GiB would wrap to -2^31 (trimming off for good)


def tune() -> bool:
    if os.environ.get("PGH_MALLOC_TUNE", "1") == "0":
        return False
    try:
        libc = C.CDLL("libc.so.6")
        mallopt = libc.mallopt
    except (OSError, AttributeError):  # not glibc: nothing to tune
        return False
    mallopt.argtypes = [C.c_int, C.c_int]
    mallopt.restype = C.c_int
    ok = mallopt(M_MMAP_THRESHOLD, MMAP_THRESHOLD) == 1
    ok = mallopt(M_TRIM_THRESHOLD, TRIM_THRESHOLD) == 1 and ok
    return ok
