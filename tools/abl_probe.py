"""Diagnostics: wall and kernel time of the bench search under ablation builds of the
specialised kernel (QI_JIT_DEFINES, e.g. QI_ABL_NOREC) -- no golden check, counts printed.

    QI_JIT_DEFINES=QI_ABL_NOREC python tools/abl_probe.py [steps] [tag]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import quorum_intersection_amd as qa  # noqa: E402
from quorum_intersection_amd import fbas_gen  # noqa: E402
from quorum_intersection_amd.distributed import DeviceSearch, distributed_search  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
tag = sys.argv[2] if len(sys.argv) > 2 else os.environ.get("QI_JIT_DEFINES", "base")
fb = qa.FBAS(fbas_gen.two_tier(10, 256), device=0)
be = DeviceSearch(fb, jit=2)
for _ in range(2):
    distributed_search(be, device="cuda")
ms, kms, res = [], [], None
for _ in range(steps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = distributed_search(be, device="cuda")
    torch.cuda.synchronize()
    ms.append(1e3 * (time.perf_counter() - t0))
    kms.append(be.kernel_ms)
ms.sort()
kms.sort()
print(json.dumps({"tag": tag, "ms_median": round(ms[len(ms) // 2], 3), "kernel_ms_median": round(kms[len(kms) // 2], 3),
                  "launches": be.launches, "nodes": res.nodes, "evals": res.evals}), flush=True)
