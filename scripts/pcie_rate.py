#!/usr/bin/env python3
"""PCIe-inclusive rate of the C2 join: the reference's Run(tableA, tableB)
hands host tables to the joiner, so the GPU path uploads them first. Times
the upload (pinned and pageable host memory) and upload + join.
Prints one JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch
    import partitionedhashjoin_amd as phj
    nR, nS = 10_000_000, 200_000_000
    c = phj.Context(0)
    c.generate_sequential(0, nR, 1)
    c.generate_zipf(1, nS, 1.05, 1, nR, 20240601)
    R = c.download(0)
    S = c.download(1)
    p = phj.radix_params((8, 8))
    out = {}
    for kind in ("pageable", "pinned"):
        if kind == "pinned":
            Rt = torch.from_numpy(R).pin_memory()
            St = torch.from_numpy(S).pin_memory()
            Rh, Sh = Rt.numpy(), St.numpy()
        else:
            Rh, Sh = R, S
        c.upload(0, Rh)
        c.upload(1, Sh)
        c.join(p)
        t0 = time.perf_counter()
        c.upload(0, Rh)
        c.upload(1, Sh)
        t1 = time.perf_counter()
        r = c.join(p)
        t2 = time.perf_counter()
        gb = (R.nbytes + S.nbytes) / 1e9
        out[kind] = {"upload_ms": (t1 - t0) * 1e3, "upload_GBps": gb / (t1 - t0),
                     "join_ms": (t2 - t1) * 1e3, "tuples_per_s_pcie_inclusive": (nR + nS) / (t2 - t0),
                     "matches": r.matches}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
