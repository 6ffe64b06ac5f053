import os, sys, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import partitionedhashjoin_amd as phj
p = phj.radix_params((8, 8))
with phj.Context(0) as c:
    c.generate_sequential(0, 10_000_000, 1)
    c.generate_zipf(1, 200_000_000, 1.05, 1, 10_000_000, 20240601)
    c.prepare(p)
    for _ in range(3): c.join(p)
    c.synchronize()
    for rep in range(2):
        t = time.perf_counter()
        tot = 0.0
        for _ in range(30):
            r = c.join(p); tot += r.total_ms
        dt = (time.perf_counter() - t) / 30 * 1e3
        print(os.environ.get("V", ""), f"{dt:.4f} ms/step wall, device span {tot/30:.4f}", flush=True)
