#!/usr/bin/env python3
"""Headline benchmark: BASELINE.json metric on config C2.

  "probe+build tuples/sec at 10M⋈200M; achieved HBM GB/s vs roofline, 1/2/4/8 GPU"
  C2: RadixCluster 2-pass (8+8 radix bits), 10M ⋈ 200M, Murmur3, Zipf s=1.05.

One step = one full join over the resident relations (partition R and S,
build, probe, count back on the host), exactly HashJoiner::Run
(src/RadixCluster/HashJoin.hpp:190-241). Relations are generated on the
device before the timed region (the reference also times after generation,
src/main.cpp:254 vs :100-102).

N=1:  python bench.py [--steps K --warmup W]
N>1:  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
      Both relations are range-sharded (strong scaling: the 10M⋈200M
      workload is fixed); each rank's context (phj_ctx_create_rank) runs the
      multi-GPU member step in libphj_hip.so: the partitioned build keys are
      all-gathered and the count all-reduced over RCCL (csrc/phj_group.h).

Rank 0 prints ONE JSON line. `roofline` is for the dominant kernel (longest
per-step device time), from hipEvents on the stream the kernels run on;
`cpu_baseline` times the oracle's restatement of the reference RadixCluster
path (-p 1024, XXH3: its best published configuration) on this host.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)
NR, NS, ALPHA, GEN_SEED = 10_000_000, 200_000_000, 1.05, 20240601


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=["c2", "c4", "c5"],
                    help="c2: radix 8+8 murmur3 s=1.05; c4: no-partitioning xxh3; c5: radix s=1.25")
    ap.add_argument("--skew", type=float, default=None, help="Zipf skew of S (default: the config's)")
    ap.add_argument("--primary", type=int, default=NR)
    ap.add_argument("--secondary", type=int, default=NS)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: the core share - 1 (cpu_threads)")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--no-traffic", action="store_true", help="skip the rocprofv3 PMC passes")
    ap.add_argument("--all-timers", action="store_true",
                    help="time every phase in the timed loop (default: PHJ_LEAN_TIMERS, only S's pass 1 and the "
                         "LDS join; each event between two kernels delays the second by ~4 us)")
    ap.add_argument("--timers-per-step", dest="timers_deferred", action="store_false",
                    help="read each step's timers inside it (default: one device defers the readout past the timed "
                         "loop, PHJ_DEFER_TIMERS)")
    ap.add_argument("--exchange", action="store_true",
                    help="at one GPU, run the N>1 step (RCCL all-gather + all-reduce) on a world of one")
    return ap.parse_args()


def config_params(phj, name):
    if name == "c4":
        return phj.nopart_params(hash=phj.HASH_XXH3), ALPHA, \
            "C4: NoPartitioning, global table in HBM, XXH3, 10M⋈200M, Zipf s=1.05"
    if name == "c5":
        return phj.radix_params((8, 8), hash=phj.HASH_MURMUR3), 1.25, \
            "C5: RadixCluster 2-pass 8+8, Murmur3, 10M⋈200M, Zipf s=1.25"
    return phj.radix_params((8, 8), hash=phj.HASH_MURMUR3), ALPHA, \
        "C2: RadixCluster 2-pass 8+8, Murmur3, 10M⋈200M, Zipf s=1.05"


def probe_phase(per_step, nR, nS, ms_per_step, traffic=None):
    """The north star's probe-phase figure (target >= 60 % of the HBM roofline
    at 1 GPU). SURVEY.md §8(d) prices the probe phase at 16 B per R and per S
    tuple (3.36 GB at 10M⋈200M: >= 60 % means <= 0.70 ms), assuming one fused
    build + probe kernel. That is what the probe kernel is here:
    k_cluster_probe (csrc/phj_cluster.h) builds each cluster's table from R's
    codes in LDS and probes S's pass-1 codes against it, in one launch whose
    time the library reports as the `build` and `probe` timers, split by the
    kernel's own clocks (`build.big`: the HBM tables of clusters beyond the
    LDS limit, a separate launch, none at C2). The same byte count over three
    spans, so rounds compare like for like:
      frac_survey_def              - over the whole LDS join kernel (build + probe
                                     timers: the figure the target is read against)
      frac_survey_def_probe_only   - over its probe share alone
      frac_survey_def_span         - over the step minus S's pass 1: the whole
                                     critical path after it (gaps, the count)
    and frac_bytes_read: the bytes the kernel reads by design (8 B per S code
    and per R code) over its time. With PHJ_CLUSTER=0 the build is k_ht_fill
    beside S's pass 1 and the probe k_probe_ht; `ms` is then the probe alone."""
    if "probe" not in per_step:
        return None
    probe_ms = per_step["probe"][0]
    build_ms = per_step.get("build", (0.0, 0))[0]
    fused = "build.big" in per_step   # the LDS join: build and probe are one launch
    ms = probe_ms + build_ms if fused else probe_ms
    if ms <= 0:
        return None
    b_def, b_read = 16 * (nR + nS), 8 * (nS + nR)
    frac = lambda b, t: b / (t * 1e-3) / 1e9 / HBM_PEAK_GBS if t > 0 else None
    span_ms = ms_per_step - per_step.get("S.p1.scatter", (0.0, 0))[0]
    return {"kernel": "k_cluster_probe: LDS build + probe, one launch" if fused else "k_probe_ht (probe timer)",
            "ms": ms, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "target": "frac_survey_def >= 0.60",
            "bytes_survey_def": b_def, "achieved_survey_def": b_def / (ms * 1e-3) / 1e9,
            "frac_survey_def": frac(b_def, ms),
            "build_ms_in_kernel": build_ms if fused else None, "probe_only_ms": probe_ms,
            "frac_survey_def_probe_only": frac(b_def, probe_ms),
            "span_ms": span_ms, "frac_survey_def_span": frac(b_def, span_ms),
            "bytes_read": b_read, "achieved_bytes_read": b_read / (ms * 1e-3) / 1e9,
            "frac_bytes_read": frac(b_read, ms),
            # HBM bytes of the probe kernel's launch from the PMC passes (k_cluster_probe's own
            # counters; its big-cluster companion is build.big's / not attributed), or null
            "traffic": (traffic or {}).get("probe"),
            "target_ms_survey_def": b_def / (0.6 * HBM_PEAK_GBS * 1e9) * 1e3,
            "note": ("frac_survey_def is a time target, not a bandwidth: the survey prices the phase at 16 B per "
                     "R and S tuple (a phase that re-reads the tuples); here pass 1 already reduced each tuple to "
                     "an 8-B code, so the phase reads 8 B per tuple and the figure can exceed 1. Its bandwidth is "
                     "frac_bytes_read")}


def pmc_traffic(args, verbose):
    """HBM bytes per launch of each join phase from rocprofv3 PMC counters
    (scripts/pmc.py: the memory-side read requests by size and WRITE_SIZE in
    separate passes, child processes run BEFORE this process touches the GPU;
    request sizes calibrated in scripts/pmc_calib.hip). Returns {timer name:
    bytes} ({} if unavailable)."""
    import shutil
    if not shutil.which("rocprofv3"):
        return {}
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import pmc
    try:
        per = pmc.collect([pmc.READ_COUNTERS, ["WRITE_SIZE"]], args.config, args.primary, args.secondary)
    except Exception as e:  # profiler unavailable: traffic stays null
        if verbose:
            print(f"pmc passes failed: {e}", file=sys.stderr)
        return {}
    return pmc.hbm_bytes(per)


def host_cpu():
    """The host's CPU model and the core share this process may use: nproc
    (os.cpu_count: the whole machine), the affinity mask and the cgroup CPU
    quota (a GPU box grants one GPU's share of a larger machine)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    nproc = os.cpu_count() or 1
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = nproc
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    return {"model": model, "nproc": nproc, "affinity": affinity, "cgroup_quota": quota}


def cpu_threads(cpu):
    """The reference sizes its pool hardware_concurrency() - 1 (src/main.cpp:235).
    On a GPU box nproc counts the whole machine while one GPU's share is 16
    cores (the pool's rule), so the pool is min(nproc, affinity, quota, 16) - 1."""
    share = min(x for x in (cpu["nproc"], cpu["affinity"], cpu["cgroup_quota"] or 10**9, 16))
    return max(1, share - 1)


def cpu_baseline(ctx, nR, nS, threads, verbose):
    """The oracle's restatement of the reference's three published CPU legs
    (results/1.05/figure.dat cols 2, 3 and 8: NoPartitioning, RadixCluster
    -p 32 and -p 1024, XXH3, LinearProbing 3-slot 1.25x) on this host's cores,
    over the same device-generated relations (copied back), once each.
    `value` is the best RadixCluster leg (-p 1024, the reference's best
    published configuration); every leg is in `legs`."""
    from oracle import oracle as O
    R = ctx.download(0)
    S = ctx.download(1)
    cpu = host_cpu()
    legs = {}
    runs = 3   # per leg; the median is reported (one run differed 2x from box to box)

    def median_run(fn, key):
        res = [fn() for _ in range(runs)]
        res.sort(key=key)
        return res[runs // 2], [key(r) for r in res]

    # RadixCluster: Run()'s wall from SetPartitioningPhaseBegin to the end of
    # Join(); the partitioned copies are allocated before the timer, as in the
    # reference (RadixCluster/HashJoin.hpp:195-198)
    for P in (1024, 32):
        res, all_ms = median_run(lambda: O.join_radix(R, S, P=P, radix=False, part_hash=O.HASH_XXH3, part_seed=1,
                                                      table_hash=O.HASH_XXH3, table_seed=2, ratio=1.25,
                                                      workers=threads), lambda r: r.wall_ms)
        legs[f"radix_p{P}"] = {"ms": res.wall_ms, "runs_ms": all_ms, "partition_ms": res.partition_ms,
                               "build_ms": res.build_ms, "probe_ms": res.probe_ms, "matches": int(res.matches),
                               "tuples_per_s": (nR + nS) / (res.wall_ms * 1e-3)}
    # NoPartitioning: the reference reports probe from the build start
    # (Results.hpp:202), i.e. build + probe, the table allocation included
    res, all_ms = median_run(lambda: O.join_nopart(R, S, hash_kind=O.HASH_XXH3, seed=2, ratio=1.25, workers=threads),
                             lambda r: r.probe_ms)
    legs["nopartitioning"] = {"ms": res.probe_ms, "runs_ms": all_ms, "build_ms": res.build_ms, "probe_ms": res.probe_ms,
                              "matches": int(res.matches), "tuples_per_s": (nR + nS) / (res.probe_ms * 1e-3)}
    del R, S
    if verbose:
        print(f"cpu baseline: {legs} on {cpu}", file=sys.stderr)
    best = legs["radix_p1024"]
    desc = "; ".join(f"{k} {v['ms']:.0f} ms" for k, v in legs.items())
    return {
        "value": best["tuples_per_s"],
        "unit": "tuples/s",
        "cores": threads,
        "kind": "port",
        "sample": f"full {nR // 10**6}M⋈{nS // 10**6}M workload (the bench's relations copied back), median of "
                  f"{runs} runs per leg of the oracle's restatement of the reference's published CPU legs, XXH3, "
                  f"LinearProbing 3-slot 1.25x, {threads} worker threads (hardware_concurrency()-1 over "
                  f"this box's {min(16, cpu['affinity'])}-core share; nproc {cpu['nproc']}, {cpu['model']}): "
                  f"{desc}; value = radix -p 1024 (reference phase semantics)",
        "legs": legs,
        "host": cpu,
        "matches": {k: v["matches"] for k, v in legs.items()},
    }


def main():
    args = parse()
    # stdout carries exactly one JSON line: libraries that print banners there
    # (RCCL prints its version on communicator init) are sent to stderr
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # PMC passes first: child processes, before this process initialises the GPU
    traffic = {} if (world > 1 or args.no_traffic) else pmc_traffic(args, args.verbose)
    import torch
    import torch.distributed as dist
    import partitionedhashjoin_amd as phj
    from partitionedhashjoin_amd.distributed import generate_shards, rank_context

    exchange = world > 1 or args.exchange
    if exchange:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29571")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    nR, nS = args.primary, args.secondary
    params, alpha, workload = config_params(phj, args.config)
    if args.skew is not None:
        alpha = args.skew
        workload += f" (skew overridden: {alpha})"
    # the join is one C call per step on this rank's context: a single-device
    # phj_join at N=1; at N>1 (or --exchange) the multi-GPU member step of
    # csrc/phj_group.h (R partition + RCCL all-gather of the build keys beside
    # the S partition, fused join, RCCL all-reduce of the count)
    ctx = rank_context(local_rank, rank, world, dist if exchange else None, exchange=args.exchange)
    generate_shards(ctx, nR, nS, alpha, GEN_SEED, rank, world)
    torch.cuda.synchronize()
    # correctness gate at full size: every generated S key lies in [1, |R|]
    local_inrange = ctx.count_in_range(1, 1, nR)
    ctx.prepare(params)   # workspace allocated outside the timed region

    radix = params.algo == phj.ALGO_RADIX

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    # the warm-up steps run the timed steps' own flags (below)
    defer = args.timers_deferred and params.algo == phj.ALGO_RADIX
    timed_params = params
    if defer:
        timed_params = type(params).from_buffer_copy(params)
        # (lean on one device: 7 us faster there, 8 us slower in the W=8 rehearsal's member step)
        lean = world == 1 and not exchange and not args.all_timers
        timed_params.flags = params.flags | phj.DEFER_TIMERS | (phj.LEAN_TIMERS if lean else 0)
    for _ in range(args.warmup):
        ctx.join(timed_params)
    if defer:
        ctx.timers_report()   # a clean slate

    barrier()
    t0 = time.perf_counter()
    acc = {}
    matches = None
    exch = 0.0

    def accumulate(timers):
        for name, ms, nbytes in timers:
            a = acc.setdefault(name, [0.0, 0])
            a[0] += ms
            a[1] += nbytes

    # one device: PHJ_DEFER_TIMERS keeps the timer readout (event queries, the
    # LDS join's clock split) out of the timed steps; the events are recorded
    # inside them and summed by timers_report after the loop
    # (at N>1 each rank's context has one member: the same, per rank); one
    # device: PHJ_LEAN_TIMERS also leaves R's pass-1 timer out (--all-timers)
    results = [ctx.join(timed_params) for _ in range(args.steps)]
    barrier()
    elapsed = time.perf_counter() - t0
    # each step's timers are its own HIP events, recorded in the timed region;
    # they are read out here, after it (Python bookkeeping is not the join)
    for res in results:
        matches = res.matches
        exch += res.exchange_ms
        if not defer:
            accumulate(res.timers())
    if defer:
        rep = ctx.timers_report().timers()
        accumulate(rep)
        exch = sum(ms for name, ms, _ in rep if name == "exchange")

    def allsum(x):
        if world == 1:
            return int(x)
        t = torch.tensor([int(x)], dtype=torch.int64, device="cuda")
        dist.all_reduce(t)
        return int(t.item())

    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    inrange = allsum(local_inrange)
    # a non-trivial full-size check after the timed region (the default inputs'
    # answer is always |S|): R shifted to [1 + SHIFT, |R| + SHIFT] makes the
    # hottest Zipf keys miss; the join must count exactly the S keys in range
    # It runs the timed steps' own flags (DEFER|LEAN on one device: the count
    # polled from pinned host memory, S's chunk state cleared by the previous
    # join's last workgroup), three joins back to back, then the plain flags
    shift = 3
    generate_shards(ctx, nR, nS, alpha, GEN_SEED, rank, world, start=1 + shift)
    shifted_expect = allsum(ctx.count_in_range(1, 1 + shift, nR))
    shifted_runs, shifted_ms = [], []   # (host wall time per join: the misses' probe cost)
    for p in [timed_params] * 3 + [params]:
        t_join = time.perf_counter()
        shifted_runs.append(ctx.join(p).matches)
        shifted_ms.append(round((time.perf_counter() - t_join) * 1e3, 4))
    if defer:
        ctx.timers_report()   # (the check's deferred timers are not the bench's)
    shifted_got = shifted_runs[0]
    shifted_ok = all(m == shifted_expect for m in shifted_runs) and shifted_expect < inrange
    generate_shards(ctx, nR, nS, alpha, GEN_SEED, rank, world)

    if rank == 0:
        per_step = {k: (v[0] / args.steps, v[1] / args.steps) for k, v in acc.items()}
        # the dominant kernel of the critical path: the R partition runs on its
        # own stream beside S, and at N=1 its first timer also spans the wait for
        # the persistent S scatter to free the CUs
        crit = {k: v for k, v in per_step.items() if not k.startswith("R.") and k != "exchange"} or per_step
        if crit:
            dom_name, (dom_ms, dom_bytes) = max(crit.items(), key=lambda kv: kv[1][0])
        else:   # no timers recorded (PHJ_TIMERS=0): the roofline is unmeasured
            dom_name, dom_ms, dom_bytes = None, 0.0, 0
        achieved = dom_bytes / (dom_ms * 1e-3) / 1e9 if dom_ms > 0 else None
        value = (nR + nS) * args.steps / elapsed
        out = {
            "metric": "probe+build tuples/sec at 10M⋈200M; achieved HBM GB/s vs roofline, 1/2/4/8 GPU",
            "value": value,
            "unit": "tuples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic (device-generated Sequential R + seeded Zipf S, reference generators)",
            "config": {"workload": workload, "primary": nR, "secondary": nS,
                       "radix_bits": list(params.radix_bits) if params.algo == phj.ALGO_RADIX else None,
                       "hash": "murmur3" if params.hash == phj.HASH_MURMUR3 else "xxh3",
                       "skew": alpha, "parallelism": f"range-shard x{world}"
                       + (" (exchange path)" if exchange and world == 1 else "")},
            "matches": int(matches),
            "expected_matches": inrange,
            "shifted_check": {"build_start": 1 + shift, "expected": shifted_expect, "matches": shifted_got,
                              "runs": shifted_runs, "wall_ms": shifted_ms, "flags": int(timed_params.flags),
                              "plain_flags": int(params.flags)},
            "correct": int(matches) == inrange and shifted_ok,
            "exchange_ms": exch / args.steps if exchange else None,
            "roofline": {"bound": "hbm", "kernel": dom_name, "achieved": achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS if achieved is not None else None,
                         "traffic": traffic.get(dom_name), "algorithmic_bytes": dom_bytes,
                         "ms": dom_ms},
            "probe_phase": probe_phase(per_step, nR, nS, elapsed * 1e3 / args.steps, traffic) if radix else None,
            "kernels_ms": {k: round(v[0], 4) for k, v in sorted(per_step.items())},
            "kernels_traffic_bytes": {k: int(v) for k, v in sorted(traffic.items())} or None,
        }
        if world == 1 and not args.no_cpu_baseline:
            threads = args.cpu_threads or cpu_threads(host_cpu())
            cb = cpu_baseline(ctx, nR, nS, threads, args.verbose)
            out["cpu_baseline"] = {k: cb[k] for k in ("value", "unit", "cores", "kind", "sample")}
            out["cpu_legs"] = cb["legs"]
            out["cpu_host"] = cb["host"]
            out["cpu_matches_gpu"] = all(m == int(matches) for m in cb["matches"].values())
        print(json.dumps(out), file=json_out, flush=True)
    ctx.close()
    if exchange:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
