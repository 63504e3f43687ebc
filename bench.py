#!/usr/bin/env python3
"""Benchmark: batched KKT Newton-steps/sec of the parallel-in-time IPM hot path on MI355X.

Metric (BASELINE.json): "KKT Newton-steps/sec at (horizon N x batch)".  One step = one batched
KKT solve (paroc.par_bwd_pass + par_fwd_pass replacement, noc_kkt_solve) of cart-pole
trajectories with horizon N = 200, the LQ blocks being the real first Newton iterate (bp = 0.1)
produced on the device by the linearisation kernels, resident in HBM before timing.

Scaling (north_star: "cartpole N=200 batch=4096 at 1, 2, 4 and 8 GPUs"): by default the GLOBAL
batch of 4096 trajectories (BASELINE config c3) is split over the ranks with
noc.distributed.shard_bounds (strong scaling; at --gpus 1 this is c3 itself).  --batch B instead
gives every rank B trajectories (weak scaling; c5 = --batch 8192 on 8 GPUs).  No collective on the
data path; one all-reduce(max) of the timing.  value = global trajectories x steps / the slowest
rank's time.  Roofline: the slowest rank's algorithmic bytes per launch / its
launch time vs the 8 TB/s HBM peak.  cpu_baseline: the plain-C restatement of the reference's
sequential Riccati (oracle/kkt_ref.c, OpenMP) on a bounded sample of the same blocks, rank 0,
N=1 only.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--global-batch G | --batch B]
Multi-GPU: `python bench.py --gpus N` starts N ranks itself (torch.distributed.run as a child
process, before any GPU call in the parent, which only relays rank 0's line and exit code); under
an external launcher (`python -m torch.distributed.run --nproc-per-node N bench.py --gpus N`) the
ranks are the launcher's.  --gpus must equal the world size, else the bench refuses to run.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ip-parallel-optimal-control_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
CONFIG_LABEL = {("cartpole", 200, 4096): "BASELINE c3",
                ("pendulum", 100, 1024): "BASELINE c2",
                ("linear8", 512, 16384): "BASELINE c4",
                ("cartpole", 200, 65536): "BASELINE c5 (8192 per GPU on 8 GPUs)"}


def algorithmic_bytes(nx, nu, N, B):
    """read A,B,Q,M,R,ru once + write dx,du once per stage, + P per trajectory."""
    per_stage = 8 * (2 * nx * nx + 2 * nx * nu + nu * nu + nu + nx + nu)
    return B * N * per_stage + B * 8 * nx * nx


def pmc_traffic(path, key):
    """HBM bytes per launch of the KKT kernel from a committed rocprofv3 --pmc summary (JSON written
    by tools/pmc_traffic.py) -- only if it was measured on THIS build of the KKT kernels (its
    source_hash equals the current sources'), else None.  Returns (bytes or None, note)."""
    from noc._lib import source_hash
    try:
        with open(path) as fh:
            d = json.load(fh)
    except Exception as e:
        return None, f"no PMC summary ({e!r})"
    if key not in d:
        return None, f"no PMC pass for {key} in {os.path.relpath(path, ROOT)}"
    raw = d.get(key + "_raw", {})
    cur = source_hash(raw.get("kernel_filter", "kkt_scan"))
    if raw.get("source_hash") != cur:
        return None, (f"stale: {key} was profiled on KKT sources {raw.get('source_hash')}, this "
                      f"build is {cur} (re-run the FETCH_SIZE / WRITE_SIZE passes)")
    return d[key], (f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE of this build ({cur}), "
                    f"{raw.get('correction', '')}")


def cpu_baseline(blocks, sample, seconds=10.0, problem="cartpole"):
    """Time the C restatement of the sequential KKT solve on `sample` trajectories (the same
    blocks, relaid out to the natural layout)."""
    sys.path.insert(0, ROOT)
    from oracle import kkt_ref
    nat = blocks["engine"].natural_blocks()
    nat["reg"] = blocks["reg"]
    host = {k: nat[k][:sample].cpu().numpy() for k in ("A", "B", "Q", "R", "M", "r", "P", "reg")}
    del nat
    cores = len(os.sched_getaffinity(0))
    cores = min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)))
    ref = kkt_ref.solve(*(host[k] for k in ("A", "B", "Q", "R", "M", "r", "P", "reg")),
                        threads=cores)
    reps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        kkt_ref.solve(*(host[k] for k in ("A", "B", "Q", "R", "M", "r", "P", "reg")), threads=cores)
        reps += 1
    dt = time.perf_counter() - t0
    # the survey's 1-core figure: same sample, one thread, a quarter of the time
    reps1, t1 = 0, time.perf_counter()
    while time.perf_counter() - t1 < seconds / 4:
        kkt_ref.solve(*(host[k] for k in ("A", "B", "Q", "R", "M", "r", "P", "reg")), threads=1)
        reps1 += 1
    dt1 = time.perf_counter() - t1
    return dict(value=reps * sample / dt, unit="trajectory-KKT-steps/s", cores=cores, kind="port",
                value_1core=reps1 * sample / dt1,
                sample=f"{sample} {problem} trajectories x N={host['A'].shape[1]}, {reps} repeats "
                       f"({dt:.1f} s) of the OpenMP C sequential Riccati (oracle/kkt_ref.c); "
                       f"value_1core: {reps1} repeats ({dt1:.1f} s) on one thread"), ref


def residual_vs_seq_ref(out, ref, sample):
    """BASELINE metric's 'fp64 residual vs seq ref': max relative deviation of the GPU step from
    the sequential-Riccati restatement (oracle/kkt_ref.c) on the sampled trajectories."""
    import numpy as np
    res = {}
    for k in ("dx", "du", "pred"):
        got = getattr(out, k)[:sample].double().cpu().numpy()
        want = ref[k]
        res[k] = float(np.max(np.abs(got - want)) / max(1.0, float(np.max(np.abs(want)))))
    res["feasible_equal"] = bool(np.array_equal(out.feasible[:sample].cpu().numpy(),
                                                ref["feasible"]))
    res["max"] = max(res["dx"], res["du"], res["pred"])
    res["tolerance"] = 1e-10
    res["sample"] = sample
    return res


def allreduce(vals, op="sum"):
    """All-reduce of a few fp64 scalars over the bench's process group (RCCL on the GPUs; the
    gloo rehearsal mode reduces on the host)."""
    import torch
    import torch.distributed as dist
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([float(v) for v in vals], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
    return t.tolist()


def ipm_solve_rate(problem, N, B, rank, world, G, lo, seed=11):
    """End-to-end: the whole interior-point solve (P:228-254) of this rank's B trajectories with
    the persistent kernel (noc_ipm_solve, one launch), timed with HIP events; over ranks the wall
    time is the max and the solve counts are summed.  Reported beside the KKT metric:
    kkt_solves_per_s = KKT solves actually COMPUTED / wall time (the identical retries at the rp
    clip that are accounted without recomputation, ws.repeats, are excluded;
    kkt_solves_reference_equivalent_per_s counts them as the reference would).  The rank solves
    trajectories lo..lo+B-1 of ONE global batch of G (shard_initial_conditions), so the summed
    counts of N ranks are those of the 1-rank solve of the same G trajectories."""
    import torch
    import torch.distributed as dist
    from noc import problems
    from noc import _lib
    from noc.ipm import BatchedIPM, persistent_supported
    ocp = problems.make_problem(problem, N)
    if not persistent_supported(ocp.family, N):
        # c4 (linear8) is LQ-only in the reference (LM:64-84: par_bwd_pass / par_fwd_pass, no
        # interior-point loop), so its KKT line is already the end-to-end step
        return {"skipped": "no persistent instance for this family / horizon (c4 is LQ-only in "
                           "the reference: one KKT solve per MPC step, LM:67-84)"}
    x0, u0 = problems.shard_initial_conditions(problem, N, G, lo, lo + B, seed=seed)
    eng = BatchedIPM(ocp.family, N, B, persistent=True)
    eng.load(u0, x0)
    eng.solve(max_steps=eng.PROBE_SOLVES + 8)  # warm-up: both launches of the probe schedule (their kernels loaded)

    def timed(flags, schedule="auto"):
        eng.load(u0, x0)
        eng.ws.flags = flags
        torch.cuda.synchronize()
        if pg():
            dist.barrier()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        eng.solve_persistent(schedule=schedule)  # incl. the probe launch / launch-order pass
        ev1.record()
        torch.cuda.synchronize()
        eng.ws.flags = 0
        return ev0.elapsed_time(ev1)

    # every retry recomputed (NOC_WS_NO_REPEAT_SKIP), then the default: the identical retries at
    # the rp clip accounted without recomputation -- bit-identical results, checked here
    ms_all = timed(_lib.WS_NO_REPEAT_SKIP)
    U_all = eng.t["u"].clone()
    ms_index = timed(0, "index")
    # the schedule "auto" replaces when the batch exceeds the resident waves (else not timed)
    beyond = B > eng._resident_slots()
    ms_cost = timed(0, "cost") if beyond else -1.0
    U_cost = eng.t["u"].clone()
    ms = timed(0)
    identical = bool(torch.equal(U_all, eng.t["u"])) and bool(torch.equal(U_cost, eng.t["u"]))
    U, its, solves = (t.cpu() for t in eng.result())
    reps = eng.t["repeats"].cpu()
    done = int((eng.t["phase"] == 3).sum().item())
    tot = [float(solves.sum()), float(done), float(its.double().sum()), float(B),
           float(reps.sum()), float(not identical)]
    mx = [ms, float(solves.max()), ms_all, ms_index, ms_cost]
    if pg():
        tot = allreduce(tot, "sum")
        mx = allreduce(mx, "max")
    computed = tot[0] - tot[4]
    return {"what": "whole barrier schedule, noc_ipm_solve (one wave per trajectory, one launch "
                    "per rank)",
            "trajectories": int(tot[3]), "wall_ms": mx[0], "kkt_solves": int(tot[0]),
            "kkt_solves_per_s": computed / (mx[0] * 1e-3),
            "kkt_solves_computed": int(computed),
            "kkt_solves_reference_equivalent_per_s": tot[0] / (mx[0] * 1e-3),
            "repeats_accounted": int(tot[4]),
            "wall_ms_recompute_all": mx[2],
            "wall_ms_index_order": mx[3],
            "wall_ms_initial_cost_order": mx[4] if mx[4] >= 0 else None,
            "schedule": "when the batch exceeds the resident waves: a probe launch of every "
                        "trajectory's first BatchedIPM.PROBE_SOLVES KKT solves, then the rest "
                        "resumed by descending total cost (timed inside wall_ms)",
            "bit_identical_to_recompute_all": tot[5] == 0,
            "mean_newton_iters": tot[2] / max(tot[3], 1.0), "max_kkt_solves": int(mx[1]),
            "converged": int(tot[1])}


BENCH_SEED = 1234  # the global batch's seed (the same on every rank)


def pg():
    """True when this run has a process group (launched ranks): barriers and max / sum / gather
    over the ranks go through it."""
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized()


def parse_slice(text):
    """--slice r/W -> (r, W)"""
    try:
        r, w = (int(v) for v in text.split("/"))
    except ValueError:
        sys.exit(f"bench.py: --slice wants r/W (e.g. 3/8), got {text!r}")
    if not (w >= 1 and 0 <= r < w):
        sys.exit(f"bench.py: --slice {text}: need 0 <= r < W")
    return r, w


def rank_shard(args, world, rank):
    """(B, G, lo, scaling): this rank's trajectories lo..lo+B-1 of the global batch G.  Strong
    scaling (default): G = --global-batch split by noc.distributed.shard_bounds; weak (--batch B):
    G = B x world, rank r owning [rB, (r+1)B).  --slice r/W (one process, no process group): what
    rank r of a W-rank strong-scaling run solves, on this one GPU -- the per-GPU work of the
    north-star curve's W-GPU point, measured slice by slice (tools/slice_curve.py)."""
    if getattr(args, "slice", None):
        from noc.distributed import shard_bounds
        r, w = parse_slice(args.slice)
        lo, hi = shard_bounds(args.global_batch, w, r)
        return hi - lo, args.global_batch, lo, f"slice {r}/{w} of a strong-scaling run"
    if args.batch is not None:
        return args.batch, args.batch * world, rank * args.batch, "weak"
    from noc.distributed import shard_bounds
    lo, hi = shard_bounds(args.global_batch, world, rank)
    return hi - lo, args.global_batch, lo, "strong"


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(n, argv):
    """`bench.py --gpus n` without a launcher: start n ranks (one process per GPU) with
    torch.distributed.run as a CHILD process -- the parent has touched no GPU -- and return its
    exit code.  Rank 0 prints the JSON line straight to the inherited stdout."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}",
           os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def dry_run_line(args, world, rank):
    """NOC_BENCH_DRYRUN=1 (CPU tests): the launcher, process group, max-over-ranks timing and the
    JSON assembly, with no GPU work -- value is null, so it can never pass for a measurement."""
    import torch.distributed as dist
    from noc import problems
    B, G, lo, scaling = rank_shard(args, world, rank)
    x0, u0 = problems.shard_initial_conditions(args.problem, args.horizon, G, lo, lo + B,
                                               seed=BENCH_SEED)
    dump = os.environ.get("NOC_BENCH_DRYRUN_DUMP")
    if dump:  # this rank's inputs, for the CPU test that they are a slice of the 1-rank inputs
        import numpy as np
        np.savez(os.path.join(dump, f"rank{rank}_of{world}.npz"), x0=x0, u0=u0, lo=lo, G=G)
    if pg():
        dist.barrier()
    t = [0.0]
    if pg():
        t = allreduce(t, "max")
        ranks = allgather_float(float(rank))
    else:
        ranks = [0.0]
    return {"metric": "KKT Newton-steps/sec at (horizon N x batch)", "value": None,
            "unit": "trajectory-KKT-steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": None, "higher_is_better": True,
            "dry_run": True, "data": "dry run: no GPU work (launcher / process-group rehearsal)",
            "rccl_world_size": world, "ranks_seen": [int(r) for r in ranks],
            "scaling": scaling, "config": {"global_batch": G, "batch_per_gpu": B}}


def allgather_float(v):
    """One fp64 scalar from every rank, in rank order (per-rank kernel times in the line)."""
    import torch
    import torch.distributed as dist
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([float(v)], dtype=torch.float64, device=dev)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [float(o.item()) for o in out]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--problem", default="cartpole")
    ap.add_argument("--horizon", type=int, default=200)
    ap.add_argument("--global-batch", type=int, default=4096,
                    help="total trajectories, split over the ranks (strong scaling; default c3)")
    ap.add_argument("--batch", type=int, default=None,
                    help="trajectories per GPU instead (weak scaling)")
    ap.add_argument("--slice", default=None,
                    help="r/W: solve only rank r's shard of a W-rank strong-scaling run, on one "
                         "GPU without a process group (value then counts the slice only)")
    ap.add_argument("--lanes", type=int, default=0)
    ap.add_argument("--layout", choices=["tiled", "natural"], default="tiled",
                    help="HBM layout of the LQ blocks (tiled = what the linearisation kernels write)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-sample", type=int, default=512)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-ipm", action="store_true", help="skip the end-to-end solve line")
    ap.add_argument("--no-graph", action="store_true",
                    help="launch every step from Python instead of replaying a HIP graph of the "
                         "K timed steps (small configs then measure the host's launch rate)")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    args = ap.parse_args()
    if args.gpus < 1:
        sys.exit(f"bench.py: --gpus must be >= 1 (got {args.gpus})")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher: become one (nothing has touched the GPU in this process)
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.slice and (args.gpus != 1 or args.batch is not None):
        sys.exit("bench.py: --slice runs one process on one GPU (--gpus 1) of the strong-scaling "
                 "global batch (no --batch)")
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} "
                 f"ranks; refusing to report a line whose n_gpus would not be what was asked")

    import torch
    import torch.distributed as dist
    # NOC_BENCH_REHEARSAL=1: every rank on cuda:0 over gloo -- rehearses the N > 1 code path on a
    # one-GPU box (timings then share one GPU and mean nothing).  NOC_BENCH_DRYRUN=1: no GPU at all
    # (CPU tests of the launcher / process group / JSON line; value null).
    rehearsal = os.environ.get("NOC_BENCH_REHEARSAL") == "1"
    dry = os.environ.get("NOC_BENCH_DRYRUN") == "1"
    if rehearsal:
        local = 0
    if not dry:
        torch.cuda.set_device(local)
    # a process group whenever a launcher started this process (world 1 included: the RCCL
    # init / barrier / all-reduce / all-gather then run on the hardware even on one GPU)
    if world > 1 or "WORLD_SIZE" in os.environ:
        if rehearsal or dry:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    if dry:
        line = dry_run_line(args, world, rank)
        if rank == 0:
            print(json.dumps(line), flush=True)
        if pg():
            dist.destroy_process_group()
        return
    from noc import lqt, problems, _lib

    N = args.horizon
    B, G, lo, scaling = rank_shard(args, world, rank)
    # lanes 8..64: the parallel-in-time scan on the lane-interleaved layout; lanes 1: the
    # horizon-sequential group solve on the grouped layout (the nx = 8 default).  Either way the
    # blocks are what the device linearisation writes for that solver.  Every rank linearises its
    # slice of ONE global batch (one seed), so N ranks solve exactly the 1-rank problem.
    blocks = problems.make_bench_blocks(args.problem, N=N, batch=B, seed=BENCH_SEED,
                                        lanes=args.lanes, natural=(args.layout == "natural"),
                                        shard=(G, lo))
    tb = blocks["tiled"]
    nx, nu, lanes = tb.nx, tb.nu, tb.lanes
    if args.layout == "tiled":
        out = lqt.kkt_solve_tiled(tb, reg=blocks["reg"], want_gains=False)

        def step():
            lqt.kkt_solve_tiled(tb, reg=blocks["reg"], out=out)
    else:
        nat = [blocks[k] for k in ("A", "B", "Q", "R", "M", "r", "P")]
        out = lqt.kkt_solve(*nat, reg=blocks["reg"], lanes=lanes, want_gains=False)

        def step():
            lqt.kkt_solve(*nat, reg=blocks["reg"], lanes=lanes, out=out)

    # The K timed steps are one HIP graph (captured once, replayed once): a c2-sized launch runs
    # ~10 us, less than a Python + ctypes launch takes on the host, so eager launches would time
    # the host.  The graph holds exactly K kernel launches on the same buffers.
    graph = None
    if not args.no_graph:
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            step()  # allocator / library warm-up on the capture stream
        torch.cuda.current_stream().wait_stream(side)
        g1, graph = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(g1):
            step()
        with torch.cuda.graph(graph):
            for _ in range(args.steps):
                step()
    for _ in range(args.warmup):
        if graph is not None:
            g1.replay()
        else:
            step()
    torch.cuda.synchronize()
    if pg():
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    if graph is not None:
        graph.replay()
    else:
        for _ in range(args.steps):
            step()
    ev1.record()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    if pg():
        dist.barrier()
    torch.cuda.synchronize()
    kern_ms = ev0.elapsed_time(ev1) / args.steps          # HIP-event time per launch (stream)
    ms = wall * 1e3 / args.steps
    rank_kern_ms = [kern_ms]
    if pg():
        rank_kern_ms = allgather_float(kern_ms)
        ms, kern_ms = allreduce([ms, kern_ms], "max")
    feasible_frac = float(out.feasible.float().mean())
    # trajectories this run solved per step: the global batch (every rank's shard), or one slice
    solved = B if args.slice else G
    value = solved * args.steps / (ms * args.steps / 1e3)
    abytes = algorithmic_bytes(nx, nu, N, B)
    if pg():  # the slowest rank's bytes (shards differ by at most one trajectory)
        abytes = int(allreduce([abytes], "max")[0])
    achieved = abytes / (kern_ms * 1e-3) / 1e9
    traffic, traffic_note = pmc_traffic(args.pmc_json, f"{args.problem}_N{N}_B{B}")
    # what limits the launch below the HBM roofline (DESIGN.md §3.1 stamps): with at most one
    # wave per SIMD the per-wave dependent chain (combine levels, load latency) sets the time;
    # above it the blocks' three passes (one from HBM, two from the memory-side cache)
    simds = 4 * torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
    waves = -(-B * lanes // 64) if lanes >= 8 else -(-B // 8)
    if lanes < 8:
        limiter = "hbm: two sweeps (blocks + gains), group solve"
    elif waves <= simds:
        limiter = (f"latency: {waves / simds:.2f} waves per SIMD, the per-wave chain of combine "
                   "levels and load latencies, not bytes")
    else:
        limiter = (f"memory: {waves / simds:.2f} waves per SIMD; one HBM pass over the blocks and "
                   "two re-reads served by the memory-side cache")
    result = {
        "metric": "KKT Newton-steps/sec at (horizon N x batch)",
        "value": value,
        "unit": "trajectory-KKT-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms,
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "f64",
        "data": f"synthetic: first Newton iterate (bp=0.1) of random-start {args.problem} "
                "problems, linearised on device",
        "config": {"workload": f"{args.problem} nx={nx} nu={nu} N={N} global batch={G} "
                               f"({CONFIG_LABEL.get((args.problem, N, G), 'custom')}), "
                               f"{B} per GPU",
                   "layout": args.layout,
                   "horizon": N, "batch_per_gpu": B, "global_batch": G,
                   "lanes_per_trajectory": lanes, "parallelism": f"trajectory-sharded x{world}"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_note": traffic_note,
                     "algorithmic_bytes_per_launch": abytes, "kernel_ms": kern_ms,
                     "limiter": limiter},
        "rccl_world_size": dist.get_world_size() if pg() else 1,
        "process_group": (dist.get_backend() if pg() else None),
        "per_rank_kernel_ms": rank_kern_ms,
        "feasible_fraction": feasible_frac,
        "launch": "eager" if graph is None else "hip_graph (the K timed steps captured once, one replay)",
        "build_hash": _lib.load().noc_build_hash().decode(),  # == the tree's (checked by load())
    }
    if args.slice:
        result["config"]["slice"] = args.slice
        result["config"]["slice_trajectories"] = [lo, lo + B]
    if not args.no_ipm:
        result["ipm_solve"] = ipm_solve_rate(args.problem, N, B, rank, world, G, lo)
    if rank == 0 and world == 1 and not args.no_cpu:
        try:
            sample = min(args.cpu_sample, B)
            result["cpu_baseline"], ref = cpu_baseline(blocks, sample, args.cpu_seconds,
                                                             args.problem)
            result["residual_vs_seq_ref"] = residual_vs_seq_ref(out, ref, sample)
        except Exception as e:  # reported, never fatal
            result["cpu_baseline"] = {"value": None, "error": repr(e)}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if pg():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
