"""bench.py -- pod-node pair scores/s and placements/s of the MI355X placement
engine on BASELINE.json's headline workload:

  synthetic 10k nodes x 100k pending pods, dense int8 latency matrix and
  pod->node traffic (rack/zone locality, 8 bound peers per pod), clusterloader2-
  shaped requests -- all generated in HBM before the timed region.

One step = one full placement pass: resource-fit filter over all pod x node
pairs, the WA x L contraction on MFMA with the fused top-4 epilogue, the
per-pod merge (+ RCCL all-gather across node shards when N > 1), and the
greedy commit with capacity update; the placements and integer scores are
copied back to the host.  The reference-mode vote scorer (scheduler.go:248-394
on one fresh 10k-node snapshot per pod, 48 GB) is timed too and reported under
"reference_mode".

  python bench.py [--gpus N] [--steps K] [--warmup W]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

`--gpus N > 1` without a launcher (no WORLD_SIZE in the environment) starts
the N rank processes itself (launch_ranks: RANK / LOCAL_RANK / WORLD_SIZE and
a file:// rendezvous per child, before this process touches the GPU) and
relays rank 0's line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_I8_TOPS = 5033.2     # dense int8 MFMA, 256 CU x 4 SIMD x 2048 op/clk x 2.4 GHz
PEAK_BF16_TFLOPS = 2516.6  # dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0      # HBM3E spec (MI355X_MICROARCH.md)
SEED = 0x4E4153


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--nodes", type=int, default=10000)
    ap.add_argument("--pods", type=int, default=100000)
    ap.add_argument("--dtype", default="i8", choices=["i8", "bf16"])
    ap.add_argument("--peers", type=int, default=8)
    ap.add_argument("--no-reference-mode", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget-s", type=float, default=20.0)
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the other BASELINE configs (C1/C2/C5/C4 lines under 'configs', "
                         "one GPU only)")
    ap.add_argument("--c4", action="store_true",
                    help="run C4 (50k nodes x 500k pods, node-sharded) also when --gpus > 1")
    ap.add_argument("--rccl-world1", action="store_true",
                    help="diagnostic: at --gpus 1 place through a one-rank RCCL communicator "
                         "(every chunk's all-gather + cross-rank merge runs)")
    ap.add_argument("--vote-node-shard", action="store_true",
                    help="reference mode with the node axis sharded over the ranks (partial "
                         "records all-gathered over RCCL) instead of pods split across ranks")
    ap.add_argument("--rehearse-world", type=int, default=0,
                    help="diagnostic at --gpus 1: time rank 0 of a G-GPU node-sharded pass "
                         "(its node columns; the other ranks' lists are shifted copies of its "
                         "own; placements not meaningful, RCCL over a one-rank communicator)")
    ap.add_argument("--commit-cus", type=int, default=None,
                    help="NAS_OPT_COMMIT_CUS for the headline pass (world 1): CUs per XCD kept "
                         "for the commit stream (default: the engine's)")
    ap.add_argument("--synth-profile", type=int, default=0, choices=[0, 1],
                    help="generator of the C3 inputs (NAS_OPT_SYNTH_PROFILE): 0 racks / zones "
                         "with bound peers (default), 1 uniform over the full int8 range "
                         "(SURVEY.md §8(d)'s operand distribution; configs.C3_fullrange)")
    ap.add_argument("--only", choices=["place", "vote", "score", "pmc", "C1", "C2", "C2_f32",
                                       "C3_bf16", "C3_fullrange", "C5", "C4", "C4_shardG2"],
                    default=None,
                    help="profile helper: run only one path (pmc: the score and vote legs, "
                         "what the in-run PMC passes profile)")
    ap.add_argument("--no-pmc", action="store_true",
                    help="skip the in-run rocprofv3 PMC passes (roofline.traffic then null)")
    return ap.parse_args()


def _cgroup_cpus():
    """CPU quota of this process's cgroup in CPUs (cgroup v2 cpu.max, else v1
    cfs quota / period), or None when unlimited / unknown."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = float(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = float(f.read())
        return None if q <= 0 else q / per
    except (OSError, ValueError):
        return None


def cpu_info():
    """Host CPU model and the cores this process may use (for the CPU
    baselines).  `affinity` is what sched_getaffinity shows -- the whole
    machine on the GPU pool's boxes --, `usable` the box's CPU share the
    baselines run on: OMP_NUM_THREADS as the pool exports it (16 per GPU), else
    the cgroup CPU quota, else the affinity count."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count()
    quota = _cgroup_cpus()
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or None
    if omp:
        usable, why = min(omp, affinity), (
            "OMP_NUM_THREADS (the box's CPU share as the GPU pool exports it: 16 CPUs per GPU "
            "of a machine whose affinity mask shows all of its cores; worker pools are sized to "
            "that share, and threads past it only contend with the other GPUs' jobs)")
    elif quota:
        usable, why = max(1, min(int(quota), affinity)), "cgroup CPU quota"
    else:
        usable, why = affinity, "sched_getaffinity (no quota, no OMP_NUM_THREADS)"
    return {"model": model, "nproc": os.cpu_count(), "affinity": affinity,
            "cgroup_quota_cpus": quota, "omp_num_threads": omp, "usable": usable,
            "usable_source": why}


def host_threads():
    """Threads for the pods-parallel CPU baselines: every usable core."""
    return cpu_info()["usable"] or 1


def pmc_traffic(args, profile=0):
    """HBM-side bytes per launch of the dominant kernels, measured in this run:
    two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE: they do not fit one
    pass on gfx950) over a child `bench.py --only pmc` of the same workload,
    FETCH_SIZE doubled per MI355X_MICROARCH.md's gfx950 note.  Runs BEFORE this
    process touches the GPU (the child is a separate process).  Returns
    {kernel: {"fetch": B, "write": B, "bytes": B}} or {} (with the reason)."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return {}, "rocprofv3 not found"
    child = [sys.executable, os.path.abspath(__file__), "--only", "pmc", "--steps", "1",
             "--warmup", "0", "--no-pmc", "--nodes", str(args.nodes), "--pods", str(args.pods),
             "--dtype", args.dtype, "--peers", str(args.peers), "--synth-profile", str(profile)]
    if profile != args.synth_profile:  # (a config line's inputs: the score leg only)
        child.append("--no-reference-mode")
    out = {}
    tmp = tempfile.mkdtemp(prefix="nas_pmc_", dir="/tmp")
    env = dict(os.environ, TMPDIR="/tmp")
    try:
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(tmp, ctr)
            r = subprocess.run(["timeout", "-s", "KILL", "150", prof, "--pmc", ctr,
                                "--output-format", "csv", "-d", d, "-o", "p", "--"] + child,
                               cwd="/tmp", env=env, stdout=subprocess.DEVNULL,
                               stderr=subprocess.DEVNULL)
            if r.returncode != 0:
                return {}, f"rocprofv3 --pmc {ctr} exited {r.returncode}"
            per = {}
            for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
                with open(f) as fh:
                    for row in csv.DictReader(fh):
                        if row["Counter_Name"] != ctr:
                            continue
                        k = row["Kernel_Name"].replace("(anonymous namespace)", "").split("(")[0]
                        k = k.split("<")[0].split("::")[-1].replace("void ", "").strip()
                        key = (k, row["Dispatch_Id"])
                        per[key] = per.get(key, 0.0) + float(row["Counter_Value"])
            mult = 2.0 if ctr == "FETCH_SIZE" else 1.0
            for (k, _), kb in per.items():
                rec = out.setdefault(k, {})
                name = "fetch" if ctr == "FETCH_SIZE" else "write"
                rec[name] = max(rec.get(name, 0.0), kb * 1024.0 * mult)  # the largest dispatch
        for rec in out.values():
            rec["bytes"] = rec.get("fetch", 0.0) + rec.get("write", 0.0)
        return out, None
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def visible_gpus():
    """GPUs this process could use, counted without initialising the GPU
    (torch.cuda.device_count does not, on this image); 0 without torch / GPUs."""
    try:
        import torch
        return int(torch.cuda.device_count())
    except Exception:  # noqa: BLE001 -- no torch / no runtime: the CPU rank logic
        return 0


def launch_ranks(child_argv, n, ndev, timeout_s=None, extra_env=None):
    """Start n rank processes of `child_argv` (one per GPU: LOCAL_RANK = r mod
    ndev, so more ranks than GPUs share them -- RCCL then refuses and bench.py
    falls back to its host exchange) with RANK / LOCAL_RANK / WORLD_SIZE and a
    file:// gloo rendezvous (NAS_DIST_INIT: no TCP port to collide).  Wait for
    all of them; as soon as one exits non-zero (or the deadline passes) kill
    the others, so no rank is left waiting for a dead peer; always reap.
    Rank 0's stdout goes to a file (bench.py prints its one JSON line there);
    every rank's stderr is inherited.  Returns (rc, rank 0's stdout): rc is
    the first failing rank's exit code (128 + signal for a signal), else 0."""
    import shutil
    import subprocess
    import tempfile
    tmp = tempfile.mkdtemp(prefix="nas_ranks_", dir="/tmp")
    out0 = os.path.join(tmp, "rank0.out")
    procs, failed = [], None

    def die_with_parent():
        # a rank must not outlive this launcher (a driver that kills it on a
        # deadline would otherwise leave the ranks on the GPUs): SIGKILL on
        # the parent's death (Linux PR_SET_PDEATHSIG)
        try:
            import ctypes
            ctypes.CDLL(None).prctl(1, 9)
        except Exception:  # noqa: BLE001 -- best effort off Linux
            pass
    try:
        with open(out0, "w") as f0:
            for r in range(n):
                env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r % ndev if ndev else r),
                           WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0",
                           NAS_DIST_INIT="file://" + os.path.join(tmp, "rdv"),
                           MASTER_ADDR="127.0.0.1", **(extra_env or {}))
                procs.append(subprocess.Popen(child_argv, env=env, preexec_fn=die_with_parent,
                                              stdout=f0 if r == 0 else subprocess.DEVNULL))
            deadline = None if timeout_s is None else time.monotonic() + timeout_s
            rcs = [None] * n
            while any(rc is None for rc in rcs):
                for i, p in enumerate(procs):
                    if rcs[i] is None:
                        rcs[i] = p.poll()
                        if rcs[i] not in (None, 0) and failed is None:
                            failed = rcs[i]
                if failed is not None:
                    break
                if deadline is not None and time.monotonic() > deadline:
                    failed = 124
                    print(f"launch_ranks: deadline of {timeout_s} s passed", file=sys.stderr)
                    break
                time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
            p.wait()
        text = open(out0).read() if os.path.exists(out0) else ""
        shutil.rmtree(tmp, ignore_errors=True)
    if failed is not None and failed < 0:
        failed = 128 - failed
    return (failed or 0), text


def self_launch(args):
    """`bench.py --gpus N` (N > 1) with no launcher: N rank processes of this
    same command line, one per GPU (launch_ranks), started before this process
    makes any GPU call; rank 0's JSON line is relayed on stdout (with
    config.launcher saying so) and the exit code is the first failing rank's."""
    ndev = visible_gpus()
    print(f"bench.py: no WORLD_SIZE in the environment; starting {args.gpus} rank processes "
          f"({ndev} GPU(s) visible, file:// rendezvous)", file=sys.stderr, flush=True)
    rc, text = launch_ranks([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], args.gpus,
                            ndev)
    lines = [ln for ln in text.splitlines() if ln.startswith("{")]
    if lines:
        out = json.loads(lines[-1])
        out.setdefault("config", {})["launcher"] = (
            f"bench.py self-launch: {args.gpus} rank processes on {ndev} visible GPU(s), "
            f"gloo file:// rendezvous")
        print(json.dumps(out), flush=True)
    elif rc == 0:
        print("bench.py: rank 0 printed no result line", file=sys.stderr)
        rc = 1
    return rc


class Dist:
    def __init__(self, gpus):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        if self.world != gpus:
            raise SystemExit(f"--gpus {gpus} but WORLD_SIZE={self.world}")
        self.pg = None
        import torch
        self.torch = torch
        if self.world > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            # torchrun's env:// store by default; NAS_DIST_INIT (e.g. a file://
            # rendezvous, as the CPU tests use) replaces it
            init = os.environ.get("NAS_DIST_INIT", "env://")
            dist.init_process_group("gloo", init_method=init, rank=self.rank,
                                    world_size=self.world)
            self.dist = dist
        # (no GPU: the rank logic alone, as the CPU gloo tests run it)
        self.gpu = torch.cuda.is_available()
        if self.gpu:
            torch.cuda.set_device(self.local)

    def barrier_sync(self):
        if self.gpu:
            self.torch.cuda.synchronize()
        if self.world > 1:
            self.dist.barrier()
        if self.gpu:
            self.torch.cuda.synchronize()

    def max(self, x):
        if self.world == 1:
            return x
        t = self.torch.tensor([x], dtype=self.torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def bcast_bytes(self, b):
        if self.world == 1:
            return b
        obj = [b]
        self.dist.broadcast_object_list(obj, src=0)
        return obj[0]


def agree(d, ok):
    """True only if `ok` holds on every rank (gloo MIN); every rank must call."""
    if d.world == 1:
        return ok
    t = d.torch.tensor([1 if ok else 0], dtype=d.torch.int64)
    d.dist.all_reduce(t, op=d.dist.ReduceOp.MIN)
    return bool(t.item())


def host_all_gather(d):
    """sharded.place_dist_shard's exchange over the gloo process group: every
    rank's (keys, bounds) in rank order."""
    torch = d.torch

    def ag(keys, bounds):
        k = torch.from_numpy(np.ascontiguousarray(keys).view(np.int64))
        b = torch.from_numpy(np.ascontiguousarray(bounds).view(np.int64))
        ks = [torch.empty_like(k) for _ in range(d.world)]
        bs = [torch.empty_like(b) for _ in range(d.world)]
        d.dist.all_gather(ks, k)
        d.dist.all_gather(bs, b)
        return [(x.numpy().view(np.uint64), y.numpy().view(np.uint64)) for x, y in zip(ks, bs)]
    return ag


def time_steps(d, fn, steps, warmup):
    for _ in range(warmup):
        fn()
    d.barrier_sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    d.barrier_sync()
    return d.max(time.perf_counter() - t0)


def bench_place(args, d, eng):
    """Returns (elapsed, per-stage times, placements, the engine to use from
    here on, how the node shards exchange their lists)."""
    N, P = args.nodes, args.pods
    if args.rehearse_world > 1:
        assert d.world == 1, "--rehearse-world runs on one GPU"
        eng.set_option("REHEARSE_WORLD", args.rehearse_world)  # diagnostic option
    exchange = None
    if d.world > 1 or args.rccl_world1 or args.rehearse_world > 1:
        exchange = "rccl all-gather (nas_comm_init)"
        err = None
        try:
            eng.set_option("COMM_TIMEOUT_MS", 60000)
            uid = d.bcast_bytes(eng.comm_unique_id() if d.rank == 0 else None)
            eng.comm_init(uid, d.rank, d.world)
            eng.synth_cluster(SEED, N, P, args.dtype, peers=args.peers, profile=args.synth_profile)
            if args.rehearse_world > 1:
                # the stand-in lists repeat this rank's few best nodes G times,
                # so herds would drain them at once; with 64x capacity no list
                # runs dry and the pass times scoring + exchange + merge + the
                # full commit walk
                eng.upload_capacity(np.minimum(eng.get_capacity().astype(np.int64) * 64,
                                               2**31 - 1).astype(np.int32))
            eng.reset_capacity()
            eng.place()  # first collectives (connection setup) inside the deadline
        except Exception as e:  # noqa: BLE001 -- decided together below
            err = repr(e)[:300]
        if not agree(d, err is None):
            if d.world == 1:
                raise RuntimeError(f"RCCL path failed: {err}")
            # RCCL unusable on this node: the same kernels on the same node
            # shards, candidate lists exchanged through the host over gloo
            # (sharded.place_dist_shard) -- slower, reported as such
            print(f"rank {d.rank}: RCCL path failed ({err or 'on another rank'}); "
                  "host exchange over gloo", file=sys.stderr, flush=True)
            eng.close()
            from kubernetesnetawarescheduler_amd import Engine
            eng = Engine(d.local)
            eng.set_shard(d.rank, d.world)
            exchange = f"host gloo all-gather (RCCL failed: {err or 'on another rank'})"
            eng.synth_cluster(SEED, N, P, args.dtype, peers=args.peers, profile=args.synth_profile)
            return bench_place_host(args, d, eng) + (eng, exchange)
    else:
        eng.synth_cluster(SEED, N, P, args.dtype, peers=args.peers, profile=args.synth_profile)
    if args.commit_cus is not None:
        eng.set_option("COMMIT_CUS", args.commit_cus)
    keys = ("cost_ms", "fit_ms", "merge_ms", "commit_ms", "total_ms", "cost_launches",
            "rescore_rounds", "unschedulable")
    acc = dict.fromkeys(keys, 0.0)
    state = {"node": None}
    # placements and integer scores come back every step (into reused arrays)
    outs = (np.empty(P, np.int32), None, np.empty(P, np.int64))

    def step():
        eng.reset_capacity()
        node, _, score = eng.place(out=outs)
        t = eng.timings()
        for k in keys:
            acc[k] += t[k]
        state["node"] = node

    for _ in range(args.warmup):
        step()
    for k in keys:
        acc[k] = 0.0
    # timed steps record only the events the pass synchronises on; the
    # per-stage device times come from separate steps with stage timings on
    eng.set_option("STAGE_TIMINGS", 0)
    elapsed = time_steps(d, step, args.steps, 0)
    eng.set_option("STAGE_TIMINGS", 1)
    per = {k: v / args.steps for k, v in acc.items()}
    for k in keys:
        acc[k] = 0.0
    n_stage = 3
    for _ in range(n_stage):
        step()
    per.update({k: acc[k] / n_stage for k in ("cost_ms", "fit_ms", "merge_ms", "commit_ms",
                                                "total_ms")})
    return elapsed, per, state["node"], eng, exchange


def bench_place_host(args, d, eng):
    """The placement pass with the node shards' lists exchanged through the
    host (fallback when RCCL is unusable): score, gloo all-gather, merge,
    replicated commit, rescore windows -- sharded.place_dist_shard."""
    from kubernetesnetawarescheduler_amd import sharded
    P = args.pods
    ag = host_all_gather(d)
    state = {"node": None, "rounds": 0}

    def step():
        eng.reset_capacity()
        node, _, rounds = sharded.place_dist_shard(eng, P, ag)
        state["node"], state["rounds"] = node, rounds

    elapsed = time_steps(d, step, args.steps, args.warmup)
    per = {"cost_ms": 0.0, "fit_ms": 0.0, "merge_ms": 0.0, "commit_ms": 0.0, "total_ms": 0.0,
           "rescore_rounds": float(state["rounds"]),
           "unschedulable": float((state["node"] < 0).sum())}
    return elapsed, per, state["node"]


def bench_cost_kernel(args, d, eng):
    """Roofline of the dominant kernel: one full-size scoring pass (fit + one
    k_cost_topk launch over all pods + merge) on one stream, HIP events
    around the k_cost_topk launch."""
    eng.reset_capacity()
    eng.score()  # warm-up launch (tools/check_roofline.py drops it too)
    ms = []
    for _ in range(max(3, args.steps)):
        eng.score()
        t = eng.timings()
        assert t["cost_launches"] == 1
        ms.append(t["cost_ms"])
    return float(np.mean(ms)), ms


def bench_fit_kernel(args, d, eng, reps=10):
    """Roofline of the resource-fit filter (north star kernel (1)): the
    standalone nas_filter over all pod x node pairs of the workload (one k_fit
    launch, HIP events around it on its stream).  In the placement pass the
    wide cost tile decides the fit itself (k_cost.hip, fused fit); this is the
    filter as its own HBM-bound kernel.  Algorithmic bytes: the mask written
    once (P x ceil(N/64) x 8 B) plus capacities and requests read once."""
    N, P = args.nodes, args.pods
    # the filter covers this context's node shard (a rehearsal's rank 0 holds
    # the first N / G nodes)
    G = args.rehearse_world or d.world
    r = 0 if args.rehearse_world else d.rank
    nloc = (r + 1) * N // G - r * N // G
    eng.reset_capacity()
    eng.filter(want_mask=False)  # warm-up
    ms = []
    for _ in range(reps):
        eng.filter(want_mask=False)
        ms.append(eng.timings()["fit_ms"])
    fit_ms = float(np.mean(ms))
    algo = P * ((nloc + 63) // 64) * 8.0 + 3 * 4.0 * (nloc + P)
    return {"kernel": "k_fit (nas_filter, standalone)", "bound": "hbm",
            "achieved": algo / (fit_ms * 1e-3) / 1e9, "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": algo / (fit_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, "launch_ms": fit_ms,
            "launch_ms_min": min(ms), "launches": reps, "bytes_per_launch": algo,
            "note": "mask write P*ceil(N/64)*8 B + capacities and requests 12*(N+P) B per launch; "
                    "HIP events around the one launch.  The standalone filter only: in the "
                    "world-1 placement pass the wide cost kernel decides the fit itself after "
                    "its main loop (fused fit), so no k_fit launch runs there"}


def vendor_gemm_reference(args, d, reps=5):
    """Known-good ceiling reference for the dominant kernel, measured in this
    run (cdna_hip_programming.md §5.4 rule 10): the vendor library's plain
    GEMM (hipBLASLt through torch._int_mm / torch.matmul) at the shape
    k_cost_topk launches -- Mp x Kp nodes x K, Pp pods, both operands
    K-contiguous -- on operands with the C3 value ranges (latency 1..105,
    traffic 0..2).  The library writes the whole product to HBM (int32 4.1 GB
    at C3); k_cost_topk fuses the fit mask and the top-8 reduction instead.
    `frac` uses the same 2*P*N*N_local op count as the roofline object, so the
    two fractions compare directly.  Not the product path: a measurement aid."""
    import torch
    N, P = args.nodes, args.pods
    nloc = N // max(d.world, args.rehearse_world)
    r = lambda x, m: (x + m - 1) // m * m  # noqa: E731
    M, K, Pp = r(nloc, 256), r(N, 128 if args.dtype == "i8" else 64), r(P, 256)
    dev = torch.device("cuda", d.local)
    g = torch.Generator(device=dev)
    g.manual_seed(SEED)
    A = torch.randint(1, 106, (M, K), generator=g, device=dev, dtype=torch.int32).to(torch.int8)
    Bt = torch.randint(0, 3, (Pp, K), generator=g, device=dev, dtype=torch.int32).to(torch.int8)
    if args.dtype == "i8":
        B = Bt.t()  # [K][Pp] view of the pod rows: K contiguous, as WA is stored
        fn = lambda: torch._int_mm(A, B)  # noqa: E731
        lib, peak = "hipBLASLt int8 GEMM (torch._int_mm), int32 output", PEAK_I8_TOPS
    else:
        A, B = A.to(torch.bfloat16), Bt.to(torch.bfloat16).t()
        fn = lambda: torch.matmul(A, B)  # noqa: E731
        lib, peak = "hipBLASLt bf16 GEMM (torch.matmul), bf16 output", PEAK_BF16_TFLOPS
    try:
        fn()
        torch.cuda.synchronize()
        ms = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ms.append(e0.elapsed_time(e1))
        ms_mean = float(np.mean(ms))
        ops = 2.0 * P * N * nloc
        return {"library": lib, "shape": {"nodes": M, "k": K, "pods": Pp},
                "launch_ms": ms_mean, "launch_ms_min": min(ms), "launches": reps,
                "achieved": ops / (ms_mean * 1e-3) / 1e12, "frac": ops / (ms_mean * 1e-3) / 1e12 / peak,
                "note": "plain GEMM, whole product stored to HBM, C3 value ranges; same op count "
                        "and peak as the roofline object"}
    except Exception as e:  # noqa: BLE001 -- a library refusal is reported, not fatal
        return {"library": lib, "error": str(e)[:200]}
    finally:
        del A, Bt, B
        torch.cuda.empty_cache()


def bench_host(args):
    """SURVEY.md §8(f) next-1 / next-2 on the host (libnas_host.so, no GPU):
    a snapshot refresh -- every node's node-exporter text parsed with the
    reference's Go semantics (scheduler.go:275-331, :396-549) into the SoA
    arrays nas_upload_snapshot takes, one thread and the host's share of
    threads -- and the pairwise latency matrix from all-pairs iperf3 reports
    (scheduler.go:503-530 per pair).  The reference parses 5 scraped bodies
    per pod, sequentially, inside its scheduling loop."""
    import ctypes as C
    from kubernetesnetawarescheduler_amd import hostlib as H
    from kubernetesnetawarescheduler_amd.exporter_text import exporter_body, iperf_report
    rng = np.random.default_rng(SEED)
    n = args.nodes
    names = [f"raspiworker{i}" for i in range(n)]
    bodies = [exporter_body(names[i], rng.choice([6e8, 1.2e9, 1.5e9, 1.8e9], 4),
                            float(rng.integers(5e8, 9e9)), float(rng.integers(1e8, 5e8)),
                            int(rng.integers(0, 3e6)), int(rng.integers(0, 3e6)),
                            int(rng.integers(0, 9))).encode() for i in range(n)]
    nbytes = sum(len(b) for b in bodies)
    arr = (C.c_char_p * n)(*bodies)
    lens = (C.c_size_t * n)(*[len(b) for b in bodies])
    nm = (C.c_char_p * n)(*[x.encode() for x in names])
    outs = [np.zeros(n, np.float64), np.zeros(n, np.float64)] + [np.zeros(n, np.int64) for _ in range(3)]
    status = np.zeros(n, np.int32)
    ptrs = [o.ctypes.data_as(C.c_void_p) for o in outs] + [status.ctypes.data_as(C.c_void_p)]
    cores = cpu_info()
    threads = cores["usable"] or 1

    def run(t, reps=5):
        ms = []
        for _ in range(reps):
            t0 = time.perf_counter()
            rc = H.hostlib().nas_host_snapshot_from_bodies(n, arr, lens, nm, *ptrs, t)
            ms.append((time.perf_counter() - t0) * 1e3)
            assert rc == 0
        return float(np.median(ms)), [o.copy() for o in outs]

    ms1, r1 = run(1)
    msT, rT = run(threads)
    same = all(np.array_equal(a, b) for a, b in zip(r1, rT)) and not status.any()
    # spot-check against the one-node entry point (the ingest tests pin it)
    spot = all(H.node_metrics(bodies[i], names[i]) ==
               (r1[0][i], r1[1][i], int(r1[2][i]), int(r1[3][i]), int(r1[4][i]))
               for i in range(0, n, max(1, n // 64)))
    g = 100
    reps = [[None if i == j else iperf_report(float(rng.uniform(2e8, 9.4e8))).encode()
             for j in range(g)] for i in range(g)]
    flat = [reps[i][j] for i in range(g) for j in range(g)]
    rarr = (C.c_char_p * (g * g))(*flat)
    rlen = (C.c_size_t * (g * g))(*[0 if x is None else len(x) for x in flat])
    L = np.zeros((g, g), np.float32)
    lm = []
    for _ in range(3):
        t0 = time.perf_counter()
        assert H.hostlib().nas_host_latency_matrix_us(g, rarr, rlen, L.ctypes.data_as(C.c_void_p)) == 0
        lm.append((time.perf_counter() - t0) * 1e3)
    lm_ms = float(np.median(lm))
    return {"snapshot_ingest": {"nodes": n, "bytes": nbytes, "ms_1_thread": ms1,
                                "nodes_per_s_1_thread": n / (ms1 * 1e-3), "threads": threads,
                                "ms": msT, "nodes_per_s": n / (msT * 1e-3),
                                "MB_per_s": nbytes / (msT * 1e-3) / 1e6,
                                "thread_count_free": same, "matches_node_metrics": spot},
            "latency_matrix_us": {"nodes": g, "reports": g * (g - 1), "ms": lm_ms,
                                  "reports_per_s": g * (g - 1) / (lm_ms * 1e-3)},
            "cpu": cores,
            "note": "host mirror (libnas_host.so), CPU only; synthetic node-exporter 0.18 "
                    "bodies and iperf3 -J reports (exporter_text.py)"}


def bench_vote(args, d, eng):
    N = args.nodes
    if args.vote_node_shard:
        # node axis sharded (SURVEY.md §8(e) vote row): every rank holds its
        # node slice of all P snapshots; partial records are all-gathered
        # over RCCL and merged, every rank returns all P decisions
        S = args.pods
        lo, hi = d.rank * N // d.world, (d.rank + 1) * N // d.world
        if not eng.has_comm:
            uid = d.bcast_bytes(eng.comm_unique_id() if d.rank == 0 else None)
            eng.comm_init(uid, d.rank, d.world)
        eng.synth_snapshots_shard(SEED, N, lo, hi - lo, S)
    else:
        S = args.pods // d.world
        eng.synth_snapshots(SEED + d.rank, N, S)
    rng = np.random.default_rng(SEED)
    o1 = rng.permutation(N).astype(np.int32)
    o2 = rng.permutation(N + 1).astype(np.int32)
    eng.upload_orders(o1, o2)
    vote_ms = [0.0]

    def step():
        eng.score_reference(S)
        vote_ms[0] += eng.timings()["vote_ms"]

    for _ in range(args.warmup):
        step()
    vote_ms[0] = 0.0
    elapsed = time_steps(d, step, args.steps, 0)
    best, win = eng.score_reference(S)
    return elapsed, vote_ms[0] / args.steps, S, (o1, o2, best, win)


def cpu_baseline_place(args, eng, gpu_nodes, N=None, dtype=None, first=64):
    """Oracle (C restatement, OpenMP) on a bounded sample of the same workload:
    the first Ps pods against all N nodes.  Sequential greedy over pods 0..Ps-1
    depends only on those pods, so the GPU's placements for them must match."""
    import oracle
    N = N or args.nodes
    dtype = dtype or args.dtype
    threads = host_threads()
    os.environ["OMP_NUM_THREADS"] = str(threads)
    _, L, cap, req = eng.read_inputs(0, 0, want_L=True)
    Ps, spent, t_total, pods_done = first, 0.0, 0.0, 0
    placements = None
    while True:
        WA, _, _, _ = eng.read_inputs(0, Ps, want_L=False)
        t0 = time.perf_counter()
        node, _, _ = oracle.place(WA, L, req[:Ps], cap, dtype)
        dt = time.perf_counter() - t0
        spent += dt
        t_total, pods_done, placements = dt, Ps, node
        if dt > args.cpu_budget_s / 2 or Ps >= 16384:
            break
        Ps *= 2
    match = bool((gpu_nodes[:pods_done] == placements).all())
    return {"value": pods_done * N / t_total, "unit": "pair-scores/s", "cores": threads,
            "cores_note": "every usable core (cpu.usable, cpu.usable_source)",
            "kind": "port",
            "sample": f"oracle/oracle.c or_place (sequential greedy, cost rows on {threads} "
                      f"OpenMP threads) on the first {pods_done} pods x {N} nodes of the same "
                      f"workload, {t_total:.2f} s",
            "placements_per_s": pods_done / t_total,
            "gpu_matches_oracle_on_sample": match}


def cpu_baseline_vote(args, eng, ref):
    """Literal restatement of scheduler.go:250-394 (single thread, the
    reference's single Schedule goroutine) on sampled snapshots."""
    import oracle
    o1, o2, best, win = ref
    N = args.nodes
    snaps, idx = [], list(range(0, eng.snap_count, 3))
    t_total, done, ok = 0.0, 0, True
    for s in idx:
        snap = eng.read_snapshot(s)
        t0 = time.perf_counter()
        b, w, _ = oracle.vote(snap, o1, o2)
        t_total += time.perf_counter() - t0
        done += 1
        ok &= (b == best[s]) and (list(w) == win[s].tolist())
        if t_total > args.cpu_budget_s / 2:
            break
    out = {"value": done * N / t_total, "unit": "pair-scores/s", "cores": 1, "kind": "port",
           "sample": f"oracle or_vote_literal (C restatement of scheduler.go:250-394 over plain "
                     f"arrays, one thread like wait.Until(Schedule)) on {done} sampled snapshots "
                     f"x {N} nodes",
           "gpu_matches_oracle_on_sample": bool(ok), "cpu": cpu_info()}
    # the same loop over Go-style maps (oracle/gomap.cpp): nodeMetricsMap
    # filled per pod (:281-331 minus the scrape), range loops over unordered
    # maps (:334-394); the GPU is checked on the map orders it walked
    S_g = min(64, eng.snap_count)
    snaps = [eng.read_snapshot(s) for s in range(S_g)]
    batch = {k: np.stack([x[k] for x in snaps]) for k in snaps[0]}
    del snaps
    b_g, o1_g, o2_g, (fill_ns, loop_ns) = oracle.vote_gomap(batch)
    eng.upload_pod_orders(o1_g, o2_g)  # pod p: snapshot p with its own walked orders
    best_g, _ = eng.score_reference(S_g, pod_snapshot=np.arange(S_g, dtype=np.int32))
    eng.upload_orders(o1, o2)
    tot = (fill_ns + loop_ns) * 1e-9
    out["go_maps"] = {"value": S_g * N / tot, "unit": "pair-scores/s", "cores": 1,
                      "loop_only_value": S_g * N / (loop_ns * 1e-9),
                      "sample": f"oracle/gomap.cpp: {S_g} snapshots x {N} nodes, "
                                f"std::unordered_map<std::string, ...> for nodeMetricsMap and "
                                f"nodePriorities, map fill {fill_ns * 1e-6:.1f} ms + loops "
                                f"{loop_ns * 1e-6:.1f} ms",
                      "gpu_matches_oracle_on_sample": bool((best_g == b_g).all())}
    # the same loop pods-parallel over the host's cores (BASELINE.md plan)
    threads = host_threads()
    os.environ["OMP_NUM_THREADS"] = str(threads)
    S = min(2048, eng.snap_count)
    snaps = [eng.read_snapshot(s) for s in range(S)]
    batch = {k: np.stack([x[k] for x in snaps]) for k in snaps[0]}
    del snaps
    reps, t_par = 0, 0.0
    while t_par < 2.0:
        t0 = time.perf_counter()
        b, w = oracle.vote_batch(batch, o1, o2)
        t_par += time.perf_counter() - t0
        reps += 1
    out["pods_parallel"] = {"value": reps * S * N / t_par, "unit": "pair-scores/s",
                            "cores": threads,
                            "cores_note": "every usable core (cpu.usable, cpu.usable_source)",
                            "sample": f"or_vote_batch over {S} snapshots x {N} "
                                                        f"nodes, OpenMP over pods, {reps} reps",
                            "gpu_matches_oracle_on_sample": bool((b == best[:S]).all() and
                                                                 (w == win[:S]).all())}
    return out


def _timed_place(d, eng, steps, warmup):
    """Timed placement passes with stage timings off (only the events the
    pass synchronises on, as in the headline); one more pass with them on
    fills res["t"] (stages, rescore counts)."""
    res = {}
    # results land in buffers allocated once, as a serving caller keeps them
    # (and as the headline's passes do): fresh arrays every step put ~5 MB of
    # first-touch page faults per C5 pass into the timed region
    n = eng.n_clusters * eng.n_pods
    outs = (np.empty(n, np.int32), np.empty(n, np.float32), np.empty(n, np.int64))

    def step():
        eng.reset_capacity()
        res["node"], _, res["score"] = eng.place(out=outs)
        res["t"] = eng.timings()

    for _ in range(warmup):
        step()
    eng.set_option("STAGE_TIMINGS", 0)
    t = time_steps(d, step, steps, 0)
    eng.set_option("STAGE_TIMINGS", 1)
    node, score = res["node"].copy(), res["score"].copy()
    step()
    assert (res["node"] == node).all() and (res["score"] == score).all()
    return t, res


def config_c1(args, d, eng):
    """configs[0]: the reference's own CPU-sized case, ~10 nodes x 100 pods,
    reference-mode vote scoring (one snapshot per pod), checked against the
    oracle's literal restatement of scheduler.go:250-394."""
    import oracle
    N, S = 10, 100
    eng.synth_snapshots(SEED, N, S)
    rng = np.random.default_rng(SEED)
    o1, o2 = rng.permutation(N).astype(np.int32), rng.permutation(N + 1).astype(np.int32)
    eng.upload_orders(o1, o2)
    t = time_steps(d, lambda: eng.score_reference(S), args.steps, args.warmup)
    best, win = eng.score_reference(S)
    ok = True
    snaps = [eng.read_snapshot(s) for s in range(S)]
    for s in range(S):
        b, w, _ = oracle.vote(snaps[s], o1, o2)
        ok &= b == best[s] and list(w) == win[s].tolist()
    # configs[0] IS "the reference Go scheduler on CPU": its per-pod loop over
    # Go-style maps (oracle/gomap.cpp, one thread like wait.Until(Schedule)),
    # timed on the same 100 snapshots, and the GPU checked on the map orders
    # that run walked
    batch = {k: np.stack([x[k] for x in snaps]) for k in snaps[0]}
    reps, fill, loop = 0, 0, 0
    t_end = time.perf_counter() + 2.0
    while time.perf_counter() < t_end:
        b_g, o1_g, o2_g, (f_ns, l_ns) = oracle.vote_gomap(batch)
        fill, loop, reps = fill + f_ns, loop + l_ns, reps + 1
    eng.upload_orders(o1_g, o2_g)
    best_g, _ = eng.score_reference(S)
    cpu_ms = (fill + loop) * 1e-6 / reps
    cpu_base = {"value": S * N / (cpu_ms * 1e-3), "unit": "pair-scores/s", "cores": 1,
                "kind": "port", "ms_per_step": cpu_ms, "loop_only_ms": loop * 1e-6 / reps,
                "sample": f"oracle/gomap.cpp (scheduler.go:281-394 over std::unordered_map, "
                          f"map fill + loops), the same {S} snapshots, {reps} repetitions",
                "gpu_matches_on_its_map_orders": bool((best_g == b_g).all()), "cpu": cpu_info()}
    # extended mode on the same shape: every pod sends
    # 100 MB (customNetworkBenchmark/*.data:2) to one bound server pod, seeded
    # 10 x 10 int8 latency, Raspberry-Pi-sized capacity
    P = S
    L = rng.integers(1, 100, (N, N)).astype(np.int8)
    L = np.triu(L, 1) + np.triu(L, 1).T
    server = int(rng.integers(0, N))
    WA = np.zeros((P, N), np.int8)
    WA[:, server] = 100
    free = np.tile(np.array([[4000, 4 << 20, 110]], np.int32), (N, 1))
    req = np.stack([rng.integers(1, 540, P), rng.integers(7_464, 303_749, P), np.ones(P)],
                   1).astype(np.int32)
    eng.upload_latency(L, "i8")
    eng.upload_capacity(free)
    eng.upload_pods(req)
    eng.upload_traffic(WA, "i8")
    te, res = _timed_place(d, eng, args.steps, args.warmup)
    want, wcost, _ = oracle.place(WA, L, req, free, "i8")
    ok_ext = (res["node"] == want).all() and (res["score"] == wcost).all()
    return {"workload": f"C1: reference-mode vote, {N} nodes x {S} pods (one snapshot per pod); "
                        f"extended mode on the same shape (100 MB per pod to one server pod)",
            "value": S * N / (t / args.steps), "unit": "pair-scores/s",
            "ms_per_step": t * 1e3 / args.steps, "matches_oracle": bool(ok),
            "cpu_baseline": cpu_base,
            "extended": {"ms_per_step": te * 1e3 / args.steps,
                         "placements_per_s": P / (te / args.steps), "matches_oracle": bool(ok_ext)},
            "bound": "latency: one nas_score_reference call (a few tens of microseconds of launch "
                     "and copy; 48 KB of snapshots) per step -- the HBM or MFMA roofline does not "
                     "apply at 1000 pairs",
            "note": "launch-latency bound: one score_reference / nas_place call per step"}


def config_c2(args, d, eng):
    """configs[1]: clusterloader2-derived 1k x 10k, sparse (CSR) pod
    communication graph; the whole placement is checked against the oracle."""
    import oracle
    from kubernetesnetawarescheduler_amd import workloads
    N, P = 1000, 10000
    c = workloads.c2_cluster(SEED, N, P)
    eng.upload_latency(c["L"], "i8")
    eng.upload_capacity(c["free"])
    eng.upload_pods(c["req"])
    eng.upload_traffic_csr(c["row_ptr"], c["peer_node"], c["weight"], "i8", N)
    t, res = _timed_place(d, eng, args.steps, args.warmup)
    stages = {k: res["t"][k] for k in ("fit_ms", "cost_ms", "merge_ms", "commit_ms", "total_ms",
                                        "rescore_rounds", "rescored_pods", "commit_rounds")}
    WA = workloads.csr_to_dense(c["row_ptr"], c["peer_node"], c["weight"], N)
    t0 = time.perf_counter()
    want, wcost, wfree = oracle.place(WA, c["L"], c["req"], c["free"], "i8")
    t_cpu = time.perf_counter() - t0
    ok = (res["node"] == want).all() and (res["score"] == wcost).all() \
        and (eng.get_capacity() == wfree).all()
    ms = t * 1e3 / args.steps
    return {"workload": f"C2: clusterloader2 requests, {N} nodes x {P} pods, CSR traffic "
                        f"({len(c['peer_node'])} nnz, exact int32 aggregation), latency "
                        f"U[50,500] us in 4-us int8 steps",
            "value": P * N / (ms * 1e-3), "unit": "pair-scores/s", "ms_per_step": ms,
            "placements_per_s": P / (ms * 1e-3), "unschedulable": res["t"]["unschedulable"],
            "matches_oracle": bool(ok), "oracle_check": f"all {P} pods, scores and capacity",
            "stages_ms": stages,
            "bound": "latency: the contraction is 2e10 int8 ops (~4 us at the MFMA peak); a pass "
                     "is the pipeline's launches plus the commit's stops -- each gathered rescore "
                     "slot (stale scan, compact, gather, fit, cost, merge, commit) is a chain of "
                     "dependent small launches (stages_ms: device-side sums)",
            "cpu_baseline": {"value": P * N / t_cpu, "unit": "pair-scores/s",
                             "cores": int(os.environ.get("OMP_NUM_THREADS", "1")), "kind": "port",
                             "ms_per_step": t_cpu * 1e3,
                             "sample": "oracle/oracle.c or_place on the whole C2 workload"}}


def config_c5(args, d, eng, B=64, N=5000, P=5000, sample=1024):
    """configs[4]: 64 independent 5k-node clusters (5k pending pods each) in
    one batched nas_place; cluster 0's first `sample` pods checked against the
    oracle (sequential greedy over a prefix depends only on that prefix)."""
    import oracle
    eng.synth_batch(SEED, B, N, P, "i8", peers=args.peers)
    t, res = _timed_place(d, eng, args.steps, args.warmup)
    WA, L, cap, req = eng.read_inputs(0, sample, want_L=True)
    t0 = time.perf_counter()
    want, wcost, _ = oracle.place(WA, L, req[:sample], cap, "i8")
    t_cpu = time.perf_counter() - t0
    ok = (res["node"][0, :sample] == want).all() and (res["score"][0, :sample] == wcost).all()
    ms = t * 1e3 / args.steps
    # roofline of the batched contraction: the k_cost_topk launches over all
    # clusters (nas_score: a wide and a narrow one back to back), HIP events
    # around both; 2 * B * P * N * N int8 ops
    eng.reset_capacity()
    cms = []
    for _ in range(4):
        eng.score()
        cms.append(eng.timings()["cost_ms"])
    cost_ms = float(np.median(cms[1:]))
    kpad = -(-N // 128) * 128
    ops = 2.0 * B * P * N * kpad
    return {"workload": f"C5: batch of {B} clusters x {N} nodes x {P} pods (synthetic, seeded)",
            "value": B * P * N / (ms * 1e-3), "unit": "pair-scores/s", "ms_per_step": ms,
            "placements_per_s": B * P / (ms * 1e-3), "unschedulable": res["t"]["unschedulable"],
            "rescore_rounds": res["t"]["rescore_rounds"], "matches_oracle": bool(ok),
            "oracle_check": f"cluster 0, first {sample} pods",
            "roofline": {"kernel": "k_cost_topk (batched: 256 x 384 tiles over the first 4,608 pods "
                                   "of every cluster, 256 x 256 over the rest, back to back)",
                         "bound": "mfma",
                         "achieved": ops / (cost_ms * 1e-3) / 1e12, "peak": PEAK_I8_TOPS,
                         "unit": "TFLOP/s", "frac": ops / (cost_ms * 1e-3) / 1e12 / PEAK_I8_TOPS,
                         "launch_ms": cost_ms, "launches": 3, "ops_per_launch": ops},
            "cpu_baseline": {"value": sample * N / t_cpu, "unit": "pair-scores/s",
                             "cores": int(os.environ.get("OMP_NUM_THREADS", "1")), "kind": "port",
                             "sample": f"oracle or_place on cluster 0's first {sample} pods"}}


def config_c3_bf16(args, d, eng):
    """The headline C3 shape on the bf16 path (fp32 accumulation): a
    placement pass timed like the headline, and the roofline of its full-size
    k_cost_topk launch against the dense bf16 MFMA peak.  Parity of the bf16
    path (candidates within 1e-5 of fp64) is the GPU suite's job."""
    N, P = args.nodes, args.pods
    eng.synth_cluster(SEED, N, P, "bf16", peers=args.peers)
    t, res = _timed_place(d, eng, args.steps, args.warmup)
    ms = t * 1e3 / args.steps
    eng.reset_capacity()
    # one untimed launch, then the mean of six (one box's run had three
    # launches averaging 20.7 ms against 12.9-13.0 ms on every other run, its
    # pass unaffected: six keep one such launch from halving the line's frac;
    # the samples are in the line)
    cms = []
    for _ in range(7):
        eng.score()
        cms.append(eng.timings()["cost_ms"])
    cost_ms = float(np.mean(cms[1:]))
    ops = 2.0 * P * N * N
    return {"workload": f"C3 in bf16: {N} nodes x {P} pods, dense bf16 latency + traffic",
            "dtype": "bf16xbf16->f32", "value": P * N / (ms * 1e-3), "unit": "pair-scores/s",
            "ms_per_step": ms, "placements_per_s": P / (ms * 1e-3),
            "unschedulable": res["t"]["unschedulable"], "rescore_rounds": res["t"]["rescore_rounds"],
            "roofline": {"kernel": "k_cost_topk<bf16>", "bound": "mfma",
                         "achieved": ops / (cost_ms * 1e-3) / 1e12, "peak": PEAK_BF16_TFLOPS,
                         "unit": "TFLOP/s",
                         "frac": ops / (cost_ms * 1e-3) / 1e12 / PEAK_BF16_TFLOPS,
                         "launch_ms": cost_ms, "launches": len(cms) - 1,
                         "launch_ms_samples": [round(c, 4) for c in cms[1:]],
                         "ops_per_launch": ops}}


_TRAFFIC_FULLRANGE = {}


def config_c3_fullrange(args, d, eng, sample=2048):
    """The headline C3 shape (10k nodes x 100k pods, int8) on SURVEY.md
    §8(d)'s own operand distribution: latency and traffic
    uniform over the full int8 range (NAS_OPT_SYNTH_PROFILE 1 -- U{1..127}
    for U[1, 1000] us, U{0..127} for U[0, 1)), no rack / zone locality and no
    bound-peer structure.  The cost kernel is power-limited, so its rate
    depends on operand entropy: this line states whether >= 1e11 pair scores/s
    holds on full-range operands.  A placement pass timed like the headline,
    its own k_cost_topk roofline (with its PMC traffic when collected) and the
    first `sample` pods checked against the sequential oracle."""
    import oracle
    N, P = args.nodes, args.pods
    eng.synth_cluster(SEED, N, P, "i8", peers=args.peers, profile=1)
    t, res = _timed_place(d, eng, args.steps, args.warmup)
    ms = t * 1e3 / args.steps
    eng.reset_capacity()
    cms = []
    for _ in range(max(4, args.steps // 2 + 1)):
        eng.score()
        cms.append(eng.timings()["cost_ms"])
    cost_ms = float(np.mean(cms[1:]))
    ops = 2.0 * P * N * N
    WA, L, cap, req = eng.read_inputs(0, sample, want_L=True)
    t0 = time.perf_counter()
    want, wcost, _ = oracle.place(WA, L, req[:sample], cap, "i8")
    t_cpu = time.perf_counter() - t0
    ok = bool((res["node"][:sample] == want).all() and (res["score"][:sample] == wcost).all())
    tr = _TRAFFIC_FULLRANGE.get("k_cost_topk", {}).get("bytes")
    value = P * N / (ms * 1e-3)
    return {"workload": f"C3 on the full int8 range: {N} nodes x {P} pods, latency U{{1..127}} "
                        f"(symmetric, zero diagonal), traffic U{{0..127}} to every node, "
                        f"clusterloader2-shaped requests", "dtype": "i8xi8->i32",
            "value": value, "unit": "pair-scores/s", "ms_per_step": ms,
            "placements_per_s": P / (ms * 1e-3), "meets_1e11": bool(value >= 1e11),
            "unschedulable": res["t"]["unschedulable"], "rescore_rounds": res["t"]["rescore_rounds"],
            "matches_oracle": ok, "oracle_check": f"first {sample} pods: placements and scores",
            "operands": {"WA_min": int(WA.min()), "WA_max": int(WA.max()),
                         "WA_mean": float(WA.mean()), "L_offdiag_min": int(L[~np.eye(N, dtype=bool)].min()),
                         "L_max": int(L.max()), "L_symmetric": bool((L == L.T).all())},
            "roofline": {"kernel": "k_cost_topk<int8> (wide tile)", "bound": "mfma",
                         "achieved": ops / (cost_ms * 1e-3) / 1e12, "peak": PEAK_I8_TOPS,
                         "unit": "TFLOP/s", "frac": ops / (cost_ms * 1e-3) / 1e12 / PEAK_I8_TOPS,
                         "traffic": tr, "traffic_unit": "B/launch",
                         "launch_ms": cost_ms, "launches": len(cms) - 1, "ops_per_launch": ops},
            "cpu_baseline": {"value": sample * N / t_cpu, "unit": "pair-scores/s",
                             "cores": int(os.environ.get("OMP_NUM_THREADS", "1")), "kind": "port",
                             "sample": f"oracle or_place on the first {sample} pods"}}


def config_c2_f32(args, d, eng):
    """C2 with measured float latencies (microseconds, unquantised) and float
    traffic (MB): the fp32 path (v_mfma_f32_32x32x2_f32, exact fp32 products).
    Placements equal the fp64 sequential oracle up to the first pod whose two
    best fitting nodes are within the 1e-5 relative tolerance."""
    import oracle
    from kubernetesnetawarescheduler_amd import workloads
    N, P = 1000, 10000
    c = workloads.c2_cluster(SEED, N, P)
    rng = np.random.default_rng(SEED + 1)
    Lf = c["L"].astype(np.float32) * 4.0 + rng.uniform(0.0, 4.0, (N, N)).astype(np.float32)
    Lf = np.triu(Lf, 1) + np.triu(Lf, 1).T
    wf = c["weight"].astype(np.float32) * rng.uniform(0.9, 1.1, len(c["weight"])).astype(np.float32)
    eng.upload_latency(Lf, "f32")
    eng.upload_capacity(c["free"])
    eng.upload_pods(c["req"])
    eng.upload_traffic_csr(c["row_ptr"], c["peer_node"], wf, "f32", N)
    t, res = _timed_place(d, eng, args.steps, args.warmup)
    ms = t * 1e3 / args.steps
    WA = workloads.csr_to_dense(c["row_ptr"], c["peer_node"], wf.astype(np.float64), N)
    want, _, _ = oracle.place(WA.astype(np.float32), Lf, c["req"], c["free"], "f32")
    diff = np.nonzero(res["node"] != want)[0]
    eng.reset_capacity()
    cms = []
    for _ in range(4):
        eng.score()
        cms.append(eng.timings()["cost_ms"])
    cost_ms = float(np.mean(cms[1:]))
    ops32 = 2.0 * P * N * (-(-N // 32) * 32)
    ops = 6 * ops32  # the bf16 MFMA work of the six-segment split (k_misc.hip k_split6)
    return {"workload": f"C2 in fp32: {N} nodes x {P} pods, float latency (us) and CSR "
                        f"traffic (MB)", "dtype": "f32 (3-plane bf16 split)xf32->f32",
            "value": P * N / (ms * 1e-3), "unit": "pair-scores/s", "ms_per_step": ms,
            "placements_per_s": P / (ms * 1e-3), "unschedulable": res["t"]["unschedulable"],
            "identical_to_fp64_oracle_pods": int(diff[0]) if len(diff) else P,
            "roofline": {"kernel": "k_cost_topk<bf16> on the fp32 operands' six-segment split",
                         "bound": "mfma",
                         "achieved": ops / (cost_ms * 1e-3) / 1e12, "peak": PEAK_BF16_TFLOPS,
                         "unit": "TFLOP/s",
                         "frac": ops / (cost_ms * 1e-3) / 1e12 / PEAK_BF16_TFLOPS,
                         "launch_ms": cost_ms, "launches": 3, "ops_per_launch": ops,
                         "fp32_equivalent_tflops": ops32 / (cost_ms * 1e-3) / 1e12,
                         "note": "160 workgroups on 256 CUs: occupancy-bound at this size"},
            "bound": "latency (like C2): the contraction is 1.2e11 bf16 FLOPs (~0.05 ms at the "
                     "bf16 peak) on 160 workgroups; the pass is launches plus the commit's stops"}


def config_c4(args, d, eng, N=50000, P=500000):
    """configs[3]: 50k nodes x 500k pods, node axis sharded over the ranks."""
    if d.world > 1:
        uid = d.bcast_bytes(eng.comm_unique_id() if d.rank == 0 else None)
        eng.comm_init(uid, d.rank, d.world)
    eng.synth_cluster(SEED, N, P, "i8", peers=args.peers)
    steps = max(1, min(args.steps, 2))
    t, res = _timed_place(d, eng, steps, 1)
    if d.world == 1:
        _C4_WORLD1.update(node=res["node"].copy(), score=res["score"].copy())
    ms = t * 1e3 / steps
    # pass-level roofline: 2 * P * N * K int8 ops per pass (K = N padded to
    # 128) over the whole pass's wall time -- the cost launches (two scoring
    # streams) dominate; fit, merges and the replicated commit overlap them
    ops = 2.0 * P * N * (-(-N // 128) * 128)
    out = {"workload": f"C4: {N} nodes x {P} pods, node-sharded x{d.world}",
           "value": P * N / (ms * 1e-3), "unit": "pair-scores/s", "ms_per_step": ms,
           "steps": steps, "placements_per_s": P / (ms * 1e-3),
           "unschedulable": res["t"]["unschedulable"], "rescore_rounds": res["t"]["rescore_rounds"],
           "stages_ms": {k: res["t"][k] for k in ("fit_ms", "cost_ms", "merge_ms", "commit_ms")},
           "stages_note": "device-side sums per pass; cost_ms adds the two scoring streams' "
                          "overlapping launches",
           "bound": f"mfma: {ops:.3g} int8 ops per pass ({ops / PEAK_I8_TOPS / 1e12 * 1e3:.0f} ms "
                    f"at the dense peak on one GPU)",
           "roofline": {"kernel": "whole pass (k_cost_topk dominates)", "bound": "mfma",
                        "achieved": ops / (ms * 1e-3) / 1e12, "peak": PEAK_I8_TOPS * d.world,
                        "unit": "TFLOP/s", "frac": ops / (ms * 1e-3) / 1e12 / (PEAK_I8_TOPS * d.world),
                        "ops_per_pass": ops, "gpus": d.world}}
    if d.world == 1 and d.rank == 0 and not args.no_cpu_baseline:
        cb = cpu_baseline_place(args, eng, res["node"], N=N, dtype="i8", first=4)
        cb["sample"] = cb["sample"].replace("of the same workload", "of the C4 workload")
        out["cpu_baseline"] = cb
    return out


_C4_WORLD1 = {}


def config_c4_shard(args, d, eng, G=2, N=50000, P=500000):
    """configs[3]'s node split at its own size on ONE GPU: G virtual node
    shards (nas_set_shard contexts, each scoring N/G node columns over the full
    K), lists exchanged and merged on the host, the commit replayed on every
    shard (sharded.place_local_shards).  The shards run one after another on
    the same GPU, so this is G x one shard's work plus the host exchange -- a
    check of the multi-GPU split's geometry and results at size, NOT a
    multi-GPU timing.  Placements and scores are compared with the world-1
    C4 pass of the same seed (configs.C4, same run)."""
    from kubernetesnetawarescheduler_amd import Engine
    from kubernetesnetawarescheduler_amd.sharded import place_local_shards
    engines = [eng] + [Engine(d.local) for _ in range(G - 1)]
    try:
        for r, e in enumerate(engines):
            e.set_shard(r, G)
            e.synth_cluster(SEED, N, P, "i8", peers=args.peers)
        res = {}

        def step():
            for e in engines:
                e.reset_capacity()
            res["node"], res["score"], res["rounds"] = place_local_shards(engines, P)

        t = time_steps(d, step, 1, 1)
        caps = [e.get_capacity() for e in engines]
    finally:
        for e in engines[1:]:
            e.close()
    ms = t * 1e3
    out = {"workload": f"C4: {N} nodes x {P} pods as {G} virtual node shards on one GPU, "
                       f"host exchange (sharded.place_local_shards)",
           "value": P * N / (ms * 1e-3), "unit": "pair-scores/s", "ms_per_step": ms, "steps": 1,
           "rescore_rounds": res["rounds"], "unschedulable": int((res["node"] < 0).sum()),
           "shards_agree_on_capacity": bool(all((c == caps[0]).all() for c in caps)),
           "note": "the G shards' scoring runs serially on one GPU and the lists cross the host: "
                   "a correctness run of the multi-GPU split at its size, not a scaling number"}
    w1 = _C4_WORLD1.get("node")
    if w1 is not None:
        out["equals_world1"] = bool((w1 == res["node"]).all() and
                                    (_C4_WORLD1["score"] == res["score"]).all())
    return out


def run_configs(args, d, only=None):
    """The other BASELINE configs, each on a fresh context (one GPU)."""
    from kubernetesnetawarescheduler_amd import Engine
    out = {}
    for name, fn in (("C1", config_c1), ("C2", config_c2), ("C2_f32", config_c2_f32),
                     ("C3_bf16", config_c3_bf16), ("C3_fullrange", config_c3_fullrange),
                     ("C5", config_c5), ("C4", config_c4),
                     ("C4_shardG2", config_c4_shard)):
        if only and name != only:
            continue
        with Engine(d.local) as e:
            out[name] = fn(args, d, e)
    return out


def _claim_stdout():
    """The contract is ONE JSON line on stdout; RCCL (and HIP runtime libraries)
    print banners there from native code.  Point fd 1 at stderr for the run and
    keep the original stdout for the result line."""
    sys.stdout.flush()
    keep = os.dup(1)
    os.dup2(2, 1)
    return os.fdopen(keep, "w")


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args))
    result_out = _claim_stdout()
    traffic, traffic_why = {}, "not collected (--no-pmc or a multi-GPU run)"
    if (not args.no_pmc and args.only is None and args.gpus == 1
            and int(os.environ.get("WORLD_SIZE", "1")) == 1):
        traffic, traffic_why = pmc_traffic(args)  # before this process initialises the GPU
        if not args.no_configs and args.dtype == "i8" and args.synth_profile == 0:
            # configs.C3_fullrange's own launch traffic (its inputs, score leg only)
            _TRAFFIC_FULLRANGE.update(pmc_traffic(args, profile=1)[0])
    d = Dist(args.gpus)
    from kubernetesnetawarescheduler_amd import Engine
    eng = Engine(d.local)
    N, P = args.nodes, args.pods
    out = {"metric": "pod-node pair scores/sec and placements/sec at 10k nodes x 100k pods",
           "unit": "pair-scores/s", "n_gpus": d.world, "steps": args.steps,
           "warmup": args.warmup, "higher_is_better": True, "scaling": "strong",
           "vs_baseline": None, "dtype": "i8xi8->i32" if args.dtype == "i8" else "bf16xbf16->f32",
           "data": "synthetic (seeded, generated in HBM)",
           "config": {"workload": f"C3: {N} nodes x {P} pods, dense {args.dtype} latency + "
                                  f"traffic, racks of 32 / zones of 16 racks, {args.peers} "
                                  f"peers per pod, clusterloader2-shaped requests",
                      "nodes": N, "pods": P, "parallelism": f"node-sharded x{d.world}",
                      "candidates_per_pod": 8}}
    gpu_nodes = None
    cfg_only = args.only if args.only and args.only.startswith("C") else None
    if cfg_only:  # one config line alone (profiling)
        eng.close()
        out["configs"] = run_configs(args, d, cfg_only)
        if d.rank == 0:
            print(json.dumps(out), file=result_out, flush=True)
        return
    if args.rehearse_world > 1:
        out["rehearsal"] = (f"rank 0 of a {args.rehearse_world}-GPU node-sharded pass on one GPU: "
                            "its node columns scored, the other ranks' lists stood in for by "
                            "shifted copies; NOT a multi-GPU measurement, placements not checked")
    if args.only not in ("vote", "score", "pmc"):
        elapsed, per, gpu_nodes, eng, exchange = bench_place(args, d, eng)
        if exchange:
            out["config"]["exchange"] = exchange
        out["value"] = P * N / (elapsed / args.steps)
        out["ms_per_step"] = elapsed * 1e3 / args.steps
        out["placements_per_s"] = P / (elapsed / args.steps)
        out["stages_ms"] = {k: per[k] for k in ("fit_ms", "cost_ms", "merge_ms", "commit_ms",
                                                "total_ms")}
        out["stages_note"] = ("device-side sums per step (3 extra steps with stage timings on; "
                              "the timed steps record only synchronising events); scoring runs "
                              "in chunks on two streams with merge + commit pipelined on a "
                              "third, so stages overlap")
        out["rescore_rounds"] = per["rescore_rounds"]
        out["unschedulable"] = per["unschedulable"]
    if args.only not in ("vote",):
        if gpu_nodes is None:
            eng.synth_cluster(SEED, N, P, args.dtype, peers=args.peers, profile=args.synth_profile)
        cost_ms, samples = bench_cost_kernel(args, d, eng)
        nloc = N // max(d.world, args.rehearse_world)
        ops = 2.0 * P * N * nloc
        achieved = ops / (cost_ms * 1e-3) / 1e12
        peak = PEAK_I8_TOPS if args.dtype == "i8" else PEAK_BF16_TFLOPS
        out["roofline"] = {"kernel": "k_cost_topk", "bound": "mfma", "achieved": achieved,
                           "peak": peak, "unit": "TFLOP/s",
                           "op_type": "int8 ops (2 per MAC) vs the dense int8 MFMA peak"
                                      if args.dtype == "i8" else "bf16 FLOPs",
                           "frac": achieved / peak,
                           "traffic": traffic.get("k_cost_topk", {}).get("bytes"),
                           "traffic_unit": "B/launch",
                           "traffic_note": ("beyond-L2 bytes of the largest k_cost_topk dispatch "
                                            "(rocprofv3 FETCH_SIZE x 2, which counts the L2's "
                                            "memory-side requests incl. Infinity Cache hits, "
                                            "+ WRITE_SIZE) in this run"
                                            if traffic else traffic_why),
                           "launch_ms": cost_ms, "launches": len(samples),
                           "launch_ms_min": min(samples), "ops_per_launch": ops,
                           "note": "mean over the timed launches of one launch over all pods x "
                                   "this rank's node columns (nas_score), HIP events on its "
                                   "stream; 2*P*N*N_local ops; tools/check_roofline.py compares "
                                   "it with the rocprofv3 kernel trace of the same command"}
        if d.gpu and d.world == 1 and args.only is None:
            out["roofline"]["vendor_gemm"] = vendor_gemm_reference(args, d)
    if args.only not in ("vote",) and d.gpu:
        fr = bench_fit_kernel(args, d, eng)
        fr["traffic"] = traffic.get("k_fit", {}).get("bytes")
        fr["traffic_unit"] = "B/launch"
        out["fit_roofline"] = fr
    if not args.no_reference_mode and args.only in (None, "vote", "pmc"):
        elapsed, vote_ms, S, ref = bench_vote(args, d, eng)
        pods_total = S if args.vote_node_shard else S * d.world
        nloc = (d.rank + 1) * N // d.world - d.rank * N // d.world if args.vote_node_shard else N
        bytes_launch = 48.0 * nloc * S
        out["reference_mode"] = {
            "value": pods_total * N / (elapsed / args.steps), "unit": "pair-scores/s",
            "ms_per_step": elapsed * 1e3 / args.steps,
            "sharding": "node axis, RCCL all-gather of partial records" if args.vote_node_shard
                        else "pods (independent snapshots), no collective",
            "workload": f"vote scorer, one fresh {N}-node snapshot per pod ({pods_total} pods)",
            "roofline": {"kernel": "k_vote_partial" if args.vote_node_shard else "k_vote",
                         "bound": "hbm",
                         "achieved": bytes_launch / (vote_ms * 1e-3) / 1e9, "peak": PEAK_HBM_GBS,
                         "unit": "GB/s",
                         "frac": bytes_launch / (vote_ms * 1e-3) / 1e9 / PEAK_HBM_GBS,
                         "traffic": traffic.get("k_vote", {}).get("bytes"),
                         "traffic_unit": "B/launch", "launch_ms": vote_ms, "bytes_per_launch": bytes_launch}}
        if (d.rank == 0 and d.world == 1 and not args.no_cpu_baseline and not args.vote_node_shard
                and args.only != "pmc"):
            out["reference_mode"]["cpu_baseline"] = cpu_baseline_vote(args, eng, ref)
    if d.rank == 0 and d.world == 1 and not args.no_cpu_baseline and gpu_nodes is not None:
        # the vote path freed nothing; re-synthesise the cluster inputs (same seed)
        eng.synth_cluster(SEED, N, P, args.dtype, peers=args.peers, profile=args.synth_profile)
        out["cpu_baseline"] = cpu_baseline_place(args, eng, gpu_nodes)
    eng.close()
    if d.world == 1 and not args.no_configs and args.only is None:
        out["configs"] = run_configs(args, d)
    if d.rank == 0 and d.world == 1 and args.only is None and not args.no_configs:
        out["host"] = bench_host(args)
    if args.c4 and "C4" not in out.get("configs", {}):
        from kubernetesnetawarescheduler_amd import Engine
        with Engine(d.local) as e:
            out.setdefault("configs", {})["C4"] = config_c4(args, d, e)
    if d.rank == 0:
        print(json.dumps(out), file=result_out, flush=True)


if __name__ == "__main__":
    main()
