"""Benchmark: local-BA LM iterations/s on MI355X (BASELINE.json metric).

One "step" is one Levenberg-Marquardt iteration (OptimizationAlgorithmLevenberg::solve:
linearize + Schur + dense reduced-camera solve + update + re-evaluation) of the GP local BA on a
synthetic BASELINE config-1 window (50 optimisable KF + 1 fixed, 20k landmarks, ~120k
observations, 4 asynchronous cameras, fp64), with the early-stop rule disabled so the iteration
count is fixed.  Inputs are resident in HBM before the timed region.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

With N > 1 every rank optimises its own window (window farming, BASELINE config 3): windows are
cut from one trajectory so neighbouring windows share keyframes and landmarks, and at every
window boundary (each --window-iters iterations) the owners of shared landmarks publish their
estimates with one all_gather over RCCL (xGMI).  value = iterations of all ranks / max-rank time.

`python bench.py --gpus N` with N > 1 and no WORLD_SIZE in the environment launches the N rank
processes itself (torch.distributed.run as a child process, before anything touches the GPU) and
exits with its status; rank 0's line is the job's line.  Under a launcher, WORLD_SIZE must equal
--gpus.  --dry-launch prints the launch (command and rank environment) and exits.
"""
import argparse
import ctypes
import glob
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "amc-slam_amd"))

METRIC = "local-BA iterations/sec (50 KF, 20k landmarks, 120k obs) at 1/2/4/8 MI355X"


def metric_for(config, W):
    """BASELINE.json's metric string for its own configuration (configs[1]); the same form for the others
    (global BA for the global-BA shapes, configs[2] and configs[4])."""
    if config == "cfg1_local_50kf":
        return METRIC
    from amc_lba.synth import CONFIGS
    glob = bool(CONFIGS.get(config, {}).get("global_ba"))
    n_kf = int((W.kfs["fixed"] == 0).sum())
    return (f"{'global' if glob else 'local'}-BA iterations/sec ({n_kf} KF, {len(W.lm) // 1000}k landmarks, "
            f"{len(W.obs) // 1000}k obs) at 1/2/4/8 MI355X")


def s8d_sweep_bytes(win):
    """SURVEY.md §8(d)'s B_sweep exactly as the survey defines it: 72 B per observation + 288 B per unique
    (KF, landmark) Hpl block + 96 B per landmark + 2 x (1152 B per KF pair + 96 B per KF).  The kernel no
    longer writes the Hpl blocks (they stay in LDS), but this is the figure the north-star's HBM target is
    quoted on, so it is reported as such (roofline_s8d)."""
    n_obs = len(win.obs)
    n_lm = len(np.unique(win.obs["lm"]))
    n_kf = int((win.kfs["fixed"] == 0).sum())
    return 72 * n_obs + 288 * int(win.n_pairs) + 96 * n_lm + 2 * (1152 * max(n_kf - 1, 0) + 96 * n_kf)


def launch_ranks(args, argv):
    """--gpus N > 1 without a launcher: run the N ranks as a child torch.distributed.run (one process per
    GPU, RCCL over xGMI, rendezvous on 127.0.0.1) and return its exit status; None when this process is
    the (only) rank.  Nothing here touches the GPU, so the children own the devices."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != args.gpus:
            print(f"bench.py: WORLD_SIZE={ws} but --gpus {args.gpus}", file=sys.stderr)
            return 2
        return None
    if args.gpus <= 1:
        return None
    import socket
    with socket.socket() as sk:   # a free rendezvous port
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + \
        [a for a in argv if a != "--dry-launch"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    if args.dry_launch:
        print(json.dumps({"launch": cmd, "nproc": args.gpus, "master_addr": "127.0.0.1", "master_port": port,
                          "env": {"HSA_ENABLE_IPC_MODE_LEGACY": env["HSA_ENABLE_IPC_MODE_LEGACY"]}}), flush=True)
        return 0
    return subprocess.run(cmd, env=env).returncode


HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
FP64_PEAK_TFLOPS = 78.6        # MI355X fp64 vector/matrix spec


def sweep_bytes(win):
    """SURVEY.md §8(d) algorithmic bytes of the residual/Jacobian/J^T W J sweep per launch, as this kernel
    moves them: 72 B per observation of compulsory input, 96 B per landmark (Hll + bl), 2 x (1152 B per
    KF-pair Hpp block + 96 B per KF).  §8(d)'s 288 B per (KF, landmark) Hpl block is not written any more:
    a regular tile's Hpl stays in LDS from its computation to its elimination and k_update back-substitutes
    in the sample space; only the heavy landmarks' segment blocks (none at config 1) are
    stored."""
    n_obs = len(win.obs)
    n_lm = len(np.unique(win.obs["lm"]))
    n_kf = int((win.kfs["fixed"] == 0).sum())
    n_kfpairs = max(n_kf - 1, 0)
    return 72 * n_obs + 96 * n_lm + 2 * (1152 * n_kfpairs + 96 * n_kf)


def sweep_flops(win):
    """Algorithmic fp64 FLOPs of the sweep as this implementation formulates it: per
    observation, residual (~60) and the Jacobian w.r.t. its pose sample and point (~150); per row,
    the sample-space products M += s J1^T J1, g += s J1^T e (27 FMA), G += s J1^T Jp (18 FMA) and
    Hll / bl (12 FMA); per (observation, KF side) the Hpl block N_side^T G (12 x 3 x 6 FMA).  The
    24 x 24 expansion N^T M N happens once per pose sample (k_prior_lin), not per row."""
    k = win.obs["kind"]
    gp = np.isin(k, (0, 1))
    rows = np.where(np.isin(k, (1, 3)), 3, 2)
    sides = np.where(gp, 2, 1)
    f = 60 + 150 + 2 * (27 + 18 + 12) * rows + 2 * 216 * sides
    return float(f.sum())


def schur_terms(win):
    """The landmark elimination fused into the sweep kernel (k_lin_schur): per landmark
    with P non-fixed KF blocks, Dinv (72 B written), and the Schur complement it adds to S: one 12 x 12
    block per pair of its KFs (a <= b), and a 12-vector of the reduced rhs per KF.  Algorithmic bytes:
    72 B per landmark + 1152 B per distinct coupled KF pair + 96 B per KF (the reduced system's
    pieces, written once); FLOPs: per landmark 2 x 3 x (12P)(12P + 1) / 2 (sum_m Hpl Dinv Hpl^T, upper
    half) + 2 x 36 P (rhs) + ~60 (3 x 3 inverse / LDL^T)."""
    o = win.obs
    fixed = win.kfs["fixed"].astype(bool)
    ks = np.concatenate([np.stack([o["lm"], o["kf_b"]], 1), np.stack([o["lm"], o["kf_a"]], 1)])
    ks = ks[(ks[:, 1] >= 0)]
    ks = ks[~fixed[ks[:, 1]]]
    ks = np.unique(ks, axis=0)
    lm_ids, starts, counts = np.unique(ks[:, 0], return_index=True, return_counts=True)
    pairs = set()
    flops = 0.0
    for s, c in zip(starts, counts):
        kk = ks[s:s + c, 1]
        P = len(kk)
        flops += 3.0 * (12 * P) * (12 * P + 1) + 72.0 * P + 60.0
        for a in range(P):
            for b in range(a, P):
                pairs.add((int(kk[a]), int(kk[b])))
    n_kf = int((~fixed).sum())
    return 72 * len(lm_ids) + 1152 * len(pairs) + 96 * n_kf, flops


def pmc_summary(workload, kernel):
    """The committed rocprofv3 PMC summary (scripts/pmc_linearize.sh + pmc_summary.py) of `kernel` for THIS library
    build (its lib_sha256 must match the loaded library's digest): (dict, file name) or (None, why)."""
    import amc_lba
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"pmc_{kernel}_*.json")))
    digest = amc_lba.lib_digest()
    stale = []
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("workload") != workload:
            continue
        if d.get("lib_sha256") != digest:
            stale.append(os.path.basename(f))
            continue
        return d, os.path.basename(f)
    return None, (f"no PMC summary of this library build ({digest}); stale: {stale}" if stale else "no PMC summary")


def pmc_traffic(workload, kernel="k_lin_schur"):
    """HBM bytes per launch of the kernel from the committed rocprofv3 PMC summary (FETCH_SIZE
    doubled per the gfx950 correction + WRITE_SIZE, MI355X_MICROARCH.md §HBM) of THIS library build
    (the summary's lib_sha256 must match the loaded library's digest), or (None, why)."""
    import amc_lba
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"pmc_{kernel}_*.json")))
    digest = amc_lba.lib_digest()
    stale = []
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("workload") != workload or not d.get("hbm_bytes_per_launch"):
            continue
        if d.get("lib_sha256") != digest:
            stale.append(os.path.basename(f))
            continue
        return float(d["hbm_bytes_per_launch"]), os.path.basename(f)
    return None, (f"no PMC summary of this library build ({digest}); stale: {stale}" if stale else "no PMC summary")


def cpu_model():
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline_omp(config, seconds, threads):
    """The same oracle built with OpenMP (oracle/_build/liblba_oracle_omp.so: the per-edge error and
    Jacobian passes, the landmark inverses, the Schur complement by pose-block rows and the landmark
    back-substitution on `threads` threads, like g2o's G2O_USE_OPENMP build, block_solver.hpp:378-380,527;
    the dense LDLT stays serial as Eigen's is; results bitwise the serial build's), timed in a child
    process (the other library) on the same window."""
    env = dict(os.environ, ORC_LIB=os.path.join(ROOT, "oracle", "_build", "liblba_oracle_omp.so"),
               OMP_NUM_THREADS=str(threads), _BENCH_OMP_CHILD="1")
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "--config", config, "--cpu-seconds", str(seconds)],
                       env=env, capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        return {"error": r.stderr[-300:]}
    d = json.loads(r.stdout.strip().splitlines()[-1])
    d.update({"cores": threads, "kind": "port", "cpu": cpu_model()})
    return d


def cpu_baseline(win, seconds):
    """The oracle (C restatement of the reference CPU path, single thread, like the reference's
    G2O_USE_OPENMP OFF build) on the same window: a bounded number of LM iterations."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import orc
    o = orc.Oracle(win, early_stop=0)
    t = time.perf_counter()
    o.optimize(1)
    t_cal = time.perf_counter() - t
    n = int(max(1, min(50, round(seconds / max(t_cal, 1e-6)))))
    o2 = orc.Oracle(win, early_stop=0)
    t = time.perf_counter()
    n_run, _ = o2.optimize(n)
    dt = time.perf_counter() - t
    threads = os.environ.get("OMP_NUM_THREADS") if orc.LIB.endswith("_omp.so") else "1"
    return {"value": n_run / dt, "unit": "LM iterations/s", "cores": 1, "kind": "port", "cpu": cpu_model(),
            "sample": f"{n_run} LM iterations of the same {win.name} window, oracle/{os.path.basename(orc.LIB)} "
                      f"(-O3, {threads} thread(s)), {dt:.1f} s"}


def localgpba_map_calls(device, passes=3, seed=7):
    """The caller's real window (SURVEY.md 8(d), round-5 verdict item 6): Optimizer::LocalGPBA as LocalMapping calls it
    (src/LocalMapping.cc:131, once per new keyframe; src/Optimizer.cc:713-1432) through the C++ host adapter
    lbamap_local_gpba -- the temporal window of the keyframe (10 keyframes, or 25 with bLarge), its covisible / fixed
    keyframes and local points, set-up, optimize(10), the outlier post-pass and the write-back, all in the call -- on a
    synthetic 40-keyframe, 4-camera map, called for keyframes 20..39 in order as the mapping thread would (every call
    updates the map), `passes` times from a fresh map (the first call of a map creates its engine and is not timed).
    Beside it the same windows' LM on the CPU oracle (lbamap_build_window's flat window from a fresh map, then
    optimize(10); one thread, and the OpenMP build) on every fifth of those windows (the oracle takes seconds per
    window).  The CPU rate counts the LM only (the adapter's window build, C++ in both, is reported beside it: through
    Python here it is an upper bound)."""
    from amc_lba import mapsnap as ms
    from amc_lba.abi import make_config
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import orc
    snap = ms.make_map(n_kf=40, n_lm=8000, obs_per_lm=6, n_cam=4, seed=seed)
    kfs = list(range(20, 40))
    out = {}
    for large in (False, True):
        times, parts, bad = [], [], 0
        for _ in range(passes):
            m = ms.LocalGPBAMap(snap)
            for i, kf in enumerate(kfs):
                t = time.perf_counter()
                rc, res = m.local_gpba(kf, large=large, device=device)
                dt = time.perf_counter() - t
                bad += rc != 0
                if i > 0:
                    times.append(dt)
                    parts.append(list(res.ms_phase))
            m.close()
        m = ms.LocalGPBAMap(snap)
        wins, t_build = [], 0.0
        for kf in kfs:
            t = time.perf_counter()
            W, _, _, _ = m.build_window(kf, large=large)
            t_build += time.perf_counter() - t
            wins.append(W)
        m.close()
        t_build /= len(kfs)
        # the call's two engine parts on the same windows (one engine, as the adapter's): lba_set_problem and
        # lba_optimize(10); the rest of a call is the adapter's C++ window build, post-pass and write-back
        import amc_lba
        p = amc_lba.Problem(wins[0], device=device)
        p.optimize(10)
        t_set, t_opt10, ph = [], [], []
        for W in wins[1:]:
            t = time.perf_counter()
            p.set_window(W)
            t_set.append(time.perf_counter() - t)
            ph.append(p.setup_phases())
            t = time.perf_counter()
            p.optimize(10)
            t_opt10.append(time.perf_counter() - t)
        p.close()
        cpu = {}
        sample = wins[4::5]
        for tag, lib_omp in (("1_thread", False), ("openmp", True)):
            t_opt = 0.0
            for W in sample:
                o = orc.Oracle(W, cfg=make_config(**W.cfg), omp=lib_omp)
                t = time.perf_counter()
                o.optimize(10)
                t_opt += time.perf_counter() - t
            t_opt /= len(sample)
            cpu[tag] = {"calls_per_s": 1.0 / t_opt, "optimize_ms": t_opt * 1e3, "windows": len(sample)}
        cpu["openmp"]["threads"] = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or None
        g = float(np.mean(times))
        out["large" if large else "normal"] = {
            "window_keyframes_mean": float(np.mean([len(W.kfs) for W in wins])),
            "optimisable_kf_mean": float(np.mean([int((W.kfs["fixed"] == 0).sum()) for W in wins])),
            "landmarks_mean": float(np.mean([len(W.lm) for W in wins])),
            "observations_mean": float(np.mean([len(W.obs) for W in wins])),
            "gpu_calls_per_s": 1.0 / g, "gpu_ms_per_call_mean": g * 1e3,
            "gpu_ms_per_call_median": float(np.median(times)) * 1e3, "calls_timed": len(times), "failed_calls": bad,
            "call_parts_ms_median": dict(zip(("window_build", "set_problem", "optimize", "post_pass_write_back"),
                                             np.median(np.array(parts), axis=0).tolist())),
            "engine_set_problem_ms_median": float(np.median(t_set)) * 1e3,
            "engine_optimize10_ms_median": float(np.median(t_opt10)) * 1e3,
            "engine_set_problem_phases_ms_median": {k: float(np.median([d[k] for d in ph])) for k in ph[0]},
            "window_build_ms_python": t_build * 1e3, "cpu_oracle": cpu,
            "speedup_vs_cpu_1_thread": (1.0 / g) / cpu["1_thread"]["calls_per_s"]}
    out["note"] = ("lbamap_local_gpba per call: window build + lba_set_problem + lba_optimize(10) + post-pass + "
                   "write-back (synthetic 40-keyframe map, 8000 points, 4 cameras, keyframes 20..39 in order); CPU: "
                   "optimize(10) of the same windows (every fifth) through oracle/ (a C restatement of g2o's LM, not "
                   "g2o itself), the window build not counted")
    return out


def main():
    if os.environ.get("_BENCH_OMP_CHILD"):   # cpu_baseline_omp's child: the oracle alone, one JSON line
        ap = argparse.ArgumentParser()
        ap.add_argument("--config", default="cfg1_local_50kf")
        ap.add_argument("--cpu-seconds", type=float, default=12.0)
        a, _ = ap.parse_known_args()
        from amc_lba.synth import make_config_window
        print(json.dumps(cpu_baseline(make_config_window(a.config), a.cpu_seconds)), flush=True)
        return
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=None,
                    help="untimed LM iterations before the timed ones (default: 100 for config 1, ~20 ms of work that "
                         "brings the GPU to its steady clocks -- 5 left the 20-step value ~2 %% low, "
                         "profiles/r8g_warmup.txt; 5 for config 0, whose small window converges within 100 and then "
                         "rejects trials; 2 for the global-BA configs, whose iterations take ms each)")
    ap.add_argument("--config", default="cfg1_local_50kf")
    ap.add_argument("--window-iters", type=int, default=10, help="LM iterations per window (LocalGPBA optimize(10))")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--seed", type=int, default=20250912)
    ap.add_argument("--sweep-events", choices=("every", "sampled", "off"), default="sampled",
                    help="HIP events around k_lin_schur / k_chol_flow dispatches in the timed run: every trial, "
                         "every 10th trial (default: the events idle the device ~5 us each) or none")
    ap.add_argument("--gba-solve", choices=("split", "replicated"), default="split",
                    help="config 4 over N ranks: distributed factorisation (default) or the replicated solve")
    ap.add_argument("--solve", choices=("auto", "band", "dense"), default="auto",
                    help="reduced-system solve: L^-1 tiles (dense) or substitution (band); auto picks by size")
    ap.add_argument("--dry-launch", action="store_true",
                    help="with --gpus N > 1 and no launcher: print the rank launch and exit (no GPU)")
    ap.add_argument("--f32-residual", action="store_true",
                    help="BASELINE configs[4]'s fp32 residuals + fp64 accumulate (LBA_FLAG_F32_RESIDUAL; default fp64)")
    args = ap.parse_args()
    if args.warmup is None:   # (from the name: nothing may load the library before launch_ranks)
        args.warmup = 100 if args.config == "cfg1_local_50kf" else (2 if "global" in args.config else 5)
    rc = launch_ranks(args, sys.argv[1:])
    if rc is not None:
        sys.exit(rc)
    if os.environ.get("_BENCH_RANK_PROBE"):   # (tests: a launched rank reports its environment, no GPU)
        # (one write(2) of the whole line, under PIPE_BUF: the ranks share the pipe, and print's separate writes of
        # the text and the newline could interleave with another rank's)
        os.write(1, (json.dumps({k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                                                  "HSA_ENABLE_IPC_MODE_LEGACY")}) + "\n").encode())
        return

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import amc_lba
    from amc_lba import farm
    from amc_lba.synth import make_config_window

    # global BA (config 4): one problem partitioned over the ranks (--gba-solve split: the distributed
    # factorisation, each rank factors its subtree of the nested dissection and the top separators' tiles are
    # all-reduced over RCCL every LM trial; replicated: landmarks l % N, the whole reduced system all-reduced and
    # factored by every rank); otherwise window farming (config 3) or a single window
    gba = args.config.startswith("cfg4")
    solve_flag = {"auto": 0, "band": amc_lba.abi.FLAG_BAND_SOLVE, "dense": amc_lba.abi.FLAG_DENSE_SOLVE}[args.solve]
    if args.f32_residual:
        solve_flag |= amc_lba.abi.FLAG_F32_RESIDUAL
    # the timed run records the dispatch timestamps of every k_lin_schur and k_chol_flow launch
    # (LBA_FLAG_TIME_SWEEP): the rooflines below are measured live, per launch, over the timed region
    flags = solve_flag | {"every": amc_lba.abi.FLAG_TIME_SWEEP, "off": 0,
                          "sampled": amc_lba.abi.FLAG_TIME_SWEEP | amc_lba.abi.FLAG_TIME_SAMPLED}[args.sweep_events]
    ex, full = None, None
    t_setup = time.perf_counter()
    # large set-ups (config 4: ~35 s of window generation, then the engine's preprocessing) report
    # progress, so a watchdog that looks for output does not take them for a hang
    import threading
    setup_done = threading.Event()

    def _progress():
        while not setup_done.wait(20.0):
            print(f"[bench rank {rank}] setting up ({time.perf_counter() - t_setup:.0f} s)", file=sys.stderr, flush=True)
    threading.Thread(target=_progress, daemon=True).start()
    if gba:
        from amc_lba.gba import partition_window
        full = make_config_window(args.config, seed=args.seed)
        split = world > 1 and args.gba_solve == "split"
        win, _ = partition_window(full, rank, world, amc_lba.partition_assign(full, world) if split else None)
        if split:
            flags |= amc_lba.abi.FLAG_SUBTREE_SOLVE
        rid = None
        if world > 1:
            idt = torch.zeros(128, dtype=torch.uint8, device=torch.device("cuda", local))
            if rank == 0:
                idt.copy_(torch.frombuffer(bytearray(amc_lba.rccl_unique_id()), dtype=torch.uint8))
            dist.broadcast(idt, 0)
            rid = bytes(idt.cpu().numpy().tobytes())
        prob = amc_lba.Problem(win, device=local, early_stop=0, flags=flags, rccl_id=rid, rank=rank, nranks=world)
    else:
        if world > 1:
            win, shared = farm.make_rank_window(args.config, rank, world, seed=args.seed)
        else:
            win = make_config_window(args.config, seed=args.seed)
        prob = amc_lba.Problem(win, device=local, early_stop=0, flags=flags)
        if world > 1:
            # window-boundary exchange inside the engine: its own RCCL communicator (in-place
            # ncclAllGather on the window's stream), owner -> slot tables matched once here
            idt = torch.zeros(128, dtype=torch.uint8, device=torch.device("cuda", local))
            if rank == 0:
                idt.copy_(torch.frombuffer(bytearray(amc_lba.rccl_unique_id()), dtype=torch.uint8))
            dist.broadcast(idt, 0)
            prob.set_farm_rccl(bytes(idt.cpu().numpy().tobytes()), rank, world)
            ex = farm.DeviceExchange(prob, win, shared)
    t_setup = time.perf_counter() - t_setup
    setup_done.set()

    # warmup (not timed)
    sinfo = prob.solver_info()   # (panels, tiles, chain, dissection levels, fill: reported below)
    try:
        sflops = prob.solver_flops()   # (the solve's algorithmic FLOPs below)
    except AttributeError:             # (an older library under A/B)
        sflops = (float("nan"), float("nan"))
    if args.warmup > 0:
        prob.optimize(args.warmup)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    done, ms_k, n_k, trials, ms_s, n_s = 0, 0.0, 0, 0, 0.0, 0
    while done < args.steps:
        it = min(args.window_iters, args.steps - done)
        n, st = prob.optimize(it)
        done += n
        ms_k += st.ms_k_linearize
        n_k += st.n_k_linearize
        ms_s += st.ms_k_solve
        n_s += st.n_k_solve
        trials += st.trials
        if ex is not None:
            ex.exchange()               # window boundary: publish owned shared keyframes / landmarks
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([dt], device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())

    # per-kernel launch durations for the rooflines: the timed run carries events on one trial in ten only (they idle
    # the device ~5 us each); a further, untimed optimize with events on every trial's k_lin_schur and k_chol_flow
    # dispatches averages >= 20 launches of each (the same problem, continuing from the timed run's state)
    meas_iters = max(20, args.window_iters)
    cfg_m = amc_lba.abi.LbaConfig.from_buffer_copy(prob.cfg)
    cfg_m.flags = (cfg_m.flags | amc_lba.abi.FLAG_TIME_SWEEP) & ~amc_lba.abi.FLAG_TIME_SAMPLED
    prob._check(amc_lba.lib().lba_set_config(prob.h, ctypes.byref(cfg_m)))
    mk_ms, mk_n, ms_ms, ms_n = 0.0, 0, 0.0, 0
    while mk_n < meas_iters:
        _, st_m = prob.optimize(args.window_iters)
        mk_ms += st_m.ms_k_linearize
        mk_n += st_m.n_k_linearize
        ms_ms += st_m.ms_k_solve
        ms_n += st_m.n_k_solve
        if st_m.n_k_linearize == 0:
            break
    prob._check(amc_lba.lib().lba_set_config(prob.h, ctypes.byref(prob.cfg)))

    # the data-path collectives, measured after the timed region (untimed): the farm's window-boundary
    # exchange (pack, in-place ncclAllGather, unpack on the window's stream) and, for the distributed global-BA
    # factorisation, an RCCL all-reduce of the per-trial size over the same ranks
    comm = None
    if world > 1 and ex is not None:
        cnt = torch.tensor([float(ex.counts[0]), float(ex.counts[1])], device="cuda")
        allc = [torch.zeros_like(cnt) for _ in range(world)]
        dist.all_gather(allc, cnt)
        kcap = int(max(c[0].item() for c in allc))
        lcap = int(max(c[1].item() for c in allc))
        stride_b = (13 * kcap + 3 * lcap) * 8
        reps = 20
        torch.cuda.synchronize()
        dist.barrier()
        t = time.perf_counter()
        for _ in range(reps):
            ex.exchange()
        torch.cuda.synchronize()
        te = torch.tensor([(time.perf_counter() - t) / reps], device="cuda")
        dist.all_reduce(te, op=dist.ReduceOp.MAX)
        comm = {"kind": "window-boundary exchange (k_farm_pack, in-place ncclAllGather, k_farm_unpack)",
                "bytes_per_rank": stride_b, "bytes_gathered": stride_b * world,
                "us_per_boundary": float(te.item()) * 1e6, "boundaries_timed": (done + args.window_iters - 1) //
                args.window_iters, "published": {"kf": ex.counts[0], "lm": ex.counts[1]},
                "received": {"kf": ex.counts[2], "lm": ex.counts[3]}}
    elif world > 1 and gba:
        si = prob.split_info()
        nb = int(si["allreduce_bytes"])
        buf = torch.ones(max(nb // 8, 1), dtype=torch.float64, device="cuda")
        reps = 20
        for _ in range(3):
            dist.all_reduce(buf)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(reps):
            dist.all_reduce(buf)
        torch.cuda.synchronize()
        te = torch.tensor([(time.perf_counter() - t) / reps], device="cuda")
        dist.all_reduce(te, op=dist.ReduceOp.MAX)
        comm = {"kind": ("per-trial all-reduce of the top separators' tiles + bS + b_p" if args.gba_solve == "split"
                         else "per-trial all-reduce of every tile of S + bS + b_p"),
                "bytes_per_trial": nb, "replicated_bytes_per_trial": int(si["replicated_allreduce_bytes"]),
                "us_per_trial": float(te.item()) * 1e6,
                "timing": "torch.distributed all_reduce (RCCL) of the same byte count over the same ranks, after the "
                          "timed region",
                "rank_flops_share": si["rank_flops"] / max(si["system_flops"], 1.0)}

    phase, set_problem_ms, set_problem_phases = None, None, None
    if world == 1:
        # phase breakdown from a separate, untimed run with every phase evented
        prob.close()
        ph = amc_lba.Problem(win, device=local, early_stop=0, flags=amc_lba.abi.FLAG_TIME_PHASES | solve_flag)
        n_ph, st_ph = ph.optimize(args.window_iters)
        # per LM iteration: k_lin_schur (linearisation + landmark elimination, every trial), k_expand +
        # k_assemble, the reduced-system solve, k_update + k_eval
        phase = {name: getattr(st_ph, k) / max(n_ph, 1) for name, k in
                 (("lin_schur", "ms_linearize"), ("expand_assemble", "ms_schur"), ("solve", "ms_solve"),
                  ("update_eval", "ms_update_eval"))}
        phase["trials"] = st_ph.trials / max(n_ph, 1)
        # one LocalGPBA call = lba_set_problem (host preprocessing of the window + host->device upload,
        # outside the timed region above) + optimize(window_iters): time a set_problem on the engine
        kfs, lm, obs, pri, vel, cams = ph._keep
        L = amc_lba.lib()
        sp, sp_ph = [], []   # (median of seven set-ups: one sample is at the mercy of the host's scheduling)
        for _ in range(7):
            t_sp = time.perf_counter()
            rc = L.lba_set_problem(ph.h, amc_lba.ptr(kfs), len(kfs), amc_lba.ptr(lm), len(lm), amc_lba.ptr(obs),
                                   len(obs), amc_lba.ptr(pri), len(pri), amc_lba.ptr(vel), len(vel), amc_lba.ptr(cams),
                                   len(cams))
            torch.cuda.synchronize()
            sp.append((time.perf_counter() - t_sp) * 1e3 if rc == 0 else float("nan"))
            if rc == 0:
                sp_ph.append(ph.setup_phases())
        set_problem_ms = float(np.median(sp)) if all(np.isfinite(sp)) else None
        set_problem_phases = ({k: float(np.median([d[k] for d in sp_ph])) for k in sp_ph[0]} if sp_ph else None)
        ph.close()
    if rank == 0:
        # window farm: every rank runs its own window (weak scaling); global BA: one problem (strong)
        total_iters = done if gba else done * world
        W = full if gba else win
        value = total_iters / dt
        # launch averages from the dedicated run (the timed run's sampled events are reported beside them)
        live_k_ms, live_s_ms = ms_k / max(n_k, 1), ms_s / max(n_s, 1)
        if mk_n:
            ms_k, n_k = mk_ms, mk_n
        if ms_n:
            ms_s, n_s = ms_ms, ms_n
        k_ms = ms_k / max(n_k, 1)
        B_schur, F_schur = schur_terms(win)
        B = sweep_bytes(win) + B_schur
        B_s8d = s8d_sweep_bytes(win)
        F = sweep_flops(win) + F_schur
        s_ms = ms_s / max(n_s, 1)
        npose = 12 * int((win.kfs["fixed"] == 0).sum())
        # algorithmic FLOPs of one solve from the symbolic structure of L (lba_solver_flops): the tile
        # factorisation + the two substitutions (dense Cholesky np^3/3 when the system has no sparsity)
        F_fac, F_sub = sflops
        F_solve = F_fac + F_sub
        solve_note = ("tile Cholesky of the nested-dissection-ordered reduced camera system: per column with m "
                      "tiles below the diagonal 32^3/3 + 2 m 32^3 + m (m - 1) 32^3, plus two substitutions "
                      "(lba_solver_flops, exact for the symbolic structure); the dependent panel chain, not the "
                      "FLOPs, sets its time")
        # SURVEY.md 8(d)'s algorithmic FLOPs of the dense solve: n^3 / 3 + 2 n^2, n = 12 n_kf_opt.  That is the local
        # window's solver (LinearSolverDense, linear_solver_dense.h:65-113); the global-BA shapes go through the sparse
        # LinearSolverEigen (linear_solver_eigen.h:94-124), whose work is the symbolic structure's: their solve is
        # priced in the structural FLOPs (the dense count of a 60k-dof system would put the kernel far above peak)
        from amc_lba.synth import CONFIGS
        glob_shape = bool(CONFIGS.get(args.config, {}).get("global_ba"))
        F_s8d = npose ** 3 / 3.0 + 2.0 * npose ** 2
        F_price = F_solve if glob_shape else F_s8d
        price_note = ("the symbolic structure's FLOPs (lba_solver_flops): the reference's global BA solves with the "
                      "sparse LinearSolverEigen" if glob_shape else
                      "SURVEY.md 8(d): n^3/3 + 2 n^2, n = 12 n_kf_opt (the dense LDLT's count)")
        chol_pmc, chol_pmc_src = pmc_summary(args.config, "k_chol_flow")
        achieved = B / (k_ms * 1e-3) / 1e9 if n_k else None
        achieved_f = F / (k_ms * 1e-3) / 1e12 if n_k else None
        workload = f"{args.config}: {win.name or args.config} synthetic window"
        traffic, traffic_src = pmc_traffic(args.config)
        line = {
            "metric": metric_for(args.config, W),
            "value": value,
            "unit": "LM iterations/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt * 1e3 / done,
            "higher_is_better": True,
            "scaling": "strong" if gba else "weak",
            "vs_baseline": None,
            "dtype": "f32 residuals + f64 accumulate" if args.f32_residual else "f64",
            "data": "synthetic (deterministic generator, amc_lba/synth.py, seed %d)" % args.seed,
            "config": {"workload": workload, "n_kf": int(len(W.kfs)), "n_opt_kf": int((W.kfs["fixed"] == 0).sum()),
                       "n_lm": int(len(W.lm)), "n_obs": int(len(W.obs)), "n_pairs": int(W.n_pairs),
                       "n_cam": int(len(W.cams)), "window_iters": args.window_iters, "solve": args.solve,
                       "parallelism": ((f"distributed factorisation x{world} (subtree per rank, RCCL all-reduce of the "
                                        "top per trial)" if args.gba_solve == "split" else
                                        f"landmark partition x{world} (RCCL all-reduce per trial)") if gba else
                                       f"window farm x{world}") if world > 1 else "single window",
                       "window_build_and_setup_s": t_setup},   # (the synthetic window generation in Python + lba_set_problem)
            # the sweep's algorithmic intensity (F / B ~ 44 FLOP/B at config 1) is above the fp64 ridge point
            # (78.6 TF / 8 TB/s ~ 10 FLOP/B): its roofline is fp64 compute; the HBM view is kept beside it
            "roofline": {"bound": "mfma", "kernel": "k_lin_schur", "achieved": achieved_f,
                         "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": (achieved_f / FP64_PEAK_TFLOPS) if n_k else None,
                         "traffic": traffic, "traffic_source": traffic_src, "flops_per_launch": F,
                         "bytes_per_launch": B, "intensity_flop_per_byte": F / B,
                         "avg_launch_ms": k_ms, "timed_launches": n_k,
                         "note": "fp64 (VALU FMAs and v_mfma_f64) against the 78.6 TF fp64 peak"},
            # SURVEY.md §8(d)'s figure, the one the north-star's >= 70 % HBM target is quoted on
            "roofline_s8d": {"kernel": "k_lin_schur", "bound": "hbm", "bytes_per_launch": B_s8d,
                             "achieved": B_s8d / (k_ms * 1e-3) / 1e9 if n_k else None, "peak": HBM_PEAK_GBS,
                             "unit": "GB/s", "frac": (B_s8d / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS) if n_k else None,
                             "note": "72 n_obs + 288 n_pairs + 96 n_lm + 2 (1152 n_kfpairs + 96 n_kf) over the live "
                                     "average k_lin_schur launch"},
            "roofline_hbm": {"kernel": "k_lin_schur", "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                             "unit": "GB/s", "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                             "bytes_per_launch": B, "traffic": traffic, "traffic_source": traffic_src},
            "roofline_solve": {"kernel": "k_chol_flow", "bound": "mfma", "flops_per_launch": F_price,
                               "achieved": F_price / (s_ms * 1e-3) / 1e12 if n_s else None,
                               "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                               "frac": (F_price / (s_ms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS) if n_s else None,
                               "traffic": (chol_pmc or {}).get("hbm_bytes_per_launch"), "traffic_source": chol_pmc_src,
                               "avg_launch_ms": s_ms, "timed_launches": n_s,
                               "flops_note": price_note, "flops_s8d_dense": F_s8d,
                               "flops_structural": F_solve,
                               "frac_structural": (F_solve / (s_ms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS) if n_s else None,
                               "note": solve_note,
                               "solver": sinfo, "flops_factor": F_fac, "flops_substitution": F_sub},
            "live_sampled_ms": {"k_lin_schur": live_k_ms, "k_chol_flow": live_s_ms,
                                "note": "the timed run's own sampled dispatch events (one trial in ten)"},
            "trials_per_step": trials / max(done, 1),
            "phases_ms_per_step": phase,
        }
        # the contract's `roofline` is the DOMINANT kernel's (the longer average launch); the sweep's stays beside it
        line["roofline_sweep"] = line["roofline"]
        if chol_pmc is not None:
            sq = chol_pmc.get("sq_per_launch_median", {})
            line["roofline_solve"]["mfma_pmc"] = {
                "mfma_f64_flops_per_launch": sq.get("mfma_f64_flops"),
                "mfma_busy_frac_of_all_simds": sq.get("mfma_busy_frac_of_all_simds"),
                "SQ_INSTS_VALU_MFMA_F64": sq.get("SQ_INSTS_VALU_MFMA_F64"),
                "SQ_INSTS_VALU_FMA_F64": sq.get("SQ_INSTS_VALU_FMA_F64"),
                "source": chol_pmc_src}
        if gba:   # the sweep's figures are rank 0's landmark partition's
            line["roofline_sweep"]["note"] = "k_lin_schur of rank 0's landmark partition"
        if n_s and s_ms > k_ms:
            line["roofline"] = dict(line["roofline_solve"], dominant=True)
        else:
            line["roofline"] = dict(line["roofline_sweep"], dominant=True)
        if comm is not None:
            line["collective"] = comm
        if world == 1 and not gba:   # LocalGPBA-equivalent calls (optimize(window_iters))
            calls = {"optimize_calls_per_s": value / args.window_iters, "set_problem_ms": set_problem_ms,
                     "set_problem_phases_ms": set_problem_phases}
            if set_problem_ms is not None:
                calls["calls_per_s_with_set_problem"] = 1.0 / (args.window_iters / value + set_problem_ms * 1e-3)
            line["localgpba_calls"] = calls
            if not args.no_cpu and args.config == "cfg1_local_50kf":
                line["localgpba_map_calls"] = localgpba_map_calls(local)
        if not args.no_cpu and world == 1 and not gba:   # (the oracle's dense LDLT of S = 60000^2 is hours)
            line["cpu_baseline"] = cpu_baseline(win, args.cpu_seconds)
            # secondary: the OpenMP build of the oracle on this rank's share of the host's cores
            # (OMP_NUM_THREADS: the GPU box's CPU share for one GPU, 16 on this pool; os.cpu_count() is the whole
            # machine's, which the pool does not let one GPU's job occupy)
            omp_threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
            line["cpu_baseline_omp"] = cpu_baseline_omp(args.config, args.cpu_seconds, omp_threads)
            line["cpu_baseline_omp"]["nproc"] = os.cpu_count()
            # speed-up against the best CPU baseline measured (both are ports of g2o's algorithm, oracle/,
            # not g2o itself: the reference's build is not available here)
            cands = [("port, 1 thread", line["cpu_baseline"].get("value"))]
            if line["cpu_baseline_omp"] and line["cpu_baseline_omp"].get("value"):
                cands.append((f"port, OpenMP {line['cpu_baseline_omp'].get('cores')} threads",
                              line["cpu_baseline_omp"]["value"]))
            best = max((c for c in cands if c[1]), key=lambda c: c[1])
            line["speedup_vs_cpu"] = {"value": value / best[1], "against": best[0],
                                      "all": {k: value / v for k, v in cands if v}}
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
