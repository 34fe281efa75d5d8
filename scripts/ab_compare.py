"""A/B of library builds / set-up variants on one window: final state after optimize(N) (bitwise
comparison against the first variant) and LM iterations per second over repeated optimize(10) calls.

    python scripts/ab_compare.py --variant base: --variant dpp:AMC_LBA_LIB=amc-slam_amd/lib/exp/x.so \
        --variant unfused:LBA_NO_FUSED_EVAL=1 [--config cfg1_local_50kf] [--calls 30]

Each variant runs in its own process (its environment selects the build and the set-up knobs).
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

if os.environ.get("_AB_CHILD"):
    sys.path.insert(0, os.path.join(ROOT, "amc-slam_amd"))
    import amc_lba
    from amc_lba.synth import make_config_window
    cfg, iters, calls, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    extra = json.loads(sys.argv[5]) if len(sys.argv) > 5 else {}
    w = make_config_window(cfg, **extra)
    p = amc_lba.Problem(w, early_stop=0)
    n, st = p.optimize(iters)
    kfs, lm = p.state()
    np.savez(out, kq=kfs["q"], kt=kfs["t"], kv=kfs["vel"], lm=lm, chi=np.array([st.chi2_initial, st.chi2_final]),
             n=np.array([n]))
    p.close()
    # timing: repeated optimize(10) from the same start (set_state back to the window's initial estimate)
    p = amc_lba.Problem(w, early_stop=0)
    k0, l0 = p.state()
    p.optimize(10)
    its, t = 0, 0.0
    for _ in range(calls):
        p.set_state(k0, l0)
        t0 = time.perf_counter()
        m, _ = p.optimize(10)
        t += time.perf_counter() - t0
        its += m
    print(json.dumps({"its_per_s": its / t, "ms_per_it": 1e3 * t / its, "iters": int(n),
                      "chi2": [st.chi2_initial, st.chi2_final]}), flush=True)
    sys.exit(0)

ap = argparse.ArgumentParser()
ap.add_argument("--variant", action="append", required=True, help="name:ENV=VAL,ENV=VAL")
ap.add_argument("--config", default="cfg1_local_50kf")
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--calls", type=int, default=30)
ap.add_argument("--window-kw", default="{}", help="extra make_config_window keywords (JSON)")
ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "ab"))
args = ap.parse_args()
os.makedirs(args.out, exist_ok=True)
ref = None
for v in args.variant:
    name, _, envs = v.partition(":")
    env = dict(os.environ, _AB_CHILD="1")
    for kv in filter(None, envs.split(",")):
        k, _, val = kv.partition("=")
        env[k] = val if not val.startswith("amc-slam_amd/") else os.path.join(ROOT, val)
    path = os.path.join(args.out, f"{args.config}_{name}.npz")
    r = subprocess.run([sys.executable, os.path.abspath(__file__), args.config, str(args.iters), str(args.calls), path,
                        args.window_kw], env=env, capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        print(f"{name}: FAILED rc={r.returncode}\n{r.stderr[-2000:]}", flush=True)
        sys.exit(1)
    res = json.loads(r.stdout.strip().splitlines()[-1])
    d = dict(np.load(path))
    if ref is None:
        ref = d
        same = "reference"
    else:
        diffs = {k: float(np.max(np.abs(d[k] - ref[k]))) for k in ref if d[k].shape == ref[k].shape}
        bad = {k: x for k, x in diffs.items() if x != 0.0}
        same = "bitwise identical" if not bad else f"differs: {bad}"
    print(f"{name:12s} {res['its_per_s']:8.1f} LM it/s  {res['ms_per_it']:.4f} ms/it  iters {res['iters']}  "
          f"chi2 {res['chi2'][1]:.10g}  {same}", flush=True)
