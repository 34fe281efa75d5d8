"""Bitwise comparison of LM runs between two builds of the engine (A/B of a kernel change that must not move a
result bit): python scripts/cmp_libs.py <lib A> <lib B> [config] -- each build in its own child process."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(cfg):
    sys.path.insert(0, os.path.join(ROOT, "amc-slam_amd"))
    import numpy as np
    from amc_lba import Problem
    from amc_lba.synth import make_config_window
    win = make_config_window(cfg)
    p = Problem(win, early_stop=0)
    n, st = p.optimize(10)
    kf, lm = p.state()
    h = lambda a: __import__("hashlib").sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]   # noqa: E731
    print(json.dumps({"n": n, "trials": st.trials, "chi2": st.chi2_final, "kf_t": h(kf["t"]), "kf_q": h(kf["q"]),
                      "lm": h(lm)}))


if __name__ == "__main__":
    if sys.argv[1] == "--child":
        child(sys.argv[2])
        sys.exit(0)
    cfg = sys.argv[3] if len(sys.argv) > 3 else "cfg1_local_50kf"
    out = []
    for lib in sys.argv[1:3]:
        env = dict(os.environ, AMC_LBA_LIB=lib) if lib != "main" else dict(os.environ)
        r = subprocess.run([sys.executable, __file__, "--child", cfg], env=env, capture_output=True, text=True, timeout=300)
        out.append(json.loads(r.stdout.strip().splitlines()[-1]))
        print(lib, out[-1])
    print("bitwise identical" if out[0] == out[1] else "DIFFERENT")
