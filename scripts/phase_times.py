"""Per-phase cycle breakdown of k_lin_schur (linearisation phases, then elimination phases; diagnostics).

Runs a window with LBA_PHASE_TIMING set (the library then records clock64() at the phase boundaries of
every workgroup and dumps them when the problem is destroyed), then prints per-phase averages and how
the per-tile time depends on the tile shape.

    python scripts/phase_times.py [--config cfg1_local_50kf] [--iters 3] [--out gpurun_out/phases.txt]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "amc-slam_amd"))

LIN_PHASES = ["obs residual+J1 -> LDS", "sample M/g", "Hll/bl (+Dinv, LDL)", "Hpl = N^T G"]
SCHUR_PHASES = ["W = Hpl L^-T", "S partials (VALU)", "rhs partials"]
SHAPE = ["nobs", "nsmp", "npair", "nlm", "nsent", "nkf"]


def load(path):
    raw = open(path, "rb").read()
    nt = int(np.frombuffer(raw[:4], np.int32)[0])
    off = 4
    lin = np.frombuffer(raw[off:off + nt * 16 * 8], np.uint64).reshape(nt, 16).astype(np.int64)
    off += nt * 16 * 8
    sch = np.frombuffer(raw[off:off + nt * 16 * 8], np.uint64).reshape(nt, 16).astype(np.int64)
    off += nt * 16 * 8
    shape = np.frombuffer(raw[off:off + 6 * nt * 4], np.int32).reshape(6, nt)
    off += 6 * nt * 4
    chol = bs = cft = None
    if len(raw) > off:
        nb = int(np.frombuffer(raw[off:off + 4], np.int32)[0])
        off += 4
        chol = np.frombuffer(raw[off:off + nb * 16 * 8], np.uint64).reshape(nb, 16).astype(np.int64)
        off += nb * 16 * 8
        bs = np.frombuffer(raw[off:off + nb * 16 * 8], np.uint64).reshape(nb, 16).astype(np.int64)
        off += nb * 16 * 8
        W = 8 + 2 * 16   # CF_TDBG_STRIDE
        if len(raw) >= off + 4096 * W * 8:
            cft = np.frombuffer(raw[off:off + 4096 * W * 8], np.uint64).reshape(4096, W).astype(np.int64)
    return nt, lin, sch, shape, chol, bs, cft


def report(name, stamps, phases, shape, out):
    live = stamps[:, len(phases)] != 0   # (segment tiles of heavy landmarks have no elimination stamps)
    stamps, shape = stamps[live], shape[:, live]
    d = np.diff(stamps[:, :len(phases) + 1], axis=1)
    tot = stamps[:, len(phases)] - stamps[:, 0]
    out.append(f"== {name}: {stamps.shape[0]} workgroups, cycles per workgroup (clock64)")
    out.append(f"   total: mean {tot.mean():10.0f}  p50 {np.median(tot):10.0f}  p95 {np.percentile(tot, 95):10.0f}  max {tot.max():10.0f}")
    for i, ph in enumerate(phases):
        out.append(f"   {ph:24s} mean {d[:, i].mean():10.0f} ({100 * d[:, i].mean() / tot.mean():5.1f} %)  p95 {np.percentile(d[:, i], 95):10.0f}")
    for j, s in enumerate(SHAPE):
        v = shape[j].astype(float)
        c = np.corrcoef(v, tot)[0, 1] if v.std() > 0 else float("nan")
        out.append(f"   shape {s:6s} mean {v.mean():7.1f} max {v.max():6.0f}  corr(total) {c:+.2f}")


def timeline(lin, shape, out):
    """Wall-clock (s_memrealtime, 100 MHz) start / end of every tile workgroup of the last relinearising launch
    (slots 12 / 13; a gated launch returns before its first stamp and k_update's stamps of the same rows use
    slots 5..11 / 14 / 15): the span, how the tiles' start times spread (dispatch rounds) and which tiles end
    last."""
    st, en = lin[:, 12], lin[:, 13]
    ok = (st > 0) & (en > 0)
    if not ok.any():
        return
    st, en = st[ok], en[ok]
    idx = np.nonzero(ok)[0]
    t0 = st.min()
    s_us, e_us = (st - t0) / 100.0, (en - t0) / 100.0
    d = e_us - s_us
    out.append(f"== k_lin_schur timeline (us, tiles of the last launch): span {e_us.max():.2f}, tile duration "
               f"mean {d.mean():.2f} p50 {np.median(d):.2f} p95 {np.percentile(d, 95):.2f} max {d.max():.2f}")
    for q in (0.5, 0.75, 0.9, 1.0):
        out.append(f"   start time quantile {q:4.2f}: {np.quantile(s_us, q):7.2f}   end time quantile {q:4.2f}: {np.quantile(e_us, q):7.2f}")
    late = np.argsort(-e_us)[:8]
    for k in late:
        t = idx[k]
        out.append(f"   late tile {t:5d}: start {s_us[k]:6.2f} end {e_us[k]:6.2f} dur {d[k]:6.2f}  shape "
                   + " ".join(f"{n}={shape[j, t]}" for j, n in enumerate(SHAPE)))
    # a list-scheduling estimate: the measured durations on S slots, in index order vs longest first
    for slots in (768,):
        for name, order in (("index order", np.arange(len(d))), ("longest first", np.argsort(-d))):
            fin = np.zeros(slots)
            for k in order:
                j = fin.argmin()
                fin[j] += d[k]
            out.append(f"   list schedule on {slots} slots, {name}: makespan {fin.max():.2f} us")


def update_timeline(lin, n_gp, n_kfb, out):
    """k_update workgroups of the last launch (slots 14 / 15): GP-pair sample rebuilds, KF blocks,
    landmark blocks; when each kind ends."""
    st, en = lin[:, 14], lin[:, 15]
    ok = (st > 0) & (en > 0)
    if not ok.any():
        return
    t0 = st[ok].min()
    idx = np.nonzero(ok)[0]
    s_us, e_us = (st[ok] - t0) / 100.0, (en[ok] - t0) / 100.0
    out.append(f"== k_update timeline (us): span {e_us.max():.2f}")
    gpi = idx[idx < n_gp]
    if len(gpi) and (lin[gpi, 5] > 0).all():   # GP-pair rebuild phases (gp_pair_prep stamps, slots 5..10)
        cols = [14, 5, 6, 7, 8, 9, 10, 15]
        names = ["KF trial states + log(T12) + Ad(T12^-1)", "Jr^-1(xi12), ad(v2)", "w2, A1", "B1, D",
                 "sample lanes (exp, pose, Ad, Jr)", "N blocks", "tail"]
        d = np.diff(lin[np.ix_(gpi, cols)].astype(np.int64), axis=1) / 100.0
        out.append("   GP-pair rebuild phases (us, mean / max): " +
                   "; ".join(f"{nm} {d[:, k].mean():.2f} / {d[:, k].max():.2f}" for k, nm in enumerate(names)))
    tli = idx[idx >= n_gp + n_kfb]
    if len(tli) and (lin[tli, 5] > 0).all() and (lin[tli, 6] > 0).all():   # bs_tile stamps, slots 5 / 6
        d = np.diff(lin[np.ix_(tli, [14, 5, 6, 15])].astype(np.int64), axis=1) / 100.0
        out.append("   landmark-tile phases (us, mean / max): " +
                   "; ".join(f"{nm} {d[:, k].mean():.2f} / {d[:, k].max():.2f}"
                             for k, nm in enumerate(["t_s = N x", "observations G^T t", "landmarks, scale sum"])))
    for name, sel in (("GP pairs", idx < n_gp), ("KF blocks", (idx >= n_gp) & (idx < n_gp + n_kfb)),
                      ("landmark blocks", idx >= n_gp + n_kfb)):
        if sel.any():
            d = e_us[sel] - s_us[sel]
            out.append(f"   {name:16s} n {sel.sum():5d}  start max {s_us[sel].max():6.2f}  end max {e_us[sel].max():6.2f}  "
                       f"duration mean {d.mean():6.2f} max {d.max():6.2f}")


def exp_asm_timeline(sch, out):
    """k_exp_asm workgroups of the last launch (slots 8.. of the elimination rows; workgroups below n_tiles only):
    the sample expansions (start / expanded / published) and the assembly blocks (start / Schur partials in /
    samples in / stored)."""
    x = sch[:, 8:12]
    live = x[:, 0] > 0
    if not live.any():
        return
    t0 = x[live, 0].min()
    exp = live & (x[:, 3] == 0) & (x[:, 2] > 0)
    asm = live & (x[:, 3] > 0)
    f = lambda v: (v - t0) / 100.0   # noqa: E731
    out.append(f"== k_exp_asm timeline (us from the first workgroup's start): {exp.sum()} expansions, {asm.sum()} "
               f"assembly blocks stamped")
    if exp.any():
        e = x[exp]
        out.append(f"   expansions: start max {f(e[:, 0]).max():6.2f}  expanded mean {f(e[:, 1]).mean():6.2f} max "
                   f"{f(e[:, 1]).max():6.2f}  published max {f(e[:, 2]).max():6.2f}")
    if asm.any():
        a = x[asm]
        out.append(f"   assembly: start median {np.median(f(a[:, 0])):6.2f} max {f(a[:, 0]).max():6.2f}  partials in "
                   f"median {np.median(f(a[:, 1])):6.2f}  samples in median {np.median(f(a[:, 2])):6.2f} max "
                   f"{f(a[:, 2]).max():6.2f}  stored median {np.median(f(a[:, 3])):6.2f} max {f(a[:, 3]).max():6.2f}")
        a = a[(a[:, 1] > 0) & (a[:, 2] > 0)]   # (the rhs blocks have no partial / sample stamps)
        if len(a):
            out.append(f"   S-block durations (us): partial sums mean {(a[:, 1] - a[:, 0]).mean() / 100:5.2f}, wait for "
                       f"samples mean {(a[:, 2] - a[:, 1]).mean() / 100:5.2f}, rest mean {(a[:, 3] - a[:, 2]).mean() / 100:5.2f}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg1_local_50kf")
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "phases.txt"))
    ap.add_argument("--dump", default="/tmp/lba_phase_times.bin")
    args = ap.parse_args()
    os.environ["LBA_PHASE_TIMING"] = args.dump
    from amc_lba import Problem
    from amc_lba.synth import make_config_window
    win = make_config_window(args.config)
    p = Problem(win, early_stop=0)
    p.optimize(args.iters)
    p.close()
    nt, lin, sch, shape, chol, bs, cft = load(args.dump)
    out = [f"config {args.config}: {nt} tiles"]
    report("k_lin_schur (linearisation)", lin, LIN_PHASES, shape, out)
    report("k_lin_schur (elimination)", sch, SCHUR_PHASES, shape, out)
    timeline(lin, shape, out)
    exp_asm_timeline(sch, out)
    gp = win.obs["kind"] <= 1   # MONO_GP, STEREO_GP
    n_gp = len(set(zip(win.obs["kf_a"][gp].tolist(), win.obs["kf_b"][gp].tolist())))
    update_timeline(lin, n_gp, (len(win.kfs) + 63) // 64, out)
    np.savez_compressed(os.path.splitext(args.out)[0] + "_raw.npz", lin=lin, sch=sch, shape=shape)
    if chol is not None:
        npan = int((chol[:, 0] != 0).sum())
        c = chol[:npan].astype(np.int64)
        t0 = c[:, 0].min()
        out.append(f"== k_chol_flow panels (us from the first panel task start): start / own updates done / "
                   f"- / - / factor start / factor end / published")
        for j in range(npan):
            v = [(c[j, k] - t0) / 100.0 if c[j, k] else float("nan") for k in range(7)]
            out.append("   panel %3d: " % j + " ".join(f"{x:7.2f}" for x in v))
            w = [(c[j, 8 + k] - t0) / 100.0 if c[j, 8 + k] else float("nan") for k in range(7)]
            out.append("   (j+1,j)  : " + " ".join(f"{x:7.2f}" for x in w))
        yx = [((c[j, 7] - t0) / 100.0, (c[j, 15] - t0) / 100.0) for j in range(npan)]
        out.append("   forward block y_j published / solution block x_j written:")
        out.append("   " + "  ".join(f"{j}:{y:.1f}/{x:.1f}" for j, (y, x) in enumerate(yx)))
        pub = [(c[j, 6] - t0) / 100.0 for j in range(npan) if c[j, 6]]
        ys = [y for y, _ in yx if c[0, 7] and y > 0]
        xs = [x for _, x in yx if x > 0]
        if pub and ys and xs:   # the solve's tail after the factorisation (band mode: the substitution chains)
            order = sorted(range(npan), key=lambda j: yx[j][1])
            out.append(f"   tail: last panel published {max(pub):.2f}, last y_j {max(ys):.2f}, last x_j {max(xs):.2f}; "
                       "x_j in completion order (first 24): " +
                       " ".join(f"{j}:{yx[j][1]:.1f}" for j in order[:24]))
        b2 = bs[:npan].astype(np.int64)
        for rr in range(2):
            out.append(f"   L^-1 tiles of row {npan - 2 + rr}: j: start / terms done / L_ii^-1 out / published")
            for j in range(npan - 2 + rr):
                v = [(b2[j, 4 * rr + k] - t0) / 100.0 if b2[j, 4 * rr + k] else float("nan") for k in range(4)]
                out.append(f"     {j:3d}: " + " ".join(f"{x:7.2f}" for x in v))
        if cft is not None:
            out.append("   factor tasks (ticket: i j lookahead | start / last blocking wait done (panel) / loop done / "
                       "lookahead factors done / loop+lookahead done / published)")
            for tk in range(4096):
                r = cft[tk]
                if r[0] == 0:
                    continue
                f = lambda x: (x - t0) / 100.0 if x else float("nan")
                ii, jj, la, pp = r[4] & 4095, (r[4] >> 12) & 4095, (r[4] >> 24) & 1, (r[4] >> 32) & 4095
                out.append(f"     {tk:4d}: ({ii:2d},{jj:2d}) la={la} | {f(r[0]):7.2f} {f(r[3]):7.2f} (p={pp:2d}) "
                           f"{f(r[5]):7.2f} {f(r[6]):7.2f} {f(r[1]):7.2f} {f(r[2]):7.2f}  factor {r[7]} cycles")
                if ii == jj and len(r) > 8:   # the panel task's update list: entry end (panel, * = waited)
                    ent = [f"{r[9 + 2 * e] & 0xffffff}{'*' if (r[9 + 2 * e] >> 24) & 1 else ''}:{f(r[8 + 2 * e]):.2f}"
                           for e in range(16) if r[8 + 2 * e]]
                    out.append("            entries " + " ".join(ent))
    text = "\n".join(out)
    print(text)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    open(args.out, "w").write(text + "\n")


if __name__ == "__main__":
    main()
