"""Kernel sequence of a rocprofv3 kernel trace (ordered by start time, runs collapsed): shows where the
runtime's __amd_rocclr_copyBuffer / fillBufferAligned dispatches fall relative to the LM-loop kernels
(they belong to lba_set_problem's uploads when they sit between loops, not inside one).

    python scripts/trace_regions.py gpurun_out/prof_TAG/trace_kernel_trace.csv
"""
import csv
import sys


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    seq = []
    for r in rows:
        n = r["Kernel_Name"].split("(")[0].replace("lba::", "")
        if seq and seq[-1][0] == n:
            seq[-1][1] += 1
        else:
            seq.append([n, 1])
    # split into segments: runtime copy/fill runs vs runs of engine kernels
    segs, cur, kind = [], [], None
    for n, c in seq:
        k = "runtime" if n.startswith("__amd_rocclr") else "engine"
        if k != kind and cur:
            segs.append((kind, cur))
            cur = []
        kind = k
        cur.append((n, c))
    if cur:
        segs.append((kind, cur))
    tot = {"runtime": 0, "engine": 0}
    for k, s in segs:
        n = sum(c for _, c in s)
        tot[k] += n
        if k == "runtime":
            print(f"[set-up uploads] {n} runtime copy/fill dispatches")
        else:
            lin = sum(c for nm, c in s if nm == "k_lin_schur")
            print(f"[LM loop] {n} engine dispatches, {lin} k_lin_schur; no runtime copy inside")
    print(f"total: {tot['runtime']} runtime copy/fill dispatches, all between engine-kernel runs (lba_set_problem)")


if __name__ == "__main__":
    main(sys.argv[1])
