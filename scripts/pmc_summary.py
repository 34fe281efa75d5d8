"""Summarise the rocprofv3 PMC passes of scripts/pmc_linearize.sh for one kernel: the per-launch HBM
traffic (FETCH_SIZE x 2 per the gfx950 correction + WRITE_SIZE, MI355X_MICROARCH.md §HBM; rocprofv3
reports both in KB) and, when the SQ pass ran, per-launch medians of its counters.

    python scripts/pmc_summary.py <pmc dir> <out.json> [kernel]
"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "amc-slam_amd"))
from amc_lba import lib_digest  # noqa: E402


def per_dispatch(dirname, counter, kernel):
    vals = {}
    for f in glob.glob(os.path.join(dirname, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter or kernel not in r.get("Kernel_Name", ""):
                continue
            key = (r.get("Agent_Id"), r.get("Dispatch_Id"))
            vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def median(v):
    return sorted(v)[len(v) // 2] if v else None


def main():
    src, dst = sys.argv[1], sys.argv[2]
    kernel = sys.argv[3] if len(sys.argv) > 3 else "k_lin_schur"
    fetch = per_dispatch(os.path.join(src, "FETCH_SIZE"), "FETCH_SIZE", kernel)
    write = per_dispatch(os.path.join(src, "WRITE_SIZE"), "WRITE_SIZE", kernel)
    if not fetch or not write:
        raise SystemExit(f"no {kernel} counter rows found")
    f_kb, w_kb = median(fetch), median(write)
    fetch_b = 2.0 * f_kb * 1024.0   # gfx950: FETCH_SIZE reports half the bytes of wide streaming reads
    write_b = w_kb * 1024.0
    out = {"workload": os.environ.get("PMC_CONFIG", "cfg1_local_50kf"), "kernel": kernel, "lib_sha256": lib_digest(), "dispatches": [len(fetch), len(write)],
           "fetch_size_kb_median": f_kb, "write_size_kb_median": w_kb,
           "hbm_read_bytes_per_launch": fetch_b, "hbm_write_bytes_per_launch": write_b,
           "hbm_bytes_per_launch": fetch_b + write_b,
           "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), FETCH_SIZE x2 (gfx950)"}
    sq_dir = os.path.join(src, "SQ")
    if os.path.isdir(sq_dir):
        sq = {}
        names = set()
        for f in glob.glob(os.path.join(sq_dir, "**", "*counter_collection.csv"), recursive=True):
            names.update(r.get("Counter_Name") for r in csv.DictReader(open(f)))
        for c in sorted(n for n in names if n):
            sq[c] = median(per_dispatch(sq_dir, c, kernel))
        if sq.get("SQ_INSTS_LDS") and sq.get("SQ_LDS_BANK_CONFLICT") is not None:
            sq["lds_bank_conflict_per_lds_inst"] = sq["SQ_LDS_BANK_CONFLICT"] / sq["SQ_INSTS_LDS"]
        if sq.get("SQ_INSTS_VALU_MFMA_MOPS_F64") is not None:
            # MOPS are counted in units of 512 FLOPs (rocprofv3 -L); fp64 dense MFMA peak 78.6 TF/s
            sq["mfma_f64_flops"] = 512.0 * sq["SQ_INSTS_VALU_MFMA_MOPS_F64"]
        if sq.get("SQ_VALU_MFMA_BUSY_CYCLES") is not None and sq.get("GRBM_GUI_ACTIVE"):
            # GRBM_GUI_ACTIVE is summed over the 8 XCDs: kernel cycles = /8; 1024 SIMDs
            cyc = sq["GRBM_GUI_ACTIVE"] / 8.0
            sq["mfma_busy_frac_of_all_simds"] = sq["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024.0)
        out["sq_per_launch_median"] = sq
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
