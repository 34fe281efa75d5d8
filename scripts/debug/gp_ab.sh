# k_update GP-chain diagnostics (lib/exp/gpdiag.so: stamps after the staging loads and the trial states) and the
# scalar-load variant of the pair's index record (lib/exp/shab.so) against the main build
set -u
cd ${GRAFT_REPO_ROOT:-/root/repo}
X=$PWD/amc-slam_amd/lib/exp
AMC_LBA_LIB=$X/gpdiag.so timeout -k 10 300 python scripts/phase_times.py --out gpurun_out/r5x_gpdiag_phases.txt > gpurun_out/r5x.log 2>&1 || exit 1
grep -A6 "k_update timeline" gpurun_out/r5x_gpdiag_phases.txt
timeout -k 10 300 python scripts/cmp_libs.py main $X/shab.so > gpurun_out/r5x_cmp_shab.txt 2>&1 || exit 1
tail -1 gpurun_out/r5x_cmp_shab.txt
bash scripts/prof_ab.sh r5x shab || exit 1
AMC_LBA_LIB=$X/shab.so timeout -k 10 300 python scripts/phase_times.py --out gpurun_out/r5x_shab_phases.txt > /dev/null 2>&1 || exit 1
grep -A6 "k_update timeline" gpurun_out/r5x_shab_phases.txt
