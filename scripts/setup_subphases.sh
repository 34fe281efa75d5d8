# lba_set_problem host sub-phases (LBA_SETUP_TIMING) at 1 and 8 threads on this machine's host
cd ${GRAFT_REPO_ROOT:-.}
for th in 1 8; do
  echo "== threads $th"
  LBA_SETUP_TIMING=1 LBA_SETUP_THREADS=$th timeout -k 5 120 python -c "
import sys; sys.path.insert(0,'amc-slam_amd')
import amc_lba
from amc_lba.synth import make_config_window
w = make_config_window('cfg1_local_50kf')
for i in range(5): amc_lba.setup_host_profile(w)
" 2>&1 | tail -14
done
lscpu | grep -E "Model name|^CPU\(s\)|Thread|MHz" | head -5
