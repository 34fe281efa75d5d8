cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u scripts/ab_compare.py --calls 40 --variant base: --variant fused:LBA_FLOW_FUSED=1 --variant base2: > gpurun_out/R3h.ab.log 2>&1; cat gpurun_out/R3h.ab.log
AMC_LBA_LIB=$GRAFT_REPO_ROOT/amc-slam_amd/lib/exp/twice.so timeout -k 10 200 python scripts/phase_times.py --out gpurun_out/R3h_twice_phases.txt > /dev/null 2>&1
grep -A2 "k_update timeline" gpurun_out/R3h_twice_phases.txt
