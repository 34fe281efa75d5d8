cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u scripts/ab_compare.py --calls 40 --variant base: --variant nowait:LBA_NO_UPD_WAIT=1 --variant inl:AMC_LBA_LIB=amc-slam_amd/lib/exp/inl.so --variant inl_nowait:AMC_LBA_LIB=amc-slam_amd/lib/exp/inl.so,LBA_NO_UPD_WAIT=1 --variant base2: > gpurun_out/R3e.ab.log 2>&1; cat gpurun_out/R3e.ab.log
