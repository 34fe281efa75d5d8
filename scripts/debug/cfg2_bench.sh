set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config cfg2_global_500kf --steps 5 --warmup 2 --no-cpu > gpurun_out/cfg2_bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_cfg2 -o trace -- python3 $GRAFT_REPO_ROOT/bench.py --config cfg2_global_500kf --steps 5 --warmup 2 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/cfg2_prof.log 2>&1
