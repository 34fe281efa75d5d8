cd $GRAFT_REPO_ROOT
E=$PWD/amc-slam_amd/lib/exp
timeout -k 10 300 python scripts/cmp_libs.py $E/pipe3.so $E/head.so > gpurun_out/r8h_cmp.txt 2>&1; cat gpurun_out/r8h_cmp.txt
timeout -k 10 300 python scripts/cmp_libs.py $E/pipe3.so $E/head.so cfg2_global_500kf >> gpurun_out/r8h_cmp.txt 2>&1; tail -3 gpurun_out/r8h_cmp.txt
for c in cfg1_local_50kf cfg2_global_500kf; do for r in 1 2 3; do for v in head pipe3; do
  echo -n "$c $v: "
  AMC_LBA_LIB=$E/$v.so timeout -k 10 300 python bench.py --config $c --steps ${S:-100} --warmup 5 --no-cpu 2>/dev/null | grep "^{" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value'],1), 'ms/step', round(d['ms_per_step']*1e3,2), 'solve us', round(d['roofline_solve']['avg_launch_ms']*1e3,1), 'sweep us', round(d['roofline_sweep']['avg_launch_ms']*1e3,1), 'trials', d['trials_per_step'])" || exit 1
done; done; done
