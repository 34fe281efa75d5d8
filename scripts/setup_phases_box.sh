cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for th in 8 1; do
  echo "== threads $th"
  LBA_SETUP_THREADS=$th timeout -k 10 200 python scripts/setup_phases_gpu.py > gpurun_out/r3ao_sp_$th.log 2>&1 || exit 1
  tail -32 gpurun_out/r3ao_sp_$th.log
done
lscpu | grep -E "Model name|MHz" | head -3
