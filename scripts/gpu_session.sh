#!/bin/bash
# GPU session driver: every GPU step under its own time limit, chained so the first failure ends it.
#   gpurun -- 'bash scripts/gpu_session.sh TAG STEP...'
# steps: list (rocprofv3 -L), bench (200-step config-1 line), drv (driver-shaped 20-step bench with CPU baseline),
#        tests (whole -m gpu suite), quick (parity subset), prof (kernel-trace stats), phases (in-kernel stamps)
set -u
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
T=$1; shift
python - <<'PY' || exit 3
import sys; sys.path.insert(0, 'amc-slam_amd')
import build
r = build.stale()
if r: print('STALE LIBRARY:', r); sys.exit(1)
PY
for s in "$@"; do
  case $s in
    list) (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 -L > $OLDPWD/gpurun_out/${T}_counters.txt 2>&1); rc=$? ;;
    bench) timeout -k 10 300 python bench.py --steps ${STEPS:-200} --warmup 10 --no-cpu > gpurun_out/${T}_bench.log 2>&1; rc=$?
           grep '^{' gpurun_out/${T}_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', round(d['value'],1), 'ms', round(d['ms_per_step']*1e3,2), 'sweep', round(d.get('roofline_sweep', d['roofline'])['avg_launch_ms']*1e3,2), 'solve', round(d['roofline_solve']['avg_launch_ms']*1e3,2))" ;;
    drv) timeout -k 10 600 python bench.py > gpurun_out/${T}_drv.log 2>&1; rc=$?; tail -c 600 gpurun_out/${T}_drv.log ;;
    tests) timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -rf --durations=15 --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_pytest.log ;;
    quick) timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_parity.py} > gpurun_out/${T}_quick.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_quick.log ;;
    prof) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OLDPWD/gpurun_out/prof_$T -o run -- python3 $OLDPWD/bench.py --steps 25 --warmup 3 --no-cpu > $OLDPWD/gpurun_out/${T}_prof.log 2>&1); rc=$?
          f=$(ls gpurun_out/prof_$T/*/run_kernel_stats.csv gpurun_out/prof_$T/run_kernel_stats.csv 2>/dev/null | head -1)
          [ -n "$f" ] && python scripts/kstats.py $f 28 | tee gpurun_out/${T}_kernel_stats.txt ;;
    pmc) KERNEL=${KERNEL:-k_lin_schur} bash scripts/pmc_linearize.sh $T; rc=$? ;;
    pmcchol) KERNEL=k_chol_flow SQ_COUNTERS="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_FMA_F64 GRBM_GUI_ACTIVE" bash scripts/pmc_linearize.sh $T; rc=$? ;;
    micro) /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 scripts/micro/$MICRO.hip -o /tmp/$MICRO && timeout -k 10 120 /tmp/$MICRO > gpurun_out/${T}_$MICRO.txt 2>&1; rc=$?; cat gpurun_out/${T}_$MICRO.txt ;;
    cfgs) rc=0; for c in ${CFGS:-cfg2_global_500kf cfg4_global_5k}; do
            timeout -k 10 300 python bench.py --config $c --steps ${CSTEPS:-5} --warmup 2 --no-cpu > gpurun_out/${T}_bench_$c.log 2>&1 || { rc=$?; break; }
            grep '^{' gpurun_out/${T}_bench_$c.log | tail -1; done ;;
    phases) timeout -k 10 300 python scripts/phase_times.py --out gpurun_out/${T}_phases.txt > gpurun_out/${T}_phases.log 2>&1; rc=$? ;;
    *) echo "unknown step $s"; rc=2 ;;
  esac
  echo "step $s rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
