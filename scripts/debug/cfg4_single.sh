#!/bin/bash
# config 4 (5k KF / 1M landmarks / 6M obs global BA) on one GPU: the whole problem, band solve
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1000 python bench.py --config cfg4_global_5k --steps ${STEPS:-3} --warmup 1 --window-iters 3 --no-cpu > gpurun_out/cfg4_single.log 2>&1
