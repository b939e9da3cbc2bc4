#!/bin/bash
# profiles/run_r01_sweep.sh — one GPU call: occupancy sweep of k_walk / k_emit
# (bench.py --sweep), then the PMC traffic passes (run_pmc.sh) and the SQ /
# TCC pass of run_pmc_walk.sh, all on the C3 workload.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/gpurun_out
SW="MQM_WALK_OCC=1;MQM_WALK_OCC=5;MQM_WALK_OCC=6;MQM_WALK_OCC=8;MQM_EMIT64_OCC=6;MQM_EMIT64_OCC=8;MQM_EMIT16_OCC=6;MQM_EMIT16_OCC=8"
timeout -k 10 500 python3 -u $ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline --sweep "$SW" \
  > $ROOT/gpurun_out/sweep.json 2> $ROOT/gpurun_out/sweep.log
bash $ROOT/profiles/run_pmc.sh
