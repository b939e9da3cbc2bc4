#!/bin/bash
# profiles/run_pmc_sq.sh — issue / wait / occupancy counters of the match
# kernels (C3 bench, 2 steps) in ONE rocprofv3 --pmc pass (8 SQ + 2 TCC slots,
# MI355X_MICROARCH.md §rocprofv3 PMC slots).  Run on the GPU box from the repo
# root; writes gpurun_out/pmc_sq/ and prints a per-kernel summary.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
P="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD TCC_HIT_sum TCC_MISS_sum"
timeout -s KILL 600 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $ROOT/gpurun_out/pmc_sq -o pmc -- \
  python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $ROOT/gpurun_out/pmc_sq.json 2> $ROOT/gpurun_out/pmc_sq.log
python3 $ROOT/profiles/pmc_summary.py $(dirname $(find $ROOT/gpurun_out/pmc_sq -name "pmc_counter_collection.csv" | head -1)) \
  > $ROOT/gpurun_out/pmc_sq_summary.txt
cat $ROOT/gpurun_out/pmc_sq_summary.txt
