#!/bin/bash
# profiles/run_pmc_walk.sh — occupancy / latency / translation counters of the
# match kernels (C3 bench, 2 steps), one rocprofv3 --pmc pass per counter set
# (MI355X_MICROARCH.md: per-block counter slots).  Run on the GPU box from the
# repo root; writes gpurun_out/pmcw_<pass>/.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
P1="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum"
P2="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_VMEM TCC_HIT_sum TCC_MISS_sum"
i=0
for P in "$P1" "$P2"; do
  i=$((i + 1))
  timeout -s KILL 600 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $ROOT/gpurun_out/pmcw_$i -o pmc -- \
    python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $ROOT/gpurun_out/pmcw_$i.json 2> $ROOT/gpurun_out/pmcw_$i.log
done
