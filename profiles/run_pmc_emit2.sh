#!/bin/bash
# profiles/run_pmc_emit2.sh — LDS / VMEM issue and stall counters of the
# emit kernels on the C3 bench (2 steps), one rocprofv3 --pmc pass per set.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
P2="SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVES TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum"
i=0
for P in "$P1" "$P2"; do
  i=$((i + 1))
  timeout -s KILL 600 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $ROOT/gpurun_out/pmcf_$i -o pmc -- \
    python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $ROOT/gpurun_out/pmcf_$i.json 2> $ROOT/gpurun_out/pmcf_$i.log
done
