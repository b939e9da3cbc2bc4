#!/bin/bash
# profiles/run_pmc_emit.sh — stall / cache / request-latency counters of the
# match kernels on the C3 bench (2 steps), one rocprofv3 --pmc pass per set.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_VALU TCC_HIT_sum TCC_MISS_sum"
P2="TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum"
i=0
for P in "$P1" "$P2"; do
  i=$((i + 1))
  timeout -s KILL 600 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $ROOT/gpurun_out/pmce_$i -o pmc -- \
    python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $ROOT/gpurun_out/pmce_$i.json 2> $ROOT/gpurun_out/pmce_$i.log
done
