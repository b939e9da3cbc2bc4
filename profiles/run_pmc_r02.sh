#!/bin/bash
# profiles/run_pmc_r02.sh TAG [ARGS...] — rocprofv3 PMC passes over the C3
# bench (MI355X_MICROARCH.md §rocprofv3: one pass per counter group, FETCH_SIZE
# and WRITE_SIZE in separate passes, <= 8 SQ / 4 TCC counters per pass).
# Counters missing from `rocprofv3 -L` are dropped from their pass.  Each pass
# under its own `timeout -s KILL`.  Summaries: profiles/pmc_summary.py.
set -euo pipefail
TAG=$1
shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --host-topics 0 --latency-topics 0 --steady-steps 0 --pipeline 0 $*"
timeout -s KILL 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
PASSES=(
  "FETCH_SIZE"
  "WRITE_SIZE"
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
  "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_THREAD_CYCLES_VALU SQ_INSTS_SMEM TCC_HIT_sum TCC_MISS_sum"
  "SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"
)
i=0
for P in "${PASSES[@]}"; do
  i=$((i + 1))
  keep=""
  for c in $P; do
    if grep -qw "$c" $OUT/counters.txt; then keep="$keep $c"; else echo "[pmc] $c not listed, dropped"; fi
  done
  [ -z "$keep" ] && continue
  echo "[pmc] pass $i:$keep $(date +%T)"
  timeout -s KILL 240 rocprofv3 --pmc $keep --kernel-trace --output-format csv -d $OUT/pmc_$i -o pmc -- \
    python3 $ROOT/bench.py $ARGS > $OUT/pmc_$i.json 2> $OUT/pmc_$i.log
done
for d in $OUT/pmc_*/; do
  f=$(find $d -name "pmc_counter_collection.csv" | head -1)
  [ -n "$f" ] && python3 $ROOT/profiles/pmc_summary.py $(dirname $f) >> $OUT/pmc_summary.txt
done
echo "[pmc] done $(date +%T)"
