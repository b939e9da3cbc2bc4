#!/bin/bash
# profiles/run_r01_emit_u.sh — sweep of k_emit's solo entries in flight per
# lane (MQM_EMIT_U64 / MQM_EMIT_U16) on C3, then the C3 parity-critical GPU
# tests for the default variant.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/emitu
mkdir -p $OUT
cd $ROOT
SW="MQM_EMIT_U64=4;MQM_EMIT_U64=2;MQM_EMIT_U64=8;MQM_EMIT_U16=8;MQM_EMIT_U64=8,MQM_EMIT_U16=8;MQM_EMIT_U64=4"
timeout -k 10 500 python3 -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --sweep "$SW" \
  > $OUT/sweep.json 2> $OUT/sweep.log
MQM_EMIT_U64=8 MQM_EMIT_U16=8 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 250 --timeout-method thread > $OUT/pytest_u8.log 2>&1
echo done
