#!/bin/bash
# profiles/run_r01_head.sh — one GPU call that checks HEAD end to end: the GPU
# parity tests, the default bench line (C3, with the CPU baseline) and the
# rocprofv3 --kernel-trace --stats summary of the same bench command.
# Every GPU step has its own time limit; the first failure ends the script.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/head
mkdir -p $OUT
cd $ROOT
timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1
timeout -k 10 420 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o prof -- \
  python3 $ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline \
  > $OUT/bench_under_rocprof.json 2> $OUT/rocprof.log
echo done
