#!/bin/bash
# profiles/run_r01_flatten.sh — after the parallel flattener: GPU parity tests,
# headline bench, churn bench (flatten phases traced to churn.log).
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/flat
mkdir -p $OUT
cd $ROOT
timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1
timeout -k 10 420 python3 -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.log
MQM_FLATTEN_TRACE=1 timeout -k 10 600 python3 -u bench.py --workload churn --steps 5 --warmup 1 \
  > $OUT/churn.json 2> $OUT/churn.log
echo done
