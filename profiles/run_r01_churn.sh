#!/bin/bash
# profiles/run_r01_churn.sh — GPU tests (incl. tests/test_commit.py) and the
# incremental-commit bench (bench.py --workload churn) on C3.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/churn
mkdir -p $OUT
cd $ROOT
timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1
timeout -k 10 600 python3 -u bench.py --workload churn --steps 5 --warmup 1 > $OUT/churn.json 2> $OUT/churn.log
echo done
