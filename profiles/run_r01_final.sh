#!/bin/bash
# profiles/run_r01_final.sh — end-of-session check of HEAD: every GPU test,
# smoke(), the default bench line (with CPU baseline), its rocprofv3 kernel
# stats, and the churn bench with the flattener phases traced.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/final
mkdir -p $OUT
cd $ROOT
timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 420 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o prof -- \
  python3 $ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline \
  > $OUT/bench_under_rocprof.json 2> $OUT/rocprof.log
cd $ROOT
MQM_FLATTEN_TRACE=1 timeout -k 10 600 python3 -u bench.py --workload churn --steps 5 --warmup 1 \
  > $OUT/churn.json 2> $OUT/churn.log
echo done
