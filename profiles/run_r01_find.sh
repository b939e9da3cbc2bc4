#!/bin/bash
# profiles/run_r01_find.sh — GPU parity (all GPU tests) of the default build,
# then the C3 bench over find_hits batching (MQM_FIND_STEP 8 default / 4 / 1).
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/find
mkdir -p $OUT
cd $ROOT
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1
for v in default v_step4 v_step1; do
  lib=$ROOT/maxmq_amd/_lib/$v/libmqmatch.so
  [ $v = default ] && lib=$ROOT/maxmq_amd/_lib/libmqmatch.so
  MQM_LIB=$lib timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --host-topics 0 \
    > $OUT/bench_$v.json 2> $OUT/bench_$v.log
  echo "$v $(python3 -c "import json;d=json.load(open('$OUT/bench_$v.json'));print(d['value'],d['kernel_ms'])")" | tee -a $OUT/sweep.txt
done
