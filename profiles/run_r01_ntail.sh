#!/bin/bash
# profiles/run_r01_ntail.sh — GPU parity of the default build, then the C3
# bench over kernel variants (make variant): base / record-tail 16-B loads /
# non-temporal output stores / both (default build).
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/ntail
mkdir -p $OUT
cd $ROOT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1
for v in v_base v_tail v_nt default; do
  lib=$ROOT/maxmq_amd/_lib/$v/libmqmatch.so
  [ $v = default ] && lib=$ROOT/maxmq_amd/_lib/libmqmatch.so
  MQM_LIB=$lib timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline \
    > $OUT/bench_$v.json 2> $OUT/bench_$v.log
  echo "$v $(python3 -c "import json;d=json.load(open('$OUT/bench_$v.json'));print(d['value'],d['kernel_ms'])")" | tee -a $OUT/sweep.txt
done
