#!/bin/bash
# profiles/run_r01_pad.sh — GPU parity (all GPU tests), then the C3 bench with
# segment starts padded to 16 entries (default) and unpadded (MQM_DPAD=1), and
# the rocprofv3 kernel stats of the default.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pad
mkdir -p $OUT
cd $ROOT
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1
for p in 16 1; do
  MQM_DPAD=$p timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --host-topics 0 \
    > $OUT/bench_pad$p.json 2> $OUT/bench_pad$p.log
  echo "pad$p $(python3 -c "import json;d=json.load(open('$OUT/bench_pad$p.json'));print(d['value'],d['kernel_ms'])")" | tee -a $OUT/sweep.txt
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o prof -- \
  python3 $ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline --host-topics 0 \
  > $OUT/bench_under_rocprof.json 2> $OUT/rocprof.log
echo done
