#!/bin/bash
# profiles/run_pmc.sh — HBM traffic of one match batch from rocprofv3 PMC
# counters, in two separate passes (FETCH_SIZE takes 3 TCC slots, WRITE_SIZE 2:
# MI355X_MICROARCH.md §rocprofv3 PMC slots).  Run on the GPU box from the repo
# root; writes gpurun_out/pmc_{fetch,write}/ and profiles/traffic.json via
# profiles/pmc_to_traffic.py.
set -euo pipefail
CFG=${CFG:-3}
STEPS=${STEPS:-2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace --output-format csv \
    -d $ROOT/gpurun_out/pmc_$C -o pmc -- \
    python3 $ROOT/bench.py --config $CFG --steps $STEPS --warmup 1 --no-cpu-baseline --host-topics 0 --latency-topics 0 \
    > $ROOT/gpurun_out/pmc_$C.json 2> $ROOT/gpurun_out/pmc_$C.log
done
python3 $ROOT/profiles/pmc_to_traffic.py $ROOT/gpurun_out $((STEPS + 1)) > $ROOT/gpurun_out/traffic.json
cat $ROOT/gpurun_out/traffic.json
