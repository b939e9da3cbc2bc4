#!/bin/bash
# profiles/run_r02.sh TAG STEP... — round-2 GPU runs, each step under its own
# time limit, chained so that the first failure ends the call.
#   tests   : every -m gpu test                         -> gpurun_out/TAG/pytest_gpu.log
#   quick   : the -m gpu tests except the full-size ones -> gpurun_out/TAG/pytest_quick.log
#   smoke   : __graft_entry__.smoke()
#   bench   : the default bench line (C3)               -> gpurun_out/TAG/bench.json
#   fast    : bench without CPU baseline / host path     -> gpurun_out/TAG/bench_fast.json
#   prof    : rocprofv3 kernel trace + stats of `fast`   -> gpurun_out/TAG/prof/
#   profser : `prof` with the merges serialised behind the solo copy (MQM_NO_OVERLAP=1): per-kernel times
#   shim    : the Go shim's call sequence from 4 threads  -> gpurun_out/TAG/pytest_shim.log
#   variants: `fast` once per tuning build maxmq_amd/_lib/<name>/ (make variant) -> bench_fast_<name>.json
#   calib   : FETCH_SIZE / WRITE_SIZE on known byte counts (tools/calib_fetch) -> gpurun_out/TAG/calib_*
set -euo pipefail
TAG=$1
shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
FAST="--steps 10 --warmup 3 --no-cpu-baseline --host-topics 0 --latency-topics 0"
for step in "$@"; do
  echo "[run_r02] $step $(date +%T)"
  case $step in
    tests) timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread \
             > $OUT/pytest_gpu.log 2>&1 ;;
    quick) timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
             -k "not full_size and not 20m and not 5m" > $OUT/pytest_quick.log 2>&1 ;;
    smoke) timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 ;;
    bench) timeout -k 10 600 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.log ;;
    fast) timeout -k 10 400 python3 -u bench.py $FAST > $OUT/bench_fast.json 2> $OUT/bench_fast.log ;;
    lanes) for L in 4 16; do MQM_WALK_LANES=$L timeout -k 10 400 python3 -u bench.py $FAST \
             > $OUT/bench_fast_lanes$L.json 2> $OUT/bench_fast_lanes$L.log; done ;;
    c4shard) timeout -k 10 600 python3 -u bench.py --config 4 --shard 0/8 $FAST \
             > $OUT/bench_c4_shard0of8.json 2> $OUT/bench_c4_shard0of8.log ;;
    host) timeout -k 10 600 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline \
             > $OUT/bench_host.json 2> $OUT/bench_host.log ;;
    c4prof) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv \
             -d $OUT/prof_c4 -o prof -- python3 $ROOT/bench.py --config 4 --shard 0/8 --steps 3 --warmup 1 \
             --no-cpu-baseline --host-topics 0 --latency-topics 0 > $OUT/c4_under_rocprof.json 2> $OUT/rocprof_c4.log) ;;
    prof) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv \
             -d $OUT/prof -o prof -- python3 $ROOT/bench.py $FAST \
             > $OUT/bench_under_rocprof.json 2> $OUT/rocprof.log) ;;
    nobloom) MQM_NO_BLOOM=1 timeout -k 10 400 python3 -u bench.py $FAST > $OUT/bench_fast_nobloom.json \
             2> $OUT/bench_fast_nobloom.log ;;
    edgeload) for L in 0.12 0.35; do MQM_EDGE_LOAD=$L timeout -k 10 400 python3 -u bench.py $FAST \
             > $OUT/bench_fast_load$L.json 2> $OUT/bench_fast_load$L.log || exit 1; done ;;
    nooverlap) MQM_NO_OVERLAP=1 timeout -k 10 400 python3 -u bench.py $FAST > $OUT/bench_fast_nooverlap.json \
             2> $OUT/bench_fast_nooverlap.log ;;
    ret) timeout -k 10 600 python3 -u -m pytest tests/test_gpu_retained.py -m gpu -x -v --timeout 300 \
             --timeout-method thread > $OUT/pytest_ret.log 2>&1 ;;
    rev) timeout -k 10 600 python3 -u bench.py --workload reverse --steps 5 --warmup 1 --no-cpu-baseline \
             > $OUT/bench_reverse.json 2> $OUT/bench_reverse.log ;;
    revfull) timeout -k 10 900 python3 -u bench.py --workload reverse --steps 5 --warmup 1 \
             > $OUT/bench_reverse_full.json 2> $OUT/bench_reverse_full.log ;;
    revprof) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
             -d $OUT/prof_rev -o prof -- python3 $ROOT/bench.py --workload reverse --steps 3 --warmup 1 \
             --no-cpu-baseline > $OUT/rev_under_rocprof.json 2> $OUT/rocprof_rev.log) ;;
    revpmc) (cd /tmp && export TMPDIR=/tmp && for C in FETCH_SIZE WRITE_SIZE; do
             timeout -s KILL 600 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/revpmc_$C -o pmc \
             -- python3 $ROOT/bench.py --workload reverse --steps 2 --warmup 1 --no-cpu-baseline \
             > $OUT/revpmc_$C.json 2> $OUT/revpmc_$C.log || exit 1; done) ;;
    batching) timeout -k 10 300 python3 -u -m pytest tests/test_gpu_batching.py -m gpu -x -v --timeout 240 \
             --timeout-method thread > $OUT/pytest_batching.log 2>&1 ;;
    shim) timeout -k 10 300 python3 -u -m pytest tests/test_gpu_shim.py -m gpu -x -v --timeout 240 \
             --timeout-method thread > $OUT/pytest_shim.log 2>&1 ;;
    calib) (cd /tmp && export TMPDIR=/tmp && for C in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
             tag=$(echo $C | cut -d' ' -f1); timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv \
             -d $OUT/calib_$tag -o calib -- $ROOT/tools/_build/calib_fetch > $OUT/calib_$tag.txt 2>&1 || exit 1; done) ;;
    variants) for L in maxmq_amd/_lib/*/libmqmatch.so; do V=$(basename $(dirname $L)); [ "$V" = asan ] && continue;
             MQM_LIB=$ROOT/$L timeout -k 10 400 python3 -u bench.py $FAST > $OUT/bench_fast_$V.json 2> $OUT/bench_fast_$V.log || exit 1; done ;;
    profser) (cd /tmp && export TMPDIR=/tmp MQM_NO_OVERLAP=1 && timeout -k 10 500 rocprofv3 --kernel-trace --stats \
             --output-format csv -d $OUT/profser -o prof -- python3 $ROOT/bench.py $FAST \
             > $OUT/bench_under_rocprof_serial.json 2> $OUT/rocprof_serial.log) ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[run_r02] done $(date +%T)"
