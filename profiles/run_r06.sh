#!/bin/bash
# profiles/run_r06.sh TAG STEP... — round-6 GPU runs, each step under its own
# time limit, chained so that the first failure ends the call.
#   stampt  : served churn test with recycled snapshot buffers (no quarantine) and version stamps checked
#   recyclet: served + churn tests with recycled snapshot buffers, no quarantine
#   pathab  : `fast` with the walk's path filter, without it (MQM_PATH_FILTER=0), with it again
#   pairab  : `fast` with the paired-position window copy (MQM_WINCOPY_PAIR=1), then without
#   pairpar : parity subset with the paired window copy
#   cooppar : parity + queued tests with the cooperative walk loads (MQM_WALK_COOP=1)
#   coopab  : `fast` with / without / with the cooperative walk loads
#   tests   : every -m gpu test                          -> gpurun_out/TAG/pytest_gpu.log
#   serve   : the per-publish server tests (incl. served calls under Subscribe/Unsubscribe churn)
#   ab / c4ab: `fast` (C3) / the C4 shard bench with the round-5 walk (paired node slots) and long-part
#             copy, then each switched off (MQM_SLOTS=1 switches the slot walk on, MQM_LONG_PART=0 the long copy off)
#   revstats: the C5 reverse bench with the per-level item mix (MQM_REV_STATS=1)
#   revab   : the C5 reverse bench without and with level tasks (MQM_REV_TASKS=1)
#   node    : the sharded node step with two rank processes and the HIP matcher (tests/test_gpu_node_step.py)
#   churnserve: the churn workload with the served-calls-under-churn legs (one per rebuild thread count)
#   edges   : the device-built edge table equals the host's (digests), async commits on the GPU
#   vecab   : the 4-positions-per-lane window copy (MQM_WINCOPY_VEC=1): parity subset, then C3 / C4 shard A/B
#   ident   : the Identifiers parity tests (batch, DFS, runs, batching collector)
#   c4test  : the C4 shard 0/8 full-batch test            -> gpurun_out/TAG/pytest_c4.log
#   ret     : the retained (reverse-match) tests           -> gpurun_out/TAG/pytest_ret.log
#   nobloom : the edge-case / random-op parity tests with the edge filter off (MQM_NO_BLOOM=1)
#   fastt   : small-batch path + batching collector + shim tests -> gpurun_out/TAG/pytest_fast.log
#   quick   : every -m gpu test except the full-size ones
#   lat     : C3 bench with the per-publish legs (single topic, 64 native callers direct / batched)
#   c4pmc / pmc: FETCH_SIZE / WRITE_SIZE passes (C4 shard / C3) -> traffic_c4.json / traffic.json
#   freeprobe: tools/_build/free_probe (does hipFree wait for a running kernel?) -> free_probe.txt
#   calib   : tools/_build/calib_fetch (random-gather / cooperative-gather rates) -> calib_kernels.txt
#   duplex  : tools/_build/duplex_probe (H2D / D2H alone and at once, DMA and kernel copies) -> duplex_probe.txt
#   hostab  : the host-path legs with DMA / kernel result copies (MQM_D2H_KERNEL=1), 4 / 8 HW queues
#   hostthreads: the host-path legs on 4 / 12 / 16 caller threads
#   kcopyt  : the runs-form tests, kernel copy-out parity included
#   freshtest: the MQM_CFG_FRESH tests (every mutation visible at once) + the served / churn tests
#   xcdab   : `fast` with / without the XCD-affine walk parts (MQM_WALK_XCD=1), on the batch as generated and sorted
#   xcdpar  : parity + queued tests with the XCD-affine walk
#   sortab  : `fast` with the walk in prefix order (default), in batch order (MQM_WALK_SORT=0), in prefix order again
#   freshleg: the churn workload with one plain and one MQM_CFG_FRESH served leg (2 build threads, 20 s each)
#   c2      : the C2 bench line (1M filters, 10M topics) with roofline and CPU baseline -> bench_c2.json
#   c4fast  : the C4 shard bench without CPU baseline
#   pipe    : `fast` with pipelined steps on 2 and 3 contexts -> bench_fast_pipe{2,3}.json
#   par     : the parity and queued-call GPU tests only
#   smoke   : __graft_entry__.smoke()
#   bench   : the default bench line (C3)                -> gpurun_out/TAG/bench.json
#   fast    : bench without CPU baseline / host path      -> gpurun_out/TAG/bench_fast.json
#   prof    : rocprofv3 kernel trace + stats of `fast`, one batch at a time (pipelined batches overlap
#             their kernels, so per-kernel durations would mix)  -> gpurun_out/TAG/prof/
#   c4shard : C4 shard 0/8 bench line with roofline and CPU baseline
#   c4prof  : rocprofv3 kernel stats of the C4 shard bench
#   c4host  : the C4 shard bench with the host-path legs (runs / packed forms: the per-shard end-to-end rate)
#   revprof : rocprofv3 kernel trace + stats of the C5 reverse bench
#   revpmc  : FETCH_SIZE / WRITE_SIZE passes of the C5 reverse bench -> traffic_reverse.json
#   rev     : C5 reverse bench line (full 50M retained, CPU baseline, full-size selfcheck)
#   counters / c4counters: the five rocprofv3 --pmc passes (profiles/run_pmc_r02.sh) over C3 / the C4
#             shard -> c3_counters.txt (profiles/derive_counters.py), traffic.json
set -euo pipefail
TAG=$1
shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
FAST="--steps 10 --warmup 3 --no-cpu-baseline --host-topics 0 --latency-topics 0 --steady-steps 0"
PYT="python3 -u -m pytest -x -v --timeout-method thread"
for step in "$@"; do
  echo "[run_r06] $step $(date +%T)"
  case $step in
    tests) timeout -k 10 1000 $PYT tests -m gpu --timeout 600 --durations=15 > $OUT/pytest_gpu.log 2>&1 ;;
    stampt) MQM_SNAP_RECYCLE=1 MQM_RECYCLE_QUARANTINE_MS=0 MQM_SNAP_STAMP=1 timeout -k 10 500 $PYT -s \
             tests/test_gpu_serve_churn.py -m gpu --timeout 300 > $OUT/pytest_stamp.log 2>&1 ;;
    verifyt) MQM_SNAP_RECYCLE=1 MQM_RECYCLE_QUARANTINE_MS=0 MQM_SNAP_VERIFY=1 timeout -k 10 500 $PYT -s \
             tests/test_gpu_serve_churn.py -m gpu --timeout 300 > $OUT/pytest_verify.log 2>&1 ;;
    recyclematrix)  # served churn tests with recycled snapshot buffers (no quarantine), per edge-build memory; each variant 3x
          for V in scratch:X=0 pool:MQM_EDGE_POOL=1 hostedges:MQM_HOST_EDGES=1; do
            N=${V%%:*}; E=${V#*:}
            for k in 1 2 3; do
              env $E MQM_SNAP_RECYCLE=1 MQM_RECYCLE_QUARANTINE_MS=0 timeout -k 10 300 $PYT -s tests/test_gpu_serve_churn.py \
                -m gpu --timeout 200 > $OUT/pytest_recycle_${N}_$k.log 2>&1 && echo "$N $k passed" >> $OUT/matrix.txt \
                || echo "$N $k FAILED: $(grep -o '[0-9]* of [0-9]* results differ' $OUT/pytest_recycle_${N}_$k.log | head -2 | tr '\n' ' ')" >> $OUT/matrix.txt
            done
          done ;;
    recyclet) MQM_SNAP_RECYCLE=1 MQM_RECYCLE_QUARANTINE_MS=0 timeout -k 10 500 $PYT -s \
             tests/test_gpu_serve_churn.py tests/test_gpu_serve.py -m gpu --timeout 300 > $OUT/pytest_recycle.log 2>&1 ;;
    pathab) for V in path:X=0 nopath:MQM_PATH_FILTER=0 path2:X=0; do
          N=${V%%:*}; E=${V#*:}
          env $E timeout -k 10 400 python3 -u bench.py $FAST > $OUT/bench_fast_$N.json 2> $OUT/bench_fast_$N.log || exit 1
        done ;;
    pairab) for V in pair:MQM_WINCOPY_PAIR=1 base:X=0; do
          N=${V%%:*}; E=${V#*:}
          env $E timeout -k 10 400 python3 -u bench.py $FAST --ident-steps 0 > $OUT/bench_fast_$N.json 2> $OUT/bench_fast_$N.log || exit 1
        done ;;
    pairpar) MQM_WINCOPY_PAIR=1 timeout -k 10 500 $PYT tests/test_gpu_parity.py -m gpu --timeout 300 \
             -k "config_vs_oracle or edge_cases or kat or full_size" > $OUT/pytest_pair.log 2>&1 ;;
    cooppar) MQM_WALK_COOP=1 timeout -k 10 600 $PYT tests/test_gpu_parity.py tests/test_gpu_queued.py -m gpu --timeout 300 \
             > $OUT/pytest_coop.log 2>&1 ;;
    coopab) for V in coop:MQM_WALK_COOP=1 base:X=0 coop2:MQM_WALK_COOP=1; do
          N=${V%%:*}; E=${V#*:}
          env $E timeout -k 10 400 python3 -u bench.py $FAST --ident-steps 0 > $OUT/bench_fast_$N.json 2> $OUT/bench_fast_$N.log || exit 1
        done ;;
    churnt) timeout -k 10 500 $PYT tests/test_gpu_serve_churn.py -m gpu --timeout 300 > $OUT/pytest_churn.log 2>&1 ;;
    serve) timeout -k 10 600 $PYT tests/test_gpu_serve.py tests/test_gpu_serve_churn.py tests/test_gpu_shim.py -m gpu \
             --timeout 300 > $OUT/pytest_serve.log 2>&1 ;;
    ab) for V in base:X=0 long:MQM_LONG_PART=256 desccopy:MQM_DESC_COPY=1; do
          N=${V%%:*}; E=${V#*:}
          env $E timeout -k 10 400 python3 -u bench.py $FAST > $OUT/bench_fast_$N.json 2> $OUT/bench_fast_$N.log || exit 1
        done ;;
    c4ab) for V in base:X=0 long:MQM_LONG_PART=256; do
          N=${V%%:*}; E=${V#*:}
          env $E timeout -k 10 600 python3 -u bench.py --config 4 --shard 0/8 $FAST > $OUT/bench_c4_$N.json \
            2> $OUT/bench_c4_$N.log || exit 1
        done ;;
    ntab) for V in base:MQM_NT_STORE=0 nt:X=0 base2:MQM_NT_STORE=0 nt2:X=0; do
          N=${V%%:*}; E=${V#*:}
          env $E timeout -k 10 400 python3 -u bench.py $FAST --ident-steps 0 > $OUT/bench_fast_$N.json 2> $OUT/bench_fast_$N.log || exit 1
        done ;;
    c4ntab) for V in base:MQM_NT_STORE=0 nt:X=0; do
          N=${V%%:*}; E=${V#*:}
          env $E timeout -k 10 600 python3 -u bench.py --config 4 --shard 0/8 $FAST --ident-steps 0 > $OUT/bench_c4_$N.json \
            2> $OUT/bench_c4_$N.log || exit 1
        done ;;
    ntpar) MQM_NT_STORE=1 timeout -k 10 500 $PYT tests/test_gpu_parity.py -m gpu --timeout 300 \
             -k "config_vs_oracle or edge_cases or kat" > $OUT/pytest_nt.log 2>&1 ;;
    revstats) MQM_REV_STATS=1 timeout -k 10 600 python3 -u bench.py --workload reverse --steps 2 --warmup 1 \
             --no-cpu-baseline > $OUT/bench_rev_stats.json 2> $OUT/bench_rev_stats.log ;;
    node) timeout -k 10 400 $PYT tests/test_gpu_node_step.py -m gpu --timeout 300 > $OUT/pytest_node.log 2>&1 ;;
    revab) for V in base:X=0 tasks:MQM_REV_TASKS=1; do
          N=${V%%:*}; E=${V#*:}
          env $E timeout -k 10 600 python3 -u bench.py --workload reverse --steps 3 --warmup 1 --no-cpu-baseline \
            > $OUT/bench_rev_$N.json 2> $OUT/bench_rev_$N.log || exit 1
        done ;;
    churnserve) timeout -k 10 1100 python3 -u bench.py --workload churn --steps 3 --warmup 1 --serve-churn-s 30 \
             > $OUT/bench_churn.json 2> $OUT/bench_churn.log ;;
    flat) timeout -k 10 700 $PYT tests/test_gpu_retained.py tests/test_gpu_edges.py tests/test_commit.py \
             tests/test_gpu_serve_churn.py tests/test_gpu_parity.py -m gpu --timeout 300 --durations=10 \
             > $OUT/pytest_flat.log 2>&1 ;;
    churnfast) MQM_FAST_REPLAY=1 timeout -k 10 700 python3 -u bench.py --workload churn --steps 2 --warmup 1 \
             --serve-churn-s 30 --churn-build-threads 4,2 > $OUT/bench_churnfast.json 2> $OUT/bench_churnfast.log ;;
    churnslow) MQM_FAST_REPLAY=0 timeout -k 10 700 python3 -u bench.py --workload churn --steps 2 --warmup 1 \
             --serve-churn-s 30 --churn-build-threads 4,2 > $OUT/bench_churnslow.json 2> $OUT/bench_churnslow.log ;;
    edges) timeout -k 10 400 $PYT tests/test_gpu_edges.py tests/test_commit.py -m gpu --timeout 200 \
             > $OUT/pytest_edges.log 2>&1 ;;
    churndiag) timeout -k 10 520 python3 -u bench.py --workload churn --steps 2 --warmup 1 --serve-churn-s 12 \
             --churn-build-threads 4,16,-1 > $OUT/bench_churn.json 2> $OUT/bench_churn.log ;;
    vecab) MQM_WINCOPY_VEC=1 timeout -k 10 500 $PYT tests/test_gpu_parity.py tests/test_gpu_fast.py -m gpu --timeout 300 \
             -k "config_vs_oracle or edge_cases or full_size_c3 or kat" > $OUT/pytest_vec.log 2>&1 &&
           for V in base:X=0 vec:MQM_WINCOPY_VEC=1; do
             N=${V%%:*}; E=${V#*:}
             env $E timeout -k 10 400 python3 -u bench.py $FAST --ident-steps 0 > $OUT/bench_fast_$N.json 2> $OUT/bench_fast_$N.log || exit 1
             env $E timeout -k 10 600 python3 -u bench.py --config 4 --shard 0/8 $FAST --ident-steps 0 > $OUT/bench_c4_$N.json \
               2> $OUT/bench_c4_$N.log || exit 1
           done ;;
    ident) timeout -k 10 500 $PYT tests/test_gpu_parity.py tests/test_gpu_runs.py tests/test_gpu_batching.py -m gpu \
             --timeout 200 -k "ident or batched" > $OUT/pytest_ident.log 2>&1 ;;
    c4test) timeout -k 10 600 $PYT tests/test_gpu_c4_shard.py -m gpu --timeout 500 > $OUT/pytest_c4.log 2>&1 ;;
    ret) timeout -k 10 600 $PYT tests/test_gpu_retained.py -m gpu --timeout 300 > $OUT/pytest_ret.log 2>&1 ;;
    nobloom) MQM_NO_BLOOM=1 timeout -k 10 400 $PYT tests/test_gpu_parity.py -m gpu --timeout 200 \
             -k "edge_cases or random_ops or config_vs_oracle" > $OUT/pytest_nobloom.log 2>&1 ;;
    fastt) timeout -k 10 500 $PYT tests/test_gpu_fast.py tests/test_gpu_batching.py tests/test_gpu_shim.py -m gpu \
             --timeout 200 > $OUT/pytest_fast.log 2>&1 ;;
    quick) timeout -k 10 600 $PYT tests -m gpu --timeout 300 -k "not full_size and not 20m and not 5m and not config4" \
             > $OUT/pytest_quick.log 2>&1 ;;
    lat) timeout -k 10 600 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --host-topics 0 \
             > $OUT/bench_lat.json 2> $OUT/bench_lat.log ;;
    hostab) for V in dma:X=0 kern:MQM_D2H_KERNEL=1 hwq8:GPU_MAX_HW_QUEUES=8 kernhwq8:MQM_D2H_KERNEL=1:GPU_MAX_HW_QUEUES=8; do
          N=${V%%:*}; E=$(echo ${V#*:} | tr ':' ' ')
          env $E timeout -k 10 500 python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --latency-topics 0 \
            --steady-steps 0 --ident-steps 0 > $OUT/bench_host_$N.json 2> $OUT/bench_host_$N.log || exit 1
        done ;;
    hostthreads) for T in ${HOST_THREADS:-4 12 16}; do
          timeout -k 10 500 python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --latency-topics 0 \
            --steady-steps 0 --ident-steps 0 --host-threads $T > $OUT/bench_host_t$T.json 2> $OUT/bench_host_t$T.log || exit 1
        done ;;
    kcopyt) timeout -k 10 400 $PYT tests/test_gpu_runs.py -m gpu --timeout 200 > $OUT/pytest_kcopy.log 2>&1 ;;
    freshtest) timeout -k 10 600 $PYT -s tests/test_gpu_fresh.py tests/test_gpu_serve_churn.py tests/test_gpu_serve.py -m gpu \
             --timeout 300 > $OUT/pytest_fresh.log 2>&1 ;;
    xcdab) for V in base:X=0 xcd:MQM_WALK_XCD=1; do
          N=${V%%:*}; E=${V#*:}
          env $E timeout -k 10 400 python3 -u bench.py $FAST --ident-steps 0 > $OUT/bench_fast_$N.json 2> $OUT/bench_fast_$N.log || exit 1
          env $E timeout -k 10 400 python3 -u bench.py $FAST --ident-steps 0 --sort-topics > $OUT/bench_fast_sorted_$N.json \
            2> $OUT/bench_fast_sorted_$N.log || exit 1
        done ;;
    xcdpar) MQM_WALK_XCD=1 timeout -k 10 600 $PYT tests/test_gpu_parity.py tests/test_gpu_queued.py -m gpu --timeout 300 \
             > $OUT/pytest_xcd.log 2>&1 ;;
    sortab) for V in sorted:X=0 batch:MQM_WALK_SORT=0 sorted2:X=0; do
          N=${V%%:*}; E=${V#*:}
          env $E timeout -k 10 400 python3 -u bench.py $FAST > $OUT/bench_fast_$N.json 2> $OUT/bench_fast_$N.log || exit 1
        done ;;
    freshleg) timeout -k 10 900 python3 -u bench.py --workload churn --steps 2 --warmup 1 --serve-churn-s 20 \
             --churn-build-threads 2 > $OUT/bench_churn.json 2> $OUT/bench_churn.log ;;
    c2) timeout -k 10 600 python3 -u bench.py --config 2 --steps 10 --warmup 3 --host-topics 0 --latency-topics 0 \
             --steady-steps 0 --cpu-seconds 10 > $OUT/bench_c2.json 2> $OUT/bench_c2.log ;;
    c4fast) timeout -k 10 600 python3 -u bench.py --config 4 --shard 0/8 $FAST > $OUT/bench_c4_fast.json 2> $OUT/bench_c4_fast.log ;;
    c4pmc) (cd /tmp && export TMPDIR=/tmp && for C in FETCH_SIZE WRITE_SIZE; do
             timeout -s KILL 400 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/c4pmc/pmc_$C -o pmc \
             -- python3 $ROOT/bench.py --config 4 --shard 0/8 --steps 1 --warmup 1 --no-cpu-baseline --host-topics 0 \
             --latency-topics 0 --steady-steps 0 > $OUT/c4pmc_$C.json 2> $OUT/c4pmc_$C.log || exit 1; done) &&
             python3 profiles/pmc_to_traffic.py $OUT/c4pmc > $OUT/traffic_c4.json ;;
    pmc) (cd /tmp && export TMPDIR=/tmp && for C in FETCH_SIZE WRITE_SIZE; do
             timeout -s KILL 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/pmc/pmc_$C -o pmc \
             -- python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --host-topics 0 \
             --latency-topics 0 --steady-steps 0 > $OUT/pmc_$C.json 2> $OUT/pmc_$C.log || exit 1; done) &&
             python3 profiles/pmc_to_traffic.py $OUT/pmc > $OUT/traffic.json ;;
    pipe) for P in 2 3; do timeout -k 10 400 python3 -u bench.py $FAST --pipeline $P > $OUT/bench_fast_pipe$P.json \
             2> $OUT/bench_fast_pipe$P.log || exit 1; done ;;
    par) timeout -k 10 600 $PYT tests/test_gpu_parity.py tests/test_gpu_queued.py -m gpu --timeout 300 \
             > $OUT/pytest_par.log 2>&1 ;;
    duplex) (timeout -k 10 200 tools/_build/duplex_probe 128 16 && timeout -k 10 200 tools/_build/duplex_probe 32 64 \
             && timeout -k 10 200 tools/_build/duplex_probe 128 16 2048) > $OUT/duplex_probe.txt 2>&1 ;;
    l2probe) timeout -k 10 120 tools/_build/l2_probe > $OUT/l2_probe.txt 2>&1 ;;
    reuseprobe) timeout -k 10 120 tools/_build/reuse_probe > $OUT/reuse_probe.txt 2>&1 ;;
    pollprobe) timeout -k 10 120 tools/_build/poll_probe > $OUT/poll_probe.txt 2>&1 ;;
    freeprobe) timeout -k 10 60 tools/_build/free_probe > $OUT/free_probe.txt 2>&1 ;;
    calib) timeout -k 10 120 tools/_build/calib_fetch > $OUT/calib_kernels.txt 2>&1 ;;
    smoke) timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 ;;
    bench) timeout -k 10 600 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.log ;;
    fast) timeout -k 10 400 python3 -u bench.py $FAST > $OUT/bench_fast.json 2> $OUT/bench_fast.log ;;
    prof) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv \
             -d $OUT/prof -o prof -- python3 $ROOT/bench.py $FAST --pipeline 0 \
             > $OUT/bench_under_rocprof.json 2> $OUT/rocprof.log) ;;
    c4shard) timeout -k 10 700 python3 -u bench.py --config 4 --shard 0/8 --steps 5 --warmup 2 --host-topics 0 \
             --latency-topics 0 --cpu-seconds 10 > $OUT/bench_c4_shard0of8.json 2> $OUT/bench_c4_shard0of8.log ;;
    c4prof) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv \
             -d $OUT/prof_c4 -o prof -- python3 $ROOT/bench.py --config 4 --shard 0/8 --steps 3 --warmup 1 --pipeline 0 \
             --no-cpu-baseline --host-topics 0 --latency-topics 0 > $OUT/c4_under_rocprof.json 2> $OUT/rocprof_c4.log) ;;
    c4host) timeout -k 10 700 python3 -u bench.py --config 4 --shard 0/8 --steps 3 --warmup 1 --no-cpu-baseline \
             --latency-topics 0 --steady-steps 0 > $OUT/bench_c4_host.json 2> $OUT/bench_c4_host.log ;;
    rev) timeout -k 10 900 python3 -u bench.py --workload reverse --steps 5 --warmup 1 --cpu-seconds 10 \
             > $OUT/bench_reverse.json 2> $OUT/bench_reverse.log ;;
    revnt) for V in nt:X=0 plain:MQM_REV_NT=0; do
          N=${V%%:*}; E=${V#*:}
          env $E timeout -k 10 600 python3 -u bench.py --workload reverse --steps 5 --warmup 1 --no-cpu-baseline \
            > $OUT/bench_reverse_$N.json 2> $OUT/bench_reverse_$N.log || exit 1
        done ;;
    revpmc) (cd /tmp && export TMPDIR=/tmp && for C in FETCH_SIZE WRITE_SIZE; do
             timeout -s KILL 500 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $OUT/revpmc/pmc_$C -o pmc \
             -- python3 $ROOT/bench.py --workload reverse --steps 1 --warmup 1 --no-cpu-baseline \
             > $OUT/revpmc_$C.json 2> $OUT/revpmc_$C.log || exit 1; done) &&
             python3 profiles/pmc_to_traffic.py $OUT/revpmc > $OUT/traffic_reverse.json ;;
    revprof) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
             -d $OUT/prof_rev -o prof -- python3 $ROOT/bench.py --workload reverse --steps 2 --warmup 1 --no-cpu-baseline \
             > $OUT/rev_under_rocprof.json 2> $OUT/rocprof_rev.log) ;;
    counters) bash profiles/run_pmc_r02.sh $TAG/pmc_c3 > $OUT/pmc_c3.log 2>&1 &&
             python3 profiles/derive_counters.py $OUT/pmc_c3 --json $OUT/c3_counters.json > $OUT/c3_counters.txt &&
             python3 profiles/pmc_to_traffic.py $OUT/pmc_c3 > $OUT/traffic.json ;;
    c4counters) bash profiles/run_pmc_r02.sh $TAG/pmc_c4 --config 4 --shard 0/8 > $OUT/pmc_c4.log 2>&1 &&
             python3 profiles/derive_counters.py $OUT/pmc_c4 --json $OUT/c4_counters.json > $OUT/c4_counters.txt &&
             python3 profiles/pmc_to_traffic.py $OUT/pmc_c4 > $OUT/traffic_c4.json ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[run_r06] done $(date +%T)"
