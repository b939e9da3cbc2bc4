#!/usr/bin/env python3
"""bench.py — publish-routing match throughput on MI355X.

One "step" = one TopicsIndex.Subscribers pass (topics.go:484-555) of the HIP
path over a batch of publish topics already resident in HBM, through the C ABI
(mqm_match_device_async on one of --pipeline contexts, default 2: a step
submits its batch and collects the one submitted two steps earlier, and every
timed batch is complete before the timed region ends; --pipeline 0: one
blocking mqm_match_device per step): tokenize + walk -> scans -> solo copy +
merges -> per-topic segments of deliveries + shared candidates.  Workload (BASELINE.json `metric` is quoted "at 10M filters"):
configs[2], 10M wildcard-heavy filters (40% '+', 10% '#', topics Zipf(1.2)
over filter rank), 10M-topic batch, synthetic (tools/mqgen, seed 0x4D510003).

N > 1 (torchrun, one rank per GPU, RCCL): --mode replicas (default) gives
every rank the full trie and its own 10M-topic batch (weak scaling, no
data-path collective); --mode sharded splits the subscribers by client range
and every shard matches the whole batch: with --gather host (default) each
shard's runs-form result lands in pinned host memory over its own PCIe link
(no data-path collective; DESIGN §6: the node step is PCIe-bound there), with
--gather device rank 0's batch is RCCL-broadcast and every shard's dense
per-topic lists go back to rank 0 over RCCL send/recv, where
mqm_gather_shards lays them out as the node-wide CSR, in chunks of topics
sized so one gathered chunk fits --gather-budget-gb on rank 0
(maxmq_amd/shard.py node_step / plan_chunk); --mode hybrid runs GPUs /
--shards independent replica groups of --shards subscriber shards each (own
process group, own batch, own leader).

Rank 0 prints ONE JSON line.  `roofline.achieved` = algorithmic bytes of the
match pipeline (B = T + 8N + 8P + 8V + 8S + 8D, per-topic walk
counters from the oracle on the CPU sample) / its HIP-event time per batch.
`cpu_baseline` = oracle/mochi_ref.c (C restatement of the reference matcher,
kind "port") on this host's cores over a time-bounded sample of the batch.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=3, help="BASELINE configs index + 1 (mqgen config)")
    ap.add_argument("--filters", type=int, default=0, help="override n_filters")
    ap.add_argument("--topics", type=int, default=0, help="override n_topics")
    ap.add_argument("--mode", choices=["replicas", "sharded", "hybrid"], default="replicas",
                    help="replicas: full trie per GPU, own batch each; sharded: subscriber shards over all GPUs, "
                         "one batch; hybrid: --shards subscriber shards x (GPUs / --shards) topic replicas")
    ap.add_argument("--shards", type=int, default=2, help="hybrid: subscriber shards per replica group")
    ap.add_argument("--gather", choices=["host", "device"], default="host",
                    help="sharded/hybrid: host = every shard runs the host path (runs form) over the whole batch "
                         "and its clients' deliveries land in its own pinned host memory over its own PCIe link "
                         "(no data-path collective); device = the shards' dense lists go to the group leader "
                         "over RCCL and mqm_gather_shards lays out one node-wide CSR there (bound by the "
                         "leader's xGMI ingress, DESIGN §6)")
    ap.add_argument("--gather-budget-gb", type=float, default=48.0,
                    help="sharded/hybrid: HBM the group leader may hold for one gathered chunk (received lists "
                         "+ laid-out node CSR); topics per gather are sized from it (shard.plan_chunk)")
    ap.add_argument("--shard", default="",
                    help="R/N: this one GPU matches shard R of the N-way subscriber-sharded config "
                         "(the per-shard cost of a node run, e.g. --config 4 --shard 0/8)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline time budget")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (0 = one per CPU this process may run on, BASELINE.md §2)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--host-topics", type=int, default=500000,
                    help="PCIe-inclusive host path (mqm_match_batch): topics per call, outside the timed region; 0 = skip")
    ap.add_argument("--host-passes", type=int, default=8,
                    help="host-path legs: passes over the batch in the to_host leg (many calls: no start / tail effect)")
    ap.add_argument("--host-threads", type=int, default=4,
                    help="host path: concurrent callers (each its own stream), batches overlapped across them "
                         "(4: the best of 4 / 8 / 12 / 16 measured, r06i / r06j — more callers queue more copies "
                         "behind each other's and their kernels behind them)")
    ap.add_argument("--sort-topics", action="store_true",
                    help="(diagnostic, not a bench line) the device batch reordered by its first 8 bytes: how much "
                         "of the walk is prefix locality (with MQM_WALK_XCD=1: one XCD per eighth of the batch)")
    ap.add_argument("--pipeline", type=int, default=2,
                    help="timed steps through the queued device API on this many contexts / streams (a step "
                         "submits its batch and waits for the one submitted that many steps earlier; every "
                         "batch's result is complete before the timed region ends): a broker streaming batches, "
                         "one batch's walk overlapping the previous one's emission (2: 746.7M vs 712.5M topics/s "
                         "blocking on one box, 3: 727.8M, profiles/r04/r04ac); 0 = one blocking "
                         "mqm_match_device call per step")
    ap.add_argument("--steady-steps", type=int, default=20,
                    help="steady-state leg: batches queued back to back on two contexts (0 = skip)")
    ap.add_argument("--ident-steps", type=int, default=3,
                    help="Identifiers leg (the drop-in's MQM_CFG_IDENTIFIERS configuration): blocking batches "
                         "with and without the Identifiers pass; 0 = skip")
    ap.add_argument("--latency-topics", type=int, default=2000,
                    help="single-topic mqm_subscribers calls timed for the per-publish latency; 0 = skip")
    ap.add_argument("--conc-threads", type=int, default=64,
                    help="latency leg: concurrent single-topic callers (direct, then batched)")
    ap.add_argument("--conc-calls", type=int, default=200, help="latency leg: calls per concurrent caller")
    ap.add_argument("--workload", choices=["forward", "reverse", "churn"], default="forward",
                    help="forward: Subscribers (headline); reverse: Messages over retained topics (config 5); "
                         "churn: Subscribe/Unsubscribe at rate with background snapshot rebuilds")
    ap.add_argument("--churn-ops", type=int, default=1000000, help="churn: mutations per round (half unsubscribes)")
    ap.add_argument("--serve-churn-s", type=float, default=30.0,
                    help="churn: seconds of per-publish calls (64 native callers through MQM_CFG_SERVE) while "
                         "--churn-rate Subscribe/Unsubscribe per second run (0 = skip)")
    ap.add_argument("--churn-rate", type=float, default=100000.0, help="churn: mutations/s during the served leg")
    ap.add_argument("--churn-build-threads", default="2,4,16,-1",
                    help="churn: comma-separated host thread counts for the background rebuild "
                         "(mqm_build_threads), one served-under-churn leg each (-1: no rebuild during the leg)")
    ap.add_argument("--churn-fresh-legs", default="2",
                    help="churn: build thread counts of the served-under-churn legs with MQM_CFG_FRESH corrections "
                         "on (mqm_fresh_policy; the legs above run with them off: the snapshot's view)")
    ap.add_argument("--retained", type=int, default=50000000, help="reverse: retained topics")
    ap.add_argument("--sweep", default="",
                    help="tuning sweep before the measurement: ';'-separated variants of "
                         "'ENV=V,ENV=V' (runtime knobs, e.g. MQM_RESOLVE_MIN=769); per-variant kernel ms to stderr")
    ap.add_argument("--traffic-json", default="",
                    help="PMC-derived HBM bytes per batch (profiles/pmc_to_traffic.py); default: the file of this "
                         "workload, profiles/traffic.json (config 3) or profiles/traffic_c4.json (config 4 shard), "
                         "none for other workloads")
    return ap.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def _heartbeat(period=60.0):
    """a progress line every `period` s while long host phases (generation,
    index build, CPU baseline) run, so a watchdog never mistakes them for a hang"""
    import threading

    t0 = time.time()

    def beat():
        while True:
            time.sleep(period)
            log(f"[heartbeat] {time.time() - t0:.0f}s")

    threading.Thread(target=beat, daemon=True).start()


def spawn_ranks(args):
    """--gpus N > 1 outside torchrun: start N rank processes (one per GPU) with
    torch.distributed.run and exit with its status.  Runs before anything
    touches the GPU (the parent never initialises HIP)."""
    import socket
    import subprocess

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    log(f"[bench] starting {args.gpus} ranks: {' '.join(cmd)}")
    return subprocess.call(cmd, env=env)


def cpu_threads(args):
    """one thread per CPU this process may actually run on —
    its affinity mask, capped by its cgroup CPU quota (the GPU box grants a
    16-CPU share of a 2 x 64-core host: more threads would only time-slice) —
    unless --cpu-threads says otherwise."""
    info = host_info()
    avail = info.get("cpus_affinity") or os.cpu_count() or 1
    q = info.get("cgroup_cpu_quota")
    if q:
        avail = min(avail, max(1, int(q)))
    return max(1, args.cpu_threads or avail)


def host_info():
    """visible CPUs, affinity, cgroup CPU quota, physical cores, model"""
    info = {"cpus_visible": os.cpu_count()}
    try:
        info["cpus_affinity"] = len(os.sched_getaffinity(0))
    except AttributeError:
        pass
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()
            info["cgroup_cpu_quota"] = None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        pass
    try:
        cores, model = set(), ""
        phys = core = None
        with open("/proc/cpuinfo") as fh:
            for ln in fh:
                k, _, v = ln.partition(":")
                k, v = k.strip(), v.strip()
                if k == "model name":
                    model = v
                elif k == "physical id":
                    phys = v
                elif k == "core id":
                    core = v
                elif not k and phys is not None:
                    cores.add((phys, core))
        info["physical_cores"] = len(cores) or None
        info["model"] = model
    except OSError:
        pass
    return info


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    _heartbeat()
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    import maxmq_amd
    from maxmq_amd import shard
    from tools import mqgen

    if args.workload == "reverse":
        return run_reverse(args, dist, rank, world, local, dev)
    if args.workload == "churn":
        return run_churn(args, dist, rank, world, local, dev)

    overrides = {}
    if args.filters:
        overrides["n_filters"] = args.filters
    if args.topics:
        overrides["n_topics"] = args.topics
    sharded = args.mode in ("sharded", "hybrid") and world > 1
    shard_of = tuple(int(x) for x in args.shard.split("/")) if args.shard else None
    if sharded:
        # replica groups of k subscriber shards (sharded: one group of all ranks)
        k = world if args.mode == "sharded" else args.shards
        groups, lay = shard.hybrid_layout(world, k)
        pgs = [dist.new_group(g_) for g_ in groups]  # every rank creates every group, in order
        grp, my_shard = lay[rank]
        pg, leader = pgs[grp], groups[grp][0]
    t0 = time.time()
    if sharded:  # this rank's client range only (a 100M-filter config is never whole on one host)
        w = shard.generated_shard(args.config, k, my_shard, **overrides)
    elif shard_of:
        w = shard.generated_shard(args.config, shard_of[1], shard_of[0], **overrides)
    else:
        w = mqgen.generate(args.config, **overrides)
    n = len(w.topics)
    log(f"[rank {rank}] generated {len(w.filters)} filters / {n} topics in {time.time() - t0:.1f}s")

    # ---- build the index (host store -> snapshot -> HBM) -------------------------------
    t0 = time.time()
    idx = maxmq_amd.TopicsIndex(device=local, autocommit=False)
    idx.subscribe_workload(w)
    idx.commit()
    snap = idx.snapshot_stats()
    log(f"[rank {rank}] index built in {time.time() - t0:.1f}s: {snap}")

    if args.sort_topics:
        sdata, soffs = _sorted_by_prefix(w.topics.data, w.topics.offs)
        tb = torch.from_numpy(sdata).to(dev)
        to = torch.from_numpy(soffs.view(np.int64)).to(dev)
        log(f"[rank {rank}] device batch sorted by its first 8 bytes (diagnostic)")
    else:
        tb = torch.from_numpy(w.topics.data).to(dev)
        to = torch.from_numpy(w.topics.offs.view(np.int64)).to(dev)
    stream = torch.cuda.current_stream(dev)
    chunk = n
    if sharded and args.gather == "host":
        # every shard runs the host path over the group's whole batch: the
        # batch is node input in host memory (every rank process holds the
        # same generated topics, as a shared pinned buffer would); each shard
        # matches it against its client range and its deliveries land in its
        # own pinned host memory, consumed on its caller threads (iterate)
        hrun, _, hper, hnb, _, _ = host_runner(idx, w, args, "runs")
        for _ in range(2):
            hrun(args.host_threads, 0)
        log(f"[rank {rank}] group {grp} shard {my_shard}/{k}: host gather, {hnb} calls of {hper} topics per step")
    if sharded and args.gather == "device":
        from maxmq_amd.devbuf import copy_from_ptr

        # shard client id -> node client id (the generator's global client
        # index), every shard's map held by its group leader, which lays the
        # gathered lists out
        mine = torch.from_numpy(shard.local_client_map(w).astype(np.int32)).to(dev)
        cmaps = shard.gather_maps(dist, mine, dst=leader, group=pg)
        bufs, node, cache = {}, {}, {}

        def grow(buf, key, count, dtype):
            if key not in buf or buf[key].numel() < count:
                buf.pop(key, None)
                buf[key] = torch.empty(max(int(count * 1.25), 1), dtype=dtype, device=dev)
            return buf[key][:count]

        def match_chunk(c0, c1):
            """this shard's dense CSR of topics [c0, c1) (the offsets array is
            absolute into the batch bytes, so a chunk is a pointer offset)"""
            m = c1 - c0
            idx.match_device(tb.data_ptr(), to.data_ptr() + 8 * c0, m, stream.cuda_stream)
            d = idx.dense_device(stream.cuda_stream)
            nd, ns = int(d.n_deliveries), int(d.n_shared)
            o = copy_from_ptr(grow(bufs, "offs", m + 1, torch.int64), d.offsets)
            dl = copy_from_ptr(grow(bufs, "d", nd, torch.int64), d.deliveries)
            so = copy_from_ptr(grow(bufs, "soffs", m + 1, torch.int64), d.shared_offsets)
            sl = copy_from_ptr(grow(bufs, "s", ns, torch.int32), d.shared)
            return o, dl, so, sl

        def layout(c0, c1, parts, sparts):
            """group leader: the chunk's node-wide CSRs (mqm_gather_shards*)"""
            m = c1 - c0
            tot = sum(int(p[1].numel()) for p in parts)
            stot = sum(int(p[1].numel()) for p in sparts)
            maxmq_amd.gather_shards(m, [(o.data_ptr(), dl.data_ptr(), cmaps[i].data_ptr(), cmaps[i].numel())
                                        for i, (o, dl) in enumerate(parts)],
                                    grow(node, "offs", m + 1, torch.int64).data_ptr(),
                                    grow(node, "d", tot, torch.int64).data_ptr(), stream.cuda_stream)
            maxmq_amd.gather_shards_shared(m, [(o.data_ptr(), sl.data_ptr()) for o, sl in sparts],
                                           grow(node, "soffs", m + 1, torch.int64).data_ptr(),
                                           grow(node, "s", stot, torch.int32).data_ptr(), stream.cuda_stream)

        # topics per gather: the group's deliveries per topic over the batch's
        # first topics, summed over its shards, against the leader's budget
        probe = min(n, 200000)
        _, pdl, _, psl = match_chunk(0, probe)
        tot = torch.tensor([pdl.numel(), psl.numel()], dtype=torch.float64, device=dev)
        dist.all_reduce(tot, group=pg)
        dpt, spt = float(tot[0]) / probe, float(tot[1]) / probe
        chunk = shard.plan_chunk(n, dpt * 1.1, spt * 1.1, args.gather_budget_gb * 1e9)
        log(f"[rank {rank}] group {grp} shard {my_shard}/{k}: {dpt:.0f} node deliveries per topic -> "
            f"{chunk} topics per gather ({(n + chunk - 1) // chunk} gathers per step)")

    pipe = {}
    if args.pipeline > 0 and not sharded:
        pipe["streams"] = [torch.cuda.Stream(dev) for _ in range(args.pipeline)]
        pipe["ctxs"] = [idx.match_context() for _ in range(args.pipeline)]
        pipe["pend"] = [False] * args.pipeline
        pipe["k"] = 0

    def drain():
        """pipelined steps: wait for every batch still in flight (their results)"""
        out = []
        for c in range(args.pipeline):
            if pipe["pend"][c]:
                out.append(pipe["ctxs"][c].wait())
                pipe["pend"][c] = False
        return out

    def step():
        if pipe:
            # the queued device API: submit this step's batch on the next
            # context, collect the batch that context held (submitted
            # `--pipeline` steps ago); the device always has the next batches
            # queued, so one batch's walk overlaps another's emission
            c = pipe["k"] % args.pipeline
            pipe["k"] += 1
            r_ = pipe["ctxs"][c].wait() if pipe["pend"][c] else None
            pipe["ctxs"][c].submit(tb.data_ptr(), to.data_ptr(), n, pipe["streams"][c].cuda_stream)
            pipe["pend"][c] = True
            return r_, (int(r_.n_deliveries) if r_ else 0), (int(r_.n_shared) if r_ else 0)
        if sharded and args.gather == "host":
            _, nd_ = hrun(hnb, 1)
            return None, nd_, 0
        if sharded:
            # the publish batch enters at the group leader and is broadcast over
            # xGMI (RCCL); every shard matches it chunk by chunk and its dense
            # lists go back to the leader (RCCL send/recv), laid out there
            nd_, ns_ = shard.node_step(dist, tb, to, match_chunk, layout, chunk, src=leader, group=pg, cache=cache)
            return None, nd_, ns_
        r_ = idx.match_device(tb.data_ptr(), to.data_ptr(), n, stream.cuda_stream)
        return r_, int(r_.n_deliveries), int(r_.n_shared)

    for _ in range(args.warmup):
        step()
    if pipe:
        drain()
        # the index's own workspace (the isolated batches timed per stage after
        # the timed region) sized now, so those batches allocate nothing
        idx.match_device(tb.data_ptr(), to.data_ptr(), n, stream.cuda_stream)
    torch.cuda.synchronize(dev)
    if args.sweep:
        run_sweep(args, idx, step, dev, rank)
    idx.profile(True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    deliveries = 0
    shared = 0
    fallback = 0
    big = 0
    why = {}
    lists = {}
    results = []
    for _ in range(args.steps):
        results.append(step())
    if pipe:  # the batches still in flight belong to the timed steps
        results += [(r_, int(r_.n_deliveries), int(r_.n_shared)) for r_ in drain()]
    for r, nd_, ns_ in results:
        deliveries += nd_
        shared += ns_
        if r is None:  # sharded node step: per-shard kernel statistics are not summed over chunks
            continue
        fallback = int(r.n_fallback)
        big = int(r.n_big)
        why = dict(zip(["frontier", "hits", "levels", "shared_hits", "raw_entries"], list(r.fallback_why)))
        lists = {"resolve": int(r.n_resolve), "merge_small": int(r.n_merge_small), "merge_wave": int(r.n_merge_wave),
                 "solo_ranges": int(r.n_solo_ranges), "solo_deliveries": int(r.n_solo), "group_merge": int(r.n_big), "tier2": int(r.n_tier2), "tier3": int(r.n_tier3),
                 "multi_entries_by_tier": [int(x) for x in r.multi_entries]}
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    if pipe:
        # kernel times of the stages: isolated (blocking) batches on the index's
        # own workspace after the timed region (the pipelined contexts overlap
        # batches, so a batch has no device time of its own there)
        # (the contexts stay open until the end: freeing their ~30 GB of
        # workspace here slowed the host-path leg that follows, 113M vs 156M
        # topics/s on one box, r04al / r04am)
        idx.profile(False)
        idx.profile(True)
        for _ in range(3):
            idx.match_device(tb.data_ptr(), to.data_ptr(), n, stream.cuda_stream)
        torch.cuda.synchronize(dev)
    prof = idx.profile_read()
    idx.profile(False)
    if dist:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        dsum = torch.tensor([deliveries, shared], dtype=torch.float64, device=dev)
        dist.all_reduce(dsum)
        deliveries, shared = int(dsum[0].item()), int(dsum[1].item())

    if sharded:
        # every shard of a group walks the group's batch: node-wide lists of n
        # topics per step and group
        topics_total = n * args.steps * len(groups)
    else:
        topics_total = n * args.steps * world
    value = topics_total / dt
    out = None
    if rank == 0:
        calls = max(prof["calls"], 1)
        kms = {k: prof[f"{k}_ms"] / calls for k in ("walk", "dedupe", "total")}
        cpu = None
        stats = None
        # per-GPU side measurements at N = 1 only (the contract's cpu_baseline
        # leg; host path and latency are per-GPU properties too); at N > 1 the
        # oracle runs only a short sample for the roofline's algorithmic bytes
        host = host_path(idx, w, args, "runs") if args.host_topics and world == 1 else None
        if host:
            host["packed"] = host_path(idx, w, args, "packed")
        steady = steady_state(idx, tb, to, n, dev, args) if world == 1 and not shard_of and args.steady_steps else None
        gproxy = gather_proxy(idx, tb, to, n, dev, args, shard_of[1]) if world == 1 and shard_of else None
        lat = latency(idx, w, args) if args.latency_topics and world == 1 else None
        ident = identifiers_leg(idx, tb, to, n, dev, args) if args.ident_steps and world == 1 else None
        if not args.no_cpu_baseline:
            if world == 1:
                cpu, stats = cpu_baseline(w, args)
            else:
                short = argparse.Namespace(**dict(vars(args), cpu_seconds=min(args.cpu_seconds, 2.0)))
                _, stats = cpu_baseline(w, short)
        tj = args.traffic_json
        if not tj and not args.filters and not args.topics:  # counters are per workload
            if args.config == 3 and not shard_of:
                tj = os.path.join(ROOT, "profiles", "traffic.json")
            elif args.config == 4 and shard_of:
                tj = os.path.join(ROOT, "profiles", "traffic_c4.json")
        roof = roofline(stats, n, kms, tj, dt * 1e3 / args.steps if pipe else None)
        out = {
            "metric": "publish topics matched/sec (node) + matched deliveries/sec at 10M filters",
            "value": value,
            "unit": "topics/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "strong" if sharded and len(groups) == 1 else "weak",
            "vs_baseline": None,
            "dtype": "u8/u32 (byte+integer matching)",
            "data": "synthetic (tools/mqgen, deterministic seed); inputs resident in HBM",
            "config": {
                "workload": (f"mqgen config {args.config} shard {shard_of[0]}/{shard_of[1]} (client range), " if shard_of
                             else f"mqgen config {args.config} {args.mode} over {world} GPU(s) ({len(groups)} "
                                  f"group(s) of {k} subscriber shards, " + (
                                      f"{chunk} topics per gather to the group leader" if args.gather == "device" else
                                      "each shard's results to its own pinned host memory, runs form") + "), rank 0 holds "
                             if sharded else f"mqgen config {args.config}: ") + f"{len(w.filters)} filters "
                            f"({w.params['p_plus']:.0%} '+', {w.params['p_hash']:.0%} '#', "
                            f"topic Zipf s={w.params['topic_zipf_s']}), {n}-topic batch, depth<={w.params['max_depth']}",
                "filters": len(w.filters),
                "topics_per_batch": n,
                "pipeline": (f"{args.pipeline} contexts / streams (queued device API)" if pipe else
                             "one blocking mqm_match_device per step"),
                "parallelism": (f"shard{shard_of[0]}of{shard_of[1]}" if shard_of else
                                f"hybrid{k}x{len(groups)}" if sharded and args.mode == "hybrid" else f"{args.mode}{world}"),
            },
            "deliveries_per_s": deliveries / dt,
            "shared_candidates_per_s": shared / dt,
            "deliveries_per_topic": deliveries / max(topics_total, 1),
            "fallback_topics_per_batch": fallback,
            "big_topics_per_batch": big,
            "fallback_reasons": why,
            "emit_lists": lists,
            "kernel_ms": kms,
            "snapshot": snap,
            "roofline": roof,
            "cpu_baseline": cpu,
            "host_path": host,
            "gather_proxy": gproxy,
            # SURVEY §8(d)'s end-to-end definition (pinned topics in -> usable
            # per-topic rows in host memory), beside the HBM-resident `value`
            "end_to_end": ({"value": host["value"], "unit": "topics/s", "form": host["form"],
                            "definition": "SURVEY 8(d): pinned topics in -> CSR result in pinned host memory",
                            "with_every_delivery_read": host["legs"]["iterate"]["value"]} if host else None),
            "steady_state": steady,
            "single_topic_latency": lat,
            "identifiers": ident,
        }
        print(json.dumps(out), flush=True)
    for c in pipe.get("ctxs", []):
        c.close()
    if dist:
        dist.barrier()
        dist.destroy_process_group()


def identifiers_leg(idx, tb, to, n, dev, args):
    """The drop-in's real configuration: the Go shim creates its index with
    MQM_CFG_IDENTIFIERS, because Subscription.Merge always
    builds the Identifiers map (packets.go:250-259).  --ident-steps blocking
    batches of the same 10M topics, each mqm_match_device followed by
    mqm_identifiers_device (k_ident over the walk's records), against the same
    number of blocking batches without it; inputs resident in HBM."""
    import torch

    stream = torch.cuda.current_stream(dev)

    def timed(with_ids):
        idx.match_device(tb.data_ptr(), to.data_ptr(), n, stream.cuda_stream)  # warm
        if with_ids:
            idx.identifiers_device(stream.cuda_stream)
        torch.cuda.synchronize(dev)
        t_ids, nid = 0.0, 0
        t0 = time.perf_counter()
        for _ in range(args.ident_steps):
            idx.match_device(tb.data_ptr(), to.data_ptr(), n, stream.cuda_stream)
            if with_ids:
                t1 = time.perf_counter()
                d = idx.identifiers_device(stream.cuda_stream)  # (synchronises: it reads the total back)
                t_ids += time.perf_counter() - t1
                nid = int(d.n_idents)
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / args.ident_steps, t_ids / args.ident_steps, nid

    plain, _, _ = timed(False)
    after, ids_after, nid = timed(True)  # the pass after the match
    idx.identifiers_early(True)  # the pass beside the match's merges (mqm_identifiers_early)
    try:
        both, ids, nid_e = timed(True)
    finally:
        idx.identifiers_early(False)
    assert nid_e == nid, (nid_e, nid)
    return {"value": n / both, "unit": "topics/s", "ms_per_step": both * 1e3, "match_only_ms_per_step": plain * 1e3,
            "identifiers_extra_ms": (both - plain) * 1e3, "identifiers_share_of_step": (both - plain) / both,
            "collect_ms": ids * 1e3,
            "after_the_match": {"value": n / after, "ms_per_step": after * 1e3, "identifiers_pass_ms": ids_after * 1e3},
            "listed_sids_per_topic": nid / n,
            "what": "blocking mqm_match_device + mqm_identifiers_device per 10M-topic batch (the shim's "
                    "MQM_CFG_IDENTIFIERS configuration), the pass beside the merges (mqm_identifiers_early; "
                    "after_the_match: run after it), vs blocking mqm_match_device alone"}


def steady_state(idx, tb, to, n, dev, args):
    """SURVEY §8(d) steady state: --steady-steps batches queued back to back
    through the queued device API (mqm_match_device_async), two contexts on
    two streams, the host waiting only for the batch queued two steps earlier
    (so the device always has the next batch queued).  Inputs resident in
    HBM; the same batch each time."""
    import torch

    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    ctxs = [idx.match_context(), idx.match_context()]
    for c, st in zip(ctxs, streams):  # size each context (its first batch is exact)
        c.submit(tb.data_ptr(), to.data_ptr(), n, st.cuda_stream)
        c.wait()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    pend = [False, False]
    dsum = 0
    for k in range(args.steady_steps):
        c = k % 2
        if pend[c]:
            dsum += int(ctxs[c].wait().n_deliveries)
        ctxs[c].submit(tb.data_ptr(), to.data_ptr(), n, streams[c].cuda_stream)
        pend[c] = True
    for c in (0, 1):
        if pend[c]:
            dsum += int(ctxs[c].wait().n_deliveries)
    dt = time.perf_counter() - t0
    requeued = sum(c.requeued() for c in ctxs)
    for c in ctxs:
        c.close()
    return {"value": args.steady_steps * n / dt, "unit": "topics/s", "batches": args.steady_steps,
            "ms_per_batch": dt * 1e3 / args.steady_steps, "deliveries_per_s": dsum / dt, "contexts": 2,
            "requeued_batches": requeued,
            "note": "mqm_match_device_async on 2 contexts / 2 streams, host waits only for the batch queued two "
                    "steps earlier; no read-back inside a batch (outputs sized by the contexts' first batch)"}


def _sorted_by_prefix(data, offs):
    """(--sort-topics) the batch reordered by the big-endian key of each
    topic's first 8 bytes (zero past its end), stable"""
    o = offs.astype(np.int64)
    lens = np.diff(o)
    pad = np.concatenate([data, np.zeros(8, np.uint8)])
    key = np.zeros(len(lens), np.uint64)
    for k in range(8):
        b = pad[o[:-1] + k].astype(np.uint64)
        b[lens <= k] = 0
        key |= b << np.uint64(56 - 8 * k)
    perm = np.argsort(key, kind="stable")
    lp = lens[perm]
    no = np.zeros(len(lens) + 1, np.int64)
    np.cumsum(lp, out=no[1:])
    src = np.repeat(o[:-1][perm] - no[:-1], lp) + np.arange(no[-1], dtype=np.int64)
    return np.ascontiguousarray(data[src]), no.astype(np.uint64)


def host_path(idx, w, args, form="runs"):
    """The boundary's host form as a broker drives it (SURVEY §8d end to end):
    topics in pinned host memory -> H2D -> the match pipeline -> result D2H
    into pinned, library-owned blocks -> consumed on the calling thread.
    --host-threads native callers (tools/conc_driver.cpp mqd_host_path; no
    interpreter lock) each take --host-topics-topic batches of the C3 batch in
    turn, each with its own workspace and HIP stream (include/mqmatch.h,
    Threading), so one batch's copies and consumption overlap another's
    kernels.  form "packed": mqm_match_batch_packed (4 B per delivery over
    PCIe); "runs": mqm_match_batch_runs (8 B per solo run, 4 B per merged
    winner).  Consumption: "to_host" (the result in host memory), "iterate"
    (every delivery read once, as the cgo shim's loop over a topic's
    subscribers), "expand" (plain packed rows, mqm_result_expand).  Timed
    outside the headline's region.  `pcie_bound` = the same bytes at the link
    rates measured here (H2D and D2H run concurrently)."""
    import ctypes as C

    import torch

    from maxmq_amd import capi

    L = capi.lib()
    run, fn, per, nb, dp, op = host_runner(idx, w, args, form)
    # warm every caller's context (workspace sizing, pinned result blocks):
    # contexts come from a pool, so only concurrent calls create one each
    for _ in range(2):
        run(args.host_threads, 0)
    # the bytes one batch moves (batch 0), for the PCIe model
    res = C.c_void_p()
    capi.check("host path", fn(idx._h, C.c_void_p(dp), C.c_void_p(op), per, C.byref(res)))
    win = int(C.cast(L.mqm_result_offsets(res), C.POINTER(C.c_uint64))[per])
    sh = int(C.cast(L.mqm_result_shared_offsets(res), C.POINTER(C.c_uint64))[per])
    ro, rr, rw, nw = C.c_void_p(), C.c_void_p(), C.c_void_p(), C.c_uint64()
    n_runs = 0
    if L.mqm_result_runs(res, C.byref(ro), C.byref(rr), C.byref(rw), C.byref(nw)) == 0:
        n_runs = int(C.cast(ro, C.POINTER(C.c_uint64))[per])
    L.mqm_result_free(res)
    out_per_batch = 8 * n_runs + 4 * win + 4 * sh + (24 if form == "runs" else 16) * per
    legs = {}
    ph = (C.c_double * 6)()
    for consume, name in ((0, "to_host"), (1, "iterate"), (2, "expand")):
        L.mqm_batch_host_us(idx._h, ph)  # (reset)
        calls = nb * (args.host_passes if consume == 0 else 1)  # (the headline leg: steady state over many calls)
        dt, nd = run(calls, consume)
        legs[name] = {"value": calls * per / dt, "deliveries_per_s": nd / dt,
                      "ms_per_call": dt * 1e3 * args.host_threads / calls, "calls": calls}
        if L.mqm_batch_host_us(idx._h, ph) == 0:  # where a call's time goes (mean us per phase)
            legs[name]["phases_us"] = dict(zip(("front_ctx", "h2d", "match", "runs_densify", "d2h_sync"),
                                               (round(ph[i], 1) for i in range(5))))
    # link rates: 1 GiB pinned <-> device, each direction alone
    dev = torch.device("cuda", torch.cuda.current_device())
    g = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
    h = torch.empty(1 << 30, dtype=torch.uint8).pin_memory()
    rates = {}
    for name, (dst, src) in {"h2d": (g, h), "d2h": (h, g)}.items():
        dst.copy_(src)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(3):
            dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        rates[name] = 3 * (1 << 30) / (time.perf_counter() - t1)
    # both directions at once (two streams; tools/duplex_probe: each direction
    # slows to ~48 of ~57 GB/s while the other runs)
    g2 = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
    h2 = torch.empty(1 << 30, dtype=torch.uint8).pin_memory()
    sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(3):
        with torch.cuda.stream(sa):
            g.copy_(h, non_blocking=True)
        with torch.cuda.stream(sb):
            h2.copy_(g2, non_blocking=True)
    torch.cuda.synchronize()
    rates["both"] = 3 * (1 << 30) / (time.perf_counter() - t1)  # per direction
    del g, h, g2, h2
    n = nb * per
    in_b = int(w.topics.offs[n]) + 8 * n
    out_b = out_per_batch * nb
    bound_s = max(in_b / rates["h2d"], out_b / rates["d2h"])
    # the same bytes when the smaller direction overlaps the larger one at the
    # concurrent rate, the rest of the larger at its own rate
    ov = min(in_b, out_b) / rates["both"]
    rest = (max(in_b, out_b) - min(in_b, out_b)) / (rates["d2h"] if out_b >= in_b else rates["h2d"])
    duplex_s = max(bound_s, ov + rest)
    # SURVEY §8(d)'s end-to-end definition: topics in pinned host memory ->
    # the CSR result in pinned host memory ("to_host"; the runs form's CSR is
    # runs + winners); "iterate" adds the consumer reading every delivery
    best = legs["to_host"]
    return {"value": best["value"], "unit": "topics/s", "consume": "to_host", "form": form, "legs": legs,
            "topics_per_call": per, "calls": nb, "threads": args.host_threads,
            "d2h_bytes_per_topic": out_b / n, "runs_per_topic": n_runs / per, "winners_per_topic": win / per,
            "h2d_GBps": rates["h2d"] / 1e9, "d2h_GBps": rates["d2h"] / 1e9,
            "pcie_bound_topics_per_s": n / bound_s, "frac_of_pcie_bound": best["value"] / (n / bound_s),
            "both_directions_GBps": rates["both"] / 1e9, "pcie_duplex_bound_topics_per_s": n / duplex_s,
            "frac_of_duplex_bound": best["value"] / (n / duplex_s),
            "note": "pinned topics in -> match -> result into pinned blocks -> consumed on the calling thread (" +
                    ("mqm_match_batch_runs: 8-B solo runs of the host word table + 4-B merged winners"
                     if form == "runs" else "mqm_match_batch_packed: 4-B packed words") +
                    "); native caller threads (tools/conc_driver.cpp); pcie_bound = max(H2D bytes / H2D rate, "
                    "D2H bytes / D2H rate), each rate alone; duplex bound: the smaller direction overlapped at "
                    "the both-at-once rate"}


def gather_proxy(idx, tb, to, n, dev, args, shards=8):
    """Single-GPU proxy of the device-gather node step (`--gather device`,
    DESIGN §6): this shard's dense result of one planned chunk stands in for
    each of `shards` shards; timed on this GPU: the densify + copy-out a shard
    does per chunk, the D2D copies of the other shards' lists (a lower bound of
    their xGMI transfer: local HBM, not links) and mqm_gather_shards' layout of
    the node-wide CSR.  The xGMI time of the same bytes is projected at 7 links
    x 153 GB/s into the leader (MI355X_MICROARCH / the prompt's figure), the
    ideal; RCCL point-to-point reaches a fraction of it."""
    import torch

    import maxmq_amd
    from maxmq_amd import shard
    from maxmq_amd.devbuf import copy_from_ptr

    st = torch.cuda.current_stream(dev)
    probe = min(n, 200000)
    idx.match_device(tb.data_ptr(), to.data_ptr(), probe, st.cuda_stream)
    d = idx.dense_device(st.cuda_stream)
    dpt = int(d.n_deliveries) / probe
    chunk = shard.plan_chunk(n, shards * dpt * 1.1, 0.0, args.gather_budget_gb * 1e9)
    chunk = min(chunk, n)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    ev[0].record(st)
    idx.match_device(tb.data_ptr(), to.data_ptr(), chunk, st.cuda_stream)
    ev[1].record(st)
    d = idx.dense_device(st.cuda_stream)
    nd = int(d.n_deliveries)
    offs = copy_from_ptr(torch.empty(chunk + 1, dtype=torch.int64, device=dev), d.offsets)
    dl = copy_from_ptr(torch.empty(nd, dtype=torch.int64, device=dev), d.deliveries)
    ev[2].record(st)
    recv = [torch.empty_like(dl) for _ in range(shards - 1)]
    for r in recv:
        r.copy_(dl)
    ev[3].record(st)
    torch.cuda.synchronize(dev)
    out_o = torch.empty(chunk + 1, dtype=torch.int64, device=dev)
    out_d = torch.empty(shards * nd, dtype=torch.int64, device=dev)
    parts = [(offs.data_ptr(), dl.data_ptr(), 0, 0)] + [(offs.data_ptr(), r.data_ptr(), 0, 0) for r in recv]
    t0 = time.perf_counter()
    maxmq_amd.gather_shards(chunk, parts, out_o.data_ptr(), out_d.data_ptr(), st.cuda_stream)
    torch.cuda.synchronize(dev)
    layout_ms = (time.perf_counter() - t0) * 1e3
    ingress = (shards - 1) * nd * 8
    xgmi_ms = ingress / (7 * 153e9) * 1e3
    step_chunks = (n + chunk - 1) // chunk
    per_chunk_ms = ev[0].elapsed_time(ev[1]) + ev[1].elapsed_time(ev[2]) + max(xgmi_ms, ev[2].elapsed_time(ev[3])) + layout_ms
    del recv, out_d
    return {"shards": shards, "chunk_topics": chunk, "chunks_per_step": step_chunks,
            "deliveries_per_topic_per_shard": dpt, "leader_ingress_bytes_per_chunk": ingress,
            "match_ms": ev[0].elapsed_time(ev[1]), "densify_copy_ms": ev[1].elapsed_time(ev[2]),
            "d2d_copies_ms": ev[2].elapsed_time(ev[3]), "layout_ms": layout_ms,
            "xgmi_ideal_ms": xgmi_ms, "projected_step_ms": per_chunk_ms * step_chunks,
            "projected_node_topics_per_s": n / (per_chunk_ms * step_chunks * 1e-3),
            "note": "one GPU standing in for every shard (its own chunk result copied shards - 1 times); "
                    "serial stages, no overlap; xGMI at the 7 x 153 GB/s ideal into the leader"}


def host_runner(idx, w, args, form="runs"):
    """The native host-path driver (tools/conc_driver.cpp mqd_host_path) over
    --host-topics-topic batches of w's topics in pinned memory -> (run,
    batch entry point, topics per call, calls per pass, data / offsets
    pointers); run(n_batches, consume) -> (seconds, deliveries)."""
    import ctypes as C

    import torch

    from maxmq_amd import capi

    L = capi.lib()
    D, _ = _driver()
    vp = C.c_void_p

    class HApi(C.Structure):
        _fields_ = [("batch", vp), ("offsets", vp), ("packed", vp), ("runs", vp), ("expand", vp), ("result_free", vp)]

    fn = L.mqm_match_batch_runs if form == "runs" else L.mqm_match_batch_packed
    api = HApi(C.cast(fn, vp), C.cast(L.mqm_result_offsets, vp), C.cast(L.mqm_result_packed, vp),
               C.cast(L.mqm_result_runs, vp), C.cast(L.mqm_result_expand, vp), C.cast(L.mqm_result_free, vp))
    D.mqd_host_path.argtypes = [C.POINTER(HApi), vp, vp, vp, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, C.c_int,
                                C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    D.mqd_host_path.restype = C.c_int64
    per = min(args.host_topics, len(w.topics))
    nb = max(1, len(w.topics) // per)
    data = torch.from_numpy(w.topics.data).pin_memory()
    offs = torch.from_numpy(w.topics.offs[: nb * per + 1].astype(np.int64)).pin_memory()
    dp, op = data.data_ptr(), offs.data_ptr()
    d, c = C.c_uint64(), C.c_uint64()
    keep = (data, offs, api)  # alive as long as run is

    def run(n_batches, consume):
        ns = D.mqd_host_path(C.byref(keep[2]), idx._h, C.c_void_p(dp), C.c_void_p(op), per, n_batches, nb,
                             args.host_threads, consume, C.byref(d), C.byref(c))
        if ns < 0:
            raise RuntimeError(f"host path ({form}) call failed")
        return ns * 1e-9, d.value

    return run, fn, per, nb, dp, op


def _driver():
    """tools/_build/libmqdrive.so: native threads issuing mqm_subscribers
    calls (the reference's one-goroutine-per-connection call shape)"""
    import ctypes as C

    from maxmq_amd import capi

    L = capi.lib()
    D = C.CDLL(os.path.join(ROOT, "tools", "_build", "libmqdrive.so"))

    class Api(C.Structure):
        _fields_ = [("subscribers", C.c_void_p), ("offsets", C.c_void_p), ("result_free", C.c_void_p)]

    api = Api(C.cast(L.mqm_subscribers, C.c_void_p), C.cast(L.mqm_result_offsets, C.c_void_p),
              C.cast(L.mqm_result_free, C.c_void_p))
    D.mqd_concurrent.argtypes = [C.POINTER(Api), C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_int, C.c_int,
                                 C.c_void_p, C.POINTER(C.c_uint64)]
    D.mqd_concurrent.restype = C.c_int64
    return D, api


def latency(idx, w, args):
    """Per-publish latency and throughput of the reference's call shape: one
    Subscribers(topic) per call (server.go:776) through mqm_subscribers, host
    in / host out, issued by native threads (tools/conc_driver.cpp): one
    caller, then --conc-threads concurrent callers (one goroutine per
    connection, listeners/tcp.go:83) each calling directly, then through the
    MQM_CFG_BATCHING collector, then through the MQM_CFG_SERVE persistent
    server (one caller, then the concurrent callers)."""
    import ctypes as C

    D, api = _driver()
    n = min(max(args.latency_topics, args.conc_threads * args.conc_calls), len(w.topics))
    data = np.ascontiguousarray(w.topics.data[: int(w.topics.offs[n])])
    offs = np.ascontiguousarray(w.topics.offs[: n + 1].astype(np.uint64))

    def run(threads, calls):
        lat = np.zeros(threads * calls, np.uint64)
        dsum = C.c_uint64()
        ns = D.mqd_concurrent(C.byref(api), idx._h, data.ctypes.data_as(C.c_void_p), offs.ctypes.data_as(C.c_void_p),
                              n, threads, calls, lat.ctypes.data_as(C.c_void_p), C.byref(dsum))
        if ns < 0:
            raise RuntimeError("mqm_subscribers failed in the driver")
        us = lat.astype(np.float64) / 1e3
        return {"topics_per_s": threads * calls / (ns * 1e-9), "p50_us": float(np.median(us)),
                "p90_us": float(np.percentile(us, 90)), "p99_us": float(np.percentile(us, 99)),
                "deliveries_per_topic": dsum.value / (threads * calls)}

    single = min(args.latency_topics, n)
    run(1, 50)  # warm
    one = run(1, single)
    out = {"unit": "us", "calls": single, "p50": one["p50_us"], "p90": one["p90_us"], "p99": one["p99_us"],
           "topics_per_s": one["topics_per_s"], "driver": "native threads (tools/conc_driver.cpp)"}
    T, per = args.conc_threads, args.conc_calls
    run(T, 20)  # warm: every caller's context (stream, workspace, pinned blocks) exists before timing
    idx.direct_host_us()  # (reset)
    conc = {"threads": T, "calls_per_thread": per, "direct": run(T, per)}
    conc["direct"]["phases_us"] = idx.direct_host_us()
    idx.batching_policy(0, 0)  # MQM_CFG_BATCHING on from here
    run(T, 20)
    b0, t0_ = idx.batching_stats()
    conc["batched"] = run(T, per)
    b1, t1 = idx.batching_stats()
    conc["batched"]["mean_batch"] = (t1 - t0_) / max(1, b1 - b0)
    out["concurrent"] = conc
    # MQM_CFG_SERVE: the persistent server (fast.hip k_serve) answers every
    # call through a ring of pinned slots, no launch / stream synchronisation
    # per call; --conc-threads workgroups, so every concurrent caller has one
    idx.serve_policy(T, 20000)
    run(1, 50)
    one = run(1, single)
    single_dev_us = idx.serve_device_us()
    served = {"device_us_single": single_dev_us, "p50": one["p50_us"], "p90": one["p90_us"], "p99": one["p99_us"], "topics_per_s": one["topics_per_s"]}
    run(T, 20)
    s0 = idx.serve_stats()
    served["concurrent"] = dict(run(T, per), threads=T, calls_per_thread=per)
    s1 = idx.serve_stats()
    served["ring_share"] = (s1[0] - s0[0]) / max(1, (s1[0] - s0[0]) + (s1[1] - s0[1]))
    served["launches"] = s1[2]
    served["device_us_per_call"] = idx.serve_device_us()
    served["grid"] = T
    out["served"] = served
    return out


def run_sweep(args, idx, step, dev, rank):
    """time every variant of --sweep (env knobs read per batch by match.hip)"""
    import torch

    results = []
    for var in [v for v in args.sweep.split(";") if v.strip()]:
        kv = dict(x.split("=", 1) for x in var.split(",") if x.strip())
        old = {k: os.environ.get(k) for k in kv}
        os.environ.update(kv)
        step()
        torch.cuda.synchronize(dev)
        idx.profile(True)
        for _ in range(max(args.steps, 3)):
            step()
        torch.cuda.synchronize(dev)
        prof = idx.profile_read()
        idx.profile(False)
        calls = max(prof["calls"], 1)
        res = {"variant": var, **{f"{k}_ms": prof[f"{k}_ms"] / calls for k in ("walk", "dedupe", "total")}}
        results.append(res)
        if rank == 0:
            log(f"[sweep] {json.dumps(res)}")
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return results


def run_churn(args, dist, rank, world, local, dev):
    """Incremental Subscribe/Unsubscribe at rate on the
    headline workload: the index runs with MQM_CFG_ASYNC_COMMIT.  A round =
    --churn-ops mutations (half Unsubscribes of existing (filter, client)
    pairs, half Subscribes of existing filters by new clients) applied to the
    host store + delta log, then mqm_commit_async while match steps keep
    running on the front snapshot.  `value` = mutations/s the store absorbs;
    the line also carries the rebuild time (replay + flatten + upload) and the
    match throughput before / during / after the rebuild."""
    import torch

    import maxmq_amd
    from tools import mqgen
    from tools.mqgen import Strings

    overrides = {}
    if args.filters:
        overrides["n_filters"] = args.filters
    if args.topics:
        overrides["n_topics"] = args.topics
    w = mqgen.generate(args.config, **overrides)
    n = len(w.topics)
    t0 = time.time()
    # (MQM_CFG_FRESH: the overlay is kept from the start; the served legs switch
    # its corrections on or off with mqm_fresh_policy)
    idx = maxmq_amd.TopicsIndex(device=local, autocommit=False, async_commit=True,
                                fresh=bool(args.churn_fresh_legs.strip()))
    idx.subscribe_workload(w)
    idx.commit()
    if idx.fresh:
        idx.fresh_policy(False)  # (on for the fresh_* served legs only)
    build_s = time.time() - t0
    log(f"[rank {rank}] async index built in {build_s:.1f}s: {idx.commit_state()}")
    tb = torch.from_numpy(w.topics.data).to(dev)
    to = torch.from_numpy(w.topics.offs.view(np.int64)).to(dev)
    stream = torch.cuda.current_stream(dev)

    def timed_steps(k):
        ts = []
        for _ in range(k):
            t = time.perf_counter()
            idx.match_device(tb.data_ptr(), to.data_ptr(), n, stream.cuda_stream)
            torch.cuda.synchronize(dev)
            ts.append(time.perf_counter() - t)
        return ts

    timed_steps(args.warmup)
    before = timed_steps(args.steps)
    rng = np.random.default_rng(0x4D51C0DE)
    half = args.churn_ops // 2
    sel = rng.choice(len(w.filters), size=half, replace=False)
    un_f = Strings.from_list([w.filters[int(i)] for i in sel])
    un_c = Strings.from_list([w.clients[int(i)] for i in sel])
    sel2 = rng.choice(len(w.filters), size=half, replace=False)
    sub_f = Strings.from_list([w.filters[int(i)] for i in sel2])
    sub_c = Strings.from_list([f"churn-{j}" for j in range(half)])
    t0 = time.perf_counter()
    existed = idx.unsubscribe_many(un_f, un_c)
    is_new = idx.subscribe_many(sub_c, sub_f, w.qos[sel2], w.no_local[sel2], w.rap[sel2], w.rh[sel2], w.ident[sel2])
    mut_s = time.perf_counter() - t0
    st0 = idx.commit_state()
    t0 = time.perf_counter()
    idx.commit_async()
    submit_ms = (time.perf_counter() - t0) * 1e3
    during = []
    t_pub = None
    while len(during) < 2000 and time.perf_counter() - t0 < 300:
        during += timed_steps(1)
        if idx.commit_state()["builds"] > st0["builds"]:
            t_pub = time.perf_counter() - t0
            break
    if t_pub is None:
        idx.commit_poll(wait=True)
        t_pub = time.perf_counter() - t0
    st = idx.commit_state()
    after = timed_steps(args.steps)
    assert st["snapshot_version"] == st["store_version"], st
    med = lambda x: float(np.median(x)) * 1e3 if x else None  # noqa: E731
    out = {
        "metric": "incremental Subscribe/Unsubscribe mutations/sec absorbed, background snapshot rebuild at 10M filters",
        "value": args.churn_ops / mut_s,
        "unit": "mutations/s",
        "n_gpus": 1,
        "higher_is_better": True,
        "config": {"workload": f"mqgen config {args.config}: {len(w.filters)} filters, {n}-topic match batches; "
                               f"{half} unsubscribes + {half} subscribes per round",
                   "filters": len(w.filters)},
        "unsubscribes_existed": int(existed.sum()),
        "subscribes_new": int(is_new.sum()),
        "initial_build_s": build_s,
        "submit_ms": submit_ms,
        "rebuild_ms": st["last_build_ms"],
        "rebuild_ops": st["last_build_ops"],
        "publish_after_ms": t_pub * 1e3,
        "match_ms_median": {"before": med(before), "during_rebuild": med(during), "after": med(after)},
        "match_steps_during_rebuild": len(during),
        "commit_state": st,
    }
    if args.serve_churn_s > 0:
        out["served_under_churn"] = serve_churn(idx, w, args)
    if rank == 0:
        print(json.dumps(out), flush=True)


def serve_churn(idx, w, args):
    """Per-publish Subscribers(topic) calls through the persistent server
    (MQM_CFG_SERVE) on the async index while --churn-rate Subscribe /
    Unsubscribe per second run on another thread (the reference takes both
    concurrently: server.go:1013 / topics.go:303-321 beside server.go:776).
    Native threads (tools/conc_driver.cpp mqd_serve_churn): --conc-threads
    callers for --serve-churn-s seconds, first with no mutations (baseline),
    then with them.  The index rebuilds in the background
    (mqm_commit_policy: submit 50 ms after the first unsubmitted mutation;
    logs coalesce while a build runs), and callers match the newest published
    snapshot without taking the index lock.  Visibility lag of a mutation = the
    first return of a call whose result's snapshot version includes it, minus
    the mutation's time."""
    import ctypes as C

    from maxmq_amd import capi
    from tools.mqgen import Strings

    L = capi.lib()
    D = C.CDLL(os.path.join(ROOT, "tools", "_build", "libmqdrive.so"))

    class Api(C.Structure):
        _fields_ = [(x, C.c_void_p) for x in ("subscribers", "offsets", "result_free", "version", "subscribe",
                                              "unsubscribe", "state")]

    class Out(C.Structure):
        _fields_ = [(x, C.c_uint64) for x in ("calls", "deliveries", "mutations", "failed_mutations")] + [
            ("slow_ns", C.c_uint64 * 256), ("slow_t_us", C.c_uint64 * 256), ("n_pub", C.c_uint64),
            ("pub_t_us", C.c_uint64 * 256), ("pub_builds", C.c_uint64 * 256)]

    api = Api(*[C.cast(getattr(L, f), C.c_void_p) for f in (
        "mqm_subscribers", "mqm_result_offsets", "mqm_result_free", "mqm_result_snapshot_version", "mqm_subscribe",
        "mqm_unsubscribe", "mqm_commit_state_get")])
    vp = C.c_void_p
    D.mqd_serve_churn.argtypes = [C.POINTER(Api), vp, vp, vp, C.c_uint32, C.c_int, C.c_double, C.c_uint32,
                                  C.c_uint32, vp, vp, vp, vp, C.c_uint32, C.c_double, vp, vp, vp, vp, C.c_uint64, vp,
                                  vp, C.POINTER(Out)]
    D.mqd_serve_churn.restype = C.c_int64
    n = min(len(w.topics), 1 << 20)
    data = np.ascontiguousarray(w.topics.data[: int(w.topics.offs[n])])
    offs = np.ascontiguousarray(w.topics.offs[: n + 1].astype(np.uint64))
    m = 200000
    rng = np.random.default_rng(0x5EC4)
    sel = rng.choice(len(w.filters), size=m, replace=False)
    fl = Strings.from_list([w.filters[int(i)] for i in sel])
    cl = Strings.from_list([f"churner-{j}" for j in range(m)])
    T = args.conc_threads
    idx.commit_policy(0, 50)
    idx.serve_policy(T, 20000)
    p = lambda a: a.ctypes.data_as(vp)  # noqa: E731

    def run(seconds, rate):
        cap = int(seconds * 40000) + 1000  # calls per thread (>= 40k/s per caller)
        sample = 16
        lat = np.zeros(T * cap, np.uint32)
        done = np.zeros(T, np.uint32)
        per_s = cap // sample + 1
        s_t = np.zeros(T * per_s, np.uint32)
        s_v = np.zeros(T * per_s, np.uint64)
        mcap = int(seconds * rate * 1.2) + 1000 if rate > 0 else 1
        m_t = np.zeros(mcap, np.uint32)
        m_v = np.zeros(mcap, np.uint64)
        o = Out()
        st0 = idx.commit_state()
        c0 = idx.serve_counters()
        ns = D.mqd_serve_churn(C.byref(api), idx._h, p(data), p(offs), n, T, seconds, cap, sample, p(cl.data),
                               p(cl.offs), p(fl.data), p(fl.offs), m, rate, p(lat), p(done), p(s_t), p(s_v), mcap,
                               p(m_t), p(m_v), C.byref(o))
        if ns < 0:
            raise RuntimeError("mqm_subscribers failed in the churn driver")
        st1 = idx.commit_state()
        us = np.concatenate([lat[k * cap: k * cap + int(done[k])] for k in range(T)]).astype(np.float64) / 1e3
        r = {"seconds": ns * 1e-9, "calls": int(o.calls), "topics_per_s": o.calls / (ns * 1e-9),
             "p50_us": float(np.median(us)), "p99_us": float(np.percentile(us, 99)),
             "p999_us": float(np.percentile(us, 99.9)), "max_us": float(us.max()),
             "deliveries_per_topic": o.deliveries / max(1, o.calls),
             "p9999_us": float(np.percentile(us, 99.99)),
             "calls_over_ms": {str(t): int((us > t * 1e3).sum()) for t in (1, 10, 100, 1000)},
             "slowest_calls": sorted(([round(o.slow_ns[k] / 1e6, 3), round(o.slow_t_us[k] / 1e6, 3)]
                                      for k in range(min(T, 256))), reverse=True)[:8],
             "publishes_at_s": [round(o.pub_t_us[i] / 1e6, 3) for i in range(int(o.n_pub))],
             "snapshots_published": st1["builds"] - st0["builds"], "last_build_ms": st1["last_build_ms"]}
        if rate > 0:
            nm = int(o.mutations)
            r.update({"mutations": nm, "mutations_per_s": nm / (ns * 1e-9), "failed_mutations": int(o.failed_mutations)})
            # visibility: sampled calls in return order, the newest version seen so far
            keep = np.concatenate([np.arange(k * per_s, k * per_s + (int(done[k]) + sample - 1) // sample)
                                   for k in range(T)])
            order = np.argsort(s_t[keep], kind="stable")
            tr, vr = s_t[keep][order].astype(np.float64), np.maximum.accumulate(s_v[keep][order])
            pos = np.searchsorted(vr, m_v[:nm], side="left")  # first call whose result includes mutation k
            seen = pos < len(vr)
            lag = (tr[np.minimum(pos, len(vr) - 1)] - m_t[:nm].astype(np.float64))[seen] / 1e3
            r["visibility_lag_ms"] = ({"p50": float(np.median(lag)), "p99": float(np.percentile(lag, 99)),
                                       "max": float(lag.max())} if len(lag) else None)
            r["mutations_seen_by_a_call"] = float(seen.mean()) if nm else None
            ph = (C.c_double * 5)()
            capi.check("mqm_build_phases_ms", L.mqm_build_phases_ms(idx._h, ph))
            r["last_build_phases_ms"] = {"replay": ph[0], "flatten": ph[1], "upload": ph[2],
                                         "build_threads": int(ph[3]), "kept_shape": bool(ph[4])}
        r["host_phase_max"] = idx.serve_host_max_us()
        # the served path's safety nets during the leg (all 0 in a healthy run:
        # forced relaunches, slot / result timeouts; stale = decoded again on
        # the batch path because the result's host snapshot was gone)
        c1 = idx.serve_counters()
        r["serve_counters"] = {k: c1[k] - c0[k] for k in c1}
        return r

    run(2.0, 0)  # warm: the server, every caller's path
    base = run(min(args.serve_churn_s, 10.0), 0)
    legs = {}
    fresh_on = idx.fresh
    plan = [(int(x), False) for x in str(args.churn_build_threads).split(",") if x.strip()]
    if fresh_on:
        plan += [(int(x), True) for x in str(args.churn_fresh_legs).split(",") if x.strip()]
    for bt, fresh in plan:
        # bt < 0: no background rebuild during the leg (the mutations' own cost)
        capi.check("mqm_build_threads", L.mqm_build_threads(max(bt, 0)))
        if fresh_on:
            idx.fresh_policy(fresh)
        idx.commit_async()  # (the previous leg's mutations built and published: a fresh
        idx.commit_poll(wait=True)  # leg's overlay starts from that snapshot)
        idx.commit_policy(0, 50 if bt >= 0 else 0)
        f0 = idx.fresh_stats() if fresh else None
        name = ("fresh_" if fresh else "") + (f"build_threads_{bt}" if bt >= 0 else "no_rebuild")
        legs[name] = run(args.serve_churn_s, args.churn_rate)
        if fresh:
            f1 = idx.fresh_stats()
            fs = {k: f1[k] - f0[k] if k not in ("held_clients", "max_batch_age_ns", "max_round_ns",
                                                 "max_copy_wait_ns") else f1[k] for k in f1}
            fs["read_us_per_corrected_call"] = fs["read_ns"] / max(1, fs["calls_corrected"]) / 1e3
            fs["scan_us_per_corrected_call"] = fs["scan_ns"] / max(1, fs["calls_corrected"]) / 1e3
            legs[name]["fresh"] = fs
        log(f"[serve churn] {name}: {legs[name]}")
    if fresh_on:
        idx.fresh_policy(False)
    capi.check("mqm_build_threads", L.mqm_build_threads(0))
    idx.commit_policy(0, 50)
    return {"threads": T, "driver": "native threads (tools/conc_driver.cpp mqd_serve_churn)",
            "index": "MQM_CFG_ASYNC_COMMIT | MQM_CFG_SERVE" + (" | MQM_CFG_FRESH" if idx.fresh else "") +
                     ", commit_policy(0 ops, 50 ms); fresh_* legs: the calls corrected for every mutation so far "
                     "(include/mqmatch.h MQM_CFG_FRESH), the other legs: the published snapshot's view",
            "baseline_no_mutations": base, "under_churn": legs, "target_rate": args.churn_rate}


def run_reverse(args, dist, rank, world, local, dev):
    """Messages (topics.go:426-480) for a batch of subscription filters against
    the retained topics (BASELINE configs[4]): mqgen config 5's filters (5%
    $SHARE, 20% '+', 5% '#') also subscribed, `--retained` topics retained.
    A step = one mqm_messages_device call over the whole filter batch, inputs
    resident in HBM (device-side worklist counters: one read-back per call)."""
    import torch

    import maxmq_amd
    from tools import mqgen

    cfg = 5
    nf = args.filters or 1000000
    t0 = time.time()
    w = mqgen.generate(cfg, n_filters=nf, n_topics=args.retained)
    log(f"[rank {rank}] generated {len(w.filters)} filters / {len(w.topics)} retained topics in {time.time() - t0:.1f}s")
    t0 = time.time()
    idx = maxmq_amd.TopicsIndex(device=local, autocommit=False)
    idx.subscribe_workload(w)
    refs = np.arange(len(w.topics), dtype=np.uint64)
    idx.retain_many(w.topics, refs)
    idx.commit()
    snap = idx.snapshot_stats()
    log(f"[rank {rank}] index built in {time.time() - t0:.1f}s: {snap} retained={idx.retained_len()}")
    fb = torch.from_numpy(w.filters.data).to(dev)
    fo = torch.from_numpy(w.filters.offs.view(np.int64)).to(dev)
    stream = torch.cuda.current_stream(dev)
    n = len(w.filters)

    def step():
        return idx.messages_device(fb.data_ptr(), fo.data_ptr(), n, stream.cuda_stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    refs_out = items = ranges = skipped = 0
    for _ in range(args.steps):
        r = step()
        refs_out += int(r.n_refs)
        items += int(r.n_items)
        skipped += int(r.n_skipped)
        ranges += int(r.n_ranges)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    # full-size property check, outside the timed region: the same call twice
    # gives the same per-filter counts and the same checksum of every filter's
    # refs (order-independent: sum of mixed refs per filter)
    check = reverse_selfcheck(idx, fb, fo, n, dev, stream)
    if rank == 0:
        steps = args.steps
        tbytes = int(w.filters.offs[-1])
        # algorithmic bytes per batch, for the work this pipeline performs
        # (SURVEY §8d's forward model applied to the reverse walk): filter bytes
        # + offsets in/out (16 B) + per (filter, node) item actually loaded an
        # 8-B key probe and an 8-B descriptor read (16 B; the reference's items
        # that the literal-edge index jumps over are not charged, they are
        # reported as reference_items) + per retained hit one ref read and one
        # written (16 B)
        loaded = (items - skipped) / steps
        per_batch = tbytes + 16 * n + 16 * loaded + 16 * refs_out / steps
        achieved = per_batch / (dt / steps) / 1e9
        traffic = None  # PMC bytes per call (profiles/traffic_reverse.json, pmc_to_traffic.py --per-call)
        tj = os.path.join(ROOT, "profiles", "traffic_reverse.json")
        if os.path.exists(tj) and not args.filters and args.retained == 50_000_000:
            try:
                with open(tj) as fh:
                    traffic = json.load(fh).get("hbm_bytes_per_batch")
            except Exception:
                traffic = None
        cpu = None
        if not args.no_cpu_baseline:
            cpu = cpu_reverse(w, refs, args)
        out = {
            "metric": "retained reverse match: filters matched/sec + retained hits/sec",
            "value": n * steps * world / dt,
            "unit": "filters/s",
            "n_gpus": world,
            "steps": steps,
            "warmup": args.warmup,
            "ms_per_step": dt * 1e3 / steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8/u32 (byte+integer matching)",
            "data": "synthetic (tools/mqgen config 5, deterministic seed); inputs resident in HBM",
            "config": {"workload": f"mqgen config 5: {n} filters vs {len(w.topics)} retained topics "
                                   f"(+ the filters subscribed), depth<=8",
                       "filters_per_batch": n, "retained": len(w.topics), "parallelism": f"replicas{world}"},
            "retained_hits_per_s": refs_out * world / dt,
            "hits_per_filter": refs_out / (n * steps),
            "items_per_filter": (items - skipped) / (n * steps),
            "reference_items_per_filter": items / (n * steps),
            "selfcheck": check,
            "snapshot": snap,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "algorithmic_bytes_per_batch": per_batch,
                         "model": "T + 16 N + 16 x items loaded + 16 x retained hits",
                         "kernel": "reverse-match pipeline per batch (k_flt_*, k_level per depth, k_emit_*, "
                                   "k_task_copy; wall time, one read-back per call)"},
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


def reverse_selfcheck(idx, fb, fo, n, dev, stream):
    """Two mqm_messages_device calls on the full batch: identical per-filter
    counts and identical per-filter checksums of the refs (sum of splitmix64
    of every ref, order-independent), plus every ref below the retained count."""
    import torch

    from maxmq_amd.devbuf import dev_view_copy, segment_checksums

    def once():
        m = idx.messages_device(fb.data_ptr(), fo.data_ptr(), n, stream.cuda_stream)
        torch.cuda.synchronize(dev)
        offs = dev_view_copy(m.offsets, n + 1, torch.int64, dev)
        sums = segment_checksums(offs, m.refs, torch.int64)
        return offs, sums

    o1, s1 = once()
    o2, s2 = once()
    cnt = o1[1:] - o1[:-1]
    return {"run_to_run_counts_equal": bool(torch.equal(o1, o2)),
            "run_to_run_ref_checksums_equal": bool(torch.equal(s1, s2)),
            "offsets_monotone": bool((cnt >= 0).all()), "refs": int(o1[-1])}


def cpu_reverse(w, refs, args):
    """oracle/mochi_ref.c scan_messages over a time-bounded sample of the filters."""
    from oracle.binding import OracleIndex

    threads = cpu_threads(args)
    t0 = time.time()
    ora = OracleIndex()
    ora.subscribe_workload(w)
    ora.retain_many(w.topics, refs)
    build_s = time.time() - t0
    f = w.filters
    n = len(f)
    done, busy, hits, chunk = 0, 0.0, 0, 2000
    while done < n and busy < args.cpu_seconds:
        hi = min(n, done + chunk)
        o = (f.offs[done:hi + 1] - f.offs[done]).astype(np.uint64)
        d = f.data[int(f.offs[done]):int(f.offs[hi])]
        t1 = time.perf_counter()
        mo, _ = ora.messages(d, o, nthreads=threads)
        busy += time.perf_counter() - t1
        hits += int(mo[-1])
        done = hi
        chunk = min(chunk * 2, 100000)
    ora.close()
    host = host_info()
    out = {"value": done / busy, "unit": "filters/s", "cores": threads, "kind": "port", "host": host,
           "sample": f"first {done} filters ({busy:.1f}s of matching, index build {build_s:.0f}s excluded); "
                     f"C restatement of mochi v2.2.12 TopicsIndex.Messages (oracle/mochi_ref.c); Go toolchain "
                     f"unavailable",
           "retained_hits_per_s": hits / busy}
    out.update(cores_note(done / busy / threads, threads, host))  # (per-thread share of the parallel rate)
    return out


def cpu_baseline(w, args):
    """oracle/mochi_ref.c over a time-bounded sample (chunks of the same batch,
    from the front) on this host's cores; index build excluded."""
    from oracle.binding import OracleIndex

    threads = cpu_threads(args)
    t0 = time.time()
    ora = OracleIndex()
    ora.subscribe_workload(w)
    build_s = time.time() - t0
    data, offs = w.topics.data, w.topics.offs
    n = len(offs) - 1
    chunk = 20000
    done = 0
    busy = 0.0
    tot = None
    while done < n and busy < args.cpu_seconds:
        hi = min(n, done + chunk)
        o = (offs[done:hi + 1] - offs[done]).astype(np.uint64)
        d = data[int(offs[done]):int(offs[hi])]
        t1 = time.perf_counter()
        _, _, st = ora.match_counts(d, o, nthreads=threads)
        busy += time.perf_counter() - t1
        tot = st if tot is None else {k: tot[k] + st[k] for k in tot}
        done = hi
        chunk = min(chunk * 2, 400000)
    # single-thread rate over the front of the same sample (<= ~3 s)
    st_done, st_busy, st_chunk = 0, 0.0, 5000
    while st_done < done and st_busy < min(3.0, args.cpu_seconds / 4):
        hi = min(done, st_done + st_chunk)
        o = (offs[st_done:hi + 1] - offs[st_done]).astype(np.uint64)
        d = data[int(offs[st_done]):int(offs[hi])]
        t1 = time.perf_counter()
        ora.match_counts(d, o, nthreads=1)
        st_busy += time.perf_counter() - t1
        st_done = hi
    ora.close()
    cpu = {
        "value": done / busy,
        "unit": "topics/s",
        "cores": threads,
        "kind": "port",
        "sample": f"first {done} topics of the batch ({busy:.1f}s of matching, index build {build_s:.0f}s "
                  f"excluded); C restatement of mochi v2.2.12 TopicsIndex (oracle/mochi_ref.c); Go toolchain "
                  f"unavailable",
        "deliveries_per_s": tot["deliveries"] / busy,
        "single_thread_value": st_done / st_busy if st_busy > 0 else None,
        "host": host_info(),
    }
    cpu.update(cores_note(cpu["single_thread_value"], threads, cpu["host"]))
    return cpu, tot


def cores_note(single, threads, host):
    """BASELINE.md §2 asks for one thread per core.  The GPU box grants this
    process a cgroup CPU quota (16 CPUs of a 2 x 64-core host): more threads
    than the quota only time-slice, so `cores` is the quota.  For scale, the
    single-thread rate times the host's physical cores (an upper bound: linear
    scaling, no memory-bandwidth or SMT limit) is reported beside it."""
    phys = host.get("physical_cores")
    out = {"cores_note": f"{threads} threads = the CPUs this process may use (cgroup quota "
                         f"{host.get('cgroup_cpu_quota')}); host has {phys} physical cores"}
    if single and phys:
        out["projected_all_physical_cores"] = single * phys
    return out


def roofline(stats, n, kms, traffic_json, step_ms=None):
    """B = T + 8N + 8P + 8V + 8S + 8D algorithmic bytes per
    batch (per-topic counters of the oracle's walk over the CPU sample, scaled
    to the batch) over the device time of the whole match pipeline (k_walk,
    scans, k_emit<16|64>, k_multi, k_dfs: first to last kernel, HIP events on
    the launch stream).  `stages` splits it by kernel: k_walk (HIP events
    around it) moves T + 8N + 8P + 8V, everything after it (scans, route,
    solo copy, merges) 8S + 8D.  `traffic` = HBM bytes per batch of the same
    kernels from rocprofv3 FETCH_SIZE / WRITE_SIZE (profiles/traffic.json from
    profiles/pmc_to_traffic.py over a profiles/run_pmc_r02.sh run, reads
    converted per access shape as tools/calib_fetch calibrated them).
    With pipelined steps (--pipeline) batches overlap, so `achieved` divides by
    the time per step (throughput); the stages keep the isolated batch's kernel
    times."""
    total_ms = step_ms if step_ms else kms["total"]
    if not stats or not stats["topics"] or total_ms <= 0:
        return {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None,
                "traffic": None}
    k = stats["topics"]
    walk_b = (stats["topic_bytes"] + 8 * k + 8 * stats["probes"] + 8 * stats["visits"]) / k * n
    emit_b = (8 * stats["gathered"] + 8 * stats["deliveries"]) / k * n
    bytes_per_launch = walk_b + emit_b
    achieved = bytes_per_launch / (total_ms * 1e-3) / 1e9
    traffic = walk_traffic = None
    if traffic_json and os.path.exists(traffic_json):
        try:
            with open(traffic_json) as fh:
                tj = json.load(fh)
            traffic, walk_traffic = tj.get("hbm_bytes_per_batch"), tj.get("walk_bytes_per_batch")
        except Exception:
            traffic = None

    def stage(b, ms):
        return {"bytes": b, "ms": ms, "achieved": b / (ms * 1e-3) / 1e9 if ms > 0 else None,
                "frac": b / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS if ms > 0 else None}

    return {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
            "algorithmic_bytes_per_topic": bytes_per_launch / n, "algorithmic_bytes_per_batch": bytes_per_launch,
            "kernel": "match pipeline per batch: k_walk + scans + k_route + solo copy (k_desc, k_winmap, k_wincopy) "
                      "+ merges (k_resolve; heavy topics k_merge_small, k_merge, k_multi) + k_shared (+ k_dfs)",
            "time_basis": ("ms per pipelined step (batches overlap)" if step_ms else
                           "device time of one batch (HIP events, first to last kernel)"),
            "ms": total_ms, "isolated_batch_ms": kms["total"],
            "stages": {"walk": dict(stage(walk_b, kms["walk"]), traffic=walk_traffic),
                       "emission": stage(emit_b, kms["dedupe"])}}


if __name__ == "__main__":
    main()
