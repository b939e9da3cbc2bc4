"""HBM traffic per batch of the match kernels from rocprofv3 FETCH_SIZE /
WRITE_SIZE passes (profiles/run_pmc_r02.sh output) -> profiles/traffic.json.

Measurement infrastructure.  Calibration (tools/calib_fetch on the GPU box,
profiles/r02/r02i/calib_*): FETCH_SIZE = (L2 -> memory read requests) x 64 B,
where a 16-B/lane coalesced stream issues one request per 128-B line (so its
bytes are 2 x FETCH_SIZE, as MI355X_MICROARCH.md §HBM says) and a random
gather of 8, 32 or 64 B per lane issues one request per 64-B sector (its bytes
are 1 x FETCH_SIZE).  Reads are therefore converted per kernel by its access
shape: x1 for the gather kernels (trie walk, merges), x2 for the streaming
copies.  WRITE_SIZE is exact for 4..16-B/lane stores (same calibration).
usage: pmc_to_traffic.py <pmc dir> [> profiles/traffic.json]
"""
import collections
import csv
import glob
import json
import os
import re
import sys

GATHER = ("k_walk", "k_merge_small", "k_merge", "k_multi", "k_multi_part", "k_resolve", "k_dfs", "k_shared",
          "k_level")  # (reverse match: k_level walks the trie and the edge index)
STREAM = ("k_desc", "k_winmap", "k_wincopy", "k_route", "k_table_sizes",
          "k_flt_count", "k_flt_fill", "k_emit_count", "k_emit_place", "k_task_copy")


def kname(s):
    """kernel name with its template argument when it has one (k_multi<2048>
    -> k_multi2048: the workgroup merge tiers are reported apart)"""
    m = re.match(r"(?:void )?(?:mqm::\(anonymous namespace\)::)?(k_\w+)(?:<(\d+)[,>])?", s)
    if not m:
        return None
    return m.group(1) + (m.group(2) if m.group(1) in ("k_multi", "k_resolve") and m.group(2) else "")


def base(k):
    return re.sub(r"\d+$", "", k) if k else k


root = sys.argv[1]
# --last-call: sum every launch of the last call in each pass (the reverse
# match launches k_level once per trie depth; a call starts with k_flt_count)
last_call = "--last-call" in sys.argv
sums = {c: collections.defaultdict(float) for c in ("FETCH_SIZE", "WRITE_SIZE")}
disp = {c: collections.defaultdict(set) for c in ("FETCH_SIZE", "WRITE_SIZE")}
for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    with open(path) as fh:
        rows = list(csv.DictReader(fh))
    cut = 0
    if last_call:
        starts = [int(r["Dispatch_Id"]) for r in rows if kname(r.get("Kernel_Name", "")) == "k_flt_count"]
        cut = max(starts) if starts else 0
    for row in rows:
        c = row.get("Counter_Name")
        k = kname(row.get("Kernel_Name", ""))
        if c not in sums or base(k) not in GATHER + STREAM or int(row["Dispatch_Id"]) < cut:
            continue
        sums[c][k] += float(row["Counter_Value"])
        disp[c][k].add((path, row["Dispatch_Id"]))
kib = 1024.0
# per batch: a kernel may launch more than once per batch (the k_multi tiers
# share one name here), so divide by the batches (k_walk launches once each)
div = (lambda c, k: 1) if last_call else (lambda c, k: len(disp[c]["k_walk"]) or len(disp[c][k]))
reads = {k: v * kib * (1 if base(k) in GATHER else 2) / div("FETCH_SIZE", k) for k, v in sums["FETCH_SIZE"].items()}
writes = {k: v * kib / div("WRITE_SIZE", k) for k, v in sums["WRITE_SIZE"].items()}
out = {
    "read_bytes_per_batch_by_kernel": reads,
    "write_bytes_per_batch_by_kernel": writes,
    "walk_bytes_per_batch": reads.get("k_walk", 0) + writes.get("k_walk", 0),
    "hbm_bytes_per_batch": sum(reads.values()) + sum(writes.values()),
    "note": ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes, per launch of each match kernel; "
             "reads = FETCH_SIZE KiB x 1 (gather kernels: one request per 64-B sector) or x 2 (streaming "
             "copies: one request per 128-B line), calibrated by tools/calib_fetch; writes = WRITE_SIZE KiB"),
}
print(json.dumps(out, indent=1))
