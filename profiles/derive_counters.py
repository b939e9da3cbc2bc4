"""Per-kernel derived counters from the rocprofv3 --pmc passes of
profiles/run_pmc_r02.sh:  python3 derive_counters.py PMC_DIR [--json OUT]

Measurement infrastructure (not product code).  For every match kernel, per
launch (averaged over the launches the passes saw):

  ms              kernel duration (kernel trace of the PMC passes)
  fetch_req_M     L2 -> memory read requests (FETCH_SIZE KiB * 1024 / 64:
                  tools/calib_fetch shows one request per 64-B sector miss of a
                  random gather and per 128-B line of a 16-B/lane stream, so
                  requests, not FETCH_SIZE bytes, are comparable across access
                  shapes)
  hbm_read_GB     read bytes: requests x 64 B for gathers (lower bound), x 128 B
                  for streams (upper bound) -> both reported
  write_GB        WRITE_SIZE (exact for 4..16-B/lane stores, calibration)
  l2_hit          TCC_HIT / (TCC_HIT + TCC_MISS)
  waves_per_cu    SQ_WAVE_CYCLES * 4 / (duration * clock * CUs): mean resident
                  wavefronts per CU (SQ cycle counters tick every 4 cycles)
  lane_util       SQ_THREAD_CYCLES_VALU / (SQ_ACTIVE_INST_VALU * 64): active
                  lanes per VALU instruction (1 - divergence)
  wait_mem, wait_issue, active   SQ_WAIT_ANY, SQ_WAIT_INST_ANY,
                  SQ_ACTIVE_INST_ANY as fractions of SQ_WAVE_CYCLES
  lds_conflict    SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS
  ta_busy         TA_BUSY_avr per launch / (duration * clock / 4)
"""
import collections
import csv
import glob
import json
import os
import re
import sys

CLOCK_HZ = 2.4e9
CUS = 256


def kname(s):
    m = re.search(r"(k_\w+(<[^>]*>)?)", s)
    return m.group(1) if m else None


def main():
    d = sys.argv[1]
    cnt = collections.defaultdict(lambda: collections.defaultdict(float))
    ndisp = collections.defaultdict(lambda: collections.defaultdict(set))
    dur = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "pmc_*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = kname(r["Kernel_Name"])
            if not k:
                continue
            c = r["Counter_Name"]
            cnt[k][c] += float(r["Counter_Value"])
            ndisp[k][c].add((f, r["Dispatch_Id"]))
    for f in glob.glob(os.path.join(d, "pmc_*", "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = kname(r["Kernel_Name"])
            if k:
                dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    out = {}
    for k in sorted(cnt):
        v = {c: cnt[k][c] / max(1, len(ndisp[k][c])) for c in cnt[k]}
        if not dur[k]:
            continue
        t = sorted(dur[k])[len(dur[k]) // 2]
        g = v.get
        row = {"ms": t * 1e3}
        if "FETCH_SIZE" in v:
            req = v["FETCH_SIZE"] * 1024 / 64
            row["fetch_req_M"] = req / 1e6
            row["hbm_read_GB_gather"] = req * 64 / 1e9
            row["hbm_read_GB_stream"] = req * 128 / 1e9
        if "WRITE_SIZE" in v:
            row["write_GB"] = v["WRITE_SIZE"] * 1024 / 1e9
        if "TCC_HIT_sum" in v:
            row["l2_hit"] = g("TCC_HIT_sum") / max(1.0, g("TCC_HIT_sum") + g("TCC_MISS_sum"))
        if "SQ_WAVE_CYCLES" in v:
            wc = g("SQ_WAVE_CYCLES")
            row["waves_per_cu"] = wc * 4 / (t * CLOCK_HZ * CUS)
            row["wait_mem"] = g("SQ_WAIT_ANY", 0) / wc
            row["wait_issue"] = g("SQ_WAIT_INST_ANY", 0) / wc
            row["active"] = g("SQ_ACTIVE_INST_ANY", 0) / wc
        if "SQ_THREAD_CYCLES_VALU" in v and "SQ_INSTS_VALU" in v:
            row["lane_util"] = g("SQ_THREAD_CYCLES_VALU") / max(1.0, g("SQ_INSTS_VALU") * 64)
        if "SQ_LDS_BANK_CONFLICT" in v and "SQ_INSTS_LDS" in v:
            row["lds_conflict_per_inst"] = g("SQ_LDS_BANK_CONFLICT") / max(1.0, g("SQ_INSTS_LDS"))
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS"):
            if c in v:
                row[c] = v[c]
        if "TA_BUSY_avr" in v:
            row["ta_busy"] = g("TA_BUSY_avr") / (t * CLOCK_HZ)
        out[k] = {a: (round(b, 4) if isinstance(b, float) else b) for a, b in row.items()}
    cols = ["ms", "fetch_req_M", "write_GB", "l2_hit", "waves_per_cu", "lane_util", "wait_mem", "wait_issue",
            "active", "lds_conflict_per_inst", "ta_busy"]
    print("kernel".ljust(16) + "".join(c[:12].rjust(13) for c in cols))
    for k, row in out.items():
        print(k[:16].ljust(16) + "".join(
            (f"{row[c]:.3f}" if c in row else "-").rjust(13) for c in cols))
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
