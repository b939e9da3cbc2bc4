"""Per-kernel average of rocprofv3 --pmc counter CSVs: python3 pmc_summary.py DIR..."""
import collections
import csv
import re
import sys

for d in sys.argv[1:]:
    rows = list(csv.DictReader(open(f"{d}/pmc_counter_collection.csv")))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in rows:
        m = re.search(r"(k_\w+(<[^>]*>)?)", r["Kernel_Name"])
        if not m:
            continue
        agg[m.group(1)][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[m.group(1)].add(r["Dispatch_Id"])
    for k, cs in agg.items():
        nd = len(disp[k])
        print(d, k, nd, {c: round(v / nd) for c, v in cs.items()})
