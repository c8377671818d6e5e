"""Mean of each rocprofv3 --pmc counter per gine kernel (template args kept).
    python tools/pmc_kernels.py run_counter_collection.csv [...]"""
import collections
import csv
import re
import sys

for f in sys.argv[1:]:
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        if "gine" not in r["Kernel_Name"]:
            continue
        m = re.search(r"(k_\w+<[^>]*>|k_\w+)", r["Kernel_Name"])
        agg[m.group(1)][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        print(k, {c: round(sum(x) / len(x)) for c, x in v.items()})
