"""Summarise rocprofv3 --pmc CSV output per kernel (mean counter value per dispatch).
    python tools/pmc_summary.py gpurun_out/<tag>/<pass>/run_counter_collection.csv [...]
With --traffic-json OUT, writes {kernel: HBM bytes per launch} using the gfx950
correction of MI355X_MICROARCH.md (FETCH_SIZE reports half of a wide streaming read:
bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024)."""
import argparse
import collections
import csv
import json
import re


def short(name):
    n = name.replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", n).replace("void ", "")
    return n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--traffic-json")
    ap.add_argument("--filter", default="gine::")
    ap.add_argument("--config", default="cfg2", help="bench configuration the counters ran on")
    ap.add_argument("--tree-hash", default=None,
                    help="bench.source_tree_hash() of the tree the counters ran on")
    a = ap.parse_args()
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in a.files:
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if a.filter and a.filter not in k:
                continue
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    counters = sorted({c for k in vals for c in vals[k]})
    print("kernel".ljust(48) + "".join(c[:16].rjust(17) for c in counters))
    traffic = {}
    for k in sorted(vals):
        row = {c: (sum(v) / len(v) if v else float("nan")) for c, v in vals[k].items()}
        print(k[:48].ljust(48) + "".join(f"{row.get(c, float('nan')):17.1f}" for c in counters))
        if "FETCH_SIZE" in row and "WRITE_SIZE" in row:
            traffic[k] = round((2 * row["FETCH_SIZE"] + row["WRITE_SIZE"]) * 1024)
    if a.traffic_json:
        traffic["_config"] = a.config
        if a.tree_hash:
            traffic["_tree"] = a.tree_hash
        json.dump(traffic, open(a.traffic_json, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
