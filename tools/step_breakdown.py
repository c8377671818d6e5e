"""Per-training-step kernel breakdown from a rocprofv3 kernel trace (CSV).

Splits the trace into steps at the flat-AdamW tick kernel (one per step), takes the median
step among the last ``--steps`` ones, and prints time per kernel family.
    python tools/step_breakdown.py gpurun_out/<tag>/prof/run_kernel_trace.csv [--steps 10]
"""
import argparse
import collections
import csv
import re
import statistics


def family(name: str) -> str:
    n = re.sub(r"\(.*", "", name.replace("(anonymous namespace)::", "")).replace("void ", "")
    n = re.sub(r"<.*", "", n) if n.startswith("at::") else n
    if n.startswith("Cijk_"):
        return "rocBLAS/hipBLASLt GEMM " + re.search(r"MT\w+?_", n).group(0)[:-1]
    n = n.replace("gine::(anonymous namespace)::", "gine::")
    return n[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--marker", default="k_adamw")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    cuts = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    steps = [rows[cuts[k] + 1:cuts[k + 1] + 1] for k in range(len(cuts) - 1)][-a.steps:]
    spans = [(int(s[-1]["End_Timestamp"]) - int(s[0]["Start_Timestamp"])) / 1e3 for s in steps]
    busy = [sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in s) / 1e3
            for s in steps]
    med = sorted(range(len(steps)), key=lambda k: spans[k])[len(steps) // 2]
    step = steps[med]
    print(f"{len(cuts)} steps in trace; median step span {spans[med]:.1f} us, kernel-busy "
          f"{busy[med]:.1f} us, {len(step)} kernels (spans: min {min(spans):.1f} "
          f"median {statistics.median(spans):.1f} max {max(spans):.1f})")
    tot, cnt = collections.Counter(), collections.Counter()
    for r in step:
        f = family(r["Kernel_Name"])
        tot[f] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        cnt[f] += 1
    for f, t in tot.most_common():
        print(f"{t:9.1f} us {cnt[f]:4d}x {t / cnt[f]:8.2f} us/launch  {f}")


if __name__ == "__main__":
    main()
