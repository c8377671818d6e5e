"""Per-kernel pipe utilisation from tools/gpu_pipes.sh's two PMC passes: every counter
divided by SQ_BUSY_CU_CYCLES of the same kernel (ratios comparable between kernels).
    python tools/pipes_summary.py gpurun_out/<tag>"""
import collections
import csv
import re
import sys


def short(name: str) -> str:
    m = re.search(r"(gine::(?:\(anonymous namespace\)::)?(\w+)(<[^()]*>)?)", name)
    if not m:
        return name[:40]
    return (m.group(2) + (m.group(3) or ""))[:46]


def load(path):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        vals[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in vals.items()}


def main():
    base = sys.argv[1]
    a = load(f"{base}/pmc_A/run_counter_collection.csv")
    b = load(f"{base}/pmc_B/run_counter_collection.csv")
    cols = [("mfma", "SQ_VALU_MFMA_BUSY_CYCLES", a), ("valu", "SQ_ACTIVE_INST_VALU", a),
            ("lds", "SQ_ACTIVE_INST_LDS", a), ("vmem", "SQ_ACTIVE_INST_VMEM", a),
            ("wait", "SQ_WAIT_ANY", a), ("ldsidx", "SQ_LDS_IDX_ACTIVE", b),
            ("ldsconf", "SQ_LDS_BANK_CONFLICT", b), ("ldsfull", "SQ_LDS_DATA_FIFO_FULL", b),
            ("tafull", "SQ_VMEM_TA_ADDR_FIFO_FULL", b)]
    print("kernel".ljust(48) + "busyCU(k)".rjust(10) + "".join(n.rjust(9) for n, _, _ in cols))
    rows = sorted(a.items(), key=lambda kv: -kv[1].get("SQ_BUSY_CU_CYCLES", 0))
    for k, d in rows:
        busy = d.get("SQ_BUSY_CU_CYCLES", 0)
        if busy < 1e5:
            continue
        line = k.ljust(48) + f"{busy / 1e3:10.0f}"
        for _, c, src in cols:
            v = src.get(k, {}).get(c)
            line += f"{v / busy:9.3f}" if v is not None else " " * 9
        print(line)


if __name__ == "__main__":
    main()
