"""Per-step totals of a rocprofv3 counter_collection.csv written for tools/step_bytes.py:
every dispatch after the cumsum marker kernel, summed per counter and per kernel family.
Usage: python tools/step_bytes_summary.py counter_collection.csv STEPS"""
import csv
import sys
from collections import defaultdict


def main(path, steps):
    rows = list(csv.DictReader(open(path)))
    key = "Dispatch_Id" if rows and "Dispatch_Id" in rows[0] else "Correlation_Id"
    rows.sort(key=lambda r: int(r.get(key, 0) or 0))
    start = None
    for r in rows:
        if "cumsum" in r.get("Kernel_Name", "").lower() or "scan" in r.get("Kernel_Name", "").lower():
            start = int(r[key])
    if start is None:
        sys.exit("marker kernel not found")
    tot = defaultdict(float)
    fam = defaultdict(lambda: defaultdict(float))
    for r in rows:
        if int(r[key]) <= start:
            continue
        try:
            v = float(r["Counter_Value"])
        except (KeyError, ValueError):
            continue
        c = r["Counter_Name"]
        k = r.get("Kernel_Name", "?").replace("(anonymous namespace)::", "").replace("void ", "")
        k = k.split("<")[0].split("(")[0][:40]
        tot[c] += v
        fam[k][c] += v
    for c, v in tot.items():
        print(f"{c}: {v / steps / 1e3:.1f} MB per step (FETCH_SIZE / WRITE_SIZE are in KB)")
    c0 = next(iter(tot))
    print(f"\n| kernel family | {c0} MB/step |\n|---|---:|")
    for k, d in sorted(fam.items(), key=lambda kv: -kv[1][c0]):
        print(f"| `{k}` | {d[c0] / steps / 1e3:.1f} |")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
