"""Per-kernel averages of a rocprofv3 counter_collection.csv (one row per dispatch x counter)."""
import csv
import sys
from collections import defaultdict


def main(path):
    rows = list(csv.DictReader(open(path)))
    agg = defaultdict(lambda: defaultdict(list))
    for r in rows:
        k = r.get("Kernel_Name", "?").replace("(anonymous namespace)::", "").replace("void ", "")
        k = k.split("(")[0][:48]
        try:
            v = float(r.get("Counter_Value", "nan"))
        except ValueError:
            continue
        agg[k][r.get("Counter_Name", "?")].append(v)
    names = sorted({c for d in agg.values() for c in d})
    print("| kernel | dispatches | " + " | ".join(f"mean {n}" for n in names) + " |")
    print("|---|---:|" + "---:|" * len(names))
    order = sorted(agg.items(), key=lambda kv: -max(len(v) for v in kv[1].values()))
    for k, d in order:
        n = max(len(v) for v in d.values())
        cells = []
        for c in names:
            v = d.get(c, [])
            cells.append(f"{sum(v) / len(v):.3g}" if v else "")
        print(f"| `{k}` | {n} | " + " | ".join(cells) + " |")


if __name__ == "__main__":
    main(sys.argv[1])
