"""Summarise a rocprofv3 kernel_stats.csv (per-kernel totals) into markdown for profiles/."""
import csv
import sys
from pathlib import Path


def main(stats_csv, steps, title):
    rows = list(csv.DictReader(open(stats_csv)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    out = [f"# {title}", "", f"Source: `{stats_csv}` (rocprofv3 --kernel-trace --stats), "
           f"{steps} profiled steps (incl. warmup).", "",
           f"GPU kernel time: {tot / 1e6:.2f} ms total, {tot / 1e6 / steps:.2f} ms/step", "",
           "| kernel | calls/step | ms/step | % | avg us |", "|---|---:|---:|---:|---:|"]
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        t = float(r["TotalDurationNs"])
        if t / tot < 0.001:
            continue
        out.append(f"| `{r['Name'][:60]}` | {int(r['Calls']) / steps:.1f} | {t / 1e6 / steps:.3f} | "
                   f"{100 * t / tot:.1f} | {float(r['AverageNs']) / 1e3:.1f} |")
    return "\n".join(out) + "\n"


if __name__ == "__main__":
    print(main(sys.argv[1], int(sys.argv[2]), sys.argv[3]))
