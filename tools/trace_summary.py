"""Summarise a rocprofv3 kernel_trace.csv of a bench run into per-step numbers.

Steps are delimited by the one-per-step ``k_augment`` dispatch (the step's first kernel; the
optimizer update is issued per stage since round 5, so ``k_lars_update`` is no longer one per step).  Prints (1) per-kernel
totals averaged over the last ``--steps`` complete steps and (2) the ordered dispatch list of
the final step (name, grid, µs) so kernels can be mapped back to layers.

Usage: python tools/trace_summary.py TRACE.csv [--steps 5] [--list] > out.md
"""
import argparse
import csv
from collections import OrderedDict


def _name(k: str, n: int) -> str:
    k = k.replace("(anonymous namespace)::", "").replace("void ", "")
    return k.split("(")[0][:n]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--list", action="store_true")
    ap.add_argument("--marker", default="k_augment")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    if len(ends) < a.steps + 1:
        raise SystemExit(f"only {len(ends)} steps in trace")
    lo = ends[-a.steps - 1] + 1
    hi = ends[-1] + 1
    sel = rows[lo:hi]
    tot = OrderedDict()
    for r in sel:
        name = _name(r["Kernel_Name"], 70)
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        c = tot.setdefault(name, [0, 0.0])
        c[0] += 1
        c[1] += d
    wall = (int(sel[-1]["End_Timestamp"]) - int(sel[0]["Start_Timestamp"])) / 1e3 / a.steps
    busy = sum(v[1] for v in tot.values()) / a.steps
    print(f"steps={a.steps} wall/step={wall / 1e3:.3f} ms  kernel-busy/step={busy / 1e3:.3f} ms\n")
    print("| kernel | calls/step | ms/step | % |\n|---|---:|---:|---:|")
    for k, (n, t) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        print(f"| `{k}` | {n / a.steps:.1f} | {t / a.steps / 1e3:.3f} | {100 * t / a.steps / busy:.1f} |")
    if a.list:
        print("\n## last step, in order\n\n| # | kernel | grid | LDS | us |\n|---|---|---:|---:|---:|")
        last = rows[ends[-2] + 1:ends[-1] + 1]
        for i, r in enumerate(last):
            name = _name(r["Kernel_Name"], 60)
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            grid = r.get("Grid_Size_X", r.get("Grid_Size", "?"))
            lds = r.get("Group_Segment_Size", r.get("LDS_Block_Size", "?"))
            print(f"| {i} | `{name}` | {grid} | {lds} | {d:.1f} |")


if __name__ == "__main__":
    main()
