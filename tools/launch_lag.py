"""Host-late vs dependency idle: joins a rocprofv3 kernel trace with its HIP API trace
(``--kernel-trace --hip-runtime-trace``) by correlation id.  For every idle gap of the GPU
(no kernel on any queue) inside the last STEPS steps, the kernel that ends the gap was either
enqueued by the host only after the GPU went idle (host-late: the issuing thread fell behind) or
enqueued earlier and held back by a dependency (event wait / stream barrier / boundary cost).

usage: python tools/launch_lag.py DIR [STEPS] [MARKER]   (DIR holds run_kernel_trace.csv and
run_hip_api_trace.csv)"""
import csv
import re


def _short(name: str) -> str:
    """Kernel base name from a (possibly untruncated) demangled rocprofv3 name."""
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    return re.split(r"[<(]", name, 1)[0]
import os
import sys


def main():
    d = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    marker = sys.argv[3] if len(sys.argv) > 3 else "k_augment"
    api = {}
    with open(os.path.join(d, "run_hip_api_trace.csv")) as f:
        for r in csv.DictReader(f):
            if "Launch" in r["Function"] or "launch" in r["Function"]:
                api[int(r["Correlation_Id"])] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    ks = []
    with open(os.path.join(d, "run_kernel_trace.csv")) as f:
        for r in csv.DictReader(f):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                       _short(r["Kernel_Name"])[:32], int(r["Correlation_Id"])))
    ks.sort()
    starts = [i for i, k in enumerate(ks) if k[2].startswith(marker)]
    lo, hi = starts[-steps - 1], starts[-1]
    sel = ks[lo:hi]
    cur_e = sel[0][1]
    late = dep = 0
    late_n = dep_n = 0
    worst = []
    for s, e, name, cid in sel[1:]:
        if s > cur_e + 1000:
            gap = s - cur_e
            a = api.get(cid)
            if a is not None and a[1] > cur_e:
                late += min(gap, a[1] - cur_e)
                dep += gap - min(gap, a[1] - cur_e)
                late_n += 1
                worst.append((min(gap, a[1] - cur_e), name, "host-late"))
            else:
                dep += gap
                dep_n += 1
                worst.append((gap, name, "dependency"))
        cur_e = max(cur_e, e)
    print(f"idle per step: host-late {late / steps / 1e3:.1f} us ({late_n / steps:.1f} gaps), "
          f"dependency/boundary {dep / steps / 1e3:.1f} us ({dep_n / steps:.1f} gaps)")
    agg = {}
    for g, n, kind in worst:
        agg[(n, kind)] = agg.get((n, kind), 0) + g
    for (n, kind), g in sorted(agg.items(), key=lambda kv: -kv[1])[:15]:
        print(f"  {g / steps / 1e3:8.1f} us/step  {kind:10s} before {n}")


if __name__ == "__main__":
    main()
