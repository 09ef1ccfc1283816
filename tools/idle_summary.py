"""GPU idle time per training step from a rocprofv3 kernel trace: the union of all kernels'
[start, end) intervals (any queue) over the last STEPS steps, and the gaps between them.  Idle
time inside a step is either host starvation (the issuing thread fell behind the GPU) or a
dependency bubble (a kernel waiting on an event from another stream).

usage: python tools/idle_summary.py run_kernel_trace.csv [STEPS] [STEP_MARKER_KERNEL]
Steps are delimited by the first kernel of each step (default: k_augment)."""
import csv
import re


def _short(name: str) -> str:
    """Kernel base name from a (possibly untruncated) demangled rocprofv3 name."""
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    return re.split(r"[<(]", name, 1)[0]
import sys


def main():
    path = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    marker = sys.argv[3] if len(sys.argv) > 3 else "k_augment"
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), _short(r["Kernel_Name"]),
                         int(r["Queue_Id"])))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if r[2].startswith(marker)]
    if len(starts) < steps + 1:
        sys.exit(f"only {len(starts)} step markers")
    lo, hi = starts[-steps - 1], starts[-1]
    sel = rows[lo:hi]
    t0, t1 = sel[0][0], rows[hi][0]
    busy, gaps = 0, []
    cur_s, cur_e = sel[0][0], sel[0][1]
    prev_name = sel[0][2]
    for s, e, name, q in sel[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, prev_name, name))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        prev_name = name if e >= cur_e else prev_name
    busy += cur_e - cur_s
    wall = t1 - t0
    idle = wall - busy
    print(f"steps={steps} wall/step={wall / steps / 1e6:.3f} ms  busy/step={busy / steps / 1e6:.3f} ms"
          f"  idle/step={idle / steps / 1e6:.3f} ms ({100.0 * idle / wall:.1f}%)")
    buckets = [(0, 1000), (1000, 5000), (5000, 20000), (20000, 10 ** 12)]
    for a, b in buckets:
        g = [x for x in gaps if a <= x[0] < b]
        print(f"  gaps {a / 1e3:>5.0f}-{b / 1e3 if b < 10 ** 12 else float('inf'):>5.0f} us: "
              f"{len(g) / steps:6.1f}/step  {sum(x[0] for x in g) / steps / 1e3:8.1f} us/step")
    agg = {}
    for d, a, b in gaps:
        k = (a.split("(")[0][:40], b.split("(")[0][:40])
        agg[k] = agg.get(k, 0) + d
    print("largest idle transitions (prev kernel -> next kernel):")
    for (a, b), d in sorted(agg.items(), key=lambda kv: -kv[1])[:12]:
        print(f"  {d / steps / 1e3:8.1f} us/step  {a} -> {b}")


if __name__ == "__main__":
    main()
