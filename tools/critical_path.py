"""Approximate critical path of one bench step from a rocprofv3 kernel trace.

Walks back from the step's last kernel: the predecessor of a kernel is the kernel (any queue)
whose end is the latest at or before that kernel's start (+1 µs of launch skew); a same-queue
kernel ending within 10 µs of that one is preferred (a side-queue kernel starved of CUs by it
ends just after it).  Prints the
chain's time per kernel family, the idle gaps along it, and the chain itself (last step).

usage: python tools/critical_path.py run_kernel_trace.csv [--list]"""
import collections
import csv
import re
import sys


def main():
    rows = []
    for r in csv.DictReader(open(sys.argv[1])):
        n = re.sub(r"^void ", "", r["Kernel_Name"])
        n = re.sub(r"\(anonymous namespace\)::", "", n)
        n = re.split(r"[<(]", n, 1)[0]
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n, int(r["Queue_Id"]),
                     int(r.get("Grid_Size", 0) or 0)))
    rows.sort()
    st = [i for i, r in enumerate(rows) if r[2].startswith("k_augment")]
    sel = rows[st[-2]:st[-1]]
    t0 = sel[0][0]
    chain = [sel[-1]]
    cur = sel[-1]
    while True:
        cands = [r for r in sel if r[1] <= cur[0] + 1000 and r is not cur and r[0] < cur[0]]
        if not cands:
            break
        p = max(cands, key=lambda r: r[1])
        # a side-queue kernel whose blocks only got CUs once a main-queue kernel drained ends a
        # few µs after it: credit the same-queue kernel, the one that actually held the chip
        same = [r for r in cands if r[3] == cur[3] and r[1] >= p[1] - 10000]
        if same:
            p = max(same, key=lambda r: r[1])
        chain.append(p)
        cur = p
    chain.reverse()
    wall = (sel[-1][1] - t0) / 1e3
    busy = collections.defaultdict(lambda: [0, 0.0])
    gap = 0.0
    for a, b in zip(chain, chain[1:]):
        gap += max(0, b[0] - a[1]) / 1e3
    for r in chain:
        busy[r[2]][0] += 1
        busy[r[2]][1] += (r[1] - r[0]) / 1e3
    tot = sum(v[1] for v in busy.values())
    print(f"step span {wall:.1f} us; chain {len(chain)} kernels, {tot:.1f} us in kernels, "
          f"{gap:.1f} us in gaps\n")
    print("| kernel | on chain | us | % of span |\n|---|---:|---:|---:|")
    for k, (c, t) in sorted(busy.items(), key=lambda kv: -kv[1][1]):
        print(f"| `{k}` | {c} | {t:.1f} | {100 * t / wall:.1f} |")
    if "--list" in sys.argv:
        print("\n| t (us) | kernel | queue | grid | us | gap before |\n|---:|---|---:|---:|---:|---:|")
        prev = None
        for r in chain:
            g = (r[0] - prev[1]) / 1e3 if prev else 0.0
            print(f"| {(r[0] - t0) / 1e3:.1f} | `{r[2]}` | {r[3]} | {r[4]} | "
                  f"{(r[1] - r[0]) / 1e3:.1f} | {g:.1f} |")
            prev = r


if __name__ == "__main__":
    main()
