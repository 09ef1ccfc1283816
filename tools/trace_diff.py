"""Per-kernel difference of two rocprofv3 kernel traces of bench steps (e.g. N = 1 vs the
forced-comm N > 1 step): wall per step, busy per queue, and the kernels whose time or count per
step changed most.  Steps are delimited by the first kernel of each step (k_augment).

usage: python tools/trace_diff.py A.csv B.csv [STEPS] > out.md"""
import collections
import csv
import re
import sys


def load(path, steps):
    rows = []
    for r in csv.DictReader(open(path)):
        n = re.sub(r"^void ", "", r["Kernel_Name"])
        n = re.sub(r"\(anonymous namespace\)::", "", n)
        n = re.split(r"[<(]", n, 1)[0]
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n, int(r["Queue_Id"])))
    rows.sort()
    st = [i for i, r in enumerate(rows) if r[2].startswith("k_augment")]
    sel = rows[st[-steps - 1]:st[-1]]
    tot = collections.defaultdict(lambda: [0, 0.0])
    q = collections.defaultdict(float)
    for s, e, n, qq in sel:
        tot[n][0] += 1
        tot[n][1] += (e - s) / 1e3
        q[qq] += (e - s) / 1e3
    wall = (rows[st[-1]][0] - rows[st[-steps - 1]][0]) / 1e3 / steps
    return ({k: (c / steps, t / steps) for k, (c, t) in tot.items()},
            sorted((t / steps for t in q.values()), reverse=True), wall)


def main():
    a_path, b_path = sys.argv[1], sys.argv[2]
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    a, qa, wa = load(a_path, steps)
    b, qb, wb = load(b_path, steps)
    print(f"wall/step: A {wa:.1f} us, B {wb:.1f} us (B - A = {wb - wa:+.1f} us)\n")
    print("busy per queue (us/step, largest first): A", [round(v, 1) for v in qa],
          " B", [round(v, 1) for v in qb], "\n")
    print("| kernel | A calls | A us | B calls | B us | B - A us |")
    print("|---|---:|---:|---:|---:|---:|")
    keys = sorted(set(a) | set(b), key=lambda k: -abs(b.get(k, (0, 0))[1] - a.get(k, (0, 0))[1]))
    for k in keys[:30]:
        ca, ta = a.get(k, (0, 0))
        cb, tb = b.get(k, (0, 0))
        print(f"| `{k}` | {ca:.0f} | {ta:.1f} | {cb:.0f} | {tb:.1f} | {tb - ta:+.1f} |")


if __name__ == "__main__":
    main()
