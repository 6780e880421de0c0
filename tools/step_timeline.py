"""One training step's kernel timeline from a rocprofv3 kernel trace.

Steps are cut at a marker kernel launched once per step (default
sample_kernel). For the last --steps steps it prints span, GPU-busy time
(union of kernel intervals over every queue) and idle gaps; for the median
step the kernel sequence with durations and the gap before each launch, and
per-kernel totals per step.

    python tools/step_timeline.py <kernel_trace.csv> [--marker sample_kernel] [--steps 8]
"""
from __future__ import annotations

import argparse
import csv
import re
from collections import defaultdict


def short(name: str) -> str:
    n = re.sub(r"^void ", "", name)
    n = re.sub(r"\(.*$", "", n)
    n = n.replace("bbgr::", "")
    return n[:70]


def load(path: str):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                         short(r["Kernel_Name"]), r.get("Grid_Size_X", r.get("Grid_Size", ""))))
    rows.sort()
    return rows


def busy(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="sample_kernel")
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--index", type=int, default=None,
                    help="print this segment (counted from the first marker) instead of "
                         "the median of the last --steps")
    a = ap.parse_args()
    rows = load(a.trace)
    marks = [i for i, r in enumerate(rows) if a.marker in r[2]]
    if len(marks) < 2:
        raise SystemExit(f"fewer than 2 '{a.marker}' launches in the trace")
    steps = [(marks[k], marks[k + 1]) for k in range(len(marks) - 1)]
    steps = steps[a.index:a.index + 1] if a.index is not None else steps[-a.steps:]
    stats = []
    for i0, i1 in steps:
        seg = rows[i0:i1]
        span = rows[i1][0] - seg[0][0]
        stats.append((span, busy([(s, e) for s, e, _, _ in seg]), i0, i1))
    print("step  span_us  busy_us  idle_us  launches")
    for span, b, i0, i1 in stats:
        print(f"      {span / 1e3:8.1f} {b / 1e3:8.1f} {(span - b) / 1e3:8.1f} {i1 - i0:6d}")
    med = sorted(stats)[len(stats) // 2]
    _, _, i0, i1 = med
    seg = rows[i0:i1]
    print(f"\nmedian step: span {med[0] / 1e3:.1f} us, busy {med[1] / 1e3:.1f} us")
    print("   start_us   dur_us  gap_us  kernel [grid]")
    t0, last_end = seg[0][0], seg[0][0]
    for s, e, n, g in seg:
        print(f"{(s - t0) / 1e3:10.1f} {(e - s) / 1e3:8.1f} {(s - last_end) / 1e3:7.1f}  {n} [{g}]")
        last_end = max(last_end, e)
    tot = defaultdict(lambda: [0, 0])
    for s, e, n, _ in seg:
        tot[n][0] += 1
        tot[n][1] += e - s
    print("\nper step: calls  total_us  kernel")
    for n, (c, t) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        print(f"{c:6d} {t / 1e3:9.1f}  {n}")


if __name__ == "__main__":
    main()
