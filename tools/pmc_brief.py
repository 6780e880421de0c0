"""Per-kernel FETCH_SIZE / WRITE_SIZE of the store-policy A/B passes
(tools/gpu_run.sh storeab): one table per policy, KiB per dispatch averaged
by (kernel, grid), plus the per-dispatch sequence of the user-side products
(grid 40000000) so a single amplified launch of a step stands out.

    python tools/pmc_brief.py gpurun_out/<tag> > gpurun_out/<tag>/pmc_brief.txt
"""
import collections
import csv
import glob
import json
import os
import sys


def load(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    return rows


def main(out):
    res = {}
    for pol in ("split", "nt", "none"):
        per = collections.defaultdict(lambda: collections.defaultdict(list))
        seq = collections.defaultdict(list)
        for c in ("WRITE_SIZE", "FETCH_SIZE"):
            for r in load(os.path.join(out, f"pmc_{pol}_{c}")):
                key = f"{r['Kernel_Name']}@{r['Grid_Size']}"
                v = float(r["Counter_Value"])
                per[key][c].append(v)
                if r["Grid_Size"] == "40000000":
                    seq[c].append((int(r.get("Dispatch_Id", 0) or 0), r["Kernel_Name"], v))
        if not per:
            continue
        print(f"== policy {pol}")
        print(f"{'kernel@grid':48s} {'n':>4s} {'FETCH KiB':>12s} {'WRITE KiB':>12s}")
        tab = {}
        for key in sorted(per):
            f, w = per[key]["FETCH_SIZE"], per[key]["WRITE_SIZE"]
            fa = sum(f) / len(f) if f else float("nan")
            wa = sum(w) / len(w) if w else float("nan")
            tab[key] = {"n": max(len(f), len(w)), "fetch_kib": fa, "write_kib": wa}
            print(f"{key:48s} {max(len(f), len(w)):4d} {fa:12.0f} {wa:12.0f}")
        print("user-side sequence (dispatch, kernel, WRITE KiB):")
        for d, k, v in sorted(seq["WRITE_SIZE"])[-12:]:
            print(f"   {d:6d} {k:36s} {v:10.0f}")
        res[pol] = tab
    json.dump(res, open(os.path.join(out, "pmc_brief.json"), "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
