"""Summarise a tools/profile_box.sh run into profiles/<round>/<tag>_*.

    python tools/summarize_profile.py r01

Inputs : gpurun_out/prof_<tag>/{trace,fetch,write}/run_*.csv (rocprofv3)
Outputs: profiles/<round>/<tag>_kernel_stats.csv   (rocprofv3 --stats summary, verbatim)
         profiles/<round>/<tag>_summary.json/.md   (per-kernel avg time, PMC bytes)
         profiles/spmm_traffic.json        (read by bench.py: roofline.traffic)
         profiles/step_traffic.json        (read by bench.py: roofline.step_*; the
                                            PMC bytes of one whole training step)

HBM bytes per the MI355X guide (MI355X_MICROARCH.md §HBM, cdna_hip_programming
§7): FETCH_SIZE and WRITE_SIZE in KiB from separate passes; on gfx950
FETCH_SIZE reports 1/2 of the bytes of a wide coalesced stream, so
hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024. The 2x read correction is
calibrated for 16-B-per-lane streams (checked here on adam_kernel, whose
bytes are known); for the SpMM's 256-B row gathers it is applied as the
guide prescribes and the raw counters are kept beside it. Infinity-Cache
(MALL) hits are counted by FETCH_SIZE, so the figure bounds HBM traffic
from above.
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def round_dir(tag: str) -> str:
    """profiles/ keeps each round's records in its own directory (r5x: round5)."""
    import re
    if re.match(r"r6[a-z]", tag):
        return "round6"
    if re.match(r"r5[a-z]", tag):
        return "round5"
    if re.match(r"r4[a-z]", tag):
        return "round4"
    if re.match(r"r3([a-z]|$)", tag):
        return "round3"
    return "round1-2"


def commit_id(src=None):
    """BBGR_COMMIT, else this checkout's HEAD (the profile's tree is the one
    gpurun sent; summarise right after the run), '+dirty' if files differ."""
    c = os.environ.get("BBGR_COMMIT")
    if c:
        return c
    if src and os.path.exists(os.path.join(src, "commit.txt")):   # written by profile_box.sh
        c = open(os.path.join(src, "commit.txt")).read().strip()
        if c and c != "unknown":
            return c
    import subprocess
    try:
        head = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short=12", "HEAD"],
                              capture_output=True, text=True, check=True).stdout.strip()
        dirty = subprocess.run(["git", "-C", ROOT, "status", "--porcelain", "--untracked-files=no"],
                               capture_output=True, text=True, check=True).stdout.strip()
        return head + ("+dirty" if dirty else "")
    except (OSError, subprocess.CalledProcessError):
        return None


def _bench_line(src: str) -> dict:
    lines = open(os.path.join(src, "trace_bench.json")).read().strip().splitlines()
    return json.loads(lines[-1])


def bench_steps(src: str) -> int:
    """The timed steps of the trace pass's bench run (its own JSON line)."""
    return int(_bench_line(src)["steps"])


def bench_ms_per_step(src: str) -> float:
    return float(_bench_line(src)["ms_per_step"])


def main(tag: str):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    top = os.path.join(ROOT, "profiles")
    dst = os.path.join(top, round_dir(tag))
    os.makedirs(dst, exist_ok=True)
    commit = commit_id(src)   # before this run rewrites the tracked traffic files
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"),
                os.path.join(dst, f"{tag}_kernel_stats.csv"))
    stats = {r["Name"]: r for r in csv.DictReader(
        open(os.path.join(src, "trace", "run_kernel_stats.csv")))}

    def marked(rows, grid_of):
        """(begin, end) dispatch ids of bench.py's two profile_marker_kernel
        launches (grids of 1 and 2 workgroups of 64) around the timed steps."""
        ids = {}
        for r in rows:
            if "profile_marker_kernel" in r["Kernel_Name"]:
                ids[grid_of(r)] = int(r["Dispatch_Id"])
        return (ids[64], ids[128]) if 64 in ids and 128 in ids else None

    def pmc(kind):
        rows = list(csv.DictReader(open(os.path.join(src, kind, "run_counter_collection.csv"))))
        win = marked(rows, lambda r: int(r["Grid_Size"]))
        d, dw = collections.defaultdict(list), collections.defaultdict(list)
        for r in rows:
            key = (r["Kernel_Name"], int(r["Grid_Size"]))
            d[key].append(float(r["Counter_Value"]))
            if win and win[0] < int(r["Dispatch_Id"]) < win[1]:
                dw[key].append(float(r["Counter_Value"]))
        return d, dw, win

    (fetch, fetch_w, fwin), (write, write_w, wwin) = pmc("fetch"), pmc("write")
    # per-dispatch durations by (kernel, grid) from the trace pass; those
    # between the markers (the timed steps) kept apart
    trows = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv"))))
    tgrid = lambda r: int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])  # noqa: E731
    twin = marked(trows, tgrid)
    dur, dur_w = collections.defaultdict(list), collections.defaultdict(list)
    for r in trows:
        key = (r["Kernel_Name"], tgrid(r))
        t = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        dur[key].append(t)
        if twin and twin[0] < int(r["Dispatch_Id"]) < twin[1]:
            dur_w[key].append(t)
    kernels = {}
    for key in sorted(set(fetch) | set(dur)):
        name, grid = key
        f, w, t = fetch.get(key, []), write.get(key, []), dur.get(key, [])
        e = {"kernel": name, "grid": grid, "dispatches": len(t),
             "avg_us": (sum(t) / len(t) / 1e3) if t else None}
        if f and w:
            fk, wk = sum(f) / len(f), sum(w) / len(w)
            e.update(FETCH_SIZE_KiB=fk, WRITE_SIZE_KiB=wk,
                     hbm_bytes_corrected=(2 * fk + wk) * 1024,
                     hbm_bytes_raw=(fk + wk) * 1024)
            if e["avg_us"]:
                e["hbm_GBps_corrected"] = e["hbm_bytes_corrected"] / (e["avg_us"] * 1e3)
        kernels[f"{name}@{grid}"] = e
    summary = {"tag": tag, "stats": {k: {"calls": int(v["Calls"]),
                                         "avg_us": float(v["AverageNs"]) / 1e3,
                                         "pct": float(v["Percentage"])}
                                     for k, v in stats.items()},
               "kernels": kernels}
    json.dump(summary, open(os.path.join(dst, f"{tag}_summary.json"), "w"), indent=1)
    # bench.py's roofline kernel: the full-CSR item<-user product, symbol
    # spmm_kernel (one row per 16-lane group; the user-row products are
    # spmm_pair_kernel, the frontier ones spmm_masked_*, the fused-Adam one
    # spmm_adam_*). Its per-launch PMC bytes feed roofline.traffic; the commit
    # the profile was taken at travels with it (BBGR_COMMIT, set by the caller:
    # the GPU box has no .git).
    dom = [e for e in kernels.values()
           if e["kernel"] == "spmm_kernel" and "hbm_bytes_corrected" in e]
    # only a profile of the C4 bench feeds bench.py's roofline.traffic
    if dom and os.environ.get("BBGR_TRAFFIC_JSON", "1") != "0":
        n = sum(e["dispatches"] for e in dom)
        avg = sum(e["hbm_bytes_corrected"] * e["dispatches"] for e in dom) / n
        avg_us = sum(e["avg_us"] * e["dispatches"] for e in dom) / n
        json.dump({"tag": tag, "commit": commit,
                   "kernel": "spmm_kernel (full-CSR item<-user product)",
                   "hbm_bytes_per_launch_corrected": avg,
                   "fetch_KiB_per_launch": sum(e["FETCH_SIZE_KiB"] * e["dispatches"]
                                               for e in dom) / n,
                   "write_KiB_per_launch": sum(e["WRITE_SIZE_KiB"] * e["dispatches"]
                                               for e in dom) / n,
                   "avg_us": avg_us, "dispatches": n,
                   "per_grid": {f'{e["kernel"]}@{e["grid"]}': e["hbm_bytes_corrected"]
                                for e in dom},
                   "source": f"profiles/{round_dir(tag)}/{tag}_summary.json"},
                  open(os.path.join(top, "spmm_traffic.json"), "w"), indent=1)
    # the whole step: the dispatches between bench.py's two marker kernels
    # (the timed steps; BBGR_PROFILE_MARKS=1 in profile_box.sh) in each pass,
    # counted per kernel: per_step = count / steps must be an integer for every
    # kernel (a row-list launch's grid follows its list, so grids vary from
    # step to step: they are listed per kernel, not counted apart); bytes and
    # time are the window's own dispatches summed / steps.
    if twin and fwin and wwin and os.environ.get("BBGR_TRAFFIC_JSON", "1") != "0":
        steps = int(os.environ.get("BBGR_PROFILE_STEPS") or bench_steps(src))
        by_name = collections.defaultdict(list)
        for key in dur_w:
            by_name[key[0]].append(key)
        step_k, irregular = {}, {}
        for name, keys in sorted(by_name.items()):
            n = sum(len(dur_w[k]) for k in keys)
            nf = sum(len(fetch_w.get(k, [])) for k in keys)
            nw = sum(len(write_w.get(k, [])) for k in keys)
            e = {"per_step": n / steps,
                 "us_per_step": sum(sum(dur_w[k]) for k in keys) / steps / 1e3,
                 "grids": sorted(k[1] for k in keys for _ in dur_w[k]),
                 "dispatches_in_window": {"trace": n, "fetch": nf, "write": nw}}
            if nf == n and nw == n:
                e["hbm_bytes_per_step_corrected"] = sum(
                    2 * sum(fetch_w[k]) + sum(write_w[k]) for k in keys) * 1024 / steps
            if len(e["grids"]) > 8:
                e["grids"] = sorted(set(e["grids"]))
            (step_k if n % steps == 0 and nf == n and nw == n else irregular)[name] = e
        tot_b = sum(e["hbm_bytes_per_step_corrected"] for e in step_k.values())
        tot_us = sum(e["us_per_step"] for e in step_k.values())
        step_ms = bench_ms_per_step(src)
        json.dump({"tag": tag, "commit": commit, "steps": steps,
                   "selection": "kernels dispatched between the bench's two profile markers "
                                "(the timed steps); per_step an exact integer per kernel",
                   "hbm_bytes_per_step_corrected": tot_b,
                   "kernel_us_per_step_pmc": tot_us,
                   "trace_ms_per_step": step_ms,
                   "kernels": {k: {**e, "per_step": int(e["per_step"])}
                               for k, e in step_k.items()},
                   "irregular": irregular or None,
                   "note": "2*FETCH_SIZE+WRITE_SIZE (gfx950 read correction) summed over the "
                           "kernels of one timed step; FETCH_SIZE counts Infinity-Cache hits, "
                           "so this bounds the step's HBM bytes from above; kernel_us_per_step "
                           "<= trace_ms_per_step (the trace pass's own bench line)",
                   "source": f"profiles/{round_dir(tag)}/{tag}_summary.json"},
                  open(os.path.join(top, "step_traffic.json"), "w"), indent=1)
    with open(os.path.join(dst, f"{tag}_summary.md"), "w") as fh:
        fh.write(f"# rocprofv3 summary {tag}\n\n| kernel | calls | avg us | % |\n|---|---|---|---|\n")
        for k, v in sorted(summary["stats"].items(), key=lambda kv: -kv[1]["pct"])[:15]:
            fh.write(f"| {k} | {v['calls']} | {v['avg_us']:.1f} | {v['pct']:.2f} |\n")
        fh.write("\n| kernel@grid | dispatches | avg us | FETCH KiB | WRITE KiB | HBM GB (2F+W) | GB/s |\n"
                 "|---|---|---|---|---|---|---|\n")
        for k, e in kernels.items():
            if "hbm_bytes_corrected" in e:
                fh.write(f"| {k} | {e['dispatches']} | {e['avg_us'] or 0:.1f} | "
                         f"{e['FETCH_SIZE_KiB']:.0f} | {e['WRITE_SIZE_KiB']:.0f} | "
                         f"{e['hbm_bytes_corrected'] / 1e9:.3f} | "
                         f"{e.get('hbm_GBps_corrected', 0):.0f} |\n")
    print(open(os.path.join(dst, f"{tag}_summary.md")).read())


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
