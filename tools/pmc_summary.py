"""Summarize a tools/profile.sh run into profiles/ (committed evidence).

    python tools/pmc_summary.py gpurun_out/prof rNN [--no-json]

PROF_DEST=dir: write there instead of profiles/ (on the GPU box: under gpurun_out/, so the
summaries come back while the raw traces, over gpurun's 64 MiB return limit, are deleted).
--no-json: the two CSVs only (a profile of another workload than the bench default's, e.g.
config 5's share, leaves the bench's pmc_traffic.json alone).

Writes
  profiles/<tag>_kernel_stats.csv  rocprofv3 --kernel-trace --stats summary (copied)
  profiles/<tag>_pmc.csv           per kernel template instance: dispatches, average duration,
                                   FETCH_SIZE / WRITE_SIZE / SQ counters per dispatch, HBM bytes
  profiles/pmc_traffic.json        per bench stage (bench.py's kernel names): HBM bytes, VALU
                                   wave-instructions and SQ counters per launch, stamped with the
                                   kernel sources' hash (bench.src_stamp()) and the workload size;
                                   bench.py uses an entry only when both match.
HBM bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: rocprofv3 reports KB, and on gfx950
FETCH_SIZE counts half the bytes of wide coalesced reads (MI355X_MICROARCH.md §HBM); other
access widths are uncalibrated there, so the figure is an estimate for gather-heavy kernels.
The radix passes are stages per template instance (radix_downsweep<8> ...), as the library's
profile names are; a stage with several instances gets the launch-weighted average per launch.
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STAGE_OF = {"count_tile_kernel": "count", "count_tile32_kernel": "count32",
            "tile_union_kernel": "tile_union", "edge_union_kernel": "edge_union",
            "slab_root_labels_list_kernel": "slab_root_labels",
            "tcell_kernel": "tslot", "thalo_kernel": "tstage"}


def symbol(name):
    """'void dbscan::(anonymous namespace)::foo_kernel<1536, 6>(args)' -> 'foo_kernel<1536, 6>'"""
    n = name.replace("(anonymous namespace)::", "")
    if n.startswith("void "):
        n = n[5:]
    depth, cut = 0, len(n)
    for i, c in enumerate(n):  # the argument list starts at the first '(' outside <...>
        if c == "<":
            depth += 1
        elif c == ">":
            depth -= 1
        elif c == "(" and depth == 0:
            cut = i
            break
    n = n[:cut].strip()
    head = n.split("<")[0]
    return head.split("::")[-1] + n[len(head):]


def stage_of(sym):
    base = sym.split("<")[0]
    if base in STAGE_OF:
        return STAGE_OF[base]
    if base == "bucket_msd_kernel":  # the MSD pass
        return "bucket_msd"
    if base == "bucket_lsd_kernel":  # the segmented passes, per digit width
        return f"bucket_lsd<{sym[len(base) + 1:-1].strip()}>"
    if base == "count_wave_kernel":  # instances by lanes per tile: the library's profile names
        seg = int(sym[len(base) + 1:-1].split(",")[1])
        return {64: "count_wave", 32: "count_tiny", 16: "count_tiny16"}[seg]
    if not base.endswith("_kernel"):
        return None
    st = base[:-len("_kernel")]
    # the radix passes are profiled per template instance (bench.py's names carry the width)
    return st + sym[len(base):] if st.startswith("radix_") else st


def main():
    src, tag = sys.argv[1], sys.argv[2]
    prof = os.environ.get("PROF_DEST") or os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"),
                os.path.join(prof, f"{tag}_kernel_stats.csv"))
    stamp = open(os.path.join(src, "src_sha")).read().strip()
    line = [l for l in open(os.path.join(src, "trace.log")) if l.startswith("{")][-1]
    n_points = json.loads(line)["config"]["n_points"]
    # durations and dispatch counts per instance from the kernel trace
    dur, cnt = defaultdict(float), defaultdict(int)
    for r in csv.DictReader(open(glob.glob(os.path.join(src, "trace", "**", "run_kernel_trace.csv"),
                                           recursive=True)[0])):
        s = symbol(r["Kernel_Name"])
        dur[s] += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
        cnt[s] += 1
    # counters: mean per dispatch, per instance
    ctr = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(src, "pmc*", "**", "run_counter_collection.csv"),
                              recursive=True)):
        for r in csv.DictReader(open(f)):
            ctr[symbol(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    names = sorted(set(ctr) | set(cnt), key=lambda s: -dur.get(s, 0.0))
    cols = sorted({c for s in ctr for c in ctr[s]})
    rows = []
    for s in names:
        avg = {c: (sum(v) / len(v)) for c, v in ctr[s].items()}
        hbm = (2 * avg.get("FETCH_SIZE", 0.0) + avg.get("WRITE_SIZE", 0.0)) * 1024
        rows.append((s, cnt.get(s, 0), dur[s] / cnt[s] if cnt.get(s) else None, hbm, avg))
    with open(os.path.join(prof, f"{tag}_pmc.csv"), "w") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "dispatches_in_trace", "avg_ns", "hbm_bytes_per_launch_est"] + cols)
        for s, c, a, hbm, avg in rows:
            w.writerow([s, c, f"{a:.0f}" if a else "", f"{hbm:.0f}"] +
                       [f"{avg[k]:.1f}" if k in avg else "" for k in cols])
    stages = defaultdict(lambda: {"instances": {}})
    for s, c, a, hbm, avg in rows:
        st = stage_of(s)
        if not st or not c:
            continue
        stages[st]["instances"][s] = {"launches_in_trace": c, "avg_ns": a,
                                      "hbm_bytes_per_launch": round(hbm), "counters": avg}
    out = {}
    for st, d in stages.items():
        inst = d["instances"]
        tot = sum(v["launches_in_trace"] for v in inst.values())
        wavg = lambda key: sum(v[key] * v["launches_in_trace"] for v in inst.values()) / tot
        cavg = lambda c: sum(v["counters"].get(c, 0.0) * v["launches_in_trace"]
                             for v in inst.values()) / tot
        valu = {c[len("SQ_INSTS_VALU_"):]: round(cavg(c), 1) for c in cols
                if c.startswith("SQ_INSTS_VALU_") and c.split("_")[-1] in ("F32", "F64")}
        sq = {c: round(cavg(c), 1) for c in cols if c.startswith("SQ_")}
        out[st] = {"hbm_bytes_per_launch": round(wavg("hbm_bytes_per_launch")),
                   "avg_ns": round(wavg("avg_ns"), 1), "valu_insts_per_launch": valu, "sq": sq,
                   "instances": {k: {kk: vv for kk, vv in v.items() if kk != "counters"}
                                 for k, v in inst.items()}}
    if "--no-json" in sys.argv[3:]:
        out = None
    if out is not None:
        with open(os.path.join(prof, "pmc_traffic.json"), "w") as f:
            json.dump({"src_sha": stamp, "n_points": n_points,
                       "source": f"profiles/{tag}_pmc.csv", "stages": out}, f, indent=1,
                      sort_keys=True)
    for s, c, a, hbm, avg in rows[:25]:
        print(f"{s:40s} n={c:4d} avg_ns={a or 0:10.0f} hbm={hbm:14.0f}")


if __name__ == "__main__":
    main()
