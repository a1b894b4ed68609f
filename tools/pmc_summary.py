"""Summarize a tools/profile.sh run into profiles/ (committed evidence).

    python tools/pmc_summary.py gpurun_out/prof r01

Writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied)
  profiles/<tag>_pmc.csv            per-kernel average FETCH_SIZE / WRITE_SIZE per dispatch
  profiles/pmc_traffic.json         HBM bytes per launch for the bench's stages, read by bench.py
HBM bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: rocprofv3 reports KB, and on gfx950
FETCH_SIZE counts half the bytes of wide coalesced reads (MI355X_MICROARCH.md §HBM); other
access widths are uncalibrated there, so the figure is an estimate for gather-heavy kernels.
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
def stage_of(kernel):
    """bench.py's per-kernel name (the klaunch names in csrc/fit.hip): the kernel's base name
    without `_kernel`; count_tile_kernel is "count"."""
    if kernel == "count_tile_kernel":
        return "count"
    if kernel == "count_tile32_kernel":
        return "count32"
    return kernel[:-len("_kernel")] if kernel.endswith("_kernel") else None




def base(name):
    n = name.replace("(anonymous namespace)::", "")
    if n.startswith("void "):
        n = n[5:]
    n = n.split("(")[0]
    n = n.split("::")[-1]
    return n.split("<")[0].strip()


def per_kernel(path, counter):
    acc = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] == counter:
                acc[base(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    src, tag = sys.argv[1], sys.argv[2]
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"),
                os.path.join(prof, f"{tag}_kernel_stats.csv"))
    fetch = per_kernel(os.path.join(src, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(src, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    stats = {}
    with open(os.path.join(src, "trace", "run_kernel_stats.csv")) as f:
        for r in csv.DictReader(f):
            stats[base(r["Name"])] = float(r["AverageNs"])
    rows, traffic = [], {}
    for k in sorted(set(fetch) | set(write)):
        fb = fetch.get(k, 0.0) * 2 * 1024
        wb = write.get(k, 0.0) * 1024
        rows.append((k, fetch.get(k, 0.0), write.get(k, 0.0), fb + wb, stats.get(k)))
        st = stage_of(k)
        if st:
            traffic[st] = {"kernel": k, "bytes_per_launch": round(fb + wb),
                           "fetch_kb": fetch.get(k), "write_kb": write.get(k),
                           "avg_ns": stats.get(k), "source": f"profiles/{tag}_pmc.csv"}
    with open(os.path.join(prof, f"{tag}_pmc.csv"), "w") as f:
        f.write("kernel,fetch_size_kb_avg,write_size_kb_avg,hbm_bytes_per_launch_est,avg_ns\n")
        for r in rows:
            f.write(f"{r[0]},{r[1]:.1f},{r[2]:.1f},{r[3]:.0f},{r[4] if r[4] else ''}\n")
    with open(os.path.join(prof, "pmc_traffic.json"), "w") as f:
        json.dump(traffic, f, indent=1, sort_keys=True)
    for r in rows:
        print(f"{r[0]:28s} fetchKB={r[1]:12.1f} writeKB={r[2]:12.1f} est_bytes={r[3]:14.0f}")


if __name__ == "__main__":
    main()
