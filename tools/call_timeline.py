"""Where one seam call's time goes, from a rocprofv3 trace of tools/call_trace.py (HIP runtime API,
kernels, memory copies).  Calls are cut at the end of each synchronizing API call; for each
block of calls (separated by >= 10 ms idle) the medians over its calls of:
  host->first API   wall from the previous call's return to this call's first HIP API entry
  api               every HIP API call of one call (count, total time, the longest ones)
  launch->start     the first kernel's (or copy's) API entry to its start on the GPU
  gpu span          first GPU operation start to last GPU operation end, and the kernels' sum
  end->return       last GPU operation end to the synchronizing call's return
    python3 tools/call_timeline.py gpurun_out/ct"""
import csv
import glob
import os
import statistics as S
import sys
from collections import defaultdict

root = sys.argv[1]


def load(pat):
    fs = glob.glob(os.path.join(root, "**", pat), recursive=True)
    rows = []
    for f in fs:
        rows += list(csv.DictReader(open(f)))
    return rows


api = load("*hip_api_trace.csv")
ker = load("*kernel_trace.csv")
cpy = load("*memory_copy_trace.csv")
gpu = {}  # correlation id -> (start, end, name)
for r in ker:
    gpu[int(r["Correlation_Id"])] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                                     r["Kernel_Name"].split("(")[0].replace("void ", ""))
for r in cpy:
    gpu[int(r["Correlation_Id"])] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                                     r.get("Direction", "copy"))
# API calls of the thread that made the most calls (the probe's main thread)
by_tid = defaultdict(list)
for r in api:
    by_tid[r["Thread_Id"]].append(r)
calls = max(by_tid.values(), key=len)
calls = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"],
                 int(r["Correlation_Id"])) for r in calls))
SYNC = ("hipStreamSynchronize", "hipEventSynchronize", "hipDeviceSynchronize")
segs, cur = [], []
for c in calls:
    cur.append(c)
    if c[2] in SYNC:
        segs.append(cur)
        cur = []
# blocks: a new block when the gap before a segment exceeds 10 ms
blocks, blk, prev_end = [], [], None
for s in segs:
    if prev_end is not None and s[0][0] - prev_end > 10_000_000:
        blocks.append(blk)
        blk = []
    blk.append((s, prev_end))
    prev_end = s[-1][1]
blocks.append(blk)
for bi, blk in enumerate(blocks):
    if len(blk) < 20:
        continue
    rows = defaultdict(list)
    names = defaultdict(list)
    for s, pe in blk[6:]:  # past the warm calls
        ops = [gpu[c[3]] for c in s if c[3] in gpu]
        if not ops:
            continue
        first_api = s[0][0]
        if pe is not None:
            rows["host gap before call"].append(first_api - pe)
        rows["api calls"].append(len(s))
        rows["api time total"].append(sum(c[1] - c[0] for c in s))
        launch = [c for c in s if c[3] in gpu][0]
        rows["first API entry -> first launch API entry"].append(launch[0] - first_api)
        g0 = min(o[0] for o in ops)
        g1 = max(o[1] for o in ops)
        rows["launch API entry -> GPU start"].append(g0 - launch[0])
        rows["gpu span"].append(g1 - g0)
        rows["gpu busy (sum)"].append(sum(o[1] - o[0] for o in ops))
        rows["GPU end -> sync return"].append(s[-1][1] - g1)
        rows["first API entry -> sync return"].append(s[-1][1] - first_api)
        for o in ops:
            names[o[2]].append(o[1] - o[0])
        for c in s:
            names["API " + c[2]].append(c[1] - c[0])
    print(f"block {bi}: {len(blk)} calls")
    for k, v in rows.items():
        print(f"  {k:42s} {S.median(v) / 1e3:8.1f} us")
    for k, v in sorted(names.items(), key=lambda kv: -sum(kv[1])):
        print(f"    {k[:70]:70s} n={len(v):4d} median {S.median(v) / 1e3:7.1f} us")
