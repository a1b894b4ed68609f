"""Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE for the fit's gather patterns (tooling).

    python tools/pmc_calibrate.py build            # hipcc tools/calib.hip -> tools/libcalib.so
    rocprofv3 --pmc FETCH_SIZE -d DIR -o run -- python tools/pmc_calibrate.py run
    python tools/pmc_calibrate.py report DIR

Three kernels with known bytes, each over arrays far larger than the 256 MiB Infinity Cache:
stream16 (coalesced 16 B/lane: the guide's calibrated case, FETCH_SIZE = 1/2 of the bytes),
gather32 (a random 32-B record per lane inside bands of 40 000 records, as gather_bucket reads
the bucketed sort's records; its 4-B index stream coalesced) and gather4 (a random 4-B word
per lane over the whole array, as permute_out_bucket reads the labels; 4-B index stream and
4-B output stream coalesced).  report prints FETCH_SIZE per known byte for each."""
import ctypes
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libcalib.so")
N = 1 << 26  # 64 M lanes per kernel


def build():
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                    os.path.join(HERE, "calib.hip"), "-o", LIB], check=True)


def run():
    import numpy as np
    import torch

    L = ctypes.CDLL(LIB)
    L.calib_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                            ctypes.c_void_p]
    dev = "cuda"
    sink = torch.zeros(N, dtype=torch.float64, device=dev)
    a16 = torch.rand(N, 2, dtype=torch.float64, device=dev)
    band = 40_000
    g = torch.Generator(device="cpu").manual_seed(1)
    base = torch.arange(N, dtype=torch.int64) // band * band
    idx32 = (base + torch.randint(0, band, (N,), generator=g)).clamp(max=N - 1).to(torch.int32)
    rec = torch.rand(N, 4, dtype=torch.float64, device=dev)
    idx4 = torch.randperm(N, generator=g).to(torch.int32)
    w = torch.randint(0, 1 << 30, (N,), dtype=torch.int32, device=dev)
    out4 = torch.zeros(N, dtype=torch.int32, device=dev)
    i32, i4 = idx32.to(dev), idx4.to(dev)
    torch.cuda.synchronize()
    for _ in range(2):
        assert L.calib_run(0, a16.data_ptr(), None, N, sink.data_ptr()) == 0
        assert L.calib_run(1, rec.data_ptr(), i32.data_ptr(), N, sink.data_ptr()) == 0
        assert L.calib_run(2, w.data_ptr(), i4.data_ptr(), N, out4.data_ptr()) == 0
    print("ok", flush=True)


KNOWN = {"stream16": 16 * N, "gather32": (32 + 4) * N, "gather4": (4 + 4) * N}


def report(d):
    import csv
    import glob

    rows = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "")
            for name in KNOWN:
                if name in k and r.get("Counter_Name") in ("FETCH_SIZE", "WRITE_SIZE"):
                    rows.setdefault((name, r["Counter_Name"]), []).append(float(r["Counter_Value"]))
    for (name, ctr), v in sorted(rows.items()):
        kb = sum(v) / len(v)
        print(f"{name:9s} {ctr:10s} {kb * 1024 / 1e6:10.1f} MB per launch; known read bytes "
              f"{KNOWN[name] / 1e6:10.1f} MB; ratio {kb * 1024 / KNOWN[name]:.3f}")


if __name__ == "__main__":
    {"build": build, "run": run}.get(sys.argv[1], lambda: report(sys.argv[2]))()
