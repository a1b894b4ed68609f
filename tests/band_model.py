"""Host model of the band form's staging capacity (small.hip band_fit_kernel: band_make_grid
with its total-cell bound scaled by the launch's workgroups, the rows taken along the axis that
makes them shorter, the row-cost ranges and each workgroup's staged row span): whether a
partition overflows a workgroup's staging (kStError 3 -> the tiled recall).  Test
infrastructure: tests/test_gpu_band.py derives its exact expected recall counts from it, and
tools/band_overflow_sim.py runs it over the seam's G(10^7) partitions (where it reproduced the
GPU's 6 recalls of the rows-along-y form exactly)."""
import numpy as np

K_CAP, K_CELLS, K_MAXWG, K_C0 = 7168, 7168, 64, 2


def cells(vmax, vmin, h):
    return np.floor((vmax * 0.5 - vmin * 0.5) * (2.0 / h)) + 1.0


def band_overflows(x, y, eps, gscale=True):
    """True when some workgroup of the band fit would stage more than its capacity.  gscale:
    the grid's total-cell bound scaled by the launch's workgroups (G / kBandMaxWG)."""
    m = x.size
    G = min(K_MAXWG, max(16, (m + 255) // 256))
    fin = np.isfinite(x) & np.isfinite(y)
    xf, yf = x[fin], y[fin]
    nf = xf.size
    if nf == 0:
        return False, 0, 0
    xmin, xmax, ymin, ymax = xf.min(), xf.max(), yf.min(), yf.max()
    R = max(abs(eps) * (1.0 + 2.0 ** -40), 2.0 ** -500)
    h0 = R * (1.0 + 2.0 ** -16)
    hx = hy = h0
    kNx, kNy, kAll = K_CELLS // 3, K_CAP - 1, 24.0 * K_CELLS
    if gscale:
        kAll = 24.0 * K_CELLS * G / K_MAXWG
    for _ in range(4096):
        cx, cy = cells(xmax, xmin, hx), cells(ymax, ymin, hy)
        if cx <= kNx and cy <= kNy and cx * cy <= kAll:
            break
        if cx / kNx >= cy / kNy:
            hx *= 2.0
        else:
            hy *= 2.0
    nx, ny = int(cx), int(cy)
    invy = 2.0 / hy
    qy = np.floor(2.0 * ((yf * 0.5 - ymin * 0.5) * invy)).astype(np.int64)
    qy = np.clip(qy, 0, 2 * ny - 1)
    row = qy >> 1
    pts = np.bincount(row, minlength=ny).astype(np.int64)
    qtot = int((pts * (K_C0 * nx + pts)).sum())
    tw = qtot + nx * nx * ny
    rmax = max(1, K_CELLS // nx - 2)
    pmax = K_CAP // 2
    fpt = (3 * tw + G * pmax - 1) // (G * pmax)
    fr = (3 * tw + G * rmax - 1) // (G * rmax)
    bcell = max(nx, (fr + nx - 1) // nx)
    a = np.maximum(K_C0 * nx + pts, fpt)
    cost = pts * a + nx * bcell
    C = np.concatenate([[0], np.cumsum(cost)])
    par = np.concatenate([[0], np.cumsum(pts)])
    T = int(C[-1])
    worst = 0
    for g in range(G):
        lo = g * T // G
        hi = T if g + 1 == G else (g + 1) * T // G
        ra = int(np.searchsorted(C, lo, side="right") - 1)
        rb = int(np.searchsorted(C, hi, side="right") - 1)
        if lo >= hi:
            continue
        sa = ra - 1 if ra > 0 else 0
        sb = rb + 2 if rb + 2 < ny else ny
        S = int(par[sb] - par[sa])
        worst = max(worst, S)
        if S > K_CAP or (sb - sa) * nx > K_CELLS:
            return True, nx, ny
    return False, nx, ny


def band_recall(x, y, eps):
    """The shipped kernel: gscale grid, transposed when its rows would be longer than its
    columns (nx > ny)."""
    o, nx, ny = band_overflows(x, y, eps)
    if nx > ny:
        return band_overflows(y, x, eps)[0]
    return o
