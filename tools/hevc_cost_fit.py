"""Fit and check the HEVC slice planner's CU cost model (hevc_core.h cu_cost) against measured bin
tokens, and simulate the P-picture slice layout it produces.

    # on the GPU box: per-unit tables of a few P pictures
    python tools/hevc_session_timing.py --width 3840 --height 2160 --bitrate-kbps 18000 \\
        --frames 14 --report 3 --dump gpurun_out/cufit/desk
    # anywhere:
    python tools/hevc_cost_fit.py gpurun_out/cufit/desk_11.npy gpurun_out/cufit/desk_13.npy

Each table row is one 16x16 unit in raster order: (type, cbf, sum of last+1, coded sub-blocks,
est_bytes, measured tokens).  Prints the least-squares fit of coded units (with an AMVP / intra
term), the mean tokens of units without residual per type, and for each picture the slowest slice
(in tokens) the layout rule floor(prefix * S / T) gives with the current model, compared with the
best contiguous partition into the same number of slices by the measured tokens.
"""
import argparse

import numpy as np


def model_current(typ, cbf, lsum, sb, eb):
    """cu_cost of csrc/codec/hevc_core.h (round 5 fit; the unit type is not known at layout time)."""
    v = np.floor((2 * lsum + 104 * sb + 31 * eb) / 8)
    return np.where(cbf == 0, 1.0, np.where(v > 5, v - 4, 1))


def model_round4(typ, cbf, lsum, sb, eb):
    return np.where(cbf == 0, 4.0, 1 + np.floor(lsum / 4) + 15 * sb + np.floor(21 * eb / 8))


def slices(t, model, units_w, max_slices=200, cost_per_slice=2048):
    typ, cbf, lsum, sb, eb, tok = t.T
    n = len(t)
    x, y = np.arange(n) % units_w, np.arange(n) // units_w
    ctb = (y // 2) * ((units_w + 1) // 2) + (x // 2)
    nct = int(ctb.max()) + 1
    ce = np.bincount(ctb, model(typ, cbf, lsum, sb, eb), nct)
    ct = np.bincount(ctb, tok, nct)
    total = ce.sum()
    s = int(min(max_slices, max(1, total // cost_per_slice)))
    pre = np.concatenate([[0], np.cumsum(ce)[:-1]])
    sid = np.minimum(np.floor(pre * s / total), s - 1).astype(int)
    rank = np.cumsum(np.concatenate([[True], sid[1:] != sid[:-1]])) - 1
    per = np.bincount(rank, ct)
    return per, ct


def best_partition(ct, k):
    def fits(cap):
        cnt, acc = 1, 0.0
        for v in ct:
            if v > cap:
                return False
            if acc + v > cap:
                cnt, acc = cnt + 1, v
            else:
                acc += v
        return cnt <= k
    lo, hi = float(ct.max()), float(ct.sum())
    while hi - lo > 1:
        mid = (lo + hi) / 2
        lo, hi = (lo, mid) if fits(mid) else (mid, hi)
    return hi


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tables", nargs="+")
    ap.add_argument("--units-w", type=int, default=240, help="16x16 units per row (3840 / 16)")
    a = ap.parse_args()
    ts = [np.load(p).astype(np.float64) for p in a.tables]
    allt = np.concatenate(ts)
    typ, cbf, lsum, sb, eb, tok = allt.T
    m = cbf > 0
    X = np.stack([np.ones(m.sum()), lsum[m], sb[m], eb[m], (typ[m] >= 2).astype(float)], 1)
    coef, *_ = np.linalg.lstsq(X, tok[m], rcond=None)
    print("coded units: tokens ~ %.2f + %.3f (last+1) + %.2f sub-blocks + %.2f bytes + %.2f [AMVP/intra,"
          " final type: not known to the planner]" % tuple(coef))
    for ty in range(4):
        u = (cbf == 0) & (typ == ty)
        if u.any():
            print("no residual, type %d: %d units, %.2f tokens" % (ty, u.sum(), tok[u].mean()))
    for p, t in zip(a.tables, ts):
        cur, ct = slices(t, model_current, a.units_w)
        old, _ = slices(t, model_round4, a.units_w)
        print("%s: %d slices, slowest %d tokens (round-4 model %d), median %d, best partition %d" % (
            p, len(cur), cur.max(), old.max(), np.median(cur), best_partition(ct, len(cur))))


if __name__ == "__main__":
    main()
