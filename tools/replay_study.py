"""Off-GPU study of recorded free races (AMG_REPLAY_DUMP dumps of
tests/async_band.replay_check): for one case, the oracle's replays of each
run -- the end order, the row-time model, and `samples` sequential orders
consistent with the recorded update windows (each correction placed at a
uniformly random time inside its [start, end] window) -- beside the device's
relres.

usage: python tools/replay_study.py DUMPDIR CASE [--samples 20]
"""
import argparse
import ctypes
import glob
import json
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_package  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dump")
    ap.add_argument("case")
    ap.add_argument("--samples", type=int, default=20)
    a = ap.parse_args()
    amg = load_package()
    from oracle import pyoracle as oracle
    from async_band import _per_rank, replay_tables, sliced_replay, timed_band, torn_replay
    z = np.load(os.path.join(a.dump, a.case + ".npz"))
    host = {}
    for key in ("A", "P", "R"):
        host[key] = []
        lev = 0
        while f"{key}{lev}_shape" in z:
            nr, nc = z[f"{key}{lev}_shape"]
            host[key].append(oracle.Csr(int(nr), int(nc), z[f"{key}{lev}_rowptr"], z[f"{key}{lev}_col"],
                                        z[f"{key}{lev}_val"]))
            lev += 1
    opts = amg.default_opts()
    raw = z["opts"].tobytes()
    ctypes.memmove(ctypes.addressof(opts), raw, min(len(raw), ctypes.sizeof(opts)))
    f = z["f"]
    blocks = {int(k[3:]): z[k] for k in z.files if k.startswith("blk")} or None
    L = len(host["A"])
    rng = np.random.default_rng(0)
    for fn in sorted(glob.glob(os.path.join(a.dump, a.case + "_run*.json"))):
        d = json.load(open(fn))
        comp = d["composed"]
        ends, starts, rs = d["ends"], d["starts"], d["rs"]
        E = _per_rank(ends)
        S = _per_rank(starts) if starts is not None else E
        if rs is not None and len(rs) > 2:
            base = sliced_replay(amg, oracle, host, f, opts, E, rs, composed=comp, blocks=blocks)
        else:
            base = timed_band(amg, oracle, host, f, opts, replay_tables([np.asarray(x) for x in E[0]], L),
                              blocks=blocks, composed=comp)[0]
        tm = torn_replay(amg, oracle, host, f, opts, E, S, rs=rs, composed=comp, blocks=blocks)
        samp = []
        for _ in range(a.samples):
            T = []
            for e_r, s_r in zip(E, S):
                tr = []
                for k in range(L):
                    e = np.asarray(e_r[k], dtype=np.float64)
                    s = np.asarray(s_r[k], dtype=np.float64) if k < len(s_r) and len(s_r[k]) >= len(e) else e
                    s = s[:len(e)]
                    tr.append(s + (e - s) * rng.random(len(e)))
                T.append(tr)
            if rs is not None and len(rs) > 2:
                samp.append(sliced_replay(amg, oracle, host, f, opts, T, rs, composed=comp, blocks=blocks))
            else:
                samp.append(timed_band(amg, oracle, host, f, opts, replay_tables(T[0], L), blocks=blocks,
                                       composed=comp)[0])
        rel = d["rel"]
        print(f"{a.case} run {d['run']}: device {rel:.4e} | end order {base:.4e} ({rel / base:.2f}x) | row-time "
              f"{tm:.4e} | window orders [{min(samp):.4e}, {max(samp):.4e}] -> device/[lo,hi] "
              f"{rel / min(samp):.2f}-{rel / max(samp):.2f}")


if __name__ == "__main__":
    main()


def random_rowtime(amg, oracle, host, f, opts, E, S, rs, rng, block=256, composed=False, blocks=None):
    """the row-time model with the rows of each update pass reached in a random
    order of `block`-row pieces (a kernel's workgroups do not run in row order)"""
    from async_band import _replay_slices
    L = len(host["A"])
    n0 = host["A"][0].nrows
    rs = list(rs) if rs is not None else [0, n0]
    cuts, tabs = [0], []
    for r in range(len(E)):
        a, b = rs[r], rs[r + 1]
        nb = max(1, (b - a + block - 1) // block)
        for k_ in range(nb):
            lo_, hi_ = a + k_ * block, min(b, a + (k_ + 1) * block)
            tab = []
            for k in range(L):
                e = np.asarray(E[r][k], dtype=np.float64)
                s = np.asarray(S[r][k], dtype=np.float64) if k < len(S[r]) and len(S[r][k]) >= len(e) else e
                s = s[:len(e)]
                tab.append(s + (e - s) * rng.random(len(e)))
            tabs.append(tab)
            cuts.append(hi_)
    return _replay_slices(amg, oracle, host, f, opts, cuts, tabs, composed=composed, blocks=blocks)
