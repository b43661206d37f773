"""The replay of a DMEM_AsyncSmooth run (test infrastructure).

amg_dist_async_jacobi (DMEM_Smooth.cpp:16-313: Jacobi in residual-update form,
ghost deltas exchanged asynchronously) logs, per rank, the order in which its
work entered the compute stream (amg_dist_async_jacobi_log): every relaxation
update (with its acceleration coefficients), every interior product
r -= A_own e_k, and every ghost delta applied, r -= A_offd e_p[j] (peer p's
relaxation j).  Which of the peer's relaxations a rank's residual has seen when
it relaxes is the whole nondeterminism of the asynchronous smoother; given the
logs it is fixed, and this module recomputes the run on the host: every rank's
update u = r ./ s (s = a_ii / w, 1 where a_ii = 0; or the L1 row norm), the
acceleration branch of ajac_update_k (DMEM_ChebyUpdate's async form,
DMEM_Misc.cpp:650-663), x += e, and the residual updates in the logged order,
with a peer's delta j taken from that peer's own replayed relaxation j.  A
device run must match its replay to rounding (the device sums each row in its
local CSR order, the host in the global one)."""
import numpy as np
import scipy.sparse as sp


def host_csr(nrows, ncols, rowptr, col, val):
    return sp.csr_matrix((np.asarray(val, dtype=np.float64), np.asarray(col), np.asarray(rowptr)),
                         shape=(nrows, ncols))


def ajac_replay(A, f, rs, logs, omega, l1=None):
    """A: global scipy CSR; f: global right-hand side; rs: row starts of the
    ranks; logs: per rank the (events, 5) array of async_jacobi_log; l1: global
    L1 row norms (ASYNC_L1_JACOBI) or None.  Returns (x, r): the replayed
    iterate and incrementally kept residual, global"""
    A = sp.csr_matrix(A)
    R = len(rs) - 1
    diag = A.diagonal()
    sc = np.asarray(l1, dtype=np.float64) if l1 is not None else np.where(diag == 0.0, 1.0, diag / omega)
    blk = {}
    for q in range(R):
        for p in range(R):
            B = A[rs[q]:rs[q + 1], rs[p]:rs[p + 1]]
            if p == q or B.nnz:
                blk[q, p] = B.tocsr()
    r = [np.array(f[rs[q]:rs[q + 1]], dtype=np.float64) for q in range(R)]
    x = [np.zeros(rs[q + 1] - rs[q]) for q in range(R)]
    d = [np.zeros(rs[q + 1] - rs[q]) for q in range(R)]
    hist = [dict() for _ in range(R)]
    last = [-1] * R
    ptr = [0] * R
    while any(ptr[q] < len(logs[q]) for q in range(R)):
        moved = False
        for q in range(R):
            s_q = sc[rs[q]:rs[q + 1]]
            while ptr[q] < len(logs[q]):
                t, a, b, c, dd = (float(v) for v in logs[q][ptr[q]])
                t = int(t)
                if t == 1:  # ajac_update_k
                    k, am = int(a), int(b)
                    u = 0.0 + r[q] / s_q
                    if am == 1:
                        d[q] = u.copy()
                    elif am == 2:
                        dp = d[q]
                        d[q] = c * dp + dd * u
                        u = c * dp + dd * u
                    elif am == 3:
                        u = dd * u
                    e = 0.0 + 1.0 * u
                    x[q] = x[q] + 1.0 * e
                    hist[q][k] = e
                    last[q] = k
                elif t == 2:  # interior product r -= A_own e_k
                    r[q] = r[q] - blk[q, q] @ hist[q][int(a)]
                elif t == 3:  # peer p's delta j
                    p, j = int(a), int(b)
                    if last[p] < j:
                        break  # the peer has not relaxed that far yet in the replay
                    if (q, p) in blk:  # (a peer with no coupling contributes nothing)
                        r[q] = r[q] - blk[q, p] @ hist[p][j]
                elif t == 4:  # every peer's delta of sweep k
                    k = int(a)
                    peers = [p for p in range(R) if p != q and (q, p) in blk]
                    if any(last[p] < k for p in peers):
                        break
                    g = sum(blk[q, p] @ hist[p][k] for p in peers)
                    r[q] = r[q] - g
                else:
                    raise ValueError(f"rank {q}: event type {t}")
                ptr[q] += 1
                moved = True
        if not moved:
            raise RuntimeError(f"replay stuck at events {ptr} of {[len(v) for v in logs]}")
    return np.concatenate(x), np.concatenate(r)


def check_replay(A, f, rs, logs, x_dev, rel_dev, omega, l1=None, rtol=1e-9, what=""):
    """the device run (assembled iterate x_dev, relres rel_dev) against the replay
    of its own logged schedule: iterate within rtol of its largest entry, relres
    within rtol"""
    xr, rr = ajac_replay(A, f, rs, logs, omega, l1=l1)
    rel_rep = np.linalg.norm(f - A @ xr) / np.linalg.norm(f)
    err = float(np.max(np.abs(x_dev - xr)) / max(np.max(np.abs(xr)), 1e-300))
    late = sum(int(np.count_nonzero(L[:, 0] == 3)) for L in logs)
    print(f"  {what}: device relres {rel_dev:.10e}, replay {rel_rep:.10e} ({late} ghost deltas, "
          f"max |x - x_replay| / max |x| = {err:.2e})")
    assert err <= rtol, (what, err)
    assert abs(rel_dev - rel_rep) <= rtol * rel_rep, (what, rel_dev, rel_rep)
    return rel_rep
