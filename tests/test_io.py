"""Binary triplet matrix files (-problem file, csrc/amg_io.cpp) on the host:
the library's readers against a plain-Python restatement of the reference's
(ReadBinary_fread_HypreParCSR Misc.cpp:800-915, ParReadBinary_fread
DMEM_BuildMatrix.cpp:1488-1560) plus hypre's IJ assembly (first position,
last value, diagonal first -- third party, parity unpinned), write/read round
trips of PrintCSRMatrix (Misc.cpp:753-797) and TextToBin (TextToBin.cpp:5-39)."""
import numpy as np
import pytest


def ref_read(recs, symm, remove_disc):
    """Misc.cpp:800-915 record by record, then the IJ assembly."""
    num_rows = int(recs[0]["i"])
    col_count = [0] * num_rows
    flag = [0] * len(recs)
    for k in range(1, len(recs)):
        col_count[recs[k]["j"] - 1] += 1
        flag[k] = 1
    shift = [0] * num_rows
    if remove_disc:
        disc = [0] * num_rows
        for k in range(1, len(recs)):
            if flag[k] and col_count[recs[k]["i"] - 1] <= 1:
                flag[k] = 0
                disc[recs[k]["i"] - 1] = 1
                num_rows -= 1
        shift = list(np.cumsum(disc))
    rows = [[] for _ in range(num_rows)]
    for k in range(1, len(recs)):
        if not flag[k]:
            continue
        r = int(recs[k]["i"]) - shift[recs[k]["i"] - 1]
        c = int(recs[k]["j"]) - shift[recs[k]["j"] - 1]
        rows[r - 1].append((c - 1, float(recs[k]["val"])))
        if symm and r != c:
            rows[c - 1].append((r - 1, float(recs[k]["val"])))
    return assemble(rows, 0)


def assemble(rows, row0):
    rowptr, col, val = [0], [], []
    for r, ent in enumerate(rows):
        order, vals = [], {}
        for c, v in ent:
            if c not in vals:
                order.append(c)
            vals[c] = v
        if r + row0 in vals:
            order.remove(r + row0)
            order.insert(0, r + row0)
        col += order
        val += [vals[c] for c in order]
        rowptr.append(len(col))
    return np.array(rowptr, np.int32), np.array(col, np.int32), np.array(val, np.float64)


def records(n, entries):
    rec = np.zeros(len(entries) + 1, dtype=[("i", "<i4"), ("j", "<i4"), ("val", "<f8")])
    rec[0] = (n, n, 0.0)
    for k, (i, j, v) in enumerate(entries):
        rec[k + 1] = (i, j, v)
    return rec


def check_same(got, want):
    n, _, rowptr, col, val = got
    assert np.array_equal(rowptr, want[0])
    assert np.array_equal(col, want[1])
    assert np.array_equal(val.view(np.uint64), want[2].view(np.uint64))


def lower_triangle_entries(A):
    ent = []
    for i in range(A.nrows):
        for k in range(A.rowptr[i], A.rowptr[i + 1]):
            if A.col[k] <= i:
                ent.append((i + 1, int(A.col[k]) + 1, float(A.val[k])))
    return ent


def test_write_read_roundtrip(amg, oracle, tmp_path):
    A = oracle.laplace_7pt(6, 5, 4)
    p = tmp_path / "lap.bin"
    amg.io.write(p, A.nrows, A.ncols, A.rowptr, A.col, A.val, binary=1)
    recs = np.fromfile(p, dtype=amg.io.RECORD)
    assert recs.size == A.rowptr[-1] + 1 and recs[0]["i"] == A.nrows and recs[0]["j"] == A.ncols
    n, m, rowptr, col, val = amg.io.read(p, symm=0)
    assert (n, m) == (A.nrows, A.ncols)
    assert np.array_equal(rowptr, A.rowptr) and np.array_equal(col, A.col)
    assert np.array_equal(val.view(np.uint64), A.val.view(np.uint64))
    # the text form through TextToBin
    t = tmp_path / "lap.txt"
    amg.io.write(t, A.nrows, A.ncols, A.rowptr, A.col, A.val, binary=0)
    amg.io.text_to_bin(t, tmp_path / "lap2.bin")
    n2, _, rp2, c2, v2 = amg.io.read(tmp_path / "lap2.bin", symm=0)
    assert n2 == A.nrows and np.array_equal(rp2, A.rowptr) and np.array_equal(c2, A.col)
    assert np.array_equal(v2, A.val)  # %.16e round-trips fp64


def test_symmetric_file(amg, oracle, tmp_path):
    """SMEM's -problem file reads a lower triangle with symm_flag = 1 and gets
    the whole matrix back (rows diagonal-first, mirrored entries after the
    row's own in file order)."""
    A = oracle.laplace_7pt(5)
    rec = records(A.nrows, lower_triangle_entries(A))
    p = tmp_path / "lower.bin"
    rec.tofile(p)
    got = amg.io.read(p, symm=1)
    check_same(got, ref_read(rec, 1, 0))
    # same entries per row as the full matrix
    n, _, rowptr, col, val = got
    for i in range(n):
        a = dict(zip(A.col[A.rowptr[i]:A.rowptr[i + 1]], A.val[A.rowptr[i]:A.rowptr[i + 1]]))
        b = dict(zip(col[rowptr[i]:rowptr[i + 1]], val[rowptr[i]:rowptr[i + 1]]))
        assert a == b and col[rowptr[i]] == i


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_ragged_duplicates_disconnected(amg, tmp_path, seed):
    """Random files: shuffled records, repeated (row, col) pairs, zero values,
    rows without a diagonal, empty rows and disconnected points; both flags."""
    rng = np.random.default_rng(seed)
    n = 40
    ent = []
    for i in range(1, n + 1):
        if i % 7 == 3:
            continue  # empty row
        if i % 5 != 1:
            ent.append((i, i, float(rng.uniform(1, 4))))
        for _ in range(int(rng.integers(0, 5))):
            j = int(rng.integers(1, n + 1))
            ent.append((i, j, float(rng.choice([0.0, rng.uniform(-1, 1)]))))
    ent += [(9, 9, 2.0), (17, 17, 3.0)]  # extra diagonal records
    ent += [ent[4], (ent[6][0], ent[6][1], -7.5)]  # a repeat and an overwrite
    order = rng.permutation(len(ent))
    rec = records(n, [ent[k] for k in order])
    p = tmp_path / "r.bin"
    rec.tofile(p)
    for symm in (0, 1):
        check_same(amg.io.read(p, symm=symm, remove_disconnected=0), ref_read(rec, symm, 0))


@pytest.mark.parametrize("seed", [0, 1])
def test_remove_disconnected(amg, oracle, tmp_path, seed):
    """remove_disconnected_points_flag: isolated points (a diagonal record and
    nothing else in their column) dropped and the other rows renumbered, read
    with and without symm."""
    rng = np.random.default_rng(seed)
    A = oracle.laplace_7pt(4, 3, 3)
    iso = sorted(rng.choice(np.arange(A.nrows + 6), 6, replace=False))
    # global numbering with the isolated points interleaved
    keep = [g for g in range(A.nrows + 6) if g not in iso]
    # the whole matrix: with a lower triangle the last row's column holds only
    # its diagonal, so the reference would take it for disconnected and drop
    # num_rows once per record of that row (its "TODO: fix this"), leaving
    # renumbered rows past the end -- an error here
    ent = [(keep[i] + 1, keep[int(A.col[k])] + 1, float(A.val[k])) for i in range(A.nrows)
           for k in range(A.rowptr[i], A.rowptr[i + 1])]
    ent += [(g + 1, g + 1, float(rng.uniform(1, 2))) for g in iso]
    rec = records(A.nrows + 6, [ent[k] for k in rng.permutation(len(ent))])
    p = tmp_path / "iso.bin"
    rec.tofile(p)
    for symm in (0, 1):
        got = amg.io.read(p, symm=symm, remove_disconnected=1)
        check_same(got, ref_read(rec, symm, 1))
    n, _, rowptr, col, val = amg.io.read(p, symm=0, remove_disconnected=1)
    assert n == A.nrows and np.array_equal(rowptr, A.rowptr)
    for i in range(n):  # the same rows (record order shuffled), diagonal first
        s = slice(rowptr[i], rowptr[i + 1])
        assert col[rowptr[i]] == i and dict(zip(col[s], val[s])) == dict(zip(A.col[s], A.val[s]))
    # a lower triangle with the flag: the reference's row count goes wrong
    low = records(A.nrows, lower_triangle_entries(A))
    low.tofile(tmp_path / "low.bin")
    with pytest.raises(amg.AmgError):
        amg.io.read(tmp_path / "low.bin", symm=1, remove_disconnected=1)


def test_partition_file(amg, oracle, tmp_path):
    """ParReadBinary_fread: one rank's rows [lo, hi] (global), zero values skipped."""
    A = oracle.laplace_7pt(4)
    lo, hi = 17, 40
    ent = [(i + 1, int(A.col[k]) + 1, float(A.val[k])) for i in range(lo - 1, hi)
           for k in range(A.rowptr[i], A.rowptr[i + 1])]
    ent.insert(3, (lo, lo + 1, 0.0))
    rec = records(hi - lo + 1, ent)
    p = tmp_path / "part_2_1"
    rec.tofile(p)
    first, got = amg.io.read_part(p, A.ncols)
    assert first == lo - 1
    rows = [[] for _ in range(hi - lo + 1)]
    for i, j, v in ent:
        if abs(v) > 0:
            rows[i - lo].append((j - 1, v))
    check_same(got, assemble(rows, lo - 1))


def test_errors(amg, tmp_path):
    with pytest.raises(amg.AmgError):
        amg.io.read(tmp_path / "missing.bin")
    rec = records(3, [(1, 1, 1.0), (4, 1, 1.0)])
    rec.tofile(tmp_path / "bad.bin")
    with pytest.raises(amg.AmgError):
        amg.io.read(tmp_path / "bad.bin")
