"""Host side of the drop-in CLI (CPU only): option handling and exit codes,
the SQLite loader against the reference's fixture arrays, and the fmt-exact
number format.  The GPU leg is tests/test_gpu_cli.py."""
import gzip
import os
import shutil
import struct
import subprocess

import numpy as np
import pytest

from helpers import GOLDEN, gpath, text
from parfastaai_amd import formats as fm

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.environ.get("PFAAI_CLI", os.path.join(ROOT, "parfastaai_amd", "lib", "par_fastaai_amd"))  # (tools/sanitize.py)


def run(*args, **kw):
    return subprocess.run([CLI, *args], capture_output=True, text=True, **kw)


def unpack(tmp_path, name):
    out = tmp_path / name
    with gzip.open(gpath(name)) as fi, open(out, "wb") as fo:
        shutil.copyfileobj(fi, fo)
    return str(out)


def test_cli_exit_codes(tmp_path):
    assert run().returncode == 106                               # RequiredError
    assert run("/nonexistent.db", "o.csv").returncode == 105     # ValidationError (ExistingFile)
    db = unpack(tmp_path, "xdb_subset1.db")
    assert run(db).returncode == 106
    assert run(db, "o.csv", "-q", "/nonexistent.txt").returncode == 105
    assert run(db, "o.csv", "--bogus").returncode == 109         # ExtrasError
    assert run("--help").returncode == 0


@pytest.mark.parametrize("name", ["xdb_subset1", "xdb_subset2"])
def test_loader_matches_reference_arrays(tmp_path, name):
    db = unpack(tmp_path, name + ".db")
    pre = str(tmp_path / "dump")
    r = run(db, str(tmp_path / "o.csv"), "--dump-arrays", pre)
    assert r.returncode == 0, r.stderr
    assert np.array_equal(fm.read_vec_i32(pre + "_lc_array.bin"), fm.read_vec_i32(gpath(name + "_lc_array.bin")))
    assert np.array_equal(fm.read_f_array(pre + "_f_array.bin"), fm.read_f_array(gpath(name + "_f_array.bin")))
    assert np.array_equal(fm.read_matrix_i32(pre + "_t_matrix.bin"), fm.read_matrix_i32(gpath(name + "_t_matrix.bin")))


def test_qt_loader_matches_reference_arrays(tmp_path):
    t = unpack(tmp_path, "xdb_subset1.db")
    q = unpack(tmp_path, "xdb_subset2.db")
    pre = str(tmp_path / "dump")
    r = run(t, str(tmp_path / "o.csv"), "-r", q, "--dump-arrays", pre)
    assert r.returncode == 0, r.stderr
    assert np.array_equal(fm.read_vec_i32(pre + "_lc_array.bin"), fm.read_vec_i32(gpath("xdb_qt_lc_array.bin")))
    assert np.array_equal(fm.read_f_array(pre + "_f_array.bin"), fm.read_f_array(gpath("xdb_qt_f_array.bin")))
    assert np.array_equal(fm.read_matrix_i32(pre + "_t_matrix.bin"), fm.read_matrix_i32(gpath("xdb_qt_t_matrix.bin")))


def test_bad_query_list_exit_3(tmp_path):
    # validate_subset (main.cpp:204-232): unknown genome -> error box, rc 3
    db = unpack(tmp_path, "xdb_subset1.db")
    ql = unpack(tmp_path, "qsub_test_bad_input.txt")
    r = run(db, str(tmp_path / "o.csv"), "-q", ql)
    assert r.returncode == 3 and "missing from the database" in r.stdout


def test_overlapping_qt_exit_3(tmp_path):
    # validate_qry2tgt (main.cpp:268-300): subset1 vs itself-overlapping combo DB
    t = unpack(tmp_path, "xdb_subset_combo12.db")
    q = unpack(tmp_path, "xdb_subset1.db")
    r = run(t, str(tmp_path / "o.csv"), "-r", q)
    assert r.returncode == 3 and "overlapping" in r.stdout


def test_fmt_double_matches_fmt10(tmp_path):
    rng = np.random.default_rng(7)
    vals = np.concatenate([
        rng.random(2000), rng.random(200) * 1e-3, rng.random(50) * 1e-6, rng.random(50) * 1e17,
        [0.0, 1.0, 0.5, 1e-4, 1e-5, 0.0001234, 1e16, 1e15, 123456789012345.0, 2.0, 1.0009481433436662,
         9.999999999999999e-05, 5e-324, 1.7976931348623157e308, 0.1, 100.0],
    ])
    f = tmp_path / "v.txt"
    f.write_text("\n".join(float(v).hex() for v in vals) + "\n")
    r = run("--format-selftest", str(f))
    assert r.returncode == 0
    assert r.stdout.splitlines() == [fm.fmt_double(v) for v in vals]


def test_fmt_rule_on_fixture_csv():
    # every cell of the reference's CSV fixtures re-formats to itself
    for name in ["xanthodb_aji_matrix_wheader.csv", "xdb_subset1_aji_matrix_wheader.csv",
                 "qsub_test_output_matrix_wheader.csv"]:
        for line in text(name).splitlines()[1:]:
            for cell in line.split(",")[1:]:
                assert fm.fmt_double(float(cell)) == cell


def _f_from_g(G_off, G_tet, n_ids, P):
    """F (protein, genome) ordered by (tetramer, protein, genome) and Lc from
    genome-major lists: the host statement of what pfaai_load builds on the
    device from G (stable sort by tetramer * P + protein)."""
    lens = np.diff(G_off)
    lst = np.repeat(np.arange(n_ids * P, dtype=np.int64), lens)
    g, p = lst // P, lst % P
    t = G_tet.astype(np.int64)
    order = np.lexsort((g, p, t))
    F = np.stack([p[order], g[order]], axis=1).astype(np.int32)
    return F, np.bincount(t, minlength=160000).astype(np.int32)


def _read_i64_vec(path):
    raw = open(path, "rb").read()
    n = struct.unpack("<Q", raw[:8])[0]
    return np.frombuffer(raw[8:8 + 8 * n], dtype=np.int64)


@pytest.mark.parametrize("name", ["xdb_subset1", "xdb_subset2"])
def test_genomes_loader_gives_reference_f(tmp_path, name):
    """The default ingest (`<p>_genomes` -> G): F built from G equals the
    reference's F fixture, Lc and T too (the GPU does this build)."""
    db = unpack(tmp_path, name + ".db")
    pre = str(tmp_path / "g")
    r = run(db, str(tmp_path / "o.csv"), "--dump-genomes", pre)
    assert r.returncode == 0, r.stderr
    assert "<p>_genomes -> G" in r.stdout
    G_off, G_tet = _read_i64_vec(pre + "_g_off.bin"), fm.read_vec_i32(pre + "_g_tet.bin")
    T = fm.read_matrix_i32(pre + "_t_matrix.bin")
    P, n = T.shape
    assert len(G_off) == n * P + 1 and G_off[-1] == len(G_tet)
    for k in range(n * P):  # strictly ascending lists
        assert (np.diff(G_tet[G_off[k]:G_off[k + 1]]) > 0).all()
    F, Lc = _f_from_g(G_off, G_tet, n, P)
    assert np.array_equal(F, fm.read_f_array(gpath(name + "_f_array.bin")))
    assert np.array_equal(Lc, fm.read_vec_i32(gpath(name + "_lc_array.bin")))
    assert np.array_equal(T, fm.read_matrix_i32(gpath(name + "_t_matrix.bin")))


def test_genomes_loader_qt(tmp_path):
    """-r: both DBs' lists, query ids offset by nT; F from G restricted to the
    tetramers present in both DBs (the reference's inner join) is the
    reference's QT F, and T is its QT T."""
    t = unpack(tmp_path, "xdb_subset1.db")
    q = unpack(tmp_path, "xdb_subset2.db")
    pre = str(tmp_path / "g")
    r = run(t, str(tmp_path / "o.csv"), "-r", q, "--dump-genomes", pre)
    assert r.returncode == 0, r.stderr
    G_off, G_tet = _read_i64_vec(pre + "_g_off.bin"), fm.read_vec_i32(pre + "_g_tet.bin")
    T = fm.read_matrix_i32(pre + "_t_matrix.bin")
    assert np.array_equal(T, fm.read_matrix_i32(gpath("xdb_qt_t_matrix.bin")))
    P, n = T.shape
    F, _ = _f_from_g(G_off, G_tet, n, P)
    ref = fm.read_f_array(gpath("xdb_qt_f_array.bin"))
    # keep the (tetramer, protein) runs holding both a target and a query genome
    lens = np.diff(G_off)
    lst = np.repeat(np.arange(n * P, dtype=np.int64), lens)
    tet = np.sort(G_tet.astype(np.int64) * P + lst % P, kind="stable")  # run key per F entry, F order
    nT = 4
    key_t = set(np.unique(tet[F[:, 1] < nT]).tolist())
    key_q = set(np.unique(tet[F[:, 1] >= nT]).tolist())
    both = np.array([k in key_t and k in key_q for k in tet])
    assert np.array_equal(F[both], ref)


def test_genomes_loader_falls_back_when_orientations_disagree(tmp_path):
    """The `<p>_genomes` ingest is taken only when every protein's genome
    lists hold as many memberships as its `<p>_tetras` blobs (the reference's
    F source, scp_db.hpp:161-216); a DB whose two orientations disagree is
    read through `<p>_tetras`, so the output stays the reference's."""
    import sqlite3

    from parfastaai_amd import syn

    db = str(tmp_path / "s.db")
    syn.write_db(db, n_genomes=12, n_prot=4, clade_size=4)
    r = run(db, str(tmp_path / "o.csv"), "--dump-genomes", str(tmp_path / "g"))
    assert r.returncode == 0 and "<p>_genomes -> G" in r.stdout, r.stdout + r.stderr
    con = sqlite3.connect(db)
    gid, blob = con.execute("SELECT genome_id, tetramers FROM `SYN00002.1_genomes` LIMIT 1").fetchone()
    t = np.frombuffer(blob, "<i4")
    extra = next(x for x in range(159999, 0, -1) if x not in set(t.tolist()))  # a tetramer F does not list
    con.execute("UPDATE `SYN00002.1_genomes` SET tetramers = ? WHERE genome_id = ?",
                (np.sort(np.r_[t, extra]).astype("<i4").tobytes(), gid))
    con.commit()
    con.close()
    r = run(db, str(tmp_path / "o.csv"), "--dump-genomes", str(tmp_path / "g"))
    assert r.returncode == 0 and "<p>_tetras -> F" in r.stdout, r.stdout + r.stderr


def test_genomes_loader_falls_back_at_equal_counts(tmp_path):
    """Exact check, not a count: the `<p>_genomes` lists of one protein hold
    as many memberships as its `<p>_tetras` blobs but a different one
    (make_ref_vectors.mutate_equal_count) -> the `<p>_tetras` path (the CSV
    against the reference binary's: tests/test_gpu_cli.py); the same for
    the query DB of -r."""
    import make_ref_vectors as mk
    from parfastaai_amd import syn

    _, kw = mk.CASES["mismatch24"]
    db = str(tmp_path / "m.db")
    syn.write_db(db, **kw)
    r = run(db, str(tmp_path / "o.csv"), "--dump-genomes", str(tmp_path / "g"))
    assert r.returncode == 0 and "<p>_genomes -> G" in r.stdout, r.stdout + r.stderr
    mk.mutate_equal_count(db)
    r = run(db, str(tmp_path / "o.csv"), "--dump-genomes", str(tmp_path / "g"))
    assert r.returncode == 0 and "<p>_tetras -> F" in r.stdout, r.stdout + r.stderr
    # -r: an intact target DB with a mutated query DB, and the other way round
    q, qm = str(tmp_path / "q.db"), str(tmp_path / "qm.db")
    syn.write_db(q, genome_prefix="qry", **kw)
    syn.write_db(qm, genome_prefix="qry", **kw)
    mk.mutate_equal_count(qm)
    t = str(tmp_path / "t.db")
    syn.write_db(t, **kw)
    r = run(t, str(tmp_path / "o.csv"), "-r", q, "--dump-genomes", str(tmp_path / "g"))
    assert r.returncode == 0 and "<p>_genomes -> G" in r.stdout, r.stdout + r.stderr
    for a, b in ((t, qm), (db, q)):
        r = run(a, str(tmp_path / "o.csv"), "-r", b, "--dump-genomes", str(tmp_path / "g"))
        assert r.returncode == 0 and "<p>_tetras -> F" in r.stdout, r.stdout + r.stderr
