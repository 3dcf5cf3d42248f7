"""Config C1 through the SQLite loader (CPU): the reference's 20-genome test
DB, rebuilt from its committed arrays and names by tools/rebuild_xantho_db
(the DB is a missing blob upstream), read by the drop-in CLI's loader.

  * the loader's arrays equal the reference's xanthodb_{lc,f,t} fixtures (the
    `<p>_tetras` path), and F built from the `<p>_genomes` path equals them too;
  * the reference's own known-answer checks on that DB (pfaai_tests.cpp):
    tetramerOccCounts("PF00119.20", [2060, 2144]) gives Lc[2060] = 20,
    Lc[2100] = 20, Lc[2140] = 3, Lc[2144] = 17 (:129-137); F spot values
    F[Lp[2000]] = (5, 0), F[Lp[2415] - 1] = (35, 0x13), F[Lp[2415]] =
    (74, 0x11) (:154-171); the first four T rows (:139-152, == the T fixture);
  * where the reference binary was built here (oracle/_ref), it reproduces
    the reference's CSV fixtures byte for byte on the rebuilt DB -- the
    rebuild is faithful.
The GPU leg (CLI CSV on this DB) is tests/test_gpu_cli.py::test_cli_c1_rebuilt_db.
"""
import gzip
import os
import shutil
import subprocess

import numpy as np
import pytest

from helpers import GOLDEN, gpath, text
from parfastaai_amd import formats as fm

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# PFAAI_CLI / PFAAI_REBUILD_TOOL: the sanitizer builds of tools/sanitize.py
CLI = os.environ.get("PFAAI_CLI", os.path.join(ROOT, "parfastaai_amd", "lib", "par_fastaai_amd"))
TOOL = os.environ.get("PFAAI_REBUILD_TOOL", os.path.join(ROOT, "tools", "_build", "rebuild_xantho_db"))
REF = os.path.join(ROOT, "oracle", "_ref", "par_fastaai.x")


def rebuild_xantho(tmp):
    """Rebuild the C1 DB into tmp; returns its path."""
    ins = []
    for f in ("xanthodb_f_array.bin", "xanthodb_lc_array.bin", "xanthodb_t_matrix.bin"):
        out = os.path.join(tmp, f)
        with gzip.open(gpath(f)) as fi, open(out, "wb") as fo:
            shutil.copyfileobj(fi, fo)
        ins.append(out)
    db = os.path.join(tmp, "modified_xantho_fastaai2.db")
    r = subprocess.run([TOOL, *ins, os.path.join(GOLDEN, "xantho_names.txt"), db], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return db


def test_c1_loader_arrays_and_known_answers(tmp_path):
    db = rebuild_xantho(str(tmp_path))
    pre = str(tmp_path / "d")
    r = subprocess.run([CLI, db, str(tmp_path / "o.csv"), "--dump-arrays", pre], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    Lc = fm.read_vec_i32(pre + "_lc_array.bin")
    F = fm.read_f_array(pre + "_f_array.bin")
    T = fm.read_matrix_i32(pre + "_t_matrix.bin")
    assert np.array_equal(Lc, fm.read_vec_i32(gpath("xanthodb_lc_array.bin")))
    assert np.array_equal(F, fm.read_f_array(gpath("xanthodb_f_array.bin")))
    assert np.array_equal(T, fm.read_matrix_i32(gpath("xanthodb_t_matrix.bin")))
    Lp = np.concatenate([[0], np.cumsum(Lc)])
    # tetramerOccCounts("PF00119.20" = protein 0, [2060, 2144])
    tet = np.repeat(np.arange(160000), Lc)
    p0 = F[:, 0] == 0
    lc0 = np.bincount(tet[p0], minlength=160000)
    assert (lc0[2060], lc0[2100], lc0[2140], lc0[2144]) == (20, 20, 3, 17)
    assert tuple(F[Lp[2000]]) == (5, 0)
    assert tuple(F[Lp[2415] - 1]) == (35, 0x13)
    assert tuple(F[Lp[2415]]) == (74, 0x11)


def test_c1_genomes_path_gives_reference_f(tmp_path):
    from test_cli_host import _f_from_g, _read_i64_vec
    db = rebuild_xantho(str(tmp_path))
    pre = str(tmp_path / "g")
    r = subprocess.run([CLI, db, str(tmp_path / "o.csv"), "--dump-genomes", pre], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    G_off, G_tet = _read_i64_vec(pre + "_g_off.bin"), fm.read_vec_i32(pre + "_g_tet.bin")
    F, Lc = _f_from_g(G_off, G_tet, 20, 80)
    assert np.array_equal(F, fm.read_f_array(gpath("xanthodb_f_array.bin")))
    assert np.array_equal(Lc, fm.read_vec_i32(gpath("xanthodb_lc_array.bin")))


@pytest.mark.skipif(not os.path.exists(REF), reason="reference binary not built here (oracle/build_ref.sh)")
def test_c1_rebuilt_db_reproduces_reference_csvs(tmp_path):
    db = rebuild_xantho(str(tmp_path))
    out = tmp_path / "ref.csv"
    subprocess.run([REF, db, str(out)], capture_output=True, check=True)
    assert out.read_text() == text("xanthodb_aji_matrix_wheader.csv")
    q = tmp_path / "q.txt"
    q.write_text(text("qsub_test_input.txt"))
    subprocess.run([REF, "-q", str(q), db, str(out)], capture_output=True, check=True)
    assert out.read_text() == text("qsub_test_output_matrix_wheader.csv")
