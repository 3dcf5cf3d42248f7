"""End-to-end drop-in check (GPU): the C++ CLI par_fastaai_amd (SQLite
loader -> C ABI -> HIP engine -> CSV / cereal bin) reproduces the reference
CLI's output files byte for byte."""
import gzip
import os
import shutil
import subprocess

import numpy as np
import pytest

from helpers import gpath, text
from parfastaai_amd import formats as fm
from parfastaai_amd import syn

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "parfastaai_amd", "lib", "par_fastaai_amd")


def unpack(tmp_path, name):
    out = tmp_path / name
    with gzip.open(gpath(name)) as fi, open(out, "wb") as fo:
        shutil.copyfileobj(fi, fo)
    return str(out)


def run(*args):
    r = subprocess.run([CLI, *args], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return r


@pytest.mark.parametrize("devs", [[], ["--devices", "0,0"]], ids=["1dev", "2ctx"])
@pytest.mark.parametrize("name", ["xdb_subset1", "xdb_subset2"])
def test_cli_csv_bytes(tmp_path, name, devs):
    db = unpack(tmp_path, name + ".db")
    out = tmp_path / "out.csv"
    r = run(db, str(out), "--bin", str(tmp_path / "o"), *devs)
    # the drop-in runs the benchmarked path: <p>_genomes -> G, F (and G_pos / G_end) built on the GPU,
    # k_rows_pl walking from G_pos to G_end (pfaai_run_walk), the narrow rows as the 512-thread launch
    assert "<p>_genomes -> G" in r.stdout and "; k_rows_pl; walk G_pos..G_end, 512-thread narrow rows)" in r.stdout, \
        r.stdout
    assert out.read_text() == text(name + "_aji_matrix_wheader.csv")
    J = fm.read_jac(str(tmp_path / "o_jac.bin"))
    Jr = fm.read_jac(gpath(name + "_jac.bin"))
    assert np.array_equal(J, Jr)
    assert np.array_equal(fm.read_vec_f64(str(tmp_path / "o_aji.bin")), fm.read_vec_f64(gpath(name + "_aji.bin")))


def test_cli_qt_ref_compat_bins(tmp_path):
    t = unpack(tmp_path, "xdb_subset1.db")
    q = unpack(tmp_path, "xdb_subset2.db")
    run(t, str(tmp_path / "out.csv"), "-r", q, "--ref-compat", "--bin", str(tmp_path / "o"))
    assert np.array_equal(fm.read_jac(str(tmp_path / "o_jac.bin")), fm.read_jac(gpath("xdb_qt_jac.bin")))
    assert np.array_equal(fm.read_vec_f64(str(tmp_path / "o_aji.bin")), fm.read_vec_f64(gpath("xdb_qt_aji.bin")))


def test_cli_qt_correct_equals_merged_db_block(tmp_path):
    """Correct QT semantics = the target x query block of an all-vs-all run on
    the merged DB (xdb_subset_combo12.db)."""
    t = unpack(tmp_path, "xdb_subset1.db")
    q = unpack(tmp_path, "xdb_subset2.db")
    c = unpack(tmp_path, "xdb_subset_combo12.db")
    run(t, str(tmp_path / "qt.csv"), "-r", q, "--corrected")
    run(c, str(tmp_path / "all.csv"), "--corrected")
    qr, qc, QM = fm.read_csv_matrix(str(tmp_path / "qt.csv"))
    ar, ac, AM = fm.read_csv_matrix(str(tmp_path / "all.csv"))
    rows = [ar.index(n) for n in qr]
    cols = [ac.index(n) for n in qc]
    assert np.array_equal(QM, AM[np.ix_(rows, cols)])


@pytest.mark.parametrize("devs", [[], ["--devices", "0,0,0"]], ids=["1dev", "3ctx"])
@pytest.mark.parametrize("case", ["all48", "qsub40", "qt12", "qt8x12"])
def test_cli_vs_reference_binary_on_syn(tmp_path, case, devs):
    """The CLI's CSV equals the reference binary's, on one context and with the
    rows split over three contexts (--devices 0,0,0: the multi-GPU path, one
    host thread per context, on the box's one GPU; -q too since round 6 --
    each context's query-query cells merged into the triangle)."""
    import make_ref_vectors as mk
    kind, kw = mk.CASES[case]
    kw = dict(kw)
    out = str(tmp_path / "out.csv")
    if kind == "all":
        db = str(tmp_path / "s.db")
        syn.write_db(db, **kw)
        run(db, out, *devs)
    elif kind == "qsub":
        query = kw.pop("query")
        db = str(tmp_path / "s.db")
        g = syn.write_db(db, **kw)
        ql = tmp_path / "q.txt"
        ql.write_text("\n".join(g["genome_set"][i] for i in query) + "\n")
        run(db, out, "-q", str(ql), *devs)
    else:
        nT, nQ = kw.pop("n_tgt"), kw.pop("n_qry")
        tdb, qdb = str(tmp_path / "t.db"), str(tmp_path / "q.db")
        syn.write_db(tdb, n_genomes=nT, **kw)
        syn.write_db(qdb, n_genomes=nQ, genome_prefix="qry", genome_seed=syn.DEFAULT_SEED + 1,
                     n_clades=(nT + kw["clade_size"] - 1) // kw["clade_size"], clade_mod=True, **kw)
        run(tdb, out, "-r", qdb, "--ref-compat", *devs)
    assert open(out).read() == text(f"ref_{case}.csv")


def test_cli_orientations_disagree_at_equal_counts(tmp_path):
    """A DB whose `<p>_genomes` blobs hold as many but other memberships than
    its `<p>_tetras` blobs (make_ref_vectors.mutate_equal_count): the exact
    membership check sends it through `<p>_tetras`, and the CSV equals the
    reference binary's on that DB (tests/golden/ref_mismatch24.csv.gz) --
    trusting `<p>_genomes` would print other values."""
    import make_ref_vectors as mk
    _, kw = mk.CASES["mismatch24"]
    db = str(tmp_path / "m.db")
    syn.write_db(db, **kw)
    out = tmp_path / "o.csv"
    r = run(db, str(out))
    assert "<p>_genomes -> G" in r.stdout
    intact = out.read_text()
    mk.mutate_equal_count(db)
    r = run(db, str(out))
    assert "<p>_tetras -> F" in r.stdout, r.stdout
    assert out.read_text() == text("ref_mismatch24.csv")
    assert intact == text("ref_mismatch24.csv")  # (the reference ignores the `<p>_genomes` contents)


@pytest.mark.parametrize("name", ["xdb_subset1", "xdb_subset2"])
def test_cli_stream_aji_equals_reference_bin(tmp_path, name):
    """--stream-aji (pfaai_stream, tiles of 7 pairs) writes the reference's
    own <prefix>_aji.bin bytes."""
    db = unpack(tmp_path, name + ".db")
    out = tmp_path / "s_aji.bin"
    run(db, str(tmp_path / "unused.csv"), "--stream-aji", str(out), "--tile-pairs", "7")
    assert np.array_equal(fm.read_vec_f64(str(out)), fm.read_vec_f64(gpath(name + "_aji.bin")))
    assert not (tmp_path / "unused.csv").exists()


def test_cli_stream_aji_qt_ref_compat(tmp_path):
    t = unpack(tmp_path, "xdb_subset1.db")
    q = unpack(tmp_path, "xdb_subset2.db")
    out = tmp_path / "s_aji.bin"
    run(t, str(tmp_path / "unused.csv"), "-r", q, "--ref-compat", "--stream-aji", str(out), "--tile-pairs", "50")
    assert np.array_equal(fm.read_vec_f64(str(out)), fm.read_vec_f64(gpath("xdb_qt_aji.bin")))


@pytest.mark.parametrize("loader", ["genomes", "tetras"])
def test_cli_both_loaders_same_bytes(tmp_path, loader):
    """--loader tetras (F from `<p>_tetras`, G built on the GPU) and the default
    G ingest (F built on the GPU) write the same bytes, for -q and -r too."""
    db = unpack(tmp_path, "xdb_subset1.db")
    q = unpack(tmp_path, "xdb_subset2.db")
    r = run(db, str(tmp_path / "a.csv"), "--loader", loader)
    assert "; k_rows_pl; walk G_pos..G_end" in r.stdout, r.stdout
    assert (tmp_path / "a.csv").read_text() == text("xdb_subset1_aji_matrix_wheader.csv")
    r = run(db, str(tmp_path / "b.csv"), "-r", q, "--loader", loader, "--ref-compat", "--bin", str(tmp_path / "b"))
    assert "; k_rows_pl; walk run table + splitters)" in r.stdout, r.stdout
    assert np.array_equal(fm.read_vec_f64(str(tmp_path / "b_aji.bin")), fm.read_vec_f64(gpath("xdb_qt_aji.bin")))


@pytest.mark.parametrize("compat", [[], ["--corrected"]], ids=["default", "corrected"])
def test_cli_c1_rebuilt_db(tmp_path, compat):
    """Config C1 end to end: the reference's 20-genome DB (rebuilt from its
    fixtures, tests/test_c1_loader.py) through par_fastaai_amd -- CSV byte-
    identical to the reference's xanthodb_aji_matrix_wheader.csv, and the -q
    run to qsub_test_output_matrix_wheader.csv."""
    from test_c1_loader import rebuild_xantho
    db = rebuild_xantho(str(tmp_path))
    out = tmp_path / "o.csv"
    r = run(db, str(out), *compat)
    assert "; k_rows_pl; walk G_pos..G_end" in r.stdout, r.stdout
    assert out.read_text() == text("xanthodb_aji_matrix_wheader.csv")
    q = tmp_path / "q.txt"
    q.write_text(text("qsub_test_input.txt"))
    run(db, str(out), "-q", str(q), *compat)
    assert out.read_text() == text("qsub_test_output_matrix_wheader.csv")
    # -q with its query rows split over three contexts (round 6)
    r = run(db, str(out), "-q", str(q), "--devices", "0,0,0", *compat)
    assert "AJI (MI355X x3)" in r.stdout, r.stdout
    assert out.read_text() == text("qsub_test_output_matrix_wheader.csv")


@pytest.mark.parametrize("name", ["xdb_subset1", "xdb_subset2"])
def test_cli_stream_csv_bytes(tmp_path, name):
    """--stream-csv (pfaai_stream_matrix tiles of 3 whole rows, formatted as
    they arrive) writes the reference's CSV byte for byte."""
    db = unpack(tmp_path, name + ".db")
    out = tmp_path / "out.csv"
    r = run(db, str(out), "--stream-csv", "--tile-rows", "3")
    assert "CSV (streamed)" in r.stdout, r.stdout
    assert out.read_text() == text(name + "_aji_matrix_wheader.csv")


@pytest.mark.parametrize("case", ["all48", "qsub40", "qt12", "qt8x12"])
def test_cli_stream_csv_vs_reference_binary_on_syn(tmp_path, case):
    import make_ref_vectors as mk
    kind, kw = mk.CASES[case]
    kw = dict(kw)
    out = str(tmp_path / "out.csv")
    s = ["--stream-csv", "--tile-rows", "5"]
    if kind == "all":
        db = str(tmp_path / "s.db")
        syn.write_db(db, **kw)
        run(db, out, *s)
    elif kind == "qsub":
        query = kw.pop("query")
        db = str(tmp_path / "s.db")
        g = syn.write_db(db, **kw)
        ql = tmp_path / "q.txt"
        ql.write_text("\n".join(g["genome_set"][i] for i in query) + "\n")
        run(db, out, "-q", str(ql), *s)
    else:
        nT, nQ = kw.pop("n_tgt"), kw.pop("n_qry")
        tdb, qdb = str(tmp_path / "t.db"), str(tmp_path / "q.db")
        syn.write_db(tdb, n_genomes=nT, **kw)
        syn.write_db(qdb, n_genomes=nQ, genome_prefix="qry", genome_seed=syn.DEFAULT_SEED + 1,
                     n_clades=(nT + kw["clade_size"] - 1) // kw["clade_size"], clade_mod=True, **kw)
        run(tdb, out, "-r", qdb, "--ref-compat", *s)
    assert open(out).read() == text(f"ref_{case}.csv")


def test_cli_stream_csv_c1_qsub(tmp_path):
    from test_c1_loader import rebuild_xantho
    db = rebuild_xantho(str(tmp_path))
    q = tmp_path / "q.txt"
    q.write_text(text("qsub_test_input.txt"))
    out = tmp_path / "o.csv"
    run(db, str(out), "-q", str(q), "--stream-csv", "--tile-rows", "2")
    assert out.read_text() == text("qsub_test_output_matrix_wheader.csv")
    run(db, str(out), "--stream-csv")
    assert out.read_text() == text("xanthodb_aji_matrix_wheader.csv")


def test_cli_stream_csv_40k_bounded_rss(tmp_path):
    """40,000 genomes: the default writer holds the JAC vector (16 GB), the AJI
    vector (6.4 GB) and the dense matrix (12.8 GB); --stream-csv holds the
    loaded DB plus two 256 MB pinned tiles, so the CLI's peak RSS stays far
    below any of them.  The CSV (~25 GB) goes to /dev/null; its bytes are
    pinned by the fixture tests above (same code path)."""
    import sys
    db = str(tmp_path / "s40k.db")
    syn.write_db(db, n_genomes=40000, n_prot=12, clade_size=40)
    # peak RSS of the CLI alone: a fresh interpreter whose only child it is
    probe = ("import resource, subprocess, sys\n"
             "r = subprocess.run(sys.argv[1:], capture_output=True, text=True)\n"
             "sys.stdout.write(r.stdout + r.stderr)\n"
             "print('PEAK_KB', resource.getrusage(resource.RUSAGE_CHILDREN).ru_maxrss)\n"
             "sys.exit(r.returncode)\n")
    r = subprocess.run([sys.executable, "-c", probe, CLI, db, "/dev/null", "--stream-csv"],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "CSV (streamed)" in r.stdout, r.stdout
    peak_kb = int(r.stdout.split("PEAK_KB")[1])
    print(r.stdout)
    assert peak_kb < 4_000_000, peak_kb  # < 4 GB, vs 35 GB for the default writer


@pytest.mark.parametrize("case", ["zero3", "zero30"])
def test_cli_default_is_reference_exact_on_zero_overlap(tmp_path, case):
    """One drop-in default: on DBs whose genome pairs may
    share no tetramer, `par_fastaai_amd in.db out.csv` prints the reference
    binary's bytes (the pair gets the J of E[0]'s protein, algorithm_impl.hpp:
    90-91); --corrected writes AJI 0 for exactly those pairs and the oracle's
    corrected values everywhere."""
    import make_ref_vectors as mk
    import oracle as O
    from helpers import dense_all, sets_problem

    kw = mk.CASES[case][1]
    db = str(tmp_path / "z.db")
    syn.write_db_sets(db, mk.sets_for(case), **kw)
    out = tmp_path / "out.csv"
    run(db, str(out))
    assert out.read_text() == text(f"ref_{case}.csv")
    run(db, str(out), "--stream-csv", "--tile-rows", "4")
    assert out.read_text() == text(f"ref_{case}.csv")
    run(db, str(out), "--corrected")
    n = kw["n_genomes"]
    r = O.Problem(sets_problem(mk.sets_for(case), n, kw["n_prot"]), compat=False).ref_run()
    names = syn.genome_names(n)
    assert out.read_text() == fm.csv_text(names, names, dense_all(r["AJI"], n))


def test_cli_fast_exit_writes_complete_outputs(tmp_path):
    """The CLI leaves by std::_Exit after flushing (skipping the HIP
    runtime's exit-time teardown); every output -- CSV, --bin's three cereal
    files, --stream-csv, --stream-aji -- must be byte-identical to a run that
    returns from main normally (PFAAI_CLI_FAST_EXIT=0), with the same exit
    code."""
    db = unpack(tmp_path, "xdb_subset1.db")
    outs = {}
    for fast in ("1", "0"):
        d = tmp_path / f"fast{fast}"
        d.mkdir()
        env = dict(os.environ, PFAAI_CLI_FAST_EXIT=fast)
        for args in ([str(d / "a.csv"), "--bin", str(d / "b")], [str(d / "s.csv"), "--stream-csv", "--tile-rows", "3"],
                     [str(d / "u.csv"), "--stream-aji", str(d / "s_aji.bin")]):
            r = subprocess.run([CLI, db, *args], capture_output=True, text=True, timeout=300, env=env)
            outs.setdefault(args[1], []).append(r.returncode)
        outs[fast] = {f: (d / f).read_bytes() for f in ("a.csv", "b_jac.bin", "b_aji.bin", "b_aji_matrix.bin",
                                                        "s.csv", "s_aji.bin")}
    assert outs["1"] == outs["0"]
    assert all(rc == [0, 0] for k, rc in outs.items() if k not in ("0", "1"))
    assert outs["1"]["a.csv"].decode() == text("xdb_subset1_aji_matrix_wheader.csv")


@pytest.mark.timeout(600)
def test_cli_c2_csv_equals_reference_binary(tmp_path):
    """Config C2 end to end (SYN 2 000 x 100 SQLite DB -> CSV, 86 MB): the
    CLI's CSV hashes to the SHA-256 of the reference binary's CSV on the same
    DB (tests/golden/full_digests.json "C2_cli_csv", made in the container by
    oracle/_ref/par_fastaai.x -- the reference built from its own sources),
    and the run takes the benchmarked kernel form."""
    import hashlib
    import json

    with open(os.path.join(ROOT, "tests", "golden", "full_digests.json")) as f:
        want = json.load(f)["C2_cli_csv"]
    db = str(tmp_path / "c2.db")
    syn.write_db(db, 2000, 100)
    out = tmp_path / "c2.csv"
    r = run(db, str(out))
    assert "<p>_genomes -> G" in r.stdout and "; k_rows_pl; walk G_pos..G_end, 512-thread narrow rows)" in r.stdout, \
        r.stdout
    assert out.stat().st_size == want["bytes"]
    assert hashlib.sha256(out.read_bytes()).hexdigest() == want["sha256"]
