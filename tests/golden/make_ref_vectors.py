"""Golden vectors produced by the reference itself on synthetic databases.

Builds small SYN databases (parfastaai_amd/syn.py, deterministic), runs the
reference CLI compiled from its own sources (oracle/_ref/par_fastaai.x, see
oracle/build_ref.sh) on them and stores its output CSVs gzip'd under
tests/golden/ref_<case>.csv.gz.  The tests regenerate the same arrays with
syn.generate() and compare the HIP engine's matrix with these files.

Run in the build container (needs oracle/_ref/par_fastaai.x):
    python tests/golden/make_ref_vectors.py
"""
import gzip
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from parfastaai_amd import syn  # noqa: E402

REF = os.path.join(ROOT, "oracle", "_ref", "par_fastaai.x")

# name -> (kind, kwargs)
CASES = {
    # all-vs-all, 48 genomes x 24 SCPs, clades of 8
    "all48": ("all", dict(n_genomes=48, n_prot=24, clade_size=8)),
    # all-vs-all with sparse proteins (has=0.6) so some pairs miss proteins
    "all32_sparse": ("all", dict(n_genomes=32, n_prot=16, clade_size=4, has=0.6, keep=0.7)),
    # query subset (-q) with a sorted list of 7 genomes out of 40
    "qsub40": ("qsub", dict(n_genomes=40, n_prot=20, clade_size=5, query=[1, 4, 9, 10, 22, 31, 39])),
    # query-vs-target (-r), 12 targets x 12 queries (nQ == nT keeps the
    # reference's column map intact; its T-index quirk is reproduced under
    # ref-compat and pinned here)
    "qt12": ("qt", dict(n_tgt=12, n_qry=12, n_prot=20, clade_size=4)),
    # -r with more queries than targets: the reference's rows overlap (its
    # column placement of the quirky JAC ids, ds_impl.hpp:434-436 +
    # main.cpp:149) -- --stream-csv must still print these bytes
    "qt8x12": ("qt", dict(n_tgt=8, n_qry=12, n_prot=20, clade_size=4)),
    # explicit memberships (syn.write_db_sets) with pairs that share no
    # tetramer in any protein: the reference gives them the
    # J of E[0]'s protein; the drop-in CLI's default must print the same bytes
    "zero3": ("sets", dict(n_genomes=3, n_prot=2)),
    "zero30": ("sets", dict(n_genomes=30, n_prot=3)),
    # a DB whose `<p>_genomes` blobs disagree with its `<p>_tetras` blobs at
    # equal membership counts (mutate_equal_count): the reference reads F from
    # `<p>_tetras` and only the lengths of `<p>_genomes` (scp_db.hpp:161-262),
    # so a drop-in that trusted `<p>_genomes` would print other values
    "mismatch24": ("mismatch", dict(n_genomes=24, n_prot=6, clade_size=4)),
}


def mutate_equal_count(db, acc="SYN00002.1", k=3):
    """Replace one tetramer of the k-th `<acc>_genomes` blob by one the blob
    does not hold (same length, still a sorted set): the two orientations
    then hold equally many but different memberships."""
    import sqlite3

    import numpy as np

    con = sqlite3.connect(db)
    gid, blob = con.execute(f"SELECT genome_id, tetramers FROM `{acc}_genomes` ORDER BY genome_id LIMIT 1 OFFSET {k}"
                            ).fetchone()
    t = np.frombuffer(blob, "<i4").copy()
    have = set(t.tolist())
    t[len(t) // 2] = next(x for x in range(159999, 0, -1) if x not in have)
    con.execute(f"UPDATE `{acc}_genomes` SET tetramers = ? WHERE genome_id = ?",
                (np.sort(t).astype("<i4").tobytes(), gid))
    con.commit()
    con.close()


def sets_for(name):
    """The memberships {(genome, protein): tetramers} of a "sets" case."""
    import numpy as np

    if name == "zero3":  # genome 2 shares no tetramer with genome 0 (tests/test_gpu_parity.py::_zero_overlap_ds)
        blocks = {(5, 0): [0, 1], (9, 0): [1, 2], (11, 1): [0, 1], (20, 1): [2], (30, 0): [0]}
        out = {}
        for (t, p), gs in blocks.items():
            for g in gs:
                out.setdefault((g, p), []).append(t)
        return out
    # zero30: 30 genomes, 3 proteins, 2-4 tetramers each drawn from 60 ids in
    # three disjoint ranges per genome group, some proteins missing: many
    # pairs share nothing at all
    rng = np.random.default_rng(30)
    out = {}
    for g in range(30):
        grp = g % 3
        for p in range(3):
            if rng.random() < 0.8:
                out[(g, p)] = [int(x) for x in rng.choice(np.arange(grp * 20, grp * 20 + 20) + 1000 * p,
                                                          size=int(rng.integers(2, 5)), replace=False)]
    return out


def run_ref(args, out_csv):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run([REF, *args, out_csv], capture_output=True, text=True, env=env)
    if r.returncode != 0:
        raise RuntimeError(f"reference failed ({r.returncode}): {r.stderr[-2000:]}")


def main():
    if not os.path.exists(REF):
        sys.exit("oracle/_ref/par_fastaai.x missing: run oracle/build_ref.sh")
    with tempfile.TemporaryDirectory() as td:
        for name, (kind, kw) in CASES.items():
            if len(sys.argv) > 1 and name not in sys.argv[1:]:
                continue
            out = os.path.join(td, name + ".csv")
            if kind == "all":
                db = os.path.join(td, name + ".db")
                syn.write_db(db, **kw)
                run_ref([db], out)
            elif kind == "qsub":
                kw = dict(kw)
                query = kw.pop("query")
                db = os.path.join(td, name + ".db")
                g = syn.write_db(db, **kw)
                ql = os.path.join(td, name + ".txt")
                with open(ql, "w") as f:
                    f.write("\n".join(g["genome_set"][i] for i in query) + "\n")
                run_ref([db, "-q", ql], out)
            elif kind == "sets":
                db = os.path.join(td, name + ".db")
                syn.write_db_sets(db, sets_for(name), **kw)
                run_ref([db], out)
            elif kind == "mismatch":
                db = os.path.join(td, name + ".db")
                syn.write_db(db, **kw)
                mutate_equal_count(db)
                run_ref([db], out)
            else:
                kw = dict(kw)
                nT, nQ = kw.pop("n_tgt"), kw.pop("n_qry")
                tdb, qdb = os.path.join(td, name + "_t.db"), os.path.join(td, name + "_q.db")
                syn.write_db(tdb, n_genomes=nT, **kw)
                syn.write_db(qdb, n_genomes=nQ, genome_prefix="qry", genome_seed=syn.DEFAULT_SEED + 1,
                             n_clades=(nT + kw["clade_size"] - 1) // kw["clade_size"], clade_mod=True, **kw)
                run_ref([tdb, "-r", qdb], out)
            with open(out, "rb") as fi, gzip.GzipFile(os.path.join(HERE, f"ref_{name}.csv.gz"), "wb", mtime=0) as fo:
                fo.write(fi.read())
            print("wrote", name)


if __name__ == "__main__":
    main()
