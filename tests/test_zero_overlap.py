"""SURVEY §8a row Z -- genome pairs that share no tetramer in any protein.

The reference leaves their extents at 0/0 (algorithm_impl.hpp:90-91), so they
get S = J of E[0]'s protein and N = 1; main.cpp:143-154 prints that.  The
golden CSVs tests/golden/ref_zero{3,30}.csv.gz are the reference binary's own
output on two such DBs (tests/golden/make_ref_vectors.py, syn.write_db_sets).
CPU: the oracle's compat mode reproduces them byte for byte (pins the oracle
for this quirk).  GPU (tests/test_gpu_cli.py): the drop-in CLI's DEFAULT
output equals them, and --corrected writes 0 for exactly those cells."""
import numpy as np
import pytest

import make_ref_vectors as mk
import oracle as O
from helpers import dense_all, sets_problem, text
from parfastaai_amd import formats as fm
from parfastaai_amd import syn


@pytest.mark.parametrize("case", ["zero3", "zero30"])
def test_oracle_compat_reproduces_reference_csv(case):
    kw = mk.CASES[case][1]
    n, P = kw["n_genomes"], kw["n_prot"]
    pb = sets_problem(mk.sets_for(case), n, P)
    r = O.Problem(pb, compat=True).ref_run()
    names = syn.genome_names(n)
    assert fm.csv_text(names, names, dense_all(r["AJI"], n)) == text(f"ref_{case}.csv")
    # the case really has zero-overlap pairs, and the corrected mode differs exactly there
    rc = O.Problem(pb, compat=False).ref_run()
    zero = rc["N"] == 0
    assert zero.any()
    assert np.all(rc["AJI"][zero] == 0) and np.any(r["AJI"][zero] != 0)
    assert np.array_equal(r["AJI"][~zero], rc["AJI"][~zero])
