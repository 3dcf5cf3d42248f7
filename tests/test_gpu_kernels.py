"""Kernel-level GPU checks: the row kernels' exact small-integer division is
bit-identical to IEEE '/', and every selectable row-kernel variant
(PFAAI_ROWS_KERNEL, read by pfaai_run) reproduces the oracle bit-exactly."""
import os

import numpy as np
import pytest

import oracle as O
from parfastaai_amd import syn
from parfastaai_amd.datastruct import ParFAAIData
from parfastaai_amd.impl import ParFAAIImpl

pytestmark = pytest.mark.gpu


def test_exact_division(engine):
    # T entries are < 2^16 (checked at load): c <= 65535 and c <= d < 2^17,
    # the whole domain, 6.4e9 quotients
    assert engine.debug_div_check(65535, (1 << 17) - 1) == 0


@pytest.fixture(scope="module")
def syn_problem():
    g = syn.generate(300, 24, clade_size=10)
    ds = ParFAAIData.from_split(g["Lp"], g["F_prot"], g["F_genome"], g["T"]).with_genome_major(g["G_off"], g["G_tet"])
    ref = O.Problem(ds.problem()).ref_run()
    return ds, ref


@pytest.mark.parametrize("variant", ["pl", "v2", "pl512", "fused", "worklist"])
def test_row_kernel_variants(engine, syn_problem, variant):
    ds, ref = syn_problem
    os.environ["PFAAI_ROWS_KERNEL"] = variant
    try:
        impl = ParFAAIImpl(ds, engine=engine)
        impl.run()
    finally:
        os.environ.pop("PFAAI_ROWS_KERNEL", None)
    jac = impl.getJAC()
    assert impl.n_events() == ref["n_events"]
    assert np.array_equal(jac["N"], ref["N"]) and np.array_equal(jac["S"], ref["S"])
    assert np.array_equal(impl.getAJI(), ref["AJI"])
