"""F construction on the device (pfaai_build_f; SURVEY §8b, north_star
"E/F-array construction (device radix sort of (tetramer, genome) tuples)"):
from the `<p>_genomes` triples it must reproduce the reference's own F / Lc /
T fixtures bit for bit, and the synthetic generator's F (the reference
loader's order, tools/syn_gen.c) at scale."""
import numpy as np
import pytest

from parfastaai_amd import _capi, syn
from parfastaai_amd import formats as fm
from helpers import gpath

pytestmark = pytest.mark.gpu


def _triples_from_G(g):
    """(genome, protein)-major walk of the genome-major lists."""
    G, P = g["T"].shape[1], g["T"].shape[0]
    lens = np.diff(g["G_off"])
    gp = np.repeat(np.arange(G * P, dtype=np.int64), lens)
    return (gp % P).astype(np.int32), (gp // P).astype(np.int32), g["G_tet"]


@pytest.mark.parametrize("name", ["xanthodb", "xdb_subset1", "xdb_subset2"])
def test_build_f_reproduces_reference_fixtures(engine, name):
    F = fm.read_f_array(gpath(f"{name}_f_array.bin"))      # (n, 2) [protein, genome], ref order
    Lc = fm.read_vec_i32(gpath(f"{name}_lc_array.bin"))
    T = fm.read_matrix_i32(gpath(f"{name}_t_matrix.bin"))
    t = np.repeat(np.arange(160000, dtype=np.int32), Lc)
    # the blobs' order: protein-major, genome, then tetramer
    o = np.lexsort((t, F[:, 1], F[:, 0]))
    out = engine.build_f(F[o, 0], F[o, 1], t[o], T.shape[0], T.shape[1])
    assert np.array_equal(out["Lc"], Lc)
    assert np.array_equal(out["F_prot"], F[:, 0]) and np.array_equal(out["F_genome"], F[:, 1])
    assert np.array_equal(out["T"], T)


@pytest.mark.parametrize("n,P", [(400, 30), (3000, 100)])
def test_build_f_equals_loader_order_syn(engine, n, P):
    g = syn.generate(n, P)
    p, gg, t = _triples_from_G(g)
    out = engine.build_f(p, gg, t, P, n)
    assert np.array_equal(out["Lp"], g["Lp"])
    assert np.array_equal(out["F_prot"], g["F_prot"]) and np.array_equal(out["F_genome"], g["F_genome"])
    assert np.array_equal(out["T"], g["T"])


def test_build_f_rejects_unordered_genomes_and_empty(engine):
    with pytest.raises(_capi.PfaaiError):
        engine.build_f([0, 0], [5, 3], [7, 7], 1, 10)
    out = engine.build_f([], [], [], 3, 4)
    assert out["Lp"][-1] == 0 and out["T"].sum() == 0
