"""The load-time transposition sort (pfaai_sort.hpp):
F <-> G on the device by a stable LSD radix sort of 64-bit records in one,
two or three passes of <= 11-bit digits.

  * both orientations given: one sort of F by (genome, protein) must accept
    exactly the caller's G -- a swapped tetramer or a shifted list bound is
    refused -- and its G_pos drives the benchmark kernel (WK 3) to the
    oracle's results;
  * F only: G_off from T, verified against the sorted keys; an inconsistent
    T (a count that is not the list length) falls back to the general radix
    sort, and the results still follow the reference's formula with that T;
  * G only: F by the protein-major enumeration sorted by tetramer (no
    G_pos: Lp from the sorted tetramers), long lists included;
  * key widths that take one, two and three passes, and record counts that
    are not a multiple of the 8192-record tile -- bit-exact against the
    oracle and against each other.
"""
import numpy as np
import pytest

import oracle as O
from parfastaai_amd import _capi, syn
from parfastaai_amd.datastruct import ParFAAIData

pytestmark = pytest.mark.gpu


def _problem(n, P, **kw):
    g = syn.generate(n, P, **kw)
    return ParFAAIData.from_split(g["Lp"], g["F_prot"], g["F_genome"], g["T"]).with_genome_major(
        g["G_off"], g["G_tet"]).problem()


def _strip(pb, drop):
    return {k: v for k, v in pb.items() if k not in drop}


def _check_rows(engine, pb, rows, res):
    aji, S, N = res
    pr = O.Problem(pb)
    n = pb["n_ids"]
    for a in rows:
        So, No, _ = pr.dense_rows(a, a + 1)
        b = np.arange(a + 1, n)
        k = n * a + b - (a + 2) * (a + 1) // 2
        assert np.array_equal(N[k], No[0, b]) and np.array_equal(S[k], So[0, b]), a


@pytest.mark.parametrize("n,P,kw,passes", [
    (20, 40, dict(clade_size=5), 1),          # g * P + p < 2^11: one pass
    (701, 37, dict(clade_size=9), 2),          # 15-bit keys, |F| not a multiple of the tile
    (3000, 1500, dict(clade_size=10, has=0.02), 3),  # 23-bit keys: three 8-bit passes
])
def test_orientations_agree_across_pass_counts(engine, n, P, kw, passes):
    pb = _problem(n, P, **kw)
    assert (n * P).bit_length() <= 11 * passes
    results = {}
    for drop, want in (((), "g_checked"), (("G_off", "G_tet"), "g_from_f"), (("Lp", "F_prot", "F_genome"), "f_from_g")):
        engine.load(**_strip(pb, drop))
        assert engine.load_info() == want, drop
        results[want] = engine.compute(0)
        assert engine.stats()["n_events"] == O.Problem(pb).count_e()
    for k in ("g_from_f", "f_from_g"):
        for a, b in zip(results[k], results["g_checked"]):
            assert np.array_equal(a, b), k
    _check_rows(engine, pb, (0, 1, n // 2, n - 2), results["g_checked"])


def test_both_given_refuses_a_g_that_is_not_the_transpose(engine):
    pb = _problem(300, 24, clade_size=10)
    G_off, G_tet = pb["G_off"], pb["G_tet"]
    # (1) one tetramer of one list replaced by another id (still an ascending set)
    bad = G_tet.copy()
    k0, k1 = int(G_off[5 * 24 + 3]), int(G_off[5 * 24 + 4])
    lst = set(bad[k0:k1].tolist())
    new = next(t for t in range(159999, 0, -1) if t not in lst)
    bad[k0:k1] = np.sort(np.r_[bad[k0:k1 - 1], new])
    with pytest.raises(_capi.PfaaiError):
        engine.load(**dict(pb, G_tet=bad))
    # (2) one entry moved from a list to its neighbour: same |G|, same G_tet, shifted bound
    off = G_off.copy()
    j = next(j for j in range(1000, len(off) - 1) if off[j + 1] - off[j] > 1 and off[j] - off[j - 1] > 1)
    off[j] += 1
    with pytest.raises(_capi.PfaaiError):
        engine.load(**dict(pb, G_off=off))
    engine.load(**pb)  # the real transpose is accepted
    assert engine.load_info() == "g_checked"


def _swap(G_off, G_tet, la, lb):
    """G_tet with one tetramer of list la exchanged for one of list lb (each
    absent from the other list): same G_off, every list still ascending --
    the memberships {(la, t1), (lb, t2)} become {(la, t2), (lb, t1)}, an XOR
    parallelogram of the check's codes."""
    A = G_tet[G_off[la]:G_off[la + 1]].tolist()
    B = G_tet[G_off[lb]:G_off[lb + 1]].tolist()
    t1 = next(t for t in A if t not in set(B))
    t2 = next(t for t in B if t not in set(A))
    out = G_tet.copy()
    out[G_off[la]:G_off[la + 1]] = sorted([t for t in A if t != t1] + [t2])
    out[G_off[lb]:G_off[lb + 1]] = sorted([t for t in B if t != t2] + [t1])
    return out


@pytest.mark.parametrize("rows", [None, (40, 90)])
def test_both_given_refuses_swapped_tetramers(engine, rows):
    """One tetramer exchanged between two genomes' lists of one protein, and
    between two proteins' lists of one genome: |G|, G_off and every list
    length are unchanged, so only the membership sums can see it -- refused
    by a full load and by a rank load whose block holds the lists."""
    P = 24
    pb = _problem(300, P, clade_size=10)
    G_off, G_tet = pb["G_off"], pb["G_tet"]
    load = (lambda **kw: engine.load(**kw)) if rows is None else (lambda **kw: engine.load(rows=rows, **kw))
    for la, lb in ((50 * P + 3, 61 * P + 3), (70 * P + 2, 70 * P + 9)):
        with pytest.raises(_capi.PfaaiError):
            load(**dict(pb, G_tet=_swap(G_off, G_tet, la, lb)))
    load(**pb)
    assert engine.load_info() == "g_checked"


def test_both_given_without_gpos_checks_membership_without_a_sort(engine):
    """Where the row kernels use no G_pos (-q subsets; all-vs-all past 20 480
    genomes) the both-given load runs only the membership sums (k_hash_f over
    F, k_gend over G) and no sort: a G with one tetramer replaced is still
    refused, and the real transpose gives the oracle's S / N."""
    from parfastaai_amd.datastruct import ParFAAIQSubData

    g = syn.generate(400, 20, clade_size=10)
    q = [g["genome_set"][i] for i in range(2, 400, 9)]
    pb = ParFAAIQSubData.from_split(g["Lp"], g["F_prot"], g["F_genome"], g["T"], g["genome_set"], q
                                    ).with_genome_major(g["G_off"], g["G_tet"]).problem()
    G_off, G_tet = pb["G_off"], pb["G_tet"]
    bad = G_tet.copy()
    k0, k1 = int(G_off[7 * 20 + 2]), int(G_off[7 * 20 + 3])
    lst = set(bad[k0:k1].tolist())
    new = next(t for t in range(159999, 0, -1) if t not in lst)
    bad[k0:k1] = np.sort(np.r_[bad[k0:k1 - 1], new])
    with pytest.raises(_capi.PfaaiError):
        engine.load(**dict(pb, G_tet=bad))
    # a membership moved to another genome's list of the same protein: same
    # |G|, every list still ascending, the triple (g, p, t) changed
    g_a, g_b, p = 3, 4, 5
    la = G_tet[G_off[g_a * 20 + p]:G_off[g_a * 20 + p + 1]]
    lb = G_tet[G_off[g_b * 20 + p]:G_off[g_b * 20 + p + 1]]
    t = next((x for x in la.tolist() if x not in set(lb.tolist())), None)
    if t is not None and len(la) > 1:
        lists = [G_tet[G_off[k]:G_off[k + 1]].tolist() for k in range(len(G_off) - 1)]
        lists[g_a * 20 + p].remove(t)
        lists[g_b * 20 + p] = sorted(lists[g_b * 20 + p] + [t])
        off2 = np.r_[0, np.cumsum([len(x) for x in lists])].astype(G_off.dtype)
        tet2 = np.concatenate([np.asarray(x, dtype=G_tet.dtype) for x in lists])
        with pytest.raises(_capi.PfaaiError):
            engine.load(**dict(pb, G_off=off2, G_tet=tet2))
    engine.load(**pb)
    assert engine.load_info() == "g_checked"
    aji, S, N = engine.compute(0)
    want = O.Problem(pb).ref_run()
    assert np.array_equal(S, want["S"]) and np.array_equal(N, want["N"])


def test_f_only_inconsistent_t_takes_the_general_sort(engine):
    """T is an input of the formula (J = c / (T[p][A] + T[p][B] - c)); when it
    is not the list lengths of F, G_off cannot come from it: the general
    radix sort builds G, and S / N follow the reference with that T."""
    pb = _strip(_problem(200, 16, clade_size=8), ("G_off", "G_tet"))
    T = pb["T"].copy()
    T[3, 7] += 2
    pb = dict(pb, T=T)
    engine.load(**pb)
    assert engine.load_info() == "legacy"
    res = engine.compute(0)
    _check_rows(engine, pb, (0, 7, 100, 198), res)


@pytest.mark.parametrize("given", ["both", "g_only"])
def test_g_given_inconsistent_t_takes_the_clamped_walk(engine, given):
    """the WK 3 walk divides without the denominator clamp, which
    is safe only when T is every (genome, protein) list's length (t_exact,
    checked at load).  G handed over (with F, or alone) with one T entry
    larger than its list length: the load must not take the clamp-free
    form -- the run takes the run table + splitters walk -- and S / N follow
    the reference with that T (oracle, bit-exact)."""
    pb = _problem(200, 16, clade_size=8)
    T = pb["T"].copy()
    T[3, 7] += 2
    T[0, 150] += 1
    pb = dict(pb, T=T)
    if given == "g_only":
        pb = _strip(pb, ("Lp", "F_prot", "F_genome"))
    engine.load(**pb)
    res = engine.compute(0)
    assert engine.stats()["walk"] == "splitters", engine.stats()
    full = pb if given == "both" else dict(_problem(200, 16, clade_size=8), T=T)
    _check_rows(engine, full, (0, 3, 7, 100, 150, 198), res)


def test_g_only_long_list(engine):
    """A (genome, protein) list of 9 000 tetramers: the G-only sort's records
    (tetramer | protein | genome) carry no list offset, so it still takes the
    transposition sort; the fused row kernel takes the long list; results
    equal the F + G load and the oracle."""
    rng = np.random.default_rng(5)
    n, P = 30, 3
    sets = {(g, p): np.unique(rng.integers(0, 4000, 60)) for g in range(n) for p in range(P)}
    sets[(4, 1)] = np.arange(0, 18000, 2)
    from helpers import sets_problem
    pb = sets_problem({k: v.tolist() for k, v in sets.items()}, n, P)
    engine.load(**pb)
    ref = engine.compute(0)
    engine.load(**_strip(pb, ("Lp", "F_prot", "F_genome")))
    assert engine.load_info() == "f_from_g"
    got = engine.compute(0)
    assert engine.stats()["rows_kernel"] == "fused"
    for a, b in zip(got, ref):
        assert np.array_equal(a, b)
    _check_rows(engine, pb, (0, 4, 20), ref)
