"""The half neighbour list (k_pairs_half, window sums in k_excl): every pair
evaluated once (kept by the atom of the lower x cell, or within one x cell by the smaller x),
the partner's share summed in 64-bit fixed point.  Used on one rank in fp64
when the box has >= 4 cells per axis; cf_options.pair_list = CF_PAIR_LIST_FULL selects
the full two-sided list for comparison.

Tolerances (written here): against the oracle forces <= 1e-8 kJ/mol/nm, energy <= 1e-9 |E| +
1e-8; half vs full list forces <= 2e-12 max|F| + 1e-9 (the fixed point rounds each j-side term to
2^-34; the i-side sums run in another order).
The fallbacks -- an overflowed list, a j-side term too large for the fixed point -- hand the
evaluation to the fp64 cell rescan, which must give the same answer.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from oracle import Oracle  # noqa: E402
from openmmcoul import HipCalcCoulForceKernel  # noqa: E402
from openmmcoul import testsystems as ts  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _kernel(system, force, half, algo=0, skin=0.0, precision="double", cluster=True, cap=0):
    """half: the half list (the cluster-pair form unless cluster=False: the per-atom half list);
    else the full two-sided list (cf_options.pair_list); cap: a list capacity that overflows
    (cf_options.list_capacity: cluster-pair entries per i-cluster, per-atom entries per sub-list)."""
    pl = ("cluster" if cluster else "atom_half") if half else "full"
    k = HipCalcCoulForceKernel(kspace_algo=algo, precision=precision, pair_list=pl,
                               list_capacity=cap).initialize(system, force)
    if skin:
        k.set_neighbor_skin(skin)
    return k


def _eval(k, pos, box):
    e, f = k.execute_host(pos, box)   # the first evaluation builds the cells (and picks the list kind)
    return e, f, k.dedq(), k.energy_terms()


@pytest.mark.parametrize("cluster", [False, True], ids=["atom_list", "cluster_list"])
@pytest.mark.parametrize("nw,algo", [(4000, 0), (7000, 2)])
def test_half_list_matches_full_list_and_oracle(nw, algo, cluster):
    system, force, pos, box = ts.water_box(nw, cutoff=1.0, ewald_tol=1e-4, every_bond_angle=5)
    eh, fh, dh, th = _eval(_kernel(system, force, True, algo, cluster=cluster), pos, box)
    ef, ff, df, tf = _eval(_kernel(system, force, False, algo), pos, box)
    # (the per-atom half list measured 2.0e-9 at 4000 waters, |F| ~ 1e3: the same bar for both)
    assert np.abs(fh - ff).max() <= 2e-12 * np.abs(ff).max() + 1e-9, np.abs(fh - ff).max()
    assert np.abs(dh - df).max() <= 1e-10 * np.abs(df).max()
    assert abs(th[2] - tf[2]) <= 1e-11 * abs(tf[2]) + 1e-9
    ref = Oracle(force, box).execute(pos, box)
    tol = 1e-8 if algo == 0 else 2.5e-6
    assert np.abs(fh - ref["forces"]).max() <= tol
    assert abs(eh - ref["energy"]) <= 1e-9 * np.abs(ref["terms"]).sum() + 1e-8


def test_half_list_bitwise_reproducible_with_skin():
    system, force, pos, box = ts.water_box(4000, cutoff=1.0, ewald_tol=1e-3)
    k = _kernel(system, force, True, skin=0.1)
    rng = np.random.default_rng(5)
    x = pos.copy()
    outs = []
    for _ in range(3):
        outs.append(k.execute_host(x, box))
        x = x + rng.normal(scale=0.003, size=x.shape)
    k2 = _kernel(system, force, True, skin=0.1)
    x = pos.copy()
    rng = np.random.default_rng(5)
    for e, f in outs:
        e2, f2 = k2.execute_host(x, box)
        assert e2 == e and np.array_equal(f2, f)
        x = x + rng.normal(scale=0.003, size=x.shape)


def test_half_list_fallback_on_list_overflow():
    # a list capacity (cf_options.list_capacity) far below the density: every list overflows, the
    # half-list evaluation is flagged and k_excl rescans every atom in fp64.  (Before round 6 a
    # default box 2.5x wider did this; the capacity now also follows the current box's density.)
    system, force, pos, box = ts.water_box(4000, cutoff=1.0, ewald_tol=1e-4)
    big = [[2.5 * box[i][j] for j in range(3)] for i in range(3)]
    system.setDefaultPeriodicBoxVectors(*big)
    # (the checker is the full-list kernel on the same default box: the oracle's k-sum over the
    # 16x larger k-vector set of the wide default box takes minutes on one host core)
    k = _kernel(system, force, True, cluster=False, cap=24)
    ef, ff = _kernel(system, force, False).execute_host(pos, box)
    for _ in range(2):
        e, f = k.execute_host(pos, box)
        assert np.abs(f - ff).max() <= 2e-12 * np.abs(ff).max() + 1e-9
        assert abs(e - ef) <= 1e-12 * abs(ef) + 1e-9


def test_half_list_fallback_on_fixed_point_range():
    # two waters 0.02 nm apart: a pair force of ~1e5 kJ/mol/nm exceeds the fixed point's 2^16
    system, force, pos, box = ts.water_box(4000, cutoff=1.0, ewald_tol=1e-4)
    p = pos.copy()
    p[3:6] = p[0:3] + np.array([0.02, 0.0, 0.0])
    k = _kernel(system, force, True)
    e, f = k.execute_host(p, box)
    ref = Oracle(force, box).execute(p, box)
    assert np.abs(f - ref["forces"]).max() <= 1e-8 * max(1.0, np.abs(ref["forces"]).max() / 1e3)
    assert abs(e - ref["energy"]) <= 1e-9 * np.abs(ref["terms"]).sum() + 1e-8


def _sparse_gas():
    # 300 waters at 1/8 of water density, rc 0.7 + skin 0.1: 5 cells per axis with ~7 atoms per
    # cell, so 64 consecutive cell-sorted atoms span more cells than the box has along z -- the
    # wave builder's block frame does not fit and those rows cannot use the half list
    return ts.water_box(300, cutoff=0.7, ewald_tol=1e-4, density=ts.WATER_DENSITY / 8, every_bond_angle=3)


def _dense_overflow():
    # a default box 2.5x larger (16x lower density); since round 6 the automatic capacity follows the
    # current box too, so the overflow is forced with cf_options.list_capacity
    system, force, pos, box = ts.water_box(4000, cutoff=1.0, ewald_tol=1e-4)
    system.setDefaultPeriodicBoxVectors(*[[2.5 * box[i][j] for j in range(3)] for i in range(3)])
    return system, force, pos, box


@pytest.mark.parametrize("make,cluster,cap", [(_sparse_gas, False, 0), (_dense_overflow, False, 24), (_dense_overflow, True, 24)],
                         ids=["block_frame_misfit", "list_overflow", "cluster_list_overflow"])
def test_half_list_fallbacks_persist_over_kept_lists(make, cluster, cap):
    """A fallback raised when the list is BUILT (rows the builder could not encode, overflowed
    rows) must hold on every later evaluation that keeps that list under a skin: each step is
    compared with the full list rebuilt from scratch (pair_list "full", skin 0) on the same positions.
    (The cluster-pair list has no block frame: the sparse gas runs it without a fallback, checked
    against the oracle below.)"""
    system, force, pos, box = make()
    k = _kernel(system, force, True, skin=0.1, cluster=cluster, cap=cap)
    ref = _kernel(system, force, False)
    rng = np.random.default_rng(11)
    x = pos.copy()
    for step in range(5):
        e, f = k.execute_host(x, box)
        ef, ff = ref.execute_host(x, box)
        # (the rescan of a kept rc + skin list walks cells of another size than the reference's
        # full list: the same pairs in another summation order, ~2e-12 of |F|)
        assert np.abs(f - ff).max() <= 1e-8, (step, np.abs(f - ff).max())
        assert abs(e - ef) <= 1e-12 * abs(ef) + 1e-9, (step, e, ef)
        x = x + rng.normal(scale=0.002, size=x.shape)
    fb = k.fallback_stats()
    assert fb[0] == 5 and fb[2] & 2, fb   # every evaluation took the fp64 rescan (list reason)
    builds, evals = k.neighbor_stats()
    assert evals == 5 and builds < evals   # the later steps did keep the list


def test_half_list_sparse_gas_matches_oracle_with_skin():
    system, force, pos, box = _sparse_gas()
    k = _kernel(system, force, True, skin=0.1)
    orc = Oracle(force, box)
    x = pos.copy()
    rng = np.random.default_rng(3)
    for _ in range(3):
        e, f = k.execute_host(x, box)
        r = orc.execute(x, box)
        assert np.abs(f - r["forces"]).max() <= 1e-8
        assert abs(e - r["energy"]) <= 1e-9 * np.abs(r["terms"]).sum() + 1e-8
        x = x + rng.normal(scale=0.002, size=x.shape)


@pytest.mark.parametrize("cluster", [False, True], ids=["atom_list", "cluster_list"])
def test_half_list_mixed_precision(cluster):
    # the fp32 half-list kernel (the per-atom list, and the cluster-pair list -- the mixed default since
    # round 5) against the fp32 full list and the fp64 half list (same k-space)
    system, force, pos, box = ts.water_box(4000, cutoff=1.0, ewald_tol=1e-4, every_bond_angle=5)
    em, fm, dm, tm = _eval(_kernel(system, force, True, 0, precision="mixed", cluster=cluster), pos, box)
    ef, ff, df, tf = _eval(_kernel(system, force, False, 0, precision="mixed"), pos, box)
    ed, fd, dd, td = _eval(_kernel(system, force, True, 0), pos, box)
    rms = lambda a, b: np.sqrt(((a - b) ** 2).sum(1).mean() / (b ** 2).sum(1).mean())
    assert rms(fm, ff) <= 1e-5 and np.abs(fm - ff).max() <= 0.05
    assert rms(fm, fd) <= 1e-5 and np.abs(fm - fd).max() <= 0.05
    assert np.abs(dm - dd).max() <= 1e-5 * np.abs(dd).max()
    assert abs(em - ed) <= 1e-9 * np.abs(td).sum()
