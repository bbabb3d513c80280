"""The octant (eighth-shell) cluster-pair list (cf_kernels_es.hip: k_es_build,
k_pairs_es): a block per cell owns the 8 cells of its octant, evaluates the octant's 14 cell pairs
(the self pair and 13 pairs with the others) and sums both sides of every pair in 64-bit fixed
point; each atom's sums are added from the 8 octants that hold it.  It must evaluate exactly the
reference's pair set (RCK:559-593): checked against the per-atom half list (pair_list
"atom_half"), the full two-sided list (pair_list "full"), the 18-cell cluster list and the oracle.

Tolerances (written here): against the other lists forces <= 2e-12 max|F| + 1e-9 kJ/mol/nm (the
same pairs; both sides in 2^-34 fixed point, the i side summed per row in another order: ~1e-12 of
|F| ~ 1e3), dE/dq <= 1e-10 relative, direct energy <= 1e-11 relative; against the oracle forces
<= 1e-8 (exact k-space) or 1e-6 (grid k-space) and energy <= 1e-9 of sum |terms|."""
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


def _kernel(system, force, pair_list="octant", algo=0, skin=0.0, precision="double", cap=0):
    k = HipCalcCoulForceKernel(kspace_algo=algo, precision=precision, pair_list=pair_list,
                               list_capacity=cap).initialize(system, force)
    if skin:
        k.set_neighbor_skin(skin)
    return k


def _eval(k, pos, box):
    e, f = k.execute_host(pos, box)
    return e, f, k.dedq(), k.energy_terms()


def _shuffled(nw, seed=2, **kw):
    system, force, pos, box = ts.water_box(nw, **kw)
    perm = np.random.default_rng(seed).permutation(nw)
    return system, force, pos.reshape(nw, 3, 3)[perm].reshape(-1, 3), box


def _close(a, b):
    (fa, da, ta), (fb, db, tb) = a, b
    assert np.abs(fa - fb).max() <= 2e-12 * np.abs(fb).max() + 1e-9, np.abs(fa - fb).max()
    assert np.abs(da - db).max() <= 1e-10 * np.abs(db).max(), np.abs(da - db).max()
    assert abs(ta[2] - tb[2]) <= 1e-11 * abs(tb[2]) + 1e-9, (ta[2], tb[2])


@pytest.mark.parametrize("nw,algo,shuffle", [(4000, 0, False), (7000, 2, False), (4000, 0, True)])
def test_octant_list_matches_other_lists_and_oracle(nw, algo, shuffle):
    mk = _shuffled if shuffle else ts.water_box
    system, force, pos, box = mk(nw, cutoff=1.0, ewald_tol=1e-4, every_bond_angle=5)
    k = _kernel(system, force, "octant", algo)
    eo, fo, do, to = _eval(k, pos, box)
    assert k.pair_list() == "octant"
    assert k.fallback_stats()[0] == 0
    for pl in ("atom_half", "full", "cluster"):
        _, f, d, t = _eval(_kernel(system, force, pl, algo), pos, box)
        _close((fo, do, to), (f, d, t))
    ref = Oracle(force, box).execute(pos, box)
    assert np.abs(fo - ref["forces"]).max() <= (1e-8 if algo == 0 else 1e-6)
    assert abs(eo - ref["energy"]) <= 1e-9 * np.abs(ref["terms"]).sum() + 1e-8


def test_octant_list_odd_cells_and_exclusions():
    # partial clusters, molecules straddling cell faces, sparse cells; rc 0.9
    system, force, pos, box = ts.water_box(2345, cutoff=0.9, ewald_tol=1e-4, every_bond_angle=3)
    k = _kernel(system, force)
    e, f, d, t = _eval(k, pos, box)
    ref = Oracle(force, box).execute(pos, box)
    assert np.abs(f - ref["forces"]).max() <= 1e-8
    assert np.abs(d - ref["dedq"]).max() <= 1e-9 * np.abs(ref["dedq"]).max()
    assert abs(e - ref["energy"]) <= 1e-9 * np.abs(ref["terms"]).sum() + 1e-8
    assert k.fallback_stats()[0] == 0


def test_octant_list_energy_only_and_forces_only_flags():
    # the pair energy is returned per block through the fixed-order energy sum with or without
    # forces (RCK:592: real-space energy regardless of includeEnergy)
    system, force, pos, box = ts.water_box(4000, cutoff=1.0, ewald_tol=1e-4, every_bond_angle=5)
    k = _kernel(system, force)
    ref = _kernel(system, force, "full")
    for fl in (True, False):
        e, f = k.execute_host(pos, box, includeForces=fl)
        er, fr = ref.execute_host(pos, box, includeForces=fl)
        assert abs(e - er) <= 1e-12 * abs(er) + 1e-9


def test_octant_list_trajectory_with_skin_matches_rebuilt_list():
    system, force, pos, box = _shuffled(4000, cutoff=1.0, ewald_tol=1e-4)
    k = _kernel(system, force, skin=0.15)
    ref = _kernel(system, force, "atom_half")
    rng = np.random.default_rng(7)
    x = pos.copy()
    for _ in range(8):
        e, f = k.execute_host(x, box)
        er, fr = ref.execute_host(x, box)
        assert np.abs(f - fr).max() <= 2e-12 * np.abs(fr).max() + 1e-9
        assert abs(e - er) <= 1e-11 * abs(er) + 1e-8
        x = x + np.array([0.03, 0.015, 0.0075]) + rng.normal(scale=0.003, size=x.shape)
    builds, evals = k.neighbor_stats()
    assert evals == 8 and 1 < builds < evals, (builds, evals)
    assert k.fallback_stats()[0] == 0


def test_octant_list_bitwise_reproducible_with_skin():
    # integer window sums of per-row i-side totals: the bits do not depend on which wave took
    # which row, nor on the block schedule
    system, force, pos, box = ts.water_box(4000, cutoff=1.0, ewald_tol=1e-3)
    outs = []
    for _ in range(2):
        k = _kernel(system, force, skin=0.1)
        rng = np.random.default_rng(5)
        x = pos.copy()
        run = []
        for _ in range(3):
            run.append(k.execute_host(x, box))
            x = x + rng.normal(scale=0.003, size=x.shape)
        outs.append(run)
        k.destroy()
    for (e1, f1), (e2, f2) in zip(*outs):
        assert e1 == e2 and np.array_equal(f1, f2)


def test_octant_list_overflow_falls_back_on_every_kept_list():
    # a row capacity of 8 entries (cf_options.list_capacity) overflows every long row at build:
    # every evaluation that keeps the list takes the fp64 rescan, with the reference's answer
    system, force, pos, box = ts.water_box(4000, cutoff=1.0, ewald_tol=1e-4)
    k = _kernel(system, force, skin=0.1, cap=8)
    ref = _kernel(system, force, "full")
    rng = np.random.default_rng(11)
    x = pos.copy()
    for step in range(4):
        e, f = k.execute_host(x, box)
        ef, ff = ref.execute_host(x, box)
        assert np.abs(f - ff).max() <= 1e-8, (step, np.abs(f - ff).max())
        assert abs(e - ef) <= 1e-12 * abs(ef) + 1e-9
        x = x + rng.normal(scale=0.002, size=x.shape)
    fb = k.fallback_stats()
    assert fb[0] == 4 and fb[2] & 2, fb
    builds, evals = k.neighbor_stats()
    assert evals == 4 and builds < evals


def test_octant_list_fixed_point_range_fallback():
    system, force, pos, box = ts.water_box(4000, cutoff=1.0, ewald_tol=1e-4)
    p = pos.copy()
    p[3:6] = p[0:3] + np.array([0.02, 0.0, 0.0])
    k = _kernel(system, force)
    e, f = k.execute_host(p, box)
    ref = Oracle(force, box).execute(p, box)
    assert np.abs(f - ref["forces"]).max() <= 1e-8 * max(1.0, np.abs(ref["forces"]).max() / 1e3)
    assert abs(e - ref["energy"]) <= 1e-9 * np.abs(ref["terms"]).sum() + 1e-8
    assert k.fallback_stats()[2] & 4


@pytest.mark.parametrize("shear", [(0.3, -0.25, 0.2), (-0.5, 0.5, -0.5)])
def test_octant_list_triclinic_box(shear):
    # reduced triclinic boxes (cells in fractional coordinates): each octant position's lattice
    # translation gives the reference's c, b, a minimum image for the pairs within rc
    system, force, pos, box = ts.triclinic_water_box(4000, cutoff=0.7, ewald_tol=1e-4, shear=shear)
    k = _kernel(system, force)
    e, f, d, t = _eval(k, pos, box)
    assert k.pair_list() == "octant"
    assert k.fallback_stats() == (0, 0, 0), k.fallback_stats()
    ref = Oracle(force, box).execute(pos, box)
    assert np.abs(f - ref["forces"]).max() <= 1e-8
    assert abs(e - ref["energy"]) <= 1e-9 * np.abs(ref["terms"]).sum() + 1e-8


def test_octant_list_mixed_precision():
    # the fp32 pair term on the octant list against the fp32 full list and the fp64 octant list
    system, force, pos, box = ts.water_box(4000, cutoff=1.0, ewald_tol=1e-4, every_bond_angle=5)
    em, fm, dm, tm = _eval(_kernel(system, force, "octant", precision="mixed"), pos, box)
    ef, ff, df, tf = _eval(_kernel(system, force, "full", precision="mixed"), pos, box)
    ed, fd, dd, td = _eval(_kernel(system, force, "octant"), pos, box)
    rms = lambda a, b: np.sqrt(((a - b) ** 2).sum(1).mean() / (b ** 2).sum(1).mean())
    assert rms(fm, ff) <= 1e-5 and np.abs(fm - ff).max() <= 0.05
    assert rms(fm, fd) <= 1e-5 and np.abs(fm - fd).max() <= 0.05
    assert np.abs(dm - dd).max() <= 1e-5 * np.abs(dd).max()
    assert abs(em - ed) <= 1e-9 * np.abs(td).sum()
