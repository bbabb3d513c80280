"""The cluster-pair half list (cf_kernels_cluster.hip: k_cl_build, k_pairs_cq):
clusters of <= 4 cell-sorted atoms, one list entry per cluster pair with a 16-bit pair mask
(exclusions, the self pair's triangle, partial clusters), an fp32 cutoff prefilter whose hits are
compacted into per-atom queues, and the fp64 pair term with the exact r <= rc test.  It must
evaluate exactly the reference's pair set (RCK:559-593): checked against the per-atom half list
(pair_list "atom_half"), the full two-sided list (pair_list "full") and the oracle.

Tolerances (written here): cluster vs per-atom half list forces <= 2e-12 max|F| + 1e-9 kJ/mol/nm
(the same pairs; the partner side in 2^-34 fixed point, the i side summed in another order:
~1e-12 of |F| ~ 1e3), dE/dq <= 1e-10 relative,
direct energy <= 1e-11 relative; against the oracle forces <= 1e-8 (exact k-space) and energy
<= 1e-9 of sum |terms|."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from oracle import Oracle  # noqa: E402
from openmmcoul import testsystems as ts  # noqa: E402
from tests.test_gpu_half import _eval, _kernel  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _shuffled(nw, seed=2, **kw):
    """A water box whose molecules are numbered in random order: a cell sorted by atom index
    would give clusters spread over the whole cell; the z-column sort keeps them compact."""
    system, force, pos, box = ts.water_box(nw, **kw)
    perm = np.random.default_rng(seed).permutation(nw)
    p3 = pos.reshape(nw, 3, 3)[perm].reshape(-1, 3)
    return system, force, p3, box


@pytest.mark.parametrize("nw,algo,shuffle", [(4000, 0, False), (7000, 2, False), (4000, 0, True)])
def test_cluster_list_matches_atom_lists_and_oracle(nw, algo, shuffle):
    mk = _shuffled if shuffle else ts.water_box
    system, force, pos, box = mk(nw, cutoff=1.0, ewald_tol=1e-4, every_bond_angle=5)
    ec, fc, dc, tc = _eval(_kernel(system, force, True, algo), pos, box)
    ea, fa, da, ta = _eval(_kernel(system, force, True, algo, cluster=False), pos, box)
    ef, ff, df, tf = _eval(_kernel(system, force, False, algo), pos, box)
    for f, d, t in ((fa, da, ta), (ff, df, tf)):
        assert np.abs(fc - f).max() <= 2e-12 * np.abs(f).max() + 1e-9, np.abs(fc - f).max()
        assert np.abs(dc - d).max() <= 1e-10 * np.abs(d).max()
        assert abs(tc[2] - t[2]) <= 1e-11 * abs(t[2]) + 1e-9
    ref = Oracle(force, box).execute(pos, box)
    assert np.abs(fc - ref["forces"]).max() <= (1e-8 if algo == 0 else 2.5e-6)
    assert abs(ec - ref["energy"]) <= 1e-9 * np.abs(ref["terms"]).sum() + 1e-8


def test_cluster_list_trajectory_with_skin_matches_rebuilt_list():
    # kept lists over an MD-like trajectory (atoms drift, the list is kept, then rebuilt): every
    # step equal to the per-atom half list rebuilt from scratch on the same positions
    system, force, pos, box = _shuffled(4000, cutoff=1.0, ewald_tol=1e-4)
    # (a drift of the whole box plus small noise: noise large enough to force rebuilds by itself
    # would push atoms of different molecules into each other, past the fixed point's range -- a
    # fallback, tested in test_gpu_half.py)
    k = _kernel(system, force, True, skin=0.15)
    ref = _kernel(system, force, True, cluster=False)
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
    fb = k.fallback_stats()
    assert fb[0] == 0, fb


def test_cluster_list_odd_cells_and_exclusions():
    # atoms per cell not a multiple of 4 (partial clusters), exclusions between clusters of
    # different cells (molecules straddling cell faces), an atom count that leaves a few cells
    # with very few atoms
    system, force, pos, box = ts.water_box(2345, cutoff=0.9, ewald_tol=1e-4, every_bond_angle=3)
    ec, fc, dc, tc = _eval(_kernel(system, force, True), pos, box)
    ref = Oracle(force, box).execute(pos, box)
    assert np.abs(fc - ref["forces"]).max() <= 1e-8
    assert np.abs(dc - ref["dedq"]).max() <= 1e-9 * np.abs(ref["dedq"]).max()
    assert abs(ec - ref["energy"]) <= 1e-9 * np.abs(ref["terms"]).sum() + 1e-8


@pytest.mark.parametrize("world", [2, 4])
def test_cluster_list_on_several_ranks_opt_in(world):
    """The ownership-filtered cluster-pair list on several ranks (pair_list "cluster", opt-in: slower
    than the full per-atom list at W = 4/8): `world` handles on this GPU, the k-space
    buffers summed by hand, against one rank -- each rank evaluates the cluster pairs that touch
    its atoms, k_excl gathers its atoms' partner-side sums."""
    from openmmcoul import HipCalcCoulForceKernel
    from tests.test_gpu_configs import _decomposed
    system, force, pos, box = ts.water_box(4000, cutoff=1.0, ewald_tol=1e-4, every_bond_angle=5)
    k = HipCalcCoulForceKernel(kspace_algo=2).initialize(system, force)
    e1, f1 = k.execute_host(pos, box)
    d1, t1 = k.dedq(), k.energy_terms()
    k.destroy()
    ew, fw, dw, _ = _decomposed(system, force, pos, box, world, 2, pair_list="cluster")
    assert abs(ew - e1) <= 1e-11 * np.abs(t1).sum()
    assert np.abs(fw - f1).max() <= 2e-12 * np.abs(f1).max() + 1e-9
    assert np.abs(dw - d1).max() <= 2e-12 * np.abs(d1).max() + 1e-9

