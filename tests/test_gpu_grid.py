"""GPU parity of the grid reciprocal path (kspace_algo = 2: ES-kernel spreading, pruned
DFT, interpolation) against the oracle restatement of
ReferenceCoulKernels.cpp:513-556 and against the exact fp64-MFMA k-sum.

The grid evaluates the reference's own truncated k-sum (same k-set, weights and current
box); its only error is the ES-kernel quadrature error, set by the kernel width W.
Tolerances (written here; north star: forces within 1e-5 kJ/mol/nm):
  forces   max |dF|         <= 2.5e-6 kJ/mol/nm (default W = 13: 5e-8 on the bench's C3 positions; W = 14 ~1e-8)
  energy   |dE|             <= 1e-9 |E| + 1e-8 kJ/mol
  dE/dq    max |d(dE/dq)|   <= 1e-9 max|dE/dq| + 1e-9
  charges  max |dq|         <= 1e-12 e (untouched by the k-space method)
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from oracle import Oracle  # noqa: E402
from openmmcoul import HipCalcCoulForceKernel, ChargeFluxError, _cabi  # noqa: E402
from openmmcoul import testsystems as ts  # noqa: E402
from openmmcoul.distributed import device_buffer_as_tensor  # noqa: E402

GRID = HipCalcCoulForceKernel.KSPACE_GRID
F_TOL = 2.5e-6   # the grid k-space budget: a quarter of the north star's 1e-5


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _compare(got, ref, f_tol=F_TOL, e_rel=1e-9):
    e, f, q, dq, terms = got
    assert abs(e - ref["energy"]) <= e_rel * abs(ref["energy"]) + 1e-8, (e, ref["energy"])
    if dq is not None:
        assert np.abs(f - ref["forces"]).max() <= f_tol, np.abs(f - ref["forces"]).max()
        scale = np.abs(ref["dedq"]).max()
        assert np.abs(dq - ref["dedq"]).max() <= 1e-9 * scale + 1e-9, np.abs(dq - ref["dedq"]).max()
    assert np.abs(q - ref["charges"]).max() <= 1e-12
    for a, b in zip(terms, ref["terms"]):
        assert abs(a - b) <= e_rel * max(abs(b), 1.0) + 1e-8, (terms, ref["terms"])


def _run(kernel, pos, box, fl=True, en=True):
    e, f = kernel.execute_host(pos, box, fl, en)
    return e, f, kernel.charges(), (kernel.dedq() if fl else None), kernel.energy_terms()


@pytest.mark.parametrize("nw,rc,tol", [(100, 0.6, 1e-5), (400, 0.7, 1e-4)])
def test_grid_small_boxes(nw, rc, tol):
    system, force, pos, box = ts.water_box(nw, cutoff=rc, ewald_tol=tol, every_bond_angle=3)
    k = HipCalcCoulForceKernel(kspace_algo=GRID).initialize(system, force)
    o = Oracle(force, box)
    for fl, en in ((True, True), (True, False), (False, True)):
        _compare(_run(k, pos, box, fl, en), o.execute(pos, box, fl, en))


@pytest.mark.parametrize("width", [12, 14, 16])
def test_grid_c2_parity(width):
    system, force, pos, box = ts.make("C2")
    k = HipCalcCoulForceKernel(kspace_algo=GRID, grid_width=width).initialize(system, force)
    assert k.ewald_params()[1] == (7, 7, 7)
    _compare(_run(k, pos, box), Oracle(force, box).execute(pos, box))


def test_grid_c2_golden_fixture():
    import os
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "c2.npz"))
    system, force, pos, box = ts.make("C2")
    k = HipCalcCoulForceKernel(kspace_algo=GRID).initialize(system, force)
    e, f = k.execute_host(pos, box)
    assert abs(e - float(d["energy"])) <= 1e-9 * abs(float(d["energy"]))
    assert np.abs(f - d["forces"]).max() <= F_TOL


def test_grid_nacl_madelung_atoms_on_grid_points():
    # ions sit exactly on grid points (first taps at the support edge: phi = 0 there)
    system, force, pos, box = ts.nacl_crystal(cells=4, a=0.5, cutoff=1.0, ewald_tol=1e-10)
    k = HipCalcCoulForceKernel(kspace_algo=GRID).initialize(system, force)
    e, f = k.execute_host(pos, box)
    expect = -(len(pos) / 2) * 1.747564594633182 * 138.935456 / 0.25
    assert e == pytest.approx(expect, rel=2e-9)
    assert np.abs(f).max() < F_TOL


def test_grid_moved_box_and_wrapped_positions():
    system, force, pos, box = ts.water_box(400, cutoff=0.7, ewald_tol=1e-4)
    p2 = pos + np.array([3.1, -7.4, 12.0])
    box2 = box * 1.02
    k = HipCalcCoulForceKernel(kspace_algo=GRID).initialize(system, force)
    _compare(_run(k, p2, box2), Oracle(force, box).execute(p2, box2))


def test_grid_noncubic_box():
    system, force, pos, box = ts.water_box(400, cutoff=0.7, ewald_tol=1e-4)
    box2 = box.copy()
    box2[0, 0] *= 1.3
    box2[2, 2] *= 0.95
    system.setDefaultPeriodicBoxVectors(*box2)
    k = HipCalcCoulForceKernel(kspace_algo=GRID).initialize(system, force)
    o = Oracle(force, box2)
    assert k.ewald_params()[1] == o.ewald()[1]
    _compare(_run(k, pos, box2), o.execute(pos, box2))


@pytest.mark.parametrize("nw,rc,tol,min_per_bin", [(1500, 1.5, 1e-3, 128), (800, 1.3, 1e-3, 64)])
def test_grid_dense_bins(nw, rc, tol, min_per_bin):
    # few, crowded 8^3 bins (a short k-sum on a small grid): bins of more than 64 and more
    # than 128 members take k_g_order_taps' LDS and global-memory ranking paths
    system, force, pos, box = ts.water_box(nw, cutoff=rc, ewald_tol=tol, every_bond_angle=3)
    k = HipCalcCoulForceKernel(kspace_algo=GRID).initialize(system, force)
    ng = k.grid_shape()
    per_bin = len(pos) / np.prod([n // 8 for n in ng])
    print("grid", ng, "mean atoms per bin", per_bin)
    assert per_bin > min_per_bin
    _compare(_run(k, pos, box), Oracle(force, box).execute(pos, box))


def test_grid_device_api_deterministic():
    system, force, pos, box = ts.water_box(1500, cutoff=1.0, ewald_tol=1e-4)
    stream = torch.cuda.current_stream().cuda_stream
    k = HipCalcCoulForceKernel(stream=stream, kspace_algo=GRID).initialize(system, force)
    e_h, f_h = k.execute_host(pos, box)
    pt = torch.tensor(pos, dtype=torch.float64, device="cuda")
    outs = []
    for _ in range(2):
        f = torch.zeros_like(pt)
        e = torch.zeros(1, dtype=torch.float64, device="cuda")
        k.execute_device(pt, box, True, True, f, e)
        torch.cuda.synchronize()
        outs.append((e.item(), f.cpu().numpy()))
    assert outs[0][0] == outs[1][0] and np.array_equal(outs[0][1], outs[1][1])  # bitwise reproducible
    assert outs[0][0] == e_h and np.array_equal(outs[0][1], f_h)


@pytest.mark.parametrize("world,shuffled,precision", [(2, False, "double"), (4, False, "double"), (8, False, "double"),
                                                     (4, True, "double"), (4, False, "mixed")])
def test_grid_multi_rank_decomposition_on_one_gpu(world, shuffled, precision):
    # W ranks of an atom decomposition driven on one GPU (the all-reduce done by hand): each
    # rank spreads / transforms only the grid x-planes its atoms reach.  Contiguous ranks of
    # the lattice-ordered box are x-slabs (rank 0's straddles the periodic boundary: its H
    # atoms wrap to x ~ L); shuffled molecules make every rank span the box (full range).
    system, force, pos, box = ts.water_box(2400, cutoff=1.0, ewald_tol=1e-4, every_bond_angle=4)
    if shuffled:   # permute molecule positions within each topology class
        rng = np.random.default_rng(11)
        w = pos.reshape(-1, 3, 3).copy()
        kinds = np.arange(len(w)) % 4 == 3
        for cls in (kinds, ~kinds):
            ids = np.flatnonzero(cls)
            w[ids] = w[rng.permutation(ids)]
        pos = w.reshape(-1, 3)
    stream = torch.cuda.current_stream().cuda_stream
    pt = torch.tensor(pos, dtype=torch.float64, device="cuda")
    single = HipCalcCoulForceKernel(stream=stream, kspace_algo=GRID, precision=precision).initialize(system, force)
    e1, f1 = single.execute_host(pos, box)
    t1 = single.energy_terms()
    ks = [HipCalcCoulForceKernel(stream=stream, rank=r, world_size=world, kspace_algo=GRID,
                                 precision=precision).initialize(system, force)
          for r in range(world)]
    for step in range(2):   # the second evaluation checks that the x-slab state re-arms
        for k in ks:
            k.begin(pt, box, True, True)
        bufs = [device_buffer_as_tensor(*k.kspace_buffer(), "cuda") for k in ks]
        total = sum(bufs[1:], bufs[0].clone())
        for b in bufs:
            b.copy_(total)
        f = torch.zeros_like(pt)
        es = []
        for k in ks:
            e = torch.zeros(1, dtype=torch.float64, device="cuda")
            k.end(f, e)
            es.append(e)
        torch.cuda.synchronize()
        if precision == "double":
            assert sum(x.item() for x in es) == pytest.approx(e1, rel=1e-11)
        else:   # one mixed rank walks the half list (each pair once), several the full list: the
            # fp32 pair terms round differently (observed 2.4e-3 kJ/mol = 2e-9 of sum|terms|;
            # the mixed-precision energy bar against fp64 is 1e-8 of sum|terms|)
            assert abs(sum(x.item() for x in es) - e1) <= 1e-8 * np.abs(t1).sum()
        if precision == "double":
            assert np.abs(f.cpu().numpy() - f1).max() < 1e-8
        else:   # fp32 per-lane force sums: the list kind (half on one rank, full on several) and the
            # rank's lanes-per-atom choice change their rounding (observed 2.5e-3 = 1.0e-6 of max|F|)
            assert np.abs(f.cpu().numpy() - f1).max() < 1e-5 * np.abs(f1).max()


def test_grid_c3_matches_exact_mfma_path():
    # full C3 (96k atoms, kmax 31): grid path against the exact fp64-MFMA k-sum
    system, force, pos, box = ts.make("C3")
    ka = HipCalcCoulForceKernel(kspace_algo=0).initialize(system, force)
    kg = HipCalcCoulForceKernel(kspace_algo=GRID).initialize(system, force)
    ea, fa = ka.execute_host(pos, box)
    eg, fg = kg.execute_host(pos, box)
    assert abs(eg - ea) <= 1e-9 * abs(ea) + 1e-8, (eg, ea)
    assert np.abs(fg - fa).max() <= F_TOL, np.abs(fg - fa).max()
    da, dg = ka.dedq(), kg.dedq()
    assert np.abs(dg - da).max() <= 1e-9 * np.abs(da).max() + 1e-9
    ta, tg = ka.energy_terms(), kg.energy_terms()
    assert tg[1] == pytest.approx(ta[1], rel=1e-10)


def test_grid_options_validation():
    system, force, pos, box = ts.water_box(100, cutoff=0.6)
    with pytest.raises(ChargeFluxError):
        HipCalcCoulForceKernel(kspace_algo=GRID, grid_width=3).initialize(system, force)
    with pytest.raises(ChargeFluxError):
        HipCalcCoulForceKernel(kspace_algo=7).initialize(system, force)


def _with_dft8(flag, system, force, **kw):
    # flag "0": the GEMM stages (CF_VARIANT_GEMM_DFT), "1": the factorized stages (default)
    v = _cabi.CF_VARIANT_GEMM_DFT if flag == "0" else 0
    return HipCalcCoulForceKernel(kspace_algo=GRID, variants=v, **kw).initialize(system, force)


@pytest.mark.parametrize("case", ["C2", "noncubic", "odd_kmax_12k", "C3"])
def test_grid_dft8_matches_gemm_stages(case):
    # the factorized DFT stages (ng = 8Q: 8-point DFTs + Q-term sums per mode)
    # evaluate the same pruned sums as the fp64-MFMA GEMM stages; only the summation order
    # differs: energy, dE/dq and forces equal to <= 1e-12 relative
    if case == "C2":
        system, force, pos, box = ts.make("C2")
    elif case == "C3":
        system, force, pos, box = ts.make("C3")
    elif case == "noncubic":
        system, force, pos, box = ts.water_box(400, cutoff=0.7, ewald_tol=1e-4)
        box = box.copy()
        box[0, 0] *= 1.3
        box[2, 2] *= 0.95
        system.setDefaultPeriodicBoxVectors(*box)
    else:
        system, force, pos, box = ts.water_box(4000, cutoff=1.0, ewald_tol=1e-4)
    out = []
    for flag in ("0", "1"):
        k = _with_dft8(flag, system, force)
        e, f = k.execute_host(pos, box)
        out.append((e, f, k.dedq(), k.energy_terms()))
        k.destroy()
    (e0, f0, d0, t0), (e1, f1, d1, t1) = out
    scale = sum(abs(t) for t in t0)
    assert abs(e1 - e0) <= 1e-12 * scale, (e0, e1)
    assert np.abs(f1 - f0).max() <= 1e-12 * np.abs(f0).max(), np.abs(f1 - f0).max()
    assert np.abs(d1 - d0).max() <= 1e-12 * np.abs(d0).max(), np.abs(d1 - d0).max()


@pytest.mark.parametrize("case,width,spread", [("C2", 14, 0), ("C2", 13, 0), ("w4k", 14, 0), ("w4k", 14, 2),
                                               ("w4k", 8, 0), ("w4k", 11, 0), ("w4k", 16, 0), ("w4k", 12, 0),
                                               ("w4k", 9, 0)])
def test_grid_interp2_matches_interp(case, width, spread):
    """The two-atoms-per-wave interpolation (k_g_interp2: taps in registers, DPP row broadcasts,
    x rows split by parity over the two rows of a half-wave) against the one-atom form
    (CF_VARIANT_INTERP1), even and odd kernel widths, with either spread (spread = 2:
    CF_VARIANT_VECTOR_SPREAD): the same sums in another order, forces and dE/dq equal to <= 1e-12
    relative, energy unchanged (not interpolated)."""
    if case == "C2":
        system, force, pos, box = ts.make("C2")
    else:
        system, force, pos, box = ts.water_box(4000, cutoff=1.0, ewald_tol=1e-4, every_bond_angle=5)
    out = []
    for v in (_cabi.CF_VARIANT_INTERP1, 0):
        k = HipCalcCoulForceKernel(kspace_algo=GRID, grid_width=width, variants=v | spread | (
            _cabi.CF_VARIANT_INTERP2 if width <= 8 else 0)).initialize(system, force)
        e, f = k.execute_host(pos, box)
        out.append((e, f, k.dedq()))
        k.destroy()
    (e0, f0, d0), (e1, f1, d1) = out
    assert e1 == e0
    assert np.abs(f1 - f0).max() <= 1e-12 * np.abs(f0).max(), np.abs(f1 - f0).max()
    assert np.abs(d1 - d0).max() <= 1e-12 * np.abs(d0).max(), np.abs(d1 - d0).max()


@pytest.mark.parametrize("case,width", [("C2", 8), ("w4k", 8), ("w4k", 7), ("w4k", 6), ("w4k", 5), ("w4k", 4)])
def test_grid_interp4_matches_interp(case, width):
    """The four-atoms-per-wave interpolation (k_g_interp4, W <= 8: one atom per 16-lane row, y
    taps by bank-masked row broadcasts) against the one-atom form (CF_VARIANT_INTERP1) and the
    two-atom form (CF_VARIANT_INTERP2), even and odd widths: forces and dE/dq equal to <= 1e-12
    relative, energy unchanged (not interpolated)."""
    if case == "C2":
        system, force, pos, box = ts.make("C2")
    else:
        system, force, pos, box = ts.water_box(4000, cutoff=1.0, ewald_tol=1e-4, every_bond_angle=5)
    out = []
    for v in (_cabi.CF_VARIANT_INTERP1, _cabi.CF_VARIANT_INTERP2, 0):
        k = HipCalcCoulForceKernel(kspace_algo=GRID, grid_width=width, variants=v).initialize(system, force)
        e, f = k.execute_host(pos, box)
        out.append((e, f, k.dedq()))
        k.destroy()
    e0, f0, d0 = out[0]
    for e1, f1, d1 in out[1:]:
        assert e1 == e0
        assert np.abs(f1 - f0).max() <= 1e-12 * np.abs(f0).max(), np.abs(f1 - f0).max()
        assert np.abs(d1 - d0).max() <= 1e-12 * np.abs(d0).max(), np.abs(d1 - d0).max()


def _odd_tile_box():
    """A water box whose grid has an odd number of 8-point bins along x (ng = round8(2 (2K - 1)),
    cf_kernels_grid.hip grid_plan), so the matrix-core spread's last 16-wide x tile is a half tile."""
    for n in (700, 900, 1100, 1300, 1500, 1800, 2100):
        system, force, pos, box = ts.water_box(n, cutoff=0.9, ewald_tol=1e-4)
        k = HipCalcCoulForceKernel(kspace_algo=GRID).initialize(system, force)
        kx = k.ewald_params()[1][0]
        k.destroy()
        if ((-(-2 * (2 * kx - 1) // 8)) % 2) == 1:
            return system, force, pos, box
    pytest.skip("no odd-bin box among the sizes tried")


@pytest.mark.parametrize("case,width", [("C2", 14), ("w4k", 14), ("w4k", 13), ("w4k", 11), ("w4k", 8), ("w4k", 5),
                                        ("small", 14), ("tric", 12), ("odd", 14), ("odd", 8)])
def test_grid_spread_mfma_matches_vector_spread(case, width):
    """The matrix-core spread (k_g_spread_mfma: 16x8x8 tiles, v_mfma_f64_16x16x4 over groups of
    4 source atoms) against the vector spread (CF_VARIANT_VECTOR_SPREAD, k_g_spread_tile): the same
    grid sums in another order, so energy, forces and dE/dq equal to <= 1e-12 relative, and the
    matrix form bitwise reproducible run to run.  'small' has a small grid (few x-bins per
    16-wide tile), 'tric' a reduced triclinic box, 'odd' an odd number of x-bins (a half tile
    at the end of every x row, as C5's 264-point grid)."""
    if case == "C2":
        system, force, pos, box = ts.make("C2")
    elif case == "small":
        system, force, pos, box = ts.water_box(300, cutoff=0.9, ewald_tol=1e-4)
    elif case == "tric":
        system, force, pos, box = ts.water_box(2000, cutoff=0.9, ewald_tol=1e-4)
        box = box.copy()
        box[1, 0] = 0.3 * box[0, 0]
        box[2, 0] = -0.2 * box[0, 0]
        box[2, 1] = 0.25 * box[1, 1]
        system.setDefaultPeriodicBoxVectors(*box)
    elif case == "odd":
        system, force, pos, box = _odd_tile_box()
    else:
        system, force, pos, box = ts.water_box(4000, cutoff=1.0, ewald_tol=1e-4, every_bond_angle=5)
    out = []
    # the vector form, then the matrix form at every width twice (the default uses it for W > 9)
    for v in (_cabi.CF_VARIANT_VECTOR_SPREAD, _cabi.CF_VARIANT_MFMA_SPREAD, _cabi.CF_VARIANT_MFMA_SPREAD):
        k = HipCalcCoulForceKernel(kspace_algo=GRID, grid_width=width, variants=v).initialize(system, force)
        e, f = k.execute_host(pos, box)
        out.append((e, f, k.dedq(), k.energy_terms()))
        k.destroy()
    (e0, f0, d0, t0), (e1, f1, d1, _), (e2, f2, d2, _) = out
    scale = sum(abs(t) for t in t0)
    assert abs(e1 - e0) <= 1e-12 * scale, (e0, e1)
    assert np.abs(f1 - f0).max() <= 1e-12 * np.abs(f0).max(), np.abs(f1 - f0).max()
    assert np.abs(d1 - d0).max() <= 1e-12 * np.abs(d0).max(), np.abs(d1 - d0).max()
    assert e2 == e1 and np.array_equal(f2, f1) and np.array_equal(d2, d1)


@pytest.mark.parametrize("rounds", [3, 8])
def test_grid_bin_rounds_bitwise(rounds):
    """k_g_bin and k_assemble_energy with several 256-atom rounds per block (the default from
    262144 owned atoms up; CF_VARIANT_BLOCK_ROUNDS forces it at a small size): the provisional ranks come
    from atomics in any order and k_g_order_taps restores the stable order, so forces and dE/dq
    are bitwise equal to the one-round launch -- including a ragged last block; the energy is
    the same fixed-order sum regrouped (per-thread chunk sums, fewer block partials): <= 1e-13
    relative, and bitwise reproducible run to run."""
    system, force, pos, box = ts.water_box(4000, cutoff=1.0, ewald_tol=1e-4, every_bond_angle=5)
    out = []
    for r in (1, rounds):
        k = HipCalcCoulForceKernel(kspace_algo=GRID, variants=_cabi.CF_VARIANT_BLOCK_ROUNDS(r)).initialize(system,
                                                                                                          force)
        e, f = k.execute_host(pos, box)
        e2, f2 = k.execute_host(pos, box)   # the ticket re-armed by the last block
        out.append((e, f, k.dedq()))
        assert e2 == e and np.array_equal(f2, f)
        k.destroy()
    (e0, f0, d0), (e1, f1, d1) = out
    assert abs(e1 - e0) <= 1e-13 * abs(e0), (e0, e1)
    assert np.array_equal(f1, f0) and np.array_equal(d1, d0)
