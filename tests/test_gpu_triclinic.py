"""GPU parity for reduced triclinic boxes (OpenMM's form a = (ax,0,0), b = (bx,by,0),
c = (cx,cy,cz)).  The reference takes the minimum image with the box vectors
(getDeltaRPeriodic: c, b, a in turn; ReferenceCoulKernels.cpp:567, 601 and the flux terms
RCK:53-55) and the reciprocal k-set and weights from the box diagonals only, on unwrapped
positions (RCK:513-547).  Here the real space uses the same box-vector minimum image, with cells
that are parallelepipeds in fractional coordinates (O(N): cf_api.hip set_cells,
cf_kernels_core.hip k_cell_hist; boxes under 3 cells per direction use all pairs), the k-space paths are
unchanged (both evaluate the diagonal-only sum on per-axis wrapped coordinates, which leave
every factor e^{i k_a x_a} unchanged).
Tolerances as in test_gpu_parity.py (exact k-sum: forces 1e-8) and test_gpu_grid.py (grid: 2.5e-6).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from oracle import Oracle  # noqa: E402
from openmmcoul import HipCalcCoulForceKernel  # noqa: E402
from openmmcoul import testsystems as ts  # noqa: E402

EXACT = HipCalcCoulForceKernel.KSPACE_EXACT_MFMA
GRID = HipCalcCoulForceKernel.KSPACE_GRID


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _compare(k, pos, box, ref, f_tol, fl=True, en=True):
    e, f = k.execute_host(pos, box, fl, en)
    assert abs(e - ref["energy"]) <= 1e-9 * abs(ref["energy"]) + 1e-8, (e, ref["energy"])
    if fl:
        assert np.abs(f - ref["forces"]).max() <= f_tol, np.abs(f - ref["forces"]).max()
        scale = np.abs(ref["dedq"]).max()
        assert np.abs(k.dedq() - ref["dedq"]).max() <= 1e-9 * scale + 1e-9
    assert np.abs(k.charges() - ref["charges"]).max() <= 1e-12
    for a, b in zip(k.energy_terms(), ref["terms"]):
        assert abs(a - b) <= 1e-9 * max(abs(b), 1.0) + 1e-8, (k.energy_terms(), ref["terms"])


@pytest.mark.parametrize("algo,f_tol", [(EXACT, 1e-8), (GRID, 2.5e-6)])
def test_triclinic_vs_oracle(algo, f_tol):
    system, force, pos, box = ts.triclinic_water_box(300, cutoff=0.7)
    k = HipCalcCoulForceKernel(kspace_algo=algo).initialize(system, force)
    o = Oracle(force, box)
    for fl, en in ((True, True), (True, False), (False, True)):
        _compare(k, pos, box, o.execute(pos, box, fl, en), f_tol, fl, en)


@pytest.mark.parametrize("algo,f_tol", [(EXACT, 1e-8), (GRID, 2.5e-6)])
def test_triclinic_moved_and_lattice_shifted(algo, f_tol):
    # atoms displaced and some moved by whole box vectors (the reference's k-sum uses the
    # unwrapped positions, so a lattice shift changes it: both sides see the same positions)
    system, force, pos, box = ts.triclinic_water_box(300, cutoff=0.7, shear=(-0.4, 0.35, -0.3))
    rng = np.random.default_rng(3)
    p2 = pos + rng.normal(scale=0.01, size=pos.shape)
    p2[::7] += box[1]
    p2[::11] -= box[2]
    p2[::13] += box[0] + box[2]
    k = HipCalcCoulForceKernel(kspace_algo=algo).initialize(system, force)
    _compare(k, p2, box, Oracle(force, box).execute(p2, box), f_tol)


def test_triclinic_with_skin_trajectory_and_box_switch():
    # persistent list with skin over a short trajectory, then an orthorhombic box and back:
    # every evaluation matches the oracle (the list is rebuilt when the box changes)
    system, force, pos, box = ts.triclinic_water_box(300, cutoff=0.7)
    k = HipCalcCoulForceKernel(kspace_algo=EXACT).initialize(system, force)
    k.set_neighbor_skin(0.1)
    o = Oracle(force, box)
    rng = np.random.default_rng(9)
    p = pos.copy()
    for step in range(4):
        p = p + rng.normal(scale=0.004, size=p.shape)
        _compare(k, p, box, o.execute(p, box), 1e-8)
    ortho = np.diag(np.diag(box))
    _compare(k, p, ortho, o.execute(p, ortho), 1e-8)
    _compare(k, p, box, o.execute(p, box), 1e-8)


@pytest.mark.parametrize("algo", [EXACT, GRID])
def test_triclinic_two_rank_split_on_one_gpu(algo):
    # atom decomposition (the all-reduce of the k-space buffer done by hand) on a triclinic box
    from openmmcoul.distributed import device_buffer_as_tensor
    system, force, pos, box = ts.triclinic_water_box(300, cutoff=0.7)
    stream = torch.cuda.current_stream().cuda_stream
    pt = torch.tensor(pos, dtype=torch.float64, device="cuda")
    e1, f1 = HipCalcCoulForceKernel(stream=stream, kspace_algo=algo).initialize(system, force).execute_host(pos, box)
    ks = [HipCalcCoulForceKernel(stream=stream, rank=r, world_size=2, kspace_algo=algo).initialize(system, force)
          for r in range(2)]
    for k in ks:
        k.begin(pt, box, True, True)
    bufs = [device_buffer_as_tensor(*k.kspace_buffer(), "cuda") for k in ks]
    total = bufs[0] + bufs[1]
    for b in bufs:
        b.copy_(total)
    f = torch.zeros_like(pt)
    es = []
    for k in ks:
        e = torch.zeros(1, dtype=torch.float64, device="cuda")
        k.end(f, e)
        es.append(e)
    torch.cuda.synchronize()
    assert (es[0] + es[1]).item() == pytest.approx(e1, rel=1e-11)
    assert np.abs(f.cpu().numpy() - f1).max() < 1e-8


def test_non_reduced_box_rejected():
    from openmmcoul import ChargeFluxError
    system, force, pos, box = ts.triclinic_water_box(300, cutoff=0.7)
    k = HipCalcCoulForceKernel(kspace_algo=EXACT).initialize(system, force)
    bad = box.copy()
    bad[1, 0] = 0.7 * box[0, 0]
    with pytest.raises(ChargeFluxError):
        k.execute_host(pos, bad)
    bad = box.copy()
    bad[0, 2] = 0.1
    with pytest.raises(ChargeFluxError):
        k.execute_host(pos, bad)


@pytest.mark.parametrize("algo", [EXACT, GRID])
def test_triclinic_mixed_precision(algo):
    # the fp32 full-list pair kernel (k_pairs_mixed) with the box-vector minimum image formed in
    # fp64; bars of tests/test_gpu_mixed.py (RMS-relative force error 1e-4, energy 1e-7 of
    # sum |terms|; the pair kernel alone, exact k-sum: 1e-5)
    system, force, pos, box = ts.triclinic_water_box(300, cutoff=0.7)
    k = HipCalcCoulForceKernel(kspace_algo=algo, precision="mixed").initialize(system, force)
    ref = Oracle(force, box).execute(pos, box)
    e, f = k.execute_host(pos, box)
    d = f - ref["forces"]
    err = np.sqrt((d ** 2).sum(1).mean() / (ref["forces"] ** 2).sum(1).mean())
    assert err <= (1e-5 if algo == EXACT else 1e-4), err
    assert abs(e - ref["energy"]) <= 1e-7 * np.abs(ref["terms"]).sum()


# ---- the O(N) cell path at sizes where it runs (>= 4 cells per lattice direction) ----------------
# 4000 waters (12 000 atoms), rc 0.7 nm: 6 cells per direction in fractional coordinates, the
# wave builder and the half list (one rank).  The oracle's triclinic pair search is all pairs.
def _big(shear=(0.3, -0.25, 0.2), n=4000):
    return ts.triclinic_water_box(n, cutoff=0.7, ewald_tol=1e-4, shear=shear)


def _kernel(system, force, algo, half=True, skin=0.0, precision="double"):
    k = HipCalcCoulForceKernel(kspace_algo=algo, precision=precision,
                               pair_list="auto" if half else "full").initialize(system, force)
    if skin:
        k.set_neighbor_skin(skin)
    return k


@pytest.mark.parametrize("shear", [(0.3, -0.25, 0.2), (-0.5, 0.5, -0.5), (0.45, 0.0, 0.0)])
def test_triclinic_cell_path_vs_oracle_12k(shear):
    system, force, pos, box = _big(shear)
    ref = Oracle(force, box).execute(pos, box)
    for half in (True, False):
        k = _kernel(system, force, EXACT, half)
        _compare(k, pos, box, ref, 1e-8)
        assert k.fallback_stats() == (0, 0, 0), k.fallback_stats()   # the fast paths, not the rescan


def test_triclinic_cell_path_lattice_shifted_atoms_and_grid():
    system, force, pos, box = _big((-0.4, 0.35, -0.3))
    rng = np.random.default_rng(5)
    p2 = pos + rng.normal(scale=0.01, size=pos.shape)
    p2[::7] += box[1]
    p2[::11] -= box[2]
    p2[::13] += box[0] - box[1] + box[2]
    ref = Oracle(force, box).execute(p2, box)
    _compare(_kernel(system, force, GRID), p2, box, ref, 2.5e-6)


def test_triclinic_cell_path_skin_trajectory_half_and_full():
    # a kept list (skin) over moved steps, the half list and the full list, each step vs the oracle
    system, force, pos, box = _big()
    o = Oracle(force, box)
    ks = [_kernel(system, force, EXACT, half, skin=0.1) for half in (True, False)]
    rng = np.random.default_rng(2)
    p = pos.copy()
    for step in range(3):
        ref = o.execute(p, box)
        for k in ks:
            _compare(k, p, box, ref, 1e-8)
        p = p + rng.normal(scale=0.004, size=p.shape)
    builds, evals = ks[0].neighbor_stats()
    assert evals == 3 and builds < 3


def test_triclinic_cell_path_mixed_precision():
    system, force, pos, box = _big()
    ref = Oracle(force, box).execute(pos, box)
    e, f = _kernel(system, force, EXACT, precision="mixed").execute_host(pos, box)
    d = f - ref["forces"]
    assert np.sqrt((d ** 2).sum(1).mean() / (ref["forces"] ** 2).sum(1).mean()) <= 1e-5
    assert abs(e - ref["energy"]) <= 1e-7 * np.abs(ref["terms"]).sum()


def test_triclinic_cell_path_two_ranks():
    from openmmcoul.distributed import device_buffer_as_tensor
    system, force, pos, box = _big()
    stream = torch.cuda.current_stream().cuda_stream
    pt = torch.tensor(pos, dtype=torch.float64, device="cuda")
    e1, f1 = HipCalcCoulForceKernel(stream=stream, kspace_algo=GRID).initialize(system, force).execute_host(pos, box)
    ks = [HipCalcCoulForceKernel(stream=stream, rank=r, world_size=2, kspace_algo=GRID).initialize(system, force)
          for r in range(2)]
    for k in ks:
        k.begin(pt, box, True, True)
    bufs = [device_buffer_as_tensor(*k.kspace_buffer(), "cuda") for k in ks]
    total = bufs[0] + bufs[1]
    for b in bufs:
        b.copy_(total)
    f = torch.zeros_like(pt)
    es = []
    for k in ks:
        e = torch.zeros(1, dtype=torch.float64, device="cuda")
        k.end(f, e)
        es.append(e)
    torch.cuda.synchronize()
    assert (es[0] + es[1]).item() == pytest.approx(e1, rel=1e-11)
    assert np.abs(f.cpu().numpy() - f1).max() < 1e-8
