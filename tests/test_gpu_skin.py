"""Persistent neighbour list with a skin (cf_set_neighbor_skin).

The reference rebuilds its voxel-hash list on every call (ReferenceCoulKernels.cpp:559).
With a skin the HIP path keeps the list while no atom has moved more than skin/2; the
evaluated pair set must be exactly the same, so results must agree with a rebuild-every-call
kernel to rounding (only the fp64 summation order may differ) and with the oracle.

Tolerances: energy rel 1e-11, forces max |dF| 1e-8 kJ/mol/nm against the skin-0 kernel;
the usual oracle tolerances (test_gpu_parity.py) at the end of the trajectory.
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


def _pair(system, force, skin):
    ref = HipCalcCoulForceKernel().initialize(system, force)
    sk = HipCalcCoulForceKernel().initialize(system, force).set_neighbor_skin(skin)
    return ref, sk


def _same(a, b, e_rel=1e-11, f_abs=1e-8):
    (ea, fa), (eb, fb) = a, b
    assert ea == pytest.approx(eb, rel=e_rel, abs=1e-8)
    assert np.abs(fa - fb).max() <= f_abs, np.abs(fa - fb).max()


# 400 waters rc 0.7: 2 cells/dim at rc+skin -> brute-force list path;
# 4000 waters rc 1.0: 4 cells/dim -> wave-cooperative list path (periodic seams)
@pytest.mark.parametrize("nw,rc,tol", [(400, 0.7, 1e-4), (4000, 1.0, 1e-3)])
def test_skin_trajectory_matches_rebuild_every_call(nw, rc, tol):
    system, force, pos, box = ts.water_box(nw, cutoff=rc, ewald_tol=tol, every_bond_angle=5)
    ref, sk = _pair(system, force, 0.1)
    rng = np.random.default_rng(7)
    x = pos.copy()
    for step in range(30):
        _same(sk.execute_host(x, box), ref.execute_host(x, box))
        x = x + rng.normal(scale=0.004, size=x.shape)   # ~0.007 nm per step per atom
    builds, evals = sk.neighbor_stats()
    assert evals == 30
    assert 2 <= builds < evals, (builds, evals)       # reused, and rebuilt when atoms moved
    assert ref.neighbor_stats()[0] == 30
    if nw <= 400:
        o = Oracle(force, box).execute(x, box)
        e, f = sk.execute_host(x, box)
        assert e == pytest.approx(o["energy"], rel=1e-9)
        assert np.abs(f - o["forces"]).max() <= 1e-8


def test_skin_rebuilds_on_wrap_and_box_change():
    system, force, pos, box = ts.water_box(400, cutoff=0.7, ewald_tol=1e-4)
    ref, sk = _pair(system, force, 0.1)
    _same(sk.execute_host(pos, box), ref.execute_host(pos, box))
    b0 = sk.neighbor_stats()[0]
    # an atom re-wrapped by a full box vector: a jump of L must force a rebuild
    x = pos.copy()
    x[5, 0] += box[0, 0]
    _same(sk.execute_host(x, box), ref.execute_host(x, box))
    assert sk.neighbor_stats()[0] == b0 + 1
    # unchanged positions: list reused
    _same(sk.execute_host(x, box), ref.execute_host(x, box))
    assert sk.neighbor_stats()[0] == b0 + 1
    # a new box (barostat-like scaling): rebuild
    box2 = box * 1.002
    x2 = x * 1.002
    _same(sk.execute_host(x2, box2), ref.execute_host(x2, box2))
    assert sk.neighbor_stats()[0] == b0 + 2


def test_skin_capped_by_small_box():
    # 100 waters, L = 1.44 nm, rc 0.6: the requested 0.3 nm skin is capped at L/2 - rc
    system, force, pos, box = ts.water_box(100, cutoff=0.6, ewald_tol=1e-4)
    ref, sk = _pair(system, force, 0.3)
    rng = np.random.default_rng(3)
    x = pos.copy()
    for _ in range(8):
        _same(sk.execute_host(x, box), ref.execute_host(x, box))
        x = x + rng.normal(scale=0.01, size=x.shape)
    o = Oracle(force, box).execute(x, box)
    e, f = sk.execute_host(x, box)
    assert e == pytest.approx(o["energy"], rel=1e-9)
    assert np.abs(f - o["forces"]).max() <= 1e-8


def test_skin_two_rank_split_phase_matches_single():
    # 2 ranks on one device through the split-phase API with a skin: sum of rank energies
    # and the union of owned forces equal the single-rank result
    system, force, pos, box = ts.water_box(2400, cutoff=1.0, ewald_tol=1e-3)
    stream = torch.cuda.current_stream().cuda_stream
    single = HipCalcCoulForceKernel(stream=stream).initialize(system, force)
    ranks = [HipCalcCoulForceKernel(stream=stream, rank=r, world_size=2).initialize(system, force)
             .set_neighbor_skin(0.1) for r in range(2)]
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(11)
    x = pos.copy()
    for _ in range(6):
        e1, f1 = single.execute_host(x, box)
        p = torch.tensor(x, dtype=torch.float64, device=dev)
        f = torch.zeros_like(p)
        bufs = [k.kspace_tensor(dev) for k in ranks]
        for k in ranks:
            k.begin(p, box, True, True)
        torch.cuda.synchronize()
        tot = bufs[0] + bufs[1]
        bufs[0].copy_(tot)
        bufs[1].copy_(tot)
        es = []
        for k in ranks:
            e = torch.zeros(1, dtype=torch.float64, device=dev)
            k.end(f, e)
            es.append(e)
        torch.cuda.synchronize()
        assert (es[0] + es[1]).item() == pytest.approx(e1, rel=1e-11)
        assert np.abs(f.cpu().numpy() - f1).max() < 1e-8
        x = x + rng.normal(scale=0.01, size=x.shape)
    assert all(k.neighbor_stats()[0] < 6 for k in ranks)
