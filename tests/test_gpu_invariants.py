"""Physics checks of the HIP path itself, independent of the oracle:
finite-difference gradients including the charge-flux chain rule, dE/dq against a charge
derivative, translation and lattice invariance, two point charges, and zero flux constants
reproducing plain Ewald.  fp64, through the C-ABI."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from openmmcoul import CoulForce, HipCalcCoulForceKernel, ONE_4PI_EPS0, System  # noqa: E402
from openmmcoul import testsystems as ts  # noqa: E402

GRID = HipCalcCoulForceKernel.KSPACE_GRID


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _fd_check(k, pos, box, atoms, h=1e-6, tol=2e-4):
    # central differences of the energy against the returned forces (F = -dE/dx with the
    # flux chain rule, ReferenceCoulKernels.cpp:626-632); same bar as the oracle's own check
    _, f = k.execute_host(pos, box)
    for i in atoms:
        for d in range(3):
            p1, p2 = pos.copy(), pos.copy()
            p1[i, d] += h
            p2[i, d] -= h
            e1, _ = k.execute_host(p1, box, includeForces=False)
            e2, _ = k.execute_host(p2, box, includeForces=False)
            fd = -(e1 - e2) / (2 * h)
            assert f[i, d] == pytest.approx(fd, abs=tol, rel=1e-6), (i, d, f[i, d], fd)


def test_fd_no_pbc_cluster():
    system, force, pos, _ = ts.cluster_c1()
    k = HipCalcCoulForceKernel().initialize(system, force)
    _fd_check(k, pos, None, atoms=[0, 1, 2, 3, 4, 5, 100, 200, 255])


@pytest.mark.parametrize("algo", [0, GRID])
def test_fd_pbc_flux_box(algo):
    system, force, pos, box = ts.water_box(40, cutoff=0.5, ewald_tol=1e-6, every_bond_angle=3)
    k = HipCalcCoulForceKernel(kspace_algo=algo).initialize(system, force)
    _fd_check(k, pos, box, atoms=[0, 1, 2, 6, 7, 8, 30, 61])


def test_dedq_is_charge_derivative():
    system, force, pos, box = ts.water_box(40, cutoff=0.5, ewald_tol=1e-6, every_bond_angle=3)
    k = HipCalcCoulForceKernel().initialize(system, force)
    k.execute_host(pos, box)
    dedq = k.dedq()
    h = 1e-6
    for i in (0, 4, 11):
        q, s, e = force.getParticleParameters(i)
        es = []
        for dq in (h, -h):
            force.setParticleParameters(i, q + dq, s, e)
            k.copyParametersToContext(force)
            es.append(k.execute_host(pos, box, includeForces=False)[0])
        force.setParticleParameters(i, q, s, e)
        k.copyParametersToContext(force)
        assert dedq[i] == pytest.approx((es[0] - es[1]) / (2 * h), rel=1e-6, abs=1e-5)


def test_translation_and_lattice_invariance():
    system, force, pos, _ = ts.cluster_c1()
    _, f = HipCalcCoulForceKernel().initialize(system, force).execute_host(pos, None)
    assert np.abs(f.sum(axis=0)).max() < 1e-8 * np.abs(f).max() * len(pos)   # sum F = 0 without PBC
    system, force, pos, box = ts.water_box(400, cutoff=0.7, ewald_tol=1e-5, every_bond_angle=3)
    for algo in (0, GRID):
        k = HipCalcCoulForceKernel(kspace_algo=algo).initialize(system, force)
        e0, f0 = k.execute_host(pos, box)
        p2 = pos.copy()
        p2[3:6] += box[0]           # one whole water moved by a lattice vector
        p2[90:93] -= 2 * box[2]
        p2[600:603] += box[1] - box[0]
        e1, f1 = k.execute_host(p2, box)
        assert e1 == pytest.approx(e0, rel=1e-10)
        assert np.abs(f1 - f0).max() <= 1e-7 * np.abs(f0).max()


def test_two_point_charges():
    f = CoulForce()
    f.addParticle(0.7, 0.0, 0.0)
    f.addParticle(-1.3, 0.0, 0.0)
    s = System()
    s.addParticle(1.0)
    s.addParticle(1.0)
    pos = np.array([[0.1, 0.2, 0.3], [0.5, -0.2, 0.9]])
    e, frc = HipCalcCoulForceKernel().initialize(s, f).execute_host(pos, None)
    d = pos[0] - pos[1]
    r = np.linalg.norm(d)
    assert e == pytest.approx(ONE_4PI_EPS0 * 0.7 * -1.3 / r, rel=1e-14)
    fe = ONE_4PI_EPS0 * 0.7 * -1.3 / r ** 3 * d
    assert np.abs(frc[0] - fe).max() <= 1e-12 * np.abs(fe).max()
    assert np.abs(frc[1] + fe).max() <= 1e-12 * np.abs(fe).max()


def test_zero_flux_constants_reproduce_plain_ewald():
    # every flux constant 0 -> charges stay q0 and the chain rule adds nothing: the same
    # energy and forces as the force without any flux term
    system, force, pos, box = ts.water_box(300, cutoff=0.7, ewald_tol=1e-5, every_bond_angle=3)
    plain = CoulForce()
    for i in range(force.getNumParticles()):
        plain.addParticle(*force.getParticleParameters(i))
    for kx in range(force.getNumExceptions()):
        plain.addException(*force.getExceptionParameters(kx))
    plain.setUsesPeriodicBoundaryConditions(True)
    plain.setCutoffDistance(0.7)
    plain.setEwaldErrorTolerance(1e-5)
    force._fbond_par = [(0.0, b) for _, b in force._fbond_par]
    force._fangle_par = [(0.0, t) for _, t in force._fangle_par]
    force._fwater_par = [(0.0, 0.0, 0.0, b0, ub0) for _, _, _, b0, ub0 in force._fwater_par]
    for algo in (0, GRID):
        e1, f1 = HipCalcCoulForceKernel(kspace_algo=algo).initialize(system, force).execute_host(pos, box)
        e2, f2 = HipCalcCoulForceKernel(kspace_algo=algo).initialize(system, plain).execute_host(pos, box)
        assert e1 == pytest.approx(e2, rel=1e-13)
        assert np.abs(f1 - f2).max() <= 1e-12 * np.abs(f2).max()
