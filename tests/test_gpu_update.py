"""updateParametersInContext (cf_update_parameters): after new charges, LJ
and flux parameters on the same topology, the HIP path must equal a freshly created handle
and the oracle on the new parameters.  Tolerances as in test_gpu_parity.py."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from oracle import Oracle  # noqa: E402
from openmmcoul import ChargeFluxError, Context, HipCalcCoulForceKernel, System, _cabi  # noqa: E402
from openmmcoul import testsystems as ts  # noqa: E402
from tests.test_gpu_parity import _compare, _run  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _perturb(force, rng, distinct_lj=False):
    for i in range(force.getNumParticles()):
        q, s, e = force.getParticleParameters(i)
        if distinct_lj:   # > 64 distinct LJ parameter sets: the per-atom LJ gather path
            s, e = s + 1e-6 * i, e + 1e-8 * i
        elif e > 0:
            s, e = s * 1.02, e * 0.9
        force.setParticleParameters(i, q * 1.05, s, e)
    for k in range(force.getNumFluxWaters()):
        po, h1, h2, k1, k2, kub, b0, ub0 = force.getFluxWaterParameters(k)
        force._fwater_par[k] = (k1 * 1.1, k2 - 0.05, kub, b0, ub0)
    for k in range(force.getNumFluxBonds()):
        force._fbond_par[k] = (force._fbond_par[k][0] * 0.9, force._fbond_par[k][1])
    for k in range(force.getNumFluxAngles()):
        force._fangle_par[k] = (force._fangle_par[k][0] + 0.02, force._fangle_par[k][1])


@pytest.mark.parametrize("algo,skin,distinct", [(0, 0.0, False), (2, 0.1, False), (2, 0.1, True)])
def test_update_matches_fresh_handle_and_oracle(algo, skin, distinct):
    system, force, pos, box = ts.water_box(400, cutoff=0.7, ewald_tol=1e-4, every_bond_angle=3)
    k = HipCalcCoulForceKernel(kspace_algo=algo).initialize(system, force)
    k.set_neighbor_skin(skin)
    e0, _ = k.execute_host(pos, box)
    _perturb(force, np.random.default_rng(3), distinct)
    k.copyParametersToContext(force)
    got = _run(k, pos, box)
    assert abs(got[0] - e0) > 1e-3 * abs(e0)   # the update took effect
    fresh = HipCalcCoulForceKernel(kspace_algo=algo).initialize(system, force)
    ref_h = _run(fresh, pos, box)
    assert abs(got[0] - ref_h[0]) <= 1e-12 * abs(ref_h[0])
    assert np.abs(got[1] - ref_h[1]).max() <= 1e-12 * np.abs(ref_h[1]).max() + 1e-9
    _compare(got, Oracle(force, box).execute(pos, box), f_tol=2.5e-6 if algo == 2 else 1e-8)


def test_update_no_pbc_through_context():
    system, force, pos, _ = ts.cluster_c1()
    ctx = Context(system)
    ctx.setPositions(pos)
    e0 = ctx.getState(getEnergy=True).getPotentialEnergy()
    _perturb(force, np.random.default_rng(5))
    force.updateParametersInContext(ctx)
    st = ctx.getState(getEnergy=True, getForces=True)
    ref = Oracle(force).execute(pos, None)
    assert st.getPotentialEnergy() != e0
    assert abs(st.getPotentialEnergy() - ref["energy"]) <= 1e-9 * abs(ref["energy"]) + 1e-8
    assert np.abs(st.getForces() - ref["forces"]).max() <= 1e-8


def test_update_rejects_topology_changes():
    system, force, pos, box = ts.water_box(100, cutoff=0.6, every_bond_angle=3)
    k = HipCalcCoulForceKernel().initialize(system, force)
    f2 = ts.water_box(100, cutoff=0.6, every_bond_angle=3)[1]
    f2._exclusions[0] = (0, 5)
    with pytest.raises(ChargeFluxError) as ei:
        k.copyParametersToContext(f2)
    assert ei.value.code == _cabi.CF_ERR_INVALID
    f3 = ts.water_box(100, cutoff=0.6, every_bond_angle=3)[1]
    f3._fwater_idx[0] = (f3._fwater_idx[0][0], f3._fwater_idx[0][2], f3._fwater_idx[0][1])
    with pytest.raises(ChargeFluxError):
        k.copyParametersToContext(f3)
    f4 = ts.water_box(100, cutoff=0.6, every_bond_angle=3)[1]
    f4.setCutoffDistance(0.5)
    with pytest.raises(ChargeFluxError):
        k.copyParametersToContext(f4)
    # the handle still works with its original parameters
    e, _ = k.execute_host(pos, box)
    ref = Oracle(force, box).execute(pos, box)
    assert abs(e - ref["energy"]) <= 1e-9 * abs(ref["energy"]) + 1e-8
    ctx = Context(System())
    with pytest.raises(ValueError):
        force.updateParametersInContext(ctx)
