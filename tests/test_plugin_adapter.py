"""The OpenMM plugin's C++ layer (openmm-chargeflux_amd/plugin/include: CoulHipMarshal.h,
CoulHipKernelCore.h — what HipCalcCoulForceKernel::initialize / execute / copyParametersToContext
run, plugin/src/HipCoulKernels.cpp) compiled against a C++ CoulForce with the reference's API
(tests/cpp/CoulForceStandIn.h; CoulForce.h:22-133) and driven through tests/cpp/libcf_adapter_test.so.

CPU: the adapter reads every particle, exception and flux term through the reference getters in
the reference's order (ReferenceCoulKernels.cpp:230-284, 385-391) and produces the same cf_params
as the Python mirror.  GPU: the plugin path evaluates C1/C2 equal to the oracle (exact k-sum:
forces <= 1e-8 kJ/mol/nm; grid: <= 1e-6), including a parameter update.
"""
import numpy as np
import pytest

from openmmcoul import testsystems as ts
from tests.cpp import adapter

CASES = {"C1": lambda: ts.cluster_c1(), "C2": lambda: ts.make("C2"),
         "mixed_terms": lambda: ts.water_box(300, cutoff=0.7, every_bond_angle=2)}


@pytest.mark.parametrize("name", list(CASES))
def test_adapter_marshals_like_the_mirror(name):
    system, force, pos, box = CASES[name]()
    out, scal, box_out = adapter.marshal(force, box)
    ref = force.arrays()
    for k, v in ref.items():
        assert out[k].shape == v.reshape(out[k].shape).shape, k
        assert np.array_equal(out[k], v.reshape(out[k].shape)), k
    assert scal[0] == (1 if force.usesPeriodicBoundaryConditions() else 0)
    assert scal[1] == force.getCutoffDistance() and scal[2] == force.getEwaldErrorTolerance()
    assert np.array_equal(box_out, np.zeros((3, 3)) if box is None else box)


def test_adapter_checks_particle_count():
    # the System's particle count (ReferenceCoulKernels.cpp:231) must equal the force's
    system, force, pos, box = ts.cluster_c1()
    with pytest.raises(RuntimeError, match="different numbers of particles"):
        adapter.marshal(force, box, n_system=force.getNumParticles() + 1)


torch = pytest.importorskip("torch")


@pytest.fixture()
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


@pytest.mark.gpu
@pytest.mark.parametrize("name,algo,f_tol", [("C1", 0, 1e-8), ("C2", 0, 1e-8), ("C2", 2, 1e-6),
                                              ("mixed_terms", 0, 1e-8)])
def test_plugin_path_matches_oracle(_gpu, name, algo, f_tol):
    from oracle import Oracle
    system, force, pos, box = CASES[name]()
    db = None if box is None else np.array(system.getDefaultPeriodicBoxVectors())
    e, f = adapter.execute(force, db, pos, box, kspace_algo=algo)
    ref = Oracle(force, box).execute(pos, box)
    assert abs(e - ref["energy"]) <= 1e-9 * abs(ref["energy"]) + 1e-8, (e, ref["energy"])
    assert np.abs(f - ref["forces"]).max() <= f_tol, np.abs(f - ref["forces"]).max()


@pytest.mark.gpu
def test_plugin_parameter_update_matches_oracle(_gpu):
    from oracle import Oracle
    system, force, pos, box = ts.water_box(300, cutoff=0.7, every_bond_angle=2)
    import copy
    f2 = copy.deepcopy(force)
    rng = np.random.default_rng(2)
    for i in range(f2.getNumParticles()):
        q, s, e = f2.getParticleParameters(i)
        f2.setParticleParameters(i, q * (1 + 0.05 * rng.standard_normal()), s, e)
    f2._fwater_par = [(k1 * 1.1, k2, kub, b0, ub0) for (k1, k2, kub, b0, ub0) in f2._fwater_par]
    db = np.array(system.getDefaultPeriodicBoxVectors())
    e, f = adapter.execute(force, db, pos, box, kspace_algo=0, update_to=f2)
    ref = Oracle(f2, box).execute(pos, box)
    assert abs(e - ref["energy"]) <= 1e-9 * abs(ref["energy"]) + 1e-8
    assert np.abs(f - ref["forces"]).max() <= 1e-8


@pytest.mark.gpu
def test_plugin_reports_the_rescan_fallback_once(_gpu, capfd):
    """Two waters 0.02 nm apart: a partner-side term beyond the half list's fixed-point range sends
    every evaluation to the fp64 rescan (correct, slow).  The plugin counts them
    (KernelCore::fallback_evaluations) and says so once on stderr, not once per step."""
    system, force, pos, box = ts.water_box(4000, cutoff=1.0, ewald_tol=1e-4)
    p = pos.copy()
    p[3:6] = p[0:3] + np.array([0.02, 0.0, 0.0])
    e, f, n = adapter.execute_count(force, box, p, box, 3)
    assert n >= 3, n
    err = capfd.readouterr().err
    assert err.count("fp64 rescan fallback") == 1, err
    # a normal box: no fallback, no message
    e, f, n = adapter.execute_count(force, box, pos, box, 2)
    assert n == 0
    assert "fallback" not in capfd.readouterr().err
