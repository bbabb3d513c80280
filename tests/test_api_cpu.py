"""CPU tests of the boundary: the C-ABI library loads and exports every symbol that
include/chargeflux.h declares; the Python mirror of CoulForce keeps the reference API
(openmmapi/include/CoulForce.h:22-133, python/openmmcoul.i:50-76)."""
import ctypes as C
import os
import re

import pytest
import torch

from openmmcoul import CoulForce, HipCalcCoulForceKernel, ChargeFluxError, _cabi
from openmmcoul import testsystems as ts

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "chargeflux.h")


def _declared():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"CF_EXPORT\s+[\w\s\*]+?\b(cf_\w+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    names = _declared()
    assert len(names) >= 18
    lib = C.CDLL(_cabi.LIB_PATH)
    for n in names:
        assert hasattr(lib, n), n
    assert {n for n, _, _ in _cabi.SIGNATURES} == set(names)


def test_api_version_and_error_without_device():
    lib = _cabi.load_library()
    assert lib.cf_api_version() == 4   # 3: cf_options.handover, pair_list, variants, list_capacity; 4: guards, cf_compute_openmm
    if torch.cuda.is_available():
        pytest.skip("a HIP device is present")
    system, force, pos, box = ts.water_box(20, cutoff=0.4)
    with pytest.raises(ChargeFluxError) as ei:
        HipCalcCoulForceKernel().initialize(system, force)
    assert ei.value.code == _cabi.CF_ERR_HIP


def test_null_arguments_are_rejected():
    lib = _cabi.load_library()
    h = C.c_void_p()
    assert lib.cf_create(None, None, C.byref(h)) == _cabi.CF_ERR_INVALID
    assert b"null" in lib.cf_last_error()
    assert lib.cf_compute_end(None, None, None) == _cabi.CF_ERR_INVALID
    assert lib.cf_destroy(None) == _cabi.CF_OK


def test_coulforce_defaults_and_accessors():
    f = CoulForce()
    assert f.getCutoffDistance() == 1.0          # CoulForce.cpp:13
    assert f.getEwaldErrorTolerance() == 1e-4    # CoulForce.cpp:14
    assert f.usesPeriodicBoundaryConditions() is False
    f.addParticle(-0.8, 0.3, 0.6)
    f.addParticle(0.4, 0.0, 0.0)
    f.addParticle(0.4, 0.0, 0.0)
    assert f.getNumParticles() == 3
    f.setParticleParameters(1, 0.41, 0.01, 0.02)
    assert f.getParticleParameters(1) == (0.41, 0.01, 0.02)
    f.addException(0, 1)
    assert f.getNumExceptions() == 1 and f.getExceptionParameters(0) == (0, 1)
    f.addFluxBond(0, 1, -0.8, 0.1)
    f.addFluxAngle(1, 0, 2, 0.1, 1.8)
    f.addFluxWater(0, 1, 2, -1.0, 0.2, 0.5, 0.1, 0.15)
    assert f.getFluxBondParameters(0) == (0, 1, -0.8, 0.1)
    assert f.getFluxAngleParameters(0) == (1, 0, 2, 0.1, 1.8)
    assert f.getFluxWaterParameters(0) == (0, 1, 2, -1.0, 0.2, 0.5, 0.1, 0.15)
    assert (f.getNumFluxBonds(), f.getNumFluxAngles(), f.getNumFluxWaters()) == (1, 1, 1)
    f.setCutoffDistance(0.9)
    f.setEwaldErrorTolerance(5e-4)
    f.setUsesPeriodicBoundaryConditions(True)
    assert (f.getCutoffDistance(), f.getEwaldErrorTolerance(), f.usesPeriodicBoundaryConditions()) == (0.9, 5e-4, True)
    assert CoulForce.isinstance(f) and CoulForce.cast(f) is f
    with pytest.raises(IndexError):
        f.getParticleParameters(3)
    assert HipCalcCoulForceKernel.Name() == "CalcCoulForce"   # CoulKernels.h:17-19


def test_cparams_layout_matches_storage():
    system, force, pos, box = ts.water_box(30, cutoff=0.4, every_bond_angle=3)
    p, keep = force.to_cparams(box)
    assert p.num_particles == 90
    assert p.num_exceptions == 90
    assert p.num_flux_waters == 20 and p.num_flux_bonds == 20 and p.num_flux_angles == 10
    assert p.use_pbc == 1 and p.cutoff == 0.4
    assert [p.default_box[i] for i in (0, 4, 8)] == [box[0, 0]] * 3
    assert p.flux_water_params[5 * 3 + 4] == ts.FW[4]
