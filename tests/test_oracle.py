"""CPU tests of the oracle (oracle/cf_oracle.c): physics known-answer tests that pin the
restatement of ReferenceCoulKernels.cpp, since the reference ships no fixtures and cannot
be built here (parity unpinned against the reference itself)."""
import math

import numpy as np
import pytest

from oracle import Oracle
from openmmcoul import CoulForce, ONE_4PI_EPS0
from openmmcoul import testsystems as ts

MADELUNG_NACL = 1.747564594633182


def test_two_charges_no_pbc():
    f = CoulForce()
    f.addParticle(1.0, 0.0, 0.0)
    f.addParticle(-0.5, 0.0, 0.0)
    o = Oracle(f)
    pos = np.array([[0.1, 0.2, 0.3], [0.4, 0.2, 0.3]])
    r = o.execute(pos)
    expect = ONE_4PI_EPS0 * 1.0 * -0.5 / 0.3
    assert r["energy"] == pytest.approx(expect, rel=1e-14)
    fx = -expect / 0.3  # F0 = -dE/dx0 = -E/r > 0: attractive, atom 0 pulled toward +x
    assert r["forces"][0, 0] == pytest.approx(fx, rel=1e-13)
    assert r["forces"][1, 0] == pytest.approx(-fx, rel=1e-13)
    assert r["dedq"][0] == pytest.approx(ONE_4PI_EPS0 * -0.5 / 0.3, rel=1e-14)


def test_lj_pair_no_pbc():
    # LJ stored as (sigma/2, 2 sqrt(eps)) -> 4 sqrt(e1 e2) [(s/r)^12-(s/r)^6], s = (s1+s2)/2
    f = CoulForce()
    f.addParticle(0.0, 0.3, 0.5)
    f.addParticle(0.0, 0.34, 0.8)
    o = Oracle(f)
    r0 = 0.37
    e = o.execute(np.array([[0, 0, 0], [r0, 0, 0]]))["energy"]
    s = 0.32
    expect = 4 * math.sqrt(0.5 * 0.8) * ((s / r0) ** 12 - (s / r0) ** 6)
    assert e == pytest.approx(expect, rel=1e-13)


def test_ewald_params_match_survey_table():
    # alpha / kmax of configs C2, C3, C5 as tabulated in SURVEY.md §8 (computed from the
    # reference initialize(), ReferenceCoulKernels.cpp:401-420)
    for nw, tol, alpha, kmax in ((1000, 1e-3, 2.49291, 7), (32000, 1e-4, 2.91842, 31), (256000, 1e-4, 2.91842, 65)):
        L = (nw / ts.WATER_DENSITY) ** (1 / 3)
        f = CoulForce()
        f.addParticle(0.0, 0.0, 0.0)
        f.setUsesPeriodicBoundaryConditions(True)
        f.setEwaldErrorTolerance(tol)
        a, k = Oracle(f, np.diag([L, L, L])).ewald()
        assert a == pytest.approx(alpha, abs=5e-6)
        assert k == (kmax, kmax, kmax)


def test_nacl_madelung():
    system, force, pos, box = ts.nacl_crystal(cells=4, a=0.5, cutoff=1.0, ewald_tol=1e-10)
    o = Oracle(force, box)
    r = o.execute(pos, box)
    n = len(pos)
    expect = -(n / 2) * MADELUNG_NACL * ONE_4PI_EPS0 / 0.25
    assert r["energy"] == pytest.approx(expect, rel=2e-9)
    # perfect crystal: every force vanishes by symmetry
    assert np.abs(r["forces"]).max() < 1e-6


def _fd_check(o, pos, box, atoms, h=1e-6, tol=2e-4):
    r = o.execute(pos, box)
    for i in atoms:
        for d in range(3):
            p1, p2 = pos.copy(), pos.copy()
            p1[i, d] += h
            p2[i, d] -= h
            e1 = o.execute(p1, box, include_forces=False)["energy"]
            e2 = o.execute(p2, box, include_forces=False)["energy"]
            fd = -(e1 - e2) / (2 * h)
            assert r["forces"][i, d] == pytest.approx(fd, abs=tol, rel=1e-6), (i, d)


def test_finite_difference_no_pbc_cluster():
    system, force, pos, _ = ts.cluster_c1()
    o = Oracle(force)
    _fd_check(o, pos, None, atoms=[0, 1, 2, 3, 4, 5, 100, 200, 255])


def test_finite_difference_pbc_flux_box():
    system, force, pos, box = ts.water_box(40, cutoff=0.5, ewald_tol=1e-6, every_bond_angle=3)
    o = Oracle(force, box)
    _fd_check(o, pos, box, atoms=[0, 1, 2, 6, 7, 8, 30, 61])


def test_dedq_matches_charge_derivative():
    # q_i = q0_i + flux deltas  =>  dE/dq0_i == dE/dq_i (self + recip + direct + excl)
    system, force, pos, box = ts.water_box(40, cutoff=0.5, ewald_tol=1e-6, every_bond_angle=3)
    r = Oracle(force, box).execute(pos, box)
    h = 1e-6
    for i in (0, 4, 11):
        q, s, e = force.getParticleParameters(i)
        force.setParticleParameters(i, q + h, s, e)
        ep = Oracle(force, box).execute(pos, box, include_forces=False)["energy"]
        force.setParticleParameters(i, q - h, s, e)
        em = Oracle(force, box).execute(pos, box, include_forces=False)["energy"]
        force.setParticleParameters(i, q, s, e)
        assert r["dedq"][i] == pytest.approx((ep - em) / (2 * h), rel=1e-6, abs=1e-5)


def test_charge_conservation_and_flux_formulas():
    system, force, pos, box = ts.water_box(60, cutoff=0.5, every_bond_angle=4)
    r = Oracle(force, box).execute(pos, box)
    q0 = force.arrays()["charges"]
    assert r["charges"].sum() == pytest.approx(q0.sum(), abs=1e-12)
    # FluxWater O charge: dqO = -(dqH1 + dqH2)  (ReferenceCoulKernels.cpp:188-193)
    o = 0
    k1, k2, kub, b0, ub0 = ts.FW
    r12 = np.linalg.norm(pos[1] - pos[0]); r13 = np.linalg.norm(pos[2] - pos[0]); r23 = np.linalg.norm(pos[2] - pos[1])
    dq2 = k1 * (r12 - b0) + k2 * (r13 - b0) + kub * (r23 - ub0)
    dq3 = k1 * (r13 - b0) + k2 * (r12 - b0) + kub * (r23 - ub0)
    assert r["charges"][1] == pytest.approx(ts.Q_H + dq2, abs=1e-14)
    assert r["charges"][2] == pytest.approx(ts.Q_H + dq3, abs=1e-14)
    assert r["charges"][o] == pytest.approx(ts.Q_O - dq2 - dq3, abs=1e-14)


def test_translation_invariance():
    system, force, pos, _ = ts.cluster_c1()
    r = Oracle(force).execute(pos)
    assert np.abs(r["forces"].sum(axis=0)).max() < 1e-8
    system, force, pos, box = ts.water_box(40, cutoff=0.5, ewald_tol=1e-6)
    o = Oracle(force, box)
    e0 = o.execute(pos, box)["energy"]
    p2 = pos.copy()
    p2[3:6] += box[0]          # move one whole water by a lattice vector
    p2[9:12] -= 2 * box[2]
    assert o.execute(p2, box)["energy"] == pytest.approx(e0, rel=1e-10)


def test_energy_flag_quirk():
    # periodic: self + real + exclusion energy are returned even without includeEnergy
    # (ReferenceCoulKernels.cpp:507-510, 592, 619, 633); the reciprocal term is not.
    system, force, pos, box = ts.water_box(40, cutoff=0.5)
    o = Oracle(force, box)
    full = o.execute(pos, box, True, True)
    part = o.execute(pos, box, True, False)
    t = full["terms"]
    assert part["energy"] == pytest.approx(t[0] + t[2] + t[3], rel=1e-13)
    assert full["energy"] == pytest.approx(t.sum(), rel=1e-13)
    # non-periodic: nothing without includeEnergy
    system, force, pos, _ = ts.cluster_c1()
    assert Oracle(force).execute(pos, None, True, False)["energy"] == 0.0


def test_triclinic_reduced_box_accepted_and_validated():
    # OpenMM's reduced form a = (ax,0,0), b = (bx,by,0), c = (cx,cy,cz), |bx|,|cx| <= ax/2, |cy| <= by/2
    system, force, pos, box = ts.triclinic_water_box(60, cutoff=0.5)
    o = Oracle(force, box)
    r = o.execute(pos, box)
    assert np.isfinite(r["energy"]) and np.isfinite(r["forces"]).all()
    bad = box.copy()
    bad[0, 1] = 0.1            # a must lie along x
    with pytest.raises(Exception):
        Oracle(force, bad)
    bad = box.copy()
    bad[1, 0] = 0.6 * box[0, 0]   # |bx| > ax/2
    with pytest.raises(Exception):
        Oracle(force, bad)


def test_finite_difference_triclinic_box():
    # the box-vector minimum image (getDeltaRPeriodic) in the pair and flux terms and the
    # reference's diagonal-only k-sum on unwrapped positions (RCK:513-567) are FD-consistent
    system, force, pos, box = ts.triclinic_water_box(60, cutoff=0.5, ewald_tol=1e-6)
    o = Oracle(force, box)
    _fd_check(o, pos, box, atoms=[0, 1, 2, 6, 7, 8, 30, 61, 120, 179])


def test_triclinic_zero_shear_equals_orthorhombic():
    system, force, pos, box = ts.triclinic_water_box(60, cutoff=0.5, shear=(0.0, 0.0, 0.0))
    o = Oracle(force, box)
    r1 = o.execute(pos, box)
    r2 = o.execute(pos, np.diag(np.diag(box)))
    assert r1["energy"] == r2["energy"] and np.array_equal(r1["forces"], r2["forces"])


def test_coulomb_constant_is_a_parameter():
    """k_e (ONE_4PI_EPS0 of the loading OpenMM, ReferenceCoulKernels.cpp:7) enters every
    electrostatic term linearly and nothing else: E(k_e) = k_e E_c + E_LJ, likewise F and dE/dq
    (charges and dq/dx do not depend on it).  0 selects 138.935456 with identical bits; the C2
    golden fixture (made at 138.935456) is reproduced bit-for-bit by the explicit value."""
    system, force, pos, box = ts.water_box(200, cutoff=0.8, ewald_tol=1e-4, every_bond_angle=3)
    r0 = Oracle(force, box).execute(pos, box)
    rd = Oracle(force, box, one_4pi_eps0=ONE_4PI_EPS0).execute(pos, box)
    assert r0["energy"] == rd["energy"] and np.array_equal(r0["forces"], rd["forces"])
    ks = [100.0, 138.93545764438198, 200.0]
    rs = [Oracle(force, box, one_4pi_eps0=k).execute(pos, box) for k in ks]
    for key in ("energy", "forces", "dedq"):
        a, b, c = (np.asarray(r[key], np.float64) for r in rs)
        slope = (c - a) / (ks[2] - ks[0])
        pred = a + slope * (ks[1] - ks[0])
        assert np.abs(pred - b).max() <= 1e-9 * max(1.0, np.abs(b).max()), key
    assert np.array_equal(rs[0]["charges"], rs[2]["charges"])
    with pytest.raises(ValueError, match="one_4pi_eps0"):
        Oracle(force, box, one_4pi_eps0=-1.0)
