"""Synthetic systems of SURVEY.md §8(d): flexible charge-flux water boxes (C2-C5) and the
256-atom non-periodic cluster (C1).  Data are synthetic (no network, no datasets)."""
from __future__ import annotations

import math

import numpy as np

from .force import CoulForce
from .kernel import System

SEED = 20261015
R_OH = 0.09572
THETA_HOH = math.radians(104.52)
Q_O, Q_H = -0.834, 0.417
SIG_O, EPS_O = 0.315061, 0.636386
WATER_DENSITY = 33.43  # molecules / nm^3
# FluxWater (k1, k2, kub, b0, ub0) and the bond/angle variant used by every 10th molecule
FW = (-1.0, 0.2, 0.5, 0.09572, 0.15139)
FB = (-0.8, 0.09572)
FA = (0.1, 1.82421813)


def _random_rotations(rng, n):
    q = rng.normal(size=(n, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    w, x, y, z = q.T
    return np.stack([
        np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)], -1),
        np.stack([2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)], -1),
        np.stack([2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)], -1),
    ], 1)


def _water_geometry(rng, centres):
    n = len(centres)
    h = THETA_HOH / 2
    local = np.array([[0, 0, 0], [R_OH * math.sin(h), R_OH * math.cos(h), 0],
                      [-R_OH * math.sin(h), R_OH * math.cos(h), 0]])
    rot = _random_rotations(rng, n)
    return centres[:, None, :] + np.einsum("nij,kj->nki", rot, local)


def add_water(force: CoulForce, o: int, flux_bond_angle: bool):
    h1, h2 = o + 1, o + 2
    force.addException(o, h1)
    force.addException(o, h2)
    force.addException(h1, h2)
    if flux_bond_angle:
        force.addFluxBond(o, h1, *FB)
        force.addFluxBond(o, h2, *FB)
        force.addFluxAngle(h1, o, h2, *FA)
    else:
        force.addFluxWater(o, h1, h2, *FW)


def water_box(n_waters: int, cutoff: float = 1.0, ewald_tol: float = 1e-4, seed: int = SEED,
              density: float = WATER_DENSITY, every_bond_angle: int = 10):
    """Periodic cubic water box.  Returns (system, force, positions[N,3], box[3,3])."""
    rng = np.random.default_rng(seed)
    L = (n_waters / density) ** (1.0 / 3.0)
    m = int(math.ceil(n_waters ** (1.0 / 3.0) - 1e-9))
    a = L / m
    idx = np.array([(i, j, k) for i in range(m) for j in range(m) for k in range(m)][:n_waters], dtype=np.float64)
    centres = (idx + 0.5) * a + rng.uniform(-0.02, 0.02, size=(n_waters, 3))
    pos = _water_geometry(rng, centres).reshape(-1, 3)
    force = CoulForce()
    system = System()
    for w in range(n_waters):
        for q, s, e, mass in ((Q_O, SIG_O, EPS_O, 15.999), (Q_H, 0.0, 0.0, 1.008), (Q_H, 0.0, 0.0, 1.008)):
            force.addParticle(q, s, e)
            system.addParticle(mass)
    for w in range(n_waters):
        add_water(force, 3 * w, every_bond_angle > 0 and w % every_bond_angle == every_bond_angle - 1)
    force.setUsesPeriodicBoundaryConditions(True)
    force.setCutoffDistance(cutoff)
    force.setEwaldErrorTolerance(ewald_tol)
    box = np.diag([L, L, L])
    system.setDefaultPeriodicBoxVectors(*box)
    system.addForce(force)
    return system, force, pos, box


def triclinic_water_box(n_waters: int, cutoff: float = 0.7, ewald_tol: float = 1e-4, seed: int = SEED,
                        shear=(0.3, -0.25, 0.2), every_bond_angle: int = 3):
    """Periodic water box with a reduced triclinic cell a = (L,0,0), b = (sb L, L, 0),
    c = (sc L, scy L, L) (OpenMM's reduced form: |shears| <= 1/2).  Molecule centres sit on
    the lattice's own fractional grid, so no two periodic images overlap.  Returns
    (system, force, positions[N,3], box[3,3] with the box vectors as rows)."""
    rng = np.random.default_rng(seed)
    L = (n_waters / WATER_DENSITY) ** (1.0 / 3.0)
    m = int(math.ceil(n_waters ** (1.0 / 3.0) - 1e-9))
    box = np.array([[L, 0.0, 0.0], [shear[0] * L, L, 0.0], [shear[1] * L, shear[2] * L, L]])
    idx = np.array([(i, j, k) for i in range(m) for j in range(m) for k in range(m)][:n_waters], dtype=np.float64)
    frac = (idx + 0.5) / m + rng.uniform(-0.005, 0.005, size=(n_waters, 3))
    centres = frac @ box
    pos = _water_geometry(rng, centres).reshape(-1, 3)
    force = CoulForce()
    system = System()
    for w in range(n_waters):
        for q, s, e, mass in ((Q_O, SIG_O, EPS_O, 15.999), (Q_H, 0.0, 0.0, 1.008), (Q_H, 0.0, 0.0, 1.008)):
            force.addParticle(q, s, e)
            system.addParticle(mass)
    for w in range(n_waters):
        add_water(force, 3 * w, every_bond_angle > 0 and w % every_bond_angle == every_bond_angle - 1)
    force.setUsesPeriodicBoundaryConditions(True)
    force.setCutoffDistance(cutoff)
    force.setEwaldErrorTolerance(ewald_tol)
    system.setDefaultPeriodicBoxVectors(*box)
    system.addForce(force)
    return system, force, pos, box


def cluster_c1(seed: int = SEED):
    """C1: 256-atom non-periodic cluster: 64 waters (32 FluxWater, 32 bond+angle) in a
    1.3 nm cube plus 64 LJ ions (+-1 e, sigma 0.3 nm, eps 0.5 kJ/mol)."""
    rng = np.random.default_rng(seed)
    a = 1.3 / 4
    grid = np.array([(i, j, k) for i in range(4) for j in range(4) for k in range(4)], dtype=np.float64)
    wcent = (grid + 0.25) * a + rng.uniform(-0.02, 0.02, size=(64, 3))
    icent = (grid + 0.75) * a + rng.uniform(-0.02, 0.02, size=(64, 3))
    wpos = _water_geometry(rng, wcent).reshape(-1, 3)
    force = CoulForce()
    system = System()
    for w in range(64):
        for q, s, e, mass in ((Q_O, SIG_O, EPS_O, 15.999), (Q_H, 0.0, 0.0, 1.008), (Q_H, 0.0, 0.0, 1.008)):
            force.addParticle(q, s, e)
            system.addParticle(mass)
    for w in range(64):
        add_water(force, 3 * w, w % 2 == 1)
    for i in range(64):
        force.addParticle(1.0 if i % 2 == 0 else -1.0, 0.3, 0.5)
        system.addParticle(22.99 if i % 2 == 0 else 35.45)
    pos = np.concatenate([wpos, icent])
    system.addForce(force)
    return system, force, pos, None


def nacl_crystal(cells: int = 4, a: float = 0.5, cutoff: float = 1.0, ewald_tol: float = 1e-10):
    """Rock-salt crystal (Madelung known answer): cells^3 conventional cells, lattice a."""
    force = CoulForce()
    system = System()
    pos = []
    basis = [(0, 0, 0), (0.5, 0.5, 0), (0.5, 0, 0.5), (0, 0.5, 0.5)]
    for i in range(cells):
        for j in range(cells):
            for k in range(cells):
                for b in basis:
                    for shift, q in (((0, 0, 0), 1.0), ((0.5, 0, 0), -1.0)):
                        r = (np.array([i, j, k]) + np.array(b) + np.array(shift)) * a
                        pos.append(r)
                        force.addParticle(q, 0.0, 0.0)
                        system.addParticle(1.0)
    L = cells * a
    force.setUsesPeriodicBoundaryConditions(True)
    force.setCutoffDistance(cutoff)
    force.setEwaldErrorTolerance(ewald_tol)
    box = np.diag([L, L, L])
    system.setDefaultPeriodicBoxVectors(*box)
    system.addForce(force)
    return system, force, np.array(pos), box


CONFIGS = {
    "C1": dict(kind="cluster"),
    "C2": dict(kind="box", n_waters=1000, cutoff=1.0, ewald_tol=1e-3),
    "C3": dict(kind="box", n_waters=32000, cutoff=1.0, ewald_tol=1e-4),
    "C5": dict(kind="box", n_waters=256000, cutoff=1.0, ewald_tol=1e-4),
}


def make(config: str):
    c = CONFIGS[config]
    if c["kind"] == "cluster":
        return cluster_c1()
    return water_box(c["n_waters"], cutoff=c["cutoff"], ewald_tol=c["ewald_tol"])
