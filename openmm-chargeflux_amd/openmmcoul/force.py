"""CoulForce — parameter container of the charge-flux electrostatics force.

Mirror of CoulPlugin::CoulForce (reference: openmmapi/include/CoulForce.h:16-150,
openmmapi/src/CoulForce.cpp:12-144) with the same method names, argument order and
defaults (cutoff 1.0 nm, Ewald tolerance 1e-4, no PBC).  The SWIG surface
python/openmmcoul.i:50-76 is a subset of this.  Index errors raise IndexError instead
of the reference's unchecked std::vector access.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _cabi


class CoulForce:
    def __init__(self):
        # CoulForce.cpp:12-16
        self._cutoff = 1.0
        self._ewald_tol = 1e-4
        self._pbc = False
        self._charges: list[float] = []
        self._sigma: list[float] = []
        self._eps: list[float] = []
        self._exclusions: list[tuple[int, int]] = []
        self._fbond_idx: list[tuple[int, int]] = []
        self._fbond_par: list[tuple[float, float]] = []
        self._fangle_idx: list[tuple[int, int, int]] = []
        self._fangle_par: list[tuple[float, float]] = []
        self._fwater_idx: list[tuple[int, int, int]] = []
        self._fwater_par: list[tuple[float, float, float, float, float]] = []
        self._group = 0

    # ---- particles (CoulForce.cpp:18-38) ----------------------------------------
    def addParticle(self, charge, sigma, epsilon):
        self._charges.append(float(charge))
        self._sigma.append(float(sigma))
        self._eps.append(float(epsilon))
        return len(self._charges) - 1

    def getNumParticles(self):
        return len(self._charges)

    def getParticleParameters(self, index):
        self._check(index, len(self._charges), "particle")
        return self._charges[index], self._sigma[index], self._eps[index]

    def setParticleParameters(self, index, charge, sigma, epsilon):
        self._check(index, len(self._charges), "particle")
        self._charges[index] = float(charge)
        self._sigma[index] = float(sigma)
        self._eps[index] = float(epsilon)

    # ---- cutoff / PBC / Ewald (CoulForce.cpp:40-76) ---------------------------------
    def getCutoffDistance(self):
        return self._cutoff

    def setCutoffDistance(self, cutoff):
        self._cutoff = float(cutoff)

    def usesPeriodicBoundaryConditions(self):
        return self._pbc

    def setUsesPeriodicBoundaryConditions(self, ifPeriod):
        self._pbc = bool(ifPeriod)

    def setEwaldErrorTolerance(self, tol):
        self._ewald_tol = float(tol)

    def getEwaldErrorTolerance(self):
        return self._ewald_tol

    # ---- exceptions (CoulForce.cpp:56-68) -------------------------------------------
    def addException(self, p1, p2):
        self._exclusions.append((int(p1), int(p2)))
        return len(self._exclusions) - 1

    def getNumExceptions(self):
        return len(self._exclusions)

    def getExceptionParameters(self, index):
        self._check(index, len(self._exclusions), "exception")
        return self._exclusions[index]

    # ---- flux terms (CoulForce.cpp:78-140) --------------------------------------------
    def addFluxBond(self, p1, p2, k, b):
        self._fbond_idx.append((int(p1), int(p2)))
        self._fbond_par.append((float(k), float(b)))
        return len(self._fbond_idx) - 1

    def getFluxBondParameters(self, index):
        self._check(index, len(self._fbond_idx), "flux bond")
        return (*self._fbond_idx[index], *self._fbond_par[index])

    def getNumFluxBonds(self):
        return len(self._fbond_idx)

    def addFluxAngle(self, p1, p2, p3, k, theta):
        self._fangle_idx.append((int(p1), int(p2), int(p3)))
        self._fangle_par.append((float(k), float(theta)))
        return len(self._fangle_idx) - 1

    def getFluxAngleParameters(self, index):
        self._check(index, len(self._fangle_idx), "flux angle")
        return (*self._fangle_idx[index], *self._fangle_par[index])

    def getNumFluxAngles(self):
        return len(self._fangle_idx)

    def addFluxWater(self, po, ph1, ph2, k1, k2, kub, b0, ub0):
        self._fwater_idx.append((int(po), int(ph1), int(ph2)))
        self._fwater_par.append((float(k1), float(k2), float(kub), float(b0), float(ub0)))
        return len(self._fwater_idx) - 1

    def getFluxWaterParameters(self, index):
        self._check(index, len(self._fwater_idx), "flux water")
        return (*self._fwater_idx[index], *self._fwater_par[index])

    def getNumFluxWaters(self):
        return len(self._fwater_idx)

    # ---- OpenMM Force surface used by the Context mirror --------------------------------
    def getForceGroup(self):
        return self._group

    def setForceGroup(self, group):
        if not 0 <= group <= 31:
            raise ValueError("force group must be in [0, 31]")
        self._group = int(group)

    def updateParametersInContext(self, context):
        """Copy this force's current charges, LJ and flux-term parameters into a Context
        (OpenMM's updateParametersInContext convention; the reference lacks it, SURVEY §8(f)
        #4).  The topology -- which particles the flux terms and exceptions connect -- as well
        as periodicity, cutoff and Ewald tolerance must be unchanged."""
        context._update_force_parameters(self)

    # SWIG %extend helpers (python/openmmcoul.i:67-75)
    @staticmethod
    def cast(force):
        if not isinstance(force, CoulForce):
            raise TypeError("not a CoulForce")
        return force

    @staticmethod
    def isinstance(force):
        return isinstance(force, CoulForce)

    # ---- bulk views ---------------------------------------------------------------------
    def arrays(self):
        """Flat numpy views of the storage, same layout as CoulForce.h:138-149."""
        f64, i32 = np.float64, np.int32
        return {
            "charges": np.asarray(self._charges, f64),
            "sigmas": np.asarray(self._sigma, f64),
            "epsilons": np.asarray(self._eps, f64),
            "exceptions": np.asarray(self._exclusions, i32).reshape(-1, 2),
            "fbond_idx": np.asarray(self._fbond_idx, i32).reshape(-1, 2),
            "fbond_par": np.asarray(self._fbond_par, f64).reshape(-1, 2),
            "fangle_idx": np.asarray(self._fangle_idx, i32).reshape(-1, 3),
            "fangle_par": np.asarray(self._fangle_par, f64).reshape(-1, 2),
            "fwater_idx": np.asarray(self._fwater_idx, i32).reshape(-1, 3),
            "fwater_par": np.asarray(self._fwater_par, f64).reshape(-1, 5),
        }

    def to_cparams(self, default_box=None, one_4pi_eps0=0.0):
        """Build the C-ABI cf_params.  Returns (params, keepalive) — keep the second
        object alive while the struct is in use.  one_4pi_eps0: the Coulomb constant of the
        OpenMM the force is evaluated for (0 = 138.935456, the OpenMM 7.x value; include/chargeflux.h)."""
        a = {k: np.ascontiguousarray(v) for k, v in self.arrays().items()}
        p = _cabi.cf_params()
        dp = lambda x: x.ctypes.data_as(C.POINTER(C.c_double))
        ip = lambda x: x.ctypes.data_as(C.POINTER(C.c_int32))
        p.num_particles = len(a["charges"])
        p.charges, p.sigmas, p.epsilons = dp(a["charges"]), dp(a["sigmas"]), dp(a["epsilons"])
        p.num_exceptions = len(a["exceptions"])
        p.exceptions = ip(a["exceptions"])
        p.num_flux_bonds = len(a["fbond_idx"])
        p.flux_bond_idx, p.flux_bond_params = ip(a["fbond_idx"]), dp(a["fbond_par"])
        p.num_flux_angles = len(a["fangle_idx"])
        p.flux_angle_idx, p.flux_angle_params = ip(a["fangle_idx"]), dp(a["fangle_par"])
        p.num_flux_waters = len(a["fwater_idx"])
        p.flux_water_idx, p.flux_water_params = ip(a["fwater_idx"]), dp(a["fwater_par"])
        p.use_pbc = 1 if self._pbc else 0
        p.cutoff = self._cutoff
        p.ewald_tol = self._ewald_tol
        box = np.zeros(9) if default_box is None else np.asarray(default_box, np.float64).reshape(9)
        for k in range(9):
            p.default_box[k] = float(box[k])
        p.one_4pi_eps0 = float(one_4pi_eps0)
        return p, a

    @staticmethod
    def _check(index, n, what):
        if not 0 <= index < n:
            raise IndexError(f"{what} index {index} out of range [0, {n})")
