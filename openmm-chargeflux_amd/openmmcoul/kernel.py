"""The HIP implementation of CalcCoulForceKernel, plus a minimal OpenMM-shaped
System/Context/State so the force can be driven (and tested) the way the reference is
driven from OpenMM.

Reference interfaces mirrored:
  CalcCoulForceKernel::{Name, initialize, execute}   openmmapi/include/CoulKernels.h:15-38
  CoulForceImpl::{initialize, calcForcesAndEnergy}   openmmapi/src/CoulForceImpl.cpp:16-27
  System::getDefaultPeriodicBoxVectors               (used at ReferenceCoulKernels.cpp:399-400)

Device arrays are torch tensors (PyTorch is plumbing here: device memory and streams);
host arrays are numpy.  Every evaluation runs in libchargeflux_hip.so — there is no
Python or CPU compute path.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _cabi
from .force import CoulForce

DP = C.POINTER(C.c_double)


def _dp(a: np.ndarray):
    return a.ctypes.data_as(DP)


class System:
    """Minimal stand-in for openmm.System (particle count + default box + forces)."""

    def __init__(self):
        self._masses: list[float] = []
        self._box = np.diag([2.0, 2.0, 2.0]).astype(np.float64)
        self._forces: list = []

    def addParticle(self, mass):
        self._masses.append(float(mass))
        return len(self._masses) - 1

    def getNumParticles(self):
        return len(self._masses)

    def setDefaultPeriodicBoxVectors(self, a, b, c):
        self._box = np.array([a, b, c], dtype=np.float64).reshape(3, 3)

    def getDefaultPeriodicBoxVectors(self):
        return [self._box[0].copy(), self._box[1].copy(), self._box[2].copy()]

    def addForce(self, force):
        self._forces.append(force)
        return len(self._forces) - 1

    def getForces(self):
        return list(self._forces)


def _box9(box) -> np.ndarray:
    if box is None:
        return np.zeros(9)
    return np.ascontiguousarray(np.asarray(box, dtype=np.float64).reshape(9))


class HipCalcCoulForceKernel:
    """CalcCoulForceKernel on MI355X.  initialize() ~ ReferenceCalcCoulForceKernel::initialize
    (ReferenceCoulKernels.cpp:230-422); execute() ~ ...::execute (:424-636)."""

    @staticmethod
    def Name():
        return "CalcCoulForce"

    # reciprocal-sum algorithms (cf_options.kspace_algo, include/chargeflux.h)
    KSPACE_EXACT_MFMA = 0   # exact k-sum, fp64 MFMA separable form
    KSPACE_EXACT_VALU = 1   # exact k-sum, direct sincos (check path)
    KSPACE_GRID = 2         # same k-sum via ES-kernel grid (spread, pruned DFT, interpolate)

    PAIR_LISTS = {"auto": _cabi.CF_PAIR_LIST_AUTO, "cluster": _cabi.CF_PAIR_LIST_CLUSTER,
                  "atom_half": _cabi.CF_PAIR_LIST_ATOM_HALF, "full": _cabi.CF_PAIR_LIST_FULL}
    HANDOVERS = {"event": _cabi.CF_HANDOVER_EVENT, "memory": _cabi.CF_HANDOVER_MEMORY}

    def __init__(self, device: int = 0, stream=None, rank: int = 0, world_size: int = 1, kspace_algo: int = 0,
                 grid_width: int = 0, precision: str = "double", one_4pi_eps0: float = 0.0,
                 pair_list: str = "auto", handover: str = "event", variants: int = 0, list_capacity: int = 0):
        """one_4pi_eps0: ONE_4PI_EPS0 of the OpenMM the force is evaluated for (the reference
        takes it from openmm/reference/SimTKOpenMMRealType.h, ReferenceCoulKernels.cpp:7);
        0 = 138.935456 (OpenMM 7.x), _cabi.ONE_4PI_EPS0_CODATA2018 for OpenMM 8.x.
        pair_list, handover, variants, list_capacity: cf_options fields (include/chargeflux.h):
        the neighbour-list kind ("auto", "cluster", "atom_half", "full"), the second stream's
        fork / join ("event" or the opt-in "memory"), CF_VARIANT_* bits (alternative kernels of the
        same sums) and the cluster-pair list capacity (0 = automatic)."""
        if pair_list not in self.PAIR_LISTS:
            raise ValueError(f"pair_list must be one of {sorted(self.PAIR_LISTS)}")
        if handover not in self.HANDOVERS:
            raise ValueError(f"handover must be one of {sorted(self.HANDOVERS)}")
        self._pair_list = self.PAIR_LISTS[pair_list]
        self._handover = self.HANDOVERS[handover]
        self._variants = int(variants)
        self._list_capacity = int(list_capacity)
        self._lib = _cabi.load_library()
        self._ke = float(one_4pi_eps0)
        self._grid_width = grid_width
        if precision not in ("double", "mixed"):
            raise ValueError("precision must be 'double' or 'mixed'")
        self._precision = _cabi.CF_PRECISION_MIXED if precision == "mixed" else _cabi.CF_PRECISION_DOUBLE
        self._h = C.c_void_p()
        self._device = device
        self._stream = stream
        self._rank, self._world = rank, world_size
        self._algo = kspace_algo
        self._n = 0
        self._pbc = False

    # -------------------------------------------------------------------------------
    def initialize(self, system, force: CoulForce):
        if system.getNumParticles() != force.getNumParticles():
            raise _cabi.ChargeFluxError(_cabi.CF_ERR_INVALID,
                                        "System and CoulForce have different numbers of particles")
        a, b, c = system.getDefaultPeriodicBoxVectors()
        box = np.array([a, b, c], dtype=np.float64).reshape(9)
        params, keep = force.to_cparams(box, self._ke)
        opt = _cabi.cf_options()
        opt.device = self._device
        opt.stream = C.c_void_p(self._stream) if self._stream else None
        opt.rank, opt.world_size, opt.kspace_algo = self._rank, self._world, self._algo
        opt.grid_width = self._grid_width
        opt.precision = self._precision
        opt.handover, opt.pair_list = self._handover, self._pair_list
        opt.variants, opt.list_capacity = self._variants, self._list_capacity
        self.destroy()
        _cabi.check(self._lib.cf_create(C.byref(params), C.byref(opt), C.byref(self._h)), self._lib)
        del keep
        self._n = force.getNumParticles()
        self._pbc = force.usesPeriodicBoundaryConditions()
        return self

    def copyParametersToContext(self, force: CoulForce):
        """New charges / LJ / flux parameters on the same topology (cf_update_parameters; the
        reference has no updateParametersInContext)."""
        if force.getNumParticles() != self._n:
            raise _cabi.ChargeFluxError(_cabi.CF_ERR_INVALID, "the number of particles has changed")
        params, keep = force.to_cparams(None, self._ke)
        _cabi.check(self._lib.cf_update_parameters(self._h, C.byref(params)), self._lib)
        del keep

    def destroy(self):
        if self._h:
            self._lib.cf_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass

    # -------------------------------------------------------------------------------
    def ewald_params(self):
        alpha = C.c_double()
        kmax = (C.c_int32 * 3)()
        _cabi.check(self._lib.cf_get_ewald_params(self._h, C.byref(alpha), kmax), self._lib)
        return alpha.value, tuple(kmax)

    def grid_shape(self):
        """Grid points per axis of the grid reciprocal path ((0, 0, 0) for the exact paths)."""
        ng = (C.c_int32 * 3)()
        w = C.c_int32()
        _cabi.check(self._lib.cf_get_grid_shape(self._h, ng, C.byref(w)), self._lib)
        return tuple(ng)

    def grid_width(self) -> int:
        """ES kernel width W the grid reciprocal path uses (0 for the exact paths)."""
        ng = (C.c_int32 * 3)()
        w = C.c_int32()
        _cabi.check(self._lib.cf_get_grid_shape(self._h, ng, C.byref(w)), self._lib)
        return int(w.value)

    def set_neighbor_skin(self, skin: float):
        """Persistent neighbour list with a skin (nm); 0 = rebuild on every execute (the
        reference's behaviour, ReferenceCoulKernels.cpp:559).  See include/chargeflux.h."""
        _cabi.check(self._lib.cf_set_neighbor_skin(self._h, float(skin)), self._lib)
        return self

    def set_graph(self, enable: bool = True):
        """Replay single-rank evaluations as a captured hipGraph (cf_set_graph): the same kernels
        in the same order, without the per-launch host cost."""
        _cabi.check(self._lib.cf_set_graph(self._h, 1 if enable else 0), self._lib)
        return self

    def set_overlap(self, enable: bool = True):
        """Second stream for the grid path (cf_set_overlap, default on): off launches every kernel
        on the handle's stream, so that kernel durations are the kernels' own; same results."""
        _cabi.check(self._lib.cf_set_overlap(self._h, 1 if enable else 0), self._lib)
        return self

    def graph_stats(self):
        """(captures, replays) since set_graph(True)."""
        c, r = C.c_int64(), C.c_int64()
        _cabi.check(self._lib.cf_get_graph_stats(self._h, C.byref(c), C.byref(r)), self._lib)
        return c.value, r.value

    def pair_list(self):
        """The direct-space list in use: "cluster", "atom_half" or "full" ("auto" before the first
        periodic evaluation and without PBC) -- cf_get_pair_list."""
        k = C.c_int32()
        _cabi.check(self._lib.cf_get_pair_list(self._h, C.byref(k)), self._lib)
        return {v: n for n, v in self.PAIR_LISTS.items()}[k.value]

    def neighbor_stats(self):
        """(list builds, evaluations) since initialize."""
        b, e = C.c_int64(), C.c_int64()
        _cabi.check(self._lib.cf_get_neighbor_stats(self._h, C.byref(b), C.byref(e)), self._lib)
        return b.value, e.value

    def fallback_stats(self):
        """(evaluations that fell back to the fp64 rescan of every atom, list rows rescanned
        after a full-list overflow, union of the reasons: 1 window > 4096 atoms, 2 list overflow /
        unplaceable rows, 4 fixed-point range) since initialize: slow-path diagnostics."""
        a, b, r = C.c_int64(), C.c_int64(), C.c_int32()
        _cabi.check(self._lib.cf_get_fallback_stats(self._h, C.byref(a), C.byref(b), C.byref(r)), self._lib)
        return a.value, b.value, r.value

    def owned_range(self):
        lo, hi = C.c_int32(), C.c_int32()
        _cabi.check(self._lib.cf_get_owned_range(self._h, C.byref(lo), C.byref(hi)), self._lib)
        return lo.value, hi.value

    @staticmethod
    def _flags(include_forces, include_energy):
        return (_cabi.CF_INCLUDE_FORCES if include_forces else 0) | (_cabi.CF_INCLUDE_ENERGY if include_energy else 0)

    def execute_host(self, positions, box=None, includeForces=True, includeEnergy=True, forces=None):
        """Host-memory execute: positions (N,3) nm; forces (N,3) float64 array ADDED to
        (created if None).  Returns (energy, forces)."""
        pos = np.ascontiguousarray(np.asarray(positions, dtype=np.float64).reshape(self._n, 3))
        if forces is None:
            forces = np.zeros((self._n, 3))
        if forces.dtype != np.float64 or not forces.flags.c_contiguous or forces.shape != (self._n, 3):
            raise ValueError("forces must be a C-contiguous float64 (N,3) array")
        e = C.c_double()
        b9 = _box9(box)
        _cabi.check(self._lib.cf_compute_host(self._h, _dp(pos), _dp(b9), self._flags(includeForces, includeEnergy),
                                              _dp(forces), C.byref(e)), self._lib)
        return e.value, forces

    def execute_device(self, positions, box=None, includeForces=True, includeEnergy=True, forces=None, energy=None):
        """Device execute on torch tensors (float64, cuda): forces (N,3) ADDED to, energy
        (1,) overwritten.  Asynchronous on the kernel's stream."""
        b9 = _box9(box)
        fptr = forces.data_ptr() if forces is not None else None
        eptr = energy.data_ptr() if energy is not None else None
        _cabi.check(self._lib.cf_compute(self._h, C.c_void_p(positions.data_ptr()), _dp(b9),
                                         self._flags(includeForces, includeEnergy), C.c_void_p(fptr),
                                         C.c_void_p(eptr)), self._lib)

    def execute_openmm(self, posq, atom_index, padded_n, box=None, includeForces=True, includeEnergy=True,
                       force_buffer=None, energy_buffer=None, posq_correction=None):
        """Execute on an OpenMM GPU platform's own buffers (cf_compute_openmm; the reference's CUDA
        platform binds them at CudaCoulKernels.cpp:523-600): posq (N, 4) float64 or float32 torch
        tensor in the platform's sorted order, atom_index (N,) int32 (sorted slot -> atom),
        force_buffer (3 * padded_n,) int64 fixed point (2^-32 kJ/mol/nm, x | y | z planes by sorted
        slot) ADDED to, energy_buffer a one-element float64 / float32 tensor ADDED to; posq_correction
        (N, 4) float32 for the mixed-precision platform.  posq is never written."""
        import torch
        kind = _cabi.CF_POSQ_FLOAT4 if posq.dtype == torch.float32 else _cabi.CF_POSQ_DOUBLE4
        ekind = _cabi.CF_ENERGY_FLOAT if (energy_buffer is not None and energy_buffer.dtype == torch.float32) \
            else _cabi.CF_ENERGY_DOUBLE
        b9 = _box9(box)
        ptr = lambda t: C.c_void_p(t.data_ptr()) if t is not None else None
        _cabi.check(self._lib.cf_compute_openmm(self._h, ptr(posq), ptr(posq_correction), kind, ptr(atom_index),
                                                int(padded_n), _dp(b9), self._flags(includeForces, includeEnergy),
                                                ptr(force_buffer), ptr(energy_buffer), ekind), self._lib)

    def device_errors(self):
        """CF_GUARD_* bits of the device index guards tripped so far (0 = none; synchronises)."""
        v = C.c_int32()
        _cabi.check(self._lib.cf_get_device_errors(self._h, C.byref(v)), self._lib)
        return v.value

    # split-phase (multi-GPU): begin -> all-reduce kspace_buffer -> end
    def begin(self, positions, box=None, includeForces=True, includeEnergy=True):
        self._b9 = _box9(box)
        _cabi.check(self._lib.cf_compute_begin(self._h, C.c_void_p(positions.data_ptr()), _dp(self._b9),
                                               self._flags(includeForces, includeEnergy)), self._lib)

    def kspace_buffer(self):
        ptr, n = C.c_void_p(), C.c_int64()
        _cabi.check(self._lib.cf_kspace_buffer(self._h, C.byref(ptr), C.byref(n)), self._lib)
        return ptr.value, n.value

    def kspace_tensor(self, device):
        """The structure-factor buffer as a zero-copy torch tensor (None without PBC)."""
        ptr, n = self.kspace_buffer()
        if not n:
            return None
        from .distributed import device_buffer_as_tensor
        return device_buffer_as_tensor(ptr, n, device)

    def direct(self):
        """Launch the direct-space kernels of the begun evaluation now (optional; lets a
        multi-rank caller overlap them with the S(k) all-reduce)."""
        _cabi.check(self._lib.cf_compute_direct(self._h), self._lib)

    def end(self, forces=None, energy=None):
        fptr = forces.data_ptr() if forces is not None else None
        eptr = energy.data_ptr() if energy is not None else None
        _cabi.check(self._lib.cf_compute_end(self._h, C.c_void_p(fptr), C.c_void_p(eptr)), self._lib)

    def execute(self, context, includeForces, includeEnergy):
        """OpenMM-style execute(ContextImpl&, bool, bool) -> energy (ReferenceCoulKernels.cpp:424)."""
        return context._execute_kernel(self, includeForces, includeEnergy)

    # diagnostics ----------------------------------------------------------------------
    def charges(self):
        out = np.zeros(self._n)
        _cabi.check(self._lib.cf_get_charges(self._h, _dp(out)), self._lib)
        return out

    def dedq(self):
        out = np.zeros(self._n)
        _cabi.check(self._lib.cf_get_dedq(self._h, _dp(out)), self._lib)
        return out

    def energy_terms(self):
        out = np.zeros(4)
        _cabi.check(self._lib.cf_get_energy_terms(self._h, _dp(out)), self._lib)
        return out

    # phase names in cf_get_timing order (bit p of cf_set_timing_mask)
    PHASES = ("flux_terms", "atoms_prep", "cell_sort", "neighbor_list", "kspace_tables", "kspace_sfac",
              "kspace_coeffs", "kspace_force", "direct_pairs", "assemble", "energy", "grid_sort", "grid_spread",
              "grid_dft_fwd", "grid_dft_inv", "grid_interp", "direct_excl")

    def set_timing(self, enable=True, phases=None):
        """Per-kernel HIP-event timing of every phase, or only of the named phases."""
        if phases is None:
            _cabi.check(self._lib.cf_set_timing(self._h, 1 if enable else 0), self._lib)
        else:
            mask = 0
            for p in phases:
                mask |= 1 << self.PHASES.index(p)
            _cabi.check(self._lib.cf_set_timing_mask(self._h, mask if enable else 0), self._lib)

    def timing(self):
        """{phase: (total_ms, launches)} recorded since set_timing(True)."""
        nmax = 32
        names = C.create_string_buffer(16 * nmax)
        tot = (C.c_double * nmax)()
        calls = (C.c_int32 * nmax)()
        nph = C.c_int32()
        _cabi.check(self._lib.cf_get_timing(self._h, nmax, names, tot, calls, C.byref(nph)), self._lib)
        out = {}
        for p in range(nph.value):
            nm = names.raw[16 * p:16 * p + 16].split(b"\0")[0].decode()
            out[nm] = (tot[p], calls[p])
        return out

    def synchronize(self):
        _cabi.check(self._lib.cf_synchronize(self._h), self._lib)


class State:
    def __init__(self, energy, forces):
        self._e, self._f = energy, forces

    def getPotentialEnergy(self):
        return self._e

    def getForces(self, asNumpy=True):
        return self._f


class Context:
    """Minimal OpenMM-Context mirror: owns one HipCalcCoulForceKernel per CoulForce in the
    System (CoulForceImpl::initialize, CoulForceImpl.cpp:16-21) and evaluates them with the
    force-group test of CoulForceImpl::calcForcesAndEnergy (CoulForceImpl.cpp:23-27)."""

    def __init__(self, system: System, device: int = 0, kspace_algo: int = 0, grid_width: int = 0,
                 precision: str = "double", one_4pi_eps0: float = 0.0):
        self._system = system
        self._n = system.getNumParticles()
        self._pos = np.zeros((self._n, 3))
        a, b, c = system.getDefaultPeriodicBoxVectors()
        self._box = np.array([a, b, c], dtype=np.float64)
        self._impls = []
        for f in system.getForces():
            if isinstance(f, CoulForce):
                k = HipCalcCoulForceKernel(device=device, kspace_algo=kspace_algo, grid_width=grid_width,
                                           precision=precision, one_4pi_eps0=one_4pi_eps0).initialize(system, f)
                self._impls.append((f, k))

    def setPositions(self, positions):
        self._pos = np.ascontiguousarray(np.asarray(positions, dtype=np.float64).reshape(self._n, 3))

    def setPeriodicBoxVectors(self, a, b, c):
        self._box = np.array([a, b, c], dtype=np.float64)

    def kernels(self):
        return [k for _, k in self._impls]

    def _update_force_parameters(self, force):
        hit = False
        for f, k in self._impls:
            if f is force:
                k.copyParametersToContext(force)
                hit = True
        if not hit:
            raise ValueError("this CoulForce is not part of the Context's System")

    def _execute_kernel(self, kernel, include_forces, include_energy):
        forces = np.zeros((self._n, 3))
        e, _ = kernel.execute_host(self._pos, self._box, include_forces, include_energy, forces)
        self._last_forces = forces
        return e

    def getState(self, getEnergy=False, getForces=False, groups=-1):
        energy = 0.0
        forces = np.zeros((self._n, 3))
        for f, k in self._impls:
            if (groups & (1 << f.getForceGroup())) == 0:
                continue
            e, _ = k.execute_host(self._pos, self._box, bool(getForces), bool(getEnergy), forces)
            energy += e
        return State(energy if getEnergy else None, forces if getForces else None)
