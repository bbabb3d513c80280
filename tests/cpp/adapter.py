"""TEST INFRASTRUCTURE ONLY — ctypes access to tests/cpp/libcf_adapter_test.so, the OpenMM
plugin's C++ layer (openmm-chargeflux_amd/plugin/include) instantiated on a C++ CoulForce with
the reference's API (tests/cpp/CoulForceStandIn.h).  Built by openmm-chargeflux_amd/plugin/Makefile
(part of __graft_entry__.build())."""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libcf_adapter_test.so")
DP, IP = C.POINTER(C.c_double), C.POINTER(C.c_int32)


class Flat(C.Structure):
    _fields_ = [("n", C.c_int), ("q", DP), ("sig", DP), ("eps", DP), ("ne", C.c_int), ("ex", IP),
                ("nb", C.c_int), ("bi", IP), ("bp", DP), ("na", C.c_int), ("ai", IP), ("ap", DP),
                ("nw", C.c_int), ("wi", IP), ("wp", DP), ("pbc", C.c_int), ("cutoff", C.c_double),
                ("tol", C.c_double)]


def load():
    if not os.path.exists(LIB):
        raise RuntimeError(f"{LIB} missing: run __graft_entry__.build()")
    L = C.CDLL(LIB)
    L.cfa_last_error.restype = C.c_char_p
    L.cfa_marshal.argtypes = [C.POINTER(Flat), C.c_int, DP, DP, DP, DP, IP, IP, DP, IP, DP, IP, DP, DP, DP]
    L.cfa_execute_count.argtypes = [C.POINTER(Flat), DP, C.c_int, DP, DP, C.c_int, DP, DP, C.POINTER(C.c_longlong)]
    L.cfa_execute.argtypes = [C.POINTER(Flat), C.POINTER(Flat), DP, C.c_int, C.c_int, DP, DP, C.c_int, C.c_int,
                              DP, DP]
    return L


def flat(force):
    """Flat arrays of an openmmcoul.CoulForce (the Python mirror) -> (Flat, keepalive)."""
    a = {k: np.ascontiguousarray(v) for k, v in force.arrays().items()}
    f = Flat()
    dp = lambda x: x.ctypes.data_as(DP)
    ip = lambda x: x.ctypes.data_as(IP)
    f.n = len(a["charges"])
    f.q, f.sig, f.eps = dp(a["charges"]), dp(a["sigmas"]), dp(a["epsilons"])
    f.ne, f.ex = len(a["exceptions"]), ip(a["exceptions"])
    f.nb, f.bi, f.bp = len(a["fbond_idx"]), ip(a["fbond_idx"]), dp(a["fbond_par"])
    f.na, f.ai, f.ap = len(a["fangle_idx"]), ip(a["fangle_idx"]), dp(a["fangle_par"])
    f.nw, f.wi, f.wp = len(a["fwater_idx"]), ip(a["fwater_idx"]), dp(a["fwater_par"])
    f.pbc = 1 if force.usesPeriodicBoundaryConditions() else 0
    f.cutoff, f.tol = force.getCutoffDistance(), force.getEwaldErrorTolerance()
    return f, a


def marshal(force, box, n_system=None):
    """The cf_params the plugin's adapter builds (for a System of n_system particles, default
    the force's count), as numpy arrays."""
    L = load()
    f, keep = flat(force)
    n, e, b, a, w = f.n, f.ne, f.nb, f.na, f.nw
    out = {"charges": np.zeros(n), "sigmas": np.zeros(n), "epsilons": np.zeros(n),
           "exceptions": np.zeros((e, 2), np.int32), "fbond_idx": np.zeros((b, 2), np.int32),
           "fbond_par": np.zeros((b, 2)), "fangle_idx": np.zeros((a, 3), np.int32), "fangle_par": np.zeros((a, 2)),
           "fwater_idx": np.zeros((w, 3), np.int32), "fwater_par": np.zeros((w, 5))}
    scal, box_out = np.zeros(3), np.zeros(9)
    b9 = np.zeros(9) if box is None else np.ascontiguousarray(np.asarray(box, np.float64).reshape(9))
    ptr = lambda x: x.ctypes.data_as(IP if x.dtype == np.int32 else DP)
    rc = L.cfa_marshal(C.byref(f), f.n if n_system is None else n_system, ptr(b9), *[ptr(out[k]) for k in ("charges", "sigmas", "epsilons", "exceptions",
                                                                    "fbond_idx", "fbond_par", "fangle_idx",
                                                                    "fangle_par", "fwater_idx", "fwater_par")],
                       ptr(scal), ptr(box_out))
    if rc:
        raise RuntimeError(L.cfa_last_error().decode())
    del keep
    return out, scal, box_out.reshape(3, 3)


def execute(force, default_box, pos, box, kspace_algo=2, precision=0, include_forces=True, include_energy=True,
            update_to=None):
    """KernelCore::initialize + execute_host through the plugin layer -> (energy, forces)."""
    L = load()
    f, keep = flat(force)
    f2, keep2 = flat(update_to) if update_to is not None else (None, None)
    db = np.ascontiguousarray(np.asarray(default_box if default_box is not None else np.zeros((3, 3)),
                                         np.float64).reshape(9))
    b9 = np.zeros(9) if box is None else np.ascontiguousarray(np.asarray(box, np.float64).reshape(9))
    p = np.ascontiguousarray(np.asarray(pos, np.float64).reshape(-1, 3))
    forces = np.zeros_like(p)
    e = C.c_double()
    rc = L.cfa_execute(C.byref(f), C.byref(f2) if f2 is not None else None, db.ctypes.data_as(DP), kspace_algo,
                       precision, p.ctypes.data_as(DP), b9.ctypes.data_as(DP), int(include_forces),
                       int(include_energy), forces.ctypes.data_as(DP), C.byref(e))
    if rc:
        raise RuntimeError(f"cfa_execute failed ({rc}): {L.cfa_last_error().decode()}")
    del keep, keep2
    return e.value, forces


def execute_count(force, default_box, pos, box, calls, kspace_algo=2):
    """KernelCore::initialize + `calls` x execute_host -> (energy, forces summed over the calls,
    KernelCore::fallback_evaluations())."""
    L = load()
    f, keep = flat(force)
    db = np.ascontiguousarray(np.asarray(default_box, np.float64).reshape(9))
    b9 = np.ascontiguousarray(np.asarray(box, np.float64).reshape(9))
    p = np.ascontiguousarray(np.asarray(pos, np.float64).reshape(-1, 3))
    forces = np.zeros_like(p)
    e = C.c_double()
    n = C.c_longlong()
    rc = L.cfa_execute_count(C.byref(f), db.ctypes.data_as(DP), kspace_algo, p.ctypes.data_as(DP),
                             b9.ctypes.data_as(DP), int(calls), forces.ctypes.data_as(DP), C.byref(e), C.byref(n))
    if rc:
        raise RuntimeError(f"cfa_execute_count failed ({rc}): {L.cfa_last_error().decode()}")
    del keep
    return e.value, forces, n.value
