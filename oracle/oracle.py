"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of the CPU restatement in cf_oracle.c.

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker
(and the serial CPU baseline "port").  Never imported by the product package.

PARITY UNPINNED: the reference has no tests/golden vectors and cannot be built here
(it requires OpenMM headers and libraries, absent from this image).  This restatement
is pinned only by the physics known-answer tests in tests/test_oracle.py.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libcf_oracle.so")
DP = C.POINTER(C.c_double)


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        L.cfo_create.restype = C.c_void_p
        L.cfo_create.argtypes = [C.c_void_p, C.c_char_p, C.c_int]
        L.cfo_destroy.argtypes = [C.c_void_p]
        L.cfo_ewald.argtypes = [C.c_void_p, DP, C.POINTER(C.c_int32)]
        L.cfo_execute.restype = C.c_double
        L.cfo_execute.argtypes = [C.c_void_p, DP, DP, C.c_int, C.c_int, DP, DP, DP, DP]
        L.cfo_execute_klimit.restype = C.c_double
        L.cfo_execute_klimit.argtypes = [C.c_void_p, DP, DP, C.c_int, C.c_int, DP, DP, C.c_int64]
        L.cfo_time_sample.restype = C.c_int
        L.cfo_time_sample.argtypes = [C.c_void_p, DP, DP, C.c_int64, DP, DP, C.POINTER(C.c_int64)]
        _lib = L
    return _lib


def _dp(a):
    return a.ctypes.data_as(DP)


class Oracle:
    """Reference-semantics evaluator of a CoulForce (ReferenceCoulKernels.cpp:230-636)."""

    def __init__(self, force, default_box=None, one_4pi_eps0=0.0):
        # build the same cf_params the product consumes (layout from include/chargeflux.h)
        import sys
        sys.path.insert(0, os.path.join(os.path.dirname(HERE), "openmm-chargeflux_amd"))
        params, self._keep = force.to_cparams(default_box, one_4pi_eps0)   # 0: 138.935456 (OpenMM 7.x)
        err = C.create_string_buffer(256)
        self._h = lib().cfo_create(C.byref(params), err, 256)
        if not self._h:
            raise ValueError(err.value.decode())
        self.n = force.getNumParticles()

    def __del__(self):
        if getattr(self, "_h", None):
            lib().cfo_destroy(self._h)
            self._h = None

    def ewald(self):
        a = C.c_double()
        k = (C.c_int32 * 3)()
        lib().cfo_ewald(self._h, C.byref(a), k)
        return a.value, tuple(k)

    def execute(self, pos, box=None, include_forces=True, include_energy=True):
        """Returns dict(energy, forces, terms, charges, dedq)."""
        pos = np.ascontiguousarray(np.asarray(pos, np.float64).reshape(self.n, 3))
        b9 = np.zeros(9) if box is None else np.ascontiguousarray(np.asarray(box, np.float64).reshape(9))
        f = np.zeros((self.n, 3))
        terms = np.zeros(4)
        q = np.zeros(self.n)
        dedq = np.zeros(self.n)
        e = lib().cfo_execute(self._h, _dp(pos), _dp(b9), int(include_forces), int(include_energy), _dp(f),
                              _dp(terms), _dp(q), _dp(dedq))
        return {"energy": e, "forces": f, "terms": terms, "charges": q, "dedq": dedq}

    def terms_without_recip(self, pos, box):
        """Energy terms (self, 0, direct, exclusion) with the reciprocal loop skipped."""
        pos = np.ascontiguousarray(np.asarray(pos, np.float64).reshape(self.n, 3))
        b9 = np.ascontiguousarray(np.asarray(box, np.float64).reshape(9))
        f = np.zeros((self.n, 3))
        terms = np.zeros(4)
        lib().cfo_execute_klimit(self._h, _dp(pos), _dp(b9), 0, 1, _dp(f), _dp(terms), 0)
        return terms

    def time_sample(self, pos, box, k_count):
        """CPU-baseline sample: (t_nonrecip, t_recip_for_k_count, k_total)."""
        pos = np.ascontiguousarray(np.asarray(pos, np.float64).reshape(self.n, 3))
        b9 = np.ascontiguousarray(np.asarray(box, np.float64).reshape(9))
        tn, tr, kt = C.c_double(), C.c_double(), C.c_int64()
        rc = lib().cfo_time_sample(self._h, _dp(pos), _dp(b9), int(k_count), C.byref(tn), C.byref(tr), C.byref(kt))
        if rc != 0:
            raise ValueError("time_sample requires a periodic system")
        return tn.value, tr.value, kt.value
