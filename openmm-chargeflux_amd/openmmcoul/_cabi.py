"""ctypes binding of the C-ABI declared in include/chargeflux.h.

This is the reference-side binding a Python user of `openmmcoul` goes through (the
reference's own Python surface is the SWIG module python/openmmcoul.i; see
INTEGRATION.md).  The product library is ``openmm-chargeflux_amd/libchargeflux_hip.so``;
loading fails loudly when it is missing — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(_PKG_ROOT, "libchargeflux_hip.so")

CF_OK = 0
CF_ERR_INVALID = -1
CF_ERR_HIP = -2
CF_ERR_STATE = -3
CF_ERR_NOMEM = -4
CF_PRECISION_DOUBLE = 0
CF_PRECISION_MIXED = 1
CF_HANDOVER_EVENT = 0
CF_HANDOVER_MEMORY = 1
CF_PAIR_LIST_AUTO = 0
CF_PAIR_LIST_CLUSTER = 1
CF_PAIR_LIST_ATOM_HALF = 2
CF_PAIR_LIST_FULL = 3
CF_VARIANT_GEMM_DFT = 1
CF_VARIANT_VECTOR_SPREAD = 2
CF_VARIANT_MFMA_SPREAD = 4
CF_VARIANT_INTERP1 = 8
CF_VARIANT_INTERP2 = 16


def CF_VARIANT_BLOCK_ROUNDS(r: int) -> int:
    return (int(r) & 15) << 8


CF_GUARD_CELL_BOUNDS = 1
CF_GUARD_CLUSTER_TABLE = 2
CF_GUARD_LIST_ENTRY = 4
CF_GUARD_GRID_BINS = 8
CF_GUARD_NEIGHBOR = 16
CF_GUARD_ATOM_INDEX = 32
CF_GUARD_REBUILD_FLAG = 64
CF_POSQ_DOUBLE4 = 0
CF_POSQ_FLOAT4 = 1
CF_ENERGY_DOUBLE = 0
CF_ENERGY_FLOAT = 1
CF_INCLUDE_FORCES = 1
CF_INCLUDE_ENERGY = 2
ONE_4PI_EPS0 = 138.935456                    # OpenMM 7.x headers: cf_params.one_4pi_eps0 = 0
ONE_4PI_EPS0_CODATA2018 = 138.93545764438198  # OpenMM 8.x headers (CODATA 2018)


class cf_params(C.Structure):
    _fields_ = [
        ("num_particles", C.c_int32),
        ("charges", C.POINTER(C.c_double)),
        ("sigmas", C.POINTER(C.c_double)),
        ("epsilons", C.POINTER(C.c_double)),
        ("num_exceptions", C.c_int32),
        ("exceptions", C.POINTER(C.c_int32)),
        ("num_flux_bonds", C.c_int32),
        ("flux_bond_idx", C.POINTER(C.c_int32)),
        ("flux_bond_params", C.POINTER(C.c_double)),
        ("num_flux_angles", C.c_int32),
        ("flux_angle_idx", C.POINTER(C.c_int32)),
        ("flux_angle_params", C.POINTER(C.c_double)),
        ("num_flux_waters", C.c_int32),
        ("flux_water_idx", C.POINTER(C.c_int32)),
        ("flux_water_params", C.POINTER(C.c_double)),
        ("use_pbc", C.c_int32),
        ("cutoff", C.c_double),
        ("ewald_tol", C.c_double),
        ("default_box", C.c_double * 9),
        ("one_4pi_eps0", C.c_double),
    ]


class cf_options(C.Structure):
    _fields_ = [
        ("device", C.c_int32),
        ("stream", C.c_void_p),
        ("rank", C.c_int32),
        ("world_size", C.c_int32),
        ("kspace_algo", C.c_int32),
        ("grid_width", C.c_int32),
        ("precision", C.c_int32),
        ("handover", C.c_int32),
        ("pair_list", C.c_int32),
        ("variants", C.c_int32),
        ("list_capacity", C.c_int32),
        ("reserved", C.c_int32 * 1),
    ]


DP = C.POINTER(C.c_double)

# (name, restype, argtypes) for every symbol in include/chargeflux.h
SIGNATURES = [
    ("cf_api_version", C.c_int, []),
    ("cf_last_error", C.c_char_p, []),
    ("cf_create", C.c_int, [C.POINTER(cf_params), C.POINTER(cf_options), C.POINTER(C.c_void_p)]),
    ("cf_destroy", C.c_int, [C.c_void_p]),
    ("cf_get_ewald_params", C.c_int, [C.c_void_p, DP, C.POINTER(C.c_int32)]),
    ("cf_get_owned_range", C.c_int, [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    ("cf_get_grid_shape", C.c_int, [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    ("cf_compute", C.c_int, [C.c_void_p, C.c_void_p, DP, C.c_int, C.c_void_p, C.c_void_p]),
    ("cf_compute_begin", C.c_int, [C.c_void_p, C.c_void_p, DP, C.c_int]),
    ("cf_kspace_buffer", C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_int64)]),
    ("cf_compute_direct", C.c_int, [C.c_void_p]),
    ("cf_compute_end", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    ("cf_compute_host", C.c_int, [C.c_void_p, DP, DP, C.c_int, DP, DP]),
    ("cf_get_charges", C.c_int, [C.c_void_p, DP]),
    ("cf_get_dedq", C.c_int, [C.c_void_p, DP]),
    ("cf_get_energy_terms", C.c_int, [C.c_void_p, DP]),
    ("cf_synchronize", C.c_int, [C.c_void_p]),
    ("cf_set_timing", C.c_int, [C.c_void_p, C.c_int]),
    ("cf_set_timing_mask", C.c_int, [C.c_void_p, C.c_uint32]),
    ("cf_get_timing", C.c_int, [C.c_void_p, C.c_int32, C.c_char_p, DP, C.POINTER(C.c_int32),
                                C.POINTER(C.c_int32)]),
    ("cf_partition", C.c_int, [C.POINTER(cf_params), C.c_int32, C.c_int32, C.POINTER(C.c_int32),
                               C.POINTER(C.c_int32)]),
    ("cf_set_neighbor_skin", C.c_int, [C.c_void_p, C.c_double]),
    ("cf_update_parameters", C.c_int, [C.c_void_p, C.POINTER(cf_params)]),
    ("cf_get_neighbor_stats", C.c_int, [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    ("cf_set_graph", C.c_int, [C.c_void_p, C.c_int]),
    ("cf_set_overlap", C.c_int, [C.c_void_p, C.c_int]),
    ("cf_get_fallback_stats", C.c_int, [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int64),
                                        C.POINTER(C.c_int32)]),
    ("cf_get_graph_stats", C.c_int, [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    ("cf_get_pair_list", C.c_int, [C.c_void_p, C.POINTER(C.c_int32)]),
    ("cf_get_device_errors", C.c_int, [C.c_void_p, C.POINTER(C.c_int32)]),
    ("cf_compute_openmm", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_int32, DP,
                                    C.c_int, C.c_void_p, C.c_void_p, C.c_int32]),
]

_lib = None
_lock = threading.Lock()


class ChargeFluxError(Exception):
    """Raised for a non-zero C-ABI return code (the reference raises OpenMMException,
    which SWIG maps to Python Exception: python/openmmcoul.i:26-33)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"[{code}] {msg}")
        self.code = code


def load_library(path: str | None = None):
    """Load libchargeflux_hip.so (raises if absent: the product has no fallback)."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise RuntimeError(
                f"HIP extension {p} not found; build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "or `make -C openmm-chargeflux_amd/csrc` (no CPU fallback exists)")
        lib = C.CDLL(p, mode=C.RTLD_GLOBAL)
        for name, res, args in SIGNATURES:
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if path is None:
            _lib = lib
        return lib


def check(rc: int, lib=None):
    if rc != CF_OK:
        lib = lib or load_library()
        msg = lib.cf_last_error()
        raise ChargeFluxError(rc, msg.decode() if msg else "unknown error")
