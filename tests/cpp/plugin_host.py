"""TEST INFRASTRUCTURE ONLY — ctypes access to tests/cpp/libcf_plugin_host.so, which plays
OpenMM's part for the compiled plugin libOpenMMCoulHIP.so (built by `make -C
openmm-chargeflux_amd/plugin compat` against tests/cpp/openmm_compat and the reference's own
openmmapi/include headers).  One process holds one platform registry, as OpenMM does."""
import ctypes as C
import os

import numpy as np

from tests.cpp.adapter import DP, IP, Flat, flat

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libcf_plugin_host.so")
COMPAT_LIB = os.path.join(HERE, "openmm_compat", "lib")
PLUGIN7 = os.path.join(COMPAT_LIB, "plugins", "libOpenMMCoulHIP.so")       # ONE_4PI_EPS0 138.935456
PLUGIN8 = os.path.join(COMPAT_LIB, "plugins_openmm8", "libOpenMMCoulHIP.so")   # 138.93545764438198
SYMBOLS = ("registerPlatforms", "registerKernelFactories", "registerCoulHipKernelFactories",
           "coulHipRegistrationReport")

_L = None
_plugins = {}


def available():
    return all(os.path.exists(p) for p in (LIB, PLUGIN7, PLUGIN8))


def lib():
    global _L
    if _L is None:
        L = C.CDLL(LIB)
        L.cfh_last_error.restype = C.c_char_p
        L.cfh_registration_report.restype = C.c_char_p
        L.cfh_load_plugin.argtypes = [C.c_char_p, C.POINTER(C.c_int), C.POINTER(C.c_void_p)]
        L.cfh_register.argtypes = [C.c_void_p]
        L.cfh_register_foreign_factory.argtypes = [C.c_char_p]
        L.cfh_kernel_owner.argtypes = [C.c_char_p, C.POINTER(C.c_int)]
        L.cfh_factory_rejects_name.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.c_int]
        L.cfh_execute.argtypes = [C.POINTER(Flat), DP, C.c_char_p, DP, DP, C.c_int, C.c_int, DP, DP]
        L.cfh_serialize.argtypes = [C.POINTER(Flat), C.c_int, C.c_char_p, C.c_int, C.POINTER(C.c_int)]
        L.cfh_deserialize.argtypes = [C.c_char_p, C.POINTER(C.c_void_p)]
        L.cfh_force_counts.argtypes = [C.c_void_p, IP, DP]
        L.cfh_force_arrays.argtypes = [C.c_void_p, DP, DP, DP, IP, IP, DP, IP, DP, IP, DP]
        L.cfh_force_serialize.argtypes = [C.c_void_p, C.c_char_p, C.c_int, C.POINTER(C.c_int)]
        L.cfh_force_free.argtypes = [C.c_void_p]
        L.cfh_init()
        _L = L
    return _L


def _check(rc):
    if rc != 0:
        raise RuntimeError(lib().cfh_last_error().decode())


def load_plugin(path):
    """dlopen the plugin (once per path) -> (handle, names of the entry points found)."""
    if path not in _plugins:
        found, h = C.c_int(), C.c_void_p()
        _check(lib().cfh_load_plugin(path.encode(), C.byref(found), C.byref(h)))
        _plugins[path] = (h, tuple(n for k, n in enumerate(SYMBOLS) if found.value >> k & 1))
    return _plugins[path]


def register(path):
    """Make `path`'s factory the registered one (its registerCoulHipKernelFactories)."""
    h, _ = load_plugin(path)
    _check(lib().cfh_register(h))


def report():
    return lib().cfh_registration_report().decode()


def register_foreign(platform):
    _check(lib().cfh_register_foreign_factory(platform.encode()))


def owner(platform):
    """0: no CalcCoulForce kernel, 1: the HIP kernel, 2: another plugin's."""
    o = C.c_int()
    _check(lib().cfh_kernel_owner(platform.encode(), C.byref(o)))
    return o.value


def factory_rejects(platform, name):
    msg = C.create_string_buffer(512)
    rc = lib().cfh_factory_rejects_name(platform.encode(), name.encode(), msg, 512)
    return rc == 0, msg.value.decode()


def execute(force, default_box, pos, box, platform="Reference", include_forces=True, include_energy=True,
            forces=None):
    """Platform::createKernel("CalcCoulForce") -> initialize(System, CoulForce) -> execute
    (ContextImpl) with ReferencePlatform::PlatformData buffers -> (energy, forces)."""
    f, keep = flat(force)
    db = None if default_box is None else np.ascontiguousarray(np.asarray(default_box, np.float64).reshape(9))
    b9 = None if box is None else np.ascontiguousarray(np.asarray(box, np.float64).reshape(9))
    p = np.ascontiguousarray(np.asarray(pos, np.float64).reshape(-1, 3))
    out = np.zeros_like(p) if forces is None else np.ascontiguousarray(forces, np.float64).copy()
    e = C.c_double()
    _check(lib().cfh_execute(C.byref(f), None if db is None else db.ctypes.data_as(DP), platform.encode(),
                             p.ctypes.data_as(DP), None if b9 is None else b9.ctypes.data_as(DP),
                             int(include_forces), int(include_energy), out.ctypes.data_as(DP), C.byref(e)))
    del keep
    return e.value, out


def serialize(force, force_group=0):
    """XmlSerializer::serialize<CoulForce>(force, "Force") through the plugin's CoulForceProxy."""
    f, keep = flat(force)
    need = C.c_int()
    _check(lib().cfh_serialize(C.byref(f), force_group, None, 0, C.byref(need)))
    buf = C.create_string_buffer(need.value)
    _check(lib().cfh_serialize(C.byref(f), force_group, buf, need.value, C.byref(need)))
    del keep
    return buf.value.decode()


def deserialize(xml):
    """XmlSerializer::deserialize -> (arrays like CoulForce.arrays(), scal (pbc, cutoff, tol, group),
    the re-serialized text)."""
    h = C.c_void_p()
    _check(lib().cfh_deserialize(xml.encode(), C.byref(h)))
    try:
        cnt = (C.c_int * 5)()
        scal = np.zeros(4)
        _check(lib().cfh_force_counts(h, cnt, scal.ctypes.data_as(DP)))
        n, e, b, a, w = cnt
        out = {"charges": np.zeros(n), "sigmas": np.zeros(n), "epsilons": np.zeros(n),
               "exceptions": np.zeros((e, 2), np.int32), "fbond_idx": np.zeros((b, 2), np.int32),
               "fbond_par": np.zeros((b, 2)), "fangle_idx": np.zeros((a, 3), np.int32),
               "fangle_par": np.zeros((a, 2)), "fwater_idx": np.zeros((w, 3), np.int32),
               "fwater_par": np.zeros((w, 5))}
        ptr = lambda x: x.ctypes.data_as(IP if x.dtype == np.int32 else DP)
        _check(lib().cfh_force_arrays(h, *[ptr(out[k]) for k in out]))
        need = C.c_int()
        _check(lib().cfh_force_serialize(h, None, 0, C.byref(need)))
        buf = C.create_string_buffer(need.value)
        _check(lib().cfh_force_serialize(h, buf, need.value, C.byref(need)))
        return out, scal, buf.value.decode()
    finally:
        lib().cfh_force_free(h)
