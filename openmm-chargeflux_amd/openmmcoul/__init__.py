"""openmmcoul — MI355X-native ChargeFlux (CoulForce) evaluator.

Same module name and CoulForce surface as the reference's SWIG module
(python/openmmcoul.i); every evaluation runs in the HIP library libchargeflux_hip.so.
"""
from ._cabi import ChargeFluxError, load_library, ONE_4PI_EPS0
from .force import CoulForce
from .kernel import Context, HipCalcCoulForceKernel, State, System
from .serialization import XmlSerializer

__all__ = ["CoulForce", "HipCalcCoulForceKernel", "Context", "State", "System", "ChargeFluxError",
           "load_library", "ONE_4PI_EPS0", "XmlSerializer"]
