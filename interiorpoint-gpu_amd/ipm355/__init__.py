"""ipm355 -- MI355X-native interior-point Newton hot path behind the
LPSolver / QPSolver / SOCPSolver API of fdeguire03/InteriorPoint-GPU.

Host code: this package (Python, mirrors the reference's classes).
Device code: libipm355.so (hand-written HIP for gfx950, C ABI in include/ipm355.h).
"""
from ._lib import IPMBackendError, load_library  # noqa: F401
from .device import set_linesearch_mode  # noqa: F401
from .lasso import LassoSolver  # noqa: F401
from .function_manager import (FunctionManagerLP, FunctionManagerPhase1, FunctionManagerQP,  # noqa: F401
                               FunctionManagerSOCP, FunctionManagerSOCPPhase1)
from .newton import *  # noqa: F401,F403
from .phase_one import PhaseOneSolver  # noqa: F401
from .solvers import LPSolver, QPSolver, SOCPSolver  # noqa: F401

__all__ = ["LPSolver", "QPSolver", "SOCPSolver", "LassoSolver", "PhaseOneSolver", "FunctionManagerLP", "FunctionManagerQP",
           "FunctionManagerPhase1", "FunctionManagerSOCP", "FunctionManagerSOCPPhase1", "IPMBackendError",
           "load_library"]
