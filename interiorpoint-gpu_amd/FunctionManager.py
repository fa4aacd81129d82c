"""Drop-in module (reference FunctionManager.py): device-backed barrier oracles."""
from ipm355.function_manager import (FunctionManagerLP, FunctionManagerPhase1, FunctionManagerQP,  # noqa: F401
                                     FunctionManagerSOCP, FunctionManagerSOCPPhase1)
