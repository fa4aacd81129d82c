"""Drop-in module: `from LPSolver import LPSolver` as with the reference's flat layout (LPSolver.py)."""
from ipm355.solvers import LPSolver  # noqa: F401
