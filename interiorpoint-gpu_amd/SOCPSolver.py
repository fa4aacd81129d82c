"""Drop-in module: `from SOCPSolver import SOCPSolver` as with the reference's flat layout (SOCPSolver.py)."""
from ipm355.solvers import SOCPSolver  # noqa: F401
