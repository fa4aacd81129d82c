"""Drop-in module: `from QPSolver import QPSolver` as with the reference's flat layout (QPSolver.py)."""
from ipm355.solvers import QPSolver  # noqa: F401
