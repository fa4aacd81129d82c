"""Drop-in module: `from LassoSolver import LassoSolver` as with the reference's flat layout (LassoSolver.py)."""
from ipm355.lasso import LassoSolver  # noqa: F401
