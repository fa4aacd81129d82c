"""Drop-in module (reference NewtonSolverInfeasibleStart.py)."""
from ipm355.newton import *  # noqa: F401,F403
