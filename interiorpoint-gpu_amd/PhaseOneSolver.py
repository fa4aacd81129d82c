"""Drop-in module (reference PhaseOneSolver.py)."""
from ipm355.phase_one import PhaseOneSolver  # noqa: F401
