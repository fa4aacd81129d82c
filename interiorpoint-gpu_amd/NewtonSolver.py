"""Drop-in module (reference NewtonSolver.py): Newton solvers run by libipm355.so."""
from ipm355.newton import (NewtonSolver, NewtonSolverCG, NewtonSolverCholesky, NewtonSolverDiagonal,  # noqa: F401
                           NewtonSolverDirect, NewtonSolverNPLstSq, NewtonSolverNPSolve)
