"""CPU checks of the C-ABI boundary: the library loads and exports every entry point
declared in include/ipm355.h, and the ctypes struct layouts match the header (no GPU calls)."""
import ctypes
import os
import re

import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "ipm355.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ipm_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from ipm355 import _lib
    lib = _lib.load_library()
    names = declared_functions()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # every declared function also has a ctypes prototype
    assert set(names) <= set(_lib.EXPORTS), set(names) - set(_lib.EXPORTS)


def test_version_and_workspace_query_without_gpu():
    from ipm355 import _lib
    lib = _lib.load_library()
    assert lib.ipm_version() == 1
    d = _lib.ProblemDesc()
    d.kind = _lib.KIND_QP
    d.n = 2048
    d.m = 512
    d.C = 1  # non-null marker; only sizes are read
    d.ldc = 2048
    ws = lib.ipm_workspace_bytes(ctypes.byref(d))
    # H and the least-squares backup's eigenvectors (Q9: carved up front, never grown on the hot
    # path) dominate: 2 x 2048^2 doubles
    assert 2 * 2048 * 2048 * 8 <= ws < 2048 * 2048 * 8 * 4


def test_struct_sizes_match_header_layout():
    from ipm355 import _lib
    # ipm_problem_desc: 4 int32 + 8-byte fields ... computed by ctypes with C alignment
    assert ctypes.sizeof(_lib.NewtonOpts) == 4 * 4 + 4 * 8 + 8 + 8
    assert ctypes.sizeof(_lib.NewtonResult) == 4 * 4 + 6 * 8
    assert ctypes.sizeof(_lib.ProblemDesc) % 8 == 0


def test_product_path_fails_loudly_without_gpu():
    import numpy as np
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from ipm355 import IPMBackendError, LPSolver
    with pytest.raises(IPMBackendError):
        LPSolver(c=np.ones(3), check_cvxpy=False)
