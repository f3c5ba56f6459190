"""Shared test helpers: canonical SHA-256 digests of CSR arrays (matches tests/golden/make_golden.py)."""
import hashlib

import numpy as np


def digest(row_ptr, col, val, vdtype="<u4"):
    return {
        "nnz": int(len(col)),
        "row_ptr": hashlib.sha256(np.asarray(row_ptr, dtype="<u8").tobytes()).hexdigest(),
        "col": hashlib.sha256(np.asarray(col, dtype="<u4").tobytes()).hexdigest(),
        "val": hashlib.sha256(np.asarray(val, dtype=vdtype).tobytes()).hexdigest(),
    }


def assert_digest(got, want, what=""):
    for k in ("nnz", "row_ptr", "col", "val"):
        assert got[k] == want[k], f"{what}: {k} mismatch"
