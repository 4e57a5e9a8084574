"""Test helper: the reference's ctypes marshalling restated (mlp_utils.py:33-164).

The reference module itself imports the loma compiler and wandb at import time, so tests restate
its behaviour: separately allocated rows (not contiguous), Python-list conversion, readback via
per-element indexing.
"""
import ctypes

import numpy as np


def to_ctypes(arr):
    """mlp_utils.convert_ndim_array_to_ndim_ctypes: float -> c_float, int -> c_int rows."""
    a = np.asarray(arr)
    ct = ctypes.c_int if np.issubdtype(a.dtype, np.integer) else ctypes.c_float
    lst = a.tolist()
    if a.ndim == 1:
        return (ct * len(lst))(*lst)
    if a.ndim == 2:
        LP = ctypes.POINTER(ct)
        rows = (LP * len(lst))()
        keep = []
        for i, r in enumerate(lst):
            row = (ct * len(r))(*r)
            keep.append(row)
            rows[i] = row
        p = ctypes.cast(rows, ctypes.POINTER(LP))
        p._keep = (rows, keep)
        return p
    if a.ndim == 3:
        LP = ctypes.POINTER(ct)
        LPP = ctypes.POINTER(LP)
        top = (LPP * len(lst))()
        keep = []
        for i, plane in enumerate(lst):
            rows = (LP * len(plane))()
            for j, r in enumerate(plane):
                row = (ct * len(r))(*r)
                keep.append(row)
                rows[j] = row
            keep.append(rows)
            top[i] = rows
        p = ctypes.cast(top, ctypes.POINTER(LPP))
        p._keep = (top, keep)
        return p
    raise ValueError("Unsupported number of dimensions")


def from_ctypes(p, shape):
    """mlp_utils.lp_lp_c_float_to_numpy / lp_lp_lp_c_float_to_numpy."""
    out = np.zeros(shape, np.float32)
    if len(shape) == 2:
        for r in range(shape[0]):
            for c in range(shape[1]):
                out[r, c] = p[r][c]
    else:
        for d in range(shape[0]):
            for r in range(shape[1]):
                for c in range(shape[2]):
                    out[d, r, c] = p[d][r][c]
    return out
