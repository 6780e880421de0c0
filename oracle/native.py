"""ORACLE — test infrastructure, NOT product code.

ctypes binding of oracle/lib/liboracle.so (built from oracle/csrc by
oracle/Makefile, also from __graft_entry__.build()): the C restatements whose
fp32 arithmetic must match the device bit for bit (fmaf chains)."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "lib", "liboracle.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            subprocess.run(["make", "-C", _HERE], check=True, stdout=subprocess.DEVNULL)
        L = ctypes.CDLL(_LIB)
        P = ctypes.c_void_p
        L.oracle_full_topk.argtypes = [ctypes.c_int64, P, P, P, P, ctypes.c_int64, P,
                                       ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                       ctypes.c_int32, P, P]
        L.oracle_full_topk.restype = None
        L.oracle_score_chain.argtypes = [P, P, ctypes.c_int32]
        L.oracle_score_chain.restype = ctypes.c_float
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def full_topk(users, tr_ptr, tr_idx, uf, itf, k):
    """Top-k (score desc, item asc) of the masked fp32 fma-chain scores
    (oracle/csrc/eval_full.c). Returns (items [n,k] int32, scores [n,k] f32)."""
    users = np.ascontiguousarray(users, np.int64)
    tr_ptr = np.ascontiguousarray(tr_ptr, np.int32)
    tr_idx = np.ascontiguousarray(tr_idx, np.int32)
    uf = np.ascontiguousarray(uf, np.float32)
    itf = np.ascontiguousarray(itf, np.float32)
    n = users.size
    items = np.empty((n, k), np.int32)
    scores = np.empty((n, k), np.float32)
    lib().oracle_full_topk(n, _p(users), _p(tr_ptr), _p(tr_idx), _p(uf), uf.shape[1], _p(itf),
                           itf.shape[1], uf.shape[1], itf.shape[0], k, _p(items), _p(scores))
    return items, scores


def score_chain(a, b):
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    return float(lib().oracle_score_chain(_p(a), _p(b), a.size))
