"""CPU: libbbgr.so loads, exports every symbol include/bbgr.h declares, and the
ctypes struct layouts agree with the C header (no compute calls: no GPU here)."""
import ctypes
import re
import subprocess

import pytest

from bbgr import _lib


def test_library_exports_every_header_symbol():
    L = _lib.lib()
    syms = _lib.header_symbols()
    assert len(syms) >= 18
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    assert set(_lib._SIGNATURES) == set(syms)


def test_nm_lists_symbols_as_exported_text():
    out = subprocess.run(["nm", "-D", "--defined-only", str(_lib.LIB_PATH)],
                         capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (bbgr_\w+)", out))
    assert set(_lib.header_symbols()) <= exported


def test_abi_version_and_error_text():
    L = _lib.lib()
    assert L.bbgr_abi_version() == 11
    assert isinstance(L.bbgr_last_error(), bytes)


def _c_sizeof(struct_name: str) -> int:
    src = f'#include "bbgr.h"\n#include <stdio.h>\nint main(){{printf("%zu", sizeof({struct_name}));}}'
    exe = "/tmp/bbgr_sizeof_" + struct_name
    subprocess.run(["gcc", "-x", "c", "-", "-I", str(_lib.HEADER_PATH.parent), "-o", exe],
                   input=src, text=True, check=True)
    return int(subprocess.run([exe], capture_output=True, text=True, check=True).stdout)


@pytest.mark.parametrize("cname,pyty", [("bbgr_csr", _lib.CsrStruct),
                                        ("bbgr_spmm_args", _lib.SpmmArgs),
                                        ("bbgr_bpr_args", _lib.BprArgs),
                                        ("bbgr_eval_args", _lib.EvalArgs)])
def test_struct_layout_matches_header(cname, pyty):
    assert _c_sizeof(cname) == ctypes.sizeof(pyty)


def test_invalid_arguments_rejected_without_gpu():
    """Argument validation happens before any HIP call."""
    L = _lib.lib()
    rc = L.bbgr_spmm(None, None, None)
    assert rc == -1 and b"null" in L.bbgr_last_error()
    rc = L.bbgr_adam(-1, None, None, None, None, 1e-3, 0.9, 0.999, 1e-8, 0.0, 1.0, 1.0, 1.0,
                     None)
    assert rc == -1
    with pytest.raises(_lib.BbgrError, match="BBGR_ERR_INVALID"):
        _lib.call("bbgr_bpr_reduce", 0, None, 0.0, 0.0, None, None)


def test_comm_entry_points_validate_without_gpu():
    """The RCCL exchange ABI rejects bad handles / sizes before touching RCCL;
    destroying a null communicator is a no-op."""
    L = _lib.lib()
    assert L.bbgr_allreduce_items(None, None, 16, None) == -1
    assert L.bbgr_allreduce_items(ctypes.c_void_p(16), None, 16, None) == -1
    assert L.bbgr_comm_init(None, 2, 0, None) == -1
    ids = (ctypes.c_uint8 * 128)()
    comm = ctypes.c_void_p()
    assert L.bbgr_comm_init(ctypes.byref(comm), 2, 2, ids) == -1    # rank >= nranks
    assert L.bbgr_comm_unique_id(None) == -1
    assert L.bbgr_comm_destroy(None) == 0


def test_gpu_required_is_loud():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        _lib.require_gpu()


def test_eval_workspace_query_without_gpu():
    """Size queries (workspace=NULL) are host-only: covered bytes + chunk
    partials (+ the per-lane top-K lists for full ranking)."""
    a = _lib.EvalArgs()
    a.n_users, a.n_items, a.d, a.k_max, a.n_k, a.n_neg = 10000, 5000, 64, 20, 2, 99
    a.ks[0], a.ks[1] = 10, 20
    a.lduf = a.ldif = 64
    a.users = a.te_indptr = a.te_indices = a.tr_indptr = a.tr_indices = 16
    a.uf = a.itf = a.topk = a.item_pop = a.sums = 16
    n = ctypes.c_size_t(0)
    _lib.call("bbgr_eval_sampled", ctypes.byref(a), None, ctypes.byref(n), None)
    assert n.value >= 2 * 5000 + 8 * 2 * 3 * 10
    m = ctypes.c_size_t(0)
    _lib.call("bbgr_eval_full", ctypes.byref(a), None, ctypes.byref(m), None)
    assert m.value >= n.value + 10000 * 2 * 24 * 8
    a.k_max = 40
    with pytest.raises(_lib.BbgrError, match="k_max <= 32"):
        _lib.call("bbgr_eval_full", ctypes.byref(a), None, ctypes.byref(m), None)
