"""ctypes binding of libbbgr.so (the C ABI declared in include/bbgr.h).

The shared library is the product: every device computation of this package
goes through it. There is no CPU fallback — if the library is missing, or
no GPU is visible when a kernel is called, this module raises.

torch is imported first so that libbbgr.so binds to the HIP runtime torch
already loaded (both carry SONAME libamdhip64.so.7): one runtime, one device
context, torch's caching allocator owns every buffer we touch, and every call
is ordered on torch's current stream.
"""
from __future__ import annotations

import ctypes
import os
import re
from pathlib import Path

import torch  # noqa: F401  (must load torch's HIP runtime before libbbgr.so)

PKG_DIR = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("BBGR_LIB", PKG_DIR / "lib" / "libbbgr.so"))   # override: A/B builds
HEADER_PATH = PKG_DIR.parent / "include" / "bbgr.h"

BBGR_OK = 0
STATUS = {0: "BBGR_OK", -1: "BBGR_ERR_INVALID", -2: "BBGR_ERR_UNSUPPORTED",
          -3: "BBGR_ERR_HIP", -4: "BBGR_ERR_WORKSPACE"}

OP_GS, OP_METHOD_A, OP_J, OP_SYM = 0, 1, 2, 3
NEG_CAP = 65536

c_int32 = ctypes.c_int32
c_int64 = ctypes.c_int64
c_float = ctypes.c_float
c_double = ctypes.c_double
c_void_p = ctypes.c_void_p
c_size_t = ctypes.c_size_t
c_uint64 = ctypes.c_uint64


class BbgrError(RuntimeError):
    """A libbbgr entry point returned a negative bbgr_status."""

    def __init__(self, fn: str, rc: int, msg: str):
        super().__init__(f"{fn} failed: {STATUS.get(rc, rc)}: {msg}")
        self.rc = rc


class CsrStruct(ctypes.Structure):
    _fields_ = [
        ("n_rows", c_int32), ("n_cols", c_int32), ("nnz", c_int64),
        ("indptr", c_void_p), ("indices", c_void_p),
        ("long_threshold", c_int32), ("chunk_edges", c_int32),
        ("n_chunks", c_int32), ("n_split", c_int32),
        ("chunks", c_void_p), ("split", c_void_p),
    ]


class SpmmArgs(ctypes.Structure):
    _fields_ = [
        ("d", c_int32),
        ("x", c_void_p), ("ldx", c_int64),
        ("weight_mode", c_int32),
        ("edge_val", c_void_p), ("col_scale", c_void_p), ("col_scale_s", c_float),
        ("y", c_void_p), ("ldy", c_int64),
        ("y_scale", c_void_p), ("y_scale_s", c_float),
        ("add", c_void_p), ("ldadd", c_int64),
        ("add_scale", c_void_p), ("add_scale_s", c_float),
        ("acc_in", c_void_p), ("ldacc_in", c_int64),
        ("acc_out", c_void_p), ("ldacc_out", c_int64),
        ("acc_scale", c_void_p), ("acc_scale_s", c_float),
        ("gamma", c_float),
        ("partial", c_void_p),
        ("src_mask", c_void_p),
        ("row_mask", c_void_p),
        ("acc_mask", c_void_p),
        ("add_mask", c_void_p),
        ("row_list", c_void_p),
        ("n_row_list", c_int64),
        ("use_range", c_int32),
        ("range", c_int32 * 6),
        ("adam_param", c_void_p), ("adam_exp_avg", c_void_p), ("adam_exp_avg_sq", c_void_p),
        ("adam_ld", c_int64), ("adam_lr", c_float), ("adam_beta1", c_float),
        ("adam_beta2", c_float), ("adam_eps", c_float), ("adam_weight_decay", c_float),
        ("adam_bias_correction1", c_float), ("adam_bias_correction2_sqrt", c_float),
        ("stream_from", c_int32), ("stream_out_from", c_int32),
        ("adam_bc_table", c_void_p), ("adam_state", c_void_p),
        ("y_map", c_void_p), ("acc_map", c_void_p), ("add_map", c_void_p),
        ("src_bits", c_void_p),
        ("row_count", c_void_p),
        ("acc_in_map", c_void_p),
        ("adam_grad", c_void_p), ("adam_grad_ld", c_int64), ("adam_grad_scale", c_float),
        ("adam_map", c_void_p),
        ("adam_moments_unmapped", c_int32),
        ("tag_out", c_void_p), ("tag_mask", c_void_p), ("src_tagged", c_void_p),
        ("adam_mirror", c_void_p), ("src_mask_bits", c_void_p),
    ]


class BprArgs(ctypes.Structure):
    _fields_ = [
        ("batch", c_int64), ("d", c_int32),
        ("n_users", c_int64), ("n_items", c_int64),
        ("users", c_void_p), ("pos", c_void_p), ("neg", c_void_p),
        ("uf", c_void_p), ("lduf", c_int64),
        ("itf", c_void_p), ("ldif", c_int64),
        ("ue", c_void_p), ("ldue", c_int64),
        ("ie", c_void_p), ("ldie", c_int64),
        ("pop", c_void_p),
        ("reg", c_float), ("lambda_fair", c_float),
        ("parts", c_void_p), ("dloss", c_void_p),
        ("g_uf", c_void_p), ("ldguf", c_int64),
        ("g_if", c_void_p), ("ldgif", c_int64),
        ("g_ue", c_void_p), ("ldgue", c_int64),
        ("g_ie", c_void_p), ("ldgie", c_int64),
        ("contrib", c_void_p), ("ldcontrib", c_int64),
        ("scores_out", c_void_p), ("scores", c_void_p),
    ]


class EvalArgs(ctypes.Structure):
    _fields_ = [
        ("n_users", c_int64), ("users", c_void_p),
        ("te_indptr", c_void_p), ("te_indices", c_void_p),
        ("tr_indptr", c_void_p), ("tr_indices", c_void_p),
        ("uf", c_void_p), ("lduf", c_int64), ("itf", c_void_p), ("ldif", c_int64),
        ("d", c_int32), ("n_items", c_int32), ("n_neg", c_int32), ("k_max", c_int32),
        ("n_k", c_int32), ("ks", c_int32 * 8),
        ("seed", c_uint64), ("counter", c_uint64),
        ("item_pop", c_void_p), ("self_info_denom", c_float), ("group", c_void_p),
        ("pos_rank", c_void_p), ("topk", c_void_p), ("topk_score", c_void_p),
        ("cand_out", c_void_p), ("fail_count", c_void_p), ("sums", c_void_p),
        ("cand_in", c_void_p),
    ]


class Pcg64State(ctypes.Structure):
    """bbgr_pcg64: numpy's PCG64 bit_generator.state (128-bit state and
    increment as two 64-bit halves, the buffered 32-bit output)."""
    _fields_ = [
        ("state_hi", c_uint64), ("state_lo", c_uint64),
        ("inc_hi", c_uint64), ("inc_lo", c_uint64),
        ("has_uint32", c_int32), ("uinteger", ctypes.c_uint32),
    ]


class BatchArgs(ctypes.Structure):
    """bbgr_batch_args (bbgr_batch_begin / bbgr_batch_end)."""
    _fields_ = [
        ("batch", c_int64), ("users", c_void_p), ("pos", c_void_p), ("neg", c_void_p),
        ("n_users", c_int64), ("n_items", c_int64),
        ("user_indptr", c_void_p), ("user_indices", c_void_p),
        ("mask_u", c_void_p), ("mask_i", c_void_p),
        ("list", c_void_p), ("count", c_void_p),
        ("slot_map", c_void_p), ("slot_bits", c_void_p),
        ("g_u", c_void_p), ("g_i", c_void_p), ("g_side", c_void_p),
        ("ld_gu", c_int64), ("ld_gi", c_int64), ("ld_side", c_int64),
        ("d", c_int32),
    ]


class RowsMarkArgs(ctypes.Structure):
    """bbgr_rows_mark_args (bbgr_rows_mark)."""
    _fields_ = [
        ("n_users_listed", c_int64), ("n_items_listed", c_int64),
        ("users", c_void_p), ("items", c_void_p),
        ("n_users", c_int64), ("n_items", c_int64),
        ("user_rank", c_void_p), ("item_rank", c_void_p),
        ("user_indptr", c_void_p), ("user_indices", c_void_p),
        ("mask_u", c_void_p), ("mask_i", c_void_p), ("frontier", c_void_p),
        ("mask_u_in", c_void_p), ("mask_i_in", c_void_p),
        ("user_list", c_void_p), ("user_count", c_void_p),
        ("frontier_list", c_void_p), ("frontier_count", c_void_p),
    ]


_P = c_void_p
_SIGNATURES = {
    "bbgr_abi_version": ([], c_int32),
    "bbgr_last_error": ([], ctypes.c_char_p),
    "bbgr_device_info": ([ctypes.c_int, _P, ctypes.c_char_p, ctypes.c_int], c_int32),
    "bbgr_sync": ([_P], c_int32),
    "bbgr_profile_marker": ([c_int32, _P], c_int32),
    "bbgr_csr_build": ([c_int64, _P, _P, c_int32, c_int32, _P, _P, _P, _P,
                        ctypes.POINTER(c_size_t), _P], c_int32),
    "bbgr_csr_plan_count": ([ctypes.POINTER(CsrStruct), ctypes.POINTER(c_int32),
                             ctypes.POINTER(c_int32), _P, ctypes.POINTER(c_size_t), _P],
                            c_int32),
    "bbgr_csr_plan_build": ([ctypes.POINTER(CsrStruct), _P, _P, _P,
                             ctypes.POINTER(c_size_t), _P], c_int32),
    "bbgr_operator_scales": ([c_int32, c_int32, c_int32, _P, _P, _P, _P, _P, _P, _P,
                              _P, _P, _P, _P, _P], c_int32),
    "bbgr_gather_scale": ([c_int64, _P, _P, _P, _P], c_int32),
    "bbgr_degree_count": ([c_int64, _P, c_int32, _P, _P], c_int32),
    "bbgr_degree_count_ws": ([c_int64, _P, c_int32, _P, _P, ctypes.POINTER(c_size_t), _P],
                             c_int32),
    "bbgr_degree_order": ([c_int32, _P, _P, _P, _P, ctypes.POINTER(c_size_t), _P], c_int32),
    "bbgr_relabel": ([c_int64, _P, _P, _P, _P], c_int32),
    "bbgr_spmm": ([ctypes.POINTER(CsrStruct), ctypes.POINTER(SpmmArgs), _P], c_int32),
    "bbgr_epilogue": ([c_int32, _P, c_int64, ctypes.POINTER(SpmmArgs), _P], c_int32),
    "bbgr_bpr": ([ctypes.POINTER(BprArgs), _P], c_int32),
    "bbgr_bpr_reduce": ([c_int64, _P, c_float, c_float, _P, _P], c_int32),
    "bbgr_adam": ([c_int64, _P, _P, _P, _P, c_float, c_float, c_float, c_float,
                   c_float, c_float, c_float, c_float, _P], c_int32),
    "bbgr_adam_dev": ([c_int64, _P, _P, _P, _P, c_float, c_float, c_float, c_float,
                       c_float, c_float, _P, _P, _P], c_int32),
    "bbgr_step_begin": ([_P, _P], c_int32),
    "bbgr_mark_rows": ([c_int64, _P, ctypes.c_uint8, _P, c_int64, _P], c_int32),
    "bbgr_comm_unique_id": ([_P], c_int32),
    "bbgr_comm_init": ([_P, c_int32, c_int32, _P], c_int32),
    "bbgr_comm_destroy": ([_P], c_int32),
    "bbgr_allreduce_items": ([_P, _P, c_int64, _P], c_int32),
    "bbgr_comm_allreduce": ([_P, _P, c_int64, c_int32, c_int32, _P], c_int32),
    "bbgr_comm_allgather": ([_P, _P, _P, c_int64, c_int32, _P], c_int32),
    "bbgr_ewa_normalize": ([ctypes.POINTER(CsrStruct), _P, _P, _P, _P, c_int64, c_int32, c_int32,
                            c_float, c_float, c_float, _P, _P, _P, _P,
                            ctypes.POINTER(c_size_t), _P], c_int32),
    "bbgr_scatter_add_rows": ([c_int64, _P, _P, c_int64, _P, c_int64, c_int32, c_int64, _P,
                               ctypes.POINTER(c_size_t), _P], c_int32),
    "bbgr_scatter_plan": ([c_int64, _P, c_int64, _P, ctypes.POINTER(c_size_t), _P], c_int32),
    "bbgr_scatter_apply": ([c_int64, c_int64, _P, _P, c_int64, _P, c_int64, _P, c_int64, c_int32,
                            _P], c_int32),
    "bbgr_mark_neighbors": ([c_int64, _P, _P, _P, ctypes.c_uint8, _P, _P], c_int32),
    "bbgr_mark_slots": ([c_int64, _P, _P, _P, _P, c_int32, _P], c_int32),
    "bbgr_batch_begin": ([ctypes.POINTER(BatchArgs), _P], c_int32),
    "bbgr_mask_pack": ([c_int64, _P, _P, _P], c_int32),
    "bbgr_batch_end": ([ctypes.POINTER(BatchArgs), _P], c_int32),
    "bbgr_rows_mark": ([ctypes.POINTER(RowsMarkArgs), _P], c_int32),
    "bbgr_mark_list": ([c_int64, _P, _P, _P, _P, c_int64, _P, _P, _P], c_int32),
    "bbgr_slots_from_perms": ([c_int64, _P, _P, _P, _P, _P], c_int32),
    "bbgr_transpose_slots": ([ctypes.POINTER(CsrStruct), ctypes.POINTER(CsrStruct), _P, _P],
                             c_int32),
    "bbgr_mark_neighbors_of_mask": ([c_int64, _P, _P, _P, _P, ctypes.c_uint8, _P, _P],
                                    c_int32),
    "bbgr_row_support": ([c_int64, c_int32, _P, c_int64, _P, _P, _P, _P, _P], c_int32),
    "bbgr_rows_zero": ([c_int64, _P, _P, c_int64, c_int32, _P], c_int32),
    "bbgr_rows_axpy": ([c_int64, _P, c_float, _P, c_int64, _P, c_int64, c_int32, _P],
                       c_int32),
    "bbgr_pop_cdf": ([c_int32, _P, c_double, _P, _P, ctypes.POINTER(c_size_t), _P],
                     c_int32),
    "bbgr_sample": ([c_int64, _P, _P, _P, c_int32, _P, c_float, c_int32, c_uint64,
                     c_uint64, _P, _P, _P, _P], c_int32),
    "bbgr_sample_dev": ([c_int64, _P, _P, _P, c_int32, _P, c_float, c_int32, c_uint64,
                         _P, _P, _P, _P, _P], c_int32),
    "bbgr_shuffle": ([c_int64, _P, _P, c_uint64, c_uint64, _P,
                      ctypes.POINTER(c_size_t), _P], c_int32),
    "bbgr_eval_sampled": ([ctypes.POINTER(EvalArgs), _P, ctypes.POINTER(c_size_t), _P],
                          c_int32),
    "bbgr_eval_full": ([ctypes.POINTER(EvalArgs), _P, ctypes.POINTER(c_size_t), _P], c_int32),
    "bbgr_eval_draw_candidates": ([ctypes.POINTER(Pcg64State), c_int64, _P, _P, _P, _P, _P,
                                   c_int64, c_int32, _P], c_int32),
    "bbgr_nonempty_rows": ([c_int32, _P, _P, _P, _P, ctypes.POINTER(c_size_t), _P],
                           c_int32),
    "bbgr_mask_to_list": ([c_int64, _P, _P, _P, _P, ctypes.POINTER(c_size_t), _P], c_int32),
    "bbgr_list_offsets": ([c_int32, _P, _P, _P, _P, _P], c_int32),
    "bbgr_list_positions": ([c_int64, _P, _P, _P, _P], c_int32),
    "bbgr_rows_gather": ([c_int64, _P, _P, c_int64, _P, c_int64, c_int32, _P], c_int32),
    "bbgr_rows_copy": ([c_int64, _P, _P, c_int64, _P, c_int64, c_int32, _P], c_int32),
    "bbgr_first_slot": ([c_int64, _P, c_int64, _P, _P, _P], c_int32),
    "bbgr_ego_slots": ([c_int64, _P, _P, _P, c_int64, c_int64, _P, _P, _P, _P, _P, _P, _P, _P],
                       c_int32),
    "bbgr_graph_rows": ([c_int64, _P, c_int64, _P, _P, _P], c_int32),
    "bbgr_ego_rows": ([c_int64, c_int32, _P, _P, _P, _P, _P, _P, c_int64, _P, c_int64, _P,
                       c_float, _P, _P, c_int64, _P, c_int64, c_float, _P, _P], c_int32),
    "bbgr_rows_add_slots": ([c_int64, _P, _P, _P, _P, c_int64, _P, c_int64, c_int32, c_int64,
                             _P], c_int32),
    "bbgr_rows_add_unique": ([c_int64, _P, _P, c_int64, _P, c_int64, c_int32, c_int64, _P],
                             c_int32),
    # blueprint names, thin forms of the entry points above
    "bbgr_spmm_f32": ([ctypes.POINTER(CsrStruct), _P, c_int64, _P, c_int64, c_int32, _P, _P,
                       _P, c_float, _P], c_int32),
    "bbgr_bpr_fwd_bwd": ([ctypes.POINTER(BprArgs), _P], c_int32),
    "bbgr_adam_f32": ([c_int64, _P, _P, _P, _P, c_float, c_float, c_float, c_float,
                       c_float, c_float, c_float, c_float, _P], c_int32),
    "bbgr_negsample": ([c_int64, _P, _P, _P, c_int32, _P, c_float, c_int32, c_uint64,
                        c_uint64, _P, _P, _P, _P], c_int32),
}

_lib = None


def header_symbols(header: Path = HEADER_PATH) -> list[str]:
    """Every `bbgr_*(` function declared in include/bbgr.h."""
    text = header.read_text()
    return sorted(set(re.findall(r"\b(bbgr_[a-z0-9_]+)\s*\(", text)))


def lib() -> ctypes.CDLL:
    """Load libbbgr.so (once). Raises loudly if it was not built."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise ImportError(
                f"libbbgr.so not found at {LIB_PATH}; build it with "
                f"`python -c 'import __graft_entry__ as g; g.build()'` or "
                f"`make -C {PKG_DIR / 'csrc'}`")
        handle = ctypes.CDLL(str(LIB_PATH), mode=os.RTLD_NOW | os.RTLD_GLOBAL)
        for name, (argtypes, restype) in _SIGNATURES.items():
            fn = getattr(handle, name)
            fn.argtypes = argtypes
            fn.restype = restype
        if handle.bbgr_abi_version() != 11:
            raise ImportError("libbbgr.so ABI version mismatch")
        _lib = handle
    return _lib


def check(fn_name: str, rc: int) -> None:
    if rc != BBGR_OK:
        msg = lib().bbgr_last_error()
        raise BbgrError(fn_name, rc, msg.decode() if msg else "")


def call(fn_name: str, *args) -> None:
    check(fn_name, getattr(lib(), fn_name)(*args))


def require_gpu(t: torch.Tensor | None = None) -> None:
    if not torch.cuda.is_available():
        raise RuntimeError("bbgr kernels need a ROCm GPU (torch.cuda.is_available() is False); "
                           "there is no CPU fallback")
    if t is not None and not t.is_cuda:
        raise ValueError("bbgr kernels take device tensors; got a CPU tensor")


def stream_handle() -> int:
    return torch.cuda.current_stream().cuda_stream


def ptr(t: torch.Tensor | None):
    return None if t is None else t.data_ptr()


def ld(t: torch.Tensor | None) -> int:
    if t is None:
        return 0
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError("tables must be 2-D with unit column stride")
    return t.stride(0)


def byte_mask(n: int, device) -> torch.Tensor:
    """A zeroed 1-byte-per-row mask of n rows whose storage covers whole 4-byte
    words: bbgr_mark_list flags rows with 32-bit atomics on the word holding
    the byte, so the last row may touch up to 3 bytes past n."""
    return torch.zeros((int(n) + 3) // 4 * 4, dtype=torch.uint8, device=device)[: int(n)]


def check_word_padded(mask: torch.Tensor, n: int, what: str = "mask") -> None:
    """Refuse a mask for bbgr_mark_list whose storage ends inside the last word."""
    have = mask.untyped_storage().nbytes() - mask.storage_offset() * mask.element_size()
    need = (int(n) + 3) // 4 * 4
    if mask.dtype != torch.uint8 or have < need or mask.data_ptr() % 4:
        raise ValueError(f"{what}: bbgr_mark_list needs a 4-byte aligned uint8 mask whose "
                         f"storage covers {need} bytes (have {have}); use _lib.byte_mask")


def workspace_query(fn_name: str, *args_before_ws, args_after=()) -> int:
    """Run an entry point in size-query mode (workspace=NULL)."""
    n = c_size_t(0)
    call(fn_name, *args_before_ws, None, ctypes.byref(n), *args_after)
    return n.value
