"""Drop-in for the model layer of version_1/lightgcn_cu_pop_long_tail_exposure.py
(byte-identical to "lightgcn_cu_pop_Degree-Aware Message.py"): Method A,
popularity damping alpha_i = 1/log1p(max(deg_i,1)) on BOTH operators
(:362-396), Gauss-Seidel propagation (:424-442), uniform negatives.
"""
from __future__ import annotations

from ._lib import OP_METHOD_A
from .lightgcn_cu_pop import LightGCN, _build

__all__ = ["build_message_passing_mats", "LightGCN", "evaluate_sampled",
           "evaluate_full_ranking"]


def build_message_passing_mats(train_edges_2xE, num_users: int, num_items: int, cred_u,
                               device: str):
    """M_ui = w_base*alpha_i, M_iu = c_u*w_base*alpha_i (:379-392)."""
    return _build(train_edges_2xE, num_users, num_items, cred_u, device, OP_METHOD_A)


def evaluate_sampled(model, train_csr, test_csr, num_items: int, device: str, **cfg):
    """version_1/lightgcn_cu_pop_long_tail_exposure.py:485-545 (same arguments; precision / recall / ndcg per K):
    bbgr.evaluation.evaluate_sampled, candidates drawn on the device."""
    from .evaluation import evaluate_sampled_reference
    return evaluate_sampled_reference(model, train_csr, test_csr, num_items, device, **cfg)


def evaluate_full_ranking(model, train_csr, test_csr, num_items: int, device: str, **cfg):
    """version_1/lightgcn_cu_pop_long_tail_exposure.py:547-610 (same arguments; precision / recall / ndcg per K):
    bbgr.evaluation.evaluate_full."""
    from .evaluation import evaluate_full_ranking_reference
    return evaluate_full_ranking_reference(model, train_csr, test_csr, num_items, device, **cfg)
