"""ORACLE — test infrastructure, NOT product code.

CPU restatements of the reference's hot path used ONLY as the checker by
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg. Nothing in
the bbgr package imports this directory.

  oracle.ref_numpy : float64 numpy/scipy restatement (the parity truth)
  oracle.ref_torch : fp32 torch restatement using the reference's own torch
                     calls (sparse_coo_tensor().coalesce(), torch.sparse.mm,
                     stack().mean(0), the bpr_loss expression, torch.optim.Adam)
                     — the "reference CPU path" timed as cpu_baseline.

Pinning: the reference publishes no tests, fixtures or golden vectors, and
importing/running the reference Python here was refused by the environment
(SURVEY §8c), so this oracle is pinned by hand-derived known-answer tests
(tests/test_oracle.py: closed-form 2x2 / 3x4 graphs, duplicate edge, isolated
item, ln 2 loss at zero embeddings) and by cross-agreement of the two
independent restatements. Against the reference itself it is
"parity unpinned" (see DESIGN.md §Oracle).
"""
