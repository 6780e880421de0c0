"""MI355X-native LightGCN propagation + BPR training path (import name: ``bbgr``).

Hot path of ishika28/Beyond-Binary-Fake-User-Detection-A-Credibility-Aware-
Graph-based-Recommender-System rebuilt on hand-written gfx950 HIP kernels
behind the reference's own module API:

  bbgr.lightgcn_cu_pop   Version-2/lighgcn_cu_pop.py   (GS order, credibility)
  bbgr.lightgcn_cu_pop_long_tail_exposure              (Method A damping)
  bbgr.lightgcn_cu       lightgcn_cu.py                (Jacobi order, L_fair)
  bbgr.lightgcn          lightgcn.py / lightgcn-1.py   (symmetric A_hat)
  bbgr.trainer           fused native training step (sampler + fwd + BPR + bwd + Adam)
  bbgr.distributed       user-row sharded training over RCCL
  bbgr.sampler, bbgr.optim, bbgr.bpr, bbgr.propagate, bbgr.graph

All device compute goes through libbbgr.so (C ABI: include/bbgr.h).
"""
__version__ = "0.1.0"
