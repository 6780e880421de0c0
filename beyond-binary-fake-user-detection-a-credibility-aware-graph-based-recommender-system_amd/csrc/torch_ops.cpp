// torch_ops.cpp — the drop-in path's operators registered from C++
// (TORCH_LIBRARY(bbgr)): libbbgr_torch.so, loaded by bbgr/ops.py with
// torch.ops.load_library. The reference's models call torch.sparse.mm inside
// their propagate() and rely on autograd for the backward
// (Version-2/lighgcn_cu_pop.py:472-508, lightgcn_cu.py:420-463,
// lightgcn.py:318-349, the step at Version-2:858-863); these operators are the
// drop-in for exactly that surface:
//
//   bbgr::propagate(u0, i0, pair_key, num_layers, order) -> (u_final, i_final)
//   bbgr::propagate_backward(gU, gI, pair_key, num_layers, order) -> (grad_u0, grad_i0)
//   bbgr::propagate_backward_rows(iu, vu, gI, num_users, pair_key, num_layers, order,
//                                 ii=None, vi=None)
//   bbgr::jacobi_layer(u, i, pair_key) -> (new_i, new_u)          (+ _backward)
//   bbgr::propagate_sym(x0, pair_key, num_layers) -> x_final       (+ _backward)
//   bbgr::bpr_loss(uf, itf, ue, ie, users, pos, neg, reg, pop, lambda_fair) -> loss
//   bbgr::bpr_loss_backward(...) -> (g_uf, g_if, g_ue, g_ie)
//   bbgr::bpr_loss_sparse_ego(..., sparse_uf) -> loss
//   bbgr::_register_pair / _unregister_pair / _counters            (host bookkeeping)
//
// Each has a CUDA(=HIP) kernel that issues libbbgr launches on torch's current
// stream (graph-capturable, no host sync), a Meta kernel (torch.compile traces
// through it) and, for the forward ops, an Autograd kernel whose backward is
// itself a registered op. The sparse operators are not tensors: an operator
// pair (four CSR products + scale vectors, bbgr/propagate.OperatorPair) is
// registered once from Python and the ops look it up by key.
#include <ATen/ATen.h>
#include <ATen/core/dispatch/Dispatcher.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <torch/autograd.h>
#include <torch/library.h>

#include <atomic>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "bbgr.h"

using at::Tensor;
using torch::autograd::AutogradContext;
using torch::autograd::variable_list;

namespace bbgr_torch {

static void check(int rc, const char *what) {
  TORCH_CHECK(rc == BBGR_OK, "bbgr: ", what, " failed (", rc, "): ", bbgr_last_error());
}

static hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

static bool capturing() {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(cur_stream(), &st) != hipSuccess) return false;
  return st != hipStreamCaptureStatusNone;
}

template <class T>
static T *p(const Tensor &t) {
  return t.defined() ? t.data_ptr<T>() : nullptr;
}
static const float *cf(const c10::optional<Tensor> &t) {
  return t && t->defined() ? t->data_ptr<float>() : nullptr;
}
static int64_t ld(const Tensor &t) {
  if (!t.defined()) return 0;
  TORCH_CHECK(t.dim() == 2 && t.stride(1) == 1, "bbgr: tables must be 2-D with unit column stride");
  return t.stride(0);
}
static void check_table(const char *name, const Tensor &t, int64_t rows, int64_t d) {
  TORCH_CHECK(t.scalar_type() == at::kFloat, name, " must be float32");
  TORCH_CHECK(t.is_cuda(), name, " must be a device tensor");
  TORCH_CHECK(t.dim() == 2 && t.size(0) == rows && t.size(1) == d, name, " has shape ",
              t.sizes(), ", expected [", rows, ", ", d, "]");
  TORCH_CHECK(t.stride(1) == 1, name, " must have unit column stride");
}

// -- operator pairs (registered from Python) ----------------------------------
struct Product {
  bbgr_csr csr{};      // internal ids
  bbgr_csr csr_in{};   // input-id column indices (input-order pairs)
  bool has_in = false;
  const float *vals = nullptr, *in_scale = nullptr, *out_scale = nullptr;
  const float *first_vals = nullptr;
  bool cols_by_degree = false, rows_by_degree = false;
  int64_t hot_bytes = 192LL << 20;

  // propagate.Csr.stream_from / stream_out_from
  int32_t stream_from(int d) const {
    if (!cols_by_degree) return 0;
    if ((int64_t)csr.n_cols * 4 * d <= hot_bytes) return 0;
    return (int32_t)std::max<int64_t>(1, std::min<int64_t>(csr.n_cols / 8, hot_bytes / (4 * d)));
  }
  int32_t stream_out_from(int d) const {
    if (!rows_by_degree) return 0;
    if ((int64_t)csr.n_rows * 4 * d <= hot_bytes) return 0;
    return (int32_t)std::max<int64_t>(1, std::min<int64_t>(csr.n_rows / 8, hot_bytes / (4 * d)));
  }
};

struct Pair {
  Product fi, fu, bi, bu;   // fwd item<-user, fwd user<-item, their transposes
  int64_t U = 0, I = 0;
  const float *feed_fwd_iu = nullptr, *feed_fwd_ui = nullptr;
  const float *feed_bwd_iu = nullptr, *feed_bwd_ui = nullptr;
  bool io = false;   // input-order tables over a degree-ordered graph
  Tensor user_map, item_map, user_rank64, item_rank64, item_map64;
  std::vector<Tensor> keep;   // every registered tensor, alive while registered
  mutable Tensor u2i_slots;   // user-CSR slot -> item-CSR slot (built at first use)
  mutable std::once_flag u2i_once;
  // the rows backward's frontier buffers, one set per stream (reused: the slot
  // bitmap is cleared again after each use; frontier_bits / release_bits)
  struct FrontierBufs {
    Tensor bits, list, count, ws, mbits;
  };
  mutable std::mutex fb_mu;
  mutable std::map<int64_t, FrontierBufs> fb;
  // 0..U-1 / 0..I-1 (int32): the identity acc_in_map of the last layer of an
  // input-order chain, made once instead of two fills per call
  mutable std::once_flag iota_once;
  mutable Tensor iota_u, iota_i;
  // the in-backward Adam's two [I, d] item tables (the rows backward's gI and
  // the item Adam's gradient side table), one set per stream, all-zero between
  // calls: a call writes the batch items' rows only and clears them again, so
  // no step pays two 256 MB (C4) zero fills (bpr_adam_backward). At most
  // kItemTableSets sets are kept (the least recently used stream's set is
  // dropped): a caller that steps on a new stream per epoch or worker holds a
  // bounded 2 x [I, d] each, not one more set per stream.
  struct ItemTables {
    Tensor gi, grad;
    uint64_t tick = 0;
  };
  static constexpr size_t kItemTableSets = 2;
  mutable std::mutex it_mu;
  mutable std::map<int64_t, ItemTables> it;
  mutable uint64_t it_tick = 0;
  // the set for stream `skey` (it_mu held), evicting the LRU set first when full
  ItemTables &item_tables(int64_t skey) const {
    auto f = it.find(skey);
    if (f == it.end()) {
      if (it.size() >= kItemTableSets) {
        auto lru = it.begin();
        for (auto j = it.begin(); j != it.end(); ++j)
          if (j->second.tick < lru->second.tick) lru = j;
        it.erase(lru);
      }
      f = it.emplace(skey, ItemTables{}).first;
    }
    f->second.tick = ++it_tick;
    return f->second;
  }
};

static std::mutex g_mu;
static std::unordered_map<int64_t, std::shared_ptr<Pair>> g_pairs;
// split-row workspaces: (indptr, d, stream or -1 for graph captures) -> buffer
static std::map<std::tuple<const void *, int, int64_t>, Tensor> g_ws;
static std::atomic<int64_t> g_rows_backward{0}, g_dense_backward{0};

static std::shared_ptr<Pair> pair_of(int64_t key) {
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_pairs.find(key);
  TORCH_CHECK(it != g_pairs.end(), "bbgr ops: no operator pair registered under key ", key);
  return it->second;
}

// partial workspace of a product's split rows (n_chunks*(d+1) floats, zeroed
// once; every launch leaves the arrival counters zero). A graph capture gets a
// set of its own, allocated inside the capture (its zero fill then replays).
static float *workspace(const Product &pr, int d, const at::Device &dev) {
  if (pr.csr.n_split == 0) return nullptr;
  const int64_t skey = capturing() ? -1 : (int64_t)(intptr_t)cur_stream();
  auto key = std::make_tuple((const void *)pr.csr.indptr, d, skey);
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_ws.find(key);
  if (it == g_ws.end()) {
    Tensor w = at::zeros({(int64_t)pr.csr.n_chunks * (d + 1)},
                         at::TensorOptions().dtype(at::kFloat).device(dev));
    it = g_ws.emplace(key, w).first;
  }
  return it->second.data_ptr<float>();
}

// -- one fused SpMM launch (propagate.spmm) ------------------------------------
// One parameter table's Adam step (torch.optim.Adam semantics, host bias
// corrections): bbgr.optim.FusedAdam in backward mode hands these over.
struct AdamTable {
  Tensor p, m, v;
  float lr = 1e-3f, beta1 = 0.9f, beta2 = 0.999f, eps = 1e-8f, wd = 0.f;
  float bc1 = 1.f, bc2s = 1.f;
  bool moments_graph = false;   // m, v in the graph's row order (adam_moments_unmapped)
  // p is then graph-ordered too (the optimizer's master copy) and every updated
  // row is also written to this caller-order table (bbgr_spmm_args.adam_mirror)
  Tensor mirror;
};

struct Opts {
  Tensor y;
  const float *y_scale = nullptr;
  float y_scale_s = 1.f;
  Tensor add;
  const float *add_scale = nullptr;
  float add_scale_s = 1.f;
  Tensor acc_in, acc_out;
  const float *acc_scale = nullptr;
  float acc_scale_s = 1.f;
  float gamma = 1.f;
  const uint8_t *src_mask = nullptr, *row_mask = nullptr, *add_mask = nullptr;
  const uint8_t *acc_mask = nullptr;
  const int32_t *y_map = nullptr, *acc_map = nullptr, *add_map = nullptr;
  const int32_t *acc_in_map = nullptr;
  bool src_input = false;
  const int64_t *row_list = nullptr, *row_count = nullptr;   // device-length row list
  int64_t n_row_list = 0;
  const uint32_t *src_bits = nullptr;                         // slot bitmap of src_mask
  const uint32_t *src_mask_bits = nullptr;                    // src_mask packed (bbgr_mask_pack)
  // fused Adam on this launch's rows (bbgr_spmm_args.adam_*; null: none)
  const AdamTable *adam = nullptr;
  const float *adam_grad = nullptr;   // its gradient table (nullable: the row value)
  int64_t adam_grad_ld = 0;
  float adam_grad_scale = 1.f;
  const int32_t *adam_map = nullptr;  // its row map (nullable: y_map's)
};


static void spmm(const Product &pr, const Tensor &x, bool first, const Opts &o) {
  bbgr_spmm_args a;
  std::memset(&a, 0, sizeof a);
  const int d = (int)x.size(1);
  a.d = d;
  a.x = x.data_ptr<float>();
  a.ldx = ld(x);
  if (pr.vals) {
    a.weight_mode = 1;
    a.edge_val = pr.vals;
  } else if (first && pr.in_scale) {
    TORCH_CHECK(pr.first_vals, "bbgr: first-layer edge values not registered");
    a.weight_mode = 1;
    a.edge_val = pr.first_vals;
  }
  a.col_scale_s = 1.f;
  a.y = p<float>(o.y);
  a.ldy = ld(o.y);
  a.y_scale = o.y_scale;
  a.y_scale_s = o.y_scale_s;
  a.add = p<float>(o.add);
  a.ldadd = ld(o.add);
  a.add_scale = o.add_scale;
  a.add_scale_s = o.add_scale_s;
  a.acc_in = p<float>(o.acc_in);
  a.ldacc_in = ld(o.acc_in);
  a.acc_out = p<float>(o.acc_out);
  a.ldacc_out = ld(o.acc_out);
  a.acc_scale = o.acc_scale;
  a.acc_scale_s = o.acc_scale_s;
  a.gamma = o.gamma;
  a.partial = workspace(pr, d, x.device());
  a.src_mask = o.src_mask;
  a.row_mask = o.row_mask;
  a.add_mask = o.add_mask;
  a.acc_mask = o.acc_mask;
  a.y_map = o.y_map;
  a.acc_map = o.acc_map;
  a.add_map = o.add_map;
  a.acc_in_map = o.acc_in_map;
  a.row_list = o.row_list;
  a.n_row_list = o.n_row_list;
  a.row_count = o.row_count;
  a.src_bits = o.src_bits;
  a.src_mask_bits = o.src_mask ? o.src_mask_bits : nullptr;
  if (o.adam) {
    const AdamTable &A = *o.adam;
    a.adam_param = A.p.data_ptr<float>();
    a.adam_exp_avg = A.m.data_ptr<float>();
    a.adam_exp_avg_sq = A.v.data_ptr<float>();
    a.adam_ld = ld(A.p);
    a.adam_lr = A.lr;
    a.adam_beta1 = A.beta1;
    a.adam_beta2 = A.beta2;
    a.adam_eps = A.eps;
    a.adam_weight_decay = A.wd;
    a.adam_bias_correction1 = A.bc1;
    a.adam_bias_correction2_sqrt = A.bc2s;
    a.adam_grad = o.adam_grad;
    a.adam_grad_ld = o.adam_grad_ld;
    a.adam_grad_scale = o.adam_grad_scale;
    a.adam_map = o.adam_map;
    a.adam_moments_unmapped = A.moments_graph ? 1 : 0;
    if (A.mirror.defined()) a.adam_mirror = A.mirror.data_ptr<float>();
  }
  // input-order source rows carry no hot prefix; mapped output rows neither
  a.stream_from = o.src_input ? 0 : pr.stream_from(d);
  a.stream_out_from = o.y_map ? 0 : pr.stream_out_from(d);
  TORCH_CHECK(!o.src_input || pr.has_in, "bbgr: product has no input-id columns");
  check(bbgr_spmm(o.src_input ? &pr.csr_in : &pr.csr, &a, cur_stream()), "bbgr_spmm");
}

static at::TensorOptions f32(const Tensor &like) {
  return at::TensorOptions().dtype(at::kFloat).device(like.device());
}
static at::TensorOptions u8(const Tensor &like) {
  return at::TensorOptions().dtype(at::kByte).device(like.device());
}

// -- K-layer chains (propagate.forward_steps / backward_steps, no sharding) ----
// The layer-mean accumulators of an input-order pair (K >= 2) stay in the
// graph's order between layers: layer 1 reads the caller's u0 / i0 through
// the map (acc_in_map) into an internal table, the middle layers update it in
// place with no map, and layer K writes the caller's rows (acc_map) from it
// (acc_in_map = identity). Same arithmetic per row, so the same bits; at C4
// the mapped (random-row) accumulator passes cost ~0.45 ms per user product.
struct AccPlan {
  Tensor in, out;
  const int32_t *in_map = nullptr, *out_map = nullptr;
};

static Tensor iota32(int64_t n, const Tensor &like) {
  return at::arange(n, at::TensorOptions().dtype(at::kInt).device(like.device()));
}

// the pair's cached identity maps; a graph capture makes its own (the fill
// then replays with it)
static std::pair<Tensor, Tensor> pair_iotas(const Pair &P, const Tensor &like) {
  if (capturing()) return {iota32(P.U, like), iota32(P.I, like)};
  std::call_once(P.iota_once, [&] {
    P.iota_u = iota32(P.U, like);
    P.iota_i = iota32(P.I, like);
    check(bbgr_sync(cur_stream()), "bbgr_sync");   // once: filled before any stream reads it
  });
  return {P.iota_u, P.iota_i};
}

static AccPlan acc_plan(int64_t k, int64_t K, const Tensor &x0, const Tensor &caller,
                        Tensor &internal, const int32_t *map, const Tensor &iota) {
  AccPlan a;
  if (!map || K < 2) {   // one table throughout (mapped or not)
    a.in = k == 1 ? x0 : caller;
    a.out = caller;
    a.in_map = a.out_map = map;
    return a;
  }
  a.in = k == 1 ? x0 : internal;
  a.out = k == K ? caller : internal;
  a.in_map = k == 1 ? map : (k == K ? iota.data_ptr<int32_t>() : nullptr);
  a.out_map = k == K ? map : nullptr;
  return a;
}

static void set_acc(Opts &o, const AccPlan &a) {
  o.acc_in = a.in;
  o.acc_out = a.out;
  o.acc_map = a.out_map;
  o.acc_in_map = a.in_map;
}

static std::tuple<Tensor, Tensor> forward_chain(const Pair &P, const Tensor &u0, const Tensor &i0,
                                                int64_t K, bool gs, Tensor acc_u = Tensor(),
                                                Tensor acc_i = Tensor()) {
  const int64_t U = P.U, I = P.I, d = u0.size(1);
  check_table("user table", u0, U, d);
  check_table("item table", i0, I, d);
  if (!acc_u.defined()) acc_u = at::empty({U, d}, f32(u0));
  if (!acc_i.defined()) acc_i = at::empty({I, d}, f32(u0));
  if (K == 0) {
    acc_u.copy_(u0);
    acc_i.copy_(i0);
    return {acc_u, acc_i};
  }
  const float gl = (float)(1.0 / (double)(K + 1));   // as the Python float
  const int32_t *am_u = P.io ? P.user_map.data_ptr<int32_t>() : nullptr;
  const int32_t *am_i = P.io ? P.item_map.data_ptr<int32_t>() : nullptr;
  Tensor int_u, int_i, iota_u, iota_i;   // internal-order accumulators (input-order pair)
  if (P.io && K >= 2) {
    int_u = at::empty({U, d}, f32(u0));
    int_i = at::empty({I, d}, f32(u0));
    std::tie(iota_u, iota_i) = pair_iotas(P, u0);
  }
  if (gs) {   // Version-2:482-487: i_k = M_iu u_{k-1}; u_k = M_ui i_k
    Tensor bufU = at::empty({U, d}, f32(u0)), bufI = at::empty({I, d}, f32(u0));
    for (int64_t k = 1; k <= K; ++k) {
      const float g = k == K ? gl : 1.f;
      Opts oi;
      oi.y = bufI;
      oi.y_scale = P.feed_fwd_iu;
      set_acc(oi, acc_plan(k, K, i0, acc_i, int_i, am_i, iota_i));
      oi.acc_scale = P.fi.out_scale;
      oi.gamma = g;
      oi.src_input = P.io && k == 1;
      spmm(P.fi, k == 1 ? u0 : bufU, k == 1, oi);
      Opts ou;
      if (k < K) ou.y = bufU;
      ou.y_scale = P.feed_fwd_ui;
      set_acc(ou, acc_plan(k, K, u0, acc_u, int_u, am_u, iota_u));
      ou.acc_scale = P.fu.out_scale;
      ou.gamma = g;
      spmm(P.fu, bufI, false, ou);
    }
  } else {    // lightgcn_cu.py:429-447: both sides from layer k-1
    Tensor bufU[2] = {at::empty({U, d}, f32(u0)), at::empty({U, d}, f32(u0))};
    Tensor bufI[2] = {at::empty({I, d}, f32(u0)), at::empty({I, d}, f32(u0))};
    int cur = 0;
    for (int64_t k = 1; k <= K; ++k) {
      const float g = k == K ? gl : 1.f;
      const int nxt = 1 - cur;
      Opts oi;
      if (k < K) oi.y = bufI[nxt];
      oi.y_scale = P.feed_fwd_iu;
      set_acc(oi, acc_plan(k, K, i0, acc_i, int_i, am_i, iota_i));
      oi.acc_scale = P.fi.out_scale;
      oi.gamma = g;
      oi.src_input = P.io && k == 1;
      spmm(P.fi, k == 1 ? u0 : bufU[cur], k == 1, oi);
      Opts ou;
      if (k < K) ou.y = bufU[nxt];
      ou.y_scale = P.feed_fwd_ui;
      set_acc(ou, acc_plan(k, K, u0, acc_u, int_u, am_u, iota_u));
      ou.acc_scale = P.fu.out_scale;
      ou.gamma = g;
      ou.src_input = P.io && k == 1;
      spmm(P.fu, k == 1 ? i0 : bufI[cur], k == 1, ou);
      cur = nxt;
    }
  }
  return {acc_u, acc_i};
}

// Several zeroed byte regions from ONE fill (a launch each costs ~5 us at the
// drop-in step's batch sizes): region k holds sizes[k] bytes at a 256-byte
// aligned offset, so a region also views as a wider type, and a byte mask's
// last word lies inside its region (bbgr_mark_list sets bytes with word
// atomics).
struct ZeroArena {
  Tensor buf;
  std::vector<int64_t> off, len;
  ZeroArena(const Tensor &like, std::initializer_list<int64_t> sizes) {
    int64_t o = 0;
    for (int64_t n : sizes) {
      off.push_back(o);
      len.push_back(n);
      o += (std::max<int64_t>(n, 1) + 255) / 256 * 256;
    }
    buf = at::zeros({o}, u8(like));
  }
  Tensor bytes(size_t k) const { return buf.narrow(0, off[k], len[k]); }
};

// ids in [0, n) -> rank[ids] (graph order), anything else -> -1 (skipped by
// the marking kernels)
static Tensor to_graph_rows(const Tensor &ids, int64_t n, const Tensor &rank64) {
  Tensor out = at::empty_like(ids);
  check(bbgr_graph_rows(ids.numel(), ids.data_ptr<int64_t>(), n,
                        rank64.defined() ? rank64.data_ptr<int64_t>() : nullptr,
                        out.data_ptr<int64_t>(), cur_stream()),
        "bbgr_graph_rows");
  return out;
}

// BBGR_ROWS_MARK=0 keeps forward_rows' separate marking launches (A/B, tests)
static bool rows_mark_fused() {
  const char *e = std::getenv("BBGR_ROWS_MARK");
  return !(e && e[0] == '0');
}

// The GS finals at the listed rows only (bbgr::propagate_rows): u_final at
// `users`, i_final at `items` (the caller's rows: input ids of an input-order
// pair); every other row of the two returned tables is left unwritten. The
// dense layers 1..K-1 run as in forward_chain, with their layer-mean
// accumulators touched at the listed rows only (acc_mask); layer K computes
// the item frontier (listed items and N(listed users)) as a device-length row
// list and the listed users only. The same per-row arithmetic as the dense
// chain, so the listed rows hold the dense chain's bits. A training step that
// reads the finals only at its batch rows (the reference's get_user_item_emb
// -> bpr_loss, Version-2:858-859) skips the two last-layer full products and
// the full-table accumulator passes. Jacobi order: the dense chain.
// graph_tables: u0 / i0 are the GRAPH-ordered copies of the caller's tables
// (the in-backward optimizer's master copies, input-order pair, K >= 2): the
// first products gather them through the internal column indices (the hot
// prefix of the degree order) and the layer-1 accumulators read them unmapped;
// the returned finals are in the caller's order as always. Same values, same
// per-row arithmetic: bitwise the caller-order call.
static std::tuple<Tensor, Tensor> forward_rows(const Pair &P, const Tensor &u0, const Tensor &i0,
                                               int64_t K, bool gs, const Tensor &users_,
                                               const Tensor &items_, bool graph_tables = false) {
  TORCH_CHECK(!graph_tables || (gs && K >= 2 && P.io),
              "propagate_rows_graph: an input-order GS pair and num_layers >= 2");
  if (!gs || K == 0) return forward_chain(P, u0, i0, K, gs);
  const int64_t U = P.U, I = P.I, d = u0.size(1);
  check_table("user table", u0, U, d);
  check_table("item table", i0, I, d);
  Tensor users = users_.to(at::kLong).contiguous().view({-1});
  Tensor items = items_.to(at::kLong).contiguous().view({-1});
  Tensor acc_u = at::empty({U, d}, f32(u0)), acc_i = at::empty({I, d}, f32(u0));
  const hipStream_t st = cur_stream();
  // every zeroed mask and counter of the call in one fill: mu, mi, fr (+ the
  // caller-order mu_in, mi_in of an input-order pair), ucount, fcount
  ZeroArena za(u0, {U, I, I, P.io ? U : 0, P.io ? I : 0, 16});
  Tensor mu = za.bytes(0), mi = za.bytes(1), fr = za.bytes(2);
  Tensor ulist = at::empty({std::max<int64_t>(users.numel(), 1)}, users.options());
  Tensor flist = at::empty({std::max<int64_t>(I, 1)}, users.options());
  Tensor counts = za.bytes(5).view(at::kLong);
  Tensor ucount = counts.narrow(0, 0, 1), fcount = counts.narrow(0, 1, 1);
  Tensor mu_in = P.io ? za.bytes(3) : mu, mi_in = P.io ? za.bytes(4) : mi;
  const bbgr_csr &uc = P.fu.csr;
  // masks in the graph's order (mu / mi), in the caller's (mu_in / mi_in; an
  // input-order pair), the distinct listed users (the last user product's
  // rows) and the item frontier (the last item product's: listed items and
  // every neighbour of a listed user) as device-length lists
  if (rows_mark_fused()) {   // one launch (bbgr_rows_mark)
    bbgr_rows_mark_args a{};
    a.n_users_listed = users.numel();
    a.n_items_listed = items.numel();
    a.users = users.data_ptr<int64_t>();
    a.items = items.data_ptr<int64_t>();
    a.n_users = U;
    a.n_items = I;
    a.user_rank = P.io ? P.user_rank64.data_ptr<int64_t>() : nullptr;
    a.item_rank = P.io ? P.item_rank64.data_ptr<int64_t>() : nullptr;
    a.user_indptr = uc.indptr;
    a.user_indices = uc.indices;
    a.mask_u = mu.data_ptr<uint8_t>();
    a.mask_i = mi.data_ptr<uint8_t>();
    a.frontier = fr.data_ptr<uint8_t>();
    a.mask_u_in = P.io ? mu_in.data_ptr<uint8_t>() : nullptr;
    a.mask_i_in = P.io ? mi_in.data_ptr<uint8_t>() : nullptr;
    a.user_list = ulist.data_ptr<int64_t>();
    a.user_count = ucount.data_ptr<int64_t>();
    a.frontier_list = flist.data_ptr<int64_t>();
    a.frontier_count = fcount.data_ptr<int64_t>();
    check(bbgr_rows_mark(&a, st), "bbgr_rows_mark");
  } else {   // BBGR_ROWS_MARK=0: the separate launches (A/B, tests)
    Tensor ui = to_graph_rows(users, U, P.io ? P.user_rank64 : Tensor());
    Tensor ii = to_graph_rows(items, I, P.io ? P.item_rank64 : Tensor());
    check(bbgr_mark_list(ui.numel(), ui.data_ptr<int64_t>(), nullptr, nullptr,
                         mu.data_ptr<uint8_t>(), U, ulist.data_ptr<int64_t>(),
                         ucount.data_ptr<int64_t>(), st),
          "bbgr_mark_list");
    check(bbgr_mark_rows(ii.numel(), ii.data_ptr<int64_t>(), 1, mi.data_ptr<uint8_t>(), I, st),
          "bbgr_mark_rows");
    check(bbgr_mark_list(ii.numel(), ii.data_ptr<int64_t>(), nullptr, nullptr,
                         fr.data_ptr<uint8_t>(), I, flist.data_ptr<int64_t>(),
                         fcount.data_ptr<int64_t>(), st),
          "bbgr_mark_list");
    check(bbgr_mark_list(ui.numel(), ui.data_ptr<int64_t>(), uc.indptr, uc.indices,
                         fr.data_ptr<uint8_t>(), I, flist.data_ptr<int64_t>(),
                         fcount.data_ptr<int64_t>(), st),
          "bbgr_mark_list");
    if (P.io) {
      check(bbgr_mark_rows(users.numel(), users.data_ptr<int64_t>(), 1,
                           mu_in.data_ptr<uint8_t>(), U, st),
            "bbgr_mark_rows");
      check(bbgr_mark_rows(items.numel(), items.data_ptr<int64_t>(), 1,
                           mi_in.data_ptr<uint8_t>(), I, st),
            "bbgr_mark_rows");
    }
  }
  const float gl = (float)(1.0 / (double)(K + 1));
  const int32_t *am_u = P.io ? P.user_map.data_ptr<int32_t>() : nullptr;
  const int32_t *am_i = P.io ? P.item_map.data_ptr<int32_t>() : nullptr;
  Tensor int_u, int_i, iota_u, iota_i;
  if (P.io && K >= 2) {
    int_u = at::empty({U, d}, f32(u0));
    int_i = at::empty({I, d}, f32(u0));
    std::tie(iota_u, iota_i) = pair_iotas(P, u0);
  }
  Tensor bufU = at::empty({U, d}, f32(u0)), bufI = at::empty({I, d}, f32(u0));
  for (int64_t k = 1; k <= K; ++k) {
    const float g = k == K ? gl : 1.f;
    Opts oi;
    oi.y = bufI;
    oi.y_scale = P.feed_fwd_iu;
    AccPlan ai = acc_plan(k, K, i0, acc_i, int_i, am_i, iota_i);
    if (graph_tables && k == 1) ai.in_map = nullptr;   // i0 already in the graph's order
    set_acc(oi, ai);
    oi.acc_mask = (ai.out_map ? mi_in : mi).data_ptr<uint8_t>();
    oi.acc_scale = P.fi.out_scale;
    oi.gamma = g;
    oi.src_input = P.io && k == 1 && !graph_tables;
    if (k == K) {   // the item frontier, listed on the device
      oi.row_mask = fr.data_ptr<uint8_t>();
      oi.row_list = flist.data_ptr<int64_t>();
      oi.n_row_list = I;
      oi.row_count = fcount.data_ptr<int64_t>();
    }
    spmm(P.fi, k == 1 ? u0 : bufU, k == 1, oi);
    Opts ou;
    if (k < K) ou.y = bufU;
    ou.y_scale = P.feed_fwd_ui;
    AccPlan au = acc_plan(k, K, u0, acc_u, int_u, am_u, iota_u);
    if (graph_tables && k == 1) au.in_map = nullptr;
    set_acc(ou, au);
    ou.acc_mask = (au.out_map ? mu_in : mu).data_ptr<uint8_t>();
    ou.acc_scale = P.fu.out_scale;
    ou.gamma = g;
    if (k == K) {   // the listed users only
      ou.row_mask = mu.data_ptr<uint8_t>();
      ou.row_list = ulist.data_ptr<int64_t>();
      ou.n_row_list = users.numel();
      ou.row_count = ucount.data_ptr<int64_t>();
    }
    spmm(P.fu, bufI, false, ou);
  }
  return {acc_u, acc_i};
}

// grad_support: (su, si, si_int) — su / si index the rows of gU / gI (input
// order for an input-order pair), si_int the item CSR rows (GS: the first
// item product's output support). Undefined = no masks.
struct Support {
  Tensor su, si, si_int;
  // GS rows backward (d >= 64): the item frontier as a device-length row list
  // and the slot bitmap of the listed users' edges in item-CSR order, for the
  // first item product (bbgr_spmm_args.row_list / row_count / src_bits)
  Tensor flist, fcount, bits;
  // si_int packed one bit per item (bbgr_mask_pack): the first user product's
  // per-edge test (bbgr_spmm_args.src_mask_bits)
  Tensor si_bits;
  // gU (and su) in the graph's own row order instead of the caller's: the
  // rows backward builds its gU table itself, so every user product adds it
  // without the row map (add_mask read at the row, not at user_map[row]) and
  // the first products gather it through the internal column indices
  bool gu_internal = false;
  // gI given as rows (the rows backward with ii / vi): gI is zero off the
  // listed rows, so the GS weight gradient gI/(K+1) is formed on those rows
  // of a zeroed table instead of a pass over the whole of gI
  Tensor gi_rows;
};

// user-CSR slot -> item-CSR slot holding the same edge, the k-th copy of a
// duplicate pair mapped to the k-th copy: stable sorts of both CSRs' edge
// keys (user * I + item, internal ids). Unlike bbgr_transpose_slots (a binary
// search per edge) it needs no column order inside the rows: an input-order
// pair's rows keep their columns in the caller's id order. One-time per pair.
static const Tensor &u2i_slots(const Pair &P, const at::Device &dev) {
  // built once per pair under the pair's own flag (not the registry mutex, so
  // pair_of / workspace lookups on other threads never wait for the sorts);
  // repeat_interleave is told its output size, so nothing syncs with the host
  std::call_once(P.u2i_once, [&] {
    const bbgr_csr &uc = P.fu.csr, &ic = P.bi.csr;
    const int64_t nnz = uc.nnz;
    const auto i32 = at::TensorOptions().dtype(at::kInt).device(dev);
    Tensor out = at::empty({std::max<int64_t>(nnz, 1)}, i32);
    if (nnz > 0) {
      auto rows_of = [&](const int32_t *indptr, int64_t n) {
        Tensor ptr = at::from_blob(const_cast<int32_t *>(indptr), {n + 1}, i32);
        Tensor cnt = (ptr.narrow(0, 1, n) - ptr.narrow(0, 0, n)).to(at::kLong);
        // (the optional output size selects the repeats-only overload; a plain
        // int64 would bind to repeat_interleave(self, repeats) instead)
        return at::repeat_interleave(cnt, std::optional<int64_t>(nnz));
      };
      Tensor uidx = at::from_blob(const_cast<int32_t *>(uc.indices), {nnz}, i32).to(at::kLong);
      Tensor iidx = at::from_blob(const_cast<int32_t *>(ic.indices), {nnz}, i32).to(at::kLong);
      Tensor ka = rows_of(uc.indptr, P.U) * P.I + uidx;
      Tensor kb = iidx * P.I + rows_of(ic.indptr, P.I);
      Tensor sa = std::get<1>(at::sort(ka, /*stable=*/true, /*dim=*/0, /*descending=*/false));
      Tensor sb = std::get<1>(at::sort(kb, /*stable=*/true, /*dim=*/0, /*descending=*/false));
      out.index_put_({sa}, sb.to(at::kInt));
    }
    P.u2i_slots = out;
  });
  return P.u2i_slots;
}

// the flagged rows of mask [n] as an ascending device list + device count,
// into the caller's buffers (list >= n rows, count 1, ws grown as needed)
static void mask_list(const Tensor &mask, Tensor &list, Tensor &cnt, Tensor &ws) {
  const int64_t n = mask.numel();
  const auto i64 = at::TensorOptions().dtype(at::kLong).device(mask.device());
  size_t need = 0;
  check(bbgr_mask_to_list(n, mask.data_ptr<uint8_t>(), nullptr, nullptr, nullptr, &need,
                          cur_stream()),
        "bbgr_mask_to_list (size)");
  if (!ws.defined() || (size_t)ws.numel() < need)
    ws = at::empty({(int64_t)std::max<size_t>(need, 1)}, u8(mask));
  if (!list.defined() || list.numel() < std::max<int64_t>(n, 1))
    list = at::empty({std::max<int64_t>(n, 1)}, i64);
  if (!cnt.defined()) cnt = at::empty({1}, i64);
  size_t have = (size_t)ws.numel();
  check(bbgr_mask_to_list(n, mask.data_ptr<uint8_t>(), list.data_ptr<int64_t>(),
                          cnt.data_ptr<int64_t>(), ws.data_ptr(), &have, cur_stream()),
        "bbgr_mask_to_list");
}

// BBGR_DROPIN_BITS=0 keeps the mask-only first item product (A/B, tests)
static bool dropin_bits_enabled() {
  const char *e = std::getenv("BBGR_DROPIN_BITS");
  return !(e && e[0] == '0');
}

// Support.flist / fcount / bits for the listed users ui (internal ids): the
// first backward item product then visits the frontier's rows only and tests
// edge liveness 64 slots per load, bitwise the mask-only product (the same
// live edges in the same order; DESIGN §3 "Frontier products")
// Buffers are per pair and stream and reused: the bitmap is all-zero between
// uses (release_bits clears the listed users' bits after the chain, as
// FusedTrainer does), the list / count / hipcub workspace are overwritten. A
// graph capture gets fresh ones (their zero fill is then part of the graph).
// The returned lock (the pair's frontier mutex) is held by the caller until
// release_bits has been issued: another host thread's backward on the same
// stream then issues its marking after this one's clear, so stream order keeps
// each chain's bitmap, list and count its own. Only the host-side issue is
// serialised; the GPU work of different streams still overlaps.
// frontier_bits applies (its list then feeds the first item product)
static bool listed_frontier(const Pair &P, int64_t d) {
  return d >= 64 && dropin_bits_enabled() && P.fu.csr.nnz > 0;
}

static std::unique_lock<std::mutex> frontier_bits(const Pair &P, Support &s, const Tensor &ui,
                                                  int64_t d) {
  std::unique_lock<std::mutex> g(P.fb_mu, std::defer_lock);
  if (!listed_frontier(P, d)) return g;
  const Tensor &slots = u2i_slots(P, ui.device());
  const int64_t nbits = P.bi.csr.nnz / 32 + 4;
  const auto i32 = at::TensorOptions().dtype(at::kInt).device(ui.device());
  Pair::FrontierBufs fresh, *b = &fresh;
  if (!capturing()) {
    g.lock();
    b = &P.fb[(int64_t)(intptr_t)cur_stream()];
  }
  if (!b->bits.defined()) b->bits = at::zeros({nbits}, i32);
  const Tensor &mi = s.si_int.defined() ? s.si_int : s.si;
  if (!s.flist.defined()) {   // (rows_backward's list_marks listed it while marking)
    mask_list(mi, b->list, b->count, b->ws);
    s.flist = b->list;
    s.fcount = b->count;
  }
  // the packed item mask (every word rewritten per call: nothing to clear;
  // BBGR_MASK_BITS=0 keeps the byte test, A/B)
  const char *mb_env = std::getenv("BBGR_MASK_BITS");
  if (!(mb_env && mb_env[0] == '0')) {
    if (!b->mbits.defined()) b->mbits = at::empty({P.I / 32 + 1}, i32);
    check(bbgr_mask_pack(P.I, mi.data_ptr<uint8_t>(),
                         reinterpret_cast<uint32_t *>(b->mbits.data_ptr<int32_t>()),
                         cur_stream()),
          "bbgr_mask_pack");
    s.si_bits = b->mbits;
  }
  s.bits = b->bits;
  check(bbgr_mark_slots(ui.numel(), ui.data_ptr<int64_t>(), P.fu.csr.indptr,
                        slots.data_ptr<int32_t>(),
                        reinterpret_cast<uint32_t *>(s.bits.data_ptr<int32_t>()), 1,
                        cur_stream()),
        "bbgr_mark_slots");
  return g;
}

// clear the listed users' bits again once the chain has read them (stream order)
static void release_bits(const Pair &P, const Support &s, const Tensor &ui) {
  if (!s.bits.defined()) return;
  check(bbgr_mark_slots(ui.numel(), ui.data_ptr<int64_t>(), P.fu.csr.indptr,
                        P.u2i_slots.data_ptr<int32_t>(),
                        reinterpret_cast<uint32_t *>(s.bits.data_ptr<int32_t>()), 0,
                        cur_stream()),
        "bbgr_mark_slots (clear)");
}

// The drop-in's in-backward Adam (GS, K >= 2; bbgr_torch::bpr_adam_backward):
// the user step rides on the last user product, which then writes no gradient
// table; the item step on the last item product (a dense launch over every
// item row), reading its gradient gl * item_grad from a caller-order side
// table (gI + (K+1) * ego rows, formed before the chain); the batch users'
// ego-L2 rows enter gU just before the last user product (gU[r] += (K+1) *
// ego[r], so G = out * T + gl * gU carries them), as FusedTrainer does.
static void index_add_rows(Tensor &dst, const Tensor &index, const Tensor &src);

// The sort of a deterministic row scatter, kept to apply to several tables
// over the same index list (bbgr_scatter_plan / bbgr_scatter_apply).
struct RowPlan {
  Tensor ws, idx;
  int64_t n = 0, n_dst = 0;
  bool defined() const { return ws.defined(); }
};

static RowPlan plan_rows(const Tensor &index, int64_t n_dst) {
  RowPlan r;
  r.idx = index.to(at::kLong).contiguous();
  r.n = r.idx.numel();
  r.n_dst = n_dst;
  size_t need = 0;
  check(bbgr_scatter_plan(r.n, r.idx.data_ptr<int64_t>(), n_dst, nullptr, &need, cur_stream()),
        "bbgr_scatter_plan (size)");
  r.ws = at::empty({(int64_t)std::max<size_t>(need, 1)},
                   at::TensorOptions().dtype(at::kByte).device(index.device()));
  size_t have = (size_t)r.ws.numel();
  check(bbgr_scatter_plan(r.n, r.idx.data_ptr<int64_t>(), n_dst, r.ws.data_ptr(), &have,
                          cur_stream()),
        "bbgr_scatter_plan");
  return r;
}

// dst.index_add_(0, idx, src) (then src2 continuing each row's sum) in the
// plan's order: bitwise index_add_rows over [src; src2] with [idx; idx]
static void apply_rows(const RowPlan &r, Tensor &dst, const Tensor &src_,
                       const Tensor &src2_ = Tensor()) {
  TORCH_CHECK(dst.size(0) == r.n_dst, "apply_rows: destination rows differ from the plan's");
  const Tensor src = src_.contiguous(), src2 = src2_.defined() ? src2_.contiguous() : Tensor();
  TORCH_CHECK(src.size(0) >= r.n && src.size(1) == dst.size(1) &&
                  (!src2.defined() || (src2.size(0) >= r.n && src2.size(1) == dst.size(1))),
              "apply_rows: shapes");
  check(bbgr_scatter_apply(r.n, r.n_dst, r.ws.data_ptr(), src.data_ptr<float>(), ld(src),
                           src2.defined() ? src2.data_ptr<float>() : nullptr,
                           src2.defined() ? ld(src2) : 0, dst.data_ptr<float>(), ld(dst),
                           (int32_t)dst.size(1), cur_stream()),
        "bbgr_scatter_apply");
}

struct StepAdam {
  AdamTable user, item;
  Tensor item_grad;                 // [I, d], caller's row order
  Tensor ego_u_vals;                // (K+1) * ego rows, aligned with the users' rows
  // the sorts of the step's two index lists: the batch items (gI and the
  // item gradient) and the batch users' gU rows (set by rows_backward; gU
  // and the ego rows added before the user Adam)
  RowPlan item_plan, user_plan;
  // the users' scatter in first-slot form instead of user_plan (defined:
  // bbgr_rows_add_slots over user_rows, the rows of the batch's user slots)
  Tensor user_slot, user_count, user_rows;
};

// dst[user_rows[k]] += the first-slot sums of src's rows (bbgr_rows_add_slots):
// bitwise apply_rows over a plan of user_rows (a stable sort's segments)
static void add_slot_rows(const StepAdam &sa, Tensor &dst, const Tensor &src_) {
  const Tensor src = src_.contiguous();
  const int64_t n = sa.user_rows.numel();
  TORCH_CHECK(src.size(0) >= n && src.size(1) == dst.size(1) && sa.user_slot.numel() >= n,
              "add_slot_rows: shapes");
  check(bbgr_rows_add_slots(n, sa.user_slot.data_ptr<int64_t>(),
                            sa.user_count.data_ptr<int32_t>(), sa.user_rows.data_ptr<int64_t>(),
                            src.data_ptr<float>(), ld(src), dst.data_ptr<float>(), ld(dst),
                            (int32_t)dst.size(1), dst.size(0), cur_stream()),
        "bbgr_rows_add_slots");
}

// BBGR_USER_SORT=1 keeps the user scatter's sort (A/B, tests)
static bool users_sorted_scatter() {
  const char *e = std::getenv("BBGR_USER_SORT");
  return e && e[0] == '1';
}

static std::tuple<Tensor, Tensor> backward_chain(const Pair &P, const Tensor &gU, const Tensor &gI,
                                                 int64_t K, bool gs, const Support &s,
                                                 Tensor gu0 = Tensor(), Tensor gi0 = Tensor(),
                                                 const StepAdam *sa = nullptr) {
  const int64_t U = P.U, I = P.I, d = gU.size(1);
  check_table("user grad", gU, U, d);
  check_table("item grad", gI, I, d);
  TORCH_CHECK(!sa || (gs && K >= 2), "bbgr: the in-backward Adam needs the GS order and K >= 2");
  if (!sa && !gu0.defined()) gu0 = at::empty({U, d}, f32(gU));
  if (!sa && !gi0.defined()) gi0 = at::empty({I, d}, f32(gU));
  if (K == 0) {
    gu0.copy_(gU);
    gi0.copy_(gI);
    return {gu0, gi0};
  }
  const float gl = (float)(1.0 / (double)(K + 1));   // as the Python float
  const uint8_t *su = p<uint8_t>(s.su), *si = p<uint8_t>(s.si);
  const uint8_t *si_int = s.si_int.defined() ? p<uint8_t>(s.si_int) : si;
  const int32_t *um = P.io ? P.user_map.data_ptr<int32_t>() : nullptr;
  const int32_t *im = P.io ? P.item_map.data_ptr<int32_t>() : nullptr;
  const int32_t *um_add = s.gu_internal ? nullptr : um;   // gU's row map
  const bool gu_in = P.io && !s.gu_internal;              // gU in input order
  if (gs) {   // Gi_k = gI' + M_ui^T Gu_k ; Gu_{k-1} = gU' + M_iu^T Gi_k ; Gu_K = gU'
    Tensor bufU = at::empty({U, d}, f32(gU)), bufI = at::empty({I, d}, f32(gU));
    for (int64_t k = K; k >= 1; --k) {
      const bool first = k == K;
      Opts oi;
      oi.y = bufI;
      oi.y_scale = P.feed_bwd_iu;
      oi.y_scale_s = first ? gl : 1.f;
      oi.add = gI;
      oi.add_mask = si;
      oi.add_scale = P.bu.in_scale;
      oi.add_scale_s = gl;
      oi.src_mask = first ? su : nullptr;
      oi.row_mask = first ? si_int : nullptr;
      oi.add_map = im;
      oi.src_input = gu_in && first;
      if (first && s.bits.defined()) {
        oi.row_list = s.flist.data_ptr<int64_t>();
        oi.n_row_list = I;
        oi.row_count = s.fcount.data_ptr<int64_t>();
        oi.src_bits = reinterpret_cast<const uint32_t *>(s.bits.data_ptr<int32_t>());
      }
      if (sa && k == 1) {   // the item Adam rides on the last item product
        oi.adam = &sa->item;
        oi.adam_grad = sa->item_grad.data_ptr<float>();
        oi.adam_grad_ld = ld(sa->item_grad);
        oi.adam_grad_scale = gl;
        oi.adam_map = im;   // bufI is in the graph's order, the weights in the caller's
      }
      spmm(P.bi, first ? gU : bufU, first, oi);
      Opts ou;
      ou.add = gU;
      ou.add_mask = su;
      ou.add_map = um_add;
      ou.src_mask = first ? si_int : nullptr;
      if (first && s.si_bits.defined())
        ou.src_mask_bits = reinterpret_cast<const uint32_t *>(s.si_bits.data_ptr<int32_t>());
      ou.add_scale_s = gl;
      if (k > 1) {
        ou.y = bufU;
        ou.y_scale = P.feed_bwd_ui;
        ou.add_scale = P.bi.in_scale;
      } else if (sa) {   // the user Adam: no gradient table, ego rows in gU first
        Tensor g = gU;
        if (sa->user_slot.defined())
          add_slot_rows(*sa, g, sa->ego_u_vals);
        else
          apply_rows(sa->user_plan, g, sa->ego_u_vals);
        ou.y_scale = P.bu.out_scale;
        ou.y_map = um;   // the Adam's rows: the caller's order
        ou.adam = &sa->user;
      } else {
        ou.y = gu0;
        ou.y_scale = P.bu.out_scale;
        ou.y_map = um;
      }
      spmm(P.bu, bufI, false, ou);
    }
    if (sa) return {Tensor(), Tensor()};
    // GS: i0 only feeds the layer mean. The Tensor overload with a CPU 0-dim
    // float: the Scalar overload of mul.out computes into a temporary and
    // copies it (a second 256 MB pass at C4); the same float product either way
    const Tensor glt = at::scalar_tensor(gl, at::TensorOptions().dtype(at::kFloat));
    if (s.gi_rows.defined()) {   // gI holds values on its listed rows only
      gi0.zero_();
      gi0.index_copy_(0, s.gi_rows, at::mul(gI.index_select(0, s.gi_rows), glt));
    } else {
      at::mul_out(gi0, gI, glt);
    }
  } else {    // Jacobi: Gu_{k-1} = gU' + M_iu^T Gi_k ; Gi_{k-1} = gI' + M_ui^T Gu_k
    Tensor bufU[2] = {at::empty({U, d}, f32(gU)), at::empty({U, d}, f32(gU))};
    Tensor bufI[2] = {at::empty({I, d}, f32(gU)), at::empty({I, d}, f32(gU))};
    int cur = 0;
    for (int64_t k = K; k >= 1; --k) {
      const bool first = k == K;
      const int nxt = 1 - cur;
      const float ys = first ? gl : 1.f;
      const Tensor &xu = first ? gI : bufI[cur];   // input of BU (item table)
      const Tensor &xi = first ? gU : bufU[cur];   // input of BI (user table)
      Opts ou, oi;
      ou.y_scale_s = oi.y_scale_s = ys;
      ou.add = gU;
      ou.add_mask = su;
      ou.add_map = um_add;
      ou.add_scale_s = gl;
      ou.src_mask = first ? si : nullptr;
      ou.src_input = P.io && first;
      oi.add = gI;
      oi.add_mask = si;
      oi.add_map = im;
      oi.add_scale_s = gl;
      oi.src_mask = first ? su : nullptr;
      oi.src_input = gu_in && first;
      if (k > 1) {
        ou.y = bufU[nxt];
        ou.y_scale = P.feed_bwd_ui;
        ou.add_scale = P.bi.in_scale;
        oi.y = bufI[nxt];
        oi.y_scale = P.feed_bwd_iu;
        oi.add_scale = P.bu.in_scale;
      } else {
        ou.y = gu0;
        ou.y_scale = P.bu.out_scale;
        ou.y_map = um;
        oi.y = gi0;
        oi.y_scale = P.bi.out_scale;
        oi.y_map = im;
      }
      spmm(P.bu, xu, first, ou);
      spmm(P.bi, xi, first, oi);
      cur = nxt;
    }
  }
  return {gu0, gi0};
}

// -- gradient supports (ops.grad_support / the rows path) ----------------------
static Support io_support(const Pair &P, const Tensor &mu, const Tensor &mi, bool gs,
                          const Tensor &users /* input ids or undefined */) {
  Support s{mu, mi, Tensor()};
  if (!gs) return s;
  Tensor mi_int = mi.index_select(0, P.item_map64);
  const bbgr_csr &uc = P.fu.csr;
  if (users.defined()) {
    Tensor ui = P.user_rank64.index_select(0, users).contiguous();
    check(bbgr_mark_neighbors(ui.numel(), ui.data_ptr<int64_t>(), uc.indptr, uc.indices, 1,
                              mi_int.data_ptr<uint8_t>(), cur_stream()),
          "bbgr_mark_neighbors");
  } else {
    check(bbgr_mark_neighbors_of_mask(P.U, mu.data_ptr<uint8_t>(), P.user_map.data_ptr<int32_t>(),
                                      uc.indptr, uc.indices, 1, mi_int.data_ptr<uint8_t>(),
                                      cur_stream()),
          "bbgr_mark_neighbors_of_mask");
  }
  s.si = mi_int.index_select(0, P.item_rank64);
  s.si_int = mi_int;
  return s;
}

// the gradients' row support, read off the tables (bbgr_row_support): users
// with a nonzero gU row; items with a nonzero gI row plus, for GS, every
// neighbour of a flagged user. Bitwise the dense chain (skipped rows are zero).
static Support grad_support(const Pair &P, const Tensor &gU, const Tensor &gI, bool gs) {
  const int64_t U = P.U, I = P.I, d = gU.size(1);
  Tensor mu = at::empty({std::max<int64_t>(U, 1)}, u8(gU));
  Tensor mi = at::empty({std::max<int64_t>(I, 1)}, u8(gU));
  check(bbgr_row_support(I, (int32_t)d, gI.data_ptr<float>(), ld(gI), mi.data_ptr<uint8_t>(),
                         nullptr, nullptr, nullptr, cur_stream()),
        "bbgr_row_support");
  if (P.io) {
    check(bbgr_row_support(U, (int32_t)d, gU.data_ptr<float>(), ld(gU), mu.data_ptr<uint8_t>(),
                           nullptr, nullptr, nullptr, cur_stream()),
          "bbgr_row_support");
    return io_support(P, mu.narrow(0, 0, U), mi.narrow(0, 0, I), gs, Tensor());
  }
  const bbgr_csr &uc = P.fu.csr;
  check(bbgr_row_support(U, (int32_t)d, gU.data_ptr<float>(), ld(gU), mu.data_ptr<uint8_t>(),
                         gs ? uc.indptr : nullptr, gs ? uc.indices : nullptr,
                         gs ? mi.data_ptr<uint8_t>() : nullptr, cur_stream()),
        "bbgr_row_support");
  return Support{mu.narrow(0, 0, U), mi.narrow(0, 0, I), Tensor()};
}

// dst.index_add_(0, index, src) summed per destination in ascending source
// order (bbgr_scatter_add_rows; deterministic)
static void index_add_rows(Tensor &dst, const Tensor &index, const Tensor &src) {
  Tensor idx = index.to(at::kLong).contiguous();
  const int64_t n = idx.numel();
  TORCH_CHECK(src.size(0) >= n && src.size(1) == dst.size(1), "index_add_rows: shapes");
  size_t need = 0;
  const int32_t d = (int32_t)dst.size(1);
  check(bbgr_scatter_add_rows(n, idx.data_ptr<int64_t>(), src.data_ptr<float>(), ld(src),
                              dst.data_ptr<float>(), ld(dst), d, dst.size(0), nullptr, &need,
                              cur_stream()),
        "bbgr_scatter_add_rows (size)");
  Tensor ws = at::empty({(int64_t)std::max<size_t>(need, 1)}, u8(dst));
  size_t have = (size_t)ws.numel();
  check(bbgr_scatter_add_rows(n, idx.data_ptr<int64_t>(), src.data_ptr<float>(), ld(src),
                              dst.data_ptr<float>(), ld(dst), d, dst.size(0), ws.data_ptr(),
                              &have, cur_stream()),
        "bbgr_scatter_add_rows");
}

static bool is_gs(c10::string_view order) {
  if (order == "gs") return true;
  TORCH_CHECK(order == "jacobi", "unknown propagation order ", order);
  return false;
}

// -- CUDA (HIP) kernels ---------------------------------------------------------
static std::tuple<Tensor, Tensor> propagate_cuda(const Tensor &u0, const Tensor &i0, int64_t key,
                                                 int64_t K, c10::string_view order) {
  auto P = pair_of(key);
  return forward_chain(*P, u0.contiguous(), i0.contiguous(), K, is_gs(order));
}

static std::tuple<Tensor, Tensor> propagate_rows_cuda(const Tensor &u0, const Tensor &i0,
                                                      const Tensor &users, const Tensor &items,
                                                      int64_t key, int64_t K,
                                                      c10::string_view order) {
  auto P = pair_of(key);
  return forward_rows(*P, u0.contiguous(), i0.contiguous(), K, is_gs(order), users, items);
}

// bbgr::propagate_rows_graph — propagate_rows (GS) from the graph-ordered
// master copies of the weights (no autograd: the in-backward step's forward)
static std::tuple<Tensor, Tensor> propagate_rows_graph_cuda(const Tensor &u0g, const Tensor &i0g,
                                                            const Tensor &users,
                                                            const Tensor &items, int64_t key,
                                                            int64_t K) {
  auto P = pair_of(key);
  return forward_rows(*P, u0g.contiguous(), i0g.contiguous(), K, true, users, items, true);
}

static std::tuple<Tensor, Tensor> propagate_backward_cuda(const Tensor &gU_, const Tensor &gI_,
                                                          int64_t key, int64_t K,
                                                          c10::string_view order) {
  auto P = pair_of(key);
  const bool gs = is_gs(order);
  Tensor gU = gU_.contiguous(), gI = gI_.contiguous();
  g_dense_backward++;
  return backward_chain(*P, gU, gI, K, gs, grad_support(*P, gU, gI, gs));
}

// dL/d(u_final) given as rows: vu[k] adds to user iu[k]. The dense gU is
// formed on the listed rows only (zeroed, then summed in ascending k) and the
// masks come from the list: every read of gU in a K >= 1 chain is masked to
// those rows, so the rest is never touched (K = 0 copies gU whole: zeroed).
static std::tuple<Tensor, Tensor> rows_backward(const std::shared_ptr<Pair> &P, const Tensor &iu_,
                                                const Tensor &vu, const Tensor &gI_, int64_t K,
                                                bool gs, const c10::optional<Tensor> &ii_,
                                                const c10::optional<Tensor> &vi_,
                                                StepAdam *sa = nullptr,
                                                const Tensor &gi_zeroed = Tensor());

static std::tuple<Tensor, Tensor> propagate_backward_rows_cuda(
    const Tensor &iu_, const Tensor &vu, const Tensor &gI_, int64_t num_users, int64_t key,
    int64_t K, c10::string_view order, const c10::optional<Tensor> &ii_,
    const c10::optional<Tensor> &vi_) {
  auto P = pair_of(key);
  TORCH_CHECK(num_users == P->U, "propagate_backward_rows: num_users does not match the pair");
  return rows_backward(P, iu_, vu, gI_, K, is_gs(order), ii_, vi_);
}

// the body of propagate_backward_rows; `sa`: the in-backward Adam (no gradient
// tables returned); `gi_zeroed`: an all-zero [I, d] table to form gI in (rows
// ii only) instead of a fresh zero fill
static std::tuple<Tensor, Tensor> rows_backward(const std::shared_ptr<Pair> &P, const Tensor &iu_,
                                                const Tensor &vu, const Tensor &gI_, int64_t K,
                                                bool gs, const c10::optional<Tensor> &ii_,
                                                const c10::optional<Tensor> &vi_, StepAdam *sa,
                                                const Tensor &gi_zeroed) {
  const int64_t U = P->U, I = P->I, d = vu.size(1);
  Tensor iu = iu_.to(at::kLong).contiguous();
  // dL/d(i_final) as rows too (vi[k] adds to item ii[k]; gI_ is then only a
  // [I, d] placeholder): gI is summed on those rows of a zeroed table (the GS
  // item product's addend is read on its whole output support, N(users)
  // included) and its support is the list itself instead of a 256 MB
  // bbgr_row_support scan; the GS weight gradient gI/(K+1) is formed on the
  // listed rows only (Support.gi_rows)
  const bool gi_rows = ii_.has_value() && ii_->defined();
  TORCH_CHECK(gi_rows == (vi_.has_value() && vi_->defined()),
              "propagate_backward_rows: ii and vi go together");
  Tensor ii, gI;
  if (gi_rows) {
    ii = ii_->to(at::kLong).contiguous();
    TORCH_CHECK(vi_->dim() == 2 && vi_->size(0) == ii.numel() && vi_->size(1) == d,
                "propagate_backward_rows: vi must be [len(ii), d]");
    gI = gi_zeroed.defined() ? gi_zeroed
                             : at::zeros({std::max<int64_t>(I, 1), d}, f32(vu)).narrow(0, 0, I);
    if (sa && sa->item_plan.defined()) apply_rows(sa->item_plan, gI, *vi_);
    else index_add_rows(gI, ii, vi_->contiguous());
  } else {
    gI = gI_.contiguous();
  }
  // input-order pair, K >= 1: gU never leaves this op, so it is formed in the
  // graph's row order (row user_rank[iu[k]]) and the chain reads it unmapped
  // (Support.gu_internal); the same values at the same rows of the products
  const bool gu_int = P->io && K >= 1;
  Tensor ru = gu_int ? P->user_rank64.index_select(0, iu).contiguous() : iu;
  Tensor gU;
  if (K == 0) {
    gU = at::zeros({std::max<int64_t>(U, 1), d}, f32(vu)).narrow(0, 0, U);
  } else {
    gU = at::empty({std::max<int64_t>(U, 1), d}, f32(vu)).narrow(0, 0, U);
    gU.index_fill_(0, ru, 0.0);
  }
  if (sa) {   // the ego rows land on the same gU rows as vu: one sort for both
    if (sa->user_slot.defined()) {   // first slots + counts: no sort
      sa->user_rows = ru;
      add_slot_rows(*sa, gU, vu);
    } else {
      sa->user_plan = plan_rows(ru, U);
      apply_rows(sa->user_plan, gU, vu);
    }
  } else {
    index_add_rows(gU, ru, vu.contiguous());
  }
  // input-order pair, GS, gI as rows, the first item product on a row list:
  // the item frontier is marked in the graph's order straight from the batch
  // items and N(batch users), and listed while it is marked (bbgr_mark_list:
  // no mask scan, no input-order mask to permute); the list's order is
  // unspecified and the product's rows are independent of it (bitwise)
  const bool list_marks = gu_int && gs && gi_rows && iu.numel() > 0 && listed_frontier(*P, d);
  // mu (and mi when it is marked from the list; the graph-order item mask and
  // the list's count when list_marks) zeroed by one fill
  ZeroArena za(vu, {U, gi_rows && !list_marks ? I : 0, list_marks ? I : 0, list_marks ? 8 : 0});
  Tensor mu = za.bytes(0);
  Tensor mi = gi_rows ? za.bytes(1) : at::empty({std::max<int64_t>(I, 1)}, u8(vu)).narrow(0, 0, I);
  check(bbgr_mark_rows(ru.numel(), ru.data_ptr<int64_t>(), 1, mu.data_ptr<uint8_t>(), U,
                       cur_stream()),
        "bbgr_mark_rows");
  if (list_marks) {
    // (nothing reads the input-order item mask on this path)
  } else if (gi_rows) {
    check(bbgr_mark_rows(ii.numel(), ii.data_ptr<int64_t>(), 1, mi.data_ptr<uint8_t>(), I,
                         cur_stream()),
          "bbgr_mark_rows");
  } else {
    check(bbgr_row_support(I, (int32_t)d, gI.data_ptr<float>(), ld(gI),
                           mi.data_ptr<uint8_t>(), nullptr, nullptr, nullptr, cur_stream()),
          "bbgr_row_support");
  }
  g_rows_backward++;
  Support s;
  if (list_marks) {
    Tensor mi_int = za.bytes(2);
    Tensor cnt = za.bytes(3).view(at::kLong);
    Tensor list = at::empty({std::max<int64_t>(I, 1)}, iu.options());
    Tensor ii_int = to_graph_rows(ii, I, P->item_rank64);
    const Tensor &ui = ru;   // (gu_int here: the batch users' graph rows)
    const bbgr_csr &uc = P->fu.csr;
    check(bbgr_mark_list(ii_int.numel(), ii_int.data_ptr<int64_t>(), nullptr, nullptr,
                         mi_int.data_ptr<uint8_t>(), I, list.data_ptr<int64_t>(),
                         cnt.data_ptr<int64_t>(), cur_stream()),
          "bbgr_mark_list");
    check(bbgr_mark_list(ui.numel(), ui.data_ptr<int64_t>(), uc.indptr, uc.indices,
                         mi_int.data_ptr<uint8_t>(), I, list.data_ptr<int64_t>(),
                         cnt.data_ptr<int64_t>(), cur_stream()),
          "bbgr_mark_list");
    s = Support{mu.narrow(0, 0, U), mi_int.index_select(0, P->item_rank64), mi_int};
    s.flist = list;
    s.fcount = cnt;
    s.gu_internal = gu_int;
  } else if (P->io) {
    s = io_support(*P, mu.narrow(0, 0, U), mi.narrow(0, 0, I), gs, iu);
    s.gu_internal = gu_int;
  } else {
    if (gs) {   // the first item product's output support: N(listed users)
      const bbgr_csr &uc = P->fu.csr;
      check(bbgr_mark_neighbors(iu.numel(), iu.data_ptr<int64_t>(), uc.indptr, uc.indices, 1,
                                mi.data_ptr<uint8_t>(), cur_stream()),
            "bbgr_mark_neighbors");
    }
    s = Support{mu.narrow(0, 0, U), mi.narrow(0, 0, I), Tensor()};
  }
  if (gi_rows && K >= 1) s.gi_rows = ii;
  std::unique_lock<std::mutex> fb_lock;
  if (gs && K >= 1 && iu.numel() > 0)
    fb_lock = frontier_bits(*P, s, ru, d);
  // the bitmap must be all-zero again on every exit: the clear is issued
  // after the chain, also when the chain throws (then best effort: a clear
  // that fails too leaves the error of the chain as the one reported)
  struct Release {
    const Pair &P;
    const Support &s;
    const Tensor &ru;
    bool armed = true;
    ~Release() {
      if (!armed) return;
      try {
        release_bits(P, s, ru);
      } catch (...) {
      }
    }
  } rel{*P, s, ru};
  auto out = backward_chain(*P, gU, gI, K, gs, s, Tensor(), Tensor(), sa);
  rel.armed = false;
  release_bits(*P, s, ru);
  return out;
}

static std::tuple<Tensor, Tensor> jacobi_layer_cuda(const Tensor &u_, const Tensor &i_, int64_t key) {
  auto P = pair_of(key);
  Tensor u = u_.contiguous(), i = i_.contiguous();
  const int64_t d = u.size(1);
  check_table("user table", u, P->U, d);
  check_table("item table", i, P->I, d);
  Tensor new_i = at::empty({P->I, d}, f32(u)), new_u = at::empty({P->U, d}, f32(u));
  Opts oi, ou;
  oi.y = new_i;
  oi.y_scale = P->fi.out_scale;
  oi.src_input = P->io;
  oi.y_map = P->io ? P->item_map.data_ptr<int32_t>() : nullptr;
  ou.y = new_u;
  ou.y_scale = P->fu.out_scale;
  ou.src_input = P->io;
  ou.y_map = P->io ? P->user_map.data_ptr<int32_t>() : nullptr;
  spmm(P->fi, u, true, oi);
  spmm(P->fu, i, true, ou);
  return {new_i, new_u};
}

// (d/du, d/di): M_iu^T g_i on the user rows, M_ui^T g_u on the item rows
static std::tuple<Tensor, Tensor> jacobi_layer_backward_cuda(const Tensor &g_i, const Tensor &g_u,
                                                             int64_t key) {
  auto P = pair_of(key);
  const int64_t d = g_i.size(1);
  Tensor gu = at::empty({P->U, d}, f32(g_i)), gi = at::empty({P->I, d}, f32(g_i));
  Opts ou, oi;
  ou.y = gu;
  ou.y_scale = P->bu.out_scale;
  ou.src_input = P->io;
  ou.y_map = P->io ? P->user_map.data_ptr<int32_t>() : nullptr;
  oi.y = gi;
  oi.y_scale = P->bi.out_scale;
  oi.src_input = P->io;
  oi.y_map = P->io ? P->item_map.data_ptr<int32_t>() : nullptr;
  spmm(P->bu, g_i.contiguous(), true, ou);
  spmm(P->bi, g_u.contiguous(), true, oi);
  return {gu, gi};
}

// lightgcn.py's one stacked [users; items] table: Jacobi on the two blocks
static Tensor propagate_sym_cuda(const Tensor &x0_, int64_t key, int64_t K) {
  auto P = pair_of(key);
  Tensor x0 = x0_.contiguous();
  Tensor out = at::empty_like(x0);
  forward_chain(*P, x0.narrow(0, 0, P->U), x0.narrow(0, P->U, P->I), K, false,
                out.narrow(0, 0, P->U), out.narrow(0, P->U, P->I));
  return out;
}

static Tensor propagate_sym_backward_cuda(const Tensor &g_, int64_t key, int64_t K) {
  auto P = pair_of(key);
  Tensor g = g_.contiguous();
  Tensor gx = at::empty_like(g);
  Tensor gU = g.narrow(0, 0, P->U), gI = g.narrow(0, P->U, P->I);
  g_dense_backward++;
  backward_chain(*P, gU, gI, K, false, grad_support(*P, gU, gI, false), gx.narrow(0, 0, P->U),
                 gx.narrow(0, P->U, P->I));
  return gx;
}

// -- BPR --------------------------------------------------------------------
static bbgr_bpr_args bpr_args(const Tensor &users, const Tensor &pos, const Tensor &neg,
                              const Tensor &uf, const Tensor &itf, const Tensor &ue,
                              const Tensor &ie, double reg, const c10::optional<Tensor> &pop,
                              double lambda_fair) {
  TORCH_CHECK(users.numel() == pos.numel() && pos.numel() == neg.numel(),
              "users, pos_items, neg_items must have equal length");
  TORCH_CHECK(!ue.defined() || ue.size(0) == uf.size(0), "ego and final tables differ in rows");
  TORCH_CHECK(!ie.defined() || ie.size(0) == itf.size(0), "ego and final tables differ in rows");
  bbgr_bpr_args a;
  std::memset(&a, 0, sizeof a);
  a.batch = users.numel();
  a.d = (int32_t)uf.size(1);
  a.n_users = uf.size(0);
  a.n_items = itf.size(0);
  a.users = users.data_ptr<int64_t>();
  a.pos = pos.data_ptr<int64_t>();
  a.neg = neg.data_ptr<int64_t>();
  a.uf = uf.data_ptr<float>();
  a.lduf = ld(uf);
  a.itf = itf.data_ptr<float>();
  a.ldif = ld(itf);
  a.ue = p<float>(ue);
  a.ldue = ld(ue);
  a.ie = p<float>(ie);
  a.ldie = ld(ie);
  a.pop = cf(pop);
  a.reg = (float)reg;
  a.lambda_fair = (float)lambda_fair;
  return a;
}

static Tensor idx64(const Tensor &t) { return t.to(at::kLong).contiguous(); }

static Tensor bpr_loss_cuda(const Tensor &uf_, const Tensor &itf_, const Tensor &ue_,
                            const Tensor &ie_, const Tensor &users_, const Tensor &pos_,
                            const Tensor &neg_, double reg, const c10::optional<Tensor> &pop,
                            double lambda_fair) {
  Tensor uf = uf_.contiguous(), itf = itf_.contiguous(), ue = ue_.contiguous(),
         ie = ie_.contiguous();
  Tensor users = idx64(users_), pos = idx64(pos_), neg = idx64(neg_);
  const int64_t B = users.numel();
  TORCH_CHECK(B > 0, "empty batch");
  Tensor parts = at::empty({3 * B}, f32(uf));
  Tensor out = at::empty({}, f32(uf));
  bbgr_bpr_args a = bpr_args(users, pos, neg, uf, itf, ue, ie, reg, pop, lambda_fair);
  a.parts = parts.data_ptr<float>();
  check(bbgr_bpr(&a, cur_stream()), "bbgr_bpr");
  check(bbgr_bpr_reduce(B, parts.data_ptr<float>(), (float)reg, (float)lambda_fair,
                        out.data_ptr<float>(), cur_stream()),
        "bbgr_bpr_reduce");
  return out;
}

// deterministic: per-triple gradient rows of the final tables (contrib), each
// destination summed in ascending triple order (bbgr_scatter_add_rows)
static std::tuple<Tensor, Tensor, Tensor, Tensor> bpr_loss_backward_cuda(
    const Tensor &dloss, const Tensor &uf_, const Tensor &itf_, const Tensor &ue_,
    const Tensor &ie_, const Tensor &users_, const Tensor &pos_, const Tensor &neg_, double reg,
    const c10::optional<Tensor> &pop, double lambda_fair) {
  Tensor uf = uf_.contiguous(), itf = itf_.contiguous(), ue = ue_.contiguous(),
         ie = ie_.contiguous();
  Tensor users = idx64(users_), pos = idx64(pos_), neg = idx64(neg_);
  Tensor g_uf = at::zeros_like(uf), g_if = at::zeros_like(itf), g_ue = at::zeros_like(ue),
         g_ie = at::zeros_like(ie);
  const int64_t B = users.numel();
  Tensor contrib = at::empty({3 * B, uf.size(1)}, f32(uf));
  Tensor dl = dloss.to(at::kFloat).contiguous().reshape({});
  bbgr_bpr_args a = bpr_args(users, pos, neg, uf, itf, ue, ie, reg, pop, lambda_fair);
  a.dloss = dl.data_ptr<float>();
  a.g_ue = g_ue.data_ptr<float>();
  a.ldgue = ld(g_ue);
  a.g_ie = g_ie.data_ptr<float>();
  a.ldgie = ld(g_ie);
  a.contrib = contrib.data_ptr<float>();
  a.ldcontrib = ld(contrib);
  check(bbgr_bpr(&a, cur_stream()), "bbgr_bpr");
  index_add_rows(g_uf, users, contrib.narrow(0, 0, B));
  index_add_rows(g_if, at::cat({pos, neg}), contrib.narrow(0, B, 2 * B));
  return {g_uf, g_if, g_ue, g_ie};
}

// slot[b] = position of the first occurrence of ids[b] (device-only): stable
// sort, then each sorted value's first sorted position by a binary search
// (a lower bound; one launch instead of a cummax scan and its masks)
// slot[b] = first b' with ids[b'] == ids[b] (ids in [0, n_rows)): bbgr_first_slot
// over a per-(device, n_rows) scratch of INT32_MAX rows, kept between calls
// (each call leaves it all INT32_MAX, in stream order); one per stream, like
// the workspaces. At most kFirstSlotScratch tables are kept (the least
// recently used is dropped): a process cycling through streams or model sizes
// holds a bounded n_rows int32 each (20 MB for U = 5M). An entry inherited by a
// new stream at a recycled address is still all INT32_MAX once the old
// stream's work has drained, which destroying a stream waits for.
// `role` keeps tables a single launch uses side by side apart: bbgr_ego_slots
// takes a user and an item table at once, which must not be one buffer when
// U == I (0 = first_slot, 1 = ego users, 2 = ego items). Role 3 holds
// bbgr_ego_rows' counts, filled with (and left at) 0 instead of INT32_MAX.
static constexpr size_t kFirstSlotScratch = 8;
static Tensor slot_scratch(int64_t n_rows, const at::Device &dev, int64_t role = 0,
                           int32_t fill = 0x7fffffff) {
  static std::mutex mu;
  static std::map<std::tuple<int64_t, int64_t, int64_t, int64_t>, std::pair<Tensor, uint64_t>>
      scratch;
  static uint64_t tick = 0;
  const auto fresh = [&] {
    return at::full({std::max<int64_t>(n_rows, 1)}, fill,
                    at::TensorOptions().dtype(at::kInt).device(dev));
  };
  if (capturing()) return fresh();   // a captured step fills its own (the fill replays with it)
  std::lock_guard<std::mutex> lk(mu);
  const auto key =
      std::make_tuple((int64_t)dev.index(), n_rows, (int64_t)(intptr_t)cur_stream(), role);
  auto it = scratch.find(key);
  if (it == scratch.end()) {
    if (scratch.size() >= kFirstSlotScratch) {
      auto lru = scratch.begin();
      for (auto j = scratch.begin(); j != scratch.end(); ++j)
        if (j->second.second < lru->second.second) lru = j;
      scratch.erase(lru);
    }
    it = scratch.emplace(key, std::make_pair(fresh(), uint64_t(0))).first;
  }
  it->second.second = ++tick;
  return it->second.first;
}

static Tensor first_slot(const Tensor &ids_, int64_t n_rows) {
  Tensor ids = ids_.to(at::kLong).contiguous();
  Tensor slot = at::empty_like(ids);
  Tensor first = slot_scratch(n_rows, ids.device());
  check(bbgr_first_slot(ids.numel(), ids.data_ptr<int64_t>(), n_rows, first.data_ptr<int32_t>(),
                        slot.data_ptr<int64_t>(), cur_stream()),
        "bbgr_first_slot");
  return slot;
}

// the ego-L2 gradient as compact rows (bpr.ego_grad_rows): every occurrence of
// a row adds into the row of its FIRST occurrence (the others stay +0.0), so
// each table row's sum is formed exactly as in the dense path
static std::tuple<Tensor, Tensor, Tensor, Tensor> ego_grad_rows(const Tensor &dl,
                                                                const Tensor &users,
                                                                const Tensor &pos,
                                                                const Tensor &neg,
                                                                const Tensor &ue,
                                                                const Tensor &ie, double reg,
                                                                double scale = 1.0,
                                                                Tensor *user_slots = nullptr) {
  const int64_t B = users.numel(), d = ue.size(1), U = ue.size(0), I = ie.size(0);
  TORCH_CHECK(U > 0 && I > 0, "ego_grad_rows: empty table");
  // one int64 block: iu [B], ii [2B], cu [B], sp [B], sn [B]
  Tensor ix = at::empty({6 * B}, users.options());
  Tensor iu = ix.narrow(0, 0, B), ii = ix.narrow(0, B, 2 * B), cu = ix.narrow(0, 3 * B, B),
         sp = ix.narrow(0, 4 * B, B), sn = ix.narrow(0, 5 * B, B);
  Tensor fu = slot_scratch(U, users.device(), 1), fi = slot_scratch(I, users.device(), 2);
  check(bbgr_ego_slots(B, users.data_ptr<int64_t>(), pos.data_ptr<int64_t>(),
                       neg.data_ptr<int64_t>(), U, I, fu.data_ptr<int32_t>(),
                       fi.data_ptr<int32_t>(), iu.data_ptr<int64_t>(), ii.data_ptr<int64_t>(),
                       cu.data_ptr<int64_t>(), sp.data_ptr<int64_t>(), sn.data_ptr<int64_t>(),
                       cur_stream()),
        "bbgr_ego_slots");
  // every row written (zero off the first slots): no fill; the counts scratch
  // is zero between calls
  Tensor g = at::empty({3 * B, d}, f32(ue));
  Tensor gu = g.narrow(0, 0, B), gi = g.narrow(0, B, 2 * B);
  Tensor cnt = slot_scratch(3 * B, users.device(), 3, 0);
  const Tensor uec = ue.contiguous(), iec = ie.contiguous();
  // user_slots: (cu, the users' first-slot counts) for bbgr_rows_add_slots
  Tensor cnt_u;
  if (user_slots) {
    cnt_u = at::empty({std::max<int64_t>(B, 1)}, at::TensorOptions().dtype(at::kInt).device(
                                                     users.device()));
    user_slots[0] = cu;
    user_slots[1] = cnt_u;
  }
  check(bbgr_ego_rows(B, (int32_t)d, cu.data_ptr<int64_t>(), sp.data_ptr<int64_t>(),
                      sn.data_ptr<int64_t>(), iu.data_ptr<int64_t>(), ii.data_ptr<int64_t>(),
                      uec.data_ptr<float>(), ld(uec), iec.data_ptr<float>(), ld(iec),
                      dl.data_ptr<float>(), (float)reg, cnt.data_ptr<int32_t>(),
                      gu.data_ptr<float>(), ld(gu), gi.data_ptr<float>(), ld(gi), (float)scale,
                      user_slots ? cnt_u.data_ptr<int32_t>() : nullptr, cur_stream()),
        "bbgr_ego_rows");
  return {gu, gi, iu, ii};
}

// bbgr::bpr_adam_backward — the drop-in step's backward with the optimizer in
// it (bbgr.optim.FusedAdam(fuse_backward=True); GS, K >= 2; eager only):
// dL/d(finals) as the BPR kernel's per-triple rows scaled by dloss (as
// bpr_loss_sparse_ego's backward), the ego-L2 rows in first-slot form
// (ego_grad_rows), then propagate_backward_rows' chain with the user Adam on
// its last user product and the item Adam on its last item product (StepAdam).
// Updates u0, i0 and their moments in place; no gradient table is written.
// Versus the separate step (gradients, then bbgr_adam) the ego rows are added
// before the last products' epilogues instead of after them: the same terms,
// rounded in another order (FusedTrainer's order).
static void bpr_adam_backward_cuda(const Tensor &dloss, const Tensor &uf_, const Tensor &itf_,
                                   const Tensor &u0, const Tensor &i0, const Tensor &users_,
                                   const Tensor &pos_, const Tensor &neg_, double reg,
                                   int64_t key, int64_t K, const Tensor &m_u, const Tensor &v_u,
                                   const Tensor &m_i, const Tensor &v_i, double lr, double beta1,
                                   double beta2, double eps, double wd, double bc1_u,
                                   double bc2s_u, double bc1_i, double bc2s_i,
                                   bool moments_graph, const c10::optional<Tensor> &u_graph,
                                   const c10::optional<Tensor> &i_graph) {
  auto P = pair_of(key);
  TORCH_CHECK(K >= 2, "bpr_adam_backward: the in-backward Adam needs num_layers >= 2");
  const int64_t d = u0.size(1), U = P->U, I = P->I;
  check_table("user weights", u0, U, d);
  check_table("item weights", i0, I, d);
  for (const Tensor *t : {&u0, &i0, &m_u, &v_u, &m_i, &v_i})
    TORCH_CHECK(t->is_contiguous() && t->scalar_type() == at::kFloat,
                "bpr_adam_backward: weights and moments must be contiguous fp32");
  TORCH_CHECK(m_u.sizes() == u0.sizes() && v_u.sizes() == u0.sizes() &&
                  m_i.sizes() == i0.sizes() && v_i.sizes() == i0.sizes(),
              "bpr_adam_backward: moment shapes");
  Tensor users = idx64(users_), pos = idx64(pos_), neg = idx64(neg_);
  Tensor uf = uf_.contiguous(), itf = itf_.contiguous();
  const int64_t B = users.numel();
  Tensor dl = dloss.to(at::kFloat).contiguous().reshape({});
  Tensor contrib = at::empty({3 * B, d}, f32(uf));
  bbgr_bpr_args a = bpr_args(users, pos, neg, uf, itf, u0, i0, reg, c10::nullopt, 0.0);
  a.dloss = dl.data_ptr<float>();
  a.contrib = contrib.data_ptr<float>();
  a.ldcontrib = ld(contrib);
  check(bbgr_bpr(&a, cur_stream()), "bbgr_bpr");
  // the ego rows come scaled by K + 1 (one rounding, as at::mul(rows, K + 1));
  // the users' first slots and counts replace the user scatter's sort
  Tensor uslots[2];
  auto eg = ego_grad_rows(dl, users, pos, neg, u0, i0, reg, (double)(K + 1),
                          users_sorted_scatter() ? nullptr : uslots);
  const Tensor &ru = std::get<0>(eg), &ri = std::get<1>(eg), &iu = std::get<2>(eg),
               &ii = std::get<3>(eg);
  StepAdam sa;
  sa.user_slot = uslots[0];
  sa.user_count = uslots[1];
  sa.user = AdamTable{u0, m_u, v_u, (float)lr, (float)beta1, (float)beta2, (float)eps, (float)wd,
                      (float)bc1_u, (float)bc2s_u};
  sa.item = AdamTable{i0, m_i, v_i, (float)lr, (float)beta1, (float)beta2, (float)eps, (float)wd,
                      (float)bc1_i, (float)bc2s_i};
  // moments in the graph's row order: only the caller-order weight rows are
  // read and written through the row maps (an input-order pair; otherwise the
  // two orders are one)
  sa.user.moments_graph = sa.item.moments_graph = moments_graph && P->io;
  // graph-ordered master copies of the weights: the Adam reads and writes them
  // with the moments (streamed) and writes the caller's rows only (mirror)
  const bool masters = u_graph.has_value() && u_graph->defined();
  TORCH_CHECK(masters == (i_graph.has_value() && i_graph->defined()),
              "bpr_adam_backward: u_graph and i_graph go together");
  if (masters) {
    TORCH_CHECK(sa.user.moments_graph, "bpr_adam_backward: master copies need an input-order "
                                       "pair with graph-ordered moments");
    TORCH_CHECK(u_graph->sizes() == u0.sizes() && i_graph->sizes() == i0.sizes() &&
                    u_graph->is_contiguous() && i_graph->is_contiguous() &&
                    u_graph->scalar_type() == at::kFloat && i_graph->scalar_type() == at::kFloat,
                "bpr_adam_backward: master copies shaped like the weights (contiguous fp32)");
    sa.user.p = *u_graph;
    sa.user.mirror = u0;
    sa.item.p = *i_graph;
    sa.item.mirror = i0;
  }
  sa.ego_u_vals = ru;
  // the item gradient / gl: the BPR rows, then the ego rows, per item in
  // ascending source order
  // (one sort of the 2B item ids serves this scatter and rows_backward's gI)
  Tensor vi = contrib.narrow(0, B, 2 * B);
  sa.item_plan = plan_rows(ii, I);
  // the two [I, d] item tables: kept all-zero per stream and cleared again at
  // the batch items' rows (ii, clamped to [0, I)), the only rows written
  // (eager only; a table set is dropped, not reused, when the chain throws)
  // (a graph capture gets fresh tables: their fills are then part of the graph)
  const bool cached = !capturing();
  const int64_t skey = (int64_t)(intptr_t)cur_stream();
  std::unique_lock<std::mutex> lk(P->it_mu, std::defer_lock);
  Pair::ItemTables fresh, *tp = &fresh;
  if (cached) {
    lk.lock();
    tp = &P->item_tables(skey);
  }
  Pair::ItemTables &t = *tp;
  if (!t.gi.defined() || t.gi.size(1) != d || t.gi.device() != uf.device()) {
    t.gi = at::zeros({std::max<int64_t>(I, 1), d}, f32(uf));
    t.grad = at::zeros({std::max<int64_t>(I, 1), d}, f32(uf));
  }
  Tensor gi = t.gi.narrow(0, 0, I);
  sa.item_grad = t.grad.narrow(0, 0, I);
  struct Drop {   // a throw leaves rows written: forget the set (fresh zeros next call)
    const Pair &P;
    int64_t key;
    bool armed = true;
    ~Drop() {
      if (armed) P.it.erase(key);
    }
  } drop{*P, skey, cached};
  apply_rows(sa.item_plan, sa.item_grad, vi, ri);
  rows_backward(P, iu, contrib.narrow(0, 0, B), i0, K, true, ii, vi, &sa, gi);
  if (cached)
    for (Tensor *z : {&gi, &sa.item_grad})
      check(bbgr_rows_zero(ii.numel(), ii.data_ptr<int64_t>(), z->data_ptr<float>(), ld(*z),
                           (int32_t)d, cur_stream()),
            "bbgr_rows_zero");
  drop.armed = false;
}

// -- Meta kernels (shapes only; torch.compile traces through them) ---------------
static std::tuple<Tensor, Tensor> propagate_meta(const Tensor &u0, const Tensor &i0, int64_t,
                                                 int64_t, c10::string_view) {
  return {at::empty_like(u0), at::empty_like(i0)};
}
static std::tuple<Tensor, Tensor> propagate_rows_meta(const Tensor &u0, const Tensor &i0,
                                                      const Tensor &, const Tensor &, int64_t,
                                                      int64_t, c10::string_view) {
  return {at::empty_like(u0), at::empty_like(i0)};
}
static std::tuple<Tensor, Tensor> propagate_backward_rows_meta(
    const Tensor &, const Tensor &vu, const Tensor &gI, int64_t num_users, int64_t, int64_t,
    c10::string_view, const c10::optional<Tensor> &, const c10::optional<Tensor> &) {
  return {at::empty({num_users, vu.size(1)}, vu.options()), at::empty_like(gI)};
}
static std::tuple<Tensor, Tensor> jacobi_layer_meta(const Tensor &u, const Tensor &i, int64_t) {
  return {at::empty_like(i), at::empty_like(u)};
}
static std::tuple<Tensor, Tensor> jacobi_layer_backward_meta(const Tensor &g_i, const Tensor &g_u,
                                                             int64_t) {
  return {at::empty_like(g_u), at::empty_like(g_i)};
}
static Tensor propagate_sym_meta(const Tensor &x0, int64_t, int64_t) { return at::empty_like(x0); }
static Tensor bpr_loss_meta(const Tensor &uf, const Tensor &, const Tensor &, const Tensor &,
                            const Tensor &, const Tensor &, const Tensor &, double,
                            const c10::optional<Tensor> &, double) {
  return at::empty({}, uf.options());
}
static std::tuple<Tensor, Tensor, Tensor, Tensor> bpr_loss_backward_meta(
    const Tensor &, const Tensor &uf, const Tensor &itf, const Tensor &ue, const Tensor &ie,
    const Tensor &, const Tensor &, const Tensor &, double, const c10::optional<Tensor> &,
    double) {
  return {at::empty_like(uf), at::empty_like(itf), at::empty_like(ue), at::empty_like(ie)};
}
static Tensor bpr_loss_sparse_ego_meta(const Tensor &uf, const Tensor &, const Tensor &,
                                       const Tensor &, const Tensor &, const Tensor &,
                                       const Tensor &, double, const c10::optional<Tensor> &,
                                       double, bool) {
  return at::empty({}, uf.options());
}
static Tensor bpr_loss_sparse_ego_cuda(const Tensor &uf, const Tensor &itf, const Tensor &ue,
                                       const Tensor &ie, const Tensor &users, const Tensor &pos,
                                       const Tensor &neg, double reg,
                                       const c10::optional<Tensor> &pop, double lambda_fair, bool) {
  return bpr_loss_cuda(uf, itf, ue, ie, users, pos, neg, reg, pop, lambda_fair);
}

// -- dispatcher handles (autograd kernels call below the Autograd key) ----------
template <class Sig>
static c10::TypedOperatorHandle<Sig> op(const char *name) {
  return c10::Dispatcher::singleton().findSchemaOrThrow(name, "").typed<Sig>();
}
using PropSig = std::tuple<Tensor, Tensor>(const Tensor &, const Tensor &, int64_t, int64_t,
                                           c10::string_view);
using RowsSig = std::tuple<Tensor, Tensor>(const Tensor &, const Tensor &, const Tensor &, int64_t,
                                           int64_t, int64_t, c10::string_view,
                                           const c10::optional<Tensor> &,
                                           const c10::optional<Tensor> &);
using LayerSig = std::tuple<Tensor, Tensor>(const Tensor &, const Tensor &, int64_t);
using SymSig = Tensor(const Tensor &, int64_t, int64_t);
using BprSig = Tensor(const Tensor &, const Tensor &, const Tensor &, const Tensor &,
                      const Tensor &, const Tensor &, const Tensor &, double,
                      const c10::optional<Tensor> &, double);
using BprBwdSig = std::tuple<Tensor, Tensor, Tensor, Tensor>(
    const Tensor &, const Tensor &, const Tensor &, const Tensor &, const Tensor &, const Tensor &,
    const Tensor &, const Tensor &, double, const c10::optional<Tensor> &, double);
using BprSeSig = Tensor(const Tensor &, const Tensor &, const Tensor &, const Tensor &,
                        const Tensor &, const Tensor &, const Tensor &, double,
                        const c10::optional<Tensor> &, double, bool);

// -- autograd -------------------------------------------------------------------
struct PropagateFn : public torch::autograd::Function<PropagateFn> {
  static variable_list forward(AutogradContext *ctx, const Tensor &u0, const Tensor &i0,
                               int64_t key, int64_t K, c10::string_view order) {
    ctx->saved_data["key"] = key;
    ctx->saved_data["K"] = K;
    ctx->saved_data["order"] = std::string(order);
    ctx->saved_data["su"] = u0.sizes().vec();
    ctx->saved_data["si"] = i0.sizes().vec();
    at::AutoDispatchBelowADInplaceOrView g;
    static auto h = op<PropSig>("bbgr::propagate");
    auto r = h.call(u0, i0, key, K, order);
    return {std::get<0>(r), std::get<1>(r)};
  }
  static variable_list backward(AutogradContext *ctx, variable_list go) {
    auto r = propagate_grads(ctx, go);
    return {r.first, r.second, Tensor(), Tensor(), Tensor()};
  }

  // (grad u0, grad i0) of the linear K-layer chain: a function of dL/d(finals)
  // alone, so the rows forward (PropagateRowsFn) shares it
  static std::pair<Tensor, Tensor> propagate_grads(AutogradContext *ctx, variable_list go) {
    const int64_t key = ctx->saved_data["key"].toInt(), K = ctx->saved_data["K"].toInt();
    const std::string order = ctx->saved_data["order"].toStringRef();
    const auto su = ctx->saved_data["su"].toIntVector(), si = ctx->saved_data["si"].toIntVector();
    Tensor gU = go[0], gI = go[1];
    if (gU.defined() && gU.layout() == at::kSparse) {
      // a BPR-shaped gradient handed over as rows (bbgr::bpr_loss_sparse_ego):
      // dL/d(u_final) always, dL/d(i_final) too when it arrives sparse
      Tensor vals = gU._values();
      static auto h = op<RowsSig>("bbgr::propagate_backward_rows");
      c10::optional<Tensor> ii, vi;
      if (gI.defined() && gI.is_sparse()) {
        ii = gI._indices().select(0, 0);
        vi = gI._values();
        gI = at::empty(si, vals.options());   // shape only: never read
      } else if (!gI.defined()) {
        gI = at::zeros(si, vals.options());
      }
      auto r = h.call(gU._indices().select(0, 0), vals, gI, su[0], key, K, order, ii, vi);
      return {std::get<0>(r), std::get<1>(r)};
    }
    if (gU.defined() && gU.is_sparse()) gU = gU.to_dense();
    if (gI.defined() && gI.is_sparse()) gI = gI.to_dense();
    const Tensor &ref = gU.defined() ? gU : gI;
    if (!gU.defined()) gU = at::zeros(su, ref.options());
    if (!gI.defined()) gI = at::zeros(si, ref.options());
    static auto h = op<PropSig>("bbgr::propagate_backward");
    auto r = h.call(gU, gI, key, K, order);
    return {std::get<0>(r), std::get<1>(r)};
  }
};

using PropRowsSig = std::tuple<Tensor, Tensor>(const Tensor &, const Tensor &, const Tensor &,
                                               const Tensor &, int64_t, int64_t,
                                               c10::string_view);

// bbgr::propagate_rows: the finals valid at the listed rows only; the backward
// is propagate's (the chain is linear: its gradient does not read the forward
// values), so a BPR gradient over those rows flows exactly as through
// bbgr::propagate
struct PropagateRowsFn : public torch::autograd::Function<PropagateRowsFn> {
  static variable_list forward(AutogradContext *ctx, const Tensor &u0, const Tensor &i0,
                               const Tensor &users, const Tensor &items, int64_t key, int64_t K,
                               c10::string_view order) {
    ctx->saved_data["key"] = key;
    ctx->saved_data["K"] = K;
    ctx->saved_data["order"] = std::string(order);
    ctx->saved_data["su"] = u0.sizes().vec();
    ctx->saved_data["si"] = i0.sizes().vec();
    at::AutoDispatchBelowADInplaceOrView g;
    static auto h = op<PropRowsSig>("bbgr::propagate_rows");
    auto r = h.call(u0, i0, users, items, key, K, order);
    return {std::get<0>(r), std::get<1>(r)};
  }
  static variable_list backward(AutogradContext *ctx, variable_list go) {
    auto r = PropagateFn::propagate_grads(ctx, go);
    return {r.first, r.second, Tensor(), Tensor(), Tensor(), Tensor(), Tensor()};
  }
};

struct JacobiLayerFn : public torch::autograd::Function<JacobiLayerFn> {
  static variable_list forward(AutogradContext *ctx, const Tensor &u, const Tensor &i,
                               int64_t key) {
    ctx->saved_data["key"] = key;
    ctx->saved_data["su"] = u.sizes().vec();
    ctx->saved_data["si"] = i.sizes().vec();
    at::AutoDispatchBelowADInplaceOrView g;
    static auto h = op<LayerSig>("bbgr::jacobi_layer");
    auto r = h.call(u, i, key);
    return {std::get<0>(r), std::get<1>(r)};
  }
  static variable_list backward(AutogradContext *ctx, variable_list go) {
    const int64_t key = ctx->saved_data["key"].toInt();
    const auto su = ctx->saved_data["su"].toIntVector(), si = ctx->saved_data["si"].toIntVector();
    Tensor g_i = go[0], g_u = go[1];
    const Tensor &ref = g_i.defined() ? g_i : g_u;
    if (!g_i.defined()) g_i = at::zeros(si, ref.options());
    if (!g_u.defined()) g_u = at::zeros(su, ref.options());
    if (g_i.is_sparse()) g_i = g_i.to_dense();
    if (g_u.is_sparse()) g_u = g_u.to_dense();
    static auto h = op<LayerSig>("bbgr::jacobi_layer_backward");
    auto r = h.call(g_i, g_u, key);
    return {std::get<0>(r), std::get<1>(r), Tensor()};
  }
};

struct PropagateSymFn : public torch::autograd::Function<PropagateSymFn> {
  static Tensor forward(AutogradContext *ctx, const Tensor &x0, int64_t key, int64_t K) {
    ctx->saved_data["key"] = key;
    ctx->saved_data["K"] = K;
    at::AutoDispatchBelowADInplaceOrView g;
    static auto h = op<SymSig>("bbgr::propagate_sym");
    return h.call(x0, key, K);
  }
  static variable_list backward(AutogradContext *ctx, variable_list go) {
    Tensor g = go[0].is_sparse() ? go[0].to_dense() : go[0];
    static auto h = op<SymSig>("bbgr::propagate_sym_backward");
    return {h.call(g, ctx->saved_data["key"].toInt(), ctx->saved_data["K"].toInt()), Tensor(),
            Tensor()};
  }
};

struct BprFn : public torch::autograd::Function<BprFn> {
  static Tensor forward(AutogradContext *ctx, const Tensor &uf, const Tensor &itf,
                        const Tensor &ue, const Tensor &ie, const Tensor &users,
                        const Tensor &pos, const Tensor &neg, double reg,
                        const c10::optional<Tensor> &pop, double lambda_fair) {
    ctx->save_for_backward({uf, itf, ue, ie, users, pos, neg});
    ctx->saved_data["reg"] = reg;
    ctx->saved_data["lam"] = lambda_fair;
    ctx->saved_data["pop"] = pop ? c10::IValue(*pop) : c10::IValue();
    at::AutoDispatchBelowADInplaceOrView g;
    static auto h = op<BprSig>("bbgr::bpr_loss");
    return h.call(uf, itf, ue, ie, users, pos, neg, reg, pop, lambda_fair);
  }
  static variable_list backward(AutogradContext *ctx, variable_list go) {
    auto s = ctx->get_saved_variables();
    c10::optional<Tensor> pop;
    if (!ctx->saved_data["pop"].isNone()) pop = ctx->saved_data["pop"].toTensor();
    static auto h = op<BprBwdSig>("bbgr::bpr_loss_backward");
    auto r = h.call(go[0], s[0], s[1], s[2], s[3], s[4], s[5], s[6],
                    ctx->saved_data["reg"].toDouble(), pop, ctx->saved_data["lam"].toDouble());
    return {std::get<0>(r), std::get<1>(r), std::get<2>(r), std::get<3>(r), Tensor(), Tensor(),
            Tensor(), Tensor(), Tensor(), Tensor()};
  }
};

// bbgr::bpr_loss whose backward returns the ego-table gradients as sparse COO
// batch rows (eager drop-in step; autograd adds them into propagate's dense
// table in place) and, with sparse_uf, dL/d(u_final) as sparse rows too
// (consumed by propagate's backward without a zero-filled table)
struct BprSparseEgoFn : public torch::autograd::Function<BprSparseEgoFn> {
  static Tensor forward(AutogradContext *ctx, const Tensor &uf, const Tensor &itf,
                        const Tensor &ue, const Tensor &ie, const Tensor &users,
                        const Tensor &pos, const Tensor &neg, double reg,
                        const c10::optional<Tensor> &pop, double lambda_fair, bool sparse_uf) {
    ctx->save_for_backward({uf, itf, ue, ie, users, pos, neg});
    ctx->saved_data["reg"] = reg;
    ctx->saved_data["lam"] = lambda_fair;
    ctx->saved_data["pop"] = pop ? c10::IValue(*pop) : c10::IValue();
    ctx->saved_data["sparse_uf"] = sparse_uf;
    at::AutoDispatchBelowADInplaceOrView g;
    static auto h = op<BprSeSig>("bbgr::bpr_loss_sparse_ego");
    return h.call(uf, itf, ue, ie, users, pos, neg, reg, pop, lambda_fair, sparse_uf);
  }
  static variable_list backward(AutogradContext *ctx, variable_list go) {
    auto s = ctx->get_saved_variables();
    Tensor uf = s[0].contiguous(), itf = s[1].contiguous(), ue = s[2].contiguous(),
           ie = s[3].contiguous();
    Tensor users = idx64(s[4]), pos = idx64(s[5]), neg = idx64(s[6]);
    c10::optional<Tensor> pop;
    if (!ctx->saved_data["pop"].isNone()) pop = ctx->saved_data["pop"].toTensor();
    const double reg = ctx->saved_data["reg"].toDouble();
    const int64_t B = users.numel();
    Tensor dl = go[0].to(at::kFloat).contiguous().reshape({});
    Tensor contrib = at::empty({3 * B, uf.size(1)}, f32(uf));
    bbgr_bpr_args a = bpr_args(users, pos, neg, uf, itf, ue, ie, reg, pop,
                               ctx->saved_data["lam"].toDouble());
    a.dloss = dl.data_ptr<float>();
    a.contrib = contrib.data_ptr<float>();
    a.ldcontrib = ld(contrib);
    check(bbgr_bpr(&a, cur_stream()), "bbgr_bpr");
    auto eg = ego_grad_rows(dl, users, pos, neg, ue, ie, reg);
    const Tensor &ru = std::get<0>(eg), &ri = std::get<1>(eg), &iu = std::get<2>(eg),
                 &ii = std::get<3>(eg);
    Tensor g_uf, g_if;
    if (ctx->saved_data["sparse_uf"].toBool()) {
      // dL/d(u_final) and dL/d(i_final) as rows, summed by propagate's rows
      // backward (bitwise the dense tables on their rows). A dropped triple's
      // rows are +0.0 (the kernel zeroes them): clamped ids add nothing
      g_uf = at::sparse_coo_tensor(iu.unsqueeze(0), contrib.narrow(0, 0, B), uf.sizes());
      g_if = at::sparse_coo_tensor(ii.unsqueeze(0), contrib.narrow(0, B, 2 * B), itf.sizes());
    } else {
      g_uf = at::zeros_like(uf);
      index_add_rows(g_uf, users, contrib.narrow(0, 0, B));
      g_if = at::zeros_like(itf);
      index_add_rows(g_if, at::cat({pos, neg}), contrib.narrow(0, B, 2 * B));
    }
    Tensor g_ue = at::sparse_coo_tensor(iu.unsqueeze(0), ru, ue.sizes());
    Tensor g_ie = at::sparse_coo_tensor(ii.unsqueeze(0), ri, ie.sizes());
    return {g_uf, g_if, g_ue, g_ie, Tensor(), Tensor(), Tensor(), Tensor(), Tensor(), Tensor(),
            Tensor()};
  }
};

static std::tuple<Tensor, Tensor> propagate_autograd(const Tensor &u0, const Tensor &i0,
                                                     int64_t key, int64_t K,
                                                     c10::string_view order) {
  auto r = PropagateFn::apply(u0, i0, key, K, order);
  return {r[0], r[1]};
}
static std::tuple<Tensor, Tensor> propagate_rows_autograd(const Tensor &u0, const Tensor &i0,
                                                          const Tensor &users,
                                                          const Tensor &items, int64_t key,
                                                          int64_t K, c10::string_view order) {
  auto r = PropagateRowsFn::apply(u0, i0, users, items, key, K, order);
  return {r[0], r[1]};
}
static std::tuple<Tensor, Tensor> jacobi_layer_autograd(const Tensor &u, const Tensor &i,
                                                        int64_t key) {
  auto r = JacobiLayerFn::apply(u, i, key);
  return {r[0], r[1]};
}
static Tensor propagate_sym_autograd(const Tensor &x0, int64_t key, int64_t K) {
  return PropagateSymFn::apply(x0, key, K);
}
static Tensor bpr_loss_autograd(const Tensor &uf, const Tensor &itf, const Tensor &ue,
                                const Tensor &ie, const Tensor &users, const Tensor &pos,
                                const Tensor &neg, double reg, const c10::optional<Tensor> &pop,
                                double lambda_fair) {
  return BprFn::apply(uf, itf, ue, ie, users, pos, neg, reg, pop, lambda_fair);
}
static Tensor bpr_loss_sparse_ego_autograd(const Tensor &uf, const Tensor &itf, const Tensor &ue,
                                           const Tensor &ie, const Tensor &users,
                                           const Tensor &pos, const Tensor &neg, double reg,
                                           const c10::optional<Tensor> &pop, double lambda_fair,
                                           bool sparse_uf) {
  return BprSparseEgoFn::apply(uf, itf, ue, ie, users, pos, neg, reg, pop, lambda_fair,
                               sparse_uf);
}

// -- registration of operator pairs ---------------------------------------------
// tensors: per product (fwd_item, fwd_user, bwd_item, bwd_user) 9 entries
//   [indptr, indices, chunks, split, vals, in_scale, out_scale, first_vals,
//    input_indices], then feed_fwd_iu, feed_fwd_ui, feed_bwd_iu, feed_bwd_ui,
//   then user_map, item_map, user_rank, item_rank (input-order pairs).
// meta: per product 10 ints [n_rows, n_cols, nnz, long_threshold, chunk_edges,
//   n_chunks, n_split, cols_by_degree, rows_by_degree, hot_bytes], then U, I.
static constexpr int kTensPerProduct = 9, kMetaPerProduct = 10;

static void register_pair(int64_t key, const std::vector<c10::optional<Tensor>> &t,
                          const std::vector<int64_t> &m) {
  TORCH_CHECK(t.size() == 4 * kTensPerProduct + 8, "_register_pair: tensor list of ", t.size());
  TORCH_CHECK(m.size() == 4 * kMetaPerProduct + 2, "_register_pair: meta list of ", m.size());
  auto P = std::make_shared<Pair>();
  auto get = [&](size_t j) -> Tensor {
    if (!t[j] || !t[j]->defined()) return Tensor();
    P->keep.push_back(*t[j]);
    return *t[j];
  };
  Product *prods[4] = {&P->fi, &P->fu, &P->bi, &P->bu};
  for (int q = 0; q < 4; ++q) {
    Product &pr = *prods[q];
    const size_t b = (size_t)q * kTensPerProduct;
    const int64_t *mm = m.data() + q * kMetaPerProduct;
    Tensor indptr = get(b), indices = get(b + 1), chunks = get(b + 2), split = get(b + 3);
    TORCH_CHECK(indptr.defined() && indices.defined() && indptr.scalar_type() == at::kInt &&
                    indices.scalar_type() == at::kInt,
                "_register_pair: int32 indptr / indices");
    pr.csr.n_rows = (int32_t)mm[0];
    pr.csr.n_cols = (int32_t)mm[1];
    pr.csr.nnz = mm[2];
    pr.csr.indptr = indptr.data_ptr<int32_t>();
    pr.csr.indices = indices.data_ptr<int32_t>();
    pr.csr.long_threshold = (int32_t)mm[3];
    pr.csr.chunk_edges = (int32_t)mm[4];
    pr.csr.n_chunks = (int32_t)mm[5];
    pr.csr.n_split = (int32_t)mm[6];
    pr.csr.chunks = chunks.defined() ? chunks.data_ptr<int32_t>() : nullptr;
    pr.csr.split = split.defined() ? split.data_ptr<int32_t>() : nullptr;
    pr.cols_by_degree = mm[7] != 0;
    pr.rows_by_degree = mm[8] != 0;
    pr.hot_bytes = mm[9];
    Tensor vals = get(b + 4), in_scale = get(b + 5), out_scale = get(b + 6),
           first = get(b + 7), in_idx = get(b + 8);
    pr.vals = vals.defined() ? vals.data_ptr<float>() : nullptr;
    pr.in_scale = in_scale.defined() ? in_scale.data_ptr<float>() : nullptr;
    pr.out_scale = out_scale.defined() ? out_scale.data_ptr<float>() : nullptr;
    pr.first_vals = first.defined() ? first.data_ptr<float>() : nullptr;
    if (in_idx.defined()) {
      pr.has_in = true;
      pr.csr_in = pr.csr;
      pr.csr_in.indices = in_idx.data_ptr<int32_t>();
    }
  }
  const size_t f = 4 * kTensPerProduct;
  Tensor a = get(f), b = get(f + 1), c = get(f + 2), d = get(f + 3);
  P->feed_fwd_iu = a.defined() ? a.data_ptr<float>() : nullptr;
  P->feed_fwd_ui = b.defined() ? b.data_ptr<float>() : nullptr;
  P->feed_bwd_iu = c.defined() ? c.data_ptr<float>() : nullptr;
  P->feed_bwd_ui = d.defined() ? d.data_ptr<float>() : nullptr;
  Tensor um = get(f + 4), im = get(f + 5), ur = get(f + 6), ir = get(f + 7);
  P->U = m[4 * kMetaPerProduct];
  P->I = m[4 * kMetaPerProduct + 1];
  if (um.defined()) {
    TORCH_CHECK(im.defined() && ur.defined() && ir.defined(), "_register_pair: partial io maps");
    P->io = true;
    P->user_map = um;
    P->item_map = im;
    P->item_map64 = im.to(at::kLong);
    P->user_rank64 = ur.to(at::kLong);
    P->item_rank64 = ir.to(at::kLong);
    TORCH_CHECK(P->fi.has_in && P->fu.has_in && P->bi.has_in && P->bu.has_in,
                "_register_pair: input-order pair without input-id columns");
  }
  std::lock_guard<std::mutex> g(g_mu);
  g_pairs[key] = P;
}

static void unregister_pair(int64_t key) {
  std::lock_guard<std::mutex> g(g_mu);
  auto it = g_pairs.find(key);
  if (it == g_pairs.end()) return;
  const Pair &P = *it->second;
  for (const Product *pr : {&P.fi, &P.fu, &P.bi, &P.bu}) {   // its split-row workspaces
    for (auto w = g_ws.begin(); w != g_ws.end();) {
      if (std::get<0>(w->first) == (const void *)pr->csr.indptr) w = g_ws.erase(w);
      else ++w;
    }
  }
  g_pairs.erase(it);
}

// (rows-path backwards, dense backwards) issued so far: tests check which
// backward the autograd graph took
static std::vector<int64_t> counters() { return {g_rows_backward.load(), g_dense_backward.load()}; }

// the in-backward Adam's cached item table sets of a pair (tests bound it)
static int64_t item_table_sets(int64_t key) {
  auto P = pair_of(key);
  std::lock_guard<std::mutex> lk(P->it_mu);
  return (int64_t)P->it.size();
}

}  // namespace bbgr_torch

TORCH_LIBRARY(bbgr, m) {
  m.def("propagate(Tensor u0, Tensor i0, int pair_key, int num_layers, str order) -> (Tensor, Tensor)");
  m.def("propagate_backward(Tensor gU, Tensor gI, int pair_key, int num_layers, str order) -> (Tensor, Tensor)");
  m.def("propagate_rows(Tensor u0, Tensor i0, Tensor users, Tensor items, int pair_key, "
        "int num_layers, str order) -> (Tensor, Tensor)");
  m.def("propagate_backward_rows(Tensor iu, Tensor vu, Tensor gI, int num_users, int pair_key, "
        "int num_layers, str order, Tensor? ii=None, Tensor? vi=None) -> (Tensor, Tensor)");
  m.def("jacobi_layer(Tensor u, Tensor i, int pair_key) -> (Tensor, Tensor)");
  m.def("jacobi_layer_backward(Tensor g_i, Tensor g_u, int pair_key) -> (Tensor, Tensor)");
  m.def("propagate_sym(Tensor x0, int pair_key, int num_layers) -> Tensor");
  m.def("propagate_sym_backward(Tensor g, int pair_key, int num_layers) -> Tensor");
  m.def("bpr_loss(Tensor uf, Tensor itf, Tensor ue, Tensor ie, Tensor users, Tensor pos, "
        "Tensor neg, float reg, Tensor? pop, float lambda_fair) -> Tensor");
  m.def("bpr_loss_backward(Tensor dloss, Tensor uf, Tensor itf, Tensor ue, Tensor ie, "
        "Tensor users, Tensor pos, Tensor neg, float reg, Tensor? pop, float lambda_fair) "
        "-> (Tensor, Tensor, Tensor, Tensor)");
  m.def("bpr_loss_sparse_ego(Tensor uf, Tensor itf, Tensor ue, Tensor ie, Tensor users, "
        "Tensor pos, Tensor neg, float reg, Tensor? pop, float lambda_fair, bool sparse_uf) "
        "-> Tensor");
  m.def("bpr_adam_backward(Tensor dloss, Tensor uf, Tensor itf, Tensor(a!) u0, Tensor(b!) i0, "
        "Tensor users, Tensor pos, Tensor neg, float reg, int pair_key, int num_layers, "
        "Tensor(c!) m_u, Tensor(d!) v_u, Tensor(e!) m_i, Tensor(f!) v_i, float lr, float beta1, "
        "float beta2, float eps, float weight_decay, float bc1_u, float bc2s_u, float bc1_i, "
        "float bc2s_i, bool moments_graph=False, Tensor(g!)? u_graph=None, "
        "Tensor(h!)? i_graph=None) -> ()");
  m.def("propagate_rows_graph(Tensor u0g, Tensor i0g, Tensor users, Tensor items, "
        "int pair_key, int num_layers) -> (Tensor, Tensor)");
  m.def("_register_pair(int key, Tensor?[] tensors, int[] meta) -> ()",
        &bbgr_torch::register_pair);
  m.def("_unregister_pair(int key) -> ()", &bbgr_torch::unregister_pair);
  m.def("_counters() -> int[]", &bbgr_torch::counters);
  m.def("_item_table_sets(int key) -> int", &bbgr_torch::item_table_sets);
}

TORCH_LIBRARY_IMPL(bbgr, CUDA, m) {
  m.impl("propagate", &bbgr_torch::propagate_cuda);
  m.impl("propagate_rows", &bbgr_torch::propagate_rows_cuda);
  m.impl("propagate_backward", &bbgr_torch::propagate_backward_cuda);
  m.impl("propagate_backward_rows", &bbgr_torch::propagate_backward_rows_cuda);
  m.impl("jacobi_layer", &bbgr_torch::jacobi_layer_cuda);
  m.impl("jacobi_layer_backward", &bbgr_torch::jacobi_layer_backward_cuda);
  m.impl("propagate_sym", &bbgr_torch::propagate_sym_cuda);
  m.impl("propagate_sym_backward", &bbgr_torch::propagate_sym_backward_cuda);
  m.impl("bpr_loss", &bbgr_torch::bpr_loss_cuda);
  m.impl("bpr_loss_backward", &bbgr_torch::bpr_loss_backward_cuda);
  m.impl("bpr_loss_sparse_ego", &bbgr_torch::bpr_loss_sparse_ego_cuda);
  m.impl("bpr_adam_backward", &bbgr_torch::bpr_adam_backward_cuda);
  m.impl("propagate_rows_graph", &bbgr_torch::propagate_rows_graph_cuda);
}

TORCH_LIBRARY_IMPL(bbgr, Meta, m) {
  m.impl("propagate", &bbgr_torch::propagate_meta);
  m.impl("propagate_rows", &bbgr_torch::propagate_rows_meta);
  m.impl("propagate_backward", &bbgr_torch::propagate_meta);
  m.impl("propagate_backward_rows", &bbgr_torch::propagate_backward_rows_meta);
  m.impl("jacobi_layer", &bbgr_torch::jacobi_layer_meta);
  m.impl("jacobi_layer_backward", &bbgr_torch::jacobi_layer_backward_meta);
  m.impl("propagate_sym", &bbgr_torch::propagate_sym_meta);
  m.impl("propagate_sym_backward", &bbgr_torch::propagate_sym_meta);
  m.impl("bpr_loss", &bbgr_torch::bpr_loss_meta);
  m.impl("bpr_loss_backward", &bbgr_torch::bpr_loss_backward_meta);
  m.impl("bpr_loss_sparse_ego", &bbgr_torch::bpr_loss_sparse_ego_meta);
}

TORCH_LIBRARY_IMPL(bbgr, Autograd, m) {
  m.impl("propagate", &bbgr_torch::propagate_autograd);
  m.impl("propagate_rows", &bbgr_torch::propagate_rows_autograd);
  m.impl("jacobi_layer", &bbgr_torch::jacobi_layer_autograd);
  m.impl("propagate_sym", &bbgr_torch::propagate_sym_autograd);
  m.impl("bpr_loss", &bbgr_torch::bpr_loss_autograd);
  m.impl("bpr_loss_sparse_ego", &bbgr_torch::bpr_loss_sparse_ego_autograd);
}
