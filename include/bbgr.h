/*
 * bbgr.h — C ABI of the MI355X-native LightGCN propagation + BPR training path.
 *
 * One shared library (libbbgr.so, hipcc --offload-arch=gfx950) exports every entry
 * point below. Plain pointers and sizes only: no torch types cross this boundary.
 *
 * Conventions (every entry point):
 *   - Caller-owned DEVICE buffers; no allocation inside hot calls. Entry points that
 *     need scratch take (workspace, workspace_bytes); call them once with
 *     workspace == NULL to query the size.
 *   - Stream-ordered on the hipStream_t passed as `stream` (NULL = default stream).
 *     No host synchronisation except in the entry points documented as "syncs"
 *     (one-time operator planning only).
 *   - Return BBGR_OK (0) or a negative bbgr_status; bbgr_last_error() gives text.
 *   - Re-entrant across distinct streams.
 *   - Index arrays are int32 for CSR structure (nnz < 2^31), int64 for batch
 *     index vectors (they are torch.long in the reference).
 *
 * What each entry point replaces in the reference (paths relative to the
 * reference repo root) is cited on its declaration.
 */
#ifndef BBGR_H
#define BBGR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BBGR_ABI_VERSION 11

typedef enum {
  BBGR_OK = 0,
  BBGR_ERR_INVALID = -1,     /* bad argument (null pointer, size, alignment) */
  BBGR_ERR_UNSUPPORTED = -2, /* valid but not implemented (e.g. emb dim) */
  BBGR_ERR_HIP = -3,         /* a HIP runtime call failed; see bbgr_last_error() */
  BBGR_ERR_WORKSPACE = -4    /* workspace missing or too small */
} bbgr_status;

typedef void *bbgr_stream_t; /* a hipStream_t */

/* ------------------------------------------------------------------------- */
/* Library                                                                    */
/* ------------------------------------------------------------------------- */
int bbgr_abi_version(void);
/* Text for the most recent failure on the calling host thread. */
const char *bbgr_last_error(void);
/* Device properties the planner uses (CU count, arch name). */
int bbgr_device_info(int device, int *cu_count, char *arch_name, int arch_name_len);
/* Blocks until `stream` has drained (the one explicit sync). */
int bbgr_sync(bbgr_stream_t stream);
/* An empty kernel, profile_marker_kernel, of `tag` workgroups (1 <= tag <=   */
/* 1024; ABI 10): bench.py brackets its timed steps with tags 1 / 2 so a      */
/* rocprofv3 trace can be cut at them by dispatch order                       */
/* (tools/summarize_profile.py).                                              */
int bbgr_profile_marker(int32_t tag, bbgr_stream_t stream);

/* ------------------------------------------------------------------------- */
/* CSR structure                                                              */
/*   Replaces: sparse_coo_tensor(...).coalesce() in                           */
/*     Version-2/lighgcn_cu_pop.py:443,450; lightgcn_cu.py:393,397;          */
/*     lightgcn.py:363,372 — and edges_to_user_csr, Version-2:309-327.        */
/*   Duplicate (row,col) pairs are KEPT as repeated entries; summing repeated */
/*   entries in the SpMM is what coalesce()'s value-sum does.                 */
/* ------------------------------------------------------------------------- */

/* Build a row-sorted CSR with columns sorted inside each row (stable:
 * duplicates keep their input order). `perm_out` (nullable) receives, for every
 * CSR slot, the input edge id it came from — used to permute per-edge values.
 * Device arrays: rows[nnz], cols[nnz] -> indptr[n_rows+1], indices[nnz]. */
int bbgr_csr_build(int64_t nnz, const int32_t *rows, const int32_t *cols,
                   int32_t n_rows, int32_t n_cols, int32_t *indptr,
                   int32_t *indices, int32_t *perm_out, void *workspace,
                   size_t *workspace_bytes, bbgr_stream_t stream);

/* Load-balance plan for the SpMM. Rows with degree > long_threshold are cut
 * into chunks of at most chunk_edges edges; each chunk is one 256-thread
 * workgroup. Rows cut into >1 chunk ("split rows") are finished by a fix-up
 * pass. chunks[n_chunks][4] = {row, e_begin, e_end, slot (-1: sole chunk)};
 * split[n_split][4] = {row, slot_begin, n_slots, 0}.                         */
typedef struct {
  int32_t n_rows;
  int32_t n_cols;
  int64_t nnz;
  const int32_t *indptr;  /* [n_rows+1] device */
  const int32_t *indices; /* [nnz] device */
  int32_t long_threshold; /* 0 => default (256) */
  int32_t chunk_edges;    /* 0 => default (2048) */
  int32_t n_chunks;
  int32_t n_split;
  const int32_t *chunks; /* [n_chunks*4] device */
  const int32_t *split;  /* [n_split*4] device */
} bbgr_csr;

/* Counts chunks and split rows for csr->long_threshold / chunk_edges (fills
 * csr-side values into *n_chunks / *n_split). SYNCS `stream` (one-time). */
int bbgr_csr_plan_count(const bbgr_csr *csr, int32_t *n_chunks, int32_t *n_split,
                        void *workspace, size_t *workspace_bytes,
                        bbgr_stream_t stream);
/* Fills chunks[n_chunks*4] and split[n_split*4] (sizes from plan_count). */
int bbgr_csr_plan_build(const bbgr_csr *csr, int32_t *chunks, int32_t *split,
                        void *workspace, size_t *workspace_bytes,
                        bbgr_stream_t stream);

/* out[s] = the slot of b holding the edge of slot s of a, b being a's        */
/* transpose with column-sorted rows (the k-th copy of a duplicate pair maps   */
/* to the k-th copy). One-time; feeds bbgr_mark_slots.                         */
int bbgr_transpose_slots(const bbgr_csr *a, const bbgr_csr *b, int32_t *out,
                         bbgr_stream_t stream);
/* The same map from the two CSR builds' permutations (bbgr_csr_build's      */
/* perm_out of a and of b over ONE edge list: slot -> edge id): out[s] =      */
/* inv(perm_b)[perm_a[s]]. Two O(nnz) passes instead of a binary search per   */
/* edge; equal to bbgr_transpose_slots (the builds' sorts are stable, so the  */
/* k-th copy of a duplicate pair is the k-th in edge order on both sides).    */
/* scratch: nnz int32, distinct from out.                                     */
int bbgr_slots_from_perms(int64_t nnz, const int32_t *perm_a, const int32_t *perm_b,
                          int32_t *out, int32_t *scratch, bbgr_stream_t stream);

/* ------------------------------------------------------------------------- */
/* Vertex order (a one-time relabelling before the CSR build)                 */
/*   The reference indexes users / items in id-map order (Version-2:227-303). */
/*   Numbering the rows of a table by descending degree packs its most        */
/*   gathered rows into one address range: the SpMM then streams the cold     */
/*   rows (bbgr_spmm_args.stream_from) and keeps the hot ones cached. Every   */
/*   operator is permutation-equivariant, so the result is the same model up */
/*   to the row order (and fp32 summation order inside a row).                */
/* ------------------------------------------------------------------------- */
/* degree[j] = number of e < n_ids with ids[e] == j, j < n (exact).           */
int bbgr_degree_count(int64_t n_ids, const int32_t *ids, int32_t n, int32_t *degree,
                      bbgr_stream_t stream);
/* The same with a workspace (query with workspace == NULL): below 4M ids, 8  */
/* replicated counter arrays (one per XCD's workgroups) summed at the end     */
/* (power-law ids contend 8x less; 32*n bytes); from 4M ids on, a radix sort */
/* of the ids, a run-length encode and one scatter of the run lengths (no    */
/* atomics; ~4*n_ids + 8*n bytes + sort scratch). Ids must lie in [0, n).    */
int bbgr_degree_count_ws(int64_t n_ids, const int32_t *ids, int32_t n, int32_t *degree,
                         void *workspace, size_t *workspace_bytes, bbgr_stream_t stream);
/* perm[new] = old id, rank[old] = new id, by descending degree; equal degrees */
/* keep ascending id (stable). Workspace query with workspace == NULL.        */
int bbgr_degree_order(int32_t n, const int32_t *degree, int32_t *perm, int32_t *rank,
                      void *workspace, size_t *workspace_bytes, bbgr_stream_t stream);
/* out[e] = map[ids[e]] for e < n (out may alias ids).                        */
int bbgr_relabel(int64_t n, const int32_t *ids, const int32_t *map, int32_t *out,
                 bbgr_stream_t stream);

/* ------------------------------------------------------------------------- */
/* Operator scale vectors                                                     */
/*   Replaces the numpy weight math of build_message_passing_mats             */
/*   (Version-2/lighgcn_cu_pop.py:429-452), its Method-A variant              */
/*   (version_1/lightgcn_cu_pop_long_tail_exposure.py:362-396),               */
/*   build_cred_weighted_mats (lightgcn_cu.py:368-399) and build_norm_adj     */
/*   (lightgcn.py:352-372).                                                   */
/*                                                                            */
/* Every operator of the reference factors as diag(row) * A * diag(col) over  */
/* the 0/1(+multiplicity) adjacency A:                                        */
/*   item<-user  M = diag(p) A_iu diag(q)      user<-item  M = diag(s) A_ui diag(t)
 *   GS / J : p = t = b, q = c*a, s = a    (a = 1/sqrt(max(deg_u,1)),         */
/*                                          b = 1/sqrt(max(deg_i,1)))         */
/*   Method A: p = t = b*alpha, alpha = 1/log1p(max(deg_i,1))                 */
/*   S (symmetric N x N): p = t = deg_i^-1/2, q = s = deg_u^-1/2 (inf -> 0)   */
/* Outputs (device, fp32): deg_u[U], deg_i[I], p[I], q[U], s[U], t[I],        */
/* pt[I] = p*t, qs[U] = q*s. cred (nullable => all ones) is clipped to [0,1]  */
/* by the caller as the reference loader does.                                */
/* ------------------------------------------------------------------------- */
typedef enum {
  BBGR_OP_GS = 0,       /* Version-2/lighgcn_cu_pop.py (credibility inside messages) */
  BBGR_OP_METHOD_A = 1, /* version_1/lightgcn_cu_pop_long_tail_exposure.py     */
  BBGR_OP_J = 2,        /* lightgcn_cu.py (same weights as GS, Jacobi order)  */
  BBGR_OP_SYM = 3       /* lightgcn.py symmetric normalised adjacency         */
} bbgr_op_kind;

int bbgr_operator_scales(int32_t kind, int32_t n_users, int32_t n_items,
                         const int32_t *indptr_u, const int32_t *indptr_i,
                         const float *cred, float *deg_u, float *deg_i,
                         float *p, float *q, float *s, float *t, float *pt,
                         float *qs, bbgr_stream_t stream);

/* out[e] = scale[indices[e]] for e < nnz: a column scale expanded into CSR
 * slot order, so a chain's first SpMM streams 4 coalesced bytes per edge
 * (weight_mode 1) instead of gathering scale[col] at random (weight_mode 2). */
int bbgr_gather_scale(int64_t nnz, const int32_t *indices, const float *scale,
                      float *out, bbgr_stream_t stream);

/* ------------------------------------------------------------------------- */
/* Fused CSR-SpMM (the hot kernel)                                            */
/*   Replaces torch.sparse.mm at Version-2/lighgcn_cu_pop.py:483-484,         */
/*   lightgcn_cu.py:431,434, lightgcn.py:323 and the autograd backward of     */
/*   each (transposed operator), plus the stack(...).mean(0) layer mean       */
/*   (Version-2:488-489) as a fused accumulate epilogue.                      */
/*                                                                            */
/* For every row r of A:                                                      */
/*   T_r = sum_{e in row r} w_e * x[col_e, :]                                  */
/*        w_e = 1                     (weight_mode 0)                          */
/*        w_e = edge_val[e]           (weight_mode 1, CSR slot order)          */
/*        w_e = col_scale[col_e]*col_scale_s   (weight_mode 2)                 */
/*   y[r]       = ys_r * T_r + as_r * add[r]            (if y   != NULL)      */
/*                ys_r = (y_scale ? y_scale[r] : 1) * y_scale_s               */
/*                as_r = (add_scale ? add_scale[r] : 1) * add_scale_s         */
/*   acc_out[r] = (acc_in[r] + cs_r * T_r) * gamma       (if acc_out != NULL) */
/*                cs_r = (acc_scale ? acc_scale[r] : 1) * acc_scale_s;        */
/*                acc_in NULL => 0                                            */
/* Tables are fp32 row-major with leading dimension ld* (floats, multiple of  */
/* 4, 16-byte aligned base). d in {64, 128, 256}, or 8, 16, 32 for the      */
/* column slices of a column-sharded model (narrow rows: d/4 lanes gather one */
/* row, 16/(d/4) edges per load round, slot sums added by a fixed xor tree).  */
/* src_mask (nullable, [n_cols] bytes): edges whose column is 0 in the mask    */
/*   are skipped — exact when x is zero on those rows (sparse gradients).     */
/* row_mask (nullable, [n_rows] bytes): rows that are 0 are not computed and  */
/*   not written (only the flagged rows of the outputs are needed).           */
/* acc_mask (nullable, [n_rows]): acc_in/acc_out touched only on flagged rows */
/* add_mask (nullable, [n_rows]): add[r] read only on flagged rows (treated   */
/*   as 0 elsewhere — exact when add is zero off the mask).                   */
/* row_list (nullable, int64 [n_row_list]): compute only these rows (short    */
/*   rows on a grid sized by the list; long rows need row_mask set for their  */
/*   chunk workgroups: a row_list without row_mask is rejected when the plan  */
/*   has chunks). Listed rows must be distinct. Launches with any mask or list run as */
/*   `spmm_masked_kernel`, full-CSR launches as `spmm_kernel`.                */
/* use_range != 0: compute only rows [range[0], range[1]), whose long-row     */
/*   chunks are [range[2], range[3]) and split rows [range[4], range[5]) of   */
/*   the plan (all three are row-ordered, so a row range maps to contiguous   */
/*   chunk / split ranges). Lets the sharded step all-reduce item partial     */
/*   sums chunk by chunk, overlapped with the next chunk's SpMM. Combined     */
/*   with row_list (+ row_mask): the short rows are the list's entries (the   */
/*   caller passes the slice of its sorted list inside [range[0], range[1])) */
/*   and the range selects the chunk / split-row sub-ranges only.             */
/* adam_param (nullable): fused optimizer step. The row value the y output    */
/*   would receive (g = ys*T + as*add) is the gradient of that row of         */
/*   adam_param, and bbgr_adam's update (same math, same rounding) is applied */
/*   in place to adam_param / adam_exp_avg / adam_exp_avg_sq (row stride      */
/*   adam_ld). y may then be NULL: the gradient table is never written nor    */
/*   re-read (the last backward product of the training step, V2:862-863).   */
/*   Every row of the launch must be computed (no masks / row lists).         */
/* stream_from > 0: source rows with index >= stream_from are gathered with   */
/*   non-temporal (streaming) loads, so they do not evict the rows below it  */
/*   from L2 / Infinity Cache. Meant for a source table in descending-degree  */
/*   order (bbgr_degree_order), where rows [0, stream_from) are the hot set.  */
/*   Results are unchanged; 0 = every row loaded with the default policy.     */
/* stream_out_from > 0: output rows >= stream_out_from are stored streaming   */
/*   (y, and the fused-Adam parameter row), and the fused Adam's moments are  */
/*   streamed in and out: the next product gathers this table, and only its  */
/*   hot prefix (output table in degree order) is worth keeping cached.       */
/* adam_state (nullable, with adam_bc_table): the fused Adam reads its step t */
/*   from device memory (bbgr_step_begin's state[0]) and its bias corrections */
/*   from adam_bc_table[2(t-1)], [2(t-1)+1] instead of the two float fields,  */
/*   so a captured step (hipGraph) replays with the right t every time.       */
/* y_map / acc_map / add_map (nullable, int32 [n_rows]): row maps of the      */
/*   epilogue's tables. CSR row r writes row y_map[r] of y (and updates row   */
/*   y_map[r] of the fused Adam's tables), reads / writes row acc_map[r] of    */
/*   acc_in / acc_out and reads row add_map[r] of add; acc_mask / add_mask    */
/*   index the mapped rows. Scale vectors stay indexed by r. Lets a graph      */
/*   numbered by descending degree serve tables the caller holds in its own    */
/*   (input) order: the drop-in modules' first products gather input-order    */
/*   rows through input-id column indices, and these maps place every        */
/*   input-order output row, so no table is permuted. stream_out_from must be */
/*   0 when y_map is set.                                                      */
/* src_bits (nullable, with src_mask, d >= 64): a bitmap over this CSR's      */
/*   slots, bit e set iff src_mask[indices[e]] != 0 (bbgr_mark_slots of the    */
/*   source rows' edges). The gather then tests liveness on the bitmap (64     */
/*   edges per test) and loads only live edges' indices: a first backward      */
/*   product over a few batch rows' edges stops scanning every index of the  */
/*   row. Results are bitwise those of src_mask alone (same edges, same      */
/*   order); bits of padding: 3 words beyond nnz/32, readable. With src_bits  */
/*   the rows of one chunk (long_threshold < deg <= chunk_edges) are summed by */
/*   the row's lane group in the chunk workgroup's order (bitwise the same):  */
/*   a listed launch must then list them (row_mask alone no longer sums them) */
/* acc_in_map (nullable, int32 [n_rows]): acc_in's own row map — row r reads */
/*   acc_in row acc_in_map[r] while acc_out is placed by acc_map. Lets a chain */
/*   keep its layer-mean accumulator in the graph's (degree) order between    */
/*   layers: the first layer reads the caller's table through its map, the   */
/*   last writes the caller's order, the middle ones touch no map (random    */
/*   256-byte rows cost ~30 % of a user-side product at C4).                  */
/* row_count (nullable, DEVICE int64, with row_list): the list holds           */
/*   min(n_row_list, *row_count) rows; n_row_list is its capacity. For a list  */
/*   built on the stream (a captured step): a fixed grid of short-row          */
/*   workgroups walks it, so the host never reads the length.                  */
/* adam_grad (nullable, with adam_param; ABI 6): the fused Adam's gradient is */
/*   adam_grad_scale * adam_grad[row] (row stride adam_grad_ld) instead of the */
/*   row value, and y is written as usual: an item-row product of the GS      */
/*   backward carries the item table's Adam step, whose gradient (the sparse  */
/*   BPR rows / (K+1) + ego rows) is final before the product runs, so the   */
/*   separate pass over the item table (28 B / parameter) overlaps the        */
/*   product's gathers. Same rounding as bbgr_adam with grad_scale.          */
/* adam_map (nullable, int32 [n_rows]; ABI 7): the fused Adam's rows (param, */
/*   exp_avg, exp_avg_sq and adam_grad) of CSR row r are row adam_map[r]      */
/*   instead of y_map's: a product that writes y in the graph's order while  */
/*   the weights live in the caller's (the drop-in's in-backward item Adam). */
/* adam_moments_unmapped (ABI 9): nonzero keeps exp_avg / exp_avg_sq at the  */
/*   launch's own row r (the graph's order) while the param and adam_grad    */
/*   follow adam_map: the drop-in optimizer stores its moments in the graph's */
/*   order, so only the caller-order weight row is read and written at       */
/*   random (bbgr.optim.FusedAdam converts them at its state_dict boundary). */
/* src_mask_bits (nullable, with src_mask; ABI 10): the same mask packed one */
/*   bit per source row (bit c & 31 of word c >> 5; bbgr_mask_pack), read by */
/*   the per-edge liveness test instead of the bytes: fewer L2 requests for   */
/*   the same test (degree-ordered hub columns share lines). Bitwise the byte */
/*   mask's result.                                                            */
/* adam_mirror (nullable, with adam_moments_unmapped; ABI 10): adam_param is */
/*   then in the launch's row order as well (row r, like the moments), and   */
/*   every updated param row is also stored to adam_mirror row adam_map[r]   */
/*   (y_map[r] without adam_map), stride adam_ld: the drop-in optimizer keeps */
/*   a graph-ordered master copy of a weight table, streamed with its        */
/*   moments, and the caller's table is only written (no random row read).   */
/* tag_out (nullable, int32 [nnz], with tag_mask [n_cols] bytes; ABI 10): a  */
/*   full launch (no masks, list, range or fused Adam) also writes            */
/*   tag_out[e] = indices[e] with bit 31 set where tag_mask[indices[e]] == 0, */
/*   for every slot e of the CSR. src_tagged (nullable, ABI 10): a launch     */
/*   reads its column indices from src_tagged instead, an index with bit 31   */
/*   set being a dead source skipped as src_mask would skip it (so src_mask   */
/*   and src_bits must be NULL): the src-masked backward user product reads   */
/*   the frontier from the copy the forward's first user product wrote, with  */
/*   no mask load between an index and its gather. Bitwise the src_mask       */
/*   launch. Both need a two-row CSR (nnz <= 24 n_rows) and d >= 64.          */
/* partial: n_chunks*d floats followed by n_chunks int32 arrival counters     */
/*   (zero when allocated; each launch leaves them zero): the last chunk of a */
/*   split row to arrive sums the row's partials in chunk order in the same  */
/*   launch (no separate fix-up kernel). Needed when csr->n_split > 0. Two    */
/*   launches that may run at once (different streams) need two buffers.     */
/* ------------------------------------------------------------------------- */
typedef struct {
  int32_t d;
  const float *x;
  int64_t ldx;
  int32_t weight_mode;
  const float *edge_val;
  const float *col_scale;
  float col_scale_s;
  float *y;
  int64_t ldy;
  const float *y_scale;
  float y_scale_s;
  const float *add;
  int64_t ldadd;
  const float *add_scale;
  float add_scale_s;
  const float *acc_in;
  int64_t ldacc_in;
  float *acc_out;
  int64_t ldacc_out;
  const float *acc_scale;
  float acc_scale_s;
  float gamma;
  float *partial;
  const uint8_t *src_mask;
  const uint8_t *row_mask;
  const uint8_t *acc_mask;
  const uint8_t *add_mask;
  const int64_t *row_list;
  int64_t n_row_list;
  int32_t use_range;
  int32_t range[6];
  float *adam_param;
  float *adam_exp_avg;
  float *adam_exp_avg_sq;
  int64_t adam_ld;
  float adam_lr;
  float adam_beta1;
  float adam_beta2;
  float adam_eps;
  float adam_weight_decay;
  float adam_bias_correction1;
  float adam_bias_correction2_sqrt;
  int32_t stream_from;
  int32_t stream_out_from;
  const float *adam_bc_table;
  const int64_t *adam_state;
  const int32_t *y_map;
  const int32_t *acc_map;
  const int32_t *add_map;
  const uint32_t *src_bits;
  const int64_t *row_count;
  const int32_t *acc_in_map;
  const float *adam_grad;
  int64_t adam_grad_ld;
  float adam_grad_scale;
  const int32_t *adam_map;
  int32_t adam_moments_unmapped;
  int32_t *tag_out;
  const uint8_t *tag_mask;
  const int32_t *src_tagged;
  float *adam_mirror;
  const uint32_t *src_mask_bits;
} bbgr_spmm_args;

int bbgr_spmm(const bbgr_csr *csr, const bbgr_spmm_args *args,
              bbgr_stream_t stream);

/* The SpMM epilogue alone, with T read from a dense table t[n_rows, ldt]
 * (args->x / weight fields ignored; row_mask, acc_mask, add_mask honoured). Used after the RCCL all-reduce of
 * per-rank item partial sums in the user-row-sharded multi-GPU step, where
 * the epilogue cannot run before the sum is complete.
 * args->row_list (nullable): t is COMPACT, t[n_row_list, ldt]; its row j is
 * the sum of output row row_list[j] (< n_rows, the output tables' row count).
 * The sparse frontier exchange all-reduces only those rows. */
int bbgr_epilogue(int32_t n_rows, const float *t, int64_t ldt,
                  const bbgr_spmm_args *args, bbgr_stream_t stream);

/* ------------------------------------------------------------------------- */
/* Fused BPR loss: gather -> dot -> log-sigmoid -> (+reg, +fair) -> grads     */
/*   Replaces LightGCN.bpr_loss, Version-2/lighgcn_cu_pop.py:495-508          */
/*   (== lightgcn.py:333-349 with ego offset; lightgcn_cu.py:635-648 adds     */
/*   lambda_fair * mean(pop[pos] * pos_score)) and its autograd backward.     */
/*                                                                            */
/* Per triple b (u, p, n):                                                    */
/*   s+ = <uf[u], if[p]>, s- = <uf[u], if[n]>                                 */
/*   parts[3b+0] = -log(sigmoid(s+ - s-) + 1e-12)                             */
/*   parts[3b+1] = |ue[u]|^2 + |ie[p]|^2 + |ie[n]|^2   (ego tables)           */
/*   parts[3b+2] = pop ? pop[p] * s+ : 0                                      */
/* loss = mean(parts0) + reg * mean(parts1) + lambda_fair * mean(parts2).     */
/* If grads requested, with G = dloss ? *dloss : 1 (device scalar):           */
/*   g_uf[u] += .., g_if[p] += .., g_if[n] += ..   (dense tables, atomics)    */
/*   g_ue[u] += 2 reg G/B ue[u], g_ie[p|n] += 2 reg G/B ie[p|n]               */
/* Any grad pointer may be NULL to skip it. Index vectors are int64.          */
/* contrib (nullable, [3*batch rows], ld ldcontrib): deterministic mode. The  */
/*   g_uf / g_if terms are NOT scattered; instead row b receives the user    */
/*   term of triple b, row batch+b its pos-item term, row 2*batch+b its      */
/*   neg-item term (zero rows for skipped triples). bbgr_scatter_add_rows   */
/*   then sums them per destination row in a fixed order (bitwise            */
/*   reproducible training step).                                            */
/* A triple with an index outside [0,n_users) / [0,n_items) (e.g. the        */
/* sampler's -1 for a user without positives) contributes zero everywhere.   */
/* Column-sharded tables (each rank holds d of the model's columns): a first  */
/*   call with scores_out writes this shard's (s+, s-, |ue|^2+|ie+|^2+|ie-|^2) */
/*   per triple and nothing else; the caller sums them over the shards        */
/*   (all-reduce, 12 B per triple) and a second call with scores uses the     */
/*   complete sums for the loss parts and the gradient coefficients, writing  */
/*   this shard's columns of the gradient rows.                               */
/* d: 8, 16, 32, 64, 128 or 256 (narrow widths: column shards).               */
/* ------------------------------------------------------------------------- */
typedef struct {
  int64_t batch;
  int32_t d;
  int64_t n_users;                 /* rows of uf / ue (bounds check) */
  int64_t n_items;                 /* rows of itf / ie (bounds check) */
  const int64_t *users;
  const int64_t *pos;
  const int64_t *neg;
  const float *uf; int64_t lduf;   /* final user table */
  const float *itf; int64_t ldif;  /* final item table */
  const float *ue; int64_t ldue;   /* ego user table */
  const float *ie; int64_t ldie;   /* ego item table */
  const float *pop;                /* nullable, [I] */
  float reg;
  float lambda_fair;
  float *parts;                    /* nullable, [3*batch] */
  const float *dloss;              /* nullable device scalar */
  float *g_uf; int64_t ldguf;
  float *g_if; int64_t ldgif;
  float *g_ue; int64_t ldgue;
  float *g_ie; int64_t ldgie;
  float *contrib; int64_t ldcontrib;
  float *scores_out;               /* nullable, [3*batch]: see below */
  const float *scores;             /* nullable, [3*batch]: see below */
} bbgr_bpr_args;

int bbgr_bpr(const bbgr_bpr_args *args, bbgr_stream_t stream);

/* loss[0] = sum(parts0)/B + reg*sum(parts1)/B + lambda_fair*sum(parts2)/B,
 * fixed-order (deterministic) reduction in one workgroup. */
int bbgr_bpr_reduce(int64_t batch, const float *parts, float reg,
                    float lambda_fair, float *loss, bbgr_stream_t stream);

/* ------------------------------------------------------------------------- */
/* Adam (torch.optim.Adam defaults: amsgrad=False, maximize=False)            */
/*   Replaces opt.step() at Version-2/lighgcn_cu_pop.py:863 (Adam lr=1e-3,    */
/*   :793). Host computes bias_correction1 = 1-beta1^t and                    */
/*   bias_correction2_sqrt = sqrt(1-beta2^t) in double, as torch does.        */
/*   m = lerp(m, g, 1-beta1); v = beta2 v + (1-beta2) g^2;                    */
/*   p -= (lr/bc1) * m / (sqrt(v)/bc2_sqrt + eps)   (+ weight_decay*p in g)   */
/*   with g = grad_scale * grad[i] (1.0 = plain Adam; the GS item gradient    */
/*   gI/(K+1) is folded in this way instead of materialising it).             */
/* ------------------------------------------------------------------------- */
int bbgr_adam(int64_t n, float *param, const float *grad, float *exp_avg,
              float *exp_avg_sq, float lr, float beta1, float beta2, float eps,
              float weight_decay, float grad_scale, float bias_correction1,
              float bias_correction2_sqrt, bbgr_stream_t stream);

/* ------------------------------------------------------------------------- */
/* Device-resident step state (graph-captured training steps)                 */
/*   A training step captured once into a hipGraph (torch.cuda.CUDAGraph) and */
/*   replayed must not bake the host's per-step scalars into kernel args.     */
/*   state[4] int64 on the device: state[0] = Adam step t, state[1] = this    */
/*   step's sampler counter, state[2] = the next one, state[3] = the number   */
/*   of steps bc_table holds (>= 1). bbgr_step_begin (one lane): t += 1;      */
/*   state[1] = state[2]; state[2] += 1 -- the same sequence the host keeps   */
/*   for an eager step (counter used, then incremented).                      */
/*   bc_table[2(t-1)] = 1 - beta1^t, bc_table[2(t-1)+1] = sqrt(1 - beta2^t),  */
/*   computed on the host in double as torch does, rounded to float: the     */
/*   device constants are then bit-identical to the host ones.               */
/*   bbgr_adam_dev / bbgr_sample_dev: bbgr_adam / bbgr_sample with t and the  */
/*   counter read from state. Every reader clamps t to [1, state[3]]: a table */
/*   of >= ~20k steps is exact past its end (both corrections are 1.0f).      */
/* ------------------------------------------------------------------------- */
int bbgr_step_begin(int64_t *state, bbgr_stream_t stream);
int bbgr_adam_dev(int64_t n, float *param, const float *grad, float *exp_avg,
                  float *exp_avg_sq, float lr, float beta1, float beta2, float eps,
                  float weight_decay, float grad_scale, const float *bc_table,
                  const int64_t *state, bbgr_stream_t stream);

/* ------------------------------------------------------------------------- */
/* Row utilities for the fused training step                                  */
/* ------------------------------------------------------------------------- */
/* Row utilities skip negative indices (the sampler's -1 "no item").        */
/* table[idx[k], :d] = 0 for k < n (restores all-zero gradient tables). */
int bbgr_rows_zero(int64_t n, const int64_t *idx, float *table, int64_t ld,
                   int32_t d, bbgr_stream_t stream);
/* dst[idx[k], :] += alpha * src[idx[k], :] (atomic; duplicates sum). */
int bbgr_rows_axpy(int64_t n, const int64_t *idx, float alpha, const float *src,
                   int64_t ldsrc, float *dst, int64_t lddst, int32_t d,
                   bbgr_stream_t stream);

/* dst[idx[k], :d] = src[idx[k], :d] for k < n (ABI 6; idx[k] < 0 skipped,  */
/* repeated rows write the same value). d and both ld multiples of 4, tables */
/* 16-byte aligned. Copies a sparse table's batch rows into another.         */
int bbgr_rows_copy(int64_t n, const int64_t *idx, const float *src, int64_t ldsrc,
                   float *dst, int64_t lddst, int32_t d, bbgr_stream_t stream);

/* dst[k, :d] = src[idx[k], :d] for k < n (zero row where idx[k] < 0). d and
 * both ld multiples of 4, tables 16-byte aligned. Compacts frontier rows for
 * the sparse multi-GPU exchange (the inverse is bbgr_epilogue's row_list). */
int bbgr_rows_gather(int64_t n, const int64_t *idx, const float *src, int64_t ldsrc,
                     float *dst, int64_t lddst, int32_t d, bbgr_stream_t stream);

/* bbgr_scatter_add_rows for DISTINCT indices (ABI 6): dst[idx[k], :d] +=     */
/* (0 + src[k, :d]), the same additions a one-addend segment makes, in one   */
/* launch without the sort (a training batch of distinct users). Negative or */
/* >= n_dst indices are skipped; repeated indices are the caller's error.    */
int bbgr_rows_add_unique(int64_t n, const int64_t *idx, const float *src, int64_t ldsrc,
                         float *dst, int64_t lddst, int32_t d, int64_t n_dst,
                         bbgr_stream_t stream);

/* slot[k] = the first k' <= k with ids[k'] == ids[k], for k < n (ABI 6; ids */
/* in [0, n_rows)). first: int32 [n_rows] scratch holding INT32_MAX at every */
/* row (left so on return). The BPR ego rows' "add into the row of the first */
/* occurrence" without a sort: an atomic minimum per row (order-free, so    */
/* deterministic), a gather, and a reset of the touched rows.              */
int bbgr_first_slot(int64_t n, const int64_t *ids, int64_t n_rows, int32_t *first,
                    int64_t *slot, bbgr_stream_t stream);

/* The ego rows' slots of a batch of B (user, pos, neg) triples in three     */
/* launches (ABI 8; bpr.ego_grad_rows, the drop-in step's BPR backward,      */
/* Version-2/lighgcn_cu_pop.py:389-397):                                      */
/*   iu[b] = clamp(users[b], 0, n_users - 1);                                 */
/*   ii[b] = clamp(pos[b], 0, n_items - 1), ii[B + b] = clamp(neg[b], ...);   */
/*   cu[b] = the first b' with iu[b'] == iu[b], or -1 when any id of triple  */
/*           b lies outside its table;                                        */
/*   sp[b] / sn[b] = the first j with ii[j] == ii[b] / ii[B + b].             */
/* first_u [n_users] / first_i [n_items]: int32 scratch holding INT32_MAX at */
/* every row (left so on return), as bbgr_first_slot's.                       */
int bbgr_ego_slots(int64_t B, const int64_t *users, const int64_t *pos, const int64_t *neg,
                   int64_t n_users, int64_t n_items, int32_t *first_u, int32_t *first_i,
                   int64_t *iu, int64_t *ii, int64_t *cu, int64_t *sp, int64_t *sn,
                   bbgr_stream_t stream);

/* The ego-L2 gradient rows of a batch in first-slot form (ABI 10; the       */
/* drop-in step's BPR backward), from bbgr_ego_slots' outputs: slot s of     */
/* g_u [B, d] (s < B, user iu[s]) and of g_i [2B, d] (item ii[s]) receives    */
/* y = (2 reg dloss / B) * e, e its ego row (ue[iu[s]] / ie[ii[s]]), added n  */
/* times from +0.0, n = the slot's occurrences as a first slot (cu / sp / sn) */
/* among the valid triples (cu[b] >= 0); other slots are written zero. Bitwise */
/* bbgr_bpr's ego rows over the compact tables (identical addends, so its     */
/* float atomics' order cannot matter) without their serialisation on a       */
/* popular item's row. counts: int32 [3B] scratch, zero on entry and return.  */
/* scale: every written row is that sum times scale (one rounding; 1 = the    */
/* sum itself; the in-backward Adam's (K+1) * ego rows without a mul launch). */
/* counts_u_out (nullable, int32 [B]): slot s < B's user count n (0 off the   */
/* first slots), for bbgr_rows_add_slots over the same cu.                    */
int bbgr_ego_rows(int64_t B, int32_t d, const int64_t *cu, const int64_t *sp, const int64_t *sn,
                  const int64_t *iu, const int64_t *ii, const float *ue, int64_t ldue,
                  const float *ie, int64_t ldie, const float *dloss, float reg, int32_t *counts,
                  float *g_u, int64_t ldgu, float *g_i, int64_t ldgi, float scale,
                  int32_t *counts_u_out, bbgr_stream_t stream);

/* A row scatter in first-slot form (ABI 10): for every k < n with          */
/* counts[k] > 0 (a leader: counts[k] valid slots k' have slot[k'] == k;    */
/* bbgr_ego_slots' cu and bbgr_ego_rows' counts_u_out), dst[rows[k], :d] +=  */
/* (0 + src[k] + src[k2] + ...) over k and those k' > k in ascending order.  */
/* Bitwise bbgr_scatter_add_rows of the batch's rows (a stable sort's        */
/* segment sums) when the slots of invalid triples (slot -1) hold zero rows, */
/* without the sort (a batch of distinct users: one read per row).          */
int bbgr_rows_add_slots(int64_t n, const int64_t *slot, const int32_t *counts,
                        const int64_t *rows, const float *src, int64_t ldsrc, float *dst,
                        int64_t lddst, int32_t d, int64_t n_dst, bbgr_stream_t stream);

/* out[k] = rank[ids[k]] (rank NULL: ids[k]) for ids[k] in [0, n_rows), else */
/* -1 (ABI 8): a caller's row ids as graph rows in one launch                */
/* (bbgr::propagate_rows' batch lists; the marking kernels skip the -1).     */
int bbgr_graph_rows(int64_t n, const int64_t *ids, int64_t n_rows, const int64_t *rank,
                    int64_t *out, bbgr_stream_t stream);

/* Deterministic index_add_: dst[idx[k], :d] += src[k, :d] for k < n, with   */
/* the addends of each destination row summed in ascending k and added once  */
/* (stable radix sort of idx, then one segment sum per row). Negative or     */
/* >= n_dst indices are skipped. Replaces the autograd scatter of the BPR    */
/* gradient and Tensor.index_add_ (main.py:645-650 scatter_add).             */
int bbgr_scatter_add_rows(int64_t n, const int64_t *idx, const float *src, int64_t ldsrc,
                          float *dst, int64_t lddst, int32_t d, int64_t n_dst,
                          void *workspace, size_t *workspace_bytes, bbgr_stream_t stream);
/* bbgr_scatter_add_rows in two halves (ABI 8), so one sort serves several  */
/* scatters over the same index list (the drop-in backward scatters its     */
/* item rows into two tables and its user rows twice).                      */
/* bbgr_scatter_plan: the stable order of idx into `plan` (device; query    */
/* plan_bytes with plan == NULL: bbgr_scatter_add_rows' workspace size).    */
int bbgr_scatter_plan(int64_t n, const int64_t *idx, int64_t n_dst, void *plan,
                      size_t *plan_bytes, bbgr_stream_t stream);
/* bbgr_scatter_apply: dst[r, :d] += (the ascending sum over k with         */
/* idx[k] == r of src[k, :d], continued over src2[k, :d] when src2 is not    */
/* NULL), each row added once: bitwise bbgr_scatter_add_rows over the        */
/* concatenation [src; src2] with the index list [idx; idx]. n, n_dst and    */
/* idx as planned; the plan may be applied any number of times.             */
int bbgr_scatter_apply(int64_t n, int64_t n_dst, const void *plan, const float *src,
                       int64_t ldsrc, const float *src2, int64_t ldsrc2, float *dst,
                       int64_t lddst, int32_t d, bbgr_stream_t stream);

/* ------------------------------------------------------------------------- */
/* Credibility-GNN edge weights, main.py:677-701:       */
/*   CredModel.ewa_raw: w = max(beta*clamp(attr[:,col_verified],0,1) +       */
/*                              gamma*attr[:,col_align], 0)                  */
/*   CredModel.normalize_per_dst: w~ = w / (sum of w over the edge's dst +   */
/*                                1e-12 (eps))                               */
/* csr: destination-row CSR of the edges (bbgr_csr_build with perm_out);     */
/* perm[k]: input edge id of CSR slot k. w_in (nullable, input-edge order)   */
/* replaces the EWA formula (normalize_per_dst on given weights). Outputs    */
/* (each nullable): w_raw and w_edge in input-edge order, w_csr in CSR order */
/* (the edge values of the aggregation SpMM, CredModel.aggregate = bbgr_spmm */
/* over this CSR). The csr must carry its load-balance plan; per-row sums    */
/* follow it in a fixed order (bitwise deterministic). dst (nullable, input  */
/* order): each edge's destination row; with it w_edge is written by one     */
/* coalesced pass over the edges instead of a scatter through perm.          */
/* Workspace: raw weights in CSR order, per-row sums, chunk partials (+ raw  */
/* weights in input order when w_in and w_raw are both NULL).                */
/* ------------------------------------------------------------------------- */
int bbgr_ewa_normalize(const bbgr_csr *csr, const int32_t *perm, const int32_t *dst,
                       const float *w_in,
                       const float *edge_attr, int64_t lda, int32_t col_verified,
                       int32_t col_align, float beta, float gamma, float eps,
                       float *w_raw, float *w_edge, float *w_csr, void *workspace,
                       size_t *workspace_bytes, bbgr_stream_t stream);

/* mask[idx[k]] = value for k < n; indices outside [0, n_rows) (the sampler's
 * -1, or a caller's stale tail) are skipped. */
int bbgr_mark_rows(int64_t n, const int64_t *idx, uint8_t value, uint8_t *mask,
                   int64_t n_rows, bbgr_stream_t stream);
/* For each listed row r = rows[k]: mask[indices[e]] = value for every edge e of
 * row r (the neighbourhood frontier of a batch). */
int bbgr_mark_neighbors(int64_t n, const int64_t *rows, const int32_t *indptr,
                        const int32_t *indices, uint8_t value, uint8_t *mask,
                        bbgr_stream_t stream);
/* Flag rows in mask and list each newly flagged row once: indptr == NULL —
 * the rows rows[k] (k < n; negative / >= n_rows skipped); else every column
 * indices[e] of every edge e of row rows[k]. A row whose byte was 0 is set to
 * 1 and appended at list[(*count)++] (count: DEVICE int64, list order
 * unspecified; rows already flagged are not listed again). mask: 4-byte
 * aligned, its allocation a whole number of 4-byte words. The frontier of a
 * step as a row list without a scan of the mask (bbgr_spmm_args.row_count). */
int bbgr_mark_list(int64_t n, const int64_t *rows, const int32_t *indptr,
                   const int32_t *indices, uint8_t *mask, int64_t n_rows, int64_t *list,
                   int64_t *count, bbgr_stream_t stream);
/* Slot bitmaps (bbgr_spmm_args.src_bits). tmap = bbgr_transpose_slots of the  */
/* CSR whose rows are listed: for every edge e of row rows[k] (k < n), bit     */
/* tmap[e] of bits is set (set != 0), or its whole 32-bit word cleared          */
/* (set == 0: restores an all-zero bitmap after use). Negative rows skipped.   */
int bbgr_mark_slots(int64_t n, const int64_t *rows, const int32_t *indptr,
                    const int32_t *tmap, uint32_t *bits, int32_t set,
                    bbgr_stream_t stream);
/* A training step's batch bookkeeping in one launch each (ABI 10; the fused  */
/* trainer's frontier step). bbgr_batch_begin = bbgr_mark_rows(users, 1,      */
/* mask_u) + bbgr_mark_list(pos, neg -> mask_i, list) + (user_indptr != NULL) */
/* bbgr_mark_list(every neighbour of the users -> mask_i, list) +            */
/* (slot_bits != NULL) bbgr_mark_slots(users, set); the same masks, list SET */
/* (its order unspecified either way) and bits. bbgr_batch_end restores them:*/
/* mask_u / mask_i bytes of the users, items and neighbours to 0, the slot    */
/* words to 0, *count to 0 (list != NULL), and zeroes the step's sparse       */
/* gradient rows: g_u at the users, g_i and g_side (each nullable) at pos and */
/* neg (d columns). Ids outside the tables (the sampler's -1) are skipped.    */
typedef struct {
  int64_t batch;
  const int64_t *users, *pos, *neg;   /* internal row ids */
  int64_t n_users, n_items;
  const int32_t *user_indptr, *user_indices;   /* user CSR; NULL: no neighbours */
  uint8_t *mask_u, *mask_i;
  int64_t *list, *count;              /* item frontier list (nullable together) */
  const int32_t *slot_map;            /* with slot_bits (nullable together) */
  uint32_t *slot_bits;
  float *g_u, *g_i, *g_side;          /* bbgr_batch_end only, nullable */
  int64_t ld_gu, ld_gi, ld_side;
  int32_t d;
} bbgr_batch_args;
int bbgr_batch_begin(const bbgr_batch_args *args, bbgr_stream_t stream);
/* bits[w] = OR over b < 32 of (mask[32 w + b] != 0) << b, for every word    */
/* w < ceil(n / 32) (ABI 10): a byte mask packed for bbgr_spmm_args.         */
/* src_mask_bits (the bits past n are 0).                                    */
int bbgr_mask_pack(int64_t n, const uint8_t *mask, uint32_t *bits, bbgr_stream_t stream);
int bbgr_batch_end(const bbgr_batch_args *args, bbgr_stream_t stream);
/* The row marking of one bbgr::propagate_rows call in one launch (ABI 11): */
/* the listed users users[k] (k < n_users_listed) and items items[k] (k <    */
/* n_items_listed), caller ids, mapped to graph rows through user_rank /     */
/* item_rank (NULL: the ids are the rows). The same masks, list SETS (orders */
/* unspecified) and counts as bbgr_mark_list(user rows -> mask_u, user_list) */
/* + bbgr_mark_rows(item rows, 1, mask_i) + bbgr_mark_list(item rows ->      */
/* frontier, frontier_list) + (user_indptr != NULL) bbgr_mark_list(every     */
/* neighbour of the user rows in the graph-order user CSR -> frontier,       */
/* frontier_list) + (each nullable) bbgr_mark_rows(users, 1, mask_u_in) and  */
/* bbgr_mark_rows(items, 1, mask_i_in) in the caller's order. Ids outside    */
/* the tables (the sampler's -1) are skipped. mask_u / frontier: 4-byte      */
/* aligned whole words (bbgr_mark_list); the counts are DEVICE int64.        */
typedef struct {
  int64_t n_users_listed, n_items_listed;
  const int64_t *users, *items;                /* caller ids */
  int64_t n_users, n_items;
  const int64_t *user_rank, *item_rank;        /* caller id -> graph row; nullable */
  const int32_t *user_indptr, *user_indices;   /* graph-order user CSR; nullable together */
  uint8_t *mask_u, *mask_i, *frontier;         /* graph order */
  uint8_t *mask_u_in, *mask_i_in;              /* caller order; nullable */
  int64_t *user_list, *user_count, *frontier_list, *frontier_count;
} bbgr_rows_mark_args;
int bbgr_rows_mark(const bbgr_rows_mark_args *args, bbgr_stream_t stream);
/* The same for every CSR row r < n_rows flagged in row_mask: row_mask[r], or
 * row_mask[row_map[r]] when row_map is given (a mask kept in the caller's
 * vertex order over a CSR numbered by descending degree). */
int bbgr_mark_neighbors_of_mask(int64_t n_rows, const uint8_t *row_mask,
                                const int32_t *row_map, const int32_t *indptr,
                                const int32_t *indices, uint8_t value, uint8_t *mask,
                                bbgr_stream_t stream);

/* mask[r] = 1 if row r of x [n_rows, d] (leading dimension ldx) holds a
 * nonzero, else 0 (every row written; -0.0 counts as zero). With a CSR
 * (indptr, indices over the rows of x): nbr_mask[indices[e]] = 1 for every edge
 * of a flagged row (other entries untouched). The gradient support of a
 * backward pass whose caller did not say which rows are live (the registered
 * propagate_backward op: BPR gradients touch only the batch rows). */
int bbgr_row_support(int64_t n_rows, int32_t d, const float *x, int64_t ldx, uint8_t *mask,
                     const int32_t *indptr, const int32_t *indices, uint8_t *nbr_mask,
                     bbgr_stream_t stream);

/* ------------------------------------------------------------------------- */
/* Item exchange over RCCL (the sharded step's per-layer all-reduce of item   */
/* partial sums) for callers without torch.distributed.        */
/* RCCL is resolved at run time (librccl.so.1: the copy already loaded in the */
/* process, else the library path). The communicator is an ncclComm_t.       */
/* ------------------------------------------------------------------------- */
/* id_out: 128 bytes (ncclUniqueId) to hand to every rank (rank 0 creates).  */
int bbgr_comm_unique_id(uint8_t *id_out);
/* Collective over nranks processes (blocks until all have joined); the      */
/* calling thread's current HIP device is the rank's GPU.                    */
int bbgr_comm_init(void **comm_out, int32_t nranks, int32_t rank, const uint8_t *id);
int bbgr_comm_destroy(void *comm);
/* In-place sum over the ranks of items[count] (fp32), stream-ordered.       */
int bbgr_allreduce_items(void *comm, float *items, int64_t count, bbgr_stream_t stream);
/* The sharded step's other collectives on the same communicator (ABI 6), so */
/* a caller can keep EVERY collective of a step on its compute stream, in    */
/* issue order (no hop to a comm stream and back): in-place all-reduce of    */
/* buf[count] and all-gather of count elements per rank into recv[nranks *   */
/* count] (rank-major). dtype: bbgr_dtype; op: bbgr_redop.                   */
typedef enum { BBGR_DT_U8 = 0, BBGR_DT_I32 = 1, BBGR_DT_I64 = 2, BBGR_DT_F32 = 3 } bbgr_dtype;
typedef enum { BBGR_RED_SUM = 0, BBGR_RED_MAX = 1, BBGR_RED_MIN = 2 } bbgr_redop;
int bbgr_comm_allreduce(void *comm, void *buf, int64_t count, int32_t dtype, int32_t op,
                        bbgr_stream_t stream);
int bbgr_comm_allgather(void *comm, const void *send, void *recv, int64_t count,
                        int32_t dtype, bbgr_stream_t stream);

/* ------------------------------------------------------------------------- */
/* Negative / positive sampling                                               */
/*   Replaces the per-user host loop of Version-2/lighgcn_cu_pop.py:835-849:  */
/*   sample_pos_item (:339-343), sample_neg_item_popmix (:349-376),           */
/*   user_has_item (:330-336), uniform sample_neg_item (lightgcn.py:296-300), */
/*   and pop_prob = (deg_i+1)^gamma / (sum + 1e-12)  (:805-810).              */
/* RNG: Philox4x32-10, key = seed, counter = (counter, slot, draw).           */
/* ------------------------------------------------------------------------- */
/* cdf[i] = normalised inclusive prefix sum of (deg_i + 1)^gamma (fp64), the
 * table numpy's Generator.choice(p=pop_prob) searches. */
int bbgr_pop_cdf(int32_t n_items, const int32_t *indptr_i, double gamma,
                 double *cdf, void *workspace, size_t *workspace_bytes,
                 bbgr_stream_t stream);

/* For each b < batch, user u = users[b]:
 *   pos[b] = indices[indptr[u] + floor(U01 * deg_u)]   (-1 if deg_u == 0)
 *   neg[b] = first of <= max_tries candidates not in row u, each drawn from
 *            the pop CDF with probability mix_pop (cdf != NULL) else uniform;
 *            then uniform draws until one is not in row u (capped at
 *            BBGR_NEG_CAP draws; -1 and *fail_count += 1 if none found).
 * indices must be sorted within each row (bbgr_csr_build guarantees it). */
#define BBGR_NEG_CAP 65536
int bbgr_sample(int64_t batch, const int64_t *users, const int32_t *indptr,
                const int32_t *indices, int32_t n_items, const double *cdf,
                float mix_pop, int32_t max_tries, uint64_t seed,
                uint64_t counter, int64_t *pos, int64_t *neg,
                int32_t *fail_count, bbgr_stream_t stream);
int bbgr_sample_dev(int64_t batch, const int64_t *users, const int32_t *indptr,
                    const int32_t *indices, int32_t n_items, const double *cdf,
                    float mix_pop, int32_t max_tries, uint64_t seed,
                    const int64_t *state, int64_t *pos, int64_t *neg,
                    int32_t *fail_count, bbgr_stream_t stream);

/* out = a random permutation of in[0..n) (Philox keys + radix sort), the
 * device form of rng.shuffle(train_users) (Version-2:821). */
int bbgr_shuffle(int64_t n, const int64_t *in, int64_t *out, uint64_t seed,
                 uint64_t counter, void *workspace, size_t *workspace_bytes,
                 bbgr_stream_t stream);

/* Users with at least one edge: out[0..*count) ascending (Version-2:797-798).
 * *count is a DEVICE int64. */
int bbgr_nonempty_rows(int32_t n_rows, const int32_t *indptr, int64_t *out,
                       int64_t *count, void *workspace, size_t *workspace_bytes,
                       bbgr_stream_t stream);

/* Rows flagged in mask[n] (any non-zero byte): out[0..*count) ascending.
 * *count is a DEVICE int64. Same workspace protocol. */
int bbgr_mask_to_list(int64_t n, const uint8_t *mask, int64_t *out, int64_t *count,
                      void *workspace, size_t *workspace_bytes, bbgr_stream_t stream);

/* offs[k] = number of entries of the ascending list[0..*count) below
 * bounds[k] (k < n_bounds; *count is a DEVICE int64): the split of a
 * bbgr_mask_to_list row list at row-range boundaries, computed on the stream
 * so the host copies n_bounds values instead of scanning the mask. */
int bbgr_list_offsets(int32_t n_bounds, const int64_t *bounds, const int64_t *list,
                      const int64_t *count, int64_t *offs, bbgr_stream_t stream);

/* pos[list[j]] = j for j < *count (n_max >= *count: the launch size; list
 * entries < the length of pos; other entries of pos are left alone). With
 * pos as an SpMM's y_map, a row-list product writes listed row list[j]
 * straight to row j of a compact table (the sparse item exchange's payload). */
int bbgr_list_positions(int64_t n_max, const int64_t *list, const int64_t *count,
                        int32_t *pos, bbgr_stream_t stream);

/* ------------------------------------------------------------------------- */
/* Evaluation                                            */
/*   bbgr_eval_sampled replaces evaluate_sampled,                             */
/*   Version-2/lighgcn_cu_pop.py:536-650; bbgr_eval_full replaces             */
/*   evaluate_full_ranking, :652-752 (both + metrics_at_k :514-531,           */
/*   novelty_stats_for_items :390-405).                                       */
/* users[n_users]: the evaluated users (rows of the test CSR that are not     */
/* empty, ascending). group[b]: bit0 = top-pct credibility user, bit1 =       */
/* bottom-pct (make_cred_groups :405-422; nullable).                          */
/* Sampled: pos uniform from the test row, n_neg negatives uniform from       */
/*   [0, n_items) rejecting test and train items (duplicates allowed),        */
/*   1+n_neg candidates scored <uf[u], itf[c]> and ranked descending, ties    */
/*   in candidate order (pos first). Writes pos_rank[n_users],                */
/*   topk[n_users*k_max] (-1 padded), optional cand_out[n_users*(1+n_neg)].   */
/*   cand_in (nullable, ABI 10): the candidates are taken from                */
/*   cand_in[b*(1+n_neg) + c] (c = 0 the positive) instead of drawn; the      */
/*   reference's own numpy stream, drawn by bbgr_eval_draw_candidates.        */
/* Full: every item scored <uf[u], itf[i]> with fp32 MFMA (one fmaf chain    */
/*   per score, components in the order 0, d/2, 1, d/2+1, ...), train items   */
/*   set to -1e9, ranked by (score desc, item asc); topk[n_users*k_max] and   */
/*   optional topk_score[n_users*k_max]. k_max <= 32, d in {64, 128}.         */
/* Both write sums[n_k*11] (double) per K =                                   */
/*   {sum P, sum R, sum NDCG, sum avg log(pop+1), sum avg self-info,          */
/*    sum R over high-cred users, sum R over low-cred users, #high, #low,     */
/*    #evaluated users, #distinct top-K items (coverage numerator)},          */
/* reduced in a fixed order (bitwise reproducible).                           */
/* ------------------------------------------------------------------------- */
typedef struct {
  int64_t n_users;
  const int64_t *users;
  const int32_t *te_indptr;
  const int32_t *te_indices;
  const int32_t *tr_indptr;
  const int32_t *tr_indices;
  const float *uf;
  int64_t lduf;
  const float *itf;
  int64_t ldif;
  int32_t d;
  int32_t n_items;
  int32_t n_neg;           /* sampled only */
  int32_t k_max;
  int32_t n_k;
  int32_t ks[8];
  uint64_t seed;           /* sampled only */
  uint64_t counter;        /* sampled only */
  const float *item_pop;
  float self_info_denom;   /* total_train_interactions + n_items */
  const uint8_t *group;
  int32_t *pos_rank;       /* sampled only */
  int32_t *topk;
  float *topk_score;       /* full only, nullable */
  int32_t *cand_out;       /* sampled only, nullable */
  int32_t *fail_count;     /* sampled only, nullable */
  double *sums;
  const int32_t *cand_in;  /* sampled only, nullable (ABI 10) */
} bbgr_eval_args;

int bbgr_eval_sampled(const bbgr_eval_args *args, void *workspace, size_t *workspace_bytes,
                      bbgr_stream_t stream);
int bbgr_eval_full(const bbgr_eval_args *args, void *workspace, size_t *workspace_bytes,
                   bbgr_stream_t stream);

/* The reference's candidate draws, bit for bit (HOST code, host arrays; ABI  */
/* 10). evaluate_sampled (Version-2/lighgcn_cu_pop.py:554-589, the same loop  */
/* in lightgcn.py:406-429, lightgcn_cu.py:496-519,                            */
/* version_1/lightgcn_cu_pop_long_tail_exposure.py:494-517) draws from        */
/* np.random.default_rng(seed + 999), per evaluated user u in order:          */
/*   pos = gt[rng.integers(0, len(gt))]  (gt = the user's test row)           */
/*   repeat until n_neg: j = rng.integers(0, n_items); skip j if j is in gt   */
/*   or user_has_item(train, u, j) (np.searchsorted in the train row, :330);  */
/*   otherwise append j (duplicates kept).                                    */
/* rng is numpy's PCG64 bit generator state (bit_generator.state: the 128-bit */
/* state and increment, has_uint32, uinteger), advanced in place exactly as   */
/* numpy advances it: scalar integers(0, n) on int64 is Lemire's bounded      */
/* draw on buffered 32-bit outputs (n - 1 < 2^32; 64-bit outputs above).      */
/* cand[b*(1+n_neg) + c]: c = 0 the positive, 1.. the negatives. users must   */
/* have non-empty test rows. Returns BBGR_ERR_INVALID if a user cannot get    */
/* n_neg negatives (the reference's loop would not end).                      */
typedef struct {
  uint64_t state_hi, state_lo;   /* the 128-bit LCG state */
  uint64_t inc_hi, inc_lo;       /* the 128-bit increment (odd) */
  int32_t has_uint32;
  uint32_t uinteger;
} bbgr_pcg64;
int bbgr_eval_draw_candidates(bbgr_pcg64 *rng, int64_t n_users, const int64_t *users,
                              const int64_t *te_indptr, const int64_t *te_indices,
                              const int64_t *tr_indptr, const int64_t *tr_indices,
                              int64_t n_items, int32_t n_neg, int32_t *cand);

/* ------------------------------------------------------------------------- */
/* Blueprint names (SURVEY §8(b)'s ABI sketch), thin forms of the above.      */
/* ------------------------------------------------------------------------- */
/* Y = diag(row_scale) A diag(col_scale) X (either scale NULL = ones), one    */
/* fused launch; acc (nullable, leading dimension ldy): acc += acc_scale * Y  */
/* (the layer-mean accumulation). For plans without split rows               */
/* (A->n_split == 0); otherwise use bbgr_spmm with a partial workspace.       */
int bbgr_spmm_f32(const bbgr_csr *A, const float *X, int64_t ldx, float *Y, int64_t ldy,
                  int32_t d, const float *row_scale, const float *col_scale, float *acc,
                  float acc_scale, bbgr_stream_t stream);
/* = bbgr_bpr (loss parts and gradients in one launch). */
int bbgr_bpr_fwd_bwd(const bbgr_bpr_args *args, bbgr_stream_t stream);
/* = bbgr_adam. */
int bbgr_adam_f32(int64_t n, float *param, const float *grad, float *exp_avg,
                  float *exp_avg_sq, float lr, float beta1, float beta2, float eps,
                  float weight_decay, float grad_scale, float bias_correction1,
                  float bias_correction2_sqrt, bbgr_stream_t stream);
/* = bbgr_sample (pop-mix negatives + uniform positives). */
int bbgr_negsample(int64_t batch, const int64_t *users, const int32_t *indptr,
                   const int32_t *indices, int32_t n_items, const double *cdf,
                   float mix_pop, int32_t max_tries, uint64_t seed, uint64_t counter,
                   int64_t *pos, int64_t *neg, int32_t *fail_count, bbgr_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* BBGR_H */
