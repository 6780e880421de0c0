/* Host-side ABI check under AddressSanitizer + UndefinedBehaviorSanitizer.
 *
 * Built by `make -C <pkg>/csrc sanitize` from the library's host code only
 * (--cuda-host-only: kernels are stubs, so nothing here may reach a launch)
 * and run by tests/test_sanitize.py on the CPU. It drives every entry
 * point's argument validation and error reporting: each call must return a
 * negative bbgr_status with a message, without touching the device, and
 * without any sanitizer report (invalid reads, overflows, UB in the checks).
 */
#include <stdio.h>
#include <string.h>

#include "bbgr.h"

static int failures = 0;

static void expect_error(const char *what, int rc) {
  const char *msg = bbgr_last_error();
  if (rc >= 0 || !msg || !*msg) {
    fprintf(stderr, "FAIL %s: rc=%d msg=%s\n", what, rc, msg ? msg : "(null)");
    ++failures;
  }
}

static void expect_ok(const char *what, int rc) {
  if (rc != 0) {
    fprintf(stderr, "FAIL %s: rc=%d (%s)\n", what, rc, bbgr_last_error());
    ++failures;
  }
}

int main(void) {
  if (bbgr_abi_version() != BBGR_ABI_VERSION) {
    fprintf(stderr, "FAIL abi version %d\n", bbgr_abi_version());
    return 1;
  }
  bbgr_csr csr;
  memset(&csr, 0, sizeof csr);
  bbgr_spmm_args a;
  memset(&a, 0, sizeof a);
  float f4[16] __attribute__((aligned(16)));
  memset(f4, 0, sizeof f4);

  expect_error("spmm null csr", bbgr_spmm(NULL, &a, NULL));
  expect_error("spmm null args", bbgr_spmm(&csr, NULL, NULL));
  csr.n_rows = -1;
  expect_error("spmm negative rows", bbgr_spmm(&csr, &a, NULL));
  csr.n_rows = 4;
  csr.n_cols = 4;
  csr.nnz = 0;
  csr.indptr = (const int32_t *)f4;
  a.d = 48;
  expect_error("spmm unsupported d", bbgr_spmm(&csr, &a, NULL));
  a.d = 64;
  a.x = f4;
  a.ldx = 63;   /* ld not a multiple of 4 and < d */
  expect_error("spmm bad ld", bbgr_spmm(&csr, &a, NULL));
  a.ldx = 64;
  a.weight_mode = 1;   /* needs edge values */
  expect_error("spmm weight_mode 1 without values", bbgr_spmm(&csr, &a, NULL));
  a.weight_mode = 0;
  a.adam_param = f4;   /* fused Adam without moments */
  expect_error("spmm adam without moments", bbgr_spmm(&csr, &a, NULL));
  a.adam_param = NULL;
  a.use_range = 1;
  a.range[0] = 3;
  a.range[1] = 2;      /* row0 > row1 */
  expect_error("spmm bad range", bbgr_spmm(&csr, &a, NULL));
  a.use_range = 0;
  a.row_list = (const int64_t *)f4;
  a.n_row_list = -5;
  expect_error("spmm negative row list", bbgr_spmm(&csr, &a, NULL));

  expect_error("epilogue null args", bbgr_epilogue(4, f4, 64, NULL, NULL));
  expect_error("epilogue negative rows", bbgr_epilogue(-1, f4, 64, &a, NULL));
  expect_error("bpr null", bbgr_bpr(NULL, NULL));
  expect_error("adam negative n", bbgr_adam(-1, f4, f4, f4, f4, 1e-3f, 0.9f, 0.999f, 1e-8f,
                                            0.f, 1.f, 0.1f, 0.03f, NULL));
  expect_error("adam null tensor", bbgr_adam(4, NULL, f4, f4, f4, 1e-3f, 0.9f, 0.999f, 1e-8f,
                                             0.f, 1.f, 0.1f, 0.03f, NULL));
  expect_ok("adam empty", bbgr_adam(0, NULL, NULL, NULL, NULL, 1e-3f, 0.9f, 0.999f, 1e-8f,
                                    0.f, 1.f, 0.1f, 0.03f, NULL));
  expect_error("adam_dev null state", bbgr_adam_dev(4, f4, f4, f4, f4, 1e-3f, 0.9f, 0.999f,
                                                    1e-8f, 0.f, 1.f, f4, NULL, NULL));
  expect_error("step_begin null", bbgr_step_begin(NULL, NULL));
  expect_error("sample bad sizes", bbgr_sample(1, NULL, NULL, NULL, 0, NULL, 0.f, 5, 1, 0,
                                               NULL, NULL, NULL, NULL));
  expect_error("sample_dev null state", bbgr_sample_dev(1, NULL, NULL, NULL, 5, NULL, 0.f, 5,
                                                        1, NULL, NULL, NULL, NULL, NULL));
  expect_error("plan count null", bbgr_csr_plan_count(NULL, NULL, NULL, NULL, NULL, NULL));
  expect_error("plan build null", bbgr_csr_plan_build(NULL, NULL, NULL, NULL, NULL, NULL));
  expect_error("shuffle null size", bbgr_shuffle(4, NULL, NULL, 1, 1, NULL, NULL, NULL));
  expect_error("mark_rows bad", bbgr_mark_rows(-1, NULL, 1, NULL, 4, NULL));
  expect_error("rows_zero bad", bbgr_rows_zero(-1, NULL, NULL, 64, 64, NULL));
  expect_error("row_support bad ld", bbgr_row_support(4, 64, f4, 32, NULL, NULL, NULL, NULL,
                                                      NULL));
  expect_error("row_support csr without nbr", bbgr_row_support(4, 64, f4, 64, (uint8_t *)f4,
                                                               (const int32_t *)f4, NULL, NULL,
                                                               NULL));
  expect_ok("row_support empty", bbgr_row_support(0, 64, NULL, 64, NULL, NULL, NULL, NULL, NULL));
  expect_error("spmm_f32 null csr", bbgr_spmm_f32(NULL, f4, 64, f4, 64, 64, NULL, NULL, NULL,
                                                   0.f, NULL));
  csr.n_split = 1;
  expect_error("spmm_f32 split rows", bbgr_spmm_f32(&csr, f4, 64, f4, 64, 64, NULL, NULL, NULL,
                                                     0.f, NULL));
  csr.n_split = 0;
  expect_error("bpr_fwd_bwd null", bbgr_bpr_fwd_bwd(NULL, NULL));
  expect_error("adam_f32 negative n", bbgr_adam_f32(-1, f4, f4, f4, f4, 1e-3f, 0.9f, 0.999f,
                                                    1e-8f, 0.f, 1.f, 1.f, 1.f, NULL));
  expect_error("allreduce null comm", bbgr_allreduce_items(NULL, f4, 4, NULL));
  expect_error("comm_allreduce null comm", bbgr_comm_allreduce(NULL, f4, 4, BBGR_DT_F32,
                                                               BBGR_RED_SUM, NULL));
  expect_error("comm_allreduce bad dtype", bbgr_comm_allreduce((void *)f4, f4, 4, 9,
                                                               BBGR_RED_SUM, NULL));
  expect_error("comm_allgather null comm", bbgr_comm_allgather(NULL, f4, f4, 4, BBGR_DT_F32,
                                                               NULL));
  expect_error("first_slot bad n", bbgr_first_slot(-1, NULL, 4, NULL, NULL, NULL));
  expect_error("first_slot null", bbgr_first_slot(4, NULL, 4, NULL, NULL, NULL));
  expect_ok("first_slot empty", bbgr_first_slot(0, NULL, 4, NULL, NULL, NULL));
  expect_error("ego_slots bad B", bbgr_ego_slots(-1, NULL, NULL, NULL, 4, 4, NULL, NULL, NULL, NULL,
                                                  NULL, NULL, NULL, NULL));
  expect_error("ego_slots empty table", bbgr_ego_slots(0, NULL, NULL, NULL, 0, 4, NULL, NULL, NULL,
                                                       NULL, NULL, NULL, NULL, NULL));
  expect_error("ego_slots null", bbgr_ego_slots(4, NULL, NULL, NULL, 4, 4, NULL, NULL, NULL, NULL,
                                                NULL, NULL, NULL, NULL));
  expect_ok("ego_slots empty", bbgr_ego_slots(0, NULL, NULL, NULL, 4, 4, NULL, NULL, NULL, NULL,
                                              NULL, NULL, NULL, NULL));
  expect_error("graph_rows bad n", bbgr_graph_rows(-1, NULL, 4, NULL, NULL, NULL));
  {
    size_t sz = 0;
    expect_error("scatter_plan no size", bbgr_scatter_plan(4, NULL, 4, NULL, NULL, NULL));
    expect_error("scatter_plan bad n", bbgr_scatter_plan(-1, NULL, 4, NULL, &sz, NULL));
  }
  expect_error("scatter_apply bad d", bbgr_scatter_apply(4, 4, NULL, NULL, 8, NULL, 0, NULL, 8, 12,
                                                         NULL));
  expect_error("scatter_apply null", bbgr_scatter_apply(4, 4, NULL, NULL, 64, NULL, 0, NULL, 64, 64,
                                                        NULL));
  expect_ok("scatter_apply empty", bbgr_scatter_apply(0, 4, NULL, NULL, 64, NULL, 0, NULL, 64, 64,
                                                      NULL));
  expect_error("graph_rows null", bbgr_graph_rows(4, NULL, 4, NULL, NULL, NULL));
  expect_ok("graph_rows empty", bbgr_graph_rows(0, NULL, 4, NULL, NULL, NULL));
  expect_error("rows_copy bad d", bbgr_rows_copy(4, NULL, f4, 64, f4, 64, 6, NULL));
  expect_ok("rows_copy empty", bbgr_rows_copy(0, NULL, NULL, 64, NULL, 64, 64, NULL));
  expect_error("rows_add_unique bad ld", bbgr_rows_add_unique(4, NULL, f4, 32, f4, 64, 64, 8,
                                                              NULL));
  expect_ok("rows_add_unique empty", bbgr_rows_add_unique(0, NULL, NULL, 64, NULL, 64, 64, 8,
                                                          NULL));
  {
    size_t need = 0;   /* sort path from 4M ids: a workspace query only */
    expect_ok("degree_count_ws sort query",
              bbgr_degree_count_ws((int64_t)1 << 23, NULL, 1000, NULL, NULL, &need, NULL));
    if (need < ((size_t)1 << 25)) {
      fprintf(stderr, "degree_count_ws sort workspace too small: %zu\n", need);
      ++failures;
    }
  }
  {
    bbgr_rows_mark_args r;
    memset(&r, 0, sizeof r);
    expect_error("rows_mark null args", bbgr_rows_mark(NULL, NULL));
    expect_error("rows_mark empty tables", bbgr_rows_mark(&r, NULL));
    r.n_users = r.n_items = 4;
    expect_ok("rows_mark nothing listed", bbgr_rows_mark(&r, NULL));
    r.n_users_listed = 2;
    expect_error("rows_mark null arrays", bbgr_rows_mark(&r, NULL));
    r.n_users_listed = -1;
    expect_error("rows_mark negative count", bbgr_rows_mark(&r, NULL));
  }
  expect_error("eval sampled null", bbgr_eval_sampled(NULL, NULL, NULL, NULL));
  expect_error("eval full null", bbgr_eval_full(NULL, NULL, NULL, NULL));

  if (failures) {
    fprintf(stderr, "%d failures\n", failures);
    return 1;
  }
  printf("abi host check ok\n");
  return 0;
}
