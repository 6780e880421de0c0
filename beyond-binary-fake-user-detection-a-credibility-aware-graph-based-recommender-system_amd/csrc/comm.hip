// RCCL item exchange behind the C ABI (bbgr_allreduce_items).
//
// The sharded step sums each rank's item-row partial sums over the ranks
// (one all-reduce per item product, pipelined over row ranges). These entry
// points let a C / FFI caller do that without torch.distributed: a
// communicator from an exchanged unique id, and an in-place fp32 sum on a
// caller stream. RCCL is resolved at run time from the copy already loaded in
// the process (torch's, SONAME librccl.so.1) or loaded from the library path,
// so libbbgr.so has no link-time RCCL dependency and never mixes two copies.
#include <dlfcn.h>
#include <rccl/rccl.h>
#include <string.h>

#include "common.h"

namespace bbgr {

struct RcclApi {
  ncclResult_t (*get_unique_id)(ncclUniqueId *);
  ncclResult_t (*comm_init_rank)(ncclComm_t *, int, ncclUniqueId, int);
  ncclResult_t (*comm_destroy)(ncclComm_t);
  ncclResult_t (*all_reduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t,
                             ncclComm_t, hipStream_t);
  ncclResult_t (*all_gather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t,
                             hipStream_t);
  const char *(*error_string)(ncclResult_t);
  bool ok;
};

static RcclApi &rccl() {
  static RcclApi api = [] {
    RcclApi a = {};
    void *h = dlopen("librccl.so.1", RTLD_NOLOAD | RTLD_LAZY);
    if (!h) h = dlopen("librccl.so.1", RTLD_LAZY | RTLD_GLOBAL);
    if (!h) return a;
    a.get_unique_id = reinterpret_cast<decltype(a.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
    a.comm_init_rank = reinterpret_cast<decltype(a.comm_init_rank)>(dlsym(h, "ncclCommInitRank"));
    a.comm_destroy = reinterpret_cast<decltype(a.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
    a.all_reduce = reinterpret_cast<decltype(a.all_reduce)>(dlsym(h, "ncclAllReduce"));
    a.all_gather = reinterpret_cast<decltype(a.all_gather)>(dlsym(h, "ncclAllGather"));
    a.error_string = reinterpret_cast<decltype(a.error_string)>(dlsym(h, "ncclGetErrorString"));
    a.ok = a.get_unique_id && a.comm_init_rank && a.comm_destroy && a.all_reduce &&
           a.all_gather;
    return a;
  }();
  return api;
}

static int rccl_fail(ncclResult_t r, const char *what) {
  const char *msg = rccl().error_string ? rccl().error_string(r) : "?";
  set_error("%s: RCCL error %d (%s)", what, (int)r, msg);
  return BBGR_ERR_HIP;
}

static bool nccl_dtype(int32_t dt, ncclDataType_t *t) {
  switch (dt) {
    case BBGR_DT_U8: *t = ncclUint8; return true;
    case BBGR_DT_I32: *t = ncclInt32; return true;
    case BBGR_DT_I64: *t = ncclInt64; return true;
    case BBGR_DT_F32: *t = ncclFloat32; return true;
    default: return false;
  }
}

static bool nccl_op(int32_t op, ncclRedOp_t *o) {
  switch (op) {
    case BBGR_RED_SUM: *o = ncclSum; return true;
    case BBGR_RED_MAX: *o = ncclMax; return true;
    case BBGR_RED_MIN: *o = ncclMin; return true;
    default: return false;
  }
}

#define BBGR_RCCL(call, what)                              \
  do {                                                     \
    ncclResult_t r_ = (call);                              \
    if (r_ != ncclSuccess) return rccl_fail(r_, what);     \
  } while (0)

}  // namespace bbgr

using namespace bbgr;

extern "C" int bbgr_comm_unique_id(uint8_t *id_out) {
  BBGR_REQUIRE(id_out, "bbgr_comm_unique_id: null id_out");
  BBGR_REQUIRE(rccl().ok, "bbgr_comm_unique_id: librccl.so.1 not found");
  ncclUniqueId id;
  BBGR_RCCL(rccl().get_unique_id(&id), "ncclGetUniqueId");
  memcpy(id_out, id.internal, NCCL_UNIQUE_ID_BYTES);
  return BBGR_OK;
}

extern "C" int bbgr_comm_init(void **comm_out, int32_t nranks, int32_t rank,
                              const uint8_t *id) {
  BBGR_REQUIRE(comm_out && id && nranks > 0 && rank >= 0 && rank < nranks,
               "bbgr_comm_init: bad arguments");
  BBGR_REQUIRE(rccl().ok, "bbgr_comm_init: librccl.so.1 not found");
  ncclUniqueId uid;
  memcpy(uid.internal, id, NCCL_UNIQUE_ID_BYTES);
  ncclComm_t comm = nullptr;
  BBGR_RCCL(rccl().comm_init_rank(&comm, nranks, uid, rank), "ncclCommInitRank");
  *comm_out = comm;
  return BBGR_OK;
}

extern "C" int bbgr_comm_destroy(void *comm) {
  if (!comm) return BBGR_OK;
  BBGR_REQUIRE(rccl().ok, "bbgr_comm_destroy: librccl.so.1 not found");
  BBGR_RCCL(rccl().comm_destroy(static_cast<ncclComm_t>(comm)), "ncclCommDestroy");
  return BBGR_OK;
}

extern "C" int bbgr_allreduce_items(void *comm, float *items, int64_t count,
                                    bbgr_stream_t stream) {
  BBGR_REQUIRE(comm && count >= 0 && (count == 0 || items), "bbgr_allreduce_items: bad args");
  if (count == 0) return BBGR_OK;
  BBGR_REQUIRE(rccl().ok, "bbgr_allreduce_items: librccl.so.1 not found");
  BBGR_RCCL(rccl().all_reduce(items, items, (size_t)count, ncclFloat32, ncclSum,
                              static_cast<ncclComm_t>(comm), as_stream(stream)),
            "ncclAllReduce");
  return BBGR_OK;
}

extern "C" int bbgr_comm_allreduce(void *comm, void *buf, int64_t count, int32_t dtype,
                                   int32_t op, bbgr_stream_t stream) {
  ncclDataType_t t;
  ncclRedOp_t o;
  BBGR_REQUIRE(comm && count >= 0 && (count == 0 || buf) && nccl_dtype(dtype, &t) &&
                   nccl_op(op, &o),
               "bbgr_comm_allreduce: bad args");
  if (count == 0) return BBGR_OK;
  BBGR_REQUIRE(rccl().ok, "bbgr_comm_allreduce: librccl.so.1 not found");
  BBGR_RCCL(rccl().all_reduce(buf, buf, (size_t)count, t, o, static_cast<ncclComm_t>(comm),
                              as_stream(stream)),
            "ncclAllReduce");
  return BBGR_OK;
}

extern "C" int bbgr_comm_allgather(void *comm, const void *send, void *recv, int64_t count,
                                   int32_t dtype, bbgr_stream_t stream) {
  ncclDataType_t t;
  BBGR_REQUIRE(comm && count >= 0 && (count == 0 || (send && recv)) && nccl_dtype(dtype, &t),
               "bbgr_comm_allgather: bad args");
  if (count == 0) return BBGR_OK;
  BBGR_REQUIRE(rccl().ok, "bbgr_comm_allgather: librccl.so.1 not found");
  BBGR_RCCL(rccl().all_gather(send, recv, (size_t)count, t, static_cast<ncclComm_t>(comm),
                              as_stream(stream)),
            "ncclAllGather");
  return BBGR_OK;
}
