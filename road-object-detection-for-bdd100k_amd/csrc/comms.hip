// comms.hip — the data-parallel reduce point of the C ABI: one RCCL
// communicator per process and an in-place, stream-ordered bucket all-reduce (sum) of the flat
// gradient — the exchange train.py's single-device optimizer step (net_tools.py:645-651) turns
// into under data parallelism.  RCCL is bound at run time (dlopen of librccl.so.1: the copy the
// process has already loaded, PyTorch's, is reused, so librod adds no second RCCL and no link
// dependency).  The communicator is created from a 128-byte unique id that rank 0 makes
// (rod_rccl_unique_id) and the caller distributes (any rendezvous: torch.distributed's store in
// rod/ddp.py).  Nothing here allocates device memory; the all-reduce is stream-ordered and
// capturable into a HIP graph like any RCCL collective.
#include <dlfcn.h>
#include <string.h>

#include <mutex>

#include "rod_common.h"

namespace {

// ncclUniqueId is a struct of 128 bytes passed BY VALUE to ncclCommInitRank
struct Uid {
  char internal[128];
};

typedef int (*InitRankFn)(void**, int, Uid, int);

std::mutex g_mu;
void* g_lib = nullptr;
int (*g_get_uid)(Uid*) = nullptr;
InitRankFn g_init_rank = nullptr;
int (*g_allreduce)(const void*, void*, size_t, int, int, void*, hipStream_t) = nullptr;
int (*g_allgather)(const void*, void*, size_t, int, void*, hipStream_t) = nullptr;
int (*g_destroy)(void*) = nullptr;
const char* (*g_errstr)(int) = nullptr;
void* g_comm = nullptr;
int g_world = 0;

bool bind() {
  if (g_lib) return true;
  void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);   // the process's RCCL (PyTorch's)
  if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!h) {
    ::rod::set_error("rod_rccl: cannot load librccl.so.1: %s", dlerror());
    return false;
  }
  g_get_uid = (int (*)(Uid*))dlsym(h, "ncclGetUniqueId");
  g_init_rank = (InitRankFn)dlsym(h, "ncclCommInitRank");
  g_allreduce = (int (*)(const void*, void*, size_t, int, int, void*, hipStream_t))dlsym(h, "ncclAllReduce");
  g_allgather = (int (*)(const void*, void*, size_t, int, void*, hipStream_t))dlsym(h, "ncclAllGather");
  g_destroy = (int (*)(void*))dlsym(h, "ncclCommDestroy");
  g_errstr = (const char* (*)(int))dlsym(h, "ncclGetErrorString");
  if (!g_get_uid || !g_init_rank || !g_allreduce || !g_allgather || !g_destroy) {
    ::rod::set_error("rod_rccl: librccl.so.1 lacks the nccl* entry points");
    return false;
  }
  g_lib = h;
  return true;
}

// ncclDataType_t of a librod dtype code (-1: not a collective type)
int nccl_type(int dtype) {
  return dtype == ROD_F32 ? 7 /* ncclFloat32 */ : dtype == ROD_BF16 ? 9 /* ncclBfloat16 */
                                                  : dtype == ROD_I32 ? 2 /* ncclInt32 */ : -1;
}

int fail(const char* what, int rc) {
  ::rod::set_error("%s: RCCL error %d (%s)", what, rc, g_errstr ? g_errstr(rc) : "?");
  return rc > 0 ? rc : ROD_EINVAL;
}

}  // namespace

extern "C" {

int rod_rccl_unique_id(void* out) {
  ROD_CHECK_ARG(out, "rod_rccl_unique_id: NULL output");
  std::lock_guard<std::mutex> lk(g_mu);
  if (!bind()) return ROD_EINVAL;
  Uid u;
  const int rc = g_get_uid(&u);
  if (rc) return fail("rod_rccl_unique_id", rc);
  memcpy(out, u.internal, sizeof(u.internal));
  return 0;
}

int rod_rccl_init(int rank, int world, const void* uid) {
  ROD_CHECK_ARG(uid && world >= 1 && rank >= 0 && rank < world, "rod_rccl_init: bad rank %d / world %d", rank,
                world);
  std::lock_guard<std::mutex> lk(g_mu);
  if (!bind()) return ROD_EINVAL;
  ROD_CHECK_ARG(!g_comm, "rod_rccl_init: a communicator exists (rod_rccl_destroy first)");
  Uid u;
  memcpy(u.internal, uid, sizeof(u.internal));
  void* comm = nullptr;
  const int rc = g_init_rank(&comm, world, u, rank);
  if (rc) return fail("rod_rccl_init", rc);
  g_comm = comm;
  g_world = world;
  return 0;
}

int rod_allreduce_bucket(void* ptr, long count, int dtype, void* stream) {
  ROD_CHECK_ARG(g_comm, "rod_allreduce_bucket: no communicator (rod_rccl_init)");
  ROD_CHECK_ARG(ptr && count >= 0, "rod_allreduce_bucket: bad buffer");
  const int nt = nccl_type(dtype);
  ROD_CHECK_ARG(nt >= 0, "rod_allreduce_bucket: bad dtype %d", dtype);
  if (count == 0) return 0;
  const int rc = g_allreduce(ptr, ptr, (size_t)count, nt, 0 /* ncclSum */, g_comm, ROD_STREAM(stream));
  if (rc) return fail("rod_allreduce_bucket", rc);
  return 0;
}

int rod_allgather(const void* send, void* recv, long count, int dtype, void* stream) {
  ROD_CHECK_ARG(g_comm, "rod_allgather: no communicator (rod_rccl_init)");
  ROD_CHECK_ARG(send && recv && count >= 0, "rod_allgather: bad buffer");
  const int nt = nccl_type(dtype);
  ROD_CHECK_ARG(nt >= 0, "rod_allgather: bad dtype %d", dtype);
  if (count == 0) return 0;
  const int rc = g_allgather(send, recv, (size_t)count, nt, g_comm, ROD_STREAM(stream));
  if (rc) return fail("rod_allgather", rc);
  return 0;
}

int rod_rccl_world(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  return g_comm ? g_world : 0;
}

int rod_rccl_destroy(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_comm) return 0;
  const int rc = g_destroy(g_comm);
  g_comm = nullptr;
  g_world = 0;
  if (rc) return fail("rod_rccl_destroy", rc);
  return 0;
}

}  // extern "C"
