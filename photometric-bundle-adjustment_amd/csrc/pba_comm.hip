// pba_comm.hip — the collective of the multi-GPU Gauss-Newton loop (include/pba.h, pba_comm_*).
//
// The loop's two sums per LM trial (the banded partial reduced camera systems, then the trial's point-part scalars)
// are enqueued on the engine's stream, so the host never waits for them:
//   * RCCL: ncclAllReduce in place on the engine stream — the one-process-per-GPU path over xGMI.  librccl.so.1 is
//     opened on first use (the same library object torch's ProcessGroupNCCL loaded when torch is in the process).
//   * in-process group: n engines of one process (one host thread each, one device) standing in for ranks, summed in
//     rank order through events and a device kernel — the one-GPU rehearsal of the same stream-ordered loop.
#include <hip/hip_runtime.h>

#include <dlfcn.h>

#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "pba_internal.h"

using namespace pba::detail;

namespace {

// ---- RCCL, resolved at run time -------------------------------------------------------------------------------
// The subset of rccl.h used here (ncclResult_t is an int enum, ncclDataType_t ncclFloat64 = 8, ncclRedOp_t ncclSum = 0).
struct NcclId { char internal[128]; };
typedef int (*GetUniqueIdFn)(NcclId*);
typedef int (*CommInitRankFn)(void** comm, int n, NcclId id, int rank);
typedef int (*CommDestroyFn)(void* comm);
typedef int (*AllReduceFn)(const void*, void*, size_t, int, int, void*, hipStream_t);
typedef const char* (*ErrorStringFn)(int);
constexpr int kNcclFloat64 = 8, kNcclSum = 0;

struct Rccl {
  GetUniqueIdFn get_unique_id = nullptr;
  CommInitRankFn comm_init_rank = nullptr;
  CommDestroyFn comm_destroy = nullptr;
  AllReduceFn all_reduce = nullptr;
  ErrorStringFn error_string = nullptr;
  bool ok = false;
  std::string error;
};

const Rccl& rccl() {
  static Rccl r = [] {
    Rccl x;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      const char* m = dlerror();
      x.error = std::string("librccl.so.1 not loadable: ") + (m ? m : "?");
      return x;
    }
    x.get_unique_id = reinterpret_cast<GetUniqueIdFn>(dlsym(h, "ncclGetUniqueId"));
    x.comm_init_rank = reinterpret_cast<CommInitRankFn>(dlsym(h, "ncclCommInitRank"));
    x.comm_destroy = reinterpret_cast<CommDestroyFn>(dlsym(h, "ncclCommDestroy"));
    x.all_reduce = reinterpret_cast<AllReduceFn>(dlsym(h, "ncclAllReduce"));
    x.error_string = reinterpret_cast<ErrorStringFn>(dlsym(h, "ncclGetErrorString"));
    x.ok = x.get_unique_id && x.comm_init_rank && x.comm_destroy && x.all_reduce;
    if (!x.ok) x.error = "librccl.so.1 lacks an nccl* entry point";
    return x;
  }();
  return r;
}

std::string nccl_error(int rc) {
  const Rccl& r = rccl();
  return "RCCL error " + std::to_string(rc) + (r.error_string ? std::string(": ") + r.error_string(rc) : std::string());
}

// ---- in-process group -----------------------------------------------------------------------------------------
constexpr int kMaxLocalRanks = 16;
struct StagePtrs { const double* p[kMaxLocalRanks]; };

// out[i] = Σ_q stage_q[i] in rank order (every rank computes the same bits)
__global__ void local_sum_kernel(StagePtrs s, int n_ranks, double* __restrict__ out, long long count) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (long long)gridDim.x * blockDim.x) {
    double v = 0.0;
    for (int q = 0; q < n_ranks; ++q) v += s.p[q][i];
    out[i] = v;
  }
}

struct LocalGroup {
  int n = 0;
  std::mutex m;
  std::condition_variable cv;
  int arrived = 0;
  long long generation = 0;
  std::vector<double*> stage;
  std::vector<long long> cap;
  std::vector<hipEvent_t> ev_in, ev_out;
  std::vector<char> out_recorded;

  void barrier() {
    std::unique_lock<std::mutex> lk(m);
    const long long gen = generation;
    if (++arrived == n) {
      arrived = 0;
      ++generation;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return generation != gen; });
    }
  }
  ~LocalGroup() {
    for (double* p : stage)
      if (p) (void)hipFree(p);
    for (hipEvent_t e : ev_in)
      if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : ev_out)
      if (e) (void)hipEventDestroy(e);
  }
};

}  // namespace

struct pba_comm {
  int kind = 0;  // 0: RCCL, 1: in-process group
  int rank = 0, n_ranks = 1, device = 0;
  void* nccl = nullptr;
  std::shared_ptr<LocalGroup> group;
};

namespace pba {
namespace detail {

int comm_rank(const pba_comm* c) { return c->rank; }
int comm_size(const pba_comm* c) { return c->n_ranks; }

// Σ over the ranks of count doubles at buf (device memory), in place, enqueued on stream.  Every rank calls it with the
// same count in the same order.
int comm_allreduce(pba_comm* c, double* buf, long long count, hipStream_t stream) {
  if (count <= 0) return PBA_OK;
  if (c->kind == 0) {
    const int rc = rccl().all_reduce(buf, buf, (size_t)count, kNcclFloat64, kNcclSum, c->nccl, stream);
    if (rc != 0) return fail(PBA_ERR_DEVICE, "ncclAllReduce: " + nccl_error(rc));
    return PBA_OK;
  }
  LocalGroup& G = *c->group;
  const int r = c->rank;
  if (count > G.cap[r]) {  // every rank grows at the same call: no stage is in use once the device is idle
    G.barrier();
    PBA_HIP(hipDeviceSynchronize());
    if (G.stage[r]) PBA_HIP(hipFree(G.stage[r]));
    G.stage[r] = nullptr;
    PBA_HIP(hipMalloc(&G.stage[r], sizeof(double) * (size_t)count));
    G.cap[r] = count;
    G.barrier();
  }
  // this rank's stage is rewritten only after every rank has read it in the previous sum
  for (int q = 0; q < G.n; ++q)
    if (G.out_recorded[q]) PBA_HIP(hipStreamWaitEvent(stream, G.ev_out[q], 0));
  PBA_HIP(hipMemcpyAsync(G.stage[r], buf, sizeof(double) * (size_t)count, hipMemcpyDeviceToDevice, stream));
  PBA_HIP(hipEventRecord(G.ev_in[r], stream));
  G.barrier();  // every rank's stage copy is enqueued and its event recorded
  StagePtrs s{};
  for (int q = 0; q < G.n; ++q) {
    if (q != r) PBA_HIP(hipStreamWaitEvent(stream, G.ev_in[q], 0));
    s.p[q] = G.stage[q];
  }
  const int grid = (int)std::min<long long>(1024, (count + 255) / 256);
  local_sum_kernel<<<grid, 256, 0, stream>>>(s, G.n, buf, count);
  PBA_HIP(hipGetLastError());
  PBA_HIP(hipEventRecord(G.ev_out[r], stream));
  G.out_recorded[r] = 1;
  G.barrier();  // every rank has enqueued its waits on this sum's events before any rank records them again
  return PBA_OK;
}

}  // namespace detail
}  // namespace pba

extern "C" {

int pba_comm_unique_id(void* id) {
  if (!id) return fail(PBA_ERR_INVALID_ARGUMENT, "null id");
  const Rccl& r = rccl();
  if (!r.ok) return fail(PBA_ERR_DEVICE, r.error);
  NcclId x{};
  const int rc = r.get_unique_id(&x);
  if (rc != 0) return fail(PBA_ERR_DEVICE, "ncclGetUniqueId: " + nccl_error(rc));
  std::memcpy(id, &x, sizeof x);
  return PBA_OK;
}

int pba_comm_init(const void* id, int32_t n_ranks, int32_t rank, int32_t device, pba_comm** out) {
  if (!id || !out || n_ranks <= 0 || rank < 0 || rank >= n_ranks) return fail(PBA_ERR_INVALID_ARGUMENT, "bad communicator arguments");
  *out = nullptr;
  const Rccl& r = rccl();
  if (!r.ok) return fail(PBA_ERR_DEVICE, r.error);
  PBA_HIP(hipSetDevice(device));
  NcclId x;
  std::memcpy(&x, id, sizeof x);
  void* comm = nullptr;
  const int rc = r.comm_init_rank(&comm, n_ranks, x, rank);
  if (rc != 0) return fail(PBA_ERR_DEVICE, "ncclCommInitRank: " + nccl_error(rc));
  pba_comm* c = new pba_comm();
  c->kind = 0;
  c->rank = rank;
  c->n_ranks = n_ranks;
  c->device = device;
  c->nccl = comm;
  *out = c;
  return PBA_OK;
}

int pba_comm_init_local(int32_t n_ranks, int32_t device, pba_comm** comms) {
  if (!comms || n_ranks <= 0 || n_ranks > kMaxLocalRanks) return fail(PBA_ERR_INVALID_ARGUMENT, "bad local group arguments");
  PBA_HIP(hipSetDevice(device));
  auto g = std::make_shared<LocalGroup>();
  g->n = n_ranks;
  g->stage.assign(n_ranks, nullptr);
  g->cap.assign(n_ranks, 0);
  g->ev_in.assign(n_ranks, nullptr);
  g->ev_out.assign(n_ranks, nullptr);
  g->out_recorded.assign(n_ranks, 0);
  for (int q = 0; q < n_ranks; ++q) {
    PBA_HIP(hipEventCreateWithFlags(&g->ev_in[q], hipEventDisableTiming));
    PBA_HIP(hipEventCreateWithFlags(&g->ev_out[q], hipEventDisableTiming));
  }
  for (int q = 0; q < n_ranks; ++q) {
    pba_comm* c = new pba_comm();
    c->kind = 1;
    c->rank = q;
    c->n_ranks = n_ranks;
    c->device = device;
    c->group = g;
    comms[q] = c;
  }
  return PBA_OK;
}

int pba_comm_destroy(pba_comm* c) {
  if (!c) return PBA_OK;
  if (c->kind == 0 && c->nccl) (void)rccl().comm_destroy(c->nccl);
  delete c;
  return PBA_OK;
}

int pba_comm_allreduce(pba_comm* c, double* d_buf, int64_t count, void* hip_stream) {
  if (!c || (count > 0 && !d_buf) || count < 0) return fail(PBA_ERR_INVALID_ARGUMENT, "bad allreduce arguments");
  PBA_HIP(hipSetDevice(c->device));
  return comm_allreduce(c, d_buf, count, static_cast<hipStream_t>(hip_stream));
}

int pba_comm_rank(const pba_comm* c) { return c ? c->rank : -1; }
int pba_comm_size(const pba_comm* c) { return c ? c->n_ranks : 0; }

}  // extern "C"
