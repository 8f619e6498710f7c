// beast_comm_*: the library's own RCCL communicator (beast_comm_init / destroy and
// the comm argument of the training call), for a caller that drives several GPUs without
// torch.distributed.  The collectives are the ones this path needs and nothing more:
//   * all-reduce MIN / MAX / SUM -- §8e's running bounds (update_weights_bounds*,
//     beast/beast_bspline_tokenizer.py:362-389), the quantile histograms (fit_parameters,
//     :428 process_group) and the BPE setup's token range / code-point presence;
//   * all-gather and all-gather-v -- the replicated BPE loop's one exchange of every rank's
//     distinct words (beast_tokenizer_amd/bpe_train.py GpuBpeOps.gather_words).
// RCCL is bound at run time (dlopen of librccl.so.1 on the first communicator), so the library
// itself needs no RCCL to load, and inside a torch process the RCCL torch already mapped is the
// one used (same soname) rather than a second copy.  One process per GPU is the intended form
// (beast_comm_init_rank over a unique id the caller distributes); beast_comm_init is SURVEY's
// single-process form (ncclCommInitAll: one handle per listed device), whose collectives must be
// issued inside beast_comm_group_start / _end or from one host thread per handle.
//
// beast_comm_init_virtual (SURVEY §4.3 "N virtual ranks on one device", tests): N handles on one
// device, one caller thread per handle; each collective synchronises the caller's stream and
// meets the other ranks in host memory (a barrier, the rank-ordered reduction, a second barrier
// before the staging slots are reused).  It runs every multi-rank code path of the library --
// rank offsets, all-gather-v displacements, the sharded loop's per-pass reductions -- on a
// one-GPU box, where RCCL cannot form a world > 1.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <vector>

#include "common.h"

namespace {

// the rendezvous of a virtual world: one staging slot per rank, a generation barrier
struct VirtualGroup {
  int world = 0;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  bool broken = false;   // a rank timed out: every later barrier fails at once
  int refs = 0;
  std::vector<std::vector<unsigned char>> slot;
};

}  // namespace

struct beast_comm {
  ncclComm_t nc;
  int world, rank, device;
  VirtualGroup* vg;   // non-null: a virtual rank
  int32_t* scratch;   // device int32[4] on `device`: status agreement
};

namespace {

struct Rccl {
  ncclResult_t (*get_unique_id)(ncclUniqueId*);
  ncclResult_t (*init_rank)(ncclComm_t*, int, ncclUniqueId, int);
  ncclResult_t (*init_all)(ncclComm_t*, int, const int*);
  ncclResult_t (*destroy)(ncclComm_t);
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t);
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t);
  ncclResult_t (*broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
  ncclResult_t (*group_start)();
  ncclResult_t (*group_end)();
  const char* (*error_string)(ncclResult_t);
  bool ok = false;
};

Rccl g_rccl;
std::once_flag g_rccl_once;

void rccl_load() {
  // the copy already mapped (torch's), else the system one
  void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL | RTLD_NOLOAD);
  if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!h) return;
  bool all = true;
  auto sym = [&](auto& fn, const char* name) {
    fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
    all = all && fn != nullptr;
  };
  sym(g_rccl.get_unique_id, "ncclGetUniqueId");
  sym(g_rccl.init_rank, "ncclCommInitRank");
  sym(g_rccl.init_all, "ncclCommInitAll");
  sym(g_rccl.destroy, "ncclCommDestroy");
  sym(g_rccl.all_reduce, "ncclAllReduce");
  sym(g_rccl.all_gather, "ncclAllGather");
  sym(g_rccl.broadcast, "ncclBroadcast");
  sym(g_rccl.group_start, "ncclGroupStart");
  sym(g_rccl.group_end, "ncclGroupEnd");
  sym(g_rccl.error_string, "ncclGetErrorString");
  g_rccl.ok = all;
}

const Rccl* rccl() {
  std::call_once(g_rccl_once, rccl_load);
  return g_rccl.ok ? &g_rccl : nullptr;
}

int nccl_fail(ncclResult_t r, const char* what) {
  beast::set_error("%s: RCCL error %d (%s)", what, (int)r, g_rccl.error_string ? g_rccl.error_string(r) : "?");
  return BEAST_E_HIP;
}

#define BEAST_NCCL(call, what)                          \
  do {                                                  \
    const ncclResult_t r_ = (call);                     \
    if (r_ != ncclSuccess) return nccl_fail(r_, what);  \
  } while (0)

#define BEAST_NEED_RCCL(R)                                                                           \
  const Rccl* R = rccl();                                                                            \
  BEAST_REQUIRE_CODE(R != nullptr, BEAST_E_UNSUPPORTED, "beast_comm: librccl.so.1 could not be loaded")

bool dtype_of(int dt, ncclDataType_t* out, size_t* bytes) {
  switch (dt) {
    case BEAST_DT_U8: *out = ncclUint8; *bytes = 1; return true;
    case BEAST_DT_I32: *out = ncclInt32; *bytes = 4; return true;
    case BEAST_DT_U32: *out = ncclUint32; *bytes = 4; return true;
    case BEAST_DT_I64: *out = ncclInt64; *bytes = 8; return true;
    case BEAST_DT_U64: *out = ncclUint64; *bytes = 8; return true;
    case BEAST_DT_F32: *out = ncclFloat32; *bytes = 4; return true;
    case BEAST_DT_F64: *out = ncclFloat64; *bytes = 8; return true;
    default: return false;
  }
}

bool op_of(int op, ncclRedOp_t* out) {
  switch (op) {
    case BEAST_OP_SUM: *out = ncclSum; return true;
    case BEAST_OP_MIN: *out = ncclMin; return true;
    case BEAST_OP_MAX: *out = ncclMax; return true;
    default: return false;
  }
}

// a scratch int32[4] on `device` (the current device is restored)
int alloc_scratch(int device, int32_t** out) {
  int prev = 0;
  BEAST_HIP(hipGetDevice(&prev), "hipGetDevice");
  BEAST_HIP(hipSetDevice(device), "hipSetDevice");
  const hipError_t e = hipMalloc(reinterpret_cast<void**>(out), 4 * sizeof(int32_t));
  (void)hipSetDevice(prev);
  BEAST_HIP(e, "communicator scratch");
  return BEAST_OK;
}

// ---------------------------------------------------------------- virtual ranks --
// a barrier of the virtual world; fails (every rank alike) when a rank does not arrive within the
// timeout -- a rank that returned early must not leave the others blocked forever
int vbarrier(VirtualGroup* g, const char* what) {
  std::unique_lock<std::mutex> lk(g->mu);
  BEAST_REQUIRE_CODE(!g->broken, BEAST_E_HIP, "%s: a virtual rank failed to arrive earlier; the group is broken", what);
  const uint64_t gen = g->gen;
  if (++g->arrived == g->world) {
    g->arrived = 0;
    ++g->gen;
    g->cv.notify_all();
    return BEAST_OK;
  }
  const bool ok = g->cv.wait_for(lk, std::chrono::seconds(120), [&] { return g->gen != gen || g->broken; });
  if (!ok || g->broken) {
    g->broken = true;
    g->cv.notify_all();
    beast::set_error("%s: virtual ranks did not all arrive (timeout or an earlier failure)", what);
    return BEAST_E_HIP;
  }
  return BEAST_OK;
}

// stage `bytes` of this rank's device buffer into its slot (the stream synchronised first, so the
// buffer holds what the stream-ordered caller wrote)
int vstage(beast_comm* c, const void* send, size_t bytes, hipStream_t s, const char* what) {
  BEAST_HIP(hipStreamSynchronize(s), what);
  std::vector<unsigned char>& slot = c->vg->slot[c->rank];
  slot.resize(bytes);
  if (bytes) {
    BEAST_HIP(hipMemcpyAsync(slot.data(), send, bytes, hipMemcpyDeviceToHost, s), what);
    BEAST_HIP(hipStreamSynchronize(s), what);
  }
  return BEAST_OK;
}

template <class T>
void vreduce(VirtualGroup* g, int op, int64_t count, std::vector<unsigned char>& out) {
  out.assign(g->slot[0].begin(), g->slot[0].end());
  T* acc = reinterpret_cast<T*>(out.data());
  for (int r = 1; r < g->world; ++r) {   // rank order, as a deterministic reduction
    const T* x = reinterpret_cast<const T*>(g->slot[r].data());
    for (int64_t i = 0; i < count; ++i) {
      if (op == BEAST_OP_SUM) acc[i] = static_cast<T>(acc[i] + x[i]);
      else if (op == BEAST_OP_MIN) acc[i] = x[i] < acc[i] ? x[i] : acc[i];
      else acc[i] = acc[i] < x[i] ? x[i] : acc[i];
    }
  }
}

int v_allreduce(beast_comm* c, const void* send, void* recv, int64_t count, int dtype, int op, size_t eb, hipStream_t s) {
  const size_t bytes = (size_t)count * eb;
  if (int rc = vstage(c, send, bytes, s, "virtual allreduce")) return rc;
  if (int rc = vbarrier(c->vg, "virtual allreduce")) return rc;
  std::vector<unsigned char> out;
  switch (dtype) {
    case BEAST_DT_U8: vreduce<uint8_t>(c->vg, op, count, out); break;
    case BEAST_DT_I32: vreduce<int32_t>(c->vg, op, count, out); break;
    case BEAST_DT_U32: vreduce<uint32_t>(c->vg, op, count, out); break;
    case BEAST_DT_I64: vreduce<int64_t>(c->vg, op, count, out); break;
    case BEAST_DT_U64: vreduce<uint64_t>(c->vg, op, count, out); break;
    case BEAST_DT_F32: vreduce<float>(c->vg, op, count, out); break;
    default: vreduce<double>(c->vg, op, count, out); break;
  }
  if (int rc = vbarrier(c->vg, "virtual allreduce")) return rc;   // every rank has read the slots
  BEAST_HIP(hipMemcpyAsync(recv, out.data(), bytes, hipMemcpyHostToDevice, s), "virtual allreduce");
  BEAST_HIP(hipStreamSynchronize(s), "virtual allreduce");   // `out` is freed on return
  return BEAST_OK;
}

// rank r's counts[r] x eb bytes at recv + displs[r] x eb (all-gather: counts = count, displs = r x count)
int v_gather(beast_comm* c, const void* send, void* recv, const int64_t* counts, const int64_t* displs, size_t eb,
             hipStream_t s) {
  if (int rc = vstage(c, send, (size_t)counts[c->rank] * eb, s, "virtual allgather")) return rc;
  if (int rc = vbarrier(c->vg, "virtual allgather")) return rc;
  std::vector<std::vector<unsigned char>> all(c->world);
  for (int r = 0; r < c->world; ++r) all[r] = c->vg->slot[r];
  if (int rc = vbarrier(c->vg, "virtual allgather")) return rc;
  for (int r = 0; r < c->world; ++r)
    if (counts[r] > 0)
      BEAST_HIP(hipMemcpyAsync(static_cast<unsigned char*>(recv) + (size_t)displs[r] * eb, all[r].data(),
                               (size_t)counts[r] * eb, hipMemcpyHostToDevice, s),
                "virtual allgather");
  BEAST_HIP(hipStreamSynchronize(s), "virtual allgather");   // `all` is freed on return
  return BEAST_OK;
}

}  // namespace

extern "C" size_t beast_comm_id_bytes(void) { return NCCL_UNIQUE_ID_BYTES; }

extern "C" int beast_comm_unique_id(void* id_out) {
  BEAST_REQUIRE(id_out != nullptr, "beast_comm_unique_id: null pointer");
  BEAST_NEED_RCCL(R);
  ncclUniqueId id;
  BEAST_NCCL(R->get_unique_id(&id), "ncclGetUniqueId");
  std::memcpy(id_out, &id, sizeof(id));
  return BEAST_OK;
}

extern "C" int beast_comm_init_rank(int world, int rank, const void* id, int device, beast_comm** out) {
  BEAST_REQUIRE(id != nullptr && out != nullptr, "beast_comm_init_rank: null pointer");
  BEAST_REQUIRE(world >= 1 && rank >= 0 && rank < world && device >= 0,
                "beast_comm_init_rank: bad rank %d of world %d on device %d", rank, world, device);
  *out = nullptr;
  BEAST_NEED_RCCL(R);
  int32_t* scratch = nullptr;
  if (int rc = alloc_scratch(device, &scratch)) return rc;
  // RCCL binds the communicator to the current device: switch for the init, then restore the
  // caller's
  int prev = 0;
  BEAST_HIP(hipGetDevice(&prev), "hipGetDevice");
  BEAST_HIP(hipSetDevice(device), "hipSetDevice");
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  ncclComm_t nc = nullptr;
  const ncclResult_t r = R->init_rank(&nc, world, uid, rank);
  (void)hipSetDevice(prev);
  if (r != ncclSuccess) (void)hipFree(scratch);
  BEAST_NCCL(r, "ncclCommInitRank");
  *out = new beast_comm{nc, world, rank, device, nullptr, scratch};
  return BEAST_OK;
}

extern "C" int beast_comm_init(int ndev, const int* devs, beast_comm** out) {
  BEAST_REQUIRE(ndev >= 1 && devs != nullptr && out != nullptr, "beast_comm_init: bad arguments");
  BEAST_NEED_RCCL(R);
  std::vector<int32_t*> scratch(ndev, nullptr);
  for (int i = 0; i < ndev; ++i)
    if (int rc = alloc_scratch(devs[i], &scratch[i])) {
      for (int32_t* p : scratch) (void)hipFree(p);
      return rc;
    }
  std::vector<ncclComm_t> nc(ndev, nullptr);
  const ncclResult_t r = R->init_all(nc.data(), ndev, devs);
  if (r != ncclSuccess)
    for (int32_t* p : scratch) (void)hipFree(p);
  BEAST_NCCL(r, "ncclCommInitAll");
  for (int i = 0; i < ndev; ++i) out[i] = new beast_comm{nc[i], ndev, i, devs[i], nullptr, scratch[i]};
  return BEAST_OK;
}

extern "C" int beast_comm_init_virtual(int n, int device, beast_comm** out) {
  BEAST_REQUIRE(n >= 1 && n <= 64 && device >= 0 && out != nullptr, "beast_comm_init_virtual: bad arguments");
  std::vector<int32_t*> scratch(n, nullptr);
  for (int i = 0; i < n; ++i)
    if (int rc = alloc_scratch(device, &scratch[i])) {
      for (int32_t* p : scratch) (void)hipFree(p);
      return rc;
    }
  VirtualGroup* g = new VirtualGroup();
  g->world = n;
  g->refs = n;
  g->slot.resize(n);
  for (int i = 0; i < n; ++i) out[i] = new beast_comm{nullptr, n, i, device, g, scratch[i]};
  return BEAST_OK;
}

extern "C" int beast_comm_destroy(beast_comm* c) {
  if (c == nullptr) return BEAST_OK;
  if (c->scratch) (void)hipFree(c->scratch);
  if (c->vg != nullptr) {
    VirtualGroup* g = c->vg;
    bool last;
    {
      std::lock_guard<std::mutex> lk(g->mu);
      last = --g->refs == 0;
    }
    delete c;
    if (last) delete g;
    return BEAST_OK;
  }
  BEAST_NEED_RCCL(R);
  const ncclResult_t r = R->destroy(c->nc);
  delete c;
  BEAST_NCCL(r, "ncclCommDestroy");
  return BEAST_OK;
}

extern "C" int beast_comm_info(const beast_comm* c, int* world, int* rank, int* device) {
  BEAST_REQUIRE(c != nullptr, "beast_comm_info: null communicator");
  if (world) *world = c->world;
  if (rank) *rank = c->rank;
  if (device) *device = c->device;
  return BEAST_OK;
}

extern "C" int beast_comm_group_start(void) {
  BEAST_NEED_RCCL(R);
  BEAST_NCCL(R->group_start(), "ncclGroupStart");
  return BEAST_OK;
}

extern "C" int beast_comm_group_end(void) {
  BEAST_NEED_RCCL(R);
  BEAST_NCCL(R->group_end(), "ncclGroupEnd");
  return BEAST_OK;
}

extern "C" int beast_comm_allreduce(beast_comm* c, const void* send, void* recv, int64_t count, int dtype, int op,
                                    void* stream) {
  BEAST_REQUIRE(c != nullptr && count >= 0 && (count == 0 || (send && recv)), "beast_comm_allreduce: bad arguments");
  ncclDataType_t dt;
  ncclRedOp_t ro;
  size_t eb;
  BEAST_REQUIRE(dtype_of(dtype, &dt, &eb) && op_of(op, &ro), "beast_comm_allreduce: unknown dtype %d / op %d", dtype, op);
  if (count == 0) return BEAST_OK;
  if (c->vg) return v_allreduce(c, send, recv, count, dtype, op, eb, beast::as_stream(stream));
  BEAST_NEED_RCCL(R);
  BEAST_NCCL(R->all_reduce(send, recv, (size_t)count, dt, ro, c->nc, beast::as_stream(stream)), "ncclAllReduce");
  return BEAST_OK;
}

extern "C" int beast_comm_allgather(beast_comm* c, const void* send, void* recv, int64_t count, int dtype,
                                    void* stream) {
  BEAST_REQUIRE(c != nullptr && count >= 0 && (count == 0 || (send && recv)), "beast_comm_allgather: bad arguments");
  ncclDataType_t dt;
  size_t eb;
  BEAST_REQUIRE(dtype_of(dtype, &dt, &eb), "beast_comm_allgather: unknown dtype %d", dtype);
  if (count == 0) return BEAST_OK;
  if (c->vg) {
    std::vector<int64_t> counts(c->world, count), displs(c->world);
    for (int r = 0; r < c->world; ++r) displs[r] = (int64_t)r * count;
    return v_gather(c, send, recv, counts.data(), displs.data(), eb, beast::as_stream(stream));
  }
  BEAST_NEED_RCCL(R);
  BEAST_NCCL(R->all_gather(send, recv, (size_t)count, dt, c->nc, beast::as_stream(stream)), "ncclAllGather");
  return BEAST_OK;
}

// rank r's counts[r] elements land at recv + displs[r] on every rank: one broadcast per rank in
// one group (RCCL has no all-gather-v); counts / displs are HOST arrays [world], the same on
// every rank.  A rank with nothing to send is skipped by all ranks alike.
extern "C" int beast_comm_allgatherv(beast_comm* c, const void* send, void* recv, const int64_t* counts,
                                     const int64_t* displs, int dtype, void* stream) {
  BEAST_REQUIRE(c != nullptr && counts != nullptr && displs != nullptr, "beast_comm_allgatherv: null pointer");
  ncclDataType_t dt;
  size_t eb;
  BEAST_REQUIRE(dtype_of(dtype, &dt, &eb), "beast_comm_allgatherv: unknown dtype %d", dtype);
  bool any = false;
  for (int r = 0; r < c->world; ++r) {
    BEAST_REQUIRE(counts[r] >= 0 && displs[r] >= 0, "beast_comm_allgatherv: negative count / displacement");
    any = any || counts[r] > 0;
  }
  if (!any) return BEAST_OK;
  BEAST_REQUIRE(recv != nullptr && (counts[c->rank] == 0 || send != nullptr), "beast_comm_allgatherv: null buffer");
  hipStream_t s = beast::as_stream(stream);
  if (c->vg) return v_gather(c, send, recv, counts, displs, eb, s);
  BEAST_NEED_RCCL(R);
  BEAST_NCCL(R->group_start(), "ncclGroupStart");
  ncclResult_t first = ncclSuccess;
  for (int r = 0; r < c->world; ++r) {
    if (counts[r] == 0) continue;
    char* dst = static_cast<char*>(recv) + (size_t)displs[r] * eb;
    const ncclResult_t e = R->broadcast(r == c->rank ? send : dst, dst, (size_t)counts[r], dt, r, c->nc, s);
    if (first == ncclSuccess) first = e;
  }
  const ncclResult_t e = R->group_end();
  BEAST_NCCL(first, "ncclBroadcast");
  BEAST_NCCL(e, "ncclGroupEnd");
  return BEAST_OK;
}

namespace beast {

int comm_max_i32(beast_comm* c, int v, int* out, hipStream_t s) {
  *out = v;
  if (c == nullptr || c->world == 1) return BEAST_OK;
  int32_t h[4] = {v, 0, 0, 0};
  BEAST_HIP(hipMemcpyAsync(c->scratch, h, sizeof(int32_t), hipMemcpyHostToDevice, s), "status upload");
  if (int rc = beast_comm_allreduce(c, c->scratch, c->scratch, 1, BEAST_DT_I32, BEAST_OP_MAX, s)) return rc;
  BEAST_HIP(hipMemcpyAsync(h, c->scratch, sizeof(int32_t), hipMemcpyDeviceToHost, s), "status read");
  BEAST_HIP(hipStreamSynchronize(s), "stream sync");
  *out = h[0];
  return BEAST_OK;
}

int comm_agree(beast_comm* c, int rc, hipStream_t s) {
  if (c == nullptr || c->world == 1) return rc;
  // the worst failure code over the ranks (codes are negative; 0 = every rank succeeded)
  int worst = 0;
  const int crc = comm_max_i32(c, rc == BEAST_OK ? 0 : -rc, &worst, s);
  if (rc != BEAST_OK) return rc;   // this rank's own error and message
  if (crc != BEAST_OK) return crc;
  if (worst == 0) return BEAST_OK;
  set_error("beast_comm: another rank of the communicator failed (code %d); every rank returns it", -worst);
  return -worst;
}

}  // namespace beast
