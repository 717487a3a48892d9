// The one collective of a trial-sharded Monte-Carlo run: a
// SUM all-reduce of the int64 success counts [n_N][n_p][2] over RCCL (xGMI on
// one node).  The reference is single-process (Pd_plotter.py:176-235 counts
// successes in one loop); this is what lets a C caller of cvd_mc_run shard the
// global trial range over GPUs and still get the single-process counts.
//
// Two entry shapes:
//   - cvd_allreduce_counts: one process driving ndev devices
//     (ncclCommInitAll, one grouped ncclAllReduce); communicators are cached
//     per device list for the life of the process;
//   - cvd_comm_*: one process per GPU (ncclGetUniqueId on rank 0, distributed
//     by the caller, ncclCommInitRank), the shape torchrun launches.
//
// librccl is opened on first use: the copy already mapped into the process
// (PyTorch's, same soname librccl.so.1) when there is one, so one RCCL and one
// HIP runtime serve both; otherwise the system's (CVD_RCCL_LIB overrides).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/cvd.h"
#include "cvd_internal.h"

using cvd::set_error;

namespace {

struct Rccl {
  bool ok = false;
  std::string err;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  decltype(&ncclCommInitAll) init_all = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
};

Rccl& rccl() {
  static Rccl R;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = nullptr;
    if (const char* e = std::getenv("CVD_RCCL_LIB")) h = ::dlopen(e, RTLD_NOW | RTLD_LOCAL);
    if (!h) h = ::dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL | RTLD_NOLOAD);   // already mapped (torch)
    if (!h) h = ::dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = ::dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) { R.err = std::string("RCCL: cannot open librccl.so.1: ") + ::dlerror(); return; }
    bool all = true;
    auto sym = [&](auto& f, const char* name) {
      f = reinterpret_cast<std::remove_reference_t<decltype(f)>>(::dlsym(h, name));
      if (!f) all = false;
    };
    sym(R.get_unique_id, "ncclGetUniqueId");
    sym(R.init_rank, "ncclCommInitRank");
    sym(R.init_all, "ncclCommInitAll");
    sym(R.all_reduce, "ncclAllReduce");
    sym(R.group_start, "ncclGroupStart");
    sym(R.group_end, "ncclGroupEnd");
    sym(R.destroy, "ncclCommDestroy");
    sym(R.error_string, "ncclGetErrorString");
    if (!all) { R.err = "RCCL: missing symbols in librccl"; return; }
    R.ok = true;
  });
  return R;
}

int nccl_fail(const char* what, ncclResult_t r) {
  set_error(std::string("RCCL ") + what + ": " + rccl().error_string(r));
  return CVD_E_HIP;
}

struct DeviceGuard {
  int cur = 0;
  DeviceGuard() { (void)hipGetDevice(&cur); }
  ~DeviceGuard() { (void)hipSetDevice(cur); }
};

std::mutex g_mu;
std::map<std::vector<int>, std::vector<ncclComm_t>> g_comms;   // device list -> communicators

}  // namespace

struct cvd_comm {
  ncclComm_t comm = nullptr;
  int device = 0;
};

extern "C" int cvd_allreduce_counts(int64_t* const* d_counts, int64_t len, int32_t ndev, const int32_t* devices,
                                    void* const* streams) {
  if (!d_counts || !devices || ndev < 1 || len < 0) { set_error("bad allreduce arguments"); return CVD_E_INVALID; }
  for (int i = 0; i < ndev; ++i)
    if (!d_counts[i] && len > 0) { set_error("null count buffer"); return CVD_E_INVALID; }
  Rccl& R = rccl();
  if (!R.ok) { set_error(R.err); return CVD_E_UNSUPPORTED; }
  if (len == 0) return CVD_OK;
  DeviceGuard guard;
  std::lock_guard<std::mutex> lk(g_mu);
  std::vector<int> key(devices, devices + ndev);
  auto it = g_comms.find(key);
  if (it == g_comms.end()) {
    std::vector<ncclComm_t> comms((size_t)ndev, nullptr);
    ncclResult_t r = R.init_all(comms.data(), ndev, key.data());
    if (r != ncclSuccess) return nccl_fail("ncclCommInitAll", r);
    it = g_comms.emplace(key, std::move(comms)).first;
  }
  ncclResult_t r = R.group_start();
  if (r != ncclSuccess) return nccl_fail("ncclGroupStart", r);
  for (int i = 0; i < ndev; ++i) {
    if (hipSetDevice(devices[i]) != hipSuccess) {
      (void)R.group_end();
      set_error("hipSetDevice failed");
      return CVD_E_HIP;
    }
    r = R.all_reduce(d_counts[i], d_counts[i], (size_t)len, ncclInt64, ncclSum, it->second[(size_t)i],
                     streams ? (hipStream_t)streams[i] : nullptr);
    if (r != ncclSuccess) {
      (void)R.group_end();
      return nccl_fail("ncclAllReduce", r);
    }
  }
  r = R.group_end();
  if (r != ncclSuccess) return nccl_fail("ncclGroupEnd", r);
  return CVD_OK;
}

extern "C" int cvd_comm_unique_id(uint8_t* id_out) {
  if (!id_out) { set_error("null id buffer"); return CVD_E_INVALID; }
  Rccl& R = rccl();
  if (!R.ok) { set_error(R.err); return CVD_E_UNSUPPORTED; }
  ncclUniqueId id;
  ncclResult_t r = R.get_unique_id(&id);
  if (r != ncclSuccess) return nccl_fail("ncclGetUniqueId", r);
  static_assert(sizeof(id) == CVD_COMM_ID_BYTES, "ncclUniqueId size");
  std::memcpy(id_out, &id, sizeof(id));
  return CVD_OK;
}

extern "C" int cvd_comm_init(const uint8_t* id, int32_t nranks, int32_t rank, int32_t device, cvd_comm** out) {
  if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks || device < 0) {
    set_error("bad comm arguments");
    return CVD_E_INVALID;
  }
  *out = nullptr;
  Rccl& R = rccl();
  if (!R.ok) { set_error(R.err); return CVD_E_UNSUPPORTED; }
  DeviceGuard guard;
  if (hipSetDevice(device) != hipSuccess) { set_error("hipSetDevice failed"); return CVD_E_HIP; }
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  auto* c = new cvd_comm();
  c->device = device;
  ncclResult_t r = R.init_rank(&c->comm, nranks, uid, rank);
  if (r != ncclSuccess) {
    delete c;
    return nccl_fail("ncclCommInitRank", r);
  }
  *out = c;
  return CVD_OK;
}

extern "C" int cvd_comm_allreduce_counts(cvd_comm* comm, int64_t* d_counts, int64_t len, void* stream) {
  if (!comm || (!d_counts && len > 0) || len < 0) { set_error("bad allreduce arguments"); return CVD_E_INVALID; }
  if (len == 0) return CVD_OK;
  Rccl& R = rccl();
  DeviceGuard guard;
  if (hipSetDevice(comm->device) != hipSuccess) { set_error("hipSetDevice failed"); return CVD_E_HIP; }
  ncclResult_t r = R.all_reduce(d_counts, d_counts, (size_t)len, ncclInt64, ncclSum, comm->comm, (hipStream_t)stream);
  if (r != ncclSuccess) return nccl_fail("ncclAllReduce", r);
  return CVD_OK;
}

extern "C" void cvd_comm_destroy(cvd_comm* comm) {
  if (!comm) return;
  if (comm->comm && rccl().ok) (void)rccl().destroy(comm->comm);
  delete comm;
}
