// gevws_comm.cpp -- multi-GPU at the C ABI for ONE process that drives several
// GPUs (a gev server whose NumLoops event loops are placed on the node's
// devices round-robin, load_balance.go:7-14 / server.go:80-91): an RCCL
// communicator over those devices (ncclCommInitAll) and the one collective the
// decode path has -- the all-reduce(sum) of each device's decoded {frames,
// payload bytes, errors}.  Payloads never cross GPUs.
//
// RCCL is loaded on first use (dlopen of librccl.so.1): a process that already
// holds one (torch's bundled RCCL has the same SONAME) shares it, and the
// decode library keeps no link-time dependency on RCCL.  The one-process-per-GPU
// form (torch.distributed over RCCL, bench.py) needs none of this.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstring>
#include <mutex>
#include <vector>

#include "gevws.h"

namespace {

struct Rccl {
  void* h = nullptr;
  decltype(&ncclCommInitAll) comm_init_all = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  bool ok = false;
};

Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    const char* names[] = {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"};
    for (const char* n : names) {
      r.h = dlopen(n, RTLD_NOW | RTLD_NOLOAD);  // one already in the process (e.g. torch's)
      if (r.h) break;
    }
    for (const char* n : names) {
      if (r.h) break;
      r.h = dlopen(n, RTLD_NOW | RTLD_GLOBAL);
    }
    if (!r.h) {
      fprintf(stderr, "[gevws] RCCL not found (librccl.so.1): %s\n", dlerror());
      return;
    }
    r.comm_init_all = (decltype(r.comm_init_all))dlsym(r.h, "ncclCommInitAll");
    r.comm_destroy = (decltype(r.comm_destroy))dlsym(r.h, "ncclCommDestroy");
    r.all_reduce = (decltype(r.all_reduce))dlsym(r.h, "ncclAllReduce");
    r.group_start = (decltype(r.group_start))dlsym(r.h, "ncclGroupStart");
    r.group_end = (decltype(r.group_end))dlsym(r.h, "ncclGroupEnd");
    r.error_string = (decltype(r.error_string))dlsym(r.h, "ncclGetErrorString");
    r.ok = r.comm_init_all && r.comm_destroy && r.all_reduce && r.group_start && r.group_end && r.error_string;
    if (!r.ok) fprintf(stderr, "[gevws] RCCL: missing symbols\n");
  });
  return r;
}

// {frames, payload_len, errors} of a decode summary -> int64[3] on the device
__global__ void k_counts_of(const gevws_summary* __restrict__ s, int64_t* __restrict__ out) {
  if (threadIdx.x == 0) {
    out[0] = (int64_t)s->frames;
    out[1] = (int64_t)s->payload_len;
    out[2] = (int64_t)s->errors;
  }
}

}  // namespace

struct gevws_comm {
  std::vector<int> devices;
  std::vector<ncclComm_t> comms;
};

extern "C" {

gevws_comm* gevws_comm_create(const int* devices, int n) {
  if (!devices || n <= 0) return nullptr;
  Rccl& r = rccl();
  if (!r.ok) return nullptr;
  const int visible = gevws_device_count();
  for (int i = 0; i < n; ++i)
    if (devices[i] < 0 || devices[i] >= visible) {
      fprintf(stderr, "[gevws] gevws_comm_create: device %d not available (%d visible)\n", devices[i], visible);
      return nullptr;
    }
  auto* c = new gevws_comm();
  c->devices.assign(devices, devices + n);
  c->comms.resize(n);
  int prev = 0;
  (void)hipGetDevice(&prev);
  const ncclResult_t e = r.comm_init_all(c->comms.data(), n, devices);
  (void)hipSetDevice(prev);
  if (e != ncclSuccess) {
    fprintf(stderr, "[gevws] ncclCommInitAll: %s\n", r.error_string(e));
    delete c;
    return nullptr;
  }
  return c;
}

void gevws_comm_destroy(gevws_comm* c) {
  if (!c) return;
  Rccl& r = rccl();
  for (ncclComm_t m : c->comms)
    if (m && r.ok) (void)r.comm_destroy(m);
  delete c;
}

int gevws_comm_size(const gevws_comm* c) { return c ? (int)c->devices.size() : 0; }

int gevws_counts_allreduce_async(gevws_comm* c, gevws_ctx* const* ctxs, const gevws_summary* const* d_summaries,
                                 int64_t* const* d_counts) {
  if (!c || !ctxs || !d_summaries || !d_counts) return GEVWS_ERR_INVALID;
  Rccl& r = rccl();
  if (!r.ok) return GEVWS_ERR_DEVICE;
  const int n = (int)c->devices.size();
  for (int i = 0; i < n; ++i)
    if (!ctxs[i] || gevws_ctx_device(ctxs[i]) != c->devices[i] || !d_summaries[i] || !d_counts[i])
      return GEVWS_ERR_INVALID;
  int prev = 0;
  (void)hipGetDevice(&prev);
  int st = GEVWS_OK;
  for (int i = 0; i < n && st == GEVWS_OK; ++i) {
    (void)hipSetDevice(c->devices[i]);
    hipStream_t s = (hipStream_t)gevws_ctx_stream(ctxs[i]);
    // the summary is written by the context's last decode, on whatever stream
    // the caller gave it: order the read (and the reduce behind it) after that
    if (gevws_ctx_order_after_last(ctxs[i], s) != GEVWS_OK) {
      st = GEVWS_ERR_DEVICE;
      break;
    }
    k_counts_of<<<1, 64, 0, s>>>(d_summaries[i], d_counts[i]);
    if (hipGetLastError() != hipSuccess) st = GEVWS_ERR_DEVICE;
  }
  if (st == GEVWS_OK) {
    // one group: every device's all-reduce progresses together (a single
    // thread drives all the ranks)
    ncclResult_t e = r.group_start();
    for (int i = 0; i < n && e == ncclSuccess; ++i) {
      (void)hipSetDevice(c->devices[i]);
      e = r.all_reduce(d_counts[i], d_counts[i], 3, ncclInt64, ncclSum, c->comms[i],
                       (hipStream_t)gevws_ctx_stream(ctxs[i]));
    }
    const ncclResult_t g = r.group_end();
    if (e != ncclSuccess || g != ncclSuccess) {
      fprintf(stderr, "[gevws] ncclAllReduce: %s\n", r.error_string(e != ncclSuccess ? e : g));
      st = GEVWS_ERR_DEVICE;
    }
  }
  (void)hipSetDevice(prev);
  return st;
}

int gevws_counts_allreduce(gevws_comm* c, gevws_ctx* const* ctxs, const gevws_summary* const* d_summaries,
                           int64_t* const* d_counts, int64_t h_total[3]) {
  int st = gevws_counts_allreduce_async(c, ctxs, d_summaries, d_counts);
  if (st != GEVWS_OK) return st;
  int prev = 0;
  (void)hipGetDevice(&prev);
  for (size_t i = 0; i < c->devices.size(); ++i) {
    (void)hipSetDevice(c->devices[i]);
    if (hipStreamSynchronize((hipStream_t)gevws_ctx_stream(ctxs[i])) != hipSuccess) st = GEVWS_ERR_DEVICE;
  }
  if (st == GEVWS_OK && h_total) {
    (void)hipSetDevice(c->devices[0]);
    if (hipMemcpy(h_total, d_counts[0], 3 * sizeof(int64_t), hipMemcpyDeviceToHost) != hipSuccess)
      st = GEVWS_ERR_DEVICE;
  }
  (void)hipSetDevice(prev);
  return st;
}

}  // extern "C"
