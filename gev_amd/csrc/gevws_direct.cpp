// gevws_direct.cpp -- direct dispatch of a context's live passes (opt-in,
// gevws_ctx_set_direct).  A live pass is one kernel (the one-launch decode)
// whose completion the host learns from the mapped completion word, so the
// HIP runtime's launch path -- argument marshalling, its queue bookkeeping,
// ~3.5 us of host time a pass on the 100-connection loop -- buys it nothing.
// Here the context owns an AQL queue of its own (hsa_queue_create) and writes
// each pass's dispatch packet into it: the kernel's arguments into a slot of
// a kernarg ring in host memory the GPU reads, the packet body, then its
// header with a release store, then the doorbell.
//
// The kernel objects are the ones the HIP runtime loaded for this library
// (k_decode_small_direct, both shapes), found through the ROCr loader
// extension's executable list after a hipFuncGetAttributes has made the
// runtime load them.  Ordering: packets on the queue run one after another
// (barrier bit); against the context's stream, a call that enqueues there
// after direct passes first waits for their completion words
// (direct_drain), and a direct pass after stream work waits for that work's
// event on the host.
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <hsa/hsa_ven_amd_loader.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>

#include "gevws_internal.hpp"

struct DirectQueue {
  hsa_agent_t agent{};
  hsa_queue_t* q = nullptr;
  struct Kernel {
    uint64_t object = 0;
    uint32_t kernarg_bytes = 0, group_bytes = 0, private_bytes = 0;
  } k[2];  // [0] narrow shape, [1] wide
  static constexpr uint32_t kSlots = 64;  // kernarg ring (<= the queue's packets)
  static constexpr uint32_t kSlotBytes = 512;
  uint8_t* kernargs = nullptr;  // kSlots x kSlotBytes, fine-grained host memory
  uint32_t slot_seq[kSlots] = {};  // the completion number of the dispatch that last used a slot
  bool slot_used[kSlots] = {};     // ... if that dispatch may not have signalled yet
  const volatile uint32_t* flag_host = nullptr;  // the completion word the dispatches signal (host address)
  uint32_t* flag_dev = nullptr;
  uint32_t last_seq = 0;  // the last dispatch's completion number
  uint64_t dispatched = 0;
  int failed = 0;  // set by the queue's error callback (a faulting packet): no further dispatch or wait
};

namespace gevws_impl {

const void* direct_kernel_stub(int wide);  // gevws_walk.hip

namespace {

bool hsa_ready() {
  static const bool ok = hsa_init() == HSA_STATUS_SUCCESS;
  return ok;
}

struct AgentMatch {
  uint32_t domain, bdf;  // the HIP device's PCI domain and bus / device (function dropped)
  hsa_agent_t found{};
  bool hit = false;
};

hsa_status_t find_agent(hsa_agent_t a, void* data) {
  auto* m = static_cast<AgentMatch*>(data);
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS || t != HSA_DEVICE_TYPE_GPU)
    return HSA_STATUS_SUCCESS;
  uint32_t bdfid = 0, domain = 0;
  if (hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdfid) != HSA_STATUS_SUCCESS ||
      hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &domain) != HSA_STATUS_SUCCESS)
    return HSA_STATUS_SUCCESS;
  if (domain == m->domain && (bdfid >> 3) == m->bdf) {
    m->found = a;
    m->hit = true;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

struct SymbolSearch {
  hsa_agent_t agent;
  DirectQueue* dq;
  int found = 0;
};

hsa_status_t on_symbol(hsa_executable_t, hsa_agent_t, hsa_executable_symbol_t sym, void* data) {
  auto* s = static_cast<SymbolSearch*>(data);
  hsa_symbol_kind_t kind;
  if (hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_TYPE, &kind) != HSA_STATUS_SUCCESS ||
      kind != HSA_SYMBOL_KIND_KERNEL)
    return HSA_STATUS_SUCCESS;
  uint32_t len = 0;
  if (hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_NAME_LENGTH, &len) != HSA_STATUS_SUCCESS)
    return HSA_STATUS_SUCCESS;
  std::string name(len, '\0');
  if (hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_NAME, &name[0]) != HSA_STATUS_SUCCESS)
    return HSA_STATUS_SUCCESS;
  if (name.find("k_decode_small_direct") == std::string::npos) return HSA_STATUS_SUCCESS;
  // SmallShape<256, 65536> / SmallShape<1024, 131072>
  const int wide = name.find("ILj1024E") != std::string::npos ? 1 : name.find("ILj256E") != std::string::npos ? 0 : -1;
  if (wide < 0 || s->dq->k[wide].object) return HSA_STATUS_SUCCESS;
  DirectQueue::Kernel& k = s->dq->k[wide];
  if (hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &k.object) != HSA_STATUS_SUCCESS ||
      hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &k.kernarg_bytes) !=
          HSA_STATUS_SUCCESS ||
      hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &k.group_bytes) !=
          HSA_STATUS_SUCCESS ||
      hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &k.private_bytes) !=
          HSA_STATUS_SUCCESS) {
    k.object = 0;
    return HSA_STATUS_SUCCESS;
  }
  ++s->found;
  return HSA_STATUS_SUCCESS;
}

hsa_status_t on_executable(hsa_executable_t exe, void* data) {
  auto* s = static_cast<SymbolSearch*>(data);
  (void)hsa_executable_iterate_agent_symbols(exe, s->agent, on_symbol, data);
  return s->found == 2 ? HSA_STATUS_INFO_BREAK : HSA_STATUS_SUCCESS;
}

hsa_status_t find_kernarg_pool(hsa_amd_memory_pool_t pool, void* data) {
  hsa_amd_segment_t seg;
  uint32_t flags = 0;
  if (hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg) != HSA_STATUS_SUCCESS ||
      seg != HSA_AMD_SEGMENT_GLOBAL ||
      hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags) != HSA_STATUS_SUCCESS ||
      !(flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT))
    return HSA_STATUS_SUCCESS;
  *static_cast<hsa_amd_memory_pool_t*>(data) = pool;
  return HSA_STATUS_INFO_BREAK;
}

hsa_status_t find_cpu_kernarg_pool(hsa_agent_t a, void* data) {
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS || t != HSA_DEVICE_TYPE_CPU)
    return HSA_STATUS_SUCCESS;
  auto* pool = static_cast<hsa_amd_memory_pool_t*>(data);
  (void)hsa_amd_agent_iterate_memory_pools(a, find_kernarg_pool, pool);
  return pool->handle ? HSA_STATUS_INFO_BREAK : HSA_STATUS_SUCCESS;
}

// The runtime's report of an asynchronous queue error (a packet that
// faulted): recorded, so waits and dispatches on this queue fail at once.
void on_queue_error(hsa_status_t status, hsa_queue_t*, void* data) {
  __atomic_store_n(&static_cast<DirectQueue*>(data)->failed, 1, __ATOMIC_RELEASE);
  const char* msg = nullptr;
  (void)hsa_status_string(status, &msg);
  fprintf(stderr, "[gevws] direct dispatch queue error: %s\n", msg ? msg : "?");
}

void close_queue(DirectQueue* dq) {
  if (!dq) return;
  if (dq->q) (void)hsa_queue_destroy(dq->q);
  if (dq->kernargs) (void)hsa_amd_memory_pool_free(dq->kernargs);
  delete dq;
}

// The context's queue, kernels and kernarg ring, or nullptr.
DirectQueue* open_queue(gevws_ctx* ctx) {
  if (!hsa_ready()) return nullptr;
  int domain = 0, bus = 0, dev = 0;
  if (hipDeviceGetAttribute(&domain, hipDeviceAttributePciDomainId, ctx->device) != hipSuccess ||
      hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, ctx->device) != hipSuccess ||
      hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, ctx->device) != hipSuccess)
    return nullptr;
  AgentMatch m{(uint32_t)domain, ((uint32_t)bus << 5) | (uint32_t)dev};
  if (hsa_iterate_agents(find_agent, &m) != HSA_STATUS_INFO_BREAK || !m.hit) return nullptr;
  auto* dq = new DirectQueue;
  dq->agent = m.found;
  // the runtime loads a module's code objects on first use: make it load these
  for (int w = 0; w < 2; ++w) {
    hipFuncAttributes fa;
    if (hipFuncGetAttributes(&fa, direct_kernel_stub(w)) != hipSuccess) {
      close_queue(dq);
      return nullptr;
    }
  }
  hsa_ven_amd_loader_1_03_pfn_t ld;
  memset(&ld, 0, sizeof(ld));
  SymbolSearch s{dq->agent, dq};
  if (hsa_system_get_major_extension_table(HSA_EXTENSION_AMD_LOADER, 1, sizeof(ld), &ld) != HSA_STATUS_SUCCESS ||
      !ld.hsa_ven_amd_loader_iterate_executables) {
    close_queue(dq);
    return nullptr;
  }
  (void)ld.hsa_ven_amd_loader_iterate_executables(on_executable, &s);
  if (s.found != 2) {
    close_queue(dq);
    return nullptr;
  }
  for (const auto& k : dq->k)
    if (k.kernarg_bytes > DirectQueue::kSlotBytes || k.kernarg_bytes < sizeof(DirectDecodeArgs) || k.private_bytes) {
      close_queue(dq);  // (a layout this file does not expect: launch through HIP instead)
      return nullptr;
    }
  uint32_t qmin = 0;
  (void)hsa_agent_get_info(dq->agent, HSA_AGENT_INFO_QUEUE_MIN_SIZE, &qmin);
  uint32_t qsize = 64;
  while (qsize < qmin) qsize *= 2;
  if (hsa_queue_create(dq->agent, qsize, HSA_QUEUE_TYPE_SINGLE, on_queue_error, dq, UINT32_MAX, UINT32_MAX, &dq->q) !=
      HSA_STATUS_SUCCESS) {
    dq->q = nullptr;
    close_queue(dq);
    return nullptr;
  }
  hsa_amd_memory_pool_t pool{};
  if (hsa_iterate_agents(find_cpu_kernarg_pool, &pool) != HSA_STATUS_INFO_BREAK || !pool.handle ||
      hsa_amd_memory_pool_allocate(pool, DirectQueue::kSlots * DirectQueue::kSlotBytes, 0,
                                   reinterpret_cast<void**>(&dq->kernargs)) != HSA_STATUS_SUCCESS ||
      hsa_amd_agents_allow_access(1, &dq->agent, nullptr, dq->kernargs) != HSA_STATUS_SUCCESS) {
    close_queue(dq);
    return nullptr;
  }
  memset(dq->kernargs, 0, DirectQueue::kSlots * DirectQueue::kSlotBytes);
  return dq;
}

// Spins until the completion word carries seq or later (false past 10 s, or
// at once once the queue has reported an error).
bool wait_word(const DirectQueue* dq, const volatile uint32_t* w, uint32_t seq) {
  const auto t0 = std::chrono::steady_clock::now();
  for (uint64_t i = 1;; ++i) {
    if ((int32_t)(__atomic_load_n(w, __ATOMIC_ACQUIRE) - seq) >= 0) return true;
    if ((i & 1023) == 0 && (__atomic_load_n(&dq->failed, __ATOMIC_ACQUIRE) ||
                            std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10)))
      return false;
    __builtin_ia32_pause();
  }
}

}  // namespace

int direct_drain(gevws_ctx* ctx) {
  DirectQueue* dq = ctx->direct;
  if (!dq || !dq->dispatched || !dq->flag_host) return GEVWS_OK;
  return wait_word(dq, dq->flag_host, dq->last_seq) ? GEVWS_OK : GEVWS_ERR_DEVICE;
}

// One live pass written into the context's queue (the kernel: shape `wide`,
// nwg workgroups), or false: launch it through HIP instead.  The caller has
// filled a.done / a.seq with the completion word and this pass's number.
bool direct_dispatch(gevws_ctx* ctx, int wide, const DirectDecodeArgs& a) {
  if (!ctx->direct && !(ctx->direct = open_queue(ctx))) {
    ctx->direct_enabled = false;  // (this process cannot: HIP launches from here on)
    return false;
  }
  DirectQueue* dq = ctx->direct;
  if (__atomic_load_n(&dq->failed, __ATOMIC_ACQUIRE)) return false;
  const DirectQueue::Kernel& k = dq->k[wide];
  // the completion word's host address (the pass waits on it; so do drains)
  if (dq->flag_dev != a.done) {
    if (dq->dispatched && direct_drain(ctx) != GEVWS_OK) return false;
    hipPointerAttribute_t pa;
    if (hipPointerGetAttributes(&pa, a.done) != hipSuccess || !pa.hostPointer) return false;
    dq->flag_dev = a.done;
    dq->flag_host = static_cast<const volatile uint32_t*>(pa.hostPointer);
    dq->dispatched = 0;
    memset(dq->slot_used, 0, sizeof(dq->slot_used));  // (drained above)
  }
  // work the context enqueued on its stream before this pass runs first
  if (ctx->has_last && !ctx->last_direct &&
      (last_event(ctx) != GEVWS_OK || hipEventSynchronize(ctx->last_done) != hipSuccess))
    return false;
  // The packet slot and the kernarg slot are claimed only once both are free
  // (a single-producer queue: nothing else moves the write index), so a
  // failed wait leaves no half-claimed slot for the packet processor to stall on.
  hsa_queue_t* q = dq->q;
  const uint64_t idx = hsa_queue_load_write_index_relaxed(q);
  const auto t0 = std::chrono::steady_clock::now();
  while (idx - hsa_queue_load_read_index_scacquire(q) >= q->size) {
    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10)) return false;
    __builtin_ia32_pause();
  }
  // the kernarg slot: free once the dispatch that used it last has signalled
  const uint32_t slot = (uint32_t)(idx % DirectQueue::kSlots);
  if (dq->slot_used[slot] && !wait_word(dq, dq->flag_host, dq->slot_seq[slot])) return false;
  uint8_t* karg = dq->kernargs + (size_t)slot * DirectQueue::kSlotBytes;
  memcpy(karg, &a, sizeof(a));
  dq->slot_seq[slot] = a.seq;
  dq->slot_used[slot] = true;
  auto* pkt = static_cast<hsa_kernel_dispatch_packet_t*>(q->base_address) + (idx & (q->size - 1));
  const uint32_t nt = wide ? 1024u : 256u;
  pkt->workgroup_size_x = (uint16_t)nt;
  pkt->workgroup_size_y = 1;
  pkt->workgroup_size_z = 1;
  pkt->reserved0 = 0;
  pkt->grid_size_x = a.nwg * nt;
  pkt->grid_size_y = 1;
  pkt->grid_size_z = 1;
  pkt->private_segment_size = k.private_bytes;
  pkt->group_segment_size = k.group_bytes;
  pkt->kernel_object = k.object;
  pkt->kernarg_address = karg;
  pkt->reserved2 = 0;
  pkt->completion_signal = hsa_signal_t{0};
  // system-scope fences: the pass's input may have just been written by the
  // host or a copy engine (agent scope measured within run noise, r06r)
  const uint16_t header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                          (1 << HSA_PACKET_HEADER_BARRIER) |
                          (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                          (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
  const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
  hsa_queue_store_write_index_screlease(q, idx + 1);
  __atomic_store_n(reinterpret_cast<uint32_t*>(pkt), (uint32_t)header | ((uint32_t)setup << 16), __ATOMIC_RELEASE);
  hsa_signal_store_screlease(q->doorbell_signal, (hsa_signal_value_t)idx);
  dq->last_seq = a.seq;
  ++dq->dispatched;
  ++ctx->direct_dispatches;
  ctx->last_direct = true;
  return true;
}

void direct_forget_flag(gevws_ctx* ctx) {
  DirectQueue* dq = ctx->direct;
  if (!dq) return;
  if (ctx->last_direct) {
    (void)direct_drain(ctx);
    ctx->last_direct = false;
  }
  dq->flag_host = nullptr;  // (the word may be freed next)
  dq->flag_dev = nullptr;
  dq->dispatched = 0;
  memset(dq->slot_used, 0, sizeof(dq->slot_used));  // every slot free: its dispatch has signalled
}

void direct_close(gevws_ctx* ctx) {
  if (!ctx->direct) return;
  (void)direct_drain(ctx);
  close_queue(ctx->direct);
  ctx->direct = nullptr;
}

}  // namespace gevws_impl
