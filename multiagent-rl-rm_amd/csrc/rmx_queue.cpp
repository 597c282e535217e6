// rmx_queue.cpp — the engine's own AQL queue: rmx_step_seq's K dependent step launches written as K kernel-dispatch
// packets into an HSA queue of the engine's (one per device), one doorbell, one completion signal waited on by
// spinning.  A HIP graph of the same K launches pays ~12 us more per window on the host (hipGraphLaunch, the stream
// synchronisation): profiles/r04_ab_log.md "aql".  The kernels are the library's own step_fast_kernel
// instantiations: the gfx950 code object of rmx_fast.hip, embedded in librmx.so at link time (Makefile), loaded
// once per device through the HSA loader.  Kernel arguments live in device memory (host-memory kernargs made a
// 20-step window 10x slower: every wave reads them across PCIe), rewritten only where they changed since the
// previous window.
//
// Robustness (round 5):
// - every kernel the queue dispatches is checked against the code object's own metadata (the NT_AMDGPU_METADATA
//   note, MessagePack): its explicit arguments must be StepArgs' layout and its hidden arguments only those the queue
//   writes, at the offsets it writes them.  A kernel that fails (e.g. a debugging printf adds hidden_printf_buffer,
//   which would read 0 here) is refused and its windows run on the caller's stream;
// - the queue is found by the device's PCI location (domain, bus, device; the partition bits ignored) and, if several
//   agents share it, by UUID; no match leaves the queue unavailable (stream path), not an error;
// - every wait has a deadline; a window that faults or times out inactivates the queue (no packet of it keeps running
//   on the caller's columns) and retires it: that call fails, later windows run on the stream.
//
// Dispatch timing (round 6, rmx_queue_timing / rmx_queue_times): the queue has HSA dispatch profiling enabled from
// its creation; with timing on (a stride m), packets 0, m, 2m, ... and the window's last one carry a completion signal
// of their own, so the command processor stamps those dispatches' start (packet processing) and end (completion) —
// the timestamps a kernel trace reads, with the window's packets still back to back behind one doorbell (a tracer's
// queue interception hands them to the device one at a time: profiles/r06_ab_log.md "trace").  A stamped packet costs
// the command processor ~1.2 us more than an unstamped one (its completion is signalled), so a sparse stride leaves
// the cadence as it is and the span between stamps measures it (profiles/r06_ab_log.md "cp stamps").
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "rmx_comd.h"
#include "rmx_internal.h"

// the embedded code object (build/rmx_fast_co.S)
extern "C" const char rmx_fast_co_begin[];
extern "C" const char rmx_fast_co_end[];

namespace rmx {
namespace {

constexpr uint32_t kQueueSize = 1024;  // packets; a window longer than that is written lap by lap
constexpr size_t kSlotAlign = 64;
constexpr double kWaitSeconds = 60.0;  // a window (or ring room for it) not there after this is an error
constexpr int kMaxTimed = 4096;        // dispatch timing: at most this many stamped packets per window
constexpr int kBell = 16;              // a window's doorbell rings after its first packet and every kBell packets

// ---- code-object metadata: which step kernels the queue may dispatch (rmx_comd.cpp) ---------------------------

// Code object v5 hidden arguments, at the first 8-aligned offset after the explicit ones (what the HIP runtime
// writes for a 1-D launch): block counts, group sizes, remainders, global offsets (0), grid dimensions, dynamic LDS
constexpr size_t kHiddenBase = (sizeof(StepArgs) + 7) & ~size_t(7);
constexpr CoLayout kLayout = {offsetof(StepArgs, p), sizeof(FastParams), kHiddenBase};

const CoCheck& embedded_check() {
  static const CoCheck c = check_code_object(reinterpret_cast<const unsigned char*>(rmx_fast_co_begin),
                                             (size_t)(rmx_fast_co_end - rmx_fast_co_begin), kLayout);
  return c;
}

// ---- the queue ----------------------------------------------------------------------------------------------

struct Kernel {
  uint64_t object;
  uint32_t kargs, group, priv;
};

struct DeviceQueue {
  std::mutex mu;
  int state = kQueueUnused;
  std::string err;  // why the queue is unavailable or retired
  std::string inject;  // RMX_QUEUE_INJECT at init (tests): "init" fails the init, "window" fails the first window
  hsa_agent_t agent{};
  hsa_code_object_reader_t reader{};
  hsa_executable_t exec{};
  hsa_queue_t* q = nullptr;
  hsa_signal_t done{};
  uint64_t tick_hz = 0;
  std::unordered_map<std::string, Kernel> kernels;
  char* kargs_dev = nullptr;  // device-memory kernarg slots
  size_t kargs_cap = 0;
  std::vector<unsigned char> kargs_img;  // what kargs_dev holds, in its first kargs_valid bytes
  size_t kargs_valid = 0;
  std::vector<unsigned char> scratch;
  std::atomic<int> fault{0};  // set by the runtime's queue-error callback (a faulting kernel, a bad packet)
  // the previous window's packets (bodies without the header word) under its key
  uint64_t last_key = 0;
  std::vector<hsa_kernel_dispatch_packet_t> built;
  int64_t windows = 0, uploads = 0, packets = 0, stream_windows = 0;
  // dispatch timing: the stride (0 off), one signal per stamped packet, the last timed window's stamps
  int timing = 0;
  bool profiled = false;
  bool early = true;  // ring the doorbell while the window's packets are written (RMX_QUEUE_EARLY=0: at the end)
  std::vector<hsa_signal_t> tsig;
  std::vector<uint64_t> times;  // [n][packet, start, end] (ns) of the last timed window
};

constexpr int kMaxDevices = 64;
DeviceQueue g_dev[kMaxDevices];

std::string hsa_msg(const char* what, hsa_status_t s) {
  const char* m = nullptr;
  hsa_status_string(s, &m);
  return std::string(what) + ": " + (m ? m : "hsa error") + " (" + std::to_string((int)s) + ")";
}

#define HSA_OR_FAIL(expr, what)           \
  do {                                    \
    hsa_status_t s_ = (expr);             \
    if (s_ != HSA_STATUS_SUCCESS) {       \
      d.err = hsa_msg(what, s_);          \
      return false;                       \
    }                                     \
  } while (0)

struct AgentMatch {
  uint32_t bus_dev, domain;  // (bus << 8) | (device << 3), as in the low 16 bits of HSA's BDF id
  char uuid[16];
  bool have_uuid;
  std::vector<hsa_agent_t> at_location;
  std::vector<bool> uuid_match;
};

hsa_status_t match_agent(hsa_agent_t a, void* user) {
  auto* m = static_cast<AgentMatch*>(user);
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS || t != HSA_DEVICE_TYPE_GPU)
    return HSA_STATUS_SUCCESS;
  uint32_t bdf = 0, domain = 0;
  if (hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf) != HSA_STATUS_SUCCESS ||
      hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &domain) != HSA_STATUS_SUCCESS)
    return HSA_STATUS_SUCCESS;
  // bus and device only: the function bits, and what a partitioned GPU's topology puts above bit 16, differ
  if ((bdf & 0xFFF8u) != m->bus_dev || domain != m->domain) return HSA_STATUS_SUCCESS;
  char u[24] = {0};
  bool same = false;
  if (m->have_uuid && hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_UUID, u) == HSA_STATUS_SUCCESS &&
      std::strncmp(u, "GPU-", 4) == 0 && std::strlen(u) == 20)
    same = std::memcmp(u + 4, m->uuid, 16) == 0;  // HIP's UUID bytes are the 16 hex digits of the HSA string
  m->at_location.push_back(a);
  m->uuid_match.push_back(same);
  return HSA_STATUS_SUCCESS;
}

void on_queue_error(hsa_status_t, hsa_queue_t*, void* data) { static_cast<DeviceQueue*>(data)->fault.store(1); }

// the HSA agent of HIP device `device`, the embedded code object loaded for it, a queue; false leaves d.err set
bool init(DeviceQueue& d, int device) {
  if (const char* v = std::getenv("RMX_QUEUE_INJECT")) d.inject = v;
  if (d.inject == "init") {
    d.err = "rmx queue: init failure injected (RMX_QUEUE_INJECT=init)";
    return false;
  }
  const CoCheck& co = embedded_check();
  if (!co.err.empty()) {
    d.err = "rmx queue: the embedded step code object: " + co.err;
    return false;
  }
  int bus = 0, dev = 0, dom = 0;
  if (hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, device) != hipSuccess ||
      hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, device) != hipSuccess ||
      hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, device) != hipSuccess) {
    d.err = "rmx queue: cannot read the device's PCI location";
    return false;
  }
  AgentMatch m{((uint32_t)bus << 8) | ((uint32_t)dev << 3), (uint32_t)dom, {0}, false, {}, {}};
  hipDevice_t hd;
  hipUUID hu;
  m.have_uuid = hipDeviceGet(&hd, device) == hipSuccess && hipDeviceGetUuid(&hu, hd) == hipSuccess;
  if (m.have_uuid) std::memcpy(m.uuid, hu.bytes, 16);
  HSA_OR_FAIL(hsa_init(), "hsa_init");
  HSA_OR_FAIL(hsa_iterate_agents(match_agent, &m), "hsa_iterate_agents");
  // one agent at the location is the device; several (a partitioned GPU): the one whose UUID is the device's
  size_t pick = m.at_location.size();
  if (m.at_location.size() == 1) pick = 0;
  for (size_t i = 0; i < m.at_location.size() && m.at_location.size() > 1; ++i)
    if (m.uuid_match[i]) pick = pick == m.at_location.size() ? i : m.at_location.size() + 1;  // two matches: none
  if (pick >= m.at_location.size()) {
    d.err = m.at_location.empty() ? "rmx queue: no HSA agent at the device's PCI location"
                                  : "rmx queue: several HSA agents at the device's PCI location, none by UUID";
    return false;
  }
  d.agent = m.at_location[pick];
  HSA_OR_FAIL(hsa_code_object_reader_create_from_memory(rmx_fast_co_begin, (size_t)(rmx_fast_co_end - rmx_fast_co_begin),
                                                        &d.reader),
              "code object reader");
  HSA_OR_FAIL(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &d.exec),
              "executable");
  HSA_OR_FAIL(hsa_executable_load_agent_code_object(d.exec, d.agent, d.reader, nullptr, nullptr), "code object load");
  HSA_OR_FAIL(hsa_executable_freeze(d.exec, nullptr), "executable freeze");
  HSA_OR_FAIL(hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP_FREQUENCY, &d.tick_hz), "timestamp frequency");
  HSA_OR_FAIL(hsa_queue_create(d.agent, kQueueSize, HSA_QUEUE_TYPE_SINGLE, on_queue_error, &d, UINT32_MAX,
                               UINT32_MAX, &d.q),
              "queue create");
  // (without its completion interrupt — a GPU-only signal, the host spin-polls either — windows ran the same:
  // profiles/r06_ab_log.md "cp stamps")
  HSA_OR_FAIL(hsa_signal_create(1, 0, nullptr, &d.done), "signal create");
  // dispatch profiling from the start: the command processor stamps a dispatch only if the queue had it enabled
  // before its first packet (enabled later, on a queue that had run windows, the stamps stayed 0 or stale: r06k);
  // only packets with a completion signal are stamped, and untimed windows give one to the last packet only
  // (RMX_QUEUE_PROFILE=0 at the first window: off, and rmx_queue_times reports no stamps — the A/B of its cost)
  const char* ev = std::getenv("RMX_QUEUE_EARLY");
  d.early = !(ev && std::strcmp(ev, "0") == 0);
  const char* pv = std::getenv("RMX_QUEUE_PROFILE");
  d.profiled = !(pv && std::strcmp(pv, "0") == 0);
  // optional: a queue that cannot be profiled still runs every window, it just has no stamps
  if (d.profiled) d.profiled = hsa_amd_profiling_set_profiler_enabled(d.q, 1) == HSA_STATUS_SUCCESS;
  return true;
}

const Kernel* kernel(DeviceQueue& d, const char* symbol) {
  auto it = d.kernels.find(symbol);
  if (it != d.kernels.end()) return &it->second;
  hsa_executable_symbol_t sym;
  if (hsa_executable_get_symbol_by_name(d.exec, symbol, &d.agent, &sym) != HSA_STATUS_SUCCESS) return nullptr;
  Kernel k{};
  if (hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &k.object) != HSA_STATUS_SUCCESS ||
      hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &k.kargs) !=
          HSA_STATUS_SUCCESS ||
      hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &k.group) !=
          HSA_STATUS_SUCCESS ||
      hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &k.priv) !=
          HSA_STATUS_SUCCESS)
    return nullptr;
  return &d.kernels.emplace(symbol, k).first->second;
}

void write_kernargs(unsigned char* slot, const StepLaunch& L) {
  std::memcpy(slot, &L.args, sizeof(StepArgs));
  unsigned char* h = slot + kHiddenBase;
  const uint32_t counts[3] = {L.grid, 1, 1};
  const uint16_t sizes[3] = {(uint16_t)L.block, 1, 1};
  const uint16_t grid_dims = 1;
  std::memcpy(h + 0, counts, sizeof(counts));
  std::memcpy(h + 12, sizes, sizeof(sizes));  // remainders (18..23) stay 0: the grid is whole workgroups
  std::memcpy(h + 64, &grid_dims, sizeof(grid_dims));
  std::memcpy(h + 120, &L.lds, sizeof(uint32_t));
}

// The window's packets into d.built and its kernel arguments into device memory (only the span that changed).
// 0 built; kQueueStream: a kernel the metadata check refused (nothing changed); -1 an error
int build_window(DeviceQueue& d, const StepLaunch* L, int K, std::string* err) {
  // resolve the kernels; one kernarg slot size for the window
  std::vector<const Kernel*> ks((size_t)K);
  size_t slot = 0;
  const CoCheck& co = embedded_check();
  for (int i = 0; i < K; ++i) {
    auto r = co.refused.find(L[i].symbol);
    if (r != co.refused.end()) {
      *err = std::string("rmx queue: ") + L[i].symbol + " refused: " + r->second;
      return kQueueStream;
    }
    ks[i] = kernel(d, L[i].symbol);
    if (!ks[i]) {
      *err = std::string("rmx queue: the code object has no ") + L[i].symbol;
      return -1;
    }
    if (ks[i]->kargs < kHiddenBase + kHiddenUsed) {
      *err = std::string("rmx queue: unexpected kernarg segment of ") + L[i].symbol;
      return -1;
    }
    if (L[i].block == 0 || L[i].block > 1024 || L[i].grid == 0 || (uint64_t)L[i].grid * L[i].block > 0xFFFFFFFFull) {
      *err = "rmx queue: bad launch geometry";
      return -1;
    }
    slot = std::max(slot, ((size_t)ks[i]->kargs + kSlotAlign - 1) & ~(kSlotAlign - 1));
  }
  const size_t bytes = slot * (size_t)K;
  d.scratch.assign(bytes, 0);
  for (int i = 0; i < K; ++i) write_kernargs(d.scratch.data() + slot * i, L[i]);
  if (bytes > d.kargs_cap) {
    if (d.kargs_dev) (void)hipFree(d.kargs_dev);
    d.kargs_dev = nullptr;
    d.kargs_valid = 0;
    if (hipMalloc(&d.kargs_dev, bytes) != hipSuccess) {
      d.kargs_cap = 0;
      *err = "rmx queue: kernarg allocation failed";
      return -1;
    }
    d.kargs_cap = bytes;
  }
  // upload the span that differs from what the device holds (another window on the same buffers: nothing)
  const size_t same = std::min(bytes, d.kargs_valid);
  size_t lo = 0, hi = bytes;
  while (lo < same && d.scratch[lo] == d.kargs_img[lo]) ++lo;
  if (bytes <= d.kargs_valid)
    while (hi > lo && d.scratch[hi - 1] == d.kargs_img[hi - 1]) --hi;
  if (lo < hi) {
    d.kargs_valid = std::min(d.kargs_valid, lo);  // a failed copy leaves the rest unknown
    if (hipMemcpy(d.kargs_dev + lo, d.scratch.data() + lo, hi - lo, hipMemcpyHostToDevice) != hipSuccess) {
      *err = "rmx queue: kernarg upload failed";
      return -1;
    }
    if (d.kargs_img.size() < hi) d.kargs_img.resize(hi);
    std::memcpy(d.kargs_img.data() + lo, d.scratch.data() + lo, hi - lo);
    d.kargs_valid = std::max(d.kargs_valid, hi);
    ++d.uploads;
  }
  d.built.assign((size_t)K, hsa_kernel_dispatch_packet_t{});
  for (int i = 0; i < K; ++i) {
    hsa_kernel_dispatch_packet_t& pk = d.built[(size_t)i];
    pk.workgroup_size_x = (uint16_t)L[i].block;
    pk.workgroup_size_y = 1;
    pk.workgroup_size_z = 1;
    pk.grid_size_x = L[i].grid * L[i].block;
    pk.grid_size_y = 1;
    pk.grid_size_z = 1;
    pk.private_segment_size = ks[i]->priv;
    pk.group_segment_size = ks[i]->group + L[i].lds;
    pk.kernel_object = ks[i]->object;
    pk.kernarg_address = d.kargs_dev + slot * i;
  }
  return 0;
}

// A window failed (a fault, or no completion / ring room by the deadline): stop the packet processor so that no
// packet of it keeps reading or writing the caller's columns after the call returns, and retire the queue.
int retire(DeviceQueue& d, const char* why, std::string* err) {
  if (d.q) (void)hsa_queue_inactivate(d.q);
  d.state = kQueueRetired;
  d.err = why;
  d.last_key = 0;
  *err = d.err;
  return -1;
}

using Clock = std::chrono::steady_clock;

}  // namespace

int queue_run(int device, const StepLaunch* L, int K, uint64_t key, std::string* err) {
  if (device < 0 || device >= kMaxDevices || K <= 0) {
    *err = "rmx queue: bad device or window length";
    return -1;
  }
  DeviceQueue& d = g_dev[device];
  std::lock_guard<std::mutex> lock(d.mu);
  if (d.state == kQueueUnused) {
    d.state = init(d, device) ? kQueueReady : kQueueUnavailable;
    if (d.state == kQueueUnavailable && d.err.empty()) d.err = "rmx queue: init failed";
  }
  if (d.state != kQueueReady) {  // unavailable or retired: the caller's stream serves the window
    *err = d.err;
    ++d.stream_windows;
    return kQueueStream;
  }
  if (!key || key != d.last_key || d.built.size() != (size_t)K) {
    d.last_key = 0;
    const int b = build_window(d, L, K, err);
    if (b == kQueueStream) ++d.stream_windows;
    if (b) return b;
    d.last_key = key;
  }
  if (d.inject == "window") {  // tests: the first window fails as a timed-out one would, without submitting it
    d.inject.clear();
    ++d.windows;
    return retire(d, "rmx queue: a window did not complete (injected, RMX_QUEUE_INJECT=window)", err);
  }
  // K packets, each behind the previous one (barrier bit), every fence at agent scope, as a HIP stream's kernel
  // dispatches carry them: the acquire invalidates the CUs' caches before a step reads, the release writes the L2s'
  // dirty lines back to the memory side after it (where the other XCDs, copy engines and the host's copies read) —
  // what the window needs for device-memory inputs written by earlier kernels or copies and outputs read after it.
  // System scope (host-coherent memory) cost ~4 us more per window (profiles/r04_ab_log.md aql).
  hsa_queue_t* q = d.q;
  const uint64_t size = q->size;
  // dispatch timing: packets 0, m, 2m, ... (m = d.timing) get completion signals of their own, the last one keeps
  // d.done, which the command processor stamps as well; stamp j of the window is packet stamped_packet(j)
  const int m = d.timing;
  const int n_stride = m > 0 && d.profiled && K >= 2 ? (K - 2) / m + 1 : 0;  // stamped packets before the last one
  const int n_timed = m > 0 && d.profiled ? std::min(n_stride + 1, kMaxTimed) : 0;
  auto stamped_packet = [&](int j) { return j == n_timed - 1 ? K - 1 : j * m; };
  std::vector<int> sig_of((size_t)(n_timed ? K : 0), -1);
  for (int j = 0; j + 1 < n_timed; ++j) sig_of[(size_t)stamped_packet(j)] = j;
  while ((int)d.tsig.size() < n_timed) {
    hsa_signal_t sg;  // nobody waits on it: no completion interrupt (an interrupt signal made every packet ~5 us: r06k)
    if (hsa_amd_signal_create(1, 0, nullptr, HSA_AMD_SIGNAL_AMD_GPU_ONLY, &sg) != HSA_STATUS_SUCCESS) {
      *err = "rmx queue: timing signal create failed";
      return -1;
    }
    d.tsig.push_back(sg);
  }
  for (int j = 0; j + 1 < n_timed; ++j) hsa_signal_store_relaxed(d.tsig[(size_t)j], 1);
  d.times.clear();
  const Clock::time_point deadline =
      Clock::now() + std::chrono::duration_cast<Clock::duration>(std::chrono::duration<double>(kWaitSeconds));
  hsa_signal_store_relaxed(d.done, 1);
  auto* ring = static_cast<hsa_kernel_dispatch_packet_t*>(q->base_address);
  // A doorbell's packets never wrap around the ring's end: a profiler's queue interception (rocprofv3
  // --kernel-trace) reads them as one contiguous span and faulted on a window across the end.  A window that would
  // cross it starts at slot 0 instead, behind no-op barrier packets up to the end (the queue is empty here: the
  // previous window was waited for).
  const uint64_t w0 = hsa_queue_load_write_index_relaxed(q);
  const uint64_t off = w0 & (size - 1);
  const uint64_t pad = off && off + std::min<uint64_t>((uint64_t)K, size) > size ? size - off : 0;
  const uint64_t base = hsa_queue_add_write_index_relaxed(q, pad + (uint64_t)K) + pad;
  for (uint64_t j = 0; j < pad; ++j) {
    auto* bp = reinterpret_cast<hsa_barrier_and_packet_t*>(ring + ((w0 + j) & (size - 1)));
    std::memset(reinterpret_cast<char*>(bp) + 4, 0, sizeof(*bp) - 4);
    __atomic_store_n(reinterpret_cast<uint32_t*>(bp), (uint32_t)(HSA_PACKET_TYPE_BARRIER_AND << HSA_PACKET_HEADER_TYPE),
                     __ATOMIC_RELEASE);
  }
  if (pad) hsa_signal_store_screlease(q->doorbell_signal, (hsa_signal_value_t)(base - 1));
  ++d.windows;
  // the doorbell rings after the first packet and every kBell after it, not only after the last: the command processor
  // starts the window while the host still writes its packets (~35 ns each) and never runs out of them (a step takes
  // 2.4-3.6 us); RMX_QUEUE_EARLY=0 at the first window rings once, at the end (the A/B)
  const int bell = d.early ? kBell : 0;
  for (int i = 0; i < K; ++i) {
    const uint64_t idx = base + (uint64_t)i;
    if (i > 0 && (idx & (size - 1)) == 0)  // a window longer than the ring: each lap is its own doorbell
      hsa_signal_store_screlease(q->doorbell_signal, (hsa_signal_value_t)(idx - 1));
    // room in the ring: the packet processor has consumed packet idx - size (bounded, as the completion wait)
    for (uint32_t spin = 0; idx - hsa_queue_load_read_index_scacquire(q) >= size; ++spin) {
      if (d.fault.load()) return retire(d, "rmx queue: the queue faulted", err);
      if ((spin & 1023u) == 1023u && Clock::now() > deadline)
        return retire(d, "rmx queue: no ring room for a window's packets (the packet processor stalled)", err);
    }
    hsa_kernel_dispatch_packet_t* pk = ring + (idx & (size - 1));
    const hsa_kernel_dispatch_packet_t& b = d.built[(size_t)i];
    // the body after the first word (header + setup), which is stored last
    std::memcpy(reinterpret_cast<char*>(pk) + 4, reinterpret_cast<const char*>(&b) + 4, sizeof(b) - 4);
    pk->completion_signal = i == K - 1 ? d.done : n_timed && sig_of[(size_t)i] >= 0 ? d.tsig[(size_t)sig_of[(size_t)i]]
                                                                                   : hsa_signal_t{0};
    const uint16_t header = (uint16_t)((HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                                       (1 << HSA_PACKET_HEADER_BARRIER) |
                                       (HSA_FENCE_SCOPE_AGENT << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                       (HSA_FENCE_SCOPE_AGENT << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
    const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
    __atomic_store_n(reinterpret_cast<uint32_t*>(pk), (uint32_t)header | ((uint32_t)setup << 16), __ATOMIC_RELEASE);
    ++d.packets;
    if (bell && i + 1 < K && (i == 0 || (i + 1) % bell == 0))
      hsa_signal_store_screlease(q->doorbell_signal, (hsa_signal_value_t)idx);
  }
  hsa_signal_store_screlease(q->doorbell_signal, (hsa_signal_value_t)(base + (uint64_t)K - 1));
  const double left = std::max(0.0, std::chrono::duration<double>(deadline - Clock::now()).count());
  const uint64_t timeout = (uint64_t)(left * (double)d.tick_hz);
  const hsa_signal_value_t v =
      hsa_signal_wait_scacquire(d.done, HSA_SIGNAL_CONDITION_LT, 1, timeout, HSA_WAIT_STATE_ACTIVE);
  if (d.fault.load()) return retire(d, "rmx queue: the queue faulted", err);
  if (v >= 1) return retire(d, "rmx queue: a window did not complete", err);
  if (n_timed) {  // a packet starts after the previous one completed (barrier bit): every stamped signal is final here
    d.times.resize(3 * (size_t)n_timed);
    for (int j = 0; j < n_timed; ++j) {
      hsa_amd_profiling_dispatch_time_t t{};
      const hsa_signal_t sg = j == n_timed - 1 ? d.done : d.tsig[(size_t)j];
      if (hsa_amd_profiling_get_dispatch_time(d.agent, sg, &t) != HSA_STATUS_SUCCESS) {
        d.times.clear();
        *err = "rmx queue: hsa_amd_profiling_get_dispatch_time failed";
        return -1;
      }
      d.times[3 * (size_t)j] = (uint64_t)stamped_packet(j);
      // system timestamp ticks -> ns
      d.times[3 * (size_t)j + 1] = (uint64_t)((double)t.start * 1e9 / (double)d.tick_hz);
      d.times[3 * (size_t)j + 2] = (uint64_t)((double)t.end * 1e9 / (double)d.tick_hz);
    }
  }
  return 0;
}

void queue_set_timing(int device, int every) {
  if (device < 0 || device >= kMaxDevices) return;
  DeviceQueue& d = g_dev[device];
  std::lock_guard<std::mutex> lock(d.mu);
  d.timing = std::max(every, 0);  // (the last timed window's stamps stay readable until the next window)
}

int64_t queue_times(int device, uint64_t* out, int64_t cap) {
  if (device < 0 || device >= kMaxDevices) return 0;
  DeviceQueue& d = g_dev[device];
  std::lock_guard<std::mutex> lock(d.mu);
  const int64_t n = (int64_t)d.times.size() / 3;
  if (out && cap > 0) std::memcpy(out, d.times.data(), sizeof(uint64_t) * 3 * (size_t)std::min(n, cap));
  return n;
}

void queue_note_stream(int device) {
  if (device < 0 || device >= kMaxDevices) return;
  DeviceQueue& d = g_dev[device];
  std::lock_guard<std::mutex> lock(d.mu);
  ++d.stream_windows;
}

void queue_info(int device, QueueInfo* out) {
  *out = QueueInfo{};
  if (device < 0 || device >= kMaxDevices) return;
  DeviceQueue& d = g_dev[device];
  std::lock_guard<std::mutex> lock(d.mu);
  out->windows = d.windows;
  out->uploads = d.uploads;
  out->packets = d.packets;
  out->stream_windows = d.stream_windows;
  out->state = d.state;
}

int code_object_check(const void* co, size_t bytes, int64_t* n_step, int64_t* n_refused, std::string* first) {
  const CoCheck local = co ? check_code_object(static_cast<const unsigned char*>(co), bytes, kLayout) : CoCheck{};
  const CoCheck& c = co ? local : embedded_check();
  *n_step = c.n_step;
  *n_refused = (int64_t)c.refused.size();
  first->clear();
  if (!c.err.empty()) {
    *first = c.err;
    return -1;
  }
  // the first refused symbol in name order (deterministic for the caller)
  std::string best;
  for (const auto& kv : c.refused)
    if (best.empty() || kv.first < best) best = kv.first;
  if (!best.empty()) *first = best + ": " + c.refused.at(best);
  return 0;
}

}  // namespace rmx
