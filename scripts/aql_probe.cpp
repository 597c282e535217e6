// aql_probe.cpp — diagnostic (not product): what a K-step window costs on the host when the K dependent launches go
// through a HIP graph (hipGraphLaunch + hipStreamSynchronize) versus AQL packets written straight into an HSA queue
// of our own (K prebuilt packets, one doorbell, a spin-wait on the last packet's completion signal).  The kernel is a
// copy of config 2's step I/O at 65,536 envs (13 dword loads, 8 dword stores per lane, 64-thread workgroups), built
// as a raw gfx950 code object (aql_probe_kernel.hip) and loaded into both runtimes.
//   make -C scripts aql_probe && ./scripts/aql_probe scripts/aql_probe_kernel.hsaco
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <vector>

#define HK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));                 \
      exit(1);                                                                                  \
    }                                                                                           \
  } while (0)
#define SK(x)                                                                                   \
  do {                                                                                          \
    hsa_status_t s_ = (x);                                                                      \
    if (s_ != HSA_STATUS_SUCCESS) {                                                             \
      const char* m_ = nullptr;                                                                 \
      hsa_status_string(s_, &m_);                                                               \
      fprintf(stderr, "%s:%d hsa %d %s\n", __FILE__, __LINE__, (int)s_, m_ ? m_ : "");          \
      exit(1);                                                                                  \
    }                                                                                           \
  } while (0)

struct Args {  // the kernel's explicit arguments (no hidden arguments: the kernel reads no blockDim / gridDim)
  int n, blk;
  int* c[5];
  int* t;
  int* act;
  int* rew;
  unsigned char* done;
};

static hsa_agent_t g_gpu, g_cpu;
static int g_bdf = -1;
static hsa_amd_memory_pool_t g_kpool;

static hsa_status_t find_agents(hsa_agent_t a, void*) {
  hsa_device_type_t t;
  SK(hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t));
  if (t == HSA_DEVICE_TYPE_CPU && g_cpu.handle == 0) g_cpu = a;
  if (t == HSA_DEVICE_TYPE_GPU) {
    uint32_t bdf = 0;
    SK(hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf));
    if ((int)bdf == g_bdf) g_gpu = a;
  }
  return HSA_STATUS_SUCCESS;
}
static hsa_status_t find_kpool(hsa_amd_memory_pool_t p, void*) {
  hsa_amd_segment_t seg;
  SK(hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg));
  if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
  uint32_t flags = 0;
  SK(hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags));
  if (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT) {
    g_kpool = p;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main(int argc, char** argv) {
  const char* path = argc > 1 ? argv[1] : "scripts/aql_probe_kernel.hsaco";
  const int N = 65536, BLK = 64, REPS = 400;
  HK(hipSetDevice(0));
  int bus = 0, dev = 0;
  HK(hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, 0));
  HK(hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, 0));
  g_bdf = (bus << 8) | (dev << 3);
  Args a;
  a.n = N;
  a.blk = BLK;
  for (int k = 0; k < 5; ++k) HK(hipMalloc(&a.c[k], 4 * 2 * N));
  HK(hipMalloc(&a.t, 4 * N));
  HK(hipMalloc(&a.act, 4 * 2 * N));
  HK(hipMalloc(&a.rew, 4 * 2 * N));
  HK(hipMalloc(&a.done, N));
  for (int k = 0; k < 5; ++k) HK(hipMemset(a.c[k], 0, 4 * 2 * N));
  HK(hipMemset(a.t, 0, 4 * N));
  HK(hipMemset(a.act, 0, 4 * 2 * N));
  HK(hipDeviceSynchronize());

  std::ifstream f(path, std::ios::binary);
  std::vector<char> co((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  if (co.empty()) {
    fprintf(stderr, "no code object at %s\n", path);
    return 1;
  }
  // ---- HIP: the same code object as a module, launched K times inside a graph ----
  hipModule_t mod;
  hipFunction_t fn;
  HK(hipModuleLoadData(&mod, co.data()));
  HK(hipModuleGetFunction(&fn, mod, "copy_step_io"));
  hipStream_t st;
  HK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  using clk = std::chrono::steady_clock;
  auto hip_window = [&](int K) {
    hipGraph_t g;
    hipGraphExec_t ge;
    HK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    for (int i = 0; i < K; ++i) {
      Args ai = a;
      size_t sz = sizeof(ai);
      void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &ai, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
      HK(hipModuleLaunchKernel(fn, N / BLK, 1, 1, BLK, 1, 1, 0, st, nullptr, cfg));
    }
    HK(hipStreamEndCapture(st, &g));
    HK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    HK(hipGraphLaunch(ge, st));
    HK(hipStreamSynchronize(st));
    std::vector<double> w;
    for (int r = 0; r < REPS; ++r) {
      const auto t0 = clk::now();
      HK(hipGraphLaunch(ge, st));
      HK(hipStreamSynchronize(st));
      w.push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count());
    }
    HK(hipGraphExecDestroy(ge));
    HK(hipGraphDestroy(g));
    return median(w);
  };

  // ---- HSA: our own queue, prebuilt packets ----
  SK(hsa_init());
  SK(hsa_iterate_agents(find_agents, nullptr));
  if (!g_gpu.handle) {
    fprintf(stderr, "no HSA agent with BDF %x\n", g_bdf);
    return 1;
  }
  hsa_status_t ps = hsa_amd_agent_iterate_memory_pools(g_cpu, find_kpool, nullptr);
  if (ps != HSA_STATUS_INFO_BREAK && ps != HSA_STATUS_SUCCESS) SK(ps);
  hsa_code_object_reader_t rd;
  SK(hsa_code_object_reader_create_from_memory(co.data(), co.size(), &rd));
  hsa_executable_t ex;
  SK(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &ex));
  SK(hsa_executable_load_agent_code_object(ex, g_gpu, rd, nullptr, nullptr));
  SK(hsa_executable_freeze(ex, nullptr));
  hsa_executable_symbol_t sym;
  SK(hsa_executable_get_symbol_by_name(ex, "copy_step_io.kd", &g_gpu, &sym));
  uint64_t kobj = 0;
  uint32_t kargsz = 0, gseg = 0, pseg = 0;
  SK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &kobj));
  SK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &kargsz));
  SK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &gseg));
  SK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &pseg));
  if (kargsz > 256 || kargsz < sizeof(Args)) {
    fprintf(stderr, "unexpected kernarg segment size %u\n", kargsz);
    return 1;
  }
  hsa_queue_t* q = nullptr;
  SK(hsa_queue_create(g_gpu, 1024, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q));
  const int KMAX = 512;
  // kernel arguments in host kernarg memory (the CP / waves read them across PCIe) or, argv[2] == "vram", in device
  // memory written once (HIP's default on this GPU: "device kernargs")
  const bool vram = argc > 2 && !std::strcmp(argv[2], "vram");
  void* karg = nullptr;
  std::vector<char> kimg(256 * KMAX, 0);
  for (int i = 0; i < KMAX; ++i) std::memcpy(kimg.data() + 256 * i, &a, sizeof(a));
  if (vram) {
    HK(hipMalloc(&karg, kimg.size()));
    HK(hipMemcpy(karg, kimg.data(), kimg.size(), hipMemcpyHostToDevice));
  } else {
    SK(hsa_amd_memory_pool_allocate(g_kpool, kimg.size(), 0, &karg));
    SK(hsa_amd_agents_allow_access(1, &g_gpu, nullptr, karg));
    std::memcpy(karg, kimg.data(), kimg.size());
  }
  hsa_signal_t done;
  SK(hsa_signal_create(1, 0, nullptr, &done));
  auto aql_window = [&](int K, int scope_acq, int scope_rel) {
    auto submit = [&]() {
      const uint64_t idx = hsa_queue_add_write_index_relaxed(q, K);
      auto* base = static_cast<hsa_kernel_dispatch_packet_t*>(q->base_address);
      for (int i = 0; i < K; ++i) {
        hsa_kernel_dispatch_packet_t* pk = base + ((idx + i) & (q->size - 1));
        pk->workgroup_size_x = BLK;
        pk->workgroup_size_y = 1;
        pk->workgroup_size_z = 1;
        pk->grid_size_x = N;
        pk->grid_size_y = 1;
        pk->grid_size_z = 1;
        pk->private_segment_size = pseg;
        pk->group_segment_size = gseg;
        pk->kernel_object = kobj;
        pk->kernarg_address = static_cast<char*>(karg) + 256 * i;
        pk->reserved2 = 0;
        pk->completion_signal = i == K - 1 ? done : hsa_signal_t{0};
        const uint16_t header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                                (1 << HSA_PACKET_HEADER_BARRIER) |
                                (scope_acq << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                (scope_rel << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
        const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
        __atomic_store_n(reinterpret_cast<uint32_t*>(pk), (uint32_t)header | ((uint32_t)setup << 16), __ATOMIC_RELEASE);
      }
      hsa_signal_store_screlease(q->doorbell_signal, (hsa_signal_value_t)(idx + K - 1));
      hsa_signal_wait_scacquire(done, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_ACTIVE);
      hsa_signal_store_relaxed(done, 1);
    };
    submit();
    std::vector<double> w;
    for (int r = 0; r < REPS; ++r) {
      const auto t0 = clk::now();
      submit();
      w.push_back(std::chrono::duration<double, std::micro>(clk::now() - t0).count());
    }
    return median(w);
  };
  for (int K : {1, 20, 500}) {
    const double th = hip_window(K);
    const double ta = aql_window(K, HSA_FENCE_SCOPE_AGENT, HSA_FENCE_SCOPE_AGENT);
    const double ts = aql_window(K, HSA_FENCE_SCOPE_SYSTEM, HSA_FENCE_SCOPE_SYSTEM);
    printf("{\"K\": %d, \"hip_graph_window_us\": %.2f, \"aql_agent_window_us\": %.2f, \"aql_system_window_us\": %.2f, "
           "\"hip_us_per_step\": %.3f, \"aql_us_per_step\": %.3f}\n", K, th, ta, ts, th / K, ta / K);
    fflush(stdout);
  }
  // check the copy ran: t was incremented once per launch everywhere
  std::vector<int> h(N);
  HK(hipMemcpy(h.data(), a.t, 4 * N, hipMemcpyDeviceToHost));
  long long expect = 0;
  for (int K : {1, 20, 500}) expect += (long long)K * (REPS + 1) * 3;
  printf("{\"t0\": %d, \"tN\": %d, \"expected\": %lld}\n", h[0], h[N - 1], expect);
  SK(hsa_signal_destroy(done));
  SK(hsa_queue_destroy(q));
  if (vram)
    HK(hipFree(karg));
  else
    SK(hsa_amd_memory_pool_free(karg));
  SK(hsa_executable_destroy(ex));
  SK(hsa_code_object_reader_destroy(rd));
  SK(hsa_shut_down());
  return 0;
}
