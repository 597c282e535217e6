// floor_bench.hip — launch-chain floors on MI355X for the step kernel's shape (diagnostic, not product).
// Graph-captured chains of K dependent launches; reports us per launch for:
//   null      : empty kernel, same grid
//   copy_dw   : the step kernel's exact traffic pattern (per env: t r/w, per agent 5 cols r/w + action r
//               + reward w, env_done w), dword per lane, no compute
//   copy_dw4  : same bytes, 4 envs per thread with 16-B loads/stores
// Build: hipcc -O3 --offload-arch=gfx950 floor_bench.hip -o floor_bench
#include <execinfo.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <signal.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

// SIGSEGV / SIGABRT: the raw backtrace and this process's mappings, so a fault inside a library (a round-2
// record showed one under rocprofv3's kernel trace) can be symbolized offline (addr2line on library + offset).
void fault_report(int sig) {
  void* pcs[64];
  const int n = backtrace(pcs, 64);
  dprintf(2, "floor_bench: signal %d; backtrace:\n", sig);
  backtrace_symbols_fd(pcs, n, 2);
  dprintf(2, "floor_bench: /proc/self/maps:\n");
  const int fd = open("/proc/self/maps", 0);
  if (fd >= 0) {
    char buf[4096];
    ssize_t k;
    while ((k = read(fd, buf, sizeof(buf))) > 0) (void)!write(2, buf, (size_t)k);
    close(fd);
  }
  signal(sig, SIG_DFL);
  raise(sig);
}

struct Cols {
  int* c[5];  // pos_x pos_y rm_q flags ep_ret  [A][N]
  int* t;     // [N]
  int* act;   // [A][N]
  int* rew;   // [A][N]
  unsigned char* done;
  long long N;
  int A;
};

__global__ void null_kernel(Cols) {}

__global__ void __launch_bounds__(256) copy_dw(Cols p) {
  long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= p.N) return;
  int t = p.t[e];
  int v[2][6];
#pragma unroll
  for (int a = 0; a < 2; ++a) {
#pragma unroll
    for (int k = 0; k < 5; ++k) v[a][k] = p.c[k][a * p.N + e];
    v[a][5] = p.act[a * p.N + e];
  }
  p.t[e] = t + 1;
#pragma unroll
  for (int a = 0; a < 2; ++a) {
#pragma unroll
    for (int k = 0; k < 5; ++k) p.c[k][a * p.N + e] = v[a][k] + v[a][5];
    p.rew[a * p.N + e] = v[a][5];
  }
  p.done[e] = (unsigned char)t;
}

// copy_dw with sc1 (write-through) buffer stores, as the fast-path step kernels store
__device__ __forceinline__ void st_sc1(int* base, long long i, int v) {
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b32(v, r, (unsigned)(i * 4), 0, 16);
}
__global__ void __launch_bounds__(256) copy_sc1(Cols p) {
  long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= p.N) return;
  int t = p.t[e];
  int v[2][6];
#pragma unroll
  for (int a = 0; a < 2; ++a) {
#pragma unroll
    for (int k = 0; k < 5; ++k) v[a][k] = p.c[k][a * p.N + e];
    v[a][5] = p.act[a * p.N + e];
  }
  st_sc1(p.t, e, t + 1);
#pragma unroll
  for (int a = 0; a < 2; ++a) {
#pragma unroll
    for (int k = 0; k < 5; ++k) st_sc1(p.c[k], a * p.N + e, v[a][k] + v[a][5]);
    st_sc1(p.rew, a * p.N + e, v[a][5]);
  }
  p.done[e] = (unsigned char)t;
}

// copy_sc1 with a dependent chain of `chain` VALU ops between the loads and the stores (models the step
// logic's latency), or without loads / without stores
template <int CHAIN>
__global__ void __launch_bounds__(256) copy_chain(Cols p, int mode) {
  long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= p.N) return;
  int v[2][6];
  int t = 1;
  if (mode != 2) {  // mode 2: stores only
    t = p.t[e];
#pragma unroll
    for (int a = 0; a < 2; ++a) {
#pragma unroll
      for (int k = 0; k < 5; ++k) v[a][k] = p.c[k][a * p.N + e];
      v[a][5] = p.act[a * p.N + e];
    }
  } else {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int k = 0; k < 6; ++k) v[a][k] = (int)e + k + a;
  }
  int x = v[0][0] ^ v[1][5];
#pragma unroll
  for (int i = 0; i < CHAIN; ++i) asm volatile("v_mad_u32_u24 %0, %0, 3, 1" : "+v"(x));
  if (mode == 1) {  // loads only: one conditional store keeps the loads alive
    int acc = t + x;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int k = 0; k < 6; ++k) acc ^= v[a][k];
    if (acc == 0x7fffffff) p.t[e] = acc;
    return;
  }
  st_sc1(p.t, e, t + 1 + (x & 0));
#pragma unroll
  for (int a = 0; a < 2; ++a) {
#pragma unroll
    for (int k = 0; k < 5; ++k) st_sc1(p.c[k], a * p.N + e, v[a][k] + v[a][5] + x);
    st_sc1(p.rew, a * p.N + e, v[a][5]);
  }
  p.done[e] = (unsigned char)t;
}

// a packed-state layout's I/O at A = 2 (experiment): per agent two state words (x|y|q|flag bits, agent_steps),
// ep_ret and the action loaded; the two state words and the reward stored (ep_ret rarely changes: not stored)
__global__ void __launch_bounds__(64) copy_packed(Cols p) {
  long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= p.N) return;
  int t = p.t[e];
  int v[2][4];
#pragma unroll
  for (int a = 0; a < 2; ++a) {
#pragma unroll
    for (int k = 0; k < 3; ++k) v[a][k] = p.c[k][a * p.N + e];
    v[a][3] = p.act[a * p.N + e];
  }
  st_sc1(p.t, e, t + 1);
#pragma unroll
  for (int a = 0; a < 2; ++a) {
#pragma unroll
    for (int k = 0; k < 2; ++k) st_sc1(p.c[k], a * p.N + e, v[a][k] + v[a][3]);
    st_sc1(p.rew, a * p.N + e, v[a][3] ^ v[a][2]);
  }
  p.done[e] = (unsigned char)t;
}
// the current layout's I/O with the default store set (rm_q / ep_ret not stored), 64-thread workgroups
__global__ void __launch_bounds__(64) copy_current(Cols p) {
  long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= p.N) return;
  int t = p.t[e];
  int v[2][6];
#pragma unroll
  for (int a = 0; a < 2; ++a) {
#pragma unroll
    for (int k = 0; k < 5; ++k) v[a][k] = p.c[k][a * p.N + e];
    v[a][5] = p.act[a * p.N + e];
  }
  st_sc1(p.t, e, t + 1);
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    st_sc1(p.c[0], a * p.N + e, v[a][0] + v[a][5]);
    st_sc1(p.c[1], a * p.N + e, v[a][1] + v[a][5]);
    st_sc1(p.c[3], a * p.N + e, v[a][3] + v[a][5]);
    st_sc1(p.rew, a * p.N + e, v[a][5] ^ v[a][2] ^ v[a][4]);
  }
  p.done[e] = (unsigned char)t;
}

// The default step kernel's I/O for a BASELINE config's shape (A agents, optional shaping column), 64-thread
// workgroups, sc1 stores of exactly the words it stores by default (kSkipRare: x, y, flags, reward per agent, t
// and env_done per env, shaping when present; rm_q and ep_ret loaded, not stored): the copy floor of that config.
template <int A, bool SHAPING>
__global__ void __launch_bounds__(64) copy_cfg(Cols p, int* shaping) {
  long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= p.N) return;
  int t = p.t[e];
  int v[A][6];
#pragma unroll
  for (int a = 0; a < A; ++a) {
#pragma unroll
    for (int k = 0; k < 5; ++k) v[a][k] = p.c[k][a * p.N + e];
    v[a][5] = p.act[a * p.N + e];
  }
  st_sc1(p.t, e, t + 1);
#pragma unroll
  for (int a = 0; a < A; ++a) {
    st_sc1(p.c[0], a * p.N + e, v[a][0] + v[a][5]);
    st_sc1(p.c[1], a * p.N + e, v[a][1] + v[a][5]);
    st_sc1(p.c[3], a * p.N + e, v[a][3] + v[a][5]);
    st_sc1(p.rew, a * p.N + e, v[a][5] ^ v[a][2] ^ v[a][4]);
    if (SHAPING) st_sc1(shaping, a * p.N + e, v[a][5] + v[a][2]);
  }
  p.done[e] = (unsigned char)t;
}

// copy_cfg plus exactly one dependent 4-B gather per agent after the column loads, into a 16 KB table (the merged
// lookup's shape: config 3's 4-B merged table is 10.8 KB, an L2 hit); the gathered word feeds every store, so the
// store burst waits for it as the step's does.  copy_cfg_gather - copy_cfg = the lookup's latency alone.
constexpr int kGatherEntries = 4096;
template <int A, bool SHAPING>
__global__ void __launch_bounds__(64) copy_cfg_gather(Cols p, int* shaping, const int* tbl) {
  long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= p.N) return;
  int t = p.t[e];
  int v[A][6];
#pragma unroll
  for (int a = 0; a < A; ++a) {
#pragma unroll
    for (int k = 0; k < 5; ++k) v[a][k] = p.c[k][a * p.N + e];
    v[a][5] = p.act[a * p.N + e];
  }
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<int*>(tbl), 0, kGatherEntries * 4, 0x00020000);
  int g[A];
#pragma unroll
  for (int a = 0; a < A; ++a) {  // every agent's gather in flight together
    const unsigned idx = (unsigned)(v[a][0] * 37 + v[a][1] * 11 + v[a][2] * 5 + v[a][5]) & (kGatherEntries - 1);
    g[a] = __builtin_amdgcn_raw_buffer_load_b32(r, idx * 4u, 0, 0);
  }
  st_sc1(p.t, e, t + 1);
#pragma unroll
  for (int a = 0; a < A; ++a) {
    st_sc1(p.c[0], a * p.N + e, v[a][0] + v[a][5] + (g[a] & 1));
    st_sc1(p.c[1], a * p.N + e, v[a][1] + v[a][5] + (g[a] & 2));
    st_sc1(p.c[3], a * p.N + e, v[a][3] + v[a][5] + (g[a] & 4));
    st_sc1(p.rew, a * p.N + e, v[a][5] ^ v[a][2] ^ v[a][4] ^ g[a]);
    if (SHAPING) st_sc1(shaping, a * p.N + e, v[a][5] + v[a][2] + g[a]);
  }
  p.done[e] = (unsigned char)(t ^ g[0]);
}

__global__ void __launch_bounds__(256) copy_dw4(Cols p) {
  long long e4 = ((long long)blockIdx.x * blockDim.x + threadIdx.x);
  if (e4 * 4 >= p.N) return;
  int4 t = reinterpret_cast<int4*>(p.t)[e4];
  int4 v[2][6];
#pragma unroll
  for (int a = 0; a < 2; ++a) {
#pragma unroll
    for (int k = 0; k < 5; ++k) v[a][k] = reinterpret_cast<int4*>(p.c[k] + a * p.N)[e4];
    v[a][5] = reinterpret_cast<int4*>(p.act + a * p.N)[e4];
  }
  t.x += 1; t.y += 1; t.z += 1; t.w += 1;
  reinterpret_cast<int4*>(p.t)[e4] = t;
#pragma unroll
  for (int a = 0; a < 2; ++a) {
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      int4 w = v[a][k];
      w.x += v[a][5].x; w.y += v[a][5].y; w.z += v[a][5].z; w.w += v[a][5].w;
      reinterpret_cast<int4*>(p.c[k] + a * p.N)[e4] = w;
    }
    reinterpret_cast<int4*>(p.rew + a * p.N)[e4] = v[a][5];
  }
  reinterpret_cast<uchar4*>(p.done)[e4] = make_uchar4(t.x, t.y, t.z, t.w);
}

// Graphs are destroyed only at exit when FLOOR_KEEP_GRAPHS is set (the round-2 SIGSEGV under the kernel tracer
// came right after the first graphs of a size were destroyed).
static std::vector<std::pair<hipGraphExec_t, hipGraph_t>> g_kept;

// FLOOR_EAGER=1: the chain as K eager launches (no graph): the form a kernel-trace pass can run (under
// rocprofv3 --kernel-trace, graph replays of these chains die in the tool's HSA intercept; profiles/r03_ab_log.md)
template <typename F>
double time_chain_eager(F launch, int K, hipStream_t s) {
  for (int i = 0; i < K; ++i) launch(s);
  CK(hipStreamSynchronize(s));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CK(hipEventRecord(a, s));
    for (int i = 0; i < K; ++i) launch(s);
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return best * 1e3 / K;
}

template <typename F>
double time_chain(F launch, int K, hipStream_t s) {
  if (std::getenv("FLOOR_EAGER")) return time_chain_eager(launch, K, s);
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int i = 0; i < K; ++i) launch(s);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CK(hipEventRecord(a, s));
    CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
  }
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  if (std::getenv("FLOOR_KEEP_GRAPHS")) {
    g_kept.push_back({ge, g});
  } else {
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  return best * 1e3 / K;
}

int main(int argc, char** argv) {
  signal(SIGSEGV, fault_report);
  signal(SIGABRT, fault_report);
  const int K = 500;
  const long long all_sizes[] = {64, 4096, 65536, 262144, 1048576, 4194304, 8388608};
  std::vector<long long> sizes(all_sizes, all_sizes + 7);
  if (argc > 1 && !std::strcmp(argv[1], "cfg")) sizes = {65536};  // the per-config floors only
  hipStream_t s;
  CK(hipStreamCreate(&s));
  for (long long N : sizes) {
    Cols p;
    p.N = N;
    p.A = 2;
    for (int k = 0; k < 5; ++k) CK(hipMalloc(&p.c[k], sizeof(int) * 2 * N));
    CK(hipMalloc(&p.t, sizeof(int) * N));
    CK(hipMalloc(&p.act, sizeof(int) * 2 * N));
    CK(hipMalloc(&p.rew, sizeof(int) * 2 * N));
    CK(hipMalloc(&p.done, N));
    const unsigned g1 = (unsigned)((N + 255) / 256), g4 = (unsigned)((N / 4 + 255) / 256);
    double tn = time_chain([&](hipStream_t st) { hipLaunchKernelGGL(null_kernel, dim3(g1), dim3(256), 0, st, p); }, K, s);
    double t1 = time_chain([&](hipStream_t st) { hipLaunchKernelGGL(copy_dw, dim3(g1), dim3(256), 0, st, p); }, K, s);
    double t4 = N >= 1024 ? time_chain([&](hipStream_t st) { hipLaunchKernelGGL(copy_dw4, dim3(g4 ? g4 : 1), dim3(256), 0, st, p); }, K, s) : 0;
    double ts = time_chain([&](hipStream_t st) { hipLaunchKernelGGL(copy_sc1, dim3(g1), dim3(256), 0, st, p); }, K, s);
    const double bytes = N * 2 * 52.5;
    printf("{\"n_envs\": %lld, \"null_us\": %.3f, \"copy_dw_us\": %.3f, \"copy_sc1_us\": %.3f, \"copy_dw4_us\": %.3f, \"copy_dw_TBs\": %.2f, \"copy_dw4_TBs\": %.2f",
           N, tn, t1, ts, t4, bytes / t1 / 1e6, t4 > 0 ? bytes / t4 / 1e6 : 0.0);
    if (N == 8388608) {  // the step's exact I/O (13 loads, 14 sc1 stores per lane) at the bandwidth-regime size
      const double tc = time_chain([&](hipStream_t st) { hipLaunchKernelGGL(copy_chain<0>, dim3(g1), dim3(256), 0, st, p, 0); }, 20, s);
      printf(", \"chain0_us\": %.3f, \"chain0_TBs\": %.2f", tc, bytes / tc / 1e6);
    }
    if (N == 65536) {  // dependent-chain, loads-only and stores-only variants at the headline size
      auto run = [&](auto kern, int mode) {
        return time_chain([&](hipStream_t st) { hipLaunchKernelGGL(kern, dim3(g1), dim3(256), 0, st, p, mode); }, K, s);
      };
      printf(", \"chain0_us\": %.3f", run(copy_chain<0>, 0));
      printf(", \"chain64_us\": %.3f", run(copy_chain<64>, 0));
      printf(", \"chain128_us\": %.3f", run(copy_chain<128>, 0));
      printf(", \"chain256_us\": %.3f", run(copy_chain<256>, 0));
      printf(", \"chain512_us\": %.3f", run(copy_chain<512>, 0));
      double tl = run(copy_chain<0>, 1);
      double tw = run(copy_chain<0>, 2);
      printf(", \"loads_only_us\": %.3f, \"stores_only_us\": %.3f", tl, tw);
      const unsigned g64 = (unsigned)((N + 63) / 64);
      const double tcur = time_chain([&](hipStream_t st) { hipLaunchKernelGGL(copy_current, dim3(g64), dim3(64), 0, st, p); }, K, s);
      const double tpk = time_chain([&](hipStream_t st) { hipLaunchKernelGGL(copy_packed, dim3(g64), dim3(64), 0, st, p); }, K, s);
      printf(", \"copy_current64_us\": %.3f, \"copy_packed64_us\": %.3f", tcur, tpk);
      // per BASELINE config: the default step's own I/O shape (A = 2, 1, 4, 3 + shaping), 64-thread workgroups
      int* sh = nullptr;
      int* c4[5];
      int *act4, *rew4, *t4;
      CK(hipMalloc(&sh, sizeof(int) * 4 * N));
      Cols q = p;  // A = 4 columns for configs 4 / 5
      for (int k = 0; k < 5; ++k) {
        CK(hipMalloc(&c4[k], sizeof(int) * 4 * N));
        q.c[k] = c4[k];
      }
      CK(hipMalloc(&act4, sizeof(int) * 4 * N));
      CK(hipMalloc(&rew4, sizeof(int) * 4 * N));
      CK(hipMalloc(&t4, sizeof(int) * N));
      q.act = act4, q.rew = rew4, q.t = t4;
      auto cfg = [&](auto kern, const Cols& cc) {
        return time_chain([&](hipStream_t st) { hipLaunchKernelGGL(kern, dim3(g64), dim3(64), 0, st, cc, sh); }, K, s);
      };
      printf(", \"copy_cfg2_us\": %.3f, \"copy_cfg3_us\": %.3f, \"copy_cfg4_us\": %.3f, \"copy_cfg5_us\": %.3f",
             cfg(copy_cfg<2, false>, q), cfg(copy_cfg<1, false>, q), cfg(copy_cfg<4, false>, q), cfg(copy_cfg<3, true>, q));
      int* tbl = nullptr;  // the gather table: small words, zero-initialised then filled with a pattern
      CK(hipMalloc(&tbl, sizeof(int) * kGatherEntries));
      {
        std::vector<int> h(kGatherEntries);
        for (int i = 0; i < kGatherEntries; ++i) h[i] = (i * 2654435761u) >> 20;
        CK(hipMemcpy(tbl, h.data(), sizeof(int) * kGatherEntries, hipMemcpyHostToDevice));
      }
      auto cfgg = [&](auto kern, const Cols& cc) {
        return time_chain([&](hipStream_t st) { hipLaunchKernelGGL(kern, dim3(g64), dim3(64), 0, st, cc, sh, tbl); }, K, s);
      };
      printf(", \"copy_cfg2_gather_us\": %.3f, \"copy_cfg3_gather_us\": %.3f, \"copy_cfg4_gather_us\": %.3f, "
             "\"copy_cfg5_gather_us\": %.3f",
             cfgg(copy_cfg_gather<2, false>, q), cfgg(copy_cfg_gather<1, false>, q), cfgg(copy_cfg_gather<4, false>, q),
             cfgg(copy_cfg_gather<3, true>, q));
      CK(hipFree(tbl));
      for (int k = 0; k < 5; ++k) CK(hipFree(c4[k]));
      CK(hipFree(act4));
      CK(hipFree(rew4));
      CK(hipFree(t4));
      CK(hipFree(sh));
    }
    printf("}\n");
    fflush(stdout);
    for (int k = 0; k < 5; ++k) CK(hipFree(p.c[k]));
    CK(hipFree(p.t));
    CK(hipFree(p.act));
    CK(hipFree(p.rew));
    CK(hipFree(p.done));
  }
  return 0;
}
