// Cost probe of the per-env numpy PCG64 on gfx950 (diagnostic, not product): shader cycles per
// pcg_next64 in a dependent chain, per seed_pcg64, and per 32-bit draw of the random-start shuffle's flat loop,
// one wave per SIMD (1,024 waves) and one wave alone.
// Build: hipcc -O3 --offload-arch=gfx950 -I../multiagent-rl-rm_amd/csrc pcg_probe.hip -o pcg_probe
#include <hip/hip_runtime.h>

#include <cstdio>

#include "rmx_device.h"

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
      return 1;                                                                \
    }                                                                          \
  } while (0)

using rmx::Pcg;

__global__ void probe(int mode, int iters, unsigned long long* out, unsigned long long* sink) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  Pcg r = {0x1234ull + e, 0x9876ull * e, 0x5555ull, 0x7777ull | 1ull};
  uint64_t acc = 0;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  if (mode == 0) {  // dependent pcg_next64
    for (int i = 0; i < iters; ++i) acc ^= rmx::pcg_next64(r);
  } else if (mode == 1) {  // seed_pcg64 (SeedSequence + two steps)
    for (int i = 0; i < iters; ++i) {
      r = rmx::seed_pcg64(acc + (uint64_t)e + (uint64_t)i);
      acc ^= r.lo;
    }
  } else if (mode == 2) {  // pcg_step only
    for (int i = 0; i < iters; ++i) {
      rmx::pcg_step(r);
      acc ^= r.lo;
    }
  } else {  // 64x64 -> low 64 multiplies in a chain
    uint64_t x = r.lo | 1ull;
    for (int i = 0; i < iters; ++i) x = x * 0x4385DF649FCCF645ull + 1ull;
    acc = x;
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) out[e >> 6] = t1 - t0;
  if (acc == 0x12345) sink[0] = acc;
}

int main() {
  unsigned long long *out, *sink;
  CK(hipMalloc(&out, sizeof(unsigned long long) * 4096));
  CK(hipMalloc(&sink, 8));
  const char* names[] = {"pcg_next64", "seed_pcg64", "pcg_step", "mul64 chain"};
  unsigned long long h[4096];
  for (int mode = 0; mode < 4; ++mode) {
    for (int waves : {1, 1024}) {
      const int iters = mode == 1 ? 64 : 1024;
      hipLaunchKernelGGL(probe, dim3(waves), dim3(64), 0, 0, mode, iters, out, sink);
      CK(hipDeviceSynchronize());
      hipLaunchKernelGGL(probe, dim3(waves), dim3(64), 0, 0, mode, iters, out, sink);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(h, out, sizeof(unsigned long long) * waves, hipMemcpyDeviceToHost));
      double s = 0;
      for (int w = 0; w < waves; ++w) s += (double)h[w];
      std::printf("{\"op\": \"%s\", \"waves\": %d, \"memtime_ticks_per_iter\": %.1f}\n", names[mode], waves,
                  s / waves / iters);
    }
  }
  return 0;
}
