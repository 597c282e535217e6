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

__global__ void probe_shuffle(int n, int active, uint16_t* ws, unsigned long long* out, unsigned long long* sink) {
  __shared__ unsigned char lds[256 * 64 + 512];
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  rmx::Pcg r = rmx::seed_pcg64(1234u + e);
  int32_t slot[2] = {0, 1};
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) < active) rmx::shuffle_slots<2>(r, n, ws + (int64_t)e * rmx::shuffle_stride(n), 2, slot);
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) out[e >> 6] = t1 - t0;
  if (slot[0] == 12345 + slot[1]) sink[0] = r.lo;
}

// branch-free draw loop: every draw stores at index i (a rejected draw's byte is overwritten by the accepted one);
// JUMP: two outputs per iteration from one state (s1 = M s + c, s2 = M^2 s + c (M + 1)), independent chains
template <bool JUMP>
__global__ void probe_draws2(int n, int active, unsigned long long* out, unsigned long long* sink) {
  __shared__ unsigned char lds[256 * 24];
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  rmx::Pcg r = rmx::seed_pcg64(1234u + e);
  uint32_t acc = 0, lane = threadIdx.x & 63;
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  if ((int)lane < active) {
    int32_t i = n - 1;
    uint32_t mask = 127;
    auto take = [&](uint32_t d) {
      const uint32_t v = d & mask;
      lds[((((uint32_t)i >> 2) << 6) + lane) * 4u + ((uint32_t)i & 3u)] = (unsigned char)v;
      const int32_t ok = (i > 0 && v <= (uint32_t)i) ? 1 : 0;
      i -= ok;
      mask = (uint32_t)i <= (mask >> 1) ? (mask >> 1) : mask;
    };
    auto outf = [](uint64_t hi, uint64_t lo) {
      const uint64_t x = hi ^ lo;
      const unsigned rot = (unsigned)(hi >> 58);
      return (x >> rot) | (x << ((64u - rot) & 63u));
    };
    if (!JUMP) {
      while (i > 0) {
        const uint64_t o = rmx::pcg_next64(r);
        take((uint32_t)o);
        take((uint32_t)(o >> 32));
      }
    } else {
      // c2 = c * (M + 1) mod 2^128, M2 = M^2 mod 2^128 (compile-time)
      constexpr uint64_t MH = 0x2360ED051FC65DA4ull, ML = 0x4385DF649FCCF645ull;
      constexpr unsigned __int128 M = ((unsigned __int128)MH << 64) | ML;
      constexpr unsigned __int128 M2 = M * M;
      const unsigned __int128 c = ((unsigned __int128)r.ihi << 64) | r.ilo;
      const unsigned __int128 c2 = c * (M + 1);
      unsigned __int128 st = ((unsigned __int128)r.hi << 64) | r.lo;
      while (i > 0) {
        const unsigned __int128 s1 = st * M + c, s2 = st * M2 + c2;
        const uint64_t o1 = outf((uint64_t)(s1 >> 64), (uint64_t)s1), o2 = outf((uint64_t)(s2 >> 64), (uint64_t)s2);
        take((uint32_t)o1);
        take((uint32_t)(o1 >> 32));
        take((uint32_t)o2);
        take((uint32_t)(o2 >> 32));
        st = s2;
      }
      r.lo = (uint64_t)st;
    }
    acc = (uint32_t)i;
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[e >> 6] = t1 - t0;
  if (acc == 0x12345u) sink[0] = r.lo + lds[lane];
}

// the random-start draw loop in isolation: 0 no store, 1 LDS byte store, 2 global u16 store
template <int STORE>
__global__ void probe_draws(int n, int active, uint16_t* ws, unsigned long long* out, unsigned long long* sink) {
  __shared__ unsigned char lds[256 * 24];
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  rmx::Pcg r = rmx::seed_pcg64(1234u + e);
  uint32_t acc = 0, lane = threadIdx.x & 63;
  uint16_t* row = ws + (int64_t)e * 96;
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  if ((int)lane < active) {
    int32_t i = n - 1;
    uint32_t mask = 127;
    auto take = [&](uint32_t d) {
      const uint32_t v = d & mask;
      if (i > 0 && v <= (uint32_t)i) {
        if (STORE == 1) lds[((((uint32_t)i >> 2) << 6) + lane) * 4u + ((uint32_t)i & 3u)] = (unsigned char)v;
        if (STORE == 2) row[i] = (uint16_t)v;
        acc += v;
        --i;
        mask = (uint32_t)i <= (mask >> 1) ? (mask >> 1) : mask;
      }
    };
    while (i > 0) {
      const uint64_t o = rmx::pcg_next64(r);
      take((uint32_t)o);
      take((uint32_t)(o >> 32));
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) out[e >> 6] = t1 - t0;
  if (acc == 0x12345u) sink[0] = r.lo + lds[lane];
}

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
  uint16_t* ws;
  CK(hipMalloc(&ws, sizeof(uint16_t) * 96 * 65536));
  for (int active : {1, 4, 64}) {
    for (int waves : {1, 1024}) {
      hipLaunchKernelGGL(probe_shuffle, dim3(waves), dim3(64), 0, 0, 89, active, ws, out, sink);
      CK(hipDeviceSynchronize());
      hipLaunchKernelGGL(probe_shuffle, dim3(waves), dim3(64), 0, 0, 89, active, ws, out, sink);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(h, out, sizeof(unsigned long long) * waves, hipMemcpyDeviceToHost));
      double sm = 0;
      for (int w = 0; w < waves; ++w) sm += (double)h[w];
      std::printf("{\"op\": \"shuffle_slots n=89 (global row)\", \"active_lanes\": %d, \"waves\": %d, \"memtime_ticks\": %.0f}\n",
                  active, waves, sm / waves);
    }
  }
  for (int store : {0, 1, 2}) {
    for (int active : {1, 64}) {
      for (int waves : {1, 1024}) {
        auto k = store == 0 ? probe_draws<0> : store == 1 ? probe_draws<1> : probe_draws<2>;
        hipLaunchKernelGGL(k, dim3(waves), dim3(64), 0, 0, 89, active, ws, out, sink);
        CK(hipDeviceSynchronize());
        hipLaunchKernelGGL(k, dim3(waves), dim3(64), 0, 0, 89, active, ws, out, sink);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h, out, sizeof(unsigned long long) * waves, hipMemcpyDeviceToHost));
        double sm = 0;
        for (int w = 0; w < waves; ++w) sm += (double)h[w];
        std::printf("{\"op\": \"draw loop n=89\", \"store\": %d, \"active_lanes\": %d, \"waves\": %d, \"memtime_ticks\": %.0f}\n",
                    store, active, waves, sm / waves);
      }
    }
  }
  for (int jump : {0, 1}) {
    for (int active : {1, 64}) {
      const int waves = 1024;
      auto k = jump ? probe_draws2<true> : probe_draws2<false>;
      hipLaunchKernelGGL(k, dim3(waves), dim3(64), 0, 0, 89, active, out, sink);
      CK(hipDeviceSynchronize());
      hipLaunchKernelGGL(k, dim3(waves), dim3(64), 0, 0, 89, active, out, sink);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(h, out, sizeof(unsigned long long) * waves, hipMemcpyDeviceToHost));
      double sm = 0;
      for (int w = 0; w < waves; ++w) sm += (double)h[w];
      std::printf("{\"op\": \"branch-free draw loop n=89\", \"jump2\": %d, \"active_lanes\": %d, \"waves\": %d, \"memtime_ticks\": %.0f}\n",
                  jump, active, waves, sm / waves);
    }
  }
  return 0;
}
