// rmx_device.h — device helpers shared by the gfx950 kernels (action hash, per-wave statistics).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rmx_internal.h"

namespace rmx {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + kGolden;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// a = splitmix64(seed ^ (((t*N + e)*A + i) * GR)) >> 62
__device__ __forceinline__ int32_t hash_action(uint64_t seed, int64_t t, int64_t n_global, int64_t e, int A, int i) {
  uint64_t ctr = (((uint64_t)t * (uint64_t)n_global + (uint64_t)e) * (uint64_t)A + (uint64_t)i) * kGolden;
  return (int32_t)(splitmix64(seed ^ ctr) >> 62);
}

// Per-lane episode-statistics contribution, reduced per wave.
struct LaneStats {
  double ret;
  int episodes, successes, length;
};

// ---- wave64 sums without the LDS crossbar: DPP within each 16-lane row, then 4 readlanes ----------
// quad_perm[1,0,3,2] (0xB1), quad_perm[2,3,0,1] (0x4E), row_half_mirror (0x141), row_mirror (0x140) leave
// every lane of a row holding the row sum; lanes 15/31/47/63 are then summed in a fixed order.  Every lane
// of the wave must be active (callers reach this outside any lane-divergent branch).
template <int CTRL>
__device__ __forceinline__ uint32_t dpp32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}

template <int CTRL>
__device__ __forceinline__ double dpp64(double v) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const uint32_t lo = dpp32<CTRL>((uint32_t)b), hi = dpp32<CTRL>((uint32_t)(b >> 32));
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
  v += dpp32<0xB1>(v);
  v += dpp32<0x4E>(v);
  v += dpp32<0x141>(v);
  v += dpp32<0x140>(v);
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 15) + (uint32_t)__builtin_amdgcn_readlane((int)v, 31) +
         (uint32_t)__builtin_amdgcn_readlane((int)v, 47) + (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, lane);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), lane);
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

__device__ __forceinline__ double wave_sum_f64(double v) {
  v += dpp64<0xB1>(v);
  v += dpp64<0x4E>(v);
  v += dpp64<0x141>(v);
  v += dpp64<0x140>(v);
  return ((readlane_f64(v, 15) + readlane_f64(v, 31)) + readlane_f64(v, 47)) + readlane_f64(v, 63);
}

// The wave's slab slot, loaded by lane 0 at kernel start (its latency hides under the state loads) so
// the flush at the end is a plain store: no atomic keeps the launch alive after the last wave.
struct SlabSlot {
  double v[RMX_NSTATS];
};

__device__ __forceinline__ SlabSlot slab_prefetch(const double* __restrict__ slab) {
  SlabSlot s = {{0.0, 0.0, 0.0, 0.0}};
  if ((threadIdx.x & 63) == 0) {
    const size_t w = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const double2* q = reinterpret_cast<const double2*>(slab + w * RMX_NSTATS);
    const double2 a = q[0], b = q[1];
    s.v[0] = a.x;
    s.v[1] = a.y;
    s.v[2] = b.x;
    s.v[3] = b.y;
  }
  return s;
}

// Per-wave statistics of a whole launch (fused rollouts): shuffle-reduce, lane 0 adds into the wave's slot.
__device__ __forceinline__ void wave_flush(double* __restrict__ slab, const LaneStats& ls, bool any) {
  // `any` must be wave-uniform
  if (!any) return;
  double r = ls.ret;
  int ep = ls.episodes, sc = ls.successes, ln = ls.length;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    r += __shfl_xor(r, o, 64);
    ep += __shfl_xor(ep, o, 64);
    sc += __shfl_xor(sc, o, 64);
    ln += __shfl_xor(ln, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    // One wave owns one slab slot per launch, so the order of adds is fixed (stream order): the
    // no-return f64 atomics only avoid a load->store round trip at the end of the wave.
    const size_t w = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    double* s = slab + w * RMX_NSTATS;
    unsafeAtomicAdd(s + RMX_STAT_SUM_RETURN, r);
    unsafeAtomicAdd(s + RMX_STAT_EPISODES, (double)ep);
    unsafeAtomicAdd(s + RMX_STAT_SUCCESSES, (double)sc);
    unsafeAtomicAdd(s + RMX_STAT_SUM_LENGTH, (double)ln);
  }
}

__device__ __forceinline__ void wave_flush_slot(double* __restrict__ slab, const SlabSlot& old, const LaneStats& ls,
                                                bool any) {
  if (!any) return;  // wave-uniform
  const double r = wave_sum_f64(ls.ret);
  // episodes (<= 64) and successes (<= 512) share one word; lengths (<= 64 * 60001) get their own
  const uint32_t es = wave_sum_u32((uint32_t)ls.episodes | ((uint32_t)ls.successes << 16));
  const uint32_t ln = wave_sum_u32((uint32_t)ls.length);
  const uint32_t ep = es & 0xFFFFu, sc = es >> 16;
  if ((threadIdx.x & 63) == 0) {  // one owner per slot per launch; launches are stream-ordered
    const size_t w = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    double2* q = reinterpret_cast<double2*>(slab + w * RMX_NSTATS);
    q[0] = make_double2(old.v[0] + r, old.v[1] + (double)ep);
    q[1] = make_double2(old.v[2] + (double)sc, old.v[3] + (double)ln);
  }
}

}  // namespace rmx
