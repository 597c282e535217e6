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

// ---- numpy default_rng(seed) on the device: SeedSequence -> PCG64 (XSL-RR 128/64) ----------------
// Restated from numpy/random/bit_generator.pyx (SeedSequence.mix_entropy / generate_state) and pcg64.h
// (pcg_setseq_128_srandom_r, pcg_setseq_128_xsl_rr_64_random_r); Generator.random = (next64 >> 11) * 2^-53.
struct Pcg {
  uint64_t hi, lo, ihi, ilo;  // 128-bit state, 128-bit increment
};

__device__ __forceinline__ void pcg_step(Pcg& r) {
  constexpr uint64_t MH = 0x2360ED051FC65DA4ull, ML = 0x4385DF649FCCF645ull;
  const uint64_t nlo = r.lo * ML;
  const uint64_t nhi = __umul64hi(r.lo, ML) + r.lo * MH + r.hi * ML;
  const uint64_t slo = nlo + r.ilo;
  r.hi = nhi + r.ihi + (slo < nlo ? 1ull : 0ull);
  r.lo = slo;
}

__device__ __forceinline__ uint64_t pcg_next64(Pcg& r) {
  pcg_step(r);
  const uint64_t x = r.hi ^ r.lo;
  const unsigned rot = (unsigned)(r.hi >> 58);
  return (x >> rot) | (x << ((64u - rot) & 63u));
}

__device__ __forceinline__ uint32_t ss_hashmix(uint32_t v, uint32_t& hc) {
  v ^= hc;
  hc *= 0x931e8875u;
  v *= hc;
  return v ^ (v >> 16);
}

__device__ __forceinline__ uint32_t ss_mix(uint32_t x, uint32_t y) {
  const uint32_t r = 0xca01f9ddu * x - 0x4973f715u * y;
  return r ^ (r >> 16);
}

// FrozenLake random_start_positions (ma_frozen_lake.py:59-64, 156-172): rng.shuffle(free_cells) of a Python list
// = numpy's untyped Generator.shuffle: Fisher-Yates from the end, for i = n-1 .. 1 swap(L[i], L[j_i]) with
// j_i = random_interval(i): the smallest all-ones mask >= i, 32-bit draws rejected while (draw & mask) > i.
// numpy's PCG64 hands out a 64-bit output as two 32-bit draws, low half first (the shuffle starts on a freshly
// seeded generator, so no half is buffered before it; the half left over at the end is never used: slip draws
// read whole 64-bit outputs).  Restated and checked against numpy 2.2 in tests/test_oracle_golden.py.
//
// Only the first A slots of the shuffled list matter.  Instead of permuting an n-entry array with a dependent
// read-modify-write per swap (round 2: ~50 us per step at 65,536 envs, every wave waiting on a chain of ~180
// dependent global accesses), the draws run as one flat loop that writes each accepted j_i to the env's
// workspace row (fire-and-forget stores), then ONE pass over the row undoes the swaps for the A slots only:
// slot p ends holding the element that started at index pos, where pos runs from p through the swaps in the
// reverse of their application order (i = 1 .. n-1: pos == i -> j_i, pos == j_i -> i).  Rows are 16-B aligned
// (stride = shuffle_stride(n), rmx_internal.h) and read back 8 entries per load, two loads ahead.
template <int AMAX>
__device__ __forceinline__ void shuffle_slots(Pcg& r, int32_t n, uint16_t* __restrict__ row, int A,
                                              int32_t (&slot)[AMAX]) {
  int32_t i = n - 1;
  uint32_t mask = (uint32_t)max(i, 0);
  mask |= mask >> 1;
  mask |= mask >> 2;
  mask |= mask >> 4;
  mask |= mask >> 8;
  mask |= mask >> 16;
  auto take = [&](uint32_t d) {  // one 32-bit draw against the current i
    const uint32_t v = d & mask;
    if (i > 0 && v <= (uint32_t)i) {
      row[i] = (uint16_t)v;
      --i;
      mask = (uint32_t)i <= (mask >> 1) ? (mask >> 1) : mask;
    }
  };
  while (i > 0) {
    const uint64_t o = pcg_next64(r);
    take((uint32_t)o);
    take((uint32_t)(o >> 32));
  }
#pragma unroll
  for (int a = 0; a < AMAX; ++a) slot[a] = a;
  typedef uint4 __attribute__((may_alias)) uint4_alias;  // read back what the u16 stores wrote (no TBAA reordering)
  const uint4_alias* rv = reinterpret_cast<const uint4_alias*>(row);
  const int32_t nc = (n + 7) >> 3;
  uint4 cur = nc > 0 ? rv[0] : make_uint4(0u, 0u, 0u, 0u);
  uint4 nxt = nc > 1 ? rv[1] : make_uint4(0u, 0u, 0u, 0u);
  for (int32_t c = 0; c < nc; ++c) {
    const uint4 nn = c + 2 < nc ? rv[c + 2] : make_uint4(0u, 0u, 0u, 0u);
    const uint32_t w[4] = {cur.x, cur.y, cur.z, cur.w};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int32_t ii = c * 8 + k;
      const int32_t jj = (int32_t)((w[k >> 1] >> ((k & 1) * 16)) & 0xFFFFu);
      if (ii >= 1 && ii < n) {
#pragma unroll
        for (int a = 0; a < AMAX; ++a)
          if (a < A) slot[a] = slot[a] == ii ? jj : (slot[a] == jj ? ii : slot[a]);
      }
    }
    cur = nxt;
    nxt = nn;
  }
}

__device__ inline Pcg seed_pcg64(uint64_t seed) {
  uint32_t ent0 = (uint32_t)seed, ent1 = (uint32_t)(seed >> 32);
  const int n = (seed >> 32) ? 2 : 1;  // _coerce_to_uint32_array: little-endian 32-bit words (0 -> [0])
  uint32_t pool[4], hc = 0x43b0d7e5u;
#pragma unroll
  for (int i = 0; i < 4; ++i) pool[i] = ss_hashmix(i == 0 ? ent0 : (i == 1 && n == 2) ? ent1 : 0u, hc);
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int d = 0; d < 4; ++d)
      if (s != d) pool[d] = ss_mix(pool[d], ss_hashmix(pool[s], hc));
  uint32_t w[8], hb = 0x8b51f9ddu;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint32_t x = pool[i & 3] ^ hb;
    hb *= 0x58f38dedu;
    x *= hb;
    w[i] = x ^ (x >> 16);
  }
  const uint64_t v0 = (uint64_t)w[0] | ((uint64_t)w[1] << 32), v1 = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
  const uint64_t v2 = (uint64_t)w[4] | ((uint64_t)w[5] << 32), v3 = (uint64_t)w[6] | ((uint64_t)w[7] << 32);
  Pcg r;
  r.ihi = (v2 << 1) | (v3 >> 63);  // inc = (initseq << 1) | 1
  r.ilo = (v3 << 1) | 1ull;
  r.hi = 0;
  r.lo = 0;
  pcg_step(r);  // state = 0*M + inc
  const uint64_t lo = r.lo + v1;  // state += initstate
  r.hi = r.hi + v0 + (lo < r.lo ? 1ull : 0ull);
  r.lo = lo;
  pcg_step(r);
  return r;
}

template <typename P>  // KParams (generic kernels) or FastParams (FrozenLake slip on the fast path)
__device__ __forceinline__ uint64_t seed_of(const P& p, int64_t e_global, int32_t k) {
  return p.base_seed * p.seed_scale + (uint64_t)e_global * p.seed_env_stride + (uint64_t)k * p.seed_episode_stride;
}

// rng.choice(outcomes, p=probs) = outcomes[searchsorted(cdf, u, side="right")], intended in [0, 4).  The
// intended action's row is selected from uniform (kernel-argument) values: indexing the parameter arrays with a
// lane-varying action made the compiler fetch them per lane from the kernarg segment, dependent loads per
// agent-step (generic kernel, config 2 with slip, 65,536 envs: 6.54 -> 6.42-6.44 us per step).
__device__ __forceinline__ uint32_t sel4(uint32_t i, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  return (i & 2u) ? ((i & 1u) ? d : c) : ((i & 1u) ? b : a);
}
__device__ __forceinline__ uint32_t ufl(int32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t ufl_u64(uint64_t v) {
  const uint32_t lo = ufl((int32_t)(uint32_t)v), hi = ufl((int32_t)(uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}
template <typename P>
__device__ __forceinline__ int32_t slip_choice(const P& p, int32_t intended_action, Pcg& r) {
#ifdef RMX_DIAG
  if (p.diag & 32768) return intended_action;  // timing ablation: no draw
#endif
  const uint32_t intended = (uint32_t)intended_action;
  // Generator.random() = m * 2^-53 with m = next64 >> 11; cdf <= u is compared exactly as thr <= m on integers
  // (thr = ceil(cdf * 2^53), host slip_threshold) instead of a u64 -> f64 conversion and f64 compares
  const uint64_t m = pcg_next64(r) >> 11;
  if (p.slip_uniform) {  // one cdf for every intended action (host slip_fill): uniform thresholds, packed outcomes
    const uint32_t n = ufl(p.slip_n[0]);
    uint32_t idx = 0;
#pragma unroll
    for (int i = 0; i < 3; ++i) idx += ((uint32_t)i + 1u < n && ufl_u64(p.slip_thr[0][i]) <= m) ? 1u : 0u;
    return (int32_t)((ufl_u64(p.slip_pack) >> (3u * (4u * intended + idx))) & 7u);
  }
  // (the general form: every intended action its own cdf, selected per lane from the uniform table values)
  const uint32_t n = sel4(intended, ufl(p.slip_n[0]), ufl(p.slip_n[1]), ufl(p.slip_n[2]), ufl(p.slip_n[3]));
  uint32_t idx = 0;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const uint64_t c0 = ufl_u64(p.slip_thr[0][i]), c1 = ufl_u64(p.slip_thr[1][i]);
    const uint64_t c2 = ufl_u64(p.slip_thr[2][i]), c3 = ufl_u64(p.slip_thr[3][i]);
    const uint64_t c = (intended & 2u) ? ((intended & 1u) ? c3 : c2) : ((intended & 1u) ? c1 : c0);
    idx += ((uint32_t)i + 1u < n && c <= m) ? 1u : 0u;
  }
  uint32_t o[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
    o[j] = sel4(intended, ufl(p.slip_out[0][j]), ufl(p.slip_out[1][j]), ufl(p.slip_out[2][j]), ufl(p.slip_out[3][j]));
  return (int32_t)sel4(idx, o[0], o[1], o[2], o[3]);
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
