// rmx_sync.hip — the resident host-boundary stepper behind rmx_reset_sync / rmx_step_sync.
//
// The reference's per-call API (RMEnvironmentWrapper.reset / .step, rm_environment_wrapper.py:28-107, driven by
// frozen_lake_main.py:336-376 and office_main.py:1696-1749) hands ONE environment's actions in and wants its
// five dicts back before the next call.  Launching a kernel per call and copying the outputs back costs a
// launch, a completion signal and one or more copies every step.  Here one workgroup stays resident between
// calls instead: the env's state lives in its registers, the tables in its LDS, and a lane polls a request
// line in pinned host memory.  The host writes the actions and bumps the request number; the workgroup steps
// (the same agent_step / env_step as the generic kernels, rmx_generic.h), writes the output columns straight
// into host memory, fences at system scope and bumps the acknowledgement number, which the host polls in
// its own memory.  Each side only reads memory local to it in its poll loop.
//
// Lifetime: the workgroup exits on an exit request, after idle_ticks without a request (the host relaunches on
// the next call; rmx_capi.cpp), or after life_ticks in all.  Every wave leaves the loop together (the request
// word is broadcast through LDS), and on exit writes its state back to the bound device columns, so the
// asynchronous entry points (which end the resident workgroup first) continue from it.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rmx_device.h"
#include "rmx_generic.h"
#include "rmx_internal.h"

namespace rmx {

namespace {

constexpr uint32_t kSyncTimeout = 0;

// The seed-schedule seed of env e_global in its k-th episode under base seed `base` (rmx.h, stochastic mode).
__device__ __forceinline__ uint64_t schedule_seed(const KParams& p, uint64_t base, int64_t e_global, int32_t k) {
  return base * p.seed_scale + (uint64_t)e_global * p.seed_env_stride + (uint64_t)k * p.seed_episode_stride;
}

// The outputs of one request into the host-mapped mailbox (SyncCols' packed records): 16-B buffer stores with
// sc0 | sc1 (system scope, write-through to host memory); the caller waits for their completion (s_waitcnt)
// before the acknowledgement, so no L2 writeback or invalidate is ever needed.
constexpr int kSysCoherent = 17;  // sc0 | sc1
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int AMAX, bool QRM>
__device__ __forceinline__ void store_outputs(const SyncCols& c, const KParams& p, int64_t e, const AgentReg (&s)[AMAX],
                                              int32_t t, const AgentOut (&o)[AMAX], bool done, bool stepped,
                                              const Lds& L) {
  const int A = AMAX <= 4 ? AMAX : p.A;
  const auto rr = __builtin_amdgcn_make_buffer_rsrc(c.rec, 0, (int)(32 * A * p.N), 0x00020000);
  const auto re = __builtin_amdgcn_make_buffer_rsrc(c.envrec, 0, (int)(16 * p.N), 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(u32x4{(uint32_t)t, (uint32_t)done, 0u, 0u}, re, (uint32_t)e * 16u, 0,
                                         kSysCoherent);
#pragma unroll
  for (int a = 0; a < AMAX; ++a) {
    if (AMAX <= 4 || a < p.A) {
      const uint32_t off = ((uint32_t)e * (uint32_t)A + (uint32_t)a) * 32u;
      const uint32_t enc = (uint32_t)((s[a].y * p.W + s[a].x) * p.enc_nq[a] + s[a].q);
      __builtin_amdgcn_raw_buffer_store_b128(
          u32x4{((uint32_t)s[a].x & 0xFFFFu) | ((uint32_t)s[a].y << 16), (uint32_t)s[a].q, s[a].f,
                stepped ? __float_as_uint(o[a].reward) : 0u},
          rr, off, 0, kSysCoherent);
      __builtin_amdgcn_raw_buffer_store_b128(
          u32x4{stepped ? __float_as_uint(o[a].renv) : 0u, __float_as_uint(s[a].ret),
                stepped ? __float_as_uint(o[a].shaping) : 0u, enc},
          rr, off + 16u, 0, kSysCoherent);
      if constexpr (QRM)
        if (stepped) emit_qrm_to<true>(o[a], a, e, L, p, c.qrm_s, c.qrm_sn, c.qrm_rq, c.qrm_done);
    }
  }
}

}  // namespace

// One workgroup, thread e = env e (N <= RMX_SYNC_MAX_ENVS).  STOCH: per-env PCG64 (slip, random starts); QRM:
// the counterfactual columns are computed (compile-time, so the common instantiation carries none of their code).
template <int KIND, int AMAX, bool STOCH, bool QRM>
__global__ void __launch_bounds__(256) resident_kernel(KParams p, SyncIO io) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  __shared__ uint32_t sh_op, sh_seq, sh_acts, sh_bad;
  __shared__ uint64_t sh_seed;
#ifdef RMX_DIAG
  __shared__ uint64_t sh_t_seen;
#endif
  const int64_t N = p.N;
  const int64_t e = threadIdx.x;
  const bool live = e < N;
  AgentReg s[AMAX];
  int32_t t = 0, episode = 0;
  Pcg rng = {0, 0, 0, 0};
  uint64_t base = p.base_seed;
  if (live) {
    t = p.t[e];
#pragma unroll
    for (int a = 0; a < AMAX; ++a) {
      if (AMAX <= 4 || a < p.A) {
        const int64_t k = (int64_t)a * N + e;
        s[a] = {p.pos_x[k], p.pos_y[k], p.rm_q[k], p.flags[k], p.ep_ret[k]};
      }
    }
    if constexpr (STOCH) {
      rng = {p.rng[e], p.rng[N + e], p.rng[2 * N + e], p.rng[3 * N + e]};
      episode = p.episode[e];
    }
  }
  stage_tables(lds, p.tables, p.tables_n16);
  __syncthreads();
  const Lds L = lds_view(lds, p);
  LaneStats ls = {0.0, 0, 0, 0};
  AgentOut o[AMAX] = {};
  bool done = false, stepped = false;
  uint32_t bad_any = 0;
  uint32_t last = io.seq0;
  const uint64_t t_start = (uint64_t)wall_clock64();
  uint64_t t_idle = t_start;
  // the request word: one 16-B system-coherent load (sc0 | sc1) through a buffer descriptor
  const auto req_rsrc = __builtin_amdgcn_make_buffer_rsrc(io.req, 0, 16, 0x00020000);
  for (;;) {
    if (threadIdx.x == 0) {  // the only poller: one lane, one 16-B read per poll, s_sleep between polls
      uint32_t seq = last, ctl = kSyncTimeout, acts = 0;
      for (;;) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(req_rsrc, 0, 0, kSysCoherent);
        if (v[0] != last && v[0] == v[3]) {  // a new request, read whole (the echo rejects a torn read)
          seq = v[0];
          ctl = v[1];
          acts = v[2];
          break;
        }
        const uint64_t now = (uint64_t)wall_clock64();
        if (now - t_idle > io.idle_ticks || now - t_start > io.life_ticks) break;  // op stays kSyncTimeout
        __builtin_amdgcn_s_sleep(2);
      }
      // the action array and the seed were written before the request word and are read below with
      // system-scope loads (no cached copy exists), after the request word: no fence needed
      if ((ctl & 3u) == kSyncReset)
        sh_seed = __hip_atomic_load(&io.req->seed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      sh_seq = seq;
      sh_op = ctl;
      sh_acts = acts;
      sh_bad = 0;
#ifdef RMX_DIAG
      sh_t_seen = (uint64_t)wall_clock64();
#endif
    }
    __syncthreads();
    const uint32_t ctl = sh_op, seq = sh_seq, op = ctl & 3u;
    if (op != kSyncStep && op != kSyncReset) break;  // exit request or timeout: uniform over the workgroup
    uint32_t bad = 0;
    if (live) {
      if (op == kSyncReset) {  // rmx_reset for every env (reset_kernel) with the request's base seed
        base = sh_seed;
        t = 0;
#pragma unroll
        for (int a = 0; a < AMAX; ++a)
          if (AMAX <= 4 || a < p.A) {
            s[a] = {p.start_x[a], p.start_y[a], p.init_q[a], RMX_F_ACTIVE, 0.0f};
          }
        if constexpr (STOCH) {
          episode = 0;
          rng = seed_pcg64(schedule_seed(p, base, p.env_offset + e, 0));
          if (p.random_starts) random_starts<AMAX>(p, rng, e, s);
        }
        done = false;
        stepped = false;
      } else {
        int32_t act[AMAX];
#pragma unroll
        for (int a = 0; a < AMAX; ++a) {
          if (AMAX <= 4 || a < p.A) {
            const int64_t k = (int64_t)a * N + e;
            if (ctl & kSyncInline) {  // 4-bit fields: k = 0..6 in ctl from bit 4, k = 7..14 in the acts word
              act[a] = (int32_t)(k < 7 ? (ctl >> (4 + 4 * k)) & 15u : (sh_acts >> (4 * (k - 7))) & 15u);
            } else {
              act[a] = (int32_t)__hip_atomic_load(reinterpret_cast<const uint32_t*>(io.act) + k, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_SYSTEM);
            }
          }
        }
        if ((ctl & kSyncAutoreset) && (s[0].f & RMX_F_ENV_DONE)) {  // the loop's reset() before this step
          reset_regs<AMAX>(s, t, p);
          if constexpr (STOCH) {
            episode += 1;
            rng = seed_pcg64(schedule_seed(p, base, p.env_offset + e, episode));
            if (p.random_starts) random_starts<AMAX>(p, rng, e, s);
          }
        }
        const float disc = p.gamma_is_one ? 1.0f : p.disc[min((uint32_t)t, (uint32_t)p.max_t + 1u)];
        done = env_step<KIND, AMAX>(s, t, act, L, p, disc, o, ls, &bad, STOCH ? &rng : nullptr);
        stepped = true;
      }
      store_outputs<AMAX, QRM>(io.out, p, e, s, t, o, done, stepped, L);
    }
    bad_any |= bad;
    if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(&sh_bad, 1u);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_waitcnt(0);  // this lane's output stores are complete (gfx9: stores count in vmcnt)
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __syncthreads();  // ... for every lane; also orders the reads of sh_* before the next poll
    if (threadIdx.x == 0) {
#ifdef RMX_DIAG
      __hip_atomic_store(&io.ack->t_seen, sh_t_seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&io.ack->t_done, (uint64_t)wall_clock64(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#endif
      // {seq, bad} as one 8-B store: the host reads bad after it sees seq
      __hip_atomic_store(reinterpret_cast<uint64_t*>(io.ack), (uint64_t)seq | ((uint64_t)sh_bad << 32),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      t_idle = (uint64_t)wall_clock64();
    }
    last = seq;
  }
  // write-back: the device columns continue from the resident state (the base seed is the host's copy)
  if (live) {
    p.t[e] = t;
#pragma unroll
    for (int a = 0; a < AMAX; ++a) {
      if (AMAX <= 4 || a < p.A) {
        const int64_t k = (int64_t)a * N + e;
        p.pos_x[k] = s[a].x;
        p.pos_y[k] = s[a].y;
        p.rm_q[k] = s[a].q;
        p.flags[k] = s[a].f;
        p.ep_ret[k] = s[a].ret;
      }
    }
    if constexpr (STOCH) {
      p.rng[e] = rng.hi;
      p.rng[N + e] = rng.lo;
      p.rng[2 * N + e] = rng.ihi;
      p.rng[3 * N + e] = rng.ilo;
      p.episode[e] = episode;
    }
    // the last request's outputs into the bound output columns, as an asynchronous step leaves them
    if (stepped) {
#pragma unroll
      for (int a = 0; a < AMAX; ++a) {
        if (AMAX <= 4 || a < p.A) {
          const int64_t k = (int64_t)a * N + e;
          p.reward[k] = o[a].reward;
          if (p.renv) p.renv[k] = o[a].renv;
          if (p.shaping) p.shaping[k] = o[a].shaping;
          if constexpr (QRM) emit_qrm_to(o[a], a, e, L, p, p.qrm_s, p.qrm_sn, p.qrm_rq, p.qrm_done);
        }
      }
      if (p.env_done) p.env_done[e] = (uint8_t)done;
    }
    if (p.enc_state)
#pragma unroll
      for (int a = 0; a < AMAX; ++a)
        if (AMAX <= 4 || a < p.A) p.enc_state[(int64_t)a * N + e] = (s[a].y * p.W + s[a].x) * p.enc_nq[a] + s[a].q;
  }
  if (__any(bad_any) && (threadIdx.x & 63) == 0) atomicOr(p.err, 1u);
  wave_flush(p.slab, ls, __any(ls.episodes != 0));
}

template <int KIND, int AMAX, bool STOCH>
static void launch_resident_s(const KParams& p, const SyncIO& io, dim3 b, size_t lds, hipStream_t st) {
  if (io.out.qrm_s)
    hipLaunchKernelGGL((resident_kernel<KIND, AMAX, STOCH, true>), dim3(1), b, lds, st, p, io);
  else
    hipLaunchKernelGGL((resident_kernel<KIND, AMAX, STOCH, false>), dim3(1), b, lds, st, p, io);
}

template <int KIND, int AMAX>
static void launch_resident_a(const KParams& p, const SyncIO& io, dim3 b, size_t lds, hipStream_t st) {
  if (p.rng_on)
    launch_resident_s<KIND, AMAX, true>(p, io, b, lds, st);
  else
    launch_resident_s<KIND, AMAX, false>(p, io, b, lds, st);
}

template <int KIND>
static void launch_resident_k(const KParams& p, const SyncIO& io, dim3 b, size_t lds, hipStream_t st) {
  switch (amax_bucket(p.A)) {
    case 1: launch_resident_a<KIND, 1>(p, io, b, lds, st); break;
    case 2: launch_resident_a<KIND, 2>(p, io, b, lds, st); break;
    case 3: launch_resident_a<KIND, 3>(p, io, b, lds, st); break;
    case 4: launch_resident_a<KIND, 4>(p, io, b, lds, st); break;
    default: launch_resident_a<KIND, 8>(p, io, b, lds, st); break;
  }
}

hipError_t launch_resident(const KParams& p, const SyncIO& io, int kind, int threads, size_t lds, hipStream_t st) {
  const dim3 b((unsigned)((threads + 63) / 64 * 64));
  if (kind == RMX_FROZEN_LAKE)
    launch_resident_k<RMX_FROZEN_LAKE>(p, io, b, lds, st);
  else
    launch_resident_k<RMX_OFFICE_WORLD>(p, io, b, lds, st);
  return hipGetLastError();
}

}  // namespace rmx
