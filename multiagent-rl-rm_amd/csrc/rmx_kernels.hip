// rmx_kernels.hip — gfx950 step / rollout kernels of the grid-world + Reward-Machine engine.
//
// One thread owns one environment and runs its A agents in registers (agents of an env couple only
// through the shared timestep and the episode-end rule).  State is structure-of-
// arrays, agent-major (column[a*N + e]) so every load/store of a wave is one coalesced 256-B line.
// The static tables (per-cell can_move/hazard tile, per-agent cell->event map, dense RM
// next-state/reward/shaping tables) are staged once per workgroup into LDS with 16-B loads and
// looked up per lane.  Episode statistics are reduced per wave (ballot + shuffles) into a per-wave
// f64 slab owned by that wave: no atomics, deterministic, reduced once per report.
//
// Reference semantics restated (paths relative to Alee08/multiagent-rl-rm):
//   FrozenLake  ma_frozen_lake.py:96-154 (step), :174-187 (holes), :189-215 (terminations), :224-242 (move)
//   OfficeWorld ma_office.py:122-202 (step), :204-220 (plants), :240-257 (terminations),
//               :269-325 (move / wall collision), config_office.py:12-39 (can_move_*)
//   Wrapper     rm_environment_wrapper.py:43-107; RM step reward_machine.py:45-59
//   Loop rules  frozen_lake_main.py:345,368,375-376; office_main.py:1743-1749; success evaluation_metrics.py:248-267
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdint.h>

#include "rmx_device.h"
#include "rmx_generic.h"
#include "rmx_internal.h"

namespace rmx {

// ------------------------------------------------------------------------------------------------
// Single-step kernel: state round-trips HBM (the canonical drop-in for RMEnvironmentWrapper.step).
// ------------------------------------------------------------------------------------------------
// FEAT bits: 1 = per-env numpy PCG64 (stochastic slip and / or FrozenLake random starts), 2 = QRM
// counterfactual outputs, 4 = column words the step leaves unchanged are not stored (large N, as in the fast
// path; not combined with QRM).
// Compile-time, so the deterministic hot path carries neither the SeedSequence reseed nor the QRM stores.
template <int KIND, int AMAX, bool HASHED, int FEAT>
__global__ void __launch_bounds__(256) step_kernel(KParams p) {
  constexpr bool STOCH = (FEAT & 1) != 0;
  constexpr bool QRM = (FEAT & 2) != 0;
  constexpr bool SKIP = (FEAT & 4) != 0;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int64_t N = p.N;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = e < N;

  // 1) issue the state / action loads first so their latency overlaps the LDS staging
  AgentReg s[AMAX];
  int32_t act[AMAX];
  int32_t t = 0;
  if (live) {
    t = p.t[e];
#pragma unroll
    for (int a = 0; a < AMAX; ++a) {
      if (AMAX <= 4 || a < p.A) {
        const int64_t k = (int64_t)a * N + e;
        s[a].x = p.pos_x[k];
        s[a].y = p.pos_y[k];
        s[a].q = p.rm_q[k];
        s[a].f = p.flags[k];
        s[a].ret = p.ep_ret[k];
        act[a] = HASHED ? hash_action(p.seed, p.t_global, p.n_global, p.env_offset + e, p.A, a) : p.actions[k];
      }
    }
  }
  AgentReg s0[SKIP ? AMAX : 1];  // SKIP: the values as loaded
  if constexpr (SKIP) {
#pragma unroll
    for (int a = 0; a < AMAX; ++a) s0[a] = s[a];
  }
  const SlabSlot slot = slab_prefetch(p.slab);  // in flight with the state loads
#ifdef RMX_DIAG
  const int diag = p.diag;
  if (diag & 4) {  // copy-only: state straight back (traffic floor of this kernel's shape)
    if (live) {
      p.t[e] = t + 1;
      if (p.env_done) p.env_done[e] = (uint8_t)t;
#pragma unroll
      for (int a = 0; a < AMAX; ++a)
        if (AMAX <= 4 || a < p.A) {
          const int64_t k = (int64_t)a * N + e;
          p.pos_x[k] = s[a].x + act[a];
          p.pos_y[k] = s[a].y;
          p.rm_q[k] = s[a].q;
          p.flags[k] = s[a].f;
          p.ep_ret[k] = s[a].ret;
          p.reward[k] = 0.0f;
        }
    }
    return;
  }
  if (!(diag & 2)) {
    stage_tables(lds, p.tables, p.tables_n16);
    __syncthreads();
  }
  const Lds L = (diag & 2) ? lds_view(reinterpret_cast<const unsigned char*>(p.tables), p) : lds_view(lds, p);
#else
  stage_tables(lds, p.tables, p.tables_n16);
  __syncthreads();
  const Lds L = lds_view(lds, p);
#endif

  LaneStats ls = {0.0, 0, 0, 0};
  bool done = false;
  uint32_t bad = 0;
  AgentOut o[AMAX];
  if (live) {
    Pcg rng = {0, 0, 0, 0};
    if constexpr (STOCH) rng = {p.rng[e], p.rng[N + e], p.rng[2 * N + e], p.rng[3 * N + e]};
    if (p.autoreset && (s[0].f & RMX_F_ENV_DONE)) {
      reset_regs<AMAX>(s, t, p);
      if constexpr (STOCH) {  // env.rng = default_rng(seed of the next episode)
        const int32_t k = p.episode[e] + 1;
        p.episode[e] = k;
#ifdef RMX_DIAG
        if (!(p.diag & 16384))  // timing ablation: no reseed
#endif
        rng = seed_pcg64(seed_of(p, p.env_offset + e, k));
        if (p.random_starts) random_starts<AMAX>(p, rng, e, s);  // before any slip draw of the episode
      }
    }
    const float disc = p.gamma_is_one ? 1.0f : p.disc[min((uint32_t)t, (uint32_t)p.max_t + 1u)];
    done = env_step<KIND, AMAX>(s, t, act, L, p, disc, o, ls, &bad, STOCH ? &rng : nullptr);
    if constexpr (STOCH) {
      p.rng[e] = rng.hi;
      p.rng[N + e] = rng.lo;
      p.rng[2 * N + e] = rng.ihi;
      p.rng[3 * N + e] = rng.ilo;
    }
    p.t[e] = t;
    if (p.env_done) p.env_done[e] = (uint8_t)done;
#pragma unroll
    for (int a = 0; a < AMAX; ++a) {
      if (AMAX <= 4 || a < p.A) {
        const int64_t k = (int64_t)a * N + e;
        const AgentReg& o0 = s0[SKIP ? a : 0];
        if (!SKIP || s[a].x != o0.x) p.pos_x[k] = s[a].x;
        if (!SKIP || s[a].y != o0.y) p.pos_y[k] = s[a].y;
        if (!SKIP || s[a].q != o0.q) p.rm_q[k] = s[a].q;
        if (!SKIP || s[a].f != o0.f) p.flags[k] = s[a].f;
        if (!SKIP || __float_as_int(s[a].ret) != __float_as_int(o0.ret)) p.ep_ret[k] = s[a].ret;
        p.reward[k] = o[a].reward;
        if (p.shaping) p.shaping[k] = o[a].shaping;
        if (p.renv) p.renv[k] = o[a].renv;
        if (p.enc_state) p.enc_state[k] = (s[a].y * p.W + s[a].x) * p.enc_nq[a] + s[a].q;
        if constexpr (QRM) emit_qrm(o[a], a, e, L, p);
      }
    }
  }
  if (__any(bad)) {
    if ((threadIdx.x & 63) == 0) atomicOr(p.err, 1u);
  }
#ifdef RMX_DIAG
  if (diag & 1) return;  // no statistics flush
#endif
  wave_flush_slot(p.slab, slot, ls, __any(done));
}

// ------------------------------------------------------------------------------------------------
// Fused rollout: T autoreset steps with hashed actions, state in VGPRs, tables in LDS once.
// ------------------------------------------------------------------------------------------------
template <int KIND, int AMAX, bool STOCH>
__global__ void __launch_bounds__(256) rollout_kernel(KParams p, int32_t T, float* __restrict__ trace) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int64_t N = p.N;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = e < N;
  AgentReg s[AMAX];
  int32_t t = 0;
  if (live) {
    t = p.t[e];
#pragma unroll
    for (int a = 0; a < AMAX; ++a) {
      if (AMAX <= 4 || a < p.A) {
        const int64_t k = (int64_t)a * N + e;
        s[a].x = p.pos_x[k];
        s[a].y = p.pos_y[k];
        s[a].q = p.rm_q[k];
        s[a].f = p.flags[k];
        s[a].ret = p.ep_ret[k];
      }
    }
  }
  stage_tables(lds, p.tables, p.tables_n16);
  __syncthreads();
  const Lds L = lds_view(lds, p);
  LaneStats ls = {0.0, 0, 0, 0};
  uint32_t bad = 0;
  AgentOut o[AMAX];
  bool done = false;
  const int64_t eg = p.env_offset + e;
  Pcg rng = {0, 0, 0, 0};
  int32_t episode = 0;
  if constexpr (STOCH) {
    if (live) {
      rng = {p.rng[e], p.rng[N + e], p.rng[2 * N + e], p.rng[3 * N + e]};
      episode = p.episode[e];
    }
  }
  for (int32_t it = 0; it < T; ++it) {
    if (live) {
      int32_t act[AMAX];
#pragma unroll
      for (int a = 0; a < AMAX; ++a)
        if (AMAX <= 4 || a < p.A) act[a] = hash_action(p.seed, p.t_global + it, p.n_global, eg, p.A, a);
      if (s[0].f & RMX_F_ENV_DONE) {
        reset_regs<AMAX>(s, t, p);
        if constexpr (STOCH) {
          rng = seed_pcg64(seed_of(p, eg, ++episode));
          if (p.random_starts) random_starts<AMAX>(p, rng, e, s);
        }
      }
      const float disc = p.gamma_is_one ? 1.0f : p.disc[min((uint32_t)t, (uint32_t)p.max_t + 1u)];
      done = env_step<KIND, AMAX>(s, t, act, L, p, disc, o, ls, &bad, STOCH ? &rng : nullptr);
      if (trace) {
#pragma unroll
        for (int a = 0; a < AMAX; ++a)
          if (AMAX <= 4 || a < p.A) trace[((int64_t)it * p.A + a) * N + e] = o[a].reward;
      }
    }
  }
  if (live) {
    p.t[e] = t;
    if (p.env_done) p.env_done[e] = (uint8_t)done;
    if constexpr (STOCH) {
      p.rng[e] = rng.hi;
      p.rng[N + e] = rng.lo;
      p.rng[2 * N + e] = rng.ihi;
      p.rng[3 * N + e] = rng.ilo;
      p.episode[e] = episode;
    }
#pragma unroll
    for (int a = 0; a < AMAX; ++a) {
      if (AMAX <= 4 || a < p.A) {
        const int64_t k = (int64_t)a * N + e;
        p.pos_x[k] = s[a].x;
        p.pos_y[k] = s[a].y;
        p.rm_q[k] = s[a].q;
        p.flags[k] = s[a].f;
        p.ep_ret[k] = s[a].ret;
        p.reward[k] = o[a].reward;
        if (p.shaping) p.shaping[k] = o[a].shaping;
        if (p.renv) p.renv[k] = o[a].renv;
        if (p.enc_state) p.enc_state[k] = (s[a].y * p.W + s[a].x) * p.enc_nq[a] + s[a].q;
      }
    }
  }
  if (__any(bad)) {
    if ((threadIdx.x & 63) == 0) atomicOr(p.err, 1u);
  }
  wave_flush(p.slab, ls, __any(ls.episodes != 0));
}

// ------------------------------------------------------------------------------------------------
// Lane-per-agent layout: G lanes (power of two >= A) own one env, lane a runs agent a.  The env-level
// AND over agents (episode end) is a G-lane butterfly of shuffles; a wave covers 64/G envs and every
// load is still two-to-four fully used 128-B lines.  2-4x the waves of thread-per-env at the same
// byte count, and one agent's dependency chain per lane.
// ------------------------------------------------------------------------------------------------
template <int G>
__device__ __forceinline__ bool group_and(bool v) {
#pragma unroll
  for (int o = 1; o < G; o <<= 1) {
    const int other = __shfl_xor((int)v, o, 64);  // every lane must execute the shuffle (no short-circuit)
    v = v & (other != 0);
  }
  return v;
}

template <int KIND, int G, bool HASHED>
__global__ void __launch_bounds__(256) step_kernel_lpe(KParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int64_t N = p.N;
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t e = gid / G;
  const int a = (int)(gid & (G - 1));
  const bool env_ok = e < N;
  const bool live = env_ok && a < p.A;
  const int64_t k = (int64_t)a * N + e;

  AgentReg s = {0, 0, 0, 0u, 0.0f};
  int32_t act = RMX_WAIT, t = 0;
  if (live) {
    t = p.t[e];
    s.x = p.pos_x[k];
    s.y = p.pos_y[k];
    s.q = p.rm_q[k];
    s.f = p.flags[k];
    s.ret = p.ep_ret[k];
    act = HASHED ? hash_action(p.seed, p.t_global, p.n_global, p.env_offset + e, p.A, a) : p.actions[k];
  }
  stage_tables(lds, p.tables, p.tables_n16);
  __syncthreads();
  const Lds L = lds_view(lds, p);

  uint32_t bad = 0;
  AgentOut o = {0.0f, 0.0f, 0.0f, true, true, false, 0u, 0u, 0u};
  if (live) {
    if (p.autoreset && (s.f & RMX_F_ENV_DONE)) {  // every agent of a finished env carries the bit
      t = 0;
      s.x = p.start_x[a];
      s.y = p.start_y[a];
      s.q = p.init_q[a];
      s.f = RMX_F_ACTIVE;
      s.ret = 0.0f;
    }
    o = agent_step<KIND>(s, act, a, t + 1, L, p, &bad);
    const float disc = p.gamma_is_one ? 1.0f : p.disc[min((uint32_t)t, (uint32_t)p.max_t + 1u)];
    s.ret = fmaf(disc, o.reward, s.ret);
  }
  const bool all_term = group_and<G>(o.term);
  const bool all_trunc = group_and<G>(o.trunc);
  const bool done = env_ok && (all_term || all_trunc);
  LaneStats ls = {0.0, 0, 0, 0};
  if (live) {
    if (done) {
      s.f |= RMX_F_ENV_DONE;
      ls.ret = (double)s.ret;
      ls.successes = (o.term && s.q == p.final_q[a] && s.ret > 0.0f) ? 1 : 0;
    }
    p.pos_x[k] = s.x;
    p.pos_y[k] = s.y;
    p.rm_q[k] = s.q;
    p.flags[k] = s.f;
    p.ep_ret[k] = s.ret;
    p.reward[k] = o.reward;
    if (p.shaping) p.shaping[k] = o.shaping;
    if (p.renv) p.renv[k] = o.renv;
    if (p.enc_state) p.enc_state[k] = (s.y * p.W + s.x) * p.enc_nq[a] + s.q;
    if (p.qrm_s) emit_qrm(o, a, e, L, p);
    if (a == 0) {
      p.t[e] = t + 1;
      if (p.env_done) p.env_done[e] = (uint8_t)done;
      if (done) {
        ls.episodes = 1;
        ls.length = t + 1;
      }
    }
  }
  if (__any(bad)) {
    if ((threadIdx.x & 63) == 0) atomicOr(p.err, 1u);
  }
  wave_flush(p.slab, ls, __any(done));
}

template <int KIND, int G>
__global__ void __launch_bounds__(256) rollout_kernel_lpe(KParams p, int32_t T, float* __restrict__ trace) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int64_t N = p.N;
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t e = gid / G;
  const int a = (int)(gid & (G - 1));
  const bool env_ok = e < N;
  const bool live = env_ok && a < p.A;
  const int64_t k = (int64_t)a * N + e;
  AgentReg s = {0, 0, 0, 0u, 0.0f};
  int32_t t = 0;
  if (live) {
    t = p.t[e];
    s.x = p.pos_x[k];
    s.y = p.pos_y[k];
    s.q = p.rm_q[k];
    s.f = p.flags[k];
    s.ret = p.ep_ret[k];
  }
  stage_tables(lds, p.tables, p.tables_n16);
  __syncthreads();
  const Lds L = lds_view(lds, p);
  LaneStats ls = {0.0, 0, 0, 0};
  uint32_t bad = 0;
  AgentOut o = {0.0f, 0.0f, 0.0f, true, true, false, 0u, 0u, 0u};
  bool done = false;
  const int64_t eg = p.env_offset + e;
  for (int32_t it = 0; it < T; ++it) {
    if (live) {
      const int32_t act = hash_action(p.seed, p.t_global + it, p.n_global, eg, p.A, a);
      if (s.f & RMX_F_ENV_DONE) {
        t = 0;
        s.x = p.start_x[a];
        s.y = p.start_y[a];
        s.q = p.init_q[a];
        s.f = RMX_F_ACTIVE;
        s.ret = 0.0f;
      }
      o = agent_step<KIND>(s, act, a, t + 1, L, p, &bad);
      const float disc = p.gamma_is_one ? 1.0f : p.disc[min((uint32_t)t, (uint32_t)p.max_t + 1u)];
      s.ret = fmaf(disc, o.reward, s.ret);
      t += 1;
      if (trace) trace[((int64_t)it * p.A + a) * N + e] = o.reward;
    }
    const bool all_term = group_and<G>(o.term);
    const bool all_trunc = group_and<G>(o.trunc);
    done = env_ok && (all_term || all_trunc);
    if (live && done) {
      s.f |= RMX_F_ENV_DONE;
      ls.ret += (double)s.ret;
      ls.successes += (o.term && s.q == p.final_q[a] && s.ret > 0.0f) ? 1 : 0;
      if (a == 0) {
        ls.episodes += 1;
        ls.length += t;
      }
    }
  }
  if (live) {
    p.pos_x[k] = s.x;
    p.pos_y[k] = s.y;
    p.rm_q[k] = s.q;
    p.flags[k] = s.f;
    p.ep_ret[k] = s.ret;
    p.reward[k] = o.reward;
    if (p.shaping) p.shaping[k] = o.shaping;
    if (p.renv) p.renv[k] = o.renv;
    if (p.enc_state) p.enc_state[k] = (s.y * p.W + s.x) * p.enc_nq[a] + s.q;
    if (a == 0) {
      p.t[e] = t;
      if (p.env_done) p.env_done[e] = (uint8_t)done;
    }
  }
  if (__any(bad)) {
    if ((threadIdx.x & 63) == 0) atomicOr(p.err, 1u);
  }
  wave_flush(p.slab, ls, __any(ls.episodes != 0 || ls.successes != 0 || ls.ret != 0.0));
}

// ------------------------------------------------------------------------------------------------
// Model construction: RMEnvironmentWrapper.get_mdp (rm_environment_wrapper.py:185-283).  One thread per
// (encoded state, action) of one agent: decode (x, y, q) with the agent's encoder stride, apply the
// terminal self-loop rule (is_terminal_state_mdp), else run the same agent_step from timestep 0.
// done = 255 marks "no entry" (the reference's FrozenLake decode quirk, kept unless fix_fl).
// ------------------------------------------------------------------------------------------------
template <int KIND>
__global__ void __launch_bounds__(256) mdp_kernel(KParams p, int ag, int fix_fl, int64_t S, int32_t* __restrict__ next,
                                                 float* __restrict__ reward, uint8_t* __restrict__ done) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  stage_tables(lds, p.tables, p.tables_n16);
  __syncthreads();
  const Lds L = lds_view(lds, p);
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= S * 4) return;
  const int64_t s = i >> 2;
  const int a = (int)(i & 3);
  const int32_t nQ = p.enc_nq[ag];
  const int32_t q = (int32_t)(s % nQ), pos = (int32_t)(s / nQ);
  const bool hz = (L.cell[pos] & RMX_CELL_HAZARD) != 0;
  bool term_state = false;
  float term_r = 0.0f;
  if (KIND == RMX_FROZEN_LAKE) {
    if (hz) {
      term_state = true;
      term_r = p.hazard_penalty;
    } else if (fix_fl && q == p.final_q[ag]) {
      term_state = true;
    } else if (!fix_fl) {
      next[i] = -1;
      reward[i] = 0.0f;
      done[i] = 255;
      return;
    }
  } else {
    if (hz && p.hazard_fail) {
      term_state = true;
      term_r = p.hazard_penalty;
    } else if (q == p.final_q[ag]) {
      term_state = true;
    }
  }
  if (term_state) {
    next[i] = (int32_t)s;
    reward[i] = term_r;
    done[i] = 1;
    return;
  }
  AgentReg st = {pos % p.W, pos / p.W, q, RMX_F_ACTIVE, 0.0f};
  uint32_t bad = 0;
  const AgentOut o = agent_step<KIND>(st, a, ag, 1, L, p, &bad);
  next[i] = (int32_t)o.cell * nQ + st.q;
  reward[i] = o.reward;
  done[i] = (uint8_t)(o.term || o.trunc);
}

// ------------------------------------------------------------------------------------------------
// Reset (optionally masked), action fill, stats reduction.
// ------------------------------------------------------------------------------------------------
// write_state = 0: the reset cache only.  With the cache (kRngFixedSeed: seed_episode_stride == 0) every env's
// entry is rebuilt whatever the mask says: the base seed is the handle's, so the next autoreset of an env outside the
// mask starts from the new seed's shuffle too.
__global__ void reset_kernel(KParams p, const uint8_t* __restrict__ mask, int write_state) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= p.N) return;
  const bool cache = p.rs_cells != nullptr;
  const bool state = write_state && !(mask && !mask[e]);
  if (!state && !cache) return;
  AgentReg s[RMX_MAX_AGENTS];
  for (int a = 0; a < p.A; ++a) {
    s[a].x = p.start_x[a];
    s[a].y = p.start_y[a];
  }
  Pcg r = {0ull, 0ull, 0ull, 0ull};
  if (p.rng_on) {  // env.reset: self.rng = default_rng(seed), episode k = 0 of the schedule
    r = seed_pcg64(seed_of(p, p.env_offset + e, 0));
    if (p.random_starts) random_starts<RMX_MAX_AGENTS>(p, r, e, s);  // _sample_start_positions(rng)
  }
  if (cache) {  // A <= 4 (host): cells x | y << 8, two agents per word; then the post-shuffle generator
    for (int w = 0; w < (p.A + 1) / 2; ++w) {
      const uint32_t lo = (uint32_t)s[2 * w].x | ((uint32_t)s[2 * w].y << 8);
      const uint32_t hi = 2 * w + 1 < p.A ? ((uint32_t)s[2 * w + 1].x | ((uint32_t)s[2 * w + 1].y << 8)) : 0u;
      p.rs_cells[(int64_t)w * p.N + e] = lo | (hi << 16);
    }
    p.rs_rng[e] = r.hi;
    p.rs_rng[p.N + e] = r.lo;
    p.rs_rng[2 * p.N + e] = r.ihi;
    p.rs_rng[3 * p.N + e] = r.ilo;
  }
  if (!state) return;
  p.t[e] = 0;
  if (p.rng_on) {
    p.rng[e] = r.hi;
    p.rng[p.N + e] = r.lo;
    p.rng[2 * p.N + e] = r.ihi;
    p.rng[3 * p.N + e] = r.ilo;
    p.episode[e] = 0;
  }
  for (int a = 0; a < p.A; ++a) {
    const int64_t k = (int64_t)a * p.N + e;
    p.pos_x[k] = s[a].x;
    p.pos_y[k] = s[a].y;
    p.rm_q[k] = p.init_q[a];
    p.flags[k] = RMX_F_ACTIVE;
    p.ep_ret[k] = 0.0f;
  }
}

__global__ void fill_actions_kernel(uint64_t seed, int64_t t0, int32_t T, int64_t n_global, int64_t env_offset,
                                    int64_t N, int A, int32_t* __restrict__ out) {
  const int64_t total = (int64_t)T * A * N;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = i % N;
    const int64_t r = i / N;
    const int a = (int)(r % A);
    const int64_t s = r / A;
    out[i] = hash_action(seed, t0 + s, n_global, env_offset + e, A, a);
  }
}

// Sums of one 256-thread block in a fixed order: a DPP wave sum per statistic (rmx_device.h), then wave 0's
// thread 0 adds the four wave sums in wave order.  The returned vector is valid in thread 0 only.
__device__ __forceinline__ void block_sum(double (&wsum)[4][RMX_NSTATS], double (&acc)[RMX_NSTATS]) {
  const int wave = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < RMX_NSTATS; ++k) acc[k] = wave_sum_f64(acc[k]);
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int k = 0; k < RMX_NSTATS; ++k) wsum[wave][k] = acc[k];
  __syncthreads();
  if (threadIdx.x == 0)
#pragma unroll
    for (int k = 0; k < RMX_NSTATS; ++k) acc[k] = ((wsum[0][k] + wsum[1][k]) + wsum[2][k]) + wsum[3][k];
}

// The whole statistics report in ONE launch; inside a short timed window it is pure latency (load round
// trip, block sum, ticket round trip, partial round trip), so every step of that chain is kept short.
// Pass 1: one partial vector per block — blocks [0, n_slab_blocks) own contiguous ranges of the per-wave slab,
// the rest own contiguous env ranges of the fast path's per-env slots (es_ret == NULL: none; one row [N]: the
// step kernels sum an env's agents before its one adder), each thread a few envs with their loads in flight at once.  Integer counts
// are carried as doubles (exact below 2^53).  Pass 2: the block that takes the last ticket sums the partial
// vectors in block order and re-arms the ticket.  The partition depends only on (n_waves, N) and every sum has
// a fixed association order, so repeated reports agree bit for bit.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__) && !defined(__gfx942__)
#error "rmx_kernels.hip: stats_kernel's relaxed ticket relies on gfx94x / gfx950 store completion in vmcnt"
#endif
// Cross-XCD visibility: partials are written and read with agent-scope atomic stores / loads (the compiler's
// L2-coherent forms), and each block waits for its partial stores to complete before it takes its ticket.
// Those three accesses are the only data the two passes share, so no L2 writeback / invalidate is needed
// around the ticket: an acq_rel ticket (L2 writeback + invalidate in every block) cost 3.5 us per report.
__global__ void __launch_bounds__(256) stats_kernel(const double* __restrict__ slab, int64_t n_waves,
                                                    int n_slab_blocks, const double* __restrict__ es_ret,
                                                    const unsigned long long* __restrict__ es_cnt,
                                                    const uint32_t* __restrict__ es_succ, int64_t N,
                                                    double* __restrict__ partial, unsigned int* __restrict__ ticket,
                                                    double* __restrict__ out) {
  __shared__ double wsum[4][RMX_NSTATS];
  __shared__ int last;
  double acc[RMX_NSTATS] = {0, 0, 0, 0};
  if ((int)blockIdx.x < n_slab_blocks) {
    const int64_t chunk = (n_waves + n_slab_blocks - 1) / n_slab_blocks;
    const int64_t lo = blockIdx.x * chunk, hi = lo + chunk < n_waves ? lo + chunk : n_waves;
#pragma unroll 4
    for (int64_t w = lo + threadIdx.x; w < hi; w += 256)
#pragma unroll
      for (int k = 0; k < RMX_NSTATS; ++k) acc[k] += slab[w * RMX_NSTATS + k];
  } else {
    const int nb = (int)gridDim.x - n_slab_blocks;
    const int64_t chunk = (N + nb - 1) / nb;
    const int64_t lo = (blockIdx.x - n_slab_blocks) * chunk, hi = lo + chunk < N ? lo + chunk : N;
    uint64_t len = 0, eps = 0, succ = 0;
#pragma unroll 4
    for (int64_t e = lo + threadIdx.x; e < hi; e += 256) {
      const unsigned long long c = es_cnt[e];
      len += c & ((1ull << 40) - 1);
      eps += c >> 40;
      acc[RMX_STAT_SUM_RETURN] += es_ret[e];
      succ += es_succ[e];
    }
    acc[RMX_STAT_EPISODES] = (double)eps;
    acc[RMX_STAT_SUCCESSES] = (double)succ;
    acc[RMX_STAT_SUM_LENGTH] = (double)len;
  }
  block_sum(wsum, acc);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < RMX_NSTATS; ++k)
      __hip_atomic_store(partial + blockIdx.x * RMX_NSTATS + k, acc[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_waitcnt(0);  // the partial stores have completed (gfx9: stores count in vmcnt)
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    const unsigned int prev = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = prev == gridDim.x - 1u;
  }
  __syncthreads();  // also orders thread 0's reads of wsum[] before the second block sum overwrites it
  if (!last) return;
  double acc2[RMX_NSTATS] = {0, 0, 0, 0};
  for (int i = threadIdx.x; i < (int)gridDim.x; i += 256)
#pragma unroll
    for (int k = 0; k < RMX_NSTATS; ++k)
      acc2[k] += __hip_atomic_load(partial + i * RMX_NSTATS + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  block_sum(wsum, acc2);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < RMX_NSTATS; ++k) out[k] = acc2[k];
    __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-armed for the next report
  }
}

// ------------------------------------------------------------------------------------------------
// Host-side launchers (called from rmx_capi.cpp)
// ------------------------------------------------------------------------------------------------
template <int KIND, int AMAX, int FEAT>
static void launch_step_f(const KParams& p, int hashed, dim3 g, dim3 b, size_t lds, hipStream_t st) {
  if (hashed)
    hipLaunchKernelGGL((step_kernel<KIND, AMAX, true, FEAT>), g, b, lds, st, p);
  else
    hipLaunchKernelGGL((step_kernel<KIND, AMAX, false, FEAT>), g, b, lds, st, p);
}

template <int KIND, int AMAX>
static hipError_t launch_step_t(const KParams& p, int hashed, dim3 g, dim3 b, size_t lds, hipStream_t st) {
  const int feat = (p.rng_on ? 1 : 0) | (p.qrm_s ? 2 : (p.skip_same ? 4 : 0));
  switch (feat) {
    case 0: launch_step_f<KIND, AMAX, 0>(p, hashed, g, b, lds, st); break;
    case 1: launch_step_f<KIND, AMAX, 1>(p, hashed, g, b, lds, st); break;
    case 2: launch_step_f<KIND, AMAX, 2>(p, hashed, g, b, lds, st); break;
    case 3: launch_step_f<KIND, AMAX, 3>(p, hashed, g, b, lds, st); break;
    case 4: launch_step_f<KIND, AMAX, 4>(p, hashed, g, b, lds, st); break;
    default: launch_step_f<KIND, AMAX, 5>(p, hashed, g, b, lds, st); break;
  }
  return hipGetLastError();
}

template <int KIND>
static hipError_t launch_step_k(const KParams& p, int hashed, dim3 g, dim3 b, size_t lds, hipStream_t st) {
  switch (amax_bucket(p.A)) {
    case 1: return launch_step_t<KIND, 1>(p, hashed, g, b, lds, st);
    case 2: return launch_step_t<KIND, 2>(p, hashed, g, b, lds, st);
    case 3: return launch_step_t<KIND, 3>(p, hashed, g, b, lds, st);
    case 4: return launch_step_t<KIND, 4>(p, hashed, g, b, lds, st);
    default: return launch_step_t<KIND, 8>(p, hashed, g, b, lds, st);
  }
}

template <int KIND, int G>
static hipError_t launch_step_lpe_t(const KParams& p, int hashed, dim3 g, dim3 b, size_t lds, hipStream_t st) {
  if (hashed)
    hipLaunchKernelGGL((step_kernel_lpe<KIND, G, true>), g, b, lds, st, p);
  else
    hipLaunchKernelGGL((step_kernel_lpe<KIND, G, false>), g, b, lds, st, p);
  return hipGetLastError();
}

template <int KIND>
static hipError_t launch_step_lpe_k(const KParams& p, int hashed, dim3 g, dim3 b, size_t lds, hipStream_t st) {
  switch (lanes_per_env(p.A)) {
    case 1: return launch_step_lpe_t<KIND, 1>(p, hashed, g, b, lds, st);
    case 2: return launch_step_lpe_t<KIND, 2>(p, hashed, g, b, lds, st);
    case 4: return launch_step_lpe_t<KIND, 4>(p, hashed, g, b, lds, st);
    default: return launch_step_lpe_t<KIND, 8>(p, hashed, g, b, lds, st);
  }
}

hipError_t launch_step(const KParams& p, int hashed, int kind, int layout, dim3 g, dim3 b, size_t lds,
                       hipStream_t st) {
  if (layout == kLayoutLanePerAgent)
    return kind == RMX_FROZEN_LAKE ? launch_step_lpe_k<RMX_FROZEN_LAKE>(p, hashed, g, b, lds, st)
                                   : launch_step_lpe_k<RMX_OFFICE_WORLD>(p, hashed, g, b, lds, st);
  return kind == RMX_FROZEN_LAKE ? launch_step_k<RMX_FROZEN_LAKE>(p, hashed, g, b, lds, st)
                                 : launch_step_k<RMX_OFFICE_WORLD>(p, hashed, g, b, lds, st);
}

template <int KIND>
static hipError_t launch_rollout_k(const KParams& p, int32_t T, float* trace, dim3 g, dim3 b, size_t lds,
                                   hipStream_t st) {
  if (p.rng_on) {
    switch (amax_bucket(p.A)) {
      case 1: hipLaunchKernelGGL((rollout_kernel<KIND, 1, true>), g, b, lds, st, p, T, trace); break;
      case 2: hipLaunchKernelGGL((rollout_kernel<KIND, 2, true>), g, b, lds, st, p, T, trace); break;
      case 3: hipLaunchKernelGGL((rollout_kernel<KIND, 3, true>), g, b, lds, st, p, T, trace); break;
      case 4: hipLaunchKernelGGL((rollout_kernel<KIND, 4, true>), g, b, lds, st, p, T, trace); break;
      default: hipLaunchKernelGGL((rollout_kernel<KIND, 8, true>), g, b, lds, st, p, T, trace); break;
    }
  } else {
    switch (amax_bucket(p.A)) {
      case 1: hipLaunchKernelGGL((rollout_kernel<KIND, 1, false>), g, b, lds, st, p, T, trace); break;
      case 2: hipLaunchKernelGGL((rollout_kernel<KIND, 2, false>), g, b, lds, st, p, T, trace); break;
      case 3: hipLaunchKernelGGL((rollout_kernel<KIND, 3, false>), g, b, lds, st, p, T, trace); break;
      case 4: hipLaunchKernelGGL((rollout_kernel<KIND, 4, false>), g, b, lds, st, p, T, trace); break;
      default: hipLaunchKernelGGL((rollout_kernel<KIND, 8, false>), g, b, lds, st, p, T, trace); break;
    }
  }
  return hipGetLastError();
}

template <int KIND>
static hipError_t launch_rollout_lpe_k(const KParams& p, int32_t T, float* trace, dim3 g, dim3 b, size_t lds,
                                       hipStream_t st) {
  switch (lanes_per_env(p.A)) {
    case 1: hipLaunchKernelGGL((rollout_kernel_lpe<KIND, 1>), g, b, lds, st, p, T, trace); break;
    case 2: hipLaunchKernelGGL((rollout_kernel_lpe<KIND, 2>), g, b, lds, st, p, T, trace); break;
    case 4: hipLaunchKernelGGL((rollout_kernel_lpe<KIND, 4>), g, b, lds, st, p, T, trace); break;
    default: hipLaunchKernelGGL((rollout_kernel_lpe<KIND, 8>), g, b, lds, st, p, T, trace); break;
  }
  return hipGetLastError();
}

hipError_t launch_rollout(const KParams& p, int kind, int layout, int32_t T, float* trace, dim3 g, dim3 b,
                          size_t lds, hipStream_t st) {
  if (layout == kLayoutLanePerAgent)
    return kind == RMX_FROZEN_LAKE ? launch_rollout_lpe_k<RMX_FROZEN_LAKE>(p, T, trace, g, b, lds, st)
                                   : launch_rollout_lpe_k<RMX_OFFICE_WORLD>(p, T, trace, g, b, lds, st);
  return kind == RMX_FROZEN_LAKE ? launch_rollout_k<RMX_FROZEN_LAKE>(p, T, trace, g, b, lds, st)
                                 : launch_rollout_k<RMX_OFFICE_WORLD>(p, T, trace, g, b, lds, st);
}

hipError_t launch_reset(const KParams& p, const uint8_t* mask, int write_state, hipStream_t st) {
  const int blk = 256;
  const unsigned grid = (unsigned)((p.N + blk - 1) / blk);
  hipLaunchKernelGGL(reset_kernel, dim3(grid), dim3(blk), 0, st, p, mask, write_state);
  return hipGetLastError();
}

hipError_t launch_fill_actions(uint64_t seed, int64_t t0, int32_t T, int64_t n_global, int64_t env_offset, int64_t N,
                               int A, int32_t* out, hipStream_t st) {
  const int64_t total = (int64_t)T * A * N;
  int64_t grid = (total + 255) / 256;
  if (grid > 65536) grid = 65536;
  if (grid < 1) grid = 1;
  hipLaunchKernelGGL(fill_actions_kernel, dim3((unsigned)grid), dim3(256), 0, st, seed, t0, T, n_global, env_offset,
                     N, A, out);
  return hipGetLastError();
}

hipError_t launch_mdp(const KParams& p, int kind, int ag, int fix_fl, int64_t S, int32_t* next, float* reward,
                      uint8_t* done, size_t lds, hipStream_t st) {
  const unsigned grid = (unsigned)((S * 4 + 255) / 256);
  if (kind == RMX_FROZEN_LAKE)
    hipLaunchKernelGGL((mdp_kernel<RMX_FROZEN_LAKE>), dim3(grid), dim3(256), lds, st, p, ag, fix_fl, S, next, reward, done);
  else
    hipLaunchKernelGGL((mdp_kernel<RMX_OFFICE_WORLD>), dim3(grid), dim3(256), lds, st, p, ag, fix_fl, S, next, reward,
                       done);
  return hipGetLastError();
}

hipError_t launch_stats_reduce(const double* slab, int64_t n_waves, const double* es_ret, const unsigned long long* es_cnt,
                               const uint32_t* es_succ, int64_t N, double* partial, unsigned int* ticket,
                               double* out, hipStream_t st) {
  // one launch over both homes, ~1 slab slot / ~4 envs per thread, at most kStatsPartials blocks per home; the
  // last block to finish reduces the partials.  The pass is latency-bound: 4 envs per thread (64 blocks at
  // 65,536 envs) beat 1, 2, 8 and 16 by 0.5-3.5 us per report (profiles/r02_ab_log.md, stats)
  const int p_slab = (int)std::min<int64_t>(kStatsPartials, std::max<int64_t>(1, (n_waves + 255) / 256));
  constexpr int64_t per = 256 * kStatsEnvsPerThread;
  const int p_env = es_ret ? (int)std::min<int64_t>(kStatsPartials, std::max<int64_t>(1, (N + per - 1) / per)) : 0;
  hipLaunchKernelGGL(stats_kernel, dim3(p_slab + p_env), dim3(256), 0, st, slab, n_waves, p_slab, es_ret, es_cnt,
                     es_succ, N, partial, ticket, out);
  return hipGetLastError();
}

}  // namespace rmx
