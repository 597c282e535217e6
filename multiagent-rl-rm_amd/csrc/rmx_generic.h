// rmx_generic.h — the generic step logic shared by the generic kernels (rmx_kernels.hip) and the resident
// host-boundary stepper (rmx_sync.hip): LDS table view, one agent-step, one env-step, QRM counterfactuals,
// autoreset and FrozenLake random starts.  Reference semantics are cited in rmx_kernels.hip's header.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rmx_device.h"
#include "rmx_internal.h"

namespace rmx {

// Stage the table blob (16-B granules) into LDS; every thread of the block participates.
__device__ __forceinline__ void stage_tables(unsigned char* lds, const uint4* __restrict__ src, int n16) {
  uint4* dst = reinterpret_cast<uint4*>(lds);
  for (int i = threadIdx.x; i < n16; i += blockDim.x) dst[i] = src[i];
}

struct Lds {
  const uint16_t* cell;
  const uint8_t* ev;
  const uint8_t* nq;
  const float* rr;
  const float* sh;
  const uint8_t* qrm;  // [A][Qx] get_all_states()[:-1] order
};

__device__ __forceinline__ Lds lds_view(const unsigned char* lds, const KParams& p) {
  Lds v;
  v.cell = reinterpret_cast<const uint16_t*>(lds + p.off_cell);
  v.ev = lds + p.off_ev;
  v.nq = lds + p.off_nq;
  v.rr = reinterpret_cast<const float*>(lds + p.off_rr);
  v.sh = reinterpret_cast<const float*>(lds + p.off_sh);
  v.qrm = lds + p.off_qrm;
  return v;
}

// Per-agent state held in registers.
struct AgentReg {
  int32_t x, y, q;
  uint32_t f;
  float ret;
};

// Outcome of one agent-step (for the env-level rule and the outputs).
struct AgentOut {
  float reward, shaping, renv;
  bool term, trunc;
  bool env_term;
  uint32_t prev_cell, cell, ev;  // for the QRM counterfactuals
};

// One wrapper step for one agent.  t1 = timestep after the env increment.
template <int KIND>
__device__ __forceinline__ AgentOut agent_step(AgentReg& s, int32_t act, int a, int32_t t1, const Lds& L,
                                               const KParams& p, uint32_t* bad, Pcg* rng = nullptr) {
  const int32_t fq = p.final_q[a];
  bool active = s.f & RMX_F_ACTIVE;
  bool fail = s.f & RMX_F_FAIL;
  uint32_t steps = s.f >> RMX_F_STEPS_SHIFT;
  if ((uint32_t)act > (uint32_t)RMX_WAIT) {  // invalid action: recorded, treated as wait
    *bad = 1u;
    act = RMX_WAIT;
  }
  float renv = 0.0f;
  bool env_term, trunc;
  const uint32_t prev_cell = (uint32_t)(s.y * p.W + s.x);
  // move deltas in the kind's convention: FL up = y-1, OW up = y+1
  const int32_t up = (KIND == RMX_FROZEN_LAKE) ? -1 : 1;
  if (KIND == RMX_FROZEN_LAKE) {
    if (active && s.q != fq) {  // inactive or RM already final (pre-step) -> frozen, Renv = 0
      uint32_t c = (uint32_t)(s.y * p.W + s.x);
      int32_t mv = act;
      if (rng && p.stochastic) {  // get_stochastic_action: one rng.choice per moving agent
        if (act == RMX_WAIT)
          *bad = 1u;  // the reference's slip map has no "wait" entry (KeyError)
        else
          mv = slip_choice(p, act, *rng);
      }
      if (mv < RMX_WAIT && ((L.cell[c] >> mv) & 1u)) {
        s.x += (mv == RMX_LEFT) ? -1 : (mv == RMX_RIGHT) ? 1 : 0;
        s.y += (mv == RMX_UP) ? up : (mv == RMX_DOWN) ? -up : 0;
      }
      c = (uint32_t)(s.y * p.W + s.x);
      if (L.cell[c] & RMX_CELL_HAZARD) {  // hole: fail, Renv = penalty_amount
        fail = true;
        renv = p.hazard_penalty;
      }
      steps += 1;
    }
    trunc = (steps > (uint32_t)p.max_t) || (t1 > p.max_t);
    env_term = trunc || (s.q == fq) || fail;  // RM state read before the wrapper's RM step
  } else {
    if (active) {  // OfficeWorld: RM-final agents keep moving
      uint32_t c = (uint32_t)(s.y * p.W + s.x);
      int32_t mv = RMX_WAIT;
      if (act < RMX_WAIT) {
        if ((L.cell[c] >> act) & 1u) {
          mv = act;
        } else {  // wall collision -> (wall_penalty, "wait")
          renv = p.wall_penalty;
          fail = fail || p.wall_fail;
        }
      }
      if (rng && p.stochastic && mv != RMX_WAIT) mv = slip_choice(p, mv, *rng);  // ma_office.py:155-156
      if (mv < RMX_WAIT && ((L.cell[c] >> mv) & 1u)) {  // apply_action re-checks can_move
        s.x += (mv == RMX_LEFT) ? -1 : (mv == RMX_RIGHT) ? 1 : 0;
        s.y += (mv == RMX_UP) ? up : (mv == RMX_DOWN) ? -up : 0;
        c = (uint32_t)(s.y * p.W + s.x);
      }
      if (L.cell[c] & RMX_CELL_HAZARD) {  // plant
        renv += p.hazard_penalty;
        fail = fail || p.hazard_fail;
      }
      steps += 1;
    }
    env_term = fail;
    trunc = t1 > p.max_t;
  }
  active = active && !(env_term || trunc);
  // RM step for every agent (active or not) on its current cell
  const uint32_t cell = (uint32_t)(s.y * p.W + s.x);
  const uint32_t ev = L.ev[a * p.HW + cell];
  const uint32_t ti = ((uint32_t)(a * p.Q + s.q)) * (uint32_t)p.E + ev;
  const int32_t nq = L.nq[ti];
  const float rq = L.rr[ti];
  AgentOut o;
  o.renv = renv;
  o.reward = renv + p.reward_modifier * rq;  // rewards[name] += reward_rm * reward_modifier
  o.env_term = env_term;
  o.prev_cell = prev_cell;
  o.cell = cell;
  o.ev = ev;
  o.shaping = p.has_shaping ? L.sh[ti] : 0.0f;
  const bool rm_term = (nq == fq);
  o.term = env_term || rm_term;
  o.trunc = trunc;
  s.q = nq;
  s.f = (steps << RMX_F_STEPS_SHIFT) | (active ? RMX_F_ACTIVE : 0u) | (fail ? RMX_F_FAIL : 0u) |
        (o.term ? RMX_F_TERM : 0u) | (trunc ? RMX_F_TRUNC : 0u) | (env_term ? RMX_F_ENV_TERM : 0u) |
        (rm_term ? RMX_F_RM_TERM : 0u);
  return o;
}

// QRM counterfactual experiences of agent a (rm_environment_wrapper.py:140-183): for every RM state j of
// get_all_states()[:-1], the same detected event; missing transition => stay, reward 0 (raw reward).
// Written to the columns qs / qsn / qrq / qdone ([A][Qx][N]): the bound device columns (plain stores), or, SYS,
// the host-mapped mailbox of the resident stepper (rmx_sync.hip) as relaxed system-scope stores (write-through to
// host memory, completed by the stepper's s_waitcnt before its acknowledgement).
template <typename T>
__device__ __forceinline__ void sys_store(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void sys_store(float* p, float v) {
  __hip_atomic_store(reinterpret_cast<uint32_t*>(p), __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <bool SYS = false>
__device__ __forceinline__ void emit_qrm_to(const AgentOut& o, int a, int64_t e, const Lds& L, const KParams& p,
                                            int32_t* qs, int32_t* qsn, float* qrq, uint8_t* qdone) {
  const int Qx = p.n_qrm_max;
  const int nj = p.n_qrm[a];
  const int32_t nQ = p.enc_nq[a];
  const int32_t fq = p.final_q[a];
  auto st = [](auto* ptr, auto v) {
    if constexpr (SYS)
      sys_store(ptr, v);
    else
      *ptr = v;
  };
  for (int j = 0; j < Qx; ++j) {
    const int64_t off = ((int64_t)a * Qx + j) * p.N + e;
    if (j < nj) {
      const uint32_t qj = L.qrm[a * Qx + j];
      const uint32_t tj = ((uint32_t)(a * p.Q) + qj) * (uint32_t)p.E + o.ev;
      const int32_t nqj = L.nq[tj];
      st(qs + off, (int32_t)o.prev_cell * nQ + (int32_t)qj);
      st(qsn + off, (int32_t)o.cell * nQ + nqj);
      st(qrq + off, L.rr[tj]);
      st(qdone + off, (uint8_t)(o.env_term || nqj == fq));
    } else {
      st(qs + off, (int32_t)-1);
      st(qsn + off, (int32_t)-1);
      st(qrq + off, 0.0f);
      st(qdone + off, (uint8_t)0);
    }
  }
}

__device__ __forceinline__ void emit_qrm(const AgentOut& o, int a, int64_t e, const Lds& L, const KParams& p) {
  emit_qrm_to(o, a, e, L, p, p.qrm_s, p.qrm_sn, p.qrm_rq, p.qrm_done);
}


// One env step for all A agents of env e.  Returns true if the episode ended this step.
template <int KIND, int AMAX>
__device__ __forceinline__ bool env_step(AgentReg (&s)[AMAX], int32_t& t, const int32_t (&act)[AMAX], const Lds& L,
                                         const KParams& p, float disc, AgentOut (&o)[AMAX], LaneStats& ls,
                                         uint32_t* bad, Pcg* rng) {
  const int32_t t1 = t + 1;
  bool all_term = true, all_trunc = true;
#pragma unroll
  for (int a = 0; a < AMAX; ++a) {
    if (AMAX <= 4 || a < p.A) {
      o[a] = agent_step<KIND>(s[a], act[a], a, t1, L, p, bad, rng);  // agents draw in order (one env rng)
      s[a].ret = fmaf(disc, o[a].reward, s[a].ret);
      all_term = all_term && o[a].term;
      all_trunc = all_trunc && o[a].trunc;
    }
  }
  t = t1;
  const bool done = all_term || all_trunc;
  if (done) {
    ls.episodes += 1;
    ls.length += t1;
#pragma unroll
    for (int a = 0; a < AMAX; ++a) {
      if (AMAX <= 4 || a < p.A) {
        s[a].f |= RMX_F_ENV_DONE;
        ls.ret += (double)s[a].ret;
        ls.successes += (o[a].term && s[a].q == p.final_q[a] && s[a].ret > 0.0f) ? 1 : 0;
      }
    }
  }
  return done;
}

template <int AMAX>
__device__ __forceinline__ void reset_regs(AgentReg (&s)[AMAX], int32_t& t, const KParams& p) {
  t = 0;
#pragma unroll
  for (int a = 0; a < AMAX; ++a) {
    s[a].x = p.start_x[a];
    s[a].y = p.start_y[a];
    s[a].q = p.init_q[a];
    s[a].f = RMX_F_ACTIVE;
    s[a].ret = 0.0f;
  }
}

// FrozenLake random_start_positions (ma_frozen_lake.py:59-64, 156-172): agents start on free_cells[slot[a]] of the
// shuffled list (shuffle_slots, rmx_device.h; env e's workspace row holds its draws).
template <int AMAX>
__device__ void random_starts(const KParams& p, Pcg& r, int64_t e, AgentReg (&s)[AMAX]) {
  const int n = p.n_free;
  int32_t slot[AMAX];
  shuffle_slots<AMAX>(r, n, p.start_ws + e * (int64_t)shuffle_stride(n), AMAX <= 4 ? AMAX : p.A, slot);
#pragma unroll
  for (int a = 0; a < AMAX; ++a) {
    if (AMAX <= 4 || a < p.A) {
      const int32_t c = p.free_cells[slot[a]];
      s[a].x = c % p.W;
      s[a].y = c / p.W;
    }
  }
}

}  // namespace rmx
