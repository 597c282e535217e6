// rmx_hoststep.cpp — the host path of the step engine (rmx_hoststep.h): envs stepped on the CPU over the generic
// kernels' table blob, one env after another, agents in order.
//
// Reference semantics restated (paths relative to Alee08/multiagent-rl-rm), as the gfx950 kernels restate them:
//   wrapper step      rm_environment_wrapper.py:43-107 (rewards = Renv + reward_modifier * RQ, term = env OR RM)
//   FrozenLake        ma_frozen_lake.py:96-154 (step; inactive or RM-final agents frozen), :174-187 (holes),
//                     :189-215 (terminations, read before the RM step), :224-242 (move, up = y - 1),
//                     :244-262 (slip: rng.choice per moving agent), :59-64 / :156-172 (random starts)
//   OfficeWorld       ma_office.py:122-202 (step; RM-final agents keep moving), :204-220 (plants), :240-257
//                     (terminations), :269-325 (wall collision -> penalty + wait), :327-379 (slip after the wall check)
//   RM step           reward_machine.py:45-59 (missing (q, event) => stay, reward 0)
//   QRM experiences   rm_environment_wrapper.py:140-183
//   get_mdp           rm_environment_wrapper.py:185-283 (terminal self loops, the FrozenLake decode quirk)
//   loop rules        frozen_lake_main.py:336-376, office_main.py:1696-1749 (episode end = all terminated or all
//                     truncated; success evaluation_metrics.py:248-267)
// numpy's default_rng(seed) (SeedSequence -> PCG64), Generator.random / .choice / .shuffle are restated from
// numpy/random/bit_generator.pyx, _pcg64.pyx / pcg64.h and _generator.pyx (numpy 2.2, the reference's runtime).
#include "rmx_hoststep.h"

#include <cmath>
#include <cstring>

namespace rmx {

namespace {

typedef unsigned __int128 u128;
constexpr uint64_t kGoldenH = 0x9E3779B97F4A7C15ull;
const u128 kPcgMult = ((u128)0x2360ED051FC65DA4ull << 64) | 0x4385DF649FCCF645ull;

inline u128 pack(uint64_t hi, uint64_t lo) { return ((u128)hi << 64) | lo; }

inline void pcg_advance(HostPcg& r) {
  const u128 s = pack(r.hi, r.lo) * kPcgMult + pack(r.ihi, r.ilo);
  r.hi = (uint64_t)(s >> 64);
  r.lo = (uint64_t)s;
}

// pcg64_next64: advance, then XSL-RR of the new state
inline uint64_t pcg_next64(HostPcg& r) {
  pcg_advance(r);
  const uint64_t x = r.hi ^ r.lo;
  const unsigned rot = (unsigned)(r.hi >> 58);
  return (x >> rot) | (x << ((64u - rot) & 63u));
}

// SeedSequence(seed).generate_state(4, uint64) -> pcg_setseq_128_srandom_r(v0:v1, v2:v3)
HostPcg seed_pcg64(uint64_t seed) {
  uint32_t hc = 0x43b0d7e5u;
  auto hashmix = [&hc](uint32_t v) {
    v ^= hc;
    hc *= 0x931e8875u;
    v *= hc;
    return v ^ (v >> 16);
  };
  auto mix = [](uint32_t x, uint32_t y) {
    const uint32_t r = 0xca01f9ddu * x - 0x4973f715u * y;
    return r ^ (r >> 16);
  };
  const uint32_t ent[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  const int n_ent = (seed >> 32) ? 2 : 1;  // _coerce_to_uint32_array: little-endian words, 0 -> [0]
  uint32_t pool[4];
  for (int i = 0; i < 4; ++i) pool[i] = hashmix(i < n_ent ? ent[i] : 0u);
  for (int s = 0; s < 4; ++s)
    for (int d = 0; d < 4; ++d)
      if (s != d) pool[d] = mix(pool[d], hashmix(pool[s]));
  uint32_t w[8], hb = 0x8b51f9ddu;
  for (int i = 0; i < 8; ++i) {
    uint32_t x = pool[i & 3] ^ hb;
    hb *= 0x58f38dedu;
    x *= hb;
    w[i] = x ^ (x >> 16);
  }
  uint64_t v[4];
  for (int k = 0; k < 4; ++k) v[k] = (uint64_t)w[2 * k] | ((uint64_t)w[2 * k + 1] << 32);
  const u128 inc = (pack(v[2], v[3]) << 1) | 1u;
  HostPcg r = {0, 0, (uint64_t)(inc >> 64), (uint64_t)inc};
  pcg_advance(r);
  const u128 s = pack(r.hi, r.lo) + pack(v[0], v[1]);
  r.hi = (uint64_t)(s >> 64);
  r.lo = (uint64_t)s;
  pcg_advance(r);
  return r;
}

inline uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + kGoldenH;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// SURVEY.md §8(d)'s counter hash (include/rmx.h rmx_step_hashed)
inline int32_t hash_action(uint64_t seed, int64_t t, int64_t n_global, int64_t e, int A, int i) {
  const uint64_t ctr = (((uint64_t)t * (uint64_t)n_global + (uint64_t)e) * (uint64_t)A + (uint64_t)i) * kGoldenH;
  return (int32_t)(splitmix64(seed ^ ctr) >> 62);
}

inline uint64_t cdf_threshold(double cdf) {  // Generator.random() = m * 2^-53: cdf <= u  <=>  ceil(cdf * 2^53) <= m
  if (!(cdf == cdf)) return ~0ull;
  if (cdf <= 0.0) return 0ull;
  if (cdf >= 1.0) return (1ull << 53) + (cdf > 1.0 ? 1ull : 0ull);
  return (uint64_t)std::ceil(std::ldexp(cdf, 53));
}

}  // namespace

std::string HostEngine::init(const rmx_config& c) {
  BlobOffsets bo;
  if (!build_table_blob(c, blob, bo)) return "tables exceed 64 KiB (the generic kernels' LDS blob)";
  cfg = c;
  cell = reinterpret_cast<const uint16_t*>(blob.data() + bo.cell);
  ev = blob.data() + bo.ev;
  nq = blob.data() + bo.nq;
  rr = reinterpret_cast<const float*>(blob.data() + bo.rr);
  sh = reinterpret_cast<const float*>(blob.data() + bo.sh);
  qrm = blob.data() + bo.qrm;
  disc = discount_table(c);
  if (c.random_starts) {
    free_cells = rmx::free_cells(c);
    shuffle.resize(free_cells.size());
  }
  enc_on = c.enc_nq != nullptr;
  for (int a = 0; a < c.n_agents; ++a) {
    init_q[a] = c.init_q[a];
    final_q[a] = c.final_q[a];
    start_x[a] = c.start_xy[2 * a];
    start_y[a] = c.start_xy[2 * a + 1];
    enc_nq[a] = c.enc_nq ? c.enc_nq[a] : 0;
    n_qrm[a] = c.n_qrm_max > 0 ? c.n_qrm[a] : 0;
  }
  if (c.stochastic)
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) slip_thr[i][j] = cdf_threshold(c.slip_cdf[i][j]);
  const size_t AN = (size_t)c.n_agents * (size_t)c.n_envs, N = (size_t)c.n_envs;
  own_reward.assign(AN, 0.0f);
  own_renv.assign(AN, 0.0f);
  own_shaping.assign(c.has_shaping ? AN : 0, 0.0f);
  own_done.assign(N, 0);
  own_enc.assign(enc_on ? AN : 0, 0);
  cfg.cell = nullptr;
  cfg.cell_event = nullptr;
  cfg.next_q = nullptr;
  cfg.rm_reward = nullptr;
  cfg.shape = nullptr;
  cfg.init_q = cfg.final_q = cfg.start_xy = nullptr;
  cfg.n_qrm = cfg.enc_nq = nullptr;
  cfg.qrm_states = nullptr;
  return std::string();
}

void HostEngine::bind(const rmx_buffers& b) {
  buf = b;
  reward = b.reward;
  renv = b.renv ? b.renv : own_renv.data();
  shaping = !cfg.has_shaping ? nullptr : b.shaping ? b.shaping : own_shaping.data();
  env_done = b.env_done ? b.env_done : own_done.data();
  enc = !enc_on ? nullptr : b.enc_state ? b.enc_state : own_enc.data();
  bound = true;
  pending = false;
}

void HostEngine::reset_agents(HostAgent* s, int32_t& t) const {
  t = 0;
  for (int a = 0; a < cfg.n_agents; ++a) s[a] = {start_x[a], start_y[a], init_q[a], RMX_F_ACTIVE, 0.0f};
}

// _sample_start_positions: rng.shuffle(free_cells) (the untyped Fisher-Yates: for i = n-1 .. 1 swap x[i] with
// x[random_interval(i)], 32-bit draws masked to the smallest all-ones mask >= i and rejected while > i, each 64-bit
// output giving its low half, then its high half), agent a on the a-th cell
void HostEngine::random_starts(HostPcg& r, HostAgent* s) {
  const int32_t n = (int32_t)free_cells.size();
  std::memcpy(shuffle.data(), free_cells.data(), sizeof(uint16_t) * (size_t)n);
  bool have_half = false;
  uint32_t half = 0;
  auto next32 = [&]() {
    if (have_half) {
      have_half = false;
      return half;
    }
    const uint64_t o = pcg_next64(r);
    half = (uint32_t)(o >> 32);
    have_half = true;
    return (uint32_t)o;
  };
  for (int32_t i = n - 1; i >= 1; --i) {
    uint32_t mask = (uint32_t)i;
    mask |= mask >> 1;
    mask |= mask >> 2;
    mask |= mask >> 4;
    mask |= mask >> 8;
    mask |= mask >> 16;
    uint32_t j;
    while ((j = next32() & mask) > (uint32_t)i) {
    }
    const uint16_t tmp = shuffle[i];
    shuffle[i] = shuffle[j];
    shuffle[j] = tmp;
  }
  for (int a = 0; a < cfg.n_agents; ++a) {
    s[a].x = shuffle[a] % cfg.width;
    s[a].y = shuffle[a] / cfg.width;
  }
}

// rng.choice(outcomes, p=probs) with the intended action's row: one Generator.random() draw, searchsorted(side="right")
int32_t HostEngine::slip_choice(int32_t intended, HostPcg& r) const {
  const uint64_t m = pcg_next64(r) >> 11;
  int idx = 0;
  for (int i = 0; i + 1 < cfg.slip_n[intended] && i < 3; ++i) idx += slip_thr[intended][i] <= m ? 1 : 0;
  return cfg.slip_out[intended][idx];
}

// One wrapper step of agent a (t1: the env's timestep after its increment)
HostOut HostEngine::agent_step(HostAgent& s, int32_t act, int a, int32_t t1, HostPcg* rng, uint32_t* bad) const {
  const int32_t W = cfg.width, fq = final_q[a];
  bool active = (s.f & RMX_F_ACTIVE) != 0, fail = (s.f & RMX_F_FAIL) != 0;
  uint32_t steps = s.f >> RMX_F_STEPS_SHIFT;
  if ((uint32_t)act > (uint32_t)RMX_WAIT) {  // invalid: reported, stepped as wait
    *bad = 1u;
    act = RMX_WAIT;
  }
  const int32_t up = cfg.kind == RMX_FROZEN_LAKE ? -1 : 1;
  auto move = [&](int32_t mv) {
    s.x += mv == RMX_LEFT ? -1 : mv == RMX_RIGHT ? 1 : 0;
    s.y += mv == RMX_UP ? up : mv == RMX_DOWN ? -up : 0;
  };
  float renv = 0.0f;
  bool env_term, trunc;
  const uint32_t prev_cell = (uint32_t)(s.y * W + s.x);
  if (cfg.kind == RMX_FROZEN_LAKE) {
    if (active && s.q != fq) {  // inactive or RM already final: frozen, Renv 0
      int32_t mv = act;
      if (rng && cfg.stochastic) {
        if (act == RMX_WAIT)
          *bad = 1u;  // the slip map has no "wait" (the reference's KeyError)
        else
          mv = slip_choice(act, *rng);
      }
      if (mv < RMX_WAIT && ((cell[s.y * W + s.x] >> mv) & 1u)) move(mv);
      if (cell[s.y * W + s.x] & RMX_CELL_HAZARD) {  // hole
        fail = true;
        renv = cfg.hazard_penalty;
      }
      steps += 1;
    }
    trunc = steps > (uint32_t)cfg.max_t || t1 > cfg.max_t;
    env_term = trunc || s.q == fq || fail;  // the RM state before the wrapper's RM step
  } else {
    if (active) {  // RM-final agents keep moving
      int32_t mv = RMX_WAIT;
      if (act < RMX_WAIT) {
        if ((cell[s.y * W + s.x] >> act) & 1u) {
          mv = act;
        } else {  // wall collision: penalty, "wait"
          renv = cfg.wall_penalty;
          fail = fail || cfg.wall_fail;
        }
      }
      if (rng && cfg.stochastic && mv != RMX_WAIT) mv = slip_choice(mv, *rng);
      if (mv < RMX_WAIT && ((cell[s.y * W + s.x] >> mv) & 1u)) move(mv);  // apply_action re-checks can_move
      if (cell[s.y * W + s.x] & RMX_CELL_HAZARD) {  // plant
        renv += cfg.hazard_penalty;
        fail = fail || cfg.hazard_fail;
      }
      steps += 1;
    }
    env_term = fail;
    trunc = t1 > cfg.max_t;
  }
  active = active && !(env_term || trunc);
  // the RM steps for every agent, active or not, on its current cell
  const uint32_t c = (uint32_t)(s.y * W + s.x);
  const uint32_t e = ev[(size_t)a * cfg.width * cfg.height + c];
  const size_t ti = ((size_t)a * cfg.n_rm_states + (size_t)s.q) * cfg.n_events + e;
  const int32_t next = nq[ti];
  HostOut o;
  o.renv = renv;
  o.reward = renv + cfg.reward_modifier * rr[ti];
  o.shaping = cfg.has_shaping ? sh[ti] : 0.0f;
  o.env_term = env_term;
  o.prev_cell = prev_cell;
  o.cell = c;
  o.ev = e;
  const bool rm_term = next == fq;
  o.term = env_term || rm_term;
  o.trunc = trunc;
  s.q = next;
  s.f = (steps << RMX_F_STEPS_SHIFT) | (active ? RMX_F_ACTIVE : 0u) | (fail ? RMX_F_FAIL : 0u) |
        (o.term ? RMX_F_TERM : 0u) | (trunc ? RMX_F_TRUNC : 0u) | (env_term ? RMX_F_ENV_TERM : 0u) |
        (rm_term ? RMX_F_RM_TERM : 0u);
  return o;
}

void HostEngine::reset(const uint8_t* mask, uint64_t seed) {
  base_seed = seed;
  const int64_t N = cfg.n_envs;
  const int A = cfg.n_agents;
  const bool rng_on = cfg.stochastic || cfg.random_starts;
  for (int64_t e = 0; e < N; ++e) {
    if (mask && !mask[e]) continue;
    HostAgent s[RMX_MAX_AGENTS];
    int32_t t;
    reset_agents(s, t);
    if (rng_on) {  // env.reset: self.rng = default_rng(seed); episode 0 of the schedule
      HostPcg r = seed_pcg64(base_seed * cfg.seed_scale + (uint64_t)(cfg.env_offset + e) * cfg.seed_env_stride);
      if (cfg.random_starts) random_starts(r, s);
      buf.rng[e] = r.hi;
      buf.rng[N + e] = r.lo;
      buf.rng[2 * N + e] = r.ihi;
      buf.rng[3 * N + e] = r.ilo;
      buf.episode[e] = 0;
    }
    buf.t[e] = t;
    for (int a = 0; a < A; ++a) {
      const int64_t k = (int64_t)a * N + e;
      buf.pos_x[k] = s[a].x;
      buf.pos_y[k] = s[a].y;
      buf.rm_q[k] = s[a].q;
      buf.flags[k] = s[a].f;
      buf.ep_ret[k] = s[a].ret;
    }
  }
}

uint32_t HostEngine::step(const int32_t* actions, int autoreset, bool hashed, uint64_t seed, int64_t t_global,
                          float* trace) {
  const int64_t N = cfg.n_envs;
  const int A = cfg.n_agents;
  const bool rng_on = cfg.stochastic || cfg.random_starts;
  const int Qx = buf.qrm_s ? cfg.n_qrm_max : 0;
  uint32_t bad = 0;
  for (int64_t e = 0; e < N; ++e) {
    HostAgent s[RMX_MAX_AGENTS];
    int32_t act[RMX_MAX_AGENTS];
    int32_t t = buf.t[e];
    for (int a = 0; a < A; ++a) {
      const int64_t k = (int64_t)a * N + e;
      s[a] = {buf.pos_x[k], buf.pos_y[k], buf.rm_q[k], buf.flags[k], buf.ep_ret[k]};
      // columns a caller wrote out of range index no table outside it (the kernels' range-checked descriptors give
      // the same guarantee on the device; the values that follow are unspecified, as there)
      if ((uint32_t)s[a].x >= (uint32_t)cfg.width) s[a].x = 0;
      if ((uint32_t)s[a].y >= (uint32_t)cfg.height) s[a].y = 0;
      if ((uint32_t)s[a].q >= (uint32_t)cfg.n_rm_states) s[a].q = 0;
      act[a] = hashed ? hash_action(seed, t_global, cfg.n_envs_global, cfg.env_offset + e, A, a) : actions[k];
    }
    HostPcg rng = {0, 0, 0, 0};
    if (rng_on) rng = {buf.rng[e], buf.rng[N + e], buf.rng[2 * N + e], buf.rng[3 * N + e]};
    if (autoreset && (s[0].f & RMX_F_ENV_DONE)) {  // the loop's reset() before this step
      reset_agents(s, t);
      if (rng_on) {  // env.rng = default_rng(seed of the next episode)
        const int32_t k = buf.episode[e] + 1;
        buf.episode[e] = k;
        rng = seed_pcg64(base_seed * cfg.seed_scale + (uint64_t)(cfg.env_offset + e) * cfg.seed_env_stride +
                         (uint64_t)k * cfg.seed_episode_stride);
        if (cfg.random_starts) random_starts(rng, s);  // before any slip draw of the episode
      }
    }
    const float d = cfg.gamma == 1.0f ? 1.0f : disc[(size_t)std::min<uint32_t>((uint32_t)t, (uint32_t)cfg.max_t + 1u)];
    const int32_t t1 = (int32_t)((uint32_t)t + 1u);  // wraps as on the device (a caller-written t may be INT32_MAX)
    bool all_term = true, all_trunc = true;
    HostOut o[RMX_MAX_AGENTS];
    for (int a = 0; a < A; ++a) {  // agents in order: one env rng
      o[a] = agent_step(s[a], act[a], a, t1, rng_on ? &rng : nullptr, &bad);
      s[a].ret = std::fma(d, o[a].reward, s[a].ret);
      all_term = all_term && o[a].term;
      all_trunc = all_trunc && o[a].trunc;
    }
    t = t1;
    const bool done = all_term || all_trunc;
    if (done) {  // episode statistics (the loops' per-episode logging)
      stats[RMX_STAT_EPISODES] += 1.0;
      stats[RMX_STAT_SUM_LENGTH] += (double)t1;
      for (int a = 0; a < A; ++a) {
        s[a].f |= RMX_F_ENV_DONE;
        stats[RMX_STAT_SUM_RETURN] += (double)s[a].ret;
        stats[RMX_STAT_SUCCESSES] += (o[a].term && s[a].q == final_q[a] && s[a].ret > 0.0f) ? 1.0 : 0.0;
      }
    }
    if (rng_on) {
      buf.rng[e] = rng.hi;
      buf.rng[N + e] = rng.lo;
      buf.rng[2 * N + e] = rng.ihi;
      buf.rng[3 * N + e] = rng.ilo;
    }
    buf.t[e] = t;
    env_done[e] = (uint8_t)done;
    for (int a = 0; a < A; ++a) {
      const int64_t k = (int64_t)a * N + e;
      buf.pos_x[k] = s[a].x;
      buf.pos_y[k] = s[a].y;
      buf.rm_q[k] = s[a].q;
      buf.flags[k] = s[a].f;
      buf.ep_ret[k] = s[a].ret;
      reward[k] = o[a].reward;
      renv[k] = o[a].renv;
      if (shaping) shaping[k] = o[a].shaping;
      if (enc) enc[k] = (s[a].y * cfg.width + s[a].x) * enc_nq[a] + s[a].q;
      if (trace) trace[k] = o[a].reward;
      for (int j = 0; j < Qx; ++j) {  // QRM counterfactuals: every state of get_all_states()[:-1], same event
        const int64_t off = ((int64_t)a * Qx + j) * N + e;
        if (j < n_qrm[a]) {
          const uint32_t qj = qrm[(size_t)a * Qx + j];
          const size_t tj = ((size_t)a * cfg.n_rm_states + qj) * cfg.n_events + o[a].ev;
          const int32_t nqj = nq[tj];
          buf.qrm_s[off] = (int32_t)o[a].prev_cell * enc_nq[a] + (int32_t)qj;
          buf.qrm_sn[off] = (int32_t)o[a].cell * enc_nq[a] + nqj;
          buf.qrm_rq[off] = rr[tj];
          buf.qrm_done[off] = (uint8_t)(o[a].env_term || nqj == final_q[a]);
        } else {
          buf.qrm_s[off] = -1;
          buf.qrm_sn[off] = -1;
          buf.qrm_rq[off] = 0.0f;
          buf.qrm_done[off] = 0;
        }
      }
    }
  }
  err |= bad;
  return bad;
}

void HostEngine::fill_actions(uint64_t seed, int64_t t0, int32_t T, int32_t* out) const {
  const int64_t N = cfg.n_envs;
  const int A = cfg.n_agents;
  for (int64_t s = 0; s < T; ++s)
    for (int a = 0; a < A; ++a)
      for (int64_t e = 0; e < N; ++e)
        out[(s * A + a) * N + e] = hash_action(seed, t0 + s, cfg.n_envs_global, cfg.env_offset + e, A, a);
}

int64_t HostEngine::mdp_states(int agent) const {
  return (int64_t)cfg.width * cfg.height * enc_nq[agent];
}

// get_mdp of one agent (deterministic dynamics): every (encoded state, action) from timestep 0; terminal states
// self-loop; fix_fl = 0 keeps the reference's FrozenLake decode quirk (no entries for non-hole states)
void HostEngine::mdp(int ag, int fix_fl, int32_t* next, float* rew, uint8_t* done) const {
  const int64_t S = mdp_states(ag);
  const int32_t nQ = enc_nq[ag];
  for (int64_t i = 0; i < S * 4; ++i) {
    const int64_t st = i >> 2;
    const int act = (int)(i & 3);
    const int32_t q = (int32_t)(st % nQ), pos = (int32_t)(st / nQ);
    const bool hz = (cell[pos] & RMX_CELL_HAZARD) != 0;
    bool term_state = false;
    float term_r = 0.0f;
    if (cfg.kind == RMX_FROZEN_LAKE) {
      if (hz) {
        term_state = true;
        term_r = cfg.hazard_penalty;
      } else if (fix_fl && q == final_q[ag]) {
        term_state = true;
      } else if (!fix_fl) {
        next[i] = -1;
        rew[i] = 0.0f;
        done[i] = 255;
        continue;
      }
    } else {
      if (hz && cfg.hazard_fail) {
        term_state = true;
        term_r = cfg.hazard_penalty;
      } else if (q == final_q[ag]) {
        term_state = true;
      }
    }
    if (term_state) {
      next[i] = (int32_t)st;
      rew[i] = term_r;
      done[i] = 1;
      continue;
    }
    HostAgent s = {pos % cfg.width, pos / cfg.width, q, RMX_F_ACTIVE, 0.0f};
    uint32_t bad = 0;
    const HostOut o = agent_step(s, act, ag, 1, nullptr, &bad);
    next[i] = (int32_t)o.cell * nQ + s.q;
    rew[i] = o.reward;
    done[i] = (uint8_t)(o.term || o.trunc);
  }
}

std::string HostEngine::copy_out(const rmx_buffers& out) const {
  const int64_t A = cfg.n_agents, N = cfg.n_envs;
  if (out.shaping && !cfg.has_shaping) return "sync output column not computed: shaping";
  if (out.enc_state && !enc_on) return "sync output column not computed: enc_state";
  if ((out.qrm_s || out.qrm_sn || out.qrm_rq || out.qrm_done) && !buf.qrm_s)
    return "sync output columns not computed: QRM (bind the QRM columns)";
  const size_t AN = (size_t)(A * N), AQN = AN * (size_t)(buf.qrm_s ? cfg.n_qrm_max : 0);
  auto cp = [](void* dst, const void* src, size_t n) {
    if (dst && dst != src) std::memcpy(dst, src, n);
  };
  auto zero_or = [&](void* dst, const void* src, size_t n) {  // a reset returns no step outputs: zeros
    if (!dst) return;
    if (last_reset)
      std::memset(dst, 0, n);
    else
      cp(dst, src, n);
  };
  cp(out.pos_x, buf.pos_x, 4 * AN);
  cp(out.pos_y, buf.pos_y, 4 * AN);
  cp(out.rm_q, buf.rm_q, 4 * AN);
  cp(out.flags, buf.flags, 4 * AN);
  cp(out.ep_ret, buf.ep_ret, 4 * AN);
  cp(out.t, buf.t, 4 * (size_t)N);
  zero_or(out.reward, reward, 4 * AN);
  zero_or(out.renv, renv, 4 * AN);
  zero_or(out.shaping, shaping, 4 * AN);
  zero_or(out.env_done, env_done, (size_t)N);
  if (out.enc_state) {  // after a reset too: the encoded start state
    for (int64_t a = 0; a < A; ++a)
      for (int64_t e = 0; e < N; ++e) {
        const int64_t k = a * N + e;
        out.enc_state[k] = (buf.pos_y[k] * cfg.width + buf.pos_x[k]) * enc_nq[a] + buf.rm_q[k];
      }
  }
  cp(out.qrm_s, buf.qrm_s, 4 * AQN);
  cp(out.qrm_sn, buf.qrm_sn, 4 * AQN);
  cp(out.qrm_rq, buf.qrm_rq, 4 * AQN);
  cp(out.qrm_done, buf.qrm_done, AQN);
  return std::string();
}

}  // namespace rmx
