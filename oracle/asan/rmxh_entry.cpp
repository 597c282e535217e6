// rmxh_entry.cpp — TEST INFRASTRUCTURE ONLY: a C entry point over the engine's host-side table builders
// (multiagent-rl-rm_amd/csrc/rmx_tables.cpp, compiled unchanged next to this file) for the sanitizer build
// (oracle/Makefile `asan`, tests/test_sanitizers.py).  Runs every builder rmx_create runs, in the same
// order, on one config and reports the sizes it produced.
#include <cstring>
#include <vector>

#include "../../multiagent-rl-rm_amd/csrc/rmx_comd.h"
#include "../../multiagent-rl-rm_amd/csrc/rmx_host.h"
#include "../../multiagent-rl-rm_amd/csrc/rmx_hoststep.h"

extern "C" int rmxh_build(const rmx_config* c, long long* out /* [8] */) {
  for (int i = 0; i < 8; ++i) out[i] = -1;
  const std::string msg = rmx::validate_config(*c);
  if (!msg.empty()) return -1;
  std::vector<unsigned char> blob;
  rmx::BlobOffsets bo;
  out[0] = rmx::build_table_blob(*c, blob, bo) ? (long long)blob.size() : -1;
  out[1] = (long long)rmx::discount_table(*c).size();
  std::vector<unsigned char> fast;
  rmx::FastLayout fl;
  if (rmx::build_fast_blob(*c, fast, fl)) {
    out[2] = (long long)fast.size();
    int32_t mg_base[RMX_MAX_AGENTS] = {};
    uint32_t palb[RMX_MAX_AGENTS] = {};
    std::vector<uint32_t> merged, compact;
    if (rmx::build_merged(*c, fast, fl.off_rm, mg_base, merged)) {
      out[3] = (long long)merged.size() * 4;
      out[4] = rmx::build_compact(*c, mg_base, merged, palb, compact) ? (long long)compact.size() * 4 : -1;
      out[5] = 0;  // (the 8-B record builder was removed in round 5)
    }
  }
  out[6] = (long long)rmx::free_cells(*c).size();
  out[7] = (long long)(rmx::config_digest(*c) >> 1);  // the checkpoint digest reads every table too
  return 0;
}

// The engine queue's code-object metadata reader (rmx_comd.cpp) over caller bytes: 0 read (n_step / n_refused set),
// -1 refused as unreadable.
extern "C" int rmxh_co_check(const unsigned char* co, size_t bytes, unsigned long long fp_offset,
                             unsigned long long fp_size, unsigned long long hidden_base, long long* n_step,
                             long long* n_refused) {
  const rmx::CoCheck c = rmx::check_code_object(co, bytes, rmx::CoLayout{fp_offset, fp_size, hidden_base});
  *n_step = (long long)c.n_step;
  *n_refused = (long long)c.refused.size();
  return c.err.empty() ? 0 : -1;
}

// The engine's host path (rmx_hoststep.cpp, compiled unchanged next to this file): every HostEngine entry point the C
// ABI's host handles call, on columns in exactly-sized heap allocations (a read or write past one lands in the
// sanitizer's redzone): reset with a seed, `steps` hashed steps with autoreset (QRM columns bound when the config has
// them, one invalid action every 97 steps), a masked reset, a traced rollout, the synchronous copy-out of every column,
// and get_mdp of every agent with an encoder stride.  out[0..3]: the statistics; out[4]: a digest of the final state
// columns (compared with librmx.so's host handle on the same inputs); out[5]: 1 if an invalid action was reported.
extern "C" int rmxh_host_run(const rmx_config* c, long long steps, unsigned long long seed, double* out /* [6] */) {
  if (!rmx::validate_config(*c).empty()) return -1;
  rmx::HostEngine h;
  if (!h.init(*c).empty()) return -2;
  const size_t A = (size_t)c->n_agents, N = (size_t)c->n_envs, AN = A * N, Qx = (size_t)c->n_qrm_max;
  std::vector<int32_t> px(AN), py(AN), q(AN), t(N), enc(AN), qs(AN * Qx), qsn(AN * Qx), ep(N);
  std::vector<uint32_t> fl(AN);
  std::vector<float> ret(AN), rew(AN), renv(AN), sh(AN), qrq(AN * Qx);
  std::vector<uint8_t> done(N), qd(AN * Qx);
  std::vector<uint64_t> rng(4 * N);
  rmx_buffers b;
  std::memset(&b, 0, sizeof(b));
  b.pos_x = px.data(), b.pos_y = py.data(), b.rm_q = q.data(), b.flags = fl.data(), b.ep_ret = ret.data();
  b.t = t.data(), b.reward = rew.data(), b.env_done = done.data(), b.renv = renv.data();
  if (c->has_shaping) b.shaping = sh.data();
  if (c->enc_nq) b.enc_state = enc.data();
  if (Qx) b.qrm_s = qs.data(), b.qrm_sn = qsn.data(), b.qrm_rq = qrq.data(), b.qrm_done = qd.data();
  if (c->stochastic || c->random_starts) b.rng = rng.data(), b.episode = ep.data();
  h.bind(b);
  h.reset(nullptr, seed);
  std::vector<int32_t> act(AN);
  uint32_t bad = 0;
  for (long long s = 0; s < steps; ++s) {
    if (s % 97 == 5) {  // caller actions, one of them invalid (stepped as wait, reported)
      for (size_t k = 0; k < AN; ++k) act[k] = (int32_t)((s + k) % 4);
      act[AN / 2] = 9;
      bad |= h.step(act.data(), 1);
    } else {
      bad |= h.step(nullptr, 1, true, seed, s);
    }
  }
  // columns a caller overwrote with out-of-range values: the step must not index outside its tables
  for (size_t k = 0; k < AN; ++k) {
    px[k] = (int32_t)(k * 2654435761u) ^ 0x7ffff;
    py[k] = -(int32_t)k - 300;
    q[k] = (int32_t)(k * 40503u);
    fl[k] = (uint32_t)(k * 2246822519u);
  }
  for (size_t e = 0; e < N; ++e) t[e] = (int32_t)(e * 7919u) - 100000;
  t[0] = 0x7fffffff;  // t + 1 wraps (UBSan: no signed overflow)
  for (int it = 0; it < 5; ++it) bad |= h.step(nullptr, 1, true, seed, 777 + it);
  h.reset(nullptr, seed);
  for (int it = 0; it < 5; ++it) bad |= h.step(nullptr, 1, true, seed, 900 + it);
  std::vector<uint8_t> mask(N);
  for (size_t e = 0; e < N; e += 3) mask[e] = 1;
  h.reset(mask.data(), seed + 1);
  std::vector<float> trace(AN * 16);
  for (int it = 0; it < 16; ++it) h.step(nullptr, 1, true, seed, steps + it, trace.data() + (size_t)it * AN);
  // the synchronous calls' copy-out into separate exactly-sized columns
  std::vector<int32_t> ox(AN), oy(AN), oq(AN), ot(N), oenc(AN), oqs(AN * Qx), oqsn(AN * Qx);
  std::vector<uint32_t> ofl(AN);
  std::vector<float> oret(AN), orew(AN), orenv(AN), osh(AN), oqrq(AN * Qx);
  std::vector<uint8_t> odone(N), oqd(AN * Qx);
  rmx_buffers o;
  std::memset(&o, 0, sizeof(o));
  o.pos_x = ox.data(), o.pos_y = oy.data(), o.rm_q = oq.data(), o.flags = ofl.data(), o.ep_ret = oret.data();
  o.t = ot.data(), o.reward = orew.data(), o.env_done = odone.data(), o.renv = orenv.data();
  if (c->has_shaping) o.shaping = osh.data();
  if (c->enc_nq) o.enc_state = oenc.data();
  if (Qx) o.qrm_s = oqs.data(), o.qrm_sn = oqsn.data(), o.qrm_rq = oqrq.data(), o.qrm_done = oqd.data();
  if (!h.copy_out(o).empty()) return -3;
  h.last_reset = true;
  if (!h.copy_out(o).empty()) return -3;
  for (int a = 0; a < c->n_agents; ++a) {
    if (!c->enc_nq) break;
    const int64_t S = h.mdp_states(a);
    std::vector<int32_t> nx((size_t)S * 4);
    std::vector<float> mr((size_t)S * 4);
    std::vector<uint8_t> md((size_t)S * 4);
    h.mdp(a, 0, nx.data(), mr.data(), md.data());
    h.mdp(a, 1, nx.data(), mr.data(), md.data());
  }
  for (int k = 0; k < 4; ++k) out[k] = h.stats[k];
  uint64_t d = 0xcbf29ce484222325ull;
  auto mix = [&](const void* p, size_t n) {
    const unsigned char* x = static_cast<const unsigned char*>(p);
    for (size_t i = 0; i < n; ++i) d = (d ^ x[i]) * 0x100000001b3ull;
  };
  mix(px.data(), 4 * AN), mix(py.data(), 4 * AN), mix(q.data(), 4 * AN), mix(fl.data(), 4 * AN), mix(t.data(), 4 * N);
  out[4] = (double)(d >> 12);
  out[5] = bad ? 1.0 : 0.0;
  return 0;
}
