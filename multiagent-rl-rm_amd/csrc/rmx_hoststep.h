// rmx_hoststep.h — the engine's host path: a handle created with cfg.device == RMX_DEVICE_HOST steps its envs on
// the CPU, over the same compiled tables the gfx950 generic kernels stage into LDS (build_table_blob, rmx_tables.cpp)
// and with the same rules as their agent_step / env_step (rmx_generic.h).  It serves BASELINE config 1 — the
// reference's one-env dict API on a CPU (rm_environment_wrapper.py:28-107 under frozen_lake_main.py:336-376) — without
// a GPU and without a PCIe round trip per call, and every other entry point of include/rmx.h on host buffers.
// Plain C++ (no HIP): the sanitizer build (oracle/Makefile `asan`) compiles this file with g++.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/rmx.h"
#include "rmx_host.h"

namespace rmx {

// numpy's PCG64 (XSL-RR 128/64) state as the device's Pcg (rmx_device.h): 128-bit state and increment
struct HostPcg {
  uint64_t hi, lo, ihi, ilo;
};

struct HostAgent {  // one agent's state while its env is stepped (the device's AgentReg)
  int32_t x, y, q;
  uint32_t f;
  float ret;
};

struct HostOut {  // one agent-step's outputs (the device's AgentOut)
  float reward, shaping, renv;
  bool term, trunc, env_term;
  uint32_t prev_cell, cell, ev;
};

struct HostEngine {
  rmx_config cfg{};  // scalars (the table pointers are cleared once the tables are copied)
  // the generic kernels' blob and its section views
  std::vector<unsigned char> blob;
  const uint16_t* cell = nullptr;
  const uint8_t* ev = nullptr;
  const uint8_t* nq = nullptr;
  const float* rr = nullptr;
  const float* sh = nullptr;
  const uint8_t* qrm = nullptr;
  std::vector<float> disc;           // gamma^t, t = 0 .. max_t + 1
  std::vector<uint16_t> free_cells;  // FrozenLake random starts (x-major non-hole cells)
  std::vector<uint16_t> shuffle;     // the shuffle's working copy of free_cells
  int32_t init_q[RMX_MAX_AGENTS]{}, final_q[RMX_MAX_AGENTS]{}, start_x[RMX_MAX_AGENTS]{}, start_y[RMX_MAX_AGENTS]{};
  int32_t n_qrm[RMX_MAX_AGENTS]{}, enc_nq[RMX_MAX_AGENTS]{};
  uint64_t slip_thr[4][4]{};  // ceil(cdf * 2^53) (slip_threshold, rmx_internal.h's rule)
  bool enc_on = false;        // every agent has an encoder stride: enc_state is computed
  // bound host columns; outputs the caller did not bind go to the engine's own columns (the synchronous calls
  // return them)
  rmx_buffers buf{};
  bool bound = false;
  std::vector<float> own_reward, own_renv, own_shaping;
  std::vector<uint8_t> own_done;
  std::vector<int32_t> own_enc;
  float* reward = nullptr;
  float* renv = nullptr;
  float* shaping = nullptr;
  uint8_t* env_done = nullptr;
  int32_t* enc = nullptr;
  uint64_t base_seed = 123;
  double stats[RMX_NSTATS]{};
  uint32_t err = 0;       // an invalid action was stepped (rmx_check_errors)
  bool pending = false;   // rmx_step_sync_begin ran a step whose outputs rmx_sync_wait has not returned
  uint32_t pending_bad = 0;
  bool last_reset = false;  // the synchronous call before the copy was a reset (no step outputs)

  // "" or the reason the config cannot run on the host path (after validate_config)
  std::string init(const rmx_config& c);
  void bind(const rmx_buffers& b);
  // rmx_reset (mask: host bytes, NULL = every env)
  void reset(const uint8_t* mask, uint64_t seed);
  // rmx_step / rmx_step_hashed for every env: actions [A][N] host ints, or hashed (seed, t_global); returns 1 if an
  // action outside [0, 4] (or "wait" under FrozenLake slip) was stepped (as wait)
  uint32_t step(const int32_t* actions, int autoreset, bool hashed = false, uint64_t seed = 0, int64_t t_global = 0,
                float* trace = nullptr);
  void fill_actions(uint64_t seed, int64_t t0, int32_t T, int32_t* out) const;
  int64_t mdp_states(int agent) const;
  void mdp(int agent, int fix_fl, int32_t* next, float* reward, uint8_t* done) const;
  // the synchronous calls' outputs into caller host columns (include/rmx.h: NULL fields skipped); "" or the reason a
  // requested column is not computed
  std::string copy_out(const rmx_buffers& out) const;

 private:
  HostOut agent_step(HostAgent& s, int32_t act, int a, int32_t t1, HostPcg* rng, uint32_t* bad) const;
  void reset_agents(HostAgent* s, int32_t& t) const;
  void random_starts(HostPcg& r, HostAgent* s);
  int32_t slip_choice(int32_t intended, HostPcg& r) const;
};

}  // namespace rmx
