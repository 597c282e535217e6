// rmx_capi.cpp — the extern "C" boundary of include/rmx.h (handle lifetime, validation, uploads,
// launches).  Each entry point maps onto one reference call site; see include/rmx.h for the map.
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <exception>
#include <string>
#include <vector>

#include "rmx_host.h"
#include "rmx_hoststep.h"
#include "rmx_internal.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  return fail(RMX_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define HIP_TRY(expr, what)            \
  do {                                 \
    hipError_t _e = (expr);            \
    if (_e != hipSuccess) return hip_fail(_e, what); \
  } while (0)

// Default fast-path table mode (overridable by RMX_FAST_TABLES for tests), chosen by measurement on MI355X at
// 65,536 envs (profiles/r01_ab_log.md c12/c15/c25): the tables read from the global blob (no staging,
// no block barrier); the merged single-lookup table while it is small.
// 128 KiB: config 5's shared-section table (77 KB) beats the global blob (3.74-3.76 vs 3.86-3.87 us, r01_ab_log
// c78); its unshared 233 KB table lost (c26)
constexpr size_t kFastMergedDefaultBytes = 128 * 1024;
// Episode statistics: per-env no-return atomics are off the critical path at small N, but at large N
// their count (3 per finished env) costs 10-15 % of the step (8.4M envs: 173 vs 191-198 us); there the
// per-wave slab (one DPP reduction + one 32-B store per wave) wins.
constexpr int64_t kFastWaveStatsMinEnvs = 1 << 20;
// The same size switches the generic kernel to skipping stores of every unchanged column word and the fast
// kernel to 256-thread workgroups (the bandwidth regime).
constexpr int64_t kFastSkipMinEnvs = 1 << 20;
// Non-temporal column stores from this many env x agent instances on (see rmx_create).
constexpr int64_t kFastNtMinInstances = int64_t(1) << 23;

}  // namespace

struct rmx_handle {
  rmx_config cfg;  // scalars only (host table pointers cleared after upload)
  // cfg.device == RMX_DEVICE_HOST: the CPU path (rmx_hoststep.cpp) serves every entry point; nothing below is used
  rmx::HostEngine* host = nullptr;
  // rmx_step_seq's recorded window, reused while its inputs are unchanged: the handle's parameter block
  // (fast_params), the call's arguments; seq_key names it to the device queue (its prebuilt packets)
  std::vector<rmx::StepLaunch> seq;
  rmx::FastParams seq_base;
  const int32_t* seq_actions = nullptr;
  const double* seq_out = nullptr;
  int64_t seq_stride = 0;
  int32_t seq_k = 0;
  int seq_autoreset = -1;
  uint64_t seq_key = 0;  // 0: nothing recorded
  bool queue_off = false;  // RMX_QUEUE=0 at rmx_create: rmx_step_seq always takes the stream path
  int seq_dispatch = RMX_SEQ_NONE;  // how the last rmx_step_seq ran
  int64_t seq_recordings = 0;       // windows recorded (a repeated identical call reuses the last one)
  int device = 0;
  int block = 256;
  // measured on MI355X (scripts/variants.py): thread-per-env is faster for the HBM round-trip step
  // kernel (5.1 vs 4.0 TB/s at 4M envs, equal at 65k); lane-per-agent is 1.6-2.3x faster for the
  // register-resident fused rollout.
  int step_layout = rmx::kLayoutThreadPerEnv;
  int rollout_layout = rmx::kLayoutLanePerAgent;
  void* d_tables = nullptr;
  size_t tables_bytes = 0;  // multiple of 16
  int32_t off_cell = 0, off_ev = 0, off_nq = 0, off_rr = 0, off_sh = 0, off_qrm = 0;
  int32_t n_qrm[RMX_MAX_AGENTS]{}, enc_nq[RMX_MAX_AGENTS]{};
  float* d_disc = nullptr;
  double* d_slab = nullptr;
  int64_t n_waves = 0;
  double* d_stats = nullptr;  // [RMX_NSTATS] scratch for rmx_stats_host
  uint32_t* d_err = nullptr;
  rmx_buffers buf{};
  bool bound = false;
  uint64_t base_seed = 123;  // last rmx_reset seed (autoreset reseeds from it)
  uint64_t digest = 0;       // config_digest at rmx_create (checkpoint identity)
  int32_t diag = 0;          // RMX_DIAG builds only: diagnostic kernel variants
  unsigned long long* d_stamps = nullptr;  // RMX_DIAG builds: in-kernel stamps of the fast kernel
  int32_t init_q[RMX_MAX_AGENTS]{}, final_q[RMX_MAX_AGENTS]{}, start_x[RMX_MAX_AGENTS]{}, start_y[RMX_MAX_AGENTS]{};
  // deterministic fast path (rmx::FastParams): pre-composed move words + packed RM entries
  bool fast = false;  // the thread-per-env fast kernel (step_fast_kernel) runs this handle's steps
  int fast_wave_stats = 0;  // episode stats: 1 per-wave slab (large N), 0 per-env atomics; RMX_FAST_STATS=wave|env
  int fast_skip = 0;        // rmx::kSkipRare / kSkipRareNT (by size; RMX_FAST_SKIP=2|3 forces one)
  int generic_skip = 0;     // 1: the generic kernel skips every unchanged column word (large N)
  int fast_block = 256;     // workgroup size of the fast step kernel: 64 below 1M envs, 256 from there
  int rollout_lds = 1;      // fast rollout: tables staged into LDS (1) or read through L2 (0); RMX_ROLLOUT_LDS
  int fast_tables = rmx::kTblGlobal;  // table mode rmx::kTblGlobal / kTblMerged / kTblMerged4; RMX_FAST_TABLES
  void* d_fast = nullptr;
  void* d_merged = nullptr;  // kTblMerged table (RMX_FAST_TABLES=merged or the default where measured faster)
  size_t merged_bytes = 0;
  // fast-path episode statistics: es_ret [N] f64 | es_cnt [N] u64 | es_succ [N] u32
  unsigned char* d_es = nullptr;
  size_t es_bytes = 0;
  double* es_ret = nullptr;
  unsigned long long* es_cnt = nullptr;
  uint32_t* es_succ = nullptr;
  // rmx_step_report's fused report, in the same allocation: per-block partials [ceil(N/64)][RMX_NSTATS] | ticket
  double* rpt_partial = nullptr;
  unsigned int* rpt_ticket = nullptr;
  int32_t fast_n16 = 0, fast_off_rm = 0, fast_off_info = 0;
  uint8_t fast_qrm_q[RMX_MAX_AGENTS][rmx::kFastMaxQrm]{};  // QRM state lists for the fast kernel
  int32_t mg_base[RMX_MAX_AGENTS]{};                        // merged-table record index of each agent's section
  size_t merged4_off = 0, merged4_bytes = 0;  // kTblMerged4 records, after the 16-B records in d_merged
  uint32_t mg_palb[RMX_MAX_AGENTS]{};  // kTblMerged4: each agent's reward palette as four signed bytes
  // FrozenLake random starts: non-hole cells (x-major) and the per-env shuffle workspace [N][n_free]
  int32_t n_free = 0;
  uint16_t* d_free = nullptr;
  uint16_t* d_start_ws = nullptr;
  // random starts: the step kernel's next-episode shuffle in progress, [4][N] u64 generator | [N] index | [N] tag
  unsigned char* d_nx = nullptr;
  // slip / random starts with seed_episode_stride == 0 (rmx::kRngFixedSeed): every env's post-seed (post-shuffle)
  // generator and start cells for the current base seed (the reset cache, rmx::start_cache_bytes layout), rebuilt
  // whenever the base seed changes
  bool seed_fixed = false;
  unsigned char* d_rsc = nullptr;
  // the base seed changed without a launch on a caller stream (rmx_reset_sync): the start cache and the next-episode
  // precompute tags are brought up to date on the stream of the next fast launch, ahead of it
  bool rs_stale = false;
  // the rng columns may hold generators of another base seed than the cache's (rmx::FastParams::rs_dirty)
  bool rs_dirty = true;
  // resident host-boundary stepper (rmx_reset_sync / rmx_step_sync, rmx_sync.hip): the pinned coherent mailbox,
  // its own non-blocking stream, the completion event of the last launch and the request numbering
  unsigned char* sy_mb = nullptr;
  size_t sy_bytes = 0;
  rmx::SyncIO sy_io{};
  hipStream_t sy_stream = nullptr;
  hipEvent_t sy_done = nullptr, sy_dep = nullptr;
  bool sy_running = false;  // a resident workgroup may be executing (sy_done not yet observed complete)
  bool sy_pending = false;  // a request is posted and not yet acknowledged (rmx_step_sync_begin)
  void* sy_caller = nullptr;  // the caller's stream of the outstanding request (a relaunch orders after it)
  uint32_t sy_seq = 0;      // last request posted
  uint32_t sy_served = 0;   // requests up to this number need no service (seq0 of the next launch)
  int sy_oneshot = 0;       // RMX_SYNC=launch: one launch per request (A/B of the resident workgroup)
  uint64_t sy_idle_ticks = 0, sy_life_ticks = 0;
  bool sy_enc = false;  // the records' enc_state word is meaningful (every agent has an encoder stride)
#ifdef RMX_DIAG
  std::chrono::steady_clock::time_point sy_t_post;  // diag: when the last request was posted
  double sy_wait_ns = 0;                             // diag: post -> acknowledgement seen by the host
#endif
};

namespace {

rmx::KParams base_params(const rmx_handle* h) {
  rmx::KParams p;
  std::memset(&p, 0, sizeof(p));
  const rmx_config& c = h->cfg;
  p.tables = reinterpret_cast<const uint4*>(h->d_tables);
  p.tables_n16 = (int32_t)(h->tables_bytes / 16);
  p.skip_same = h->generic_skip;  // the generic thread-per-env kernel: every unchanged word or none
  p.off_cell = h->off_cell;
  p.off_ev = h->off_ev;
  p.off_nq = h->off_nq;
  p.off_rr = h->off_rr;
  p.off_sh = h->off_sh;
  p.off_qrm = h->off_qrm;
  p.reward_modifier = c.reward_modifier;
  p.n_qrm_max = c.n_qrm_max;
  p.stochastic = c.stochastic ? 1 : 0;
  rmx::slip_fill(p, c);
  p.seed_scale = c.seed_scale;
  p.seed_env_stride = c.seed_env_stride;
  p.seed_episode_stride = c.seed_episode_stride;
  p.base_seed = h->base_seed;
  p.rng = h->buf.rng;
  p.episode = h->buf.episode;
  p.rng_on = (c.stochastic || c.random_starts) ? 1 : 0;
  p.random_starts = c.random_starts ? 1 : 0;
  p.n_free = h->n_free;
  p.free_cells = h->d_free;
  p.start_ws = h->d_start_ws;
  if (h->d_rsc) {
    p.rs_cells = reinterpret_cast<uint32_t*>(h->d_rsc);
    p.rs_rng = reinterpret_cast<uint64_t*>(h->d_rsc + rmx::start_cache_rng_off(c.n_agents, c.n_envs));
  }
  for (int a = 0; a < RMX_MAX_AGENTS; ++a) {
    p.n_qrm[a] = h->n_qrm[a];
    p.enc_nq[a] = h->enc_nq[a];
  }
  p.W = c.width;
  p.HW = c.width * c.height;
  p.A = c.n_agents;
  p.Q = c.n_rm_states;
  p.E = c.n_events;
  p.max_t = c.max_t;
  p.N = c.n_envs;
  p.hazard_penalty = c.hazard_penalty;
  p.wall_penalty = c.wall_penalty;
  p.hazard_fail = c.hazard_fail ? 1 : 0;
  p.wall_fail = c.wall_fail ? 1 : 0;
  p.has_shaping = c.has_shaping ? 1 : 0;
  p.gamma_is_one = (c.gamma == 1.0f) ? 1 : 0;
  for (int a = 0; a < RMX_MAX_AGENTS; ++a) {
    p.init_q[a] = h->init_q[a];
    p.final_q[a] = h->final_q[a];
    p.start_x[a] = h->start_x[a];
    p.start_y[a] = h->start_y[a];
  }
  p.disc = h->d_disc;
  p.pos_x = h->buf.pos_x;
  p.pos_y = h->buf.pos_y;
  p.rm_q = h->buf.rm_q;
  p.flags = h->buf.flags;
  p.ep_ret = h->buf.ep_ret;
  p.t = h->buf.t;
  p.reward = h->buf.reward;
  p.shaping = h->buf.shaping;
  p.env_done = h->buf.env_done;
  p.renv = h->buf.renv;
  p.enc_state = h->buf.enc_state;
  if (c.n_qrm_max > 0 && h->buf.qrm_s) {
    p.qrm_s = h->buf.qrm_s;
    p.qrm_sn = h->buf.qrm_sn;
    p.qrm_rq = h->buf.qrm_rq;
    p.qrm_done = h->buf.qrm_done;
  }
  p.env_offset = c.env_offset;
  p.n_global = c.n_envs_global;
  p.slab = h->d_slab;
  p.err = h->d_err;
  p.diag = h->diag;
  return p;
}

// Random starts, the wave-cooperative finish (rmx_fast.hip rs_coop_finish): output j of a PCG64 generator in one
// jump, state_j = M^j state + (1 + M + ... + M^(j-1)) inc (mod 2^128), for j = 1..64: M^j then the sum, each as
// 4 x u32 (low word first).  Placed after the precompute columns in the handle's d_nx allocation.
static size_t nx_jump_offset(int64_t n_envs) { return (40 * (size_t)n_envs + 255) & ~(size_t)255; }
struct RsJumpTable {
  uint32_t w[64][2][4];
  RsJumpTable() {
    typedef unsigned __int128 u128;
    const u128 M = ((u128)0x2360ED051FC65DA4ull << 64) | 0x4385DF649FCCF645ull;
    u128 mj = 1, sj = 0;
    for (int j = 0; j < 64; ++j) {
      sj += mj;  // 1 + M + ... + M^j
      mj *= M;   // M^(j+1)
      const u128 v[2] = {mj, sj};
      for (int k = 0; k < 2; ++k)
        for (int q = 0; q < 4; ++q) w[j][k][q] = (uint32_t)(v[k] >> (32 * q));
    }
  }
};
static const RsJumpTable rs_jump_table;

rmx::FastParams fast_params(const rmx_handle* h) {
  rmx::FastParams p;
  std::memset(&p, 0, sizeof(p));
  const rmx_config& c = h->cfg;
  p.tables = reinterpret_cast<const uint4*>(h->d_fast);
  p.n16 = h->fast_n16;
  p.off_rm = h->fast_off_rm;
  p.off_info = h->fast_off_info;
  p.A = c.n_agents;
  p.W = c.width;
  p.E = c.n_events;
  p.max_t = c.max_t;
  p.N = (int32_t)c.n_envs;
  for (int a = 0; a < c.n_agents; ++a) {
    p.mv_base[a] = a * c.width * c.height * 5;
    p.rm_base[a] = a * c.n_rm_states * c.n_events;
    p.final_q[a] = h->final_q[a];
    p.init_q[a] = h->init_q[a];
    p.start_x[a] = h->start_x[a];
    p.start_y[a] = h->start_y[a];
  }
  p.hazard_penalty = c.hazard_penalty;
  p.wall_penalty = c.wall_penalty;
  p.has_shaping = c.has_shaping ? 1 : 0;
  p.gamma_is_one = (c.gamma == 1.0f) ? 1 : 0;
  p.tbl_mode = h->fast_tables;
  p.H = c.height;
  p.hazard_fail = c.hazard_fail ? 1 : 0;
  p.wall_fail = c.wall_fail ? 1 : 0;
  p.merged = reinterpret_cast<const uint4*>(h->d_merged);
  p.merged4 = h->merged4_bytes ? reinterpret_cast<const uint32_t*>(static_cast<unsigned char*>(h->d_merged) + h->merged4_off)
                               : nullptr;
  p.merged4_bytes = (int32_t)h->merged4_bytes;
  std::memcpy(p.mg_palb, h->mg_palb, sizeof(p.mg_palb));
  p.merged_bytes = (int32_t)h->merged_bytes;
  if (c.n_qrm_max > 0 && h->buf.qrm_s) {
    p.qrm_s = h->buf.qrm_s;
    p.qrm_sn = h->buf.qrm_sn;
    p.qrm_rq = h->buf.qrm_rq;
    p.qrm_done = h->buf.qrm_done;
    p.n_qrm_max = c.n_qrm_max;
    for (int a = 0; a < c.n_agents; ++a) {
      p.n_qrm[a] = h->n_qrm[a];
      p.enc_nq[a] = h->enc_nq[a];
      for (int j = 0; j < c.n_qrm_max && j < rmx::kFastMaxQrm; ++j) p.qrm_q[a][j] = h->fast_qrm_q[a][j];
    }
  }
  p.HW = c.width * c.height;
  for (int a = 0; a < c.n_agents; ++a) {
    p.mg_base[a] = h->mg_base[a];
    p.enc_nq[a] = h->enc_nq[a];  // QRM outputs and enc_state
  }
  p.disc = h->d_disc;
  p.pos_x = h->buf.pos_x;
  p.pos_y = h->buf.pos_y;
  p.rm_q = h->buf.rm_q;
  p.flags = h->buf.flags;
  p.ep_ret = h->buf.ep_ret;
  p.t = h->buf.t;
  p.reward = h->buf.reward;
  p.shaping = h->buf.shaping;
  p.env_done = h->buf.env_done;
  p.renv = h->buf.renv;
  p.enc_state = h->buf.enc_state;
  p.env_offset = c.env_offset;
  p.n_global = c.n_envs_global;
  p.wave_stats = h->fast_wave_stats;
  p.skip_same = h->fast_skip;
  p.block = h->fast_block;
  p.slab = h->d_slab;
  p.es_ret = h->es_ret;
  p.es_cnt = h->es_cnt;
  p.es_succ = h->es_succ;
  p.err = h->d_err;
  p.diag = h->diag;
  p.stamps = h->d_stamps;
  if (c.stochastic || c.random_starts) {  // slip and / or FrozenLake random starts on the fast path
    p.slip = (c.stochastic ? rmx::kRngSlip : 0) | (c.random_starts ? rmx::kRngStarts : 0) |
             (h->seed_fixed ? rmx::kRngFixedSeed : 0);
    p.n_free = h->n_free;
    p.free_cells = h->d_free;
    p.start_ws = h->d_start_ws;
    if (h->d_rsc) {
      p.rs_cells = reinterpret_cast<const uint32_t*>(h->d_rsc);
      p.rs_rng = reinterpret_cast<const uint64_t*>(h->d_rsc + rmx::start_cache_rng_off(c.n_agents, c.n_envs));
      p.rs_dirty = h->rs_dirty ? 1 : 0;
    }
    if (h->d_nx) {
      const size_t N = (size_t)c.n_envs;
      p.nx_rng = reinterpret_cast<uint64_t*>(h->d_nx);
      p.nx_idx = reinterpret_cast<int32_t*>(h->d_nx + 32 * N);
      p.nx_ep = reinterpret_cast<int32_t*>(h->d_nx + 36 * N);
      p.rs_jump = reinterpret_cast<const uint4*>(h->d_nx + nx_jump_offset(c.n_envs));
    }
    rmx::slip_fill(p, c);
    p.seed_scale = c.seed_scale;
    p.seed_env_stride = c.seed_env_stride;
    p.seed_episode_stride = c.seed_episode_stride;
    p.base_seed = h->base_seed;
    p.rng = h->buf.rng;
    p.episode = h->buf.episode;
  }
  return p;
}

// The fast kernels run unless QRM outputs are bound with more experiences per agent than they emit.
// With QRM outputs they run thread-per-env with the global tables (the move word carries the event the
// counterfactual RM lookups need).
bool fast_applies(const rmx_handle* h) {
  if (h->fast && (h->cfg.stochastic || h->cfg.random_starts)) {  // slip / random starts: the SLIP instantiations only
    const int tm = h->fast_tables;
    return !h->buf.qrm_s && h->fast_skip == rmx::kSkipRare && (tm == rmx::kTblMerged4 || tm == rmx::kTblMerged) &&
           h->cfg.n_envs < ((int64_t)1 << 27) &&
           // the next-episode precompute's one-byte rows (the fixed-start cache has no rows)
           (!h->cfg.random_starts || h->seed_fixed || h->n_free + 8 <= rmx::kRsRowMax);
  }
  const int qmax = h->cfg.n_agents <= 2 ? rmx::kFastMaxQrm : 8;  // register budget of the QRM lookups
  // QRM columns are [A][Qx][N]: their byte offsets must stay 32-bit as well
  return h->fast && (!h->buf.qrm_s || (h->cfg.n_qrm_max <= qmax &&
                                       (int64_t)h->cfg.n_qrm_max * h->cfg.n_agents * h->cfg.n_envs < ((int64_t)1 << 30)));
}

hipError_t reduce_stats(const rmx_handle* h, double* out, hipStream_t st) {
  double* partial = h->d_slab + (size_t)RMX_NSTATS * h->n_waves;
  unsigned int* ticket = reinterpret_cast<unsigned int*>(partial + (size_t)RMX_NSTATS * 2 * rmx::kStatsPartials);
  return rmx::launch_stats_reduce(h->d_slab, h->n_waves, h->es_ret, h->es_cnt, h->es_succ, h->cfg.n_envs, partial,
                                  ticket, out, st);
}

int validate(const rmx_config* c) {
  if (!c) return fail(RMX_E_INVALID, "config is NULL");
  const std::string msg = rmx::validate_config(*c);
  return msg.empty() ? RMX_OK : fail(RMX_E_INVALID, msg);
}

hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

int check_bound(const rmx_handle* h) {
  if (!h) return fail(RMX_E_INVALID, "handle is NULL");
  if (!h->bound) return fail(RMX_E_STATE, "buffers not bound (rmx_bind)");
  return RMX_OK;
}

int64_t threads_for(const rmx_handle* h, int layout) {
  return layout == rmx::kLayoutLanePerAgent ? h->cfg.n_envs * rmx::lanes_per_env(h->cfg.n_agents) : h->cfg.n_envs;
}

dim3 grid_for(const rmx_handle* h, int layout) {
  return dim3((unsigned)((threads_for(h, layout) + h->block - 1) / h->block));
}

// rmx_get_state / rmx_set_state blob: header, then the columns in this order (agent-major [A][N] each):
// pos_x i32, pos_y i32, rm_q i32, flags u32, ep_ret f32, t i32 [N], and when the rng columns are bound
// rng u64 [4][N], episode i32 [N].
struct StateHeader {
  char magic[8];  // "RMXSTATE"
  uint32_t version, has_rng;
  int64_t n_agents, n_envs;
  uint64_t base_seed;
  double stats[RMX_NSTATS];
  uint64_t digest;  // config_digest of the handle that wrote the blob (version 2)
  int64_t env_offset, n_envs_global;
};
constexpr uint32_t kStateVersion = 2;

struct StateCol {
  void* dev;
  size_t bytes;
};

int state_columns(const rmx_handle* h, std::vector<StateCol>& cols, bool& has_rng) {
  const size_t AN = (size_t)h->cfg.n_agents * h->cfg.n_envs, N = (size_t)h->cfg.n_envs;
  const rmx_buffers& b = h->buf;
  has_rng = b.rng != nullptr && b.episode != nullptr;
  cols = {{b.pos_x, 4 * AN}, {b.pos_y, 4 * AN}, {b.rm_q, 4 * AN}, {b.flags, 4 * AN}, {b.ep_ret, 4 * AN}, {b.t, 4 * N}};
  if (has_rng) {
    cols.push_back({b.rng, 32 * N});
    cols.push_back({b.episode, 4 * N});
  }
  return RMX_OK;
}

size_t state_blob_bytes(const std::vector<StateCol>& cols) {
  size_t n = sizeof(StateHeader);
  for (const auto& c : cols) n += c.bytes;
  return n;
}

// ---- resident host-boundary stepper (rmx_sync.hip) -----------------------------------------------------------
inline void cpu_relax() { __builtin_ia32_pause(); }

// Mailbox layout: request line | acknowledgement line | actions [A][N] | output columns in rmx_buffers order.
// The stream and the two events are created once per handle (rmx_bind frees only the mailbox, whose QRM sections
// follow the bound buffers); h->sy_mb is set last, so a failure part way leaves the next call to start over.
int sync_setup(rmx_handle* h) {
  if (h->sy_mb) return RMX_OK;
  HIP_TRY(hipSetDevice(h->device), "hipSetDevice");
  if (!h->sy_stream) HIP_TRY(hipStreamCreateWithFlags(&h->sy_stream, hipStreamNonBlocking), "resident stream");
  if (!h->sy_done) HIP_TRY(hipEventCreateWithFlags(&h->sy_done, hipEventDisableTiming), "resident event");
  if (!h->sy_dep) HIP_TRY(hipEventCreateWithFlags(&h->sy_dep, hipEventDisableTiming), "resident event");
  int khz = 0;
  HIP_TRY(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, h->device), "wall clock rate");
  const size_t A = (size_t)h->cfg.n_agents, N = (size_t)h->cfg.n_envs, AN = A * N;
  const size_t Qx = h->buf.qrm_s ? (size_t)h->cfg.n_qrm_max : 0;
  bool enc = true;
  for (int a = 0; a < h->cfg.n_agents; ++a) enc = enc && h->enc_nq[a] >= 1;
  size_t off = sizeof(rmx::SyncReq) + sizeof(rmx::SyncAck);
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off = (off + bytes + 15) & ~size_t(15);
    return o;
  };
  const size_t o_act = take(4 * AN), o_rec = take(32 * AN), o_env = take(16 * N);
  const size_t o_qs = Qx ? take(4 * AN * Qx) : 0, o_qsn = Qx ? take(4 * AN * Qx) : 0;
  const size_t o_qrq = Qx ? take(4 * AN * Qx) : 0, o_qd = Qx ? take(AN * Qx) : 0;
  h->sy_enc = enc;
  void* mb = nullptr;
  HIP_TRY(hipHostMalloc(&mb, off, hipHostMallocCoherent | hipHostMallocMapped), "mailbox hipHostMalloc");
  std::memset(mb, 0, off);
  void* dmb = nullptr;
  hipError_t e = hipHostGetDevicePointer(&dmb, mb, 0);
  if (e != hipSuccess) {
    (void)hipHostFree(mb);
    return hip_fail(e, "mailbox device pointer");
  }
  h->sy_bytes = off;
  unsigned char* d = static_cast<unsigned char*>(dmb);
  rmx::SyncIO& io = h->sy_io;
  io.req = reinterpret_cast<rmx::SyncReq*>(d);
  io.ack = reinterpret_cast<rmx::SyncAck*>(d + sizeof(rmx::SyncReq));
  io.act = reinterpret_cast<const int32_t*>(d + o_act);
  io.out = {reinterpret_cast<uint4*>(d + o_rec), reinterpret_cast<uint4*>(d + o_env),
            Qx ? reinterpret_cast<int32_t*>(d + o_qs) : nullptr, Qx ? reinterpret_cast<int32_t*>(d + o_qsn) : nullptr,
            Qx ? reinterpret_cast<float*>(d + o_qrq) : nullptr, Qx ? reinterpret_cast<uint8_t*>(d + o_qd) : nullptr};
  h->sy_mb = static_cast<unsigned char*>(mb);
  const double ticks_per_us = khz > 0 ? khz / 1000.0 : 100.0;
  double idle_us = 2000.0, life_ms = 10000.0;
  if (const char* v = std::getenv("RMX_SYNC_IDLE_US")) idle_us = std::max(0.0, std::atof(v));
  if (const char* v = std::getenv("RMX_SYNC_LIFE_MS")) life_ms = std::max(0.0, std::atof(v));
  if (const char* v = std::getenv("RMX_SYNC")) h->sy_oneshot = !std::strcmp(v, "launch") ? 1 : 0;
  h->sy_idle_ticks = (uint64_t)(idle_us * ticks_per_us);
  h->sy_life_ticks = h->sy_oneshot ? 0 : (uint64_t)(life_ms * 1000.0 * ticks_per_us);
  return RMX_OK;
}

// A host pointer into the mailbox for device pointer dp (the mailbox is mapped: same bytes, maybe another address).
template <typename T>
T* mb_host(const rmx_handle* h, T* dp) {
  const unsigned char* d0 = reinterpret_cast<const unsigned char*>(h->sy_io.req);
  return dp ? reinterpret_cast<T*>(h->sy_mb + (reinterpret_cast<const unsigned char*>(dp) - d0)) : nullptr;
}

int sync_launch(rmx_handle* h, void* stream) {
  // start after the work already enqueued on the caller's stream (e.g. the reset that wrote the columns)
  HIP_TRY(hipEventRecord(h->sy_dep, as_stream(stream)), "resident dependency");
  HIP_TRY(hipStreamWaitEvent(h->sy_stream, h->sy_dep, 0), "resident dependency");
  rmx::KParams p = base_params(h);
  rmx::SyncIO io = h->sy_io;
  io.seq0 = h->sy_served;
  io.idle_ticks = h->sy_idle_ticks;
  io.life_ticks = h->sy_life_ticks;
  HIP_TRY(rmx::launch_resident(p, io, h->cfg.kind, (int)h->cfg.n_envs, h->tables_bytes, h->sy_stream), "resident launch");
  HIP_TRY(hipEventRecord(h->sy_done, h->sy_stream), "resident event");
  h->sy_running = true;
  return RMX_OK;
}

// The request word {seq, ctl, acts, seq} goes out as ONE aligned 16-B store (x86: atomic for aligned 16-B
// vector stores), after everything it refers to (the action array, the seed): stores retire in order.
void sync_post(rmx_handle* h, uint32_t ctl, uint32_t acts) {
  rmx::SyncReq* r = mb_host(h, h->sy_io.req);
  const uint32_t seq = h->sy_seq + 1;
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  _mm_store_si128(reinterpret_cast<__m128i*>(r), _mm_set_epi32((int)seq, (int)acts, (int)ctl, (int)seq));
  h->sy_seq = seq;
}

// Post one request (launching the resident workgroup if none is running) without waiting for it.
int sync_begin(rmx_handle* h, uint32_t op, uint32_t autoreset, uint64_t seed, const int32_t* actions, void* stream) {
  uint32_t ctl = op | (autoreset ? rmx::kSyncAutoreset : 0u), acts = 0;
  if (op == rmx::kSyncReset) mb_host(h, h->sy_io.req)->seed = seed;
  if (actions) {
    const int64_t n = (int64_t)h->cfg.n_agents * h->cfg.n_envs;
    if (n <= rmx::kSyncInlineActs) {  // inline: 4-bit fields, k < 7 in ctl from bit 4, the rest in acts
      ctl |= rmx::kSyncInline;
      for (int64_t k = 0; k < n; ++k) {
        const uint32_t a = (uint32_t)actions[k] <= (uint32_t)RMX_WAIT ? (uint32_t)actions[k] : rmx::kSyncBadAct;
        if (k < 7)
          ctl |= a << (4 + 4 * k);
        else
          acts |= a << (4 * (k - 7));
      }
    } else {
      std::memcpy(const_cast<int32_t*>(mb_host(h, h->sy_io.act)), actions, sizeof(int32_t) * n);
    }
  }
  sync_post(h, ctl, acts);
#ifdef RMX_DIAG
  h->sy_t_post = std::chrono::steady_clock::now();
#endif
  h->sy_pending = true;
  h->sy_caller = stream;
  if (!h->sy_running) {
    HIP_TRY(hipSetDevice(h->device), "hipSetDevice");
    return sync_launch(h, stream);
  }
  return RMX_OK;
}

// Wait for the posted request's acknowledgement.  A workgroup that timed out before it saw the request is
// relaunched with seq0 = the last served request, so the pending one is served exactly once.
int sync_wait(rmx_handle* h) {
  if (!h->sy_pending) return fail(RMX_E_STATE, "no synchronous request is outstanding");
  const rmx::SyncAck* ack = mb_host(h, h->sy_io.ack);
  const uint32_t seq = h->sy_seq;
  int rc;
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  for (unsigned spins = 1;; ++spins) {
    if (__atomic_load_n(&ack->seq, __ATOMIC_ACQUIRE) == seq) break;
    if ((spins & 63u) == 0) {
      const auto el = clk::now() - t0;
      if (el > std::chrono::microseconds(20)) {  // a normal round trip is a few us: has the workgroup exited?
        const hipError_t q = hipEventQuery(h->sy_done);
        if (q == hipSuccess) {
          if (__atomic_load_n(&ack->seq, __ATOMIC_ACQUIRE) == seq) break;
          h->sy_running = false;
          HIP_TRY(hipSetDevice(h->device), "hipSetDevice");
          if ((rc = sync_launch(h, h->sy_caller))) return rc;
        } else if (q != hipErrorNotReady) {
          h->sy_running = false;
          h->sy_pending = false;
          return hip_fail(q, "resident stepper");
        }
        if (el > std::chrono::seconds(30)) return fail(RMX_E_HIP, "resident stepper did not acknowledge in 30 s");
      }
    }
    cpu_relax();
  }
#ifdef RMX_DIAG
  h->sy_wait_ns = std::chrono::duration<double, std::nano>(clk::now() - h->sy_t_post).count();
#endif
  h->sy_served = seq;
  h->sy_pending = false;
  if (h->sy_oneshot) {  // the workgroup exits by itself after one request: wait for it, relaunch on the next
    HIP_TRY(hipEventSynchronize(h->sy_done), "resident exit");
    h->sy_running = false;
  }
  return RMX_OK;
}

int sync_request(rmx_handle* h, uint32_t op, uint32_t autoreset, uint64_t seed, const int32_t* actions, void* stream) {
  const int rc = sync_begin(h, op, autoreset, seed, actions, stream);
  return rc ? rc : sync_wait(h);
}

// End the resident workgroup (if any): the device columns are current afterwards.
int sync_end(rmx_handle* h) {
  if (h && h->sy_pending) {  // a begun request is served first
    const int rc = sync_wait(h);
    if (rc) return rc;
  }
  if (!h || !h->sy_running) return RMX_OK;
  sync_post(h, rmx::kSyncExit, 0);
  h->sy_running = false;
  h->sy_served = h->sy_seq;  // nobody serves an exit request; later launches skip it
  HIP_TRY(hipEventSynchronize(h->sy_done), "resident exit");
  return RMX_OK;
}

#define SYNC_END_OR_RETURN(h)   \
  do {                          \
    const int _rc = sync_end(h); \
    if (_rc) return _rc;        \
  } while (0)

// Unpack the columns the caller asked for from the mailbox's records; a requested column the handle does not
// compute fails.
int sync_copy_out(const rmx_handle* h, const rmx_buffers* out) {
  if (!out) return RMX_OK;
  const int64_t A = h->cfg.n_agents, N = h->cfg.n_envs;
  const size_t AQN = (size_t)(A * N) * (size_t)(h->buf.qrm_s ? h->cfg.n_qrm_max : 0);
  const rmx::SyncCols& c = h->sy_io.out;
  if (out->shaping && !h->cfg.has_shaping) return fail(RMX_E_STATE, "sync output column not computed: shaping");
  if (out->enc_state && !h->sy_enc) return fail(RMX_E_STATE, "sync output column not computed: enc_state");
  if ((out->qrm_s || out->qrm_sn || out->qrm_rq || out->qrm_done) && !c.qrm_s)
    return fail(RMX_E_STATE, "sync output columns not computed: QRM (bind the QRM columns)");
  const uint4* rec = mb_host(h, c.rec);
  const uint4* env = mb_host(h, c.envrec);
  auto f32 = [](uint32_t v) {
    float f;
    std::memcpy(&f, &v, 4);
    return f;
  };
  for (int64_t e = 0; e < N; ++e) {
    if (out->t) out->t[e] = (int32_t)env[e].x;
    if (out->env_done) out->env_done[e] = (uint8_t)env[e].y;
    for (int64_t a = 0; a < A; ++a) {
      const uint4 w0 = rec[2 * (e * A + a)], w1 = rec[2 * (e * A + a) + 1];
      const int64_t k = a * N + e;
      if (out->pos_x) out->pos_x[k] = (int32_t)(w0.x & 0xFFFFu);
      if (out->pos_y) out->pos_y[k] = (int32_t)(w0.x >> 16);
      if (out->rm_q) out->rm_q[k] = (int32_t)w0.y;
      if (out->flags) out->flags[k] = w0.z;
      if (out->reward) out->reward[k] = f32(w0.w);
      if (out->renv) out->renv[k] = f32(w1.x);
      if (out->ep_ret) out->ep_ret[k] = f32(w1.y);
      if (out->shaping) out->shaping[k] = f32(w1.z);
      if (out->enc_state) out->enc_state[k] = (int32_t)w1.w;
    }
  }
  if (out->qrm_s) std::memcpy(out->qrm_s, mb_host(h, c.qrm_s), 4 * AQN);
  if (out->qrm_sn) std::memcpy(out->qrm_sn, mb_host(h, c.qrm_sn), 4 * AQN);
  if (out->qrm_rq) std::memcpy(out->qrm_rq, mb_host(h, c.qrm_rq), 4 * AQN);
  if (out->qrm_done) std::memcpy(out->qrm_done, mb_host(h, c.qrm_done), AQN);
  return RMX_OK;
}

int sync_check(rmx_handle* h) {
  int rc = check_bound(h);
  if (rc) return rc;
  if (h->cfg.n_envs > RMX_SYNC_MAX_ENVS)
    return fail(RMX_E_INVALID, "rmx_*_sync serve shards of at most RMX_SYNC_MAX_ENVS envs");
  return sync_setup(h);
}

// ---- host handles (cfg.device == RMX_DEVICE_HOST, rmx_hoststep.cpp) ------------------------------------------
int create_host(const rmx_config* cfg, rmx_handle** out) {
  rmx_handle* h = new rmx_handle();
  h->host = new rmx::HostEngine();
  const std::string msg = h->host->init(*cfg);
  if (!msg.empty()) {
    delete h->host;
    delete h;
    return fail(RMX_E_INVALID, msg);
  }
  h->cfg = h->host->cfg;  // scalars only
  h->device = RMX_DEVICE_HOST;
  h->digest = rmx::config_digest(*cfg);
  for (int a = 0; a < cfg->n_agents; ++a) h->enc_nq[a] = h->host->enc_nq[a];
  *out = h;
  return RMX_OK;
}

// The synchronous calls on a host handle: the step runs in rmx_step_sync_begin, rmx_sync_wait returns its outputs.
int host_sync_out(rmx_handle* h, const rmx_buffers* out, uint32_t bad) {
  if (out) {
    const std::string msg = h->host->copy_out(*out);
    if (!msg.empty()) return fail(RMX_E_STATE, msg);
  }
  if (bad) return fail(RMX_E_ACTION, "an action outside [0,4] (or wait under FrozenLake slip) was stepped (treated as wait)");
  return RMX_OK;
}

}  // namespace

extern "C" {

int rmx_abi_version(void) { return RMX_ABI_VERSION; }

int rmx_device_count(int32_t* n) {
  if (!n) return fail(RMX_E_INVALID, "n is NULL");
  int c = 0;
  const hipError_t e = hipGetDeviceCount(&c);
  *n = e == hipSuccess ? c : 0;  // no driver / no device: 0 (a host handle still works)
  return RMX_OK;
}

const char* rmx_last_error(void) { return g_err.c_str(); }

int rmx_create(const rmx_config* cfg, rmx_handle** out) {
  if (!out) return fail(RMX_E_INVALID, "out is NULL");
  *out = nullptr;
  int rc = validate(cfg);
  if (rc) return rc;
  if (cfg->device == RMX_DEVICE_HOST) {
    try {
      return create_host(cfg, out);
    } catch (const std::exception& e) {  // allocation: nothing may unwind through the C ABI
      return fail(RMX_E_INVALID, std::string("rmx_create (host): ") + e.what());
    }
  }
  if (cfg->device < 0) return fail(RMX_E_INVALID, "device must be a HIP device ordinal or RMX_DEVICE_HOST");
  HIP_TRY(hipSetDevice(cfg->device), "hipSetDevice");
  rmx_handle* h = new rmx_handle();
  h->cfg = *cfg;
  h->device = cfg->device;
  if (const char* qv = std::getenv("RMX_QUEUE")) h->queue_off = std::strcmp(qv, "0") == 0;
  if (const char* b = std::getenv("RMX_BLOCK")) {
    int v = std::atoi(b);
    if (v == 64 || v == 128 || v == 256) h->block = v;
  }
#ifdef RMX_DIAG
  if (const char* d = std::getenv("RMX_DIAG_BITS")) h->diag = std::atoi(d);
#endif
  // per-env rng (slip, random starts): one env rng, agents draw in order -> thread-per-env kernels only
  const bool rng_on = cfg->stochastic || cfg->random_starts;
  if (rng_on) h->rollout_layout = rmx::kLayoutThreadPerEnv;
  if (const char* l = std::getenv("RMX_LAYOUT")) {  // test / tuning override for both kernels
    if (!std::strcmp(l, "tpe")) h->step_layout = h->rollout_layout = rmx::kLayoutThreadPerEnv;
    if (!std::strcmp(l, "lpe") && !rng_on) h->step_layout = h->rollout_layout = rmx::kLayoutLanePerAgent;
  }
  const int A = cfg->n_agents;
  for (int a = 0; a < A; ++a) {
    h->init_q[a] = cfg->init_q[a];
    h->final_q[a] = cfg->final_q[a];
    h->start_x[a] = cfg->start_xy[2 * a];
    h->start_y[a] = cfg->start_xy[2 * a + 1];
  }
  // table blob of the generic kernels (rmx_tables.cpp)
  std::vector<unsigned char> blob;
  rmx::BlobOffsets bo;
  if (!rmx::build_table_blob(*cfg, blob, bo)) {
    delete h;
    return fail(RMX_E_INVALID, "tables exceed 64 KiB of LDS");
  }
  h->tables_bytes = blob.size();
  h->digest = rmx::config_digest(*cfg);
  h->off_cell = bo.cell;
  h->off_ev = bo.ev;
  h->off_nq = bo.nq;
  h->off_rr = bo.rr;
  h->off_sh = bo.sh;
  h->off_qrm = bo.qrm;
  if (cfg->n_qrm_max > 0) {
    for (int a = 0; a < A; ++a) {
      h->n_qrm[a] = cfg->n_qrm[a];
      for (int j = 0; j < cfg->n_qrm_max && j < rmx::kFastMaxQrm; ++j)
        h->fast_qrm_q[a][j] = cfg->qrm_states[a * cfg->n_qrm_max + j];
    }
  }
  for (int a = 0; a < A; ++a) h->enc_nq[a] = cfg->enc_nq ? cfg->enc_nq[a] : 0;
  const std::vector<float> disc = rmx::discount_table(*cfg);
  // FrozenLake random starts: the non-hole cells (x-major) and a per-env shuffle workspace
  std::vector<uint16_t> free_cells;
  if (cfg->random_starts) free_cells = rmx::free_cells(*cfg);
  h->n_free = (int32_t)free_cells.size();
  // one slab slot per wave of the larger of the two launch geometries
  const int64_t gmax = std::max(grid_for(h, h->step_layout).x, grid_for(h, h->rollout_layout).x);
  std::vector<unsigned char> fast_blob;
  std::vector<uint32_t> merged_tab;
  hipError_t e0 = hipSuccess;
  {
    // RMX_FAST=0: generic kernels only (tests / A-B timing)
    const char* fe = std::getenv("RMX_FAST");
    // RMX_FAST=0: generic only; default: the fast path wherever it applies
    const bool want = fe ? std::strcmp(fe, "0") != 0 : true;
    rmx::FastLayout fl;
    h->fast = want && h->step_layout == rmx::kLayoutThreadPerEnv && rmx::build_fast_blob(*cfg, fast_blob, fl);
    h->fast_off_rm = fl.off_rm;
    h->fast_off_info = fl.off_info;
    h->fast_n16 = (int32_t)(fast_blob.size() / 16);
    // Default table mode, measured at 65,536 envs (profiles/r01_ab_log.md c25, c26): the merged single
    // lookup while its table is small (<= 64 KiB: config 2 3.06 vs 3.10-3.15 us global, config 3 2.50-2.54
    // vs 2.75-2.78 global and 2.55-2.60 lane-resident), the global blob for larger tables (config 4 equal,
    // config 5 3.67 global vs 3.81-3.87 merged).
    // The size that decides is the deduplicated one (identical agent sections stored once).
    if (h->fast) {
      std::vector<uint32_t> probe;
      const bool ok = rmx::build_merged(*cfg, fast_blob, h->fast_off_rm, h->mg_base, probe);
      h->fast_tables = ok && probe.size() * 4 <= kFastMergedDefaultBytes ? rmx::kTblMerged : rmx::kTblGlobal;
      // 4-B records (reward from a <= 4-entry palette, no shaping): config 2 3.28-3.30 vs 3.36-3.37 us on one
      // box, equal on another; config 3 2.51-2.52 vs 2.68-2.71; config 4 4.18-4.22 vs 4.25-4.28 (r01_ab_log
      // c75, c77; 8-B {word 0, reward} records gain less).  Falls back to the 16-B records below when the
      // config is not eligible.
      // FrozenLake slip keeps the 16-B records: config 2 with slip 4.62-4.64 vs 4.78-4.84 us with 4-B records,
      // config 4 equal (r02_ab_log slipint, r02aq)
      if (h->fast_tables == rmx::kTblMerged && !cfg->stochastic) h->fast_tables = rmx::kTblMerged4;
    }
    // test override of the default (the results do not depend on it): RMX_FAST_TABLES=global|merged|merged4
    if (const char* ft = std::getenv("RMX_FAST_TABLES")) {
      if (!std::strcmp(ft, "global")) h->fast_tables = rmx::kTblGlobal;
      if (!std::strcmp(ft, "merged")) h->fast_tables = rmx::kTblMerged;
      if (!std::strcmp(ft, "merged4")) h->fast_tables = rmx::kTblMerged4;
    }
    const bool want_m4 = h->fast_tables == rmx::kTblMerged4;
    if (h->fast && (h->fast_tables == rmx::kTblMerged || want_m4) &&
        !rmx::build_merged(*cfg, fast_blob, h->fast_off_rm, h->mg_base, merged_tab))
      h->fast_tables = rmx::kTblGlobal;  // table too large: one lookup per stage
    if (want_m4 && h->fast_tables != rmx::kTblGlobal) {  // the compact records follow the 16-B ones
      std::vector<uint32_t> compact;
      // the step kernel reads the palette as signed bytes: integer rewards in [-128, 127] (every BASELINE config's);
      // other palettes take the 16-B records
      if (rmx::build_compact(*cfg, h->mg_base, merged_tab, h->mg_palb, compact)) {
        h->merged4_off = merged_tab.size() * 4;
        h->merged4_bytes = compact.size() * 4;
        merged_tab.insert(merged_tab.end(), compact.begin(), compact.end());
        while (merged_tab.size() % 4) merged_tab.push_back(0u);
      } else {
        h->fast_tables = rmx::kTblMerged;  // shaping or > 4 distinct rewards: the 16-B records
      }
    }
  }
  // slip / random starts under seed_episode_stride == 0 (the reference FrozenLake runner's reset(args.seed) every
  // episode, frozen_lake_main.py:337): every episode of an env starts from the same generator and shuffle, so the
  // fast kernels copy a cached one at each autoreset instead of reseeding and redrawing (h->fast: A <= 4, cells fit
  // the cache's 8-bit x / y)
  h->seed_fixed = h->fast && (cfg->stochastic || cfg->random_starts) && cfg->seed_episode_stride == 0;
  // one slab slot per wave of the largest launch geometry (the fast kernels use 256-thread blocks)
  h->n_waves = std::max<int64_t>(gmax * (h->block / 64), (cfg->n_envs + 255) / 256 * 4);
  h->fast_wave_stats = cfg->n_envs >= kFastWaveStatsMinEnvs ? 1 : 0;
  if (const char* fs = std::getenv("RMX_FAST_STATS")) h->fast_wave_stats = !std::strcmp(fs, "wave") ? 1 : 0;
  // fast kernel: rm_q / ep_ret stores skipped when unchanged at every size (65,536 envs: 3-5 % faster than
  // storing every word; 8.4M envs: 10-17 % faster than skipping every unchanged word, whose partial-line writes
  // of the x / y / flags columns cost more than they save; profiles/r02_ab_log.md ab3, ab4, abbig).  The generic
  // kernel (slip, random starts, A > 4) skips every unchanged word from 1M envs on (round 1, c55).
  // Once a step's columns outgrow the 256 MB Infinity Cache (>= 2^23 env x agent instances, ~440 MB per step) the
  // same stores carry the non-temporal hint (kSkipRareNT): 8.4M envs 6-24 % faster on all four configs, while at
  // 1-2M envs it is mixed (configs 3 and 5 slower) and at 65,536 envs 7-8 % slower (profiles/r02_ab_log.md pol, nt).
  h->fast_skip = cfg->n_envs * (int64_t)cfg->n_agents >= kFastNtMinInstances ? rmx::kSkipRareNT : rmx::kSkipRare;
  h->generic_skip = cfg->n_envs >= kFastSkipMinEnvs ? 1 : 0;
  // test override: RMX_FAST_SKIP=3 puts the bandwidth regime's non-temporal store mode under test at smaller sizes,
  // 2 the default store mode at larger ones (the other store modes lost their A/Bs and were removed, round 5)
  if (const char* fk = std::getenv("RMX_FAST_SKIP")) {
    const int v = std::atoi(fk);
    if (v == rmx::kSkipRare || v == rmx::kSkipRareNT) h->fast_skip = v;
  }
  // test override of the generic kernel's store mode (every unchanged word skipped: its default from 1M envs)
  if (const char* gk = std::getenv("RMX_GENERIC_SKIP")) h->generic_skip = std::atoi(gk) ? 1 : 0;
  // 64-thread workgroups at the headline size (1-3 % faster on all four configs, r01_ab_log c48), 256 in the
  // bandwidth regime (64: 15-20 % slower at 8.4M envs, c49)
  h->fast_block = cfg->n_envs >= kFastSkipMinEnvs ? 256 : 64;
  if (const char* rl = std::getenv("RMX_ROLLOUT_LDS")) h->rollout_lds = std::atoi(rl) ? 1 : 0;
#ifdef RMX_DIAG
  if (std::getenv("RMX_DIAG_STAMPS") && e0 == hipSuccess) {
    const size_t n = ((size_t)cfg->n_envs + 255) / 256 * 4 * 2 * rmx::kStamps;
    e0 = hipMalloc(&h->d_stamps, n * 8);
    if (e0 == hipSuccess) e0 = hipMemset(h->d_stamps, 0, n * 8);
  }
#endif
  if (h->fast && !h->fast_wave_stats) {  // per-env slots only in the per-env stats mode (wave mode: the slab)
    // one row [N] each: both fast layouts sum an env's agents before its one adder
    const size_t N = (size_t)cfg->n_envs;
    const size_t o_cnt = 8 * N, o_succ = o_cnt + 8 * N, o_part = (o_succ + 4 * N + 15) & ~size_t(15);
    const size_t o_ticket = (o_part + sizeof(double) * RMX_NSTATS * ((N + 63) / 64) + 127) & ~size_t(127);
    h->es_bytes = o_ticket + 128 * (1 + 32);  // root + 32 shard counters, one 128-B line each (rmx_fast.hip)
    e0 = hipMalloc(&h->d_es, h->es_bytes);
    if (e0 == hipSuccess) e0 = hipMemset(h->d_es, 0, h->es_bytes);
    if (e0 == hipSuccess) {
      h->es_ret = reinterpret_cast<double*>(h->d_es);
      h->es_cnt = reinterpret_cast<unsigned long long*>(h->d_es + o_cnt);
      h->es_succ = reinterpret_cast<uint32_t*>(h->d_es + o_succ);
      h->rpt_partial = reinterpret_cast<double*>(h->d_es + o_part);
      h->rpt_ticket = reinterpret_cast<unsigned int*>(h->d_es + o_ticket);
    }
  }
  hipError_t e;
  if ((e = e0) != hipSuccess || (e = hipMalloc(&h->d_tables, h->tables_bytes)) != hipSuccess ||
      (e = hipMemcpy(h->d_tables, blob.data(), h->tables_bytes, hipMemcpyHostToDevice)) != hipSuccess ||
      (e = hipMalloc(&h->d_disc, sizeof(float) * disc.size())) != hipSuccess ||
      (e = hipMemcpy(h->d_disc, disc.data(), sizeof(float) * disc.size(), hipMemcpyHostToDevice)) != hipSuccess ||
      // slab | 2 * kStatsPartials partial vectors | the stats launch's ticket (zeroed, re-armed by every report)
      (e = hipMalloc(&h->d_slab, sizeof(double) * (RMX_NSTATS * (h->n_waves + 2 * rmx::kStatsPartials) + 2))) != hipSuccess ||
      (e = hipMemset(h->d_slab, 0, sizeof(double) * (RMX_NSTATS * (h->n_waves + 2 * rmx::kStatsPartials) + 2))) != hipSuccess ||
      (e = hipMalloc(&h->d_stats, sizeof(double) * RMX_NSTATS)) != hipSuccess ||
      (e = hipMalloc(&h->d_err, sizeof(uint32_t))) != hipSuccess ||
      (e = hipMemset(h->d_err, 0, sizeof(uint32_t))) != hipSuccess ||
      (h->n_free > 0 &&
       // (padded to whole dwords: the fast path stages the cells as u16 pairs)
       ((e = hipMalloc(&h->d_free, sizeof(uint16_t) * (free_cells.size() + 1))) != hipSuccess ||
        (e = hipMemset(h->d_free, 0, sizeof(uint16_t) * (free_cells.size() + 1))) != hipSuccess ||
        (e = hipMemcpy(h->d_free, free_cells.data(), sizeof(uint16_t) * free_cells.size(), hipMemcpyHostToDevice)) !=
            hipSuccess ||
        (e = hipMalloc(&h->d_start_ws, sizeof(uint16_t) * (size_t)rmx::shuffle_stride((int32_t)free_cells.size()) *
                                              (size_t)cfg->n_envs)) != hipSuccess ||
        (!h->seed_fixed &&  // the next-episode precompute (its tags invalid until a step restarts it)
         ((e = hipMalloc(&h->d_nx, nx_jump_offset(cfg->n_envs) + sizeof(rs_jump_table.w))) != hipSuccess ||
          (e = hipMemset(h->d_nx + 36 * (size_t)cfg->n_envs, 0xFF, 4 * (size_t)cfg->n_envs)) != hipSuccess ||
          (e = hipMemcpy(h->d_nx + nx_jump_offset(cfg->n_envs), rs_jump_table.w, sizeof(rs_jump_table.w),
                          hipMemcpyHostToDevice)) != hipSuccess)))) ||
      (h->seed_fixed &&  // the reset cache (cells 0 = in range until the first reset fills it)
       ((e = hipMalloc(&h->d_rsc, rmx::start_cache_bytes(A, cfg->n_envs))) != hipSuccess ||
        (e = hipMemset(h->d_rsc, 0, rmx::start_cache_bytes(A, cfg->n_envs))) != hipSuccess)) ||
      (h->fast && ((e = hipMalloc(&h->d_fast, fast_blob.size())) != hipSuccess ||
                   (e = hipMemcpy(h->d_fast, fast_blob.data(), fast_blob.size(), hipMemcpyHostToDevice)) != hipSuccess)) ||
      (!merged_tab.empty() &&
       ((h->merged_bytes = h->merged4_bytes ? h->merged4_off : merged_tab.size() * 4,
         e = hipMalloc(&h->d_merged, merged_tab.size() * 4)) != hipSuccess ||
        (e = hipMemcpy(h->d_merged, merged_tab.data(), merged_tab.size() * 4, hipMemcpyHostToDevice)) != hipSuccess))) {
    rmx_destroy(h);
    return hip_fail(e, "rmx_create allocation/upload");
  }
  h->cfg.cell = nullptr;
  h->cfg.cell_event = nullptr;
  h->cfg.next_q = nullptr;
  h->cfg.rm_reward = nullptr;
  h->cfg.shape = nullptr;
  h->cfg.init_q = h->cfg.final_q = h->cfg.start_xy = nullptr;
  h->cfg.n_qrm = h->cfg.enc_nq = nullptr;
  h->cfg.qrm_states = nullptr;
  *out = h;
  return RMX_OK;
}

void rmx_destroy(rmx_handle* h) {
  if (!h) return;
  if (h->host) {
    delete h->host;
    delete h;
    return;
  }
  (void)hipSetDevice(h->device);
  (void)sync_end(h);
  if (h->sy_mb) (void)hipHostFree(h->sy_mb);
  if (h->sy_done) (void)hipEventDestroy(h->sy_done);
  if (h->sy_dep) (void)hipEventDestroy(h->sy_dep);
  if (h->sy_stream) (void)hipStreamDestroy(h->sy_stream);
  (void)hipFree(h->d_tables);
  (void)hipFree(h->d_disc);
  (void)hipFree(h->d_slab);
  (void)hipFree(h->d_stats);
  (void)hipFree(h->d_err);
  (void)hipFree(h->d_fast);
  (void)hipFree(h->d_merged);
  (void)hipFree(h->d_es);
  (void)hipFree(h->d_stamps);
  (void)hipFree(h->d_free);
  (void)hipFree(h->d_start_ws);
  (void)hipFree(h->d_nx);
  (void)hipFree(h->d_rsc);
  delete h;
}

int rmx_bind(rmx_handle* h, const rmx_buffers* b) {
  if (!h || !b) return fail(RMX_E_INVALID, "handle or buffers NULL");
  if (!b->pos_x || !b->pos_y || !b->rm_q || !b->flags || !b->ep_ret || !b->t || !b->reward)
    return fail(RMX_E_STATE, "a required state/output buffer is NULL");
  const bool any_qrm = b->qrm_s || b->qrm_sn || b->qrm_rq || b->qrm_done;
  const bool all_qrm = b->qrm_s && b->qrm_sn && b->qrm_rq && b->qrm_done;
  if (any_qrm && !all_qrm) return fail(RMX_E_STATE, "QRM outputs must be all bound or all NULL");
  if (all_qrm && h->cfg.n_qrm_max == 0) return fail(RMX_E_STATE, "QRM outputs bound but n_qrm_max == 0");
  if ((h->cfg.stochastic || h->cfg.random_starts) && (!b->rng || !b->episode))
    return fail(RMX_E_STATE, "stochastic mode / random starts need the rng and episode buffers");
  if (b->enc_state)
    for (int a = 0; a < h->cfg.n_agents; ++a)
      if (h->enc_nq[a] < 1) return fail(RMX_E_STATE, "enc_state bound but enc_nq not provided at rmx_create");
  if (h->host) {  // host columns
    h->host->bind(*b);
    h->buf = *b;
    h->bound = true;
    return RMX_OK;
  }
  SYNC_END_OR_RETURN(h);
  if (h->sy_mb) {  // the mailbox's QRM sections follow the bound buffers: rebuilt at the next sync call
    (void)hipHostFree(h->sy_mb);
    h->sy_mb = nullptr;
  }
  h->buf = *b;
  h->bound = true;
  h->rs_dirty = true;  // the new rng columns hold whatever the caller put there
  return RMX_OK;
}

// random starts: the step kernel's next-episode shuffles belong to the old seed schedule / state: tag them invalid
// (the kernel restarts a precompute whose tag is not the expected episode)
static hipError_t invalidate_next_shuffles(const rmx_handle* h, hipStream_t st) {
  if (!h->d_nx) return hipSuccess;
  const size_t N = (size_t)h->cfg.n_envs;
  return hipMemsetAsync(h->d_nx + 36 * N, 0xFF, 4 * N, st);
}

// A new base seed on stream st: the fixed-start cache rebuilt (every env), the next-episode precompute tags invalidated.
static hipError_t refresh_starts(rmx_handle* h, hipStream_t st) {
  hipError_t e = hipSuccess;
  if (h->d_rsc) e = rmx::launch_reset(base_params(h), nullptr, 0, st);
  if (e == hipSuccess) e = invalidate_next_shuffles(h, st);
  if (e == hipSuccess) h->rs_stale = false;
  return e;
}

// Before a launch on st that reads the start cache / precompute: bring them up to date if the base seed moved
// without a launch on a caller stream (rmx_reset_sync).
static int starts_current(rmx_handle* h, void* stream) {
  if (h->rs_stale) HIP_TRY(refresh_starts(h, as_stream(stream)), "start cache refresh");
  return RMX_OK;
}

int rmx_reset(rmx_handle* h, const uint8_t* env_mask_dev, uint64_t seed, void* stream) {
  int rc = check_bound(h);
  if (rc) return rc;
  if (h->host) {
    h->host->reset(env_mask_dev, seed);
    h->base_seed = seed;
    return RMX_OK;
  }
  SYNC_END_OR_RETURN(h);
  // every env's generator comes from the new seed after a full reset; after a masked one with a new seed the envs
  // outside the mask keep the old seed's until their next autoreset
  h->rs_dirty = env_mask_dev ? (h->rs_dirty || seed != h->base_seed) : false;
  h->base_seed = seed;  // the seed schedule's base (stochastic mode)
  HIP_TRY(hipSetDevice(h->device), "hipSetDevice");
  rmx::KParams p = base_params(h);
  // (with the fixed-start cache this launch also rebuilds it, for every env whatever the mask)
  HIP_TRY(rmx::launch_reset(p, env_mask_dev, 1, as_stream(stream)), "reset launch");
  HIP_TRY(invalidate_next_shuffles(h, as_stream(stream)), "reset precompute");
  h->rs_stale = false;
  return RMX_OK;
}

// The fast step's parameter block for one step (rmx_step / rmx_step_hashed)
static rmx::FastParams step_fp(const rmx_handle* h, const int32_t* actions, uint64_t seed, int64_t t_global,
                               int autoreset) {
  rmx::FastParams fp = fast_params(h);
  // slip alone: the step kernel reseeds its resetting lanes (the same generator the cache holds) instead of
  // loading the cached one on every lane: 4.65 vs 4.93 us per step at config 2 (profiles/r04_ab_log.md slipcache);
  // the fused rollout loads it once and keeps it
  if (!h->cfg.random_starts) fp.slip &= ~rmx::kRngFixedSeed;
  fp.actions = actions;
  fp.seed = seed;
  fp.t_global = t_global;
  fp.autoreset = autoreset ? 1 : 0;
  if (fp.qrm_s) fp.tbl_mode = rmx::kTblGlobal;
  return fp;
}

static int do_step(rmx_handle* h, const int32_t* actions, int hashed, uint64_t seed, int64_t t_global, int autoreset,
                   void* stream) {
  int rc = check_bound(h);
  if (rc) return rc;
  if (!hashed && !actions) return fail(RMX_E_INVALID, "actions is NULL");
  if (h->host) {
    h->host->step(actions, autoreset, hashed != 0, seed, t_global);
    return RMX_OK;
  }
  SYNC_END_OR_RETURN(h);
  HIP_TRY(hipSetDevice(h->device), "hipSetDevice");
  if ((rc = starts_current(h, stream))) return rc;
  if (fast_applies(h)) {
    const rmx::FastParams fp = step_fp(h, actions, seed, t_global, autoreset);
    HIP_TRY(rmx::launch_step_fast(fp, hashed, h->cfg.kind, as_stream(stream)), "step launch");
    return RMX_OK;
  }
  rmx::KParams p = base_params(h);
  p.actions = actions;
  p.seed = seed;
  p.t_global = t_global;
  p.autoreset = autoreset ? 1 : 0;
  HIP_TRY(rmx::launch_step(p, hashed, h->cfg.kind, h->step_layout, grid_for(h, h->step_layout), dim3(h->block), h->tables_bytes, as_stream(stream)),
          "step launch");
  return RMX_OK;
}

int rmx_step(rmx_handle* h, const int32_t* actions_dev, int autoreset, void* stream) {
  return do_step(h, actions_dev, 0, 0, 0, autoreset, stream);
}

// The fused report runs where the handle's step is the thread-per-env fast kernel with 64-thread blocks,
// per-env statistics slots, rm_q / ep_ret skip stores and global / merged tables (the default below 1M envs);
// anywhere else rmx_step_report is the step launch followed by the stats launch, with the same result.
static bool report_fuses(const rmx_handle* h) {
  const int64_t grid = (h->cfg.n_envs + 63) / 64;
  const int tm = h->fast_tables;
  return fast_applies(h) && !h->buf.qrm_s && !h->fast_wave_stats && h->fast_block == 64 &&
         h->fast_skip == rmx::kSkipRare && h->rpt_partial &&
         (tm == rmx::kTblMerged4 || tm == rmx::kTblMerged || tm == rmx::kTblGlobal) && h->n_waves <= 64 * grid;
}

// The fused report step's parameter block (report_fuses(h))
static rmx::FastParams report_fp(const rmx_handle* h, const int32_t* actions, int autoreset, double* stats_out) {
  rmx::FastParams fp = fast_params(h);
  fp.actions = actions;
  fp.autoreset = autoreset ? 1 : 0;
  const int64_t grid = (h->cfg.n_envs + 63) / 64;
  fp.rpt_out = stats_out;
  fp.rpt_partial = h->rpt_partial;
  fp.rpt_ticket = h->rpt_ticket;
  fp.rpt_cs = (int32_t)((h->n_waves + grid - 1) / grid);
  fp.rpt_n_slab = (int32_t)h->n_waves;
  return fp;
}

int rmx_step_report(rmx_handle* h, const int32_t* actions_dev, int autoreset, double* stats_out_dev, void* stream) {
  int rc = check_bound(h);
  if (rc) return rc;
  if (!actions_dev || !stats_out_dev) return fail(RMX_E_INVALID, "bad rmx_step_report arguments");
  if (h->host) {
    h->host->step(actions_dev, autoreset);
    std::memcpy(stats_out_dev, h->host->stats, sizeof(h->host->stats));
    return RMX_OK;
  }
  SYNC_END_OR_RETURN(h);
  if (!report_fuses(h)) {
    if ((rc = do_step(h, actions_dev, 0, 0, 0, autoreset, stream))) return rc;
    HIP_TRY(reduce_stats(h, stats_out_dev, as_stream(stream)), "stats launch");
    return RMX_OK;
  }
  HIP_TRY(hipSetDevice(h->device), "hipSetDevice");
  const rmx::FastParams fp = report_fp(h, actions_dev, autoreset, stats_out_dev);
  HIP_TRY(rmx::launch_step_fast(fp, 0, h->cfg.kind, as_stream(stream)), "step launch");
  return RMX_OK;
}

int rmx_step_report_fused(const rmx_handle* h) { return h && h->bound && report_fuses(h) ? 1 : 0; }

// The K launches rmx_step / rmx_step_report would issue, recorded (rmx::tl_capture) instead; false when the handle's
// step is not the thread-per-env step_fast_kernel.
static bool record_seq(rmx_handle* h, const int32_t* actions, int64_t stride, int32_t K, int autoreset,
                       double* stats_out, bool fused) {
  h->seq.resize((size_t)K);
  for (int32_t k = 0; k < K; ++k) {
    const int32_t* a = actions + (size_t)k * (size_t)stride;
    const bool rpt = fused && k == K - 1;
    const rmx::FastParams fp = rpt ? report_fp(h, a, autoreset, stats_out) : step_fp(h, a, 0, 0, autoreset);
    rmx::StepCapture cap{&h->seq[(size_t)k], false};
    rmx::tl_capture = &cap;
    (void)rmx::launch_step_fast(fp, 0, h->cfg.kind, nullptr);
    rmx::tl_capture = nullptr;
    if (!cap.ok) return false;
  }
  return true;
}

static std::atomic<uint64_t> g_seq_keys{0};
// a window's recorded launches take ~1.2 KB of host memory and ~1.3 KB of kernel arguments each
constexpr int32_t kSeqMaxSteps = 1 << 20;

static int step_seq(rmx_handle* h, const int32_t* actions_dev, int64_t action_stride, int32_t n_steps, int autoreset,
                    double* stats_out_dev, void* stream) {
  int rc = check_bound(h);
  if (rc) return rc;
  if (!actions_dev || n_steps <= 0 || action_stride < 0) return fail(RMX_E_INVALID, "bad rmx_step_seq arguments");
  if (h->host) {  // the K steps in order on the host
    h->seq_dispatch = RMX_SEQ_HOST;
    for (int32_t k = 0; k < n_steps; ++k) h->host->step(actions_dev + (size_t)k * (size_t)action_stride, autoreset);
    if (stats_out_dev) std::memcpy(stats_out_dev, h->host->stats, sizeof(h->host->stats));
    return RMX_OK;
  }
  SYNC_END_OR_RETURN(h);
  HIP_TRY(hipSetDevice(h->device), "hipSetDevice");
  if ((rc = starts_current(h, stream))) return rc;
  hipStream_t st = as_stream(stream);
  const bool fused = stats_out_dev && report_fuses(h);
  // the K calls on the caller's stream, then a synchronisation: handles whose step is not the thread-per-env fast
  // kernel, RMX_QUEUE=0, and windows the queue cannot serve
  auto on_stream = [&](int why) {
    h->seq_dispatch = why;
    for (int32_t k = 0; k < n_steps; ++k) {
      const int32_t* a = actions_dev + (size_t)k * (size_t)action_stride;
      const int r = stats_out_dev && k == n_steps - 1 ? rmx_step_report(h, a, autoreset, stats_out_dev, stream)
                                                      : do_step(h, a, 0, 0, 0, autoreset, stream);
      if (r) return r;
    }
    HIP_TRY(hipStreamSynchronize(st), "step sequence");
    return (int)RMX_OK;
  };
  if (!fast_applies(h) || h->queue_off) {
    rmx::queue_note_stream(h->device);
    return on_stream(h->queue_off && fast_applies(h) ? RMX_SEQ_STREAM_DISABLED : RMX_SEQ_STREAM_KERNEL);
  }
  // the window recorded by the previous call is this one when the parameter block and the arguments agree
  // (fast_params zero-fills the block and FastParams has no padding, rmx_internal.h: a byte compare is a field one)
  const rmx::FastParams base = fast_params(h);
  const bool same = h->seq_key && h->seq_actions == actions_dev && h->seq_stride == action_stride &&
                    h->seq_k == n_steps && h->seq_autoreset == (autoreset ? 1 : 0) && h->seq_out == stats_out_dev &&
                    std::memcmp(&base, &h->seq_base, sizeof(base)) == 0;
  if (!same) {
    h->seq_key = 0;
    if (!record_seq(h, actions_dev, action_stride, n_steps, autoreset, stats_out_dev, fused)) {
      rmx::queue_note_stream(h->device);
      return on_stream(RMX_SEQ_STREAM_KERNEL);
    }
    ++h->seq_recordings;
    std::memcpy(&h->seq_base, &base, sizeof(base));
    h->seq_actions = actions_dev;
    h->seq_out = stats_out_dev;
    h->seq_stride = action_stride;
    h->seq_k = n_steps;
    h->seq_autoreset = autoreset ? 1 : 0;
    h->seq_key = ++g_seq_keys;
  }
  // the caller's work on the stream (and a start-cache refresh) before the window
  const hipError_t q = hipStreamQuery(st);
  if (q == hipErrorNotReady) HIP_TRY(hipStreamSynchronize(st), "step sequence");
  else if (q != hipSuccess) return hip_fail(q, "step sequence");
  std::string err;
  const int qr = rmx::queue_run(h->device, h->seq.data(), n_steps, h->seq_key, &err);
  if (qr == rmx::kQueueStream) return on_stream(RMX_SEQ_STREAM_QUEUE);  // nothing was submitted
  if (qr) {
    h->seq_key = 0;
    h->seq_dispatch = RMX_SEQ_QUEUE;
    return fail(RMX_E_HIP, err);
  }
  h->seq_dispatch = RMX_SEQ_QUEUE;
  if (stats_out_dev && !fused) {  // the report's second launch (the statistics reduction) on the stream
    HIP_TRY(reduce_stats(h, stats_out_dev, st), "stats launch");
    HIP_TRY(hipStreamSynchronize(st), "step sequence");
  }
  return RMX_OK;
}

int rmx_step_seq(rmx_handle* h, const int32_t* actions_dev, int64_t action_stride, int32_t n_steps, int autoreset,
                 double* stats_out_dev, void* stream) {
  if (n_steps > kSeqMaxSteps) return fail(RMX_E_INVALID, "rmx_step_seq: more steps than one window takes");
  try {  // nothing may unwind through the C ABI (the recorded window and the queue's buffers allocate)
    return step_seq(h, actions_dev, action_stride, n_steps, autoreset, stats_out_dev, stream);
  } catch (const std::exception& e) {
    if (h) h->seq_key = 0;
    return fail(RMX_E_HIP, std::string("rmx_step_seq: ") + e.what());
  }
}

int rmx_queue_counters(const rmx_handle* h, int64_t* out3) {
  if (!h || !out3) return fail(RMX_E_INVALID, "bad rmx_queue_counters arguments");
  rmx::QueueInfo qi{0, 0, 0, 0, RMX_QUEUE_UNUSED};  // a host handle has no device queue
  if (!h->host) rmx::queue_info(h->device, &qi);
  out3[0] = qi.windows;
  out3[1] = qi.uploads;
  out3[2] = qi.packets;
  return RMX_OK;
}

int rmx_queue_info(const rmx_handle* h, int64_t* out, int32_t n) {
  if (!h || !out || n < 0) return fail(RMX_E_INVALID, "bad rmx_queue_info arguments");
  rmx::QueueInfo qi{0, 0, 0, 0, RMX_QUEUE_UNUSED};  // a host handle has no device queue
  if (!h->host) rmx::queue_info(h->device, &qi);
  const int64_t v[RMX_QUEUE_INFO_N] = {qi.windows,         qi.uploads,      qi.packets, qi.stream_windows, qi.state,
                                       h->seq_dispatch, h->seq_recordings};
  for (int32_t i = 0; i < n && i < RMX_QUEUE_INFO_N; ++i) out[i] = v[i];
  return RMX_OK;
}

int rmx_queue_timing(rmx_handle* h, int every) {
  if (!h || every < 0) return fail(RMX_E_INVALID, "bad rmx_queue_timing arguments");
  if (h->host) return RMX_OK;  // a host handle has no device queue: nothing to time
  rmx::queue_set_timing(h->device, every);
  return RMX_OK;
}

int rmx_queue_times(const rmx_handle* h, uint64_t* stamps, int64_t cap, int64_t* n) {
  if (!h || !n || cap < 0 || (cap > 0 && !stamps)) return fail(RMX_E_INVALID, "bad rmx_queue_times arguments");
  // the device's last timed window, if this handle's last window ran on the queue
  *n = h->host || h->seq_dispatch != RMX_SEQ_QUEUE ? 0 : rmx::queue_times(h->device, stamps, cap);
  return RMX_OK;
}

int rmx_code_object_check(const void* co, size_t bytes, int64_t* n_step_kernels, int64_t* n_refused, char* report,
                          size_t report_cap) {
  if (!n_step_kernels || !n_refused || (co && bytes == 0)) return fail(RMX_E_INVALID, "bad rmx_code_object_check arguments");
  try {
    std::string first;
    const int rc = rmx::code_object_check(co, bytes, n_step_kernels, n_refused, &first);
    if (report && report_cap) {
      const size_t n = std::min(first.size(), report_cap - 1);
      std::memcpy(report, first.data(), n);
      report[n] = 0;
    }
    return rc ? fail(RMX_E_INVALID, "rmx_code_object_check: " + first) : RMX_OK;
  } catch (const std::exception& e) {
    return fail(RMX_E_INVALID, std::string("rmx_code_object_check: ") + e.what());
  }
}

int rmx_step_hashed(rmx_handle* h, uint64_t seed, int64_t t_global, int autoreset, void* stream) {
  if (t_global < 0) return fail(RMX_E_INVALID, "t_global < 0");
  return do_step(h, nullptr, 1, seed, t_global, autoreset, stream);
}

int rmx_fill_actions(rmx_handle* h, uint64_t seed, int64_t t0, int32_t T, int32_t* actions_dev, void* stream) {
  if (!h || !actions_dev || T < 0 || t0 < 0) return fail(RMX_E_INVALID, "bad rmx_fill_actions arguments");
  if (T == 0) return RMX_OK;
  if (h->host) {
    h->host->fill_actions(seed, t0, T, actions_dev);
    return RMX_OK;
  }
  HIP_TRY(hipSetDevice(h->device), "hipSetDevice");
  HIP_TRY(rmx::launch_fill_actions(seed, t0, T, h->cfg.n_envs_global, h->cfg.env_offset, h->cfg.n_envs,
                                   h->cfg.n_agents, actions_dev, as_stream(stream)),
          "fill_actions launch");
  return RMX_OK;
}

int rmx_rollout(rmx_handle* h, uint64_t seed, int64_t t0, int32_t T, float* trace, void* stream) {
  int rc = check_bound(h);
  if (rc) return rc;
  if (T < 0 || t0 < 0) return fail(RMX_E_INVALID, "bad rollout length");
  if (T == 0) return RMX_OK;
  if (h->host) {  // T autoreset steps with hashed actions; the trace [T][A][N] from each step's rewards
    const size_t AN = (size_t)h->cfg.n_agents * (size_t)h->cfg.n_envs;
    for (int32_t it = 0; it < T; ++it) h->host->step(nullptr, 1, true, seed, t0 + it, trace ? trace + (size_t)it * AN : nullptr);
    return RMX_OK;
  }
  SYNC_END_OR_RETURN(h);
  HIP_TRY(hipSetDevice(h->device), "hipSetDevice");
  if ((rc = starts_current(h, stream))) return rc;
  // the fast-path rollout (merged or global tables): deterministic dynamics, and FrozenLake slip where the step
  // runs the SLIP instantiation (merged tables; fast_params sets p.slip)
  if (h->fast && ((!h->cfg.stochastic && !h->cfg.random_starts) || fast_applies(h))) {
    rmx::FastParams fp = fast_params(h);
    fp.seed = seed;
    fp.t_global = t0;
    fp.autoreset = 1;
    // tables staged into LDS once per 256-thread workgroup (amortised over T steps), merged if present
    const bool merged = fp.tbl_mode == rmx::kTblMerged || fp.tbl_mode == rmx::kTblMerged4;
    // (random starts: the 256-thread workgroup's draw areas share the LDS with the staged table)
    const size_t rs_lds = h->cfg.random_starts ? 4 * (size_t)rmx::kRsWaveLds : 0;
    if (h->rollout_lds && (!merged || ((h->merged_bytes + 15) & ~(size_t)15) + rs_lds <= rmx::kRolloutLdsMax)) {
      fp.tbl_mode = merged ? rmx::kTblMergedLds : rmx::kTblLds;
      fp.block = 256;
    } else {
      fp.tbl_mode = merged ? rmx::kTblMerged : rmx::kTblGlobal;
    }
    HIP_TRY(rmx::launch_rollout_fast(fp, h->cfg.kind, T, trace, as_stream(stream)), "rollout launch");
    return RMX_OK;
  }
  rmx::KParams p = base_params(h);
  p.seed = seed;
  p.t_global = t0;
  p.autoreset = 1;
  HIP_TRY(rmx::launch_rollout(p, h->cfg.kind, h->rollout_layout, T, trace, grid_for(h, h->rollout_layout), dim3(h->block), h->tables_bytes,
                              as_stream(stream)),
          "rollout launch");
  return RMX_OK;
}

int rmx_mdp_states(rmx_handle* h, int32_t agent, int64_t* n_states) {
  if (!h || !n_states || agent < 0 || agent >= h->cfg.n_agents) return fail(RMX_E_INVALID, "bad rmx_mdp_states arguments");
  if (h->enc_nq[agent] < 1) return fail(RMX_E_INVALID, "enc_nq not provided at rmx_create");
  *n_states = (int64_t)h->cfg.width * h->cfg.height * h->enc_nq[agent];
  return RMX_OK;
}

int rmx_mdp(rmx_handle* h, int32_t agent, int32_t fix_frozen_lake, int32_t* next_dev, float* reward_dev,
            uint8_t* done_dev, void* stream) {
  int64_t S = 0;
  int rc = rmx_mdp_states(h, agent, &S);
  if (rc) return rc;
  if (!next_dev || !reward_dev || !done_dev) return fail(RMX_E_INVALID, "rmx_mdp output is NULL");
  if (h->host) {
    h->host->mdp(agent, fix_frozen_lake ? 1 : 0, next_dev, reward_dev, done_dev);
    return RMX_OK;
  }
  HIP_TRY(hipSetDevice(h->device), "hipSetDevice");
  rmx::KParams p = base_params(h);
  HIP_TRY(rmx::launch_mdp(p, h->cfg.kind, agent, fix_frozen_lake ? 1 : 0, S, next_dev, reward_dev, done_dev,
                          h->tables_bytes, as_stream(stream)),
          "mdp launch");
  return RMX_OK;
}

int rmx_stats_device(rmx_handle* h, double* out_dev, void* stream) {
  if (!h || !out_dev) return fail(RMX_E_INVALID, "bad rmx_stats_device arguments");
  if (h->host) {  // a host handle's "device" memory is host memory
    std::memcpy(out_dev, h->host->stats, sizeof(h->host->stats));
    return RMX_OK;
  }
  SYNC_END_OR_RETURN(h);
  HIP_TRY(hipSetDevice(h->device), "hipSetDevice");
  HIP_TRY(reduce_stats(h, out_dev, as_stream(stream)), "stats launch");
  return RMX_OK;
}

int rmx_stats_host(rmx_handle* h, double* out_host) {
  if (!h || !out_host) return fail(RMX_E_INVALID, "bad rmx_stats_host arguments");
  if (h->host) {
    std::memcpy(out_host, h->host->stats, sizeof(h->host->stats));
    return RMX_OK;
  }
  SYNC_END_OR_RETURN(h);
  HIP_TRY(hipSetDevice(h->device), "hipSetDevice");
  HIP_TRY(hipDeviceSynchronize(), "sync before stats");
  HIP_TRY(reduce_stats(h, h->d_stats, nullptr), "stats launch");
  HIP_TRY(hipMemcpy(out_host, h->d_stats, sizeof(double) * RMX_NSTATS, hipMemcpyDeviceToHost), "stats copy");
  return RMX_OK;
}

int rmx_stats_clear(rmx_handle* h, void* stream) {
  if (!h) return fail(RMX_E_INVALID, "handle is NULL");
  if (h->host) {
    std::memset(h->host->stats, 0, sizeof(h->host->stats));
    return RMX_OK;
  }
  SYNC_END_OR_RETURN(h);
  HIP_TRY(hipSetDevice(h->device), "hipSetDevice");
  HIP_TRY(hipMemsetAsync(h->d_slab, 0, sizeof(double) * RMX_NSTATS * h->n_waves, as_stream(stream)), "stats clear");
  if (h->d_es) HIP_TRY(hipMemsetAsync(h->d_es, 0, h->es_bytes, as_stream(stream)), "stats clear");
  return RMX_OK;
}

#ifdef RMX_DIAG
// Diagnostic builds only (not part of include/rmx.h): the resident stepper's device-side span of the last
// request (wall-clock ticks from seeing the request to its outputs being complete) and the tick rate in kHz.
int rmx_diag_sync_span(rmx_handle* h, unsigned long long* out /* [4]: t_seen, t_done, tick kHz, host post->ack ns */) {
  if (!h || !h->sy_mb) return fail(RMX_E_STATE, "no synchronous call made");
  const rmx::SyncAck* a = mb_host(h, h->sy_io.ack);
  int khz = 0;
  HIP_TRY(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, h->device), "wall clock rate");
  out[0] = a->t_seen;
  out[1] = a->t_done;
  out[2] = (unsigned long long)khz;
  out[3] = (unsigned long long)h->sy_wait_ns;
  return RMX_OK;
}

// Diagnostic builds only (not part of include/rmx.h): copy the per-wave stamps of the last fast-kernel
// launch ([wave][2 * kStamps] u64: shader clocks, then real-time clocks) to the host.
int rmx_diag_stamps(rmx_handle* h, unsigned long long* out, int64_t max_words) {
  if (!h || !h->d_stamps) return fail(RMX_E_STATE, "no stamp buffer (set RMX_DIAG_STAMPS at rmx_create)");
  const int64_t n = (h->cfg.n_envs + 255) / 256 * 4 * 2 * rmx::kStamps;
  HIP_TRY(hipDeviceSynchronize(), "sync");
  HIP_TRY(hipMemcpy(out, h->d_stamps, 8 * std::min(n, max_words), hipMemcpyDeviceToHost), "stamps copy");
  return (int)std::min(n, max_words);
}
#endif

int rmx_step_variant(const rmx_handle* h) {
  if (!h) return fail(RMX_E_INVALID, "handle is NULL");
  if (h->host) return RMX_VARIANT_HOST;
  if (fast_applies(h)) return RMX_VARIANT_FAST;
  return h->step_layout == rmx::kLayoutLanePerAgent ? RMX_VARIANT_LANE_PER_AGENT : RMX_VARIANT_GENERIC;
}

int rmx_state_bytes(const rmx_handle* h, size_t* bytes) {
  int rc = check_bound(h);
  if (rc) return rc;
  if (!bytes) return fail(RMX_E_INVALID, "bytes is NULL");
  std::vector<StateCol> cols;
  bool has_rng = false;
  state_columns(h, cols, has_rng);
  *bytes = state_blob_bytes(cols);
  return RMX_OK;
}

int rmx_get_state(rmx_handle* h, void* host_blob, size_t bytes) {
  int rc = check_bound(h);
  if (rc) return rc;
  std::vector<StateCol> cols;
  bool has_rng = false;
  state_columns(h, cols, has_rng);
  if (!host_blob || bytes != state_blob_bytes(cols)) return fail(RMX_E_INVALID, "state blob NULL or of the wrong size");
  if (!h->host) {
    SYNC_END_OR_RETURN(h);
    HIP_TRY(hipSetDevice(h->device), "hipSetDevice");
    HIP_TRY(hipDeviceSynchronize(), "sync before get_state");
  }
  StateHeader hd;
  std::memset(&hd, 0, sizeof(hd));
  std::memcpy(hd.magic, "RMXSTATE", 8);
  hd.version = kStateVersion;
  hd.has_rng = has_rng ? 1u : 0u;
  hd.n_agents = h->cfg.n_agents;
  hd.n_envs = h->cfg.n_envs;
  hd.base_seed = h->base_seed;
  hd.digest = h->digest;
  hd.env_offset = h->cfg.env_offset;
  hd.n_envs_global = h->cfg.n_envs_global;
  if (h->host) {
    std::memcpy(hd.stats, h->host->stats, sizeof(hd.stats));
  } else {
    HIP_TRY(reduce_stats(h, h->d_stats, nullptr), "stats launch");
    HIP_TRY(hipMemcpy(hd.stats, h->d_stats, sizeof(hd.stats), hipMemcpyDeviceToHost), "stats copy");
  }
  unsigned char* dst = static_cast<unsigned char*>(host_blob);
  std::memcpy(dst, &hd, sizeof(hd));
  dst += sizeof(hd);
  for (const auto& c : cols) {
    if (h->host)
      std::memcpy(dst, c.dev, c.bytes);
    else
      HIP_TRY(hipMemcpy(dst, c.dev, c.bytes, hipMemcpyDeviceToHost), "get_state copy");
    dst += c.bytes;
  }
  return RMX_OK;
}

int rmx_set_state(rmx_handle* h, const void* host_blob, size_t bytes) {
  int rc = check_bound(h);
  if (rc) return rc;
  std::vector<StateCol> cols;
  bool has_rng = false;
  state_columns(h, cols, has_rng);
  if (!host_blob || bytes != state_blob_bytes(cols)) return fail(RMX_E_INVALID, "state blob NULL or of the wrong size");
  StateHeader hd;
  std::memcpy(&hd, host_blob, sizeof(hd));
  if (std::memcmp(hd.magic, "RMXSTATE", 8) != 0 || hd.version != kStateVersion)
    return fail(RMX_E_INVALID, "not an rmx state blob of this version");
  if (hd.n_agents != h->cfg.n_agents || hd.n_envs != h->cfg.n_envs || hd.has_rng != (has_rng ? 1u : 0u))
    return fail(RMX_E_INVALID, "state blob shape (agents, envs, rng columns) differs from the handle");
  if (hd.digest != h->digest)
    return fail(RMX_E_INVALID, "state blob was written by a handle of another scenario (map, rules, RM or slip tables)");
  if (hd.env_offset != h->cfg.env_offset || hd.n_envs_global != h->cfg.n_envs_global)
    return fail(RMX_E_INVALID, "state blob was written for another shard (env_offset / n_envs_global)");
  {  // the columns index the tables: every cell, RM state and timestep must be in range before the upload
    const size_t AN = (size_t)h->cfg.n_agents * h->cfg.n_envs, N = (size_t)h->cfg.n_envs;
    const unsigned char* c0 = static_cast<const unsigned char*>(host_blob) + sizeof(hd);
    auto col = [&](int k, size_t i) {
      int32_t v;
      std::memcpy(&v, c0 + (size_t)k * 4 * AN + 4 * i, 4);
      return v;
    };
    for (size_t i = 0; i < AN; ++i)
      if ((uint32_t)col(0, i) >= (uint32_t)h->cfg.width || (uint32_t)col(1, i) >= (uint32_t)h->cfg.height ||
          (uint32_t)col(2, i) >= (uint32_t)h->cfg.n_rm_states)
        return fail(RMX_E_INVALID, "state blob holds a cell or RM state outside the handle's tables");
    for (size_t e = 0; e < N; ++e) {
      int32_t t;
      std::memcpy(&t, c0 + 5 * 4 * AN + 4 * e, 4);
      if (t < 0) return fail(RMX_E_INVALID, "state blob holds a negative timestep");
    }
  }
  if (h->host) {
    const unsigned char* src = static_cast<const unsigned char*>(host_blob) + sizeof(hd);
    for (const auto& c : cols) {
      std::memcpy(c.dev, src, c.bytes);
      src += c.bytes;
    }
    h->base_seed = h->host->base_seed = hd.base_seed;
    std::memcpy(h->host->stats, hd.stats, sizeof(hd.stats));
    return RMX_OK;
  }
  SYNC_END_OR_RETURN(h);
  HIP_TRY(hipSetDevice(h->device), "hipSetDevice");
  HIP_TRY(hipDeviceSynchronize(), "sync before set_state");
  const unsigned char* src = static_cast<const unsigned char*>(host_blob) + sizeof(hd);
  for (const auto& c : cols) {
    HIP_TRY(hipMemcpy(c.dev, src, c.bytes, hipMemcpyHostToDevice), "set_state copy");
    src += c.bytes;
  }
  h->base_seed = hd.base_seed;
  h->rs_dirty = true;  // the restored rng columns are the blob's
  // statistics: cleared, then the saved totals placed in slab slot 0 (every report sums the whole slab)
  HIP_TRY(hipMemset(h->d_slab, 0, sizeof(double) * RMX_NSTATS * h->n_waves), "stats clear");
  if (h->d_es) HIP_TRY(hipMemset(h->d_es, 0, h->es_bytes), "stats clear");
  HIP_TRY(hipMemcpy(h->d_slab, hd.stats, sizeof(hd.stats), hipMemcpyHostToDevice), "stats restore");
  HIP_TRY(refresh_starts(h, nullptr), "restore start cache / precompute");  // the restored base seed's
  HIP_TRY(hipDeviceSynchronize(), "sync after set_state");
  return RMX_OK;
}

int rmx_check_errors(rmx_handle* h) {
  if (!h) return fail(RMX_E_INVALID, "handle is NULL");
  if (h->host) {
    const uint32_t err = h->host->err;
    h->host->err = 0;
    return err ? fail(RMX_E_ACTION, "an action outside [0,4] was stepped (treated as wait)") : RMX_OK;
  }
  SYNC_END_OR_RETURN(h);
  HIP_TRY(hipSetDevice(h->device), "hipSetDevice");
  HIP_TRY(hipDeviceSynchronize(), "sync");
  uint32_t err = 0;
  HIP_TRY(hipMemcpy(&err, h->d_err, sizeof(err), hipMemcpyDeviceToHost), "err copy");
  HIP_TRY(hipMemset(h->d_err, 0, sizeof(uint32_t)), "err clear");
  if (err & 1u) return fail(RMX_E_ACTION, "an action outside [0,4] was stepped (treated as wait)");
  return RMX_OK;
}

int rmx_reset_sync(rmx_handle* h, uint64_t seed, const rmx_buffers* out_host, void* stream) {
  if (h && h->host) {  // reset every env, then the columns after it (no step outputs: zeros)
    int rc = check_bound(h);
    if (rc) return rc;
    h->host->pending = false;
    h->host->reset(nullptr, seed);
    h->base_seed = seed;
    h->host->last_reset = true;
    return host_sync_out(h, out_host, 0);
  }
  int rc = sync_check(h);
  if (rc) return rc;
  if (h->sy_pending && (rc = sync_wait(h))) return rc;
  h->base_seed = seed;
  h->rs_dirty = false;  // the resident kernel resets every env from the new seed
  // the start cache / precompute tags follow on the stream of the next fast launch (starts_current): a memset here
  // on the caller's stream would not be ordered before a launch on another stream
  h->rs_stale = h->d_rsc || h->d_nx;
  if ((rc = sync_request(h, rmx::kSyncReset, 0, seed, nullptr, stream))) return rc;
  return sync_copy_out(h, out_host);
}

int rmx_step_sync_begin(rmx_handle* h, const int32_t* actions_host, int autoreset, void* stream) {
  if (h && h->host) {  // the step itself; rmx_sync_wait returns its outputs
    int rc = check_bound(h);
    if (rc) return rc;
    if (!actions_host) return fail(RMX_E_INVALID, "actions is NULL");
    if (h->host->pending) return fail(RMX_E_STATE, "a synchronous request is outstanding (rmx_sync_wait first)");
    h->host->pending_bad = h->host->step(actions_host, autoreset);
    h->host->pending = true;
    h->host->last_reset = false;
    return RMX_OK;
  }
  int rc = sync_check(h);
  if (rc) return rc;
  if (!actions_host) return fail(RMX_E_INVALID, "actions is NULL");
  if (h->sy_pending) return fail(RMX_E_STATE, "a synchronous request is outstanding (rmx_sync_wait first)");
  return sync_begin(h, rmx::kSyncStep, autoreset ? 1u : 0u, 0, actions_host, stream);
}

int rmx_sync_wait(rmx_handle* h, const rmx_buffers* out_host) {
  if (!h) return fail(RMX_E_INVALID, "handle is NULL");
  if (h->host) {
    if (!h->host->pending) return fail(RMX_E_STATE, "no synchronous request is outstanding");
    h->host->pending = false;
    return host_sync_out(h, out_host, h->host->pending_bad);
  }
  int rc = sync_wait(h);
  if (rc) return rc;
  if ((rc = sync_copy_out(h, out_host))) return rc;
  if (__atomic_load_n(&mb_host(h, h->sy_io.ack)->bad, __ATOMIC_RELAXED))
    return fail(RMX_E_ACTION, "an action outside [0,4] (or wait under FrozenLake slip) was stepped (treated as wait)");
  return RMX_OK;
}

int rmx_step_sync(rmx_handle* h, const int32_t* actions_host, int autoreset, const rmx_buffers* out_host,
                  void* stream) {
  const int rc = rmx_step_sync_begin(h, actions_host, autoreset, stream);
  return rc ? rc : rmx_sync_wait(h, out_host);
}

int rmx_sync_end(rmx_handle* h) {
  if (!h) return fail(RMX_E_INVALID, "handle is NULL");
  if (h->host) {  // a begun request's outputs are dropped; the columns are current
    h->host->pending = false;
    return RMX_OK;
  }
  HIP_TRY(hipSetDevice(h->device), "hipSetDevice");
  return sync_end(h);
}

}  // extern "C"
