/*
 * rmx.h — C ABI of the MI355X-native multi-agent grid-world + Reward-Machine step engine.
 *
 * Drop-in boundary for the reference hot path (paths relative to Alee08/multiagent-rl-rm):
 *   RMEnvironmentWrapper.reset / .step / .check_terminations
 *       multiagent_rlrm/multi_agent/wrappers/rm_environment_wrapper.py:28-41, 43-107, 109-120
 *   MultiAgentFrozenLake.reset / .step / check_terminations / apply_action / holes_in_the_ice
 *       multiagent_rlrm/environments/frozen_lake/ma_frozen_lake.py:43-94, 96-154, 174-242
 *   MultiAgentOfficeWorld.reset / .step / check_terminations / apply_action / apply_wall_penalty
 *       multiagent_rlrm/environments/office_world/ma_office.py:77-120, 122-202, 204-325
 *   can_move_{up,down,left,right}      multiagent_rlrm/environments/office_world/config_office.py:12-39
 *   PositionEventDetector.detect_event multiagent_rlrm/environments/frozen_lake/detect_event.py:18-33
 *   RewardMachine.step                 multiagent_rlrm/multi_agent/reward_machine.py:45-59
 *
 * The reference's per-object Python calls become batched calls over N environments x A agents whose
 * state lives in caller-owned device buffers (structure of arrays, agent-major: column[a * N + e]).
 * All device work is enqueued on the caller's HIP stream; only rmx_stats_host / rmx_check_errors
 * synchronise.  Every entry point returns 0 on success or a negative RMX_E* code; the message is
 * available from rmx_last_error() (thread-local).
 *
 * Semantics are restated, not copied; see DESIGN.md for the rule list.
 *
 * Host handles: rmx_create with cfg.device == RMX_DEVICE_HOST steps the envs on the CPU (csrc/rmx_hoststep.cpp, over
 * the same compiled tables and rules as the generic gfx950 kernels): every entry point below then takes HOST pointers
 * wherever it says "device" (buffers, actions, masks, statistics, traces), ignores the stream and completes before it
 * returns.  It is the reference's own CPU case (BASELINE config 1: one env behind the per-call dict API) without a GPU
 * or a PCIe round trip per call.  rmx_step_variant reports RMX_VARIANT_HOST; rmx_step_seq, RMX_SEQ_HOST.
 */
#ifndef RMX_H
#define RMX_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RMX_ABI_VERSION 11

/* ---- limits (tables are staged whole into LDS per workgroup) ---------------------------------- */
#define RMX_MAX_AGENTS 8
#define RMX_MAX_CELLS 4096  /* W*H */
#define RMX_MAX_RM_STATES 255
#define RMX_MAX_EVENTS 255  /* including event 0 = "no event" (detect_event -> None) */

/* ---- error codes ---------------------------------------------------------------------------- */
#define RMX_OK 0
#define RMX_E_INVALID (-1)  /* bad argument / config            -> ValueError in Python  */
#define RMX_E_HIP (-2)      /* HIP runtime error                 -> RuntimeError          */
#define RMX_E_ACTION (-3)   /* an action outside [0,4] was seen  -> ValueError            */
#define RMX_E_STATE (-4)    /* buffers not bound / wrong sizes   -> RuntimeError          */

#define RMX_DEVICE_HOST (-1) /* rmx_config.device: the host path (no GPU) */

/* ---- environment kinds ---------------------------------------------------------------------- */
#define RMX_FROZEN_LAKE 0  /* ma_frozen_lake.py: up = y-1, RM-final agents freeze, trunc => term */
#define RMX_OFFICE_WORLD 1 /* ma_office.py:      up = y+1, walls, plants, RM-final agents keep moving */

/* ---- actions: index order of action_encoder_frozen_lake.py:14-17 / action_encoder_office_world.py:10-13 */
#define RMX_UP 0
#define RMX_DOWN 1
#define RMX_LEFT 2
#define RMX_RIGHT 3
#define RMX_WAIT 4 /* ActionRL("wait"): no move, no wall collision */

/* ---- per-cell tile bits ----------------------------------------------------------------------- */
#define RMX_CELL_CAN_UP 0x01u    /* can_move_up    (boundary, and walls for OfficeWorld) */
#define RMX_CELL_CAN_DOWN 0x02u  /* can_move_down  */
#define RMX_CELL_CAN_LEFT 0x04u  /* can_move_left  */
#define RMX_CELL_CAN_RIGHT 0x08u /* can_move_right */
#define RMX_CELL_HAZARD 0x10u    /* FrozenLake hole / OfficeWorld plant */

/* ---- per-(env, agent) flags word ------------------------------------------------------------ */
#define RMX_F_ACTIVE 0x01u   /* env.active_agents[name]                                  */
#define RMX_F_FAIL 0x02u     /* env.agent_fail[name]                                     */
#define RMX_F_TERM 0x04u     /* wrapper terminations[name] (env OR RM) after this step   */
#define RMX_F_TRUNC 0x08u    /* wrapper truncations[name]                                */
#define RMX_F_ENV_TERM 0x10u /* infos[name]["env_terminated"]                            */
#define RMX_F_RM_TERM 0x20u  /* infos[name]["rm_terminated"]                             */
#define RMX_F_ENV_DONE 0x40u /* the episode of this env ended at this step (loop rule)   */
#define RMX_F_STEPS_SHIFT 16 /* bits 16..31: env.agent_steps[name]                       */

/* ---- statistics vector (rmx_stats_*): sums over finished episodes ------------------------- */
#define RMX_STAT_SUM_RETURN 0 /* sum over (env-episode, agent) of the episode return           */
#define RMX_STAT_EPISODES 1   /* number of finished env-episodes                                */
#define RMX_STAT_SUCCESSES 2  /* number of (env-episode, agent) successes (evaluation_metrics.py:248-267) */
#define RMX_STAT_SUM_LENGTH 3 /* sum over env-episodes of env.timestep at the end               */
#define RMX_NSTATS 4

typedef struct rmx_config {
  int32_t kind;        /* RMX_FROZEN_LAKE or RMX_OFFICE_WORLD                                   */
  int32_t width;       /* grid_width  (W)                                                       */
  int32_t height;      /* grid_height (H)                                                       */
  int32_t n_agents;    /* A, 1..RMX_MAX_AGENTS                                                  */
  int32_t n_rm_states; /* Q: row count of the dense RM tables (max over agents)                 */
  int32_t n_events;    /* E: 1 + number of distinct event cells (event 0 = None)                */
  int32_t max_t;       /* truncation when timestep > max_t (1000 in the reference)              */
  int32_t device;      /* HIP device ordinal the handle binds to, or RMX_DEVICE_HOST            */
  int64_t n_envs;      /* N: envs in THIS shard (one rank / GPU)                                */
  int64_t env_offset;  /* global index of env 0 of this shard (action hash, sharding)           */
  int64_t n_envs_global; /* N over all shards (action hash)                                     */
  float hazard_penalty;  /* FL penalty_amount / OW plants_penalty_value                         */
  float wall_penalty;    /* OW wall_penalty_value (ignored for FL: a boundary block is free)     */
  int32_t hazard_fail;   /* FL: 1 (holes always fail) / OW: terminate_on_plants                  */
  int32_t wall_fail;     /* OW: terminate_hit_walls                                              */
  float gamma;           /* episode-return discount for the stats (OW loop: gamma, FL loop: 1.0) */
  int32_t has_shaping;   /* 1 if shape[] is given (potential-based shaping column)               */
  float reward_modifier; /* RMEnvironmentWrapper.reward_modifier (rm_environment_wrapper.py:26,69) */
  int32_t n_qrm_max;     /* Qx: max over agents of len(get_all_states()) - 1 (QRM experiences)    */
  /* Stochastic slip (ma_frozen_lake.py:244-298, ma_office.py:327-379): numpy Generator(PCG64) per env,
   * seeded by SeedSequence(seed) at every reset (default_rng(seed)), one rng.choice draw per agent that
   * actually slips, in agent order.  seed of env e (global index) in its k-th episode since rmx_reset:
   *   seed = base_seed * seed_scale + e * seed_env_stride + k * seed_episode_stride   (mod 2^64)
   * (FrozenLake runner: reset(args.seed) every episode; OfficeWorld runner: reset(seed*1000 + episode)). */
  int32_t stochastic;           /* 0: deterministic dynamics; 1: slip tables below are used           */
  int32_t slip_n[4];            /* outcomes per intended action (<= 4)                               */
  int32_t slip_out[4][4];       /* outcome action ids (RMX_UP..RMX_WAIT) in the reference's list order */
  double slip_cdf[4][4];        /* p.cumsum() / p.cumsum()[-1] exactly as Generator.choice computes it */
  uint64_t seed_scale, seed_env_stride, seed_episode_stride;
  /* FrozenLake random_start_positions (ma_frozen_lake.py:37-39, 59-64, 156-172): at every reset the agents
   * start on the first A cells of the non-hole cells in x-major order ((x, y) for x in range(W) for y in
   * range(H)) shuffled by numpy Generator.shuffle with the env rng just seeded for that episode, i.e. BEFORE
   * any slip draw of the episode.  Needs the rng / episode buffers like stochastic mode (the same seed
   * schedule); start_xy is then unused.  FrozenLake only; at least A non-hole cells. */
  int32_t random_starts;
  /* host pointers, copied at rmx_create */
  const uint16_t* cell;       /* [H*W]       RMX_CELL_* bits, index y*W + x                   */
  const uint8_t* cell_event;  /* [A][H*W]    event id 0..E-1 detected at that cell per agent    */
  const uint8_t* next_q;      /* [A][Q][E]   RM successor; missing (q,e) => q (self loop)       */
  const float* rm_reward;     /* [A][Q][E]   RM transition reward (raw); missing => 0           */
  const float* shape;         /* [A][Q][E]   gamma*Phi(next_q) - Phi(q), or NULL                */
  const int32_t* init_q;      /* [A]         RM initial-state index (always 0 in the reference) */
  const int32_t* final_q;     /* [A]         RM final-state index (last inserted to_state)      */
  const int32_t* start_xy;    /* [A][2]      initial (x, y) per agent                           */
  /* QRM counterfactual experiences (rm_environment_wrapper.py:122-183); may be NULL if n_qrm_max == 0 */
  const int32_t* n_qrm;       /* [A]         len(rm.get_all_states()) - 1                        */
  const uint8_t* qrm_states;  /* [A][Qx]     RM-state indices in get_all_states() order (last dropped) */
  const int32_t* enc_nq;      /* [A]         rm.numbers_state() (state encoder stride, state_encoder_*.py) */
} rmx_config;

/* Caller-owned device buffers; columns are agent-major [A][N] (index a*N + e). */
typedef struct rmx_buffers {
  int32_t* pos_x;    /* [A][N] state  */
  int32_t* pos_y;    /* [A][N] state  */
  int32_t* rm_q;     /* [A][N] state: RM state index (RewardMachine.get_state_index)      */
  uint32_t* flags;   /* [A][N] state: RMX_F_* bits + agent_steps                          */
  float* ep_ret;     /* [A][N] state: running episode return (FL sum, OW discounted sum)   */
  int32_t* t;        /* [N]    state: env.timestep                                       */
  float* reward;     /* [A][N] out:   wrapper rewards[name] = Renv + reward_modifier * RQ  */
  float* shaping;    /* [A][N] out:   gamma*Phi(q') - Phi(q) (NULL: not written)          */
  uint8_t* env_done; /* [N]    out:   1 where the episode ended this step (NULL: not written) */
  float* renv;       /* [A][N] out:   infos["Renv"] (NULL: not written)                   */
  /* QRM experiences, [A][Qx][N] each (NULL: not computed).  Experience j of agent a is
   * (qrm_s, action, Renv + qrm_rq, qrm_sn, qrm_done, qrm_s / nQ, qrm_s % nQ, qrm_sn / nQ, qrm_sn % nQ,
   * qrm_rq) of rm_environment_wrapper.py:168-179, nQ = enc_nq[a]. */
  int32_t* qrm_s;    /* encoder.encode(prev position, state j)                       */
  int32_t* qrm_sn;   /* encoder.encode(new position, hypothetical next state)        */
  float* qrm_rq;     /* hypothetical RM reward (raw, not scaled by reward_modifier)  */
  uint8_t* qrm_done; /* env termination OR hypothetical next state == final          */
  /* required when cfg.stochastic or cfg.random_starts: per-env PCG64 state and episode counter */
  uint64_t* rng;     /* [4][N] state_hi, state_lo, inc_hi, inc_lo (128-bit LCG of numpy's PCG64) */
  int32_t* episode;  /* [N]    episodes started since rmx_reset (the k of the seed schedule)      */
  /* optional learner input (NULL: not written): the post-step observation encoded as the reference's
   * state encoders do, (pos_y * W + pos_x) * enc_nq[a] + rm_q (state_encoder_frozen_lake.py:23-35,
   * state_encoder_office.py:15-24).  Needs cfg.enc_nq. */
  int32_t* enc_state; /* [A][N] */
} rmx_buffers;

typedef struct rmx_handle rmx_handle;

/* Version / diagnostics */
int rmx_abi_version(void);
/* HIP devices visible to this process (0 without a driver or a device: host handles still work); no reference
 * counterpart (the reference runs on the CPU only). */
int rmx_device_count(int32_t* n);
const char* rmx_last_error(void);
/* Build provenance (no reference counterpart): "src=<first 16 hex digits of the SHA-256 of the engine
 * sources, in the Makefile's RMX_HASHED order> kern=<the same of the fast kernels' gfx950 code object>
 * abi=<RMX_ABI_VERSION> arch=<offload arch>".  A loader compares src with the sources it ships to refuse a stale
 * library; kern ties a kernel profile to the machine code it measured. */
const char* rmx_build_info(void);

/* Create a handle: validates the config, uploads tables to the device, allocates the stats slab.
 * Replaces the object graph built by frozen_lake_main.py:199-267 / office_main.py:400-605. */
int rmx_create(const rmx_config* cfg, rmx_handle** out);
void rmx_destroy(rmx_handle* h);

/* Bind caller-owned device buffers (sizes implied by cfg.n_envs and cfg.n_agents). */
int rmx_bind(rmx_handle* h, const rmx_buffers* buf);

/* RMEnvironmentWrapper.reset (rm_environment_wrapper.py:28-41) for the envs whose env_mask byte is
 * nonzero (all envs if env_mask == NULL): timestep 0, agents active at their start cells, RM at its
 * initial state, episode return 0.  `seed` becomes the base seed of the schedule above; stochastic mode
 * reseeds each reset env with episode k = 0 (deterministic dynamics ignore it). */
int rmx_reset(rmx_handle* h, const uint8_t* env_mask_dev, uint64_t seed, void* hip_stream);

/* One RMEnvironmentWrapper.step (rm_environment_wrapper.py:43-107) for every env of the shard.
 * actions_dev: int32 [A][N] device array (RMX_UP..RMX_WAIT).  If autoreset != 0, envs whose previous
 * step ended their episode (RMX_F_ENV_DONE) are reset first, mirroring the reference loops
 * (frozen_lake_main.py:336-376, office_main.py:1696-1749), then stepped with this action. */
int rmx_step(rmx_handle* h, const int32_t* actions_dev, int autoreset, void* hip_stream);

/* As rmx_step, with actions generated in-kernel by the SURVEY §8(d) counter hash
 * a = splitmix64(seed ^ (((t_global*N_global + e_global)*A + i) * 0x9E3779B97F4A7C15)) >> 62. */
int rmx_step_hashed(rmx_handle* h, uint64_t seed, int64_t t_global, int autoreset, void* hip_stream);

/* Fill actions_dev[T][A][N] with the same hash for global steps t0 .. t0+T-1 (test / bench input). */
int rmx_fill_actions(rmx_handle* h, uint64_t seed, int64_t t0, int32_t T, int32_t* actions_dev,
                     void* hip_stream);

/* Fused rollout: T autoreset steps with hashed actions, state kept in registers, per-episode stats
 * accumulated; state columns written back once at the end.  reward_trace_dev (optional, NULL = off)
 * receives float [T][A][N] rewards. */
int rmx_rollout(rmx_handle* h, uint64_t seed, int64_t t0, int32_t T, float* reward_trace_dev,
                void* hip_stream);

/* RMEnvironmentWrapper.get_mdp (rm_environment_wrapper.py:185-283) for one agent, deterministic dynamics:
 * S = W*H*enc_nq[agent] encoded states (rmx_mdp_states); outputs [S][4] device arrays: next encoded state
 * (-1 = no entry), reward, done (0/1, 255 = no entry).  Terminal states (hole / plant with
 * terminate_on_plants / RM final) self-loop.  fix_frozen_lake = 0 reproduces the reference exactly,
 * including its FrozenLake quirk (decode returns {"q": label}, so non-hole FL states get no entries);
 * 1 decodes the RM index as the OfficeWorld encoder does. Needs no bound buffers. */
int rmx_mdp_states(rmx_handle* h, int32_t agent, int64_t* n_states);
int rmx_mdp(rmx_handle* h, int32_t agent, int32_t fix_frozen_lake, int32_t* next_dev, float* reward_dev,
            uint8_t* done_dev, void* hip_stream);

/* Episode statistics accumulated since the last rmx_stats_clear (RMX_NSTATS doubles).
 * _device writes them to a device buffer (for an RCCL all-reduce), _host synchronises. */
int rmx_stats_device(rmx_handle* h, double* out_dev, void* hip_stream);
int rmx_stats_host(rmx_handle* h, double* out_host);
int rmx_stats_clear(rmx_handle* h, void* hip_stream);

/* rmx_step followed by rmx_stats_device(stats_out_dev) on the same stream: the step of a loop iteration that
 * also logs the episode statistics (frozen_lake_main.py:368-376, office_main.py:1743-1749; the vector an
 * RCCL all-reduce then sums across ranks).  Where the handle runs the default thread-per-env fast kernel
 * below 1M envs on deterministic dynamics, the report is computed inside the step launch (one launch instead of
 * two); slip handles, QRM-bound, lane-per-agent and per-wave-statistics (>= 1M envs) handles and the generic
 * kernels take the two launches.  Integer statistics are identical either way; the fused report's return sum is a
 * fixed-order sum with its own association, so it may differ from rmx_stats_device's in the last bits.
 * Like rmx_stats_device it uses the handle's reduction scratch: one report in flight per handle (calls on one
 * stream, as everything else on a handle).
 * rmx_step_report_fused: 1 if this (bound) handle fuses the report, else 0 (no device work). */
int rmx_step_report(rmx_handle* h, const int32_t* actions_dev, int autoreset, double* stats_out_dev,
                    void* hip_stream);
int rmx_step_report_fused(const rmx_handle* h);

/* n_steps iterations of the reference loops' inner step (frozen_lake_main.py:336-376, office_main.py:1696-1749) in
 * one submission: step k is rmx_step with actions_dev + k * action_stride (int32 elements, each an [A][N] array as
 * for rmx_step); with stats_out_dev != NULL the last one is rmx_step_report's (the statistics vector written
 * there).  Results identical to those n_steps calls on hip_stream.  BLOCKING: returns once the steps are complete
 * on the device (work enqueued on hip_stream before the call runs first).  Where the handle's step is the
 * thread-per-env fast kernel the launches go to the engine's own AQL queue on the device (one per device, K
 * kernel-dispatch packets and one doorbell: no per-launch runtime work); elsewhere they are the calls on hip_stream,
 * then a stream synchronisation.  1 <= n_steps <= 2^20.
 * The stream path also serves a fast handle whenever the queue cannot: RMX_QUEUE=0 in the environment at rmx_create,
 * a queue that could not be set up on the device (no HSA agent found for it, a loader error), a step kernel the queue
 * refuses (its code-object metadata lists a hidden argument the queue does not write, e.g. a debugging printf's), and
 * every window after a failed one.  A window fails (RMX_E_HIP, its results undefined) when the queue faults or does
 * not complete within 60 s; the queue is then inactivated (none of its packets keeps running) and retired for the
 * process.
 * rmx_queue_counters: that queue's windows, kernel-argument uploads and packets so far for the handle's device.
 * rmx_queue_info: out[0..n) of RMX_QUEUE_INFO_N values: [0] windows, [1] uploads, [2] packets (as above), [3] windows
 * of the device served on a stream, [4] the device queue's state (RMX_QUEUE_*), [5] how the handle's last
 * rmx_step_seq ran (RMX_SEQ_*), [6] how often the handle re-recorded its window (a repeated identical call reuses
 * the recording and uploads nothing). */
int rmx_step_seq(rmx_handle* h, const int32_t* actions_dev, int64_t action_stride, int32_t n_steps, int autoreset,
                 double* stats_out_dev, void* hip_stream);
int rmx_queue_counters(const rmx_handle* h, int64_t* out3);
#define RMX_QUEUE_INFO_N 7
#define RMX_QUEUE_UNUSED 0      /* not set up yet (no window on this device so far) */
#define RMX_QUEUE_READY 1
#define RMX_QUEUE_UNAVAILABLE 2 /* set-up failed: windows run on the stream */
#define RMX_QUEUE_RETIRED 3     /* a window failed: later windows run on the stream */
#define RMX_SEQ_NONE 0            /* no rmx_step_seq on this handle yet */
#define RMX_SEQ_QUEUE 1           /* the engine's queue */
#define RMX_SEQ_STREAM_KERNEL 2   /* the stream: the handle's step is not the thread-per-env fast kernel */
#define RMX_SEQ_STREAM_DISABLED 3 /* the stream: RMX_QUEUE=0 at rmx_create */
#define RMX_SEQ_STREAM_QUEUE 4    /* the stream: the queue is unavailable or retired, or refused a kernel */
#define RMX_SEQ_HOST 5            /* a host handle: the K steps on the CPU */
int rmx_queue_info(const rmx_handle* h, int64_t* out, int32_t n);
/* Dispatch timing of the handle's device queue (profiling; off by default).  The queue has HSA dispatch profiling
 * enabled from its creation.  rmx_queue_timing(h, m), m >= 1: from the next window on, packets 0, m, 2m, ... and the
 * window's last one carry a completion signal of their own (at most 4,096 per window), so the command processor
 * stamps those dispatches' start (packet processing) and end (completion) — the timestamps a kernel trace reads, with
 * the packets still back to back behind one doorbell.  A stamped packet costs the command processor ~1.2 us more than
 * an unstamped one: m = 1 times every dispatch at that cost, a sparse m leaves the cadence as it is and the span
 * between stamps measures it.  m = 0 turns timing off.  rmx_queue_times: the last timed window's stamps into stamps
 * ([n][3]: packet index, start, end; ns in the system timestamp domain; at most cap triples) and *n their number (0:
 * no timed window yet, the last window was untimed or ran on the stream, or a host handle); they stay readable after
 * timing is turned off, until the next window.  Results are unchanged by timing. */
int rmx_queue_timing(rmx_handle* h, int every);
int rmx_queue_times(const rmx_handle* h, uint64_t* stamps, int64_t cap, int64_t* n);
/* The queue's metadata check (no GPU needed) over a gfx950 code object (co == NULL: the step code object embedded in
 * this library): *n_step_kernels step_fast_kernel instantiations found, *n_refused of them the queue would refuse;
 * the first refused one and why into report (NUL-terminated, truncated to report_cap).  -1 (RMX_E_INVALID) if the
 * object cannot be read. */
int rmx_code_object_check(const void* co, size_t bytes, int64_t* n_step_kernels, int64_t* n_refused, char* report,
                          size_t report_cap);

/* Which step kernel rmx_step / rmx_step_hashed launch for this handle (no device work):
 * RMX_VARIANT_GENERIC thread-per-env, RMX_VARIANT_LANE_PER_AGENT, or the deterministic fast path
 * (pre-composed move words; selected when the config allows it and no QRM outputs are bound) as
 * RMX_VARIANT_FAST (thread-per-env).  At rmx_create, RMX_FAST=0 in the environment disables the fast
 * path.  RMX_VARIANT_FAST_LANE_PER_AGENT is no longer returned (round 5 removed that layout after it lost
 * its A/Bs); the value stays reserved. */
#define RMX_VARIANT_GENERIC 0
#define RMX_VARIANT_LANE_PER_AGENT 1
#define RMX_VARIANT_FAST 2
#define RMX_VARIANT_FAST_LANE_PER_AGENT 3
#define RMX_VARIANT_HOST 4 /* a host handle (cfg.device == RMX_DEVICE_HOST): the CPU path */
int rmx_step_variant(const rmx_handle* h);

/* Synchronise and report kernel-side errors (e.g. RMX_E_ACTION), then clear them. */
int rmx_check_errors(rmx_handle* h);

/* Checkpoint / resume of a rollout (the reference saves learner tables and pickles,
 * evaluation_metrics.py:193-214, office_main.py:1611-1613): everything needed to continue the bound shard
 * bit-exactly — the state columns pos_x, pos_y, rm_q, flags, ep_ret, t, the per-env rng / episode columns
 * when bound, the reset seed of the seed schedule and the episode statistics accumulated since the last
 * rmx_stats_clear — as ONE packed host blob of rmx_state_bytes() bytes (layout versioned by a header;
 * opaque to callers).  rmx_get_state synchronises the device and copies out; rmx_set_state checks the
 * header against the handle (A, N, rng columns; RMX_E_INVALID on mismatch), copies the columns into the
 * bound buffers and replaces the statistics, then synchronises. */
int rmx_state_bytes(const rmx_handle* h, size_t* bytes);
int rmx_get_state(rmx_handle* h, void* host_blob, size_t bytes);
int rmx_set_state(rmx_handle* h, const void* host_blob, size_t bytes);

/* ---- synchronous host-boundary calls: the reference's per-call dict API ---------------------------------
 * RMEnvironmentWrapper.reset(seed) / .step(actions) (rm_environment_wrapper.py:28-41, 43-107) as the reference
 * loops call them (frozen_lake_main.py:336-376, office_main.py:1696-1749): host actions in, host outputs back,
 * the call returns once they are there.  For small shards (n_envs <= RMX_SYNC_MAX_ENVS, typically 1).
 * One workgroup stays resident on the device between calls (state in registers, tables in LDS, a pinned
 * host mailbox polled by one lane): a call costs a host<->device round trip, not a kernel launch.  It exits
 * after RMX_SYNC_IDLE_US (default 2000) microseconds without a call, on rmx_sync_end, or implicitly at the
 * start of every other entry point on the handle, writing its state back to the bound device columns first.
 *   rmx_reset_sync: rmx_reset of every env with `seed` (the schedule's base seed), outputs after the reset;
 *   rmx_step_sync:  rmx_step with actions_host int32 [A][N] in host memory, outputs after the step;
 *                   RMX_E_ACTION (after stepping, the action treated as wait) for an action outside [0, 4] or
 *                   "wait" under FrozenLake slip (the reference raises KeyError);
 *   out_host:       host pointers laid out as the device columns of rmx_buffers (NULL fields are not copied;
 *                   rng / episode are ignored); shaping, enc_state and the QRM columns are available when the
 *                   handle computes them (cfg.has_shaping, cfg.enc_nq, QRM columns bound), else RMX_E_STATE;
 *   hip_stream:     the launch of the resident workgroup is ordered after the work enqueued on it so far.
 *   rmx_step_sync_begin + rmx_sync_wait: rmx_step_sync in two halves; the caller may do host work of its own
 *                   between them (no other call on the handle); rmx_sync_wait returns what rmx_step_sync would.
 * A request for N * A <= 15 actions travels inline in one 16-B request word (one host-memory read by the
 * device).  The resident workgroup runs on the handle's own non-blocking stream; a device-wide synchronisation
 * while it waits for a call returns when it times out. */
#define RMX_SYNC_MAX_ENVS 256
int rmx_reset_sync(rmx_handle* h, uint64_t seed, const rmx_buffers* out_host, void* hip_stream);
int rmx_step_sync(rmx_handle* h, const int32_t* actions_host, int autoreset, const rmx_buffers* out_host,
                  void* hip_stream);
int rmx_step_sync_begin(rmx_handle* h, const int32_t* actions_host, int autoreset, void* hip_stream);
int rmx_sync_wait(rmx_handle* h, const rmx_buffers* out_host);
int rmx_sync_end(rmx_handle* h);

#ifdef __cplusplus
}
#endif

#endif /* RMX_H */
