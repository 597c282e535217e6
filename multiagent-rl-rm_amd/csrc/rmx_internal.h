// rmx_internal.h — kernel parameter block shared by the C-ABI layer and the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cmath>
#include <string>

#include "../../include/rmx.h"
#include "rmx_layout.h"

namespace rmx {

// FrozenLake random starts: the per-env shuffle workspace row stride in u16 entries (16-B aligned rows, read
// back 8 entries per load by shuffle_slots, rmx_device.h)
__host__ __device__ constexpr int32_t shuffle_stride(int32_t n) { return (n + 7) & ~7; }
// fast-path random starts: LDS bytes per wave (one draw byte per shuffle index and lane, then 256 free cells)
__host__ __device__ constexpr int32_t rs_wave_lds(int32_t n) { return 256 * ((n + 3) >> 2) + 512; }
// random starts in the fast kernels (rs_step, rmx_fast.hip): LDS per wave (the free-cell copies, then the
// wave-cooperative finish's output blocks) and the undo's per-lane row copy in that area: 64 lanes x kRsRowMax
// <= 8 * 64 * 24 B, so the fast path takes n_free + 8 <= kRsRowMax (host)
constexpr int kRsWaveLds = 512 + 8 * 64 * (16 + 8);
constexpr int kRsRowMax = 192;
// the per-env rng features of the fast kernels' SLIP template argument (FastParams::slip).  kRngFixedSeed (with
// kRngSlip and / or kRngStarts): the reset-seed schedule has seed_episode_stride == 0 (the reference FrozenLake
// runner's rm_env.reset(args.seed) every episode, frozen_lake_main.py:337), so every episode of env e starts from the
// same default_rng(seed) and, with random starts, the same shuffle: the start cells and the post-seed (post-shuffle)
// generator are computed once per base seed into handle-owned columns (reset_kernel, rmx_kernels.hip) and an
// autoreset copies them.
constexpr int kRngSlip = 1, kRngStarts = 2, kRngFixedSeed = 4;
// the reset cache: cells u32 [(A + 1) / 2][N] (agent 2w in bits 0-15, agent 2w + 1 in bits 16-31, each
// x | y << 8; the configured starts without random starts), then the post-seed generator u64 [4][N] (state hi, lo,
// increment hi, lo) at a 256-B aligned offset
inline size_t start_cache_rng_off(int A, int64_t N) { return (4 * (size_t)((A + 1) / 2) * (size_t)N + 255) & ~(size_t)255; }
inline size_t start_cache_bytes(int A, int64_t N) { return start_cache_rng_off(A, N) + 32 * (size_t)N; }

constexpr uint64_t kGolden = 0x9E3779B97F4A7C15ull;

// slip choice threshold (host): Generator.random() = m * 2^-53 with an integer m < 2^53, so cdf <= u exactly when
// ceil(cdf * 2^53) <= m (the scaling by 2^53 is exact); NaN never compares true, cdf >= 1 never does either
inline uint64_t slip_threshold(double cdf) {
  if (!(cdf == cdf)) return ~0ull;
  if (cdf <= 0.0) return 0ull;
  if (cdf >= 1.0) return (1ull << 53) + (cdf > 1.0 ? 1ull : 0ull);
  return (uint64_t)std::ceil(std::ldexp(cdf, 53));
}

// The slip choice tables of a kernel parameter block (KParams / FastParams) from the config: per intended action the
// outcome count, the integer thresholds of its cdf and the outcomes, and the shared-cdf fast form when every intended
// action has the same count and thresholds (the outcomes 0..4 fit 3 bits each).
template <typename P>
inline void slip_fill(P& p, const rmx_config& c) {
  bool uniform = true;
  p.slip_pack = 0;
  for (int i = 0; i < 4; ++i) {
    p.slip_n[i] = c.slip_n[i];
    uniform = uniform && c.slip_n[i] == c.slip_n[0];
    for (int j = 0; j < 4; ++j) {
      p.slip_out[i][j] = c.slip_out[i][j];
      p.slip_thr[i][j] = slip_threshold(c.slip_cdf[i][j]);
      uniform = uniform && (j >= 3 || p.slip_thr[i][j] == slip_threshold(c.slip_cdf[0][j])) &&
                (uint32_t)c.slip_out[i][j] <= 7u;
      p.slip_pack |= (uint64_t)((uint32_t)c.slip_out[i][j] & 7u) << (3 * (4 * i + j));
    }
  }
  p.slip_uniform = uniform ? 1 : 0;
}

// Passed by value as the kernel argument (well under the 4 KiB kernarg limit).
struct KParams {
  // tables blob (device) staged into LDS; byte offsets of each section inside the blob
  const uint4* tables;
  int32_t tables_n16;
  int32_t off_cell, off_ev, off_nq, off_rr, off_sh, off_qrm;
  // geometry / rules
  int32_t W, HW, A, Q, E, max_t;
  int64_t N;
  float hazard_penalty, wall_penalty;
  int32_t hazard_fail, wall_fail, has_shaping, gamma_is_one;
  float reward_modifier;
  int32_t n_qrm_max;  // Qx (0: QRM off)
  // stochastic slip: numpy PCG64 per env (rng [4][N]), seed schedule, choice tables
  int32_t stochastic;
  int32_t slip_n[4], slip_out[4][4];
  uint64_t slip_thr[4][4];  // ceil(cdf * 2^53): u = m * 2^-53 (m = next64 >> 11) has cdf <= u iff thr <= m
  // the four intended actions share one cdf (every reference slip map does): the outcome is read from slip_pack,
  // 3 bits per (intended action i, choice j) at bit 3 * (4 i + j), with uniform thresholds (slip_fill)
  int32_t slip_uniform;
  uint64_t slip_pack;
  uint64_t seed_scale, seed_env_stride, seed_episode_stride, base_seed;
  uint64_t* rng;
  int32_t* episode;
  // per-env rng columns in use (slip and / or random starts); FrozenLake random_start_positions: the
  // non-hole cells (y*W + x, x-major order) and a per-env shuffle workspace [N][n_free]
  int32_t rng_on, random_starts, n_free;
  const uint16_t* free_cells;
  uint16_t* start_ws;
  int32_t* enc_state;  // [A][N] optional encoded observation (y*W + x)*enc_nq[a] + q
  int32_t n_qrm[RMX_MAX_AGENTS], enc_nq[RMX_MAX_AGENTS];
  int32_t init_q[RMX_MAX_AGENTS], final_q[RMX_MAX_AGENTS], start_x[RMX_MAX_AGENTS], start_y[RMX_MAX_AGENTS];
  const float* disc;  // [max_t + 2] gamma^t
  // caller buffers
  int32_t* pos_x;
  int32_t* pos_y;
  int32_t* rm_q;
  uint32_t* flags;
  float* ep_ret;
  int32_t* t;
  float* reward;
  float* shaping;
  uint8_t* env_done;
  float* renv;
  int32_t* qrm_s;
  int32_t* qrm_sn;
  float* qrm_rq;
  uint8_t* qrm_done;
  // per-call
  const int32_t* actions;
  uint64_t seed;
  int64_t t_global, env_offset, n_global;
  int32_t autoreset;
  double* slab;   // [n_waves][RMX_NSTATS]
  int32_t diag;   // diagnostic variant bits (only read by -DRMX_DIAG builds)
  uint32_t* err;  // kernel-side error bits
  int32_t skip_same;  // 1: column words the step leaves unchanged are not stored (large N; not with QRM)
  // kRngFixedSeed: the start cache (start_cache_bytes layout), written by reset_kernel for EVERY env (mask or not)
  uint32_t* rs_cells;
  uint64_t* rs_rng;
};

// ---- deterministic fast path: table layout and constants in rmx_layout.h (host-only, no HIP) ----

struct FastParams {
  const uint4* tables;  // [mv u32 A*HW*5][rm uint4 A*Q*E][info uint4 A], 16-B aligned sections
  int32_t n16, off_rm, off_info;
  int32_t pad6;
  const uint4* merged;                // kTblMerged table (or NULL)
  int32_t merged_bytes;               // its size: the buffer descriptor's range (out-of-range reads return 0)
  int32_t mg_base[kFastMaxAgents];    // record index of agent a's section (identical sections shared)
  int32_t pad0;                       // explicit padding: no implicit padding anywhere (see kFastParamsFieldBytes)
  // kTblMerged4: one u32 per record = the merged word 0 with bits 28-29 = palette index of the reward (mg_palb)
  const uint32_t* merged4;
  int32_t merged4_bytes;
  uint32_t mg_palb[kFastMaxAgents];  // reward_modifier * RQ palette per agent: <= 4 integers in [-128, 127], one byte each
  int32_t HW;
  // QRM counterfactual outputs (rm_environment_wrapper.py:122-183), [A][Qx][N] each, or NULL
  int32_t* qrm_s;
  int32_t* qrm_sn;
  float* qrm_rq;
  uint8_t* qrm_done;
  int32_t n_qrm_max;                                   // Qx
  int32_t n_qrm[kFastMaxAgents], enc_nq[kFastMaxAgents];
  uint8_t qrm_q[kFastMaxAgents][kFastMaxQrm];          // get_all_states()[:-1] indices
  int32_t W, H, E, max_t, N, A;
  int32_t hazard_fail, wall_fail;  // OW terminate_on_plants / terminate_hit_walls
  int32_t mv_base[kFastMaxAgents];  // a*HW*5
  int32_t rm_base[kFastMaxAgents];  // a*Q*E
  int32_t final_q[kFastMaxAgents], init_q[kFastMaxAgents], start_x[kFastMaxAgents], start_y[kFastMaxAgents];
  float hazard_penalty, wall_penalty;
  int32_t has_shaping, gamma_is_one, autoreset;
  int32_t tbl_mode;  // table mode kTbl*
  int32_t skip_same;  // kSkipNone / kSkipAll / kSkipRare: which unchanged column words are not stored (global / merged tables)
  int32_t block;      // threads per workgroup of the thread-per-env kernel in the global / merged modes (64..256)
  int32_t pad1;
  const float* disc;
  int32_t* pos_x;
  int32_t* pos_y;
  int32_t* rm_q;
  uint32_t* flags;
  float* ep_ret;
  int32_t* t;
  float* reward;
  float* shaping;
  uint8_t* env_done;
  float* renv;
  int32_t* enc_state;  // [A][N] optional encoded observation (y*W + x)*enc_nq[a] + q
  const int32_t* actions;
  uint64_t seed;
  int64_t t_global, env_offset, n_global;
  int32_t wave_stats;          // 1: per-wave slab slots (large N); 0: per-env atomic slots below
  int32_t pad2;
  double* slab;                // [waves][RMX_NSTATS] (wave_stats)
  double* es_ret;              // [N] per-env episode-return sums (the env's agents summed before the add)
  unsigned long long* es_cnt;  // [N] per-env sum of lengths | episodes << 40
  uint32_t* es_succ;           // [N] per-env successes
  uint32_t* err;
  int32_t diag;  // diagnostic ablation bits (only read by -DRMX_DIAG builds)
  int32_t pad3;
  unsigned long long* stamps;  // RMX_DIAG builds: per-wave s_memtime / s_memrealtime stamps (or NULL)
  // rmx_step_report's fused statistics report (step_fast_kernel<..., RPT = true>, 64-thread blocks, per-env
  // slots): the last block to finish writes the vector to rpt_out.  Block b also folds in the slab slots
  // [b * rpt_cs, b * rpt_cs + rpt_cs) below rpt_n_slab (the rollout kernels and a restored state write there).
  double* rpt_out;
  double* rpt_partial;       // [grid][RMX_NSTATS]
  unsigned int* rpt_ticket;  // 0 between reports (re-armed by the last block)
  int32_t rpt_cs, rpt_n_slab;
  // FrozenLake slip on the fast path (step_fast_kernel<..., SLIP>): numpy PCG64 per env, rng [4][N] (state hi,
  // lo, increment hi, lo), episode [N] of the reset-seed schedule; the choice tables as in KParams
  int32_t slip_n[4], slip_out[4][4];
  uint64_t slip_thr[4][4];  // ceil(cdf * 2^53): u = m * 2^-53 (m = next64 >> 11) has cdf <= u iff thr <= m
  // the four intended actions share one cdf (every reference slip map does): the outcome is read from slip_pack,
  // 3 bits per (intended action i, choice j) at bit 3 * (4 i + j), with uniform thresholds (slip_fill)
  int32_t slip_uniform;
  int32_t pad4;
  uint64_t slip_pack;
  uint64_t seed_scale, seed_env_stride, seed_episode_stride, base_seed;
  uint64_t* rng;
  int32_t* episode;
  // kRngSlip | kRngStarts: slip draws and / or FrozenLake random starts on the fast path (host: kSkipRare, merged
  // tables, thread-per-env, N < 2^27); random starts: the free cells and the per-env shuffle workspace
  int32_t slip;
  int32_t n_free;
  const uint16_t* free_cells;
  uint16_t* start_ws;
  // random starts in the step kernel: the next episode's shuffle in progress (generator [4][N] u64, index [N],
  // episode tag [N]; handle-owned, the draws themselves in the start_ws rows as bytes)
  uint64_t* nx_rng;
  int32_t* nx_idx;
  int32_t* nx_ep;
  // the jump table of the wave-cooperative finish: for j = 1..64, M^j then 1 + M + ... + M^(j-1) (mod 2^128,
  // the PCG64 multiplier M), each as a uint4 (low 64 bits first)
  const uint4* rs_jump;
  // kRngFixedSeed: each env's start cells and post-shuffle generator (start_cache_bytes layout)
  const uint32_t* rs_cells;
  const uint64_t* rs_rng;
  // kRngFixedSeed: 0 when every env's rng column was written from the cache's base seed (a full rmx_reset, every
  // later autoreset): its increment words equal the cache's and, without slip, so do its state words, so a reset
  // writes only the episode counter (and, with slip, the state words).  1 after a masked reset with a new seed, a
  // restore or a rebind: a reset copies the whole cached generator.
  int32_t rs_dirty;
  int32_t pad5;
};
// rmx_step_seq reuses a recorded window while the new parameter block equals the recorded one byte for byte (and
// the queue diffs kernel arguments byte for byte): that is a field compare only if FastParams has no implicit padding.
// Every field is listed here; a field added without a listing, or a new gap, fails the assertion.
#define RMX_FAST_PARAMS_FIELDS(X) X(tables) X(n16) X(off_rm) X(off_info) X(pad6) X(merged) \
   X(merged_bytes) X(mg_base) X(pad0) X(merged4) X(merged4_bytes) X(mg_palb) X(HW) X(qrm_s) X(qrm_sn) X(qrm_rq) \
   X(qrm_done) X(n_qrm_max) X(n_qrm) X(enc_nq) X(qrm_q) X(W) X(H) X(E) X(max_t) X(N) X(A) X(hazard_fail) \
   X(wall_fail) X(mv_base) X(rm_base) X(final_q) X(init_q) X(start_x) X(start_y) X(hazard_penalty) X(wall_penalty) \
   X(has_shaping) X(gamma_is_one) X(autoreset) X(tbl_mode) X(skip_same) X(block) X(pad1) X(disc) X(pos_x) X(pos_y) \
   X(rm_q) X(flags) X(ep_ret) X(t) X(reward) X(shaping) X(env_done) X(renv) X(enc_state) X(actions) X(seed) \
   X(t_global) X(env_offset) X(n_global) X(wave_stats) X(pad2) X(slab) X(es_ret) X(es_cnt) X(es_succ) X(err) X(diag) \
   X(pad3) X(stamps) X(rpt_out) X(rpt_partial) X(rpt_ticket) X(rpt_cs) X(rpt_n_slab) X(slip_n) X(slip_out) \
   X(slip_thr) X(slip_uniform) X(pad4) X(slip_pack) X(seed_scale) X(seed_env_stride) X(seed_episode_stride) \
   X(base_seed) X(rng) X(episode) X(slip) X(n_free) X(free_cells) X(start_ws) X(nx_rng) X(nx_idx) X(nx_ep) \
   X(rs_jump) X(rs_cells) X(rs_rng) X(rs_dirty) X(pad5)
#define RMX_FP_FIELD_BYTES(f) +sizeof(FastParams::f)
constexpr size_t kFastParamsFieldBytes = 0 RMX_FAST_PARAMS_FIELDS(RMX_FP_FIELD_BYTES);
#undef RMX_FP_FIELD_BYTES
static_assert(kFastParamsFieldBytes == sizeof(FastParams), "FastParams has implicit padding or an unlisted field");
constexpr int kStamps = 9;  // stamps per wave (x2: shader clock, real time)

// the thread-per-env fast step kernel (step_fast_kernel) of p.tbl_mode / p.skip_same / p.slip / p.rpt_out
hipError_t launch_step_fast(const FastParams& p, int hashed, int kind, hipStream_t st);

// ---- the engine's own AQL queue (rmx_queue.cpp): rmx_step_seq's K dependent step launches in one submission ----
// step_fast_kernel's explicit parameters in order: the kernarg segment before its hidden (implicit) arguments
struct StepArgs {
  int32_t N, blk;
  const int32_t *pos_x, *pos_y, *rm_q;
  const uint32_t* flags;
  const int32_t* t;
  const int32_t* actions;
  FastParams p;
};
static_assert(sizeof(StepArgs) == 56 + sizeof(FastParams), "step_fast_kernel's parameter list: no padding");
// one step launch recorded instead of issued: the instantiation's code-object symbol, 1-D geometry, dynamic LDS
struct StepLaunch {
  char symbol[160];
  uint32_t grid, block, lds;
  StepArgs args;
};
// While tl_capture is set, launch_step_fast records the launch into *out (ok = true) instead of issuing it; a handle
// whose step is not the thread-per-env step_fast_kernel records nothing (ok stays false) and launches nothing.
struct StepCapture {
  StepLaunch* out;
  bool ok;
};
extern thread_local StepCapture* tl_capture;
// K recorded launches on device's own queue, each behind the previous one (barrier bit), the last one's completion
// waited for (spin, with a deadline).  Returns 0 when done; kQueueStream when nothing was submitted and the caller's
// stream must run the window (the queue is unavailable or retired, or the code-object metadata check refused one of
// the window's kernels; *err says why); -1 when the window failed (*err set; a fault or timeout has inactivated and
// retired the queue, so this window's results are undefined and later windows take the stream).  Thread-safe per
// device.  key != 0 names the window's contents (L, K): the same key as the device's previous window reuses its
// packets and kernel arguments as they are.
constexpr int kQueueStream = 1;
constexpr int kQueueUnused = RMX_QUEUE_UNUSED, kQueueReady = RMX_QUEUE_READY, kQueueUnavailable = RMX_QUEUE_UNAVAILABLE,
              kQueueRetired = RMX_QUEUE_RETIRED;
int queue_run(int device, const StepLaunch* L, int K, uint64_t key, std::string* err);
// a window of `device` served on a stream for a reason outside the queue (the handle's kernel, RMX_QUEUE=0)
void queue_note_stream(int device);
struct QueueInfo {
  int64_t windows, uploads, packets, stream_windows;  // stream_windows: rmx_step_seq calls served on a stream
  int state;                                          // kQueue*
};
void queue_info(int device, QueueInfo* out);
// dispatch timing of the device's queue (rmx_queue.cpp): the stamp stride (0 off), and the last timed window's
// [n][packet, start ns, end ns]
void queue_set_timing(int device, int every);
int64_t queue_times(int device, uint64_t* out, int64_t cap);
// the queue's code-object metadata check over `co` (NULL: the embedded step code object): step kernels seen, refused,
// and the first refused one with its reason (or the reason the object could not be read: returns -1)
int code_object_check(const void* co, size_t bytes, int64_t* n_step, int64_t* n_refused, std::string* first);
// fused T-step rollout on the fast path (global or merged tables; other table modes use global)
hipError_t launch_rollout_fast(const FastParams& p, int kind, int32_t T, float* trace, hipStream_t st);

// ---- resident host-boundary stepper (rmx_step_sync / rmx_reset_sync, rmx_sync.hip) ----------------------
// One mailbox in pinned, coherent host memory per handle: a request line the host writes, an acknowledgement line
// the device writes, the actions the host writes, and the per-step output columns the device writes.  Each side
// only ever polls its OWN memory's lines: the device polls the request line (one lane), the host polls the
// acknowledgement line.
constexpr uint32_t kSyncStep = 1, kSyncReset = 2, kSyncExit = 3;
// The request is ONE 16-B word that the host writes with one aligned 16-B store and the polling lane reads with
// one 16-B system-coherent load, so a single host-memory round trip delivers it: {seq, ctl, acts, seq} (the
// repeated seq rejects a torn read).  ctl: op (bits 0-1) | autoreset (bit 2) | inline (bit 3) | actions 0..6 in
// 4-bit fields from bit 4; acts: actions 7..14.  Inline when N * A <= kSyncInlineActs (the dict API: N = 1);
// otherwise the actions are in the mailbox's action array, written before the request word.  An action outside
// [0, 4] travels as 15 (invalid: stepped as wait and reported, as in the device path).
constexpr int kSyncInlineActs = 15;
constexpr uint32_t kSyncInline = 1u << 3, kSyncAutoreset = 1u << 2, kSyncBadAct = 15u;
struct alignas(128) SyncReq {
  uint32_t seq;        // word 0
  uint32_t ctl;        // word 1
  uint32_t acts;       // word 2
  uint32_t seq_echo;   // word 3 = seq
  uint64_t seed;       // kSyncReset: the new base seed of the reset-seed schedule (read after the request word)
};
struct alignas(128) SyncAck {
  uint32_t seq;  // written last (system scope) by the device once the outputs are in host memory
  uint32_t bad;  // 1: an action outside [0, 4] (or "wait" under FrozenLake slip) was stepped by this request
  uint64_t t_seen, t_done;  // RMX_DIAG builds: wall-clock ticks when the request was seen / the outputs completed
};
// Outputs of one request, packed so that a lane writes 2A + 1 16-B records instead of ~8A + 2 scalars:
//   rec    [N][A][2]: {x | y << 16, q, flags, reward}, {renv, ep_ret, shaping, enc_state} (f32 as bits)
//   envrec [N]:       {t, env_done, 0, 0}
// and the QRM columns ([A][Qx][N], NULL when not computed).  The host unpacks into rmx_buffers columns.
struct SyncCols {
  uint4* rec;
  uint4* envrec;
  int32_t* qrm_s;
  int32_t* qrm_sn;
  float* qrm_rq;
  uint8_t* qrm_done;
};
struct SyncIO {
  SyncReq* req;         // host-mapped
  SyncAck* ack;         // host-mapped
  const int32_t* act;   // host-mapped [A][N]
  SyncCols out;         // host-mapped
  uint32_t seq0;        // requests up to this sequence number are already served
  uint32_t pad;
  uint64_t idle_ticks;  // exit after this long (wall-clock ticks) without a request ...
  uint64_t life_ticks;  // ... or this long after launch
};
hipError_t launch_resident(const KParams& p, const SyncIO& io, int kind, int threads, size_t lds, hipStream_t st);

inline int amax_bucket(int A) { return A <= 4 ? A : 8; }
// lanes per env of the lane-per-agent layout: next power of two >= A
inline int lanes_per_env(int A) { return A <= 1 ? 1 : A <= 2 ? 2 : A <= 4 ? 4 : 8; }
constexpr int kLayoutThreadPerEnv = 0;
constexpr int kLayoutLanePerAgent = 1;

hipError_t launch_step(const KParams& p, int hashed, int kind, int layout, dim3 g, dim3 b, size_t lds,
                       hipStream_t st);
hipError_t launch_rollout(const KParams& p, int kind, int layout, int32_t T, float* trace, dim3 g, dim3 b,
                          size_t lds, hipStream_t st);
// write_state = 0: only the fixed-start cache (p.rs_cells) is rebuilt, the columns are left alone
hipError_t launch_reset(const KParams& p, const uint8_t* mask, int write_state, hipStream_t st);
hipError_t launch_fill_actions(uint64_t seed, int64_t t0, int32_t T, int64_t n_global, int64_t env_offset, int64_t N,
                               int A, int32_t* out, hipStream_t st);
hipError_t launch_mdp(const KParams& p, int kind, int ag, int fix_fl, int64_t S, int32_t* next, float* reward,
                      uint8_t* done, size_t lds, hipStream_t st);
constexpr int kStatsPartials = 512;  // max blocks of each partial pass of the stats reduction
constexpr int kStatsEnvsPerThread = 4;  // per-env slots summed by each thread of the stats launch
// sums the per-wave slab and, if es_ret != NULL, the per-env slots of the fast path (FastParams: one row [N]
// each), in one launch; partial: 2 * kStatsPartials *
// RMX_NSTATS doubles; ticket: a zeroed u32 the launch leaves zeroed
hipError_t launch_stats_reduce(const double* slab, int64_t n_waves, const double* es_ret, const unsigned long long* es_cnt,
                               const uint32_t* es_succ, int64_t N, double* partial, unsigned int* ticket,
                               double* out, hipStream_t st);

}  // namespace rmx
