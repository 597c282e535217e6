// rmx_fast.hip — the thread-per-env step kernel for gfx950 (step_fast_kernel): the default step of every BASELINE config
// (A <= 4, W, H <= 255), with or without QRM outputs, and with FrozenLake / OfficeWorld slip and FrozenLake random
// starts (the SLIP instantiations); plus the fused rollout.  Same semantics as agent_step<KIND> / env_step
// (rmx_generic.h), which the parity tests pin to the oracle and the reference's golden vectors.
//
// Why a separate path: at BASELINE size (65,536 envs) every SIMD of the chip holds one or two waves, so nothing hides
// a wave's own dependency chain; a launch costs load latency + the wave's issued instructions (~4 cycles each for a
// lone wave) + the store drain.  This path shortens the chain:
//  * the tables are read straight from global memory (they stay L2-resident), not staged into LDS: staging cost a
//    block barrier behind the blob's loads (config 2 3.43 -> 3.17 us, config 5 4.09 -> 3.84 us; DESIGN §4.2,
//    profiles/r01_ab_log.md c12).  This replaces north_star's "map tiles and RM table staged into LDS";
//  * an agent-step is ONE dependent lookup where the merged table fits (kTblMerged / kTblMerged4, <= 128 KiB): a
//    record of (agent, RM state, cell, action) pre-composed on the host (rmx_tables.cpp build_merged) holding the new
//    x / y, the next RM state, the wall / hazard / fail / RM-final bits and the scaled reward (16-B records, or 4-B
//    records with a per-agent reward palette in SGPRs: config 2 3.28 vs 3.36 us, config 3 2.51 vs 2.68 us).  Larger
//    tables and QRM outputs take the global blob (kTblGlobal): a move word, then the RM entry (two lookups);
//  * column loads / stores go through buffer descriptors: SGPR base + SGPR agent offset + one shared 32-bit lane
//    offset, so there is no per-access 64-bit address arithmetic; the rarely changing rm_q / ep_ret words are stored
//    only when they change (kSkipRare);
//  * the per-agent logic is integer bit arithmetic (no exec-mask branches); wave-level sums (the statistics report)
//    are DPP row reductions, not LDS shuffles — north_star's "__ballot compaction" is replaced by them.
// One layout: thread-per-env (A agents in one lane).  Round 5 removed the table modes and layouts that lost their
// A/Bs (LDS-staged and lane-resident tables, speculative and 8-B merged records, lane-per-agent; profiles/r01_ab_log.md
// c12/c25/c26/c75, r02_ab_log.md ab3 "pair", r05_ab_log.md "prune").
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdio>
#include <cstring>
#include <type_traits>
#include <stdint.h>

#include "rmx_device.h"
#include "rmx_internal.h"

namespace rmx {

namespace {

__device__ __forceinline__ __amdgpu_buffer_rsrc_t col_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}
// Column stores are sc1 (write-through): measured on MI355X, the launch ends ~0.4 us sooner at BASELINE
// size than with default-policy stores (aux 0); nt|sc1 (18), sc0|sc1 (17), nt loads and sc1 loads were
// no better.
constexpr int kStoreAux = 16;
// kSkipRareNT (the bandwidth regime, >= 2^23 env x agent instances): nt|sc1, write-through with the non-temporal
// hint.  At 8.4M envs 6-24 % faster than sc1 alone on all four configs; at 65,536 envs 7-8 % slower
// (r02_ab_log pol, nt).  nt loads: no gain at either size, and slower combined with nt stores.
constexpr int kStoreAuxNT = 18;
__device__ __forceinline__ int32_t col_ld(__amdgpu_buffer_rsrc_t r, uint32_t lane_bytes, uint32_t sgpr_bytes) {
  return __builtin_amdgcn_raw_buffer_load_b32(r, lane_bytes, sgpr_bytes, 0);
}
#ifdef RMX_DIAG
// diagnostic builds: diag bit 32 = default-policy stores (per-store uniform branch; timing only)
__device__ __forceinline__ void col_st_d(__amdgpu_buffer_rsrc_t r, uint32_t lane_bytes, uint32_t sgpr_bytes, int32_t v,
                                         int diag) {
  if (diag & 32)
    __builtin_amdgcn_raw_buffer_store_b32(v, r, lane_bytes, sgpr_bytes, 0);
  else
    __builtin_amdgcn_raw_buffer_store_b32(v, r, lane_bytes, sgpr_bytes, kStoreAux);
}
#define col_st(r, l, s, v) col_st_d(r, l, s, v, p.diag)
#else
__device__ __forceinline__ void col_st(__amdgpu_buffer_rsrc_t r, uint32_t lane_bytes, uint32_t sgpr_bytes, int32_t v) {
  __builtin_amdgcn_raw_buffer_store_b32(v, r, lane_bytes, sgpr_bytes, kStoreAux);
}
#endif
template <int AUX = kStoreAux>
__device__ __forceinline__ void byte_st(const FastParams& p, uint32_t e, uint32_t v) {
  __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v, col_rsrc(p.env_done, (uint32_t)p.N), e, 0, AUX);
}

// Episode statistics of a finished env (evaluation_metrics.py:248-267 bookkeeping): no-return atomics
// into per-env slots, the env's agents summed in agent order before the add.  One adder per slot per launch
// and launches are stream-ordered, so every slot's value is a fixed-order sum; rmx_stats_* reduces the slots
// in a fixed order.  es_ret [N] f64 episode-return sums, es_cnt [N] u64 length | episodes << 40, es_succ [N] u32
__device__ __forceinline__ void env_stats_ret(const FastParams& p, int32_t e, double ret, uint32_t succ) {
  unsafeAtomicAdd(p.es_ret + e, ret);
  if (succ) atomicAdd(p.es_succ + e, succ);
}
__device__ __forceinline__ void env_stats_env(const FastParams& p, int32_t e, int32_t t1) {
  atomicAdd(p.es_cnt + e, (unsigned long long)(uint32_t)t1 | (1ull << 40));
}

// ---- rmx_step_report: the statistics report fused into a step launch (64-thread blocks, per-env slots) ----
// The separate report (stats_kernel) costs a dependent launch plus its own load / ticket / partial chain
// (~7 us after the steps at 65,536 envs).  Fused, the slot loads ride with the step's column loads, the lane
// adds its own episode to the loaded values (the slot's only adder in this launch, so this equals the slot
// after the atomic), every block stores one partial vector and takes a ticket, and the last block sums the
// partials in block order.  Fixed association order for a given N: repeated reports agree bit for bit
// (integer statistics are exact in f64; the return sum's association differs from stats_kernel's, so the two
// reports may differ in the last bits of the return sum only).  Cross-XCD visibility as in stats_kernel:
// agent-scope atomic stores / loads for the partials, a store wait before the relaxed ticket.
// The hand-off below relies on gfx94x / gfx950 semantics: stores count in vmcnt (so s_waitcnt(0) means "completed"),
// and the sc1 cache-policy bit on the partial stores / loads makes them write-through / L2-bypassing at device scope.
// On any other target the last block could sum stale partials without an error: refuse to build there.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__) && !defined(__gfx942__)
#error "rmx_fast.hip: the fused report's ticket hand-off is written for gfx950 (and gfx942) memory semantics"
#endif
constexpr uint32_t kRptShards = 32;    // shard counters of the fused report's ticket
constexpr uint32_t kRptLineWords = 32;  // one 128-B line per counter (root first, then the shards)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 pack2(double a, double b) {
  const unsigned long long x = (unsigned long long)__double_as_longlong(a), y = (unsigned long long)__double_as_longlong(b);
  return u32x4{(uint32_t)x, (uint32_t)(x >> 32), (uint32_t)y, (uint32_t)(y >> 32)};
}
__device__ __forceinline__ double unpack_lo(u32x4 v) {
  return __longlong_as_double((long long)(((unsigned long long)v[1] << 32) | v[0]));
}
__device__ __forceinline__ double unpack_hi(u32x4 v) {
  return __longlong_as_double((long long)(((unsigned long long)v[3] << 32) | v[2]));
}

struct ReportIn {
  double ret;
  unsigned long long cnt;
  uint32_t succ;
  double slab[RMX_NSTATS];
};

__device__ __forceinline__ ReportIn report_prefetch(const FastParams& p, int32_t e, bool live) {
  ReportIn r = {0.0, 0ull, 0u, {0.0, 0.0, 0.0, 0.0}};
  if (live) {
    r.ret = p.es_ret[e];
    r.cnt = p.es_cnt[e];
    r.succ = p.es_succ[e];
  }
  const int32_t w = (int32_t)blockIdx.x * p.rpt_cs + (int32_t)threadIdx.x;  // host: rpt_cs <= 64 = blockDim
  if ((int32_t)threadIdx.x < p.rpt_cs && w < p.rpt_n_slab) {
    const double2* q = reinterpret_cast<const double2*>(p.slab + (size_t)w * RMX_NSTATS);
    const double2 a = q[0], b = q[1];
    r.slab[0] = a.x;
    r.slab[1] = a.y;
    r.slab[2] = b.x;
    r.slab[3] = b.y;
  }
  return r;
}

__device__ __forceinline__ void report_tail(const FastParams& p, ReportIn r, uint32_t done, double rs, uint32_t sc,
                                            int32_t t1) {
  if (done) {
    r.ret += rs;
    r.cnt += (unsigned long long)(uint32_t)t1 | (1ull << 40);
    r.succ += sc;
  }
  double v[RMX_NSTATS];
  v[RMX_STAT_SUM_RETURN] = r.ret + r.slab[RMX_STAT_SUM_RETURN];
  v[RMX_STAT_EPISODES] = (double)(r.cnt >> 40) + r.slab[RMX_STAT_EPISODES];
  v[RMX_STAT_SUCCESSES] = (double)r.succ + r.slab[RMX_STAT_SUCCESSES];
  v[RMX_STAT_SUM_LENGTH] = (double)(r.cnt & ((1ull << 40) - 1)) + r.slab[RMX_STAT_SUM_LENGTH];
#pragma unroll
  for (int k = 0; k < RMX_NSTATS; ++k) v[k] = wave_sum_f64(v[k]);  // every lane holds the block sum
  // partials through a buffer descriptor with sc1 (the agent-scope atomic store / load forms): the last block
  // issues all of its partial loads before it waits on any (a chunk of 16 blocks per lane; out-of-range reads
  // of the descriptor return 0), one memory round trip per 1,024 blocks instead of one per 64
  const auto rp = col_rsrc(p.rpt_partial, gridDim.x * (uint32_t)(RMX_NSTATS * 8));
  uint32_t last = 0;
  if (threadIdx.x == 0) {
    const uint32_t o = blockIdx.x * (uint32_t)(RMX_NSTATS * 8);
    __builtin_amdgcn_raw_buffer_store_b128(pack2(v[0], v[1]), rp, o, 0, kStoreAux);
    __builtin_amdgcn_raw_buffer_store_b128(pack2(v[2], v[3]), rp, o + 16u, 0, kStoreAux);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_waitcnt(0);  // the partial stores have completed (gfx9: stores count in vmcnt)
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    // two-level ticket: one arrival per block on its shard counter (blocks b = s mod kRptShards), then one per
    // shard on the root counter from the shard's last arriver.  One counter taking all 1,024 arrivals serialises
    // them (~12 ns each, MI355X_MICROARCH.md "fanin"), ~12 us per report.  Counters are re-armed by the block
    // that saw them complete (no other block touches them again in this launch).
    const uint32_t sh = blockIdx.x % kRptShards;
    const uint32_t n_sh = (gridDim.x - sh + kRptShards - 1) / kRptShards;  // blocks of this shard
    unsigned int* ctr = p.rpt_ticket + (1u + sh) * kRptLineWords;
    if (__hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == n_sh - 1u) {
      __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t n_root = gridDim.x < kRptShards ? gridDim.x : kRptShards;
      last = __hip_atomic_fetch_add(p.rpt_ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == n_root - 1u;
    }
  }
  if (!__builtin_amdgcn_readfirstlane(last)) return;  // lane 0 is active here: its value, wave-uniform
  double acc[RMX_NSTATS] = {0.0, 0.0, 0.0, 0.0};
  constexpr uint32_t kPer = 16;
  for (uint32_t c = 0; c < gridDim.x; c += 64u * kPer) {
    u32x4 lo[kPer], hi[kPer];
#pragma unroll
    for (uint32_t j = 0; j < kPer; ++j) {
      const uint32_t o = (c + j * 64u + threadIdx.x) * (uint32_t)(RMX_NSTATS * 8);
      lo[j] = __builtin_amdgcn_raw_buffer_load_b128(rp, o, 0, kStoreAux);
      hi[j] = __builtin_amdgcn_raw_buffer_load_b128(rp, o + 16u, 0, kStoreAux);
    }
#pragma unroll
    for (uint32_t j = 0; j < kPer; ++j) {
      acc[0] += unpack_lo(lo[j]);
      acc[1] += unpack_hi(lo[j]);
      acc[2] += unpack_lo(hi[j]);
      acc[3] += unpack_hi(hi[j]);
    }
  }
#pragma unroll
  for (int k = 0; k < RMX_NSTATS; ++k) acc[k] = wave_sum_f64(acc[k]);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < RMX_NSTATS; ++k) p.rpt_out[k] = acc[k];
    __hip_atomic_store(p.rpt_ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-armed
  }
}



// Table access: from the LDS copy (staged per block) or straight from the global blob through a buffer
// descriptor (L1/L2-resident after the first touch; no staging, no block barrier).
struct LdsTables {
  const unsigned char* base;
  int32_t off_rm, off_info;
  __device__ __forceinline__ uint32_t mv(uint32_t i) const { return reinterpret_cast<const uint32_t*>(base)[i]; }
  __device__ __forceinline__ uint4 rm(uint32_t i) const { return reinterpret_cast<const uint4*>(base + off_rm)[i]; }
  __device__ __forceinline__ uint4 info(uint32_t a) const { return reinterpret_cast<const uint4*>(base + off_info)[a]; }
};
struct GlobalTables {
  __amdgpu_buffer_rsrc_t r;
  int32_t off_rm, off_info;
  __device__ __forceinline__ uint32_t mv(uint32_t i) const { return __builtin_amdgcn_raw_buffer_load_b32(r, i * 4u, 0, 0); }
  __device__ __forceinline__ uint4 rm(uint32_t i) const {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, i * 16u, off_rm, 0);
    return make_uint4(v[0], v[1], v[2], v[3]);
  }
  __device__ __forceinline__ uint4 info(uint32_t a) const {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, a * 16u, off_info, 0);
    return make_uint4(v[0], v[1], v[2], v[3]);
  }
};

struct AgentIO {
  int32_t x, y, q, act;
  uint32_t f;
  float ret;
};

struct AgentRes {
  float reward, shaping, renv;
  uint32_t term, trunc, succ;  // 0/1
};

// One wrapper step of one agent (rm_environment_wrapper.py:43-107 over ma_frozen_lake.py:96-154 /
// ma_office.py:122-202), in three stages so that a caller can issue every agent's table lookup of one
// stage before waiting on any of them (two dependent lookups per step, not two per agent):
//   move_index -> tb.mv(index) -> rm_index -> tb.rm(index) -> finish.
// The autoreset has already been applied to s.  fq = final RM state (255: none); mvb / rmb = the
// agent's table bases.
struct AgentTmp {
  uint32_t active, at_final, moving, mm;
};

// The action the agent takes this step (wait when frozen or inactive) and its activity flags.
template <int KIND>
__device__ __forceinline__ uint32_t agent_action(const AgentIO& s, uint32_t fq, uint32_t& bad, AgentTmp& k) {
  k.active = s.f & RMX_F_ACTIVE;
  k.at_final = (uint32_t)s.q == fq ? 1u : 0u;
  // FL: inactive or RM already final (pre-step) agents are frozen; OW: every active agent moves
  k.moving = (KIND == RMX_FROZEN_LAKE) ? (k.active & (k.at_final ^ 1u)) : k.active;
  bad |= (uint32_t)s.act > (uint32_t)RMX_WAIT ? 1u : 0u;
  return k.moving ? min((uint32_t)s.act, (uint32_t)RMX_WAIT) : (uint32_t)RMX_WAIT;  // invalid -> wait
}

template <int KIND>
__device__ __forceinline__ uint32_t move_index(const AgentIO& s, uint32_t fq, uint32_t mvb, const FastParams& p,
                                               uint32_t& bad, AgentTmp& k) {
  const uint32_t ac = agent_action<KIND>(s, fq, bad, k);
  const uint32_t cell = __umul24((uint32_t)s.y, (uint32_t)p.W) + (uint32_t)s.x;
  return mvb + __umul24(cell, 5u) + ac;
}

// Decodes the move word into s.x / s.y, returns the RM entry index of (q, event at the new cell).
__device__ __forceinline__ uint32_t rm_index(AgentIO& s, uint32_t m, uint32_t rmb, const FastParams& p, AgentTmp& k) {
  k.mm = k.moving ? m : 0u;  // wall / hazard / fail bits only for a moving agent
  s.x = (int32_t)(m & 0xFFu);
  s.y = (int32_t)__builtin_amdgcn_ubfe(m, 8, 8);
  return rmb + __umul24((uint32_t)s.q, (uint32_t)p.E) + __builtin_amdgcn_ubfe(m, 16, 8);
}


// r = {next_q | final << 8, reward_modifier * RQ, shaping, 0}
template <int KIND>
__device__ __forceinline__ AgentRes finish(AgentIO& s, const AgentTmp& k, uint4 r, int32_t t1, float disc,
                                           const FastParams& p) {
  const uint32_t fail = ((s.f >> 1) | (k.mm >> 26)) & 1u;
  const uint32_t steps_f = s.f + (k.moving << RMX_F_STEPS_SHIFT);  // agent_steps += 1 in the top half
  float rv;
  uint32_t trunc, env_term;
  if (KIND == RMX_FROZEN_LAKE) {
    rv = (k.mm & kMvHazard) ? p.hazard_penalty : 0.0f;
    trunc = ((steps_f >> RMX_F_STEPS_SHIFT) > (uint32_t)p.max_t || t1 > p.max_t) ? 1u : 0u;
    env_term = trunc | k.at_final | fail;  // RM state read before the wrapper's RM step
  } else {
    rv = (k.mm & kMvWall) ? p.wall_penalty : 0.0f;
    rv = (k.mm & kMvHazard) ? rv + p.hazard_penalty : rv;
    trunc = t1 > p.max_t ? 1u : 0u;
    env_term = fail;
  }
  const uint32_t still = k.active & ((env_term | trunc) ^ 1u);
  const uint32_t rm_term = __builtin_amdgcn_ubfe(r.x, 8, 1);
  s.q = (int32_t)(r.x & 0xFFu);
  AgentRes o;
  o.reward = rv + __uint_as_float(r.y);
  o.shaping = __uint_as_float(r.z);
  o.renv = rv;
  o.term = env_term | rm_term;
  o.trunc = trunc;
  s.f = (steps_f & 0xFFFF0000u) | still | (fail << 1) | (o.term << 2) | (trunc << 3) | (env_term << 4) | (rm_term << 5);
  s.ret = fmaf(disc, o.reward, s.ret);
  o.succ = (rm_term && s.ret > 0.0f) ? 1u : 0u;  // success: RM final at episode end with return > 0
  return o;
}

// Diagnostic in-kernel stamps (RMX_DIAG builds with a stamp buffer): wait for every outstanding memory
// operation, then read the shader clock and the 100 MHz real-time clock.
#ifdef RMX_DIAG
// (diag bit 0x100000: entry and exit stamps only — the wave's span with no memory waits inserted in between)
#define STAMP(i)                                                                                             \
  if (p.stamps && ((i) == 0 || (i) == 8 || !(p.diag & 0x100000))) {                                         \
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" \
                 : "=s"(st_clk[i]), "=s"(st_rt[i]));                                                           \
  }
// STAMP_VM(i, n): wait until at most n vector-memory operations are outstanding (in-order), then stamp.
#define STAMP_VM(i, n)                                                                                       \
  if (p.stamps) {                                                                                            \
    asm volatile("s_waitcnt vmcnt(%2)\n\ts_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)"         \
                 : "=s"(st_clk[i]), "=s"(st_rt[i])                                                             \
                 : "n"(n)                                                                                   \
                 : "memory");                                                                               \
  }
#else
#define STAMP(i)
#define STAMP_VM(i, n)
#endif

template <bool GTAB>
__device__ __forceinline__ auto make_tables(const unsigned char* lds, const FastParams& p) {
  if constexpr (GTAB)
    return GlobalTables{col_rsrc(p.tables, (uint32_t)p.n16 * 16u), p.off_rm, p.off_info};
  else
    return LdsTables{lds, p.off_rm, p.off_info};
}


}  // namespace

// ------------------------------------------------------------------------------------------------
// Thread-per-env: lane e runs env e's A agents.
// ------------------------------------------------------------------------------------------------
// QXB: 0 = no QRM outputs; 4 / 8 / 16 = QRM outputs with at most QXB experiences per agent (register
// budget of the counterfactual lookups, which are all issued before any store: vmcnt counts stores too).
// SKIP: which column words the step leaves unchanged are not stored again (per-lane masked store, skipped
// for the whole wave when no lane changed it).  kSkipRare (the default): rm_q and ep_ret only, which a step
// rarely changes: 3-5 % faster than kSkipNone on all four configs at 65,536 envs and 10-17 % faster than
// kSkipAll at 8.4M envs (profiles/r02_ab_log.md ab3, ab4, abbig).  kSkipAll (every unchanged word) writes
// partial lines of the x / y / flags columns, which change for most lanes, and loses at both sizes.
// The leading scalar arguments are the ones the first loads need: built with -amdgpu-kernarg-preload-count=8
// (Makefile: the 8 leading arguments, 14 SGPRs), the CP preloads them into SGPRs at wave launch, so the column
// loads issue without waiting on a kernarg fetch (FastParams, read with s_load, feeds everything later).
// RPT: rmx_step_report — the step followed by the statistics report in the same launch (report_tail).
// SLIP: the stochastic dynamics ahead of the merged-record lookup, which is then keyed by the drawn action.
//   FrozenLake (ma_frozen_lake.py:244-298): one rng.choice per active, non-frozen agent, in agent order, from the
//   env's PCG64, reseeded by the reset-seed schedule at autoreset.
//   OfficeWorld (ma_office.py:150-159, 327-379): the wall penalty follows the INTENDED action and the move the
//   drawn one, and the draw happens only for an action that was not blocked: every agent's intended record is
//   fetched first (its wall bit = can_move of the current cell), then the draws run in agent order (a blocked
//   agent waits and does not draw), then the records of the final actions, whose wall / fail bits are replaced
//   by the intended action's (a slipped move into a wall just does not move: no penalty).
// FrozenLake random_start_positions on the fast path (ma_frozen_lake.py:59-64, 156-172): this episode's start
// cells from the freshly seeded env rng.  The same draws as shuffle_slots (rmx_device.h), but the accepted j_i
// go to LDS, one byte each (n_free <= 256, host), lane-interleaved so that every access is conflict-free: byte i
// of lane l sits in dword (i >> 2) * 64 + l of the wave's area.  The undo pass then reads them back four at a
// time with no global round trip, and the x-major free cells come from a per-wave LDS copy staged by the
// whole wave (the caller's wave-uniform branch) while the draws run.  Per wave: rs_wave_lds(n) bytes (rmx_internal.h).
// Measured r03: the generic kernel's array shuffle (a dependent global read-modify-write per swap) ran config 2
// at 54.5 us per step; the global-row form of shuffle_slots at 34-35 us.

template <int A>
__device__ __forceinline__ void shuffle_slots_lds(Pcg& r, int32_t n, unsigned char* __restrict__ wl, uint32_t lane,
                                                  int32_t (&slot)[A]) {
  int32_t i = n - 1;
  uint32_t mask = (uint32_t)max(i, 0);
  mask |= mask >> 1;
  mask |= mask >> 2;
  mask |= mask >> 4;
  mask |= mask >> 8;
  auto take = [&](uint32_t d) {
    const uint32_t v = d & mask;
    if (i > 0 && v <= (uint32_t)i) {
      wl[((((uint32_t)i >> 2) << 6) + lane) * 4u + ((uint32_t)i & 3u)] = (unsigned char)v;
      --i;
      mask = (uint32_t)i <= (mask >> 1) ? (mask >> 1) : mask;
    }
  };
  while (i > 0) {
    const uint64_t o = pcg_next64(r);
    take((uint32_t)o);
    take((uint32_t)(o >> 32));
  }
  asm volatile("" ::: "memory");
#pragma unroll
  for (int a = 0; a < A; ++a) slot[a] = a;
  const uint32_t* w32 = reinterpret_cast<const uint32_t*>(wl);
  const int32_t n4 = (n + 3) >> 2;
#pragma unroll 4
  for (int32_t c = 0; c < n4; ++c) {
    const uint32_t w = w32[((uint32_t)c << 6) + lane];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int32_t ii = c * 4 + k;
      const int32_t jj = (int32_t)__builtin_amdgcn_ubfe(w, 8 * k, 8);
      if (ii >= 1 && ii < n) {
#pragma unroll
        for (int a = 0; a < A; ++a) slot[a] = slot[a] == ii ? jj : (slot[a] == jj ? ii : slot[a]);
      }
    }
  }
}

// The autoreset's reseed (env.rng = default_rng(seed of the next episode)) and, with random starts, the episode's
// start cells: lanes whose env resets draw; the wave stages the free cells if any of its lanes does (uniform).
template <int A, bool RSTART>
__device__ __forceinline__ void random_start_reset(const FastParams& p, Pcg& rng, int32_t& episode, bool rs, bool live,
                                                   int64_t e_global, unsigned char* lds, uint32_t tid, uint32_t lds_off,
                                                   int32_t (&sx)[A], int32_t (&sy)[A]) {
  const bool any_rs = RSTART && __any(rs && live);
  uint32_t fc0 = 0, fc1 = 0;
  const uint32_t lane = tid & 63u;
  const int32_t n = p.n_free;
  unsigned char* wl = lds + lds_off + (tid >> 6) * (uint32_t)rs_wave_lds(n);
  if (any_rs) {  // this wave's copy of the free cells (u16 pairs, the host pads the last one; dwords beyond read 0),
                 // in flight with the draws
    const auto rf = col_rsrc(p.free_cells, ((uint32_t)n * 2u + 3u) & ~3u);
    fc0 = __builtin_amdgcn_raw_buffer_load_b32(rf, lane * 4u, 0, 0);
    fc1 = __builtin_amdgcn_raw_buffer_load_b32(rf, lane * 4u + 256u, 0, 0);
  }
  int32_t slot[A];
  if (rs) {
    episode += 1;
    // (computed instead by the episode's last step after its stores, config 2 with slip ran 10 % slower:
    // profiles/r06_ab_log.md "lateseed")
    rng = seed_pcg64(seed_of(p, e_global, episode));
    if (RSTART && live) shuffle_slots_lds<A>(rng, n, wl, lane, slot);  // before any slip draw of the episode
  }
  if (any_rs) {
    uint32_t* cw = reinterpret_cast<uint32_t*>(wl + 256 * ((n + 3) >> 2));
    cw[lane] = fc0;
    cw[lane + 64] = fc1;
    asm volatile("" ::: "memory");
    if (rs && live) {
      const uint16_t* cells = reinterpret_cast<const uint16_t*>(cw);
#pragma unroll
      for (int a = 0; a < A; ++a) {
        const int32_t c = (int32_t)cells[slot[a]];
        sx[a] = c % p.W;
        sy[a] = c / p.W;
      }
    }
  }
}

// ---- random starts in the step kernel: the NEXT episode's shuffle, a few draws per step --------------------------
// The draws of a reset's shuffle (~65-75 PCG64 outputs for map1's 89 free cells) held a whole wave for one lane:
// ~6 % of lanes reset per step, so nearly every wave paid ~10-20 us (profiles/r03_ab_log.md randstart).  The
// shuffle of episode k+1 depends only on (env, k+1), so every lane works on its NEXT episode's generator while
// the current episode runs: kRsDrawsPerStep draws per step (the same on every lane: no divergence), the accepted
// j_i written to the env's workspace row (one byte each).  At the reset the lane finishes what is left (the
// episode was shorter than the precompute), undoes the swaps for its A slots from the row, continues the episode
// with the generator's post-shuffle state (slip draws), and starts on the episode after.  The precompute state
// (generator, remaining index, episode tag) lives in handle-owned columns; a tag that is not the expected episode
// (after rmx_reset / rmx_set_state, or steps of another kernel family) restarts it, so it is never wrong, only late.
constexpr int kRsDrawsPerStep = 8;
// step-kernel LDS per wave with random starts: the free-cell copies (512 B), then rs_coop_finish's output blocks
// (kRsWaveLds, kRsRowMax: rmx_internal.h)

// an env's PCG64 from a [4][N] u64 column set (state hi, lo, increment hi, lo; buffer descriptor: N < 2^27 on host)
__device__ __forceinline__ Pcg ld_pcg(const uint64_t* base, int32_t N, int32_t e) {
  const auto r = col_rsrc(base, (uint32_t)N * 32u);
  const uint32_t o8 = (uint32_t)e * 8u, c8 = (uint32_t)N * 8u;
  const auto w0 = __builtin_amdgcn_raw_buffer_load_b64(r, o8, 0, 0);
  const auto w1 = __builtin_amdgcn_raw_buffer_load_b64(r, o8, c8, 0);
  const auto w2 = __builtin_amdgcn_raw_buffer_load_b64(r, o8, 2u * c8, 0);
  const auto w3 = __builtin_amdgcn_raw_buffer_load_b64(r, o8, 3u * c8, 0);
  return {((uint64_t)w0[1] << 32) | w0[0], ((uint64_t)w1[1] << 32) | w1[0], ((uint64_t)w2[1] << 32) | w2[0],
          ((uint64_t)w3[1] << 32) | w3[0]};
}

// FIXED random starts: agent a's cached start cell (x | y << 8, two agents per word)
template <int A>
__device__ __forceinline__ void fixed_start_cells(const uint32_t (&fcw)[(A + 1) / 2], int32_t (&sx)[A], int32_t (&sy)[A]) {
#pragma unroll
  for (int a = 0; a < A; ++a) {
    const uint32_t c = __builtin_amdgcn_ubfe(fcw[a >> 1], 16 * (a & 1), 16);
    sx[a] = (int32_t)(c & 0xFFu);
    sy[a] = (int32_t)(c >> 8);
  }
}

struct RsNext {
  Pcg g;       // the next episode's generator, advanced through its shuffle so far
  int32_t i;   // shuffle index still to draw for (0: all drawn)
  int32_t k;   // the episode it serves
  int32_t i0;  // i as loaded (the index column is stored only when it moved)
  bool fresh;  // seeded in this step: the increment words and the tag are stored too
};

// The row a shuffle's draws leave behind is not the list of j_i but what the undo needs of it.  Undoing the swaps
// for slot p runs pos = p through i = 1 .. n-1 (pos == i -> j_i, pos == j_i -> i); once i >= A > pos, only
// "pos == j_i -> pos = i" can fire, so after the first A - 1 swaps pos follows first occurrences:
// F[x] = min { i : j_i = x, i > x } for x >= A, and min { i >= A : j_i = x } for x < A (0: none).  Drawing in
// decreasing i, the last write of F[x] is that minimum.  Row layout (bytes): F[0 .. n), j_1 .. j_{A-1} at
// n + 1 .. n + A - 1, a dummy byte at n + 7 for draws that record nothing; rows are zeroed when a shuffle starts.
// The undo then walks ~3 first-occurrence hops per slot (rs_undo_chain) instead of all n swaps.  Recording costs
// ~6 more instructions per draw: it pays from A = 3 on (config 4 24.5 -> 19.8 us per step); A <= 2 keeps the
// plain j_i row and the full undo (config 2 20.6 vs 23.7 us, same box, profiles/r03_ab_log.md rschain).
template <bool CHAIN>
__device__ __forceinline__ void rs_take(RsNext& nx, uint32_t& mask, uint32_t d, unsigned char* row, int32_t n, int A) {
  const uint32_t v = d & mask;
  const int32_t i = nx.i;
  const bool ok = i > 0 && v <= (uint32_t)i;
  if constexpr (CHAIN) {
    const bool rec = ok && ((int32_t)v < A ? i >= A : (int32_t)v < i);
    const bool ini = ok && i < A;  // (exclusive with rec)
    row[rec ? (int32_t)v : (ini ? n + i : n + 7)] = (unsigned char)(rec ? i : (int32_t)v);
  } else {
    row[i] = (unsigned char)v;  // j_i itself (rs_undo_full)
  }
  nx.i -= ok ? 1 : 0;
  mask = (uint32_t)nx.i <= (mask >> 1) ? (mask >> 1) : mask;
}

// a shuffle starts: no first occurrences yet (the row's first n bytes; 16-B aligned rows)
__device__ __forceinline__ void rs_clear_row(unsigned char* row, int32_t n) {
  uint4* r = reinterpret_cast<uint4*>(row);
  for (int32_t c = 0; c < (n + 15) >> 4; ++c) r[c] = make_uint4(0u, 0u, 0u, 0u);
}

__device__ __forceinline__ uint32_t rs_mask(int32_t i) {
  uint32_t m = (uint32_t)max(i, 0);
  m |= m >> 1;
  m |= m >> 2;
  m |= m >> 4;
  return m;  // n <= 256 on this path
}

// at most `outputs` PCG64 outputs (two draws each) of nx's shuffle
template <bool CHAIN>
__device__ __forceinline__ void rs_draws(RsNext& nx, unsigned char* row, int outputs, int32_t n, int A) {
  uint32_t mask = rs_mask(nx.i);
  for (int k = 0; k < outputs && nx.i > 0; ++k) {  // per lane: stops once its shuffle is drawn
    const uint64_t o = pcg_next64(nx.g);
    rs_take<CHAIN>(nx, mask, (uint32_t)o, row, n, A);
    rs_take<CHAIN>(nx, mask, (uint32_t)(o >> 32), row, n, A);
  }
}

// A <= 2: the row holds j_i at byte i (a rejected draw's byte overwritten by the accepted one) and the undo runs
// all n - 1 swaps for the A slots (shuffle_slots), the row's loads in flight together
template <int A>
__device__ __forceinline__ void rs_undo_full(const unsigned char* row, int32_t n, int32_t (&slot)[A]) {
#pragma unroll
  for (int a = 0; a < A; ++a) slot[a] = a;
  typedef uint4 __attribute__((may_alias)) uint4_alias;
  const uint4_alias* rv = reinterpret_cast<const uint4_alias*>(row);
  const int32_t n16 = (n + 15) >> 4;
  for (int32_t c = 0; c < n16; c += 8) {  // 128 entries per round, their loads issued together
    uint4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = c + k < n16 ? rv[c + k] : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int k = 0; k < 128; ++k) {
      const int32_t ii = c * 16 + k;
      const uint4 vk = v[k >> 4];
      const uint32_t wd = (k & 12) == 0 ? vk.x : (k & 12) == 4 ? vk.y : (k & 12) == 8 ? vk.z : vk.w;
      const int32_t jj = (int32_t)__builtin_amdgcn_ubfe(wd, 8 * (k & 3), 8);
      if (ii >= 1 && ii < n) {
#pragma unroll
        for (int a = 0; a < A; ++a) slot[a] = slot[a] == ii ? jj : (slot[a] == jj ? ii : slot[a]);
      }
    }
  }
}

// the A start slots from a completely drawn row: the first A - 1 swaps from j_1 .. j_{A-1}, then the first-
// occurrence hops (rs_take).  The row is copied into this lane's LDS area first (every load in flight at once),
// so a hop is an LDS byte read instead of a dependent global load.
template <int A>
__device__ __forceinline__ void rs_undo_chain(const unsigned char* row, int32_t n, unsigned char* lrow,
                                              int32_t (&slot)[A]) {
  typedef uint4 __attribute__((may_alias)) uint4_alias;
  const uint4_alias* rv = reinterpret_cast<const uint4_alias*>(row);
  uint4_alias* lv = reinterpret_cast<uint4_alias*>(lrow);
  const int32_t nch = (n + 8 + 15) >> 4;  // F, the initial j's, the dummy: <= kRsRowMax bytes
  uint4 v[kRsRowMax / 16];
#pragma unroll
  for (int c = 0; c < kRsRowMax / 16; ++c) v[c] = c < nch ? rv[c] : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
  for (int c = 0; c < kRsRowMax / 16; ++c)
    if (c < nch) lv[c] = v[c];
  asm volatile("" ::: "memory");
#pragma unroll
  for (int a = 0; a < A; ++a) {
    int32_t pos = a;
#pragma unroll
    for (int k = 1; k < A; ++k) {
      const int32_t jk = lrow[n + k];
      pos = pos == k ? jk : (pos == jk ? k : pos);
    }
    for (int32_t h = 0; h < n; ++h) {  // ~3 hops on average; each hop strictly increases pos
      const int32_t f = lrow[pos];
      if (f == 0) break;
      pos = f;
    }
    slot[a] = pos;
  }
}

// ---- a reset whose shuffle is not drawn yet: the whole wave generates its draws -----------------------------------
// An episode of a few steps leaves the next shuffle partly undrawn, and with 1,024 waves some wave meets such a
// reset every step; drawn by its own lane, the rest of the shuffle is a chain of up to ~65 dependent PCG64 outputs
// (r03r: ~24 us per step).  Here the generation is parallel: for each such lane L in turn, lane j of the wave
// computes L's generator state after output j+1 in one jump, s_{j+1} = M^{j+1} s + (1 + M + ... + M^j) c
// (mod 2^128; host table FastParams::rs_jump), into an LDS block of the wave (16 B per output).  Then every such
// lane scans its own block at once: XSL-RR of each state, two draws, the accepted j_i to its row as before.  64
// outputs per round; a lane whose shuffle needs more starts the next round from output 64's state.  The
// post-shuffle generator is the state of the last output used.  The XSL-RR outputs are computed in the parallel
// phase too (a lane's scan then only reads them: the output function costs more than the state step, r03 probe).
// Up to kRsCoopLanes lanes per round; LDS per wave: kRsCoopLanes * 64 * (16 + 8) B after the free-cell copies.
constexpr int kRsCoopLanes = 8;
typedef unsigned __int128 u128;
__device__ __forceinline__ uint64_t rl64(uint64_t v, int l) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l) << 32) |
         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
}

template <bool CHAIN>
__device__ __forceinline__ void rs_coop_finish(const FastParams& p, RsNext& nx, bool need, unsigned char* row,
                                               uint32_t lane, uint4* blk, int32_t n, int A) {
  uint2* outs = reinterpret_cast<uint2*>(blk + kRsCoopLanes * 64);  // the outputs of the states in blk
  if (!__any(need)) return;
  const uint4 m4 = p.rs_jump[2 * lane], s4 = p.rs_jump[2 * lane + 1];  // M^(lane+1), S_(lane+1)
  const u128 MJ = ((u128)(((uint64_t)m4.w << 32) | m4.z) << 64) | (((uint64_t)m4.y << 32) | m4.x);
  const u128 SJ = ((u128)(((uint64_t)s4.w << 32) | s4.z) << 64) | (((uint64_t)s4.y << 32) | s4.x);
  bool mine = need;
  while (true) {
    uint64_t todo = __ballot(mine && nx.i > 0);
    if (todo == 0) break;
    int slot_of_me = -1;
    for (int g = 0; g < kRsCoopLanes && todo != 0; ++g) {  // generation: one jump per lane per served lane
      const int L = __builtin_ctzll(todo);
      todo &= todo - 1;
      const u128 s = ((u128)rl64(nx.g.hi, L) << 64) | rl64(nx.g.lo, L);
      const u128 c = ((u128)rl64(nx.g.ihi, L) << 64) | rl64(nx.g.ilo, L);
      const u128 sl = MJ * s + SJ * c;
      const uint64_t hi = (uint64_t)(sl >> 64), lo = (uint64_t)sl;
      blk[g * 64 + lane] = make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
      const uint64_t x = hi ^ lo;  // the output too, here where all 64 lanes compute one each
      const unsigned rot = (unsigned)(hi >> 58);
      const uint64_t o = (x >> rot) | (x << ((64u - rot) & 63u));
      outs[g * 64 + lane] = make_uint2((uint32_t)o, (uint32_t)(o >> 32));
      slot_of_me = (int)lane == L ? g : slot_of_me;
    }
    asm volatile("" ::: "memory");
    if (slot_of_me >= 0) {  // scan: this lane's 64 outputs in order
      uint32_t mask = rs_mask(nx.i);
      const uint2* mo = outs + slot_of_me * 64;
      int q = 0;
      for (; q < 64 && nx.i > 0; ++q) {
        const uint2 o = mo[q];
        rs_take<CHAIN>(nx, mask, o.x, row, n, A);
        if (nx.i > 0) rs_take<CHAIN>(nx, mask, o.y, row, n, A);
      }
      const uint4 last = blk[slot_of_me * 64 + q - 1];  // the generator after the last output used (or output 64)
      nx.g.hi = ((uint64_t)last.w << 32) | last.z;
      nx.g.lo = ((uint64_t)last.y << 32) | last.x;
    }
    asm volatile("" ::: "memory");
  }
}

// The step kernel's autoreset reseed with random starts (incremental form): see above.  `rng` / `episode` are the
// env's current generator and episode; on a reset they become the new episode's (post-shuffle generator).
template <int A>
__device__ __forceinline__ void rs_step(const FastParams& p, Pcg& rng, int32_t& episode, RsNext& nx, bool rs, bool live,
                                        int64_t e_global, unsigned char* row, unsigned char* lds, uint32_t tid,
                                        int32_t (&sx)[A], int32_t (&sy)[A]) {
  const int32_t n = p.n_free;
  constexpr bool CHAIN = A >= 3;  // first-occurrence rows (rs_take)
  const bool any_rs = __any(rs && live);
  uint32_t fc0 = 0, fc1 = 0;
  const uint32_t lane = tid & 63u;
  if (any_rs) {  // this wave's copy of the free cells (u16 pairs; the host pads the last one), in flight meanwhile
    const auto rf = col_rsrc(p.free_cells, ((uint32_t)n * 2u + 3u) & ~3u);
    fc0 = __builtin_amdgcn_raw_buffer_load_b32(rf, lane * 4u, 0, 0);
    fc1 = __builtin_amdgcn_raw_buffer_load_b32(rf, lane * 4u + 256u, 0, 0);
  }
  if (rs) episode += 1;
  const int32_t want = rs ? episode : episode + 1;  // the episode whose shuffle the precompute must serve now
  if (live && nx.k != want) {  // (re)start: after a reset / restore / another kernel family's steps
    nx.g = seed_pcg64(seed_of(p, e_global, want));
    nx.i = n - 1;
    nx.k = want;
    nx.fresh = true;
    if constexpr (CHAIN) rs_clear_row(row, n);
  }
  int32_t slot[A];
  if (any_rs)  // resets whose shuffle is not fully drawn yet: the wave generates the rest (then it is)
    rs_coop_finish<CHAIN>(p, nx, rs && live && nx.i > 0, row, lane,
                   reinterpret_cast<uint4*>(lds + (tid >> 6) * (uint32_t)kRsWaveLds + 512u), n, A);
  if (rs) {
    if (live) {
      asm volatile("" ::: "memory");
      // every draw is in the row now: undo for the A slots (this lane's LDS area: the cooperative blocks, done)
      if constexpr (CHAIN)
        rs_undo_chain<A>(row, n, lds + (tid >> 6) * (uint32_t)kRsWaveLds + 512u + lane * (uint32_t)kRsRowMax, slot);
      else
        rs_undo_full<A>(row, n, slot);
      rng = nx.g;  // the episode's generator after its shuffle (slip draws continue from here)
      nx.g = seed_pcg64(seed_of(p, e_global, episode + 1));  // and on to the next episode
      nx.i = n - 1;
      nx.k = episode + 1;
      nx.fresh = true;
      if constexpr (CHAIN) rs_clear_row(row, n);
    } else {
      rng = seed_pcg64(seed_of(p, e_global, episode));  // tail lanes: never stored
    }
  }
  if (__any(live && nx.i > 0)) {  // this step's share of the next episode's draws, on every lane alike
    if (live) rs_draws<CHAIN>(nx, row, kRsDrawsPerStep / 2, n, A);
  }
  if (any_rs) {
    uint32_t* cw = reinterpret_cast<uint32_t*>(lds + (tid >> 6) * (uint32_t)kRsWaveLds);
    cw[lane] = fc0;
    cw[lane + 64] = fc1;
    asm volatile("" ::: "memory");
    if (rs && live) {
      const uint16_t* cells = reinterpret_cast<const uint16_t*>(cw);
#pragma unroll
      for (int a = 0; a < A; ++a) {
        const int32_t c = (int32_t)cells[slot[a]];
        sx[a] = c % p.W;
        sy[a] = c / p.W;
      }
    }
  }
}

template <int KIND, int A, bool HASHED, int TBL, int QXB = 0, int SKIP = kSkipNone, bool RPT = false,
          int SLIP = 0>
__global__ void __launch_bounds__(256) step_fast_kernel(int32_t N_arg, int32_t blk_arg, const int32_t* x_arg,
                                                        const int32_t* y_arg, const int32_t* q_arg,
                                                        const uint32_t* f_arg, const int32_t* t_arg,
                                                        const int32_t* act_arg, FastParams p) {
  constexpr bool QRM = QXB > 0;
  static_assert(TBL == kTblGlobal || TBL == kTblMerged || TBL == kTblMerged4, "step: global or merged tables");
  static_assert(!QRM || TBL == kTblGlobal, "QRM outputs need the move word's event (global tables)");
  // M4: 4-B merged records (move word + palette index of the reward): a b32 gather instead of b128
  constexpr bool M4 = TBL == kTblMerged4;
  constexpr bool MERGED = TBL == kTblMerged || M4;
  constexpr bool STATS_FIRST = KIND == RMX_FROZEN_LAKE && A <= 2;
  // SLIP = kRngSlip | kRngStarts: the env's PCG64 + episode columns (RNG), slip draws (DRAW), FrozenLake random
  // start positions at each autoreset (RSTART)
  constexpr bool RNG = SLIP != 0, DRAW = (SLIP & kRngSlip) != 0;
  constexpr bool RSTART = (SLIP & kRngStarts) != 0 && KIND == RMX_FROZEN_LAKE;
  constexpr int SAUX = SKIP == kSkipRareNT ? kStoreAuxNT : kStoreAux;
  // column store with this instantiation's cache policy (RMX_DIAG diag bit 32: default-policy stores)
  const auto st = [&](__amdgpu_buffer_rsrc_t r, uint32_t lane_bytes, uint32_t sgpr_bytes, int32_t v) {
#ifdef RMX_DIAG
    if (p.diag & 32) {
      __builtin_amdgcn_raw_buffer_store_b32(v, r, lane_bytes, sgpr_bytes, 0);
      return;
    }
#endif
    __builtin_amdgcn_raw_buffer_store_b32(v, r, lane_bytes, sgpr_bytes, SAUX);
  };
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int tid = threadIdx.x;
#ifdef RMX_DIAG
  uint64_t st_clk[kStamps] = {}, st_rt[kStamps] = {};
#endif
  STAMP(0);
  // Preloaded pointers for A >= 3 only: measured (r01_ab_log c80) 9-11 % faster for configs 4 and 5, while for
  // A <= 2 the early load burst made config 2 bimodal (3.11 or 3.55-3.77 us per step with cold actions, vs a
  // steady 3.35-3.40) and config 3 3 % slower; there the kernarg-fetched FastParams pointers are used.
  constexpr bool PRE = A >= 3;
  const int32_t N = PRE ? N_arg : p.N;
#ifdef RMX_DIAG
  // diag 65536: XCD-contiguous env ranges (workgroups are dealt round-robin to the 8 XCDs: give XCD x the
  // x-th eighth of the envs instead of every 8th workgroup's envs)
  uint32_t wg = blockIdx.x;
  if ((p.diag & 65536) && (gridDim.x & 7u) == 0) wg = (wg & 7u) * (gridDim.x >> 3) + (wg >> 3);
  const int32_t e_raw = (int32_t)(wg * blockDim.x) + tid;
#else
  const int32_t e_raw = (int32_t)blockIdx.x * (PRE ? blk_arg : (int32_t)blockDim.x) + tid;  // blk_arg == blockDim.x
#endif
  const bool live = e_raw < N;
  const int32_t e = live ? e_raw : N - 1;  // tail lanes re-read the last env and never store
  const uint32_t off = (uint32_t)e * 4u;
  const uint32_t col = (uint32_t)N * 4u;  // bytes per agent column (A*N*4 < 2^31 on the fast path)
  const uint32_t cols = col * (uint32_t)A;
  const auto r_x = col_rsrc(PRE ? x_arg : p.pos_x, cols), r_y = col_rsrc(PRE ? y_arg : p.pos_y, cols);
  const auto r_q = col_rsrc(PRE ? q_arg : p.rm_q, cols), r_f = col_rsrc(PRE ? f_arg : p.flags, cols);
  const auto r_t = col_rsrc(PRE ? t_arg : p.t, col);
  const auto r_act = col_rsrc(PRE ? act_arg : p.actions, cols), r_rew = col_rsrc(p.reward, cols);
  AgentIO s[A];
  AgentIO s0[A];  // the values as loaded: a column word that the step leaves unchanged is not stored again
  // (`t` first: issued behind agent 0's lookup it cost config 4 1 %, profiles/r06_ab_log.md "t0")
  int32_t t = col_ld(r_t, off, 0);
  __amdgpu_buffer_rsrc_t r_ret;  // built after the preloaded-pointer loads are issued (it needs a kernarg fetch)
  if constexpr (!PRE) {
    r_ret = col_rsrc(p.ep_ret, cols);
#pragma unroll
    for (int a = 0; a < A; ++a) {
      s[a].x = col_ld(r_x, off, a * col);
      s[a].y = col_ld(r_y, off, a * col);
      s[a].q = col_ld(r_q, off, a * col);
      s[a].f = (uint32_t)col_ld(r_f, off, a * col);
      s[a].ret = __int_as_float(col_ld(r_ret, off, a * col));
      s[a].act = HASHED ? hash_action(p.seed, p.t_global, p.n_global, p.env_offset + e, A, a) : col_ld(r_act, off, a * col);
      s0[a] = s[a];
    }
  } else {  // the returns last: their column pointer is the only one not preloaded (needed at the end only)
#pragma unroll
    for (int a = 0; a < A; ++a) {
      s[a].x = col_ld(r_x, off, a * col);
      s[a].y = col_ld(r_y, off, a * col);
      s[a].q = col_ld(r_q, off, a * col);
      s[a].f = (uint32_t)col_ld(r_f, off, a * col);
      s[a].act = HASHED ? hash_action(p.seed, p.t_global, p.n_global, p.env_offset + e, A, a) : col_ld(r_act, off, a * col);
      // agent-major load order (loads return in issue order, so agent 0's words land first): FrozenLake (config 4)
      // 2.9 % faster, OfficeWorld (config 5) 2.5 % slower (profiles/r05_ab_log.md "order")
      if constexpr (KIND == RMX_FROZEN_LAKE) __builtin_amdgcn_sched_barrier(0);
    }
    // keep the kernarg-dependent work below this point: the loads above issue at wave start
    __builtin_amdgcn_sched_barrier(0);
    r_ret = col_rsrc(p.ep_ret, cols);
#pragma unroll
    for (int a = 0; a < A; ++a) {
      s[a].ret = __int_as_float(col_ld(r_ret, off, a * col));
      s0[a] = s[a];
    }
  }
  // slip: the env's PCG64 state and episode counter, with the state loads (buffer descriptors: N < 2^27 on host)
  Pcg rng = {0ull, 0ull, 0ull, 0ull};
  int32_t episode = 0;
  // FIXED (seed_episode_stride == 0): an autoreset copies the env's cached generator (post-seed, and with random
  // starts post-shuffle) and, with random starts, its cached start cells (the reset cache, rmx_internal.h).  Without slip the rng columns change only at a reset, and
  // then only when they may hold another seed's generator (p.rs_dirty): read then, after the table lookups
  // (RNG_LATE), by the lanes that reset.  The episode counter rides in the first load burst (a late load of it made
  // the resetting lanes wait for its round trip before the step logic).
  constexpr bool FIXED = RNG && (SLIP & kRngFixedSeed) != 0;
  constexpr bool FCELLS = FIXED && RSTART;
  constexpr bool RNG_LATE = FIXED && !DRAW;  // (implies random starts)
  if constexpr (RNG && !RNG_LATE) {
    rng = ld_pcg(p.rng, N, e);
    episode = col_ld(col_rsrc(p.episode, (uint32_t)N * 4u), off, 0);
  }
  uint32_t fcw[FCELLS ? (A + 1) / 2 : 1] = {};  // FIXED random starts: the cached start cells, two agents per word
  Pcg frng = {0ull, 0ull, 0ull, 0ull};          // FIXED with slip: the cached post-seed (post-shuffle) generator
  if constexpr (FIXED) {
    if constexpr (FCELLS) {
      const auto r_fc = col_rsrc(p.rs_cells, col * (uint32_t)((A + 1) / 2));
#pragma unroll
      for (int w = 0; w < (A + 1) / 2; ++w) fcw[w] = (uint32_t)col_ld(r_fc, off, (uint32_t)w * col);
    }
    if constexpr (RNG_LATE) episode = col_ld(col_rsrc(p.episode, (uint32_t)N * 4u), off, 0);
    if constexpr (DRAW) {  // the state words; the increment words only when they may differ from the env's own
      if (p.rs_dirty) {
        frng = ld_pcg(p.rs_rng, N, e);
      } else {
        const auto r = col_rsrc(p.rs_rng, (uint32_t)N * 16u);
        const auto w0 = __builtin_amdgcn_raw_buffer_load_b64(r, (uint32_t)e * 8u, 0, 0);
        const auto w1 = __builtin_amdgcn_raw_buffer_load_b64(r, (uint32_t)e * 8u, (uint32_t)N * 8u, 0);
        frng.hi = ((uint64_t)w0[1] << 32) | w0[0];
        frng.lo = ((uint64_t)w1[1] << 32) | w1[0];
      }
    }
  }
  RsNext nx = {{0ull, 0ull, 0ull, 0ull}, 0, -1, 0, false};
  if constexpr (RSTART && !FIXED) {  // the next episode's shuffle in progress: generator [4][N] u64, index [N], episode tag [N]
    const auto r_nx = col_rsrc(p.nx_rng, (uint32_t)N * 32u);
    const uint32_t o8 = (uint32_t)e * 8u, c8 = (uint32_t)N * 8u;
    const auto w0 = __builtin_amdgcn_raw_buffer_load_b64(r_nx, o8, 0, 0);
    const auto w1 = __builtin_amdgcn_raw_buffer_load_b64(r_nx, o8, c8, 0);
    const auto w2 = __builtin_amdgcn_raw_buffer_load_b64(r_nx, o8, 2u * c8, 0);
    const auto w3 = __builtin_amdgcn_raw_buffer_load_b64(r_nx, o8, 3u * c8, 0);
    nx.g = {((uint64_t)w0[1] << 32) | w0[0], ((uint64_t)w1[1] << 32) | w1[0], ((uint64_t)w2[1] << 32) | w2[0],
            ((uint64_t)w3[1] << 32) | w3[0]};
    nx.i = col_ld(col_rsrc(p.nx_idx, (uint32_t)N * 4u), off, 0);
    nx.k = col_ld(col_rsrc(p.nx_ep, (uint32_t)N * 4u), off, 0);
    nx.i0 = nx.i;
  }
  // per-wave statistics mode (large N): this wave's slab slot, in flight with the state loads
  SlabSlot slot = {{0.0, 0.0, 0.0, 0.0}};
  if (p.wave_stats) slot = slab_prefetch(p.slab);
  // fused report: this env's statistics slots and this block's share of the slab, also in flight now
  ReportIn rin;
  if constexpr (RPT) rin = report_prefetch(p, e, live);
  const auto mg = col_rsrc(p.merged, MERGED ? (uint32_t)p.merged_bytes : 0u);
  const auto mg4 = col_rsrc(p.merged4, M4 ? (uint32_t)p.merged4_bytes : 0u);
#ifdef RMX_DIAG
  // diag (timing ablations, never correct results): 1 no stats, 4096 no table lookups, 8192 copy-through (the
  // loads and stores only)
  const int diag = p.diag;
  STAMP(1);
  STAMP(2);
#endif
  const auto tb = make_tables<true>(lds, p);

#ifdef RMX_DIAG
  if (diag & 8192) {  // copy-through: the kernel's loads and stores with no step logic
    if (live) {
      st(r_t, off, 0, t + 1);
      if (p.env_done) byte_st<SAUX>(p, (uint32_t)e, (uint32_t)t & 1u);
#pragma unroll
      for (int a = 0; a < A; ++a) {
        st(r_x, off, a * col, s[a].x + s[a].act);
        st(r_y, off, a * col, s[a].y);
        st(r_q, off, a * col, s[a].q);
        st(r_f, off, a * col, (int32_t)s[a].f);
        st(r_ret, off, a * col, __float_as_int(s[a].ret));
        st(r_rew, off, a * col, s[a].act);
      }
    }
    return;
  }
#endif
  // autoreset: the previous step ended this env's episode -> reference loop reset() before the step
  const bool rs = p.autoreset && (s[0].f & RMX_F_ENV_DONE);
  t = rs ? 0 : t;
  const int32_t t1 = t + 1;
  // OfficeWorld (discounted returns): gamma^t is read AFTER stage 1 has issued the table lookups.  Loads return
  // in issue order, so a discount load issued first puts its own round trip in front of the lookup's (config 3:
  // 2.36 vs 2.43 us per step, r03j).  Config 5 (A = 3) measured neutral to 1 % slower and FrozenLake 5 % slower
  // (the deferred form's scheduling barrier), so they keep the early read.
  constexpr bool LATE_DISC = KIND == RMX_OFFICE_WORLD && A == 1;
  float disc = LATE_DISC ? 1.0f : (p.gamma_is_one ? 1.0f : p.disc[min((uint32_t)t, (uint32_t)p.max_t + 1u)]);
  uint32_t bad = 0, all_term = 1u, all_trunc = 1u;
  // the reset's start cells: the configured ones, or (random starts) this episode's shuffle of the free cells
  int32_t sx[A], sy[A];
#pragma unroll
  for (int a = 0; a < A; ++a) sx[a] = p.start_x[a], sy[a] = p.start_y[a];
  if constexpr (RNG) {  // env.rng = default_rng(seed of the next episode) (rm_environment_wrapper reset)
    if constexpr (FIXED) {  // the same seed every episode: the cached generator (and shuffle's cells)
      if (rs) {
        if constexpr (FCELLS) fixed_start_cells<A>(fcw, sx, sy);
        episode += 1;
        if constexpr (DRAW) {
          rng.hi = frng.hi;
          rng.lo = frng.lo;
          if (p.rs_dirty) {
            rng.ihi = frng.ihi;
            rng.ilo = frng.ilo;
          }
        }
      }
    } else if constexpr (RSTART)
      rs_step<A>(p, rng, episode, nx, rs, live, p.env_offset + e,
                 reinterpret_cast<unsigned char*>(p.start_ws) + (size_t)e * (size_t)(2 * shuffle_stride(p.n_free)), lds,
                 (uint32_t)tid, sx, sy);
    else
      random_start_reset<A, false>(p, rng, episode, rs, live, p.env_offset + e, lds, (uint32_t)tid, 0u, sx, sy);
  }
  AgentTmp k[A];
  uint32_t m[A];
  uint32_t prev_cell[A];
  uint2 qe[A][QXB > 0 ? QXB : 1];  // QRM: {next | final << 8, raw RQ} per hypothetical RM state
  constexpr bool OW_SLIP = DRAW && KIND == RMX_OFFICE_WORLD;
  uint32_t blocked[OW_SLIP ? A : 1] = {};
  if constexpr (OW_SLIP) {
    static_assert(MERGED, "OfficeWorld slip: 16-B or 4-B merged records");
    uint32_t wi[A];
#pragma unroll
    for (int a = 0; a < A; ++a) {  // the intended action's record (word 0) of every agent, in flight together
      s[a].x = rs ? sx[a] : s[a].x;
      s[a].y = rs ? sy[a] : s[a].y;
      s[a].q = rs ? p.init_q[a] : s[a].q;
      s[a].f = rs ? RMX_F_ACTIVE : s[a].f;
      s[a].ret = rs ? 0.0f : s[a].ret;
      const uint32_t mi = move_index<KIND>(s[a], (uint32_t)p.final_q[a], 0u, p, bad, k[a]);
      const uint32_t idx = (uint32_t)p.mg_base[a] + __umul24(__umul24((uint32_t)s[a].q, (uint32_t)p.HW), 5u) + mi;
      wi[a] = M4 ? __builtin_amdgcn_raw_buffer_load_b32(mg4, idx * 4u, 0, 0)
                 : __builtin_amdgcn_raw_buffer_load_b32(mg, idx * 16u, 0, 0);
    }
#pragma unroll
    for (int a = 0; a < A; ++a) {  // apply_wall_penalty, then get_stochastic_action in agent order
      const uint32_t ac = agent_action<KIND>(s[a], (uint32_t)p.final_q[a], bad, k[a]);
      blocked[a] = (ac < (uint32_t)RMX_WAIT && (wi[a] & kMvWall)) ? 1u : 0u;
      s[a].act = (int32_t)(blocked[a] ? (uint32_t)RMX_WAIT
                                      : (ac < (uint32_t)RMX_WAIT ? (uint32_t)slip_choice(p, (int32_t)ac, rng) : ac));
    }
  }
  uint4 r[A];
  AgentRes o[A];
#pragma unroll
  for (int a = 0; a < A; ++a) {  // stage 1: every agent's move-word lookup in flight together
    // (as selects the compiler turns into one exec-masked block for every agent's words; written as bit selects that
    // stay per agent, every config measured 15-23 % slower, profiles/r05_ab_log.md "bfi")
    s[a].x = rs ? sx[a] : s[a].x;
    s[a].y = rs ? sy[a] : s[a].y;
    s[a].q = rs ? p.init_q[a] : s[a].q;
    s[a].f = rs ? RMX_F_ACTIVE : s[a].f;
    // (the return's select stays in this block although its loads are issued last: moved after the lookups, the
    // lookups issued per agent and every config ran 0-3 % slower, profiles/r05_ab_log.md "retsel")
    s[a].ret = rs ? 0.0f : s[a].ret;
    // (every outcome's record fetched before the draw instead, 18-45 % slower: profiles/r06_ab_log.md "spec")
    if constexpr (DRAW && KIND == RMX_FROZEN_LAKE) {  // get_stochastic_action for an active agent whose RM is not final
      if ((s[a].f & RMX_F_ACTIVE) && (uint32_t)s[a].q != (uint32_t)p.final_q[a]) {
        if (s[a].act == RMX_WAIT)
          bad |= 1u;  // the reference's slip map has no "wait" entry (KeyError)
        else if ((uint32_t)s[a].act < (uint32_t)RMX_WAIT)
          s[a].act = slip_choice(p, s[a].act, rng);
      }
    }
#ifdef RMX_DIAG
    if (a == 0) STAMP(3);
    if (diag & 4096) {  // no table lookups: a move word computed from the state
      const uint32_t mi = move_index<KIND>(s[a], (uint32_t)p.final_q[a], (uint32_t)p.mv_base[a], p, bad, k[a]);
      m[a] = (mi & 0x00030303u);
      continue;
    }
#endif
    // (all five actions' records fetched before the action arrived instead, 7-13 % slower: profiles/r06_ab_log.md
    // "all5")
    if constexpr (MERGED) {  // one lookup gives the move and the RM step: stage 2 only decodes
      // the record's byte offset ((q * HW + y * W + x) * 5 + ac + mg_base) * RB with 24-bit multiplies (x, y, q < 256 on
      // the fast path; garbage state stays inside 32 bits and the descriptor's range): __umul24 compiled to the
      // quarter-rate v_mul_lo_u32 / v_mad_u64_u32 (round 5, profiles/r05_ab_log.md "idx")
      const uint32_t ac = agent_action<KIND>(s[a], (uint32_t)p.final_q[a], bad, k[a]);
      constexpr uint32_t RB = M4 ? 4u : 16u;
      const uint32_t hw5 = ((uint32_t)p.HW * (5u * RB)) & 0xFFFFFFu, w5 = ((uint32_t)p.W * (5u * RB)) & 0xFFFFFFu;
      const uint32_t ro = ((uint32_t)s[a].q & 0xFFu) * hw5 + ((uint32_t)s[a].y & 0xFFu) * w5 +
                          ((uint32_t)s[a].x & 0xFFu) * (5u * RB) + (ac + (uint32_t)p.mg_base[a]) * RB;
      if constexpr (M4) {
        r[a] = make_uint4(__builtin_amdgcn_raw_buffer_load_b32(mg4, ro, 0, 0), 0u, 0u, 0u);
      } else {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(mg, ro, 0, 0);
        r[a] = make_uint4(v[0], v[1], v[2], v[3]);
      }
    } else {
      if constexpr (QRM) prev_cell[a] = (uint32_t)(s[a].y * p.W + s[a].x);  // infos prev_s: before the move
      m[a] = tb.mv(move_index<KIND>(s[a], (uint32_t)p.final_q[a], (uint32_t)p.mv_base[a], p, bad, k[a]));
    }
  }
  if constexpr (RNG_LATE) {  // FIXED without slip: a resetting lane's generator, after the lookups, if it may differ
    if (rs && live && p.rs_dirty) rng = ld_pcg(p.rs_rng, N, e);  // (else the env's generator IS the cached one)
  }
  if (LATE_DISC && !p.gamma_is_one) {
    __builtin_amdgcn_sched_barrier(0);
    disc = p.disc[min((uint32_t)t, (uint32_t)p.max_t + 1u)];
  }
#pragma unroll
  for (int a = 0; a < A; ++a) {  // stage 2
#ifdef RMX_DIAG
    if (a == 0) STAMP(4);
    if (diag & 4096) {
      const uint32_t ti = rm_index(s[a], m[a], (uint32_t)p.rm_base[a], p, k[a]);
      r[a] = make_uint4(ti & 3u, 0u, 0u, 0u);
      continue;
    }
#endif
    if constexpr (M4) {  // the palette entry (bits 28-29) as a signed byte of a uniform word: extract + convert; the
                         // float palette picked with two select levels per agent cost ~7 more instructions (round 5,
                         // profiles/r05_ab_log.md "idx"); shaping (r.z) is 0: M4 needs no shaping
      const int32_t pb = __builtin_amdgcn_readfirstlane((int)p.mg_palb[a]);
      r[a].y = __float_as_uint((float)(int32_t)__builtin_amdgcn_sbfe(pb, (r[a].x >> 25) & 0x18u, 8u));
    }
    if constexpr (OW_SLIP) {  // the wall penalty / failure of the intended action, the plant of the final cell
      const uint32_t hz = __builtin_amdgcn_ubfe(r[a].x, 25, 1);
      const uint32_t fl = (blocked[a] & (uint32_t)p.wall_fail) | (hz & (uint32_t)p.hazard_fail);
      r[a].x = (r[a].x & ~(kMvWall | kMvFail)) | (blocked[a] << 24) | (fl << 26);
    }
    if constexpr (MERGED) {
      const uint32_t w0 = r[a].x;
      k[a].mm = k[a].moving ? w0 : 0u;  // wall / hazard / fail at bits 24-26, as in the move word
      s[a].x = (int32_t)(w0 & 0xFFu);
      s[a].y = (int32_t)__builtin_amdgcn_ubfe(w0, 8, 8);
      r[a].x = __builtin_amdgcn_ubfe(w0, 16, 8) | (__builtin_amdgcn_ubfe(w0, 27, 1) << 8);
      continue;
    }
    const uint32_t ti = rm_index(s[a], m[a], (uint32_t)p.rm_base[a], p, k[a]);
    if constexpr (QRM) {  // every hypothetical RM state's entry for the same event, in flight with r[a]
      const uint32_t ev = __builtin_amdgcn_ubfe(m[a], 16, 8);
#pragma unroll
      for (int j = 0; j < QXB; ++j) {
        qe[a][j] = make_uint2(0u, 0u);
        if (j < p.n_qrm[a]) {
          const uint4 v = tb.rm((uint32_t)p.rm_base[a] + (uint32_t)p.qrm_q[a][j] * (uint32_t)p.E + ev);
          qe[a][j] = make_uint2(v.x, v.w);
        }
      }
    }
    r[a] = tb.rm(ti);
  }
  STAMP(5);
#pragma unroll
  for (int a = 0; a < A; ++a) {
    o[a] = finish<KIND>(s[a], k[a], r[a], t1, disc, p);
    all_term &= o[a].term;
    all_trunc &= o[a].trunc;
  }
  const uint32_t done = (all_term | all_trunc) & (live ? 1u : 0u);
#ifdef RMX_DIAG
  if (p.stamps) {  // make the stamp wait for the step logic (not only for memory)
    asm volatile("" ::"v"(done), "v"(s[0].f), "v"(s[A - 1].f), "v"(o[0].reward), "v"(o[A - 1].reward));
  }
#endif
  // episode statistics (evaluation_metrics.py:248-267 bookkeeping) of the envs that finished this step
  auto flush_stats = [&]() {
    if (p.wave_stats) {  // per-wave slab slot: one plain 32-B store per wave with a finished episode
      LaneStats ls = {0.0, (int)done, 0, done ? t1 : 0};
      double rsum = 0.0;
#pragma unroll
      for (int a = 0; a < A; ++a) {
        rsum += (double)s[a].ret;
        ls.successes += done ? (int)o[a].succ : 0;
      }
      ls.ret = done ? rsum : 0.0;
      wave_flush_slot(p.slab, slot, ls, __any(done));
    } else if (done) {  // per-env slots: no-return atomics from the finishing lanes only
      // thread-per-env: the agents' returns and successes summed in the lane (agent order), one adder into
      // the agent-0 slots (3 atomic instructions per wave at any A, not 1 + 2A)
      double rs = 0.0;
      uint32_t sc = 0;
#pragma unroll
      for (int a = 0; a < A; ++a) {
        rs += (double)s[a].ret;
        sc += o[a].succ;
      }
      env_stats_env(p, e, t1);
      env_stats_ret(p, e, rs, sc);
    }
  };
  // FrozenLake with A <= 2: ~6 % of the envs finish each step, so nearly every wave has stats atomics; issued
  // before the column stores their latency overlaps the store burst (config 2: 2.89-2.92 vs 3.02-3.05 us per
  // step, profiles/r02_ab_log.md ab1/ab2).  OfficeWorld episodes rarely end and A >= 3 measured neutral or
  // slower, so those keep the atomics last.
  if constexpr (STATS_FIRST) flush_stats();
  STAMP(6);
  if (live) {
    st(r_t, off, 0, t1);
    if (p.env_done) byte_st<SAUX>(p, (uint32_t)e, done);
#pragma unroll
    for (int a = 0; a < A; ++a) {
      const uint32_t f1 = s[a].f | (done ? RMX_F_ENV_DONE : 0u);
      st(r_x, off, a * col, s[a].x);
      st(r_y, off, a * col, s[a].y);
      if (SKIP == kSkipNone || s[a].q != s0[a].q) st(r_q, off, a * col, s[a].q);
      st(r_f, off, a * col, (int32_t)f1);
      if (SKIP == kSkipNone || __float_as_int(s[a].ret) != __float_as_int(s0[a].ret))
        st(r_ret, off, a * col, __float_as_int(s[a].ret));
      st(r_rew, off, a * col, __float_as_int(o[a].reward));
    }
    // the optional outputs, one wave-uniform test per column (tested inside the agent loop, the compiler re-derived
    // each condition per agent: ~4 instructions per column and agent)
    if (p.shaping) {
      const auto r = col_rsrc(p.shaping, cols);
#pragma unroll
      for (int a = 0; a < A; ++a) st(r, off, a * col, __float_as_int(o[a].shaping));
    }
    if (p.renv) {
      const auto r = col_rsrc(p.renv, cols);
#pragma unroll
      for (int a = 0; a < A; ++a) st(r, off, a * col, __float_as_int(o[a].renv));
    }
    if (p.enc_state) {  // state_encoder_*.encode of the new observation
      const auto r = col_rsrc(p.enc_state, cols);
#pragma unroll
      for (int a = 0; a < A; ++a) st(r, off, a * col, (s[a].y * p.W + s[a].x) * p.enc_nq[a] + s[a].q);
    }
    if constexpr (RNG) {
      const auto r_rng = col_rsrc(p.rng, (uint32_t)N * 32u);
      const uint32_t o8 = (uint32_t)e * 8u, c8 = (uint32_t)N * 8u;
      typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
      // the generator moves with slip draws and at a reset only (FIXED with a clean cache: not even then without slip)
      if (DRAW || (rs && (!FIXED || p.rs_dirty))) {
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{(uint32_t)rng.hi, (uint32_t)(rng.hi >> 32)}, r_rng, o8, 0, SAUX);
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{(uint32_t)rng.lo, (uint32_t)(rng.lo >> 32)}, r_rng, o8, c8, SAUX);
      }
      if (rs && FIXED && !p.rs_dirty) {  // same seed, same increment: only the episode counter moves
        st(col_rsrc(p.episode, (uint32_t)N * 4u), off, 0, episode);
      } else if (rs) {  // a reseed changes the increment words too
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{(uint32_t)rng.ihi, (uint32_t)(rng.ihi >> 32)}, r_rng, o8, 2u * c8,
                                              SAUX);
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{(uint32_t)rng.ilo, (uint32_t)(rng.ilo >> 32)}, r_rng, o8, 3u * c8,
                                              SAUX);
        st(col_rsrc(p.episode, (uint32_t)N * 4u), off, 0, episode);
      }
      if constexpr (RSTART && !FIXED) {  // the precompute moved on (draws every step; a new generator after a reset)
        const auto r_nx = col_rsrc(p.nx_rng, (uint32_t)N * 32u);
        if (nx.fresh || nx.i != nx.i0) {
          __builtin_amdgcn_raw_buffer_store_b64(u32x2{(uint32_t)nx.g.hi, (uint32_t)(nx.g.hi >> 32)}, r_nx, o8, 0, SAUX);
          __builtin_amdgcn_raw_buffer_store_b64(u32x2{(uint32_t)nx.g.lo, (uint32_t)(nx.g.lo >> 32)}, r_nx, o8, c8, SAUX);
          st(col_rsrc(p.nx_idx, (uint32_t)N * 4u), off, 0, nx.i);
        }
        if (nx.fresh) {
          __builtin_amdgcn_raw_buffer_store_b64(u32x2{(uint32_t)nx.g.ihi, (uint32_t)(nx.g.ihi >> 32)}, r_nx, o8, 2u * c8,
                                                SAUX);
          __builtin_amdgcn_raw_buffer_store_b64(u32x2{(uint32_t)nx.g.ilo, (uint32_t)(nx.g.ilo >> 32)}, r_nx, o8, 3u * c8,
                                                SAUX);
          st(col_rsrc(p.nx_ep, (uint32_t)N * 4u), off, 0, nx.k);
        }
      }
    }
  } else {
    bad = 0;
  }
#ifdef RMX_DIAG
  if (QRM && (p.diag & 131072)) {  // timing ablation: QRM lookups kept (registers), QRM stores dropped
    uint32_t keep = 0;
#pragma unroll
    for (int a = 0; a < A; ++a)
#pragma unroll
      for (int j = 0; j < (QXB > 0 ? QXB : 1); ++j) keep ^= qe[a][j].x ^ qe[a][j].y;
    if (keep == 0x7fffffffu) atomicOr(p.err, 2u);
  } else
#endif
  if constexpr (QRM) {  // QRM counterfactual experiences (rm_environment_wrapper.py:140-183)
    const int32_t Qx = p.n_qrm_max;
    const uint32_t nq_col = (uint32_t)Qx * (uint32_t)A * (uint32_t)N;
    const auto r_s = col_rsrc(p.qrm_s, nq_col * 4u), r_sn = col_rsrc(p.qrm_sn, nq_col * 4u);
    const auto r_rq = col_rsrc(p.qrm_rq, nq_col * 4u), r_dn = col_rsrc(p.qrm_done, nq_col);
#pragma unroll
    for (int a = 0; a < A; ++a) {
      const uint32_t nQ = (uint32_t)p.enc_nq[a];
      const uint32_t new_cell = (uint32_t)(s[a].y * p.W + s[a].x);
      const uint32_t env_term = (s[a].f >> 4) & 1u;  // RMX_F_ENV_TERM of this step
#pragma unroll
      for (int j = 0; j < QXB; ++j) {
        if (j >= Qx) continue;  // uniform
        const bool valid = j < p.n_qrm[a];  // missing states of a shorter RM: (-1, -1, 0, 0)
        const uint32_t so = (uint32_t)(a * Qx + j) * (uint32_t)N;
        const int32_t s_enc = valid ? (int32_t)(prev_cell[a] * nQ + p.qrm_q[a][j]) : -1;
        const int32_t sn_enc = valid ? (int32_t)(new_cell * nQ + (qe[a][j].x & 0xFFu)) : -1;
        const uint32_t dn = valid ? (env_term | ((qe[a][j].x >> 8) & 1u)) : 0u;
        if (live) {
          st(r_s, off, so * 4u, s_enc);
          st(r_sn, off, so * 4u, sn_enc);
          st(r_rq, off, so * 4u, valid ? (int32_t)qe[a][j].y : 0);
          __builtin_amdgcn_raw_buffer_store_b8((uint8_t)dn, r_dn, (uint32_t)e, so, kStoreAux);
        }
      }
    }
  }
  if (__any(bad)) {
    if ((tid & 63) == 0) atomicOr(p.err, 1u);
  }
#ifdef RMX_DIAG
  STAMP(7);
  if (!(diag & 1)) {
#endif
  if constexpr (!STATS_FIRST) flush_stats();
#ifdef RMX_DIAG
  }
  STAMP(8);
  if (p.stamps && (tid & 63) == 0) {
    unsigned long long* w = p.stamps + (((size_t)blockIdx.x * blockDim.x + tid) >> 6) * (2 * kStamps);
#pragma unroll
    for (int i = 0; i < kStamps; ++i) {
      w[i] = st_clk[i];
      w[kStamps + i] = st_rt[i];
    }
  }
#endif
  if constexpr (RPT) {  // the env's slot values after this step's adds (the same f64 add the atomic performs)
    double rs = 0.0;
    uint32_t sc = 0;
#pragma unroll
    for (int a = 0; a < A; ++a) {
      rs += (double)s[a].ret;
      sc += o[a].succ;
    }
    report_tail(p, rin, done, rs, sc, t1);
  }
}

// ------------------------------------------------------------------------------------------------
// Fused rollout on the fast path (rmx_rollout, the reference loop frozen_lake_main.py:336-376 with
// uniform random actions): thread per env, state in VGPRs for T autoreset steps, actions hashed in
// kernel, one merged-table (or move-word + RM-entry) lookup per agent-step.  Inside one launch the
// tables stay in each XCD's L2.  Statistics accumulate per lane and are flushed once per wave.
// ------------------------------------------------------------------------------------------------
// TBL: kTblGlobal / kTblMerged read the tables through L2; kTblLds / kTblMergedLds stage them into LDS
// once per workgroup (the staging is amortised over the T steps; an LDS lookup is ~5x shorter than L2).
// SLIP: the stochastic dynamics as in step_fast_kernel<..., SLIP> (the env's PCG64 and episode counter in VGPRs for
// the T steps, re-seeded at each autoreset): FrozenLake one rng.choice per active, non-frozen agent in agent order;
// OfficeWorld the intended action's record first (wall), the draw only when it was not blocked.
template <int KIND, int A, int TBL, int SLIP = 0>
__global__ void __launch_bounds__(256) rollout_fast_kernel(FastParams p, int32_t T, float* __restrict__ trace) {
  static_assert(TBL == kTblGlobal || TBL == kTblMerged || TBL == kTblLds || TBL == kTblMergedLds,
                "rollout: global / merged tables, in L2 or LDS");
  static_assert(!SLIP || TBL == kTblMerged || TBL == kTblMergedLds, "rollout slip: merged tables");
  constexpr bool RNG = SLIP != 0, DRAW = (SLIP & kRngSlip) != 0;  // as in step_fast_kernel
  constexpr bool RSTART = (SLIP & kRngStarts) != 0 && KIND == RMX_FROZEN_LAKE;
  constexpr bool OW_SLIP = DRAW && KIND == RMX_OFFICE_WORLD;
  constexpr bool MERGED = TBL == kTblMerged || TBL == kTblMergedLds;
  constexpr bool IN_LDS = TBL == kTblLds || TBL == kTblMergedLds;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int tid = threadIdx.x;
  if constexpr (IN_LDS) {  // all 16-B granules of the table, strided over the workgroup
    const uint4* src = MERGED ? p.merged : p.tables;
    const int n16 = MERGED ? p.merged_bytes / 16 : p.n16;
    for (int i = tid; i < n16; i += (int)blockDim.x) reinterpret_cast<uint4*>(lds)[i] = src[i];
    __syncthreads();
  }
  const uint32_t mg_n16 = (uint32_t)p.merged_bytes / 16u;
  // random starts: the per-wave draw / free-cell areas follow the staged table (rs_wave_lds)
  const uint32_t rs_lds_off = IN_LDS ? ((uint32_t)(MERGED ? p.merged_bytes : p.n16 * 16) + 15u) & ~15u : 0u;
  const int32_t N = p.N;
  const int32_t e_raw = (int32_t)(blockIdx.x * blockDim.x) + tid;
  const bool live = e_raw < N;
  const int32_t e = live ? e_raw : N - 1;  // tail lanes compute env N-1 again and never store
  const uint32_t off = (uint32_t)e * 4u;
  const uint32_t col = (uint32_t)N * 4u;
  const uint32_t cols = col * (uint32_t)A;
  const auto r_x = col_rsrc(p.pos_x, cols), r_y = col_rsrc(p.pos_y, cols), r_q = col_rsrc(p.rm_q, cols);
  const auto r_f = col_rsrc(p.flags, cols), r_ret = col_rsrc(p.ep_ret, cols), r_t = col_rsrc(p.t, col);
  const auto r_rew = col_rsrc(p.reward, cols);
  AgentIO s[A];
  int32_t t = col_ld(r_t, off, 0);
#pragma unroll
  for (int a = 0; a < A; ++a) {
    s[a].x = col_ld(r_x, off, a * col);
    s[a].y = col_ld(r_y, off, a * col);
    s[a].q = col_ld(r_q, off, a * col);
    s[a].f = (uint32_t)col_ld(r_f, off, a * col);
    s[a].ret = __int_as_float(col_ld(r_ret, off, a * col));
  }
  Pcg rng = {0ull, 0ull, 0ull, 0ull};
  int32_t episode = 0;
  if constexpr (RNG) {  // rng [4][N] u64 (state hi, lo, increment hi, lo), episode [N]
    rng = {p.rng[e], p.rng[(int64_t)N + e], p.rng[2 * (int64_t)N + e], p.rng[3 * (int64_t)N + e]};
    episode = p.episode[e];
  }
  // seed_episode_stride == 0 (FIXED): the env's cached generator (and random start cells), in registers for the T
  // steps; otherwise random starts carry the step kernel's next-episode precompute (rs_step) the same way
  constexpr bool FIXED = RNG && (SLIP & kRngFixedSeed) != 0;
  constexpr bool FCELLS = FIXED && RSTART;
  uint32_t fcw[FCELLS ? (A + 1) / 2 : 1] = {};
  Pcg frng = {0ull, 0ull, 0ull, 0ull};
  if constexpr (FIXED) {
    if constexpr (FCELLS)
#pragma unroll
      for (int w = 0; w < (A + 1) / 2; ++w) fcw[w] = p.rs_cells[(int64_t)w * N + e];
    frng = {p.rs_rng[e], p.rs_rng[(int64_t)N + e], p.rs_rng[2 * (int64_t)N + e], p.rs_rng[3 * (int64_t)N + e]};
  }
  RsNext nx = {{0ull, 0ull, 0ull, 0ull}, 0, -1, 0, false};
  unsigned char* rs_row = nullptr;
  if constexpr (RSTART && !FIXED) {
    nx.g = {p.nx_rng[e], p.nx_rng[(int64_t)N + e], p.nx_rng[2 * (int64_t)N + e], p.nx_rng[3 * (int64_t)N + e]};
    nx.i = p.nx_idx[e];
    nx.k = p.nx_ep[e];
    nx.i0 = nx.i;
    rs_row = reinterpret_cast<unsigned char*>(p.start_ws) + (size_t)e * (size_t)(2 * shuffle_stride(p.n_free));
  }
  const auto mg = col_rsrc(p.merged, MERGED ? (uint32_t)p.merged_bytes : 0u);
  const auto tb = make_tables<!IN_LDS>(lds, p);
  const int64_t eg = p.env_offset + e;
  // hash_action's counter ((t*N + e)*A + a)*GR advances by N*A*GR per step: one 64-bit add per
  // agent-step instead of three 64-bit multiplies (bit-identical actions)
  uint64_t ctr[A];
#pragma unroll
  for (int a = 0; a < A; ++a)
    ctr[a] = (((uint64_t)p.t_global * (uint64_t)p.n_global + (uint64_t)eg) * (uint64_t)A + (uint64_t)a) * kGolden;
  const uint64_t dctr = (uint64_t)p.n_global * (uint64_t)A * kGolden;
  LaneStats ls = {0.0, 0, 0, 0};
  uint32_t bad = 0, done = 0;
  AgentRes o[A];
  for (int32_t it = 0; it < T; ++it) {
    const bool rs = (s[0].f & RMX_F_ENV_DONE) != 0;  // the loop's reset() after a finished episode
    t = rs ? 0 : t;
    const int32_t t1 = t + 1;
    const float disc = p.gamma_is_one ? 1.0f : p.disc[min((uint32_t)t, (uint32_t)p.max_t + 1u)];
    int32_t sx[A], sy[A];
#pragma unroll
    for (int a = 0; a < A; ++a) sx[a] = p.start_x[a], sy[a] = p.start_y[a];
    if constexpr (RNG) {
      if constexpr (FIXED) {
        if (rs) {
          if constexpr (FCELLS) fixed_start_cells<A>(fcw, sx, sy);
          rng = frng;
          episode += 1;
        }
      } else if constexpr (RSTART)
        rs_step<A>(p, rng, episode, nx, rs, live, eg, rs_row, lds + rs_lds_off, (uint32_t)tid, sx, sy);
      else
        random_start_reset<A, false>(p, rng, episode, rs, live, eg, lds, (uint32_t)tid, rs_lds_off, sx, sy);
    }
    AgentTmp k[A];
    uint32_t m[A];
    uint4 r[A];
    // a merged record of this agent's (q, cell) section: from LDS or through L2
    auto record = [&](int a, uint32_t mi) {
      const uint32_t idx = (uint32_t)p.mg_base[a] + __umul24(__umul24((uint32_t)s[a].q, (uint32_t)p.HW), 5u) + mi;
      if constexpr (IN_LDS) {
        return reinterpret_cast<const uint4*>(lds)[min(idx, mg_n16 - 1u)];
      } else {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(mg, idx * 16u, 0, 0);
        return make_uint4(v[0], v[1], v[2], v[3]);
      }
    };
    uint32_t blocked[OW_SLIP ? A : 1] = {};
#pragma unroll
    for (int a = 0; a < A; ++a) {  // the action of every agent, and the autoreset
      s[a].act = (int32_t)(splitmix64(p.seed ^ ctr[a]) >> 62);  // == hash_action(seed, t_global + it, ...)
      ctr[a] += dctr;
      s[a].x = rs ? sx[a] : s[a].x;
      s[a].y = rs ? sy[a] : s[a].y;
      s[a].q = rs ? p.init_q[a] : s[a].q;
      s[a].f = rs ? RMX_F_ACTIVE : s[a].f;
      s[a].ret = rs ? 0.0f : s[a].ret;
    }
    if constexpr (OW_SLIP) {  // the intended records (wall bits), then the draws in agent order
      uint32_t wi[A];
#pragma unroll
      for (int a = 0; a < A; ++a) wi[a] = record(a, move_index<KIND>(s[a], (uint32_t)p.final_q[a], 0u, p, bad, k[a])).x;
#pragma unroll
      for (int a = 0; a < A; ++a) {
        const uint32_t ac = agent_action<KIND>(s[a], (uint32_t)p.final_q[a], bad, k[a]);
        blocked[a] = (ac < (uint32_t)RMX_WAIT && (wi[a] & kMvWall)) ? 1u : 0u;
        s[a].act = (int32_t)(blocked[a] ? (uint32_t)RMX_WAIT
                                        : (ac < (uint32_t)RMX_WAIT ? (uint32_t)slip_choice(p, (int32_t)ac, rng) : ac));
      }
    }
#pragma unroll
    for (int a = 0; a < A; ++a) {  // stage 1: every agent's lookup in flight together
      if constexpr (DRAW && KIND == RMX_FROZEN_LAKE) {  // hashed actions are 0..3: never the slip map's missing "wait"
        if ((s[a].f & RMX_F_ACTIVE) && (uint32_t)s[a].q != (uint32_t)p.final_q[a])
          s[a].act = slip_choice(p, s[a].act, rng);
      }
      if constexpr (MERGED) {
        r[a] = record(a, move_index<KIND>(s[a], (uint32_t)p.final_q[a], 0u, p, bad, k[a]));
      } else {
        m[a] = tb.mv(move_index<KIND>(s[a], (uint32_t)p.final_q[a], (uint32_t)p.mv_base[a], p, bad, k[a]));
      }
    }
#pragma unroll
    for (int a = 0; a < A; ++a) {  // stage 2
      if constexpr (OW_SLIP) {  // the intended action's wall penalty / failure, the final cell's plant
        const uint32_t hz = __builtin_amdgcn_ubfe(r[a].x, 25, 1);
        const uint32_t fl = (blocked[a] & (uint32_t)p.wall_fail) | (hz & (uint32_t)p.hazard_fail);
        r[a].x = (r[a].x & ~(kMvWall | kMvFail)) | (blocked[a] << 24) | (fl << 26);
      }
      if constexpr (MERGED) {
        const uint32_t w0 = r[a].x;
        k[a].mm = k[a].moving ? w0 : 0u;
        s[a].x = (int32_t)(w0 & 0xFFu);
        s[a].y = (int32_t)__builtin_amdgcn_ubfe(w0, 8, 8);
        r[a].x = __builtin_amdgcn_ubfe(w0, 16, 8) | (__builtin_amdgcn_ubfe(w0, 27, 1) << 8);
      } else {
        r[a] = tb.rm(rm_index(s[a], m[a], (uint32_t)p.rm_base[a], p, k[a]));
      }
    }
    uint32_t all_term = 1u, all_trunc = 1u;
#pragma unroll
    for (int a = 0; a < A; ++a) {
      o[a] = finish<KIND>(s[a], k[a], r[a], t1, disc, p);
      all_term &= o[a].term;
      all_trunc &= o[a].trunc;
    }
    done = all_term | all_trunc;
    t = t1;
    double rsum = 0.0;
    int succ = 0;
#pragma unroll
    for (int a = 0; a < A; ++a) {
      s[a].f |= done ? RMX_F_ENV_DONE : 0u;
      rsum += (double)s[a].ret;
      succ += (int)o[a].succ;
      if (trace && live) trace[((int64_t)it * A + a) * N + e] = o[a].reward;
    }
    if (done && live) {  // evaluation_metrics.py:248-267 bookkeeping of a finished episode
      ls.ret += rsum;
      ls.episodes += 1;
      ls.successes += succ;
      ls.length += t1;
    }
  }
  if (live) {
    col_st(r_t, off, 0, t);
    if (p.env_done) byte_st(p, (uint32_t)e, done);
    if constexpr (RNG) {
      p.rng[e] = rng.hi;
      p.rng[(int64_t)N + e] = rng.lo;
      p.rng[2 * (int64_t)N + e] = rng.ihi;
      p.rng[3 * (int64_t)N + e] = rng.ilo;
      p.episode[e] = episode;
    }
    if constexpr (RSTART && !FIXED) {  // the precompute where the T steps left it
      p.nx_rng[e] = nx.g.hi;
      p.nx_rng[(int64_t)N + e] = nx.g.lo;
      p.nx_rng[2 * (int64_t)N + e] = nx.g.ihi;
      p.nx_rng[3 * (int64_t)N + e] = nx.g.ilo;
      p.nx_idx[e] = nx.i;
      p.nx_ep[e] = nx.k;
    }
#pragma unroll
    for (int a = 0; a < A; ++a) {
      col_st(r_x, off, a * col, s[a].x);
      col_st(r_y, off, a * col, s[a].y);
      col_st(r_q, off, a * col, s[a].q);
      col_st(r_f, off, a * col, (int32_t)s[a].f);
      col_st(r_ret, off, a * col, __float_as_int(s[a].ret));
      col_st(r_rew, off, a * col, __float_as_int(o[a].reward));
      if (p.shaping) col_st(col_rsrc(p.shaping, cols), off, a * col, __float_as_int(o[a].shaping));
      if (p.renv) col_st(col_rsrc(p.renv, cols), off, a * col, __float_as_int(o[a].renv));
      if (p.enc_state)
        col_st(col_rsrc(p.enc_state, cols), off, a * col, (s[a].y * p.W + s[a].x) * p.enc_nq[a] + s[a].q);
    }
  } else {
    bad = 0;
  }
  if (__any(bad)) {
    if ((tid & 63) == 0) atomicOr(p.err, 1u);
  }
  wave_flush(p.slab, ls, __any(ls.episodes != 0));
}

template <int KIND, int A>
static void launch_rollout_a(const FastParams& p, int32_t T, float* trace, dim3 g, dim3 b, hipStream_t st) {
  if (p.slip) {  // host: merged tables (rmx_rollout); random starts are a FrozenLake option
    auto go = [&](auto rng_flags) {
      constexpr int R = decltype(rng_flags)::value;
      // rs_step's LDS (not with the fixed-start cache)
      const size_t rs = (R & kRngStarts) && !(R & kRngFixedSeed) ? (size_t)(b.x / 64) * (size_t)kRsWaveLds : 0;
      if (p.tbl_mode == kTblMergedLds)
        hipLaunchKernelGGL((rollout_fast_kernel<KIND, A, kTblMergedLds, R>), g, b,
                           (((size_t)p.merged_bytes + 15) & ~(size_t)15) + rs, st, p, T, trace);
      else
        hipLaunchKernelGGL((rollout_fast_kernel<KIND, A, kTblMerged, R>), g, b, rs, st, p, T, trace);
    };
    if constexpr (KIND == RMX_FROZEN_LAKE) {
      constexpr int S = kRngStarts, F = kRngStarts | kRngFixedSeed;
      if (p.slip == S) return go(std::integral_constant<int, S>{});
      if (p.slip == (kRngSlip | S)) return go(std::integral_constant<int, kRngSlip | S>{});
      if (p.slip == F) return go(std::integral_constant<int, F>{});
      if (p.slip == (kRngSlip | F)) return go(std::integral_constant<int, kRngSlip | F>{});
    }
    if (p.slip == (kRngSlip | kRngFixedSeed)) return go(std::integral_constant<int, kRngSlip | kRngFixedSeed>{});
    return go(std::integral_constant<int, kRngSlip>{});
  }
  switch (p.tbl_mode) {
    case kTblMergedLds:
      hipLaunchKernelGGL((rollout_fast_kernel<KIND, A, kTblMergedLds>), g, b, (size_t)p.merged_bytes, st, p, T, trace);
      break;
    case kTblLds:
      hipLaunchKernelGGL((rollout_fast_kernel<KIND, A, kTblLds>), g, b, (size_t)p.n16 * 16, st, p, T, trace);
      break;
    case kTblMerged: hipLaunchKernelGGL((rollout_fast_kernel<KIND, A, kTblMerged>), g, b, 0, st, p, T, trace); break;
    default: hipLaunchKernelGGL((rollout_fast_kernel<KIND, A, kTblGlobal>), g, b, 0, st, p, T, trace); break;
  }
}

template <int KIND>
static void launch_rollout_k(const FastParams& p, int32_t T, float* trace, hipStream_t st) {
  const dim3 b((unsigned)p.block), g((unsigned)(((int64_t)p.N + p.block - 1) / p.block));
  switch (p.A) {
    case 1: launch_rollout_a<KIND, 1>(p, T, trace, g, b, st); break;
    case 2: launch_rollout_a<KIND, 2>(p, T, trace, g, b, st); break;
    case 3: launch_rollout_a<KIND, 3>(p, T, trace, g, b, st); break;
    default: launch_rollout_a<KIND, 4>(p, T, trace, g, b, st); break;
  }
}

hipError_t launch_rollout_fast(const FastParams& p, int kind, int32_t T, float* trace, hipStream_t st) {
  if (kind == RMX_FROZEN_LAKE)
    launch_rollout_k<RMX_FROZEN_LAKE>(p, T, trace, st);
  else
    launch_rollout_k<RMX_OFFICE_WORLD>(p, T, trace, st);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
thread_local StepCapture* tl_capture = nullptr;

// step_fast_kernel's preloaded leading arguments (N, block size, the columns the first loads read), then p
static StepArgs step_args(const FastParams& p, uint32_t blk) {
  return StepArgs{p.N, (int32_t)blk, p.pos_x, p.pos_y, p.rm_q, p.flags, p.t, p.actions, p};
}

// Every step_fast_kernel launch: issued on st, or, under a StepCapture (rmx_step_seq), recorded for the engine's own
// queue with the instantiation's code-object symbol (its Itanium mangling: the eight template arguments, then the
// parameter list, which is fixed)
template <int KIND, int A, bool HASHED, int TBL, int QXB = 0, int SKIP = kSkipNone, bool RPT = false, int SLIP = 0>
static void go_step(dim3 g, dim3 b, size_t lds, hipStream_t st, const FastParams& p) {
  const StepArgs a = step_args(p, b.x);
  if (StepCapture* c = tl_capture) {
    StepLaunch& L = *c->out;
    snprintf(L.symbol, sizeof(L.symbol),
             "_ZN3rmx16step_fast_kernelILi%dELi%dELb%dELi%dELi%dELi%dELb%dELi%dEEEviiPKiS2_S2_PKjS2_S2_NS_"
             "10FastParamsE.kd",
             KIND, A, (int)HASHED, TBL, QXB, SKIP, (int)RPT, SLIP);
    L.grid = g.x;
    L.block = b.x;
    L.lds = (uint32_t)lds;
    // byte copies (padding included: the host compares consecutive windows' kernargs byte for byte)
    std::memset(&L.args, 0, sizeof(L.args));
    std::memcpy(&L.args, &a, offsetof(StepArgs, p));
    std::memcpy(&L.args.p, &p, sizeof(FastParams));
    c->ok = true;
    return;
  }
  hipLaunchKernelGGL((step_fast_kernel<KIND, A, HASHED, TBL, QXB, SKIP, RPT, SLIP>), g, b, lds, st, a.N, a.blk, a.pos_x,
                     a.pos_y, a.rm_q, a.flags, a.t, a.actions, a.p);
}

template <int KIND, int A, int QXB>
static void launch_qrm(const FastParams& p, int hashed, dim3 g, hipStream_t st) {
  if (hashed)
    go_step<KIND, A, true, kTblGlobal, QXB>(g, dim3(256), 0, st, p);
  else
    go_step<KIND, A, false, kTblGlobal, QXB>(g, dim3(256), 0, st, p);
}

template <int KIND, int A, int TBL>
static void launch_tpe_t(const FastParams& p, int hashed, hipStream_t st) {
  if constexpr (TBL == kTblGlobal) {
    if (p.qrm_s) {  // QRM outputs bound: the experience-count bucket (256-thread blocks, every word stored)
      const dim3 g((unsigned)(((int64_t)p.N + 255) / 256));
      if (p.n_qrm_max <= 4)
        launch_qrm<KIND, A, 4>(p, hashed, g, st);
      else if (p.n_qrm_max <= 8 || A > 2)  // host guarantees Qx <= 8 when A > 2 (register budget)
        launch_qrm<KIND, A, 8>(p, hashed, g, st);
      else if constexpr (A <= 2)
        launch_qrm<KIND, A, 16>(p, hashed, g, st);
      return;
    }
  }
  const dim3 b((unsigned)p.block), g((unsigned)(((int64_t)p.N + p.block - 1) / p.block));
  if (p.skip_same == kSkipRareNT) {  // the default from 2^23 env x agent instances on (the bandwidth regime)
    if (hashed)
      go_step<KIND, A, true, TBL, 0, kSkipRareNT>(g, b, 0, st, p);
    else
      go_step<KIND, A, false, TBL, 0, kSkipRareNT>(g, b, 0, st, p);
    return;
  }
  if constexpr (TBL == kTblMerged4 || TBL == kTblMerged) {
    if (p.slip) {  // slip / random starts (host: no QRM, N < 2^27)
      auto go = [&](auto rng_flags) {
        constexpr int R = decltype(rng_flags)::value;
        const size_t lr = (R & kRngStarts) && !(R & kRngFixedSeed) ? (size_t)(b.x / 64) * (size_t)kRsWaveLds
                                                                      : 0;  // rs_step's LDS
        if (hashed)
          go_step<KIND, A, true, TBL, 0, kSkipRare, false, R>(g, b, lr, st, p);
        else if (p.rpt_out)  // rmx_step_report (round 5: the report fused here too, as for deterministic dynamics)
          go_step<KIND, A, false, TBL, 0, kSkipRare, true, R>(g, b, lr, st, p);
        else
          go_step<KIND, A, false, TBL, 0, kSkipRare, false, R>(g, b, lr, st, p);
      };
      if constexpr (KIND == RMX_FROZEN_LAKE) {
        constexpr int S = kRngStarts, F = kRngStarts | kRngFixedSeed;
        if (p.slip == S) return go(std::integral_constant<int, S>{});
        if (p.slip == (kRngSlip | S)) return go(std::integral_constant<int, kRngSlip | S>{});
        if (p.slip == F) return go(std::integral_constant<int, F>{});
        if (p.slip == (kRngSlip | F)) return go(std::integral_constant<int, kRngSlip | F>{});
      }
      // (slip alone: the step reseeds, the host clears kRngFixedSeed there; the rollout uses the cache)
      return go(std::integral_constant<int, kRngSlip>{});
    }
  }
  if (p.rpt_out && !hashed) {  // rmx_step_report (host: 64-thread blocks, per-env slots, no QRM)
    go_step<KIND, A, false, TBL, 0, kSkipRare, true>(g, b, 0, st, p);
    return;
  }
  if (hashed)
    go_step<KIND, A, true, TBL, 0, kSkipRare>(g, b, 0, st, p);
  else
    go_step<KIND, A, false, TBL, 0, kSkipRare>(g, b, 0, st, p);
}

template <int KIND, int A>
static void launch_tpe(const FastParams& p, int hashed, hipStream_t st) {
  switch (p.tbl_mode) {
    case kTblMerged: launch_tpe_t<KIND, A, kTblMerged>(p, hashed, st); break;
    case kTblMerged4: launch_tpe_t<KIND, A, kTblMerged4>(p, hashed, st); break;
    default: launch_tpe_t<KIND, A, kTblGlobal>(p, hashed, st); break;
  }
}

template <int KIND>
static void launch_k(const FastParams& p, int hashed, hipStream_t st) {
  switch (p.A) {
    case 1: launch_tpe<KIND, 1>(p, hashed, st); break;
    case 2: launch_tpe<KIND, 2>(p, hashed, st); break;
    case 3: launch_tpe<KIND, 3>(p, hashed, st); break;
    default: launch_tpe<KIND, 4>(p, hashed, st); break;
  }
}

hipError_t launch_step_fast(const FastParams& p, int hashed, int kind, hipStream_t st) {
  if (kind == RMX_FROZEN_LAKE)
    launch_k<RMX_FROZEN_LAKE>(p, hashed, st);
  else
    launch_k<RMX_OFFICE_WORLD>(p, hashed, st);
  return hipGetLastError();
}

}  // namespace rmx
