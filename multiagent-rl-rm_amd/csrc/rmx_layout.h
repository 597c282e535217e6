// rmx_layout.h — table layouts and constants shared by the host table builders (rmx_tables.cpp, plain
// C++: builds with g++ and the sanitizers) and the gfx950 kernels.  No HIP types here.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace rmx {

// ---- deterministic fast path ------------------------------------------------------------------
// The per-cell tile and the per-agent event map are pre-composed on the host into one transition
// word per (agent, cell, action), so an agent-step is two dependent LDS lookups: move word, then the
// RM (q, event) entry.  Used for deterministic dynamics without QRM outputs, A <= 4, W, H <= 255.
//   move word  bits 0-7 x', 8-15 y', 16-23 event at (x', y'), 24 wall hit, 25 hazard at (x', y'),
//              26 the step fails the agent (FL: hole; OW: wall && terminate_hit_walls or plant &&
//              terminate_on_plants)
//   RM entry   uint4 {next_q | (next_q == final_q) << 8, f32 reward_modifier * RQ, f32 shaping, f32 raw RQ}
//   info       uint4 per agent {move-table base, RM-table base, sx | sy<<8 | init_q<<16 | final_q<<24, enc_nq}
//              (final_q 255 = none)
//   merged     uint4 [A][Q][H*W][5] (separate allocation, <= 2 MiB): the move word and the RM entry of
//              (agent, q, cell, action) in ONE lookup: {x' | y'<<8 | next_q<<16 | wall<<24 | hazard<<25 |
//              fails<<26 | (next_q == final)<<27, reward_modifier * RQ, shaping, 0}
// fast-path table modes (the values are part of the step kernels' symbol names).  Round 5 removed the step's
// LDS-staged (0, step only), lane-resident (2, 3), speculative (6) and 8-B (8) modes, which lost their A/Bs.
constexpr int kTblLds = 0;                // rollout only: the blob staged into LDS
constexpr int kTblGlobal = 1, kTblMerged = 4;
constexpr int kTblMergedLds = 5;          // rollout only: the merged table staged into LDS
constexpr int kTblMerged4 = 7;            // step: merged table as 4-B records, reward from a per-agent palette (no shaping)
constexpr size_t kRolloutLdsMax = 64 * 1024;  // LDS bytes a rollout workgroup stages at most
constexpr size_t kMergedMaxBytes = 2u << 20;
constexpr int kFastMaxAgents = 4;
constexpr int kFastMaxQrm = 16;  // QRM experiences per agent the fast kernel emits (Qx); beyond: generic
constexpr size_t kFastBlobMaxBytes = 16 * 1024;  // the fast path's blob (move words, RM entries): <= 16 KiB
constexpr uint32_t kMvWall = 1u << 24, kMvHazard = 1u << 25, kMvFail = 1u << 26;
// fast step kernel store modes (FastParams.skip_same): every column word stored (the QRM-output instantiations only) /
// the rarely-changing rm_q and ep_ret words skipped when unchanged (the default) / the same with non-temporal
// write-through stores (the bandwidth regime, from 2^23 env x agent instances).  (Mode 1, every unchanged word
// skipped, lost its A/B and was removed in round 5.)
constexpr int kSkipNone = 0, kSkipRare = 2, kSkipRareNT = 3;

}  // namespace rmx
