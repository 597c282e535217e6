// rmx_tables.cpp — host-only half of rmx_create: validation and the device-table builders.  Runs once per
// handle, never per step.  Plain C++ so the same source also builds with g++ -fsanitize=address,undefined
// (oracle/Makefile `asan`, tests/test_sanitizers.py): these builders do all the index arithmetic on
// caller-supplied sizes.
#include "rmx_host.h"

#include <string.h>

#include <algorithm>

namespace rmx {

namespace {

size_t align16(size_t x) { return (x + 15) & ~size_t(15); }

}  // namespace

std::string validate_config(const rmx_config& cr) {
  const rmx_config* c = &cr;
  if (c->kind != RMX_FROZEN_LAKE && c->kind != RMX_OFFICE_WORLD) return "unknown env kind";
  if (c->width <= 0 || c->height <= 0 || (int64_t)c->width * c->height > RMX_MAX_CELLS) return "grid size out of range";
  if (c->n_agents < 1 || c->n_agents > RMX_MAX_AGENTS) return "n_agents must be 1..8";
  if (c->n_rm_states < 1 || c->n_rm_states > RMX_MAX_RM_STATES) return "n_rm_states out of range";
  if (c->n_events < 1 || c->n_events > RMX_MAX_EVENTS) return "n_events out of range";
  if (c->n_envs < 1 || c->n_envs > (int64_t)1 << 31) return "n_envs out of range";
  if (c->env_offset < 0 || c->n_envs_global < c->env_offset + c->n_envs) return "env_offset / n_envs_global inconsistent";
  if (c->max_t < 0 || c->max_t > 60000) return "max_t out of range";
  if (!c->cell || !c->cell_event || !c->next_q || !c->rm_reward || !c->init_q || !c->final_q || !c->start_xy)
    return "a required table pointer is NULL";
  if (c->has_shaping && !c->shape) return "has_shaping set but shape is NULL";
  if (c->n_qrm_max < 0 || c->n_qrm_max > c->n_rm_states) return "n_qrm_max out of range";
  if (c->stochastic) {
    for (int i = 0; i < 4; ++i) {
      if (c->slip_n[i] < 1 || c->slip_n[i] > 4) return "slip_n must be 1..4";
      for (int j = 0; j < c->slip_n[i]; ++j) {
        if (c->slip_out[i][j] < 0 || c->slip_out[i][j] > RMX_WAIT) return "slip_out id out of range";
        if (j > 0 && !(c->slip_cdf[i][j] >= c->slip_cdf[i][j - 1])) return "slip_cdf not monotone";
      }
    }
  }
  if (c->n_qrm_max > 0 && (!c->n_qrm || !c->qrm_states || !c->enc_nq)) return "n_qrm_max > 0 but a QRM table is NULL";
  const int A = c->n_agents, Q = c->n_rm_states, E = c->n_events, HW = c->width * c->height;
  for (int a = 0; a < A; ++a) {
    const int sx = c->start_xy[2 * a], sy = c->start_xy[2 * a + 1];
    if (sx < 0 || sx >= c->width || sy < 0 || sy >= c->height) return "start cell outside grid";
    if (c->init_q[a] < 0 || c->init_q[a] >= Q) return "init_q out of range";
    if (c->final_q[a] < -1 || c->final_q[a] >= Q) return "final_q out of range";
    for (int i = 0; i < HW; ++i)
      if (c->cell_event[(size_t)a * HW + i] >= E) return "cell_event id >= n_events";
    for (int i = 0; i < Q * E; ++i)
      if (c->next_q[(size_t)a * Q * E + i] >= Q) return "next_q entry >= n_rm_states";
    if (c->enc_nq && (c->enc_nq[a] < 1 || c->enc_nq[a] > Q)) return "enc_nq must be in 1..n_rm_states";
    if (c->n_qrm_max > 0) {
      if (c->n_qrm[a] < 0 || c->n_qrm[a] > c->n_qrm_max) return "n_qrm out of range";
      for (int j = 0; j < c->n_qrm[a]; ++j)
        if (c->qrm_states[(size_t)a * c->n_qrm_max + j] >= Q) return "qrm_states entry >= n_rm_states";
    }
  }
  // every move allowed by the tile must stay on the grid (the kernels trust the tile)
  const int up = c->kind == RMX_FROZEN_LAKE ? -1 : 1;
  const int dx[4] = {0, 0, -1, 1}, dy[4] = {up, -up, 0, 0};
  for (int y = 0; y < c->height; ++y)
    for (int x = 0; x < c->width; ++x)
      for (int k = 0; k < 4; ++k)
        if ((c->cell[y * c->width + x] >> k) & 1u) {
          const int nx = x + dx[k], ny = y + dy[k];
          if (nx < 0 || nx >= c->width || ny < 0 || ny >= c->height) return "cell tile allows a move off the grid";
        }
  if (c->random_starts) {
    if (c->kind != RMX_FROZEN_LAKE) return "random_starts is a FrozenLake option (ma_frozen_lake.py:37-39)";
    if ((int64_t)free_cells(cr).size() < A) return "Not enough free cells to place all agents.";  // ma_frozen_lake.py:169-170
  }
  return std::string();
}

// FNV-1a over every input that decides what a state column means: the kind and geometry, the rules' scalars, the
// dense tables, the RM indices, the slip tables and the seed schedule (the per-shard sizes and offsets are checked
// by the blob header itself).
uint64_t config_digest(const rmx_config& c) {
  uint64_t h = 0xcbf29ce484222325ull;
  auto mix = [&](const void* p, size_t n) {
    const unsigned char* b = static_cast<const unsigned char*>(p);
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 0x100000001b3ull;
  };
  auto mixv = [&](auto v) { mix(&v, sizeof(v)); };
  const size_t A = (size_t)c.n_agents, Q = (size_t)c.n_rm_states, E = (size_t)c.n_events;
  const size_t HW = (size_t)c.width * (size_t)c.height;
  mixv(c.kind), mixv(c.width), mixv(c.height), mixv(c.n_agents), mixv(c.n_rm_states), mixv(c.n_events);
  mixv(c.max_t), mixv(c.hazard_penalty), mixv(c.wall_penalty), mixv(c.hazard_fail), mixv(c.wall_fail);
  mixv(c.gamma), mixv(c.has_shaping), mixv(c.reward_modifier), mixv(c.stochastic), mixv(c.random_starts);
  if (c.stochastic) mix(c.slip_n, sizeof(c.slip_n)), mix(c.slip_out, sizeof(c.slip_out)), mix(c.slip_cdf, sizeof(c.slip_cdf));
  mixv(c.seed_scale), mixv(c.seed_env_stride), mixv(c.seed_episode_stride);
  mix(c.cell, 2 * HW), mix(c.cell_event, A * HW), mix(c.next_q, A * Q * E), mix(c.rm_reward, 4 * A * Q * E);
  if (c.has_shaping) mix(c.shape, 4 * A * Q * E);
  mix(c.init_q, 4 * A), mix(c.final_q, 4 * A);
  if (!c.random_starts) mix(c.start_xy, 8 * A);
  return h;
}

bool build_table_blob(const rmx_config& c, std::vector<unsigned char>& blob, BlobOffsets& o) {
  const int A = c.n_agents, Q = c.n_rm_states, E = c.n_events, HW = c.width * c.height;
  size_t off = 0;
  o.cell = (int32_t)off;
  off = align16(off + sizeof(uint16_t) * HW);
  o.ev = (int32_t)off;
  off = align16(off + (size_t)A * HW);
  o.nq = (int32_t)off;
  off = align16(off + (size_t)A * Q * E);
  o.rr = (int32_t)off;
  off = align16(off + sizeof(float) * A * Q * E);
  o.sh = (int32_t)off;
  if (c.has_shaping) off = align16(off + sizeof(float) * A * Q * E);
  o.qrm = (int32_t)off;
  if (c.n_qrm_max > 0) off = align16(off + (size_t)A * c.n_qrm_max);
  if (off > 64 * 1024) return false;
  blob.assign(off, 0);
  memcpy(blob.data() + o.cell, c.cell, sizeof(uint16_t) * HW);
  memcpy(blob.data() + o.ev, c.cell_event, (size_t)A * HW);
  memcpy(blob.data() + o.nq, c.next_q, (size_t)A * Q * E);
  memcpy(blob.data() + o.rr, c.rm_reward, sizeof(float) * A * Q * E);
  if (c.has_shaping) memcpy(blob.data() + o.sh, c.shape, sizeof(float) * A * Q * E);
  if (c.n_qrm_max > 0) memcpy(blob.data() + o.qrm, c.qrm_states, (size_t)A * c.n_qrm_max);
  return true;
}

std::vector<float> discount_table(const rmx_config& c) {
  std::vector<float> disc((size_t)c.max_t + 2);
  double g = 1.0;
  for (size_t i = 0; i < disc.size(); ++i) {
    disc[i] = (float)g;
    g *= (double)c.gamma;
  }
  return disc;
}

// Pre-compose the fast-path blob: one move word per (agent, cell, action) restating agent_step<KIND>'s move /
// wall / hazard / event rules, and the RM entries with the final bit and the reward_modifier folded in.
bool build_fast_blob(const rmx_config& c, std::vector<unsigned char>& blob, FastLayout& L) {
  const int A = c.n_agents, Q = c.n_rm_states, E = c.n_events, W = c.width, H = c.height, HW = W * H;
  // slip and FrozenLake random starts run on the fast path too (step_fast_kernel<..., SLIP>, merged records)
  if (A > kFastMaxAgents || W > 255 || H > 255 || E > 255 || Q > 255)
    return false;
  if ((int64_t)A * c.n_envs >= ((int64_t)1 << 30)) return false;  // 32-bit column byte offsets (A*N*4 < 2^32)
  const size_t mv_bytes = align16(sizeof(uint32_t) * (size_t)A * HW * 5);
  const size_t rm_bytes = 16 * (size_t)A * Q * E;
  const size_t info_bytes = 16 * (size_t)A;
  // (rounds 1-4 sized this for a 256-thread block's LDS staging, plus the lane-resident sections; the limit stays)
  const size_t total = mv_bytes + rm_bytes + info_bytes;
  if (total + 4 * 128 + 4 * 3 * 64 > kFastBlobMaxBytes) return false;
  blob.assign(total, 0);
  L.off_rm = (int32_t)mv_bytes;
  L.off_info = (int32_t)(mv_bytes + rm_bytes);
  uint32_t* info = reinterpret_cast<uint32_t*>(blob.data() + L.off_info);
  for (int a = 0; a < A; ++a) {
    const uint32_t fqb = c.final_q[a] < 0 ? 255u : (uint32_t)c.final_q[a];
    info[4 * a + 0] = (uint32_t)(a * HW * 5);
    info[4 * a + 1] = (uint32_t)(a * Q * E);
    info[4 * a + 2] = (uint32_t)c.start_xy[2 * a] | ((uint32_t)c.start_xy[2 * a + 1] << 8) |
                      ((uint32_t)c.init_q[a] << 16) | (fqb << 24);
    info[4 * a + 3] = c.enc_nq ? (uint32_t)c.enc_nq[a] : 0u;  // state-encoder stride (enc_state output)
  }
  const int up = c.kind == RMX_FROZEN_LAKE ? -1 : 1;
  const int dx[4] = {0, 0, -1, 1}, dy[4] = {up, -up, 0, 0};
  uint32_t* mv = reinterpret_cast<uint32_t*>(blob.data());
  for (int a = 0; a < A; ++a)
    for (int y = 0; y < H; ++y)
      for (int x = 0; x < W; ++x)
        for (int ac = 0; ac <= RMX_WAIT; ++ac) {
          const int cix = y * W + x;
          const bool can = ac < RMX_WAIT && ((c.cell[cix] >> ac) & 1u);
          const bool wall = c.kind == RMX_OFFICE_WORLD && ac < RMX_WAIT && !can;
          const int nx = can ? x + dx[ac] : x, ny = can ? y + dy[ac] : y;
          const int nc = ny * W + nx;
          const bool haz = (c.cell[nc] & RMX_CELL_HAZARD) != 0;
          const bool failing = c.kind == RMX_FROZEN_LAKE ? haz : ((wall && c.wall_fail) || (haz && c.hazard_fail));
          const uint32_t ev = c.cell_event[(size_t)a * HW + nc];
          mv[((size_t)a * HW + cix) * 5 + ac] = (uint32_t)nx | ((uint32_t)ny << 8) | (ev << 16) | (wall ? kMvWall : 0u) |
                                                (haz ? kMvHazard : 0u) | (failing ? kMvFail : 0u);
        }
  uint32_t* rm = reinterpret_cast<uint32_t*>(blob.data() + L.off_rm);
  for (int a = 0; a < A; ++a)
    for (int i = 0; i < Q * E; ++i) {
      const size_t ti = (size_t)a * Q * E + i;
      const uint32_t nq = c.next_q[ti];
      const float mrq = c.reward_modifier * c.rm_reward[ti];
      const float shp = c.has_shaping ? c.shape[ti] : 0.0f;
      rm[4 * ti] = nq | ((int32_t)nq == c.final_q[a] ? (1u << 8) : 0u);
      memcpy(&rm[4 * ti + 1], &mrq, sizeof(float));
      memcpy(&rm[4 * ti + 2], &shp, sizeof(float));
      memcpy(&rm[4 * ti + 3], &c.rm_reward[ti], sizeof(float));  // raw RQ (QRM experiences)
    }
  return true;
}

// The merged table: for every (agent, q, cell, action) the move word of build_fast_blob and the RM entry of
// (q, event at the destination) in one 16-B record.  Agents whose sections are identical (same RM, events,
// penalties: every agent of a BASELINE FrozenLake config) share one copy, so the table the lookups touch is
// A times smaller.
bool build_merged(const rmx_config& c, const std::vector<unsigned char>& blob, int32_t off_rm, int32_t* mg_base,
                  std::vector<uint32_t>& out) {
  const int A = c.n_agents, Q = c.n_rm_states, E = c.n_events, HW = c.width * c.height;
  const size_t sec = (size_t)Q * HW * 5;  // records per agent section
  if (sec * 16 > kMergedMaxBytes) return false;
  const uint32_t* mv = reinterpret_cast<const uint32_t*>(blob.data());
  const uint32_t* rm = reinterpret_cast<const uint32_t*>(blob.data() + off_rm);
  out.clear();
  std::vector<uint32_t> s(sec * 4);
  for (int a = 0; a < A; ++a) {
    std::fill(s.begin(), s.end(), 0u);
    for (int q = 0; q < Q; ++q)
      for (int cix = 0; cix < HW; ++cix)
        for (int ac = 0; ac <= RMX_WAIT; ++ac) {
          const uint32_t m = mv[((size_t)a * HW + cix) * 5 + ac];
          const uint32_t ev = (m >> 16) & 0xFFu;
          const uint32_t* r = rm + 4 * (((size_t)a * Q + q) * E + ev);
          const size_t o = 4 * (((size_t)q * HW + cix) * 5 + ac);
          s[o] = (m & 0x0700FFFFu) | ((r[0] & 0xFFu) << 16) | (((r[0] >> 8) & 1u) << 27);
          s[o + 1] = r[1];
          s[o + 2] = r[2];
        }
    int same = -1;
    for (size_t b = 0; b < out.size() / (sec * 4) && same < 0; ++b)
      if (std::equal(s.begin(), s.end(), out.begin() + b * sec * 4)) same = (int)b;
    if (same < 0) {
      same = (int)(out.size() / (sec * 4));
      if ((out.size() + s.size()) * 4 > kMergedMaxBytes) return false;
      out.insert(out.end(), s.begin(), s.end());
    }
    mg_base[a] = (int32_t)(same * sec);
  }
  return true;
}

// One u32 per record: word 0 with the reward replaced by its index into a per-section palette of <= 4
// distinct reward bit patterns (bits 28-29), the palette as four signed bytes.  Only without shaping (the shaping
// word is dropped) and for integer rewards in [-128, 127] (the kernel converts the byte back to f32 exactly; -0.0 has
// no byte form).
bool build_compact(const rmx_config& c, const int32_t* mg_base, const std::vector<uint32_t>& merged, uint32_t* mg_palb,
                   std::vector<uint32_t>& out) {
  if (c.has_shaping) return false;
  const size_t sec = (size_t)c.n_rm_states * c.width * c.height * 5;
  const size_t n = merged.size() / 4;
  out.assign(n, 0u);
  for (size_t b = 0; b * sec < n; ++b) {  // one palette per stored section
    std::vector<uint32_t> pal;
    for (size_t i = b * sec; i < (b + 1) * sec; ++i) {
      const uint32_t w0 = merged[4 * i], rw = merged[4 * i + 1];
      if (w0 >> 28) return false;  // word-0 layout leaves bits 28-31 free
      size_t k = std::find(pal.begin(), pal.end(), rw) - pal.begin();
      if (k == pal.size()) {
        if (pal.size() == 4) return false;
        pal.push_back(rw);
      }
      out[i] = w0 | ((uint32_t)k << 28);
    }
    uint32_t packed = 0;
    for (int k = 0; k < (int)pal.size(); ++k) {
      float v;
      memcpy(&v, &pal[k], 4);
      if (!(v >= -128.0f && v <= 127.0f && v == (float)(int)v) || (v == 0.0f && (pal[k] >> 31))) return false;
      packed |= (uint32_t)(uint8_t)(int8_t)(int)v << (8 * k);
    }
    for (int a = 0; a < c.n_agents; ++a)
      if ((size_t)mg_base[a] == b * sec) mg_palb[a] = packed;
  }
  return true;
}

std::vector<uint16_t> free_cells(const rmx_config& c) {
  std::vector<uint16_t> out;
  for (int x = 0; x < c.width; ++x)
    for (int y = 0; y < c.height; ++y)
      if (!(c.cell[y * c.width + x] & RMX_CELL_HAZARD)) out.push_back((uint16_t)(y * c.width + x));
  return out;
}

}  // namespace rmx
