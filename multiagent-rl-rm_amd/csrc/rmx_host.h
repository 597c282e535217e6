// rmx_host.h — host-only half of rmx_create: config validation and the table builders (rmx_tables.cpp).
// Plain C++ (no HIP): the sanitizer build (oracle/Makefile `asan`) compiles the same source with g++.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/rmx.h"
#include "rmx_layout.h"

namespace rmx {

// "" when the config is valid, else the RMX_E_INVALID message (every check rmx_create makes before it
// touches a table: sizes, ranges of every table entry, moves the tile allows, random-start feasibility).
std::string validate_config(const rmx_config& c);

// 64-bit digest of the compiled scenario (geometry, rules, dense tables, RM indices, slip tables, seed schedule):
// rmx_get_state writes it into the checkpoint header, rmx_set_state refuses a blob whose digest differs.
uint64_t config_digest(const rmx_config& c);

// The generic kernels' table blob (staged whole into LDS): [cell u16][cell_event u8][next_q u8][rm_reward
// f32][shape f32][qrm_states u8], 16-B aligned sections.  False when it exceeds 64 KiB.
struct BlobOffsets {
  int32_t cell = 0, ev = 0, nq = 0, rr = 0, sh = 0, qrm = 0;
};
bool build_table_blob(const rmx_config& c, std::vector<unsigned char>& blob, BlobOffsets& off);

// gamma^t for t = 0 .. max_t + 1 as repeated f64 products (office_main.py:1747), stored f32.
std::vector<float> discount_table(const rmx_config& c);

// Fast-path blob (layout in rmx_layout.h).  False when the config is outside the fast path.
struct FastLayout {
  int32_t off_rm = 0, off_info = 0;
};
bool build_fast_blob(const rmx_config& c, std::vector<unsigned char>& blob, FastLayout& L);

// Merged single-lookup table (16-B records), one section per distinct agent; mg_base[a] = record index of
// agent a's section.  False when a section or the whole table exceeds kMergedMaxBytes.
bool build_merged(const rmx_config& c, const std::vector<unsigned char>& blob, int32_t off_rm, int32_t* mg_base,
                  std::vector<uint32_t>& out);
// 4-B records with a <= 4-entry reward palette per section, mg_palb[a] = the palette as four signed bytes; false when
// not eligible (shaping, > 4 distinct rewards, or a reward that is not an integer in [-128, 127] or is -0.0).
bool build_compact(const rmx_config& c, const int32_t* mg_base, const std::vector<uint32_t>& merged, uint32_t* mg_palb,
                   std::vector<uint32_t>& out);

// FrozenLake random_start_positions: the non-hole cells as y*W + x in the reference's x-major order
// (ma_frozen_lake.py:163-168).
std::vector<uint16_t> free_cells(const rmx_config& c);

}  // namespace rmx
