// rmxh_entry.cpp — TEST INFRASTRUCTURE ONLY: a C entry point over the engine's host-side table builders
// (multiagent-rl-rm_amd/csrc/rmx_tables.cpp, compiled unchanged next to this file) for the sanitizer build
// (oracle/Makefile `asan`, tests/test_sanitizers.py).  Runs every builder rmx_create runs, in the same
// order, on one config and reports the sizes it produced.
#include <vector>

#include "../../multiagent-rl-rm_amd/csrc/rmx_comd.h"
#include "../../multiagent-rl-rm_amd/csrc/rmx_host.h"

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
