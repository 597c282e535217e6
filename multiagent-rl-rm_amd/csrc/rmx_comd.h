// rmx_comd.h — the engine queue's check of a gfx950 code object's kernel metadata (host-only C++: no HIP, no HSA).
// rmx_queue.cpp writes step_fast_kernel's kernel arguments itself (StepArgs, then the code object v5 hidden arguments a
// 1-D HIP launch carries); a kernel whose NT_AMDGPU_METADATA note lists anything else (a debugging printf adds
// hidden_hostcall_buffer, which would read 0 in a queue packet) or another explicit layout is refused, and its windows
// run on the caller's stream.  The reader takes caller-supplied bytes (rmx_code_object_check): every length is bounded
// by the buffer, and the sanitizer build drives it with corrupted objects (oracle/Makefile `asan`,
// tests/test_sanitizers.py).
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <unordered_map>

namespace rmx {

// The argument image the queue writes: N and the block size (4 B each), six 8-B column pointers, the parameter block
// at fp_offset (fp_size bytes), then the hidden arguments from hidden_base (the first 8-aligned offset after it)
struct CoLayout {
  uint64_t fp_offset, fp_size, hidden_base;
};
constexpr size_t kHiddenUsed = 124;  // the hidden arguments the queue writes end at hidden_dynamic_lds_size (120, 4 B)

// every step_fast_kernel in the object: its symbol -> the reason the queue refuses it (absent: accepted)
struct CoCheck {
  std::string err;  // the object could not be read: every kernel is refused
  std::unordered_map<std::string, std::string> refused;
  int64_t n_step = 0;
};

CoCheck check_code_object(const unsigned char* co, size_t bytes, const CoLayout& L);

}  // namespace rmx
