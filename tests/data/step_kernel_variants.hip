// Negative controls for the queue's code-object metadata check (tests/test_queue_meta.py), compiled by the test to a
// gfx950 code object and never loaded or run.  Three kernels named like the engine's step kernel, with its parameter
// list: V = 0 as the engine's kernels are (accepted), V = 1 with a debugging printf (its hidden_hostcall_buffer is
// not written by the queue: refused), and an instantiation whose explicit arguments differ (refused).
#include <cstdio>

#include "rmx_internal.h"

namespace rmx {

template <int V>
__global__ void step_fast_kernel(int32_t N, int32_t blk, const int32_t* x, const int32_t* y, const int32_t* q,
                                 const uint32_t* f, const int32_t* t, const int32_t* a, FastParams p) {
  if (V == 1 && N < 0) printf("step %d\n", blk);
  if (N < 0) p.err[0] = x[0] + y[0] + q[0] + (int)f[0] + t[0] + a[0] + (int)blockDim.x;
}
template __global__ void step_fast_kernel<0>(int32_t, int32_t, const int32_t*, const int32_t*, const int32_t*,
                                             const uint32_t*, const int32_t*, const int32_t*, FastParams);
template __global__ void step_fast_kernel<1>(int32_t, int32_t, const int32_t*, const int32_t*, const int32_t*,
                                             const uint32_t*, const int32_t*, const int32_t*, FastParams);

// the same name with one column pointer fewer
template <int V>
__global__ void step_fast_kernel(int32_t N, int32_t blk, const int32_t* x, const int32_t* y, const uint32_t* f,
                                 const int32_t* t, const int32_t* a, FastParams p) {
  if (N < 0) p.err[0] = x[0] + y[0] + (int)f[0] + t[0] + a[0] + blk;
}
template __global__ void step_fast_kernel<2>(int32_t, int32_t, const int32_t*, const int32_t*, const uint32_t*,
                                             const int32_t*, const int32_t*, FastParams);

}  // namespace rmx
