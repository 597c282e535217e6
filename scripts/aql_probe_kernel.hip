// aql_probe_kernel.hip — the kernel of scripts/aql_probe.cpp (diagnostic): config 2's step I/O at 65,536 envs as a
// copy, explicit arguments only (no blockDim / gridDim: no hidden kernel arguments), built as a raw code object.
#include <hip/hip_runtime.h>

extern "C" __global__ void __launch_bounds__(64) copy_step_io(int n, int blk, int* c0, int* c1, int* c2, int* c3,
                                                              int* c4, int* t, const int* act, int* rew,
                                                              unsigned char* done) {
  const int e = (int)blockIdx.x * blk + (int)threadIdx.x;
  if (e >= n) return;
  int* c[5] = {c0, c1, c2, c3, c4};
  const int tv = t[e];
  int v[2][6];
#pragma unroll
  for (int a = 0; a < 2; ++a) {
#pragma unroll
    for (int k = 0; k < 5; ++k) v[a][k] = c[k][a * n + e];
    v[a][5] = act[a * n + e];
  }
  t[e] = tv + 1;
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    c[0][a * n + e] = v[a][0] + v[a][5];
    c[1][a * n + e] = v[a][1] + v[a][5];
    c[3][a * n + e] = v[a][3] + v[a][5];
    rew[a * n + e] = v[a][5] ^ v[a][2] ^ v[a][4];
  }
  done[e] = (unsigned char)tv;
}
