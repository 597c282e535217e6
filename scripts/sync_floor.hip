// sync_floor.hip — floors of the host<->device mailbox round trip behind rmx_step_sync (rmx_sync.hip).
// One resident lane polls a request word and answers with an acknowledgement word; the host spins on the
// acknowledgement.  Variants: where the request word lives (pinned coherent host memory, or fine-grained device
// memory the host writes through the BAR), how many host-memory words the device reads after the request (the
// actions) and writes before the acknowledgement (the outputs), and whether the outputs go out as 4-B or 16-B
// stores.  Diagnostic only (never loaded by the product).
//   hipcc -O3 --offload-arch=gfx950 -o scripts/sync_floor scripts/sync_floor.hip
//   ./scripts/sync_floor [host|vram]
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

constexpr uint32_t kExit = 0xFFFFFFFFu;

template <int READS, int WRITES, bool WIDE>
__global__ void pingpong(uint32_t* req, const uint32_t* acts, uint32_t* out, uint32_t* ack, uint64_t idle_ticks) {
  if (threadIdx.x != 0) return;
  uint32_t last = 0;
  uint64_t t_idle = (uint64_t)wall_clock64();
  for (;;) {
    uint32_t v;
    for (;;) {
      v = __hip_atomic_load(req, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
      if (v != last) break;
      if ((uint64_t)wall_clock64() - t_idle > idle_ticks) return;
      __builtin_amdgcn_s_sleep(1);
    }
    if (v == kExit) return;
    uint32_t x = v;
#pragma unroll
    for (int i = 0; i < READS; ++i) x += __hip_atomic_load(acts + 4 * i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if constexpr (WIDE) {
#pragma unroll
      for (int i = 0; i < WRITES; i += 4)
        *reinterpret_cast<uint4*>(out + i) = make_uint4(x, x + 1, x + 2, x + 3);
    } else {
#pragma unroll
      for (int i = 0; i < WRITES; ++i) out[i] = x + i;
    }
    __hip_atomic_store(ack, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    last = v;
    t_idle = (uint64_t)wall_clock64();
  }
}

// The resident stepper's form: the request as one 16-B sc0|sc1 buffer load (POLLS of them in flight, issued
// s_sleep(1) apart), outputs as sc0|sc1 (system write-through) buffer stores, s_waitcnt vmcnt(0), then the
// acknowledgement as one more sc0|sc1 store: no L2 writeback or invalidate anywhere.
template <int WRITES, int POLLS>
__global__ void pingpong_wt(uint32_t* req, uint32_t* out, uint32_t* ack, uint64_t idle_ticks) {
  if (threadIdx.x != 0) return;
  const auto rq = __builtin_amdgcn_make_buffer_rsrc(req, 0, 16, 0x00020000);
  const auto ro = __builtin_amdgcn_make_buffer_rsrc(out, 0, 4096, 0x00020000);
  const auto ra = __builtin_amdgcn_make_buffer_rsrc(ack, 0, 4, 0x00020000);
  uint32_t last = 0;
  uint64_t t_idle = (uint64_t)wall_clock64();
  for (;;) {
    uint32_t v = last;
    if constexpr (POLLS == 1) {
      for (;;) {
        const auto w = __builtin_amdgcn_raw_buffer_load_b128(rq, 0, 0, 17);
        if (w[0] != last && w[0] == w[3]) {
          v = w[0];
          break;
        }
        if ((uint64_t)wall_clock64() - t_idle > idle_ticks) return;
        __builtin_amdgcn_s_sleep(1);
      }
    } else {
      uint32_t q[POLLS];
#pragma unroll
      for (int j = 0; j < POLLS; ++j) {
        q[j] = __builtin_amdgcn_raw_buffer_load_b32(rq, 0, 0, 17);
        __builtin_amdgcn_s_sleep(1);
      }
      for (;;) {
        bool got = false;
#pragma unroll
        for (int j = 0; j < POLLS; ++j) {  // oldest first; each consumed slot is re-issued at once
          if (!got && q[j] != last) {
            v = q[j];
            got = true;
          }
          q[j] = __builtin_amdgcn_raw_buffer_load_b32(rq, 0, 0, 17);
          __builtin_amdgcn_s_sleep(1);
        }
        if (got) break;
        if ((uint64_t)wall_clock64() - t_idle > idle_ticks) return;
      }
      __builtin_amdgcn_s_waitcnt(0);  // drain the polls still in flight
    }
    if (v == kExit) return;
#pragma unroll
    for (int i = 0; i < WRITES; ++i) __builtin_amdgcn_raw_buffer_store_b32(v + i, ro, 4 * i, 0, 17);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_waitcnt(0);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_raw_buffer_store_b32(v, ra, 0, 0, 17);
    last = v;
    t_idle = (uint64_t)wall_clock64();
  }
}

template <int WRITES, int POLLS>
double run_wt(uint32_t* req_h, uint32_t* req_d, uint32_t* out_d, uint32_t* ack_h, uint32_t* ack_d, uint64_t idle,
              int iters) {
  std::memset(req_h, 0, 16);
  __atomic_store_n(ack_h, 0u, __ATOMIC_RELEASE);
  hipLaunchKernelGGL((pingpong_wt<WRITES, POLLS>), dim3(1), dim3(64), 0, 0, req_d, out_d, ack_d, idle);
  CHECK(hipGetLastError());
  double best = 1e30;
  uint32_t seq = 0;
  for (int rep = 0; rep < 5; ++rep) {
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < iters; ++i) {
      ++seq;
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      _mm_store_si128(reinterpret_cast<__m128i*>(req_h), _mm_set_epi32((int)seq, 0, 0, (int)seq));
      const auto w0 = std::chrono::steady_clock::now();
      while (__atomic_load_n(ack_h, __ATOMIC_ACQUIRE) != seq) {
        __builtin_ia32_pause();
        if (std::chrono::steady_clock::now() - w0 > std::chrono::seconds(2)) {
          std::fprintf(stderr, "no acknowledgement for request %u\n", seq);
          std::exit(2);
        }
      }
    }
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / iters;
    best = us < best ? us : best;
  }
  _mm_store_si128(reinterpret_cast<__m128i*>(req_h), _mm_set_epi32((int)kExit, 0, 0, (int)kExit));
  CHECK(hipDeviceSynchronize());
  return best;
}

template <int READS, int WRITES, bool WIDE>
double run(uint32_t* req_h, uint32_t* req_d, uint32_t* acts_d, uint32_t* out_d, uint32_t* ack_h, uint32_t* ack_d,
           uint64_t idle, int iters) {
  *req_h = 0;
  __atomic_store_n(ack_h, 0u, __ATOMIC_RELEASE);
  hipLaunchKernelGGL((pingpong<READS, WRITES, WIDE>), dim3(1), dim3(64), 0, 0, req_d, acts_d, out_d, ack_d, idle);
  CHECK(hipGetLastError());
  double best = 1e30;
  uint32_t seq = 0;
  for (int rep = 0; rep < 5; ++rep) {
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < iters; ++i) {
      ++seq;
      __atomic_store_n(req_h, seq, __ATOMIC_RELEASE);
      const auto w0 = std::chrono::steady_clock::now();
      while (__atomic_load_n(ack_h, __ATOMIC_ACQUIRE) != seq) {
        __builtin_ia32_pause();
        if (std::chrono::steady_clock::now() - w0 > std::chrono::seconds(2)) {
          std::fprintf(stderr, "no acknowledgement for request %u\n", seq);
          std::exit(2);
        }
      }
    }
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / iters;
    best = us < best ? us : best;
  }
  __atomic_store_n(req_h, kExit, __ATOMIC_RELEASE);
  CHECK(hipDeviceSynchronize());
  return best;
}

int main(int argc, char** argv) {
  const bool vram = argc > 1 && !std::strcmp(argv[1], "vram");
  int khz = 0;
  CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0));
  const uint64_t idle = (uint64_t)khz * 200;  // 200 ms
  unsigned char* host = nullptr;
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&host), 1 << 16, hipHostMallocCoherent | hipHostMallocMapped));
  std::memset(host, 0, 1 << 16);
  unsigned char* host_d = nullptr;
  CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&host_d), host, 0));
  uint32_t *req_h = reinterpret_cast<uint32_t*>(host), *req_d = reinterpret_cast<uint32_t*>(host_d);
  if (vram) {  // the request word in fine-grained device memory, written by the host through the BAR
    void* dv = nullptr;
    CHECK(hipExtMallocWithFlags(&dv, 4096, hipDeviceMallocFinegrained));
    CHECK(hipMemset(dv, 0, 4096));
    CHECK(hipDeviceSynchronize());
    req_h = req_d = static_cast<uint32_t*>(dv);
  }
  uint32_t* ack_h = reinterpret_cast<uint32_t*>(host + 256);
  uint32_t* ack_d = reinterpret_cast<uint32_t*>(host_d + 256);
  uint32_t* acts_d = reinterpret_cast<uint32_t*>(host_d + 1024);
  uint32_t* out_d = reinterpret_cast<uint32_t*>(host_d + 4096);
  const int it = 20000;
  std::printf("request in %s memory; us per round trip (best of 5 x %d)\n", vram ? "device (fine-grained)" : "host",
              it);
  std::printf("ping                 %.3f\n", run<0, 0, false>(req_h, req_d, acts_d, out_d, ack_h, ack_d, idle, it));
  std::printf("read 1               %.3f\n", run<1, 0, false>(req_h, req_d, acts_d, out_d, ack_h, ack_d, idle, it));
  std::printf("read 2               %.3f\n", run<2, 0, false>(req_h, req_d, acts_d, out_d, ack_h, ack_d, idle, it));
  std::printf("write 4 x 4B         %.3f\n", run<0, 4, false>(req_h, req_d, acts_d, out_d, ack_h, ack_d, idle, it));
  std::printf("write 16 x 4B        %.3f\n", run<0, 16, false>(req_h, req_d, acts_d, out_d, ack_h, ack_d, idle, it));
  std::printf("write 16 as 4 x 16B  %.3f\n", run<0, 16, true>(req_h, req_d, acts_d, out_d, ack_h, ack_d, idle, it));
  std::printf("read 2 + write 16    %.3f\n", run<2, 16, false>(req_h, req_d, acts_d, out_d, ack_h, ack_d, idle, it));
  std::printf("read 2 + write 16 wide %.3f\n", run<2, 16, true>(req_h, req_d, acts_d, out_d, ack_h, ack_d, idle, it));
  if (!vram) {
    std::printf("wt ping              %.3f\n", run_wt<0, 1>(req_h, req_d, out_d, ack_h, ack_d, idle, it));
    std::printf("wt write 16          %.3f\n", run_wt<16, 1>(req_h, req_d, out_d, ack_h, ack_d, idle, it));
    std::printf("wt write 16, 2 polls %.3f\n", run_wt<16, 2>(req_h, req_d, out_d, ack_h, ack_d, idle, it));
    std::printf("wt write 16, 4 polls %.3f\n", run_wt<16, 4>(req_h, req_d, out_d, ack_h, ack_d, idle, it));
  }
  // the launch-per-call alternative: one trivial kernel launch + stream synchronise
  {
    hipStream_t st;
    CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    *req_h = 0;
    double best = 1e30;
    for (int rep = 0; rep < 5; ++rep) {
      const auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < 2000; ++i) {
        __atomic_store_n(req_h, kExit, __ATOMIC_RELEASE);
        hipLaunchKernelGGL((pingpong<0, 0, false>), dim3(1), dim3(64), 0, st, req_d, acts_d, out_d, ack_d, idle);
        CHECK(hipStreamSynchronize(st));
      }
      const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / 2000;
      best = us < best ? us : best;
    }
    std::printf("launch + sync        %.3f\n", best);
    CHECK(hipStreamDestroy(st));
  }
  return 0;
}
