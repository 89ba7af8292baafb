// ICP hand-off microbenchmark (round-6 verdict item 4): the cost of one
// iteration's cross-block hand-off of k_icp_track (27 agent-scope int64 adds
// into 4 partial-sum shards, s_waitcnt, an arrival counter, the last arriver
// storing 8 release-flag copies, a relaxed agent-scope poll of copy b % 8,
// then the 108 coherent shard loads), with no lane work and no solve, for:
//   - P = 240 blocks spread over the grid (C2 level 0's co-resident grid),
//   - P = 30 or 32 blocks that share one XCD (blocks b % 8 == 0 of a
//     256-block grid: one XCD under the round-robin placement; the protocol
//     stays agent-scope, placement decides speed only),
//   - P = 32 blocks spread over the XCDs (blocks 0..31).
// Block 0 stamps s_memtime over kIters iterations; the program prints the
// mean per iteration in shader cycles and microseconds (clock from the
// kernel's wall time).  Non-participating blocks exit at once.
// build: hipcc -O3 --offload-arch=gfx950 tools/icp_barrier_bench.hip -o tools/build/icp_barrier_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr int kIters = 2000;
constexpr int kShards = 16;  // most shards a case uses
constexpr int kThreads = 256;

struct Sync {
  unsigned arrive, pad0[31];
  struct {
    unsigned v, pad[31];
  } sub[8];  // hierarchical arrival: per residue b % 8
  unsigned top, pad1[31];
  struct {
    unsigned v, pad[31];
  } release[8];
  unsigned long long sums[kIters + 1][kShards * 27];
};

// mode 0: participants are blocks 0..P-1; mode 1: blocks with b % 8 == 0 (rank b / 8)
__global__ __launch_bounds__(kThreads) void k_handoff(Sync *sy, int P, int mode, int nload, int hier, int nadd, int nsh, unsigned long long *out) {
  const int b = blockIdx.x;
  int rank;
  if (mode == 0) {
    rank = b;
    if (b >= P) return;
  } else {
    if (b % 8 != 0) return;
    rank = b / 8;
    if (rank >= P) return;
  }
  __shared__ double red[kShards * 27];
  __shared__ long long sums[27];
  unsigned long long t0 = 0;
  long long carry = 0;
  for (int it = 0; it < kIters; ++it) {
    if (it == 1 && rank == 0 && threadIdx.x == 0) t0 = __builtin_amdgcn_s_memtime();
    unsigned long long *sh = sy->sums[it];
    if (threadIdx.x < 64) {
      if (threadIdx.x < nadd)
        __hip_atomic_fetch_add(&sh[(rank % nsh) * 27 + threadIdx.x], (unsigned long long)(rank + 1 + carry),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (threadIdx.x == 0 && !hier) {
        const unsigned n = __hip_atomic_fetch_add(&sy->arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (n == (unsigned)P * (unsigned)(it + 1) - 1u)
          for (int k = 0; k < 8; ++k)
            __hip_atomic_store(&sy->release[k].v, (unsigned)(it + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else if (threadIdx.x == 0) {
        // per-residue counter (rank % 8: ranks of one residue), then the
        // residue's last arriver adds to the top counter (8 adds)
        const int r = rank & 7;
        const unsigned nr = (unsigned)((P - r + 7) / 8);  // ranks of residue r
        const unsigned n = __hip_atomic_fetch_add(&sy->sub[r].v, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (n == nr * (unsigned)(it + 1) - 1u) {
          const unsigned groups = (unsigned)(P < 8 ? P : 8);
          const unsigned m = __hip_atomic_fetch_add(&sy->top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (m == groups * (unsigned)(it + 1) - 1u)
            for (int k = 0; k < 8; ++k)
              __hip_atomic_store(&sy->release[k].v, (unsigned)(it + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
    if (threadIdx.x == 0) {
      const unsigned *flag = &sy->release[b & 7].v;
      while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)(it + 1))
        __builtin_amdgcn_s_sleep(1);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nsh * 27; i += kThreads)
      red[i] = i < nload ? __longlong_as_double((long long)__hip_atomic_load(&sh[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) : 0.0;
    __syncthreads();
    if (threadIdx.x < 27) {
      long long a = 0;
      for (int k = 0; k < nsh; ++k) a += __double_as_longlong(red[k * 27 + threadIdx.x]);
      sums[threadIdx.x] = a;
    }
    __syncthreads();
    carry = sums[0] & 1;  // a data dependency on the iteration's sums, as the solve has
  }
  if (rank == 0 && threadIdx.x == 0) {
    out[0] = __builtin_amdgcn_s_memtime() - t0;
    out[1] = (unsigned long long)sums[0];
  }
}

#define CK(x)                                                             \
  do {                                                                    \
    hipError_t e = (x);                                                   \
    if (e != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));              \
      return 1;                                                           \
    }                                                                     \
  } while (0)

int main() {
  Sync *sy;
  unsigned long long *out;
  CK(hipMalloc(&sy, sizeof(Sync)));
  CK(hipMalloc(&out, 16));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  struct Case {
    const char *name;
    int grid, P, mode, nload, hier, nadd, nsh;
  } cases[] = {{"240 blocks, spread", 240, 240, 0, 108, 0, 27, 4},   {"32 blocks, one XCD", 256, 32, 1, 108, 0, 27, 4},
               {"30 blocks, one XCD", 256, 30, 1, 108, 0, 27, 4},    {"32 blocks, spread", 32, 32, 0, 108, 0, 27, 4},
               {"70 blocks, spread", 70, 70, 0, 108, 0, 27, 4},      {"8 blocks, one XCD", 256, 8, 1, 108, 0, 27, 4},
               {"240 blocks, 12 loads", 240, 240, 0, 12, 0, 27, 4},  {"240 blocks, no loads", 240, 240, 0, 0, 0, 27, 4},
               {"300 blocks, spread", 300, 300, 0, 108, 0, 27, 4},   {"240 blocks, hier", 240, 240, 0, 108, 1, 27, 4},
               {"300 blocks, hier", 300, 300, 0, 108, 1, 27, 4},     {"70 blocks, hier", 70, 70, 0, 108, 1, 27, 4},
               {"240 hier, no adds", 240, 240, 0, 0, 1, 0, 4},  {"300 hier, no adds", 300, 300, 0, 0, 1, 0, 4},
               {"240 flat, no adds", 240, 240, 0, 0, 0, 0, 4},  {"300 hier, 8 adds", 300, 300, 0, 108, 1, 8, 4},
               {"300 hier, 8 shards", 300, 300, 0, 216, 1, 27, 8},  {"300 hier, 16 shards", 300, 300, 0, 432, 1, 27, 16},
               {"240 hier, 8 shards", 240, 240, 0, 216, 1, 27, 8},  {"300 flat, 8 shards", 300, 300, 0, 216, 0, 27, 8}};
  for (int rep = 0; rep < 2; ++rep) {
    for (const Case &c : cases) {
      CK(hipMemset(sy, 0, sizeof(Sync)));
      CK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL(k_handoff, dim3(c.grid), dim3(kThreads), 0, 0, sy, c.P, c.mode, c.nload, c.hier, c.nadd, c.nsh, out);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      unsigned long long h[2];
      CK(hipMemcpy(h, out, 16, hipMemcpyDeviceToHost));
      if (rep == 0) continue;
      const double cyc = (double)h[0] / (kIters - 1);
      const double us = ms * 1e3 / kIters;
      printf("%-22s per iteration: %8.0f shader cycles, %6.2f us (kernel wall / iterations)\n", c.name, cyc, us);
    }
  }
  return 0;
}
