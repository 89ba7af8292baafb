// SQ issue-counter calibration (round-6 verdict item 5): known VALU streams,
// so that SQ_INSTS_VALU / SQ_ACTIVE_INST_VALU / GRBM_GUI_ACTIVE can be turned
// into "fraction of SIMD issue cycles" for the kfx kernels (tools/traffic.py).
//
// Each kernel runs 8 waves per SIMD on every SIMD (2048 blocks of 256 threads
// on 256 CUs), each wave issuing kIter x 16 instructions of one kind with 16
// independent accumulators (no dependency stalls: the SIMD's issue rate is
// the bound).  Every wave stamps s_memtime (shader cycles) at its start and
// end; the program prints, per kernel, the span in shader cycles of the
// busiest SIMD's 8 waves and the issue cost per instruction it implies:
//   cycles per wave-instruction = span / (8 waves x kIter x 16).
// Counter passes (one --pmc run each, tools/valu_calib.sh) then give
// SQ_INSTS_VALU and SQ_ACTIVE_INST_VALU per dispatch for the same kernels.
// build: hipcc -O3 --offload-arch=gfx950 tools/valu_calib.hip -o tools/build/valu_calib
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <map>
#include <vector>

constexpr int kIter = 4096;

__device__ __forceinline__ unsigned long long now() { return __builtin_amdgcn_s_memtime(); }
__device__ __forceinline__ unsigned hw_id() { return (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4); }
__device__ __forceinline__ unsigned xcc_id() { return (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20); }

#define STAMP_BEGIN const unsigned long long t0 = now();
#define STAMP_END(acc)                                                                      \
  const unsigned long long t1 = now();                                                      \
  if ((threadIdx.x & 63) == 0) {                                                            \
    const size_t w = (size_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;             \
    rec[4 * w] = t0;                                                                        \
    rec[4 * w + 1] = t1;                                                                    \
    rec[4 * w + 2] = ((unsigned long long)xcc_id() << 32) | hw_id();                        \
  }                                                                                         \
  if ((acc) == 12345.678f) rec[0] = 0; /* never: keeps the stream */

// 16 independent v_add_f32 per step
__global__ __launch_bounds__(256) void k_fadd(float seed, unsigned long long *rec) {
  float a[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) a[i] = seed * (float)(threadIdx.x + i);
  STAMP_BEGIN
  for (int it = 0; it < kIter; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(seed));
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += a[i];
  STAMP_END(s)
}

// 16 independent v_pk_fma_f32 per step (packed FP32, two lanes' worth each)
__global__ __launch_bounds__(256) void k_pkfma(float seed, unsigned long long *rec) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 a[16];
  const f2 b = {seed, seed * 0.5f}, c = {seed * 0.25f, seed};
#pragma unroll
  for (int i = 0; i < 16; ++i) a[i] = f2{seed * (float)i, seed + (float)threadIdx.x};
  STAMP_BEGIN
  for (int it = 0; it < kIter; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += a[i].x + a[i].y;
  STAMP_END(s)
}

// 16 independent v_rcp_f32 per step (transcendental unit)
__global__ __launch_bounds__(256) void k_rcp(float seed, unsigned long long *rec) {
  float a[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) a[i] = 1.f + seed * (float)(threadIdx.x + i);
  STAMP_BEGIN
  for (int it = 0; it < kIter; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) asm volatile("v_rcp_f32 %0, %0" : "+v"(a[i]));
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += a[i];
  STAMP_END(s)
}

// 16 independent v_mad_u32_u24 per step (integer address arithmetic)
__global__ __launch_bounds__(256) void k_mad24(float seed, unsigned long long *rec) {
  unsigned a[16];
  const unsigned m = (unsigned)seed + 3u;
#pragma unroll
  for (int i = 0; i < 16; ++i) a[i] = threadIdx.x + (unsigned)i;
  STAMP_BEGIN
  for (int it = 0; it < kIter; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) asm volatile("v_mad_u32_u24 %0, %0, %1, %1" : "+v"(a[i]) : "v"(m));
  }
  unsigned s = 0u;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += a[i];
  STAMP_END((float)s)
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
  const int blocks = 2048, threads = 256;  // 8 waves per SIMD on 256 CUs x 4 SIMDs
  const size_t waves = (size_t)blocks * threads / 64;
  unsigned long long *rec;
  CK(hipMalloc(&rec, waves * 4 * sizeof(unsigned long long)));
  std::vector<unsigned long long> h(waves * 4);
  struct K {
    const char *name;
    void (*fn)(float, unsigned long long *);
  } ks[] = {{"k_fadd", k_fadd}, {"k_pkfma", k_pkfma}, {"k_rcp", k_rcp}, {"k_mad24", k_mad24}};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int rep = 0; rep < 2; ++rep) {  // the second round is reported (clocks warmed up)
    for (const K &k : ks) {
      CK(hipMemset(rec, 0, waves * 4 * sizeof(unsigned long long)));
      CK(hipEventRecord(e0, 0));
      hipLaunchKernelGGL(k.fn, dim3(blocks), dim3(threads), 0, 0, 1.0001f, rec);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      CK(hipMemcpy(h.data(), rec, h.size() * 8, hipMemcpyDeviceToHost));
      if (rep == 0) continue;
      // per SIMD (xcc, se, cu, simd): span of its waves, wave count
      std::map<unsigned long long, std::pair<unsigned long long, unsigned long long>> simd;
      std::map<unsigned long long, int> cnt;
      for (size_t w = 0; w < waves; ++w) {
        const unsigned long long t0 = h[4 * w], t1 = h[4 * w + 1], id = h[4 * w + 2];
        const unsigned hw = (unsigned)id, xcc = (unsigned)(id >> 32);
        // HW_ID: simd [5:4], cu [11:8], sh [12], se [15:13]
        const unsigned long long key = ((unsigned long long)xcc << 16) | (((hw >> 8) & 0xFFu) << 2) | ((hw >> 4) & 3u);
        auto it = simd.find(key);
        if (it == simd.end()) simd[key] = {t0, t1};
        else it->second = {std::min(it->second.first, t0), std::max(it->second.second, t1)};
        cnt[key] += 1;
      }
      std::vector<double> cpi;
      for (auto &kv : simd) {
        const double span = (double)(kv.second.second - kv.second.first);
        cpi.push_back(span / ((double)cnt[kv.first] * kIter * 16));
      }
      std::sort(cpi.begin(), cpi.end());
      const double instr = (double)waves * kIter * 16;
      printf("%-8s waves %zu SIMDs %zu  wall %.3f ms  wave-instr %.4g  cycles/instr per SIMD: min %.3f med %.3f max %.3f"
             "  implied clock (GHz, med) %.3f\n",
             k.name, waves, simd.size(), ms, instr, cpi.front(), cpi[cpi.size() / 2], cpi.back(),
             cpi[cpi.size() / 2] * instr / simd.size() / (ms * 1e6));
    }
  }
  CK(hipFree(rec));
  return 0;
}
