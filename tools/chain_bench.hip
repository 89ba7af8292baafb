// Dependent-chain cost of the float adds used by the vc / ray-position replays:
// v_add_f32 chains (x, y, z separate) vs v_pk_add_f32 ({x, y} packed) + v_add_f32.
// One wave per SIMD (latency) and 8 waves per SIMD (throughput); s_memtime cycles.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float pf2 __attribute__((ext_vector_type(2)));
template <int kMode>
__global__ void k_chain(float *out, unsigned long long *cyc, int n, float s0, float s1, float s2) {
  float x = threadIdx.x * 1e-3f, y = x + 1.f, z = x + 2.f;
  pf2 xy = {x, y};
  const pf2 sxy = {s0, s1};
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; i += 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (kMode == 0) {  // three scalar chains, kept scalar with an asm barrier
        asm volatile("v_add_f32 %0, %0, %1" : "+v"(x) : "v"(s0));
        asm volatile("v_add_f32 %0, %0, %1" : "+v"(y) : "v"(s1));
        asm volatile("v_add_f32 %0, %0, %1" : "+v"(z) : "v"(s2));
      } else {  // packed {x, y} + scalar z (what the compiler emits)
        xy = xy + sxy;
        z = z + s2;
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (kMode == 1) x = xy.x, y = xy.y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = x + y + z;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
int main() {
  float *out;
  unsigned long long *cyc, h[4096];
  hipMalloc(&out, 4096 * 1024 * 4);
  hipMalloc(&cyc, 4096 * 8);
  const int n = 4096;
  for (int waves : {1, 8}) {
    const int blocks = 256 * 4 * waves;  // one 64-thread block per wave: waves per SIMD
    for (int mode = 0; mode < 2; ++mode) {
      for (int rep = 0; rep < 2; ++rep) {
        if (mode == 0) hipLaunchKernelGGL(k_chain<0>, dim3(blocks), dim3(64), 0, 0, out, cyc, n, 1e-7f, 2e-7f, 3e-7f);
        else hipLaunchKernelGGL(k_chain<1>, dim3(blocks), dim3(64), 0, 0, out, cyc, n, 1e-7f, 2e-7f, 3e-7f);
        hipDeviceSynchronize();
      }
      hipMemcpy(h, cyc, 8 * std::min(blocks, 4096), hipMemcpyDeviceToHost);
      double m = 0;
      for (int b = 0; b < std::min(blocks, 4096); ++b) m += (double)h[b];
      m /= std::min(blocks, 4096);
      printf("%s waves/SIMD %d: %.1f cycles per step (3 adds)\n", mode ? "packed xy + z" : "scalar x,y,z", waves, m / n);
    }
  }
  return 0;
}
