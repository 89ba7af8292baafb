// Exhaustive check of cheap correctly-rounded primitives on gfx950 (every
// float bit pattern), used to replace IEEE sequences in the integrate and
// raycast kernels without changing a single result:
//   rcp:  y = fma(fma(-d, r, 1), r, r) with r = v_rcp_f32(d)   vs  1.f / d
//   sqrt: v_sqrt_f32(x)                                        vs  sqrtf(x)
// over the operand ranges where the cheap form is used (|d| in [2^-125, 2^125],
// x in [2^-96, inf)).  Prints mismatch counts and the first few operands.
// build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/rn_check.hip -o tools/build/rn_check
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__device__ __forceinline__ float rcp_nr(float d) {
  const float r = __builtin_amdgcn_rcpf(d);
  const float e = __builtin_fmaf(-d, r, 1.0f);
  return __builtin_fmaf(e, r, r);
}

// candidate correctly-rounded square roots for x in [2^-96, 2^126]
__device__ __forceinline__ float sqrt_v1(float x) {  // rsq + one Newton step
  const float y = __builtin_amdgcn_rsqf(x);
  const float s0 = x * y;
  const float h = 0.5f * y;
  const float r = __builtin_fmaf(-s0, s0, x);
  return __builtin_fmaf(r, h, s0);
}
__device__ __forceinline__ float sqrt_v3(float x) {  // v_sqrt + one Newton step
  const float s0 = __builtin_amdgcn_sqrtf(x);
  const float h = 0.5f * __builtin_amdgcn_rsqf(x);
  const float r = __builtin_fmaf(-s0, s0, x);
  return __builtin_fmaf(r, h, s0);
}
__device__ __forceinline__ float sqrt_fix(float x) {  // v_sqrt + +-1 ulp residual test
  const float s = __builtin_amdgcn_sqrtf(x);
  const float sd = __uint_as_float(__float_as_uint(s) - 1u);
  const float su = __uint_as_float(__float_as_uint(s) + 1u);
  const float rd = __builtin_fmaf(-sd, s, x);
  const float ru = __builtin_fmaf(-su, s, x);
  float o = rd <= 0.f ? sd : s;
  return ru > 0.f ? su : o;
}

__global__ void k_check(unsigned long long *cnt, unsigned *first) {
  const uint64_t n = 1ull << 32;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const unsigned bits = (unsigned)i;
    const float v = __uint_as_float(bits);
    const float a = fabsf(v);
    if (a >= 0x1p-125f && a <= 0x1p125f) {
      const float ref = 1.0f / v;
      const float got = rcp_nr(v);
      if (__float_as_uint(ref) != __float_as_uint(got)) {
        const unsigned long long k = atomicAdd(&cnt[0], 1ull);
        if (k < 8) first[k] = bits;
      }
    }
    if (v >= 0x1p-96f && v <= 0x1p126f) {
      const float ref = sqrtf(v);
      const float got[4] = {__builtin_amdgcn_sqrtf(v), sqrt_v1(v), sqrt_v3(v), sqrt_fix(v)};
      for (int q = 0; q < 4; ++q)
        if (__float_as_uint(ref) != __float_as_uint(got[q])) {
          const unsigned long long k = atomicAdd(&cnt[1 + q], 1ull);
          if (k < 2) first[8 + 2 * q + k] = bits;
        }
    }
  }
}

int main() {
  unsigned long long *cnt;
  unsigned *first;
  if (hipMalloc(&cnt, 64) != hipSuccess || hipMalloc(&first, 64) != hipSuccess) return 1;
  (void)hipMemset(cnt, 0, 64);
  (void)hipMemset(first, 0, 64);
  hipLaunchKernelGGL(k_check, dim3(16384), dim3(256), 0, 0, cnt, first);
  unsigned long long h[5];
  unsigned f[16];
  if (hipMemcpy(h, cnt, 40, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  if (hipMemcpy(f, first, 64, hipMemcpyDeviceToHost) != hipSuccess) return 1;
  printf("rcp_nr mismatches: %llu\n", h[0]);
  for (int i = 0; i < 8 && i < (int)h[0]; ++i) printf("  d bits 0x%08x\n", f[i]);
  const char *names[4] = {"v_sqrt_f32", "rsq+newton", "v_sqrt+newton", "v_sqrt+ulp-fix"};
  for (int q = 0; q < 4; ++q) {
    printf("%s mismatches: %llu\n", names[q], h[1 + q]);
    for (int i = 0; i < 2 && i < (int)h[1 + q]; ++i) printf("  x bits 0x%08x\n", f[8 + 2 * q + i]);
  }
  return 0;
}
