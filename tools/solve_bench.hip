// Latency of the device ICP solve (icp_update: 6x6 LU + Rodrigues + pose
// compose) in one wave, as in k_icp_track's solve phase: the kernel source is
// included so the same inlined function is timed.  Prints cycles per solve.
// build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -fno-fast-math
//        -I slam-kinectfusion_amd/csrc tools/solve_bench.hip -o tools/build/solve_bench
#include "../slam-kinectfusion_amd/csrc/kfx_kernels.hip"

#include <cstdio>
#include <random>

namespace kfx {
namespace {
__global__ void k_solve_bench(const long long *sums_in, float *out, int iters, unsigned long long *cyc) {
  __shared__ long long sums[27];
  __shared__ double sumd[27];
  if (threadIdx.x < 27) sums[threadIdx.x] = sums_in[threadIdx.x];
  __syncthreads();
  DevPose p = pose_identity();
  double x[6];
  float acc = 0.f;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    if (threadIdx.x == 0) sums[0] += (long long)(acc != 0.f);  // keeps the solve inside the loop
    __syncthreads();
    if (threadIdx.x < 27) sumd[threadIdx.x] = icp_sum_value(sums[threadIdx.x]);  // as k_icp_track
    __syncthreads();
    DevPose q = p;
    const int f = icp_update(sumd, q, x);
    acc += q.t[0] + q.R[1] + q.R[5] + (float)f;  // rotation too: the Rodrigues update stays timed
    p.t[0] = acc * 1e-30f;  // carry a dependency into the next solve
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    cyc[0] = t1 - t0;
    out[0] = acc;
  }
}
}  // namespace
}  // namespace kfx

int main() {
  // a well-conditioned system: sums of products of 2000 random rows, 2^32 fixed point
  std::mt19937 rng(1);
  std::normal_distribution<double> nd(0.0, 0.3);
  double s[27] = {};
  for (int r = 0; r < 2000; ++r) {
    double row[7];
    for (double &v : row) v = nd(rng);
    row[6] *= 0.01;
    int k = 0;
    for (int a = 0; a < 6; ++a)
      for (int b = a; b < 7; ++b) s[k++] += row[a] * row[b];
  }
  long long h[27];
  for (int k = 0; k < 27; ++k) h[k] = (long long)(s[k] * 4294967296.0);
  long long *d;
  float *o;
  unsigned long long *c;
  (void)hipMalloc(&d, sizeof(h));
  (void)hipMalloc(&o, 4);
  (void)hipMalloc(&c, 8);
  (void)hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
  const int iters = 2000;
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(kfx::k_solve_bench, dim3(1), dim3(64), 0, 0, d, o, iters, c);
    unsigned long long cy = 0;
    (void)hipMemcpy(&cy, c, 8, hipMemcpyDeviceToHost);
    std::printf("solve: %.1f cycles (s_memtime) per icp_update\n", (double)cy / iters);
  }
  return 0;
}
