// ICP coarse levels in ONE workgroup (round-3 verdict item 3), measured: the
// shipped lane phase (icp_load_cur / icp_lane), block reduction and solve
// (icp_update) of csrc/kfx_kernels.hip, compiled here for a 1024-thread block,
// iterate over a C2 level (level 2: 160x120 -> 15 360 pixels of the A2 grid;
// level 1: 320x240 -> 71 680) with __syncthreads only: no device-scope atomics,
// no grid barrier, no shard reads.  Per-iteration wall clock (100 MHz) of
// block 0, to set beside the grid-wide iteration of tools/icp_trace.py.
// Synthetic well-conditioned surface (z = 2 + ripples), previous maps = current
// maps shifted by a small rigid motion, so every pixel associates.
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off \
//          -I slam-kinectfusion_amd/csrc -I include tools/icp_l2one.hip -o tools/build/icp_l2one
// (1024 threads: 128 registers per lane, the shipped lane phase + reduce spill 232 B)
#ifndef KFX_ICP_THREADS
#define KFX_ICP_THREADS 1024  // (-DKFX_ICP_THREADS=512: 256 registers per lane instead of 128)
#endif
#define KFX_ICP_PIX 2
#include "kfx_kernels.hip"

#include <cstdio>
#include <vector>

namespace kfx {
namespace {
__global__ __launch_bounds__(kIcpThreads, 1) void k_level_one_block(LevelGeom g, int xe, int npix, int iters,
                                                            const float *cv, const float *cn, const float *pv,
                                                            const float *pn, float d2, float s2,
                                                            unsigned long long *clk, double *xo) {
  __shared__ IcpRed red;
  __shared__ double sumd[27];
  DevPose P = pose_identity();
  for (int it = 0; it < iters; ++it) {
    const unsigned long long t0 = wall_clock64();
    double acc[27];
#pragma unroll
    for (int k = 0; k < 27; ++k) acc[k] = 0.0;
    for (int p0 = 0; p0 < npix; p0 += kIcpPix * kIcpThreads) {
      const int ppl = min(kIcpPix, (npix - p0 + kIcpThreads - 1) / kIcpThreads);
      f3 n0[kIcpPix], v0[kIcpPix];
      bool ok[kIcpPix];
      icp_load_cur(g, xe, npix, 0, ppl, cv, cn, n0, v0, ok, p0);
      icp_lane(g, P, n0, v0, ok, ppl, pv, pn, d2, s2, acc, false);
    }
    const unsigned long long t1 = wall_clock64();
    const long long s = icp_block_reduce(red, acc);
    if (threadIdx.x < 27) sumd[threadIdx.x] = icp_sum_value(s);
    __syncthreads();
    const unsigned long long t2 = wall_clock64();
    DevPose p = P;
    double x[6];
    const int f = icp_update(sumd, p, x);
    if (!f) P = p;
    if (threadIdx.x < 6 && it == iters - 1) xo[threadIdx.x] = x[threadIdx.x];
    __syncthreads();  // sumd is rewritten next iteration
    const unsigned long long t3 = wall_clock64();
    if (threadIdx.x == 0) {
      clk[4 * it + 0] = t1 - t0;  // lane phase
      clk[4 * it + 1] = t2 - t1;  // block reduce
      clk[4 * it + 2] = t3 - t2;  // solve
      clk[4 * it + 3] = t3 - t0;
    }
  }
}
}  // namespace
}  // namespace kfx

int main() {
  using namespace kfx;
  for (int level = 2; level >= 1; --level) {
    const int W = 640 >> level, H = 480 >> level;
    const float f = 525.f / (float)(1 << level), cx = (W - 1) * 0.5f, cy = (H - 1) * 0.5f;
    std::vector<float> v(3 * W * H), n(3 * W * H), v2(3 * W * H), n2(3 * W * H);
    for (int y = 0; y < H; ++y)
      for (int x = 0; x < W; ++x) {
        const float X = (x - cx) / f, Y = (y - cy) / f;
        const float z = 2.f + 0.15f * sinf(7.f * X) * cosf(5.f * Y) + 0.3f * X * X;
        const float dzdx = (0.15f * 7.f * cosf(7.f * X) * cosf(5.f * Y) + 0.6f * X) / f;
        const float dzdy = (-0.15f * 5.f * sinf(7.f * X) * sinf(5.f * Y)) / f;
        const size_t i = 3 * ((size_t)y * W + x);
        v[i] = X * z, v[i + 1] = Y * z, v[i + 2] = z;
        float nx = dzdx, ny = dzdy, nz = -1.f / f;
        const float l = sqrtf(nx * nx + ny * ny + nz * nz);
        n[i] = nx / l, n[i + 1] = ny / l, n[i + 2] = nz / l;
        // previous maps: the same surface moved by 3 mm along x
        v2[i] = v[i] + 0.003f, v2[i + 1] = v[i + 1], v2[i + 2] = v[i + 2];
        n2[i] = n[i], n2[i + 1] = n[i + 1], n2[i + 2] = n[i + 2];
      }
    float *d[4];
    const std::vector<float> *src[4] = {&v, &n, &v2, &n2};
    for (int k = 0; k < 4; ++k) {
      (void)hipMalloc(&d[k], sizeof(float) * v.size());
      (void)hipMemcpy(d[k], src[k]->data(), sizeof(float) * v.size(), hipMemcpyHostToDevice);
    }
    LevelGeom g{W, H, f, f, cx, cy};
    int xe;
    const int npix = icp_npix(g, &xe);
    const int iters = 10;
    unsigned long long *clk;
    double *xo;
    (void)hipMalloc(&clk, sizeof(unsigned long long) * 4 * iters);
    (void)hipMalloc(&xo, sizeof(double) * 6);
    const float d2 = 0.1f * 0.1f, s2 = 0.5f * 0.5f;
    for (int rep = 0; rep < 3; ++rep)
      hipLaunchKernelGGL(k_level_one_block, dim3(1), dim3(kIcpThreads), 0, 0, g, xe, npix, iters, d[0], d[1], d[2], d[3], d2,
                         s2, clk, xo);
    if (hipDeviceSynchronize() != hipSuccess) {
      std::printf("kernel failed\n");
      return 1;
    }
    std::vector<unsigned long long> c(4 * iters);
    double x[6];
    (void)hipMemcpy(c.data(), clk, sizeof(unsigned long long) * c.size(), hipMemcpyDeviceToHost);
    (void)hipMemcpy(x, xo, sizeof(x), hipMemcpyDeviceToHost);
    double tot = 0, lane = 0, red = 0, sol = 0;
    for (int i = 0; i < iters; ++i) {
      lane += c[4 * i] / 100.0, red += c[4 * i + 1] / 100.0, sol += c[4 * i + 2] / 100.0, tot += c[4 * i + 3] / 100.0;
    }
    std::printf("level %d: %d pixels in one %d-thread workgroup, %d iterations: per iteration %.2f us "
                "(lane %.2f, block reduce %.2f, solve %.2f); last x = %.3g %.3g %.3g %.3g %.3g %.3g\n",
                level, npix, kIcpThreads, iters, tot / iters, lane / iters, red / iters, sol / iters, x[0], x[1], x[2], x[3], x[4],
                x[5]);
    for (int k = 0; k < 4; ++k) (void)hipFree(d[k]);
    (void)hipFree(clk);
    (void)hipFree(xo);
  }
  return 0;
}
