// PMC calibration: known-byte streams in the access widths the kfx kernels use
// (2-byte int16 tsdf/weight, 4-byte u32 rgb, 12-byte f32x3 maps), so that
// FETCH_SIZE / WRITE_SIZE can be converted to HBM bytes for those widths
// (MI355X_MICROARCH.md: only 16-B/lane streams are calibrated there).
// Each kernel touches 512 MiB (> the 256 MiB Infinity Cache) once.
// build: hipcc -O3 --offload-arch=gfx950 tools/pmc_calib.hip -o tools/build/pmc_calib
// run:   rocprofv3 --pmc FETCH_SIZE --output-format csv -d <dir> -- tools/build/pmc_calib
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

template <typename T>
__global__ void k_read(const T *__restrict__ a, size_t n, unsigned *out) {
  unsigned acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    acc += (unsigned)a[i];
  if (acc == 0x9e3779b9u) out[0] = acc;  // never true for zeroed input; keeps the loads
}

template <typename T>
__global__ void k_write(T *__restrict__ a, size_t n, T v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    a[i] = v;
}

__global__ void k_read_f3(const float *__restrict__ a, size_t n, unsigned *out) {
  float acc = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    acc += a[3 * i] + a[3 * i + 1] + a[3 * i + 2];
  if (acc == 1234.5f) out[0] = 1;
}

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                   \
      return 1;                                                                \
    }                                                                          \
  } while (0)

int main() {
  const size_t bytes = 512ull << 20;
  void *buf;
  unsigned *out;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&out, 4));
  CK(hipMemset(buf, 0, bytes));
  const dim3 grid(8192), blk(256);
  // each kernel twice: the first pass after a different kernel, the second a repeat
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(k_read<uint16_t>, grid, blk, 0, 0, (const uint16_t *)buf, bytes / 2, out);
    hipLaunchKernelGGL(k_read<uint32_t>, grid, blk, 0, 0, (const uint32_t *)buf, bytes / 4, out);
    hipLaunchKernelGGL(k_read_f3, grid, blk, 0, 0, (const float *)buf, bytes / 12, out);
    hipLaunchKernelGGL(k_write<uint16_t>, grid, blk, 0, 0, (uint16_t *)buf, bytes / 2, (uint16_t)0);
    hipLaunchKernelGGL(k_write<uint32_t>, grid, blk, 0, 0, (uint32_t *)buf, bytes / 4, 0u);
  }
  CK(hipDeviceSynchronize());
  printf("calibration kernels done: %zu bytes each\n", bytes);
  CK(hipFree(buf));
  CK(hipFree(out));
  return 0;
}
