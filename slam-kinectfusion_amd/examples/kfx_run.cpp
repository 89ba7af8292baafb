// kfx_run — the reference's main.cpp loop (main.cpp:63-98) on a dataset
// directory, over the C-ABI only (no OpenCV, no viz): depth_sensor::open /
// getFrame → kinectfusion::pipeline per frame → poses.txt (and optionally the
// point cloud PLY, main.cpp:43-44).
//   usage: kfx_run <dataset dir> [poses.txt] [cloud.ply]
#include <chrono>
#include <cstdio>
#include <vector>

#include "../../include/kfx.h"

int main(int argc, char **argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s <dataset dir> [poses.txt] [cloud.ply]\n", argv[0]);
    return 2;
  }
  const char *poses = argc > 2 ? argv[2] : "poses.txt";
  kfx_dataset *ds = nullptr;
  if (kfx_dataset_open(argv[1], &ds) != KFX_OK) {
    std::fprintf(stderr, "error: %s\n", kfx_last_error());  // "error: no camera!"
    return 1;
  }
  kfx_intrinsics intr;
  int n = 0, has_intr = 0;
  kfx_dataset_info(ds, &intr, &n, &has_intr);
  if (!has_intr) {
    std::fprintf(stderr, "error: %s/intr.txt missing or malformed\n", argv[1]);
    return 1;
  }
  kfx_params p;
  kfx_default_params(&p);  // kinectfuison_params::default_params (kinectfusion.cpp:167-190)
  kfx_ctx *ctx = nullptr;
  if (kfx_create(&intr, &p, 0, &ctx) != KFX_OK) {
    std::fprintf(stderr, "error: %s\n", kfx_last_error());
    return 1;
  }
  std::printf("KinectFusion: start (%d frames, %dx%d)\n", n, intr.width, intr.height);
  std::vector<uint8_t> bgr((size_t)intr.width * intr.height * 3);
  std::vector<float> depth((size_t)intr.width * intr.height);
  double gpu_s = 0;
  for (int k = 0; k < n; ++k) {
    if (kfx_dataset_read(ds, k, bgr.data(), depth.data()) != KFX_OK) {
      std::printf("no image! (%s)\n", kfx_last_error());
      break;
    }
    const auto t0 = std::chrono::steady_clock::now();
    const int r = kfx_pipeline(ctx, bgr.data(), depth.data());
    gpu_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (r == KFX_TRACKING_LOST) {
      std::printf("tracking fail!\n");  // kinectfusion.cpp:99
    } else if (r != KFX_OK) {
      std::fprintf(stderr, "error: %s\n", kfx_last_error());
      return 1;
    }
  }
  int frames = 0;
  kfx_get_frame_count(ctx, &frames);
  if (kfx_write_poses_txt(ctx, poses) != KFX_OK) {
    std::fprintf(stderr, "error: %s\n", kfx_last_error());
    return 1;
  }
  if (argc > 3 && kfx_save_pointcloud(ctx, argv[3], 0) != KFX_OK) {
    std::fprintf(stderr, "error: %s\n", kfx_last_error());
    return 1;
  }
  std::printf("end! %d frames, frame_count %d, %.3f ms/frame in kfx_pipeline (host frames, PCIe incl.)\n", n,
              frames, n ? 1e3 * gpu_s / n : 0.0);
  kfx_destroy(ctx);
  kfx_dataset_close(ds);
  return 0;
}
