// kinectfusion.h — header-only drop-in for the reference's kfusion/include/kinectfusion.h.
//
// Recreates kf::kinectfuison_params and kf::kinectfusion (kinectfusion.h:9-73) with the same
// names, member types and call semantics on top of the C-ABI (include/kfx.h), so the
// reference's main.cpp and depth_sensor.{h,cpp} compile unchanged: put this directory ahead of
// kfusion/include on the include path, keep the reference's types.hpp (kf::Intrinsics), drop
// kfusion/src/{kinectfusion,icp_registration,tsdf_volume}.cpp and *.cu from the build and link
// libkfx.so.  Needs OpenCV core (cv::Mat, cv::Affine3f); OpenCV-CUDA is no longer required.
//
// getRenderMap shades the last raycast on the device (kfx_render, image_process.cu:137-221).
#pragma once

#include <opencv2/core.hpp>
#include <opencv2/core/affine.hpp>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <fstream>
#include <iostream>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/kfx.h"
#include "types.hpp"  // the reference's kf::Intrinsics (types.hpp:13-29)

namespace kf {

// kinectfusion.h:9-30
struct kinectfuison_params {
  kinectfuison_params default_params() {
    kfx_params c;
    kfx_default_params(&c);
    kinectfuison_params p;
    p.pyramid_height = c.pyramid_height;
    p.dfilter_dist = c.dfilter_dist;
    p.bfilter_kernel_size = c.bfilter_kernel_size;
    p.bfilter_spatial_sigma = c.bfilter_spatial_sigma;
    p.bfilter_color_sigma = c.bfilter_color_sigma;
    p.icp_dist_threshold = c.icp_dist_threshold;
    p.icp_angle__threshold = c.icp_angle_threshold;
    p.icp_iter_count.assign(c.icp_iter_count, c.icp_iter_count + c.pyramid_height);
    p.volu_range = cv::Vec3f(c.volu_range[0], c.volu_range[1], c.volu_range[2]);
    p.volu_dims = cv::Vec3i(c.volu_dims[0], c.volu_dims[1], c.volu_dims[2]);
    p.volu_trun_dist = c.volu_trun_dist;
    p.volu_pose = cv::Affine3f().translate(cv::Vec3f(c.volu_pose.t[0], c.volu_pose.t[1], c.volu_pose.t[2]));
    p.init_cam_model_dist = 0.f;
    p.min_pose_move = c.min_pose_move;
    p.tsdf_max_weight = c.tsdf_max_weight;
    return p;
  }
  int pyramid_height;
  float dfilter_dist;
  int bfilter_kernel_size;
  float bfilter_spatial_sigma;
  float bfilter_color_sigma;
  float icp_dist_threshold;
  float icp_angle__threshold;
  std::vector<int> icp_iter_count;
  cv::Vec3f volu_range;
  cv::Affine3f volu_pose;
  float volu_trun_dist;
  float init_cam_model_dist;
  cv::Vec3i volu_dims;
  float min_pose_move;
  int tsdf_max_weight;
};

inline kfx_pose to_kfx(const cv::Affine3f &a) {
  kfx_pose p;
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) p.R[3 * i + j] = a.matrix(i, j);
    p.t[i] = a.matrix(i, 3);
  }
  return p;
}

inline cv::Affine3f from_kfx(const kfx_pose &p) {
  cv::Matx44f m = cv::Matx44f::eye();
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) m(i, j) = p.R[3 * i + j];
    m(i, 3) = p.t[i];
  }
  return cv::Affine3f(m);
}

// kinectfusion.h:31-73
class kinectfusion {
 public:
  enum DISPLAY_TYPES { PHONG, NORMAL };

  kinectfusion(const kf::Intrinsics intr, const kf::kinectfuison_params params)
      : intr_(intr), params_(params) {
    kfx_intrinsics ci{intr.width, intr.height, intr.fx, intr.fy, intr.cx, intr.cy};
    kfx_params cp;
    kfx_default_params(&cp);
    cp.pyramid_height = params.pyramid_height;
    cp.dfilter_dist = params.dfilter_dist;
    cp.bfilter_kernel_size = params.bfilter_kernel_size;
    cp.bfilter_spatial_sigma = params.bfilter_spatial_sigma;
    cp.bfilter_color_sigma = params.bfilter_color_sigma;
    cp.icp_dist_threshold = params.icp_dist_threshold;
    cp.icp_angle_threshold = params.icp_angle__threshold;
    for (int l = 0; l < KFX_MAX_LEVELS; ++l)
      cp.icp_iter_count[l] = l < (int)params.icp_iter_count.size() ? params.icp_iter_count[l] : 0;
    for (int i = 0; i < 3; ++i) {
      cp.volu_range[i] = params.volu_range[i];
      cp.volu_dims[i] = params.volu_dims[i];
    }
    cp.volu_trun_dist = params.volu_trun_dist;
    cp.volu_pose = to_kfx(params.volu_pose);
    cp.tsdf_max_weight = params.tsdf_max_weight;
    cp.min_pose_move = params.min_pose_move;
    if (kfx_create(&ci, &cp, 0, &ctx_) != KFX_OK) throw std::runtime_error(kfx_last_error());
    sync_host_state();
  }
  ~kinectfusion() { release(); }

  // kinectfusion.cpp:78-127.  Depth is CV_32FC1 millimetres (depth_sensor.cpp:191) or CV_16UC1.
  // A tracked frame prints the reference's "Frame:N||Time:Xms" line
  // (kinectfusion.cpp:122-123: wall time of the whole call) and keeps it in
  // frame_time; the bootstrap frame and a dropped frame print nothing else.
  void pipeline(cv::Mat cmap_, cv::Mat dmap_) {
    const auto start_time = std::chrono::system_clock::now();
    const int count = frame_count;
    cv::Mat c = cmap_.isContinuous() ? cmap_ : cmap_.clone();
    cv::Mat d = dmap_.isContinuous() ? dmap_ : dmap_.clone();
    int rc;
    if (d.type() == CV_16UC1)
      rc = kfx_pipeline_u16(ctx_, c.ptr<uint8_t>(), d.ptr<uint16_t>());
    else
      rc = kfx_pipeline(ctx_, c.ptr<uint8_t>(), d.ptr<float>());
    if (rc == KFX_TRACKING_LOST) std::cout << "tracking fail!" << std::endl;  // kinectfusion.cpp:99
    else if (rc != KFX_OK) throw std::runtime_error(kfx_last_error());
    sync_host_state();
    if (rc == KFX_OK && count > 1) {
      const std::chrono::duration<double, std::milli> ms = std::chrono::system_clock::now() - start_time;
      frame_time = std::to_string(ms.count());
      std::cout << "Frame:" << count << "||Time:" << ms.count() << "ms" << std::endl;
    }
  }
  void reset() {
    kfx_reset(ctx_);
    sync_host_state();
  }
  // kinectfusion.cpp:33-47: renderPhong / renderNormals (image_process.cu:137-221) on the device
  cv::Mat getRenderMap(DISPLAY_TYPES V = PHONG) {
    cv::Mat out(intr_.height, intr_.width, CV_8UC3);
    if (kfx_render(ctx_, V == NORMAL ? KFX_RENDER_NORMAL : KFX_RENDER_PHONG, out.ptr<uint8_t>()) != KFX_OK)
      throw std::runtime_error(kfx_last_error());
    return out;
  }
  // kinectfusion.cpp:142-147: 1 x N CV_32FC3 zero-crossing cloud (world frame),
  // at most the reference's 10 M buffer (tsdf_volume.cpp:67)
  cv::Mat extracePointcloud() {
    int64_t n = 0;
    if (kfx_extract_points(ctx_, nullptr, 0, &n) != KFX_OK) throw std::runtime_error(kfx_last_error());
    n = std::min<int64_t>(n, KFX_DEFAULT_CLOUD_POINTS);
    points_array_ = cv::Mat(1, (int)n, CV_32FC3);
    if (n > 0 && kfx_extract_points(ctx_, points_array_.ptr<float>(), n, &n) != KFX_OK)
      throw std::runtime_error(kfx_last_error());
    return points_array_;
  }
  // kinectfusion.cpp:148-166: ASCII PLY of the last extracted cloud
  void savePointcloud(std::string path) {
    kfx_write_ply(path.c_str(), points_array_.empty() ? nullptr : points_array_.ptr<float>(),
                  points_array_.cols);
  }
  cv::Affine3f getCurCameraPose() { return pose_record.back(); }
  void release() {
    if (ctx_) kfx_destroy(ctx_);
    ctx_ = nullptr;
  }

 public:
  std::string frame_time;
  int frame_count = 1;
  std::vector<cv::Affine3f> pose_record;

 private:
  // pose_record mirrors the device log: a tracked frame appends one pose (only
  // that pose is read), the bootstrap frame none; a reset (the log shrank)
  // re-reads the whole record.
  void sync_host_state() {
    kfx_get_frame_count(ctx_, &frame_count);
    int n = 0;
    kfx_get_pose_record(ctx_, nullptr, 0, &n);
    if (n == (int)pose_record.size()) return;
    if (n == (int)pose_record.size() + 1) {
      kfx_pose p;
      if (kfx_get_cur_camera_pose(ctx_, &p) != KFX_OK) throw std::runtime_error(kfx_last_error());
      pose_record.push_back(from_kfx(p));
      return;
    }
    std::vector<kfx_pose> ps(n);
    kfx_get_pose_record(ctx_, ps.data(), n, &n);
    pose_record.clear();
    for (const kfx_pose &p : ps) pose_record.push_back(from_kfx(p));
  }

  kfx_ctx *ctx_ = nullptr;
  cv::Mat points_array_;
  Intrinsics intr_;
  kinectfuison_params params_;
};

}  // namespace kf

// kf::file::exportPly (kinectfusion.h:77-83): the reference declares it ("TODO:
// file") but never defines or calls it (main.cpp saves through
// savePointcloud).  Here it writes the same ASCII PLY as savePointcloud
// (kinectfusion.cpp:148-166) from a 1 x N CV_32FC3 cloud, the format
// extracePointcloud returns.
namespace kf {
namespace file {
inline void exportPly(const std::string &filename, cv::Mat pointcloud) {
  cv::Mat p = pointcloud.isContinuous() ? pointcloud : pointcloud.clone();
  const int64_t n = p.empty() ? 0 : (int64_t)p.rows * p.cols;
  if (kfx_write_ply(filename.c_str(), n ? p.ptr<float>() : nullptr, n) != KFX_OK)
    throw std::runtime_error(kfx_last_error());
}
}  // namespace file
}  // namespace kf
