// main.cpp's use of kf::kinectfusion (main.cpp:54-105), against the adapter:
// construction from default_params, pipeline, render, extraction + PLY
// (savePointcloud and kf::file::exportPly),
// reset, pose_record, release.  Compiled and linked by tests/test_abi.py.
#include <fstream>
#include <iostream>

#include "kinectfusion.h"

int main(int argc, char **argv) {
  kf::Intrinsics intr{640, 480, 525.f, 525.f, 319.5f, 239.5f};
  kf::kinectfuison_params params;
  params = params.default_params();
  try {
    kf::kinectfusion kinfu(intr, params);
    cv::Mat color(480, 640, CV_8UC3), depth(480, 640, CV_32FC1);
    kinfu.pipeline(color, depth);
    cv::Mat img = kinfu.getRenderMap(kf::kinectfusion::PHONG);
    if (kinfu.frame_count % 5 == 0) kinfu.extracePointcloud();
    kinfu.savePointcloud(argc > 1 ? argv[1] : "/dev/null");
    kf::file::exportPly(argc > 2 ? argv[2] : "/dev/null", kinfu.extracePointcloud());
    std::cout << kinfu.getCurCameraPose().matrix(0, 0) << " " << kinfu.pose_record.size() << img.rows << std::endl;
    kinfu.reset();
    kinfu.release();
  } catch (const std::exception &e) {
    std::cerr << "kinectfusion: " << e.what() << std::endl;
    return 2;
  }
  return 0;
}
