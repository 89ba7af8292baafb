// Compile-check stand-in for the reference's kfusion/include/types.hpp:
// kf::Intrinsics with the same fields (types.hpp:13-29).
#pragma once
namespace kf {
struct Intrinsics {
  int width, height;
  float fx, fy, cx, cy;
  float c = 1;
};
}  // namespace kf
