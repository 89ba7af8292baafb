// Compile-check stand-in for cv::Affine3f (see ../core.hpp).
#pragma once
#include "../core.hpp"
namespace cv {
struct Affine3f {
  Matx44f matrix = Matx44f::eye();
  Affine3f() = default;
  explicit Affine3f(const Matx44f &m) : matrix(m) {}
  Affine3f translate(const Vec3f &t) const {
    Affine3f r = *this;
    for (int i = 0; i < 3; ++i) r.matrix(i, 3) += t[i];
    return r;
  }
};
}  // namespace cv
