// Compile-check stand-in for the few OpenCV core types the adapter
// (slam-kinectfusion_amd/adapter/kinectfusion.h) uses.  OpenCV is not in this
// image; this stub only lets tests/test_abi.py compile and link the adapter
// and a main.cpp-like driver against libkfx.so.  Not a product component.
#pragma once
#include <cstdint>
#include <memory>
#include <vector>

#define CV_8UC3 16
#define CV_16UC1 2
#define CV_32FC1 5
#define CV_32FC3 21

namespace cv {
template <typename T, int N>
struct Vec {
  T v[N]{};
  Vec() = default;
  Vec(T a, T b, T c) : v{a, b, c} {}
  T &operator[](int i) { return v[i]; }
  const T &operator[](int i) const { return v[i]; }
};
using Vec3f = Vec<float, 3>;
using Vec3i = Vec<int, 3>;
template <typename T, int M, int N>
struct Matx {
  T val[M * N]{};
  T &operator()(int i, int j) { return val[i * N + j]; }
  const T &operator()(int i, int j) const { return val[i * N + j]; }
  static Matx eye() {
    Matx m;
    for (int i = 0; i < (M < N ? M : N); ++i) m(i, i) = 1;
    return m;
  }
};
using Matx44f = Matx<float, 4, 4>;
class Mat {
 public:
  Mat() = default;
  Mat(int rows, int cols, int type)
      : rows(rows), cols(cols), type_(type), buf_(std::make_shared<std::vector<uint8_t>>((size_t)rows * cols * 16)) {}
  bool isContinuous() const { return true; }
  Mat clone() const { return *this; }
  int type() const { return type_; }
  bool empty() const { return !buf_ || buf_->empty(); }
  template <typename T>
  T *ptr() { return reinterpret_cast<T *>(buf_->data()); }
  int rows = 0, cols = 0;

 private:
  int type_ = 0;
  std::shared_ptr<std::vector<uint8_t>> buf_;
};
}  // namespace cv
