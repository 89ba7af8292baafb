// kfx_oracle.cpp — TEST INFRASTRUCTURE ONLY (see kfx_oracle.h for the contract).
//
// CPU restatement of the reference hot path.  Each function cites the reference
// file:line it follows.  Float expressions are written in the reference's
// evaluation order; the build uses -ffp-contract=off so nothing is fused.
// "D" = a defined deviation from the CUDA original.
#include "kfx_oracle.h"

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

namespace {

struct V3 {
  float x, y, z;
};

inline V3 add(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 scl(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline V3 mulc(V3 a, V3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
// device_types.hpp:234-236 dot: x*x + y*y + z*z, left to right
inline float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
// device_types.hpp:256-259
inline V3 cross(V3 a, V3 b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
// device_types.hpp:246-250 normalize / device_utils.cuh:64-68 __m_normalize (D: IEEE div)
inline V3 normalized(V3 v) {
  float t = std::sqrt(dot(v, v));
  return {v.x / t, v.y / t, v.z / t};
}
// PoseR * float3 (device_types.hpp:134-139): R(i,0)x + R(i,1)y + R(i,2)z
inline V3 rmul(const float *R, V3 v) {
  return {R[0] * v.x + R[1] * v.y + R[2] * v.z, R[3] * v.x + R[4] * v.y + R[5] * v.z,
          R[6] * v.x + R[7] * v.y + R[8] * v.z};
}
inline V3 ld3(const float *p, int64_t i) { return {p[3 * i], p[3 * i + 1], p[3 * i + 2]}; }
inline void st3(float *p, int64_t i, V3 v) {
  p[3 * i] = v.x;
  p[3 * i + 1] = v.y;
  p[3 * i + 2] = v.z;
}

// __float2int_rn / __float2int_rd: the result only feeds bounds checks, so any
// value outside int range maps to INT_MIN (rejected by every check).
inline int f2i_rn(float v) {
  float r = std::rint(v);
  return (r > -2.0e9f && r < 2.0e9f) ? (int)r : INT_MIN;
}
inline int f2i_rd(float v) {
  float r = std::floor(v);
  return (r > -2.0e9f && r < 2.0e9f) ? (int)r : INT_MIN;
}

inline int reflect101(int i, int n) {
  if (i < 0) i = -i;
  if (i >= n) i = 2 * n - 2 - i;
  return i;
}

const float kDivShortMax = 0.0000305185f;  // device_utils.cuh:6
const int kShortMax = 32767;               // device_utils.cuh:7
const int kMaxWeight = 64;                 // device_utils.cuh:5
const float kFix = 4294967296.0f;          // 2^32 fixed-point scale (D)

}  // namespace

extern "C" {

// Deterministic exp (D): Cody-Waite reduction + degree-7 Taylor in plain float
// ops.  The CUDA original calls ::exp (OpenCV bilateral_filter.cu); this one is
// reproducible bit-for-bit on CPU and GPU.  Returns 0 below -86 (no denormals).
float kfo_expf(float x) {
  if (!(x >= -86.0f)) return 0.0f;
  const float kf = std::rint(x * 1.44269502f);
  const float r = (x - kf * 0.693145751953125f) - kf * 1.42860677e-6f;
  float p = 1.98412698e-4f;
  p = p * r + 1.38888889e-3f;
  p = p * r + 8.33333377e-3f;
  p = p * r + 4.16666679e-2f;
  p = p * r + 1.66666672e-1f;
  p = p * r + 0.5f;
  p = p * r + 1.0f;
  p = p * r + 1.0f;
  const int k = (int)kf;
  uint32_t bits = (uint32_t)(k + 127) << 23;
  float s;
  std::memcpy(&s, &bits, 4);
  return p * s;
}

// OpenCV cudawarping pyr_down.cu: vertical 5-tap at src row 2y, then horizontal
// 5-tap at src column 2x; weights .0625 .25 .375 .25 .0625, REFLECT_101.
void kfo_pyr_down(const float *src, int w, int h, float *dst) {
  const int dw = (w + 1) / 2, dh = (h + 1) / 2;
  const float k[5] = {0.0625f, 0.25f, 0.375f, 0.25f, 0.0625f};
  std::vector<float> col(w);
  for (int y = 0; y < dh; ++y) {
    const int sy = 2 * y;
    for (int x = 0; x < w; ++x) {
      float sum = k[0] * src[(int64_t)reflect101(sy - 2, h) * w + x];
      sum = sum + k[1] * src[(int64_t)reflect101(sy - 1, h) * w + x];
      sum = sum + k[2] * src[(int64_t)reflect101(sy, h) * w + x];
      sum = sum + k[3] * src[(int64_t)reflect101(sy + 1, h) * w + x];
      sum = sum + k[4] * src[(int64_t)reflect101(sy + 2, h) * w + x];
      col[x] = sum;
    }
    for (int x = 0; x < dw; ++x) {
      const int sx = 2 * x;
      float sum = k[0] * col[reflect101(sx - 2, w)];
      sum = sum + k[1] * col[reflect101(sx - 1, w)];
      sum = sum + k[2] * col[reflect101(sx, w)];
      sum = sum + k[3] * col[reflect101(sx + 1, w)];
      sum = sum + k[4] * col[reflect101(sx + 2, w)];
      dst[(int64_t)y * dw + x] = sum;
    }
  }
}

// OpenCV cudaimgproc bilateral_filter.cu (call site kinectfusion.cpp:60-64):
// taps (cx,cy) in [x-r, x-r+ksz) x [y-r, y-r+ksz), row-major, skipping
// space2 > r*r; w = exp(space2*(-0.5/ss^2) + |v-c|^2*(-0.5/sc^2)).
// A1 (D): out of place.
void kfo_bilateral(const float *src, int w, int h, int ksz, float sigma_color,
                   float sigma_spatial, float *dst) {
  const float s_half = -0.5f / (sigma_spatial * sigma_spatial);
  const float c_half = -0.5f / (sigma_color * sigma_color);
  const int r = ksz / 2;
  const float r2 = (float)(r * r);
  for (int y = 0; y < h; ++y) {
    for (int x = 0; x < w; ++x) {
      const float center = src[(int64_t)y * w + x];
      float sum1 = 0.f, sum2 = 0.f;
      for (int cy = y - r; cy < y - r + ksz; ++cy) {
        for (int cx = x - r; cx < x - r + ksz; ++cx) {
          const float space2 = (float)((x - cx) * (x - cx) + (y - cy) * (y - cy));
          if (space2 > r2) continue;
          const float v = src[(int64_t)reflect101(cy, h) * w + reflect101(cx, w)];
          const float d = std::fabs(v - center);
          const float wgt = kfo_expf(space2 * s_half + (d * d) * c_half);
          sum1 = sum1 + wgt * v;
          sum2 = sum2 + wgt;
        }
      }
      dst[(int64_t)y * w + x] = sum1 / sum2;
    }
  }
}

// image_process.cu:8-17
void kfo_depth_truncation(float *d, int n, float max_dist) {
  for (int i = 0; i < n; ++i) {
    d[i] *= 0.001f;
    if (d[i] > max_dist) d[i] = 0.f;
  }
}

// image_process.cu:29-43 + Intrs::reproj (device_utils.cuh:22-27), D: IEEE div.
void kfo_vertex_map(const float *d, int w, int h, float fx, float fy, float cx,
                    float cy, float *vmap) {
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      const int64_t i = (int64_t)y * w + x;
      const float z = d[i];
      if (std::isnan(z)) {
        st3(vmap, i, {0.f, 0.f, 0.f});
      } else {
        st3(vmap, i, {(z * ((float)x - cx)) / fx, (z * ((float)y - cy)) / fy, z});
      }
    }
}

// image_process.cu:57-84.  Interior only; the 1-px border is 0 (Frame::reset).
void kfo_normal_map(const float *vmap, int w, int h, float *nmap) {
  for (int64_t i = 0; i < (int64_t)w * h; ++i) st3(nmap, i, {0.f, 0.f, 0.f});
  for (int y = 1; y < h - 1; ++y)
    for (int x = 1; x < w - 1; ++x) {
      const V3 l = ld3(vmap, (int64_t)y * w + x - 1);
      const V3 r = ld3(vmap, (int64_t)y * w + x + 1);
      const V3 u = ld3(vmap, (int64_t)(y - 1) * w + x);
      const V3 dn = ld3(vmap, (int64_t)(y + 1) * w + x);
      V3 n;
      if (l.z == 0 || r.z == 0 || u.z == 0 || dn.z == 0) {
        n = {0.f, 0.f, 0.f};
      } else {
        n = cross(sub(l, r), sub(u, dn));
        if (n.z > 0) n = scl(n, -1.f);
      }
      st3(nmap, (int64_t)y * w + x, normalized(n));  // 0/0 = NaN when invalid (A8)
    }
}

// image_process.cu:95-125 (A7: zeros averaged, normals not renormalised).
void kfo_resize_points_normals(const float *vbig, const float *nbig, int ws, int hs,
                               float *vsmall, float *nsmall) {
  const int wb = ws * 2;
  for (int y = 0; y < hs; ++y)
    for (int x = 0; x < ws; ++x) {
      const int64_t o = (int64_t)y * ws + x;
      st3(vsmall, o, {0.f, 0.f, 0.f});
      st3(nsmall, o, {0.f, 0.f, 0.f});
      const int64_t i00 = (int64_t)(2 * y) * wb + 2 * x, i01 = i00 + 1, i10 = i00 + wb,
                    i11 = i10 + 1;
      const V3 d00 = ld3(vbig, i00), d01 = ld3(vbig, i01), d10 = ld3(vbig, i10),
               d11 = ld3(vbig, i11);
      if (!std::isnan(d00.x * d01.x * d10.x * d11.x)) {
        st3(vsmall, o, scl(add(add(add(d00, d01), d10), d11), 0.25f));
        const V3 n00 = ld3(nbig, i00), n01 = ld3(nbig, i01), n10 = ld3(nbig, i10),
                 n11 = ld3(nbig, i11);
        st3(nsmall, o, scl(add(add(add(n00, n01), n10), n11), 0.25f));
      }
    }
}

// types.hpp:18-28
void kfo_level_intrinsics(const kfx_intrinsics *in, int level, kfx_intrinsics *out) {
  if (level == 0) {
    *out = *in;
    return;
  }
  const float s = std::pow(0.5f, (float)level);
  out->width = in->width >> level;
  out->height = in->height >> level;
  out->fx = in->fx * s;
  out->fy = in->fy * s;
  out->cx = (in->cx + 0.5f) * s - 0.5f;
  out->cy = (in->cy + 0.5f) * s - 0.5f;
}

// kinectfusion.cpp:48-76 (pyrDown on raw mm depth first, A12).
void kfo_preprocess(const float *depth_mm, int w, int h, int levels,
                    const kfx_intrinsics *intr, const kfx_params *p, float **dmap,
                    float **vmap, float **nmap) {
  std::vector<std::vector<float>> raw(levels);
  raw[0].assign(depth_mm, depth_mm + (int64_t)w * h);
  int lw = w, lh = h;
  for (int l = 1; l < levels; ++l) {
    raw[l].resize((int64_t)((lw + 1) / 2) * ((lh + 1) / 2));
    kfo_pyr_down(raw[l - 1].data(), lw, lh, raw[l].data());
    lw = (lw + 1) / 2;
    lh = (lh + 1) / 2;
  }
  for (int l = 0; l < levels; ++l) {
    kfx_intrinsics li;
    kfo_level_intrinsics(intr, l, &li);
    kfo_bilateral(raw[l].data(), li.width, li.height, p->bfilter_kernel_size,
                  p->bfilter_color_sigma, p->bfilter_spatial_sigma, dmap[l]);
    kfo_depth_truncation(dmap[l], li.width * li.height, p->dfilter_dist);
    kfo_vertex_map(dmap[l], li.width, li.height, li.fx, li.fy, li.cx, li.cy, vmap[l]);
    kfo_normal_map(vmap[l], li.width, li.height, nmap[l]);
  }
}

// ICP::findCoresp (rigid_icp.cu:46-80) + kernel_rigidICP rows/products
// (rigid_icp.cu:81-113).  Grid floor-division (A2) limits the region to
// 32*floor(w/32) x 32*floor(h/32).  D: the 27 sums are exact int64 fixed point
// (product * 2^32 rounded to nearest even) instead of fp64 block trees + f32.
void kfo_icp_accumulate(const float *cur_v, const float *cur_n, const float *pre_v,
                        const float *pre_n, int w, int h, const kfx_intrinsics *li,
                        const kfx_pose *pose, float dist_thres, float angle_thres,
                        int64_t sums[27]) {
  for (int k = 0; k < 27; ++k) sums[k] = 0;
  const int xe = (w / 32) * 32, ye = (h / 32) * 32;
  const V3 t = {pose->t[0], pose->t[1], pose->t[2]};
  for (int y = 0; y < ye; ++y)
    for (int x = 0; x < xe; ++x) {
      const int64_t i = (int64_t)y * w + x;
      const V3 ncur0 = ld3(cur_n, i);
      if (std::isnan(ncur0.x)) continue;
      const V3 vcur = add(rmul(pose->R, ld3(cur_v, i)), t);
      const int px = f2i_rn((vcur.x / vcur.z) * li->fx + li->cx);
      const int py = f2i_rn((vcur.y / vcur.z) * li->fy + li->cy);
      if (!(vcur.z > 0 && px >= 0 && py >= 0 && px < w && py < h)) continue;
      const int64_t j = (int64_t)py * w + px;
      const V3 vpre = ld3(pre_v, j);
      const V3 dd = sub(vcur, vpre);
      const float dist = std::sqrt(dot(dd, dd));
      if (!(dist <= dist_thres)) continue;
      const V3 ncur = rmul(pose->R, ncur0);
      const V3 npre = ld3(pre_n, j);
      const V3 sa = cross(ncur, npre);
      const float sine = std::sqrt(dot(sa, sa));
      if (!(sine <= angle_thres)) continue;
      const V3 c = cross(vcur, npre);
      const float row[7] = {c.x, c.y, c.z, npre.x, npre.y, npre.z,
                            dot(npre, sub(vpre, vcur))};
      int s = 0;
      for (int a = 0; a < 6; ++a)
        for (int b = a; b < 7; ++b) {
          const float prod = row[a] * row[b];
          sums[s++] += (int64_t)std::rint(prod * kFix);
        }
    }
}

// Affine3f product a*b (OpenCV affine.hpp concatenate/rotate/translate):
// R = Ra*Rb (k ascending from 0), t = Ra.row(j).dot(tb) + ta.
void kfo_pose_mul(const kfx_pose *a, const kfx_pose *b, kfx_pose *out) {
  kfx_pose r;
  for (int j = 0; j < 3; ++j) {
    for (int i = 0; i < 3; ++i) {
      float v = 0.f;
      for (int k = 0; k < 3; ++k) v += a->R[3 * j + k] * b->R[3 * k + i];
      r.R[3 * j + i] = v;
    }
    float d = 0.f;
    for (int k = 0; k < 3; ++k) d += a->R[3 * j + k] * b->t[k];
    r.t[j] = d + a->t[j];
  }
  *out = r;
}

// Affine3f::inv (DECOMP_SVD on the 4x4 in OpenCV).  D: analytic rigid inverse
// (R^T, -(R^T t)), dot sums from 0 in ascending k.
void kfo_pose_inv(const kfx_pose *a, kfx_pose *out) {
  kfx_pose r;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) r.R[3 * i + j] = a->R[3 * j + i];
  for (int j = 0; j < 3; ++j) {
    float d = 0.f;
    for (int k = 0; k < 3; ++k) d += a->R[3 * k + j] * a->t[k];
    r.t[j] = -d;
  }
  *out = r;
}

void kfo_pose_identity(kfx_pose *out) {
  std::memset(out, 0, sizeof(*out));
  out->R[0] = out->R[4] = out->R[8] = 1.f;
}

// D: cos / sin of the Rodrigues angle (cv::Affine3f(rvec, t) uses std::cos /
// std::sin).  For theta < 0.5 (every ICP increment in practice) their Taylor
// polynomials in theta^2, Horner form with fused multiply-adds (truncation
// < 1e-19 relative; within an ulp or two of the libm values, then rounded to
// float): the same operations as the kernel's det_sincos, so GPU and oracle
// agree bit for bit; larger angles use libm on both sides.
void kfo_sincos(double theta, double *s, double *c) {
  if (!(theta < 0.5)) {
    *s = std::sin(theta);
    *c = std::cos(theta);
    return;
  }
  const double x2 = theta * theta;
  double ps = -1.0 / 1307674368000.0;
  ps = std::fma(ps, x2, 1.0 / 6227020800.0);
  ps = std::fma(ps, x2, -1.0 / 39916800.0);
  ps = std::fma(ps, x2, 1.0 / 362880.0);
  ps = std::fma(ps, x2, -1.0 / 5040.0);
  ps = std::fma(ps, x2, 1.0 / 120.0);
  ps = std::fma(ps, x2, -1.0 / 6.0);
  *s = std::fma(theta, x2 * ps, theta);
  double pc = -1.0 / 87178291200.0;
  pc = std::fma(pc, x2, 1.0 / 479001600.0);
  pc = std::fma(pc, x2, -1.0 / 3628800.0);
  pc = std::fma(pc, x2, 1.0 / 40320.0);
  pc = std::fma(pc, x2, -1.0 / 720.0);
  pc = std::fma(pc, x2, 1.0 / 24.0);
  pc = std::fma(pc, x2, -0.5);
  *c = std::fma(x2, pc, 1.0);
}

// 3x3 inverse by cofactors (icp_update's block solve): returns det(m); out =
// adj(m) / det (the cofactors as one multiply and one fused multiply-subtract)
static double kfo_inv3(const double m[3][3], double out[3][3]) {
  double c[3][3];
  c[0][0] = std::fma(m[1][1], m[2][2], -(m[1][2] * m[2][1]));
  c[0][1] = std::fma(m[1][2], m[2][0], -(m[1][0] * m[2][2]));
  c[0][2] = std::fma(m[1][0], m[2][1], -(m[1][1] * m[2][0]));
  c[1][0] = std::fma(m[0][2], m[2][1], -(m[0][1] * m[2][2]));
  c[1][1] = std::fma(m[0][0], m[2][2], -(m[0][2] * m[2][0]));
  c[1][2] = std::fma(m[0][1], m[2][0], -(m[0][0] * m[2][1]));
  c[2][0] = std::fma(m[0][1], m[1][2], -(m[0][2] * m[1][1]));
  c[2][1] = std::fma(m[0][2], m[1][0], -(m[0][0] * m[1][2]));
  c[2][2] = std::fma(m[0][0], m[1][1], -(m[0][1] * m[1][0]));
  const double det = std::fma(m[0][2], c[0][2], std::fma(m[0][1], c[0][1], m[0][0] * c[0][0]));
  const double rd = 1.0 / det;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) out[i][j] = c[j][i] * rd;
  return det;
}

// icp_registration.cpp:33-42: A/b unpack (rigid_icp.cu:156-165), det check
// (cv::determinant), solve (D: 3+3 block solve instead of SVD),
// Tinc = Affine3f(rvec, t) (OpenCV Rodrigues, float/double mix), pose*Tinc (A6).
int kfo_icp_update(const int64_t sums[27], kfx_pose *pose, double x_out[6]) {
  double A[6][6], b[6];
  int s = 0;
  for (int i = 0; i < 6; ++i)
    for (int j = i; j < 7; ++j) {
      const double v = (double)sums[s++] * (1.0 / 4294967296.0);
      if (j == 6)
        b[i] = v;
      else
        A[i][j] = A[j][i] = v;
    }
  // D: A = JᵀJ is symmetric positive (semi)definite: instead of
  // cv::solve(DECOMP_SVD), a 3+3 block solve — P = A[0:3,0:3] (rotation), Q =
  // A[0:3,3:6], R = A[3:6,3:6], S = R − Qᵀ P⁻¹ Q (Schur complement), the 3×3
  // inverses by cofactors (one division each), det A = det P · det S as
  // cv::determinant's value.  Two divisions on the dependency chain instead of
  // six (the kernel's icp_update runs these exact operations).
  double P[3][3], Q[3][3], R[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      P[i][j] = A[i][j];
      Q[i][j] = A[i][j + 3];
      R[i][j] = A[i + 3][j + 3];
    }
  double Pi[3][3], Si[3][3], S[3][3], M[3][3];
  const double detP = kfo_inv3(P, Pi);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      M[i][j] = std::fma(Pi[i][2], Q[2][j], std::fma(Pi[i][1], Q[1][j], Pi[i][0] * Q[0][j]));
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      S[i][j] = std::fma(-Q[2][i], M[2][j], std::fma(-Q[1][i], M[1][j], std::fma(-Q[0][i], M[0][j], R[i][j])));
  const double detS = kfo_inv3(S, Si);
  const double det = detP * detS;
  if (std::fabs(det) < 1e-15 || std::isnan(det)) return 1;
  double y1[3], z[3], x[6];
  for (int i = 0; i < 3; ++i) y1[i] = std::fma(Pi[i][2], b[2], std::fma(Pi[i][1], b[1], Pi[i][0] * b[0]));
  for (int i = 0; i < 3; ++i)
    z[i] = std::fma(-Q[2][i], y1[2], std::fma(-Q[1][i], y1[1], std::fma(-Q[0][i], y1[0], b[3 + i])));
  for (int i = 0; i < 3; ++i) x[3 + i] = std::fma(Si[i][2], z[2], std::fma(Si[i][1], z[1], Si[i][0] * z[0]));
  for (int i = 0; i < 3; ++i)
    x[i] = std::fma(-M[i][2], x[5], std::fma(-M[i][1], x[4], std::fma(-M[i][0], x[3], y1[i])));
  if (x_out)
    for (int i = 0; i < 6; ++i) x_out[i] = x[i];
  // cv::Affine3f(Vec3f rvec, Vec3f t): the Vec3d arguments narrow to float.
  const float rv[3] = {(float)x[0], (float)x[1], (float)x[2]};
  kfx_pose inc;
  inc.t[0] = (float)x[3];
  inc.t[1] = (float)x[4];
  inc.t[2] = (float)x[5];
  const double theta = std::sqrt((double)rv[0] * rv[0] + (double)rv[1] * rv[1] +
                                 (double)rv[2] * rv[2]);
  if (theta < 2.220446049250313e-16) {
    for (int i = 0; i < 9; ++i) inc.R[i] = (i % 4 == 0) ? 1.f : 0.f;
  } else {
    double c, sn;
    kfo_sincos(theta, &sn, &c);
    const double c1 = 1.0 - c;
    const double it = 1.0 / theta;
    const float r[3] = {(float)(rv[0] * it), (float)(rv[1] * it), (float)(rv[2] * it)};
    const float rrt[9] = {r[0] * r[0], r[0] * r[1], r[0] * r[2], r[0] * r[1], r[1] * r[1],
                          r[1] * r[2], r[0] * r[2], r[1] * r[2], r[2] * r[2]};
    const float rx[9] = {0.f, -r[2], r[1], r[2], 0.f, -r[0], -r[1], r[0], 0.f};
    for (int i = 0; i < 9; ++i) {
      const float e = (i % 4 == 0) ? 1.f : 0.f;
      inc.R[i] = ((float)(c * e) + (float)(c1 * rrt[i])) + (float)(sn * rx[i]);
    }
  }
  kfo_pose_mul(pose, &inc, pose);
  return 0;
}

// icp_registration.cpp:16-46: levels high->low, iters[level] each, pose starts
// at identity (the default-constructed Affine3f; prepose is unused).
int kfo_icp_track(float **cur_v, float **cur_n, float **pre_v, float **pre_n,
                  const kfx_intrinsics *intr, const kfx_params *p, kfx_pose *cam_pose) {
  kfo_pose_identity(cam_pose);
  const float angle = std::sin(p->icp_angle_threshold * 0.017453293f);  // A14
  for (int level = p->pyramid_height - 1; level >= 0; --level) {
    kfx_intrinsics li;
    kfo_level_intrinsics(intr, level, &li);
    for (int it = 0; it < p->icp_iter_count[level]; ++it) {
      int64_t sums[27];
      kfo_icp_accumulate(cur_v[level], cur_n[level], pre_v[level], pre_n[level], li.width,
                         li.height, &li, cam_pose, p->icp_dist_threshold, angle, sums);
      if (kfo_icp_update(sums, cam_pose, nullptr)) return 1;
    }
  }
  return 0;
}

// tsdfhelper::operator() (tsdf_volume.cu:41-99).  Column (x,y) sweeps z=1..Z-1
// with vc accumulated by repeated float adds (z=0 never updated).
// One voxel's running average (tsdfhelper, tsdf_volume.cu:72-81), for a
// voxel that passed sdf >= -trunc.
void kfo_tsdf_update(int t0, int w0, float sdf, float trunc, int *q_out, int *w_out) {
  const float ts = std::fmin(1.f, sdf / trunc);
  const float pre_t = (float)t0 * kDivShortMax;
  const int pre_w = w0;
  const int new_w = (pre_w + 1 < kMaxWeight) ? pre_w + 1 : kMaxWeight;
  const float new_t = std::fma(pre_t, (float)pre_w, ts) / (float)(pre_w + 1);
  int q = (int)(new_t * (float)kShortMax);
  q = q < -kShortMax ? -kShortMax : (q > kShortMax ? kShortMax : q);
  *q_out = q;
  *w_out = new_w;
}

void kfo_integrate(int16_t *tsdf, int16_t *weight, uint8_t *rgb, const int dims[3],
                   const float vs[3], float trunc, const kfx_intrinsics *in,
                   const kfx_pose *pose, const float *dmap, const uint8_t *bgr,
                   const int32_t *cols, int64_t ncols, int64_t *n_upd, int64_t *n_col) {
  const int X = dims[0], Y = dims[1], Z = dims[2];
  const int64_t slice = (int64_t)X * Y;
  const int W = in->width, H = in->height;
  int64_t cu = 0, cc = 0;
  const int64_t total = cols ? ncols : slice;
  const float thres_color = trunc / 2;
  const V3 t = {pose->t[0], pose->t[1], pose->t[2]};
  const V3 zstep = {pose->R[2] * vs[0], pose->R[5] * vs[0], pose->R[8] * vs[0]};
  for (int64_t ci = 0; ci < total; ++ci) {
    int x, y;
    if (cols) {
      x = cols[2 * ci];
      y = cols[2 * ci + 1];
    } else {
      x = (int)(ci % X);
      y = (int)(ci / X);
    }
    const V3 vx = {(float)x * vs[0], (float)y * vs[1], 0.f * vs[2]};
    V3 vc = add(rmul(pose->R, vx), t);
    for (int z = 1; z < Z; ++z) {
      const int64_t idx = (int64_t)x + (int64_t)y * X + (int64_t)z * slice;
      vc = add(vc, zstep);
      if (vc.z <= 0) continue;
      const int u = f2i_rn((vc.x / vc.z) * in->fx + in->cx);
      const int v = f2i_rn((vc.y / vc.z) * in->fy + in->cy);
      if (u < 0 || u >= W || v < 0 || v >= H) continue;
      const float depth = dmap[(int64_t)v * W + u];
      if (depth <= 0) continue;
      const V3 xyl = {(1.f * ((float)u - in->cx)) / in->fx, (1.f * ((float)v - in->cy)) / in->fy,
                      1.f};
      const float lambda = std::sqrt(dot(xyl, xyl));
      const float sdf = -((1.f / lambda) * std::sqrt(dot(vc, vc)) - depth);
      if (sdf >= -trunc) {
        ++cu;
        int q, new_w;
        kfo_tsdf_update(tsdf[idx], weight[idx], sdf, trunc, &q, &new_w);
        tsdf[idx] = (int16_t)q;
        weight[idx] = (int16_t)new_w;
        if (sdf <= thres_color && sdf >= -thres_color) {
          ++cc;
          uint8_t *mc = rgb + 4 * idx;
          const uint8_t *px = bgr + 3 * ((int64_t)v * W + u);
          const float c = (float)(new_w + 1);
          for (int ch = 0; ch < 3; ++ch) {
            const float m = (float)(new_w * mc[ch] + px[ch]);
            mc[ch] = (uint8_t)(m / c);
          }
        }
      }
    }
  }
  if (n_upd) *n_upd = cu;
  if (n_col) *n_col = cc;
}

namespace {
struct RayCtx {
  const int16_t *tsdf;
  int X, Y, Z;
  int64_t slice;
  V3 vs, vs_inv, gd;
  int zb, zn;  // slices that may be read: [zb, zb+zn) (the whole volume unless slab)
  uint8_t *touch = nullptr;  // kfo_raycast_touched: 1 per voxel whose tsdf was read
  int64_t *reads = nullptr;  // and the number of tsdf reads
};
inline float tsdf_at(const RayCtx &c, int64_t i) {
  if (c.touch) {
    c.touch[i] = 1;
    ++*c.reads;
  }
  return (float)c.tsdf[i] * kDivShortMax;
}
// raycasthelper::voxel2tsdf (tsdf_volume.cu:178-191): nearest voxel, valid 1..dim-2
inline float voxel2tsdf(const RayCtx &c, V3 p) {
  const int x = f2i_rn(p.x * c.vs_inv.x);
  const int y = f2i_rn(p.y * c.vs_inv.y);
  const int z = f2i_rn(p.z * c.vs_inv.z);
  if (x >= c.X - 1 || y >= c.Y - 1 || z >= c.Z - 1 || x < 1 || y < 1 || z < 1) return NAN;
  if (z < c.zb || z >= c.zb + c.zn) return NAN;  // slab: not stored
  return tsdf_at(c, (int64_t)x + (int64_t)y * c.X + (int64_t)z * c.slice);
}
// interpolate (tsdf_volume.cu:137-161), terms accumulated in listed order
inline float interp(const RayCtx &c, V3 cf) {
  const int gx = f2i_rd(cf.x), gy = f2i_rd(cf.y), gz = f2i_rd(cf.z);
  if (gx < 0 || gx >= c.X - 1 || gy < 0 || gy >= c.Y - 1 || gz < 0 || gz >= c.Z - 1) return NAN;
  if (gz < c.zb || gz + 1 >= c.zb + c.zn) return NAN;  // slab: not stored
  const float a = cf.x - (float)gx, b = cf.y - (float)gy, cc = cf.z - (float)gz;
  auto T = [&](int dx, int dy, int dz) {
    return tsdf_at(c, (int64_t)(gx + dx) + (int64_t)(gy + dy) * c.X + (int64_t)(gz + dz) * c.slice);
  };
  float s = 0.f;
  s += T(0, 0, 0) * (1 - a) * (1 - b) * (1 - cc);
  s += T(0, 0, 1) * (1 - a) * (1 - b) * cc;
  s += T(0, 1, 0) * (1 - a) * b * (1 - cc);
  s += T(0, 1, 1) * (1 - a) * b * cc;
  s += T(1, 0, 0) * a * (1 - b) * (1 - cc);
  s += T(1, 0, 1) * a * (1 - b) * cc;
  s += T(1, 1, 0) * a * b * (1 - cc);
  s += T(1, 1, 1) * a * b * cc;
  return s;
}
// raycasthelper::compute_normal (tsdf_volume.cu:192-209)
inline V3 compute_normal(const RayCtx &c, V3 p) {
  V3 n;
  const float fx1 = interp(c, mulc({p.x + c.gd.x, p.y, p.z}, c.vs_inv));
  const float fx2 = interp(c, mulc({p.x - c.gd.x, p.y, p.z}, c.vs_inv));
  n.x = (fx1 - fx2) / c.gd.x;
  const float fy1 = interp(c, mulc({p.x, p.y + c.gd.y, p.z}, c.vs_inv));
  const float fy2 = interp(c, mulc({p.x, p.y - c.gd.y, p.z}, c.vs_inv));
  n.y = (fy1 - fy2) / c.gd.y;
  const float fz1 = interp(c, mulc({p.x, p.y, p.z + c.gd.z}, c.vs_inv));
  const float fz2 = interp(c, mulc({p.x, p.y, p.z - c.gd.z}, c.vs_inv));
  n.z = (fz1 - fz2) / c.gd.z;
  return normalized(n);
}
}  // namespace

// raycasthelper::operator() (tsdf_volume.cu:210-260) + intersect (:120-136).
// Slab restatement (keys != null): only slices [zb, zb+zn) may be read, only
// samples whose nearest voxel z is in [own0, own1) may end the ray, and the
// loop index (from 1) of the sample that ended it is written to keys
// (UINT32_MAX: none) — the per-slab half of the Z-slab raycast.
static void raycast_impl(const int16_t *tsdf, const int dims[3], const float vs[3],
                         const float range[3], const kfx_intrinsics *in, const kfx_pose *pose,
                         const float Rinv[9], float *vmap, float *nmap, const int32_t *pix,
                         int64_t npix, int zb, int zn, int own0, int own1, uint32_t *keys,
                         uint8_t *touch = nullptr, int64_t *reads = nullptr, float *ts_out = nullptr) {
  RayCtx c;
  c.touch = touch;
  c.reads = reads;
  c.tsdf = tsdf;
  c.X = dims[0];
  c.Y = dims[1];
  c.Z = dims[2];
  c.zb = zb;
  c.zn = zn;
  c.slice = (int64_t)c.X * c.Y;
  c.vs = {vs[0], vs[1], vs[2]};
  c.vs_inv = {1.f / vs[0], 1.f / vs[1], 1.f / vs[2]};  // raycasthelper ctor (host)
  c.gd = scl(c.vs, 0.5f);
  const float step = vs[0];
  const V3 org = {pose->t[0], pose->t[1], pose->t[2]};
  const int64_t total = pix ? npix : (int64_t)in->width * in->height;
  for (int64_t pi = 0; pi < total; ++pi) {
    int x, y;
    if (pix) {
      x = pix[2 * pi];
      y = pix[2 * pi + 1];
    } else {
      x = (int)(pi % in->width);
      y = (int)(pi / in->width);
    }
    const int64_t o = (int64_t)y * in->width + x;
    st3(vmap, o, {0.f, 0.f, 0.f});
    st3(nmap, o, {0.f, 0.f, 0.f});
    if (keys) keys[o] = UINT32_MAX;
    if (ts_out) ts_out[o] = 0.f;
    const V3 pp = {(1.f * ((float)x - in->cx)) / in->fx, (1.f * ((float)y - in->cy)) / in->fy,
                   1.f};
    const V3 dir = normalized(rmul(pose->R, pp));
    // intersect with box [0, range]
    const V3 invR = {1.f / dir.x, 1.f / dir.y, 1.f / dir.z};
    const V3 tbot = mulc(invR, sub({0.f, 0.f, 0.f}, org));
    const V3 ttop = mulc(invR, sub({range[0], range[1], range[2]}, org));
    const V3 tmin = {std::fmin(ttop.x, tbot.x), std::fmin(ttop.y, tbot.y),
                     std::fmin(ttop.z, tbot.z)};
    const V3 tmax = {std::fmax(ttop.x, tbot.x), std::fmax(ttop.y, tbot.y),
                     std::fmax(ttop.z, tbot.z)};
    const float tnear = std::fmax(std::fmax(tmin.x, tmin.y), std::fmax(tmin.x, tmin.z));
    const float tfar = std::fmin(std::fmin(tmax.x, tmax.y), std::fmin(tmax.x, tmax.z));
    float ray_len = std::fmax(tnear, 0.f);
    if (ray_len >= tfar) continue;
    const V3 vstep = mulc(dir, c.vs);
    ray_len += step;
    V3 nextp = add(org, scl(dir, ray_len));
    float tn = voxel2tsdf(c, nextp);
    uint32_t k = 0;
    for (; ray_len < tfar; ray_len += step) {
      nextp = add(nextp, vstep);
      ++k;
      const float tcur = tn;
      tn = voxel2tsdf(c, nextp);
      if (std::isnan(tn)) continue;
      if (keys) {  // slab: an event counts only at an owned sample
        const int iz = f2i_rn(nextp.z * c.vs_inv.z);
        if (iz < own0 || iz >= own1) continue;
      }
      if (tcur < 0.f && tn > 0.f) {
        if (keys) keys[o] = k;
        break;
      }
      if (tcur > 0.f && tn < 0.f) {
        const float Ts = ray_len - (vs[0] * tcur) / (tcur - tn);  // A3 (R)
        const V3 vertex = add(org, scl(dir, Ts));
        const V3 n = compute_normal(c, vertex);
        if (!std::isnan(n.x * n.y * n.z)) {
          st3(nmap, o, rmul(Rinv, n));
          st3(vmap, o, rmul(Rinv, sub(vertex, org)));
          if (keys) keys[o] = k;
          if (ts_out) ts_out[o] = Ts;
          break;
        }
      }
    }
  }
}

void kfo_raycast(const int16_t *tsdf, const int dims[3], const float vs[3],
                 const float range[3], const kfx_intrinsics *in, const kfx_pose *pose,
                 const float Rinv[9], float *vmap, float *nmap, const int32_t *pix,
                 int64_t npix) {
  raycast_impl(tsdf, dims, vs, range, in, pose, Rinv, vmap, nmap, pix, npix, 0, dims[2], 0,
               dims[2], nullptr);
}

// SURVEY.md §8d raycast roofline input: N_uniq = the distinct voxels whose
// tsdf the reference raycast reads (nearest samples + trilinear corners of the
// normals), and the total number of those reads.
void kfo_raycast_touched(const int16_t *tsdf, const int dims[3], const float vs[3],
                         const float range[3], const kfx_intrinsics *in, const kfx_pose *pose,
                         const float Rinv[9], int64_t *n_uniq, int64_t *n_reads) {
  const int64_t n = (int64_t)dims[0] * dims[1] * dims[2];
  std::vector<uint8_t> touch((size_t)n, 0);
  std::vector<float> vmap((size_t)in->width * in->height * 3), nmap(vmap.size());
  int64_t reads = 0;
  raycast_impl(tsdf, dims, vs, range, in, pose, Rinv, vmap.data(), nmap.data(), nullptr, 0, 0, dims[2], 0,
               dims[2], nullptr, touch.data(), &reads);
  int64_t u = 0;
  for (uint8_t t : touch) u += t;
  *n_uniq = u;
  *n_reads = reads;
}

void kfo_raycast_slab(const int16_t *tsdf, const int dims[3], const float vs[3],
                      const float range[3], const kfx_intrinsics *in, const kfx_pose *pose,
                      const float Rinv[9], int zb, int zn, int own0, int own1, float *vmap,
                      float *nmap, uint32_t *keys, float *ts) {
  raycast_impl(tsdf, dims, vs, range, in, pose, Rinv, vmap, nmap, nullptr, 0, zb, zn, own0, own1,
               keys, nullptr, nullptr, ts);
}

// FullScan6 (tsdf_volume.cu:307-481) in the canonical order of the GPU
// extraction (D: the reference's order comes from warp atomics): chunks of 8
// slices aligned to global multiples of 8, then 8x8 (x,y) tiles row-major,
// then z, then (y&7, x&7), then the +x/+y/+z edge.  z covers [zlo, zhi)
// (zhi <= Z-1).  Writes min(cap, total) points, returns the total.
int64_t kfo_extract_points(const int16_t *tsdf, const int16_t *weight, const int dims[3],
                           const float vs[3], const kfx_pose *aff, int zlo, int zhi, float *out,
                           int64_t cap) {
  const int X = dims[0], Y = dims[1];
  const int64_t slice = (int64_t)X * Y;
  auto idx = [&](int x, int y, int z) { return (int64_t)x + (int64_t)y * X + (int64_t)z * slice; };
  const V3 t = {aff->t[0], aff->t[1], aff->t[2]};
  int64_t n = 0;
  zlo = std::max(zlo, 0), zhi = std::min(zhi, dims[2] - 1);  // a voxel's +z neighbour must exist
  const int a0 = (zlo / 8) * 8;
  for (int c0 = a0; c0 < zhi; c0 += 8)
    for (int ty = 0; ty < Y / 8; ++ty)
      for (int tx = 0; tx < X / 8; ++tx)
        for (int z = std::max(zlo, c0); z < std::min(zhi, c0 + 8); ++z)
          for (int yy = 0; yy < 8; ++yy)
            for (int xx = 0; xx < 8; ++xx) {
              const int x = tx * 8 + xx, y = ty * 8 + yy;
              const int W = weight[idx(x, y, z)];
              const float F = (float)tsdf[idx(x, y, z)] * kDivShortMax;
              if (W == 0 || F == 1.f) continue;
              const V3 V = {((float)x + 0.5f) * vs[0], ((float)y + 0.5f) * vs[1],
                            ((float)z + 0.5f) * vs[2]};
              for (int axis = 0; axis < 3; ++axis) {
                if (axis == 0 && x + 1 >= X) continue;
                if (axis == 1 && y + 1 >= Y) continue;
                const int64_t j = idx(x + (axis == 0), y + (axis == 1), z + (axis == 2));
                const int Wn = weight[j];
                const float Fn = (float)tsdf[j] * kDivShortMax;
                if (Wn != 0 && Fn != 1.f && ((F > 0 && Fn < 0) || (F < 0 && Fn > 0))) {
                  V3 p = V;
                  const float Va = axis == 0 ? V.x : (axis == 1 ? V.y : V.z);
                  const float Vn = Va + vs[axis];
                  const float d_inv = 1.f / (std::fabs(F) + std::fabs(Fn));
                  const float cc = (Va * std::fabs(Fn) + Vn * std::fabs(F)) * d_inv;
                  if (axis == 0) p.x = cc;
                  else if (axis == 1) p.y = cc;
                  else p.z = cc;
                  if (n < cap) st3(out, n, add(rmul(aff->R, p), t));
                  ++n;
                }
              }
            }
  return n;
}

// Marching cubes (D, no reference counterpart).  Table: for
// every corner pattern, each face (corner cycle counter-clockwise seen from
// outside) links the edge where a run of inside corners begins to the edge
// where it ends; following the links gives closed loops over the cut edges,
// each fanned from its smallest edge.  Edge numbering: axis-major, within an
// axis by ascending lower corner (corner bits x | y<<1 | z<<2).
void kfo_mc_table(uint8_t *tab) {
  int ends[12][2];
  int ne = 0;
  for (int axis = 0; axis < 3; ++axis)
    for (int corner = 0; corner < 8; ++corner)
      if (((corner >> axis) & 1) == 0) {
        ends[ne][0] = corner;
        ends[ne][1] = corner + (1 << axis);
        ne++;
      }
  auto edge_of = [&](int p, int q) {
    const int a = std::min(p, q), b = std::max(p, q);
    for (int e = 0; e < 12; e++)
      if (ends[e][0] == a && ends[e][1] == b) return e;
    return -1;
  };
  std::vector<std::vector<int>> faces;
  for (int axis = 0; axis < 3; axis++) {
    const int u = (axis + 1) % 3, w = (axis + 2) % 3;
    for (int side = 0; side < 2; side++) {
      std::vector<int> f = {side << axis, (side << axis) | (1 << u), (side << axis) | (1 << u) | (1 << w),
                            (side << axis) | (1 << w)};  // CCW about +e_axis
      if (side == 0) std::reverse(f.begin(), f.end());
      faces.push_back(f);
    }
  }
  for (int pat = 0; pat < 256; pat++) {
    auto in = [&](int corner) { return ((pat >> corner) & 1) != 0; };
    std::vector<int> link(12, -1);
    for (const auto &f : faces)
      for (int i = 0; i < 4; i++) {
        const int prev = f[(i + 3) % 4], cur = f[i];
        if (!in(cur) || in(prev)) continue;
        int last = i;
        while (in(f[(last + 1) % 4])) last = (last + 1) % 4;
        link[edge_of(prev, cur)] = edge_of(f[last], f[(last + 1) % 4]);
      }
    std::vector<int> tris;
    std::vector<bool> used(12, false);
    for (int e0 = 0; e0 < 12; e0++) {
      if (link[e0] < 0 || used[e0]) continue;
      std::vector<int> loop;
      int e = e0;
      do {
        used[e] = true;
        loop.push_back(e);
        e = link[e];
      } while (e != e0);
      for (size_t k = 1; k + 1 < loop.size(); k++) {
        tris.push_back(loop[0]);
        tris.push_back(loop[k]);
        tris.push_back(loop[k + 1]);
      }
    }
    uint8_t *row = tab + 16 * pat;
    std::fill(row, row + 16, (uint8_t)0);
    row[0] = (uint8_t)(tris.size() / 3);
    for (size_t k = 0; k < tris.size(); k++) row[1 + k] = (uint8_t)tris[k];
  }
}

int64_t kfo_extract_mesh(const int16_t *tsdf, const int16_t *weight, const int dims[3], const float vs[3],
                         const kfx_pose *aff, int zlo, int zhi, float *out, int64_t cap) {
  uint8_t tab[256 * 16];
  kfo_mc_table(tab);
  const int X = dims[0], Y = dims[1];
  const int64_t slice = (int64_t)X * Y;
  auto idx = [&](int x, int y, int z) { return (int64_t)x + (int64_t)y * X + (int64_t)z * slice; };
  const V3 t = {aff->t[0], aff->t[1], aff->t[2]};
  int64_t n = 0;
  zlo = std::max(zlo, 0), zhi = std::min(zhi, dims[2] - 1);  // a cube's upper corners must exist
  for (int c0 = (zlo / 8) * 8; c0 < zhi; c0 += 8)
    for (int ty = 0; ty < Y / 8; ++ty)
      for (int tx = 0; tx < X / 8; ++tx)
        for (int z = std::max(zlo, c0); z < std::min(zhi, c0 + 8); ++z)
          for (int yy = 0; yy < 8; ++yy)
            for (int xx = 0; xx < 8; ++xx) {
              const int x = tx * 8 + xx, y = ty * 8 + yy;
              if (x + 1 >= X || y + 1 >= Y) continue;
              float F[8];
              int pat = 0;
              bool ok = true;
              for (int c = 0; c < 8; c++) {
                const int64_t i = idx(x + (c & 1), y + ((c >> 1) & 1), z + (c >> 2));
                ok = ok && weight[i] > 0;
                F[c] = (float)tsdf[i] * kDivShortMax;
                if (F[c] < 0.f) pat |= 1 << c;
              }
              if (!ok) continue;
              const uint8_t *row = tab + 16 * pat;
              for (int k = 0; k < 3 * row[0]; k++, n += (k % 3 == 0)) {
                if (n >= cap) continue;
                const int e = row[1 + k], axis = e / 4;
                int lo = -1;  // lower corner: the (e%4)-th corner with the axis bit clear
                for (int c = 0, m = 0; c < 8; c++)
                  if (!((c >> axis) & 1) && m++ == e % 4) lo = c;
                const int hi = lo | (1 << axis);
                V3 p = {((float)(x + (lo & 1)) + 0.5f) * vs[0], ((float)(y + ((lo >> 1) & 1)) + 0.5f) * vs[1],
                        ((float)(z + (lo >> 2)) + 0.5f) * vs[2]};
                const float Va = axis == 0 ? p.x : (axis == 1 ? p.y : p.z);
                const float Vn = Va + vs[axis];
                const float d_inv = 1.f / (std::fabs(F[lo]) + std::fabs(F[hi]));
                const float cc = (Va * std::fabs(F[hi]) + Vn * std::fabs(F[lo])) * d_inv;
                if (axis == 0) p.x = cc;
                else if (axis == 1) p.y = cc;
                else p.z = cc;
                st3(out, 3 * n + k % 3, add(rmul(aff->R, p), t));
              }
            }
  return n;
}

// kernel_renderNormals / kernel_renderPhong (image_process.cu:137-221) on the
// previous frame's level-0 maps.  D: __fsqrt_rn and IEEE division for
// __m_normalize's __fdividef (device_utils.cuh:50-54), pow(h, 10) as the
// product chain h2 = h*h, h4 = h2*h2, h8 = h4*h4, h8*h2; the double promotion
// of `0.5*light_coffi` is kept.  Pixels the kernel returns early on stay 0
// (the zeroed cmap).  type 0 = PHONG, 1 = NORMAL; out = w*h uchar3.
// (uchar)(x) of a value in [0, 255] (truncation); D: NaN (normals of the
// frame-1 measured maps, A8) gives 0, as the GPU conversion does
static uint8_t to_u8(float x) { return x >= 1.f ? (uint8_t)std::fmin(x, 255.f) : 0; }
void kfo_render(const float *vmap, const float *nmap, int w, int h, const float eye[3], int type,
                uint8_t *out) {
  for (int i = 0; i < w * h; ++i) {
    const V3 n = ld3(nmap, i), v = ld3(vmap, i);
    uint8_t *o = out + 3 * (size_t)i;
    o[0] = o[1] = o[2] = 0;
    if (type == 1) {
      o[0] = to_u8(std::fabs(n.x) * 255);
      o[1] = to_u8(std::fabs(n.y) * 255);
      o[2] = to_u8(std::fabs(n.z) * 255);
      continue;
    }
    if (n.x == 0 && n.y == 0 && n.z == 0) continue;
    if (v.x == 0 && v.y == 0 && v.z == 0) continue;
    const V3 kd = {0.3843f, 0.4745f, 0.580f};
    const V3 light = {500.f, 500.f, -500.f};
    const float intensity = 0.9f;
    const V3 e = normalized(sub({eye[0], eye[1], eye[2]}, v));
    const V3 l = normalized(sub(light, v));
    float lc = dot(n, l);
    if (lc <= 0) lc = -lc;
    float coef = intensity * lc;
    const V3 diffuse = scl(kd, coef);
    const V3 hv = normalized(add(l, e));
    float hc = dot(n, hv);
    if (hc < 0) hc = -hc;
    const float h2 = hc * hc, h4 = h2 * h2, h8 = h4 * h4;
    coef = intensity * (h8 * h2);
    const double spec = 0.5 * (double)coef;
    const float amb = 0.1f;
    const float k0 = (float)std::fmin(1.0, (double)(amb + diffuse.x) + spec);
    const float k1 = (float)std::fmin(1.0, (double)(amb + diffuse.y) + spec);
    const float k2 = (float)std::fmin(1.0, (double)(amb + diffuse.z) + spec);
    o[0] = to_u8(k0 * 255);
    o[1] = to_u8(k1 * 255);
    o[2] = to_u8(k2 * 255);
  }
}

int kfo_format_pose(const kfx_pose *p, char *buf, int cap) {
  return std::snprintf(buf, cap,
                       "[%.8g, %.8g, %.8g, %.8g;\n %.8g, %.8g, %.8g, %.8g;\n %.8g, %.8g, "
                       "%.8g, %.8g;\n 0, 0, 0, 1]\n",
                       p->R[0], p->R[1], p->R[2], p->t[0], p->R[3], p->R[4], p->R[5], p->t[1],
                       p->R[6], p->R[7], p->R[8], p->t[2]);
}

}  // extern "C"

// ---------------------------------------------------------------------------
// kf::kinectfusion restated (kinectfusion.cpp:9-141)
struct kfo_pipe {
  kfx_intrinsics intr;
  kfx_params p;
  int L;
  int frame_count;
  std::vector<kfx_pose> poses;
  std::vector<std::vector<float>> cd, cv, cn, pd, pv, pn;
  std::vector<int16_t> tsdf, weight;
  std::vector<uint8_t> rgb;
  int64_t last_upd = 0, last_col = 0;
  float vs[3];

  void reset_frames() {
    for (int l = 0; l < L; ++l) {
      std::fill(cd[l].begin(), cd[l].end(), 0.f);
      std::fill(cv[l].begin(), cv[l].end(), 0.f);
      std::fill(cn[l].begin(), cn[l].end(), 0.f);
      std::fill(pd[l].begin(), pd[l].end(), 0.f);
      std::fill(pv[l].begin(), pv[l].end(), 0.f);
      std::fill(pn[l].begin(), pn[l].end(), 0.f);
    }
  }
  void reset() {  // kinectfusion.cpp:133-141 (A5 D: whole volume zeroed)
    frame_count = 1;
    reset_frames();
    std::fill(tsdf.begin(), tsdf.end(), 0);
    std::fill(weight.begin(), weight.end(), 0);
    std::fill(rgb.begin(), rgb.end(), 0);
    poses.clear();
    kfx_pose I;
    kfo_pose_identity(&I);
    poses.push_back(I);
  }
  void integrate(const uint8_t *bgr) {  // TSDFVolume::integrate (tsdf_volume.cpp:42-52)
    kfx_pose inv, vol2cam;
    kfo_pose_inv(&poses.back(), &inv);
    kfo_pose_mul(&inv, &p.volu_pose, &vol2cam);
    kfo_integrate(tsdf.data(), weight.data(), rgb.data(), p.volu_dims, vs, p.volu_trun_dist,
                  &intr, &vol2cam, cd[0].data(), bgr, nullptr, 0, &last_upd, &last_col);
  }
  int process(const uint8_t *bgr, const float *depth) {  // kinectfusion.cpp:78-127
    std::vector<float *> d(L), v(L), n(L), qv(L), qn(L);
    for (int l = 0; l < L; ++l) {
      d[l] = cd[l].data();
      v[l] = cv[l].data();
      n[l] = cn[l].data();
      qv[l] = pv[l].data();
      qn[l] = pn[l].data();
    }
    kfo_preprocess(depth, intr.width, intr.height, L, &intr, &p, d.data(), v.data(), n.data());
    if (frame_count == 1) {
      integrate(bgr);
      for (int l = 0; l < L; ++l) {  // vmap/nmap swap (:88-89), copy is equivalent
        pv[l] = cv[l];
        pn[l] = cn[l];
      }
      frame_count++;
      return 0;
    }
    kfx_pose cam;
    if (kfo_icp_track(v.data(), n.data(), qv.data(), qn.data(), &intr, &p, &cam)) {
      reset();
      return 1;
    }
    kfx_pose g;
    kfo_pose_mul(&poses.back(), &cam, &g);
    poses.push_back(g);
    integrate(bgr);
    // TSDFVolume::raycast (tsdf_volume.cpp:53-62): cam2vol = vol_pose^-1 * pose,
    // Rinv = R^-1 (D: transpose instead of SVD inverse)
    kfx_pose vinv, cam2vol;
    kfo_pose_inv(&p.volu_pose, &vinv);
    kfo_pose_mul(&vinv, &poses.back(), &cam2vol);
    float Rinv[9];
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) Rinv[3 * i + j] = cam2vol.R[3 * j + i];
    kfo_raycast(tsdf.data(), p.volu_dims, vs, p.volu_range, &intr, &cam2vol, Rinv,
                pv[0].data(), pn[0].data(), nullptr, 0);
    for (int l = 1; l < L; ++l) {
      kfx_intrinsics li;
      kfo_level_intrinsics(&intr, l, &li);
      kfo_resize_points_normals(pv[l - 1].data(), pn[l - 1].data(), li.width, li.height,
                                pv[l].data(), pn[l].data());
    }
    frame_count++;
    return 0;
  }
};

extern "C" {

kfo_pipe *kfo_pipe_create(const kfx_intrinsics *intr, const kfx_params *p) {
  kfo_pipe *pp = new kfo_pipe();
  pp->intr = *intr;
  pp->p = *p;
  pp->L = p->pyramid_height;
  pp->cd.resize(pp->L);
  pp->cv.resize(pp->L);
  pp->cn.resize(pp->L);
  pp->pd.resize(pp->L);
  pp->pv.resize(pp->L);
  pp->pn.resize(pp->L);
  for (int l = 0; l < pp->L; ++l) {
    kfx_intrinsics li;
    kfo_level_intrinsics(intr, l, &li);
    const size_t n = (size_t)li.width * li.height;
    pp->cd[l].resize(n);
    pp->pd[l].resize(n);
    pp->cv[l].resize(3 * n);
    pp->cn[l].resize(3 * n);
    pp->pv[l].resize(3 * n);
    pp->pn[l].resize(3 * n);
  }
  const size_t nv = (size_t)p->volu_dims[0] * p->volu_dims[1] * p->volu_dims[2];
  pp->tsdf.resize(nv);
  pp->weight.resize(nv);
  pp->rgb.resize(4 * nv);
  for (int i = 0; i < 3; ++i) pp->vs[i] = p->volu_range[i] / (float)p->volu_dims[i];
  pp->reset();
  return pp;
}
void kfo_pipe_destroy(kfo_pipe *pp) { delete pp; }
void kfo_pipe_reset(kfo_pipe *pp) { pp->reset(); }
int kfo_pipe_process(kfo_pipe *pp, const uint8_t *bgr, const float *depth_mm) {
  return pp->process(bgr, depth_mm);
}
int kfo_pipe_frame_count(const kfo_pipe *pp) { return pp->frame_count; }
int kfo_pipe_pose_count(const kfo_pipe *pp) { return (int)pp->poses.size(); }
void kfo_pipe_get_pose(const kfo_pipe *pp, int i, kfx_pose *out) { *out = pp->poses[i]; }
int16_t *kfo_pipe_tsdf(kfo_pipe *pp) { return pp->tsdf.data(); }
int16_t *kfo_pipe_weight(kfo_pipe *pp) { return pp->weight.data(); }
uint8_t *kfo_pipe_rgb(kfo_pipe *pp) { return pp->rgb.data(); }
float *kfo_pipe_map(kfo_pipe *pp, int which, int kind, int level) {
  if (which == 0) return kind == 0 ? pp->cd[level].data() : kind == 1 ? pp->cv[level].data() : pp->cn[level].data();
  return kind == 0 ? pp->pd[level].data() : kind == 1 ? pp->pv[level].data() : pp->pn[level].data();
}
void kfo_pipe_last_counts(const kfo_pipe *pp, int64_t *n_upd, int64_t *n_col) {
  *n_upd = pp->last_upd;
  *n_col = pp->last_col;
}

}  // extern "C"
