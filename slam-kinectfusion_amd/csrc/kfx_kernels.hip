// kfx_kernels.hip — hand-written CDNA4 (gfx950) kernels of the KinectFusion hot
// path: preprocess (pyrDown, bilateral, truncation, vertex/normal maps), ICP
// (projective association + 27-term exact reduction + on-device 6x6 solve),
// TSDF integrate, raycast and pyramid resize.
//
// Every float expression follows the reference's evaluation order (file:line
// cited per kernel) and the file is compiled with -ffp-contract=off, so results
// are bit-identical to the CPU oracle (oracle/kfx_oracle.cpp) on the same inputs.
#include <algorithm>
#include <climits>
#include <cmath>
#include <limits>
#include <type_traits>

#include "kfx_internal.h"
#include "kfx_ffadd.h"

#ifndef KFX_INT_KB
#define KFX_INT_KB 4  // integrate: voxels per batch (loads in flight per lane)
#endif
#ifndef KFX_RAY_OCC
#define KFX_RAY_OCC 5  // raycast: waves per SIMD the register budget must allow (4800 waves at VGA: one round at 5)
#endif
#ifndef KFX_RAY_SLAB_OCC
#define KFX_RAY_SLAB_OCC 4  // slab and 64-bit-index raycasts: waves per SIMD (their extra registers spill at 5)
#endif
#ifndef KFX_RAY_KR
#define KFX_RAY_KR 14  // raycast: samples per batch (loads in flight per lane)
#endif
#ifndef KFX_RAY_HINT
// raycast: waves whose tile was slow in the last frame (frames are temporally
// coherent) take a higher issue priority (s_setprio) while all waves compete
#define KFX_RAY_HINT 1
#endif
#ifndef KFX_RAY_HINT_T0
#define KFX_RAY_HINT_T0 70  // priority thresholds, 1024-cycle units of last frame's wave duration
#endif
#ifndef KFX_INT_OCC
#define KFX_INT_OCC 8  // integrate: waves per SIMD the register budget is sized for
#endif
#ifndef KFX_INT_BLOCK
#define KFX_INT_BLOCK 64  // integrate: threads per block (one wave = one 8x8 column tile: wave slots refill one at a time)
#endif
#ifndef KFX_INT_CHUNKR
#define KFX_INT_CHUNKR 65  // integrate, shallow volumes: chunk c of a tile's interval gets weight (r/100)^c
#endif
#ifndef KFX_INT_ADAPT_ZN
// integrate chunking by volume (slab) depth zn, measured per config: for
// ADAPT_ZN <= zn < ADAPT_ZN_END, length-capped chunks dispatched longest-first
// by the last frame's intervals (C3: -12 % frame time); otherwise geometric
// chunks in block order (C2 and C4 slabs: the capped chunks' replay and
// prologue cost more than the tail they cut; C5's 2048-slice columns: 65536
// tiles already balance, and capping them costs long replays)
#define KFX_INT_ADAPT_ZN 1024
#endif
#ifndef KFX_INT_ADAPT_ZN_END
#define KFX_INT_ADAPT_ZN_END 2048
#endif
#ifndef KFX_INT_NC
#define KFX_INT_NC 4  // integrate, deep volumes: chunks of a full-length tile interval
#endif
#ifndef KFX_INT_MAXCHUNK
#define KFX_INT_MAXCHUNK 8  // integrate: most z-chunks per column tile
#endif
#ifndef KFX_INT_SLAB_CHUNK
#define KFX_INT_SLAB_CHUNK 96  // integrate, Z-slab contexts: chunks of at most about this many slices (with KFX_FF_MIN_SLAB 128; 128 / 64: slab sum +0.3 % / +3 %)
#endif
#ifndef KFX_FF_MIN
#define KFX_FF_MIN 768  // fast-forward replays of at least this many adds (shorter ones: the adds; A/B r3m: 384 costs C2 +8 %)
#endif
#ifndef KFX_FF_MIN_SLAB
// Z-slabs that do not start at z = 0: every chunk replays its column from
// z = 1 to past the slab's start, so the exact fast-forward pays from fewer
// adds (C4 calibrated slabs: integrate sum 1.563-1.577 -> 1.545-1.548 ms, worst
// slab 0.219-0.221 -> 0.214-0.215 ms; C2 is unaffected)
#define KFX_FF_MIN_SLAB 128
#endif
#ifndef KFX_INT_SLAB_CAPW
#define KFX_INT_SLAB_CAPW 49152  // integrate, Z-slab contexts: at most this many waves
#endif
#ifndef KFX_INT_WAVES
// integrate: target wave count (z-chunks per column tile; C2: 4 chunks of 4096
// tiles — 3 while the next frame's preprocess shared the GPU with integrate;
// with it beside the raycast, 4 measured -1.1 % frame time in 6 of 6
// alternating pairs, 2 and 5 slower or neutral: profiles/r06_int_chunks_ab.txt)
#define KFX_INT_WAVES 16384
#endif

namespace kfx {
namespace {

constexpr float kDivShortMax = 0.0000305185f;  // device_utils.cuh:6
constexpr int kShortMax = 32767;               // device_utils.cuh:7
constexpr int kMaxWeight = 64;                 // device_utils.cuh:5 (A10)
constexpr float kFixHalf = 65536.0f;           // ICP fixed point 2^32 (D) = 2^16 per factor of a product
constexpr int kDmaxShards = 16;
constexpr float kInfF = __builtin_huge_valf();

struct f3 {
  float x, y, z;
};
__device__ __forceinline__ f3 add(f3 a, f3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ f3 sub(f3 a, f3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ f3 scl(f3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ f3 mulc(f3 a, f3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
__device__ __forceinline__ float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ f3 cross(f3 a, f3 b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
__device__ __forceinline__ f3 normalized(f3 v) {
  const float t = sqrtf(dot(v, v));
  return {v.x / t, v.y / t, v.z / t};
}
__device__ __forceinline__ f3 rmul(const float *R, f3 v) {
  return {R[0] * v.x + R[1] * v.y + R[2] * v.z, R[3] * v.x + R[4] * v.y + R[5] * v.z,
          R[6] * v.x + R[7] * v.y + R[8] * v.z};
}
__device__ __forceinline__ f3 ld3(const float *p, size_t i) {
  return {p[3 * i], p[3 * i + 1], p[3 * i + 2]};
}
__device__ __forceinline__ void st3(float *p, size_t i, f3 v) {
  p[3 * i] = v.x;
  p[3 * i + 1] = v.y;
  p[3 * i + 2] = v.z;
}
// __float2int_rn / __float2int_rd, out-of-range -> INT_MIN (rejected by every
// bounds check, as the saturated CUDA result is)
__device__ __forceinline__ int f2i_rn(float v) {
  const float r = rintf(v);
  return (r > -2.0e9f && r < 2.0e9f) ? (int)r : INT_MIN;
}
__device__ __forceinline__ int f2i_rd(float v) {
  const float r = floorf(v);
  return (r > -2.0e9f && r < 2.0e9f) ? (int)r : INT_MIN;
}
__device__ __forceinline__ int reflect101(int i, int n) {
  if (i < 0) i = -i;
  if (i >= n) i = 2 * n - 2 - i;
  return i;
}
// Deterministic exp (same constants/order as the oracle's kfo_expf).
__device__ __forceinline__ float det_expf(float x) {
  if (!(x >= -86.0f)) return 0.0f;
  const float kf = rintf(x * 1.44269502f);
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
  return p * __uint_as_float((unsigned)(k + 127) << 23);
}

// x / d correctly rounded in 3 instructions given y = RN(1/d): Markstein's
// theorem (q0 = RN(x*y) is within 1 ulp, the FMA remainder is exact, one
// correction step rounds correctly).  Checked against IEEE division on 6.7e9
// operand pairs for the divisors used here (1..65 and the truncation
// distances), and for every colour quotient (tools/markstein_check.c).
__device__ __forceinline__ float div_rn(float x, float d, float y) {
  const float q0 = x * y;
  const float r = fmaf(-q0, d, x);
  return fmaf(r, y, q0);
}

// The same sequences on two independent operands (v_pk_mul/v_pk_fma_f32: the
// per-element IEEE operations of the scalar forms, two per instruction).
typedef float pf2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ pf2 pfma(pf2 a, pf2 b, pf2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ pf2 rcp_rn2(pf2 d) {
  const pf2 r = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  return pfma(pfma(-d, r, pf2{1.f, 1.f}), r, r);
}
__device__ __forceinline__ pf2 div_rn2(pf2 x, pf2 d, pf2 y) {
  const pf2 q0 = x * y;
  return pfma(pfma(-q0, d, x), y, q0);
}
__device__ __forceinline__ pf2 sqrt_rn2(pf2 x) {
  const pf2 y = {__builtin_amdgcn_rsqf(x.x), __builtin_amdgcn_rsqf(x.y)};
  const pf2 s0 = x * y;
  return pfma(pfma(-s0, s0, x), pf2{0.5f, 0.5f} * y, s0);
}

// Integrate's voxel pairs (ipf2): packed FP32 (KFX_INT_PK 1: v_pk_* ops,
// each 4 cycles per wave on gfx950, tools/valu_calib.hip) or two scalar
// operations per pair (0: 2 cycles each, no register moves to pair operands).
#ifndef KFX_INT_LDALL
#define KFX_INT_LDALL 1  // integrate: pin the batch's tsdf / weight loads before the update branches (C2 -1.5 us)
#endif
#ifndef KFX_INT_BSKIP
#define KFX_INT_BSKIP 0  // integrate: skip a batch's loads and update when no voxel of the wave passes
#endif
#ifndef KFX_INT_PK
#define KFX_INT_PK 0  // scalar pairs: C2 integrate 0.190 -> 0.178 ms with -fno-slp-vectorize
#endif
#if KFX_INT_PK
typedef pf2 ipf2;
#else
struct ipf2 {
  float x, y;
  __device__ __forceinline__ float operator[](int k) const { return k ? y : x; }
};
__device__ __forceinline__ ipf2 operator+(ipf2 a, ipf2 b) { return {a.x + b.x, a.y + b.y}; }
__device__ __forceinline__ ipf2 operator-(ipf2 a, ipf2 b) { return {a.x - b.x, a.y - b.y}; }
__device__ __forceinline__ ipf2 operator*(ipf2 a, ipf2 b) { return {a.x * b.x, a.y * b.y}; }
__device__ __forceinline__ ipf2 operator-(ipf2 a) { return {-a.x, -a.y}; }
__device__ __forceinline__ ipf2 pfma(ipf2 a, ipf2 b, ipf2 c) { return {fmaf(a.x, b.x, c.x), fmaf(a.y, b.y, c.y)}; }
__device__ __forceinline__ ipf2 rcp_rn2(ipf2 d) {
  const ipf2 r = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  return pfma(pfma(-d, r, ipf2{1.f, 1.f}), r, r);
}
__device__ __forceinline__ ipf2 div_rn2(ipf2 x, ipf2 d, ipf2 y) {
  const ipf2 q0 = x * y;
  return pfma(pfma(-q0, d, x), y, q0);
}
__device__ __forceinline__ ipf2 sqrt_rn2(ipf2 x) {
  const ipf2 y = {__builtin_amdgcn_rsqf(x.x), __builtin_amdgcn_rsqf(x.y)};
  const ipf2 s0 = x * y;
  return pfma(pfma(-s0, s0, x), ipf2{0.5f, 0.5f} * y, s0);
}
#endif

// Pixel coordinate rn((a / d) * f + c) as a float, with a / d from one
// reciprocal y = RN(1/d) shared by both image axes: div_rn(a, d, y) is the
// correctly rounded quotient (Markstein; checked on 2e10 random general pairs,
// tools/markstein_general.c).  |d| below 2^-100 (1/d near overflow) takes the
// IEEE division.
__device__ __forceinline__ float proj_rn(float a, float d, float y, float f, float c) {
  const float q = (fabsf(d) >= 7.8886091e-31f) ? div_rn(a, d, y) : a / d;
  return rintf(q * f + c);
}
// f2i_rn(v) in [0, n) tested on the rounded float (exact: integers, n < 2^24);
// NaN fails both compares like the INT_MIN of f2i_rn.
__device__ __forceinline__ bool in_range(float r, int n) { return r >= 0.f && r < (float)n; }

__device__ __forceinline__ DevPose pose_identity() {
  DevPose p;
  for (int i = 0; i < 9; ++i) p.R[i] = (i % 4 == 0) ? 1.f : 0.f;
  p.t[0] = p.t[1] = p.t[2] = 0.f;
  return p;
}
// Affine3f a*b (OpenCV concatenate/rotate/translate order)
__device__ DevPose pose_mul(const DevPose &a, const DevPose &b) {
  DevPose r;
  for (int j = 0; j < 3; ++j) {
    for (int i = 0; i < 3; ++i) {
      float v = 0.f;
      for (int k = 0; k < 3; ++k) v += a.R[3 * j + k] * b.R[3 * k + i];
      r.R[3 * j + i] = v;
    }
    float d = 0.f;
    for (int k = 0; k < 3; ++k) d += a.R[3 * j + k] * b.t[k];
    r.t[j] = d + a.t[j];
  }
  return r;
}
// Affine3f::inv (D: analytic rigid inverse)
__device__ DevPose pose_inv(const DevPose &a) {
  DevPose r;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) r.R[3 * i + j] = a.R[3 * j + i];
  for (int j = 0; j < 3; ++j) {
    float d = 0.f;
    for (int k = 0; k < 3; ++k) d += a.R[3 * k + j] * a.t[k];
    r.t[j] = -d;
  }
  return r;
}

__device__ __forceinline__ void frame_begin(DevState *st) {
  st->frame_serial += 1u;
  st->mode = (st->frame_count == 1) ? MODE_BOOT : MODE_TRACK;
  st->icp_fail = 0;
  st->n_base = st->n_poses;
  st->icp_pose = pose_identity();
  st->back = st->log[st->n_poses - 1];
}
// the frame's max-depth shards live after the level-0 dl table (one per cur buffer)
__device__ __forceinline__ unsigned *dmax_shards(const float2 *dl0, const LevelGeom &g0) {
  return (unsigned *)(const_cast<float2 *>(dl0) + (size_t)g0.w * g0.h);
}
// ... followed by the max-depth grid: the largest valid level-0 depth (m, as
// float bits; 0: none) of each 16x16-pixel block (k_preprocess_maps), the
// integrate occlusion clip's input (int_tile_clip; the allocation: kfx_api.hip dl0b)
__device__ __forceinline__ unsigned *dmax_grid(const float2 *dl0, const LevelGeom &g0) {
  return dmax_shards(dl0, g0) + kDmaxShards;
}

// z is the global slice; the view stores slices [zb, zb+zn) (tile-column
// layout, kfx_internal.h VolView)
__device__ __forceinline__ size_t vox_index(const VolView &v, int x, int y, int z) {
  return (((size_t)(y >> 3) * v.tiles_x + (x >> 3)) * (size_t)v.zn + (size_t)(z - v.zb)) * 64 +
         ((y & 7) << 3) + (x & 7);
}

// Occupancy marking (VolView::bocc / socc): some voxel of column tile (tx, ty)
// in global slices [zlo, zhi] holds a negative tsdf.  Sets, dilated by one,
// the bricks (zlo>>3)-1 .. (zhi>>3)+1 of the 3x3 tiles around (tx, ty) (lanes
// 0..8 of the calling wave) and the super-bricks (zlo>>5)-1 .. (zhi>>5)+1 of
// the 3x3 super tiles around (tx>>2, ty>>2) (lanes 9..17).  A plain read
// first skips the atomic when the bits are already set (bits are never
// cleared inside a launch, so a stale read is a subset).
template <typename W>
__device__ __forceinline__ void occ_set_bits(W *base, int lo, int hi) {
  constexpr int kb = 8 * sizeof(W);
  for (int b = lo; b <= hi;) {
    const int wi = b / kb, e = min(hi, wi * kb + kb - 1);
    const W m = (e - b == kb - 1 ? ~(W)0 : (((W)1 << (e - b + 1)) - (W)1)) << (b % kb);
    if ((base[wi] & m) != m) atomicOr(&base[wi], m);
    b = e + 1;
  }
}
__device__ void occ_mark(const VolView &v, int tx, int ty, int zlo, int zhi, int lane) {
  if (lane < 9) {
    const int x = tx + lane % 3 - 1, y = ty + lane / 3 - 1;
    if (x < 0 || y < 0 || x >= v.tiles_x || y >= v.tiles_y) return;
    occ_set_bits(v.bocc + (size_t)(y * v.tiles_x + x) * v.bw, max((zlo >> 3) - 1 - v.bz0, 0),
                 min((zhi >> 3) + 1 - v.bz0, v.nbz - 1));
  } else if (lane < 18) {
    const int k = lane - 9;
    const int x = (tx >> 2) + k % 3 - 1, y = (ty >> 2) + k / 3 - 1;
    if (x < 0 || y < 0 || x >= v.stx || y >= v.sty) return;
    occ_set_bits(v.socc + (size_t)(y * v.stx + x) * v.sw, max((zlo >> 5) - 1 - v.sz0, 0),
                 min((zhi >> 5) + 1 - v.sz0, v.nsz - 1));
  }
}
// Brick-exact marking of a chunk (integrate): bit k of u = global brick gbs + k
// (k < 62) holds a negative tsdf written by some lane of the wave (u is the
// wave OR, uniform); dilated by one brick / super-brick and OR-ed into the 3x3
// tiles / super tiles (lanes 0..8 / 9..17) like occ_mark.
__device__ void occ_mark_bricks(const VolView &v, int tile, int gbs, unsigned long long u, int lane) {
  if (!u) return;
  const int tx = tile % v.tiles_x, ty = tile / v.tiles_x;
  if (lane < 9) {
    const int x = tx + lane % 3 - 1, y = ty + lane / 3 - 1;
    if (x < 0 || y < 0 || x >= v.tiles_x || y >= v.tiles_y) return;
    unsigned long long d = (u << 1) | u | (u << 2);  // bricks gbs-1 .. gbs+62, bit k+1 = brick gbs+k
    int lb = gbs - 1 - v.bz0;                          // local brick of bit 0
    if (lb < 0) {
      d >>= -lb;
      lb = 0;
    }
    unsigned long long *w = v.bocc + (size_t)(y * v.tiles_x + x) * v.bw;
    const int w0 = lb >> 6, off = lb & 63;
    auto put = [&](int wi, unsigned long long m) {
      if (wi >= v.bw || !m) return;
      const int hi = v.nbz - wi * 64;  // valid bits of this word
      if (hi < 64) m &= (1ull << max(hi, 0)) - 1ull;
      if (m && (w[wi] & m) != m) atomicOr(&w[wi], m);
    };
    put(w0, d << off);
    if (off) put(w0 + 1, d >> (64 - off));
  } else if (lane < 18) {
    const int k = lane - 9;
    const int x = (tx >> 2) + k % 3 - 1, y = (ty >> 2) + k / 3 - 1;
    if (x < 0 || y < 0 || x >= v.stx || y >= v.sty) return;
    // super-bricks (global brick >> 2) of the set bricks, dilated by one,
    // relative to sbase = (gbs >> 2) - 1 (at most 18 bits)
    const int a = gbs & 3;  // bit m of (vhi:vlo) = global brick (gbs & ~3) + m
    const unsigned long long vlo = u << a, vhi = a ? u >> (64 - a) : 0ull;
    unsigned sm = 0u;  // bit g = super-brick (gbs >> 2) + g holds a set brick
#pragma unroll
    for (int g = 0; g < 17; ++g) sm |= (((g < 16 ? vlo >> (4 * g) : vhi) & 0xFull) != 0ull ? 1u : 0u) << g;
    sm = (sm << 1) | sm | (sm << 2);  // dilated, bit 0 = super-brick (gbs >> 2) - 1
    int ls = (gbs >> 2) - 1 - v.sz0;
    if (ls < 0) {
      sm >>= -ls;
      ls = 0;
    }
    uint32_t *w = v.socc + (size_t)(y * v.stx + x) * v.sw;
    const int w0 = ls >> 5, off = ls & 31;
    auto put = [&](int wi, unsigned m) {
      if (wi >= v.sw || !m) return;
      const int hi = v.nsz - wi * 32;
      if (hi < 32) m &= (1u << max(hi, 0)) - 1u;
      if (m && (w[wi] & m) != m) atomicOr(&w[wi], m);
    };
    put(w0, sm << off);
    if (off) put(w0 + 1, sm >> (32 - off));
  }
}
// Wave-wide [min lo, max hi] then occ_mark (all 64 lanes active).
__device__ __forceinline__ void occ_mark_wave(const VolView &v, int tile, int lo, int hi, int lane) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    lo = min(lo, __shfl_xor(lo, off));
    hi = max(hi, __shfl_xor(hi, off));
  }
  if (hi >= lo) occ_mark(v, tile % v.tiles_x, tile / v.tiles_x, lo, hi, lane);
}

// Level-indexed block decomposition for kernels that process all pyramid
// levels in one launch (16x16 pixel tiles).
struct LevelTiles {
  LevelGeom g[kMaxLevels];
  int off[kMaxLevels + 1];
  int nbx[kMaxLevels];
  int levels;
};
__device__ __forceinline__ int find_level(const LevelTiles &t, int b) {
  int l = 0;
  while (l + 1 < t.levels && b >= t.off[l + 1]) ++l;
  return l;
}
LevelTiles make_tiles(int levels, const LevelGeom *g) {
  LevelTiles t{};
  t.levels = levels;
  int acc = 0;
  for (int l = 0; l < levels; ++l) {
    t.g[l] = g[l];
    t.nbx[l] = (g[l].w + 15) / 16;
    t.off[l] = acc;
    acc += t.nbx[l] * ((g[l].h + 15) / 16);
  }
  t.off[levels] = acc;
  return t;
}

// ---------------------------------------------------------------------------
// Preprocess

__global__ void k_frame_begin(DevState *st, unsigned *dmax) {
  if (st) frame_begin(st);
  if (dmax)
    for (int i = 0; i < kDmaxShards; ++i) dmax[i] = 0u;
}

// cv::cuda::pyrDown (kinectfusion.cpp:54-55; OpenCV pyr_down.cu): vertical
// 5-tap at src row 2y for the 5 source columns, then horizontal 5-tap.
template <typename T>
__global__ __launch_bounds__(256) void k_pyr_down(const T *__restrict__ src, int w, int h,
                                                  float *__restrict__ dst, int dw, int dh,
                                                  DevState *st, unsigned *dmax) {
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0 && threadIdx.y == 0) {
    if (st) frame_begin(st);
    if (dmax)
      for (int i = 0; i < kDmaxShards; ++i) dmax[i] = 0u;
  }
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  const int y = blockIdx.y * blockDim.y + threadIdx.y;
  if (x >= dw || y >= dh) return;
  const float k0 = 0.0625f, k1 = 0.25f, k2 = 0.375f, k3 = 0.25f, k4 = 0.0625f;
  const int sy = 2 * y;
  const size_t r0 = (size_t)reflect101(sy - 2, h) * w, r1 = (size_t)reflect101(sy - 1, h) * w,
               r2 = (size_t)reflect101(sy, h) * w, r3 = (size_t)reflect101(sy + 1, h) * w,
               r4 = (size_t)reflect101(sy + 2, h) * w;
  float col[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    const int cx = reflect101(2 * x + j - 2, w);
    float s = k0 * (float)src[r0 + cx];
    s = s + k1 * (float)src[r1 + cx];
    s = s + k2 * (float)src[r2 + cx];
    s = s + k3 * (float)src[r3 + cx];
    s = s + k4 * (float)src[r4 + cx];
    col[j] = s;
  }
  float s = k0 * col[0];
  s = s + k1 * col[1];
  s = s + k2 * col[2];
  s = s + k3 * col[3];
  s = s + k4 * col[4];
  dst[(size_t)y * dw + x] = s;
}

struct BilatArgs {
  LevelTiles t;
  const float *raw[kMaxLevels];
  const uint16_t *raw0_u16;
  float *d[kMaxLevels];
  float *v[kMaxLevels];
  float *n[kMaxLevels];
  int ksz;
  float s_half, c_half;
  float max_dist;
  const float *invl;  // 1/lambda per level-0 pixel
  float2 *dl0;        // level 0: {filtered depth (m), 1/lambda} — the integrate gather
};

// cv::cuda::bilateralFilter (kinectfusion.cpp:57-65, A1 D: out of place) +
// kernal_depthTruncation (image_process.cu:8-17) + kernel_getVertexmap
// (image_process.cu:29-43) + kernel_getNormalmap (image_process.cu:57-84),
// fused, all levels in one launch.  A block owns a 16x16 tile: it stages the
// raw tile with a (r+1)-pixel halo in LDS (halo coordinates reflect-101
// mapped, exactly the taps the filter reads), filters the 18x18 ring the
// normals need, then computes normals of the 16x16 core from LDS.  Border
// normals are written 0 (the value Frame::reset leaves, types.hpp:53-62).
// Level 0 also reduces the frame's max depth (conservative integrate bound).
constexpr int kPreMaxR = 7;                    // ksz <= 15
constexpr int kPreRaw = 16 + 2 * (kPreMaxR + 1);  // 32
__global__ __launch_bounds__(256) void k_preprocess_maps(BilatArgs a) {
  const int l = find_level(a.t, blockIdx.x);
  const int local = blockIdx.x - a.t.off[l];
  const LevelGeom g = a.t.g[l];
  const int X0 = (local % a.t.nbx[l]) * 16, Y0 = (local / a.t.nbx[l]) * 16;
  const int r = a.ksz / 2, H = r + 1, side = 16 + 2 * H;
  __shared__ float sraw[kPreRaw * kPreRaw];
  __shared__ float sd[18 * 18];
  __shared__ f3 sv[18 * 18];
  const float *src = a.raw[l];
  const uint16_t *src16 = (l == 0) ? a.raw0_u16 : nullptr;
  for (int i = threadIdx.x; i < side * side; i += 256) {
    // taps of in-image pixels reflect once (create checks r < level size);
    // the clamp only keeps halo cells no output reads inside the image
    const int yy = min(max(reflect101(Y0 - H + i / side, g.h), 0), g.h - 1);
    const int xx = min(max(reflect101(X0 - H + i % side, g.w), 0), g.w - 1);
    const size_t o = (size_t)yy * g.w + xx;
    sraw[i] = src16 ? (float)src16[o] : src[o];
  }
  __syncthreads();
  // filtered depth + vertex on the 18x18 ring (pixels inside the image)
  const float r2 = (float)(r * r);
  for (int i = threadIdx.x; i < 18 * 18; i += 256) {
    const int py = i / 18, px = i % 18;
    const int x = X0 - 1 + px, y = Y0 - 1 + py;
    float dval = 0.f;
    f3 vtx = {0.f, 0.f, 0.f};
    if (x >= 0 && x < g.w && y >= 0 && y < g.h) {
      const int cyl = py + (H - 1), cxl = px + (H - 1);  // this pixel in sraw
      const float center = sraw[cyl * side + cxl];
      float sum1 = 0.f, sum2 = 0.f;
      for (int cy = y - r; cy < y - r + a.ksz; ++cy) {
        for (int cx = x - r; cx < x - r + a.ksz; ++cx) {
          const float space2 = (float)((x - cx) * (x - cx) + (y - cy) * (y - cy));
          if (space2 > r2) continue;
          const float vv = sraw[(cyl + cy - y) * side + (cxl + cx - x)];
          const float dd = fabsf(vv - center);
          const float wgt = det_expf(space2 * a.s_half + (dd * dd) * a.c_half);
          sum1 = sum1 + wgt * vv;
          sum2 = sum2 + wgt;
        }
      }
      dval = sum1 / sum2;
      dval *= 0.001f;
      if (dval > a.max_dist) dval = 0.f;
      if (isnan(dval))
        vtx = {0.f, 0.f, 0.f};
      else
        vtx = {(dval * ((float)x - g.cx)) / g.fx, (dval * ((float)y - g.cy)) / g.fy, dval};
    }
    sd[i] = dval;
    sv[i] = vtx;
  }
  __syncthreads();
  const int cx = threadIdx.x & 15, cy = threadIdx.x >> 4;
  const int x = X0 + cx, y = Y0 + cy;
  const bool in = x < g.w && y < g.h;
  const int c = (cy + 1) * 18 + (cx + 1);
  const float dval = sd[c];
  if (in) {
    const size_t o = (size_t)y * g.w + x;
    a.d[l][o] = dval;
    if (l == 0) a.dl0[o] = make_float2(dval, a.invl[o]);
    st3(a.v[l], o, sv[c]);
    f3 n = {0.f, 0.f, 0.f};
    if (x >= 1 && x < g.w - 1 && y >= 1 && y < g.h - 1) {
      const f3 lf = sv[c - 1], rt = sv[c + 1], up = sv[c - 18], dn = sv[c + 18];
      if (lf.z == 0 || rt.z == 0 || up.z == 0 || dn.z == 0) {
        n = {0.f, 0.f, 0.f};
      } else {
        n = cross(sub(lf, rt), sub(up, dn));
        if (n.z > 0) n = scl(n, -1.f);
      }
      n = normalized(n);  // 0/0 = NaN when a neighbour is invalid (A8)
    }
    st3(a.n[l], o, n);
  }
  if (l == 0) {  // block-uniform
    unsigned m = (in && dval > 0.f) ? __float_as_uint(dval) : 0u;
    for (int off = 32; off > 0; off >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, off));
    __shared__ unsigned wm[4];
    if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned b = max(max(wm[0], wm[1]), max(wm[2], wm[3]));
      if (b) atomicMax(&dmax_shards(a.dl0, a.t.g[0])[blockIdx.x % kDmaxShards], b);
      dmax_grid(a.dl0, a.t.g[0])[local] = b;  // this 16x16 block's cell (level-0 blocks are row-major)
    }
  }
}

// ---------------------------------------------------------------------------
// ICP

// ICP::findCoresp + kernel_rigidICP (rigid_icp.cu:46-113): per pixel of the
// floor-covered region (A2), the 7-vector row and its 27 products, summed as
// exact int64 fixed point (D; order-independent, so any reduction tree gives
// the oracle's sums).  Each lane takes kIcpPix pixels whose loads are issued
// together; the block reduces through LDS and writes one 27-word partial.
#ifndef KFX_ICP_XCD
#define KFX_ICP_XCD 1  // ICP: XCD-banded pixel rows per block
#endif
#ifndef KFX_ICP_PIX
#define KFX_ICP_PIX 4
#endif
constexpr int kIcpPix = KFX_ICP_PIX;
#ifndef KFX_EXTRACT_SKIP
#define KFX_EXTRACT_SKIP 1  // point / mesh extraction: waves of clear bricks read nothing
#endif
#ifndef KFX_XSWEEP_WAVES
#define KFX_XSWEEP_WAVES 65536  // extraction: units per wave grow (up to 64) while this many waves remain
#endif
#ifndef KFX_RAY_SLAB_SKIP
#define KFX_RAY_SLAB_SKIP 1  // slab raycast: rays jump over the samples before the stored slices
#endif
#ifndef KFX_RAY_N32
#define KFX_RAY_N32 1  // raycast normals: 32-bit tile-column offsets + buffer loads (kIdx32 volumes)
#endif
#ifndef KFX_ICP_PPLCAP
#define KFX_ICP_PPLCAP 256  // ICP plan: a level takes the fewest pixels per lane that keep it within this many blocks
#endif
#ifndef KFX_ICP_SLEEP
#define KFX_ICP_SLEEP 1  // ICP release poll: s_sleep units (64 clocks) between polls (0: busy poll)
#endif
#ifndef KFX_ICP_MINB
#define KFX_ICP_MINB 2  // persistent ICP: blocks per CU the register budget is sized for (co-resident grid)
#endif
#ifndef KFX_ICP_THREADS
#define KFX_ICP_THREADS 256  // ICP: threads per block
#endif
constexpr int kIcpThreads = KFX_ICP_THREADS;
constexpr int kIcpWaves = kIcpThreads / 64;
constexpr int kIcpBlockPix = kIcpThreads * kIcpPix;
constexpr unsigned long long kIcpWatchdogTicks = 20000000ull;  // >= 0.2 s of s_memrealtime
__device__ int icp_update(const double *a27, DevPose &pose, double *xo);
// rigid_icp.cu:156-165's unpack of one int64 fixed-point sum (exact scaling)
__device__ __forceinline__ double icp_sum_value(long long s) { return (double)s * (1.0 / 4294967296.0); }

// Per-lane part of one ICP iteration: kIcpPix pixels whose current-frame
// vertex/normal (n0, v0, validity ok0) are already in registers; gathers the
// previous frame's maps at the projections and accumulates the 27 products.
// Every product is rounded to an integer multiple of 2^-32 (rintf(prod *
// 2^32)); within a block the running sums are integers below 2^49 (|prod| <
// 2^7, <= 2^10 products per 27-slot), so fp64 adds are exact and equal the
// oracle's int64 sums; the block total converts to int64 exactly.
__device__ __forceinline__ void icp_lane(const LevelGeom &g, const DevPose &P,
                                         const f3 (&n0)[kIcpPix], const f3 (&v0)[kIcpPix],
                                         const bool (&ok0)[kIcpPix], int ppl,
                                         const float *__restrict__ pv,
                                         const float *__restrict__ pn, float dist2_max,
                                         float sine2_max, double (&acc)[27], bool zero = true) {
  const f3 t = {P.t[0], P.t[1], P.t[2]};
  if (zero) {  // (zero = false: add to the sums already in acc)
#pragma unroll
    for (int k = 0; k < 27; ++k) acc[k] = 0.0;
  }
  f3 vcur[kIcpPix];
  int j[kIcpPix];
  bool ok[kIcpPix];
#pragma unroll
  for (int q = 0; q < kIcpPix; ++q) {
    ok[q] = false;
    j[q] = 0;
    if (q >= ppl) continue;  // block-uniform: pixels per lane at this level
    vcur[q] = add(rmul(P.R, v0[q]), t);
    const int px = f2i_rn((vcur[q].x / vcur[q].z) * g.fx + g.cx);
    const int py = f2i_rn((vcur[q].y / vcur[q].z) * g.fy + g.cy);
    ok[q] = ok0[q] && !isnan(n0[q].x) && vcur[q].z > 0 && px >= 0 && py >= 0 && px < g.w &&
            py < g.h;
    j[q] = ok[q] ? py * g.w + px : 0;
  }
  // loads are unconditional (rejected lanes read pixel 0) so the compiler
  // issues each group back to back instead of waiting per branch
  f3 vpre[kIcpPix], npre[kIcpPix];
#pragma unroll
  for (int q = 0; q < kIcpPix; ++q) {
    if (q >= ppl) continue;
    vpre[q] = ld3(pv, j[q]);
    npre[q] = ld3(pn, j[q]);
  }
#pragma unroll
  for (int q = 0; q < kIcpPix; ++q) {
    if (!ok[q]) continue;
    // rigid_icp.cu's sqrtf(|d|^2) <= dist_thr and sqrtf(|sa|^2) <= angle_thr,
    // as one compare each: RN(sqrt(x)) is monotonic in x, so it is <= t exactly
    // when x <= sqrt_le_bound(t) (host; NaN fails both forms)
    const f3 dd = sub(vcur[q], vpre[q]);
    if (!(dot(dd, dd) <= dist2_max)) continue;
    const f3 ncur = rmul(P.R, n0[q]);
    const f3 sa = cross(ncur, npre[q]);
    if (!(dot(sa, sa) <= sine2_max)) continue;
    const f3 c = cross(vcur[q], npre[q]);
    const float row[7] = {c.x,       c.y,       c.z, npre[q].x, npre[q].y,
                          npre[q].z, dot(npre[q], sub(vpre[q], vcur[q]))};
    // rintf(RN(ra * rb) * 2^32) as rintf(RN(ra' * rb')) with x' = x * 2^16
    // (exact power-of-two scalings of finite |x| < 2^7): equal whenever the
    // product is normal, and when it is not (|ra * rb| < 2^-126) both round to
    // a zero of the product's sign
    float rs[7];
#pragma unroll
    for (int a = 0; a < 7; ++a) rs[a] = row[a] * kFixHalf;
    int s = 0;
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
      for (int b = a; b < 7; ++b) acc[s++] += (double)rintf(rs[a] * rs[b]);
  }
}

// Current-frame vertex/normal of the lane's pixels of pixel group grp.
// Blocks are dealt round-robin to the 8 XCDs; remap so that each XCD gets a
// contiguous band of work (raycast: 16x16 pixel tiles whose rays gather the
// same voxel lines; ICP: pixel rows whose correspondences gather the same
// rows of the previous maps), which then hits in that XCD's L2.  Bijective
// for any count.
__device__ __forceinline__ int xcd_remap(int b, int nb) {
  const int q = nb / 8, r = nb % 8, xcd = b % 8;
  return xcd * q + min(xcd, r) + b / 8;
}

// Pixels [p0, npix) of the floor-covered region (p0 > 0: a slab rank's band).
__device__ __forceinline__ void icp_load_cur(const LevelGeom &g, int xe, int npix, int grp,
                                             int ppl, const float *__restrict__ cv,
                                             const float *__restrict__ cn, f3 (&n0)[kIcpPix],
                                             f3 (&v0)[kIcpPix], bool (&ok)[kIcpPix], int p0 = 0) {
#pragma unroll
  for (int q = 0; q < kIcpPix; ++q) {
    const int i = p0 + grp * kIcpThreads * ppl + q * kIcpThreads + threadIdx.x;
    ok[q] = q < ppl && i < npix;
    const size_t idx = ok[q] ? (size_t)(i / xe) * g.w + (i % xe) : 0;
    n0[q] = ld3(cn, idx);
    v0[q] = ld3(cv, idx);
  }
}

// Block reduction of the block's lanes' 27 sums.  Within a wave, a reduce-scatter
// butterfly in registers: at each step a lane keeps the half of its values
// selected by one lane bit and adds its partner's copy of that half, so after
// 5 steps lane L holds value (L >> 1) summed over 32 lanes, and a last
// exchange completes the wave sum — 32 exchanges instead of 27 full
// reductions, all cross-lane VALU ops (gfx950 v_permlane32/16_swap for lane
// bits 5 and 4, DPP row_ror:8 / row_half_mirror / quad_perm for bits 3..0), no
// LDS round trips.  The 4 waves then meet in LDS.  Values are integers below
// 2^53: every order of fp64 adds is exact.  Returns, in threads 0..26, the
// block's sum k as int64.
struct IcpRed {
  double red2[(kIcpShards > kIcpWaves ? kIcpShards : kIcpWaves) * 27];  // waves' sums; also stages the shard reads
};
__device__ __forceinline__ unsigned lo32(double v) { return (unsigned)__double_as_longlong(v); }
__device__ __forceinline__ unsigned hi32(double v) {
  return (unsigned)((unsigned long long)__double_as_longlong(v) >> 32);
}
__device__ __forceinline__ double mk64(unsigned lo, unsigned hi) {
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
// Lane bits 5 / 4: v_permlane{32,16}_swap exchanges x of the upper lanes with y
// of the lower lanes, after which x + y is, in every lane, its kept value plus
// the partner's copy of it (lower lanes keep x = in[v], upper lanes y = in[N+v]).
template <int N, bool k32>
__device__ __forceinline__ void butterfly_swap(const double (&in)[2 * N], double (&out)[N]) {
#pragma unroll
  for (int v = 0; v < N; ++v) {
    const double x = in[v], y = in[N + v];
    unsigned xl, xh, yl, yh;
    if (k32) {
      const auto rl = __builtin_amdgcn_permlane32_swap(lo32(x), lo32(y), false, false);
      const auto rh = __builtin_amdgcn_permlane32_swap(hi32(x), hi32(y), false, false);
      xl = rl[0], yl = rl[1], xh = rh[0], yh = rh[1];
    } else {
      const auto rl = __builtin_amdgcn_permlane16_swap(lo32(x), lo32(y), false, false);
      const auto rh = __builtin_amdgcn_permlane16_swap(hi32(x), hi32(y), false, false);
      xl = rl[0], yl = rl[1], xh = rh[0], yh = rh[1];
    }
    out[v] = mk64(xl, xh) + mk64(yl, yh);
  }
}
template <int CTRL>
__device__ __forceinline__ double dpp64(double v) {
  return mk64((unsigned)__builtin_amdgcn_mov_dpp((int)lo32(v), CTRL, 0xf, 0xf, false),
              (unsigned)__builtin_amdgcn_mov_dpp((int)hi32(v), CTRL, 0xf, 0xf, false));
}
// Lane bits 3..1 through DPP: the partner (row_ror:8, row_half_mirror,
// quad_perm [2,3,0,1]) differs in `bit`; lanes with the bit clear keep in[v].
template <int N, int CTRL>
__device__ __forceinline__ void butterfly_dpp(const double (&in)[2 * N], double (&out)[N], int bit) {
  const bool hi = (threadIdx.x >> bit) & 1;
#pragma unroll
  for (int v = 0; v < N; ++v) {
    const double keep = hi ? in[N + v] : in[v];
    const double give = hi ? in[v] : in[N + v];
    out[v] = keep + dpp64<CTRL>(give);
  }
}
__device__ __forceinline__ long long icp_block_reduce(IcpRed &r, const double (&acc)[27]) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  double a32[32];
#pragma unroll
  for (int k = 0; k < 32; ++k) a32[k] = k < 27 ? acc[k] : 0.0;
  double a16[16], a8[8], a4[4], a2[2], a1[1];
  butterfly_swap<16, true>(a32, a16);    // lane bit 5
  butterfly_swap<8, false>(a16, a8);     // lane bit 4
  butterfly_dpp<4, 0x128>(a8, a4, 3);    // row_ror:8       (lane bit 3)
  butterfly_dpp<2, 0x141>(a4, a2, 2);    // row_half_mirror (lane bit 2)
  butterfly_dpp<1, 0x4E>(a2, a1, 1);     // quad_perm [2,3,0,1] (lane bit 1)
  const double w = a1[0] + dpp64<0xB1>(a1[0]);  // quad_perm [1,0,3,2]: value (lane >> 1)
  if ((lane & 1) == 0 && (lane >> 1) < 27) r.red2[wv * 27 + (lane >> 1)] = w;
  __syncthreads();
  long long v = 0;
  if (threadIdx.x < 27) {
    const int k = threadIdx.x;
    double a = r.red2[k];
#pragma unroll
    for (int q = 1; q < kIcpWaves; ++q) a += r.red2[27 * q + k];
    v = (long long)a;
  }
  __syncthreads();  // red2 is reused by the caller
  return v;
}

// One ICP iteration per launch (stage API seam and the fallback when the
// persistent kernel's grid cannot be co-resident).
__global__ __launch_bounds__(kIcpThreads) void k_icp_acc(LevelGeom g, int xe, int p0, int npix,
                                                 const float *__restrict__ cv,
                                                 const float *__restrict__ cn,
                                                 const float *__restrict__ pv,
                                                 const float *__restrict__ pn, float dist2_max,
                                                 float sine2_max, DevState *__restrict__ st,
                                                 unsigned long long *__restrict__ shards,
                                                 unsigned *__restrict__ ticket, int force,
                                                 int update) {
  if (!force && (st->mode != MODE_TRACK || st->icp_fail)) return;
  const DevPose P = st->icp_pose;
  f3 n0[kIcpPix], v0[kIcpPix];
  bool ok[kIcpPix];
  icp_load_cur(g, xe, npix, blockIdx.x, kIcpPix, cv, cn, n0, v0, ok, p0);
  double acc[27];
  icp_lane(g, P, n0, v0, ok, kIcpPix, pv, pn, dist2_max, sine2_max, acc);
  __shared__ IcpRed red;
  const long long bsum = icp_block_reduce(red, acc);
  // Cross-block sum + solve in the same launch: wave 0 adds the block's 27
  // sums into one of kIcpShards shard rows with device-scope int64 atomics
  // (performed at the memory side; exact and order-free), waits for them, then
  // takes a ticket.  The block drawing the last ticket reads-and-clears the
  // shards and runs icp_registration.cpp:33-42 (icp_update) on one lane.
  __shared__ int last;
  if (threadIdx.x < 64) {
    if (threadIdx.x < 27)
      __hip_atomic_fetch_add(&shards[(blockIdx.x % kIcpShards) * 27 + threadIdx.x],
                             (unsigned long long)bsum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (threadIdx.x == 0) {
      const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = (t == gridDim.x - 1);
    }
  }
  __syncthreads();
  if (!last) return;
  __shared__ double sumd[27];
  // one read-and-clear per thread (a thread's atomics serialise)
  for (int i = threadIdx.x; i < kIcpShards * 27; i += kIcpThreads)
    red.red2[i] = __longlong_as_double((long long)__hip_atomic_exchange(
        &shards[i], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  if (threadIdx.x == 0) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (threadIdx.x < 27) {
    long long a = 0;
#pragma unroll
    for (int sh = 0; sh < kIcpShards; ++sh) a += __double_as_longlong(red.red2[sh * 27 + threadIdx.x]);
    sumd[threadIdx.x] = icp_sum_value(a);
    st->sums[threadIdx.x] = a;
  }
  __syncthreads();
  if (threadIdx.x < 64 && update) {  // wave 0 solves
    DevPose p = st->icp_pose;
    double x[6];
    const int f = icp_update(sumd, p, x);
    if (threadIdx.x == 0) {
      if (f) {
        st->icp_fail = 1;
      } else {
        st->icp_pose = p;
#pragma unroll
        for (int i = 0; i < 6; ++i) st->x[i] = x[i];
      }
    }
  }
}

// ICPRegistration::rigidTransform (icp_registration.cpp:16-46) as ONE
// persistent launch: every iteration of every level, separated by a
// grid-wide arrival counter instead of a kernel boundary.  The grid (one
// block per 1024-pixel group of the largest level) is checked co-resident on
// the host (icp_persistent_ok).  Per iteration, the blocks that own pixels at
// that level add their int64 partials into the iteration's own shard slot and
// arrive; EVERY block then waits for the arrivals, reads the slot and runs the
// same solve (identical inputs and code => identical pose in every block, no
// broadcast step).  Current-frame maps stay in registers across a level's
// iterations.  A wall-clock watchdog turns a stalled barrier into a reported
// error instead of a hang.
// begin: the frame's frame_begin is folded in (overlapped frames): every block
// derives the begun state itself and block 0's thread 0, the only writer of
// these fields during the kernel, stores it first
// kStride: a level may have more pixel groups than the grid has blocks
// (IcpPlan::stride, 1280x720 level 0); block b then takes an equal contiguous
// range of that level's pixels (IcpPlan::span) in passes of up to kIcpPix per
// lane, re-reading them every iteration, their products added into the same
// lane sums (integers below 2^53 for <= 8192 pixels per block, so the fp64
// adds stay exact and the int64 totals are the oracle's); a longer range
// takes groups b, b + gridDim, ... with one block reduce per group.
template <bool kStride>
__global__ __launch_bounds__(kIcpThreads, KFX_ICP_MINB) void k_icp_track(IcpPlan pl, DevState *__restrict__ st,
                                                   IcpSync *__restrict__ sy, int begin) {
  DevPose P;
  if (begin) {
    if (blockIdx.x == 0 && threadIdx.x == 0) frame_begin(st);
    if (st->frame_count == 1) return;  // MODE_BOOT
    P = pose_identity();
  } else {
    if (st->mode != MODE_TRACK || st->icp_fail) return;  // uniform across the grid
    P = st->icp_pose;
  }
  __shared__ IcpRed red;
  __shared__ long long sums[27];
  __shared__ double sumd[27];  // the same sums unpacked (one conversion per thread, not per solver lane)
  __shared__ int sfail, sstall;
  int fail = 0;
  const bool withhold = blockIdx.x == 0 && st->debug_stall;  // test hook: never arrive at slot 0
  unsigned target = 0;  // (flat arrival counter: KFX_ICP_HIER 0)
  unsigned tsub = 0, ttop = 0;  // KFX_ICP_HIER: this block's residue's and the top counter's targets
  int slot = 0;
  for (int l = pl.levels - 1; l >= 0 && !fail; --l) {
    const LevelGeom g = pl.g[l];
    const int prank = (int)blockIdx.x;
    const bool mine = prank < pl.groups[l];
    // kStride (some level has more groups than blocks): every level takes its
    // groups b, b + gridDim.x, ... in identity order and re-reads their
    // current-frame pixels each iteration (no register-held pixels: one
    // lane-phase code path, the register budget of the plain kernel)
    constexpr bool stride = kStride;
    f3 n0[kIcpPix], v0[kIcpPix];
    bool ok[kIcpPix];
    // a level with span[l] > 0 in the plain kernel (IcpPlan::span, CU-uniform
    // level 0): this block's contiguous range of at most kIcpPix pixels per
    // lane, held in registers like a group
    int lppl = pl.ppl[l];
    if (mine && !stride) {
      const int r = KFX_ICP_XCD ? xcd_remap(blockIdx.x, pl.groups[l]) : (int)blockIdx.x;
      if (pl.span[l] > 0) {
        const int b0 = r * pl.span[l], b1 = min(pl.npix[l], b0 + pl.span[l]);
        lppl = min(kIcpPix, (b1 - b0 + kIcpThreads - 1) / kIcpThreads);
        icp_load_cur(g, pl.xe[l], b1, 0, lppl, pl.cv[l], pl.cn[l], n0, v0, ok, b0);
      } else {
        icp_load_cur(g, pl.xe[l], pl.npix[l], r, lppl, pl.cv[l], pl.cn[l], n0, v0, ok);
      }
    }
    for (int it = 0; it < pl.iters[l] && !fail; ++it, ++slot) {
      unsigned long long *sh = sy->sums + (size_t)slot * kIcpShards * 27;
      target += min(pl.groups[l], (int)gridDim.x);  // arrivals: the blocks with a group
      (void)target;
      {
        const int m = min(pl.groups[l], (int)gridDim.x), r = (int)(blockIdx.x & 7u);
        tsub += r < m ? (unsigned)((m - r + 7) / 8) : 0u;  // participants of residue r (blocks 0 .. m-1)
        ttop += (unsigned)min(m, 8);
      }
#ifdef KFX_ICP_TRACE
      const bool tr = threadIdx.x == 0 && (blockIdx.x == 0 || blockIdx.x == gridDim.x - 1);
#else
      constexpr bool tr = false;  // trace build only: the stamps' code costs ICP ~3 us per frame
#endif
      if (tr && blockIdx.x == 0) sy->trace[slot][0] = wall_clock64();
#ifdef KFX_ICP_BLOCK_TRACE
      if (threadIdx.x == 0 && blockIdx.x < 512) sy->blk[slot][blockIdx.x][0] = wall_clock64();
#endif
      if (mine) {
        long long bsum = 0;
        if (stride && pl.span[l] > 0) {
          // this block's contiguous range, in passes of up to kIcpPix pixels
          // per lane whose products add into the same lane sums (integers
          // below 2^53: exact), then one block reduce
          const int b0 = (int)blockIdx.x * pl.span[l], b1 = min(pl.npix[l], b0 + pl.span[l]);
          double acc[27];
#pragma unroll
          for (int k = 0; k < 27; ++k) acc[k] = 0.0;
          for (int p0 = b0; p0 < b1; p0 += kIcpPix * kIcpThreads) {
            const int ppl = min(kIcpPix, (b1 - p0 + kIcpThreads - 1) / kIcpThreads);
            icp_load_cur(g, pl.xe[l], b1, 0, ppl, pl.cv[l], pl.cn[l], n0, v0, ok, p0);
            icp_lane(g, P, n0, v0, ok, ppl, pl.pv[l], pl.pn[l], pl.dist2_max, pl.sine2_max, acc, false);
          }
          if (tr && blockIdx.x == 0) sy->trace[slot][8] = wall_clock64() + (acc[3] == -1.5 ? 1 : 0);
          bsum = icp_block_reduce(red, acc);
        } else if (stride) {
          // groups blockIdx.x, + gridDim.x, ...: each group's block sums are
          // added as int64 (exact), so no lane sums stay live across groups
          for (int gx = (int)blockIdx.x; gx < pl.groups[l]; gx += (int)gridDim.x) {
            double acc[27];
            icp_load_cur(g, pl.xe[l], pl.npix[l], gx, pl.ppl[l], pl.cv[l], pl.cn[l], n0, v0, ok);
            icp_lane(g, P, n0, v0, ok, pl.ppl[l], pl.pv[l], pl.pn[l], pl.dist2_max, pl.sine2_max, acc);
            if (tr && blockIdx.x == 0) sy->trace[slot][8] = wall_clock64() + (acc[3] == -1.5 ? 1 : 0);
            bsum += icp_block_reduce(red, acc);
          }
        } else {
          double acc[27];
          icp_lane(g, P, n0, v0, ok, lppl, pl.pv[l], pl.pn[l], pl.dist2_max, pl.sine2_max, acc);
          if (tr && blockIdx.x == 0) sy->trace[slot][8] = wall_clock64() + (acc[3] == -1.5 ? 1 : 0);
          bsum = icp_block_reduce(red, acc);
        }
        if (tr && blockIdx.x == 0) sy->trace[slot][9] = wall_clock64() + (bsum == -7 ? 1 : 0);
        if (threadIdx.x < 64) {
          if (threadIdx.x < 27)
            __hip_atomic_fetch_add(&sh[(prank % kIcpShards) * 27 + threadIdx.x],
                                   (unsigned long long)bsum, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
          // the partial adds are device-scope atomics (performed past the
          // non-coherent L2s); waiting for their completion orders them before
          // the arrival, and every read of them below is a coherent atomic
          // load, so no L2 writeback/invalidate fence is needed
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          if (tr && blockIdx.x == 0) sy->trace[slot][10] = wall_clock64();
#ifdef KFX_ICP_BLOCK_TRACE
          if (threadIdx.x == 0 && blockIdx.x < 512) sy->blk[slot][blockIdx.x][1] = wall_clock64();
#endif
          if (threadIdx.x == 0 && !(withhold && slot == 0)) {
            // the last arriver releases the iteration: spinners poll 8 flag
            // copies instead of the contended arrival counter
#if KFX_ICP_HIER
            // arrivals counted per residue b % 8 (one XCD each under the
            // round-robin placement; placement decides speed only): ~38
            // atomics per counter instead of 300 on one, whose serialisation
            // (~11 ns each) was ~1.7 us of every iteration's hand-off
            // (tools/icp_barrier_bench.hip); a residue's last arriver adds to
            // the top counter, whose last arriver releases
            const unsigned n = __hip_atomic_fetch_add(&sy->sub[blockIdx.x & 7u].v, 1u, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT);
            if (n == tsub - 1) {
              const unsigned m = __hip_atomic_fetch_add(&sy->top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              if (m == ttop - 1)
                for (int k = 0; k < 8; ++k)
                  __hip_atomic_store(&sy->release[k].v, (unsigned)(slot + 1), __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
            }
#else
            const unsigned n =
                __hip_atomic_fetch_add(&sy->arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (n == target - 1)
              for (int k = 0; k < 8; ++k)
                __hip_atomic_store(&sy->release[k].v, (unsigned)(slot + 1), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
#endif
          }
        }
      }
      if (tr) sy->trace[slot][blockIdx.x == 0 ? 1 : 4] = wall_clock64();
      if (threadIdx.x == 0) {
        const unsigned long long t0 = wall_clock64();
        int stalled = 0;
        const unsigned *flag = &sy->release[blockIdx.x & 7].v;
        while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)(slot + 1)) {
          if (KFX_ICP_SLEEP) __builtin_amdgcn_s_sleep(KFX_ICP_SLEEP);
          if (wall_clock64() - t0 > kIcpWatchdogTicks) {
            stalled = 1;
            break;
          }
        }
        if (stalled) st->icp_stalled = 1;  // host reports it after the frame
        sstall = stalled;
        if (tr && blockIdx.x == 0) sy->trace[slot][2] = wall_clock64();
      }
      __syncthreads();
      // read before the next two barriers: thread 0 may write sstall again at
      // the next iteration's poll (blocks that are not `mine` skip the block
      // reduce and its barrier), but only after every wave has passed them
      const int stall_seen = sstall;
      // one coherent load per thread (a thread's atomic loads serialise)
      for (int i = threadIdx.x; i < kIcpShards * 27; i += kIcpThreads)
        red.red2[i] = __longlong_as_double((long long)__hip_atomic_load(
            &sh[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      __syncthreads();
      if (threadIdx.x < 27) {
        long long a = 0;
#pragma unroll
        for (int k = 0; k < kIcpShards; ++k) a += __double_as_longlong(red.red2[k * 27 + threadIdx.x]);
        sums[threadIdx.x] = a;
        sumd[threadIdx.x] = icp_sum_value(a);
      }
      __syncthreads();
      if (tr && blockIdx.x == 0) sy->trace[slot][5] = wall_clock64();
      {  // every wave solves (every block, identical result): no broadcast of
         // the pose through LDS and no barrier after the solve.  The next
         // writes of red come after the block reduce's barrier; sums / sumd are
         // rewritten only after the next iteration's first two barriers, which
         // every wave reaches after finishing this solve
        DevPose p = P;
        double x[6];
        int f = icp_update(sumd, p, x);
        if (tr && blockIdx.x == 0) sy->trace[slot][6] = __builtin_amdgcn_readfirstlane((int)x[0]) + wall_clock64();
        if (stall_seen) f = 1;  // a stalled block stops; the others stall at the next barrier
        if (threadIdx.x < 27 && blockIdx.x == 0) st->sums[threadIdx.x] = sums[threadIdx.x];
        if (threadIdx.x == 0 && blockIdx.x == 0) {
          if (f) {
            st->icp_fail = 1;
          } else {
#pragma unroll
            for (int i = 0; i < 6; ++i) st->x[i] = x[i];
          }
        }
        if (tr && blockIdx.x == 0) sy->trace[slot][3] = wall_clock64();
        fail = __builtin_amdgcn_readfirstlane(f);
        if (!fail) {  // wave-uniform: keep the pose in SGPRs
#pragma unroll
          for (int k = 0; k < 9; ++k) P.R[k] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(p.R[k])));
#pragma unroll
          for (int k = 0; k < 3; ++k) P.t[k] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(p.t[k])));
        }
      }
    }
  }
  if (threadIdx.x == 0) {
    if (blockIdx.x == 0) {
      st->icp_pose = P;
      if (!fail) {  // integrate's vol2cam of this tracked frame, once (k_integrate)
        const DevPose gp = pose_mul(st->back, P);  // frame_pose(st, log, 1)
        st->int_v2c = pose_mul(pose_inv(gp), pl.vpose);
        st->int_tag = st->frame_serial;
      }
    }
    // exit ticket: the last block out clears the slots and the counters
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const unsigned t = __hip_atomic_fetch_add(&sy->exit, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sfail = (t == gridDim.x - 1);  // sfail is free after the loop's last barrier
  }
  __syncthreads();
  if (sfail) {  // this block drew the last exit ticket
    const int n = slot * kIcpShards * 27;
    for (int i = threadIdx.x; i < n; i += kIcpThreads)
      __hip_atomic_store(&sy->sums[i], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x == 0) {
      __hip_atomic_store(&sy->arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&sy->exit, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&sy->top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (threadIdx.x < 8) {
      __hip_atomic_store(&sy->release[threadIdx.x].v, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&sy->sub[threadIdx.x].v, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Broadcast of a double from a (wave-uniform) lane through SGPRs.
__device__ __forceinline__ double bcast(double v, int src) {
  const long long u = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(u & 0xffffffff), src);
  const int hi = __builtin_amdgcn_readlane((int)(u >> 32), src);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// icp_registration.cpp:33-42 on the device: A/b unpack (rigid_icp.cu:156-165),
// 3+3 block solve with det check (D: instead of SVD; A = JᵀJ is symmetric),
// Rodrigues, pose = pose * Tinc.  Every lane
// runs the whole solve on its own registers (identical, wave-uniform values:
// no cross-lane traffic on the critical path).  Each double operation is the
// oracle's (kfo_icp_update) in the same order, so the result is
// bit-identical.  (A partial-pivot LU spent most of its ~3.4k cycles on
// data-dependent row moves; the LDLᵀ after it ran six divisions in a row.)
// a27: the 27 sums already unpacked by
// icp_sum_value (any memory, read by all lanes; the unpack is done once per
// value by 27 threads, not 27 times per solver lane).
// D: cos / sin of the Rodrigues angle as the oracle's kfo_sincos (theta < 0.5:
// Taylor polynomials in theta^2, Horner form with fused multiply-adds; else ocml) —
// bit-identical to the oracle and far shorter than ocml's sincos.
__device__ __forceinline__ void det_sincos(double theta, double *s, double *c) {
  if (!(theta < 0.5)) {  // wave-uniform
    sincos(theta, s, c);
    return;
  }
  const double x2 = theta * theta;
  double ps = -1.0 / 1307674368000.0;
  ps = fma(ps, x2, 1.0 / 6227020800.0);
  ps = fma(ps, x2, -1.0 / 39916800.0);
  ps = fma(ps, x2, 1.0 / 362880.0);
  ps = fma(ps, x2, -1.0 / 5040.0);
  ps = fma(ps, x2, 1.0 / 120.0);
  ps = fma(ps, x2, -1.0 / 6.0);
  *s = fma(theta, x2 * ps, theta);
  double pc = -1.0 / 87178291200.0;
  pc = fma(pc, x2, 1.0 / 479001600.0);
  pc = fma(pc, x2, -1.0 / 3628800.0);
  pc = fma(pc, x2, 1.0 / 40320.0);
  pc = fma(pc, x2, -1.0 / 720.0);
  pc = fma(pc, x2, 1.0 / 24.0);
  pc = fma(pc, x2, -0.5);
  *c = fma(x2, pc, 1.0);
}

// 3x3 inverse by cofactors (the oracle's kfo_inv3): returns det(m), out = adj(m) / det
__device__ __forceinline__ double inv3(const double (&m)[3][3], double (&out)[3][3]) {
  double c[3][3];
  c[0][0] = fma(m[1][1], m[2][2], -(m[1][2] * m[2][1]));
  c[0][1] = fma(m[1][2], m[2][0], -(m[1][0] * m[2][2]));
  c[0][2] = fma(m[1][0], m[2][1], -(m[1][1] * m[2][0]));
  c[1][0] = fma(m[0][2], m[2][1], -(m[0][1] * m[2][2]));
  c[1][1] = fma(m[0][0], m[2][2], -(m[0][2] * m[2][0]));
  c[1][2] = fma(m[0][1], m[2][0], -(m[0][0] * m[2][1]));
  c[2][0] = fma(m[0][1], m[1][2], -(m[0][2] * m[1][1]));
  c[2][1] = fma(m[0][2], m[1][0], -(m[0][0] * m[1][2]));
  c[2][2] = fma(m[0][0], m[1][1], -(m[0][1] * m[1][0]));
  const double det = fma(m[0][2], c[0][2], fma(m[0][1], c[0][1], m[0][0] * c[0][0]));
  const double rd = 1.0 / det;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) out[i][j] = c[j][i] * rd;
  return det;
}

__device__ int icp_update(const double *a27, DevPose &pose, double *xo) {
  double A[6][7];  // column 6 = b
  {
    int q = 0;
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
      for (int j = i; j < 7; ++j) {
        const double v = a27[q++];
        A[i][j] = v;
        if (j < 6) A[j][i] = v;
      }
  }
  // D: 3+3 block solve (the oracle's kfo_icp_update, operation for
  // operation): P = A[0:3,0:3], Q = A[0:3,3:6], R = A[3:6,3:6], S = R − Qᵀ P⁻¹ Q;
  // 3×3 inverses by cofactors, det A = det P · det S.  Two divisions on the
  // dependency chain (the LDLᵀ it replaces had six plus two substitution
  // chains), so the per-iteration solve every lane runs is shorter.
  double P[3][3], Q[3][3], R[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      P[i][j] = A[i][j];
      Q[i][j] = A[i][j + 3];
      R[i][j] = A[i + 3][j + 3];
    }
  double Pi[3][3], Si[3][3], S[3][3], M[3][3];
  const double detP = inv3(P, Pi);
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) M[i][j] = fma(Pi[i][2], Q[2][j], fma(Pi[i][1], Q[1][j], Pi[i][0] * Q[0][j]));
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j)
      S[i][j] = fma(-Q[2][i], M[2][j], fma(-Q[1][i], M[1][j], fma(-Q[0][i], M[0][j], R[i][j])));
  const double detS = inv3(S, Si);
  const double det = detP * detS;
  if (fabs(det) < 1e-15 || isnan(det)) return 1;
  double y1[3], z[3], x[6];
#pragma unroll
  for (int i = 0; i < 3; ++i) y1[i] = fma(Pi[i][2], A[2][6], fma(Pi[i][1], A[1][6], Pi[i][0] * A[0][6]));
#pragma unroll
  for (int i = 0; i < 3; ++i) z[i] = fma(-Q[2][i], y1[2], fma(-Q[1][i], y1[1], fma(-Q[0][i], y1[0], A[3 + i][6])));
#pragma unroll
  for (int i = 0; i < 3; ++i) x[3 + i] = fma(Si[i][2], z[2], fma(Si[i][1], z[1], Si[i][0] * z[0]));
#pragma unroll
  for (int i = 0; i < 3; ++i) x[i] = fma(-M[i][2], x[5], fma(-M[i][1], x[4], fma(-M[i][0], x[3], y1[i])));
#pragma unroll
  for (int r = 0; r < 6; ++r) xo[r] = x[r];
  // cv::Affine3f(Vec3f rvec, Vec3f t): the Vec3d arguments narrow to float.
  const float rv[3] = {(float)x[0], (float)x[1], (float)x[2]};
  DevPose inc;
  inc.t[0] = (float)x[3];
  inc.t[1] = (float)x[4];
  inc.t[2] = (float)x[5];
  const double theta =
      sqrt((double)rv[0] * rv[0] + (double)rv[1] * rv[1] + (double)rv[2] * rv[2]);
  if (theta < 2.220446049250313e-16) {
#pragma unroll
    for (int q = 0; q < 9; ++q) inc.R[q] = (q % 4 == 0) ? 1.f : 0.f;
  } else {
    double sn, c;
    det_sincos(theta, &sn, &c);
    const double c1 = 1.0 - c;
    const double it = 1.0 / theta;
    const float r[3] = {(float)(rv[0] * it), (float)(rv[1] * it), (float)(rv[2] * it)};
    const float rrt[9] = {r[0] * r[0], r[0] * r[1], r[0] * r[2], r[0] * r[1], r[1] * r[1],
                          r[1] * r[2], r[0] * r[2], r[1] * r[2], r[2] * r[2]};
    const float rx[9] = {0.f, -r[2], r[1], r[2], 0.f, -r[0], -r[1], r[0], 0.f};
#pragma unroll
    for (int q = 0; q < 9; ++q) {
      const float e = (q % 4 == 0) ? 1.f : 0.f;
      inc.R[q] = ((float)(c * e) + (float)(c1 * rrt[q])) + (float)(sn * rx[q]);
    }
  }
  pose = pose_mul(pose, inc);
  return 0;
}

// kinectfusion.cpp:84-104, resolved on the device.  Frame kind: 0 = frame-1
// bootstrap (integrate at pose_record.back(), copy measured maps), 1 = tracked
// (pose_record.back() * cam_pose), 2 = ICP failure (reset(), frame dropped).
__device__ __forceinline__ int frame_kind(const DevState *st) {
  return st->mode == MODE_BOOT ? 0 : (st->icp_fail ? 2 : 1);
}
__device__ __forceinline__ DevPose frame_pose(const DevState *st, const DevPose *log, int kind) {
  (void)log;  // st->back = log[n_base - 1], copied by frame_begin (one dependent load fewer)
  const DevPose back = st->back;
  return kind == 0 ? back : pose_mul(back, st->icp_pose);
}
// pose_record push / reset (one thread of one block); only fields that no
// other block of the frame reads are written.
__device__ void frame_bookkeeping(DevState *st, DevPose *log, int kind, const DevPose &g) {
  if (kind == 2) {
    st->frame_count = 1;
    st->n_poses = 1;
    log[0] = pose_identity();
    st->last_fail = 1;
    st->fails += 1;
    return;
  }
  if (kind == 1) {
    if (st->n_base < st->pose_cap) {
      log[st->n_base] = g;
      st->n_poses = st->n_base + 1;
    } else {
      st->pose_overflow = 1;
    }
  }
  st->frame_count += 1;
  st->last_fail = 0;
}

// ---------------------------------------------------------------------------
// TSDF integrate — tsdfhelper::operator() (tsdf_volume.cu:41-99).
//
// One wave = one 8x8 tile of (x,y) columns; a lane sweeps its column in z with
// vc accumulated by repeated float adds exactly as the reference (so the
// projected pixel of every voxel is bit-identical).  A conservative z interval
// per column (frustum + max depth, computed in double with margins) skips the
// projection work outside it; the adds are still replayed there.

// Solve alpha + beta*z >= 0 into [lo, hi] (float, approximate quotient: the
// callers widen the result by 2 slices, far above the float error; a NaN
// quotient leaves the bound unchanged, an infinite one empties the interval).
__device__ __forceinline__ void clip_lin(float alpha, float beta, float &lo, float &hi) {
  if (beta > 0.f) {
    lo = fmaxf(lo, -alpha * __builtin_amdgcn_rcpf(beta));
  } else if (beta < 0.f) {
    hi = fminf(hi, -alpha * __builtin_amdgcn_rcpf(beta));
  } else if (alpha < 0.f) {
    hi = -1.f;
  }
}

// Correctly rounded reciprocal for |d| in [2^-125, 2^125]: one Newton step on
// v_rcp_f32 (checked against IEEE 1/d for every float in that range on gfx950,
// tools/rn_check.hip).
__device__ __forceinline__ float rcp_rn(float d) {
  const float r = __builtin_amdgcn_rcpf(d);
  return fmaf(fmaf(-d, r, 1.0f), r, r);
}
// Correctly rounded sqrt for x in [2^-96, 2^126]: v_rsq_f32 + one Newton step
// (exhaustively checked against IEEE sqrtf, tools/rn_check.hip).
__device__ __forceinline__ float sqrt_rn(float x) {
  const float y = __builtin_amdgcn_rsqf(x);
  const float s0 = x * y;
  return fmaf(fmaf(-s0, s0, x), 0.5f * y, s0);
}
// A column's vc values are vc0 + zs accumulated by float adds: each component
// is a multiple of 2^(min(exp(vc0), exp(zs)) - 23) (exact sums of multiples of
// a power of two round to multiples of it), so it is 0 or at least that large,
// and it stays below |vc0| + Z|zs| (x2 for rounding).  When every component
// lies in {0} u [2^-40, 2^40], rcp_rn (|vc.z| in range), the shared-reciprocal
// quotient (tools/markstein_general.c) and sqrt_rn (|vc|^2 in [2^-80, 2^82],
// or vc.z <= 0 and the voxel is rejected anyway) are all exact; otherwise the
// column takes the IEEE sequences.
__device__ __forceinline__ int exp_of(float a) { return (int)((__float_as_uint(a) >> 23) & 0xffu) - 127; }
__device__ __forceinline__ bool column_fast(f3 vc0, f3 zs, int Z) {
  const float c0[3] = {vc0.x, vc0.y, vc0.z}, s[3] = {zs.x, zs.y, zs.z};
  bool ok = true;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float bound = 2.f * (fabsf(c0[k]) + (float)(Z + 1) * fabsf(s[k]));  // < 2^40 / 1.01
    ok = ok && bound <= 0x1.fcp39f;  // false for NaN / inf poses
    int e = 1000;
    if (c0[k] != 0.f) e = min(e, exp_of(c0[k]));
    if (s[k] != 0.f) e = min(e, exp_of(s[k]));
    ok = ok && (e == 1000 || e - 23 >= -40);
  }
  return ok;
}

// 32-bit-offset buffer access (raw buffer resource; loads past num_records
// return 0 and stores are dropped, so a rejected lane passes offset ~0u).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void *p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, 0x00020000);
}
constexpr unsigned kOob = 0xFFFFFFFFu;

// Voxel storage access of k_integrate: kIdx32 (local volume <= 2^31 voxels)
// uses buffer loads/stores with 32-bit byte offsets for tsdf/weight (the
// colour array, touched only in the colour band, through a 64-bit pointer),
// else 64-bit pointers throughout.
template <bool kIdx32>
struct VoxMem;
template <>
struct VoxMem<true> {
  using Idx = unsigned;
  __amdgpu_buffer_rsrc_t t, w;
  uint32_t *c;
  __device__ VoxMem(const VolView &v) : c(v.rgb) {
    const size_t n = v.local_voxels();
    t = make_rsrc(v.tsdf, (unsigned)min(2 * n, (size_t)0xFFFFFFFFu));
    w = make_rsrc(v.weight, (unsigned)min(n, (size_t)0xFFFFFFFFu));
  }
  __device__ int16_t ld_t(Idx i) const { return __builtin_amdgcn_raw_buffer_load_b16(t, i << 1, 0, 0); }
  __device__ int16_t ld_w(Idx i) const { return (int16_t)__builtin_amdgcn_raw_buffer_load_b8(w, i, 0, 0); }
  __device__ uint32_t ld_c(Idx i) const { return c[i]; }  // only for voxels that pass
  __device__ void st_t(Idx i, int16_t x) const { __builtin_amdgcn_raw_buffer_store_b16(x, t, i << 1, 0, 0); }
  __device__ void st_w(Idx i, int16_t x) const { __builtin_amdgcn_raw_buffer_store_b8((uint8_t)x, w, i, 0, 0); }
  __device__ void st_c(Idx i, uint32_t x) const { c[i] = x; }
  static constexpr Idx kNone = 0x7FFFFFFFu;  // byte offsets past every buffer
};
template <>
struct VoxMem<false> {
  using Idx = size_t;
  int16_t *t;
  uint8_t *w;
  uint32_t *c;
  __device__ VoxMem(const VolView &v) : t(v.tsdf), w(v.weight), c(v.rgb) {}
  __device__ int16_t ld_t(Idx i) const { return t[i]; }
  __device__ int16_t ld_w(Idx i) const { return (int16_t)w[i]; }
  __device__ uint32_t ld_c(Idx i) const { return c[i]; }
  __device__ void st_t(Idx i, int16_t x) const { t[i] = x; }
  __device__ void st_w(Idx i, int16_t x) const { w[i] = (uint8_t)x; }
  __device__ void st_c(Idx i, uint32_t x) const { c[i] = x; }
  static constexpr Idx kNone = 0;  // rejected lanes read voxel 0 (never written by them)
};

// tsdf reads of k_raycast: kIdx32 (local volume < 2^31 voxels) uses a buffer
// load with a 32-bit byte offset (24-bit multiplies; rejected samples read 0
// past the buffer end without a memory access), else 64-bit pointers.
template <bool kIdx32>
struct RayMem;
template <>
struct RayMem<true> {
  __amdgpu_buffer_rsrc_t t;
  unsigned zn, tiles_x;
  int zb;
  __device__ RayMem(const VolView &v)
      : t(make_rsrc(v.tsdf, (unsigned)(2 * v.local_voxels()))), zn((unsigned)v.zn),
        tiles_x((unsigned)v.tiles_x), zb(v.zb) {}
  __device__ int16_t ld(bool valid, int x, int y, int z) const {
    const unsigned ux = (unsigned)x, uy = (unsigned)y;
    const unsigned tile = __umul24(uy >> 3, tiles_x) + (ux >> 3);
    const unsigned idx = ((__umul24(tile, zn) + (unsigned)(z - zb)) << 6) | ((uy & 7u) << 3 | (ux & 7u));
    return __builtin_amdgcn_raw_buffer_load_b16(t, valid ? idx * 2u : kOob, 0, 0);
  }
};
template <>
struct RayMem<false> {
  const VolView *v;
  __device__ RayMem(const VolView &vv) : v(&vv) {}
  __device__ int16_t ld(bool valid, int x, int y, int z) const {
    return valid ? v->tsdf[vox_index(*v, x, y, z)] : (int16_t)0;
  }
};

// One step of a long add chain (integrate's vc replay): the IEEE adds of the
// reference, kept as three scalar v_add_f32 chains — the compiler otherwise
// packs {x, y} into v_pk_add_f32, whose dependent latency makes such chains
// several times slower (tools/chain_bench.hip).
__device__ __forceinline__ f3 replay_add(f3 a, f3 b) {
  asm volatile("v_add_f32 %0, %0, %1" : "+v"(a.x) : "v"(b.x));
  asm volatile("v_add_f32 %0, %0, %1" : "+v"(a.y) : "v"(b.y));
  asm volatile("v_add_f32 %0, %0, %1" : "+v"(a.z) : "v"(b.z));
  return a;
}
// a advanced from slice z to slice za (za - z adds when za > z): the exact
// fast-forward of kfx_ffadd.h for long replays, the adds themselves (8 per
// trip) for short ones
__device__ __forceinline__ f3 replay(f3 a, f3 b, int z, int za, int ffmin = KFX_FF_MIN) {
  if (za - z >= ffmin) {
    a.x = ff_add(a.x, b.x, za - z);
    a.y = ff_add(a.y, b.y, za - z);
    a.z = ff_add(a.z, b.z, za - z);
    return a;
  }
  for (; z + 8 <= za; z += 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u) a = replay_add(a, b);
  }
  for (; z < za; ++z) a = replay_add(a, b);
  return a;
}

// Integrate's vol2cam pose of this frame (tsdf_volume.cpp:50) and the frame
// kind (2: reset); stage seams pass an explicit pose.
__device__ __forceinline__ int int_frame_pose(const DevState *st, const DevPose *log, const DevPose &vpose,
                                              const float *xpose, DevPose &P, DevPose &gp) {
  gp = pose_identity();
  if (xpose) {
    for (int i = 0; i < 9; ++i) P.R[i] = xpose[i];
    for (int i = 0; i < 3; ++i) P.t[i] = xpose[9 + i];
    return 1;
  }
  const int kind = frame_kind(st);
  if (kind != 2) {
    gp = frame_pose(st, log, kind);
    P = pose_mul(pose_inv(gp), vpose);
  }
  return kind;
}

// A column's vc at z = 0 and its per-z step (tsdf_volume.cu:53-55), and its
// conservative interval [zl, zh] of z where any check can pass (empty: zl > zh).
__device__ __forceinline__ void int_column(const VolView &v, const LevelGeom &g, const float2 *dl, const DevPose &P,
                                           int x, int y, f3 &vc, f3 &zs, int &zl, int &zh) {
  const f3 vx = {(float)x * v.vs[0], (float)y * v.vs[1], 0.f * v.vs[2]};
  vc = add(rmul(P.R, vx), {P.t[0], P.t[1], P.t[2]});
  zs = {P.R[2] * v.vs[0], P.R[5] * v.vs[0], P.R[8] * v.vs[0]};
  unsigned dm = 0u;  // the frame's max depth (k_preprocess_maps' shards)
  const unsigned *dmx = dmax_shards(dl, g);
#pragma unroll
  for (int i = 0; i < kDmaxShards; ++i) dm = max(dm, dmx[i]);
  const float dmax = __uint_as_float(dm);
  // global z = 1..Z-1 (tsdf_volume.cu:53), restricted to the stored slab
  // (the linear model vc0 + z zs of the accumulated vc, with 2 pixels and 2
  // slices of margin: the float accumulation drifts < 0.1 voxel over a column)
  const int lo0 = max(1, v.zb), hi0 = min(v.Z - 1, v.zb + v.zn - 1);
  float lo = (float)lo0, hi = (float)hi0;  // lo only grows, hi only shrinks: finite unless emptied
  {
    const float ax = vc.x, ay = vc.y, az = vc.z, sx = zs.x, sy = zs.y, sz = zs.z;
    const float M = 2.f;  // pixels
    clip_lin(az + 1e-3f, sz, lo, hi);  // vc.z > 0
    const float cxl = g.cx + 0.5f + M, cxh = (float)g.w - 0.5f + M - g.cx;
    const float cyl = g.cy + 0.5f + M, cyh = (float)g.h - 0.5f + M - g.cy;
    clip_lin(g.fx * ax + cxl * az, g.fx * sx + cxl * sz, lo, hi);
    clip_lin(cxh * az - g.fx * ax, cxh * sz - g.fx * sx, lo, hi);
    clip_lin(g.fy * ay + cyl * az, g.fy * sy + cyl * sz, lo, hi);
    clip_lin(cyh * az - g.fy * ay, cyh * sz - g.fy * sy, lo, hi);
    const float zfar = (dmax + v.trunc) * 1.02f + 0.01f;
    clip_lin(zfar - az, -sz, lo, hi);
  }
  zl = INT_MAX, zh = INT_MIN;
  if (hi >= lo) {
    zl = max(lo0, (int)floorf(lo) - 2);
    zh = min(hi0, (int)ceilf(hi) + 2);
    if (zh < zl) zl = INT_MAX, zh = INT_MIN;
  }
}

// Occlusion clip of a column tile's intervals (KFX_INT_OCCL).  A voxel can
// only be updated where its pixel's depth d satisfies d - il |vc| >= -trunc
// (tsdf_volume.cu:67-71), and il |vc| >= vc.z / 1.0011 for every in-image
// voxel, so no voxel with vc.z > (D + trunc) * 1.0011 is updated when D bounds
// the depth of every pixel it can project to.  The lanes' segments (linear vc
// model, as int_column) project into a pixel box; with 2 pixels of margin it
// covers every rounded projection, and when it spans at most kOcclCells cells
// of the frame's 16x16-pixel max-depth grid, D = their max replaces the
// frame-wide maximum in the far clip (the same form as int_column's).  Voxels
// behind every surface they project onto (a far Z-slab, the space behind a
// sphere) are then not visited at all; the result is unchanged (only voxels
// that cannot pass are dropped).  Lanes' [zl, zh] and the union [wl, wh] are
// tightened in place (wave-uniform control flow).
#ifndef KFX_INT_OCCL
#define KFX_INT_OCCL 1
#endif
#ifndef KFX_INT_OCCL_CELLS
#define KFX_INT_OCCL_CELLS 64
#endif
constexpr int kOcclCells = KFX_INT_OCCL_CELLS;
__device__ __forceinline__ void int_tile_clip(const VolView &v, const LevelGeom &g, const float2 *dl, f3 vc0, f3 zs,
                                              int lane, int &zl, int &zh, int &wl, int &wh) {
  if (!KFX_INT_OCCL || wh < wl) return;
  const bool own = zl <= zh;
  float umin = kInfF, umax = -kInfF, vmin = kInfF, vmax = -kInfF;
  bool bad = false;
  if (own) {
    const float z1 = (float)zl, z2 = (float)zh;
    const float pz1 = vc0.z + z1 * zs.z, pz2 = vc0.z + z2 * zs.z;
    bad = !(pz1 > 1e-3f) || !(pz2 > 1e-3f);
    const float i1 = __builtin_amdgcn_rcpf(pz1), i2 = __builtin_amdgcn_rcpf(pz2);
    const float u1 = g.fx * ((vc0.x + z1 * zs.x) * i1) + g.cx, u2 = g.fx * ((vc0.x + z2 * zs.x) * i2) + g.cx;
    const float w1 = g.fy * ((vc0.y + z1 * zs.y) * i1) + g.cy, w2 = g.fy * ((vc0.y + z2 * zs.y) * i2) + g.cy;
    umin = fminf(u1, u2);
    umax = fmaxf(u1, u2);
    vmin = fminf(w1, w2);
    vmax = fmaxf(w1, w2);
    bad = bad || isnan(umin + umax + vmin + vmax);
  }
  if (__any(bad)) return;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    umin = fminf(umin, __shfl_xor(umin, off));
    umax = fmaxf(umax, __shfl_xor(umax, off));
    vmin = fminf(vmin, __shfl_xor(vmin, off));
    vmax = fmaxf(vmax, __shfl_xor(vmax, off));
  }
  const int nbx = (g.w + 15) >> 4, nby = (g.h + 15) >> 4;
  // the box's cells, clamped to the image (margin: 2 px over the rounding)
  const float fu0 = fmaxf(umin - 2.5f, 0.f), fu1 = fminf(umax + 2.5f, (float)(g.w - 1));
  const float fv0 = fmaxf(vmin - 2.5f, 0.f), fv1 = fminf(vmax + 2.5f, (float)(g.h - 1));
  if (!(fu0 <= fu1) || !(fv0 <= fv1)) return;  // (the frustum clip already handles boxes off the image)
  const int cx0 = (int)fu0 >> 4, cx1 = (int)fu1 >> 4, cy0 = (int)fv0 >> 4, cy1 = (int)fv1 >> 4;
  const int nx = cx1 - cx0 + 1, ncell = nx * (cy1 - cy0 + 1);
  if (ncell > kOcclCells) return;  // a large footprint: the frame-wide bound stands
  unsigned dm = 0u;
  if (lane < ncell) dm = dmax_grid(dl, g)[(cy0 + lane / nx) * nbx + cx0 + lane % nx];
  (void)nby;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) dm = max(dm, (unsigned)__shfl_xor((int)dm, off));
  const float zfar = (__uint_as_float(dm) + v.trunc) * 1.02f + 0.01f;
  if (own) {
    float lo = (float)zl, hi = (float)zh;
    clip_lin(zfar - vc0.z, -zs.z, lo, hi);
    if (hi >= lo) {
      zh = min(zh, (int)ceilf(hi) + 2);
    } else {
      zl = INT_MAX;
      zh = INT_MIN;
    }
  }
  wl = zl;
  wh = zh;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    wl = min(wl, __shfl_xor(wl, off));
    wh = max(wh, __shfl_xor(wh, off));
  }
}

// Chunk `chunk` of the wave-uniform union interval [wl, wh] (wl <= wh):
// [za, zb], or false when this item has no chunk (length-capped mode).
__device__ __forceinline__ bool int_chunk(const VolView &v, int chunkr, int chunk, int nchunk, int wl, int wh,
                                          int &za, int &zb) {
  const int len = wh - wl + 1;
  if (v.iadapt == 1) {
    // length-capped: chunks of about zn / nchunk slices (a short interval
    // takes fewer; the surplus items, ordered last, exit)
    const int ct = min(nchunk, max(1, (int)(((long long)len * nchunk + v.zn - 1) / v.zn)));
    if (chunk >= ct) return false;
    za = wl + (int)((long long)len * chunk / ct);
    zb = wl + (int)((long long)len * (chunk + 1) / ct) - 1;
    return true;
  }
  if (chunkr >= 100) {  // equal chunks
    za = wl + (int)((long long)len * chunk / nchunk);
    zb = wl + (int)((long long)len * (chunk + 1) / nchunk) - 1;
    return true;
  }
  // chunk c gets weight r^c: the chunks dispatched last (highest item
  // index) are the shortest, so the kernel's tail waves are short
  const float r = (float)chunkr * 0.01f;
  const float den = 1.f - __powf(r, (float)nchunk);
  za = wl + (int)((float)len * ((1.f - __powf(r, (float)chunk)) / den));
  zb = chunk + 1 == nchunk ? wh : wl + (int)((float)len * ((1.f - __powf(r, (float)(chunk + 1))) / den)) - 1;
  return true;
}

// Work split: a wave owns an 8x8 tile of columns and one of gridDim.y z-chunks
// of every column's in-range interval (more waves per SIMD to hide latency);
// each lane replays the vc adds up to its chunk start, so every voxel's vc is
// the reference's bit for bit.
// kCount: count-only variant (no voxel traffic) giving N_upd / N_col, the
// algorithmic-byte inputs of the roofline.
// RN(1/d), d = 1..256 (RN(1/1) at 0), evaluated by the compiler (IEEE
// binary32 division, round to nearest): the same values as the per-block
// divisions it replaces
struct RcpTable {
  float v[257];
};
constexpr RcpTable make_rcp_table() {
  RcpTable t{};
  t.v[0] = 1.f;
  for (int i = 1; i < 257; ++i) t.v[i] = 1.f / (float)i;
  return t;
}
__constant__ RcpTable c_rtab = make_rcp_table();

template <bool kCount, bool kIdx32>
__global__ __launch_bounds__(KFX_INT_BLOCK) __attribute__((amdgpu_waves_per_eu(KFX_INT_OCC, KFX_INT_OCC))) void k_integrate(VolView v, LevelGeom g,
                                                   const float2 *__restrict__ dl,
                                                   const float *__restrict__ dmap,
                                                   const float *__restrict__ invl,
                                                   const uint8_t *__restrict__ bgr,
                                                   DevState *__restrict__ st, DevPose *log,
                                                   DevPose vpose, const float *xpose,
                                                   unsigned long long *counters) {
  // rtab[d] = RN(1/d), d = 1..256: the weight divisors of the running averages
  // (stored weights are u8, so pre_w + 1 <= 256 and no divisor falls outside)
  __shared__ float rtab[257];
  __shared__ DevPose s_pose;
  __shared__ int s_kind;
  for (int i = threadIdx.x; i < 257; i += KFX_INT_BLOCK) rtab[i] = c_rtab.v[i];
  if (threadIdx.x == 0) {  // (inline rather than int_frame_pose: that form spills in the loop)
    if (xpose) {  // stage seam: explicit vol2cam
      s_kind = 1;
      for (int i = 0; i < 9; ++i) s_pose.R[i] = xpose[i];
      for (int i = 0; i < 3; ++i) s_pose.t[i] = xpose[9 + i];
    } else {
      const int kind = frame_kind(st);
      s_kind = kind;
      DevPose gp = pose_identity();
      if (kind == 1 && blockIdx.x != 0 && st->int_tag == st->frame_serial) {
        s_pose = st->int_v2c;  // composed once by the persistent ICP (DevState::int_v2c)
      } else if (kind != 2) {
        gp = frame_pose(st, log, kind);
        s_pose = pose_mul(pose_inv(gp), vpose);  // tsdf_volume.cpp:50
      }
      if (!kCount && blockIdx.x == 0) {
        frame_bookkeeping(st, log, kind, gp);
        // the raycast after this integrate reads its pose from here (no
        // per-block pose math or LDS round trip on its critical path);
        // frame_kind / frame_pose read fields the bookkeeping leaves alone
        st->ray_kind = kind;
        if (kind == 1) st->ray_c2v = pose_mul(pose_inv(vpose), gp);  // tsdf_volume.cpp:59
      }
    }
  }
  __syncthreads();
#ifdef KFX_INT_TRACE
  const unsigned long long t_start = wall_clock64();
#endif
  static_assert(KFX_INT_BLOCK == 64, "one wave per block: block b runs item iperm[b]");
  const int lane = threadIdx.x & 63;
  const int ntiles = v.tiles_x * v.tiles_y, nchunk = v.inchunk;
  const unsigned item = v.iperm ? v.iperm[blockIdx.x] : blockIdx.x;  // chunk * tiles + tile
  const int tile = (int)(item % (unsigned)ntiles), chunk = (int)(item / (unsigned)ntiles);
  if (chunk >= nchunk) return;
  const int x = (tile % v.tiles_x) * 8 + (lane & 7);
  const int y = (tile / v.tiles_x) * 8 + (lane >> 3);
  const size_t base = (size_t)tile * v.tile_voxels() + lane;  // this column's (x, y, zb)
  if (s_kind == 2) {  // reset(): whole volume zeroed (A5 D)
    if (kCount) return;
    const int z0 = (int)((long long)v.zn * chunk / nchunk);
    const int z1 = (int)((long long)v.zn * (chunk + 1) / nchunk);
    for (int z = z0; z < z1; ++z) {  // local slices
      const size_t i = base + (size_t)z * 64;
      v.tsdf[i] = 0;
      v.weight[i] = 0;
      v.rgb[i] = 0u;
    }
    if (chunk == 0) {  // the zeroed volume holds no negative tsdf
      for (int i = lane; i < v.bw; i += 64) v.bocc[(size_t)tile * v.bw + i] = 0ull;
      const int tx = tile % v.tiles_x, ty = tile / v.tiles_x;
      if ((tx & 3) == 0 && (ty & 3) == 0)
        for (int i = lane; i < v.sw; i += 64) v.socc[(size_t)((ty >> 2) * v.stx + (tx >> 2)) * v.sw + i] = 0u;
    }
    return;
  }
  const DevPose P = s_pose;
  f3 vc, zs;
  int zl, zh, za, zb, z;
  int_column(v, g, dl, P, x, y, vc, zs, zl, zh);
  // The wave takes a chunk of the UNION of its lanes' intervals, so all 64
  // lanes step the same z and each voxel load / store of the wave is one
  // 128-B line (per-lane intervals put the lanes on different slices: one
  // line per lane); a lane only updates voxels inside its own interval.
  int wl = zl, wh = zh;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    wl = min(wl, __shfl_xor(wl, off));
    wh = max(wh, __shfl_xor(wh, off));
  }
  int_tile_clip(v, g, dl, vc, zs, lane, zl, zh, wl, wh);
  // the next frame's dispatch order (k_int_order) from this interval length
  if (!kCount && chunk == 0 && lane == 0 && v.iwork) v.iwork[tile] = wh >= wl ? (unsigned)(wh - wl + 1) : 0u;
  if (wh < wl || !int_chunk(v, KFX_INT_CHUNKR, chunk, nchunk, wl, wh, za, zb)) return;  // wave-uniform
  // (uniform by construction: tell the compiler, so that the z loop and the
  // replay run on the scalar unit)
  za = __builtin_amdgcn_readfirstlane(za);
  zb = __builtin_amdgcn_readfirstlane(zb);
  z = 1;
  // (Z-slabs: the fast-forward from a lower count, KFX_FF_MIN_SLAB — every
  // chunk of a far slab replays its column from z = 1)
  vc = replay(vc, zs, z, za, v.zb > 0 ? KFX_FF_MIN_SLAB : KFX_FF_MIN);
  z = max(z, za);
  const int la = max(za, zl), lb = min(zb, zh);  // this lane's voxels of the chunk
  const bool live = lb >= la;
  if (__all(!live)) return;

  const float trunc = v.trunc;
  const float thres_color = trunc / 2;
  // kCount: updated, coloured, visited, gathered voxels; wave batches
  unsigned cu = 0, cc = 0, cv = 0, cg = 0, cb = 0;
  // negative tsdf this lane wrote: bricks gbs .. gbs+61 as bits, beyond as a z range
  const int gbs = za >> 3;
  unsigned long long nbm = 0ull;
  int nlo = INT_MAX, nhi = -1;
  using Mem = VoxMem<kIdx32>;
  using Idx = typename Mem::Idx;
  const Mem mem(v);
  constexpr unsigned kPixB = 8u, kPixSh = 3u;
  const __amdgpu_buffer_rsrc_t rdl = make_rsrc(dl, (unsigned)(8 * g.w * g.h));
  (void)dmap;
  (void)invl;
  constexpr Idx slice = 64;  // index step per z (tile-column layout)
  Idx iz = (Idx)base + (Idx)(za - v.zb) * slice;  // voxel index of (x, y, z)
  const bool fastw = __all(!live || column_fast(vc, zs, v.Z));  // wave-uniform
  const float fw = (float)g.w, fh = (float)g.h;
  // Batches of kB voxels: positions, projections, the kB {depth, 1/lambda}
  // gathers, then the kB tsdf/weight loads are issued back to back
  // (memory-level parallelism); each voxel's arithmetic is exactly the
  // reference's (tsdf_volume.cu:56-98).
  constexpr int kB = KFX_INT_KB;
  // The z loop is instantiated once per path (fast: the packed exact
  // sequences; else IEEE division and sqrt) and the wave picks one: the fast
  // loop then carries no code or registers of the other (integrate −2 %,
  // six alternating pairs, against one loop branching on `fast` per batch).
  auto zloop = [&](auto fast_c) {
    constexpr bool fast = decltype(fast_c)::value;
  for (; z <= zb; z += kB) {
    float sdf[kB];
    unsigned pix[kB];
    bool ok[kB];
    f3 p[kB];
#pragma unroll
    for (int j = 0; j < kB; ++j) {
      vc = add(vc, zs);
      p[j] = vc;
    }
    // projection: ok = in the image in front of the camera (tsdf_volume.cu:56-66)
    if constexpr (fast) {  // the cheap exact sequences, two voxels per packed-FP32 op
      static_assert(kB % 2 == 0, "voxel pairs");
#pragma unroll
      for (int j = 0; j < kB; j += 2) {
        const ipf2 pz = {p[j].z, p[j + 1].z};
        const ipf2 yv = rcp_rn2(pz);
        const ipf2 px = {p[j].x, p[j + 1].x}, py = {p[j].y, p[j + 1].y};
        const ipf2 uu = div_rn2(px, pz, yv) * ipf2{g.fx, g.fx} + ipf2{g.cx, g.cx};
        const ipf2 vv = div_rn2(py, pz, yv) * ipf2{g.fy, g.fy} + ipf2{g.cy, g.cy};
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          // uu, vv are finite here (|vc| components in {0} u [2^-40, 2^40]).
          // rintf by the 1.5 * 2^23 bias: for |u| < 2^22 the biased sum has
          // ulp 1 and its integer (ties to even: the bias is even) is
          // rintf(u); u >= 2^22 unbiases to >= 2^22, u <= -2^22 to a negative
          // value, so one unsigned compare per axis is still the range test
          // [0, w) of rintf(u); 24-bit multiply (w, h < 2^24)
          const int iu = (int)(__float_as_uint(uu[k] + 12582912.f) - 0x4B400000u);
          const int iv = (int)(__float_as_uint(vv[k] + 12582912.f) - 0x4B400000u);
          ok[j + k] = (z + j + k >= la) & (z + j + k <= lb) & (pz[k] > 0) & ((unsigned)iu < (unsigned)g.w) & ((unsigned)iv < (unsigned)g.h);
          pix[j + k] = ok[j + k] ? __umul24((unsigned)iv, kPixB * (unsigned)g.w) + ((unsigned)iu << kPixSh) : kOob;
        }
      }
    } else {  // IEEE division (tiny or huge operands)
#pragma unroll
      for (int j = 0; j < kB; ++j) {
        const float uf = rintf((p[j].x / p[j].z) * g.fx + g.cx);
        const float vf = rintf((p[j].y / p[j].z) * g.fy + g.cy);
        ok[j] = (z + j >= la) & (z + j <= lb) & (p[j].z > 0) & (uf >= 0.f) & (uf < fw) & (vf >= 0.f) & (vf < fh);
        pix[j] = ok[j] ? ((unsigned)(int)vf * (unsigned)g.w + (unsigned)(int)uf) * kPixB : kOob;
      }
    }
    float2 d[kB];
    float n2[kB];
#pragma unroll
    for (int j = 0; j < kB; ++j) n2[j] = dot(p[j], p[j]);
#pragma unroll
    for (int j = 0; j < kB; ++j)
      d[j] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(rdl, pix[j], 0, 0));
    // sdf and the depth test (tsdf_volume.cu:67-71)
    if constexpr (fast) {
#pragma unroll
      for (int j = 0; j < kB; j += 2) {
        // d - il |vc| = -(il |vc| - d) exactly (RN is odd-symmetric); only the
        // sign of a zero sdf can differ, and no result depends on it
        const ipf2 sd = ipf2{d[j].x, d[j + 1].x} - ipf2{d[j].y, d[j + 1].y} * sqrt_rn2(ipf2{n2[j], n2[j + 1]});
        sdf[j] = sd.x;
        sdf[j + 1] = sd.y;
      }
    } else {
#pragma unroll
      for (int j = 0; j < kB; ++j) sdf[j] = -(d[j].y * sqrtf(n2[j]) - d[j].x);
    }
#pragma unroll
    for (int j = 0; j < kB; ++j) ok[j] = ok[j] & (d[j].x > 0) & (sdf[j] >= -trunc);
    if (kCount) {
      iz += (Idx)kB * slice;
      ++cb;
#pragma unroll
      for (int j = 0; j < kB; ++j) {
        cv += (z + j >= la) & (z + j <= lb);
        cg += (pix[j] != kOob);
      }
#pragma unroll
      for (int j = 0; j < kB; ++j)
        if (ok[j]) {
          ++cu;
          if (sdf[j] <= thres_color && sdf[j] >= -thres_color) ++cc;
        }
      continue;
    }
#if KFX_INT_BSKIP
    // a batch in which no voxel of any lane passes (behind the surfaces, out
    // of the image): no loads, update arithmetic or stores (wave-uniform)
    bool anyok = false;
#pragma unroll
    for (int j = 0; j < kB; ++j) anyok = anyok | ok[j];
    if (!__any(anyok)) {
      iz += (Idx)kB * slice;
      continue;
    }
#endif
    // tsdf/weight of the voxels that pass (issuing them with the depth
    // gathers, before the depth test, measured slower: the rejected voxels'
    // extra reads cost more than the saved round trip)
    int16_t t0[kB], w0[kB];
    Idx vi[kB];
#pragma unroll
    for (int j = 0; j < kB; ++j) {
      vi[j] = iz + (Idx)j * slice;
      const Idx i = ok[j] ? vi[j] : Mem::kNone;
      t0[j] = mem.ld_t(i);
      w0[j] = mem.ld_w(i);
    }
#if KFX_INT_LDALL
    // all kB voxels' loads issued together, one wait: the compiler otherwise
    // sinks a voxel's loads into its update branch (the loaded values are
    // only used there), which puts them on a round trip of their own
#pragma unroll
    for (int j = 0; j < kB; ++j) asm volatile("" ::"v"(t0[j]), "v"(w0[j]));
#endif
    iz += (Idx)kB * slice;
    // The update arithmetic of all kB voxels, two voxels per packed op and
    // without branches (voxels that do not pass compute values nobody
    // stores).  A saturated voxel (w = 64 at the tsdf fixed point T* of a
    // ts = 1 update, sdf >= trunc) needs no test: its update reproduces the
    // stored values, so the changed-value tests below skip its stores.
    int qv[kB];
#pragma unroll
    for (int j = 0; j < kB; j += 2) {
      const ipf2 tq = div_rn2(ipf2{sdf[j], sdf[j + 1]}, ipf2{trunc, trunc}, ipf2{v.inv_trunc, v.inv_trunc});
      const ipf2 ts = {fminf(1.f, tq.x), fminf(1.f, tq.y)};
      const ipf2 pt = ipf2{(float)t0[j], (float)t0[j + 1]} * ipf2{kDivShortMax, kDivShortMax};
      const ipf2 pw = {(float)w0[j], (float)w0[j + 1]};
      const ipf2 nt = div_rn2(pfma(pt, pw, ts), pw + ipf2{1.f, 1.f}, ipf2{rtab[w0[j] + 1], rtab[w0[j + 1] + 1]}) *
                     ipf2{(float)kShortMax, (float)kShortMax};
#pragma unroll
      for (int k = 0; k < 2; ++k) qv[j + k] = max(-kShortMax, min(kShortMax, (int)nt[k]));
    }
#pragma unroll
    for (int j = 0; j < kB; ++j) {
      if (!ok[j]) continue;
      const Idx i = vi[j];
      const int pre_w = w0[j];
      const int new_w = min(pre_w + 1, kMaxWeight);
      const int q = qv[j];
      if (q < 0) {
        const int k = ((z + j) >> 3) - gbs;
        if (k < 62) {
          nbm |= 1ull << k;
        } else {
          nlo = min(nlo, z + j);
          nhi = max(nhi, z + j);
        }
      }
      // saturated voxels (w = 64 at a tsdf fixed point) keep their values:
      // skipping those stores changes nothing and saves write bandwidth
      if (q != t0[j]) mem.st_t(i, (int16_t)q);
      if (new_w != pre_w) mem.st_w(i, (int16_t)new_w);
      if (sdf[j] <= thres_color && sdf[j] >= -thres_color) {  // colour band (rare)
        const uint32_t c0 = mem.ld_c(i);
        const uint8_t *px = bgr + 3 * (size_t)(pix[j] >> kPixSh);
        const float c = (float)(new_w + 1);
        const float rc = rtab[new_w + 1];
        uint32_t out = 0u;
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
          const int m0 = (int)((c0 >> (8 * ch)) & 0xffu);
          const float m = (float)(new_w * m0 + (int)px[ch]);
          out |= (uint32_t)(uint8_t)div_rn(m, c, rc) << (8 * ch);
        }
        if (out != c0) mem.st_c(i, out);
      }
    }
  }
  };
  if (fastw) zloop(std::true_type{});
  else zloop(std::false_type{});
  if (!kCount) {  // raycast skip maps
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const unsigned lo = __shfl_xor((unsigned)nbm, off), hi = __shfl_xor((unsigned)(nbm >> 32), off);
      nbm |= ((unsigned long long)hi << 32) | lo;
    }
    occ_mark_bricks(v, tile, gbs, nbm, lane);
    occ_mark_wave(v, tile, nlo, nhi, lane);
  }
#ifdef KFX_INT_TRACE
  if (!kCount && counters && lane == 0) {  // debug: per-wave timeline
    unsigned long long *r = counters + 4 * (size_t)blockIdx.x;
    r[0] = t_start;
    r[1] = wall_clock64();
    r[2] = ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32) |
           (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);
    r[3] = (unsigned long long)tile | ((unsigned long long)chunk << 32);
  }
#endif
  if (kCount) {
    const int sh = (blockIdx.x + blockIdx.y) % 16;
    atomicAdd(&counters[2 * sh], (unsigned long long)cu);
    atomicAdd(&counters[2 * sh + 1], (unsigned long long)cc);
    atomicAdd(&counters[32 + sh], (unsigned long long)cv);
    atomicAdd(&counters[48 + sh], (unsigned long long)cg);
    if (lane == 0) atomicAdd(&counters[64 + sh], (unsigned long long)cb);  // per-wave count (wave-uniform)
  }
}

// ---------------------------------------------------------------------------
// Raycast — raycasthelper (tsdf_volume.cu:120-260)

struct RayConsts {
  f3 vs, vs_inv, gd;
  float step;
  float skip_cap;  // most samples one skip replays (accumulated rounding < 0.1 voxel)
};

__device__ __forceinline__ float voxel2tsdf(const VolView &v, const RayConsts &rc, f3 p) {
  const int x = f2i_rn(p.x * rc.vs_inv.x);
  const int y = f2i_rn(p.y * rc.vs_inv.y);
  const int z = f2i_rn(p.z * rc.vs_inv.z);
  if (x >= v.X - 1 || y >= v.Y - 1 || z >= v.Z - 1 || x < 1 || y < 1 || z < 1) return NAN;
  if ((unsigned)(z - v.zb) >= (unsigned)v.zn) return NAN;  // not stored on this slab
  return (float)v.tsdf[vox_index(v, x, y, z)] * kDivShortMax;
}

__device__ __forceinline__ float interp(const VolView &v, f3 cf) {
  const int gx = f2i_rd(cf.x), gy = f2i_rd(cf.y), gz = f2i_rd(cf.z);
  if (gx < 0 || gx >= v.X - 1 || gy < 0 || gy >= v.Y - 1 || gz < 0 || gz >= v.Z - 1) return NAN;
  // slabs: an owned event's normal reads within the stored halo (DESIGN.md
  // §7); the check only keeps any other read in bounds
  if ((unsigned)(gz - v.zb) >= (unsigned)(v.zn - 1)) return NAN;
  const float a = cf.x - (float)gx, b = cf.y - (float)gy, c = cf.z - (float)gz;
  const float t000 = (float)v.tsdf[vox_index(v, gx, gy, gz)] * kDivShortMax;
  const float t001 = (float)v.tsdf[vox_index(v, gx, gy, gz + 1)] * kDivShortMax;
  const float t010 = (float)v.tsdf[vox_index(v, gx, gy + 1, gz)] * kDivShortMax;
  const float t011 = (float)v.tsdf[vox_index(v, gx, gy + 1, gz + 1)] * kDivShortMax;
  const float t100 = (float)v.tsdf[vox_index(v, gx + 1, gy, gz)] * kDivShortMax;
  const float t101 = (float)v.tsdf[vox_index(v, gx + 1, gy, gz + 1)] * kDivShortMax;
  const float t110 = (float)v.tsdf[vox_index(v, gx + 1, gy + 1, gz)] * kDivShortMax;
  const float t111 = (float)v.tsdf[vox_index(v, gx + 1, gy + 1, gz + 1)] * kDivShortMax;
  float s = 0.f;
  s += t000 * (1 - a) * (1 - b) * (1 - c);
  s += t001 * (1 - a) * (1 - b) * c;
  s += t010 * (1 - a) * b * (1 - c);
  s += t011 * (1 - a) * b * c;
  s += t100 * a * (1 - b) * (1 - c);
  s += t101 * a * (1 - b) * c;
  s += t110 * a * b * (1 - c);
  s += t111 * a * b * c;
  return s;
}

// interp for volumes whose local voxel count fits 32-bit offsets (k_raycast's
// kIdx32): the same corners, weights and sum order, but one tile-column index
// for (gx, gy, gz) and the other seven corners as offsets from it (z + 1 is
// always the next 64-voxel slice of the same column; x + 1 / y + 1 cross into
// the next tile only at x & 7 == 7 / y & 7 == 7), read by buffer loads.
__device__ __forceinline__ float interp32(const VolView &v, __amdgpu_buffer_rsrc_t t, f3 cf) {
  const int gx = f2i_rd(cf.x), gy = f2i_rd(cf.y), gz = f2i_rd(cf.z);
  if (gx < 0 || gx >= v.X - 1 || gy < 0 || gy >= v.Y - 1 || gz < 0 || gz >= v.Z - 1) return NAN;
  if ((unsigned)(gz - v.zb) >= (unsigned)(v.zn - 1)) return NAN;
  const float a = cf.x - (float)gx, b = cf.y - (float)gy, c = cf.z - (float)gz;
  const unsigned col = (unsigned)v.zn << 6;  // voxels per tile column
  const unsigned tile = __umul24((unsigned)gy >> 3, (unsigned)v.tiles_x) + ((unsigned)gx >> 3);
  const unsigned i0 = ((tile * (unsigned)v.zn + (unsigned)(gz - v.zb)) << 6) | (((unsigned)gy & 7u) << 3 | ((unsigned)gx & 7u));
  const unsigned dx = (gx & 7) == 7 ? col - 7u : 1u;
  const unsigned dy = (gy & 7) == 7 ? __umul24((unsigned)v.tiles_x, col) - 56u : 8u;
  auto ld = [&](unsigned i) {
    return (float)(int16_t)__builtin_amdgcn_raw_buffer_load_b16(t, i << 1, 0, 0) * kDivShortMax;
  };
  const float t000 = ld(i0), t001 = ld(i0 + 64u), t010 = ld(i0 + dy), t011 = ld(i0 + dy + 64u);
  const float t100 = ld(i0 + dx), t101 = ld(i0 + dx + 64u), t110 = ld(i0 + dx + dy), t111 = ld(i0 + dx + dy + 64u);
  float s = 0.f;
  s += t000 * (1 - a) * (1 - b) * (1 - c);
  s += t001 * (1 - a) * (1 - b) * c;
  s += t010 * (1 - a) * b * (1 - c);
  s += t011 * (1 - a) * b * c;
  s += t100 * a * (1 - b) * (1 - c);
  s += t101 * a * (1 - b) * c;
  s += t110 * a * b * (1 - c);
  s += t111 * a * b * c;
  return s;
}

// The 6 trilinear interpolations of compute_normal (kIdx32 volumes) with the
// loads of kG interpolations in flight together (KFX_RAY_NG: 1 = one round trip
// per interpolation, 6 = all 48 corner loads in one): the same corners,
// weights and sum order as interp32.
#ifndef KFX_RAY_NG
#define KFX_RAY_NG 1
#endif
template <int kG>
__device__ __forceinline__ f3 compute_normal_g(const VolView &v, const RayConsts &rc, f3 p) {
  const __amdgpu_buffer_rsrc_t t = make_rsrc(v.tsdf, (unsigned)(2 * v.local_voxels()));
  const unsigned col = (unsigned)v.zn << 6;
  float f[6];
#pragma unroll
  for (int g0 = 0; g0 < 6; g0 += kG) {
    int16_t raw[kG][8];
    bool ok[kG];
#pragma unroll
    for (int q = 0; q < kG; ++q) {
      const int k = g0 + q, ax = k >> 1;
      const float sgn = (k & 1) ? -1.f : 1.f;
      const f3 pq = {ax == 0 ? p.x + sgn * rc.gd.x : p.x, ax == 1 ? p.y + sgn * rc.gd.y : p.y,
                     ax == 2 ? p.z + sgn * rc.gd.z : p.z};
      const f3 cf = mulc(pq, rc.vs_inv);
      const int gx = f2i_rd(cf.x), gy = f2i_rd(cf.y), gz = f2i_rd(cf.z);
      ok[q] = !(gx < 0 || gx >= v.X - 1 || gy < 0 || gy >= v.Y - 1 || gz < 0 || gz >= v.Z - 1) &&
              (unsigned)(gz - v.zb) < (unsigned)(v.zn - 1);
      const unsigned tile = __umul24((unsigned)gy >> 3, (unsigned)v.tiles_x) + ((unsigned)gx >> 3);
      const unsigned i0 = ok[q] ? (((tile * (unsigned)v.zn + (unsigned)(gz - v.zb)) << 6) |
                                   (((unsigned)gy & 7u) << 3 | ((unsigned)gx & 7u)))
                                : 0u;
      const unsigned dx = (gx & 7) == 7 ? col - 7u : 1u;
      const unsigned dy = (gy & 7) == 7 ? __umul24((unsigned)v.tiles_x, col) - 56u : 8u;
      const unsigned o[8] = {i0, i0 + 64u, i0 + dy, i0 + dy + 64u, i0 + dx, i0 + dx + 64u, i0 + dx + dy,
                             i0 + dx + dy + 64u};
#pragma unroll
      for (int c = 0; c < 8; ++c)
        raw[q][c] = ok[q] ? (int16_t)__builtin_amdgcn_raw_buffer_load_b16(t, o[c] << 1, 0, 0) : (int16_t)0;
    }
#pragma unroll
    for (int q = 0; q < kG; ++q) {
      const int k = g0 + q, ax = k >> 1;
      const float sgn = (k & 1) ? -1.f : 1.f;
      const f3 pq = {ax == 0 ? p.x + sgn * rc.gd.x : p.x, ax == 1 ? p.y + sgn * rc.gd.y : p.y,
                     ax == 2 ? p.z + sgn * rc.gd.z : p.z};
      const f3 cf = mulc(pq, rc.vs_inv);
      const int gx = f2i_rd(cf.x), gy = f2i_rd(cf.y), gz = f2i_rd(cf.z);
      const float a = cf.x - (float)gx, b = cf.y - (float)gy, c = cf.z - (float)gz;
      auto T = [&](int i) { return (float)raw[q][i] * kDivShortMax; };
      float s = 0.f;
      s += T(0) * (1 - a) * (1 - b) * (1 - c);
      s += T(1) * (1 - a) * (1 - b) * c;
      s += T(2) * (1 - a) * b * (1 - c);
      s += T(3) * (1 - a) * b * c;
      s += T(4) * a * (1 - b) * (1 - c);
      s += T(5) * a * (1 - b) * c;
      s += T(6) * a * b * (1 - c);
      s += T(7) * a * b * c;
      f[k] = ok[q] ? s : NAN;
    }
  }
  f3 n;
  n.x = (f[0] - f[1]) / rc.gd.x;
  n.y = (f[2] - f[3]) / rc.gd.y;
  n.z = (f[4] - f[5]) / rc.gd.z;
  return normalized(n);
}

template <bool kIdx32 = false>
__device__ f3 compute_normal(const VolView &v, const RayConsts &rc, f3 p) {
  if constexpr (kIdx32 && KFX_RAY_NG > 1) return compute_normal_g<KFX_RAY_NG>(v, rc, p);
  const __amdgpu_buffer_rsrc_t t = make_rsrc(v.tsdf, kIdx32 ? (unsigned)(2 * v.local_voxels()) : 0u);
  auto ip = [&](f3 q) { return kIdx32 ? interp32(v, t, mulc(q, rc.vs_inv)) : interp(v, mulc(q, rc.vs_inv)); };
  f3 n;
  const float fx1 = ip({p.x + rc.gd.x, p.y, p.z});
  const float fx2 = ip({p.x - rc.gd.x, p.y, p.z});
  n.x = (fx1 - fx2) / rc.gd.x;
  const float fy1 = ip({p.x, p.y + rc.gd.y, p.z});
  const float fy2 = ip({p.x, p.y - rc.gd.y, p.z});
  n.y = (fy1 - fy2) / rc.gd.y;
  const float fz1 = ip({p.x, p.y, p.z + rc.gd.z});
  const float fz2 = ip({p.x, p.y, p.z - rc.gd.z});
  n.z = (fz1 - fz2) / rc.gd.z;
  return normalized(n);
}

// One wave = an 8x8 pixel tile (rays of a wave sample neighbouring voxels).
// BOOT frames copy the measured level-0 maps instead (kinectfusion.cpp:88-89).

template <bool kIdx32>
__device__ __forceinline__ size_t ray_index(const VolView &v, int x, int y, int z) {
  if (kIdx32)
    return (size_t)(((((unsigned)(y >> 3) * (unsigned)v.tiles_x + (unsigned)(x >> 3)) * (unsigned)v.zn +
                      (unsigned)(z - v.zb)) << 6) |
                    (unsigned)(((y & 7) << 3) | (x & 7)));
  return vox_index(v, x, y, z);
}

struct RayArgs {
  LevelGeom g[kMaxLevels];
  int levels;
  unsigned long long *stats;  // k_raycast<.., kStats>: 6 counters
  // kSlab: 0 unbounded march; 1 bounded by the previous frame's model
  // distance (+ margin); 2 resume: re-march unbounded the pixels whose pass-1
  // bound left them unresolved (kmin: the MIN-reduced [keys | pend] planes)
  int slab_pass;
  const uint32_t *kmin;
  float bound_abs, bound_rel;  // pass-1 margin: metres, fraction of the distance
  // start signal (overlapped frames, kfx_api.hip enqueue_frame_overlap): the
  // first wave of block 0 stores start_val to *start_sig (fine-grained device
  // memory, system scope; relaxed: it orders nothing, the launch itself implies
  // the integrate before it is complete) as the launch begins; the preprocess stream waits
  // for it (hipStreamWaitValue32) instead of an event record on this stream
  unsigned *start_sig;
  unsigned start_val;
};

__device__ void resize_tile(const RayArgs &ra, int kind, int tx0, int ty0, int lx, int ly, f3 vout,
                            f3 nout, const FrameView &cur, const FrameView &prev);

// kSlab (Z-slab sharding): the context stores slices
// [zb, zb+zn) and owns [own0, own1).  Every sample position is still the
// reference's accumulated one, but only samples whose nearest voxel lies in the
// owned slices may end the ray here; the first such event's sample index is
// written to keys[] (UINT_MAX: none) with its maps, and the ranks' results are
// combined by an all-reduce MIN over keys (the earliest event along the ray is
// the reference's result; each sample has exactly one owner).  The event at
// sample i reads samples i-1 and i and the trilinear normal at most 4 slices
// from sample i, all inside the stored halo.  Resize runs after the combine.
// Samples a ray may replay from voxel position c while every sample stays in
// the box that a clear dilated (super)brick run guarantees non-negative or
// NaN: per axis [B*b - B, B*b + 2B - 1] (open at the volume's edge columns),
// z [zl, zh]; each face with 0.2 voxel of margin (rint reaches a voxel only
// within 0.5 of it, the accumulated rounding of <= 511 adds stays below 0.1).
constexpr float kInf = __builtin_huge_valf();
__device__ __forceinline__ float axis_limit(float c, float d, float id, float lo, float hi) {
  return d > 0.f ? (hi + 0.2f - c) * id : (d < 0.f ? (c - lo + 0.2f) * id : kInf);
}
__device__ __forceinline__ float box_limit(int B, int bx, int by, int nbx, int nby, float zl, float zh,
                                           float cx, float cy, float cz, f3 dv, f3 idv) {
  const float xl = bx > 0 ? (float)(B * bx - B) : -kInf, xh = bx < nbx - 1 ? (float)(B * bx + 2 * B - 1) : kInf;
  const float yl = by > 0 ? (float)(B * by - B) : -kInf, yh = by < nby - 1 ? (float)(B * by + 2 * B - 1) : kInf;
  return fminf(fminf(axis_limit(cx, dv.x, idv.x, xl, xh), axis_limit(cy, dv.y, idv.y, yl, yh)),
               axis_limit(cz, dv.z, idv.z, zl, zh));
}

// n repeated adds p += s per component, exactly (kfx_ffadd.h)
__device__ __forceinline__ f3 ff_add3(f3 p, f3 s, int n) {
  return {ff_add_fast(p.x, s.x, n), ff_add_fast(p.y, s.y, n), ff_add_fast(p.z, s.z, n)};
}
#ifndef KFX_RAY_EXIT
#define KFX_RAY_EXIT 1  // a ray whose remaining samples all lie in a clear box ends there
#endif
#ifndef KFX_RAY_CHAIN
#define KFX_RAY_CHAIN 2  // skip lookups: boxes per round trip (1 or 2)
#endif
// The brick box's lateral (x / y) exit from voxel position (cx, cy) in cell (bx, by).
__device__ __forceinline__ float brick_lateral_exit(const VolView &v, int bx, int by, float cx, float cy, f3 dv, f3 idv) {
  const float xl = bx > 0 ? (float)(8 * bx - 8) : -kInf, xh = bx < v.tiles_x - 1 ? (float)(8 * bx + 15) : kInf;
  const float yl = by > 0 ? (float)(8 * by - 8) : -kInf, yh = by < v.tiles_y - 1 ? (float)(8 * by + 15) : kInf;
  return fminf(axis_limit(cx, dv.x, idv.x, xl, xh), axis_limit(cy, dv.y, idv.y, yl, yh));
}
// The clear box of a brick column word at voxel position (cx, cy, cz) of cell
// (bx, by, lbz): the cell's 3x3 tile box with the dilated z run of clear cells
// in the direction of travel (lim < 1: blocked).
__device__ __forceinline__ float run_box(const VolView &v, unsigned long long w, int nbits, int b, int lc, int ncell,
                                         int c0, int B, int bx, int by, int nbx, int nby, float cx, float cy, float cz,
                                         f3 dv, f3 idv) {
  float zl = -kInf, zh = kInf;
  if (dv.z > 0.f) {
    const unsigned long long up = w >> b;
    const int top = lc + (up ? __builtin_ctzll(up) : nbits - b) - 1;
    if (top < ncell - 1) zh = (float)(B * (top + c0) + 2 * B - 1);
  } else {
    const unsigned long long dn = w << (63 - b);
    const int bot = lc - (dn ? __builtin_clzll(dn) : b + 1) + 1;
    if (bot > 0) zl = (float)(B * (bot + c0) - B);
  }
  return box_limit(B, bx, by, nbx, nby, zl, zh, cx, cy, cz, dv, idv);
}
// Samples a ray may replay from voxel position (cx, cy, cz) (< 1: blocked).
// The super-brick's box when its cell is clear (its 3x3 box contains the
// brick's laterally; tools/raysim: the brick box alone adds < 1 % of lookups
// there), else the brick's.  KFX_RAY_CHAIN 2: the words of the column at the
// brick box's lateral exit point (known before any word is back) are loaded
// in the same round trip, and that column's brick box extends the run when
// the point lies inside it (a ray along a tilted surface leaves the boxes
// sideways one after another: tools/raysim variant 8, C2's slowest wave 54
// -> 36 lookup rounds).  Every sample of the run lies in one of the boxes at
// model positions c + t dv: the same 0.2-voxel margins as one box.
__device__ __forceinline__ float skip_limit(const VolView &v, float cx, float cy, float cz, f3 dv, f3 idv) {
  const int ix = (int)floorf(cx), iy = (int)floorf(cy), iz = (int)floorf(cz);
  const int bx = min(max(ix >> 3, 0), v.tiles_x - 1), by = min(max(iy >> 3, 0), v.tiles_y - 1);
  const int lbz = min(max((iz >> 3) - v.bz0, 0), v.nbz - 1);
  const int sx = min(max(ix >> 5, 0), v.stx - 1), sy = min(max(iy >> 5, 0), v.sty - 1);
  const int lsz = min(max((iz >> 5) - v.sz0, 0), v.nsz - 1);
  const unsigned long long bwd = v.bocc[(size_t)(by * v.tiles_x + bx) * v.bw + (lbz >> 6)];
  const uint32_t swd = v.socc[(size_t)(sy * v.stx + sx) * v.sw + (lsz >> 5)];
#if KFX_RAY_CHAIN >= 2
  const float t1r = brick_lateral_exit(v, bx, by, cx, cy, dv, idv);
  const float t1 = t1r < 1.0e6f ? t1r : 0.f;  // (no lateral exit: the same column, unused)
  const float c1x = cx + t1 * dv.x, c1y = cy + t1 * dv.y, c1z = cz + t1 * dv.z;
  const int ix1 = (int)floorf(c1x), iy1 = (int)floorf(c1y), iz1 = (int)floorf(c1z);
  const int bx1 = min(max(ix1 >> 3, 0), v.tiles_x - 1), by1 = min(max(iy1 >> 3, 0), v.tiles_y - 1);
  const int lbz1 = min(max((iz1 >> 3) - v.bz0, 0), v.nbz - 1);
  const unsigned long long bwd1 = v.bocc[(size_t)(by1 * v.tiles_x + bx1) * v.bw + (lbz1 >> 6)];
#endif
  const int bb = lbz & 63, sb = lsz & 31;
  const bool sclear = !((swd >> sb) & 1u), bclear = !((bwd >> bb) & 1ull);
  float lim = 0.f;
  if (sclear || bclear) {
    lim = run_box(v, sclear ? (unsigned long long)swd : bwd, sclear ? 32 : 64, sclear ? sb : bb, sclear ? lsz : lbz,
                  sclear ? v.nsz : v.nbz, sclear ? v.sz0 : v.bz0, sclear ? 32 : 8, sclear ? sx : bx, sclear ? sy : by,
                  sclear ? v.stx : v.tiles_x, sclear ? v.sty : v.tiles_y, cx, cy, cz, dv, idv);
#if KFX_RAY_CHAIN >= 2
    const int bb1 = lbz1 & 63;
    if (t1 > 0.f && t1 <= lim && !((bwd1 >> bb1) & 1ull)) {
      const float lim1 = run_box(v, bwd1, 64, bb1, lbz1, v.nbz, v.bz0, 8, bx1, by1, v.tiles_x, v.tiles_y, c1x, c1y, c1z,
                                 dv, idv);
      if (lim1 >= 1.f) lim = fmaxf(lim, t1 + lim1);
    }
#endif
  }
  return lim;
}

#ifdef KFX_RAY_TRACE
constexpr bool kTrace = true;
__device__ unsigned long long *g_ray_iter;  // per-wave iteration records (34 u64 per wave)
#else
constexpr bool kTrace = false;
#endif
template <bool kIdx32, bool kSlab, bool kStats = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu((kSlab || !kIdx32) ? KFX_RAY_SLAB_OCC : KFX_RAY_OCC))) void k_raycast(VolView v, RayArgs ra, RayConsts rc,
                                                    FrameView cur, FrameView prev,
                                                    const DevState *__restrict__ st,
                                                    const DevPose *__restrict__ log, DevPose vpose,
                                                    const float *xpose, uint32_t *keys) {
  // kStats: march statistics (rays, skip lookups, skipped samples, blocked
  // lookups, sample batches, normal passes), no stores
  unsigned st_rays = 0, st_lookups = 0, st_skipped = 0, st_blocked = 0, st_batches = 0, st_cand = 0;
#ifdef KFX_RAY_TRACE
  const unsigned long long t_start = wall_clock64();
  unsigned long long t_march = 0, t_norm = 0, t_ndone = 0;
  // wave iterations of the march loop by live-lane count: 1 | 2-4 | 5-16 | 17-64
  unsigned long long t_hist = 0;
  // per march-loop iteration (first 16): {lookup-phase cycles << 32 | batch-phase
  // cycles}, {live lanes | lookups << 8 | max replayed samples << 16}
  unsigned long long *t_it = g_ray_iter ? g_ray_iter + 34 * ((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) : nullptr;
  int t_nit = 0;
#endif
  // cam2vol = volume_pose^-1 * pose, Rinv = R^T (tsdf_volume.cpp:59-61; D:
  // transpose), computed once per frame by k_integrate (DevState::ray_c2v) and
  // read here by every wave with scalar loads: no per-block pose math, LDS
  // round trip or barrier before the march.  Stage seam: explicit cam2vol and
  // Rinv in xpose.
  const float *pose_src = xpose ? xpose : st->ray_c2v.R;  // R[9], t[3] (+ Rinv[9] in xpose)
  const int skind = xpose ? 1 : st->ray_kind;
  const size_t wave_id = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const unsigned long long t_wave0 = KFX_RAY_HINT ? __builtin_amdgcn_s_memtime() : 0ull;
  if (KFX_RAY_HINT && !kSlab && !kStats && v.rdur) {
    const unsigned d = __builtin_amdgcn_readfirstlane(v.rdur[wave_id]);
    if (d >= KFX_RAY_HINT_T0 * 7 / 4) __builtin_amdgcn_s_setprio(3);
    else if (d >= KFX_RAY_HINT_T0 * 11 / 8) __builtin_amdgcn_s_setprio(2);
    else if (d >= KFX_RAY_HINT_T0) __builtin_amdgcn_s_setprio(1);
  }
  if (!kStats && ra.start_sig && blockIdx.x == 0 && threadIdx.x == 0)
    __hip_atomic_store(ra.start_sig, ra.start_val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const LevelGeom g = ra.g[0];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int nbx = (g.w + 15) / 16;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int tx0 = (t % nbx) * 16, ty0 = (t / nbx) * 16;
  const int lx = (wv & 1) * 8 + (lane & 7), ly = (wv >> 1) * 8 + (lane >> 3);
  const int x = tx0 + lx, y = ty0 + ly;
  const bool inimg = x < g.w && y < g.h;
  const size_t o = (size_t)y * g.w + x;
  const int kind = skind;
  f3 vout = {0.f, 0.f, 0.f}, nout = {0.f, 0.f, 0.f};
  uint32_t key = kind == 0 ? 0u : UINT_MAX;  // kSlab: sample index of the decisive event
  uint32_t pend = UINT_MAX;  // kSlab pass 1: first sample not examined (march stopped at the bound)
  float hts = 0.f;                             // kSlab: Ts of the hit written to the maps
  // act: this pixel is marched and written.  Resume pass (kSlab, pass 2):
  // only the pixels this slab left pending below the earliest event any slab
  // found (MIN-reduced [keys | pend] planes: kmin[o] > own pend) march again,
  // unbounded; the others keep their pass-1 results
  bool act = inimg;
  if (kSlab && ra.slab_pass == 2) {
    const size_t np = (size_t)g.w * g.h;
    act = inimg && keys[np + o] != UINT_MAX && keys[np + o] < ra.kmin[o];
    if (!__any(act)) return;  // (k_raycast has no barrier after its setup)
  }
  if (kind == 0 && inimg) {  // frame 1: the measured maps become the model maps
    vout = ld3(cur.v[0], o);
    nout = ld3(cur.n[0], o);
  }
  if (kind == 1) {  // block-uniform
    DevPose P;
#pragma unroll
    for (int i = 0; i < 12; ++i) (i < 9 ? P.R[i] : P.t[i - 9]) = pose_src[i];
    const f3 org = {P.t[0], P.t[1], P.t[2]};
    float da[3];
    ray_dir(P.R, g, x, y, da);
    const f3 dir = {da[0], da[1], da[2]};
    const f3 invR = {1.f / dir.x, 1.f / dir.y, 1.f / dir.z};
    const f3 tbot = mulc(invR, sub({0.f, 0.f, 0.f}, org));
    const f3 ttop = mulc(invR, sub({v.range[0], v.range[1], v.range[2]}, org));
    const f3 tmin = {fminf(ttop.x, tbot.x), fminf(ttop.y, tbot.y), fminf(ttop.z, tbot.z)};
    const f3 tmax = {fmaxf(ttop.x, tbot.x), fmaxf(ttop.y, tbot.y), fmaxf(ttop.z, tbot.z)};
    const float tnear = fmaxf(fmaxf(tmin.x, tmin.y), fmaxf(tmin.x, tmin.z));
    const float tfar = fminf(fminf(tmax.x, tmax.y), fminf(tmax.x, tmax.z));
    float ray_len = fmaxf(tnear, 0.f);
    bool live = act && ray_len < tfar;
    // pass 1: samples up to kb only (the previous frame's model distance
    // along this pixel's ray, + margin; no model point: unbounded)
    uint32_t kb = UINT_MAX;
    if (kSlab && ra.slab_pass == 1 && live) {
      const f3 pv = ld3(prev.v[0], o);
      const float dprev = sqrtf(dot(pv, pv));
      if (dprev > 0.f) {
        const float kf = (dprev * (1.f + ra.bound_rel) + ra.bound_abs - ray_len) / rc.step + 1.f;
        kb = kf < 1.f ? 1u : (kf < 4.0e9f ? (uint32_t)kf : UINT_MAX);
      }
    }
    const f3 vstep = mulc(dir, rc.vs);
    ray_len += rc.step;
    f3 nextp = add(org, scl(dir, ray_len));
    // reference loop state: the carried sample (tsdf_cur for the next step)
    float tprev = live ? voxel2tsdf(v, rc, nextp) : NAN;
    // The march goes kR samples at a time.  Load phase: positions (repeated
    // nextp += vstep) and tsdf loads for the kR samples, issued back to back.
    // Scan phase: the reference's events depend only on consecutive samples
    // (tsdf_cur is the previous sample, NaN included), so with sign s in
    // {-1,0,+1} (0 = NaN) an event at j is s[j-1]*s[j] == -1: a lane builds a
    // 16-bit event mask with plain VALU math and only lanes with an event do
    // more work (a -/+ event ends the ray; a +/- event computes the normal
    // and, if it is NaN, the scan resumes at the next event).
    constexpr int kR = KFX_RAY_KR;
    int sprev = isnan(tprev) ? 0 : (tprev > 0.f ? 1 : (tprev < 0.f ? -1 : 0));
    uint32_t kbase = 1u;  // loop sample index of the batch's first sample
#if KFX_RAY_SLAB_SKIP
    if (kSlab && live) {
      // A slab stores slices [zb, zb + zn): the samples a ray takes before it
      // reaches them read no voxel (NaN: no event, tsdf_volume.cu:184-188), so
      // the ray jumps over them at once — the exact positions and ray_len of
      // that many float adds (ff_add), the sample index advanced by as many —
      // instead of marching them batch by batch (the middle slabs' rays cross
      // the whole volume before theirs).  The count keeps 1.5 voxels and one
      // sample of margin over the continuous model of the accumulated adds.
      const float czv = nextp.z * rc.vs_inv.z, dcz = vstep.z * rc.vs_inv.z;
      float nf = 0.f;
      if (dcz > 0.f) nf = ((float)v.zb - 1.5f - czv) / dcz;
      else if (dcz < 0.f) nf = (czv - ((float)(v.zb + v.zn) + 0.5f)) / -dcz;
      if (nf >= 2.f) {
        const int n0 = (int)fminf(nf, 1.0e7f) - 1;
        const float rl1 = ff_add(ray_len, rc.step, n0 - 1);
        // the reference tests ray_len < tfar before each of the n0 steps
        if (!(rl1 < tfar)) {
          live = false;  // the march ends among the skipped samples: no event here
        } else {
          nextp = {ff_add(nextp.x, vstep.x, n0), ff_add(nextp.y, vstep.y, n0), ff_add(nextp.z, vstep.z, n0)};
          ray_len = rl1 + rc.step;
          kbase += (uint32_t)n0;
          tprev = voxel2tsdf(v, rc, nextp);
          sprev = isnan(tprev) ? 0 : (tprev > 0.f ? 1 : (tprev < 0.f ? -1 : 0));
        }
      }
    }
#endif
    const RayMem<kIdx32> mem(v);
    // voxel validity 1 <= i <= dim-2 (tsdf_volume.cu:184-185) tested on the
    // rounded floats (exact integers; NaN fails like __float2int_rn's INT_MIN)
    const float hx = (float)(v.X - 2), hy = (float)(v.Y - 2), hz = (float)(v.Z - 2);
    const float szb = (float)v.zb, sze = (float)(v.zb + v.zn);
    const float so0 = (float)v.own0, so1 = (float)v.own1;
    const float fzlo = (float)max(1, kSlab ? v.zb : 1);
    const float fzhi = (float)min(v.Z - 2, kSlab ? v.zb + v.zn - 1 : v.Z - 2);
    // Hit candidates (+/- events) are not resolved inside the march: a lane
    // stops there, and once no lane of the wave is marching, all candidates
    // compute their normals in ONE pass (6 trilinear interpolations, 48
    // gathers).  A NaN normal (the reference keeps marching) resumes the march
    // after the candidate sample from the saved state — same samples, same
    // order, same result.
    bool cand = false;
    f3 cvert = {0.f, 0.f, 0.f}, r_nextp = nextp;
    float cts = 0.f;  // the candidate's Ts (slab payload)
    float r_rl = 0.f, r_tprev = 0.f;
    uint32_t ckey = 0u, r_kbase = 0u;
    // Empty-space skipping (exact): no event can happen at a sample whose
    // nearest voxel holds no negative tsdf unless the sample before it is
    // negative (every event needs a negative sample: tsdf_volume.cu:242-244).
    // With the last sample non-negative or NaN (sprev >= 0), the dilated
    // brick and super-brick map words of the current column (both loads in
    // flight together) give runs of clear cells along z in the direction of
    // travel; every voxel of the box such a run guarantees (box_limit) is
    // non-negative, and voxels outside the volume (or the stored slab) are
    // NaN.  The samples that stay inside the larger of the two boxes are only
    // replayed (nextp += vstep, ray_len += step: the reference's exact adds)
    // without loads; the last one is then loaded as the carried sample.
    const f3 dv = mulc(vstep, rc.vs_inv);  // per-sample displacement in voxels
    const f3 idv = {1.f / fabsf(dv.x), 1.f / fabsf(dv.y), 1.f / fabsf(dv.z)};
    const float rstep = 1.f / rc.step;
    const bool can_skip = !isnan(dv.x + dv.y + dv.z);
    if (kStats || kTrace) st_rays += live ? 1u : 0u;
#ifdef KFX_RAY_TRACE
    t_march = wall_clock64();
#endif
    while (__any(live || cand)) {
    while (__any(live)) {
#ifdef KFX_RAY_TRACE
      const unsigned long long t_i0 = __builtin_amdgcn_s_memtime();
      unsigned t_lk = 0, t_mx = 0;
      const int t_nl = __popcll(__ballot(live));
      t_hist += 1ull << (t_nl <= 1 ? 0 : (t_nl <= 4 ? 16 : (t_nl <= 16 ? 32 : 48)));
#endif
      if (kSlab && live && kbase > kb) {  // pass-1 bound: samples < kbase examined, no owned event
        live = false;
        pend = kbase;
      }
      if (can_skip && live && sprev >= 0) {
        uint32_t nsk = 0;
        for (;;) {
          const float cx = nextp.x * rc.vs_inv.x, cy = nextp.y * rc.vs_inv.y, cz = nextp.z * rc.vs_inv.z;
          const float lim = skip_limit(v, cx, cy, cz, dv, idv);
          if (!(lim >= 1.f)) {
            if (kStats) st_blocked += 1;
            break;
          }
#if KFX_RAY_EXIT
          if (!kSlab && (tfar - ray_len) * rstep + 2.f <= fminf(lim, rc.skip_cap)) {
            // every sample the loop has left (at most (tfar - ray_len) / step
            // + 1, 2 of margin over the accumulated rounding) lies in the
            // clear box: no event follows (tsdf_volume.cu:234), the ray ends
            // here without a hit and without replaying its last run
            if (kStats || kTrace) st_lookups += 1;
            live = false;
            break;
          }
#endif
          int n = (int)fminf(lim, rc.skip_cap);
          if (kSlab) {
            // a slab's ray ends 2 slices past its owned range (no owned
            // sample follows, below): replay no further than about there
            // (the far slabs' boxes run on to the volume's end otherwise)
            const float zx = dv.z > 0.f ? ((float)(v.own1 + 3) - cz) * idv.z
                                        : (dv.z < 0.f ? (cz - (float)(v.own0 - 4)) * idv.z : kInf);
            n = min(n, max(1, (int)fminf(zx, rc.skip_cap)));
          }
          if (kStats || kTrace) {
            st_lookups += 1;
            st_skipped += (unsigned)n;
          }
#ifdef KFX_RAY_TRACE
          t_lk += 1;
          t_mx += (unsigned)n;
#endif
          // replay: packed adds {x, y} and {z, ray_len} (the per-element IEEE
          // adds of the reference); the first nf samples provably stay below
          // tfar (2 steps of margin over the accumulated rounding)
          pf2 pxy = {nextp.x, nextp.y}, pzr = {nextp.z, ray_len};
          const pf2 sxy = {vstep.x, vstep.y}, szr = {vstep.z, rc.step};
          const int nf = min(n, max(0, (int)((tfar - ray_len) * rstep) - 2));
          int i = 0;
          for (; i + 8 <= nf; i += 8) {
#pragma unroll
            for (int u = 0; u < 8; ++u) {
              pxy = pxy + sxy;
              pzr = pzr + szr;
            }
          }
          for (; i < nf; ++i) {
            pxy = pxy + sxy;
            pzr = pzr + szr;
          }
          for (; i < n; ++i) {
            if (!(pzr.y < tfar)) {  // the loop ends inside the skipped samples: no event
              live = false;
              break;
            }
            pxy = pxy + sxy;
            pzr = pzr + szr;
          }
          nextp = {pxy.x, pxy.y, pzr.x};
          ray_len = pzr.y;
          nsk += (uint32_t)n;
          if (!live) break;
          if (kSlab) {  // past the owned range (as after a batch): no owned sample follows
            const float zf = nextp.z * rc.vs_inv.z;
            if ((dir.z >= 0.f && zf > (float)(v.own1 + 2)) || (dir.z <= 0.f && zf < (float)(v.own0 - 3))) {
              live = false;
              break;
            }
          }
        }
        if (nsk != 0u && live) {
          kbase += nsk;
          tprev = voxel2tsdf(v, rc, nextp);
          sprev = isnan(tprev) ? 0 : (tprev > 0.f ? 1 : (tprev < 0.f ? -1 : 0));
        }
        if (kSlab && live && kbase > kb) {  // the skipped samples held no event
          live = false;
          pend = kbase;
        }
      }
#ifdef KFX_RAY_TRACE
      const unsigned long long t_i1 = __builtin_amdgcn_s_memtime();
#endif
      if (!__any(live)) break;
      int16_t raw[kR];
      unsigned pm = 0u, nm = 0u, am = 0u, ownm = 0u;
      if (kStats || kTrace) st_batches += live ? 1u : 0u;
      float rl = ray_len;
      const f3 p0 = nextp;  // position before the batch's first sample
      // Interior batch: if the first and (estimated) last sample round into the
      // valid (and stored) voxel box with a half-voxel margin and the batch ends
      // before tfar, every sample of the batch is valid (positions are
      // monotone per axis along the ray), so the per-sample checks drop out.
      bool interior = !live;
      if (live) {
        const f3 ua = mulc(add(p0, vstep), rc.vs_inv);
        const f3 ub = mulc(add(p0, scl(vstep, (float)kR)), rc.vs_inv);
        interior = rl + (float)kR * rc.step < tfar && fminf(ua.x, ub.x) >= 1.f &&
                   fmaxf(ua.x, ub.x) <= hx && fminf(ua.y, ub.y) >= 1.f && fmaxf(ua.y, ub.y) <= hy &&
                   fminf(ua.z, ub.z) >= fzlo && fmaxf(ua.z, ub.z) <= fzhi;
      }
      if (kIdx32 && __all(interior)) {
#pragma unroll
        for (int j = 0; j < kR; ++j) {
          nextp = add(nextp, vstep);
          const float fx = rintf(nextp.x * rc.vs_inv.x);
          const float fy = rintf(nextp.y * rc.vs_inv.y);
          const float fz = rintf(nextp.z * rc.vs_inv.z);
          if (kSlab) ownm |= ((fz >= so0) & (fz < so1)) ? (1u << j) : 0u;
          raw[j] = mem.ld(live, (int)fx, (int)fy, (int)fz);  // dead lanes: no access, 0
          pm |= raw[j] > 0 ? (1u << j) : 0u;
          nm |= raw[j] < 0 ? (1u << j) : 0u;
          rl = rl + rc.step;
        }
        am = (1u << kR) - 1u;
      } else {
#pragma unroll
      for (int j = 0; j < kR; ++j) {
        // a is monotone in j (rl only grows), so lanes past tfar or dead
        // just keep stepping: their samples are masked off
        const bool a = live && rl < tfar;
        am |= a ? (1u << j) : 0u;
        nextp = add(nextp, vstep);
        const float fx = rintf(nextp.x * rc.vs_inv.x);
        const float fy = rintf(nextp.y * rc.vs_inv.y);
        const float fz = rintf(nextp.z * rc.vs_inv.z);
        bool val = a & (fx >= 1.f) & (fx <= hx) & (fy >= 1.f) & (fy <= hy) & (fz >= 1.f) & (fz <= hz);
        if (kSlab) {
          val = val & (fz >= szb) & (fz < sze);
          ownm |= ((fz >= so0) & (fz < so1)) ? (1u << j) : 0u;
        }
        raw[j] = mem.ld(val, (int)fx, (int)fy, (int)fz);
        pm |= (val && raw[j] > 0) ? (1u << j) : 0u;
        nm |= (val && raw[j] < 0) ? (1u << j) : 0u;
        rl = rl + rc.step;
      }
      }
      const int je = __builtin_ctz(~am);  // first sample outside [.., tfar) (kR if none)
      // an event at j needs opposite signs at samples j-1, j (tsdf_cur is the
      // previous sample; NaN = sign 0): +/- is a hit candidate, -/+ a stop
      const unsigned pprev = (pm << 1) | (sprev > 0 ? 1u : 0u);
      const unsigned nprev = (nm << 1) | (sprev < 0 ? 1u : 0u);
      const unsigned hitm = pprev & nm;
      unsigned ev = hitm | (nprev & pm);
      const float tfirst = tprev;
      sprev = ((pm >> (kR - 1)) & 1u) ? 1 : (((nm >> (kR - 1)) & 1u) ? -1 : 0);
      // tsdf_cur of the next batch's first sample; read only when it is a
      // valid positive sample (a +/- event at j = 0 needs sprev > 0)
      tprev = (float)raw[kR - 1] * kDivShortMax;
      if (kSlab) ev &= ownm;  // only owned samples may end the ray on this slab
      unsigned pend = live ? ev : 0u;
      while (__any(pend != 0u)) {
        if (pend != 0u) {
          const int j0 = __ffs(pend) - 1;
          if (!((hitm >> j0) & 1u)) {  // tsdf_cur < 0 && tsdf_next > 0: stop, no surface
            live = false;
            pend = 0u;
            key = kbase + (uint32_t)j0;
          } else {
            // sample j0's ray_len: replay the batch's adds (event samples
            // always lie before je, where every step added rc.step)
            float tc = tfirst, tn = 0.f, rj = ray_len;
#pragma unroll
            for (int j = 0; j < kR; ++j) {
              const float tj = (float)raw[j] * kDivShortMax;
              if (j + 1 == j0) tc = tj;
              if (j == j0) tn = tj;
              if (j < j0) rj += rc.step;
            }
            const float Ts = rj - (v.vs[0] * tc) / (tc - tn);  // A3 (R)
            cvert = add(org, scl(dir, Ts));
            cts = Ts;
            cand = true;
            ckey = kbase + (uint32_t)j0;
            // resume state: sample j0 was processed, the next is j0 + 1
            f3 pj = p0;
#pragma unroll
            for (int j = 0; j < kR; ++j)
              if (j <= j0) pj = add(pj, vstep);
            r_nextp = pj;
            r_rl = rj + rc.step;
            r_kbase = kbase + (uint32_t)j0 + 1u;
            r_tprev = tn;
            live = false;
            pend = 0u;
          }
        }
      }
      if (je < kR) live = false;  // left [.., tfar) inside this batch
      if (kSlab && live) {
        // z is monotonic along the ray: once the samples are more than 2
        // slices past the owned range, no owned sample follows
        const float zf = nextp.z * rc.vs_inv.z;
        if ((dir.z >= 0.f && zf > (float)(v.own1 + 2)) || (dir.z <= 0.f && zf < (float)(v.own0 - 3)))
          live = false;
      }
      ray_len = rl;
      kbase += kR;
#ifdef KFX_RAY_TRACE
      {
        const unsigned long long t_i2 = __builtin_amdgcn_s_memtime();
        unsigned lk = t_lk, mx = t_mx;
        for (int off = 32; off > 0; off >>= 1) {
          lk = max(lk, (unsigned)__shfl_xor((int)lk, off));
          mx = max(mx, (unsigned)__shfl_xor((int)mx, off));
        }
        if (t_it && lane == 0 && t_nit < 16) {
          t_it[2 + 2 * t_nit] = ((t_i1 - t_i0) << 32) | (t_i2 - t_i1);
          t_it[3 + 2 * t_nit] = (unsigned long long)t_nl | ((unsigned long long)min(lk, 255u) << 8) |
                                ((unsigned long long)mx << 16);
        }
        ++t_nit;
      }
#endif
    }
    if (kStats) st_cand += cand ? 1u : 0u;
#ifdef KFX_RAY_TRACE
    if (__any(cand) && !t_norm) t_norm = wall_clock64();
#endif
    if (cand) {  // the wave's normal pass
      cand = false;
      const f3 n = compute_normal<kIdx32 && KFX_RAY_N32>(v, rc, cvert);
      if (!isnan(n.x * n.y * n.z)) {
        // Rinv read here (scalar loads of the uniform pose; the transpose of
        // cam2vol's R, or the stage seam's explicit Rinv)
        float ri[9];
#pragma unroll
        for (int q = 0; q < 9; ++q) ri[q] = xpose ? xpose[12 + q] : pose_src[3 * (q % 3) + q / 3];
        nout = rmul(ri, n);
        vout = rmul(ri, sub(cvert, org));
        key = ckey;
        hts = cts;
      } else {  // NaN normal: keep marching after the candidate (tsdf_volume.cu:251)
        live = true;
        nextp = r_nextp;
        ray_len = r_rl;
        kbase = r_kbase;
        sprev = -1;  // the candidate sample is negative (tsdf_next < 0)
        tprev = r_tprev;
      }
    }
#ifdef KFX_RAY_TRACE
    t_ndone = wall_clock64();
#endif
    }
  }
#ifdef KFX_RAY_TRACE
  if (!kStats && ra.stats) {  // debug: per-wave {start, end, xcc<<32|hw_id, lookups<<32|batches} of lane 0
    unsigned long long *r = ra.stats + 8 * ((size_t)blockIdx.x * 4 + (threadIdx.x >> 6));
    unsigned lk = st_lookups, bt = st_batches;
    for (int off = 32; off > 0; off >>= 1) {
      lk = max(lk, (unsigned)__shfl_xor((int)lk, off));
      bt = max(bt, (unsigned)__shfl_xor((int)bt, off));
    }
    if (lane == 0) {
      r[0] = t_start;
      r[1] = wall_clock64();
      r[2] = ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32) |
             (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);
      r[3] = ((unsigned long long)lk << 32) | bt;
      r[4] = t_march;
      r[5] = t_norm;
      r[6] = t_ndone;
      r[7] = t_hist;
      if (t_it) t_it[0] = (unsigned long long)t_nit;
    }
  }
#endif
  if (kStats) {
    const unsigned c[6] = {st_rays, st_lookups, st_skipped, st_blocked, st_batches, st_cand};
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      unsigned x = c[k];
      for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
      if (lane == 0) atomicAdd(&ra.stats[k], (unsigned long long)x);
    }
    return;
  }
  if (KFX_RAY_HINT && !kSlab && !kStats && v.rdur && (threadIdx.x & 63) == 0)
    v.rdur[wave_id] = (unsigned)((__builtin_amdgcn_s_memtime() - t_wave0) >> 10);
  if (act) {
    if (kSlab) {  // key, pend + payload {Ts, nout} (kfx_internal.h slab combine)
      const size_t np = (size_t)g.w * g.h;
      keys[o] = key;
      keys[np + o] = pend;
      keys[2 * np + o] = __float_as_uint(hts);
      keys[3 * np + o] = __float_as_uint(nout.x);
      keys[4 * np + o] = __float_as_uint(nout.y);
      keys[5 * np + o] = __float_as_uint(nout.z);
    } else {
      st3(prev.v[0], o, vout);
      st3(prev.n[0], o, nout);
    }
  }
  if (kSlab) return;  // resize runs after the cross-slab combine (k_resize)
  resize_tile(ra, kind, tx0, ty0, lx, ly, vout, nout, cur, prev);
}

// SURVEY.md §8d raycast roofline input (count-only, off the frame path): the
// reference raycast (tsdf_volume.cu:210-260) marched naively, one thread per
// pixel, marking in `bits` (one bit per stored voxel) every voxel whose tsdf it
// reads (nearest samples and the trilinear corners of hit normals) and adding
// the reads to reads[0].  N_uniq = popcount(bits) (k_popcount).
__device__ __forceinline__ float touch_read(const VolView &v, uint32_t *bits, unsigned &nr, size_t i) {
  const uint32_t m = 1u << (i & 31);
  if (!(bits[i >> 5] & m)) atomicOr(&bits[i >> 5], m);
  ++nr;
  return (float)v.tsdf[i] * kDivShortMax;
}
__device__ float touch_interp(const VolView &v, uint32_t *bits, unsigned &nr, f3 cf) {
  const int gx = f2i_rd(cf.x), gy = f2i_rd(cf.y), gz = f2i_rd(cf.z);
  if (gx < 0 || gx >= v.X - 1 || gy < 0 || gy >= v.Y - 1 || gz < 0 || gz >= v.Z - 1) return NAN;
  const float a = cf.x - (float)gx, b = cf.y - (float)gy, c = cf.z - (float)gz;
  float s = 0.f;
  s += touch_read(v, bits, nr, vox_index(v, gx, gy, gz)) * (1 - a) * (1 - b) * (1 - c);
  s += touch_read(v, bits, nr, vox_index(v, gx, gy, gz + 1)) * (1 - a) * (1 - b) * c;
  s += touch_read(v, bits, nr, vox_index(v, gx, gy + 1, gz)) * (1 - a) * b * (1 - c);
  s += touch_read(v, bits, nr, vox_index(v, gx, gy + 1, gz + 1)) * (1 - a) * b * c;
  s += touch_read(v, bits, nr, vox_index(v, gx + 1, gy, gz)) * a * (1 - b) * (1 - c);
  s += touch_read(v, bits, nr, vox_index(v, gx + 1, gy, gz + 1)) * a * (1 - b) * c;
  s += touch_read(v, bits, nr, vox_index(v, gx + 1, gy + 1, gz)) * a * b * (1 - c);
  s += touch_read(v, bits, nr, vox_index(v, gx + 1, gy + 1, gz + 1)) * a * b * c;
  return s;
}
__global__ __launch_bounds__(256) void k_raycast_touch(VolView v, LevelGeom g, RayConsts rc,
                                                       const DevState *__restrict__ st,
                                                       const DevPose *__restrict__ log, DevPose vpose,
                                                       const float *xpose, uint32_t *bits,
                                                       unsigned long long *reads) {
  __shared__ DevPose s_c2v;
  __shared__ int s_kind;
  if (threadIdx.x == 0) {
    if (xpose) {
      s_kind = 1;
      for (int i = 0; i < 9; ++i) s_c2v.R[i] = xpose[i];
      for (int i = 0; i < 3; ++i) s_c2v.t[i] = xpose[9 + i];
    } else {
      s_kind = frame_kind(st);
      if (s_kind == 1) s_c2v = pose_mul(pose_inv(vpose), frame_pose(st, log, 1));
    }
  }
  __syncthreads();
  unsigned nr = 0;
  const int pi = blockIdx.x * 256 + threadIdx.x;
  if (s_kind == 1 && pi < g.w * g.h) {
    const int x = pi % g.w, y = pi / g.w;
    const DevPose P = s_c2v;
    const f3 org = {P.t[0], P.t[1], P.t[2]};
    const f3 pp = {(1.f * ((float)x - g.cx)) / g.fx, (1.f * ((float)y - g.cy)) / g.fy, 1.f};
    const f3 dir = normalized(rmul(P.R, pp));
    const f3 invR = {1.f / dir.x, 1.f / dir.y, 1.f / dir.z};
    const f3 tbot = mulc(invR, sub({0.f, 0.f, 0.f}, org));
    const f3 ttop = mulc(invR, sub({v.range[0], v.range[1], v.range[2]}, org));
    const f3 tmin = {fminf(ttop.x, tbot.x), fminf(ttop.y, tbot.y), fminf(ttop.z, tbot.z)};
    const f3 tmax = {fmaxf(ttop.x, tbot.x), fmaxf(ttop.y, tbot.y), fmaxf(ttop.z, tbot.z)};
    const float tnear = fmaxf(fmaxf(tmin.x, tmin.y), fmaxf(tmin.x, tmin.z));
    const float tfar = fminf(fminf(tmax.x, tmax.y), fminf(tmax.x, tmax.z));
    float ray_len = fmaxf(tnear, 0.f);
    if (ray_len < tfar) {
      const f3 vstep = mulc(dir, rc.vs);
      ray_len += rc.step;
      f3 nextp = add(org, scl(dir, ray_len));
      auto sample = [&](f3 p) -> float {
        const int ix = f2i_rn(p.x * rc.vs_inv.x), iy = f2i_rn(p.y * rc.vs_inv.y), iz = f2i_rn(p.z * rc.vs_inv.z);
        if (ix >= v.X - 1 || iy >= v.Y - 1 || iz >= v.Z - 1 || ix < 1 || iy < 1 || iz < 1) return NAN;
        return touch_read(v, bits, nr, vox_index(v, ix, iy, iz));
      };
      float tn = sample(nextp);
      for (; ray_len < tfar; ray_len += rc.step) {
        nextp = add(nextp, vstep);
        const float tc = tn;
        tn = sample(nextp);
        if (isnan(tn)) continue;
        if (tc < 0.f && tn > 0.f) break;
        if (tc > 0.f && tn < 0.f) {
          const float Ts = ray_len - (v.vs[0] * tc) / (tc - tn);
          const f3 p = add(org, scl(dir, Ts));
          f3 n;
          n.x = (touch_interp(v, bits, nr, mulc({p.x + rc.gd.x, p.y, p.z}, rc.vs_inv)) -
                 touch_interp(v, bits, nr, mulc({p.x - rc.gd.x, p.y, p.z}, rc.vs_inv))) / rc.gd.x;
          n.y = (touch_interp(v, bits, nr, mulc({p.x, p.y + rc.gd.y, p.z}, rc.vs_inv)) -
                 touch_interp(v, bits, nr, mulc({p.x, p.y - rc.gd.y, p.z}, rc.vs_inv))) / rc.gd.y;
          n.z = (touch_interp(v, bits, nr, mulc({p.x, p.y, p.z + rc.gd.z}, rc.vs_inv)) -
                 touch_interp(v, bits, nr, mulc({p.x, p.y, p.z - rc.gd.z}, rc.vs_inv))) / rc.gd.z;
          n = normalized(n);
          if (!isnan(n.x * n.y * n.z)) break;
        }
      }
    }
  }
  unsigned long long t = nr;
  for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off);
  if ((threadIdx.x & 63) == 0 && t) atomicAdd(reads, t);
}
__global__ __launch_bounds__(256) void k_popcount(const uint32_t *bits, size_t n, unsigned long long *out) {
  unsigned long long c = 0;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) c += __popc(bits[i]);
  for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(out, c);
}

// kernel_resizePointsNormals (image_process.cu:95-125) for levels >= 1: the
// block's 16x16 level-0 tile (this thread's values vout/nout at (lx, ly)) maps
// onto 8x8 / 4x4 / 2x2 tiles of levels 1 / 2 / 3, computed from the level
// below through LDS with the same float ops.  kind 0 (frame 1) copies the
// measured maps, kind 2 (reset) writes zeros.
__device__ void resize_tile(const RayArgs &ra, int kind, int tx0, int ty0, int lx, int ly, f3 vout,
                            f3 nout, const FrameView &cur, const FrameView &prev) {
  if (ra.levels < 2) return;
  __shared__ f3 sv[2][256], sn[2][256];
  sv[0][ly * 16 + lx] = vout;
  sn[0][ly * 16 + lx] = nout;
  __syncthreads();
  int side = 16;
  for (int l = 1; l < ra.levels; ++l) {
    const int pb = (l - 1) & 1, cb = l & 1;
    const int ps = side;
    side >>= 1;
    const LevelGeom gl = ra.g[l];
    const int X = (tx0 >> l) + (threadIdx.x % side), Y = (ty0 >> l) + (threadIdx.x / side);
    const bool act = (int)threadIdx.x < side * side && X < gl.w && Y < gl.h;
    f3 vo = {0.f, 0.f, 0.f}, no = {0.f, 0.f, 0.f};
    if ((int)threadIdx.x < side * side) {
      const int cx = threadIdx.x % side, cy = threadIdx.x / side;
      if (kind == 0) {
        if (act) {
          const size_t ol = (size_t)Y * gl.w + X;
          vo = ld3(cur.v[l], ol);
          no = ld3(cur.n[l], ol);
        }
      } else if (kind == 1) {
        const int i00 = (2 * cy) * ps + 2 * cx;
        const f3 d00 = sv[pb][i00], d01 = sv[pb][i00 + 1], d10 = sv[pb][i00 + ps],
                 d11 = sv[pb][i00 + ps + 1];
        if (!isnan(d00.x * d01.x * d10.x * d11.x)) {
          vo = scl(add(add(add(d00, d01), d10), d11), 0.25f);
          no = scl(add(add(add(sn[pb][i00], sn[pb][i00 + 1]), sn[pb][i00 + ps]),
                       sn[pb][i00 + ps + 1]),
                   0.25f);
        }
      }
      sv[cb][cy * side + cx] = vo;
      sn[cb][cy * side + cx] = no;
      if (act) {
        const size_t ol = (size_t)Y * gl.w + X;
        st3(prev.v[l], ol, vo);
        st3(prev.n[l], ol, no);
      }
    }
    __syncthreads();
  }
}

// Resize of the combined level-0 model maps (slab mode): same tiles and ops as
// the resize fused into k_raycast.
__global__ __launch_bounds__(256) void k_resize(RayArgs ra, FrameView cur, FrameView prev,
                                                const DevState *__restrict__ st,
                                                const float *xpose) {
  const int t = blockIdx.x;
  const int kind = xpose ? 1 : frame_kind(st);
  const LevelGeom g = ra.g[0];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int nbx = (g.w + 15) / 16;
  const int tx0 = (t % nbx) * 16, ty0 = (t / nbx) * 16;
  const int lx = (wv & 1) * 8 + (lane & 7), ly = (wv >> 1) * 8 + (lane >> 3);
  const int x = tx0 + lx, y = ty0 + ly;
  f3 vout = {0.f, 0.f, 0.f}, nout = {0.f, 0.f, 0.f};
  if (x < g.w && y < g.h) {
    const size_t o = (size_t)y * g.w + x;
    vout = ld3(prev.v[0], o);
    nout = ld3(prev.n[0], o);
  }
  resize_tile(ra, kind, tx0, ty0, lx, ly, vout, nout, cur, prev);
}

// Cross-slab combine, step 2 (after the all-reduce MIN of the keys): a rank
// that does not hold the earliest event of a pixel clears its payload there,
// so the all-reduce MAX of the payload bits (step 3) leaves exactly the
// winner's (kfx_internal.h slab_mask_px).
__global__ void k_slab_mask(const uint32_t *__restrict__ keys, const uint32_t *__restrict__ key_min, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) slab_mask_px(keys, key_min, const_cast<uint32_t *>(keys) + 2 * (size_t)n, (size_t)n, (size_t)i);
}
// Step 4: the level-0 model maps from the combined payload (frame kind as in
// k_raycast: frame 1 copies the measured maps, a reset frame writes zeros).
__global__ __launch_bounds__(256) void k_slab_expand(LevelGeom g, const uint32_t *__restrict__ pay, FrameView cur,
                                                     FrameView prev, const DevState *__restrict__ st,
                                                     const DevPose *__restrict__ log, DevPose vpose) {
  __shared__ DevPose s_c2v;
  __shared__ float s_rinv[9];
  __shared__ int s_kind;
  if (threadIdx.x == 0) {
    s_kind = frame_kind(st);
    if (s_kind == 1) {
      s_c2v = pose_mul(pose_inv(vpose), frame_pose(st, log, 1));
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) s_rinv[3 * i + j] = s_c2v.R[3 * j + i];
    }
  }
  __syncthreads();
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= g.w * g.h) return;
  f3 v = {0.f, 0.f, 0.f}, nm = {0.f, 0.f, 0.f};
  if (s_kind == 0) {
    v = ld3(cur.v[0], i);
    nm = ld3(cur.n[0], i);
  } else if (s_kind == 1) {
    float d[3], a[3], b[3];
    ray_dir(s_c2v.R, g, i % g.w, i / g.w, d);
    slab_expand_px(pay, (size_t)g.w * g.h, (size_t)i, s_c2v.t, d, s_rinv, a, b);
    v = {a[0], a[1], a[2]};
    nm = {b[0], b[1], b[2]};
  }
  st3(prev.v[0], i, v);
  st3(prev.n[0], i, nm);
}

struct GroupSt {
  DevState *p[kMaxGroup];
  int n;
};

// In-process group combine (several slab contexts in one process): element-wise
// MIN / MAX over the members' u32 buffers, result written back to every member.
struct GroupBufs {
  uint32_t *p[kMaxGroup];
  int n;
};
__global__ void k_group_reduce(GroupBufs in, GroupBufs out, size_t count, int is_max) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < count;
       i += (size_t)gridDim.x * blockDim.x) {
    uint32_t r = in.p[0][i];
    for (int k = 1; k < in.n; ++k) r = is_max ? max(r, in.p[k][i]) : min(r, in.p[k][i]);
    for (int k = 0; k < out.n; ++k) out.p[k][i] = r;
  }
}

// ---------------------------------------------------------------------------
// Point-cloud extraction — FullScan6 (tsdf_volume.cu:307-481): for every voxel
// with W != 0 and F != 1 (A11: never 1), a zero crossing towards the +x, +y
// and +z neighbour (W != 0, F != 1, opposite signs) gives the point
// p = (V * |Fn| + Vn * |F|) / (|F| + |Fn|) along that edge, V the voxel
// centre ((i + 0.5) * vs), transformed by the volume pose (R * p + t).
//
// The reference appends points with warp atomics (nondeterministic order, a
// nondeterministic subset when the 10 M buffer fills).  Here the order is
// canonical (D): wave = one 8x8 column tile x kExtractZ slices; points are
// ordered by (slice chunk, tile, z, lane = (y&7)*8 + (x&7), edge x/y/z), so
// the output and its first `cap` points are deterministic.  Pass 1 counts
// per wave, a scan turns counts into offsets, pass 2 writes.
constexpr int kExtractZ = 8;

__device__ __forceinline__ int extract_voxel(const VolView &v, const DevPose &aff, int x, int y,
                                             int z, f3 (&pts)[3]) {
  const size_t i = vox_index(v, x, y, z);
  const int W = v.weight[i];
  const float F = (float)v.tsdf[i] * kDivShortMax;
  if (W == 0 || F == 1.f) return 0;
  const f3 V = {((float)x + 0.5f) * v.vs[0], ((float)y + 0.5f) * v.vs[1], ((float)z + 0.5f) * v.vs[2]};
  const f3 t = {aff.t[0], aff.t[1], aff.t[2]};
  int n = 0;
  auto edge = [&](int axis, size_t j) {
    const int Wn = v.weight[j];
    const float Fn = (float)v.tsdf[j] * kDivShortMax;
    if (Wn != 0 && Fn != 1.f && ((F > 0 && Fn < 0) || (F < 0 && Fn > 0))) {
      f3 p = V;
      const float Va = axis == 0 ? V.x : (axis == 1 ? V.y : V.z);
      const float Vn = Va + v.vs[axis];
      const float d_inv = 1.f / (fabsf(F) + fabsf(Fn));
      const float c = (Va * fabsf(Fn) + Vn * fabsf(F)) * d_inv;
      if (axis == 0) p.x = c;
      else if (axis == 1) p.y = c;
      else p.z = c;
      pts[n++] = add(rmul(aff.R, p), t);
    }
  };
  if (x + 1 < v.X) edge(0, vox_index(v, x + 1, y, z));
  if (y + 1 < v.Y) edge(1, vox_index(v, x, y + 1, z));
  edge(2, vox_index(v, x, y, z + 1));  // z + 1 < Z: guaranteed by the z range
  return n;
}

// kEmit = false: counts[wave] = points of the wave; true: write them at
// offsets[wave] + rank (rank < cap only).  z in [zlo, zhi) (global slices,
// zhi <= Z - 1; a slab passes its owned range).
// Extraction waves own one tile x one 8-slice chunk (kExtractZ), i.e. one
// brick.  Every point needs a negative tsdf at the voxel or its +x/+y/+z
// neighbour, and every marching-cubes triangle a negative corner: all of them
// lie in the brick or a neighbouring one, so a clear (dilated) brick bit of
// the occupancy map proves the wave outputs nothing — it reads no voxel.
__device__ __forceinline__ bool brick_clear(const VolView &v, int tile, int c0) {
  const int lbz = (c0 >> 3) - v.bz0;
  if (lbz < 0 || lbz >= v.nbz) return false;
  return !((v.bocc[(size_t)tile * v.bw + (lbz >> 6)] >> (lbz & 63)) & 1ull);
}

// One extraction wave's brick (lanes = the tile's 64 columns, slices [z0, z1)):
// kEmit = false returns the wave's point count; true writes the points at
// base + (canonical rank) (rank < cap only) and returns the count too.
template <bool kEmit>
__device__ __forceinline__ unsigned extract_wave(const VolView &v, const DevPose &aff, int x, int y, int z0,
                                                 int z1, unsigned long long base, float *out,
                                                 unsigned long long cap) {
  const int lane = threadIdx.x & 63;
  unsigned total = 0;
  const unsigned long long below = (1ull << lane) - 1ull;
  for (int z = z0; z < z1; ++z) {
    f3 pts[3];
    const int n = extract_voxel(v, aff, x, y, z, pts);
    const unsigned long long b1 = __ballot(n >= 1), b2 = __ballot(n >= 2), b3 = __ballot(n >= 3);
    if (kEmit) {
      const unsigned long long r = base + (unsigned long long)(__popcll(b1 & below) +
                                                               __popcll(b2 & below) +
                                                               __popcll(b3 & below));
#pragma unroll
      for (int l = 0; l < 3; ++l)  // (unrolled: pts stays in registers)
        if (l < n && r + l < cap) st3(out, (size_t)(r + l), pts[l]);
    }
    const unsigned wt = (unsigned)(__popcll(b1) + __popcll(b2) + __popcll(b3));
    base += wt;
    total += wt;
  }
  return total;
}

// Marching cubes (§8 f5; C5 asks for a mesh, the reference has none).  Cube
// (x, y, z) = the 8 voxels (x+dx, y+dy, z+dz); all 8 must have weight > 0;
// corner c = dx | dy<<1 | dz<<2 is inside when its tsdf < 0.  `tab` (256 x
// 16 bytes, built by the host, kfx_api.hip mc_table) lists per configuration
// the triangles as edge indices (edge e: axis e/4, the 4 edges of an axis in
// ascending lower-corner order).  An edge vertex interpolates the two voxel
// centres as the point extraction does (FullScan6, tsdf_volume.cu:341-360),
// then the volume pose.  Triangles come out in the canonical order of the
// point cloud (8-slice chunk, tile, z, lane, triangle), 9 floats each.
__device__ __forceinline__ f3 mc_vertex(const VolView &v, const DevPose &aff, int x, int y, int z, int e,
                                        const float (&F)[8]) {
  const int a = e >> 2, k = e & 3;
  // lower corner of edge e: the k-th corner (ascending) with bit a clear
  int c = 0, m = 0;
  for (int q = 0; q < 8; ++q)
    if (!((q >> a) & 1)) {
      if (m == k) c = q;
      ++m;
    }
  const int cn = c | (1 << a);
  f3 V = {((float)(x + (c & 1)) + 0.5f) * v.vs[0], ((float)(y + ((c >> 1) & 1)) + 0.5f) * v.vs[1],
          ((float)(z + ((c >> 2) & 1)) + 0.5f) * v.vs[2]};
  const float Fa = F[c], Fb = F[cn];
  const float Va = a == 0 ? V.x : (a == 1 ? V.y : V.z);
  const float Vn = Va + v.vs[a];
  const float d_inv = 1.f / (fabsf(Fa) + fabsf(Fb));
  const float cc = (Va * fabsf(Fb) + Vn * fabsf(Fa)) * d_inv;
  if (a == 0) V.x = cc;
  else if (a == 1) V.y = cc;
  else V.z = cc;
  return add(rmul(aff.R, V), {aff.t[0], aff.t[1], aff.t[2]});
}

// One marching-cubes wave's brick (as extract_wave): triangles in the
// canonical order, 9 floats each.
template <bool kEmit>
__device__ __forceinline__ unsigned mesh_wave(const VolView &v, const DevPose &aff, const uint8_t *__restrict__ tab,
                                              int x, int y, int z0, int z1, unsigned long long base, float *out,
                                              unsigned long long cap) {
  const int lane = threadIdx.x & 63;
  unsigned total = 0;
  for (int z = z0; z < z1; ++z) {
    float F[8];
    int cfg = 0, nt = 0;
    if (x + 1 < v.X && y + 1 < v.Y) {
      bool all = true;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const size_t i = vox_index(v, x + (c & 1), y + ((c >> 1) & 1), z + ((c >> 2) & 1));
        all = all && v.weight[i] > 0;
        F[c] = (float)v.tsdf[i] * kDivShortMax;
        cfg |= (F[c] < 0.f ? 1 : 0) << c;
      }
      if (all) nt = tab[16 * cfg];
    }
    // wave prefix of the triangle counts (lane order)
    int incl = nt;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int o = __shfl_up(incl, off);
      if (lane >= off) incl += o;
    }
    if (kEmit) {
      const unsigned long long r0 = base + (unsigned long long)(incl - nt);
      for (int t = 0; t < nt; ++t) {
        if (r0 + t >= cap) break;
#pragma unroll
        for (int k = 0; k < 3; ++k)
          st3(out, (size_t)(3 * (r0 + t) + k), mc_vertex(v, aff, x, y, z, tab[16 * cfg + 1 + 3 * t + k], F));
      }
    }
    const unsigned wt = (unsigned)__shfl(incl, 63);
    base += wt;
    total += wt;
  }
  return total;
}

// Extraction with ONE read of the volume (points or marching cubes).
// Pass A (k_extract_pool): each canonical wave counts its brick's items and,
// if it has any, reserves that many slots of a pool with one 64-bit atomic
// (high bits: the wave's entry in the list of non-empty waves, low bits: the
// pool offset) and writes its items there in its own canonical order (from
// the bricks it just read: cache hits).  The reserved slots are unordered
// across waves.  Then the offset scan of the per-wave counts (canonical
// order) and pass C (k_extract_copy): one wave per listed wave copies its
// items from the pool to their canonical position.  A pool too small for
// every item (the caller's cap) sets *overflow; the counts are still complete,
// and the host then runs the emit pass of the two-pass path instead.
constexpr int kPoolListShift = 40;
constexpr unsigned long long kPoolMask = (1ull << kPoolListShift) - 1ull;
enum XMode { kXCount = 0, kXEmit = 1, kXPool = 2 };
// The extraction passes.  A unit = one tile x one 8-slice chunk (the
// canonical order's (chunk, tile)); each wave sweeps 64 consecutive units of
// one chunk (K = 1..64, xsweep_units): lane l tests unit T0 + l's brick in
// the occupancy map, a clear brick's unit has no items (count 0, no voxel
// read), and the others are processed one after another by the whole wave
// (lane = column).  At 2048^3 (16.8 M units, mostly clear) a wave per unit
// is launch-bound (count pass 8.3 ms; 64 units per wave: 6.8 ms for count +
// pool emit); small volumes keep enough waves with a small K.
// kXCount: counts[unit]; kXEmit: items at offsets[unit] (first cap only);
// kXPool: counts[unit] and the items into the pool (above).
template <int kMode, bool kMesh>
__global__ __launch_bounds__(256) void k_xsweep(VolView v, DevPose aff, int zlo, int zhi,
                                                const uint8_t *__restrict__ tab, unsigned *counts,
                                                const unsigned long long *offsets, float *out,
                                                unsigned long long cap, unsigned long long *ctr,
                                                unsigned long long *pool_at, unsigned *list, unsigned *overflow,
                                                int K) {
  const int lane = threadIdx.x & 63;
  const int ntiles = v.tiles_x * v.tiles_y;
  const int T0 = (int)(blockIdx.x * 4 + (threadIdx.x >> 6)) * K;
  if (T0 >= ntiles) return;
  // chunks are aligned to global multiples of kExtractZ (slab boundaries are
  // too), so concatenating slabs in rank order reproduces the single volume
  const int c0 = (zlo / kExtractZ) * kExtractZ + (int)blockIdx.y * kExtractZ;
  const int z0 = max(zlo, c0), z1 = min(zhi, c0 + kExtractZ);
  static_assert(kExtractZ == 8, "one brick per unit");
  const size_t ubase = (size_t)blockIdx.y * ntiles;  // unit index = ubase + tile
  const int tl = T0 + lane;
  const bool mine = lane < K && tl < ntiles;
  const bool have = mine && !(KFX_EXTRACT_SKIP && brick_clear(v, tl, c0));
  if (kMode != kXEmit && mine && !have) counts[ubase + tl] = 0u;
  unsigned long long work = __ballot(have);
  while (work) {  // wave-uniform
    const int t = __ffsll((long long)work) - 1;
    work &= work - 1ull;
    const int tile = T0 + t;
    const size_t unit = ubase + tile;
    const int x = (tile % v.tiles_x) * 8 + (lane & 7);
    const int y = (tile / v.tiles_x) * 8 + (lane >> 3);
    if (kMode == kXEmit) {
      if (kMesh)
        (void)mesh_wave<true>(v, aff, tab, x, y, z0, z1, offsets[unit], out, cap);
      else
        (void)extract_wave<true>(v, aff, x, y, z0, z1, offsets[unit], out, cap);
      continue;
    }
    const unsigned n = kMesh ? mesh_wave<false>(v, aff, tab, x, y, z0, z1, 0ull, out, 0ull)
                             : extract_wave<false>(v, aff, x, y, z0, z1, 0ull, out, 0ull);
    if (lane == 0) counts[unit] = n;
    if (kMode != kXPool || n == 0) continue;
    unsigned long long old = 0;
    if (lane == 0) old = atomicAdd(ctr, (1ull << kPoolListShift) | (unsigned long long)n);
    old = __shfl(old, 0);
    const unsigned long long base = old & kPoolMask;
    if (lane == 0) {
      list[old >> kPoolListShift] = (unsigned)unit;
      pool_at[unit] = base;
    }
    if (base + n > cap) {  // (cap = the pool's size here)
      if (lane == 0) atomicOr(overflow, 1u);
      continue;
    }
    // the items again from the brick just read (cache hits; staging them in
    // LDS during the count measured slower: occupancy)
    if (kMesh)
      (void)mesh_wave<true>(v, aff, tab, x, y, z0, z1, base, out, cap);
    else
      (void)extract_wave<true>(v, aff, x, y, z0, z1, base, out, cap);
  }
}
// Pass C: listed wave i's items from the pool to offsets[wave] (first cap
// items of the canonical order only); per = floats per item.
__global__ __launch_bounds__(256) void k_extract_copy(const unsigned *__restrict__ list, unsigned nlist,
                                                      const unsigned *__restrict__ counts,
                                                      const unsigned long long *__restrict__ pool_at,
                                                      const unsigned long long *__restrict__ offsets,
                                                      const float *__restrict__ pool, float *out,
                                                      unsigned long long cap, int per) {
  const unsigned i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= nlist) return;
  const int lane = threadIdx.x & 63;
  const unsigned w = list[i];
  const unsigned long long o = offsets[w];
  if (o >= cap) return;
  const unsigned long long n = min((unsigned long long)counts[w], cap - o);
  const float *src = pool + pool_at[w] * per;
  float *dst = out + o * per;
  for (unsigned long long k = lane; k < n * per; k += 64) dst[k] = src[k];
}

// Exclusive scan of n u32 counts into u64 offsets (one 1024-thread block per
// 4096 counts, then the block totals, then the fix-up); *total = the sum.
__global__ __launch_bounds__(1024) void k_scan_local(const unsigned *in, unsigned long long *out,
                                                     unsigned long long *bsum, size_t n) {
  __shared__ unsigned long long s[1024];
  const size_t b0 = (size_t)blockIdx.x * 4096 + threadIdx.x * 4;
  unsigned long long v[4], acc = 0;
  for (int k = 0; k < 4; ++k) {
    v[k] = (b0 + k < n) ? in[b0 + k] : 0ull;
    acc += v[k];
  }
  s[threadIdx.x] = acc;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {  // Hillis-Steele inclusive scan
    const unsigned long long t = threadIdx.x >= off ? s[threadIdx.x - off] : 0ull;
    __syncthreads();
    s[threadIdx.x] += t;
    __syncthreads();
  }
  unsigned long long run = s[threadIdx.x] - acc;
  for (int k = 0; k < 4; ++k) {
    if (b0 + k < n) out[b0 + k] = run;
    run += v[k];
  }
  if (threadIdx.x == 1023) bsum[blockIdx.x] = s[1023];
}
__global__ __launch_bounds__(1024) void k_scan_blocks(unsigned long long *bsum, int nb,
                                                      unsigned long long *total) {
  // nb <= 1024 * 64: each thread scans a contiguous run, then one block scan
  __shared__ unsigned long long s[1024];
  const int per = (nb + 1023) / 1024;
  const int b0 = threadIdx.x * per;
  unsigned long long acc = 0;
  for (int k = 0; k < per; ++k)
    if (b0 + k < nb) acc += bsum[b0 + k];
  s[threadIdx.x] = acc;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const unsigned long long t = threadIdx.x >= off ? s[threadIdx.x - off] : 0ull;
    __syncthreads();
    s[threadIdx.x] += t;
    __syncthreads();
  }
  unsigned long long run = s[threadIdx.x] - acc;
  for (int k = 0; k < per; ++k)
    if (b0 + k < nb) {
      const unsigned long long c = bsum[b0 + k];
      bsum[b0 + k] = run;
      run += c;
    }
  if (threadIdx.x == 1023) *total = s[1023];
}
__global__ void k_scan_add(unsigned long long *out, const unsigned long long *bsum, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] += bsum[i / 4096];
}

__global__ void k_inv_lambda(LevelGeom g, float *out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= g.w * g.h) return;
  const int u = i % g.w, vv = i / g.w;
  const f3 xyl = {(1.f * ((float)u - g.cx)) / g.fx, (1.f * ((float)vv - g.cy)) / g.fy, 1.f};
  const float lambda = sqrtf(dot(xyl, xyl));
  out[i] = 1.f / lambda;
}

// Reference 8-byte record {int16 tsdf, int16 weight, u8 c0,c1,c2, pad}
// (device_types.hpp:51-56), x-fastest linear order, for slices [z0, z0+nz).
__global__ void k_export_records(VolView v, int z0, int nz, uint64_t *dst) {
  const size_t n = v.slice * (size_t)nz;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const int x = (int)(i % v.X);
    const int y = (int)((i / v.X) % v.Y);
    const int z = z0 + (int)(i / v.slice);
    const size_t s = vox_index(v, x, y, z);
    const uint64_t rec = (uint64_t)(uint16_t)v.tsdf[s] | ((uint64_t)(uint16_t)v.weight[s] << 16) |
                         ((uint64_t)(v.rgb[s] & 0xffffffu) << 32);
    dst[i] = rec;
  }
}

__global__ void k_import_records(VolView v, int z0, int nz, const uint64_t *src, unsigned *bad) {
  const size_t n = v.slice * (size_t)nz;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const int x = (int)(i % v.X);
    const int y = (int)((i / v.X) % v.Y);
    const int z = z0 + (int)(i / v.slice);
    const size_t s = vox_index(v, x, y, z);
    const uint64_t rec = src[i];
    v.tsdf[s] = (int16_t)(rec & 0xffffu);
    const int w = (int16_t)((rec >> 16) & 0xffffu);
    if ((unsigned)w > 255u) *bad = 1u;  // not representable in the u8 weight store
    v.weight[s] = (uint8_t)w;
    v.rgb[s] = (uint32_t)((rec >> 32) & 0xffffffu);
  }
}

// Order-free volume checksum over the owned slices: sum of a 64-bit mix of
// (global x-fastest index, tsdf, weight, colour) per voxel, and the count of
// voxels with weight > 0 — slab sums add up to the single volume's.
__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__global__ __launch_bounds__(256) void k_checksum(VolView v, unsigned long long *out) {
  const size_t n = v.local_voxels(), per_tile = v.tile_voxels();
  unsigned long long h = 0, cnt = 0;
  for (size_t li = (size_t)blockIdx.x * 256 + threadIdx.x; li < n; li += (size_t)gridDim.x * 256) {
    const size_t tile = li / per_tile, rem = li % per_tile;
    const int z = v.zb + (int)(rem >> 6), inner = (int)(rem & 63);
    if (z < v.own0 || z >= v.own1) continue;
    const int x = (int)(tile % v.tiles_x) * 8 + (inner & 7), y = (int)(tile / v.tiles_x) * 8 + (inner >> 3);
    const unsigned long long g = (unsigned long long)x + (unsigned long long)v.X * ((unsigned long long)y + (unsigned long long)v.Y * z);
    const unsigned long long rec = ((unsigned long long)(uint16_t)v.tsdf[li] << 48) |
                                   ((unsigned long long)(uint16_t)v.weight[li] << 32) | (v.rgb[li] & 0xffffffu);
    h += mix64(g * 0x9E3779B97F4A7C15ull ^ rec);
    cnt += v.weight[li] > 0;
  }
  for (int off = 32; off > 0; off >>= 1) {
    h += __shfl_xor(h, off);
    cnt += __shfl_xor(cnt, off);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&out[0], h);
    atomicAdd(&out[1], cnt);
  }
}

// Occupancy maps of the whole stored volume (after an upload; the maps were
// cleared): wave = one brick (column tile x 8 slices), lane = one column.
__global__ __launch_bounds__(256) void k_occ_rebuild(VolView v) {
  const int lane = threadIdx.x & 63;
  const size_t w = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= (size_t)v.tiles_x * v.tiles_y * v.nbz) return;
  const int tile = (int)(w / v.nbz), lb = (int)(w % v.nbz);
  const int z0 = max((v.bz0 + lb) * 8, v.zb), z1 = min((v.bz0 + lb) * 8 + 8, v.zb + v.zn);
  int lo = INT_MAX, hi = -1;
  for (int z = z0; z < z1; ++z)
    if (v.tsdf[(size_t)tile * v.tile_voxels() + (size_t)(z - v.zb) * 64 + lane] < 0) {
      lo = min(lo, z);
      hi = max(hi, z);
    }
  occ_mark_wave(v, tile, lo, hi, lane);
}

__global__ void k_gather_columns(VolView v, const int32_t *cols, int n, int16_t *t, int16_t *w, uint32_t *c) {
  const int nz = v.own1 - v.own0;
  const size_t total = (size_t)n * nz;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int k = (int)(i / nz), z = v.own0 + (int)(i % nz);
    const size_t s = vox_index(v, cols[2 * k], cols[2 * k + 1], z);
    if (t) t[i] = v.tsdf[s];
    if (w) w[i] = v.weight[s];
    if (c) c[i] = v.rgb[s];
  }
}

__global__ void k_export_soa(VolView v, int z0, int nz, int16_t *t, int16_t *w, uint32_t *c) {
  const size_t n = v.slice * (size_t)nz;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const int x = (int)(i % v.X);
    const int y = (int)((i / v.X) % v.Y);
    const int z = z0 + (int)(i / v.slice);
    const size_t s = vox_index(v, x, y, z);
    if (t) t[i] = v.tsdf[s];
    if (w) w[i] = v.weight[s];
    if (c) c[i] = v.rgb[s];
  }
}

// kernel_renderNormals / kernel_renderPhong (image_process.cu:137-221) on the
// previous frame's level-0 maps, lit from the last pose's camera position
// (kinectfusion.cpp:33-47).  D as in the oracle (kfo_render): IEEE sqrt and
// division in __m_normalize, pow(h, 10) as h8 * h2, NaN → 0 in the uchar
// conversion; `0.5*light_coffi` stays double as in the source.
__device__ __forceinline__ uint8_t render_u8(float x) { return x >= 1.f ? (uint8_t)fminf(x, 255.f) : 0; }
__device__ __forceinline__ f3 normalized_ieee(f3 v) {
  const float t = sqrtf(dot(v, v));
  return {v.x / t, v.y / t, v.z / t};
}
__global__ __launch_bounds__(256) void k_render(const float *__restrict__ vmap, const float *__restrict__ nmap,
                                                int n, const DevState *st, const DevPose *log, int type,
                                                uint8_t *__restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const f3 nv = ld3(nmap, i), vv = ld3(vmap, i);
  uint8_t o[3] = {0, 0, 0};
  if (type == 1) {
    o[0] = render_u8(fabsf(nv.x) * 255);
    o[1] = render_u8(fabsf(nv.y) * 255);
    o[2] = render_u8(fabsf(nv.z) * 255);
  } else if (!(nv.x == 0 && nv.y == 0 && nv.z == 0) && !(vv.x == 0 && vv.y == 0 && vv.z == 0)) {
    const DevPose &P = log[st->n_poses - 1];
    const f3 kd = {0.3843f, 0.4745f, 0.580f};
    const float intensity = 0.9f;
    const f3 e = normalized_ieee(sub({P.t[0], P.t[1], P.t[2]}, vv));
    const f3 l = normalized_ieee(sub({500.f, 500.f, -500.f}, vv));
    float lc = dot(nv, l);
    if (lc <= 0) lc = -lc;
    float coef = intensity * lc;
    const f3 diffuse = scl(kd, coef);
    const f3 hv = normalized_ieee(add(l, e));
    float hc = dot(nv, hv);
    if (hc < 0) hc = -hc;
    const float h2 = hc * hc, h4 = h2 * h2, h8 = h4 * h4;
    coef = intensity * (h8 * h2);
    const double spec = 0.5 * (double)coef;
    o[0] = render_u8((float)fmin(1.0, (double)(0.1f + diffuse.x) + spec) * 255);
    o[1] = render_u8((float)fmin(1.0, (double)(0.1f + diffuse.y) + spec) * 255);
    o[2] = render_u8((float)fmin(1.0, (double)(0.1f + diffuse.z) + spec) * 255);
  }
  out[3 * (size_t)i] = o[0];
  out[3 * (size_t)i + 1] = o[1];
  out[3 * (size_t)i + 2] = o[2];
}

}  // namespace

// ---------------------------------------------------------------------------
// launchers

#ifdef KFX_INT_TRACE
static unsigned long long *g_int_trace = nullptr;
static int g_int_trace_waves = 0;
}  // namespace kfx
// debug build only: the last integrate launch's per-wave records
// {start, end, xcc_id<<32 | hw_id, chunk<<32 | tile} (wall clock, 100 MHz)
extern "C" int kfx_debug_integrate_trace(unsigned long long *out, int cap) {
  const int n = std::min(cap, kfx::g_int_trace_waves);
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpy(out, kfx::g_int_trace, sizeof(unsigned long long) * 4 * n, hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  return n;
}
namespace kfx {
#endif

void launch_frame_begin(hipStream_t s, DevState *st, float2 *dl0, LevelGeom g0) {
  hipLaunchKernelGGL(k_frame_begin, dim3(1), dim3(1), 0, s, st,
                     dl0 ? (unsigned *)(dl0 + (size_t)g0.w * g0.h) : nullptr);
}

void launch_pyr_down(hipStream_t s, const float *src, const uint16_t *src16, int w, int h,
                     float *dst, DevState *st_begin, float2 *dl0) {
  unsigned *dmax = dl0 ? (unsigned *)(dl0 + (size_t)w * h) : nullptr;  // level-0 source dims
  const int dw = (w + 1) / 2, dh = (h + 1) / 2;
  dim3 blk(64, 4), grd((dw + 63) / 64, (dh + 3) / 4);
  if (src16)
    hipLaunchKernelGGL(k_pyr_down<uint16_t>, grd, blk, 0, s, src16, w, h, dst, dw, dh, st_begin, dmax);
  else
    hipLaunchKernelGGL(k_pyr_down<float>, grd, blk, 0, s, src, w, h, dst, dw, dh, st_begin, dmax);
}

void launch_preprocess_maps(hipStream_t s, int levels, const float *const raw[kMaxLevels],
                            const uint16_t *raw0_u16, const LevelGeom *g, FrameView cur, int ksz,
                            float sigma_color, float sigma_spatial, float max_dist,
                            const float *inv_lambda, float2 *dl0) {
  BilatArgs a{};
  a.invl = inv_lambda;
  a.dl0 = dl0;
  a.t = make_tiles(levels, g);
  for (int l = 0; l < levels; ++l) {
    a.raw[l] = raw[l];
    a.d[l] = cur.d[l];
    a.v[l] = cur.v[l];
    a.n[l] = cur.n[l];
  }
  a.raw0_u16 = raw0_u16;
  a.ksz = ksz;
  a.s_half = -0.5f / (sigma_spatial * sigma_spatial);
  a.c_half = -0.5f / (sigma_color * sigma_color);
  a.max_dist = max_dist;
  hipLaunchKernelGGL(k_preprocess_maps, dim3(a.t.off[levels]), dim3(256), 0, s, a);
}

static int icp_npix(const LevelGeom &g, int *xe) {
  *xe = (g.w / 32) * 32;  // A2: grid = floor(W/32) x floor(H/32) blocks of 32x32
  return *xe * ((g.h / 32) * 32);
}

int icp_blocks(const LevelGeom &g) {
  int xe;
  const int n = icp_npix(g, &xe);
  int nb = (n + kIcpBlockPix - 1) / kIcpBlockPix;
  return nb < 1 ? 1 : nb;
}

// The largest float x with RN(sqrtf(x)) <= t (x >= 0), so that the ICP lane's
// `sqrtf(x) <= t` is the single compare `x <= bound` for every non-negative x
// (RN(sqrt) is monotonic; a NaN x fails both).  t < 0 admits nothing, t NaN
// nothing (the bound is NaN), t = +inf everything.
float sqrt_le_bound(float t) {
  if (std::isnan(t)) return t;
  if (t < 0.f) return -1.f;
  if (std::isinf(t)) return t;
  float x = t * t;
  if (std::isinf(x)) x = std::numeric_limits<float>::max();
  while (x > 0.f && std::sqrt(x) > t) x = std::nextafter(x, 0.f);
  for (;;) {
    const float n = std::nextafter(x, std::numeric_limits<float>::infinity());
    if (std::isinf(n) || std::sqrt(n) > t) break;
    x = n;
  }
  return x;
}

IcpPlan make_icp_plan(int levels, const LevelGeom *g, const int *iters, FrameView cur,
                      FrameView prev, float dist_thr, float angle_thr) {
  IcpPlan pl{};
  pl.levels = levels;
  pl.dist2_max = sqrt_le_bound(dist_thr);
  pl.sine2_max = sqrt_le_bound(angle_thr);
  for (int l = 0; l < levels; ++l) {
    pl.g[l] = g[l];
    pl.npix[l] = icp_npix(g[l], &pl.xe[l]);
    // pixels per lane: the fewest that keep the level within one block per
    // CU (256), so coarse levels spread over more waves (shorter lane phase)
    pl.ppl[l] = std::max(1, std::min(kIcpPix, (pl.npix[l] + KFX_ICP_PPLCAP * kIcpThreads - 1) / (KFX_ICP_PPLCAP * kIcpThreads)));
    pl.groups[l] = std::max(1, (pl.npix[l] + kIcpThreads * pl.ppl[l] - 1) / (kIcpThreads * pl.ppl[l]));
    pl.iters[l] = iters[l];
    pl.cv[l] = cur.v[l];
    pl.cn[l] = cur.n[l];
    pl.pv[l] = prev.v[l];
    pl.pn[l] = prev.n[l];
    pl.nblocks = std::max(pl.nblocks, pl.groups[l]);
    pl.slots += iters[l];
  }
  pl.nblocks = std::max(pl.nblocks, 1);
  return pl;
}

bool icp_headroom(const IcpPlan &pl, int device, int cus_free) {
  int per_cu = 0, cus = 0;
  const hipError_t e = pl.stride ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_icp_track<true>, kIcpThreads, 0)
                                 : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_icp_track<false>, kIcpThreads, 0);
  if (e != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
    return false;
  return (long long)per_cu * (cus - cus_free) >= pl.nblocks;
}

bool icp_persistent_ok(IcpPlan &pl, int device) {
  if (pl.slots > kIcpMaxSlots) return false;
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_icp_track<false>, kIcpThreads, 0) != hipSuccess)
    return false;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
    return false;
  pl.stride = 0;
  if ((long long)per_cu * cus >= pl.nblocks) {
    return true;
  }
  // too many groups to be co-resident: the strided kernel on the blocks that are
  int per_cu_s = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu_s, k_icp_track<true>, kIcpThreads, 0) != hipSuccess)
    return false;
  const int cap = per_cu_s * cus;
  if (cap <= 0 || (pl.nblocks + cap - 1) / cap > kIcpStrideMax) return false;
  pl.nblocks = cap;
  pl.stride = 1;
  // levels with more groups than blocks: equal contiguous ranges (every block
  // runs ceil(npix / cap) pixels instead of one or two whole groups)
  for (int l = 0; l < pl.levels; ++l) {
    pl.span[l] = 0;
    if (pl.groups[l] <= cap) continue;
    const int per = (pl.npix[l] + cap - 1) / cap;
    const int span = (per + kIcpThreads - 1) / kIcpThreads * kIcpThreads;
    // a block's fp64 sums of 2^-32-scaled products (|product| < 2^7) stay
    // exact integers below 2^53 for up to 2^14 pixels: keep a margin of 2
    if (span > 8 * kIcpPix * kIcpThreads) continue;
    pl.span[l] = span;
    pl.groups[l] = (pl.npix[l] + span - 1) / span;
  }
  return true;
}

hipError_t launch_icp_track(hipStream_t s, const IcpPlan &pl, DevState *st, IcpSync *sync, int begin, bool coop) {
  if (coop) {
    // the runtime guarantees the grid co-resident (or fails the launch), so
    // the grid barrier cannot wait on an unscheduled block (~15 us slower)
    IcpPlan a0 = pl;
    DevState *a1 = st;
    IcpSync *a2 = sync;
    int a3 = begin;
    void *args[] = {&a0, &a1, &a2, &a3};
    return hipLaunchCooperativeKernel(pl.stride ? reinterpret_cast<const void *>(k_icp_track<true>)
                                                : reinterpret_cast<const void *>(k_icp_track<false>),
                                      dim3(pl.nblocks),
                                      dim3(kIcpThreads), args, 0, s);
  }
  if (pl.stride)
    hipLaunchKernelGGL(k_icp_track<true>, dim3(pl.nblocks), dim3(kIcpThreads), 0, s, pl, st, sync, begin);
  else
    hipLaunchKernelGGL(k_icp_track<false>, dim3(pl.nblocks), dim3(kIcpThreads), 0, s, pl, st, sync, begin);
  return hipGetLastError();
}

void launch_icp(hipStream_t s, const LevelGeom &g, const float *cv, const float *cn,
                const float *pv, const float *pn, float dist_thr, float angle_thr, DevState *st,
                unsigned long long *shards, unsigned *ticket, int force, int update, int band, int nbands) {
  int xe;
  const int n = icp_npix(g, &xe);
  const int ye = n / std::max(xe, 1);  // band = whole rows of the floor-covered region
  const int p0 = xe * (int)((long long)ye * band / nbands), p1 = xe * (int)((long long)ye * (band + 1) / nbands);
  const int nb = std::max(1, (p1 - p0 + kIcpBlockPix - 1) / kIcpBlockPix);
  hipLaunchKernelGGL(k_icp_acc, dim3(nb), dim3(kIcpThreads), 0, s, g, xe, p0, p1, cv, cn, pv, pn,
                     sqrt_le_bound(dist_thr), sqrt_le_bound(angle_thr), st, shards, ticket, force, update);
}

// The solve of one ICP iteration from DevState::sums (the all-reduced partials
// of the sharded mode): icp_registration.cpp:33-42, as in k_icp_acc's last block.
__global__ void k_icp_solve(DevState *__restrict__ st) {
  if (st->mode != MODE_TRACK || st->icp_fail) return;
  __shared__ double sumd[27];
  if (threadIdx.x < 27) sumd[threadIdx.x] = icp_sum_value(st->sums[threadIdx.x]);
  __syncthreads();
  DevPose p = st->icp_pose;
  double x[6];
  const int f = icp_update(sumd, p, x);
  if (threadIdx.x == 0) {
    if (f) {
      st->icp_fail = 1;
    } else {
      st->icp_pose = p;
#pragma unroll
      for (int i = 0; i < 6; ++i) st->x[i] = x[i];
    }
  }
}
void launch_icp_solve(hipStream_t s, DevState *st) { hipLaunchKernelGGL(k_icp_solve, dim3(1), dim3(64), 0, s, st); }

// In-process group: DevState::sums of every member <- their sum (int64, exact)
__global__ void k_group_sum_icp(GroupSt g) {
  if (threadIdx.x >= 27) return;
  long long a = 0;
  for (int k = 0; k < g.n; ++k) a += g.p[k]->sums[threadIdx.x];
  for (int k = 0; k < g.n; ++k) g.p[k]->sums[threadIdx.x] = a;
}
void launch_group_sum_icp(hipStream_t s, DevState *const *st, int n) {
  GroupSt g{};
  g.n = n;
  for (int k = 0; k < n; ++k) g.p[k] = st[k];
  hipLaunchKernelGGL(k_group_sum_icp, dim3(1), dim3(64), 0, s, g);
}

// VolView::iadapt: 1 = capped chunks longest-first, 0 = geometric chunks in block order
static int integrate_mode(const VolView &v) {
  return v.zn >= KFX_INT_ADAPT_ZN && v.zn < KFX_INT_ADAPT_ZN_END ? 1 : 0;
}

int integrate_chunks(const VolView &v) {
  const int tiles = v.tiles_x * v.tiles_y;
  if (integrate_mode(v) == 1) return std::max(1, std::min(KFX_INT_NC, v.zn / 32));  // chunks of >= 32 slices
  // z-chunks so that >= KFX_INT_WAVES waves exist (16 per SIMD on 1024 SIMDs)
  int nc = (KFX_INT_WAVES + tiles - 1) / tiles;
  // Z-slabs (a context storing part of the volume's slices): also at most
  // ~KFX_INT_SLAB_CHUNK slices per chunk.  A slab's waves otherwise cover its
  // whole stored range (C4 slab 0: 344 slices, one chunk per tile: 6150
  // working waves, 70 % of the wave slots filled at the start and a tail of
  // 120-260 us waves, tools/slab_int_trace.py)
  // — as long as the slab keeps <= KFX_INT_SLAB_CAPW waves (the chunk-start
  // replays of many chunks cost more than the tail they cut: C5 slab 0, 772
  // slices of 65536 tiles, took 1.25 ms in 7 chunks against 0.85 ms in one)
  if (KFX_INT_SLAB_CHUNK > 0 && v.zn < v.Z)
    nc = std::max(nc, std::min((v.zn + KFX_INT_SLAB_CHUNK - 1) / KFX_INT_SLAB_CHUNK, KFX_INT_SLAB_CAPW / tiles));
  return std::max(1, std::min(KFX_INT_MAXCHUNK, nc));
}

// Longest-first dispatch order of k_integrate's (tile, chunk) items for the
// next frame (VolView::iadapt): item c of tile t is one of ct(len_t) capped
// chunks of len_t / ct slices, len_t = the tile's interval length in the last
// integrate (frames are temporally coherent); surplus items (c >= ct) go last.
// A counting sort into descending length buckets by one block; any
// permutation integrates the same volume (the bucket is only a priority, so
// it may use any deterministic arithmetic: the capped chunk count is counted
// with compares, the chunk length is a float quotient).  Items of the empty
// bucket (most of them) take their slots with one LDS atomic per wave.
constexpr int kOrderBuckets = 1024;
__global__ __launch_bounds__(1024) void k_int_order(const unsigned *__restrict__ work, unsigned *__restrict__ perm,
                                                    int tiles, int nchunk, int zn, int capped, int chunkr) {
  __shared__ unsigned hist[kOrderBuckets];
  __shared__ unsigned wsum[16];
  const int t = threadIdx.x, lane = t & 63;
  hist[t] = 0u;
  __syncthreads();
  const int n = tiles * nchunk;
  const float scale = (float)(kOrderBuckets - 2) / ((float)zn + 2.f);
  auto bucket = [&](int item) {
    const int tile = item % tiles, c = item / tiles;
    const unsigned len = work[tile];
    if (len == 0u) return kOrderBuckets - 1;
    int clen;
    if (capped) {
      // ct = min(nchunk, ceil(len * nchunk / zn)) = #{k < nchunk : k zn < len nchunk}
      const unsigned a = len * (unsigned)nchunk;
      int ct = 0;
      for (int k = 0; k < nchunk; ++k) ct += (unsigned)k * (unsigned)zn < a ? 1 : 0;
      if (c >= ct) return kOrderBuckets - 1;
      clen = (int)((float)len / (float)ct);
    } else {  // the chunk's length under the split k_integrate uses (geometric / equal)
      VolView q{};
      q.iadapt = 0;
      int za, zb;
      int_chunk(q, chunkr, c, nchunk, 0, (int)len - 1, za, zb);
      clen = zb - za + 1;
    }
    return kOrderBuckets - 2 - min(kOrderBuckets - 2, (int)((float)max(clen, 0) * scale));
  };
  // (n is a multiple of nothing in particular: the loop runs whole waves, the
  // lanes past n take no bucket)
  const int nw = (n + 1023) & ~1023;
  for (int i = t; i < nw; i += 1024) {
    const int b = i < n ? bucket(i) : -1;
    const unsigned long long empty = __ballot(b == kOrderBuckets - 1);
    if (b >= 0 && b != kOrderBuckets - 1) atomicAdd(&hist[b], 1u);
    if (lane == 0 && empty) atomicAdd(&hist[kOrderBuckets - 1], (unsigned)__popcll(empty));
  }
  __syncthreads();
  // exclusive scan of the 1024 bucket counts: waves, then wave totals
  const unsigned c = hist[t];
  unsigned incl = c;
  for (int off = 1; off < 64; off <<= 1) {
    const unsigned u = __shfl_up(incl, off);
    if ((t & 63) >= off) incl += u;
  }
  if ((t & 63) == 63) wsum[t >> 6] = incl;
  __syncthreads();
  unsigned base = 0;
  for (int w = 0; w < (t >> 6); ++w) base += wsum[w];
  __syncthreads();
  hist[t] = base + incl - c;
  __syncthreads();
  for (int i = t; i < nw; i += 1024) {
    const int b = i < n ? bucket(i) : -1;
    const unsigned long long empty = __ballot(b == kOrderBuckets - 1);
    unsigned e0 = 0u;
    if (lane == 0 && empty) e0 = atomicAdd(&hist[kOrderBuckets - 1], (unsigned)__popcll(empty));
    e0 = __shfl(e0, 0);
    if (b == kOrderBuckets - 1)
      perm[e0 + (unsigned)__popcll(empty & ((1ull << lane) - 1ull))] = (unsigned)i;
    else if (b >= 0)
      perm[atomicAdd(&hist[b], 1u)] = (unsigned)i;
  }
}

void launch_integrate(hipStream_t s, VolView v, LevelGeom g0, const float2 *dl0, const float *dmap,
                      const float *invl, const uint8_t *bgr, DevState *st, DevPose *log, DevPose vpose,
                      const float *xpose, unsigned long long *counters, bool order) {
  const int tiles = v.tiles_x * v.tiles_y;
  const int nchunk = integrate_chunks(v);
  v.inchunk = nchunk;
  v.iadapt = integrate_mode(v);
  if (!v.iadapt) v.iperm = nullptr, v.iwork = nullptr;  // geometric chunks in block order
  if (counters) v.iwork = nullptr;  // the count-only pass leaves the order alone
  dim3 grd(tiles * nchunk);  // one wave (block) per (tile, chunk) item
  const bool idx32 = !v.force64 && v.local_voxels() < (1ull << 31);  // 32-bit tsdf/weight byte offsets
#ifdef KFX_INT_TRACE
  static unsigned long long *trace_buf = nullptr;
  if (!trace_buf) {
    (void)hipMalloc(&trace_buf, sizeof(unsigned long long) * 4 * (1 << 20));
    g_int_trace = trace_buf;
  }
  g_int_trace_waves = (int)grd.x;
  (void)hipMemsetAsync(trace_buf, 0, sizeof(unsigned long long) * 4 * g_int_trace_waves, s);  // waves that exit early write none
  if (!counters) {
    hipLaunchKernelGGL((k_integrate<false, true>), grd, dim3(KFX_INT_BLOCK), 0, s, v, g0, dl0, dmap, invl, bgr, st,
                       log, vpose, xpose, trace_buf);
    return;
  }
#endif
#define KFX_LAUNCH_INT(C, I)                                                                             \
  hipLaunchKernelGGL((k_integrate<C, I>), grd, dim3(KFX_INT_BLOCK), 0, s, v, g0, dl0, dmap, invl, bgr, st, log, vpose, xpose, \
                     counters)
  if (counters) KFX_LAUNCH_INT(true, false);
  else if (idx32) KFX_LAUNCH_INT(false, true);
  else KFX_LAUNCH_INT(false, false);
#undef KFX_LAUNCH_INT
  if (!counters && order) launch_int_order(s, v);
}

void launch_int_order(hipStream_t s, VolView v) {
  const int tiles = v.tiles_x * v.tiles_y;
  const int nchunk = integrate_chunks(v);
  if (!integrate_mode(v) || !v.iwork || !v.iperm) return;
  hipLaunchKernelGGL(k_int_order, dim3(1), dim3(1024), 0, s, v.iwork, v.iperm, tiles, nchunk, v.zn, integrate_mode(v),
                     KFX_INT_CHUNKR);
}

#ifdef KFX_RAY_TRACE
static unsigned long long *g_ray_trace = nullptr;
static unsigned long long *g_ray_iter_host = nullptr;
static int g_ray_trace_waves = 0;
}  // namespace kfx
// debug build only: the last raycast launch's per-wave iteration records (34 u64 per wave)
extern "C" int kfx_debug_raycast_iters(unsigned long long *out, int cap) {
  const int n = std::min(cap, kfx::g_ray_trace_waves);
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpy(out, kfx::g_ray_iter_host, sizeof(unsigned long long) * 34 * n, hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  return n;
}
// debug build only: the last raycast launch's per-wave records
extern "C" int kfx_debug_raycast_trace(unsigned long long *out, int cap) {
  const int n = std::min(cap, kfx::g_ray_trace_waves);
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpy(out, kfx::g_ray_trace, sizeof(unsigned long long) * 8 * n, hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  return n;
}
namespace kfx {
#endif
void launch_raycast(hipStream_t s, VolView v, int levels, const LevelGeom *g, FrameView cur,
                    FrameView prev, const DevState *st, const DevPose *log, DevPose vpose,
                    const float *xpose, uint32_t *keys, unsigned long long *stats, const SlabPass &sp,
                    unsigned *start_sig, unsigned start_val) {
  const bool want_stats = stats != nullptr;
#ifdef KFX_RAY_TRACE
  if (!stats) {
    if (!g_ray_trace) {
      (void)hipMalloc(&g_ray_trace, sizeof(unsigned long long) * 8 * (1 << 16));
      unsigned long long *it = nullptr;
      (void)hipMalloc(&it, sizeof(unsigned long long) * 34 * (1 << 16));
      (void)hipMemcpyToSymbol(HIP_SYMBOL(g_ray_iter), &it, sizeof(it));
      g_ray_iter_host = it;
    }
    g_ray_trace_waves = (int)(((g[0].w + 15) / 16) * ((g[0].h + 15) / 16) * 4);
    stats = g_ray_trace;
  }
#endif
  RayConsts rc;
  rc.vs = {v.vs[0], v.vs[1], v.vs[2]};
  rc.vs_inv = {1.f / v.vs[0], 1.f / v.vs[1], 1.f / v.vs[2]};
  rc.gd = {v.vs[0] * 0.5f, v.vs[1] * 0.5f, v.vs[2] * 0.5f};
  rc.step = v.vs[0];
  // half an ulp of a position inside the volume is <= max_dim * 2^-23 voxels
  rc.skip_cap = std::min(511.f, std::floor(0.1f * 8388608.f / (float)std::max(v.X, std::max(v.Y, v.Z))));
  RayArgs ra{};
  ra.levels = levels;
  ra.stats = stats;
  ra.slab_pass = keys ? sp.pass : 0;
  ra.kmin = sp.kmin;
  ra.bound_abs = sp.bound_abs;
  ra.bound_rel = sp.bound_rel;
  ra.start_sig = start_sig;
  ra.start_val = start_val;
  for (int l = 0; l < levels; ++l) ra.g[l] = g[l];
  dim3 grd(((g[0].w + 15) / 16) * ((g[0].h + 15) / 16));
  // 32-bit tsdf byte offsets (24-bit operands of the tile * zn products)
  const bool idx32 = !v.force64 && v.local_voxels() < (1ull << 31) && (size_t)v.tiles_x * v.tiles_y < (1ull << 24) &&
                     v.zn < (1 << 24);
  if (want_stats) {
    if (keys && idx32)
      hipLaunchKernelGGL((k_raycast<true, true, true>), grd, dim3(256), 0, s, v, ra, rc, cur, prev, st, log,
                         vpose, xpose, keys);
    else if (keys)
      hipLaunchKernelGGL((k_raycast<false, true, true>), grd, dim3(256), 0, s, v, ra, rc, cur, prev, st, log,
                         vpose, xpose, keys);
    else if (idx32)
      hipLaunchKernelGGL((k_raycast<true, false, true>), grd, dim3(256), 0, s, v, ra, rc, cur, prev, st, log,
                         vpose, xpose, keys);
    else
      hipLaunchKernelGGL((k_raycast<false, false, true>), grd, dim3(256), 0, s, v, ra, rc, cur, prev, st, log,
                         vpose, xpose, keys);
    return;
  }
  if (keys) {
    if (idx32)
      hipLaunchKernelGGL((k_raycast<true, true>), grd, dim3(256), 0, s, v, ra, rc, cur, prev, st, log,
                         vpose, xpose, keys);
    else
      hipLaunchKernelGGL((k_raycast<false, true>), grd, dim3(256), 0, s, v, ra, rc, cur, prev, st,
                         log, vpose, xpose, keys);
  } else if (idx32) {
    hipLaunchKernelGGL((k_raycast<true, false>), grd, dim3(256), 0, s, v, ra, rc, cur, prev, st, log,
                       vpose, xpose, keys);
  } else {
    hipLaunchKernelGGL((k_raycast<false, false>), grd, dim3(256), 0, s, v, ra, rc, cur, prev, st,
                       log, vpose, xpose, keys);
  }
}

// DevState::ray_kind / ray_c2v from the current tracking state, as the
// frame's k_integrate writes them (kfx_raycast_stats: a raycast that is not
// preceded by a pipeline integrate, e.g. after kfx_stage_icp_accumulate, uses
// the current ICP pose, as k_raycast_touch does; right after a frame the
// values are the ones integrate wrote: the bookkeeping leaves the fields
// frame_kind / frame_pose read alone)
__global__ void k_ray_pose(DevState *st, const DevPose *log, DevPose vpose) {
  const int kind = frame_kind(st);
  st->ray_kind = kind;
  if (kind == 1) st->ray_c2v = pose_mul(pose_inv(vpose), frame_pose(st, log, 1));  // tsdf_volume.cpp:59
}
void launch_ray_pose(hipStream_t s, DevState *st, const DevPose *log, DevPose vpose) {
  hipLaunchKernelGGL(k_ray_pose, dim3(1), dim3(1), 0, s, st, log, vpose);
}
void launch_raycast_touch(hipStream_t s, VolView v, LevelGeom g0, const DevState *st, const DevPose *log,
                          DevPose vpose, const float *xpose, uint32_t *bits, unsigned long long *out) {
  RayConsts rc;
  rc.vs = {v.vs[0], v.vs[1], v.vs[2]};
  rc.vs_inv = {1.f / v.vs[0], 1.f / v.vs[1], 1.f / v.vs[2]};
  rc.gd = {v.vs[0] * 0.5f, v.vs[1] * 0.5f, v.vs[2] * 0.5f};
  rc.step = v.vs[0];
  rc.skip_cap = 0.f;
  const size_t words = (v.local_voxels() + 31) / 32;
  (void)hipMemsetAsync(bits, 0, words * 4, s);
  (void)hipMemsetAsync(out, 0, 16, s);
  hipLaunchKernelGGL(k_raycast_touch, dim3((g0.w * g0.h + 255) / 256), dim3(256), 0, s, v, g0, rc, st, log, vpose,
                     xpose, bits, out + 1);
  hipLaunchKernelGGL(k_popcount, dim3(2048), dim3(256), 0, s, bits, words, out);
}

void launch_resize(hipStream_t s, int levels, const LevelGeom *g, FrameView cur, FrameView prev,
                   const DevState *st, const float *xpose) {
  RayArgs ra{};
  ra.levels = levels;
  for (int l = 0; l < levels; ++l) ra.g[l] = g[l];
  dim3 grd(((g[0].w + 15) / 16) * ((g[0].h + 15) / 16));
  hipLaunchKernelGGL(k_resize, grd, dim3(256), 0, s, ra, cur, prev, st, xpose);
}

void launch_render(hipStream_t s, const float *vmap, const float *nmap, int n, const DevState *st,
                   const DevPose *log, int type, uint8_t *out) {
  hipLaunchKernelGGL(k_render, dim3((n + 255) / 256), dim3(256), 0, s, vmap, nmap, n, st, log, type, out);
}

void launch_slab_mask(hipStream_t s, const uint32_t *keys, const uint32_t *key_min, int n) {
  hipLaunchKernelGGL(k_slab_mask, dim3((n + 255) / 256), dim3(256), 0, s, keys, key_min, n);
}
void launch_slab_expand(hipStream_t s, LevelGeom g0, const uint32_t *pay, FrameView cur, FrameView prev,
                        const DevState *st, const DevPose *log, DevPose vpose) {
  hipLaunchKernelGGL(k_slab_expand, dim3((g0.w * g0.h + 255) / 256), dim3(256), 0, s, g0, pay, cur, prev, st,
                     log, vpose);
}

void launch_group_reduce(hipStream_t s, uint32_t *const *in, int n_in, uint32_t *const *out,
                         int n_out, size_t count, bool is_max) {
  GroupBufs a{}, b{};
  a.n = n_in;
  b.n = n_out;
  for (int k = 0; k < n_in; ++k) a.p[k] = in[k];
  for (int k = 0; k < n_out; ++k) b.p[k] = out[k];
  size_t blocks = (count + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(k_group_reduce, dim3((unsigned)blocks), dim3(256), 0, s, a, b, count,
                     is_max ? 1 : 0);
}

static int extract_chunks(int zlo, int zhi) {
  if (zhi <= zlo) return 0;
  const int a = (zlo / kExtractZ) * kExtractZ;
  return (zhi - a + kExtractZ - 1) / kExtractZ;
}
size_t extract_waves(const VolView &v, int zlo, int zhi) {
  return (size_t)v.tiles_x * v.tiles_y * (size_t)extract_chunks(zlo, zhi);
}
template <int kMode>
static void launch_xsweep(hipStream_t s, const VolView &v, DevPose vpose, int zlo, int zhi, const uint8_t *tab,
                          unsigned *counts, const unsigned long long *offsets, float *out, unsigned long long cap,
                          unsigned long long *ctr, unsigned long long *pool_at, unsigned *list, unsigned *overflow) {
  const int nc = extract_chunks(zlo, zhi);
  if (nc == 0) return;
  const int tiles = v.tiles_x * v.tiles_y;
  // units per wave: as many as keep >= 64 K waves (at least 1, at most 64)
  const size_t units = (size_t)tiles * nc;
  int K = 1;
  while (K < 64 && units / (size_t)(2 * K) >= (size_t)KFX_XSWEEP_WAVES) K *= 2;
  dim3 grd((tiles + 4 * K - 1) / (4 * K), nc);  // 4 waves of K units per block
  if (tab)
    hipLaunchKernelGGL((k_xsweep<kMode, true>), grd, dim3(256), 0, s, v, vpose, zlo, zhi, tab, counts, offsets, out,
                       cap, ctr, pool_at, list, overflow, K);
  else
    hipLaunchKernelGGL((k_xsweep<kMode, false>), grd, dim3(256), 0, s, v, vpose, zlo, zhi, tab, counts, offsets, out,
                       cap, ctr, pool_at, list, overflow, K);
}
void launch_extract(hipStream_t s, const VolView &v, DevPose vpose, int zlo, int zhi,
                    unsigned *counts, const unsigned long long *offsets, float *out,
                    unsigned long long cap) {
  if (offsets)
    launch_xsweep<kXEmit>(s, v, vpose, zlo, zhi, nullptr, counts, offsets, out, cap, nullptr, nullptr, nullptr, nullptr);
  else
    launch_xsweep<kXCount>(s, v, vpose, zlo, zhi, nullptr, counts, nullptr, nullptr, 0, nullptr, nullptr, nullptr, nullptr);
}
void launch_mesh(hipStream_t s, const VolView &v, DevPose vpose, int zlo, int zhi, const uint8_t *tab,
                 unsigned *counts, const unsigned long long *offsets, float *out, unsigned long long cap) {
  if (offsets)
    launch_xsweep<kXEmit>(s, v, vpose, zlo, zhi, tab, counts, offsets, out, cap, nullptr, nullptr, nullptr, nullptr);
  else
    launch_xsweep<kXCount>(s, v, vpose, zlo, zhi, tab, counts, nullptr, nullptr, 0, nullptr, nullptr, nullptr, nullptr);
}
size_t scan_blocks(size_t n) { return (n + 4095) / 4096; }
void launch_extract_pool(hipStream_t s, const VolView &v, DevPose vpose, int zlo, int zhi, const uint8_t *tab,
                         unsigned *counts, unsigned long long *ctr, unsigned long long *pool_at, unsigned *list,
                         float *pool, unsigned long long pool_cap, unsigned *overflow) {
  launch_xsweep<kXPool>(s, v, vpose, zlo, zhi, tab, counts, nullptr, pool, pool_cap, ctr, pool_at, list, overflow);
}
void launch_extract_copy(hipStream_t s, const unsigned *list, unsigned nlist, const unsigned *counts,
                         const unsigned long long *pool_at, const unsigned long long *offsets, const float *pool,
                         float *out, unsigned long long cap, int per) {
  if (nlist == 0) return;
  hipLaunchKernelGGL(k_extract_copy, dim3((nlist + 3) / 4), dim3(256), 0, s, list, nlist, counts, pool_at, offsets,
                     pool, out, cap, per);
}
void launch_scan(hipStream_t s, const unsigned *counts, unsigned long long *offsets,
                 unsigned long long *bsum, size_t n, unsigned long long *total) {
  const size_t nb = scan_blocks(n);
  hipLaunchKernelGGL(k_scan_local, dim3((unsigned)nb), dim3(1024), 0, s, counts, offsets, bsum, n);
  hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(1024), 0, s, bsum, (int)nb, total);
  hipLaunchKernelGGL(k_scan_add, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, offsets, bsum, n);
}

// Per-slice integrate work of one frame (Z-slab balancing), in
// two parts per global slice z:
//   cover[z]   = 64 x the column tiles whose union interval (integrate's
//                wave-uniform z range, int_column) contains z: the voxel slots
//                integrate's waves step through, updated or not;
//   updated[z] = the voxels of those intervals whose depth test passes
//                (sdf >= -trunc, tsdf_volume.cu:56-71).
// At pose P, from the level-0 {depth, 1/lambda} table.  An estimate for
// choosing slab cuts (vc is computed directly, not accumulated), not bit-exact
// with integrate.  One wave per 8x8 column tile; per-block LDS histograms
// (cover as a difference array), flushed once.  hist: 2Z + 1 counters.
__global__ __launch_bounds__(256) void k_slice_work(VolView v, LevelGeom g, const float2 *__restrict__ dl,
                                                    DevPose P, unsigned long long *hist) {
  extern __shared__ int lh[];  // [0, Z]: cover differences; [Z + 1, 2Z + 1): updated
  const int Z = v.Z;
  for (int i = threadIdx.x; i < 2 * Z + 1; i += blockDim.x) lh[i] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int tile = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (tile < v.tiles_x * v.tiles_y) {  // wave-uniform
    const int x = (tile % v.tiles_x) * 8 + (lane & 7), y = (tile / v.tiles_x) * 8 + (lane >> 3);
    f3 c0, zs;
    int zl, zh;
    int_column(v, g, dl, P, x, y, c0, zs, zl, zh);
    int wl = zl, wh = zh;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      wl = min(wl, __shfl_xor(wl, off));
      wh = max(wh, __shfl_xor(wh, off));
    }
    int_tile_clip(v, g, dl, c0, zs, lane, zl, zh, wl, wh);  // what k_integrate visits
    if (wl <= wh) {
      if (lane == 0) {
        atomicAdd(&lh[wl], 64);
        atomicSub(&lh[wh + 1], 64);
      }
      for (int z = wl; z <= wh; ++z) {
        bool pass = false;
        if (z >= zl && z <= zh) {
          const f3 vc = add(c0, scl(zs, (float)z));
          if (vc.z > 0.f) {
            const float iz = 1.f / vc.z;
            const int u = (int)rintf(vc.x * iz * g.fx + g.cx), w = (int)rintf(vc.y * iz * g.fy + g.cy);
            if (u >= 0 && u < g.w && w >= 0 && w < g.h) {
              const float2 d = dl[(size_t)w * g.w + u];
              pass = d.x > 0.f && d.x - d.y * sqrtf(dot(vc, vc)) >= -v.trunc;
            }
          }
        }
        const int n = __popcll(__ballot(pass));
        if (lane == 0 && n) atomicAdd(&lh[Z + 1 + z], n);
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * Z + 1; i += blockDim.x)
    if (lh[i]) atomicAdd(&hist[i], (unsigned long long)(long long)lh[i]);  // (two's complement sums)
}

void launch_slice_work(hipStream_t s, const VolView &v, DevPose vol2cam, LevelGeom g0, const float2 *dl0,
                       unsigned long long *hist) {
  VolView gv = v;  // the whole volume's slices, whatever this context stores
  gv.zb = 0;
  gv.zn = v.Z;
  const int tiles = v.tiles_x * v.tiles_y;
  hipLaunchKernelGGL(k_slice_work, dim3((tiles + 3) / 4), dim3(256), (size_t)(2 * v.Z + 1) * 4, s, gv, g0, dl0,
                     vol2cam, hist);
}

// Host frame upload by the GPU itself: the source is page-locked host memory
// mapped into the device address space (the pinned ring or a buffer the caller
// registered), read over PCIe by a small grid of 16-B loads, several in flight
// per lane, and written to the device slot.  Replaces hipMemcpyAsync, whose
// host-side cost per call (~0.15 ms for a VGA frame, tools/host_input_probe.py)
// made the caller's thread the bottleneck of kfx_pipeline_async.
struct HostFetch {
  const unsigned char *src[2];
  unsigned char *dst[2];
  size_t bytes[2];
};
#ifndef KFX_FETCH_BLOCKS
#define KFX_FETCH_BLOCKS 4  // host fetch grid (PCIe-latency bound, 4 x 256 lanes x 4 x 16 B in flight: 2.15 MB in ~0.1 ms, hidden behind the frame before it; 4 blocks beat 16 / 64 / 256 by 3-5 % of a host frame: fewer CUs taken from the frame kernels)
#endif
constexpr int kFetchUnroll = 4;
__global__ __launch_bounds__(256) void k_host_fetch(HostFetch f) {
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t nth = (size_t)gridDim.x * blockDim.x;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const unsigned char *src = f.src[s];
    unsigned char *dst = f.dst[s];
    const size_t n = f.bytes[s];
    if (!n) continue;
    if (((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst) | n) & 15u) == 0) {
      using u32x4 = unsigned __attribute__((ext_vector_type(4)));
      const u32x4 *s4 = reinterpret_cast<const u32x4 *>(src);
      u32x4 *d4 = reinterpret_cast<u32x4 *>(dst);
      const size_t n4 = n / 16;
      for (size_t i = tid; i < n4; i += nth * kFetchUnroll) {
        u32x4 v[kFetchUnroll];
#pragma unroll
        for (int u = 0; u < kFetchUnroll; ++u)
          if (i + u * nth < n4) v[u] = __builtin_nontemporal_load(s4 + i + u * nth);
#pragma unroll
        for (int u = 0; u < kFetchUnroll; ++u)
          if (i + u * nth < n4) d4[i + u * nth] = v[u];
      }
    } else {  // unaligned caller buffers: bytes
      for (size_t i = tid; i < n; i += nth) dst[i] = src[i];
    }
  }
}
void launch_host_fetch(hipStream_t s, const void *src0, void *dst0, size_t n0, const void *src1, void *dst1,
                       size_t n1) {
  HostFetch f{{static_cast<const unsigned char *>(src0), static_cast<const unsigned char *>(src1)},
              {static_cast<unsigned char *>(dst0), static_cast<unsigned char *>(dst1)},
              {n0, n1}};
  hipLaunchKernelGGL(k_host_fetch, dim3(KFX_FETCH_BLOCKS), dim3(256), 0, s, f);
}

void launch_inv_lambda(hipStream_t s, LevelGeom g0, float *inv_lambda) {
  const int n = g0.w * g0.h;
  hipLaunchKernelGGL(k_inv_lambda, dim3((n + 255) / 256), dim3(256), 0, s, g0, inv_lambda);
}

static dim3 slab_grid(const VolView &v, int nz) {
  const size_t n = v.slice * (size_t)nz;
  size_t b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  return dim3((unsigned)b);
}

void launch_export_records(hipStream_t s, VolView v, int z0, int nz, uint64_t *dst) {
  hipLaunchKernelGGL(k_export_records, slab_grid(v, nz), dim3(256), 0, s, v, z0, nz, dst);
}
void launch_import_records(hipStream_t s, VolView v, int z0, int nz, const uint64_t *src, unsigned *bad) {
  hipLaunchKernelGGL(k_import_records, slab_grid(v, nz), dim3(256), 0, s, v, z0, nz, src, bad);
}
void launch_checksum(hipStream_t s, VolView v, unsigned long long *out) {
  hipLaunchKernelGGL(k_checksum, dim3(2048), dim3(256), 0, s, v, out);
}

void launch_export_soa(hipStream_t s, VolView v, int z0, int nz, int16_t *t, int16_t *w,
                       uint32_t *c) {
  hipLaunchKernelGGL(k_export_soa, slab_grid(v, nz), dim3(256), 0, s, v, z0, nz, t, w, c);
}

void launch_gather_columns(hipStream_t s, VolView v, const int32_t *cols, int n, int16_t *t, int16_t *w,
                           uint32_t *c) {
  const size_t total = (size_t)n * (v.own1 - v.own0);
  const unsigned b = (unsigned)std::min<size_t>(8192, (total + 255) / 256);
  hipLaunchKernelGGL(k_gather_columns, dim3(std::max(1u, b)), dim3(256), 0, s, v, cols, n, t, w, c);
}

void launch_occ_rebuild(hipStream_t s, VolView v) {
  (void)hipMemsetAsync(v.bocc, 0, v.bocc_bytes(), s);
  (void)hipMemsetAsync(v.socc, 0, v.socc_bytes(), s);
  const size_t waves = (size_t)v.tiles_x * v.tiles_y * v.nbz;
  hipLaunchKernelGGL(k_occ_rebuild, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, s, v);
}

}  // namespace kfx
