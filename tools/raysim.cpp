// raysim — CPU model of k_raycast's march schedule (analysis tool, not product).
//
// Replays, lane by lane and wave by wave (8x8 pixel tiles, lanes in lockstep
// with the kernel's __any loops), the empty-space-skipping march of
// k_raycast (slam-kinectfusion_amd/csrc/kfx_kernels.hip) over a volume dumped
// by tools/raysim_gen.py, and counts per wave the dependent round trips the
// kernel makes: skip-lookup rounds, sample-batch rounds, normal passes.  The
// occupancy maps are rebuilt from the volume (bricks / super-bricks holding a
// negative tsdf, dilated by one: the kernel's marks are a superset, set when
// voxels turned negative).  Variants of the schedule are compared by modeled
// wave time (rounds x measured per-round costs, tools/ray_trace.py).
//
// build: g++ -O2 -std=c++17 -ffp-contract=off tools/raysim.cpp -o tools/build/raysim
// usage: tools/build/raysim /tmp/raysim [variant]
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

struct f3 {
  float x, y, z;
};
static f3 add(f3 a, f3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
static f3 sub(f3 a, f3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static f3 scl(f3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
static f3 mulc(f3 a, f3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
static const float kDivShortMax = 0.0000305185f;
static const float kInf = __builtin_huge_valf();

struct Vol {
  int X, Y, Z, tx, ty, nbz, stx, sty, nsz;
  std::vector<int16_t> t;
  std::vector<uint8_t> bneg, sneg;   // undilated: brick / super-brick holds a negative voxel
  std::vector<uint8_t> bocc, socc;   // dilated by one (the kernel's maps)
  std::vector<uint8_t> bdist, sdist; // Chebyshev distance (cells) to the nearest undilated-occupied cell, capped
  float vs, range;
  int16_t at(int x, int y, int z) const { return t[(size_t)z * X * Y + (size_t)y * X + x]; }
  size_t bi(int x, int y, int z) const { return ((size_t)z * ty + y) * tx + x; }
  size_t si(int x, int y, int z) const { return ((size_t)z * sty + y) * stx + x; }
};

static void dilate(const std::vector<uint8_t> &in, std::vector<uint8_t> &out, int nx, int ny, int nz) {
  out.assign(in.size(), 0);
  for (int z = 0; z < nz; ++z)
    for (int y = 0; y < ny; ++y)
      for (int x = 0; x < nx; ++x) {
        if (!in[((size_t)z * ny + y) * nx + x]) continue;
        for (int dz = -1; dz <= 1; ++dz)
          for (int dy = -1; dy <= 1; ++dy)
            for (int dx = -1; dx <= 1; ++dx) {
              const int a = x + dx, b = y + dy, c = z + dz;
              if (a < 0 || b < 0 || c < 0 || a >= nx || b >= ny || c >= nz) continue;
              out[((size_t)c * ny + b) * nx + a] = 1;
            }
      }
}
// capped chessboard distance to the nearest set cell (0 on a set cell)
static void chess(const std::vector<uint8_t> &in, std::vector<uint8_t> &d, int nx, int ny, int nz, int cap) {
  d.assign(in.size(), (uint8_t)cap);
  std::vector<uint8_t> cur = in, nxt;
  for (size_t i = 0; i < in.size(); ++i)
    if (in[i]) d[i] = 0;
  for (int r = 1; r < cap; ++r) {
    dilate(cur, nxt, nx, ny, nz);
    for (size_t i = 0; i < in.size(); ++i)
      if (nxt[i] && d[i] > r) d[i] = (uint8_t)r;
    cur.swap(nxt);
  }
}

struct Ray {
  // kernel state (k_raycast)
  bool live = false, cand = false, can_skip = true;
  f3 org, dir, vstep, nextp, dv, idv;
  float ray_len = 0, tfar = 0, tprev = 0;
  int sprev = 0;
  uint32_t kbase = 1;
  // candidate resume state
  f3 cvert, r_nextp;
  float r_rl = 0, r_tprev = 0;
  uint32_t r_kbase = 0;
  bool hit = false, trace = false;
  // per-lane counters
  int lookups = 0, batches = 0, normals = 0;
  int sup = 0;  // batches left before the next lookup (suppression policy)
};

struct Sim {
  Vol v;
  float R[9], T[3];
  int W = 640, H = 480;
  float fx = 525.f, fy = 525.f, cx = 319.5f, cy = 239.5f;
  int kR = 14;
  float skip_cap = 0;
  int variant = 0;

  float voxel2tsdf(f3 p) const {
    const float inv = 1.f / v.vs;
    const int x = (int)rintf(p.x * inv), y = (int)rintf(p.y * inv), z = (int)rintf(p.z * inv);
    if (x >= v.X - 1 || y >= v.Y - 1 || z >= v.Z - 1 || x < 1 || y < 1 || z < 1) return NAN;
    return (float)v.at(x, y, z) * kDivShortMax;
  }
  float interp(f3 cf) const {
    const int gx = (int)floorf(cf.x), gy = (int)floorf(cf.y), gz = (int)floorf(cf.z);
    if (gx < 0 || gx >= v.X - 1 || gy < 0 || gy >= v.Y - 1 || gz < 0 || gz >= v.Z - 1) return NAN;
    const float a = cf.x - (float)gx, b = cf.y - (float)gy, c = cf.z - (float)gz;
    auto T = [&](int x, int y, int z) { return (float)v.at(x, y, z) * kDivShortMax; };
    float s = 0.f;
    s += T(gx, gy, gz) * (1 - a) * (1 - b) * (1 - c);
    s += T(gx, gy, gz + 1) * (1 - a) * (1 - b) * c;
    s += T(gx, gy + 1, gz) * (1 - a) * b * (1 - c);
    s += T(gx, gy + 1, gz + 1) * (1 - a) * b * c;
    s += T(gx + 1, gy, gz) * a * (1 - b) * (1 - c);
    s += T(gx + 1, gy, gz + 1) * a * (1 - b) * c;
    s += T(gx + 1, gy + 1, gz) * a * b * (1 - c);
    s += T(gx + 1, gy + 1, gz + 1) * a * b * c;
    return s;
  }
  bool normal_ok(f3 p) const {
    const float inv = 1.f / v.vs, gd = v.vs * 0.5f;
    auto ip = [&](f3 q) { return interp(scl(q, inv)); };
    f3 n;
    n.x = (ip({p.x + gd, p.y, p.z}) - ip({p.x - gd, p.y, p.z})) / gd;
    n.y = (ip({p.x, p.y + gd, p.z}) - ip({p.x, p.y - gd, p.z})) / gd;
    n.z = (ip({p.x, p.y, p.z + gd}) - ip({p.x, p.y, p.z - gd})) / gd;
    const float l = sqrtf(n.x * n.x + n.y * n.y + n.z * n.z);
    const f3 m = {n.x / l, n.y / l, n.z / l};
    return !std::isnan(m.x * m.y * m.z);
  }

  void setup(Ray &r, int x, int y) const {
    const float p0 = (1.f * ((float)x - cx)) / fx, p1 = (1.f * ((float)y - cy)) / fy, p2 = 1.f;
    const float v0 = R[0] * p0 + R[1] * p1 + R[2] * p2;
    const float v1 = R[3] * p0 + R[4] * p1 + R[5] * p2;
    const float v2 = R[6] * p0 + R[7] * p1 + R[8] * p2;
    const float t = sqrtf(v0 * v0 + v1 * v1 + v2 * v2);
    r.dir = {v0 / t, v1 / t, v2 / t};
    r.org = {T[0], T[1], T[2]};
    const f3 invR = {1.f / r.dir.x, 1.f / r.dir.y, 1.f / r.dir.z};
    const f3 tbot = mulc(invR, sub({0.f, 0.f, 0.f}, r.org));
    const f3 ttop = mulc(invR, sub({v.range, v.range, v.range}, r.org));
    const f3 tmin = {fminf(ttop.x, tbot.x), fminf(ttop.y, tbot.y), fminf(ttop.z, tbot.z)};
    const f3 tmax = {fmaxf(ttop.x, tbot.x), fmaxf(ttop.y, tbot.y), fmaxf(ttop.z, tbot.z)};
    const float tnear = fmaxf(fmaxf(tmin.x, tmin.y), fmaxf(tmin.x, tmin.z));
    r.tfar = fminf(fminf(tmax.x, tmax.y), fminf(tmax.x, tmax.z));
    r.ray_len = fmaxf(tnear, 0.f);
    r.live = r.ray_len < r.tfar;
    r.vstep = scl(r.dir, v.vs);
    r.ray_len += v.vs;
    r.nextp = add(r.org, scl(r.dir, r.ray_len));
    r.tprev = r.live ? voxel2tsdf(r.nextp) : NAN;
    r.sprev = std::isnan(r.tprev) ? 0 : (r.tprev > 0.f ? 1 : (r.tprev < 0.f ? -1 : 0));
    const float vsi = 1.f / v.vs;
    r.dv = scl(r.vstep, vsi);
    r.idv = {1.f / fabsf(r.dv.x), 1.f / fabsf(r.dv.y), 1.f / fabsf(r.dv.z)};
    r.can_skip = !std::isnan(r.dv.x + r.dv.y + r.dv.z);
  }

  static float axis_limit(float c, float d, float id, float lo, float hi) {
    return d > 0.f ? (hi + 0.2f - c) * id : (d < 0.f ? (c - lo + 0.2f) * id : kInf);
  }
  static float box_limit(int B, int bx, int by, int nbx, int nby, float zl, float zh, float cx_, float cy_, float cz,
                         f3 dv, f3 idv) {
    const float xl = bx > 0 ? (float)(B * bx - B) : -kInf, xh = bx < nbx - 1 ? (float)(B * bx + 2 * B - 1) : kInf;
    const float yl = by > 0 ? (float)(B * by - B) : -kInf, yh = by < nby - 1 ? (float)(B * by + 2 * B - 1) : kInf;
    return fminf(fminf(axis_limit(cx_, dv.x, idv.x, xl, xh), axis_limit(cy_, dv.y, idv.y, yl, yh)),
                 axis_limit(cz, dv.z, idv.z, zl, zh));
  }
  // the z-run of clear cells from cell c along the column, in the direction of travel
  template <typename F>
  static void zrun(F occ, int lc, int n, int B, float dz, float &zl, float &zh) {
    zl = -kInf, zh = kInf;
    if (dz > 0.f) {
      int top = lc;
      while (top + 1 < n && !occ(top + 1)) ++top;
      if (top < n - 1) zh = (float)(B * top + 2 * B - 1);
    } else {
      int bot = lc;
      while (bot - 1 >= 0 && !occ(bot - 1)) --bot;
      if (bot > 0) zl = (float)(B * bot - B);
    }
  }
  // one skip lookup of the kernel (the dilated maps): samples that may be
  // replayed from the current position (lim < 1: blocked)
  float lookup_kernel(const Ray &r) const {
    const float inv = 1.f / v.vs;
    const float cxv = r.nextp.x * inv, cyv = r.nextp.y * inv, czv = r.nextp.z * inv;
    const int ix = (int)floorf(cxv), iy = (int)floorf(cyv), iz = (int)floorf(czv);
    const int bx = std::min(std::max(ix >> 3, 0), v.tx - 1), by = std::min(std::max(iy >> 3, 0), v.ty - 1);
    const int lbz = std::min(std::max(iz >> 3, 0), v.nbz - 1);
    const int sx = std::min(std::max(ix >> 5, 0), v.stx - 1), sy = std::min(std::max(iy >> 5, 0), v.sty - 1);
    const int lsz = std::min(std::max(iz >> 5, 0), v.nsz - 1);
    float lim = 0.f;
    const bool sclear = !v.socc[v.si(sx, sy, lsz)];
    if (!v.bocc[v.bi(bx, by, lbz)] && !(variant == 4 && sclear)) {
      float zl, zh;
      zrun([&](int z) { return v.bocc[v.bi(bx, by, z)] != 0; }, lbz, v.nbz, 8, r.dv.z, zl, zh);
      lim = box_limit(8, bx, by, v.tx, v.ty, zl, zh, cxv, cyv, czv, r.dv, r.idv);
    }
    if (sclear) {
      float zl, zh;
      zrun([&](int z) { return v.socc[v.si(sx, sy, z)] != 0; }, lsz, v.nsz, 32, r.dv.z, zl, zh);
      lim = fmaxf(lim, box_limit(32, sx, sy, v.stx, v.sty, zl, zh, cxv, cyv, czv, r.dv, r.idv));
    }
    return lim;
  }
  // variant: boxes of the capped chessboard distance field (radius d-1 cells of
  // undilated-clear space around the current cell; d >= 2 is the kernel's test)
  float lookup_dist(const Ray &r) const {
    const float inv = 1.f / v.vs;
    const float cxv = r.nextp.x * inv, cyv = r.nextp.y * inv, czv = r.nextp.z * inv;
    const int ix = (int)floorf(cxv), iy = (int)floorf(cyv), iz = (int)floorf(czv);
    auto lvl = [&](int B, int nx, int ny, int nz, const std::vector<uint8_t> &d) {
      const int bx = std::min(std::max(ix / B, 0), nx - 1), by = std::min(std::max(iy / B, 0), ny - 1);
      const int bz = std::min(std::max(iz / B, 0), nz - 1);
      const int dd = d[((size_t)bz * ny + by) * nx + bx];
      if (dd < 1) return 0.f;
      const int rr = dd - 1;  // clear cells within rr of (bx, by, bz)
      auto lo = [&](int b, int n) { return b - rr > 0 ? (float)(B * (b - rr)) : -kInf; };
      auto hi = [&](int b, int n) { return b + rr < n - 1 ? (float)(B * (b + rr) + B - 1) : kInf; };
      return fminf(fminf(axis_limit(cxv, r.dv.x, r.idv.x, lo(bx, nx), hi(bx, nx)),
                         axis_limit(cyv, r.dv.y, r.idv.y, lo(by, ny), hi(by, ny))),
                   axis_limit(czv, r.dv.z, r.idv.z, lo(bz, nz), hi(bz, nz)));
    };
    return fmaxf(lvl(8, v.tx, v.ty, v.nbz, v.bdist), lvl(32, v.stx, v.sty, v.nsz, v.sdist));
  }

  // variant 3: probes ahead along the ray in the same round trip: probe k at
  // sample k*m (m = floor(7.4 / max|dv|) for bricks, 31.4 for super-bricks):
  // a dilated-clear cell at the probe clears every sample within m of it
  int probesK = 8, probeS = 0;
  int suppress = 0;  // after a failed lookup, this many batches run without a lookup
  float lookup_probe(const Ray &r) const {
    const float inv = 1.f / v.vs;
    const float mx = fmaxf(fabsf(r.dv.x), fmaxf(fabsf(r.dv.y), fabsf(r.dv.z)));
    auto run = [&](int B, float reach, int nx, int ny, int nz, const std::vector<uint8_t> &occ, int K) {
      const int m = (int)floorf(reach / mx);
      if (m < 1) return 0.f;
      int k = 0;
      for (; k < K; ++k) {
        const float s = (float)(k * m);
        const float qx = r.nextp.x * inv + s * r.dv.x, qy = r.nextp.y * inv + s * r.dv.y,
                    qz = r.nextp.z * inv + s * r.dv.z;
        const int bx = std::min(std::max((int)floorf(qx) / B, 0), nx - 1);
        const int by = std::min(std::max((int)floorf(qy) / B, 0), ny - 1);
        const int bz = std::min(std::max((int)floorf(qz) / B, 0), nz - 1);
        if (floorf(qx) < 0 || floorf(qy) < 0 || floorf(qz) < 0) {
          if (occ[((size_t)bz * ny + by) * nx + bx]) break;
        } else if (occ[((size_t)bz * ny + by) * nx + bx]) break;
      }
      return (float)(k * m);  // samples [0, k*m] are clear
    };
    float lim = run(8, 7.4f, v.tx, v.ty, v.nbz, v.bocc, probesK);
    if (probeS) lim = fmaxf(lim, run(32, 31.4f, v.stx, v.sty, v.nsz, v.socc, probeS));
    return lim;
  }

  // variant 7: up to chainK lookups in one round trip, chained while each box is
  // left through a lateral (x / y) face (the next columns along the ray's xy
  // path are predictable without the loaded words): the boxes at the model
  // positions c + total * dv, total capped by skip_cap
  int chainK = 4;
  float lookup_chain(const Ray &r) const {
    const float inv = 1.f / v.vs;
    float total = 0.f;
    for (int k = 0; k < chainK; ++k) {
      const float cxv = r.nextp.x * inv + total * r.dv.x, cyv = r.nextp.y * inv + total * r.dv.y,
                  czv = r.nextp.z * inv + total * r.dv.z;
      const int ix = (int)floorf(cxv), iy = (int)floorf(cyv), iz = (int)floorf(czv);
      const int bx = std::min(std::max(ix >> 3, 0), v.tx - 1), by = std::min(std::max(iy >> 3, 0), v.ty - 1);
      const int lbz = std::min(std::max(iz >> 3, 0), v.nbz - 1);
      const int sx = std::min(std::max(ix >> 5, 0), v.stx - 1), sy = std::min(std::max(iy >> 5, 0), v.sty - 1);
      const int lsz = std::min(std::max(iz >> 5, 0), v.nsz - 1);
      float lim = 0.f, zlim = 0.f;
      auto axes = [&](int B, int cbx, int cby, int nbx, int nby, float zl, float zh, float &lz) {
        const float xl = cbx > 0 ? (float)(B * cbx - B) : -kInf, xh = cbx < nbx - 1 ? (float)(B * cbx + 2 * B - 1) : kInf;
        const float yl = cby > 0 ? (float)(B * cby - B) : -kInf, yh = cby < nby - 1 ? (float)(B * cby + 2 * B - 1) : kInf;
        lz = axis_limit(czv, r.dv.z, r.idv.z, zl, zh);
        return fminf(fminf(axis_limit(cxv, r.dv.x, r.idv.x, xl, xh), axis_limit(cyv, r.dv.y, r.idv.y, yl, yh)), lz);
      };
      const bool sclear = !v.socc[v.si(sx, sy, lsz)];
      if (sclear) {
        float zl, zh;
        zrun([&](int z) { return v.socc[v.si(sx, sy, z)] != 0; }, lsz, v.nsz, 32, r.dv.z, zl, zh);
        lim = axes(32, sx, sy, v.stx, v.sty, zl, zh, zlim);
      } else if (!v.bocc[v.bi(bx, by, lbz)]) {
        float zl, zh;
        zrun([&](int z) { return v.bocc[v.bi(bx, by, z)] != 0; }, lbz, v.nbz, 8, r.dv.z, zl, zh);
        lim = axes(8, bx, by, v.tx, v.ty, zl, zh, zlim);
      }
      if (!(lim >= 1.f)) break;
      total += lim;
      if (total >= skip_cap || lim >= zlim) break;  // capped, or left through z: the next words are not predictable
    }
    return total;
  }

  // variant 8 (implementable: every word address known before any word is
  // back): point j+1 is the lateral (x / y) exit of the BRICK box of point j's
  // cell (no loaded data needed); the words of all chainK points are loaded in
  // one round trip; the box at point 0 as the kernel (super when clear, else
  // brick), brick boxes at the others; a point extends the run while it lies
  // inside the run cleared so far
  float lookup_chain2(const Ray &r) const {
    const float inv = 1.f / v.vs;
    float T = 0.f, t = 0.f;
    for (int k = 0; k < chainK; ++k) {
      const float cxv = r.nextp.x * inv + t * r.dv.x, cyv = r.nextp.y * inv + t * r.dv.y, czv = r.nextp.z * inv + t * r.dv.z;
      const int ix = (int)floorf(cxv), iy = (int)floorf(cyv), iz = (int)floorf(czv);
      const int bx = std::min(std::max(ix >> 3, 0), v.tx - 1), by = std::min(std::max(iy >> 3, 0), v.ty - 1);
      const int lbz = std::min(std::max(iz >> 3, 0), v.nbz - 1);
      const int sx = std::min(std::max(ix >> 5, 0), v.stx - 1), sy = std::min(std::max(iy >> 5, 0), v.sty - 1);
      const int lsz = std::min(std::max(iz >> 5, 0), v.nsz - 1);
      const float xl = bx > 0 ? (float)(8 * bx - 8) : -kInf, xh = bx < v.tx - 1 ? (float)(8 * bx + 15) : kInf;
      const float yl = by > 0 ? (float)(8 * by - 8) : -kInf, yh = by < v.ty - 1 ? (float)(8 * by + 15) : kInf;
      const float tlat = fminf(axis_limit(cxv, r.dv.x, r.idv.x, xl, xh), axis_limit(cyv, r.dv.y, r.idv.y, yl, yh));
      if (t <= T || k == 0) {
        float lim = 0.f;
        const bool sclear = k == 0 && !v.socc[v.si(sx, sy, lsz)];
        if (sclear) {
          float zl, zh;
          zrun([&](int z) { return v.socc[v.si(sx, sy, z)] != 0; }, lsz, v.nsz, 32, r.dv.z, zl, zh);
          lim = box_limit(32, sx, sy, v.stx, v.sty, zl, zh, cxv, cyv, czv, r.dv, r.idv);
        } else if (!v.bocc[v.bi(bx, by, lbz)]) {
          float zl, zh;
          zrun([&](int z) { return v.bocc[v.bi(bx, by, z)] != 0; }, lbz, v.nbz, 8, r.dv.z, zl, zh);
          lim = box_limit(8, bx, by, v.tx, v.ty, zl, zh, cxv, cyv, czv, r.dv, r.idv);
        }
        if (k == 0 && !(lim >= 1.f)) return 0.f;
        if (lim >= 1.f) T = fmaxf(T, t + lim);
      }
      if (!(tlat < kInf)) break;
      t += tlat;
      if (t > T || t >= skip_cap) break;
    }
    return fminf(T, skip_cap);
  }

  // one lookup + replay; returns false when the lane leaves the lookup loop
  bool lookup_step(Ray &r, uint32_t &nsk) const {
    float lim = variant == 2 ? fmaxf(lookup_kernel(r), lookup_dist(r)) : (variant == 7 ? lookup_chain(r) : (variant == 8 ? lookup_chain2(r) : lookup_kernel(r)));
    if (variant == 3) lim = fmaxf(lim, lookup_probe(r));
    if (r.trace) {
      const float inv = 1.f / v.vs;
      const int ix = (int)floorf(r.nextp.x * inv), iy = (int)floorf(r.nextp.y * inv), iz = (int)floorf(r.nextp.z * inv);
      printf("    lookup at k=%u vox (%d,%d,%d) brick occ %d super occ %d bdist %d sdist %d -> lim %.1f\n", r.kbase, ix, iy,
             iz, (int)v.bocc[v.bi(std::min(std::max(ix >> 3, 0), v.tx - 1), std::min(std::max(iy >> 3, 0), v.ty - 1),
                                  std::min(std::max(iz >> 3, 0), v.nbz - 1))],
             (int)v.socc[v.si(std::min(std::max(ix >> 5, 0), v.stx - 1), std::min(std::max(iy >> 5, 0), v.sty - 1),
                              std::min(std::max(iz >> 5, 0), v.nsz - 1))],
             (int)v.bdist[v.bi(std::min(std::max(ix >> 3, 0), v.tx - 1), std::min(std::max(iy >> 3, 0), v.ty - 1),
                               std::min(std::max(iz >> 3, 0), v.nbz - 1))],
             (int)v.sdist[v.si(std::min(std::max(ix >> 5, 0), v.stx - 1), std::min(std::max(iy >> 5, 0), v.sty - 1),
                               std::min(std::max(iz >> 5, 0), v.nsz - 1))],
             lim);
    }
    r.lookups++;
    if (!(lim >= 1.f)) return false;
    const int n = (int)fminf(lim, skip_cap);
    float px = r.nextp.x, py = r.nextp.y, pz = r.nextp.z, rl = r.ray_len;
    const float rstep = 1.f / v.vs;
    const int nf = std::min(n, std::max(0, (int)((r.tfar - rl) * rstep) - 2));
    int i = 0;
    for (; i < nf; ++i) {
      px = px + r.vstep.x;
      py = py + r.vstep.y;
      pz = pz + r.vstep.z;
      rl = rl + v.vs;
    }
    for (; i < n; ++i) {
      if (!(rl < r.tfar)) {
        r.live = false;
        break;
      }
      px = px + r.vstep.x;
      py = py + r.vstep.y;
      pz = pz + r.vstep.z;
      rl = rl + v.vs;
    }
    r.nextp = {px, py, pz};
    r.ray_len = rl;
    nsk += (uint32_t)n;
    return r.live;
  }
  void after_skip(Ray &r, uint32_t nsk) const {
    if (nsk != 0u && r.live) {
      r.kbase += nsk;
      r.tprev = voxel2tsdf(r.nextp);
      r.sprev = std::isnan(r.tprev) ? 0 : (r.tprev > 0.f ? 1 : (r.tprev < 0.f ? -1 : 0));
    }
  }
  // one batch of kR samples (events: +/- candidate or -/+ stop)
  void batch(Ray &r) const {
    r.batches++;
    if (r.trace) printf("    batch at k=%u\n", r.kbase);
    const f3 p0 = r.nextp;
    float rl = r.ray_len;
    float raw[32];
    unsigned pm = 0, nm = 0, am = 0;
    f3 np = r.nextp;
    for (int j = 0; j < kR; ++j) {
      const bool a = r.live && rl < r.tfar;
      am |= a ? (1u << j) : 0u;
      np = add(np, r.vstep);
      const float t = a ? voxel2tsdf(np) : NAN;
      raw[j] = t;
      const bool val = !std::isnan(t);
      pm |= (val && t > 0.f) ? (1u << j) : 0u;
      nm |= (val && t < 0.f) ? (1u << j) : 0u;
      rl = rl + v.vs;
    }
    const int je = __builtin_ctz(~am);
    const unsigned pprev = (pm << 1) | (r.sprev > 0 ? 1u : 0u);
    const unsigned nprev = (nm << 1) | (r.sprev < 0 ? 1u : 0u);
    const unsigned hitm = pprev & nm;
    unsigned ev = hitm | (nprev & pm);
    const float tfirst = r.tprev;
    r.sprev = ((pm >> (kR - 1)) & 1u) ? 1 : (((nm >> (kR - 1)) & 1u) ? -1 : 0);
    r.tprev = raw[kR - 1];
    if (ev) {
      const int j0 = __builtin_ctz(ev);
      if (!((hitm >> j0) & 1u)) {
        r.live = false;
      } else {
        float tc = tfirst, tn = 0.f, rj = r.ray_len;
        for (int j = 0; j < kR; ++j) {
          if (j + 1 == j0) tc = raw[j];
          if (j == j0) tn = raw[j];
          if (j < j0) rj += v.vs;
        }
        const float Ts = rj - (v.vs * tc) / (tc - tn);
        r.cvert = add(r.org, scl(r.dir, Ts));
        r.cand = true;
        f3 pj = p0;
        for (int j = 0; j <= j0; ++j) pj = add(pj, r.vstep);
        r.r_nextp = pj;
        r.r_rl = rj + v.vs;
        r.r_kbase = r.kbase + (uint32_t)j0 + 1u;
        r.r_tprev = tn;
        r.live = false;
        return;
      }
    }
    if (je < kR) r.live = false;
    r.nextp = np;
    r.ray_len = rl;
    r.kbase += kR;
  }
  void normal(Ray &r) const {
    r.normals++;
    r.cand = false;
    if (normal_ok(r.cvert)) {
      r.hit = true;
    } else {
      r.live = true;
      r.nextp = r.r_nextp;
      r.ray_len = r.r_rl;
      r.kbase = r.r_kbase;
      r.sprev = -1;
      r.tprev = r.r_tprev;
    }
  }
};

struct WaveCost {
  int lk_rounds = 0, bt_rounds = 0, nm_rounds = 0, mixed_rounds = 0;
  double t = 0;
  int tx0 = 0, ty0 = 0;
  std::string log;  // per round: L<lanes in lookup>/<lanes skipping on> or B<live lanes>
};

// the kernel's lockstep schedule (variant 0 / 2: lookup phase until every lane
// is blocked, then one batch for all live lanes)
static WaveCost run_wave_kernel(const Sim &S, std::vector<Ray> &L, double cL, double cB, double cN) {
  WaveCost w;
  auto any = [&](auto f) {
    for (auto &r : L)
      if (f(r)) return true;
    return false;
  };
  while (any([](const Ray &r) { return r.live || r.cand; })) {
    while (any([](const Ray &r) { return r.live; })) {
      std::vector<char> in(L.size());
      std::vector<uint32_t> nsk(L.size(), 0);
      for (size_t i = 0; i < L.size(); ++i) {
        in[i] = L[i].can_skip && L[i].live && L[i].sprev >= 0 && L[i].sup == 0;
        if (L[i].sup > 0 && L[i].live) L[i].sup--;
      }
      for (;;) {
        bool a = false;
        for (size_t i = 0; i < L.size(); ++i) a |= in[i] != 0;
        if (!a) break;
        w.lk_rounds++;
        int nin = 0, non = 0;
        for (size_t i = 0; i < L.size(); ++i)
          if (in[i]) {
            ++nin;
            if (!S.lookup_step(L[i], nsk[i])) {
              in[i] = 0;
              if (nsk[i] == 0) L[i].sup = S.suppress;  // blocked at once: no skip from here
            } else ++non;
          }
        w.log += "L" + std::to_string(nin) + "/" + std::to_string(non) + " ";
      }
      for (size_t i = 0; i < L.size(); ++i) S.after_skip(L[i], nsk[i]);
      if (!any([](const Ray &r) { return r.live; })) break;
      w.bt_rounds++;
      int nl = 0;
      for (auto &r : L)
        if (r.live) {
          ++nl;
          S.batch(r);
        }
      w.log += "B" + std::to_string(nl) + " ";
    }
    if (any([](const Ray &r) { return r.cand; })) {
      w.nm_rounds++;
      for (auto &r : L)
        if (r.cand) S.normal(r);
    }
  }
  w.t = w.lk_rounds * cL + w.bt_rounds * cB + w.nm_rounds * cN;
  return w;
}

// variant 1: per-lane interleaving — each round, lanes in skip mode do one
// lookup and lanes in march mode one batch (the wave pays both when mixed)
static WaveCost run_wave_interleaved(const Sim &S, std::vector<Ray> &L, double cL, double cB, double cN) {
  WaveCost w;
  std::vector<char> skipmode(L.size());
  std::vector<uint32_t> nsk(L.size(), 0);
  for (size_t i = 0; i < L.size(); ++i) skipmode[i] = L[i].can_skip && L[i].live && L[i].sprev >= 0;
  auto any = [&](auto f) {
    for (size_t i = 0; i < L.size(); ++i)
      if (f(i)) return true;
    return false;
  };
  while (any([&](size_t i) { return L[i].live || L[i].cand; })) {
    while (any([&](size_t i) { return L[i].live; })) {
      const bool lk = any([&](size_t i) { return L[i].live && skipmode[i]; });
      const bool bt = any([&](size_t i) { return L[i].live && !skipmode[i]; });
      if (lk && bt) w.mixed_rounds++;
      if (lk) w.lk_rounds++;
      if (bt) w.bt_rounds++;
      for (size_t i = 0; i < L.size(); ++i) {
        Ray &r = L[i];
        if (!r.live) continue;
        if (skipmode[i]) {
          if (!S.lookup_step(r, nsk[i])) {
            S.after_skip(r, nsk[i]);
            nsk[i] = 0;
            skipmode[i] = 0;
          }
        } else {
          S.batch(r);
          if (r.live) skipmode[i] = r.can_skip && r.sprev >= 0;
        }
      }
    }
    if (any([&](size_t i) { return L[i].cand; })) {
      w.nm_rounds++;
      for (size_t i = 0; i < L.size(); ++i)
        if (L[i].cand) {
          S.normal(L[i]);
          if (L[i].live) skipmode[i] = 0;  // sprev = -1 after a NaN candidate
        }
    }
  }
  w.t = w.lk_rounds * cL + w.bt_rounds * cB + w.nm_rounds * cN;
  return w;
}

// variant 5: a lookup and the batch from the same position in ONE round trip
// (the batch's loads issued with the map words; used only when the lookup is
// blocked): per round each lane either skips (clear) or marches a batch
static WaveCost run_wave_fused(const Sim &S, std::vector<Ray> &L, double cL, double cB, double cN) {
  WaveCost w;
  auto any = [&](auto f) {
    for (size_t i = 0; i < L.size(); ++i)
      if (f(i)) return true;
    return false;
  };
  std::vector<uint32_t> nsk(L.size(), 0);
  while (any([&](size_t i) { return L[i].live || L[i].cand; })) {
    while (any([&](size_t i) { return L[i].live; })) {
      bool anyb = false, anyl = false;
      for (size_t i = 0; i < L.size(); ++i) {
        Ray &r = L[i];
        if (!r.live) continue;
        if (r.can_skip && r.sprev >= 0) {
          anyl = true;
          nsk[i] = 0;
          if (S.lookup_step(r, nsk[i])) {  // skipped: the loaded batch is dropped
            S.after_skip(r, nsk[i]);
            continue;
          }
          S.after_skip(r, nsk[i]);
          if (!r.live) continue;
        }
        anyb = true;
        S.batch(r);
      }
      if (anyb) w.bt_rounds++;
      else if (anyl) w.lk_rounds++;
    }
    if (any([&](size_t i) { return L[i].cand; })) {
      w.nm_rounds++;
      for (size_t i = 0; i < L.size(); ++i)
        if (L[i].cand) S.normal(L[i]);
    }
  }
  w.t = w.lk_rounds * cL + w.bt_rounds * cB + w.nm_rounds * cN;
  return w;
}

// variant 6: two phases.  Phase 1 is the kernel's schedule capped at `cap`
// wave rounds (lookups + batches); the rays still marching then go to a queue
// (candidates pending at the cap take the wave's normal pass first).  Phase 2
// marches each queued ray with a group of G lanes: a scan round (lane j looks
// up the box at sample k + j*S; the contiguous clear prefix is replayed) and a
// dense round (G consecutive samples in one round trip), repeated.
struct Phase2 {
  int cap = 20, G = 64, S = 8;
};
static int phase2_ray(const Sim &S, Ray r, const Phase2 &P, int &scans, int &denses, int &norms) {
  int rounds = 0;
  const int saved_kR = S.kR;
  Sim &M = const_cast<Sim &>(S);
  while (r.live) {
    if (r.can_skip && r.sprev >= 0) {
      ++rounds;
      ++scans;
      // lane j: box at the position of sample (carried) + j*S
      int E = 0;
      Ray q = r;
      for (int j = 0; j < P.G && q.live; ++j) {
        const int sj = j * P.S;
        if (sj > E) break;
        // advance q to sample sj (sequential adds: the exact positions)
        while ((int)(q.kbase - r.kbase) < sj && q.live) {
          if (!(q.ray_len < q.tfar)) q.live = false;
          q.nextp = add(q.nextp, q.vstep);
          q.ray_len = q.ray_len + S.v.vs;
          q.kbase++;
        }
        if (!q.live) break;
        const float lim = S.lookup_kernel(q);
        if (lim >= 1.f) E = std::max(E, sj + (int)fminf(lim, S.skip_cap));
      }
      if (E > 0) {
        uint32_t nsk = 0;
        // replay E samples from r
        for (int i = 0; i < E && r.live; ++i) {
          if (!(r.ray_len < r.tfar)) {
            r.live = false;
            break;
          }
          r.nextp = add(r.nextp, r.vstep);
          r.ray_len = r.ray_len + S.v.vs;
          ++nsk;
        }
        S.after_skip(r, nsk);
        if (!r.live) break;
      }
    }
    ++rounds;
    ++denses;
    for (int h = 0; h < (P.G + 31) / 32 && r.live; ++h) {
      M.kR = std::min(32, P.G - 32 * h);
      S.batch(r);
    }
    M.kR = saved_kR;
    if (r.cand) {
      ++rounds;
      ++norms;
      S.normal(r);
    }
  }
  return rounds;
}
static WaveCost run_wave_two_phase(const Sim &S, std::vector<Ray> &L, double cL, double cB, double cN,
                                   const Phase2 &P, std::vector<int> &queued_rounds) {
  WaveCost w;
  auto any = [&](auto f) {
    for (auto &r : L)
      if (f(r)) return true;
    return false;
  };
  int rounds = 0;
  bool capped = false;
  while (!capped && any([](const Ray &r) { return r.live || r.cand; })) {
    while (any([](const Ray &r) { return r.live; })) {
      if (rounds >= P.cap) {
        capped = true;
        break;
      }
      std::vector<char> in(L.size());
      std::vector<uint32_t> nsk(L.size(), 0);
      for (size_t i = 0; i < L.size(); ++i) in[i] = L[i].can_skip && L[i].live && L[i].sprev >= 0;
      for (;;) {
        bool a = false;
        for (size_t i = 0; i < L.size(); ++i) a |= in[i] != 0;
        if (!a) break;
        w.lk_rounds++;
        ++rounds;
        for (size_t i = 0; i < L.size(); ++i)
          if (in[i] && !S.lookup_step(L[i], nsk[i])) in[i] = 0;
        if (rounds >= P.cap) {  // lanes still in the lookup loop stop where they are
          for (size_t i = 0; i < L.size(); ++i) in[i] = 0;
        }
      }
      for (size_t i = 0; i < L.size(); ++i) S.after_skip(L[i], nsk[i]);
      if (!any([](const Ray &r) { return r.live; })) break;
      if (rounds >= P.cap) {
        capped = true;
        break;
      }
      w.bt_rounds++;
      ++rounds;
      for (auto &r : L)
        if (r.live) S.batch(r);
    }
    if (any([](const Ray &r) { return r.cand; })) {
      w.nm_rounds++;
      for (auto &r : L)
        if (r.cand) S.normal(r);
    }
  }
  for (auto &r : L)
    if (r.live) {
      int sc = 0, dn = 0, nm = 0;
      queued_rounds.push_back(phase2_ray(S, r, P, sc, dn, nm));
    }
  w.t = w.lk_rounds * cL + w.bt_rounds * cB + w.nm_rounds * cN;
  return w;
}

int main(int argc, char **argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp/raysim";
  Sim S;
  S.variant = argc > 2 ? atoi(argv[2]) : 0;
  const int cap = argc > 3 ? atoi(argv[3]) : 16;
  if (argc > 4) S.probesK = atoi(argv[4]);
  if (argc > 5) S.probeS = atoi(argv[5]);
  if (getenv("RAYSIM_SUP")) S.suppress = atoi(getenv("RAYSIM_SUP"));
  if (getenv("RAYSIM_K")) S.chainK = atoi(getenv("RAYSIM_K"));
  int dims[3];
  FILE *f = fopen((dir + "/dims.bin").c_str(), "rb");
  if (!f || fread(dims, 4, 3, f) != 3) return 1;
  fclose(f);
  const int n = dims[0];
  S.W = dims[1];
  S.H = dims[2];
  float c2v[12];
  f = fopen((dir + "/c2v.bin").c_str(), "rb");
  if (!f || fread(c2v, 4, 12, f) != 12) return 1;
  fclose(f);
  std::memcpy(S.R, c2v, 36);
  std::memcpy(S.T, c2v + 9, 12);
  Vol &v = S.v;
  v.X = v.Y = v.Z = n;
  v.range = 2.048f;
  v.vs = v.range / (float)n;
  v.t.resize((size_t)n * n * n);
  f = fopen((dir + "/tsdf.bin").c_str(), "rb");
  if (!f || fread(v.t.data(), 2, v.t.size(), f) != v.t.size()) return 1;
  fclose(f);
  v.tx = v.ty = n / 8;
  v.nbz = n / 8;
  v.stx = v.sty = (v.tx + 3) / 4;
  v.nsz = (v.nbz + 3) / 4;
  v.bneg.assign((size_t)v.tx * v.ty * v.nbz, 0);
  v.sneg.assign((size_t)v.stx * v.sty * v.nsz, 0);
  for (int z = 0; z < n; ++z)
    for (int y = 0; y < n; ++y)
      for (int x = 0; x < n; ++x)
        if (v.at(x, y, z) < 0) {
          v.bneg[v.bi(x >> 3, y >> 3, z >> 3)] = 1;
          v.sneg[v.si(x >> 5, y >> 5, z >> 5)] = 1;
        }
  dilate(v.bneg, v.bocc, v.tx, v.ty, v.nbz);
  dilate(v.sneg, v.socc, v.stx, v.sty, v.nsz);
  chess(v.bneg, v.bdist, v.tx, v.ty, v.nbz, cap);
  chess(v.sneg, v.sdist, v.stx, v.sty, v.nsz, cap);
  S.skip_cap = std::min(511.f, std::floor(0.1f * 8388608.f / (float)n));
  // per-round costs measured on MI355X (tools/ray_trace.py, C2): lookup ~1.6 us,
  // batch ~1.9 us, normal pass ~5 us
  const double cL = 1.6, cB = 1.9, cN = 5.0;
  std::vector<WaveCost> waves;
  long long tot_lk = 0, tot_bt = 0;
  Phase2 P2;
  if (getenv("RAYSIM_CAP")) P2.cap = atoi(getenv("RAYSIM_CAP"));
  if (getenv("RAYSIM_G")) P2.G = atoi(getenv("RAYSIM_G"));
  if (getenv("RAYSIM_S")) P2.S = atoi(getenv("RAYSIM_S"));
  std::vector<int> queued;  // variant 6: phase-2 rounds of each queued ray
  for (int ty0 = 0; ty0 < S.H; ty0 += 8)
    for (int tx0 = 0; tx0 < S.W; tx0 += 8) {
      std::vector<Ray> L(64);
      for (int l = 0; l < 64; ++l) {
        const int x = tx0 + (l & 7), y = ty0 + (l >> 3);
        if (x < S.W && y < S.H) S.setup(L[l], x, y);
        if (getenv("RAYSIM_PIX")) {
          int px, py;
          if (sscanf(getenv("RAYSIM_PIX"), "%d,%d", &px, &py) == 2 && px == x && py == y) {
            L[l].trace = true;
            printf("  pixel (%d,%d): dir (%.3f %.3f %.3f) dv (%.3f %.3f %.3f)\n", x, y, L[l].dir.x, L[l].dir.y, L[l].dir.z,
                   L[l].dv.x, L[l].dv.y, L[l].dv.z);
          }
        }
      }
      WaveCost w = S.variant == 1   ? run_wave_interleaved(S, L, cL, cB, cN)
                   : S.variant == 5 ? run_wave_fused(S, L, cL, cB, cN)
                   : S.variant == 6 ? run_wave_two_phase(S, L, cL, cB, cN, P2, queued)
                                    : run_wave_kernel(S, L, cL, cB, cN);
      w.tx0 = tx0;
      w.ty0 = ty0;
      if (getenv("RAYSIM_TILE")) {  // per-lane counts of one wave (x0,y0), then the busiest lane traced
        int qx, qy;
        if (sscanf(getenv("RAYSIM_TILE"), "%d,%d", &qx, &qy) == 2 && qx == tx0 && qy == ty0) {
          int best = 0;
          for (int l = 0; l < 64; ++l) {
            printf("  lane %2d px (%d,%d): lookups %d batches %d normals %d hit %d dir (%.3f %.3f %.3f)\n", l,
                   tx0 + (l & 7), ty0 + (l >> 3), L[l].lookups, L[l].batches, L[l].normals, (int)L[l].hit, L[l].dir.x,
                   L[l].dir.y, L[l].dir.z);
            if (L[l].lookups + L[l].batches > L[best].lookups + L[best].batches) best = l;
          }
          printf("  busiest lane %d: RAYSIM_PIX=%d,%d\n", best, tx0 + (best & 7), ty0 + (best >> 3));
        }
      }
      for (auto &r : L) {
        tot_lk += r.lookups;
        tot_bt += r.batches;
      }
      waves.push_back(w);
    }
  std::vector<double> t;
  std::vector<int> lk, bt;
  for (auto &w : waves) {
    t.push_back(w.t);
    lk.push_back(w.lk_rounds);
    bt.push_back(w.bt_rounds);
  }
  auto pct = [](std::vector<double> a, double q) {
    std::sort(a.begin(), a.end());
    return a[(size_t)std::min<double>(a.size() - 1, q * a.size())];
  };
  std::vector<double> lkd(lk.begin(), lk.end()), btd(bt.begin(), bt.end());
  printf("variant %d: waves %zu  lane lookups %lld  lane batches %lld\n", S.variant, waves.size(), tot_lk, tot_bt);
  printf("  lookup rounds/wave med %.0f p90 %.0f p99 %.0f max %.0f\n", pct(lkd, .5), pct(lkd, .9), pct(lkd, .99),
         pct(lkd, 1.0));
  printf("  batch rounds/wave  med %.0f p90 %.0f p99 %.0f max %.0f\n", pct(btd, .5), pct(btd, .9), pct(btd, .99),
         pct(btd, 1.0));
  printf("  modeled wave us (excl. setup) med %.1f p90 %.1f p99 %.1f max %.1f\n", pct(t, .5), pct(t, .9), pct(t, .99),
         pct(t, 1.0));
  if (S.variant == 6) {
    std::vector<double> q(queued.begin(), queued.end());
    if (q.empty()) q.push_back(0);
    double sum = 0;
    for (double x : q) sum += x;
    printf("  phase 2 (cap %d, G %d, S %d): queued rays %zu; rounds/ray mean %.2f med %.0f p90 %.0f p99 %.0f max %.0f; "
           "wave-rounds %.0f\n",
           P2.cap, P2.G, P2.S, queued.size(), sum / q.size(), pct(q, .5), pct(q, .9), pct(q, .99), pct(q, 1.0),
           sum * P2.G / 64.0);
  }
  if (getenv("RAYSIM_SLOW")) {
    std::vector<size_t> idx(waves.size());
    for (size_t i = 0; i < idx.size(); ++i) idx[i] = i;
    std::sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return waves[a].t > waves[b].t; });
    for (int k = 0; k < atoi(getenv("RAYSIM_SLOW")); ++k) {
      const WaveCost &w = waves[idx[k]];
      printf("  slow wave tile (%d,%d): %.1f us, %d lookup / %d batch / %d normal rounds\n    %s\n", w.tx0, w.ty0, w.t,
             w.lk_rounds, w.bt_rounds, w.nm_rounds, w.log.c_str());
    }
  }
  return 0;
}
