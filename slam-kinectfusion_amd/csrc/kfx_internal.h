// kfx_internal.h — types shared by the HIP kernels (kfx_kernels.hip) and the
// host runtime (kfx_api.hip).  Not part of the public ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <math.h>

namespace kfx {

constexpr int kMaxLevels = 4;

enum FrameMode : int { MODE_BOOT = 0, MODE_TRACK = 1, MODE_FAIL = 2 };

struct DevPose {
  float R[9];  // row-major
  float t[3];
};

// Per-frame tracking state, resident in device memory so the whole frame runs
// without a host round trip.
struct DevState {
  int frame_count;      // kinectfusion::frame_count (kinectfusion.h:58)
  int mode;             // FrameMode of the frame in flight
  int icp_fail;         // set by the ICP solve on det failure (icp_registration.cpp:35-37)
  int n_poses;          // pose_record.size()
  int pose_cap;         // capacity of the pose log
  int pose_overflow;
  int n_base;           // n_poses at frame start (read-only during the frame)
  int last_fail;        // 1 if the last frame hit the ICP det check (reset applied)
  DevPose icp_pose;     // camera_pose inside rigidTransform
  long long sums[27];   // last ICP sums (test seam)
  double x[6];          // last ICP increment
  int icp_stalled;      // persistent ICP barrier watchdog fired (reported as KFX_ERR_HIP)
  int fails;            // frames dropped by a tracking failure (reset) so far
  int debug_stall;      // test hook: block 0 withholds its first ICP arrival (kfx_debug_force_icp_stall)
  DevPose *log;         // the device pose log (the host keeps it current)
  DevPose back;         // log[n_poses - 1] at frame begin: the frame pose's base, one load away
  // the frame's raycast pose, written by k_integrate (block 0) before the raycast
  // runs: kind (frame_kind) and cam2vol = volume_pose^-1 * pose (tsdf_volume.cpp:59).
  // Valid right after a pipeline integrate; a raycast with no explicit pose
  // outside a frame refreshes them first (k_ray_pose, kfx_raycast_stats).
  int ray_kind;
  DevPose ray_c2v;
  // frames begun so far (frame_begin), and integrate's vol2cam of a tracked
  // frame (tsdf_volume.cpp:50) written by the persistent ICP's block 0 with
  // int_tag = that frame's serial: integrate's blocks read it instead of
  // composing the pose each (any other path leaves the tag stale)
  unsigned frame_serial, int_tag;
  DevPose int_v2c;
};

struct LevelGeom {
  int w, h;
  float fx, fy, cx, cy;
};

#ifndef KFX_ICP_SHARDS
// ICP: partial-sum rows (atomic spread vs rows every solver reads).  With the
// flat arrival counter 4 measured best (C2 ICP -3 us vs 8); with the per-XCD
// arrival counters (KFX_ICP_HIER) 8: tools/icp_barrier_bench.hip, 300 blocks
// 4.35 us per hand-off at 4 shards, 3.33 at 8, 3.19 at 16
#define KFX_ICP_SHARDS 8
#endif
#ifndef KFX_ICP_HIER
#define KFX_ICP_HIER 1  // ICP arrival: per-residue (b % 8, one XCD each) counters, then a top counter of 8
#endif
constexpr int kIcpShards = KFX_ICP_SHARDS;
constexpr int kIcpMaxSlots = 64;  // ICP iterations per frame in the persistent kernel

// Per-frame plan of the persistent ICP kernel (all levels, all iterations).
struct IcpPlan {
  int levels, nblocks, slots;
  LevelGeom g[kMaxLevels];
  int xe[kMaxLevels], npix[kMaxLevels], groups[kMaxLevels], iters[kMaxLevels];
  int ppl[kMaxLevels];  // pixels per lane at each level
  const float *cv[kMaxLevels], *cn[kMaxLevels], *pv[kMaxLevels], *pn[kMaxLevels];
  float dist2_max, sine2_max;  // sqrt_le_bound of the distance / sine thresholds
  // 1: nblocks (co-resident) is below some level's groups (k_icp_track<true>):
  // at such a level block b takes the contiguous pixels [b span, (b+1) span)
  // in passes of up to kIcpPix per lane (span[l] > 0, a multiple of the block
  // size; groups[l] is then the number of non-empty ranges)
  int stride;
  int span[kMaxLevels];
  DevPose vpose;  // the volume pose (DevState::int_v2c)
};
constexpr int kIcpStrideMax = 16;

// Device workspace of the persistent ICP kernel; zero between launches
// (the kernel's last block restores that).
struct IcpSync {
  unsigned arrive, pad0[31];   // arrivals, all iterations (own 128-B line)
  unsigned exit, pad1[31];
  struct {
    unsigned v, pad[31];
  } sub[8];                    // KFX_ICP_HIER: arrivals of the blocks b % 8 == r, all iterations
  unsigned top, pad2[31];      // KFX_ICP_HIER: residues complete, all iterations
  struct {
    unsigned v, pad[31];
  } release[8];                // iterations released so far; 8 copies polled by block % 8
  unsigned long long sums[kIcpMaxSlots * kIcpShards * 27];
  // s_memrealtime stamps of the last frame, per iteration: block 0 start /
  // arrived / released / solved, last block arrived (kfx_get_icp_trace)
  unsigned long long trace[kIcpMaxSlots][12];
#ifdef KFX_ICP_BLOCK_TRACE
  unsigned long long blk[kIcpMaxSlots][512][2];  // debug: per-block lane-phase start / arrival
#endif
};

// SoA TSDF volume.  Each z slice is tiled in 8x8 (x,y) tiles; voxel (x,y,z)
// lives at (z-zb)*slice + ((y>>3)*tiles_x + (x>>3))*64 + (y&7)*8 + (x&7).
//
// Z-slab sharding: a context stores only the global slices
// [zb, zb+zn) — its owned slices [own0, own1) plus a halo of kSlabHalo slices
// on each side, which it integrates redundantly (bit-identical to the owner's
// copy) so that raycast never needs a halo exchange.  A single-GPU volume is
// the slab zb = own0 = 0, zn = own1 = Z.  X, Y, Z are always the global dims.
constexpr int kSlabHalo = 4;
struct VolView {
  int16_t *tsdf;
  uint8_t *weight;  // D: u8 storage of the reference's int16 weight (values 0..MAX_WEIGHT; 0..255 accepted on upload)
  uint32_t *rgb;  // u8 c0,c1,c2,pad
  int X, Y, Z;
  int zb, zn;      // stored global slices [zb, zb+zn)
  int own0, own1;  // owned global slices (raycast events, point extraction)
  int tiles_x, tiles_y;
  float vs[3];     // voxel size per axis
  float range[3];  // volume_range
  float trunc;
  float inv_trunc;  // RN(1/trunc), for the exact FMA division (kfx_kernels.hip div_rn)
  size_t slice;    // voxels per z slice (= X*Y)
  // Dilated occupancy of negative tsdf (raycast empty-space skipping, DESIGN.md
  // §4): bit set <=> some voxel within one brick of this brick may hold a
  // negative tsdf (a superset: integrate only ever sets bits; reset clears).
  // Bricks are 8x8x8 voxels = one 8x8 column tile x 8 global slices (brick z
  // = z >> 3); super-bricks are 4x4x4 bricks (32^3 voxels).  Words per column:
  //   bocc[tile * bw + (lbz >> 6)] bit (lbz & 63), lbz = (z >> 3) - bz0 in [0, nbz)
  //   socc[(sy * stx + sx) * sw + (lsz >> 5)] bit (lsz & 31), lsz = (z >> 5) - sz0
  unsigned long long *bocc;
  uint32_t *socc;
  int bz0, nbz, bw;
  int sz0, nsz, sw, stx, sty;
  // Integrate dispatch order (KFX_INT_LPT): iwork[tile] = the length of the
  // tile's wave-uniform z interval in the last integrate, iperm[b] = the
  // (chunk * tiles + tile) item block b runs (longest estimated first; any
  // permutation gives the same volume), inchunk = chunks per tile.
  unsigned *iwork;
  unsigned *iperm;
  int inchunk;
  int iadapt;  // length-capped chunks + longest-first order (deep volumes), else geometric chunks
  int force64;  // kfx_debug_force_index64: integrate / raycast take the 64-bit-index kernels at any size
  unsigned *rdur;  // raycast: each wave's duration in the last frame (1024-cycle units; issue priority hint)
  __host__ __device__ size_t bocc_bytes() const { return (size_t)tiles_x * tiles_y * bw * 8; }
  __host__ __device__ size_t socc_bytes() const { return (size_t)stx * sty * sw * 4; }
  __host__ __device__ size_t local_voxels() const { return slice * (size_t)zn; }
  // Tile-column layout: the stored slices of one 8x8 column tile are one
  // contiguous run of zn * 64 voxels, z-major inside:
  //   index(x, y, z) = (tile(x, y) * zn + (z - zb)) * 64 + (y & 7) * 8 + (x & 7)
  __host__ __device__ size_t tile_voxels() const { return (size_t)zn * 64; }
};

// ---- slab raycast combine, shared by the kernels and the host entry points
// (kfx_slab_mask_payload / kfx_slab_expand) so a CPU test drives the same code.
// A slab ships per pixel only {Ts, nout} of its winning hit (the payload,
// 4 u32 planes); every rank rebuilds the vertex from Ts and the ray with the
// raycast's own float ops.
// raycasthelper (tsdf_volume.cu:217-220): dir = normalize(R * reproj(x, y, 1))
__host__ __device__ inline void ray_dir(const float *R, const LevelGeom &g, int x, int y, float d[3]) {
  const float p0 = (1.f * ((float)x - g.cx)) / g.fx, p1 = (1.f * ((float)y - g.cy)) / g.fy, p2 = 1.f;
  const float v0 = R[0] * p0 + R[1] * p1 + R[2] * p2;
  const float v1 = R[3] * p0 + R[4] * p1 + R[5] * p2;
  const float v2 = R[6] * p0 + R[7] * p1 + R[8] * p2;
  const float t = sqrtf(v0 * v0 + v1 * v1 + v2 * v2);
  d[0] = v0 / t;
  d[1] = v1 / t;
  d[2] = v2 / t;
}
// tsdf_volume.cu:247-255: vertex = org + dir * Ts, vmap = Rinv * (vertex - org)
__host__ __device__ inline void hit_vertex(const float org[3], const float dir[3], float Ts, const float *Rinv,
                                           float out[3]) {
  const float w0 = (org[0] + dir[0] * Ts) - org[0];
  const float w1 = (org[1] + dir[1] * Ts) - org[1];
  const float w2 = (org[2] + dir[2] * Ts) - org[2];
  out[0] = Rinv[0] * w0 + Rinv[1] * w1 + Rinv[2] * w2;
  out[1] = Rinv[3] * w0 + Rinv[4] * w1 + Rinv[5] * w2;
  out[2] = Rinv[6] * w0 + Rinv[7] * w1 + Rinv[8] * w2;
}
// The losers' payload is cleared after the MIN of the keys, so the MAX of the
// u32 bits leaves the winner's (0 is the smallest u32; a hit's normal is
// nonzero, so a zero normal means no surface).
__host__ __device__ inline void slab_mask_px(const uint32_t *key_local, const uint32_t *key_min, uint32_t *pay,
                                             size_t n, size_t i) {
  if (key_local[i] != key_min[i])
    for (int q = 0; q < 4; ++q) pay[q * n + i] = 0u;
}
__host__ __device__ inline void slab_expand_px(const uint32_t *pay, size_t n, size_t i, const float org[3],
                                               const float dir[3], const float *Rinv, float v[3], float nm[3]) {
  for (int q = 0; q < 3; ++q) {
    union { uint32_t u; float f; } b;
    b.u = pay[(1 + q) * n + i];
    nm[q] = b.f;
  }
  v[0] = v[1] = v[2] = 0.f;
  if ((pay[n + i] | pay[2 * n + i] | pay[3 * n + i]) == 0u) return;
  union { uint32_t u; float f; } ts;
  ts.u = pay[i];
  hit_vertex(org, dir, ts.f, Rinv, v);
}

struct FrameView {
  float *d[kMaxLevels];
  float *v[kMaxLevels];
  float *n[kMaxLevels];
};

// ---- launchers (kfx_kernels.hip) -----------------------------------------
// dl0: zero the frame's max-depth shards stored after that level-0 table
void launch_frame_begin(hipStream_t s, DevState *st, float2 *dl0, LevelGeom g0);
void launch_pyr_down(hipStream_t s, const float *src, const uint16_t *src16, int w, int h,
                     float *dst, DevState *st_begin, float2 *dl0);
// bilateral + truncation + vertex + normal maps, all levels (raw[l] = raw mm)
void launch_preprocess_maps(hipStream_t s, int levels, const float *const raw[kMaxLevels],
                            const uint16_t *raw0_u16, const LevelGeom *g, FrameView cur, int ksz,
                            float sigma_color, float sigma_spatial, float max_dist,
                            const float *inv_lambda, float2 *dl0);
int icp_blocks(const LevelGeom &g);
// one ICP iteration (rigid_icp.cu:135-169 + icp_registration.cpp:33-42) in a
// single launch; shards = 8 x 27 int64 zeroed, ticket zeroed (both self-reset)
IcpPlan make_icp_plan(int levels, const LevelGeom *g, const int *iters, FrameView cur,
                      FrameView prev, float dist_thr, float angle_thr);
bool icp_persistent_ok(IcpPlan &pl, int device);  // grid co-resident + slots fit
// the persistent ICP grid stays co-resident with `cus_free` CUs' worth of
// blocks taken by other kernels (icp_persistent_ok's plan)
bool icp_headroom(const IcpPlan &pl, int device, int cus_free);
// begin: run the frame's frame_begin inside the launch (no separate kernel)
// coop: cooperative launch (the runtime guarantees the grid co-resident)
// Returns the launch error (a refused cooperative launch: the caller falls
// back to per-iteration launches).
hipError_t launch_icp_track(hipStream_t s, const IcpPlan &pl, DevState *st, IcpSync *sync, int begin = 0,
                            bool coop = false);
// band / nbands: only rows [ye*band/nbands, ye*(band+1)/nbands) of the
// floor-covered region (a slab rank's share in the sharded ICP mode)
void launch_icp(hipStream_t s, const LevelGeom &g, const float *cv, const float *cn,
                const float *pv, const float *pn, float dist_thr, float angle_thr, DevState *st,
                unsigned long long *shards, unsigned *ticket, int force, int update, int band = 0,
                int nbands = 1);
// one ICP solve (+ pose update) from DevState::sums
void launch_icp_solve(hipStream_t s, DevState *st);
// DevState::sums of each of the n members <- their sum
void launch_group_sum_icp(hipStream_t s, DevState *const *st, int n);
// The frame's global pose, the integrate/raycast poses and the
// kinectfusion.cpp:84-104 bookkeeping are derived inside these kernels from
// DevState + pose log (no separate commit launch).  `xpose` (device, 12 or 21
// floats: pose [, Rinv]) overrides them for the stage seams; bookkeeping is
// then skipped.
// dl0: level-0 {depth m, 1/lambda} (written by launch_preprocess_maps); dmap:
// the same filtered depth alone (the frame's level-0 map); invl: 1/lambda
void launch_integrate(hipStream_t s, VolView v, LevelGeom g0, const float2 *dl0, const float *dmap,
                      const float *invl, const uint8_t *bgr, DevState *st, DevPose *log, DevPose vpose,
                      const float *xpose,
                      unsigned long long *counters /* non-null: count-only, 32 words */,
                      bool order = true /* false: the caller launches launch_int_order itself */);
// the next frame's integrate dispatch order from this frame's intervals
// (k_int_order; deep volumes only, a no-op otherwise).  It rewrites the order
// the integrate just read: enqueue it after that integrate has completed.
void launch_int_order(hipStream_t s, VolView v);
// Z-slab raycast passes: pass 0 marches every ray to its end;
// pass 1 stops at the previous frame's model distance along the ray (+
// bound_abs metres + bound_rel of the distance) and records the first sample
// it did not examine (pend plane); pass 2 re-marches, unbounded, the pixels
// whose pend lies below kmin (the MIN-reduced [keys | pend] of pass 1)
struct SlabPass {
  int pass = 0;
  const uint32_t *kmin = nullptr;
  float bound_abs = 0.f, bound_rel = 0.f;
};
// raycast of level 0 + resizePointsNormals of levels >= 1 in one launch; with
// keys != null the slab variant (owned events only, key per pixel, no resize;
// planes [key | pend | Ts | nx | ny | nz])
// stats (non-null): the statistics variant (6 counters added, nothing stored)
void launch_raycast(hipStream_t s, VolView v, int levels, const LevelGeom *g, FrameView cur,
                    FrameView prev, const DevState *st, const DevPose *log, DevPose vpose,
                    const float *xpose, uint32_t *keys, unsigned long long *stats = nullptr,
                    const SlabPass &sp = SlabPass{}, unsigned *start_sig = nullptr, unsigned start_val = 0);
// the reference raycast's distinct voxels read (out[0]) and reads (out[1]),
// count-only (bits: one bit per stored voxel, workspace)
void launch_ray_pose(hipStream_t s, DevState *st, const DevPose *log, DevPose vpose);
void launch_raycast_touch(hipStream_t s, VolView v, LevelGeom g0, const DevState *st, const DevPose *log,
                          DevPose vpose, const float *xpose, uint32_t *bits, unsigned long long *out);
// resizePointsNormals of levels >= 1 from the level-0 model maps
void launch_resize(hipStream_t s, int levels, const LevelGeom *g, FrameView cur, FrameView prev,
                   const DevState *st, const float *xpose);
// cross-slab combine: clear maps where the local key lost the MIN
// out[0] += sum of per-voxel hashes, out[1] += voxels with weight > 0 (owned slices)
void launch_checksum(hipStream_t s, VolView v, unsigned long long *out);
// renderPhong (type 0) / renderNormals (type 1) of the level-0 maps into w*h uchar3
void launch_render(hipStream_t s, const float *vmap, const float *nmap, int n, const DevState *st,
                   const DevPose *log, int type, uint8_t *out);
// keys = [key | Ts | nx | ny | nz] planes of the slab raycast (launch_raycast's keys)
void launch_slab_mask(hipStream_t s, const uint32_t *keys, const uint32_t *key_min, int n);
// level-0 model maps from the combined payload (and the frame kind)
void launch_slab_expand(hipStream_t s, LevelGeom g0, const uint32_t *pay, FrameView cur, FrameView prev,
                        const DevState *st, const DevPose *log, DevPose vpose);
constexpr int kMaxGroup = 16;
// element-wise MIN/MAX of n_in u32 buffers (any device-accessible pointers),
// result stored to each of the n_out buffers
void launch_group_reduce(hipStream_t s, uint32_t *const *in, int n_in, uint32_t *const *out,
                         int n_out, size_t count, bool is_max);
void launch_inv_lambda(hipStream_t s, LevelGeom g0, float *inv_lambda);
// device reads of mapped page-locked host memory into device buffers (two segments)
void launch_host_fetch(hipStream_t s, const void *src0, void *dst0, size_t n0, const void *src1, void *dst1,
                       size_t n1);
// point extraction (FullScan6) over global slices [zlo, zhi): offsets == null
// counts points per wave, else writes them (float3) at offsets (< cap)
size_t extract_waves(const VolView &v, int zlo, int zhi);
void launch_extract(hipStream_t s, const VolView &v, DevPose vpose, int zlo, int zhi,
                    unsigned *counts, const unsigned long long *offsets, float *out,
                    unsigned long long cap);
// marching cubes over z in [zlo, zhi) (same waves / chunks as launch_extract);
// tab: 256 x 16 bytes {n_tri, 3*n_tri edge indices}
void launch_mesh(hipStream_t s, const VolView &v, DevPose vpose, int zlo, int zhi, const uint8_t *tab,
                 unsigned *counts, const unsigned long long *offsets, float *out, unsigned long long cap);
size_t scan_blocks(size_t n);  // bsum entries launch_scan needs (<= 65536)
// one-read extraction (k_extract_pool + scan + k_extract_copy): tab = null
// for points, the marching-cubes table for triangles
void launch_extract_pool(hipStream_t s, const VolView &v, DevPose vpose, int zlo, int zhi, const uint8_t *tab,
                         unsigned *counts, unsigned long long *ctr, unsigned long long *pool_at, unsigned *list,
                         float *pool, unsigned long long pool_cap, unsigned *overflow);
void launch_extract_copy(hipStream_t s, const unsigned *list, unsigned nlist, const unsigned *counts,
                         const unsigned long long *pool_at, const unsigned long long *offsets, const float *pool,
                         float *out, unsigned long long cap, int per);
void launch_scan(hipStream_t s, const unsigned *counts, unsigned long long *offsets,
                 unsigned long long *bsum, size_t n, unsigned long long *total);
void launch_export_records(hipStream_t s, VolView v, int z0, int nz, uint64_t *dst);
void launch_import_records(hipStream_t s, VolView v, int z0, int nz, const uint64_t *src, unsigned *bad);
void launch_export_soa(hipStream_t s, VolView v, int z0, int nz, int16_t *t, int16_t *w,
                       uint32_t *c);
// clear the occupancy maps and re-mark every brick holding a negative tsdf
// (after a volume upload)
void launch_occ_rebuild(hipStream_t s, VolView v);
// z-chunks per column tile of k_integrate (the iperm item count is tiles x this)
int integrate_chunks(const VolView &v);
// per global slice: voxels passing integrate's depth test at vol2cam (an estimate, slab balancing)
void launch_slice_work(hipStream_t s, const VolView &v, DevPose vol2cam, LevelGeom g0, const float2 *dl0,
                       unsigned long long *hist);
// owned-slice records of n (x, y) columns (device cols), column-major outputs
void launch_gather_columns(hipStream_t s, VolView v, const int32_t *cols, int n, int16_t *t, int16_t *w,
                           uint32_t *c);

}  // namespace kfx
