/*
 * kfx.h — C-ABI drop-in boundary of the MI355X-native KinectFusion hot path.
 *
 * The reference exposes the hot path only as the C++ class `kf::kinectfusion`
 * (kfusion/include/kinectfusion.h:31-73) whose methods take OpenCV types.  There
 * is no FFI in the reference; this header is the plain-C seam a binding (ctypes,
 * cgo, JNI, or the header-only C++ adapter in
 * slam-kinectfusion_amd/adapter/kinectfusion.h) calls.  Every entry point below
 * names the reference interface it replaces.
 *
 * Conventions
 *   - All host buffers belong to the caller and are copied; the context owns all
 *     device memory.  No torch / HIP types cross this boundary.
 *   - Images are row-major, tightly packed (no pitch): depth f32 or u16 in
 *     millimetres (depth_sensor.cpp:191 converts PNG u16 mm -> f32 mm), colour
 *     BGR8 interleaved (cv::Mat CV_8UC3), vertex/normal maps float3 AoS.
 *   - Poses are kfx_pose {R row-major 3x3, t}; a cv::Affine3f maps 1:1.
 *   - Every function returns an int status (KFX_OK = 0).  The reference prints
 *     CUDA errors and continues (safe_call.hpp:8-14); here they are returned.
 */
#ifndef KFX_H
#define KFX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KFX_ABI_VERSION 2 /* 2: kfx_synchronize/kfx_pipeline report earlier frames; u8 weight uploads */
#define KFX_MAX_LEVELS 4

/* status codes */
#define KFX_OK 0
#define KFX_TRACKING_LOST 1 /* kinectfusion.cpp:97-101: "tracking fail!" -> reset() */
#define KFX_ERR_ARG (-1)
#define KFX_ERR_HIP (-2)
#define KFX_ERR_OOM (-3)
#define KFX_ERR_STATE (-4)
#define KFX_ERR_NO_DEVICE (-5)
#define KFX_ERR_COMM (-6)

#define KFX_COMM_ID_BYTES 128

/* kf::Intrinsics (types.hpp:13-29).  `c` (types.hpp:17) is unused on the path. */
typedef struct kfx_intrinsics {
  int width, height;
  float fx, fy, cx, cy;
} kfx_intrinsics;

/* cv::Affine3f as used on the path: rotation row-major R[3*i+j] = R(i,j). */
typedef struct kfx_pose {
  float R[9];
  float t[3];
} kfx_pose;

/* kf::kinectfuison_params (kinectfusion.h:9-30); defaults kinectfusion.cpp:167-190. */
typedef struct kfx_params {
  int pyramid_height;            /* 3 */
  float dfilter_dist;            /* 5 m depth truncation (image_process.cu:15) */
  int bfilter_kernel_size;       /* 5 */
  float bfilter_spatial_sigma;   /* 10 (pixels) */
  float bfilter_color_sigma;     /* 10 (mm) */
  float icp_dist_threshold;      /* 0.015 m */
  float icp_angle_threshold;     /* 30 degrees; stored as sinf(deg2rad) (icp_registration.cpp:5) */
  int icp_iter_count[KFX_MAX_LEVELS]; /* indexed by level: {4,5,10} */
  float volu_range[3];           /* metres, 3 */
  int volu_dims[3];              /* 512 */
  float volu_trun_dist;          /* 2.1 * range / dims */
  kfx_pose volu_pose;            /* translate(-L/2, -L/2, 0.5) */
  int tsdf_max_weight;           /* 64; the kernel uses MAX_WEIGHT (device_utils.cuh:5) */
  float min_pose_move;           /* unused by the reference path */
} kfx_params;

typedef struct kfx_ctx kfx_ctx;

/* ---- library ------------------------------------------------------------ */
int kfx_abi_version(void);
const char *kfx_last_error(void);
/* kinectfuison_params::default_params (kinectfusion.cpp:167-190). */
int kfx_default_params(kfx_params *out);

/* ---- kf::kinectfusion ---------------------------------------------------- */
/* kinectfusion::kinectfusion(intr, params) (kinectfusion.cpp:9-27).  device =
 * HIP ordinal.  Allocates frames, the TSDF volume and ICP workspaces, then
 * reset()s. */
int kfx_create(const kfx_intrinsics *intr, const kfx_params *params, int device,
               kfx_ctx **out);
/* kinectfusion::release() + ~kinectfusion() (kinectfusion.cpp:28-31,191-195). */
int kfx_destroy(kfx_ctx *ctx);
/* kinectfusion::reset() (kinectfusion.cpp:133-141): frame_count=1, frames and
 * volume zeroed (the reference's partial reset, SURVEY A5, is made total),
 * pose_record = [I]. */
int kfx_reset(kfx_ctx *ctx);

/* kinectfusion::pipeline(cmap, dmap) (kinectfusion.cpp:78-127).  Host images;
 * blocks until the frame is done.  Returns KFX_OK, or KFX_TRACKING_LOST when ICP
 * failed and the reference's reset() semantics were applied (frame dropped). */
int kfx_pipeline(kfx_ctx *ctx, const uint8_t *bgr, const float *depth_mm);
int kfx_pipeline_u16(kfx_ctx *ctx, const uint8_t *bgr, const uint16_t *depth_mm);

/* Device-resident input: frames uploaded once with kfx_stage_frames are
 * processed without PCIe traffic and without a host sync (tracking state lives
 * on the device).  kfx_synchronize waits for queued frames
 * and reports them: KFX_TRACKING_LOST if any frame completed since the last
 * status check (kfx_pipeline, kfx_synchronize) was dropped by a tracking
 * failure (reset() applied, kinectfusion.cpp:97-101), KFX_ERR_HIP if the ICP
 * barrier watchdog fired, else KFX_OK. */
int kfx_stage_frames(kfx_ctx *ctx, int n_frames, const uint8_t *bgr,
                     const float *depth_mm);
int kfx_pipeline_staged(kfx_ctx *ctx, int frame_index);
int kfx_synchronize(kfx_ctx *ctx);
/* Pipelined host input (kinectfusion::pipeline, kinectfusion.cpp:48-52, without
 * the per-frame host sync): the frame is copied into a pinned 4-slot ring and
 * uploaded on a copy stream while earlier frames run, then queued like a
 * staged frame; the call returns without waiting for the GPU (it blocks only
 * when the ring slot's previous upload is still in flight).  The caller's
 * buffers are free on return.  Tracking status: kfx_synchronize. */
int kfx_pipeline_async(kfx_ctx *ctx, const uint8_t *bgr, const float *depth_mm);
int kfx_pipeline_async_u16(kfx_ctx *ctx, const uint8_t *bgr, const uint16_t *depth_mm);
/* Zero-copy host input: page-lock a caller buffer (hipHostRegister).  A frame
 * whose depth and colour both lie in registered buffers is uploaded by
 * kfx_pipeline_async straight from them, with no host copy and no host wait;
 * such a buffer is then read asynchronously and must stay unchanged until
 * kfx_synchronize returns (or kfx_unregister_host_buffer, which waits for
 * pending uploads).  kfx_destroy unregisters what is left. */
int kfx_register_host_buffer(kfx_ctx *ctx, void *ptr, size_t bytes);
int kfx_unregister_host_buffer(kfx_ctx *ctx, void *ptr);
/* Captured hipGraphs for the per-frame launch sequence: 0 eager launches;
 * 1 (default) single-stream frames replay one graph per input, overlapped
 * staged / async frames replay their pyrDown + preprocess as a graph and
 * launch ICP, integrate and raycast eagerly; 2 as 1, and overlapped frames
 * also replay ICP + integrate + raycast as a second graph (measured slower,
 * DESIGN.md §3).  Z-slab contexts capture the same graphs, their RCCL
 * collectives (slab combine, sharded-ICP all-reduces) as graph nodes; if RCCL
 * refuses stream capture those frames launch eagerly instead.  Frames of an
 * in-process group (kfx_pipeline_group) launch eagerly when overlapped.
 * Results are identical in every mode. */
int kfx_set_graph_mode(kfx_ctx *ctx, int enabled);
/* The mode in effect: as set, lowered where a capture was refused (RCCL
 * refusing capture: 2 -> 1 for overlapped frames, 1 -> 0 for single-stream
 * frames of a communicator context). */
int kfx_get_graph_mode(kfx_ctx *ctx, int *mode);
/* Why graph mode 2 was lowered to 1 on this context (the RCCL / capture error
 * text), or "" (valid until the context is destroyed). */
const char *kfx_get_graph_note(kfx_ctx *ctx);
/* Overlap each staged frame's preprocess with the previous frame's tracking on
 * a second stream, over double-buffered frame maps (default on; staged frames
 * then launch eagerly instead of through graphs).  Results are identical. */
int kfx_set_frame_overlap(kfx_ctx *ctx, int enabled);
/* Sampled kernel timing inside a run of pipelined frames: every `every`-th
 * frame (from now, up to max_samples frames) is bracketed by HIP events on
 * the stream its kernels run on (such a frame launches eagerly instead of
 * through its graph); kfx_get_kernel_timing returns the mean ms of ICP,
 * integrate and raycast over the samples taken and starts a new sample set.
 * every = 0 turns sampling off. */
int kfx_set_kernel_timing(kfx_ctx *ctx, int every, int max_samples);
int kfx_get_kernel_timing(kfx_ctx *ctx, float out_ms[3], int *n_samples);
/* The same samples split further: ICP, integrate, local raycast (+ resize on a
 * single volume) and the slab combine (RCCL MIN/MAX all-reduces + expand +
 * resize; 0 on a single volume).  out_ms[2] + out_ms[3] is
 * kfx_get_kernel_timing's raycast figure.  Starts a new sample set too. */
int kfx_get_kernel_timing_ex(kfx_ctx *ctx, float out_ms[4], int *n_samples);
/* Run all ICP iterations of a frame as one persistent launch (default on; used
 * only when its grid fits co-resident on the device, else one launch per
 * iteration).  enabled: 0 = one launch per iteration, 1 = persistent (plain
 * launch), 2 = persistent through a cooperative launch (co-residency
 * guaranteed by the runtime, ~15 us slower per frame).  A context whose grid
 * barrier watchdog fires (the frame reports KFX_ERR_HIP and is dropped with a
 * volume reset) switches to mode 2 by itself.  Returns 1 if the persistent
 * kernel is usable on this context, 0 if not, <0 on error.  Results are
 * identical in every mode. */
int kfx_set_icp_persistent(kfx_ctx *ctx, int enabled);
/* Test hook: the next tracked frame's persistent-ICP barrier never completes
 * (its watchdog fires after 0.2 s). */
int kfx_debug_force_icp_stall(kfx_ctx *ctx);
/* Test hook: on != 0 routes integrate and raycast through the 64-bit-index
 * kernels (the path a volume of >= 2^31 stored voxels takes, A9:
 * device_utils.cuh:31, tsdf_volume.cpp:24) at any volume size, so the oracle
 * can pin them at sizes it runs.  Results are identical either way. */
int kfx_debug_force_index64(kfx_ctx *ctx, int on);
/* Measurement hook (tools/slab_record.py): device time of the sharded ICP's
 * per-rank launches for band `rank` of `world` (kfx_set_icp_allreduce's
 * k_icp_acc over the band's rows of every level + the k_icp_solve, 19
 * iterations at the default parameters) on the current frame maps, without
 * the all-reduces, which the caller prices separately; *ms = the mean of
 * `reps` runs.  The tracking state is saved before and restored after, so the
 * context's frames are unaffected. */
int kfx_debug_icp_band_ms(kfx_ctx *ctx, int rank, int world, int reps, float *ms);
/* Slab contexts (SURVEY.md §8e alternative): instead of every rank running
 * the whole ICP (default), rank r accumulates the 27 products over its band
 * of each level's rows and the exact int64 partials are all-reduced (SUM)
 * per iteration (19 collectives per frame), then every rank solves the same
 * system — poses identical to the replicated mode. */
int kfx_set_icp_allreduce(kfx_ctx *ctx, int enabled);
/* Profiling seam (trace builds, -DKFX_ICP_TRACE via tools/variants.sh; the
 * product library returns 0: the stamps' code costs ICP ~3 us per frame):
 * per ICP iteration of the last persistent-ICP frame, five s_memrealtime
 * stamps (100 MHz): block 0 start, block 0 arrived, block 0 released from the
 * barrier, block 0 solved, last block arrived.  Returns the number of
 * iterations written (<= max_iters). */
int kfx_get_icp_trace(kfx_ctx *ctx, uint64_t *out, int max_iters);

/* kinectfusion::getCurCameraPose() (kinectfusion.cpp:128-132). */
int kfx_get_cur_camera_pose(kfx_ctx *ctx, kfx_pose *out);
/* kinectfusion::frame_count (kinectfusion.h:58). */
int kfx_get_frame_count(kfx_ctx *ctx, int *out);
/* kinectfusion::pose_record (kinectfusion.h:59).  Writes min(cap, n) poses. */
int kfx_get_pose_record(kfx_ctx *ctx, kfx_pose *out, int cap, int *n);
/* main.cpp:95-98: pose_record as `Matx44f operator<<` text ("%.8g"). */
int kfx_write_poses_txt(kfx_ctx *ctx, const char *path);

/* ---- frame / volume access (Frame, TSDFVolume::Data) --------------------- */
#define KFX_FRAME_CUR 0  /* cframe: measured maps of the current frame */
#define KFX_FRAME_PREV 1 /* pframe: raycast (model) maps used as ICP target */
/* Download one pyramid level of a frame.  Any pointer may be NULL.  dmap is
 * metres (after bilateral + truncation), vmap/nmap float3 AoS. */
int kfx_get_frame_maps(kfx_ctx *ctx, int which, int level, float *dmap,
                       float *vmap, float *nmap);
/* Upload maps (test seam for ICP / resize). */
int kfx_set_frame_maps(kfx_ctx *ctx, int which, int level, const float *vmap,
                       const float *nmap);
/* TSDFVolume::Data() (tsdf_volume.cpp:4): export the volume as the
 * reference's 8-byte x-fastest records {int16 tsdf, int16 weight, u8 c0,c1,c2,
 * u8 pad=0} (device_types.hpp:51-56).  dst holds X*Y*Z*8 bytes. */
int kfx_download_tsdf(kfx_ctx *ctx, void *dst_records);
/* Import records in the same format (test seam; no reference counterpart).
 * Weights are stored as u8 on the device (the reference's never exceed
 * MAX_WEIGHT = 64): a record weight outside 0..255 fails with KFX_ERR_ARG. */
int kfx_upload_tsdf(kfx_ctx *ctx, const void *src_records);
/* SoA export: tsdf int16[N], weight int16[N], colour u8x4[N] (any may be NULL). */
int kfx_download_volume_soa(kfx_ctx *ctx, int16_t *tsdf, int16_t *weight,
                            uint8_t *rgba);

/* ---- stage entry points (kf::device seam, device_types.hpp:113-128) ------ */
/* imageProcess (kinectfusion.cpp:48-76): upload, pyrDown, bilateral,
 * depthTruncation, getVertexmap, getNormalmap into the CUR frame. */
int kfx_stage_preprocess(kfx_ctx *ctx, const uint8_t *bgr, const float *depth_mm);
/* rigidICP (rigid_icp.cu:135-169) one iteration at `level`: CUR vs PREV maps
 * under `pose`; returns the 27 sums (i<=j upper triangle with b, in the
 * reference's shift order) as int64 fixed point (value * 2^32). */
int kfx_stage_icp_accumulate(kfx_ctx *ctx, int level, const kfx_pose *pose,
                             int64_t sums[27]);
/* ICPRegistration::rigidTransform (icp_registration.cpp:16-46) on CUR vs PREV
 * maps: the whole coarse-to-fine loop.  Returns KFX_OK or KFX_TRACKING_LOST. */
int kfx_stage_icp(kfx_ctx *ctx, kfx_pose *cam_pose_out);
/* device::integrate (tsdf_volume.cu:103-111) of the CUR frame level-0 depth and
 * colour with vol2cam; optional counts of updated / colour-updated voxels. */
int kfx_stage_integrate(kfx_ctx *ctx, const kfx_pose *vol2cam,
                        int64_t *n_updated, int64_t *n_colored);
/* device::raycast (tsdf_volume.cu:264-273) into PREV level 0, with cam2vol and
 * Rinv (row-major 3x3), then resizePointsNormals for levels >= 1. */
int kfx_stage_raycast(kfx_ctx *ctx, const kfx_pose *cam2vol, const float Rinv[9]);

/* ---- timing -------------------------------------------------------------- */
/* Per-stage device milliseconds of the last kfx_pipeline* call run in
 * profiled mode (graph off): {preprocess, icp, integrate, raycast, total}. */
int kfx_set_profiling(kfx_ctx *ctx, int enabled);
int kfx_get_stage_ms(kfx_ctx *ctx, float out_ms[5]);
/* Voxel counts of the last processed frame's integrate (the algorithmic-byte
 * inputs of the roofline): voxels whose tsdf/weight were
 * updated and those whose colour was also blended.  Count-only kernel, the
 * volume is not touched. */
int kfx_integrate_counts(kfx_ctx *ctx, int64_t *n_updated, int64_t *n_colored);
/* Work statistics of the same count-only pass: out = {updated, coloured,
 * visited (voxels evaluated inside the per-column candidate z intervals),
 * gathered (visited voxels that project into the image and read a depth),
 * wave batches executed (4 voxels per lane each), 0, 0, 0} (slots 5-7 are
 * reserved; they held the dropped free-space certification's counts). */
int kfx_integrate_stats(kfx_ctx *ctx, int64_t out[8]);
/* Work statistics of the last processed frame's raycast (re-run on the same
 * state, nothing written): out = {rays marched, empty-space skip lookups,
 * samples skipped by them, lookups that found an occupied brick, 14-sample
 * batches marched (per ray), hit candidates whose normal was computed,
 * N_uniq = distinct voxels the reference raycast (tsdf_volume.cu:210-260, no
 * skipping) reads — nearest samples plus the trilinear corners of the normals
 * (0 for slab contexts), and the number of those reads}. */
int kfx_raycast_stats(kfx_ctx *ctx, int64_t out[8]);
/* Voxel records of n selected (x, y) columns over this context's owned slices
 * [own0, own1) (test seam for volumes too large to download whole): cols =
 * n int32 (x, y) pairs; each output holds n * (own1 - own0) entries, column
 * after column, z ascending (rgb: u8 c0, c1, c2, 0 per voxel).  Any output
 * may be null. */
/* Host side of the Z-slab raycast combine (the same code the
 * device combine runs, exposed for multi-process tests without a GPU): after
 * the all-reduce MIN of the keys, clear the payload {Ts, nout} planes (4 x n
 * u32) of the pixels this slab lost; after the all-reduce MAX of the payload
 * bits, rebuild the level-0 vmap/nmap (n float3 each) of a tracked frame at
 * cam2vol / Rinv (tsdf_volume.cu:246-255). */
int kfx_slab_mask_payload(const uint32_t *key_local, const uint32_t *key_min, uint32_t *payload, int64_t n);
int kfx_slab_expand(const uint32_t *payload, const kfx_intrinsics *intr, const kfx_pose *cam2vol,
                    const float Rinv[9], float *vmap, float *nmap);
int kfx_download_columns(kfx_ctx *ctx, const int32_t *cols, int n, int16_t *tsdf, int16_t *weight,
                         uint32_t *rgb);

/* ---- point cloud ------------------------------------------ */
/* Device ms of the last kfx_extract_points / kfx_extract_mesh call, three
 * phases.  A call with a buffer (cap > 0) normally reads the volume ONCE:
 * [0] the pass that counts every wave's items and writes them into an
 * unordered pool, [1] the offset scan, [2] the pool-to-canonical-order copy
 * (kfx_get_extract_passes = 1).  The two-pass path (count only, cap = 0;
 * kfx_set_extract_passes(2); or more items than cap, when the pool cannot hold
 * them all): [0] the count pass, [1] the scan, [2] the emit pass, which reads
 * the volume again (passes = 2; 0 if nothing was emitted). */
int kfx_get_extract_ms(kfx_ctx *ctx, float out_ms[3]);
/* Volume passes of the last extraction: 1 or 2 (see above). */
int kfx_get_extract_passes(kfx_ctx *ctx, int *passes);
/* 1 (default): kfx_extract_points / kfx_extract_mesh with a buffer read the
 * volume once; 2: always the count pass, the offset scan and the emit pass.
 * The output is identical. */
int kfx_set_extract_passes(kfx_ctx *ctx, int passes);
/* TSDFVolume::fetchPointCloud buffer size (tsdf_volume.cpp:67) */
#define KFX_DEFAULT_CLOUD_POINTS 10000000
/* kinectfusion::getRenderMap (kinectfusion.cpp:33-47; kernel_renderPhong /
 * kernel_renderNormals, image_process.cu:137-221): the previous frame's
 * level-0 raycast maps shaded on the device, lit from the last pose's camera
 * position; out = width*height uchar3, pixels without a surface 0. */
#define KFX_RENDER_PHONG 0
#define KFX_RENDER_NORMAL 1
int kfx_render(kfx_ctx *ctx, int type, uint8_t *out);

/* Order-free checksum of the (owned part of the) volume: out[0] = sum mod
 * 2^64 of a 64-bit mix of (x-fastest global voxel index, tsdf, weight,
 * colour) over every voxel, out[1] = voxels with weight > 0.  The sums of a
 * volume's Z-slabs equal the single volume's: a full-size property check
 * without downloading the volume. */
int kfx_volume_checksum(kfx_ctx *ctx, uint64_t out[2]);

/* kinectfusion::extracePointcloud (kinectfusion.cpp:142-147) ->
 * TSDFVolume::fetchPointCloud (tsdf_volume.cpp:63-84) -> device::extract_points
 * (FullScan6, tsdf_volume.cu:307-499): zero crossings of the volume along +x,
 * +y, +z, in volume-pose (world) coordinates.  Writes min(cap, total) points
 * (float3) to xyz (NULL with cap 0: count only) and the total to *n_points.
 * The reference's order is nondeterministic (atomics); here it is canonical
 * (slice chunk, 8x8 tile, z, lane, edge), so the first `cap` points
 * are deterministic.  A slab context extracts its owned slices; concatenating
 * slabs in rank order gives the single-volume cloud. */
int kfx_extract_points(kfx_ctx *ctx, float *xyz, int64_t cap, int64_t *n_points);
/* kinectfusion::savePointcloud (kinectfusion.cpp:148-166): ASCII PLY, x y z per
 * line with ostream's default 6 significant digits. */
int kfx_write_ply(const char *path, const float *xyz, int64_t n);
/* extract (cap <= 0: KFX_DEFAULT_CLOUD_POINTS) + kfx_write_ply */
int kfx_save_pointcloud(kfx_ctx *ctx, const char *path, int64_t cap);

/* Marching-cubes mesh of the zero level set (C5 asks for a mesh;
 * the reference has no counterpart).  A cube is 8 neighbouring voxels, all
 * with weight > 0; corners with tsdf < 0 are inside; the triangle table is
 * derived at run time (each face cuts off every run of inside corners, so
 * ambiguous faces resolve the same way from both sides: a crack-free mesh).
 * Edge vertices interpolate voxel centres as the point cloud does, in world
 * coordinates.  Triangles are 9 floats (3 vertices), in the point cloud's
 * canonical order; writes min(cap, total), *n_tris = total.  A slab meshes
 * its owned cubes: slab meshes concatenate to the single volume's. */
int kfx_extract_mesh(kfx_ctx *ctx, float *tri_xyz, int64_t cap_tris, int64_t *n_tris);
/* ASCII PLY of a triangle soup: 3n vertices (%g), n faces "3 i j k". */
int kfx_write_ply_mesh(const char *path, const float *tri_xyz, int64_t n_tris);

/* ---- dataset front-end (host only; no GPU needed) --------------------------
 * depth_sensor in its DATASET build (depth_sensor.cpp:11-46 open, :186-196
 * getFrame) without OpenCV: the PNG files of `<dir>/color` and `<dir>/depth` in
 * sorted name order (cv::glob), `<dir>/intr.txt` = the 3x3 camera matrix of
 * which the values > 0.1 are fx, cx, fy, cy, 1.  Frames come out as the
 * reference feeds them to kinectfusion::pipeline: colour = imread(IMREAD_COLOR)
 * (8-bit BGR: 16-bit samples keep the high byte, alpha dropped, grey
 * replicated, palette expanded), depth = imread(IMREAD_UNCHANGED) converted to
 * float (millimetres, one channel required).  Without intr.txt the camera is
 * left 640x480 with zero focal lengths and has_intr = 0. */
typedef struct kfx_dataset kfx_dataset;
int kfx_dataset_open(const char *dir, kfx_dataset **out);
int kfx_dataset_info(const kfx_dataset *ds, kfx_intrinsics *intr, int *n_frames, int *has_intr);
int kfx_dataset_read(const kfx_dataset *ds, int index, uint8_t *bgr, float *depth_mm);
int kfx_dataset_close(kfx_dataset *ds);
/* The PNG decoder and intr.txt parse underneath (any PNG colour type / bit
 * depth, Adam7, CRC-checked; sizes must match). */
int kfx_png_info(const char *path, int *width, int *height, int *channels, int *bit_depth);
int kfx_png_read_bgr8(const char *path, uint8_t *bgr, int width, int height);
int kfx_png_read_depth(const char *path, float *depth, int width, int height);
int kfx_parse_intr(const char *path, float out5[5]);

/* ---- Z-slab sharding (new; the reference is single-GPU) -------------------
 * One kf::kinectfusion stream split over `world` GPUs: slab
 * `rank` owns global z slices [cut(rank), cut(rank+1)) of the volume, cut(r) =
 * floor(Z*r/world) rounded down to a multiple of 8 (cut(world) = Z),
 * and stores 4 halo slices on each side, which it integrates itself.
 * Preprocess and ICP run on every slab (identical results, no collective);
 * raycast events are combined across slabs each frame (all-reduce MIN of the
 * per-pixel event sample index, then all-reduce MAX of the winner's map bits),
 * so every slab ends each frame with the same poses and model maps as a
 * single-GPU kfx_create context, bit for bit. */
int kfx_create_slab(const kfx_intrinsics *intr, const kfx_params *params, int device,
                    int rank, int world, kfx_ctx **out);
/* Work-balanced slabs: slab r owns [cuts[r], cuts[r+1]) (cuts[0] = 0,
 * cuts[world] = Z, multiples of 8, >= 8 slices each; every rank passes the
 * same cuts).  kfx_slice_work gives, per global slice, an estimate of a
 * frame's integrate cost at the first frame's pose (any context, slab or not;
 * from the frame's filtered depth: voxel slots visited plus 1/40 of the
 * slice's X*Y stored slots); kfx_slab_balance turns such a
 * histogram into cuts minimising the largest slab's stored-range work (halos
 * included).  Results stay bit-identical to the single volume for any cuts.
 * Side effect: kfx_slice_work(_parts) preprocesses the given frame into the
 * context's buffer set 0 (current-frame maps, colour input, {depth, 1/lambda}
 * table); the volume, poses and previous-frame maps are untouched.  Called on
 * a context mid-sequence, kfx_get_frame_maps(KFX_FRAME_CUR), kfx_render and
 * kfx_integrate_stats then describe this frame, not the last tracked one:
 * call it before the sequence (as bench.py does) or on a scratch context. */
int kfx_create_slab_cuts(const kfx_intrinsics *intr, const kfx_params *params, int device,
                         int rank, int world, const int *cuts, kfx_ctx **out);
int kfx_slice_work(kfx_ctx *ctx, const uint8_t *bgr, const float *depth_mm, int64_t *work);
/* The two parts kfx_slice_work measures, per global slice (it weighs cover): cover = the voxel
 * slots integrate's waves step through (64 per column tile whose z interval
 * holds the slice), updated = the voxels whose depth test passes. */
int kfx_slice_work_parts(kfx_ctx *ctx, const uint8_t *bgr, const float *depth_mm, int64_t *cover,
                         int64_t *updated);
/* kfx_slice_work of a frame seen from cam_pose (camera-to-world, as in the
 * pose record; null = the identity pose of a first frame), with its parts
 * (cover / updated may be null).  Averaging several frames of a sequence at
 * their poses gives cuts for the whole run rather than its first frame
 * (bench.py --cuts balanced). */
int kfx_slice_work_at(kfx_ctx *ctx, const uint8_t *bgr, const float *depth_mm, const kfx_pose *cam_pose,
                      int64_t *work, int64_t *cover, int64_t *updated);
int kfx_slab_balance(const int64_t *slice_work, int Z, int world, int *cuts);
/* Bounded slab raycast: a slab that combines with others over
 * a communicator or in a kfx_pipeline_group marches each ray only up to the
 * previous frame's model distance along it (+ 16 voxels + 2 %), records where
 * it stopped, and after the all-reduce of [keys | stop points] re-marches the
 * pixels no slab resolved below that point (an exact second pass), so slabs
 * behind the visible surface skip the occluded space.  mode 0: off (every
 * ray marched to its end; the default: on the benchmark scenes the slowest
 * slab holds the surfaces most rays end on, so the bound did not lower it and
 * the second pass cost more); 1: on; 2: on without the margin
 * (test: most pixels take the second pass).  Results are identical in every
 * mode.  The mode decides which collectives a frame's combine issues, so it is
 * one mode for the whole decomposition: on a context with a communicator the
 * call is collective (every rank calls it with the same mode; a mismatch, or
 * a mode outside 0..2 on any rank, returns KFX_ERR_ARG on every rank and
 * leaves the mode unchanged), the mode held at kfx_comm_init is checked the
 * same way (a mismatch there returns KFX_ERR_ARG and leaves the context
 * without a communicator, so no frame can issue mismatched collectives), and
 * kfx_pipeline_group refuses members whose modes differ. */
int kfx_set_slab_bound(kfx_ctx *ctx, int mode);
/* stored slices [zb, zb+zn), owned slices [own0, own1) */
int kfx_slab_info(kfx_ctx *ctx, int *zb, int *zn, int *own0, int *own1);
/* One process per GPU: rank 0 creates the id, every rank passes it to
 * kfx_comm_init (RCCL over xGMI); kfx_pipeline* then combine through RCCL. */
int kfx_comm_get_unique_id(uint8_t id[KFX_COMM_ID_BYTES]);
int kfx_comm_init(kfx_ctx *ctx, const uint8_t id[KFX_COMM_ID_BYTES]);
/* One process driving all slabs (members k = slab k of n, no communicator; on
 * one GPU or on several with peer access): one pipeline() frame. */
int kfx_pipeline_group(kfx_ctx **ctxs, int n, const uint8_t *bgr, const float *depth_mm);
/* kfx_download_tsdf / kfx_download_volume_soa on a slab write its owned slices
 * only (at their global offsets); kfx_upload_tsdf reads its stored slices.
 * With kfx_set_kernel_timing on the members, kfx_pipeline_group runs them one
 * after another (each alone on its GPU, as one rank per GPU would) and every
 * member's kfx_get_kernel_timing_ex reports its own ICP / integrate / local
 * raycast / combine ms. */
/* One slab frame with the exchange done by the caller over any transport
 * (gloo, MPI, ...; a slab context without a communicator):
 * kfx_slab_frame_local runs pipeline()'s frame on this slab up to its local
 * raycast and downloads its per-pixel event keys (n = width*height u32) and
 * {Ts, nx, ny, nz} payload planes (4n u32).  The caller all-reduces the keys
 * with MIN over the slabs, applies kfx_slab_mask_payload with them, all-reduces
 * the payload with MAX and passes it to kfx_slab_frame_finish, which rebuilds
 * the model maps and the pyramid on the device exactly like the RCCL combine
 * and returns pipeline()'s status. */
int kfx_slab_frame_local(kfx_ctx *ctx, const uint8_t *bgr, const float *depth_mm, uint32_t *keys,
                         uint32_t *payload);
int kfx_slab_frame_finish(kfx_ctx *ctx, const uint32_t *payload);

#ifdef __cplusplus
}
#endif
#endif /* KFX_H */
