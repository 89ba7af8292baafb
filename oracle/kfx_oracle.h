/*
 * kfx_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference KinectFusion hot path
 * (baiyuntao00/SLAM-KinectFusion, kfusion/src/{image_process.cu, rigid_icp.cu,
 * icp_registration.cpp, tsdf_volume.cu, tsdf_volume.cpp, kinectfusion.cpp}) and
 * of the OpenCV pieces it calls (cv::cuda::pyrDown, cv::cuda::bilateralFilter,
 * cv::Affine3f).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it — as the checker, never as the product.
 *
 * PARITY STATUS: the reference cannot be built here (CUDA + OpenCV, MSVC-only,
 * SURVEY.md §8c) and ships no tests or golden vectors, so this oracle is
 * "parity unpinned" against the original CUDA binary.  It is pinned instead by
 * analytic known-answer tests (tests/test_oracle_kat.py) and by the reference's
 * only data artifact (doc/poses.txt, format only).  Deviations from the CUDA
 * original are the "D" decisions of SURVEY.md Appendix A, listed in DESIGN.md.
 *
 * Single-threaded, built with -ffp-contract=off (oracle/Makefile) so every float
 * operation happens in the written order with IEEE rounding.
 */
#ifndef KFX_ORACLE_H
#define KFX_ORACLE_H

#include <stdint.h>
#include "../include/kfx.h"

#ifdef __cplusplus
extern "C" {
#endif

/* exp used by the bilateral weights (defined semantics) */
float kfo_expf(float x);

/* cv::cuda::pyrDown (kinectfusion.cpp:55): dst is ((w+1)/2) x ((h+1)/2). */
void kfo_pyr_down(const float *src, int w, int h, float *dst);
/* cv::cuda::bilateralFilter (kinectfusion.cpp:60-64), out of place (A1: D). */
void kfo_bilateral(const float *src, int w, int h, int ksz, float sigma_color,
                   float sigma_spatial, float *dst);
/* kernal_depthTruncation (image_process.cu:8-17). */
void kfo_depth_truncation(float *d, int n, float max_dist);
/* kernel_getVertexmap (image_process.cu:29-43) with level intrinsics. */
void kfo_vertex_map(const float *d, int w, int h, float fx, float fy, float cx,
                    float cy, float *vmap);
/* kernel_getNormalmap (image_process.cu:57-84); writes border = 0. */
void kfo_normal_map(const float *vmap, int w, int h, float *nmap);
/* kernel_resizePointsNormals (image_process.cu:95-125); big is 2w x 2h. */
void kfo_resize_points_normals(const float *vbig, const float *nbig, int ws,
                               int hs, float *vsmall, float *nsmall);
/* kinectfusion::imageProcess (kinectfusion.cpp:48-76) for all levels.
 * dmap/vmap/nmap are arrays of `levels` pointers. */
void kfo_preprocess(const float *depth_mm, int w, int h, int levels,
                    const kfx_intrinsics *intr, const kfx_params *p,
                    float **dmap, float **vmap, float **nmap);
/* Intrinsics::level (types.hpp:18-28). */
void kfo_level_intrinsics(const kfx_intrinsics *in, int level,
                          kfx_intrinsics *out);

/* kernel_rigidICP + reduction (rigid_icp.cu:46-169), one iteration:
 * 27 sums as int64 fixed point (product * 2^32, rounded to nearest even). */
void kfo_icp_accumulate(const float *cur_v, const float *cur_n,
                        const float *pre_v, const float *pre_n, int w, int h,
                        const kfx_intrinsics *lintr, const kfx_pose *pose,
                        float dist_thres, float angle_thres, int64_t sums[27]);
/* det check + solve + Rodrigues + pose = pose * Tinc
 * (icp_registration.cpp:33-42).  Returns 0 ok, 1 tracking failure. */
/* D: deterministic cos/sin of the Rodrigues angle (theta < 0.5: polynomial, else libm) */
void kfo_sincos(double theta, double *s, double *c);
int kfo_icp_update(const int64_t sums[27], kfx_pose *pose, double x_out[6]);
/* ICPRegistration::rigidTransform (icp_registration.cpp:16-46). */
int kfo_icp_track(float **cur_v, float **cur_n, float **pre_v, float **pre_n,
                  const kfx_intrinsics *intr, const kfx_params *p,
                  kfx_pose *cam_pose);

/* Affine3f helpers (float, OpenCV operation order; inv is analytic) */
void kfo_pose_mul(const kfx_pose *a, const kfx_pose *b, kfx_pose *out);
void kfo_pose_inv(const kfx_pose *a, kfx_pose *out);
void kfo_pose_identity(kfx_pose *out);

/* tsdfhelper / kernel_integrate (tsdf_volume.cu:34-111).  Volume is SoA:
 * tsdf int16[N], weight int16[N], rgb u8x4[N]; idx = x + y*X + z*X*Y.
 * cols: optional list of (x,y) pairs to restrict to (NULL = all columns).
 * n_upd / n_col: counts of updated / colour-updated voxels (may be NULL). */
/* One voxel's tsdf / weight running average (tsdf_volume.cu:72-81). */
void kfo_tsdf_update(int t0, int w0, float sdf, float trunc, int *q, int *new_w);
void kfo_integrate(int16_t *tsdf, int16_t *weight, uint8_t *rgb, const int dims[3],
                   const float voxel_size[3], float trunc_dist,
                   const kfx_intrinsics *intr, const kfx_pose *vol2cam,
                   const float *dmap, const uint8_t *bgr, const int32_t *cols,
                   int64_t ncols, int64_t *n_upd, int64_t *n_col);
/* raycasthelper / kernal_raycast (tsdf_volume.cu:120-273).  Writes vmap/nmap
 * of the pixels processed (misses = 0, as Frame::reset leaves them).
 * pix: optional list of (x,y) pairs (NULL = all pixels). */
void kfo_raycast(const int16_t *tsdf, const int dims[3], const float voxel_size[3],
                 const float range[3], const kfx_intrinsics *intr,
                 const kfx_pose *cam2vol, const float Rinv[9], float *vmap,
                 float *nmap, const int32_t *pix, int64_t npix);

/* Whole-pipeline restatement of kf::kinectfusion (kinectfusion.cpp:9-195). */
/* Z-slab restatement of the raycast: tsdf readable only in
 * slices [zb, zb+zn); events only at samples whose nearest voxel z is in
 * [own0, own1); keys[] = loop index of the deciding sample (UINT32_MAX none). */
/* distinct voxels read by the reference raycast (samples + normal corners) and
 * the number of reads (SURVEY.md §8d N_uniq) */
void kfo_raycast_touched(const int16_t *tsdf, const int dims[3], const float vs[3],
                         const float range[3], const kfx_intrinsics *in, const kfx_pose *pose,
                         const float Rinv[9], int64_t *n_uniq, int64_t *n_reads);
void kfo_raycast_slab(const int16_t *tsdf, const int dims[3], const float vs[3],
                      const float range[3], const kfx_intrinsics *in, const kfx_pose *pose,
                      const float Rinv[9], int zb, int zn, int own0, int own1, float *vmap,
                      float *nmap, uint32_t *keys, float *ts /* Ts of the hit per pixel (0: none), nullable */);

/* FullScan6 point extraction (tsdf_volume.cu:307-481), canonical order; x-fastest
 * volume; z in [zlo, zhi); writes min(cap, total) points, returns total. */
int64_t kfo_extract_points(const int16_t *tsdf, const int16_t *weight, const int dims[3],
                           const float vs[3], const kfx_pose *aff, int zlo, int zhi, float *out,
                           int64_t cap);

/* Marching cubes: 256 x 16 table {n_tri, 3 n_tri edges}; triangle soup of the
 * zero level set over cubes z in [zlo, zhi) in the canonical order (9 floats
 * per triangle; writes min(cap, total), returns total). */
void kfo_mc_table(uint8_t *tab);
int64_t kfo_extract_mesh(const int16_t *tsdf, const int16_t *weight, const int dims[3], const float vs[3],
                         const kfx_pose *aff, int zlo, int zhi, float *out, int64_t cap);

/* renderPhong (type 0) / renderNormals (type 1), image_process.cu:137-221:
 * w*h uchar3 from the level-0 vmap/nmap and the camera position. */
void kfo_render(const float *vmap, const float *nmap, int w, int h, const float eye[3], int type,
                uint8_t *out);

typedef struct kfo_pipe kfo_pipe;
kfo_pipe *kfo_pipe_create(const kfx_intrinsics *intr, const kfx_params *p);
void kfo_pipe_destroy(kfo_pipe *pp);
void kfo_pipe_reset(kfo_pipe *pp);
/* returns 0 (KFX_OK) or 1 (KFX_TRACKING_LOST) */
int kfo_pipe_process(kfo_pipe *pp, const uint8_t *bgr, const float *depth_mm);
int kfo_pipe_frame_count(const kfo_pipe *pp);
int kfo_pipe_pose_count(const kfo_pipe *pp);
void kfo_pipe_get_pose(const kfo_pipe *pp, int i, kfx_pose *out);
/* pointers into the pipe's state (valid until destroy) */
int16_t *kfo_pipe_tsdf(kfo_pipe *pp);
int16_t *kfo_pipe_weight(kfo_pipe *pp);
uint8_t *kfo_pipe_rgb(kfo_pipe *pp);
float *kfo_pipe_map(kfo_pipe *pp, int which, int kind, int level); /* kind 0 d,1 v,2 n */
/* last frame's stage counts (integrate n_upd, n_col) */
void kfo_pipe_last_counts(const kfo_pipe *pp, int64_t *n_upd, int64_t *n_col);

/* main.cpp:95-98 pose text (Matx44f operator<<, %.8g). */
int kfo_format_pose(const kfx_pose *p, char *buf, int cap);

#ifdef __cplusplus
}
#endif
#endif
