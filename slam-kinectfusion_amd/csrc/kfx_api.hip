// kfx_api.hip — host runtime behind the C-ABI (include/kfx.h).
//
// Owns every device buffer of one kf::kinectfusion instance, enqueues the
// per-frame kernel sequence on one HIP stream (captured once into a hipGraph),
// and keeps the tracking state on the device so a frame needs no host round
// trip.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <string>
#include <vector>

#include <rccl/rccl.h>

#include "../../include/kfx.h"
#include "kfx_internal.h"

using namespace kfx;

namespace {

thread_local std::string g_err;

int set_err(int code, const std::string &msg) {
  g_err = msg;
  return code;
}

}  // namespace

namespace kfx {
void set_error_text(const std::string &msg) { g_err = msg; }
}  // namespace kfx

namespace {

#define HIPCHK(expr)                                                                      \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess)                                                                 \
      return set_err(KFX_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));     \
  } while (0)

DevPose to_dev(const kfx_pose &p) {
  DevPose d;
  std::memcpy(d.R, p.R, sizeof(d.R));
  std::memcpy(d.t, p.t, sizeof(d.t));
  return d;
}
kfx_pose to_api(const DevPose &d) {
  kfx_pose p;
  std::memcpy(p.R, d.R, sizeof(p.R));
  std::memcpy(p.t, d.t, sizeof(p.t));
  return p;
}
DevPose identity_pose() {
  DevPose p{};
  p.R[0] = p.R[4] = p.R[8] = 1.f;
  return p;
}

// Intrinsics::level (types.hpp:18-28)
LevelGeom level_geom(const kfx_intrinsics &in, int level) {
  LevelGeom g;
  if (level == 0) {
    g = {in.width, in.height, in.fx, in.fy, in.cx, in.cy};
    return g;
  }
  const float s = std::pow(0.5f, (float)level);
  g.w = in.width >> level;
  g.h = in.height >> level;
  g.fx = in.fx * s;
  g.fy = in.fy * s;
  g.cx = (in.cx + 0.5f) * s - 0.5f;
  g.cy = (in.cy + 0.5f) * s - 0.5f;
  return g;
}

constexpr int kInitialPoseCap = 1 << 16;

}  // namespace

// per-frame stage events: [0] start, [1] preprocess done, [2] ICP done,
// [3] integrate done, [4] frame done, [5] local raycast done, [6] combine starts,
// [7] / [8] a group combine's shared part (reductions, masks, resume) starts / ends
constexpr int kStageEvents = 9;

struct kfx_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  kfx_intrinsics intr{};
  kfx_params p{};
  int L = 0;
  LevelGeom g[kMaxLevels]{};
  float angle_thr = 0.f;

  float *raw[kMaxLevels]{};  // raw[0] = f32 mm input, raw[l] = pyrDown outputs
  uint16_t *raw0_u16 = nullptr;
  uint8_t *bgr = nullptr;
  FrameView cur{}, prev{};
  float *inv_lambda = nullptr;
  float2 *dl0 = nullptr;  // level-0 {depth m, 1/lambda}, the integrate gather table (+ dmax shards)
  // cur maps, dl0 and the ICP plan over them are double-buffered: with frame
  // overlap, frame k+1's preprocess (on pstream) fills one set while frame k's
  // ICP / integrate / raycast (on stream) read the other.  cur/dl0/icp_plan
  // above alias set `par`, the one the last frame used.
  FrameView curb[2]{};
  float2 *dl0b[2]{};
  IcpPlan planb[2]{};
  int par = 0;
  bool overlap = true;
  hipStream_t pstream = nullptr;
  hipEvent_t ev_prep = nullptr, ev_free[2]{};
  // ev_free[p] elision (enqueue_frame_overlap): free_rec[p] = the last frame
  // that used set p recorded ev_free[p]; ov_linked = the last API call into
  // this context (api_seq, counted by check_ctx) enqueued an overlapped frame
  // whose ev_icp record follows its integrate
  bool free_rec[2]{};
  bool ov_linked = false;
  unsigned long long api_seq = 0, ov_api_seq = 0;
  hipEvent_t ev_icp = nullptr;  // after the last overlapped frame's ICP, or its integrate (KFX_PREP_AFTER_INT): the next preprocess starts there
  hipEvent_t ev_group = nullptr;  // kfx_pipeline_group combine: fork (member 0) / join (the others)
  // raycast start signal (KFX_PREP_SIG): fine-grained word the frame's raycast
  // stores sig_serial to as it starts; the next preprocess waits for it with
  // hipStreamWaitValue32 on its own stream (null: unsupported, ev_icp instead)
  unsigned *start_sig = nullptr;
  unsigned sig_serial = 0;
  bool sig_prev = false;    // the last overlapped frame signalled sig_serial
  bool ray_sig_on = false;  // enqueue_map: pass the signal to this raycast
  bool ov_order = false, ov_order_prev = false;    // enqueue_map: the next preprocess stream launches k_int_order (KFX_ORDER_OFF_PATH)
  unsigned frame_sig = 0;   // the serial the frame run_frame just enqueued signals (0: none)
  bool group_chain = false;     // kfx_pipeline_group member: record ev_icp after every ICP
  bool graphs_stale = false;    // a refused persistent ICP launch: captured graphs still hold it

  // sampled kernel timing (kfx_set_kernel_timing): every `timing_every`-th
  // pipelined frame records its stage events into the next unused set
  int timing_every = 0;
  unsigned long long frame_seq = 0;
  std::vector<hipEvent_t> tsets;  // kStageEvents per sample
  size_t tnext = 0;
  VolView vol{};
  DevState *st = nullptr;
  DevPose *pose_log = nullptr;
  int pose_cap = 0;
  unsigned long long *icp_shards = nullptr;  // 8 x 27 int64 + ticket (self-resetting)
  unsigned *icp_ticket = nullptr;
  IcpSync *icp_sync = nullptr;  // persistent ICP barrier + per-iteration shard slots
  IcpPlan icp_plan{};
  bool icp_persistent = false;  // plan fits and its grid is co-resident
  bool icp_persistent_enabled = true;
  bool icp_coop = false;  // cooperative launch of the persistent ICP (after a watchdog stall, or asked for)
  bool icp_sharded = false;  // slab ranks: ICP partials all-reduced (kfx_set_icp_allreduce)
  unsigned long long *counters = nullptr;
  float *xpose = nullptr;  // explicit stage poses (21 floats: pose R,t + Rinv)
  std::vector<void *> allocs;

  float *staged_depth = nullptr;
  uint8_t *staged_bgr = nullptr;
  int n_staged = 0;

  bool graph_mode = true;
  bool profiling = false;
  hipGraphExec_t graph[2] = {nullptr, nullptr};  // [u16 input], inputs in raw[0]/bgr
  std::vector<hipGraphExec_t> staged_graph;       // one per staged frame (reads it in place)
  // overlapped staged frames: per staged frame and buffer set p, [4i+2p] the
  // pyrDown/preprocess graph (pstream), [4i+2p+1] the ICP/integrate/raycast graph
  std::vector<hipGraphExec_t> ov_graph;
  bool ov_graph_full = false;  // also capture ICP/integrate/raycast (kfx_set_graph_mode 2)
  bool cap_ext = false;        // capturing: the ev_icp record becomes an event-record node
  bool ov_main_refused = false;  // the main graph's capture failed (RCCL refused capture): eager
  hipError_t cap_err = hipSuccess;  // the last capture's HIP error (capture_graph)
  std::string graph_note;           // why the main graph was dropped (kfx_get_graph_note)
  const uint8_t *last_bgr = nullptr;              // colour the last frame integrated
  hipEvent_t ev[kStageEvents]{};  // stage events; [5]: local raycast done, [6]: combine starts (slabs)
  float stage_ms[5]{};
  int pending = 0;      // frames enqueued since the last host sync
  int known_poses = 1;  // n_poses at the last sync
  int known_fails = 0;  // DevState::fails at the last status check

  // Z-slab sharding: this context owns slab `rank` of `world`
  bool slab = false;
  int rank = 0, world = 1;
  uint8_t *render = nullptr;      // kfx_render output (allocated on first use)
  uint8_t *mc_tab = nullptr;      // marching-cubes table (uploaded on first use)
  // per pixel: [key | pend | Ts | nx | ny | nz] planes (k_raycast<kSlab>): the
  // sample index of this slab's decisive event, the first sample a bounded
  // march left unexamined, and the hit payload
  uint32_t *key_local = nullptr;
  uint32_t *key_min = nullptr;    // all-reduce MIN of the [key | pend] planes over the slabs
  int slab_bound = 0;             // kfx_set_slab_bound: 0 off (default: measured no faster), 1 on, 2 no margin
  bool group_combine = false;     // kfx_pipeline_group member (in-process combine), this call only
  bool pass1_bounded = false;     // the frame's slab raycast was bounded: the combine runs pass 2
  // kfx_pipeline_async: host frames copied into a pinned ring slot, uploaded on
  // the copy stream while earlier frames run (slot reuse ordered by events)
  static constexpr int kRing = 4;
  uint8_t *ring_host = nullptr, *ring_dev = nullptr;
  uint8_t *ring_host_dev = nullptr;  // ring_host as mapped into the device address space
  size_t ring_slot = 0;  // bytes per slot: f32 depth + BGR8
  hipEvent_t ring_h2d[kRing]{}, ring_done[kRing]{};
  bool ring_used[kRing]{};
  unsigned ring_sig[kRing]{};  // the raycast start signal of the slot's last frame (0: wait ring_done)
  hipGraphExec_t ring_graph[kRing][2][4]{};  // overlapped-frame graphs per slot and [u16 input]
  int ring_next = 0;
  bool ring_ready = false;  // every ring resource above created
  struct HostReg {
    uintptr_t host;
    size_t bytes;
    uint8_t *dev;  // the same pages mapped into the device address space
  };
  std::vector<HostReg> host_regs;  // kfx_register_host_buffer ranges
  hipStream_t cstream = nullptr;
  ncclComm_t comm = nullptr;      // RCCL communicator over the slab ranks (one process per GPU)
  int *comm_chk = nullptr;        // 2 device words of the collective slab-bound check (kfx_comm_init)
  hipEvent_t xev[5]{};            // extraction pass events (kfx_get_extract_ms)
  int extract_passes = 0;         // the last extraction: 1 (single pass) or 2 (count + emit)
  int extract_mode = 1;           // kfx_set_extract_passes: 1 single pass when a buffer is given, 2 always two
  float extract_ms[3]{};          // last extraction: count pass, scan, emit pass
  bool ext_open = false;          // kfx_slab_frame_local done, kfx_slab_frame_finish due
  hipEvent_t *ext_pending = nullptr;  // that frame's timing sample
};

namespace {

int dalloc(kfx_ctx *c, void **p, size_t bytes) {
  hipError_t e = hipMalloc(p, bytes);
  if (e != hipSuccess) {
    *p = nullptr;
    return set_err(KFX_ERR_OOM, "hipMalloc(" + std::to_string(bytes) + "): " + hipGetErrorString(e));
  }
  c->allocs.push_back(*p);
  // zero on the context's (non-blocking) stream so later kernels on it are
  // ordered after the fill; a null-stream hipMemset would race with them
  e = hipMemsetAsync(*p, 0, bytes, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) return set_err(KFX_ERR_HIP, std::string("hipMemsetAsync: ") + hipGetErrorString(e));
  return KFX_OK;
}

#ifndef KFX_PREP_AFTER_ICP
#define KFX_PREP_AFTER_ICP 1  // overlapped frames: next preprocess waits for this frame's ICP
#endif
#ifndef KFX_PREP_SIG
#define KFX_PREP_SIG 1  // overlapped frames: the raycast's start signal replaces the ev_icp record
#endif
#ifndef KFX_ORDER_OFF_PATH
#define KFX_ORDER_OFF_PATH 1  // overlapped frames: k_int_order on the preprocess stream, beside the raycast
#endif
#ifndef KFX_FREE_ELIDE
#define KFX_FREE_ELIDE 1  // overlapped frames: no ev_free record when the next frame's ev_icp wait covers it
#endif
#ifndef KFX_PREP_AFTER_INT
// ... for this frame's integrate instead: the preprocess then shares the GPU
// with the raycast (memory-latency bound, 0.2-0.4 VALU issue) rather than the
// issue-bound integrate; C2 integrate -12 us, raycast +8 us, frame -0.4 to
// -1.4 % (7 alternating pairs)
#define KFX_PREP_AFTER_INT 1
#endif
#ifndef KFX_COST_UPDATED
#define KFX_COST_UPDATED 32  // slab balancing: weight of an updated voxel (64 = one visited slot; slice_cost)
#endif
#ifndef KFX_COST_SLOT
#define KFX_COST_SLOT 3  // slab balancing: weight of a stored voxel slot (64 = one visited slot)
#endif
#ifndef KFX_VOL_PAD
#define KFX_VOL_PAD 4096  // weight offset past the 2 MiB-rounded tsdf (bytes)
#endif
size_t nvox(const kfx_ctx *c) { return c->vol.local_voxels(); }

void set_par(kfx_ctx *c, int p) {
  c->par = p;
  c->cur = c->curb[p];
  c->dl0 = c->dl0b[p];
  c->icp_plan = c->planb[p];
}

void destroy_graphs(kfx_ctx *c) {
  for (auto &gx : c->graph)
    if (gx) {
      (void)hipGraphExecDestroy(gx);
      gx = nullptr;
    }
  for (auto &gx : c->staged_graph)
    if (gx) {
      (void)hipGraphExecDestroy(gx);
      gx = nullptr;
    }
  for (auto &slot : c->ring_graph)
    for (auto &gs : slot)
      for (auto &gx : gs)
        if (gx) {
          (void)hipGraphExecDestroy(gx);
          gx = nullptr;
        }
  for (auto &gx : c->ov_graph)
    if (gx) {
      (void)hipGraphExecDestroy(gx);
      gx = nullptr;
    }
}

// Frame input: depth (f32 mm, or u16 mm) and BGR8 colour, in device memory;
// ready (optional): the input is in place once this event completes (async
// host input); done (optional): recorded after the frame's last kernel.
struct FrameInput {
  const float *d32;
  const uint16_t *d16;
  const uint8_t *bgr;
  hipEvent_t ready = nullptr;
  hipEvent_t done = nullptr;
};

// ev_icp behind the ICP just enqueued on s.  While a graph is being captured
// (cap_ext) the record is added as an event-record node on the captured ICP,
// so every replay records the event for the next frame's preprocess.
int record_icp_event(kfx_ctx *c, hipStream_t s) {
  if (!c->cap_ext) {
    HIPCHK(hipEventRecord(c->ev_icp, s));
    return KFX_OK;
  }
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  unsigned long long id = 0;
  hipGraph_t g = nullptr;
  const hipGraphNode_t *deps = nullptr;
  size_t nd = 0;
  HIPCHK(hipStreamGetCaptureInfo_v2(s, &cs, &id, &g, &deps, &nd));
  if (cs != hipStreamCaptureStatusActive || !g) return set_err(KFX_ERR_HIP, "ev_icp record: stream not capturing");
  hipGraphNode_t node = nullptr;
  HIPCHK(hipGraphAddEventRecordNode(&node, g, deps, nd, c->ev_icp));
  HIPCHK(hipStreamUpdateCaptureDependencies(s, &node, 1, hipStreamSetCaptureDependencies));
  return KFX_OK;
}

// The per-frame launch sequence (kinectfusion.cpp:78-127 with the frame-1 and
// failure branches resolved on the device).  `ev` (or null) receives the stage
// events: [0] start, [1] after preprocess, [2] after ICP, [3] after integrate,
// [4] after raycast (+ slab combine); [0..1] are absent for overlapped frames.
// Slab contexts stop after their local raycast (enqueue_local) and then
// combine the slabs' raycast results (enqueue_combine).
void enqueue_pre(kfx_ctx *c, FrameInput in, hipEvent_t *ev);
void enqueue_local(kfx_ctx *c, FrameInput in, hipEvent_t *ev);
int enqueue_track(kfx_ctx *c, FrameInput in, hipEvent_t *ev, bool begin);
int enqueue_combine(kfx_ctx *c);
void enqueue_slab_resume(kfx_ctx *c, hipStream_t s);

int enqueue_frame(kfx_ctx *c, FrameInput in, hipEvent_t *ev) {
  enqueue_pre(c, in, ev);
  int r = enqueue_track(c, in, ev, false);
  if (ev) (void)hipEventRecord(ev[5], c->stream);
  if (ev && c->slab) {  // (a single volume's sample ends at [5]: no combine to time)
    (void)hipEventRecord(ev[6], c->stream);
    (void)hipEventRecord(ev[7], c->stream);  // (no shared part: [7] = [8])
    (void)hipEventRecord(ev[8], c->stream);
  }
  if (!r && c->slab) r = enqueue_combine(c);
  if (ev) (void)hipEventRecord(ev[4], c->stream);  // (the profiled frames' end)
  return r;
}

#define NCCLCHK(expr)                                                                      \
  do {                                                                                     \
    ncclResult_t e_ = (expr);                                                              \
    if (e_ != ncclSuccess)                                                                 \
      return set_err(KFX_ERR_COMM, std::string(#expr) + ": " + ncclGetErrorString(e_));    \
  } while (0)

// Cross-slab raycast combine: all-reduce MIN of the per-pixel
// event keys (with the pend plane when the slabs' marches were bounded, and
// then the resume pass for the pixels no slab resolved, and a MIN of the keys
// again), each slab clears the payload {Ts, nout} of the pixels it lost,
// all-reduce MAX of the payload bits (16 B per pixel instead of the 24 B of
// vmap|nmap), every rank rebuilds the level-0 maps from it, then the pyramid.
int enqueue_combine(kfx_ctx *c) {
  hipStream_t s = c->stream;
  const size_t np = (size_t)c->g[0].w * c->g[0].h;
  uint32_t *pay = c->key_local + 2 * np;  // [Ts | nx | ny | nz] planes after [keys | pend]
  if (c->world > 1 || c->comm) {
    if (!c->comm) return set_err(KFX_ERR_STATE, "slab context without a communicator (kfx_comm_init, or kfx_pipeline_group)");
    if (c->pass1_bounded) {
      NCCLCHK(ncclAllReduce(c->key_local, c->key_min, 2 * np, ncclUint32, ncclMin, c->comm, s));
      enqueue_slab_resume(c, s);
    }
    NCCLCHK(ncclAllReduce(c->key_local, c->key_min, np, ncclUint32, ncclMin, c->comm, s));
    launch_slab_mask(s, c->key_local, c->key_min, (int)np);
    NCCLCHK(ncclAllReduce(pay, pay, 4 * np, ncclUint32, ncclMax, c->comm, s));
  }
  launch_slab_expand(s, c->g[0], pay, c->cur, c->prev, c->st, c->pose_log, to_dev(c->p.volu_pose));
  launch_resize(s, c->L, c->g, c->cur, c->prev, c->st, nullptr);
  return KFX_OK;
}

// imageProcess (kinectfusion.cpp:48-76) into the current set
void enqueue_pre(kfx_ctx *c, FrameInput in, hipEvent_t *ev) {
  hipStream_t s = c->stream;
  if (ev) (void)hipEventRecord(ev[0], s);
  const float *raw[kMaxLevels];
  for (int l = 0; l < kMaxLevels; ++l) raw[l] = c->raw[l];
  raw[0] = in.d32;
  if (c->L > 1) {
    launch_pyr_down(s, in.d32, in.d16, c->g[0].w, c->g[0].h, c->raw[1], c->st, c->dl0);
    for (int l = 2; l < c->L; ++l)
      launch_pyr_down(s, c->raw[l - 1], nullptr, c->g[l - 1].w, c->g[l - 1].h, c->raw[l], nullptr,
                      nullptr);
  } else {
    launch_frame_begin(s, c->st, c->dl0, c->g[0]);
  }
  launch_preprocess_maps(s, c->L, raw, in.d16, c->g, c->cur, c->p.bfilter_kernel_size,
                         c->p.bfilter_color_sigma, c->p.bfilter_spatial_sigma, c->p.dfilter_dist,
                         c->inv_lambda, c->dl0);
  if (ev) (void)hipEventRecord(ev[1], s);
}

void enqueue_local(kfx_ctx *c, FrameInput in, hipEvent_t *ev) {
  enqueue_pre(c, in, ev);
  (void)enqueue_track(c, in, ev, false);
}

// Sharded ICP (kfx_set_icp_allreduce): this rank's band of
// every level's rows, the 27 exact int64 partials all-reduced over RCCL per
// iteration, every rank solving the same sums (poses identical to the
// replicated mode).
int enqueue_icp_sharded(kfx_ctx *c, bool begin) {
  hipStream_t s = c->stream;
  if (begin) launch_frame_begin(s, c->st, nullptr, c->g[0]);
  long long *sums = reinterpret_cast<long long *>(reinterpret_cast<char *>(c->st) + offsetof(DevState, sums));
  for (int level = c->L - 1; level >= 0; --level)
    for (int it = 0; it < c->p.icp_iter_count[level]; ++it) {
      launch_icp(s, c->g[level], c->cur.v[level], c->cur.n[level], c->prev.v[level], c->prev.n[level],
                 c->p.icp_dist_threshold, c->angle_thr, c->st, c->icp_shards, c->icp_ticket, 0, 0, c->rank,
                 c->world);
      NCCLCHK(ncclAllReduce(sums, sums, 27, ncclInt64, ncclSum, c->comm, s));
      launch_icp_solve(s, c->st);
    }
  return KFX_OK;
}

// The slab raycast's first pass is bounded by the previous frame's model
// (SlabPass) when the frame's combine can run the resume pass: several slabs
// combined over a communicator or in-process (kfx_pipeline_group)
SlabPass slab_pass1(kfx_ctx *c) {
  SlabPass sp;
  c->pass1_bounded = c->slab && c->slab_bound && c->world > 1 && (c->comm || c->group_combine);
  if (c->pass1_bounded) {
    sp.pass = 1;
    sp.bound_abs = c->slab_bound == 2 ? 0.f : 16.f * c->vol.vs[0];  // 16 voxels
    sp.bound_rel = c->slab_bound == 2 ? 0.f : 0.02f;
  }
  return sp;
}
// pass 2: the pixels this slab left pending below the reduced [key | pend]
void enqueue_slab_resume(kfx_ctx *c, hipStream_t s) {
  SlabPass sp;
  sp.pass = 2;
  sp.kmin = c->key_min;
  launch_raycast(s, c->vol, c->L, c->g, c->cur, c->prev, c->st, c->pose_log, to_dev(c->p.volu_pose), nullptr,
                 c->key_local, nullptr, sp);
}

// integrate + raycast of the frame whose maps are in the current set
int enqueue_map(kfx_ctx *c, FrameInput in, hipEvent_t *ev, bool rec_int = false) {
  hipStream_t s = c->stream;
  launch_integrate(s, c->vol, c->g[0], c->dl0, c->cur.d[0], c->inv_lambda, in.bgr, c->st, c->pose_log,
                   to_dev(c->p.volu_pose), nullptr, nullptr, !c->ov_order);
  if (ev) (void)hipEventRecord(ev[3], s);
  if (rec_int) {
    const int r = record_icp_event(c, s);
    if (r) return r;
  }
  launch_raycast(s, c->vol, c->L, c->g, c->cur, c->prev, c->st, c->pose_log,
                 to_dev(c->p.volu_pose), nullptr, c->slab ? c->key_local : nullptr, nullptr, slab_pass1(c),
                 c->ray_sig_on ? c->start_sig : nullptr, c->sig_serial);
  return KFX_OK;
}

// The persistent ICP launch, if this context uses it.  False when it does not,
// or when the runtime refused the launch (a cooperative grid it cannot make
// co-resident): the context then takes the per-iteration launches from now on.
bool try_icp_persistent(kfx_ctx *c, hipStream_t s, int begin) {
  if (!c->icp_persistent || !c->icp_persistent_enabled) return false;
  if (launch_icp_track(s, c->icp_plan, c->st, c->icp_sync, begin, c->icp_coop) == hipSuccess) return true;
  (void)hipGetLastError();
  c->icp_persistent_enabled = false;
  c->graphs_stale = true;  // (maybe mid-capture: run_frame drops the graphs before the next frame)
  return false;
}

// ICP, integrate and raycast of the frame whose maps are in the current set;
// begin: the frame's frame_begin has not run yet (overlapped frames)
int enqueue_track(kfx_ctx *c, FrameInput in, hipEvent_t *ev, bool begin) {
  hipStream_t s = c->stream;
  // ICPRegistration::rigidTransform (icp_registration.cpp:16-46)
  int r = KFX_OK;
  if (c->icp_sharded && c->comm) {
    r = enqueue_icp_sharded(c, begin);
  } else if (!try_icp_persistent(c, s, begin ? 1 : 0)) {  // (the persistent launch folds frame_begin in)
    if (begin) launch_frame_begin(s, c->st, nullptr, c->g[0]);
    for (int level = c->L - 1; level >= 0; --level) {
      for (int it = 0; it < c->p.icp_iter_count[level]; ++it)
        launch_icp(s, c->g[level], c->cur.v[level], c->cur.n[level], c->prev.v[level],
                   c->prev.n[level], c->p.icp_dist_threshold, c->angle_thr, c->st,
                   c->icp_shards, c->icp_ticket, 0, 1);
    }
  }
  if (ev) (void)hipEventRecord(ev[2], s);
  // overlapped frames: the next preprocess waits here; a group: the next
  // member's ICP on this device waits here
  // (with the raycast start signal the next preprocess waits for that instead)
  const bool after_int = KFX_PREP_AFTER_INT && begin && !c->group_chain && !c->ray_sig_on;
  if ((begin || c->group_chain) && !after_int && !c->ray_sig_on && !r && (r = record_icp_event(c, s))) return r;
  const int rm = enqueue_map(c, in, ev, after_int && !r);
  return r ? r : rm;
}

// Frame overlap: the preprocess of this frame runs on pstream into the set the
// previous frame is not using, concurrently with the previous frame's ICP
// (which occupies few CUs), so the per-frame critical path is ICP (with
// frame_begin folded in) + integrate + raycast.  Measured cost of the two
// cross-stream dependencies: ~9 us/frame for the wait on ev_prep, while
// dropping the ev_free ordering (unsafe) is slower, as preprocess then
// competes with integrate/raycast.
// pyrDown + preprocess of an overlapped frame into the current set, on pstream.
void enqueue_prep_overlap(kfx_ctx *c, FrameInput in) {
  hipStream_t b = c->pstream;
  const float *raw[kMaxLevels];
  for (int l = 0; l < kMaxLevels; ++l) raw[l] = c->raw[l];
  raw[0] = in.d32;
  if (c->L > 1) {
    launch_pyr_down(b, in.d32, in.d16, c->g[0].w, c->g[0].h, c->raw[1], nullptr, c->dl0);
    for (int l = 2; l < c->L; ++l)
      launch_pyr_down(b, c->raw[l - 1], nullptr, c->g[l - 1].w, c->g[l - 1].h, c->raw[l], nullptr,
                      nullptr);
  } else {
    launch_frame_begin(b, nullptr, c->dl0, c->g[0]);
  }
  launch_preprocess_maps(b, c->L, raw, in.d16, c->g, c->cur, c->p.bfilter_kernel_size,
                         c->p.bfilter_color_sigma, c->p.bfilter_spatial_sigma, c->p.dfilter_dist,
                         c->inv_lambda, c->dl0);
}

// ICP (frame_begin folded in) + integrate + raycast (+ slab combine) of an
// overlapped frame, on the frame stream.
int enqueue_main_overlap(kfx_ctx *c, FrameInput in, hipEvent_t *ev) {
  if (ev) HIPCHK(hipEventRecord(ev[1], c->stream));
  int r = enqueue_track(c, in, ev, true);
  if (ev) HIPCHK(hipEventRecord(ev[5], c->stream));
  if (ev && c->slab) {  // (a single volume's sample ends at [5])
    HIPCHK(hipEventRecord(ev[6], c->stream));
    HIPCHK(hipEventRecord(ev[7], c->stream));
    HIPCHK(hipEventRecord(ev[8], c->stream));
  }
  if (!r && c->slab) r = enqueue_combine(c);
  if (ev && c->slab) HIPCHK(hipEventRecord(ev[4], c->stream));
  return r;
}

// gx (optional): this frame's two captured graphs for the set it uses
// (ensure_ov_graphs), replayed in place of the eager launches; the cross-frame
// and cross-stream event waits stay around them.
int enqueue_frame_overlap(kfx_ctx *c, FrameInput in, hipEvent_t *ev, hipGraphExec_t *gx) {
  const int p = c->par ^ 1;
  set_par(c, p);
  hipStream_t b = c->pstream;
  // Set p was last used by the frame before last.  When the previous API call
  // enqueued the previous overlapped frame and that frame records ev_icp after
  // its integrate, the ev_icp wait below already orders this preprocess after
  // that frame's integrate, and so (one in-order stream) after everything
  // enqueued on the frame stream before it — the frame before last included:
  // no ev_free record is needed (each record between two frame kernels costs
  // the frame stream 2-5 us).  Otherwise wait for ev_free[p],
  // recorded now at the frame stream's tail if its last user did not record it.
  const bool linked = KFX_FREE_ELIDE && KFX_PREP_AFTER_ICP && c->ov_linked && c->api_seq == c->ov_api_seq + 1;
  if (!linked) {
    if (!c->free_rec[p]) HIPCHK(hipEventRecord(c->ev_free[p], c->stream));
    HIPCHK(hipStreamWaitEvent(b, c->ev_free[p], 0));  // the frame before last is done with set p
  }
  c->ov_linked = false;
  c->free_rec[p] = false;
  if (in.ready) HIPCHK(hipStreamWaitEvent(b, in.ready, 0));  // host input uploaded
#if KFX_PREP_AFTER_ICP
  // start behind the previous frame's ICP (KFX_PREP_AFTER_INT: its integrate;
  // ev_icp is recorded there; KFX_PREP_SIG: as its raycast starts, which
  // stores the frame's serial): the latency-bound persistent ICP then runs
  // alone and the preprocess shares the GPU with the raycast
  if (c->sig_prev)
    HIPCHK(hipStreamWaitValue32(b, c->start_sig, c->sig_serial, hipStreamWaitValueGte, 0xffffffffu));
  else
    HIPCHK(hipStreamWaitEvent(b, c->ev_icp, 0));
#endif
  if (gx) HIPCHK(hipGraphLaunch(gx[0], b));
  else enqueue_prep_overlap(c, in);
  // the dispatch order of this frame's integrate from the previous frame's
  // intervals, off the frame stream: the wait above (its raycast has started,
  // or ev_icp behind its integrate) orders it after the integrate that read
  // the old order, and ev_prep before this frame's integrate
  if (c->ov_order_prev) launch_int_order(b, c->vol);
  HIPCHK(hipEventRecord(c->ev_prep, b));
  HIPCHK(hipStreamWaitEvent(c->stream, c->ev_prep, 0));
  int r = KFX_OK;
  // this frame's raycast signals its start (not inside a captured main graph,
  // whose launch arguments are fixed: it records ev_icp)
  const bool use_sig = KFX_PREP_SIG && KFX_PREP_AFTER_ICP && KFX_PREP_AFTER_INT && c->start_sig && !c->group_chain &&
                       !(gx && gx[1]);
  c->sig_prev = false;
  if (use_sig) {
    if (c->sig_serial >= 0x7fffffffu) {  // wrap: restart the serials from a drained context
      HIPCHK(hipStreamSynchronize(c->stream));
      HIPCHK(hipStreamSynchronize(b));
      if (c->cstream) HIPCHK(hipStreamSynchronize(c->cstream));
      HIPCHK(hipMemset(c->start_sig, 0, 64));
      c->sig_serial = 0;
      for (unsigned &v : c->ring_sig) v = 0u;  // (their frames are complete)
    }
    c->sig_serial += 1;
    c->ray_sig_on = true;
  }
  // (not for a captured main graph: it holds its own k_int_order launch)
  c->ov_order = KFX_ORDER_OFF_PATH && KFX_PREP_AFTER_ICP && KFX_PREP_AFTER_INT && !c->group_chain && !(gx && gx[1]);
  if (gx && gx[1]) HIPCHK(hipGraphLaunch(gx[1], c->stream));
  else r = enqueue_main_overlap(c, in, ev);
  c->ray_sig_on = false;
  c->ov_order_prev = c->ov_order && !r;
  c->ov_order = false;
  c->sig_prev = use_sig && !r;
  c->frame_sig = c->sig_prev ? c->sig_serial : 0u;
  // the next overlapped frame may rely on this frame's ev_icp (recorded after
  // its integrate: enqueue_track) instead of ev_free[p]
  const bool link = KFX_FREE_ELIDE && KFX_PREP_AFTER_ICP && KFX_PREP_AFTER_INT && !c->group_chain && !r;
  if (!link) {
    HIPCHK(hipEventRecord(c->ev_free[p], c->stream));
    c->free_rec[p] = true;
  }
  c->ov_linked = link;
  c->ov_api_seq = c->api_seq;
  // (a signalling frame's input slot is released by its raycast start signal)
  if (in.done && !c->frame_sig) HIPCHK(hipEventRecord(in.done, c->stream));
  return r;
}

template <typename F>
int capture_graph(kfx_ctx *c, hipStream_t s, F &&body, hipGraphExec_t *out) {
  hipGraph_t graph = nullptr;
  c->cap_err = hipSuccess;
  HIPCHK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  const int r = body();
  const hipError_t ec = hipStreamEndCapture(s, &graph);
  c->cap_err = ec;
  if (r) {
    if (graph) (void)hipGraphDestroy(graph);
    return r;
  }
  if (ec != hipSuccess) return set_err(KFX_ERR_HIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(ec));
  hipError_t e = hipGraphInstantiate(out, graph, nullptr, nullptr, 0);
  (void)hipGraphDestroy(graph);
  if (e != hipSuccess) return set_err(KFX_ERR_HIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(e));
  // upload now: a graph's first launch otherwise pays for it (staged frames'
  // graphs are each launched only a few times)
  HIPCHK(hipGraphUpload(*out, s));
  return KFX_OK;
}

// Overlapped frames replay graphs unless they run chained in an in-process
// group (kfx_pipeline_group: cross-context event waits between the members).
bool ov_graphs_apply(const kfx_ctx *c) { return c->graph_mode && !c->group_chain; }

// The graphs of an overlapped frame for buffer set p: gx[0] pyrDown +
// preprocess (replayed on pstream) and, with kfx_set_graph_mode(ctx, 2),
// gx[1] ICP + integrate + raycast (on the frame stream; its ev_icp record is
// an event-record node, so the next frame's preprocess still starts behind
// this frame's ICP).  gx[1] is off by default: its replay measured 4-6 us per
// frame slower than the eager launches of the same three kernels (the graph
// uploaded beforehand), while the preprocess graph is neutral to slightly
// faster.
// Z-slab contexts capture the same graphs: the preprocess graph is local, and
// the main graph holds the slab combine (and the sharded ICP's all-reduces) as
// RCCL nodes when RCCL accepts stream capture; if it refuses, the main part of
// every later frame launches eagerly (kfx_get_graph_mode reports 1).
int ensure_ov_graphs(kfx_ctx *c, FrameInput in, hipGraphExec_t *gx, int p) {
  const bool main = c->ov_graph_full && !c->ov_main_refused;
  if (gx[0] && (gx[1] || !main)) return KFX_OK;
  const int keep = c->par;
  set_par(c, p);
  int r = gx[0] ? KFX_OK
                : capture_graph(c, c->pstream, [&] { enqueue_prep_overlap(c, in); return KFX_OK; }, &gx[0]);
  if (!r && !gx[1] && main) {
    c->cap_ext = true;
    r = capture_graph(c, c->stream, [&] { return enqueue_main_overlap(c, in, nullptr); }, &gx[1]);
    c->cap_ext = false;
    // only a collective that refused capture (an RCCL error inside the
    // capture, or a capture the runtime reports unsupported / invalidated)
    // drops the main graph for good; every other failure is returned
    const bool refused = r == KFX_ERR_COMM || c->cap_err == hipErrorStreamCaptureUnsupported ||
                         c->cap_err == hipErrorStreamCaptureInvalidated ||
                         c->cap_err == hipErrorStreamCaptureImplicit;
    if (r && (c->comm || c->icp_sharded) && refused) {
      c->graph_note = kfx_last_error();
      (void)hipGetLastError();
      gx[1] = nullptr;
      c->ov_main_refused = true;
      r = KFX_OK;
    }
  }
  set_par(c, keep);
  return r;
}

int build_graph(kfx_ctx *c, FrameInput in, hipGraphExec_t *out) {
  return capture_graph(c, c->stream, [&] { return enqueue_frame(c, in, nullptr); }, out);
}

int read_state(kfx_ctx *c, DevState *out) {
  HIPCHK(hipMemcpyAsync(out, c->st, sizeof(DevState), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  c->pending = 0;
  c->known_poses = out->n_poses;
  return KFX_OK;
}

template <typename T>
int write_field(kfx_ctx *c, size_t off, const T &v) {
  HIPCHK(hipMemcpyAsync(reinterpret_cast<char *>(c->st) + off, &v, sizeof(T),
                        hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return KFX_OK;
}

// Grow the device pose log if the frames about to be queued could overflow it.
int ensure_pose_capacity(kfx_ctx *c, int more) {
  if (c->known_poses + c->pending + more < c->pose_cap) return KFX_OK;
  DevState s;
  int r = read_state(c, &s);
  if (r) return r;
  if (s.n_poses + more < c->pose_cap) return KFX_OK;
  const int ncap = c->pose_cap * 2;
  DevPose *nl = nullptr;
  HIPCHK(hipMalloc(&nl, sizeof(DevPose) * (size_t)ncap));
  HIPCHK(hipMemcpyAsync(nl, c->pose_log, sizeof(DevPose) * (size_t)c->pose_cap,
                        hipMemcpyDeviceToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  for (auto &a : c->allocs)
    if (a == c->pose_log) a = nl;
  HIPCHK(hipFree(c->pose_log));
  c->pose_log = nl;
  c->pose_cap = ncap;
  r = write_field(c, offsetof(DevState, pose_cap), ncap);
  if (!r) r = write_field(c, offsetof(DevState, log), nl);
  if (r) return r;
  destroy_graphs(c);  // the integrate/raycast nodes hold the old pointer
  return KFX_OK;
}

// Capture the per-frame graph for `in` if graph mode is on and it does not
// exist yet.  RCCL calls that refuse stream capture switch the context to
// eager launches (returns KFX_OK with graph mode off).
int ensure_graph(kfx_ctx *c, FrameInput in, hipGraphExec_t *graph) {
  if (!c->graph_mode || !graph || *graph) return KFX_OK;
  int r = build_graph(c, in, graph);
  if (r && c->comm) {
    (void)hipGetLastError();
    c->graph_mode = false;
    destroy_graphs(c);
    return KFX_OK;
  }
  return r;
}

// The event set of this frame's kernel-timing sample (kfx_set_kernel_timing),
// or null when the frame is not sampled.
hipEvent_t *timing_sample(kfx_ctx *c) {
  if (c->timing_every > 0 && !c->profiling && c->frame_seq++ % c->timing_every == 0 &&
      kStageEvents * (c->tnext + 1) <= c->tsets.size())
    return &c->tsets[kStageEvents * c->tnext++];
  return nullptr;
}

// graph: the cached executable for this input (built on first use), or null
// overlap: the input stays valid until the frame completes (staged frames)
// ovg: the input's four overlapped-frame graphs (ensure_ov_graphs, two per
// buffer set), or null for eager overlapped launches
int run_frame(kfx_ctx *c, FrameInput in, hipGraphExec_t *graph, bool overlap = false,
              hipGraphExec_t *ovg = nullptr) {
  int r = ensure_pose_capacity(c, 1);
  if (r) return r;
  if (c->graphs_stale) {  // captured with the persistent ICP launch the runtime refused
    HIPCHK(hipStreamSynchronize(c->pstream));
    HIPCHK(hipStreamSynchronize(c->stream));
    destroy_graphs(c);
    c->graphs_stale = false;
  }
  c->last_bgr = in.bgr;
  c->frame_sig = 0u;
  hipEvent_t *tev = timing_sample(c);  // this frame's timing sample, if sampled
  if (overlap && c->overlap && !c->profiling) {
    hipGraphExec_t *gx = nullptr;
    if (ovg && !tev && ov_graphs_apply(c)) {  // a timing sample launches eagerly with its events
      gx = ovg + 2 * (c->par ^ 1);
      if ((r = ensure_ov_graphs(c, in, gx, c->par ^ 1))) return r;
    }
    if ((r = enqueue_frame_overlap(c, in, tev, gx))) return r;
    HIPCHK(hipGetLastError());
    c->pending += 1;
    return KFX_OK;
  }
  set_par(c, 0);  // single-stream frames (and their graphs) use set 0
  if (in.ready) HIPCHK(hipStreamWaitEvent(c->stream, in.ready, 0));
  if (c->profiling) {
    if ((r = enqueue_frame(c, in, c->ev))) return r;
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventSynchronize(c->ev[4]));
    for (int i = 0; i < 4; ++i) HIPCHK(hipEventElapsedTime(&c->stage_ms[i], c->ev[i], c->ev[i + 1]));
    HIPCHK(hipEventElapsedTime(&c->stage_ms[4], c->ev[0], c->ev[4]));
    // stage order in the events: preprocess, icp(+commit), integrate,
    // raycast(+slab combine, +resize)
  } else {
    if ((r = ensure_graph(c, in, graph))) return r;
    if (c->graph_mode && graph && *graph && !tev) {
      HIPCHK(hipGraphLaunch(*graph, c->stream));
    } else {  // eager (a timing sample is launched eagerly with its events)
      if ((r = enqueue_frame(c, in, tev))) return r;
      HIPCHK(hipGetLastError());
    }
  }
  if (in.done) HIPCHK(hipEventRecord(in.done, c->stream));
  c->pending += 1;
  return KFX_OK;
}

// Status of the frames completed since the last check: a fired ICP watchdog
// (cleared here; that frame was dropped) is an error, a tracking failure of
// any of them is KFX_TRACKING_LOST.
int check_status(kfx_ctx *c, const DevState &s) {
  const bool lost = s.fails != c->known_fails;
  c->known_fails = s.fails;
  if (s.icp_stalled) {
    // the frame's ICP failed (its volume was reset, like a tracking loss);
    // later frames launch the persistent ICP cooperatively, which guarantees
    // the co-residency its grid barrier needs
    HIPCHK(hipMemsetAsync(c->icp_sync, 0, sizeof(IcpSync), c->stream));
    int r = write_field(c, offsetof(DevState, icp_stalled), 0);
    if (!r) r = write_field(c, offsetof(DevState, debug_stall), 0);
    if (!c->icp_coop) {
      c->icp_coop = true;
      destroy_graphs(c);  // captured with the plain launch
    }
    return r ? r : set_err(KFX_ERR_HIP, "ICP grid barrier watchdog fired (grid not co-resident); "
                                        "persistent ICP switched to cooperative launches");
  }
  return lost ? KFX_TRACKING_LOST : KFX_OK;
}

int finish_frame(kfx_ctx *c) {
  DevState s;
  int r = read_state(c, &s);
  if (r) return r;
  return check_status(c, s);
}

// Slab `rank` of `world` owns global slices [Z*rank/world, Z*(rank+1)/world)
// and stores kSlabHalo more on each side (clipped to the volume).
VolView make_vol(const kfx_params &p, int rank, int world, const int *cuts = nullptr) {
  VolView v{};
  v.X = p.volu_dims[0];
  v.Y = p.volu_dims[1];
  v.Z = p.volu_dims[2];
  // slab boundaries on multiples of 8 slices (the point-extraction chunk), so
  // slab clouds concatenate to the single-volume cloud; equal slice ranges
  // unless explicit cuts are given (kfx_create_slab_cuts)
  auto cut = [&](int r) {
    if (cuts) return cuts[r];
    return r >= world ? v.Z : (int)((long long)v.Z * r / world) / 8 * 8;
  };
  v.own0 = cut(rank);
  v.own1 = cut(rank + 1);
  if (world > 1) {
    v.zb = std::max(0, v.own0 - kSlabHalo);
    v.zn = std::min(v.Z, v.own1 + kSlabHalo) - v.zb;
  } else {
    v.zb = 0;
    v.zn = v.Z;
  }
  v.tiles_x = v.X / 8;
  v.tiles_y = v.Y / 8;
  v.slice = (size_t)v.X * v.Y;
  // occupancy maps over the stored slices (bricks on global multiples of 8 / 32)
  const int zl = v.zb + v.zn - 1;
  v.bz0 = v.zb >> 3;
  v.nbz = (zl >> 3) - v.bz0 + 1;
  v.bw = (v.nbz + 63) / 64;
  v.sz0 = v.zb >> 5;
  v.nsz = (zl >> 5) - v.sz0 + 1;
  v.sw = (v.nsz + 31) / 32;
  v.stx = (v.tiles_x + 3) / 4;
  v.sty = (v.tiles_y + 3) / 4;
  for (int i = 0; i < 3; ++i) {
    v.vs[i] = p.volu_range[i] / (float)p.volu_dims[i];  // tsdf_volume.cpp:16
    v.range[i] = p.volu_range[i];
  }
  v.trunc = p.volu_trun_dist;
  v.inv_trunc = 1.f / v.trunc;
  return v;
}

int do_reset(kfx_ctx *c) {
  const size_t n = nvox(c);
  HIPCHK(hipMemsetAsync(c->vol.tsdf, 0, n * sizeof(int16_t), c->stream));
  HIPCHK(hipMemsetAsync(c->vol.weight, 0, n * sizeof(uint8_t), c->stream));
  HIPCHK(hipMemsetAsync(c->vol.rgb, 0, n * sizeof(uint32_t), c->stream));
  HIPCHK(hipMemsetAsync(c->vol.bocc, 0, c->vol.bocc_bytes(), c->stream));
  HIPCHK(hipMemsetAsync(c->vol.socc, 0, c->vol.socc_bytes(), c->stream));
  for (int l = 0; l < c->L; ++l) {
    const size_t np = (size_t)c->g[l].w * c->g[l].h;
    for (FrameView *f : {&c->curb[0], &c->curb[1], &c->prev}) {
      if (f->d[l]) HIPCHK(hipMemsetAsync(f->d[l], 0, np * 4, c->stream));
      HIPCHK(hipMemsetAsync(f->v[l], 0, np * 12, c->stream));
      HIPCHK(hipMemsetAsync(f->n[l], 0, np * 12, c->stream));
    }
  }
  DevState s{};
  s.frame_count = 1;
  s.mode = MODE_BOOT;
  s.n_poses = 1;
  s.pose_cap = c->pose_cap;
  s.icp_pose = identity_pose();
  s.log = c->pose_log;
  s.back = identity_pose();
  const DevPose I = identity_pose();
  HIPCHK(hipMemcpyAsync(c->st, &s, sizeof(s), hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->pose_log, &I, sizeof(I), hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  set_par(c, 0);
  c->pending = 0;
  c->known_poses = 1;
  c->known_fails = 0;
  return KFX_OK;
}

int check_ctx(kfx_ctx *c) {
  if (!c) return set_err(KFX_ERR_ARG, "null context");
  c->api_seq += 1;
  hipError_t e = hipSetDevice(c->device);
  if (e != hipSuccess) return set_err(KFX_ERR_HIP, std::string("hipSetDevice: ") + hipGetErrorString(e));
  return KFX_OK;
}

}  // namespace

extern "C" {

int kfx_abi_version(void) { return KFX_ABI_VERSION; }
const char *kfx_last_error(void) { return g_err.c_str(); }

int kfx_default_params(kfx_params *p) {
  if (!p) return set_err(KFX_ERR_ARG, "null params");
  std::memset(p, 0, sizeof(*p));
  p->pyramid_height = 3;
  p->bfilter_color_sigma = 10;
  p->bfilter_spatial_sigma = 10;
  p->bfilter_kernel_size = 5;
  p->dfilter_dist = 5.f;
  p->icp_angle_threshold = 30.f;
  p->icp_dist_threshold = 0.015f;
  p->icp_iter_count[0] = 4;
  p->icp_iter_count[1] = 5;
  p->icp_iter_count[2] = 10;
  for (int i = 0; i < 3; ++i) {
    p->volu_dims[i] = 512;
    p->volu_range[i] = 3.f;
  }
  p->volu_trun_dist = 2.1f * p->volu_range[0] / (float)p->volu_dims[0];
  std::memset(&p->volu_pose, 0, sizeof(p->volu_pose));
  p->volu_pose.R[0] = p->volu_pose.R[4] = p->volu_pose.R[8] = 1.f;
  p->volu_pose.t[0] = -p->volu_range[0] / 2;
  p->volu_pose.t[1] = -p->volu_range[1] / 2;
  p->volu_pose.t[2] = 0.5f;
  p->min_pose_move = 0.008f;
  p->tsdf_max_weight = 64;
  return KFX_OK;
}

static int create_impl(const kfx_intrinsics *intr, const kfx_params *params, int device,
                       int rank, int world, bool slab, kfx_ctx **out, const int *cuts = nullptr);

int kfx_create(const kfx_intrinsics *intr, const kfx_params *params, int device, kfx_ctx **out) {
  return create_impl(intr, params, device, 0, 1, false, out);
}

int kfx_create_slab(const kfx_intrinsics *intr, const kfx_params *params, int device, int rank,
                    int world, kfx_ctx **out) {
  if (world < 1 || rank < 0 || rank >= world) return set_err(KFX_ERR_ARG, "bad rank/world");
  if (params && params->volu_dims[2] < 16 * world)
    return set_err(KFX_ERR_ARG, "fewer than 16 slices per slab");
  return create_impl(intr, params, device, rank, world, true, out);
}

int kfx_create_slab_cuts(const kfx_intrinsics *intr, const kfx_params *params, int device, int rank,
                         int world, const int *cuts, kfx_ctx **out) {
  if (world < 1 || rank < 0 || rank >= world || !cuts || !params) return set_err(KFX_ERR_ARG, "bad argument");
  const int Z = params->volu_dims[2];
  if (cuts[0] != 0 || cuts[world] != Z) return set_err(KFX_ERR_ARG, "cuts must run from 0 to Z");
  for (int r = 0; r < world; ++r)
    if (cuts[r + 1] - cuts[r] < 8 || (r > 0 && cuts[r] % 8))
      return set_err(KFX_ERR_ARG, "cuts must be multiples of 8 with >= 8 slices per slab");
  return create_impl(intr, params, device, rank, world, true, out, cuts);
}

// Integrate cost of one slice from kfx_slice_work_parts, in 1/64 voxel-slot
// units: every slot a wave steps through (the occlusion-clipped intervals),
// kCostUpdated / 64 more per updated voxel (its tsdf / weight / colour
// read-modify-write) and kCostSlot / 64 per stored slot (the waves of column
// tiles outside the frustum still start and test their range).  Weights from
// a non-negative least-squares fit of per-slab integrate times of C4 and C5
// (tools/slab_fit.py): per visited slot, an updated voxel
// 0.44-0.61, a stored slot 0-0.05.
constexpr int64_t kCostUpdated = KFX_COST_UPDATED, kCostSlot = KFX_COST_SLOT;
static int64_t slice_cost(int64_t cover, int64_t updated, int64_t slots) {
  return 64 * cover + kCostUpdated * updated + kCostSlot * slots;
}

int kfx_slab_balance(const int64_t *slice_work, int Z, int world, int *cuts) {
  if (!slice_work || !cuts || world < 1 || Z < 8 * world) return set_err(KFX_ERR_ARG, "bad argument");
  // a slab integrates its stored slices (owned + kSlabHalo on each side):
  // choose cuts on multiples of 8 minimising the largest stored-range work
  // (binary search on the bound, greedy longest-prefix feasibility)
  std::vector<int64_t> pre(Z + 1, 0);
  for (int z = 0; z < Z; ++z) pre[z + 1] = pre[z] + std::max<int64_t>(0, slice_work[z]);
  auto load = [&](int a, int b) {  // work of the slab owning [a, b)
    const int lo = world > 1 ? std::max(0, a - kSlabHalo) : 0, hi = world > 1 ? std::min(Z, b + kSlabHalo) : Z;
    return pre[hi] - pre[lo];
  };
  auto plan = [&](int64_t bound, std::vector<int> &c) {  // greedy; true if world slabs suffice
    c.assign(1, 0);
    int a = 0;
    for (int r = 0; r < world; ++r) {
      if (r == world - 1) {
        c.push_back(Z);
        return load(a, Z) <= bound && Z - a >= 8;
      }
      // longest end b (multiple of 8, leaving >= 8 slices per later slab) within the bound
      const int bmax = Z - 8 * (world - 1 - r);
      int b = a + 8;
      if (load(a, b) > bound) return false;
      while (b + 8 <= bmax && load(a, b + 8) <= bound) b += 8;
      c.push_back(b);
      a = b;
    }
    return false;
  };
  int64_t lo = 0, hi = pre[Z] + 1;
  std::vector<int> best, c;
  while (lo < hi) {
    const int64_t mid = lo + (hi - lo) / 2;
    if (plan(mid, c)) {
      hi = mid;
      best = c;
    } else {
      lo = mid + 1;
    }
  }
  if (best.empty() && !plan(lo, best)) return set_err(KFX_ERR_STATE, "no feasible cuts");
  for (int r = 0; r <= world; ++r) cuts[r] = best[r];
  return KFX_OK;
}

static int create_impl(const kfx_intrinsics *intr, const kfx_params *params, int device,
                       int rank, int world, bool slab, kfx_ctx **out, const int *cuts) {
  if (!intr || !params || !out) return set_err(KFX_ERR_ARG, "null argument");
  *out = nullptr;
  const kfx_params &p = *params;
  if (p.pyramid_height < 1 || p.pyramid_height > KFX_MAX_LEVELS)
    return set_err(KFX_ERR_ARG, "pyramid_height must be 1..4");
  const int div = 1 << (p.pyramid_height - 1);
  if (intr->width <= 0 || intr->height <= 0 || intr->width % (2 * div) || intr->height % (2 * div))
    return set_err(KFX_ERR_ARG, "width/height must be positive multiples of 2^pyramid_height");
  for (int i = 0; i < 3; ++i)
    if (p.volu_dims[i] < 8 || p.volu_range[i] <= 0.f)
      return set_err(KFX_ERR_ARG, "volume dims must be >= 8 and range > 0");
  if (p.volu_dims[0] % 8 || p.volu_dims[1] % 8)
    return set_err(KFX_ERR_ARG, "volume dims x,y must be multiples of 8 (8x8 slice tiles)");
  // keeps every in-block ICP fixed-point sum an integer below 2^53 (exact fp64
  // accumulation in k_icp_acc): |point| stays below ~45 m
  if (!(p.dfilter_dist > 0.f && p.dfilter_dist <= 30.f))
    return set_err(KFX_ERR_ARG, "dfilter_dist must be in (0, 30] m");
  if (p.bfilter_kernel_size < 1 || p.bfilter_kernel_size > 15)
    return set_err(KFX_ERR_ARG, "bfilter_kernel_size must be 1..15");
  for (int l = 0; l < p.pyramid_height; ++l)
    if ((intr->width >> l) <= p.bfilter_kernel_size / 2 || (intr->height >> l) <= p.bfilter_kernel_size / 2)
      return set_err(KFX_ERR_ARG, "pyramid level smaller than the bilateral radius");
  for (int l = 0; l < p.pyramid_height; ++l)
    if (p.icp_iter_count[l] < 0) return set_err(KFX_ERR_ARG, "negative icp_iter_count");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return set_err(KFX_ERR_NO_DEVICE, "no HIP device");
  if (device < 0 || device >= ndev) return set_err(KFX_ERR_ARG, "bad device ordinal");

  kfx_ctx *c = new kfx_ctx();
  c->device = device;
  c->slab = slab;
  c->rank = rank;
  c->world = world;
  c->intr = *intr;
  c->p = p;
  c->L = p.pyramid_height;
  for (int l = 0; l < c->L; ++l) c->g[l] = level_geom(*intr, l);
  c->angle_thr = std::sin(p.icp_angle_threshold * 0.017453293f);  // icp_registration.cpp:5
  int r = KFX_OK;
  auto fail = [&](int code) {
    kfx_destroy(c);
    return code;
  };
  if (hipSetDevice(device) != hipSuccess) return fail(set_err(KFX_ERR_HIP, "hipSetDevice failed"));
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess)
    return fail(set_err(KFX_ERR_HIP, "hipStreamCreate failed"));
  for (auto &e : c->ev)
    if (hipEventCreate(&e) != hipSuccess) return fail(set_err(KFX_ERR_HIP, "hipEventCreate failed"));
  if (hipStreamCreateWithFlags(&c->pstream, hipStreamNonBlocking) != hipSuccess)
    return fail(set_err(KFX_ERR_HIP, "hipStreamCreate failed"));
  // cross-stream ordering on one device: a device-scope release suffices
  for (hipEvent_t *e : {&c->ev_prep, &c->ev_free[0], &c->ev_free[1], &c->ev_icp})
    if (hipEventCreateWithFlags(e, hipEventDisableTiming | hipEventReleaseToDevice) != hipSuccess)
      return fail(set_err(KFX_ERR_HIP, "hipEventCreate failed"));
  // group members may sit on other devices: a system-scope release
  if (hipEventCreateWithFlags(&c->ev_group, hipEventDisableTiming) != hipSuccess)
    return fail(set_err(KFX_ERR_HIP, "hipEventCreate failed"));

  for (int l = 0; l < c->L; ++l) {
    const size_t np = (size_t)c->g[l].w * c->g[l].h;
    if ((r = dalloc(c, (void **)&c->raw[l], np * 4))) return fail(r);
    for (FrameView &f : c->curb) {
      if ((r = dalloc(c, (void **)&f.d[l], np * 4))) return fail(r);
      if ((r = dalloc(c, (void **)&f.v[l], np * 12))) return fail(r);
      if ((r = dalloc(c, (void **)&f.n[l], np * 12))) return fail(r);
    }
    // prev vmap|nmap of a level are one buffer (one collective in the slab combine)
    if ((r = dalloc(c, (void **)&c->prev.v[l], np * 24))) return fail(r);
    c->prev.n[l] = c->prev.v[l] + 3 * np;
  }
  const size_t np0 = (size_t)intr->width * intr->height;
  if (slab) {
    if ((r = dalloc(c, (void **)&c->key_local, np0 * 4 * 6))) return fail(r);  // keys, pend + payload
    if ((r = dalloc(c, (void **)&c->key_min, np0 * 4 * 2))) return fail(r);
  }
  if ((r = dalloc(c, (void **)&c->raw0_u16, np0 * 2))) return fail(r);
  if ((r = dalloc(c, (void **)&c->bgr, np0 * 3))) return fail(r);
  if ((r = dalloc(c, (void **)&c->inv_lambda, np0 * 4))) return fail(r);
  // {depth, 1/lambda} per pixel + 16 max-depth shards + the 16x16-pixel max-depth grid
  const size_t grid16 = (size_t)((intr->width + 15) / 16) * ((intr->height + 15) / 16);
  for (float2 *&d : c->dl0b)
    if ((r = dalloc(c, (void **)&d, np0 * 8 + 64 + grid16 * 4))) return fail(r);
  c->vol = make_vol(p, rank, world, cuts);
  // raycast wave durations of the last frame (4 waves per 16x16 block; zeroed: no hint)
  if ((r = dalloc(c, (void **)&c->vol.rdur, grid16 * 4 * sizeof(unsigned)))) return fail(r);
  const size_t n = nvox(c);
  {
    // tsdf and weight in ONE allocation, weight (u8) at a fixed offset (2 MiB-
    // rounded + 4 KiB): with two allocations the relative physical placement
    // of tsdf[i] and weight[i] (read together by integrate) changed from run
    // to run and integrate took 172-185 us; fixed, 169-172 us
    const size_t off = ((n * 2 + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1)) + KFX_VOL_PAD;
    if ((r = dalloc(c, (void **)&c->vol.tsdf, off + n))) return fail(r);
    c->vol.weight = (uint8_t *)((char *)c->vol.tsdf + off);
  }
  if ((r = dalloc(c, (void **)&c->vol.rgb, n * 4))) return fail(r);
  if ((r = dalloc(c, (void **)&c->vol.bocc, c->vol.bocc_bytes()))) return fail(r);
  if ((r = dalloc(c, (void **)&c->vol.socc, c->vol.socc_bytes()))) return fail(r);
  {  // integrate dispatch order: identity until the first integrate has measured the intervals
    const size_t tiles = (size_t)c->vol.tiles_x * c->vol.tiles_y, items = tiles * integrate_chunks(c->vol);
    if ((r = dalloc(c, (void **)&c->vol.iwork, tiles * 4))) return fail(r);
    if ((r = dalloc(c, (void **)&c->vol.iperm, items * 4))) return fail(r);
    std::vector<unsigned> iota(items);
    for (size_t i = 0; i < items; ++i) iota[i] = (unsigned)i;
    HIPCHK(hipMemcpy(c->vol.iperm, iota.data(), items * 4, hipMemcpyHostToDevice));
  }
  {
    // the raycast start signal (KFX_PREP_SIG) needs hipStreamWaitValue32; it
    // is off under rocprofv3 counter collection (ROCPROF_COUNTER_COLLECTION),
    // whose per-dispatch serialisation hung on the waiting preprocess queue,
    // and with KFX_STREAM_SIGNAL=0 (events instead; results identical)
    const char *pmc = std::getenv("ROCPROF_COUNTER_COLLECTION"), *ss = std::getenv("KFX_STREAM_SIGNAL");
    const bool sig_ok = !(pmc && *pmc && std::strcmp(pmc, "0") != 0) && !(ss && std::strcmp(ss, "0") == 0);
    int can_wait = 0;
    if (sig_ok && hipDeviceGetAttribute(&can_wait, hipDeviceAttributeCanUseStreamWaitValue, device) == hipSuccess && can_wait &&
        hipExtMallocWithFlags((void **)&c->start_sig, 64, hipDeviceMallocFinegrained) == hipSuccess) {
      c->allocs.push_back(c->start_sig);
      HIPCHK(hipMemset(c->start_sig, 0, 64));
    } else {
      (void)hipGetLastError();
      c->start_sig = nullptr;
    }
  }
  if ((r = dalloc(c, (void **)&c->st, sizeof(DevState)))) return fail(r);
  c->pose_cap = kInitialPoseCap;
  if ((r = dalloc(c, (void **)&c->pose_log, sizeof(DevPose) * (size_t)c->pose_cap))) return fail(r);
  if ((r = dalloc(c, (void **)&c->icp_shards, sizeof(unsigned long long) * kIcpShards * 27 + 64)))
    return fail(r);
  c->icp_ticket = reinterpret_cast<unsigned *>(c->icp_shards + kIcpShards * 27);
  if ((r = dalloc(c, (void **)&c->icp_sync, sizeof(IcpSync)))) return fail(r);
  for (int b = 0; b < 2; ++b)
    c->planb[b] = make_icp_plan(c->L, c->g, c->p.icp_iter_count, c->curb[b], c->prev,
                                c->p.icp_dist_threshold, c->angle_thr);
  for (int b = 0; b < 2; ++b) c->planb[b].vpose = to_dev(c->p.volu_pose);
  // (both sets: the fit may cap nblocks and select the strided kernel)
  c->icp_persistent = icp_persistent_ok(c->planb[0], c->device) && icp_persistent_ok(c->planb[1], c->device);
  // The side streams' waits on the raycast start signal run as small spinning
  // kernels, which may be resident while the next frame's persistent ICP
  // starts: keep the signal only when the ICP grid leaves two CUs of headroom
  // (a 720p frame's strided plan fills the GPU: its grid was then not
  // co-resident and the watchdog fired), else the event path
  if (c->start_sig && c->icp_persistent &&
      !(icp_headroom(c->planb[0], c->device, 2) && icp_headroom(c->planb[1], c->device, 2)))
    c->start_sig = nullptr;  // (the word stays in allocs)
  set_par(c, 0);
  if ((r = dalloc(c, (void **)&c->counters, sizeof(unsigned long long) * 128))) return fail(r);
  if ((r = dalloc(c, (void **)&c->xpose, sizeof(float) * 32))) return fail(r);
  launch_inv_lambda(c->stream, c->g[0], c->inv_lambda);
  if ((r = do_reset(c))) return fail(r);
  *out = c;
  return KFX_OK;
}

int kfx_destroy(kfx_ctx *c) {
  if (!c) return KFX_OK;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->pstream) (void)hipStreamSynchronize(c->pstream);
  if (c->cstream) (void)hipStreamSynchronize(c->cstream);
  destroy_graphs(c);
  if (c->ring_host) (void)hipHostFree(c->ring_host);
  for (const auto &r : c->host_regs) (void)hipHostUnregister(reinterpret_cast<void *>(r.host));
  for (int k = 0; k < kfx_ctx::kRing; ++k)
    for (hipEvent_t e : {c->ring_h2d[k], c->ring_done[k]})
      if (e) (void)hipEventDestroy(e);
  if (c->cstream) (void)hipStreamDestroy(c->cstream);
  if (c->comm) (void)ncclCommDestroy(c->comm);
  for (void *a : c->allocs) (void)hipFree(a);
  for (auto &e : c->ev)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : {c->ev_prep, c->ev_free[0], c->ev_free[1], c->ev_icp, c->ev_group})
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : c->tsets) (void)hipEventDestroy(e);
  for (hipEvent_t e : c->xev)
    if (e) (void)hipEventDestroy(e);
  if (c->pstream) (void)hipStreamDestroy(c->pstream);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  // the teardown's errors (e.g. a buffer another context unregistered first)
  // must not surface in a later call's hipGetLastError check
  (void)hipGetLastError();
  return KFX_OK;
}

int kfx_reset(kfx_ctx *c) {
  int r = check_ctx(c);
  if (r) return r;
  if (c->cstream) HIPCHK(hipStreamSynchronize(c->cstream));
  HIPCHK(hipStreamSynchronize(c->pstream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return do_reset(c);
}

int kfx_pipeline(kfx_ctx *c, const uint8_t *bgr, const float *depth_mm) {
  int r = check_ctx(c);
  if (r) return r;
  if (!bgr || !depth_mm) return set_err(KFX_ERR_ARG, "null image");
  const size_t np = (size_t)c->intr.width * c->intr.height;
  HIPCHK(hipMemcpyAsync(c->raw[0], depth_mm, np * 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->bgr, bgr, np * 3, hipMemcpyHostToDevice, c->stream));
  if ((r = run_frame(c, {c->raw[0], nullptr, c->bgr}, &c->graph[0]))) return r;
  return finish_frame(c);
}

int kfx_pipeline_u16(kfx_ctx *c, const uint8_t *bgr, const uint16_t *depth_mm) {
  int r = check_ctx(c);
  if (r) return r;
  if (!bgr || !depth_mm) return set_err(KFX_ERR_ARG, "null image");
  const size_t np = (size_t)c->intr.width * c->intr.height;
  HIPCHK(hipMemcpyAsync(c->raw0_u16, depth_mm, np * 2, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->bgr, bgr, np * 3, hipMemcpyHostToDevice, c->stream));
  if ((r = run_frame(c, {c->raw[0], c->raw0_u16, c->bgr}, &c->graph[1]))) return r;
  return finish_frame(c);
}

// The device address of [p, p + n) when it lies inside one buffer registered
// with kfx_register_host_buffer, else null
static const uint8_t *host_mapped(const kfx_ctx *c, const void *p, size_t n) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  for (const auto &r : c->host_regs)
    if (a >= r.host && a + n <= r.host + r.bytes) return r.dev + (a - r.host);
  return nullptr;
}

int kfx_register_host_buffer(kfx_ctx *c, void *ptr, size_t bytes) {
  int r = check_ctx(c);
  if (r) return r;
  if (!ptr || !bytes) return set_err(KFX_ERR_ARG, "null or empty buffer");
  HIPCHK(hipHostRegister(ptr, bytes, hipHostRegisterMapped));
  void *dev = nullptr;
  const hipError_t e = hipHostGetDevicePointer(&dev, ptr, 0);
  if (e != hipSuccess || !dev) {
    (void)hipHostUnregister(ptr);
    return set_err(KFX_ERR_HIP, std::string("hipHostGetDevicePointer: ") + hipGetErrorString(e));
  }
  c->host_regs.push_back({reinterpret_cast<uintptr_t>(ptr), bytes, static_cast<uint8_t *>(dev)});
  return KFX_OK;
}

int kfx_unregister_host_buffer(kfx_ctx *c, void *ptr) {
  int r = check_ctx(c);
  if (r) return r;
  const uintptr_t a = reinterpret_cast<uintptr_t>(ptr);
  for (size_t i = 0; i < c->host_regs.size(); ++i)
    if (c->host_regs[i].host == a) {
      // uploads from it may still be queued
      if (c->cstream) HIPCHK(hipStreamSynchronize(c->cstream));
      HIPCHK(hipHostUnregister(ptr));
      c->host_regs.erase(c->host_regs.begin() + (long)i);
      return KFX_OK;
    }
  return set_err(KFX_ERR_ARG, "buffer not registered");
}

static int pipeline_async(kfx_ctx *c, const uint8_t *bgr, const void *depth, bool u16) {
  int r = check_ctx(c);
  if (r) return r;
  if (!bgr || !depth) return set_err(KFX_ERR_ARG, "null image");
  const size_t np = (size_t)c->intr.width * c->intr.height;
  if (!c->ring_ready) {  // first use: pinned + device rings, copy stream, events
    // (each resource is created once; a failure leaves ring_ready false and
    // the next call creates only what is still missing)
    c->ring_slot = (np * 4 + np * 3 + 255) & ~(size_t)255;
    if (!c->ring_host)
      HIPCHK(hipHostMalloc((void **)&c->ring_host, c->ring_slot * kfx_ctx::kRing, hipHostMallocMapped));
    if (!c->ring_host_dev) HIPCHK(hipHostGetDevicePointer((void **)&c->ring_host_dev, c->ring_host, 0));
    if (!c->ring_dev && (r = dalloc(c, (void **)&c->ring_dev, c->ring_slot * kfx_ctx::kRing))) return r;
    if (!c->cstream) {  // the lowest priority: the frame kernels are dispatched ahead of the uploads
      int lo = 0, hi = 0;
      HIPCHK(hipDeviceGetStreamPriorityRange(&lo, &hi));
      HIPCHK(hipStreamCreateWithPriority(&c->cstream, hipStreamNonBlocking, lo));
    }
    for (int k = 0; k < kfx_ctx::kRing; ++k) {
      if (!c->ring_h2d[k]) HIPCHK(hipEventCreateWithFlags(&c->ring_h2d[k], hipEventDisableTiming));
      if (!c->ring_done[k]) HIPCHK(hipEventCreateWithFlags(&c->ring_done[k], hipEventDisableTiming));
    }
    c->ring_ready = true;
  }
  const int k = c->ring_next;
  c->ring_next = (k + 1) % kfx_ctx::kRing;
  uint8_t *hs = c->ring_host + c->ring_slot * k, *ds = c->ring_dev + c->ring_slot * k;
  const size_t dbytes = np * (u16 ? 2 : 4);
  // zero copy: frames in buffers registered with kfx_register_host_buffer are
  // read by the GPU straight from the caller's pinned pages (no host copy, no
  // host wait); others are copied into the pinned ring slot first.  Either way
  // the upload is a kernel on the copy stream reading mapped host memory
  // (k_host_fetch), not hipMemcpyAsync, whose host-side cost per call was the
  // bottleneck of this path
  const uint8_t *map_d = host_mapped(c, depth, dbytes), *map_c = host_mapped(c, bgr, np * 3);
  const bool direct = map_d && map_c;
  if (!direct) {
    if (c->ring_used[k]) HIPCHK(hipEventSynchronize(c->ring_h2d[k]));  // the slot's last upload is done
    std::memcpy(hs, depth, dbytes);
    std::memcpy(hs + np * 4, bgr, np * 3);
    map_d = c->ring_host_dev + c->ring_slot * k;
    map_c = map_d + np * 4;
  }
  // the device slot is free once the frame that read it has finished (its
  // preprocess and integrate: its raycast has started, when it signals that)
  if (c->ring_used[k]) {
    if (c->ring_sig[k])
      HIPCHK(hipStreamWaitValue32(c->cstream, c->start_sig, c->ring_sig[k], hipStreamWaitValueGte, 0xffffffffu));
    else
      HIPCHK(hipStreamWaitEvent(c->cstream, c->ring_done[k], 0));
  }
  launch_host_fetch(c->cstream, map_d, ds, dbytes, map_c, ds + np * 4, np * 3);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(c->ring_h2d[k], c->cstream));
  c->ring_used[k] = true;
  FrameInput in{u16 ? c->raw[0] : (const float *)ds, u16 ? (const uint16_t *)ds : nullptr, ds + np * 4};
  in.ready = c->ring_h2d[k];
  in.done = c->ring_done[k];
  c->ring_sig[k] = 0u;
  r = run_frame(c, in, nullptr, true, c->ring_graph[k][u16 ? 1 : 0]);
  if (!r) c->ring_sig[k] = c->frame_sig;
  return r;
}

int kfx_pipeline_async(kfx_ctx *c, const uint8_t *bgr, const float *depth_mm) {
  return pipeline_async(c, bgr, depth_mm, false);
}

int kfx_pipeline_async_u16(kfx_ctx *c, const uint8_t *bgr, const uint16_t *depth_mm) {
  return pipeline_async(c, bgr, depth_mm, true);
}

int kfx_stage_frames(kfx_ctx *c, int n, const uint8_t *bgr, const float *depth_mm) {
  int r = check_ctx(c);
  if (r) return r;
  if (n <= 0 || !bgr || !depth_mm) return set_err(KFX_ERR_ARG, "bad staged frames");
  HIPCHK(hipStreamSynchronize(c->stream));
  const size_t np = (size_t)c->intr.width * c->intr.height;
  for (void *pp : {(void *)c->staged_depth, (void *)c->staged_bgr}) {
    if (!pp) continue;
    c->allocs.erase(std::remove(c->allocs.begin(), c->allocs.end(), pp), c->allocs.end());
    (void)hipFree(pp);
  }
  c->staged_depth = nullptr;
  c->staged_bgr = nullptr;
  c->n_staged = 0;
  destroy_graphs(c);
  c->staged_graph.assign(n, nullptr);
  c->ov_graph.assign(4 * (size_t)n, nullptr);
  if ((r = dalloc(c, (void **)&c->staged_depth, np * 4 * (size_t)n))) return r;
  if ((r = dalloc(c, (void **)&c->staged_bgr, np * 3 * (size_t)n))) return r;
  HIPCHK(hipMemcpyAsync(c->staged_depth, depth_mm, np * 4 * (size_t)n, hipMemcpyHostToDevice,
                        c->stream));
  HIPCHK(hipMemcpyAsync(c->staged_bgr, bgr, np * 3 * (size_t)n, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  c->n_staged = n;
  // capture every staged frame's graphs now, outside any timed frame loop
  // (overlapped frames: two per buffer set)
  for (int i = 0; i < n; ++i) {
    const FrameInput in{c->staged_depth + np * i, nullptr, c->staged_bgr + np * 3 * i};
    if (!c->overlap) r = ensure_graph(c, in, &c->staged_graph[i]);
    else if (ov_graphs_apply(c))
      for (int p = 0; p < 2 && !r; ++p) r = ensure_ov_graphs(c, in, &c->ov_graph[4 * i + 2 * p], p);
    if (r) return r;
  }
  return KFX_OK;
}

int kfx_pipeline_staged(kfx_ctx *c, int idx) {
  int r = check_ctx(c);
  if (r) return r;
  if (idx < 0 || idx >= c->n_staged) return set_err(KFX_ERR_ARG, "staged frame index out of range");
  const size_t np = (size_t)c->intr.width * c->intr.height;
  // the captured graph for this staged frame reads it in place (no copy)
  return run_frame(c, {c->staged_depth + np * idx, nullptr, c->staged_bgr + np * 3 * idx},
                   &c->staged_graph[idx], true, &c->ov_graph[4 * (size_t)idx]);
}

int kfx_synchronize(kfx_ctx *c) {
  int r = check_ctx(c);
  if (r) return r;
  HIPCHK(hipStreamSynchronize(c->pstream));
  if (c->cstream) HIPCHK(hipStreamSynchronize(c->cstream));
  DevState s;
  if ((r = read_state(c, &s))) return r;  // also waits for the frame stream
  return check_status(c, s);
}

int kfx_set_frame_overlap(kfx_ctx *c, int enabled) {
  int r = check_ctx(c);
  if (r) return r;
  HIPCHK(hipStreamSynchronize(c->stream));
  c->overlap = enabled != 0;
  return KFX_OK;
}

int kfx_set_kernel_timing(kfx_ctx *c, int every, int max_samples) {
  int r = check_ctx(c);
  if (r) return r;
  if (every < 0 || max_samples < 0) return set_err(KFX_ERR_ARG, "negative timing argument");
  HIPCHK(hipStreamSynchronize(c->stream));
  // (the extraction events c->xev are not timing samples: they stay)
  for (hipEvent_t e : c->tsets) (void)hipEventDestroy(e);
  c->tsets.clear();
  c->ext_pending = nullptr;  // pointed into tsets (kfx_slab_frame_local)
  c->tnext = 0;
  c->frame_seq = 0;
  c->timing_every = every;
  if (every == 0) return KFX_OK;
  c->tsets.assign(kStageEvents * (size_t)max_samples, nullptr);
  // timing-only events: no system-scope fence on record (a fence per event
  // cost ~6 us of GPU time each)
  for (hipEvent_t &e : c->tsets) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
  return KFX_OK;
}

int kfx_get_kernel_timing_ex(kfx_ctx *c, float out_ms[4], int *n_samples) {
  int r = check_ctx(c);
  if (r) return r;
  if (!out_ms) return set_err(KFX_ERR_ARG, "null out");
  HIPCHK(hipStreamSynchronize(c->stream));
  // sample events: [2] ICP done, [3] integrate done, [5] local raycast done,
  // [6] combine starts (group members: after the other members' local phases),
  // [4] frame done; [1] the frame's tracking starts
  // [7]..[8] the shared part of a group combine (elapsed 0 elsewhere), added
  // to the member's own combine [6]..[4]
  // (a single volume records [1], [2], [3], [5] only: every event record in
  // a sampled frame costs the run time)
  static const int kFrom[5] = {1, 2, 3, 6, 7}, kTo[5] = {2, 3, 5, 4, 8};
  const int pairs = c->slab ? 5 : 3;
  double acc[4] = {0, 0, 0, 0};
  for (size_t k = 0; k < c->tnext; ++k) {
    for (int i = 0; i < pairs; ++i) {
      float ms = 0.f;
      HIPCHK(hipEventElapsedTime(&ms, c->tsets[kStageEvents * k + kFrom[i]], c->tsets[kStageEvents * k + kTo[i]]));
      acc[i < 4 ? i : 3] += ms;
    }
  }
  for (int i = 0; i < 4; ++i) out_ms[i] = c->tnext ? (float)(acc[i] / (double)c->tnext) : 0.f;

  if (n_samples) *n_samples = (int)c->tnext;
  c->tnext = 0;
  return KFX_OK;
}

int kfx_get_kernel_timing(kfx_ctx *c, float out_ms[3], int *n_samples) {
  if (!out_ms) return set_err(KFX_ERR_ARG, "null out");
  float m[4];
  const int r = kfx_get_kernel_timing_ex(c, m, n_samples);
  if (r) return r;
  out_ms[0] = m[0];
  out_ms[1] = m[1];
  out_ms[2] = m[2] + m[3];
  return KFX_OK;
}

int kfx_set_graph_mode(kfx_ctx *c, int enabled) {
  if (!c) return set_err(KFX_ERR_ARG, "null context");
  if (enabled < 0 || enabled > 2) return set_err(KFX_ERR_ARG, "graph mode is 0, 1 or 2");
  c->graph_mode = enabled != 0;
  if (c->ov_graph_full != (enabled == 2)) {
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipStreamSynchronize(c->pstream));
    destroy_graphs(c);
    c->ov_graph_full = enabled == 2;
    c->ov_main_refused = false;
  }
  return KFX_OK;
}

int kfx_get_graph_mode(kfx_ctx *c, int *mode) {
  if (!c || !mode) return set_err(KFX_ERR_ARG, "null argument");
  *mode = !c->graph_mode ? 0 : (c->ov_graph_full && !c->ov_main_refused ? 2 : 1);
  return KFX_OK;
}

const char *kfx_get_graph_note(kfx_ctx *c) {
  return c ? c->graph_note.c_str() : "";
}

int kfx_set_icp_persistent(kfx_ctx *c, int enabled) {
  int r = check_ctx(c);
  if (r) return r;
  if (enabled < 0 || enabled > 2) return set_err(KFX_ERR_ARG, "icp persistent mode must be 0, 1 or 2");
  HIPCHK(hipStreamSynchronize(c->stream));
  const bool on = enabled != 0, coop = enabled == 2;
  if (c->icp_persistent_enabled != on || (on && c->icp_coop != coop)) destroy_graphs(c);
  c->icp_persistent_enabled = on;
  if (on) c->icp_coop = coop;
  return c->icp_persistent ? 1 : 0;
}

int kfx_debug_force_icp_stall(kfx_ctx *c) {
  int r = check_ctx(c);
  if (r) return r;
  HIPCHK(hipStreamSynchronize(c->stream));
  return write_field(c, offsetof(DevState, debug_stall), 1);
}

int kfx_debug_icp_band_ms(kfx_ctx *c, int rank, int world, int reps, float *ms) {
  int r = check_ctx(c);
  if (r) return r;
  if (!ms || world < 1 || rank < 0 || rank >= world || reps < 1) return set_err(KFX_ERR_ARG, "band rank/world/reps");
  HIPCHK(hipStreamSynchronize(c->pstream));
  HIPCHK(hipStreamSynchronize(c->stream));
  DevState saved;
  HIPCHK(hipMemcpy(&saved, c->st, sizeof(DevState), hipMemcpyDeviceToHost));
  DevState run = saved;
  run.mode = MODE_TRACK;  // (a bootstrap state would make every launch return at once)
  run.icp_fail = 0;
  hipEvent_t e[2] = {nullptr, nullptr};
  HIPCHK(hipEventCreate(&e[0]));
  HIPCHK(hipEventCreate(&e[1]));
  double total = 0.0;
  hipError_t err = hipSuccess;
  for (int k = 0; k < reps && err == hipSuccess; ++k) {
    err = hipMemcpy(c->st, &run, sizeof(DevState), hipMemcpyHostToDevice);
    if (err == hipSuccess) err = hipEventRecord(e[0], c->stream);
    for (int level = c->L - 1; level >= 0 && err == hipSuccess; --level)
      for (int it = 0; it < c->p.icp_iter_count[level]; ++it) {
        launch_icp(c->stream, c->g[level], c->cur.v[level], c->cur.n[level], c->prev.v[level], c->prev.n[level],
                   c->p.icp_dist_threshold, c->angle_thr, c->st, c->icp_shards, c->icp_ticket, 0, 0, rank, world);
        launch_icp_solve(c->stream, c->st);
      }
    if (err == hipSuccess) err = hipEventRecord(e[1], c->stream);
    if (err == hipSuccess) err = hipEventSynchronize(e[1]);
    float t = 0.f;
    if (err == hipSuccess) err = hipEventElapsedTime(&t, e[0], e[1]);
    total += t;
  }
  (void)hipEventDestroy(e[0]);
  (void)hipEventDestroy(e[1]);
  const hipError_t err2 = hipMemcpy(c->st, &saved, sizeof(DevState), hipMemcpyHostToDevice);
  if (err != hipSuccess || err2 != hipSuccess)
    return set_err(KFX_ERR_HIP, std::string("icp band timing: ") + hipGetErrorString(err != hipSuccess ? err : err2));
  *ms = (float)(total / reps);
  return KFX_OK;
}

int kfx_debug_force_index64(kfx_ctx *c, int on) {
  int r = check_ctx(c);
  if (r) return r;
  if ((c->vol.force64 != 0) != (on != 0)) {  // captured frames hold the other kernels
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipStreamSynchronize(c->pstream));
    destroy_graphs(c);
  }
  c->vol.force64 = on != 0;
  return KFX_OK;
}

int kfx_set_icp_allreduce(kfx_ctx *c, int enabled) {
  if (!c) return set_err(KFX_ERR_ARG, "null context");
  if (!c->slab) return set_err(KFX_ERR_STATE, "ICP partial all-reduce needs a slab context");
  if (c->icp_sharded != (enabled != 0)) destroy_graphs(c);
  c->icp_sharded = enabled != 0;
  return KFX_OK;
}

int kfx_get_icp_trace(kfx_ctx *c, uint64_t *out, int max_iters) {
  int r = check_ctx(c);
  if (r) return r;
  if (!out || max_iters < 0) return set_err(KFX_ERR_ARG, "null argument");
#ifdef KFX_ICP_TRACE
  const int n = std::min(max_iters, c->icp_plan.slots);
  HIPCHK(hipStreamSynchronize(c->stream));
  HIPCHK(hipMemcpy(out, c->icp_sync->trace, sizeof(uint64_t) * 12 * (size_t)n, hipMemcpyDeviceToHost));
  return n;
#else
  return 0;  // stamps exist in trace builds only (-DKFX_ICP_TRACE, tools/variants.sh)
#endif
}

int kfx_set_profiling(kfx_ctx *c, int enabled) {
  if (!c) return set_err(KFX_ERR_ARG, "null context");
  c->profiling = enabled != 0;
  return KFX_OK;
}

int kfx_get_stage_ms(kfx_ctx *c, float out[5]) {
  if (!c || !out) return set_err(KFX_ERR_ARG, "null argument");
  std::memcpy(out, c->stage_ms, sizeof(c->stage_ms));
  return KFX_OK;
}

int kfx_get_cur_camera_pose(kfx_ctx *c, kfx_pose *out) {
  int r = check_ctx(c);
  if (r) return r;
  if (!out) return set_err(KFX_ERR_ARG, "null pose");
  DevState s;
  if ((r = read_state(c, &s))) return r;
  DevPose d;
  HIPCHK(hipMemcpyAsync(&d, c->pose_log + (s.n_poses - 1), sizeof(d), hipMemcpyDeviceToHost,
                        c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  *out = to_api(d);
  return KFX_OK;
}

int kfx_get_frame_count(kfx_ctx *c, int *out) {
  int r = check_ctx(c);
  if (r) return r;
  if (!out) return set_err(KFX_ERR_ARG, "null out");
  DevState s;
  if ((r = read_state(c, &s))) return r;
  *out = s.frame_count;
  return KFX_OK;
}

int kfx_get_pose_record(kfx_ctx *c, kfx_pose *out, int cap, int *n) {
  int r = check_ctx(c);
  if (r) return r;
  if (!n) return set_err(KFX_ERR_ARG, "null n");
  DevState s;
  if ((r = read_state(c, &s))) return r;
  *n = s.n_poses;
  const int m = std::min(cap, s.n_poses);
  if (out && m > 0) {
    std::vector<DevPose> tmp(m);
    HIPCHK(hipMemcpyAsync(tmp.data(), c->pose_log, sizeof(DevPose) * m, hipMemcpyDeviceToHost,
                          c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    for (int i = 0; i < m; ++i) out[i] = to_api(tmp[i]);
  }
  return s.pose_overflow ? set_err(KFX_ERR_STATE, "pose log overflow") : KFX_OK;
}

int kfx_write_poses_txt(kfx_ctx *c, const char *path) {
  int n = 0;
  int r = kfx_get_pose_record(c, nullptr, 0, &n);
  if (r) return r;
  std::vector<kfx_pose> ps(n);
  if ((r = kfx_get_pose_record(c, ps.data(), n, &n))) return r;
  FILE *f = std::fopen(path, "w");
  if (!f) return set_err(KFX_ERR_ARG, std::string("cannot open ") + path);
  for (const kfx_pose &p : ps)  // main.cpp:96-97: outfile << matrix << std::endl
    std::fprintf(f,
                 "[%.8g, %.8g, %.8g, %.8g;\n %.8g, %.8g, %.8g, %.8g;\n %.8g, %.8g, %.8g, %.8g;\n "
                 "0, 0, 0, 1]\n",
                 p.R[0], p.R[1], p.R[2], p.t[0], p.R[3], p.R[4], p.R[5], p.t[1], p.R[6], p.R[7],
                 p.R[8], p.t[2]);
  std::fclose(f);
  return KFX_OK;
}

int kfx_get_frame_maps(kfx_ctx *c, int which, int level, float *dmap, float *vmap, float *nmap) {
  int r = check_ctx(c);
  if (r) return r;
  if (level < 0 || level >= c->L || (which != KFX_FRAME_CUR && which != KFX_FRAME_PREV))
    return set_err(KFX_ERR_ARG, "bad frame/level");
  HIPCHK(hipStreamSynchronize(c->stream));
  const FrameView &f = which == KFX_FRAME_CUR ? c->cur : c->prev;
  const size_t np = (size_t)c->g[level].w * c->g[level].h;
  if (dmap) {
    if (which == KFX_FRAME_CUR)
      HIPCHK(hipMemcpyAsync(dmap, f.d[level], np * 4, hipMemcpyDeviceToHost, c->stream));
    else
      std::memset(dmap, 0, np * 4);
  }
  if (vmap) HIPCHK(hipMemcpyAsync(vmap, f.v[level], np * 12, hipMemcpyDeviceToHost, c->stream));
  if (nmap) HIPCHK(hipMemcpyAsync(nmap, f.n[level], np * 12, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return KFX_OK;
}

int kfx_set_frame_maps(kfx_ctx *c, int which, int level, const float *vmap, const float *nmap) {
  int r = check_ctx(c);
  if (r) return r;
  if (level < 0 || level >= c->L || (which != KFX_FRAME_CUR && which != KFX_FRAME_PREV))
    return set_err(KFX_ERR_ARG, "bad frame/level");
  HIPCHK(hipStreamSynchronize(c->stream));
  const FrameView &f = which == KFX_FRAME_CUR ? c->cur : c->prev;
  const size_t np = (size_t)c->g[level].w * c->g[level].h;
  if (vmap) HIPCHK(hipMemcpyAsync(f.v[level], vmap, np * 12, hipMemcpyHostToDevice, c->stream));
  if (nmap) HIPCHK(hipMemcpyAsync(f.n[level], nmap, np * 12, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return KFX_OK;
}

static int slab_z(const kfx_ctx *c, size_t bytes_per_voxel) {
  const size_t budget = 64u << 20;
  size_t nz = budget / (c->vol.slice * bytes_per_voxel);
  if (nz < 1) nz = 1;
  if (nz > (size_t)c->vol.Z) nz = c->vol.Z;
  return (int)nz;
}

int kfx_download_tsdf(kfx_ctx *c, void *dst) {
  int r = check_ctx(c);
  if (r) return r;
  if (!dst) return set_err(KFX_ERR_ARG, "null dst");
  const int nz = slab_z(c, 8);
  uint64_t *tmp = nullptr;
  HIPCHK(hipMalloc(&tmp, c->vol.slice * 8 * (size_t)nz));
  for (int z0 = c->vol.own0; z0 < c->vol.own1; z0 += nz) {  // owned slices only
    const int k = std::min(nz, c->vol.own1 - z0);
    launch_export_records(c->stream, c->vol, z0, k, tmp);
    hipError_t e = hipMemcpyAsync((char *)dst + c->vol.slice * 8 * (size_t)z0, tmp,
                                  c->vol.slice * 8 * (size_t)k, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) {
      (void)hipFree(tmp);
      return set_err(KFX_ERR_HIP, std::string("download_tsdf: ") + hipGetErrorString(e));
    }
  }
  HIPCHK(hipFree(tmp));
  return KFX_OK;
}

int kfx_upload_tsdf(kfx_ctx *c, const void *src) {
  int r = check_ctx(c);
  if (r) return r;
  if (!src) return set_err(KFX_ERR_ARG, "null src");
  // refuse before writing anything: every stored record's weight must fit the
  // u8 weight store, so a refused upload leaves the volume and its raycast
  // skip maps untouched (the reference never holds weights above 64)
  {
    const uint64_t *rec = static_cast<const uint64_t *>(src) + c->vol.slice * (size_t)c->vol.zb;
    const size_t n = c->vol.slice * (size_t)c->vol.zn;
    uint64_t any = 0;
    for (size_t i = 0; i < n; ++i) any |= rec[i] & 0xff000000ull;  // weight bits 24..31 (or its sign)
    if (any) return set_err(KFX_ERR_ARG, "upload_tsdf: a weight outside 0..255 (u8 weight store; the reference's are 0..64)");
  }
  HIPCHK(hipStreamSynchronize(c->stream));
  const int nz = slab_z(c, 8);
  uint64_t *tmp = nullptr;
  const size_t tbytes = c->vol.slice * 8 * (size_t)nz;
  HIPCHK(hipMalloc(&tmp, tbytes + 64));
  unsigned *bad = reinterpret_cast<unsigned *>((char *)tmp + tbytes);  // weight outside 0..255
  HIPCHK(hipMemsetAsync(bad, 0, 4, c->stream));
  const int zend = c->vol.zb + c->vol.zn;
  for (int z0 = c->vol.zb; z0 < zend; z0 += nz) {  // stored slices, halo included
    const int k = std::min(nz, zend - z0);
    hipError_t e = hipMemcpyAsync(tmp, (const char *)src + c->vol.slice * 8 * (size_t)z0,
                                  c->vol.slice * 8 * (size_t)k, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) {
      launch_import_records(c->stream, c->vol, z0, k, tmp, bad);
      e = hipStreamSynchronize(c->stream);
    }
    if (e != hipSuccess) {
      (void)hipFree(tmp);
      return set_err(KFX_ERR_HIP, std::string("upload_tsdf: ") + hipGetErrorString(e));
    }
  }
  unsigned nbad = 0;
  HIPCHK(hipMemcpy(&nbad, bad, 4, hipMemcpyDeviceToHost));
  HIPCHK(hipFree(tmp));
  launch_occ_rebuild(c->stream, c->vol);  // the raycast's skip maps of the new contents
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(c->stream));
  if (nbad)  // unreachable after the host check (device-side guard; skip maps rebuilt above)
    return set_err(KFX_ERR_ARG, "upload_tsdf: a weight outside 0..255 (u8 weight store; the reference's are 0..64)");
  return KFX_OK;
}

int kfx_download_columns(kfx_ctx *c, const int32_t *cols, int n, int16_t *t, int16_t *w, uint32_t *rgb) {
  int r = check_ctx(c);
  if (r) return r;
  if (n < 0 || (n > 0 && !cols)) return set_err(KFX_ERR_ARG, "bad columns");
  for (int k = 0; k < n; ++k)
    if (cols[2 * k] < 0 || cols[2 * k] >= c->vol.X || cols[2 * k + 1] < 0 || cols[2 * k + 1] >= c->vol.Y)
      return set_err(KFX_ERR_ARG, "column outside the volume");
  if (n == 0) return KFX_OK;
  const size_t cnt = (size_t)n * (c->vol.own1 - c->vol.own0);
  char *tmp = nullptr;
  HIPCHK(hipMalloc(&tmp, (size_t)n * 8 + cnt * 8));
  int32_t *dcols = (int32_t *)tmp;
  int16_t *dt = (int16_t *)(tmp + (size_t)n * 8);
  int16_t *dw = dt + cnt;
  uint32_t *dc = (uint32_t *)(dw + cnt);
  hipError_t e = hipMemcpyAsync(dcols, cols, (size_t)n * 8, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) {
    launch_gather_columns(c->stream, c->vol, dcols, n, dt, dw, dc);
    e = hipGetLastError();
  }
  if (e == hipSuccess && t) e = hipMemcpyAsync(t, dt, cnt * 2, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess && w) e = hipMemcpyAsync(w, dw, cnt * 2, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess && rgb) e = hipMemcpyAsync(rgb, dc, cnt * 4, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  (void)hipFree(tmp);
  if (e != hipSuccess) return set_err(KFX_ERR_HIP, std::string("download_columns: ") + hipGetErrorString(e));
  return KFX_OK;
}

int kfx_slab_mask_payload(const uint32_t *key_local, const uint32_t *key_min, uint32_t *payload, int64_t n) {
  if (!key_local || !key_min || !payload || n < 0) return set_err(KFX_ERR_ARG, "null argument");
  for (int64_t i = 0; i < n; ++i) slab_mask_px(key_local, key_min, payload, (size_t)n, (size_t)i);
  return KFX_OK;
}

int kfx_slab_expand(const uint32_t *payload, const kfx_intrinsics *intr, const kfx_pose *cam2vol,
                    const float Rinv[9], float *vmap, float *nmap) {
  if (!payload || !intr || !cam2vol || !Rinv || !vmap || !nmap) return set_err(KFX_ERR_ARG, "null argument");
  const LevelGeom g = level_geom(*intr, 0);
  const size_t n = (size_t)g.w * g.h;
  for (size_t i = 0; i < n; ++i) {
    float d[3];
    ray_dir(cam2vol->R, g, (int)(i % g.w), (int)(i / g.w), d);
    slab_expand_px(payload, n, i, cam2vol->t, d, Rinv, vmap + 3 * i, nmap + 3 * i);
  }
  return KFX_OK;
}

int kfx_download_volume_soa(kfx_ctx *c, int16_t *t, int16_t *w, uint8_t *rgba) {
  int r = check_ctx(c);
  if (r) return r;
  const int nz = slab_z(c, 8);
  const size_t cap = c->vol.slice * (size_t)nz;
  char *tmp = nullptr;
  HIPCHK(hipMalloc(&tmp, cap * 8));
  int16_t *dt = (int16_t *)tmp;
  int16_t *dw = (int16_t *)(tmp + cap * 2);
  uint32_t *dc = (uint32_t *)(tmp + cap * 4);
  for (int z0 = c->vol.own0; z0 < c->vol.own1; z0 += nz) {  // owned slices only
    const int k = std::min(nz, c->vol.own1 - z0);
    const size_t cnt = c->vol.slice * (size_t)k, off = c->vol.slice * (size_t)z0;
    launch_export_soa(c->stream, c->vol, z0, k, dt, dw, dc);
    hipError_t e = hipSuccess;
    if (t) e = hipMemcpyAsync(t + off, dt, cnt * 2, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess && w) e = hipMemcpyAsync(w + off, dw, cnt * 2, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess && rgba)
      e = hipMemcpyAsync(rgba + 4 * off, dc, cnt * 4, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) {
      (void)hipFree(tmp);
      return set_err(KFX_ERR_HIP, std::string("download_soa: ") + hipGetErrorString(e));
    }
  }
  HIPCHK(hipFree(tmp));
  return KFX_OK;
}

int kfx_stage_preprocess(kfx_ctx *c, const uint8_t *bgr, const float *depth_mm) {
  int r = check_ctx(c);
  if (r) return r;
  if (!bgr || !depth_mm) return set_err(KFX_ERR_ARG, "null image");
  const size_t np = (size_t)c->intr.width * c->intr.height;
  HIPCHK(hipMemcpyAsync(c->raw[0], depth_mm, np * 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->bgr, bgr, np * 3, hipMemcpyHostToDevice, c->stream));
  c->last_bgr = c->bgr;
  HIPCHK(hipMemsetAsync(c->dl0 + np, 0, 64, c->stream));  // the max-depth shards
  for (int l = 1; l < c->L; ++l)
    launch_pyr_down(c->stream, c->raw[l - 1], nullptr, c->g[l - 1].w, c->g[l - 1].h, c->raw[l],
                    nullptr, nullptr);
  launch_preprocess_maps(c->stream, c->L, c->raw, nullptr, c->g, c->cur,
                         c->p.bfilter_kernel_size, c->p.bfilter_color_sigma,
                         c->p.bfilter_spatial_sigma, c->p.dfilter_dist, c->inv_lambda, c->dl0);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(c->stream));
  return KFX_OK;
}

int kfx_stage_icp_accumulate(kfx_ctx *c, int level, const kfx_pose *pose, int64_t sums[27]) {
  int r = check_ctx(c);
  if (r) return r;
  if (level < 0 || level >= c->L || !pose || !sums) return set_err(KFX_ERR_ARG, "bad argument");
  if ((r = write_field(c, offsetof(DevState, icp_pose), to_dev(*pose)))) return r;
  launch_icp(c->stream, c->g[level], c->cur.v[level], c->cur.n[level], c->prev.v[level],
             c->prev.n[level], c->p.icp_dist_threshold, c->angle_thr, c->st, c->icp_shards,
             c->icp_ticket, 1, 0);
  HIPCHK(hipGetLastError());
  DevState s;
  if ((r = read_state(c, &s))) return r;
  for (int k = 0; k < 27; ++k) sums[k] = s.sums[k];
  return KFX_OK;
}

int kfx_stage_icp(kfx_ctx *c, kfx_pose *out) {
  int r = check_ctx(c);
  if (r) return r;
  DevState s0;
  if ((r = read_state(c, &s0))) return r;
  DevState s = s0;
  s.mode = MODE_TRACK;
  s.icp_fail = 0;
  s.icp_pose = identity_pose();
  HIPCHK(hipMemcpyAsync(c->st, &s, sizeof(s), hipMemcpyHostToDevice, c->stream));
  if (!try_icp_persistent(c, c->stream, 0)) {
    for (int level = c->L - 1; level >= 0; --level) {
      for (int it = 0; it < c->p.icp_iter_count[level]; ++it)
        launch_icp(c->stream, c->g[level], c->cur.v[level], c->cur.n[level], c->prev.v[level],
                   c->prev.n[level], c->p.icp_dist_threshold, c->angle_thr, c->st,
                   c->icp_shards, c->icp_ticket, 0, 1);
    }
  }
  HIPCHK(hipGetLastError());
  if ((r = read_state(c, &s))) return r;
  if (s.icp_stalled) {
    HIPCHK(hipMemsetAsync(c->icp_sync, 0, sizeof(IcpSync), c->stream));
    s0.debug_stall = 0;
    HIPCHK(hipMemcpyAsync(c->st, &s0, sizeof(s0), hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (!c->icp_coop) {
      c->icp_coop = true;
      destroy_graphs(c);
    }
    return set_err(KFX_ERR_HIP, "ICP grid barrier watchdog fired (grid not co-resident); "
                                "persistent ICP switched to cooperative launches");
  }
  if (out) *out = to_api(s.icp_pose);
  const int failed = s.icp_fail;
  HIPCHK(hipMemcpyAsync(c->st, &s0, sizeof(s0), hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return failed ? KFX_TRACKING_LOST : KFX_OK;
}

// out: {updated, coloured, visited, gathered, wave batches, 0, 0, 0} of the
// last frame's integrate
static int integrate_stats_impl(kfx_ctx *c, int64_t out[8], const float *xpose) {
  HIPCHK(hipMemsetAsync(c->counters, 0, sizeof(unsigned long long) * 128, c->stream));
  launch_integrate(c->stream, c->vol, c->g[0], c->dl0, c->cur.d[0], c->inv_lambda, c->last_bgr ? c->last_bgr : c->bgr, c->st,
                   c->pose_log, to_dev(c->p.volu_pose), xpose, c->counters);
  HIPCHK(hipGetLastError());
  unsigned long long h[128];
  HIPCHK(hipMemcpyAsync(h, c->counters, sizeof(h), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  for (int k = 0; k < 8; ++k) out[k] = 0;
  for (int i = 0; i < 16; ++i) {
    out[0] += (int64_t)h[2 * i];
    out[1] += (int64_t)h[2 * i + 1];
    for (int k = 2; k < 7; ++k) out[k] += (int64_t)h[16 * k + i];
  }
  return KFX_OK;
}

static int integrate_counts_impl(kfx_ctx *c, int64_t *nu, int64_t *nc, const float *xpose) {
  int64_t s[8];
  const int r = integrate_stats_impl(c, s, xpose);
  if (r) return r;
  if (nu) *nu = s[0];
  if (nc) *nc = s[1];
  return KFX_OK;
}

int kfx_stage_integrate(kfx_ctx *c, const kfx_pose *vol2cam, int64_t *nu, int64_t *nc) {
  int r = check_ctx(c);
  if (r) return r;
  if (!vol2cam) return set_err(KFX_ERR_ARG, "null pose");
  float xp[12];
  std::memcpy(xp, vol2cam->R, sizeof(float) * 9);
  std::memcpy(xp + 9, vol2cam->t, sizeof(float) * 3);
  HIPCHK(hipMemcpyAsync(c->xpose, xp, sizeof(xp), hipMemcpyHostToDevice, c->stream));
  if (nu || nc)
    if ((r = integrate_counts_impl(c, nu, nc, c->xpose))) return r;
  launch_integrate(c->stream, c->vol, c->g[0], c->dl0, c->cur.d[0], c->inv_lambda, c->bgr, c->st, c->pose_log,
                   to_dev(c->p.volu_pose), c->xpose, nullptr);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(c->stream));
  return KFX_OK;
}

int kfx_integrate_counts(kfx_ctx *c, int64_t *nu, int64_t *nc) {
  int r = check_ctx(c);
  if (r) return r;
  return integrate_counts_impl(c, nu, nc, nullptr);
}

int kfx_raycast_stats(kfx_ctx *c, int64_t out[8]) {
  int r = check_ctx(c);
  if (r) return r;
  if (!out) return set_err(KFX_ERR_ARG, "null out");
  HIPCHK(hipMemsetAsync(c->counters, 0, sizeof(unsigned long long) * 8, c->stream));
  // the raycast's pose from the current state (as k_raycast_touch below), not
  // only the last pipeline integrate's
  launch_ray_pose(c->stream, c->st, c->pose_log, to_dev(c->p.volu_pose));
  launch_raycast(c->stream, c->vol, c->L, c->g, c->cur, c->prev, c->st, c->pose_log,
                 to_dev(c->p.volu_pose), nullptr, c->slab ? c->key_local : nullptr, c->counters);
  HIPCHK(hipGetLastError());
  unsigned long long h[8];
  HIPCHK(hipMemcpyAsync(h, c->counters, sizeof(h), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  for (int i = 0; i < 8; ++i) out[i] = i < 6 ? (int64_t)h[i] : 0;
  if (!c->slab) {  // the reference raycast's N_uniq and reads (single volume)
    uint32_t *bits = nullptr;
    HIPCHK(hipMalloc(&bits, (c->vol.local_voxels() + 31) / 32 * 4));
    launch_raycast_touch(c->stream, c->vol, c->g[0], c->st, c->pose_log, to_dev(c->p.volu_pose), nullptr, bits,
                         c->counters + 8);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(h, c->counters + 8, 16, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipFree(bits);
    if (e != hipSuccess) return set_err(KFX_ERR_HIP, std::string("raycast_touch: ") + hipGetErrorString(e));
    out[6] = (int64_t)h[0];
    out[7] = (int64_t)h[1];
  }
  return KFX_OK;
}

int kfx_integrate_stats(kfx_ctx *c, int64_t out[8]) {
  int r = check_ctx(c);
  if (r) return r;
  if (!out) return set_err(KFX_ERR_ARG, "null out");
  return integrate_stats_impl(c, out, nullptr);
}

int kfx_stage_raycast(kfx_ctx *c, const kfx_pose *cam2vol, const float Rinv[9]) {
  int r = check_ctx(c);
  if (r) return r;
  if (!cam2vol || !Rinv) return set_err(KFX_ERR_ARG, "null argument");
  float xp[21];
  std::memcpy(xp, cam2vol->R, sizeof(float) * 9);
  std::memcpy(xp + 9, cam2vol->t, sizeof(float) * 3);
  std::memcpy(xp + 12, Rinv, sizeof(float) * 9);
  if (c->slab && c->world > 1) return set_err(KFX_ERR_STATE, "stage_raycast on one slab of several");
  HIPCHK(hipMemcpyAsync(c->xpose, xp, sizeof(xp), hipMemcpyHostToDevice, c->stream));
  launch_raycast(c->stream, c->vol, c->L, c->g, c->cur, c->prev, c->st, c->pose_log,
                 to_dev(c->p.volu_pose), c->xpose, c->slab ? c->key_local : nullptr);
  if (c->slab) launch_resize(c->stream, c->L, c->g, c->cur, c->prev, c->st, c->xpose);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(c->stream));
  return KFX_OK;
}

#ifdef KFX_ICP_BLOCK_TRACE
// debug build only: per-iteration, per-block {lane-phase start, arrival} stamps
int kfx_debug_icp_blocks(kfx_ctx *c, uint64_t *out, int max_slots) {
  const int n = std::min(max_slots, c->icp_plan.slots);
  HIPCHK(hipStreamSynchronize(c->stream));
  HIPCHK(hipMemcpy(out, c->icp_sync->blk, sizeof(uint64_t) * 1024 * (size_t)n, hipMemcpyDeviceToHost));
  return n;
}
#endif

int kfx_volume_checksum(kfx_ctx *c, uint64_t out[2]) {
  int r = check_ctx(c);
  if (r) return r;
  if (!out) return set_err(KFX_ERR_ARG, "null out");
  HIPCHK(hipMemsetAsync(c->counters, 0, sizeof(unsigned long long) * 2, c->stream));
  launch_checksum(c->stream, c->vol, c->counters);
  HIPCHK(hipGetLastError());
  unsigned long long h[2];
  HIPCHK(hipMemcpyAsync(h, c->counters, sizeof(h), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  out[0] = h[0];
  out[1] = h[1];
  return KFX_OK;
}

int kfx_render(kfx_ctx *c, int type, uint8_t *out) {
  int r = check_ctx(c);
  if (r) return r;
  if (!out || (type != KFX_RENDER_PHONG && type != KFX_RENDER_NORMAL)) return set_err(KFX_ERR_ARG, "bad argument");
  const int n = c->g[0].w * c->g[0].h;
  if (!c->render && (r = dalloc(c, (void **)&c->render, 3 * (size_t)n))) return r;
  launch_render(c->stream, c->prev.v[0], c->prev.n[0], n, c->st, c->pose_log, type, c->render);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(out, c->render, 3 * (size_t)n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return KFX_OK;
}

// ---- point cloud / PLY -----------------------------------------------------

// timing events of the extraction passes (created on first use)
static int extract_events(kfx_ctx *c) {
  for (hipEvent_t &e : c->xev)
    if (!e) HIPCHK(hipEventCreate(&e));
  return KFX_OK;
}

// The slab bound decides which collectives a frame's combine issues (the
// [key | pend] MIN and the resume pass run only when bounded), so every rank of
// a communicator must hold the same mode: checked by a MIN and a MAX
// all-reduce of it (blocking; every rank is inside the same call).  A rank
// with an invalid mode enters the collective with the sentinel -1, so every
// rank returns KFX_ERR_ARG instead of the others blocking in the all-reduce;
// the scratch words are allocated at kfx_comm_init, so no local allocation
// failure can skip the collective either.
static int comm_check_slab_bound(kfx_ctx *c, int mode) {
  int *d = c->comm_chk;
  const int h0[2] = {mode, mode};
  int h[2] = {0, 0};
  int r = KFX_OK;
  const bool up = hipMemcpyAsync(d, h0, sizeof(h0), hipMemcpyHostToDevice, c->stream) == hipSuccess;
  // enter the collective even when the upload failed (its words then hold
  // the last check's values; the error is reported after the collective)
  ncclResult_t e = ncclGroupStart();
  if (e == ncclSuccess) e = ncclAllReduce(d, d, 1, ncclInt32, ncclMin, c->comm, c->stream);
  if (e == ncclSuccess) e = ncclAllReduce(d + 1, d + 1, 1, ncclInt32, ncclMax, c->comm, c->stream);
  const ncclResult_t e2 = ncclGroupEnd();
  if (e == ncclSuccess) e = e2;
  // (the upload reads h0 on this stack frame: the stream is drained before
  // returning on every path)
  const bool drained = hipStreamSynchronize(c->stream) == hipSuccess;
  if (e != ncclSuccess)
    r = set_err(KFX_ERR_COMM, std::string("slab bound check: ") + ncclGetErrorString(e));
  else if (!drained || hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess)
    r = set_err(KFX_ERR_HIP, "slab bound check: download");
  else if (!up)
    r = set_err(KFX_ERR_HIP, "slab bound check: upload");
  else if (h[0] < 0)
    r = set_err(KFX_ERR_ARG, "slab bound modes are 0, 1, 2 (a rank passed another value)");
  else if (h[0] != h[1])
    r = set_err(KFX_ERR_ARG, "ranks differ in kfx_set_slab_bound mode (every rank must pass the same mode)");
  return r;
}

int kfx_set_slab_bound(kfx_ctx *c, int mode) {
  int r = check_ctx(c);
  if (r) return r;
  const bool valid = mode >= 0 && mode <= 2;
  if (c->comm) {
    // over a communicator the call is collective: every rank passes the same
    // mode, and every rank enters the check (an invalid mode as -1)
    if ((r = comm_check_slab_bound(c, valid ? mode : -1))) return r;
  } else if (!valid) {
    return set_err(KFX_ERR_ARG, "slab bound modes are 0, 1, 2");
  }
  if (mode != c->slab_bound) {  // captured frames hold the old passes
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipStreamSynchronize(c->pstream));
    destroy_graphs(c);
  }
  c->slab_bound = mode;
  return KFX_OK;
}

int kfx_set_extract_passes(kfx_ctx *c, int passes) {
  int r = check_ctx(c);
  if (r) return r;
  if (passes != 1 && passes != 2) return set_err(KFX_ERR_ARG, "extract passes are 1 or 2");
  c->extract_mode = passes;
  return KFX_OK;
}

int kfx_get_extract_passes(kfx_ctx *c, int *passes) {
  int r = check_ctx(c);
  if (r) return r;
  if (!passes) return set_err(KFX_ERR_ARG, "null out");
  *passes = c->extract_passes;
  return KFX_OK;
}

int kfx_get_extract_ms(kfx_ctx *c, float out_ms[3]) {
  int r = check_ctx(c);
  if (r) return r;
  if (!out_ms) return set_err(KFX_ERR_ARG, "null out");
  for (int i = 0; i < 3; ++i) out_ms[i] = c->extract_ms[i];
  return KFX_OK;
}

// Extraction into the caller's buffer with ONE read of the volume
// (k_extract_pool: count + items into an unordered pool; the offset scan;
// k_extract_copy: pool -> canonical order).  If the pool (cap items) cannot
// hold every item, the counts are still complete and the emit pass of the
// two-pass path writes the first cap items instead.  Not taken (returns 0)
// for a count-only call (cap = 0), with kfx_set_extract_passes(2), or when
// the buffers cannot be allocated: the caller then runs the two-pass path.
// per = floats per item (3 per point, 9 per triangle).
constexpr int64_t kExtractPoolItems = (int64_t)1 << 23;  // single-pass pool: <= 8.4 M items (100 MB of points)
static int extract_single_pass(kfx_ctx *c, const uint8_t *tab, int zlo, int zhi, float *host, int64_t cap,
                               int per, int64_t *total_out) {
  if (cap <= 0 || cap > (int64_t)1 << 36 || c->extract_mode == 2) return 0;
  const size_t waves = extract_waves(c->vol, zlo, zhi);
  if (waves == 0) return 0;
  const size_t nb = scan_blocks(waves);
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t o_off = al(waves * 4), o_bsum = o_off + al(waves * 8), o_misc = o_bsum + al(nb * 8),
               o_at = o_misc + 256, o_list = o_at + al(waves * 8), wsb = o_list + al(waves * 4);
  char *ws = nullptr;
  float *pool = nullptr, *dout = nullptr;
  // the unordered pool holds at most kExtractPoolItems items whatever the
  // caller's cap (a larger result overflows it and takes the emit pass: the
  // counts are complete either way); the ordered output is allocated once
  // the count is known (n = min(total, cap) items, not cap)
  const int64_t pool_cap = std::min<int64_t>(cap, kExtractPoolItems);
  if (hipMalloc(&ws, wsb) != hipSuccess || hipMalloc(&pool, (size_t)pool_cap * per * sizeof(float)) != hipSuccess) {
    (void)hipGetLastError();
    if (ws) (void)hipFree(ws);
    return 0;
  }
  unsigned *counts = (unsigned *)ws;
  unsigned long long *offsets = (unsigned long long *)(ws + o_off);
  unsigned long long *bsum = (unsigned long long *)(ws + o_bsum);
  unsigned long long *misc = (unsigned long long *)(ws + o_misc);  // {total, ctr, overflow}
  unsigned long long *pool_at = (unsigned long long *)(ws + o_at);
  unsigned *list = (unsigned *)(ws + o_list);
  const DevPose vp = to_dev(c->p.volu_pose);
  int done = 0;
  hipError_t e = hipMemsetAsync(misc, 0, 256, c->stream);
  if (e == hipSuccess && extract_events(c) == KFX_OK) {
    (void)hipEventRecord(c->xev[0], c->stream);
    launch_extract_pool(c->stream, c->vol, vp, zlo, zhi, tab, counts, misc + 1, pool_at, list, pool,
                        (unsigned long long)pool_cap, (unsigned *)(misc + 2));
    (void)hipEventRecord(c->xev[1], c->stream);
    launch_scan(c->stream, counts, offsets, bsum, waves, misc);
    (void)hipEventRecord(c->xev[2], c->stream);
    e = hipGetLastError();
    unsigned long long h[3] = {0, 0, 0};
    if (e == hipSuccess) e = hipMemcpyAsync(h, misc, 24, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    const int64_t total = (int64_t)h[0], n = std::min<int64_t>(total, cap);
    const bool ovf = (unsigned)h[2] != 0;
    if (e == hipSuccess && n > 0) e = hipMalloc(&dout, (size_t)n * per * sizeof(float));
    if (e == hipSuccess && n > 0) {
      (void)hipEventRecord(c->xev[3], c->stream);
      if (!ovf)
        launch_extract_copy(c->stream, list, (unsigned)(h[1] >> 40), counts, pool_at, offsets, pool, dout,
                            (unsigned long long)n, per);
      else if (tab)
        launch_mesh(c->stream, c->vol, vp, zlo, zhi, tab, counts, offsets, dout, (unsigned long long)n);
      else
        launch_extract(c->stream, c->vol, vp, zlo, zhi, counts, offsets, dout, (unsigned long long)n);
      (void)hipEventRecord(c->xev[4], c->stream);
      e = hipGetLastError();
      if (e == hipSuccess) e = hipMemcpyAsync(host, dout, (size_t)n * per * sizeof(float), hipMemcpyDeviceToHost, c->stream);
      if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    }
    if (e == hipSuccess) {
      (void)hipEventElapsedTime(&c->extract_ms[0], c->xev[0], c->xev[1]);
      (void)hipEventElapsedTime(&c->extract_ms[1], c->xev[1], c->xev[2]);
      c->extract_ms[2] = 0.f;
      if (n > 0) (void)hipEventElapsedTime(&c->extract_ms[2], c->xev[3], c->xev[4]);
      c->extract_passes = ovf && n > 0 ? 2 : 1;
      *total_out = total;
      done = 1;
    }
  }
  (void)hipGetLastError();
  if (dout) (void)hipFree(dout);
  (void)hipFree(pool);
  (void)hipFree(ws);
  return done;
}

int kfx_extract_points(kfx_ctx *c, float *xyz, int64_t cap, int64_t *n_points) {
  int r = check_ctx(c);
  if (r) return r;
  if (cap < 0 || (cap > 0 && !xyz)) return set_err(KFX_ERR_ARG, "bad point buffer");
  HIPCHK(hipStreamSynchronize(c->stream));
  // FullScan6 visits z = 0 .. Z-2 (it reads z + 1); a slab its owned part
  const int zlo = std::max(0, c->vol.own0), zhi = std::min(c->vol.own1, c->vol.Z - 1);
  const size_t waves = extract_waves(c->vol, zlo, zhi);
  int64_t total = 0;
  if (waves > 0 && extract_single_pass(c, nullptr, zlo, zhi, xyz, cap, 3, &total)) {
    if (n_points) *n_points = total;
    return KFX_OK;
  }
  c->extract_passes = 2;
  if (waves > 0) {
    const size_t nb = scan_blocks(waves);
    char *ws = nullptr;
    const size_t bytes = waves * 4 + waves * 8 + nb * 8 + 64;
    HIPCHK(hipMalloc(&ws, bytes));
    unsigned *counts = (unsigned *)ws;
    unsigned long long *offsets = (unsigned long long *)(ws + ((waves * 4 + 7) & ~(size_t)7));
    unsigned long long *bsum = offsets + waves;
    unsigned long long *dtot = bsum + nb;
    const DevPose vp = to_dev(c->p.volu_pose);
    if ((r = extract_events(c))) return r;
    HIPCHK(hipEventRecord(c->xev[0], c->stream));
    launch_extract(c->stream, c->vol, vp, zlo, zhi, counts, nullptr, nullptr, 0);
    HIPCHK(hipEventRecord(c->xev[1], c->stream));
    launch_scan(c->stream, counts, offsets, bsum, waves, dtot);
    HIPCHK(hipEventRecord(c->xev[2], c->stream));
    unsigned long long ht = 0;
    hipError_t e = hipMemcpyAsync(&ht, dtot, 8, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    total = (int64_t)ht;
    const int64_t n = std::min<int64_t>(total, cap);
    float *dout = nullptr;
    c->extract_ms[2] = 0.f;
    if (e == hipSuccess && n > 0) {
      e = hipMalloc(&dout, (size_t)n * 12);
      if (e == hipSuccess) {
        (void)hipEventRecord(c->xev[3], c->stream);
        launch_extract(c->stream, c->vol, vp, zlo, zhi, counts, offsets, dout,
                       (unsigned long long)n);
        (void)hipEventRecord(c->xev[4], c->stream);
        e = hipMemcpyAsync(xyz, dout, (size_t)n * 12, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        if (e == hipSuccess) (void)hipEventElapsedTime(&c->extract_ms[2], c->xev[3], c->xev[4]);
        (void)hipFree(dout);
      }
    }
    (void)hipEventElapsedTime(&c->extract_ms[0], c->xev[0], c->xev[1]);
    (void)hipEventElapsedTime(&c->extract_ms[1], c->xev[1], c->xev[2]);
    (void)hipFree(ws);
    if (e != hipSuccess) return set_err(KFX_ERR_HIP, std::string("extract_points: ") + hipGetErrorString(e));
  }
  if (n_points) *n_points = total;
  return KFX_OK;
}

// Marching-cubes triangle table, derived instead of typed in: for each of the
// 256 inside/outside corner patterns, every cube face contributes one segment
// per run of inside corners along its cycle (counter-clockwise seen from
// outside), from the edge entering the run to the edge leaving it — so on an
// ambiguous face the two inside corners are cut off separately, the same way
// from both cubes sharing the face (no cracks).  Each cut edge then starts one
// segment and ends one; the segments close into loops, each loop is fanned
// from its smallest edge index.  At most 5 triangles per cube.
static void build_mc_table(uint8_t tab[256 * 16]) {
  int lo[12], hi[12], n = 0;
  for (int a = 0; a < 3; ++a)
    for (int c = 0; c < 8; ++c)
      if (!((c >> a) & 1)) {
        lo[n] = c;
        hi[n] = c | (1 << a);
        ++n;
      }
  auto eid = [&](int u, int v) {
    for (int e = 0; e < 12; ++e)
      if ((lo[e] == u && hi[e] == v) || (lo[e] == v && hi[e] == u)) return e;
    return -1;
  };
  int cyc[6][4];
  for (int a = 0, f = 0; a < 3; ++a) {
    const int b = (a + 1) % 3, c = (a + 2) % 3;
    static const int pb[4] = {0, 1, 1, 0}, pc[4] = {0, 0, 1, 1};
    for (int s = 0; s < 2; ++s, ++f)
      for (int i = 0; i < 4; ++i) {
        const int k = s ? i : 3 - i;  // the x=0 / y=0 / z=0 face reversed: outward normal -e_a
        cyc[f][i] = (s << a) | (pb[k] << b) | (pc[k] << c);
      }
  }
  std::memset(tab, 0, 256 * 16);
  for (int cfg = 0; cfg < 256; ++cfg) {
    int nxt[12];
    for (int &x : nxt) x = -1;
    for (int f = 0; f < 6; ++f) {
      bool ins[4];
      for (int i = 0; i < 4; ++i) ins[i] = (cfg >> cyc[f][i]) & 1;
      for (int i = 0; i < 4; ++i) {
        if (!ins[i] || ins[(i + 3) % 4]) continue;  // start of a run of inside corners
        int j = i;
        while (ins[(j + 1) % 4]) j = (j + 1) % 4;
        nxt[eid(cyc[f][(i + 3) % 4], cyc[f][i])] = eid(cyc[f][j], cyc[f][(j + 1) % 4]);
      }
    }
    bool seen[12] = {};
    int nt = 0;
    for (int s = 0; s < 12; ++s) {
      if (nxt[s] < 0 || seen[s]) continue;
      int loop[12], m = 0;
      for (int e = s; !seen[e]; e = nxt[e]) {
        seen[e] = true;
        loop[m++] = e;
      }
      for (int k = 1; k + 1 < m; ++k, ++nt) {
        tab[16 * cfg + 1 + 3 * nt] = (uint8_t)loop[0];
        tab[16 * cfg + 2 + 3 * nt] = (uint8_t)loop[k];
        tab[16 * cfg + 3 + 3 * nt] = (uint8_t)loop[k + 1];
      }
    }
    tab[16 * cfg] = (uint8_t)nt;
  }
}

int kfx_extract_mesh(kfx_ctx *c, float *tri_xyz, int64_t cap, int64_t *n_tris) {
  int r = check_ctx(c);
  if (r) return r;
  if (cap < 0 || (cap > 0 && !tri_xyz)) return set_err(KFX_ERR_ARG, "bad triangle buffer");
  HIPCHK(hipStreamSynchronize(c->stream));
  if (!c->mc_tab) {
    uint8_t tab[256 * 16];
    build_mc_table(tab);
    if ((r = dalloc(c, (void **)&c->mc_tab, sizeof(tab)))) return r;
    HIPCHK(hipMemcpy(c->mc_tab, tab, sizeof(tab), hipMemcpyHostToDevice));
  }
  // cubes z .. z+1 for z in the owned slices below Z-1
  const int zlo = std::max(0, c->vol.own0), zhi = std::min(c->vol.own1, c->vol.Z - 1);
  const size_t waves = extract_waves(c->vol, zlo, zhi);
  int64_t total = 0;
  if (waves > 0 && extract_single_pass(c, c->mc_tab, zlo, zhi, tri_xyz, cap, 9, &total)) {
    if (n_tris) *n_tris = total;
    return KFX_OK;
  }
  c->extract_passes = 2;
  if (waves > 0) {
    const size_t nb = scan_blocks(waves);
    char *ws = nullptr;
    HIPCHK(hipMalloc(&ws, waves * 4 + waves * 8 + nb * 8 + 64));
    unsigned *counts = (unsigned *)ws;
    unsigned long long *offsets = (unsigned long long *)(ws + ((waves * 4 + 7) & ~(size_t)7));
    unsigned long long *bsum = offsets + waves;
    unsigned long long *dtot = bsum + nb;
    const DevPose vp = to_dev(c->p.volu_pose);
    if ((r = extract_events(c))) return r;
    HIPCHK(hipEventRecord(c->xev[0], c->stream));
    launch_mesh(c->stream, c->vol, vp, zlo, zhi, c->mc_tab, counts, nullptr, nullptr, 0);
    HIPCHK(hipEventRecord(c->xev[1], c->stream));
    launch_scan(c->stream, counts, offsets, bsum, waves, dtot);
    HIPCHK(hipEventRecord(c->xev[2], c->stream));
    unsigned long long ht = 0;
    hipError_t e = hipMemcpyAsync(&ht, dtot, 8, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    total = (int64_t)ht;
    const int64_t n = std::min<int64_t>(total, cap);
    float *dout = nullptr;
    c->extract_ms[2] = 0.f;
    if (e == hipSuccess && n > 0) {
      e = hipMalloc(&dout, (size_t)n * 36);
      if (e == hipSuccess) {
        (void)hipEventRecord(c->xev[3], c->stream);
        launch_mesh(c->stream, c->vol, vp, zlo, zhi, c->mc_tab, counts, offsets, dout, (unsigned long long)n);
        (void)hipEventRecord(c->xev[4], c->stream);
        e = hipMemcpyAsync(tri_xyz, dout, (size_t)n * 36, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        if (e == hipSuccess) (void)hipEventElapsedTime(&c->extract_ms[2], c->xev[3], c->xev[4]);
        (void)hipFree(dout);
      }
    }
    (void)hipEventElapsedTime(&c->extract_ms[0], c->xev[0], c->xev[1]);
    (void)hipEventElapsedTime(&c->extract_ms[1], c->xev[1], c->xev[2]);
    (void)hipFree(ws);
    if (e != hipSuccess) return set_err(KFX_ERR_HIP, std::string("extract_mesh: ") + hipGetErrorString(e));
  }
  if (n_tris) *n_tris = total;
  return KFX_OK;
}

int kfx_write_ply_mesh(const char *path, const float *tri_xyz, int64_t n) {
  if (!path || n < 0 || (n > 0 && !tri_xyz)) return set_err(KFX_ERR_ARG, "bad argument");
  FILE *f = std::fopen(path, "w");
  if (!f) return set_err(KFX_ERR_ARG, std::string("cannot open ") + path);
  std::fprintf(f, "ply\nformat ascii 1.0\nelement vertex %lld\nproperty float x\nproperty float y\n"
               "property float z\nelement face %lld\nproperty list uchar int vertex_indices\nend_header\n",
               (long long)(3 * n), (long long)n);
  for (int64_t i = 0; i < 3 * n; ++i)
    std::fprintf(f, "%g %g %g\n", tri_xyz[3 * i], tri_xyz[3 * i + 1], tri_xyz[3 * i + 2]);
  for (int64_t i = 0; i < n; ++i)
    std::fprintf(f, "3 %lld %lld %lld\n", (long long)(3 * i), (long long)(3 * i + 1), (long long)(3 * i + 2));
  std::fclose(f);
  return KFX_OK;
}

int kfx_write_ply(const char *path, const float *xyz, int64_t n) {
  if (!path || n < 0 || (n > 0 && !xyz)) return set_err(KFX_ERR_ARG, "bad argument");
  FILE *f = std::fopen(path, "w");
  if (!f) return set_err(KFX_ERR_ARG, std::string("cannot open ") + path);
  // kinectfusion.cpp:154-165: ostream << float uses the default "%g" (6 digits)
  std::fprintf(f, "ply\nformat ascii 1.0\nelement vertex %lld\nproperty float x\nproperty float y\n"
               "property float z\nend_header\n", (long long)n);
  for (int64_t i = 0; i < n; ++i)
    std::fprintf(f, "%g %g %g\n", xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]);
  std::fclose(f);
  return KFX_OK;
}

int kfx_save_pointcloud(kfx_ctx *c, const char *path, int64_t cap) {
  if (!path) return set_err(KFX_ERR_ARG, "null path");
  if (cap <= 0) cap = KFX_DEFAULT_CLOUD_POINTS;
  int64_t total = 0;
  int r = kfx_extract_points(c, nullptr, 0, &total);
  if (r) return r;
  const int64_t n = std::min(total, cap);
  std::vector<float> pts((size_t)n * 3);
  if (n > 0 && (r = kfx_extract_points(c, pts.data(), n, &total))) return r;
  return kfx_write_ply(path, pts.data(), n);
}

// ---- Z-slab sharding -------------------------------------------------------

// slice work of a frame with the camera at cam (camera-to-world; null: the
// first frame's identity pose)
static int slice_work_parts(kfx_ctx *c, const uint8_t *bgr, const float *depth_mm, const kfx_pose *cam,
                            int64_t *cover, int64_t *updated) {
  int r = check_ctx(c);
  if (r) return r;
  if (!bgr || !depth_mm || !cover || !updated) return set_err(KFX_ERR_ARG, "null argument");
  DevPose vol2cam = to_dev(c->p.volu_pose);  // identity camera: vol2cam = volume pose
  if (cam) {  // inverse(cam) o volume pose, in double
    const kfx_pose &v = c->p.volu_pose;
    for (int i = 0; i < 3; ++i) {
      double t = 0.0;
      for (int k = 0; k < 3; ++k) t += (double)cam->R[3 * k + i] * ((double)v.t[k] - cam->t[k]);
      vol2cam.t[i] = (float)t;
      for (int j = 0; j < 3; ++j) {
        double a = 0.0;
        for (int k = 0; k < 3; ++k) a += (double)cam->R[3 * k + i] * v.R[3 * k + j];
        vol2cam.R[3 * i + j] = (float)a;
      }
    }
  }
  HIPCHK(hipStreamSynchronize(c->pstream));
  HIPCHK(hipStreamSynchronize(c->stream));
  set_par(c, 0);
  const size_t np = (size_t)c->intr.width * c->intr.height;
  HIPCHK(hipMemcpyAsync(c->raw[0], depth_mm, np * 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->bgr, bgr, np * 3, hipMemcpyHostToDevice, c->stream));
  enqueue_pre(c, {c->raw[0], nullptr, c->bgr}, nullptr);  // the frame's {depth, 1/lambda} table and max depth
  const int Z = c->vol.Z;
  const size_t n = 2 * (size_t)Z + 1;
  unsigned long long *hist = nullptr;
  HIPCHK(hipMalloc(&hist, sizeof(unsigned long long) * n));
  hipError_t e = hipMemsetAsync(hist, 0, sizeof(unsigned long long) * n, c->stream);
  if (e == hipSuccess) {
    launch_slice_work(c->stream, c->vol, vol2cam, c->g[0], c->dl0, hist);
    e = hipGetLastError();
  }
  std::vector<unsigned long long> h(n);
  if (e == hipSuccess) e = hipMemcpyAsync(h.data(), hist, sizeof(unsigned long long) * n, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  (void)hipFree(hist);
  if (e != hipSuccess) return set_err(KFX_ERR_HIP, std::string("slice_work: ") + hipGetErrorString(e));
  int64_t run = 0;
  for (int z = 0; z < Z; ++z) {
    run += (int64_t)h[z];  // prefix sum of the cover differences
    cover[z] = run;
    updated[z] = (int64_t)h[Z + 1 + z];
  }
  return KFX_OK;
}

int kfx_slice_work_parts(kfx_ctx *c, const uint8_t *bgr, const float *depth_mm, int64_t *cover, int64_t *updated) {
  return slice_work_parts(c, bgr, depth_mm, nullptr, cover, updated);
}

int kfx_slice_work_at(kfx_ctx *c, const uint8_t *bgr, const float *depth_mm, const kfx_pose *cam_pose,
                      int64_t *work, int64_t *cover, int64_t *updated) {
  if (!c || !work) return set_err(KFX_ERR_ARG, "null argument");
  std::vector<int64_t> cv(c->vol.Z), up(c->vol.Z);
  const int r = slice_work_parts(c, bgr, depth_mm, cam_pose, cv.data(), up.data());
  if (r) return r;
  const int64_t slots = (int64_t)c->vol.X * c->vol.Y;
  for (int z = 0; z < c->vol.Z; ++z) {
    work[z] = slice_cost(cv[z], up[z], slots);
    if (cover) cover[z] = cv[z];
    if (updated) updated[z] = up[z];
  }
  return KFX_OK;
}

int kfx_slice_work(kfx_ctx *c, const uint8_t *bgr, const float *depth_mm, int64_t *work) {
  return kfx_slice_work_at(c, bgr, depth_mm, nullptr, work, nullptr, nullptr);
}

int kfx_slab_info(kfx_ctx *c, int *zb, int *zn, int *own0, int *own1) {
  if (!c) return set_err(KFX_ERR_ARG, "null context");
  if (zb) *zb = c->vol.zb;
  if (zn) *zn = c->vol.zn;
  if (own0) *own0 = c->vol.own0;
  if (own1) *own1 = c->vol.own1;
  return KFX_OK;
}

int kfx_comm_get_unique_id(uint8_t id[KFX_COMM_ID_BYTES]) {
  if (!id) return set_err(KFX_ERR_ARG, "null id");
  static_assert(sizeof(ncclUniqueId) == KFX_COMM_ID_BYTES, "RCCL unique id size");
  ncclUniqueId u;
  NCCLCHK(ncclGetUniqueId(&u));
  std::memcpy(id, &u, sizeof(u));
  return KFX_OK;
}

int kfx_comm_init(kfx_ctx *c, const uint8_t id[KFX_COMM_ID_BYTES]) {
  int r = check_ctx(c);
  if (r) return r;
  if (!id) return set_err(KFX_ERR_ARG, "null id");
  if (!c->slab) return set_err(KFX_ERR_STATE, "kfx_comm_init needs a slab context (kfx_create_slab)");
  if (c->comm) return set_err(KFX_ERR_STATE, "communicator already initialised");
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  if (!c->comm_chk) {  // before the collective init: no later local failure skips a collective
    HIPCHK(hipMalloc(&c->comm_chk, 2 * sizeof(int)));
    c->allocs.push_back(c->comm_chk);
  }
  NCCLCHK(ncclCommInitRank(&c->comm, c->world, u, c->rank));
  destroy_graphs(c);
  r = comm_check_slab_bound(c, c->slab_bound);
  if (r) {  // ranks disagree: no communicator, so no frame can issue mismatched collectives
    (void)ncclCommDestroy(c->comm);
    c->comm = nullptr;
  }
  return r;
}

int kfx_pipeline_group(kfx_ctx **cs, int n, const uint8_t *bgr, const float *depth_mm) {
  if (!cs || n < 1 || n > kMaxGroup) return set_err(KFX_ERR_ARG, "group size must be 1..16");
  if (!bgr || !depth_mm) return set_err(KFX_ERR_ARG, "null image");
  for (int k = 0; k < n; ++k) {
    kfx_ctx *c = cs[k];
    if (!c || !c->slab || c->world != n || c->rank != k || c->comm)
      return set_err(KFX_ERR_ARG, "group member k must be slab k of n without a communicator");
    if (c->intr.width != cs[0]->intr.width || c->intr.height != cs[0]->intr.height)
      return set_err(KFX_ERR_ARG, "group members differ in image size");
    // the bound decides which combine passes run: one mode for the whole group
    if (c->slab_bound != cs[0]->slab_bound)
      return set_err(KFX_ERR_ARG, "group members differ in kfx_set_slab_bound mode");
  }
  const size_t np = (size_t)cs[0]->intr.width * cs[0]->intr.height;
  for (int k = 0; k < n; ++k) {  // members on other devices are read by peer access
    for (int j = 0; j < n; ++j) {
      if (cs[j]->device == cs[k]->device) continue;
      (void)hipSetDevice(cs[k]->device);
      (void)hipDeviceEnablePeerAccess(cs[j]->device, 0);
      (void)hipGetLastError();
    }
  }
  int r;
  const bool sharded = cs[0]->icp_sharded && n > 1;
  struct ChainScope {  // group_chain / group_combine hold for this call only (every exit)
    kfx_ctx **cs;
    int n;
    ~ChainScope() {
      for (int k = 0; k < n; ++k) cs[k]->group_chain = cs[k]->group_combine = false;
    }
  } chain_scope{cs, n};
  for (int k = 0; k < n; ++k) cs[k]->group_combine = n > 1;
  hipEvent_t *tev[kMaxGroup] = {};  // members' timing samples (replicated ICP only)
  for (int k = 0; k < n; ++k) {  // local phase: preprocess, ICP, integrate, slab raycast
    kfx_ctx *c = cs[k];
    if ((r = check_ctx(c))) return r;
    if ((r = ensure_pose_capacity(c, 1))) return r;
    if (c->icp_sharded != cs[0]->icp_sharded) return set_err(KFX_ERR_ARG, "group members differ in ICP mode");
    HIPCHK(hipMemcpyAsync(c->raw[0], depth_mm, np * 4, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->bgr, bgr, np * 3, hipMemcpyHostToDevice, c->stream));
    c->last_bgr = c->bgr;
    if (sharded) {
      enqueue_pre(c, {c->raw[0], nullptr, c->bgr}, nullptr);
    } else {
      // Two persistent ICP grids spinning on one device at once can each hold
      // CUs the other's grid barrier waits for (the watchdog then fires): a
      // member's ICP starts after the previous same-device member's ICP.
      // Integrates and raycasts still overlap the next member's work.
      c->group_chain = true;
      if (k > 0 && cs[k - 1]->device == c->device) HIPCHK(hipStreamWaitEvent(c->stream, cs[k - 1]->ev_icp, 0));
      tev[k] = timing_sample(c);
      enqueue_local(c, {c->raw[0], nullptr, c->bgr}, tev[k]);
      if (tev[k]) {  // timed: this member runs alone, as on a GPU of its own
        HIPCHK(hipEventRecord(tev[k][5], c->stream));  // [6] is recorded when the combine starts
        HIPCHK(hipStreamSynchronize(c->stream));
      }
    }
    HIPCHK(hipGetLastError());
  }
  if (sharded) {  // sharded ICP: per iteration, members' bands, in-process sum, solves
    DevState *sts[kMaxGroup];
    for (int k = 0; k < n; ++k) sts[k] = cs[k]->st;
    for (int level = cs[0]->L - 1; level >= 0; --level)
      for (int it = 0; it < cs[0]->p.icp_iter_count[level]; ++it) {
        for (int k = 0; k < n; ++k) {
          kfx_ctx *c = cs[k];
          if ((r = check_ctx(c))) return r;
          launch_icp(c->stream, c->g[level], c->cur.v[level], c->cur.n[level], c->prev.v[level],
                     c->prev.n[level], c->p.icp_dist_threshold, c->angle_thr, c->st, c->icp_shards,
                     c->icp_ticket, 0, 0, k, n);
          HIPCHK(hipStreamSynchronize(c->stream));
        }
        if ((r = check_ctx(cs[0]))) return r;
        launch_group_sum_icp(cs[0]->stream, sts, n);
        HIPCHK(hipStreamSynchronize(cs[0]->stream));
        for (int k = 0; k < n; ++k) {
          if ((r = check_ctx(cs[k]))) return r;
          launch_icp_solve(cs[k]->stream, cs[k]->st);
        }
      }
    for (int k = 0; k < n; ++k) {
      kfx_ctx *c = cs[k];
      if ((r = check_ctx(c))) return r;
      enqueue_map(c, {c->raw[0], nullptr, c->bgr}, nullptr);
      HIPCHK(hipGetLastError());
    }
  }
  for (int k = 0; k < n; ++k) {
    if ((r = check_ctx(cs[k]))) return r;
    HIPCHK(hipStreamSynchronize(cs[k]->stream));
  }
  // combine, with the reductions of the collective path run by one kernel over
  // every member's buffer on member 0's stream; each member's resume pass and
  // mask run on its own stream (its own device's volume), forked from and
  // joined back to member 0's stream by events.  Each member's timed combine
  // is the shared part ([7]..[8]) plus its own expand + pyramid ([6]..[4]) —
  // what one rank of the RCCL path spends, without the members queuing behind
  // each other.
  uint32_t *kin[kMaxGroup], *kout[kMaxGroup], *pay[kMaxGroup];
  for (int k = 0; k < n; ++k) {
    kin[k] = cs[k]->key_local;
    kout[k] = cs[k]->key_min;
    pay[k] = cs[k]->key_local + 2 * np;
  }
  kfx_ctx *c0 = cs[0];
  if ((r = check_ctx(c0))) return r;
  hipStream_t s0 = c0->stream;
  for (int k = 0; k < n; ++k)
    if (tev[k]) HIPCHK(hipEventRecord(tev[k][7], s0));
  // per-member work forked from s0 and joined back (each launch on its own device)
  // On an error partway, the members forked so far are still joined back to
  // s0 and member 0's device is current again, so no enqueued work is orphaned.
  auto per_member = [&](auto &&work) -> int {
    int e = KFX_OK, forked = 1;
    HIPCHK(hipEventRecord(c0->ev_group, s0));
    for (int k = 0; k < n && !e; ++k) {
      if ((e = check_ctx(cs[k]))) break;
      if (k > 0 && hipStreamWaitEvent(cs[k]->stream, c0->ev_group, 0) != hipSuccess) {
        e = set_err(KFX_ERR_HIP, "group combine: fork");
        break;
      }
      work(cs[k]);
      if (k > 0) {
        if (hipEventRecord(cs[k]->ev_group, cs[k]->stream) != hipSuccess) {
          // not joinable by its event: wait for the member's stream instead
          (void)hipStreamSynchronize(cs[k]->stream);
          e = set_err(KFX_ERR_HIP, "group combine: join record");
          break;
        }
        forked = k + 1;
      }
    }
    const int e0 = check_ctx(c0);
    for (int k = 1; k < forked; ++k)
      if (hipStreamWaitEvent(s0, cs[k]->ev_group, 0) != hipSuccess && !e) e = set_err(KFX_ERR_HIP, "group combine: join");
    return e ? e : e0;
  };
  if (c0->pass1_bounded) {  // [key | pend] MIN, then the resume passes
    launch_group_reduce(s0, kin, n, kout, n, 2 * np, false);
    if ((r = per_member([](kfx_ctx *c) { enqueue_slab_resume(c, c->stream); }))) return r;
  }
  launch_group_reduce(s0, kin, n, kout, n, np, false);
  if ((r = per_member([np](kfx_ctx *c) { launch_slab_mask(c->stream, c->key_local, c->key_min, (int)np); })))
    return r;
  launch_group_reduce(s0, pay, n, pay, n, 4 * np, true);
  for (int k = 0; k < n; ++k)
    if (tev[k]) HIPCHK(hipEventRecord(tev[k][8], s0));
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(s0));
  int status = KFX_OK;
  for (int k = 0; k < n; ++k) {
    kfx_ctx *c = cs[k];
    if ((r = check_ctx(c))) return r;
    if (tev[k]) HIPCHK(hipEventRecord(tev[k][6], c->stream));
    launch_slab_expand(c->stream, c->g[0], c->key_local + 2 * np, c->cur, c->prev, c->st, c->pose_log,
                       to_dev(c->p.volu_pose));
    launch_resize(c->stream, c->L, c->g, c->cur, c->prev, c->st, nullptr);
    if (tev[k]) {  // timed members run alone (as on a GPU of their own)
      HIPCHK(hipEventRecord(tev[k][4], c->stream));
      HIPCHK(hipStreamSynchronize(c->stream));
    }
    HIPCHK(hipGetLastError());
    c->pending += 1;
    const int s = finish_frame(c);
    if (s < 0) return s;
    if (k == 0) status = s;
    else if (s != status) return set_err(KFX_ERR_STATE, "slab members disagree on the tracking status");
  }
  return status;
}

int kfx_slab_frame_local(kfx_ctx *c, const uint8_t *bgr, const float *depth_mm, uint32_t *keys,
                         uint32_t *payload) {
  int r = check_ctx(c);
  if (r) return r;
  if (!bgr || !depth_mm || !keys || !payload) return set_err(KFX_ERR_ARG, "null argument");
  if (!c->slab || c->comm) return set_err(KFX_ERR_STATE, "kfx_slab_frame_local needs a slab context without a communicator");
  if (c->icp_sharded) return set_err(KFX_ERR_STATE, "the external combine runs the replicated ICP (kfx_set_icp_allreduce 0)");
  if ((r = ensure_pose_capacity(c, 1))) return r;
  const size_t np = (size_t)c->intr.width * c->intr.height;
  HIPCHK(hipStreamSynchronize(c->pstream));  // an overlapped frame's preprocess may still use set 0's inputs
  set_par(c, 0);
  HIPCHK(hipMemcpyAsync(c->raw[0], depth_mm, np * 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipMemcpyAsync(c->bgr, bgr, np * 3, hipMemcpyHostToDevice, c->stream));
  c->last_bgr = c->bgr;
  hipEvent_t *tev = timing_sample(c);
  enqueue_local(c, {c->raw[0], nullptr, c->bgr}, tev);
  if (tev) HIPCHK(hipEventRecord(tev[5], c->stream));
  if (tev) HIPCHK(hipEventRecord(tev[6], c->stream));  // re-recorded when the combine starts
  if (tev) HIPCHK(hipEventRecord(tev[7], c->stream));  // (no shared part on the device: [7] = [8])
  if (tev) HIPCHK(hipEventRecord(tev[8], c->stream));
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(keys, c->key_local, np * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipMemcpyAsync(payload, c->key_local + 2 * np, 4 * np * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  c->ext_pending = tev;
  c->ext_open = true;
  return KFX_OK;
}

int kfx_slab_frame_finish(kfx_ctx *c, const uint32_t *payload) {
  int r = check_ctx(c);
  if (r) return r;
  if (!payload) return set_err(KFX_ERR_ARG, "null payload");
  if (!c->ext_open) return set_err(KFX_ERR_STATE, "kfx_slab_frame_finish without kfx_slab_frame_local");
  c->ext_open = false;
  const size_t np = (size_t)c->intr.width * c->intr.height;
  uint32_t *pay = c->key_local + 2 * np;
  if (c->ext_pending) HIPCHK(hipEventRecord(c->ext_pending[6], c->stream));
  if (c->ext_pending) HIPCHK(hipEventRecord(c->ext_pending[7], c->stream));
  if (c->ext_pending) HIPCHK(hipEventRecord(c->ext_pending[8], c->stream));
  HIPCHK(hipMemcpyAsync(pay, payload, 4 * np * 4, hipMemcpyHostToDevice, c->stream));
  launch_slab_expand(c->stream, c->g[0], pay, c->cur, c->prev, c->st, c->pose_log, to_dev(c->p.volu_pose));
  launch_resize(c->stream, c->L, c->g, c->cur, c->prev, c->st, nullptr);
  if (c->ext_pending) HIPCHK(hipEventRecord(c->ext_pending[4], c->stream));
  c->ext_pending = nullptr;
  HIPCHK(hipGetLastError());
  c->pending += 1;
  return finish_frame(c);
}

}  // extern "C"
