"""kfx — Python binding of libkfx.so (the MI355X KinectFusion hot path).

`KinectFusion` mirrors the reference's `kf::kinectfusion` (kinectfusion.h:31-73):
pipeline(color, depth) / reset() / getCurCameraPose() / pose_record /
frame_count, plus the stage seams of include/kfx.h used by the parity tests.

There is no CPU fallback: constructing a KinectFusion without the HIP library or
without a GPU raises.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from .abi import (KFX_FRAME_CUR, KFX_FRAME_PREV, KFX_OK, KFX_TRACKING_LOST, Intrinsics, Params, Pose,
                  default_params, fptr, i16ptr, i64ptr, u8ptr, u16ptr)

__all__ = ["KinectFusion", "KfxError", "Dataset", "png_info", "png_read_bgr8", "png_read_depth", "parse_intr",
           "comm_unique_id", "pipeline_group", "slab_balance", "write_ply", "lib", "build", "LIB_PATH", "Intrinsics", "Params", "Pose",
           "default_params", "KFX_FRAME_CUR", "KFX_FRAME_PREV", "KFX_OK", "KFX_TRACKING_LOST", "EXPORTS"]

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("KFX_LIB_PATH") or os.path.join(_PKG, "lib", "libkfx.so")  # override: tuning runs

# every symbol include/kfx.h declares
EXPORTS = [
    "kfx_abi_version", "kfx_last_error", "kfx_default_params", "kfx_create", "kfx_destroy", "kfx_reset",
    "kfx_pipeline", "kfx_pipeline_u16", "kfx_stage_frames", "kfx_pipeline_staged", "kfx_synchronize",
    "kfx_set_graph_mode", "kfx_set_frame_overlap", "kfx_set_kernel_timing", "kfx_get_kernel_timing", "kfx_get_kernel_timing_ex", "kfx_set_icp_persistent", "kfx_debug_force_icp_stall", "kfx_debug_force_index64", "kfx_debug_icp_band_ms", "kfx_get_icp_trace", "kfx_get_cur_camera_pose", "kfx_get_frame_count", "kfx_get_pose_record",
    "kfx_write_poses_txt", "kfx_get_frame_maps", "kfx_set_frame_maps", "kfx_download_tsdf",
    "kfx_upload_tsdf", "kfx_download_volume_soa", "kfx_stage_preprocess", "kfx_stage_icp_accumulate",
    "kfx_stage_icp", "kfx_stage_integrate", "kfx_stage_raycast", "kfx_set_profiling", "kfx_get_stage_ms",
    "kfx_integrate_counts", "kfx_integrate_stats", "kfx_raycast_stats", "kfx_download_columns", "kfx_pipeline_async", "kfx_pipeline_async_u16", "kfx_register_host_buffer", "kfx_unregister_host_buffer", "kfx_slab_mask_payload", "kfx_slab_expand", "kfx_set_icp_allreduce", "kfx_create_slab", "kfx_create_slab_cuts", "kfx_slice_work", "kfx_slice_work_parts", "kfx_slice_work_at", "kfx_get_graph_mode", "kfx_get_graph_note", "kfx_slab_balance", "kfx_slab_info", "kfx_comm_get_unique_id", "kfx_comm_init",
    "kfx_pipeline_group", "kfx_slab_frame_local", "kfx_slab_frame_finish", "kfx_render", "kfx_volume_checksum", "kfx_extract_points", "kfx_write_ply", "kfx_save_pointcloud",
    "kfx_extract_mesh", "kfx_write_ply_mesh", "kfx_get_extract_ms", "kfx_set_extract_passes", "kfx_get_extract_passes", "kfx_set_slab_bound",
    "kfx_dataset_open", "kfx_dataset_info", "kfx_dataset_read", "kfx_dataset_close", "kfx_png_info",
    "kfx_png_read_bgr8", "kfx_png_read_depth", "kfx_parse_intr",
]


class KfxError(RuntimeError):
    pass


_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _PKG], check=True)
    return LIB_PATH


def lib():
    """Load libkfx.so (raises if it has not been built — no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise KfxError(f"{LIB_PATH} missing: run `make -C {_PKG}` (or __graft_entry__.build())")
    L = C.CDLL(LIB_PATH)
    P, i, f = C.POINTER, C.c_int, C.c_float
    vp = C.c_void_p
    sig = {
        "kfx_abi_version": ([], i),
        "kfx_last_error": ([], C.c_char_p),
        "kfx_default_params": ([P(Params)], i),
        "kfx_create": ([P(Intrinsics), P(Params), i, P(vp)], i),
        "kfx_destroy": ([vp], i),
        "kfx_reset": ([vp], i),
        "kfx_pipeline": ([vp, P(C.c_uint8), P(f)], i),
        "kfx_pipeline_u16": ([vp, P(C.c_uint8), P(C.c_uint16)], i),
        "kfx_stage_frames": ([vp, i, P(C.c_uint8), P(f)], i),
        "kfx_pipeline_staged": ([vp, i], i),
        "kfx_synchronize": ([vp], i),
        "kfx_set_graph_mode": ([vp, i], i),
        "kfx_set_frame_overlap": ([vp, i], i),
        "kfx_set_kernel_timing": ([vp, i, i], i),
        "kfx_get_kernel_timing": ([vp, P(C.c_float), P(C.c_int)], i),
        "kfx_get_kernel_timing_ex": ([vp, P(C.c_float), P(C.c_int)], i),
        "kfx_set_icp_persistent": ([vp, i], i),
        "kfx_debug_force_icp_stall": ([vp], i),
        "kfx_debug_force_index64": ([vp, i], i),
        "kfx_debug_icp_band_ms": ([vp, i, i, i, P(C.c_float)], i),
        "kfx_get_icp_trace": ([vp, P(C.c_uint64), i], i),
        "kfx_get_cur_camera_pose": ([vp, P(Pose)], i),
        "kfx_get_frame_count": ([vp, P(i)], i),
        "kfx_get_pose_record": ([vp, P(Pose), i, P(i)], i),
        "kfx_write_poses_txt": ([vp, C.c_char_p], i),
        "kfx_get_frame_maps": ([vp, i, i, P(f), P(f), P(f)], i),
        "kfx_set_frame_maps": ([vp, i, i, P(f), P(f)], i),
        "kfx_download_tsdf": ([vp, vp], i),
        "kfx_upload_tsdf": ([vp, vp], i),
        "kfx_download_volume_soa": ([vp, P(C.c_int16), P(C.c_int16), P(C.c_uint8)], i),
        "kfx_stage_preprocess": ([vp, P(C.c_uint8), P(f)], i),
        "kfx_stage_icp_accumulate": ([vp, i, P(Pose), P(C.c_int64)], i),
        "kfx_stage_icp": ([vp, P(Pose)], i),
        "kfx_stage_integrate": ([vp, P(Pose), P(C.c_int64), P(C.c_int64)], i),
        "kfx_stage_raycast": ([vp, P(Pose), P(f)], i),
        "kfx_set_profiling": ([vp, i], i),
        "kfx_get_stage_ms": ([vp, P(f)], i),
        "kfx_integrate_counts": ([vp, P(C.c_int64), P(C.c_int64)], i),
        "kfx_integrate_stats": ([vp, P(C.c_int64)], i),
        "kfx_raycast_stats": ([vp, P(C.c_int64)], i),
        "kfx_pipeline_async": ([vp, P(C.c_uint8), P(f)], i),
        "kfx_slab_mask_payload": ([P(C.c_uint32), P(C.c_uint32), P(C.c_uint32), C.c_int64], i),
        "kfx_set_icp_allreduce": ([vp, i], i),
        "kfx_slab_expand": ([P(C.c_uint32), P(Intrinsics), P(Pose), P(f), P(f), P(f)], i),
        "kfx_pipeline_async_u16": ([vp, P(C.c_uint8), P(C.c_uint16)], i),
        "kfx_register_host_buffer": ([vp, vp, C.c_size_t], i),
        "kfx_unregister_host_buffer": ([vp, vp], i),
        "kfx_download_columns": ([vp, P(C.c_int32), i, P(C.c_int16), P(C.c_int16), P(C.c_uint32)], i),
        "kfx_create_slab": ([P(Intrinsics), P(Params), i, i, i, P(vp)], i),
        "kfx_create_slab_cuts": ([P(Intrinsics), P(Params), i, i, i, P(i), P(vp)], i),
        "kfx_slice_work": ([vp, P(C.c_uint8), P(f), P(C.c_int64)], i),
        "kfx_slice_work_parts": ([vp, P(C.c_uint8), P(f), P(C.c_int64), P(C.c_int64)], i),
        "kfx_slice_work_at": ([vp, P(C.c_uint8), P(f), P(Pose), P(C.c_int64), P(C.c_int64), P(C.c_int64)], i),
        "kfx_get_graph_mode": ([vp, P(i)], i),
        "kfx_get_graph_note": ([vp], C.c_char_p),
        "kfx_slab_balance": ([P(C.c_int64), i, i, P(i)], i),
        "kfx_slab_info": ([vp, P(i), P(i), P(i), P(i)], i),
        "kfx_comm_get_unique_id": ([P(C.c_uint8)], i),
        "kfx_comm_init": ([vp, P(C.c_uint8)], i),
        "kfx_pipeline_group": ([P(vp), i, P(C.c_uint8), P(f)], i),
        "kfx_slab_frame_local": ([vp, P(C.c_uint8), P(f), P(C.c_uint32), P(C.c_uint32)], i),
        "kfx_slab_frame_finish": ([vp, P(C.c_uint32)], i),
        "kfx_extract_points": ([vp, P(f), C.c_int64, P(C.c_int64)], i),
        "kfx_render": ([vp, i, P(C.c_uint8)], i),
        "kfx_volume_checksum": ([vp, P(C.c_uint64)], i),
        "kfx_write_ply": ([C.c_char_p, P(f), C.c_int64], i),
        "kfx_save_pointcloud": ([vp, C.c_char_p, C.c_int64], i),
        "kfx_extract_mesh": ([vp, P(f), C.c_int64, P(C.c_int64)], i),
        "kfx_get_extract_ms": ([vp, P(f)], i),
        "kfx_set_extract_passes": ([vp, i], i),
        "kfx_set_slab_bound": ([vp, i], i),
        "kfx_get_extract_passes": ([vp, P(i)], i),
        "kfx_write_ply_mesh": ([C.c_char_p, P(f), C.c_int64], i),
        "kfx_dataset_open": ([C.c_char_p, P(vp)], i),
        "kfx_dataset_info": ([vp, P(Intrinsics), P(i), P(i)], i),
        "kfx_dataset_read": ([vp, i, P(C.c_uint8), P(f)], i),
        "kfx_dataset_close": ([vp], i),
        "kfx_png_info": ([C.c_char_p, P(i), P(i), P(i), P(i)], i),
        "kfx_png_read_bgr8": ([C.c_char_p, P(C.c_uint8), i, i], i),
        "kfx_png_read_depth": ([C.c_char_p, P(f), i, i], i),
        "kfx_parse_intr": ([C.c_char_p, P(f)], i),
    }
    for name, (args, res) in sig.items():
        try:
            fn = getattr(L, name)
        except AttributeError:  # an older build (A/B timing runs); calling it raises then
            continue
        fn.argtypes = args
        fn.restype = res
    _lib = L
    return L


def _check(rc: int, what: str, ok=(KFX_OK,)) -> int:
    if rc not in ok:
        raise KfxError(f"{what} failed ({rc}): {lib().kfx_last_error().decode(errors='replace')}")
    return rc


def slab_mask_payload(key_local: np.ndarray, key_min: np.ndarray, payload: np.ndarray) -> np.ndarray:
    """Host side of the slab combine (kfx_slab_mask_payload): payload (4, n)
    u32 with the pixels this slab lost cleared (returns a copy)."""
    u32p = C.POINTER(C.c_uint32)
    kl = np.ascontiguousarray(key_local, np.uint32).ravel()
    km = np.ascontiguousarray(key_min, np.uint32).ravel()
    pay = np.ascontiguousarray(payload, np.uint32).copy()
    _check(lib().kfx_slab_mask_payload(kl.ctypes.data_as(u32p), km.ctypes.data_as(u32p), pay.ctypes.data_as(u32p),
                                       kl.size), "kfx_slab_mask_payload")
    return pay


def slab_expand(payload: np.ndarray, intr, cam2vol: Pose, Rinv: np.ndarray):
    """Host side of the slab combine (kfx_slab_expand): level-0 (vmap, nmap)."""
    pay = np.ascontiguousarray(payload, np.uint32)
    I = Intrinsics.from_any(intr)
    vmap = np.zeros((I.height, I.width, 3), np.float32)
    nmap = np.zeros_like(vmap)
    R = np.ascontiguousarray(Rinv, np.float32).reshape(9)
    _check(lib().kfx_slab_expand(pay.ctypes.data_as(C.POINTER(C.c_uint32)), C.byref(I), C.byref(cam2vol), fptr(R),
                                 fptr(vmap), fptr(nmap)), "kfx_slab_expand")
    return vmap, nmap


def write_ply(path: str, xyz: np.ndarray):
    """kinectfusion::savePointcloud's ASCII PLY for an (N, 3) float32 array."""
    xyz = np.ascontiguousarray(xyz, np.float32)
    _check(lib().kfx_write_ply(path.encode(), fptr(xyz), xyz.shape[0]), "kfx_write_ply")


def png_info(path: str) -> tuple:
    """(width, height, channels, bit_depth) of a PNG file."""
    w, h, c, b = C.c_int(), C.c_int(), C.c_int(), C.c_int()
    _check(lib().kfx_png_info(path.encode(), C.byref(w), C.byref(h), C.byref(c), C.byref(b)), "kfx_png_info")
    return w.value, h.value, c.value, b.value


def png_read_bgr8(path: str) -> np.ndarray:
    """imread(path, IMREAD_COLOR): (H, W, 3) uint8 BGR."""
    w, h, _, _ = png_info(path)
    out = np.empty((h, w, 3), np.uint8)
    _check(lib().kfx_png_read_bgr8(path.encode(), out.ctypes.data_as(C.POINTER(C.c_uint8)), w, h),
           "kfx_png_read_bgr8")
    return out


def png_read_depth(path: str) -> np.ndarray:
    """imread(path, IMREAD_UNCHANGED).convertTo(CV_32F): (H, W) float32."""
    w, h, _, _ = png_info(path)
    out = np.empty((h, w), np.float32)
    _check(lib().kfx_png_read_depth(path.encode(), fptr(out), w, h), "kfx_png_read_depth")
    return out


def parse_intr(path: str) -> tuple:
    """intr.txt (depth_sensor.cpp:22-35): (fx, cx, fy, cy, c)."""
    out = (C.c_float * 5)()
    _check(lib().kfx_parse_intr(path.encode(), out), "kfx_parse_intr")
    return tuple(out)


class Dataset:
    """depth_sensor's DATASET mode (depth_sensor.cpp:11-46, 186-196) over the C-ABI:
    frames as kinectfusion::pipeline receives them (BGR uint8, depth float mm)."""

    def __init__(self, path: str):
        h = C.c_void_p()
        _check(lib().kfx_dataset_open(path.encode(), C.byref(h)), "kfx_dataset_open")
        self._h = h
        intr, n, has = Intrinsics(), C.c_int(), C.c_int()
        _check(lib().kfx_dataset_info(self._h, C.byref(intr), C.byref(n), C.byref(has)), "kfx_dataset_info")
        self.intrinsics, self.n_frames, self.has_intr = intr, n.value, bool(has.value)

    def __len__(self):
        return self.n_frames

    def read(self, index: int):
        w, hgt = self.intrinsics.width, self.intrinsics.height
        bgr = np.empty((hgt, w, 3), np.uint8)
        dep = np.empty((hgt, w), np.float32)
        _check(lib().kfx_dataset_read(self._h, int(index), bgr.ctypes.data_as(C.POINTER(C.c_uint8)), fptr(dep)),
               "kfx_dataset_read")
        return bgr, dep

    def close(self):
        if self._h:
            lib().kfx_dataset_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def write_ply_mesh(path: str, tris: np.ndarray):
    """ASCII PLY of an (N, 3, 3) float32 triangle soup."""
    t = np.ascontiguousarray(tris, np.float32)
    _check(lib().kfx_write_ply_mesh(path.encode(), fptr(t), t.shape[0]), "kfx_write_ply_mesh")


def comm_unique_id() -> bytes:
    """RCCL unique id (128 bytes) for kfx_comm_init; made on rank 0 and
    broadcast to the other ranks by the launcher."""
    buf = (C.c_uint8 * 128)()
    _check(lib().kfx_comm_get_unique_id(buf), "kfx_comm_get_unique_id")
    return bytes(buf)


def slab_balance(slice_work, world: int) -> list:
    """kfx_slab_balance: world + 1 slab cuts (multiples of 8) minimising the
    largest slab's stored-range work for a per-slice work histogram."""
    w = np.ascontiguousarray(slice_work, np.int64)
    cu = (C.c_int * (world + 1))()
    _check(lib().kfx_slab_balance(i64ptr(w), int(w.size), int(world), cu), "kfx_slab_balance")
    return list(cu)


def _trim(out: np.ndarray, n: int) -> np.ndarray:
    """The first n items of a cap-sized output buffer: a copy when n is well
    below the cap (a view would keep the whole cap-sized allocation alive)."""
    return out[:n].copy() if 2 * n < len(out) else out[:n]


def pipeline_group(members, color: np.ndarray, depth: np.ndarray) -> int:
    """One pipeline() frame over all Z-slabs held in this process
    (members[k] = slab k of len(members))."""
    color = np.ascontiguousarray(color, np.uint8)
    d = np.ascontiguousarray(depth, np.float32)
    hs = (C.c_void_p * len(members))(*[m._h for m in members])
    rc = lib().kfx_pipeline_group(hs, len(members), u8ptr(color), fptr(d))
    return _check(rc, "kfx_pipeline_group", ok=(KFX_OK, KFX_TRACKING_LOST))


class KinectFusion:
    """kf::kinectfusion over the C-ABI.  Images: depth (H,W) float32/uint16 mm,
    colour (H,W,3) uint8 BGR."""

    def __init__(self, intr, params: Params | None = None, device: int = 0, slab=None, cuts=None):
        """slab=(rank, world): this instance owns Z-slab `rank` of `world`
        (kfx_create_slab; with cuts, world + 1 slice boundaries:
        kfx_create_slab_cuts); combine through comm_init (one process per GPU)
        or pipeline_group (all slabs in this process)."""
        self.intr = Intrinsics.from_any(intr)
        self.params = params if params is not None else default_params()
        h = C.c_void_p()
        if slab is None:
            _check(lib().kfx_create(C.byref(self.intr), C.byref(self.params), device, C.byref(h)), "kfx_create")
        else:
            rank, world = slab
            if cuts is None:
                _check(lib().kfx_create_slab(C.byref(self.intr), C.byref(self.params), device, int(rank), int(world),
                                             C.byref(h)), "kfx_create_slab")
            else:
                cu = (C.c_int * (world + 1))(*[int(x) for x in cuts])
                _check(lib().kfx_create_slab_cuts(C.byref(self.intr), C.byref(self.params), device, int(rank),
                                                  int(world), cu, C.byref(h)), "kfx_create_slab_cuts")
        self._h = h
        self.slab = slab
        X, Y, Z = (int(d) for d in self.params.volu_dims)
        self.dims = (X, Y, Z)
        self.nvox = X * Y * Z

    def close(self):
        if getattr(self, "_h", None):
            lib().kfx_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ---- kf::kinectfusion ------------------------------------------------
    def pipeline(self, color: np.ndarray, depth: np.ndarray) -> int:
        """Returns KFX_OK or KFX_TRACKING_LOST (reset applied, frame dropped)."""
        color = np.ascontiguousarray(color, np.uint8)
        if depth.dtype == np.uint16:
            d = np.ascontiguousarray(depth)
            rc = lib().kfx_pipeline_u16(self._h, u8ptr(color), u16ptr(d))
        else:
            d = np.ascontiguousarray(depth, np.float32)
            rc = lib().kfx_pipeline(self._h, u8ptr(color), fptr(d))
        return _check(rc, "kfx_pipeline", ok=(KFX_OK, KFX_TRACKING_LOST))

    def reset(self):
        _check(lib().kfx_reset(self._h), "kfx_reset")

    def getCurCameraPose(self) -> np.ndarray:
        p = Pose()
        _check(lib().kfx_get_cur_camera_pose(self._h, C.byref(p)), "kfx_get_cur_camera_pose")
        return p.matrix()

    @property
    def frame_count(self) -> int:
        n = C.c_int()
        _check(lib().kfx_get_frame_count(self._h, C.byref(n)), "kfx_get_frame_count")
        return n.value

    @property
    def pose_record(self) -> np.ndarray:
        n = C.c_int()
        _check(lib().kfx_get_pose_record(self._h, None, 0, C.byref(n)), "kfx_get_pose_record")
        buf = (Pose * max(n.value, 1))()
        _check(lib().kfx_get_pose_record(self._h, buf, n.value, C.byref(n)), "kfx_get_pose_record")
        return np.stack([buf[i].matrix() for i in range(n.value)])

    def write_poses_txt(self, path: str):
        _check(lib().kfx_write_poses_txt(self._h, path.encode()), "kfx_write_poses_txt")

    # ---- device-resident frames ------------------------------------------
    def stage_frames(self, colors: np.ndarray, depths: np.ndarray):
        colors = np.ascontiguousarray(colors, np.uint8)
        depths = np.ascontiguousarray(depths, np.float32)
        _check(lib().kfx_stage_frames(self._h, depths.shape[0], u8ptr(colors), fptr(depths)), "kfx_stage_frames")

    def pipeline_staged(self, idx: int):
        _check(lib().kfx_pipeline_staged(self._h, int(idx)), "kfx_pipeline_staged")

    def pipeline_async(self, color, depth_mm):
        """Queue a host frame (f32 or u16 depth, mm) without waiting for the GPU
        (kfx_pipeline_async); tracking status comes with synchronize()."""
        color = np.ascontiguousarray(color, np.uint8)
        if np.asarray(depth_mm).dtype == np.uint16:
            d = np.ascontiguousarray(depth_mm, np.uint16)
            _check(lib().kfx_pipeline_async_u16(self._h, u8ptr(color), d.ctypes.data_as(C.POINTER(C.c_uint16))),
                   "kfx_pipeline_async_u16")
        else:
            d = np.ascontiguousarray(depth_mm, np.float32)
            _check(lib().kfx_pipeline_async(self._h, u8ptr(color), fptr(d)), "kfx_pipeline_async")

    def register_host_buffer(self, arr: np.ndarray):
        """Page-lock a C-contiguous array: pipeline_async then uploads frames in
        it without a host copy (keep it unchanged until synchronize())."""
        assert arr.flags["C_CONTIGUOUS"]
        _check(lib().kfx_register_host_buffer(self._h, arr.ctypes.data, arr.nbytes), "kfx_register_host_buffer")

    def unregister_host_buffer(self, arr: np.ndarray):
        _check(lib().kfx_unregister_host_buffer(self._h, arr.ctypes.data), "kfx_unregister_host_buffer")

    def synchronize(self) -> int:
        """Wait for queued frames; KFX_OK, or KFX_TRACKING_LOST if one of the
        frames completed since the last status check was dropped (reset)."""
        return _check(lib().kfx_synchronize(self._h), "kfx_synchronize", ok=(KFX_OK, KFX_TRACKING_LOST))

    def set_graph_mode(self, mode):
        """0/False eager, 1/True (default) graphs, 2 overlapped frames also
        replay ICP + integrate + raycast as a graph (kfx.h kfx_set_graph_mode)."""
        _check(lib().kfx_set_graph_mode(self._h, int(mode)), "kfx_set_graph_mode")

    def graph_mode(self) -> int:
        """The graph mode in effect (kfx_get_graph_mode: lowered where RCCL
        refused stream capture)."""
        m = C.c_int()
        _check(lib().kfx_get_graph_mode(self._h, C.byref(m)), "kfx_get_graph_mode")
        return m.value

    def graph_note(self) -> str:
        """Why graph mode 2 was lowered (RCCL / capture error text), or ""."""
        return (lib().kfx_get_graph_note(self._h) or b"").decode(errors="replace")

    def set_kernel_timing(self, every: int, max_samples: int = 1024):
        """Bracket every `every`-th pipelined frame with HIP events (0 = off)."""
        _check(lib().kfx_set_kernel_timing(self._h, int(every), int(max_samples)), "kfx_set_kernel_timing")

    def kernel_timing(self) -> dict:
        """Mean ms of ICP / integrate / raycast (+ slab combine) over the sampled
        frames, and of the local raycast and the combine apart (resets the samples)."""
        a, n = (C.c_float * 4)(), C.c_int()
        _check(lib().kfx_get_kernel_timing_ex(self._h, a, C.byref(n)), "kfx_get_kernel_timing_ex")
        return {"icp": a[0], "integrate": a[1], "raycast": a[2] + a[3], "raycast_local": a[2],
                "combine": a[3], "samples": n.value}

    def set_frame_overlap(self, on: bool):
        """Overlap staged frames' preprocess with the previous frame's tracking."""
        _check(lib().kfx_set_frame_overlap(self._h, int(on)), "kfx_set_frame_overlap")

    def set_icp_allreduce(self, on: bool):
        """Slab contexts: shard the ICP sums over the ranks (all-reduced per iteration)."""
        _check(lib().kfx_set_icp_allreduce(self._h, int(on)), "kfx_set_icp_allreduce")

    def set_icp_persistent(self, on) -> bool:
        """Persistent ICP: False = one launch per iteration, True = one persistent
        launch, 2 = persistent through a cooperative launch; returns whether the
        persistent kernel is usable here."""
        r = lib().kfx_set_icp_persistent(self._h, int(on))
        _check(min(r, 0), "kfx_set_icp_persistent")
        return bool(r)

    def debug_force_icp_stall(self):
        """Test hook: the next tracked frame's persistent-ICP barrier never completes."""
        _check(lib().kfx_debug_force_icp_stall(self._h), "kfx_debug_force_icp_stall")

    def debug_force_index64(self, on=True):
        """Test hook: integrate / raycast take the 64-bit-index kernels (the
        >= 2^31-voxel path) at any volume size."""
        _check(lib().kfx_debug_force_index64(self._h, int(on)), "kfx_debug_force_index64")

    def debug_icp_band_ms(self, rank, world, reps=5) -> float:
        """Device ms of the sharded ICP's launches for band rank of world (no
        all-reduces; the tracking state is restored afterwards)."""
        ms = C.c_float()
        _check(lib().kfx_debug_icp_band_ms(self._h, int(rank), int(world), int(reps), C.byref(ms)),
               "kfx_debug_icp_band_ms")
        return float(ms.value)

    def icp_trace(self):
        """(iterations, 5) s_memrealtime stamps of the last persistent-ICP frame."""
        import numpy as np
        out = np.zeros((64, 12), np.uint64)
        n = _check(lib().kfx_get_icp_trace(self._h, out.ctypes.data_as(C.POINTER(C.c_uint64)), 64),
                   "kfx_get_icp_trace", ok=tuple(range(65)))
        return out[:n]

    def set_profiling(self, on: bool):
        _check(lib().kfx_set_profiling(self._h, int(on)), "kfx_set_profiling")

    def stage_ms(self) -> dict:
        a = (C.c_float * 5)()
        _check(lib().kfx_get_stage_ms(self._h, a), "kfx_get_stage_ms")
        return dict(zip(["preprocess", "icp", "integrate", "raycast", "total"], a[:]))

    def integrate_counts(self):
        a, b = C.c_int64(), C.c_int64()
        _check(lib().kfx_integrate_counts(self._h, C.byref(a), C.byref(b)), "kfx_integrate_counts")
        return a.value, b.value

    def integrate_stats(self) -> dict:
        """Work of the last frame's integrate: updated / coloured / visited / gathered voxels."""
        a = (C.c_int64 * 8)()
        _check(lib().kfx_integrate_stats(self._h, a), "kfx_integrate_stats")
        return dict(zip(["updated", "colored", "visited", "gathered", "wave_batches"], a[:5]))

    def raycast_stats(self) -> dict:
        """Work of the last frame's raycast (re-run, nothing written)."""
        a = (C.c_int64 * 8)()
        _check(lib().kfx_raycast_stats(self._h, a), "kfx_raycast_stats")
        return dict(zip(["rays", "skip_lookups", "skipped_samples", "blocked_lookups", "batches",
                         "normal_candidates", "ref_uniq_voxels", "ref_reads"], a[:8]))

    def volume_checksum(self) -> tuple:
        """(hash sum mod 2^64, voxels with weight > 0) over the owned slices."""
        out = (C.c_uint64 * 2)()
        _check(lib().kfx_volume_checksum(self._h, out), "kfx_volume_checksum")
        return int(out[0]), int(out[1])

    def render(self, kind: str = "phong") -> np.ndarray:
        """getRenderMap(PHONG / NORMAL): (H, W, 3) uint8 from the last raycast."""
        out = np.empty((self.intr.height, self.intr.width, 3), np.uint8)
        _check(lib().kfx_render(self._h, 0 if kind == "phong" else 1, out.ctypes.data_as(C.POINTER(C.c_uint8))),
               "kfx_render")
        return out

    def extract_mesh(self, cap: int = 50_000_000) -> np.ndarray:
        """Marching-cubes triangles, (N, 3, 3) float32 world coordinates (canonical order)."""
        # one call into a cap-sized buffer (the library's single-pass path;
        # np.empty pages are touched only where triangles are written)
        n = C.c_int64()
        out = np.empty((max(cap, 0), 3, 3), np.float32)
        _check(lib().kfx_extract_mesh(self._h, fptr(out) if cap > 0 else None, max(cap, 0), C.byref(n)),
               "kfx_extract_mesh")
        return _trim(out, min(n.value, max(cap, 0)))

    # ---- point cloud (kinectfusion::extracePointcloud / savePointcloud) ---
    def extract_points(self, cap: int = 10_000_000) -> np.ndarray:
        """(N, 3) float32 zero-crossing points in world coordinates (canonical order)."""
        n = C.c_int64()
        out = np.empty((max(cap, 0), 3), np.float32)
        _check(lib().kfx_extract_points(self._h, fptr(out) if cap > 0 else None, max(cap, 0), C.byref(n)),
               "kfx_extract_points")
        return _trim(out, min(n.value, max(cap, 0)))

    def extract_count(self, mesh: bool = False) -> int:
        """Points (or triangles) the volume holds, without extracting them (count pass only)."""
        n = C.c_int64()
        fn = lib().kfx_extract_mesh if mesh else lib().kfx_extract_points
        _check(fn(self._h, None, 0, C.byref(n)), "kfx_extract_mesh" if mesh else "kfx_extract_points")
        return n.value

    def set_slab_bound(self, mode: int):
        """Z-slab raycast bounded by the previous frame's model (1), off (0, default),
        or bounded without margin (2, tests); results identical."""
        _check(lib().kfx_set_slab_bound(self._h, int(mode)), "kfx_set_slab_bound")

    def set_extract_passes(self, passes: int):
        """1: single-pass extraction (default); 2: count + scan + emit passes."""
        _check(lib().kfx_set_extract_passes(self._h, int(passes)), "kfx_set_extract_passes")

    def extract_ms(self) -> dict:
        """Device ms of the last extract_points / extract_mesh: the volume pass, the offset
        scan, and the pool copy (one volume read, passes = 1) or the emit pass (passes = 2)."""
        a = (C.c_float * 3)()
        _check(lib().kfx_get_extract_ms(self._h, a), "kfx_get_extract_ms")
        n = C.c_int()
        _check(lib().kfx_get_extract_passes(self._h, C.byref(n)), "kfx_get_extract_passes")
        return {"count": a[0], "scan": a[1], "emit": a[2], "passes": n.value}

    def save_pointcloud(self, path: str, cap: int = 0):
        _check(lib().kfx_save_pointcloud(self._h, path.encode(), cap), "kfx_save_pointcloud")

    # ---- Z-slab sharding -------------------------------------------------
    def slab_info(self):
        """(zb, zn, own0, own1): stored slices [zb, zb+zn), owned [own0, own1)."""
        a = [C.c_int() for _ in range(4)]
        _check(lib().kfx_slab_info(self._h, *[C.byref(x) for x in a]), "kfx_slab_info")
        return tuple(x.value for x in a)

    def slab_frame_local(self, color: np.ndarray, depth: np.ndarray):
        """Slab frame up to the local raycast (kfx_slab_frame_local): returns this
        slab's (keys (n,) u32, payload (4, n) u32) for an exchange by the caller."""
        color = np.ascontiguousarray(color, np.uint8)
        d = np.ascontiguousarray(depth, np.float32)
        n = self.intr.width * self.intr.height
        keys = np.zeros(n, np.uint32)
        pay = np.zeros((4, n), np.uint32)
        u32p = C.POINTER(C.c_uint32)
        _check(lib().kfx_slab_frame_local(self._h, u8ptr(color), fptr(d), keys.ctypes.data_as(u32p),
                                          pay.ctypes.data_as(u32p)), "kfx_slab_frame_local")
        return keys, pay

    def slab_frame_finish(self, payload: np.ndarray) -> int:
        """Finish the frame from the MAX-combined payload (kfx_slab_frame_finish)."""
        pay = np.ascontiguousarray(payload, np.uint32)
        rc = lib().kfx_slab_frame_finish(self._h, pay.ctypes.data_as(C.POINTER(C.c_uint32)))
        return _check(rc, "kfx_slab_frame_finish", ok=(KFX_OK, KFX_TRACKING_LOST))

    def slice_work(self, color: np.ndarray, depth: np.ndarray) -> np.ndarray:
        """(Z,) int64: per global slice, the estimated integrate cost of this
        frame at the first frame's pose (kfx_slice_work; slab balancing)."""
        color = np.ascontiguousarray(color, np.uint8)
        d = np.ascontiguousarray(depth, np.float32)
        out = np.zeros(self.dims[2], np.int64)
        _check(lib().kfx_slice_work(self._h, u8ptr(color), fptr(d), i64ptr(out)), "kfx_slice_work")
        return out

    def slice_work_at(self, color: np.ndarray, depth: np.ndarray, cam_pose=None):
        """(work, cover, updated), each (Z,) int64 (kfx_slice_work_at): the
        frame seen from cam_pose (4x4 camera-to-world; None = identity)."""
        color = np.ascontiguousarray(color, np.uint8)
        d = np.ascontiguousarray(depth, np.float32)
        work, cover, upd = (np.zeros(self.dims[2], np.int64) for _ in range(3))
        cam = None if cam_pose is None else C.byref(Pose.from_matrix(cam_pose))
        _check(lib().kfx_slice_work_at(self._h, u8ptr(color), fptr(d), cam, i64ptr(work), i64ptr(cover),
                                       i64ptr(upd)), "kfx_slice_work_at")
        return work, cover, upd

    def slice_work_parts(self, color: np.ndarray, depth: np.ndarray):
        """(cover, updated), each (Z,) int64 (kfx_slice_work_parts): voxel
        slots integrate's waves visit, and voxels whose depth test passes."""
        color = np.ascontiguousarray(color, np.uint8)
        d = np.ascontiguousarray(depth, np.float32)
        cover = np.zeros(self.dims[2], np.int64)
        upd = np.zeros(self.dims[2], np.int64)
        _check(lib().kfx_slice_work_parts(self._h, u8ptr(color), fptr(d), i64ptr(cover), i64ptr(upd)),
               "kfx_slice_work_parts")
        return cover, upd

    def comm_init(self, uid: bytes):
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        _check(lib().kfx_comm_init(self._h, buf), "kfx_comm_init")

    # ---- frames / volume -------------------------------------------------
    def frame_maps(self, which: int, level: int):
        li = self.intr.level(level)
        d = np.zeros((li.height, li.width), np.float32)
        v = np.zeros((li.height, li.width, 3), np.float32)
        n = np.zeros_like(v)
        _check(lib().kfx_get_frame_maps(self._h, which, level, fptr(d), fptr(v), fptr(n)), "kfx_get_frame_maps")
        return d, v, n

    def set_frame_maps(self, which: int, level: int, vmap: np.ndarray, nmap: np.ndarray):
        v = np.ascontiguousarray(vmap, np.float32)
        n = np.ascontiguousarray(nmap, np.float32)
        _check(lib().kfx_set_frame_maps(self._h, which, level, fptr(v), fptr(n)), "kfx_set_frame_maps")

    def download_tsdf(self) -> np.ndarray:
        """Reference 8-byte records as a structured array (x fastest)."""
        rec = np.zeros(self.nvox, dtype=np.dtype([("tsdf", "<i2"), ("weight", "<i2"), ("rgb", "u1", 3),
                                                  ("pad", "u1")]))
        _check(lib().kfx_download_tsdf(self._h, rec.ctypes.data_as(C.c_void_p)), "kfx_download_tsdf")
        return rec

    def upload_tsdf(self, rec: np.ndarray):
        rec = np.ascontiguousarray(rec)
        assert rec.nbytes == 8 * self.nvox
        _check(lib().kfx_upload_tsdf(self._h, rec.ctypes.data_as(C.c_void_p)), "kfx_upload_tsdf")

    def volume_soa(self):
        t = np.zeros(self.nvox, np.int16)
        w = np.zeros(self.nvox, np.int16)
        c = np.zeros(4 * self.nvox, np.uint8)
        _check(lib().kfx_download_volume_soa(self._h, i16ptr(t), i16ptr(w), u8ptr(c)), "kfx_download_volume_soa")
        return t, w, c

    def download_columns(self, cols):
        """(tsdf, weight, rgb u8x4) of (x, y) columns over the owned slices, shape (n, nz)."""
        cols = np.ascontiguousarray(cols, np.int32).reshape(-1, 2)
        n = cols.shape[0]
        _, _, o0, o1 = self.slab_info()
        t = np.zeros((n, o1 - o0), np.int16)
        w = np.zeros((n, o1 - o0), np.int16)
        c = np.zeros((n, o1 - o0), np.uint32)
        _check(lib().kfx_download_columns(self._h, cols.ctypes.data_as(C.POINTER(C.c_int32)), n, i16ptr(t),
                                          i16ptr(w), c.ctypes.data_as(C.POINTER(C.c_uint32))),
               "kfx_download_columns")
        return t, w, c.view(np.uint8).reshape(n, o1 - o0, 4)

    # ---- stage seams -----------------------------------------------------
    def stage_preprocess(self, color, depth_mm):
        color = np.ascontiguousarray(color, np.uint8)
        d = np.ascontiguousarray(depth_mm, np.float32)
        _check(lib().kfx_stage_preprocess(self._h, u8ptr(color), fptr(d)), "kfx_stage_preprocess")

    def stage_icp_accumulate(self, level: int, pose: Pose) -> np.ndarray:
        s = np.zeros(27, np.int64)
        _check(lib().kfx_stage_icp_accumulate(self._h, level, C.byref(pose), i64ptr(s)), "kfx_stage_icp_accumulate")
        return s

    def stage_icp(self):
        p = Pose()
        rc = _check(lib().kfx_stage_icp(self._h, C.byref(p)), "kfx_stage_icp", ok=(KFX_OK, KFX_TRACKING_LOST))
        return rc, p

    def stage_integrate(self, vol2cam: Pose, counts: bool = True):
        a, b = C.c_int64(), C.c_int64()
        _check(lib().kfx_stage_integrate(self._h, C.byref(vol2cam), C.byref(a) if counts else None,
                                         C.byref(b) if counts else None), "kfx_stage_integrate")
        return a.value, b.value

    def stage_raycast(self, cam2vol: Pose, Rinv: np.ndarray):
        R = np.ascontiguousarray(Rinv, np.float32).reshape(9)
        _check(lib().kfx_stage_raycast(self._h, C.byref(cam2vol), fptr(R)), "kfx_stage_raycast")
