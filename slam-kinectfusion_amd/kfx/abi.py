"""ctypes mirror of include/kfx.h structs (shared by the product binding and the
test oracle's binding — plain data layout, no behaviour)."""
from __future__ import annotations

import ctypes as C

import numpy as np

KFX_MAX_LEVELS = 4
KFX_OK = 0
KFX_TRACKING_LOST = 1
KFX_FRAME_CUR = 0
KFX_FRAME_PREV = 1


class Intrinsics(C.Structure):
    _fields_ = [("width", C.c_int), ("height", C.c_int), ("fx", C.c_float), ("fy", C.c_float),
                ("cx", C.c_float), ("cy", C.c_float)]

    @staticmethod
    def from_any(x) -> "Intrinsics":
        if isinstance(x, Intrinsics):
            return x
        return Intrinsics(int(x.width), int(x.height), float(x.fx), float(x.fy), float(x.cx), float(x.cy))

    def level(self, l: int) -> "Intrinsics":
        """Intrinsics::level (types.hpp:18-28), float32 arithmetic."""
        if l == 0:
            return Intrinsics(self.width, self.height, self.fx, self.fy, self.cx, self.cy)
        s = np.float32(0.5) ** np.float32(l)
        f32 = np.float32
        return Intrinsics(self.width >> l, self.height >> l, float(f32(self.fx) * s), float(f32(self.fy) * s),
                          float((f32(self.cx) + f32(0.5)) * s - f32(0.5)),
                          float((f32(self.cy) + f32(0.5)) * s - f32(0.5)))


class Pose(C.Structure):
    _fields_ = [("R", C.c_float * 9), ("t", C.c_float * 3)]

    @staticmethod
    def from_matrix(m) -> "Pose":
        m = np.asarray(m, dtype=np.float32)
        p = Pose()
        for i in range(3):
            for j in range(3):
                p.R[3 * i + j] = float(m[i, j])
            p.t[i] = float(m[i, 3])
        return p

    def matrix(self) -> np.ndarray:
        m = np.eye(4, dtype=np.float32)
        m[:3, :3] = np.array(self.R[:], dtype=np.float32).reshape(3, 3)
        m[:3, 3] = np.array(self.t[:], dtype=np.float32)
        return m

    @staticmethod
    def identity() -> "Pose":
        return Pose.from_matrix(np.eye(4))


class Params(C.Structure):
    _fields_ = [("pyramid_height", C.c_int), ("dfilter_dist", C.c_float), ("bfilter_kernel_size", C.c_int),
                ("bfilter_spatial_sigma", C.c_float), ("bfilter_color_sigma", C.c_float),
                ("icp_dist_threshold", C.c_float), ("icp_angle_threshold", C.c_float),
                ("icp_iter_count", C.c_int * KFX_MAX_LEVELS), ("volu_range", C.c_float * 3),
                ("volu_dims", C.c_int * 3), ("volu_trun_dist", C.c_float), ("volu_pose", Pose),
                ("tsdf_max_weight", C.c_int), ("min_pose_move", C.c_float)]


def default_params(dims: int = 512, range_m: float = 3.0) -> Params:
    """kinectfuison_params::default_params (kinectfusion.cpp:167-190), with the
    volume size/range overridable (BASELINE configs use 4 mm / 2 mm voxels)."""
    f32 = np.float32
    p = Params()
    p.pyramid_height = 3
    p.bfilter_color_sigma = 10.0
    p.bfilter_spatial_sigma = 10.0
    p.bfilter_kernel_size = 5
    p.dfilter_dist = 5.0
    p.icp_angle_threshold = 30.0
    p.icp_dist_threshold = 0.015
    for i, v in enumerate([4, 5, 10, 0]):
        p.icp_iter_count[i] = v
    for i in range(3):
        p.volu_dims[i] = dims
        p.volu_range[i] = range_m
    # 2.1f * range / dims in float (kinectfusion.cpp:183)
    p.volu_trun_dist = float(f32(2.1) * f32(range_m) / f32(dims))
    pose = np.eye(4)
    pose[:3, 3] = [float(-f32(range_m) / f32(2)), float(-f32(range_m) / f32(2)), 0.5]
    p.volu_pose = Pose.from_matrix(pose)
    p.min_pose_move = 0.008
    p.tsdf_max_weight = 64
    return p


def fptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def u8ptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_uint8))


def u16ptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_uint16))


def i16ptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_int16))


def i32ptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_int32))


def i64ptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_int64))
