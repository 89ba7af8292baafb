import sys, numpy as np
sys.path[:0] = ['slam-kinectfusion_amd', 'oracle']
import oracle as O
from kfx import KinectFusion, synth
from kfx.abi import Intrinsics, Pose, default_params
intr = synth.Intrinsics.qvga(); I = Intrinsics.from_any(intr)
bgr, dep, gt = synth.sequence(3, intr, noise=True, dropout=0.01)
p = default_params(dims=128, range_m=2.048)
kf = KinectFusion(I, p)
vol = O.Volume((128,)*3, (2.048,)*3)
for k in range(3):
    d = dep[k].astype(np.float32)
    kf.stage_preprocess(bgr[k], d)
    ds,_,_ = O.preprocess(d, I, p)
    v2c = O.pose_mul(O.pose_inv(Pose.from_matrix(gt[k])), p.volu_pose)
    g = kf.stage_integrate(v2c)
    g2 = kf.integrate_counts()
    o = O.integrate(vol, p.volu_trun_dist, I, v2c, ds[0], bgr[k])
    t,w,c = kf.volume_soa()
    print(k, "gpu", g, "again", g2, "oracle", o, "tsdf eq", np.array_equal(t, vol.tsdf), (t!=vol.tsdf).sum(), "w eq", np.array_equal(w, vol.weight), "rgb eq", np.array_equal(c, vol.rgb), "upd", (w>0).sum(), (vol.weight>0).sum())
