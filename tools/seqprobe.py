import sys; sys.path.insert(0,'/root/repo')
import numpy as np, torch
import vo_amd
from r7020e_visual_odometry_amd import vo, synthetic as syn
n=64
L,R,gt=syn.sequence(n)
P1,P2=syn.calib()
ctx=vo.Context(375,1242,16,calib=vo.calib_from(P1,P2))
dl=torch.from_numpy(L).cuda(); dr=torch.from_numpy(R).cuda()
fs=L[0].size
outs=np.concatenate([ctx.step_batch_dev(dl.data_ptr()+b*fs, dr.data_ptr()+b*fs, 16) for b in range(0,n,16)])
for i,o in enumerate(outs):
    print(i, o['status'], o['n_left'], o['n_stereo'], o['n_tracked'], o['n_inliers'], np.round(o['pose'][:3,3],2), np.round(gt[i][:3,3],2))
