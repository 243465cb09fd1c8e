import sys, os
sys.path.insert(0, '.'); sys.path.insert(0, 'oracle')
order = sys.argv[1]
if order == "torch_first":
    import torch
    torch.cuda.init()
    print("torch devices", torch.cuda.device_count())
import vo_amd
from r7020e_visual_odometry_amd import vo, synthetic as syn
import numpy as np
L, R = syn.stereo_pair(syn.SEED_BASE + 7)
ctx = vo.Context(375, 1242, 2)
k, d = ctx.sift(L)
print("sift ok", len(k))
import oracle
kr, dr = oracle.sift(L)
print("equal", len(k) == len(kr) and np.array_equal(d, dr))
if order != "torch_first":
    import torch
    print("torch devices", torch.cuda.device_count())
    x = torch.zeros(10, device="cuda")
    print("torch ok", float(x.sum()))
# torch tensors through libvo
import torch
Lb, Rb = syn.independent_pairs(2)
dl = torch.from_numpy(Lb).cuda(); dr_ = torch.from_numpy(Rb).cuda(); torch.cuda.synchronize()
st = ctx.sift_match_batch_dev(dl.data_ptr(), dr_.data_ptr(), 2)
print("batch stats", st)
with open("/proc/self/maps") as f:
    libs = sorted({l.split()[-1] for l in f if "amdhip64" in l})
print("hip runtimes mapped:", libs)
