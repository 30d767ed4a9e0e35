"""Closed loop (pair step + k_dynw) per-iteration timings and state sanity."""
import os, sys, time, ctypes as C
import numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."),
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lqr-obstacles_amd")]
import torch
import lqro
import bench
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
N = 1024
x, vg = lqro.synthetic_swarm(N)
g = lqro.synthesize_gains()
ctx = lqro.Context(lqro.config(N, 100, 100))
ctx.set_gains(g["A"], g["B"], g["L"], g["E"])
d_x = torch.from_numpy(x).to(dev); d_vg = torch.from_numpy(vg).to(dev)
d_newv = torch.zeros((N, 3), dtype=torch.float64, device=dev)
stream = torch.cuda.current_stream(dev)
def step():
    ctx.step_device(d_x.data_ptr(), d_vg.data_ptr(), d_newv.data_ptr(), stream.cuda_stream)
for k in range(3):
    step(); torch.cuda.synchronize()
    print("pre", k, ctx.timings(), ctx.stats()["inside"], flush=True)
out = bench.closed_loop(lqro, torch, dev, stream, step, ctx, d_x, d_newv, g, 0, N, 1)
print(out)
xs = d_x.cpu().numpy(); nv = d_newv.cpu().numpy(); vgn = d_vg.cpu().numpy()
print("finite", np.isfinite(xs).all(), np.isfinite(nv).all(), "max|v|", np.abs(xs[:, 3:6]).max(), "max|newv|", np.abs(nv).max())
for k in range(3):
    t0 = time.perf_counter(); step(); torch.cuda.synchronize()
    print("post", k, (time.perf_counter() - t0) * 1e3, ctx.timings(), ctx.stats(), flush=True)
