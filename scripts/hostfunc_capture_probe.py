"""Does hipGraph capture of a host function on a forked side stream work (no RCCL)?"""
import ctypes
import sys
import torch

hip = ctypes.CDLL("libamdhip64.so")
CB = ctypes.CFUNCTYPE(None, ctypes.c_void_p)
count = [0]


@CB
def cb(_):
    count[0] += 1


variant = sys.argv[1]
x = torch.ones(1024, device="cuda")
s = torch.cuda.Stream()
c = torch.cuda.Stream()
g = torch.cuda.CUDAGraph()
with torch.cuda.stream(s):
    x.mul_(2)
    torch.cuda.synchronize()
    g.capture_begin()
    x.mul_(2)
    if variant == "side":
        c.wait_stream(s)
        with torch.cuda.stream(c):
            x.add_(1)
            r = hip.hipLaunchHostFunc(ctypes.c_void_p(c.cuda_stream), cb, None)
        s.wait_stream(c)
    else:
        r = hip.hipLaunchHostFunc(ctypes.c_void_p(s.cuda_stream), cb, None)
    x.mul_(2)
    g.capture_end()
print("captured rc", r, flush=True)
g.replay()
torch.cuda.synchronize()
print(variant, "ok", count[0], float(x[0]), flush=True)
