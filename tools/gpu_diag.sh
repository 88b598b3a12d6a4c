#!/bin/bash
# (1) load order of torch's bundled HIP runtime vs liburgym.so's /opt/rocm one; (2) the box-box index reproducer
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/diag
echo "F: raw CDLL + init, then import torch"
timeout -k 5 120 python -c "
import ctypes; L=ctypes.CDLL('urgym_amd/_lib/liburgym.so'); L.urgym_create.restype=ctypes.c_void_p
h=L.urgym_create(0,4,0,64,1,0); print('handle', bool(h))
import torch; print('torch after raw lib:', torch.cuda.is_available())" 2>&1 | grep -v amdgpu.ids
echo "G: Sim via _native (torch loaded first), then torch"
timeout -k 5 120 python -c "
import sys; sys.path.insert(0,'.')
from urgym_amd._native import Sim
s=Sim(0,4); s.reset()
import torch; print('torch after Sim:', torch.cuda.is_available(), torch.zeros(1,device='cuda').device)" 2>&1 | grep -v amdgpu.ids
cd tools/micro && timeout -k 5 60 ./bbidx
