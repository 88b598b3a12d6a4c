"""Env-batch data parallelism across the GPUs of one node (one process per GPU).

Environments are independent, so the path shards with no exchange inside a
step: rank r owns the contiguous env-id range [r*n, (r+1)*n), seeds env i's
MT19937 stream with seed + i (results are independent of the world size), and
runs its shard on its own GPU.  The only collective is the per-step all-gather
of the returns (obs | reward | terminated | truncated) for a consumer that
needs the whole batch (a central policy): torch.distributed backend "nccl" is
RCCL over xGMI on MI355X; tests use "gloo" on CPU.
"""
import os
import socket
import subprocess
import sys

import torch
import torch.distributed as dist


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_command(nproc, script, argv, port):
    """torch.distributed.run command line: one process per GPU of this node, rendezvous on 127.0.0.1"""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), script] + list(argv)


def spawn_ranks(nproc, script, argv, port=None):
    """Run `script argv` as nproc ranks (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set by torch.distributed.run)
    in child processes and return their exit code.  The caller must not have touched the GPU: the ranks are
    children, never an exec of the caller."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this driver (RCCL)
    cmd = launch_command(nproc, script, argv, port or free_port())
    return subprocess.call(cmd, env=env)


def shard(total_envs, world_size, rank):
    """(env_offset, n_local) of rank's contiguous shard; total must divide evenly."""
    if total_envs % world_size:
        raise ValueError(f"total_envs {total_envs} not divisible by world_size {world_size}")
    n = total_envs // world_size
    return rank * n, n


def pack_returns(obs, reward, terminated, truncated):
    """One contiguous FP64 [n, obs_dim + 3] buffer per step -> a single all-gather."""
    n, o = obs.shape
    buf = torch.empty(n, o + 3, dtype=torch.float64, device=obs.device)
    buf[:, :o] = obs
    buf[:, o] = reward
    buf[:, o + 1] = terminated.to(torch.float64)
    buf[:, o + 2] = truncated.to(torch.float64)
    return buf


def gather_returns(obs, reward, terminated, truncated, group=None):
    """All-gather every rank's returns; result is in global env-id order (rank-major).  RCCL gathers HBM
    buffers directly; under gloo (CPU tests, single-GPU rehearsals) the buffer goes through host memory."""
    buf = pack_returns(obs, reward, terminated, truncated)
    if dist.get_backend(group) == "gloo" and buf.is_cuda:
        buf = buf.cpu()
    world = dist.get_world_size(group)
    out = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(out, buf, group=group)
    full = torch.cat(out, 0)
    o = obs.shape[1]
    return full[:, :o], full[:, o], full[:, o + 1] > 0.5, full[:, o + 2] > 0.5
