"""Env-batch data parallelism across the GPUs of one node (one process per GPU).

Environments are independent, so the path shards with no exchange inside a
step: rank r owns the contiguous env-id range [r*n, (r+1)*n), seeds env i's
MT19937 stream with seed + i (results are independent of the world size), and
runs its shard on its own GPU.  The only collective is the per-step all-gather
of the returns (obs | final_obs | reward | terminated | truncated | is_success |
substeps, ReturnGather) for a consumer that needs the whole batch (a central
policy): torch.distributed backend "nccl" is RCCL over xGMI on MI355X; tests use
"gloo" on CPU.
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


FIELDS = ("obs", "final_obs", "reward", "terminated", "truncated", "success", "substeps")


class ReturnGather:
    """The per-step all-gather of a rank's returns for a consumer of the whole batch (a central policy, an autoreset
    learner): obs | final_obs | reward | terminated | truncated | is_success | substeps (final_obs is the
    terminal observation of an autoreset env, env_*'s step() return before the reset) packed into ONE preallocated FP64
    row per env and moved with a single dist.all_gather_into_tensor (RCCL over xGMI with the nccl backend, straight
    from HBM; gloo through host memory) into a preallocated global buffer.  gather() returns views of that buffer in
    global env-id order (rank-major): no per-step allocation, list or concatenation."""

    def __init__(self, n_local, obs_dim, device, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.o = obs_dim
        self.width = 2 * obs_dim + 5
        host = dist.get_backend(group) == "gloo"
        dev = torch.device("cpu") if host else torch.device(device)
        self.send = torch.zeros(n_local, self.width, dtype=torch.float64, device=dev)
        self.recv = torch.zeros(self.world * n_local, self.width, dtype=torch.float64, device=dev)
        o = obs_dim
        self.views = {"obs": self.recv[:, :o], "final_obs": self.recv[:, o:2 * o], "reward": self.recv[:, 2 * o],
                      "terminated": self.recv[:, 2 * o + 1], "truncated": self.recv[:, 2 * o + 2],
                      "success": self.recv[:, 2 * o + 3], "substeps": self.recv[:, 2 * o + 4]}

    def gather(self, obs, final_obs, reward, terminated, truncated, success, substeps):
        o, b = self.o, self.send
        b[:, :o].copy_(obs)
        b[:, o:2 * o].copy_(final_obs)
        b[:, 2 * o].copy_(reward)
        b[:, 2 * o + 1].copy_(terminated)
        b[:, 2 * o + 2].copy_(truncated)
        b[:, 2 * o + 3].copy_(success)
        b[:, 2 * o + 4].copy_(substeps)
        dist.all_gather_into_tensor(self.recv, b, group=self.group)
        return self.views

    def decoded(self):
        """the last gather with the flags as bool and the substep counts as int32 (host-side consumers)"""
        v = self.views
        return {"obs": v["obs"], "final_obs": v["final_obs"], "reward": v["reward"], "terminated": v["terminated"] > 0.5,
                "truncated": v["truncated"] > 0.5, "success": v["success"] > 0.5, "substeps": v["substeps"].to(torch.int32)}


def gather_returns(obs, reward, terminated, truncated, final_obs=None, success=None, substeps=None, group=None,
                   as_tuple=False):
    """One-off form of ReturnGather (tests, scripts): every field gathered, missing ones as zeros; returns the
    decoded dict in global env-id order -- or, with as_tuple=True, the round-3 form (obs, reward, terminated,
    truncated) that earlier callers unpack.  Per-step loops keep one ReturnGather instead."""
    n, o = obs.shape
    g = ReturnGather(n, o, obs.device, group)
    z = torch.zeros(n, dtype=torch.float64)
    g.gather(obs, obs if final_obs is None else final_obs, reward, terminated, truncated, z if success is None else success,
             z if substeps is None else substeps)
    d = g.decoded()
    if as_tuple:
        return d["obs"], d["reward"], d["terminated"], d["truncated"]
    return d
