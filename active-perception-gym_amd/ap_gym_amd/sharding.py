"""Env sharding across GPUs (one process per GPU, torch.distributed).

Sub-envs are independent (SyncVectorEnv seeds sub-env i with seed+i and every later draw comes
from that sub-env's own streams), so rank r simply owns the contiguous block
[r*N/W, (r+1)*N/W) and seeds it with an env offset: no data-path collective is needed and the
union of the shards is bit-identical to one unsharded env.

`ShardedVectorEnv(..., gather=True)` additionally reassembles the batched step outputs (everything
except the per-reset map observation) on every rank with one all-gather over a packed byte row per
env — RCCL over xGMI on MI355X, gloo on CPU — for consumers that need the full batch.
"""

from __future__ import annotations

from typing import Callable


def shard_bounds(num_envs_total: int, rank: int, world: int) -> tuple[int, int]:
    if num_envs_total % world:
        raise ValueError(f"num_envs ({num_envs_total}) must be divisible by the world size ({world})")
    n = num_envs_total // world
    return rank * n, n


# packed per-env row: (name, bytes per env) in order; lidar width depends on the beam count
def _row_layout(beams: int):
    return [("lidar", 4 * beams), ("odometry", 8), ("time_step", 4), ("reward", 8), ("base_reward", 4),
            ("target", 8), ("loss", 4), ("terminated", 1), ("truncated", 1), ("info_mask", 1)]


class ShardedVectorEnv:
    def __init__(self, make_local: Callable[..., object], num_envs_total: int, rank: int, world: int,
                 beams: int, gather: bool = False, group=None):
        self.rank, self.world, self.gather, self.group = rank, world, gather, group
        self.offset, self.local_num_envs = shard_bounds(num_envs_total, rank, world)
        self.num_envs = num_envs_total
        self.env = make_local(num_envs=self.local_num_envs, env_offset=self.offset)
        self._layout = _row_layout(beams)
        self._row = sum(b for _, b in self._layout)
        self._row += (-self._row) % 8
        self._send = self._recv = None

    def reset(self, *, seed=None, options=None):
        return self.env.reset(seed=seed, options=options)

    def _pack(self, fields: dict):
        import torch

        n = self.local_num_envs
        if self._send is None:
            dev = fields["lidar"].device
            self._send = torch.zeros((n, self._row), dtype=torch.uint8, device=dev)
            self._recv = torch.zeros((self.world * n, self._row), dtype=torch.uint8, device=dev)
        o = 0
        for name, nb in self._layout:
            self._send[:, o:o + nb] = fields[name].contiguous().view(torch.uint8).reshape(n, nb)
            o += nb
        return self._send

    def _unpack(self, buf):
        import torch

        dtypes = {"reward": torch.float64, "terminated": torch.bool, "truncated": torch.bool,
                  "info_mask": torch.bool}
        out, o = {}, 0
        for name, nb in self._layout:
            dt = dtypes.get(name, torch.float32)
            v = buf[:, o:o + nb].contiguous().view(dt)
            out[name] = v.reshape(buf.shape[0], -1) if name in ("lidar", "odometry", "target") else v.reshape(-1)
            o += nb
        return out

    def all_gather(self, fields: dict) -> dict:
        import torch.distributed as dist

        send = self._pack(fields)
        if dist.get_backend(self.group) == "nccl":
            dist.all_gather_into_tensor(self._recv, send, group=self.group)
        else:
            dist.all_gather(list(self._recv.chunk(self.world)), send, group=self.group)
        return self._unpack(self._recv)

    def step(self, action):
        obs, rew, term, trunc, info = self.env.step(action)
        if not self.gather:
            return obs, rew, term, trunc, info
        full = self.all_gather({"lidar": obs["lidar"], "odometry": obs["odometry"], "time_step": obs["time_step"],
                                "reward": rew, "base_reward": info["base_reward"],
                                "target": info["prediction"]["target"], "loss": info["prediction"]["loss"],
                                "terminated": term, "truncated": trunc, "info_mask": info["_base_reward"]})
        gobs = {"lidar": full["lidar"], "odometry": full["odometry"], "time_step": full["time_step"]}
        ginfo = {"base_reward": full["base_reward"], "_base_reward": full["info_mask"],
                 "prediction": {"target": full["target"], "loss": full["loss"]}, "local_obs": obs}
        return gobs, full["reward"], full["terminated"], full["truncated"], ginfo

    def close(self):
        self.env.close()
