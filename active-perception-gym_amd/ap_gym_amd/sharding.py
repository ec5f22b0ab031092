"""Env sharding across GPUs (one process per GPU, torch.distributed).

Sub-envs are independent, so rank r owns the contiguous block [r*N/W, (r+1)*N/W):
  * LIDAR ids: SyncVectorEnv seeds sub-env i with seed+i and every later draw comes from that
    sub-env's own streams, so the shard simply resets with env_offset = r*N/W;
  * image ids: the vector env draws each batch from one stream, so every shard draws the whole
    batch of num_envs_total (a few microseconds on device) and keeps its slice (env_offset).
Either way the union of the shards is bit-identical to one unsharded env and no data-path
collective is needed (weak scaling).

`ShardedVectorEnv(..., gather=True)` additionally reassembles the batched outputs on every rank (after
reset and after every step) with one all-gather over a row of bytes per env — RCCL over xGMI on MI355X,
gloo on CPU — for consumers that need the full batch (the north star's obs/reward reassembly):
  LIDAR  the local env is built with packed_outputs=True: its step kernel writes every per-env output
         (lidar, odometry, time_step, reward, terminated, truncated, base_reward, target, loss, info mask,
         map_idx, reset mask, and stats / weight when logged / sparse) straight into one [N, row] buffer
         (lidar_env.lidar_output_row_layout), which is the all-gather's send buffer as is, and the gathered
         fields are strided views of the receive buffer: no packing or unpacking copies.  The per-reset map
         observation (4*H*W bytes per env) and the per-step stats history stay sharded: they are returned
         as info["local_obs"] / the local env's buffers.
  image  likewise packed_outputs=True: the fused step kernel writes reward, loss, glimpse, glimpse position, time step,
         base reward, target and the episode statistics into the row (image_env.image_output_row_layout);
         info["index"] and the localization target glimpse change only with the batch, so they are gathered on
         reset and autoreset steps only, and terminated / truncated are the same for the whole batch (episodes
         end together), so they are not gathered at all
(image_classification.py:117-151 and image_localization.py:131-181 are the outputs gathered).
`sub_batches=S` (with gather=True and packed rows) overlaps the all-gather with the steps: each rank's envs form S
sub-envs, sub-batch h of rank r holding global envs [(h*W + r)*m, +m) (m = N / (W*S)), so sub-batch h's all-gather
fills the contiguous rows [h*W*m, (h+1)*W*m) of the receive buffer and the gathered batch stays in global env order.
Each sub-env steps, then its gather is issued at once (RCCL: asynchronously on RCCL's stream, which waits for that
step's kernel only), so RCCL moves sub-batch h's rows while sub-batch h+1's step kernel runs; the current stream
waits for every gather before step() returns.  Bit-identical to S = 1 (the sub-envs are the same envs, seeded by
their global ids; image sub-envs draw the whole batch and keep their slice).  Actions are in local_env_ids order.
`gather_lag=1` (LIDAR envs with packed rows) pipelines the all-gather instead: step(a_t) launches step t, snapshots its
rows into one of two send buffers and issues their all-gather asynchronously into one of two receive buffers, then
returns the gathered outputs of step t - 1 (None on the first step after a reset; flush() returns the last step's), so
RCCL moves step t's rows while the caller works and step t + 1's kernel runs.  The outputs are those of gather=True
shifted by one call.
Envs without packed rows (e.g. test doubles) take the copying path (fields packed by copies, glimpses only with
gather_glimpse=True).  Gathered tensors are views of the receive buffer, rewritten by the next step, unless the
local env was built with copy=True (then they are cloned).
"""

from __future__ import annotations

import inspect
from typing import Callable


def shard_bounds(num_envs_total: int, rank: int, world: int) -> tuple[int, int]:
    if num_envs_total % world:
        raise ValueError(f"num_envs ({num_envs_total}) must be divisible by the world size ({world})")
    n = num_envs_total // world
    return rank * n, n


def _is_lidar(env, beams) -> bool:
    return beams is not None or hasattr(env, "lidar_beam_count")


def _accepts(fn, name: str) -> bool:
    try:
        ps = inspect.signature(fn).parameters.values()
    except (TypeError, ValueError):
        return False
    return any(p.name == name or p.kind == inspect.Parameter.VAR_KEYWORD for p in ps)


def _row_spec(env, beams, gather_glimpse: bool):
    """(name, dtype, per-env shape) of the gathered fields of `env`'s torch step outputs (copying path)."""
    import torch

    f32, f64, b8, i32, i64 = torch.float32, torch.float64, torch.bool, torch.int32, torch.int64
    if _is_lidar(env, beams):
        b = env.lidar_beam_count if beams is None else beams
        return [("lidar", f32, (b,)), ("odometry", f32, (2,)), ("time_step", f32, ()), ("reward", f64, ()),
                ("base_reward", f32, ()), ("target", f32, (2,)), ("loss", f32, ()), ("terminated", b8, ()),
                ("truncated", b8, ()), ("info_mask", b8, ())]
    from . import _native as N

    loc = env.kind == N.APG_IMAGE_LOCALIZE
    spec = [("glimpse_pos", f32, (2,)), ("time_step", f32, ()), ("reward", f64, ()), ("base_reward", f32, ()),
            ("target", f32, (2,)) if loc else ("target", i32, ()), ("loss", f32 if loc else f64, ()),
            ("index", i64, ()), ("terminated", b8, ()), ("truncated", b8, ())]
    if gather_glimpse:
        g = tuple(env.single_observation_space["glimpse"].shape)
        spec.append(("glimpse", f32, g))
        if loc:
            spec.append(("target_glimpse", f32, g))
    return spec


def _nbytes(dtype, shape) -> int:
    import torch

    n = torch.empty((), dtype=dtype).element_size()
    for s in shape:
        n *= int(s)
    return n


class ShardedVectorEnv:
    """One rank's shard of a vector env (`make_local(num_envs=, env_offset=)` builds it; image envs also
    take num_envs_total=; LIDAR envs get packed_outputs=True when gathering and make_local accepts it) plus
    the optional all-gather of the outputs."""

    def __init__(self, make_local: Callable[..., object], num_envs_total: int, rank: int, world: int,
                 beams: int | None = None, gather: bool = False, group=None, gather_glimpse: bool = False,
                 time_gather: bool = False, sub_batches: int = 1, gather_lag: int = 0):
        self.rank, self.world, self.gather, self.group = rank, world, gather, group
        self.gather_lag = int(gather_lag)
        if self.gather_lag not in (0, 1):
            raise ValueError("gather_lag must be 0 or 1")
        if self.gather_lag and (not gather or sub_batches != 1):
            raise ValueError("gather_lag=1 pipelines the all-gather: it needs gather=True and sub_batches=1")
        self.offset, self.local_num_envs = shard_bounds(num_envs_total, rank, world)
        self.num_envs = num_envs_total
        self.sub_batches = S = int(sub_batches)
        if S < 1:
            raise ValueError("sub_batches must be >= 1")
        if S > 1 and not gather:
            raise ValueError("sub_batches > 1 overlaps the all-gather with the steps: it needs gather=True")
        if num_envs_total % (world * S):
            raise ValueError(f"num_envs ({num_envs_total}) must be divisible by world size x sub_batches ({world * S})")
        # sub-batch h of rank r: global envs [(h*W + r)*m, +m), m = N / (W*S), so the all-gather of sub-batch h fills
        # rows [h*W*m, (h+1)*W*m) of the receive buffer and the gathered batch is in global env order
        self.sub_num_envs = m = num_envs_total // (world * S)
        self.sub_offsets = [self.offset] if S == 1 else [(h * world + rank) * m for h in range(S)]
        kw = {"packed_outputs": True} if gather and _accepts(make_local, "packed_outputs") else {}
        self.envs = [make_local(num_envs=m, env_offset=o, **kw) for o in self.sub_offsets]
        self.env = self.envs[0]
        self._lidar = _is_lidar(self.env, beams)
        self._packed = gather and getattr(self.env, "output_rows", None) is not None
        if S > 1 and not self._packed:
            raise ValueError("sub_batches > 1 needs envs with packed output rows (make_local(packed_outputs=True))")
        self._spec = _row_spec(self.env, beams, gather_glimpse)
        self._row = sum(_nbytes(dt, sh) for _, dt, sh in self._spec)
        self._row += (-self._row) % 8
        self._send = self._recv = None
        self._views = None
        self._index_full = None  # image envs: the gathered info["index"] (changes only with the batch)
        self._done_full = None  # image envs: gathered terminated / truncated / sparse weight constants
        self._tg_full = None  # image localization: the gathered target glimpses (change only with the batch)
        self._inv_full = self._inv2_full = None  # randomly_invert_labels: gathered inversion flags / constant 2s
        self.time_gather = time_gather
        self.gather_events: list = []  # (begin, end) torch.cuda.Event pairs around each all-gather
        if self.gather_lag and not (self._packed and self._lidar):
            raise ValueError("gather_lag=1 needs LIDAR envs with packed output rows (make_local(packed_outputs=True))")
        self._lag = None  # gather_lag: ([send] * 2, [recv] * 2, [views] * 2), allocated on the first step
        self._pending = None  # gather_lag: (all-gather work or None, buffer index) of the last step
        self._lag_t = 0

    # ------------------------------------------------------------------ collectives
    def _all_gather_into(self, recv, send, async_op: bool = False):
        """All-gather of `send` ([n, ...]) into `recv` ([world * n, ...]): RCCL in place (async_op: on RCCL's stream,
        after the work queued so far on the current stream; returns the work to wait for), gloo through host buffers
        (CPU tests, or several ranks sharing one GPU; always synchronous, returns None)."""
        import torch
        import torch.distributed as dist

        if dist.get_backend(self.group) == "nccl":
            return dist.all_gather_into_tensor(recv, send, group=self.group, async_op=async_op)
        parts = [torch.empty_like(send, device="cpu") for _ in range(self.world)]
        dist.all_gather(parts, send.cpu(), group=self.group)
        recv.copy_(torch.cat(parts))
        return None

    def _part(self, full, h: int):
        """Sub-batch h's slice of a gathered buffer: rows [h*W*m, (h+1)*W*m) (the whole buffer without sub-batches)."""
        if self.sub_batches == 1:
            return full
        k = self.world * self.sub_num_envs
        return full[h * k:(h + 1) * k]

    def _gather_parts(self, full, parts):
        """All-gather each sub-batch's local part ([m, ...]) into its slice of `full` ([N, ...])."""
        for h, p in enumerate(parts):
            self._all_gather_into(self._part(full, h), p.contiguous())
        return full

    def _timing_begin(self, like):
        import torch

        if not (self.time_gather and like.is_cuda):
            return None
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
        return ev

    def _timing_end(self, ev):
        if ev is not None:
            ev[1].record()
            self.gather_events.append(ev)

    def _rows_buffer(self, send):
        """The receive buffer of the packed rows, [N, row] uint8 (allocated once)."""
        import torch

        if self._recv is None:
            self._recv = torch.zeros((self.num_envs, send.shape[1]), dtype=torch.uint8, device=send.device)
        return self._recv

    def _all_gather_rows(self, send):
        """All-gather of a [n, row] uint8 buffer into self._recv [world * n, row] (allocated once)."""
        recv = self._rows_buffer(send)
        ev = self._timing_begin(send)
        self._all_gather_into(recv, send)
        self._timing_end(ev)
        return recv

    def _row_views(self, recv) -> dict:
        if self._views is None:
            if self._lidar:
                from .lidar_env import row_views

                self._views = row_views(recv, self.env.output_layout)
            else:
                from .image_env import image_row_views

                self._views = image_row_views(recv, self.env.output_layout)
        if getattr(self.env, "copy", False):
            return {k: v.clone() for k, v in self._views.items()}
        return self._views

    def _gathered_rows(self) -> dict:
        """The packed path: gather the local envs' output rows (every sub-batch, one after the other); field views
        of the receive buffer (cloned when the local env copies its outputs)."""
        recv = self._rows_buffer(self.env.output_rows)
        ev = self._timing_begin(recv)
        self._gather_parts(recv, [e.output_rows for e in self.envs])
        self._timing_end(ev)
        return self._row_views(recv)

    def _split_step(self, action):
        """Sub-batches: each sub-env steps, then its rows' all-gather is issued at once (RCCL: async on RCCL's
        stream, which waits for that step's kernel only), so the gather of sub-batch h overlaps the step kernel of
        sub-batch h+1; the current stream waits for every gather at the end.  Returns the sub-envs' step outputs and
        the gathered row views."""
        m = self.sub_num_envs
        outs, works, recv, ev = [], [], None, None
        for h, env in enumerate(self.envs):
            outs.append(env.step({k: v[h * m:(h + 1) * m] for k, v in action.items()}))
            if recv is None:
                recv = self._rows_buffer(env.output_rows)
                ev = self._timing_begin(recv)
            works.append(self._all_gather_into(self._part(recv, h), env.output_rows, async_op=True))
        for w in works:
            if w is not None:
                w.wait()
        self._timing_end(ev)
        return outs, self._row_views(recv)

    @staticmethod
    def _parts_of(x, key=None):
        """The per-sub-batch list of a local output (a list with sub-batches, a single value without)."""
        xs = x if isinstance(x, list) else [x]
        return [v[key] for v in xs] if key is not None else xs

    def _gathered_index(self, local_index):
        """Image envs: info["index"] of the whole batch, gathered when the batch changes (reset, autoreset)."""
        import torch

        parts = self._parts_of(local_index)
        if self._index_full is None:
            self._index_full = torch.zeros(self.num_envs, dtype=torch.int64, device=parts[0].device)
        return self._gather_parts(self._index_full, parts)

    def _gathered_target_glimpse(self, local):
        """Image localization: the target glimpses of the whole batch, gathered when the batch changes (reset,
        autoreset); not part of the packed rows."""
        import torch

        parts = self._parts_of(local)
        if self._tg_full is None:
            self._tg_full = torch.zeros((self.num_envs, *parts[0].shape[1:]), dtype=parts[0].dtype,
                                        device=parts[0].device)
        return self._gather_parts(self._tg_full, parts)

    def _gathered_inverted(self, local):
        """Image envs with randomly_invert_labels: obs["inverted_label"] of the whole batch.  It is the drawn
        inversion (int32 0/1) on reset / autoreset steps -- gathered then -- and the constant 2 (int64) on every
        other step (image_classification.py:130-141), which needs no collective."""
        import torch

        parts = self._parts_of(local)
        if parts[0].dtype == torch.int64:
            if self._inv2_full is None:
                self._inv2_full = torch.full((self.num_envs,), 2, dtype=torch.int64, device=parts[0].device)
            return self._c(self._inv2_full)
        if self._inv_full is None:
            self._inv_full = torch.zeros(self.num_envs, dtype=parts[0].dtype, device=parts[0].device)
        return self._c(self._gather_parts(self._inv_full, parts))

    def _pack(self, fields: dict):
        import torch

        n = self.local_num_envs
        if self._send is None:
            dev = fields[self._spec[0][0]].device
            self._send = torch.zeros((n, self._row), dtype=torch.uint8, device=dev)
        o = 0
        for name, dt, sh in self._spec:
            nb = _nbytes(dt, sh)
            self._send[:, o:o + nb] = fields[name].to(dt).contiguous().view(torch.uint8).reshape(n, nb)
            o += nb
        return self._send

    def _unpack(self, buf):
        out, o = {}, 0
        rows = buf.shape[0]
        for name, dt, sh in self._spec:
            nb = _nbytes(dt, sh)
            out[name] = buf[:, o:o + nb].contiguous().view(dt).reshape(rows, *sh)
            o += nb
        return out

    def all_gather(self, fields: dict) -> dict:
        """The copying path: pack `fields` (the spec's), all-gather, unpack."""
        return self._unpack(self._all_gather_rows(self._pack(fields)))

    def gather_ms(self) -> float | None:
        """Mean time of the timed all-gathers so far (synchronizes), then forgets them."""
        import torch

        if not self.gather_events:
            return None
        torch.cuda.synchronize()
        ms = sum(a.elapsed_time(b) for a, b in self.gather_events) / len(self.gather_events)
        self.gather_events.clear()
        return ms

    # ------------------------------------------------------------------ API
    def _c(self, x):
        return x.clone() if getattr(self.env, "copy", False) else x

    def _image_obs(self, v: dict) -> dict:
        obs = {k: v[k] for k in ("glimpse", "glimpse_pos", "time_step", "target_glimpse") if k in v}
        return obs

    # ------------------------------------------------------------------ gather_lag=1
    def _lag_step(self, action):
        """Step t, its rows' all-gather issued asynchronously; returns step t - 1's gathered outputs (None at first)."""
        import torch

        from .lidar_env import row_views

        self.env.step(action)
        rows = self.env.output_rows
        if self._lag is None:
            send = [torch.empty_like(rows) for _ in range(2)]
            recv = [torch.zeros((self.num_envs, rows.shape[1]), dtype=torch.uint8, device=rows.device) for _ in range(2)]
            self._lag = (send, recv, [row_views(r, self.env.output_layout) for r in recv])
        send, recv, _ = self._lag
        k = self._lag_t & 1
        # the kernel of step t + 1 rewrites output_rows while this all-gather may still read: a snapshot is sent.
        # send[k] / recv[k] are free: step t - 2's gather was waited for when step t - 1's call returned it
        send[k].copy_(rows)
        ev = self._timing_begin(rows)
        work = self._all_gather_into(recv[k], send[k], async_op=True)
        self._timing_end(ev)
        prev, self._pending = self._pending, (work, k)
        self._lag_t += 1
        return None if prev is None else self._lag_result(prev)

    def _lag_result(self, pend):
        work, k = pend
        if work is not None:
            work.wait()  # (the current stream waits for RCCL's; no host synchronization)
        v = self._lag[2][k]
        if getattr(self.env, "copy", False):
            v = {key: t.clone() for key, t in v.items()}
        gobs = {"lidar": v["lidar"], "odometry": v["odometry"], "time_step": v["time_step"]}
        info = self._packed_step_info(v, None)
        del info["local_obs"]  # (the local buffers already hold the next step)
        return gobs, v["reward"], v["terminated"], v["truncated"], info

    def flush(self):
        """gather_lag=1: the gathered outputs of the last step (None when none is pending)."""
        pend, self._pending = self._pending, None
        return None if pend is None else self._lag_result(pend)

    def reset(self, *, seed=None, options=None):
        self._pending, self._lag_t = None, 0  # (gather_lag: a pending step's outputs are dropped with its episode)
        if self.sub_batches > 1:  # (lists of the sub-envs' local outputs below)
            outs = [e.reset(seed=seed, options=options) for e in self.envs]
            obs, info = [o[0] for o in outs], [o[1] for o in outs]
        else:
            obs, info = self.env.reset(seed=seed, options=options)
        if not (self.gather and self._packed):
            # the copying path gathers step outputs only (a reset has no reward / prediction fields)
            return obs, info
        v = self._gathered_rows()
        first = self._parts_of(obs)[0]
        if not self._lidar:
            gobs = self._image_obs(v)
            if "target_glimpse" in first:
                gobs["target_glimpse"] = self._c(self._gathered_target_glimpse(self._parts_of(obs, "target_glimpse")))
            if "inverted_label" in first:
                gobs["inverted_label"] = self._gathered_inverted(self._parts_of(obs, "inverted_label"))
            return gobs, {"index": self._c(self._gathered_index(self._parts_of(info, "index"))), "local_obs": obs,
                          "local_info": info}
        gobs = {"lidar": v["lidar"], "odometry": v["odometry"], "time_step": v["time_step"]}
        return gobs, {"map_idx": v["map_idx_out"], "_map_idx": v["reset_mask"], "local_obs": obs,
                      "local_info": info}

    def _packed_step_info(self, v: dict, obs: dict, local_info: dict | None = None) -> dict:
        mask = v["info_mask"]
        target = v["target"]
        if "weight" in v:  # -sparse ids
            target = {"target": target, "_target": mask, "weight": v["weight"], "_weight": mask}
        info = {"base_reward": v["base_reward"], "_base_reward": mask,
                "prediction": {"target": target, "_target": mask, "loss": v["loss"], "_loss": mask},
                "_prediction": mask, "map_idx": v["map_idx_out"], "_map_idx": v["reset_mask"], "local_obs": obs}
        if "stats" in v:  # scalar episode statistics (the per-step history stays in the local env)
            done = v["terminated"]
            names = ("avg_euclidean_distance", "avg_mse", "final_euclidean_distance", "final_mse")
            scalar = {}
            for j, name in enumerate(names):
                scalar[name] = v["stats"][j]
                scalar["_" + name] = done
            info["stats"] = {"scalar": scalar, "_scalar": done, "length": v["stats_len"]}
            info["_stats"] = done
            # the per-step history stays local (this shard's envs; with sub-batches in each sub-env's info)
            local = local_info.get("stats") if isinstance(local_info, dict) else None
            if local is not None and "vector" in local:
                info["stats"]["vector"] = local["vector"]
                info["stats"]["_vector"] = local["_vector"]
        return info

    def _packed_image_step(self, v: dict, obs, term, trunc, info, resetting: bool):
        import torch

        n = self.num_envs
        first_obs, first_info = self._parts_of(obs)[0], self._parts_of(info)[0]
        if resetting or self._index_full is None:
            self._gathered_index(self._parts_of(info, "index"))
        cls = "label_target" in v
        target = v["label_target"] if cls else v["target_out"]
        loss = v["loss_f64"] if cls else v["loss_f32"]
        # the whole batch terminates together, never truncated, and the env knows when on the host (no device
        # read: bool(term[0]) synchronized every gathered step); the gathered flags are constant tensors
        tflag = bool(getattr(self.env, "_prev_done", False)) if hasattr(self.env, "_prev_done") else bool(term[0])
        if self._done_full is None:
            dev = target.device
            self._done_full = (torch.zeros(n, dtype=torch.bool, device=dev), torch.ones(n, dtype=torch.bool, device=dev),
                               torch.zeros(n, dtype=torch.float32, device=dev),
                               torch.ones(n, dtype=torch.float32, device=dev))
        g_term = self._c(self._done_full[1 if tflag else 0])
        g_trunc = self._c(self._done_full[0])
        pt = first_info["prediction"]["target"]
        if isinstance(pt, dict):  # -sparse ids: weight = terminated as float32
            target = {"target": target, "weight": self._c(self._done_full[3 if tflag else 2])}
        ginfo = {"index": self._c(self._index_full), "base_reward": v["base_reward"],
                 "prediction": {"target": target, "loss": loss}, "local_obs": obs}
        if "stats" in first_info:  # the vector log wrapper's scalars of the whole batch from the rows; the per-step
            done = g_term  # history ("vector") stays local to this shard's envs (each sub-env's with sub-batches)
            scalar = {}
            for j, nm in enumerate(self.env._metric_names()):
                scalar[f"final_{nm}"] = v["stats"][j]
                scalar[f"_final_{nm}"] = done
                scalar[f"avg_{nm}"] = v["stats"][2 + j]
                scalar[f"_avg_{nm}"] = done
            if cls:
                scalar.update(first_correct=v["stats_idx"][0], last_incorrect=v["stats_idx"][1])
            ginfo["stats"] = {"scalar": scalar, "_scalar": done}
            if isinstance(info, dict):
                ginfo["stats"].update(vector=info["stats"]["vector"], _vector=info["stats"]["_vector"])
        gobs = self._image_obs(v)
        if "target_glimpse" in first_obs:  # gathered when the batch changed (this step's autoreset), else the last one
            if resetting or self._tg_full is None:
                self._gathered_target_glimpse(self._parts_of(obs, "target_glimpse"))
            gobs["target_glimpse"] = self._c(self._tg_full)
        if "inverted_label" in first_obs:
            gobs["inverted_label"] = self._gathered_inverted(self._parts_of(obs, "inverted_label"))
        return gobs, v["reward"], g_term, g_trunc, ginfo

    def step(self, action):
        """`action` holds this rank's envs in local order (local_env_ids: with sub-batches, sub-batch 0's envs, then
        sub-batch 1's, ...).  Gathered outputs are in global env order; local_obs (and the image envs' per-step
        stats history) are per sub-batch lists with sub-batches."""
        if self.gather_lag:
            return self._lag_step(action)
        resetting = bool(getattr(self.env, "_prev_done", False))
        if self.sub_batches > 1:
            outs, v = self._split_step(action)
            obs, term, trunc, info = [o[0] for o in outs], outs[0][2], outs[0][3], [o[4] for o in outs]
        else:
            obs, rew, term, trunc, info = self.env.step(action)
            if not self.gather:
                return obs, rew, term, trunc, info
        if self._packed:
            if self.sub_batches == 1:
                v = self._gathered_rows()
            if not self._lidar:
                return self._packed_image_step(v, obs, term, trunc, info, resetting)
            gobs = {"lidar": v["lidar"], "odometry": v["odometry"], "time_step": v["time_step"]}
            return gobs, v["reward"], v["terminated"], v["truncated"], self._packed_step_info(v, obs, info)
        if self._lidar:
            full = self.all_gather({"lidar": obs["lidar"], "odometry": obs["odometry"], "time_step": obs["time_step"],
                                    "reward": rew, "base_reward": info["base_reward"],
                                    "target": info["prediction"]["target"], "loss": info["prediction"]["loss"],
                                    "terminated": term, "truncated": trunc, "info_mask": info["_base_reward"]})
            gobs = {"lidar": full["lidar"], "odometry": full["odometry"], "time_step": full["time_step"]}
            ginfo = {"base_reward": full["base_reward"], "_base_reward": full["info_mask"],
                     "prediction": {"target": full["target"], "loss": full["loss"]}, "local_obs": obs}
            return gobs, full["reward"], full["terminated"], full["truncated"], ginfo
        target = info["prediction"]["target"]
        if isinstance(target, dict):  # -sparse ids: {"target", "weight"}
            target = target["target"]
        fields = {"glimpse_pos": obs["glimpse_pos"], "time_step": obs["time_step"], "reward": rew,
                  "base_reward": info["base_reward"], "target": target, "loss": info["prediction"]["loss"],
                  "index": info["index"], "terminated": term, "truncated": trunc}
        for k in ("glimpse", "target_glimpse"):
            if k in obs:
                fields[k] = obs[k]
        full = self.all_gather(fields)
        gobs = {k: full[k] for k in ("glimpse", "glimpse_pos", "time_step", "target_glimpse") if k in full}
        if "inverted_label" in obs:
            gobs["inverted_label"] = self._gathered_inverted(obs["inverted_label"])
        ginfo = {"index": full["index"], "base_reward": full["base_reward"],
                 "prediction": {"target": full["target"], "loss": full["loss"]}, "local_obs": obs}
        return gobs, full["reward"], full["terminated"], full["truncated"], ginfo

    @property
    def local_env_ids(self):
        """Global ids of this rank's envs in the local order of step()'s actions and the local outputs."""
        import numpy as np

        return np.concatenate([np.arange(o, o + self.sub_num_envs) for o in self.sub_offsets])

    def check_errors(self):
        for e in self.envs:
            e.check_errors()

    def close(self):
        for e in self.envs:
            e.close()
