"""LightDarkVectorEnv — the LightDark-v0 id as one batched GPU environment.

Reference (ap_gym 0.5.0): `make_vec("LightDark-v0", N)` builds gymnasium's SyncVectorEnv over N x
ActiveRegressionLogWrapper(TimeLimit(LightDarkEnv, 50, issue_termination=True))
(ap_gym/envs/registration.py:640-647, ap_gym/envs/light_dark.py:14-155).  This class is that
composition as state in HBM plus one kernel per step (include/apgym_capi.h: apg_light_dark_*):

  reset(seed=s)   sub-env i seeded with s+i; start position uniform in [-1, 1]^2
  step(action)    NEXT_STEP autoreset; base_reward = 1 - 1e-3 |a|^2; move = project_to_unit_disc(a) * 0.15;
                  terminated when the agent leaves (-1, 1)^2 or after 50 steps
  obs             {"noisy_position": f32[N,2] = pos + N(0, 1) * (1 - brightness(pos)) * 0.3 clipped to
                   [-2, 2], "time_step": f32[N]}
  reward          float64 (SyncVectorEnv), base_reward - normalized MSE(prediction, previous position)
  info            {"base_reward", "prediction": {"target", "loss"}} with `_key` masks, and with
                  log_stats=True (the registered id) ActiveRegressionLogWrapper's episode "stats"
  sparse=True     LightDark-sparse-v0 (SparsifyWrapper per sub-env; the reference's reset of that id raises
                  KeyError('prediction') like the LIDAR ones, see lidar_env.py)

The normal draws are numpy's ziggurat over each sub-env's PCG64 stream, bit-exact on the device.
Two I/O modes as the other envs: array_backend="numpy" (default) or "torch" (device tensors, no
host synchronisation, persistent output buffers unless copy=True).
"""

from __future__ import annotations

import ctypes
from typing import Any

import numpy as np

from . import _native as N
from .loss_fn import WeightedLossFn, affine_f32, regression_loss
from .spaces import ActivePerceptionActionSpace, Box, Dict, batch_space
from .vector_env import VectorEnv

NAN_ACTION_MSG = "NaN values detected in action."
NAN_PREDICTION_MSG = "NaN values detected in prediction."


class LightDarkVectorEnv(VectorEnv):
    metadata = {"render_modes": ["rgb_array"], "render_fps": 4, "autoreset_mode": "NextStep"}
    ERROR_POLL_INTERVAL = 128  # steps between the lazy error-word copies (each costs the stream a blit + marker)
    STAT_NAMES = ("avg_euclidean_distance", "avg_mse", "final_euclidean_distance", "final_mse")

    def __init__(self, num_envs: int = 1, render_mode: str = "rgb_array", max_episode_steps: int = 50, device=None,
                 env_offset: int = 0, copy: bool = False, strict_errors: bool = False, array_backend: str = "numpy",
                 log_stats: bool = False, sparse: bool = False, render_envs=None):
        import torch

        if render_mode not in self.metadata["render_modes"]:
            raise ValueError(f"Invalid render mode: {render_mode}")
        if array_backend not in ("numpy", "torch"):
            raise ValueError("array_backend must be 'numpy' or 'torch'")
        self.num_envs = n = int(num_envs)
        self.render_mode = render_mode
        self.max_episode_steps = int(max_episode_steps)
        self.env_offset = int(env_offset)
        self.copy, self.strict_errors, self.array_backend = copy, strict_errors, array_backend
        self.log_stats, self.sparse = bool(log_stats), bool(sparse)
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.type != "cuda":
            raise ValueError("LightDarkVectorEnv runs on a GPU device (no CPU fallback)")

        # spaces (light_dark.py:48-92, time_limit.py:64-76, active_regression_env.py:55-76)
        self.single_observation_space = Dict({"noisy_position": Box(-2, 2, (2,), np.float32),
                                              "time_step": Box(-1.0, 1.0, (), np.float32)})
        self.observation_space = batch_space(self.single_observation_space, n)
        self.single_action_space = ActivePerceptionActionSpace(Box(-1, 1, (2,), np.float32),
                                                               Box(-1, 1, (2,), np.float32))
        self.action_space = batch_space(self.single_action_space, n)
        self.single_prediction_target_space = Box(-1, 1, (2,), np.float32)
        self.loss_fn = inner_loss = regression_loss(2, -1, 1)
        if self.sparse:
            self.single_prediction_target_space = Dict({"target": self.single_prediction_target_space,
                                                        "weight": Box(0, 1, (), np.float32)})
            self.loss_fn = WeightedLossFn(inner_loss)
        self.prediction_target_space = batch_space(self.single_prediction_target_space, n)

        scale, offset = affine_f32(inner_loss)
        self._cfg = N.LightDarkConfig(num_envs=n, step_limit=self.max_episode_steps, log_stats=int(self.log_stats),
                                      sparse=int(self.sparse), loss_scale=scale, loss_offset=offset)
        t, dev = torch, self.device
        self._t = T = dict(
            pos=t.zeros((n, 2), dtype=t.float32, device=dev), elapsed=t.zeros(n, dtype=t.int32, device=dev),
            flags=t.zeros(n, dtype=t.uint8, device=dev), rng=t.zeros((n, 5), dtype=t.int64, device=dev),
            stats_hist=(t.zeros((n, 2, self.max_episode_steps), dtype=t.float32, device=dev) if self.log_stats
                        else None),
            noisy_position=t.zeros((n, 2), dtype=t.float32, device=dev),
            time_step=t.zeros(n, dtype=t.float32, device=dev), reward=t.zeros(n, dtype=t.float64, device=dev),
            terminated=t.zeros(n, dtype=t.bool, device=dev), truncated=t.zeros(n, dtype=t.bool, device=dev),
            base_reward=t.zeros(n, dtype=t.float32, device=dev), target=t.zeros((n, 2), dtype=t.float32, device=dev),
            loss=t.zeros(n, dtype=t.float32, device=dev), info_mask=t.zeros(n, dtype=t.bool, device=dev),
            reset_mask=t.zeros(n, dtype=t.bool, device=dev), err=t.zeros(1, dtype=t.int32, device=dev),
            stats=t.zeros((4, n), dtype=t.float32, device=dev) if self.log_stats else None,
            stats_len=t.zeros(n, dtype=t.int32, device=dev) if self.log_stats else None,
            weight=t.zeros(n, dtype=t.float64, device=dev) if self.sparse else None)
        self._state = N.LightDarkState(*[N.ptr(T[k]) for k in ("pos", "elapsed", "flags", "rng", "stats_hist")])
        self._out = N.LightDarkOutputs(*[N.ptr(T[k]) for k in ("noisy_position", "time_step", "reward", "terminated",
                                                                "truncated", "base_reward", "target", "loss",
                                                                "info_mask", "reset_mask", "err", "stats",
                                                                "stats_len", "weight")])
        self._err_host = t.zeros(1, dtype=t.int32).pin_memory()
        self._err_event = t.cuda.Event()
        self._err_pending = False
        self._steps_since_poll = 0
        self._autoreset_host = np.zeros(n, dtype=bool)
        self._seeded = False
        self._closed = False
        self._stats_view = None
        from .render import tracked_envs

        self.render_envs = tracked_envs(render_envs, n)
        self._render_state = [dict(traj=[], pos=None, last_obs=None, last_pos=None, last_pred=None)
                              for _ in self.render_envs]

    # ------------------------------------------------------------------ properties
    @property
    def unwrapped(self):
        return self

    @property
    def prediction_space(self):
        return self.action_space["prediction"]

    @property
    def single_prediction_space(self):
        return self.single_action_space["prediction"]

    @property
    def inner_action_space(self):
        return self.action_space["action"]

    @property
    def single_inner_action_space(self):
        return self.single_action_space["action"]

    def _stream(self):
        return N.stream_handle(self.device)

    # ------------------------------------------------------------------ errors
    def _raise_error_bits(self, bits: int):
        if bits & N.APG_ERR_NAN_ACTION:
            raise ValueError(NAN_ACTION_MSG)
        if bits & N.APG_ERR_NAN_PREDICTION:
            raise ValueError(NAN_PREDICTION_MSG)

    def check_errors(self, block: bool = True):
        if block:
            import torch

            torch.cuda.synchronize(self.device)
            bits = int(self._t["err"].item())
        elif self._err_pending and self._err_event.query():
            bits = int(self._err_host.item())
            self._err_pending = False
        else:
            return
        if bits:
            self._t["err"].zero_()
            self._raise_error_bits(bits)

    def _post_launch_error_copy(self):
        if self.strict_errors:
            self.check_errors(block=True)
            return
        self._steps_since_poll += 1
        if self._err_pending or self._steps_since_poll < self.ERROR_POLL_INTERVAL:
            return
        self._steps_since_poll = 0
        self._err_host.copy_(self._t["err"], non_blocking=True)
        self._err_event.record()
        self._err_pending = True

    # ------------------------------------------------------------------ API
    def reset(self, *, seed: int | None = None, options: dict[str, Any] | None = None):
        if self._closed:
            raise RuntimeError("environment is closed")
        if seed is None and not self._seeded:
            seed = int(np.random.SeedSequence().entropy) & ((1 << 62) - 1)
        use_seed = seed is not None
        if use_seed and not isinstance(seed, (int, np.integer)):
            raise TypeError("seed must be an int (sub-env i is seeded with seed + i) or None")
        s = (int(seed) + self.env_offset) if use_seed else 0
        if s < 0 or s + self.num_envs > 2**64:
            raise ValueError("seed must be a non-negative int")
        N.check(N.lib().apg_light_dark_reset(ctypes.byref(self._cfg), ctypes.byref(self._state), s, int(use_seed),
                                             ctypes.byref(self._out), self._stream()), "apg_light_dark_reset")
        self._track_render(None)
        self._seeded = True
        self._autoreset_host[:] = False
        if self.array_backend == "numpy":
            self.check_errors(block=True)
            return self._numpy_obs(), {}
        self._post_launch_error_copy()
        return self._torch_obs(), {}

    def step(self, action):
        import torch

        if self._closed:
            raise RuntimeError("environment is closed")
        a, p = action["action"], action["prediction"]
        n = self.num_envs
        numpy_mode = self.array_backend == "numpy"
        if numpy_mode:
            if isinstance(a, torch.Tensor):
                a = a.detach().cpu().numpy()
            if isinstance(p, torch.Tensor):
                p = p.detach().cpu().numpy()
            a_np = np.ascontiguousarray(a, dtype=np.float32).reshape(n, 2)
            p_np = np.ascontiguousarray(p, dtype=np.float32).reshape(n, 2)
            active = ~self._autoreset_host
            bad_a = np.isnan(a_np).any(axis=1) & active
            bad_p = np.isnan(p_np).any(axis=1) & active
            if bad_a.any() or bad_p.any():  # first offending sub-env decides, action checked first
                i = int(np.argmax(bad_a | bad_p))
                raise ValueError(NAN_ACTION_MSG if bad_a[i] else NAN_PREDICTION_MSG)
            a_t = torch.from_numpy(a_np).to(self.device, non_blocking=True)
            p_t = torch.from_numpy(p_np).to(self.device, non_blocking=True)
        else:
            self.check_errors(block=False)
            a_t = torch.as_tensor(a, dtype=torch.float32, device=self.device).reshape(n, 2).contiguous()
            p_t = torch.as_tensor(p, dtype=torch.float32, device=self.device).reshape(n, 2).contiguous()
        N.check(N.fast().light_dark_step(N.addr(self._cfg), N.addr(self._state), a_t.data_ptr(), p_t.data_ptr(),
                                         N.addr(self._out), self._stream() or 0), "apg_light_dark_step")
        self._track_render(p_np if numpy_mode else p_t)
        if numpy_mode:
            return self._numpy_step()
        self._post_launch_error_copy()
        return self._torch_step()

    # ------------------------------------------------------------------ outputs
    def _numpy_obs(self):
        T = self._t
        return {"noisy_position": T["noisy_position"].cpu().numpy(), "time_step": T["time_step"].cpu().numpy()}

    def _torch_obs(self):
        T = self._t
        c = (lambda x: x.clone()) if self.copy else (lambda x: x)
        return {"noisy_position": c(T["noisy_position"]), "time_step": c(T["time_step"])}

    def _numpy_step(self):
        import torch

        torch.cuda.synchronize(self.device)
        T = self._t
        bits = int(T["err"].item())
        if bits:
            T["err"].zero_()
            self._raise_error_bits(bits)
        n = self.num_envs
        obs = self._numpy_obs()
        reward = T["reward"].cpu().numpy()
        term, trunc = T["terminated"].cpu().numpy(), T["truncated"].cpu().numpy()
        mask = T["info_mask"].cpu().numpy()
        info: dict[str, Any] = {}
        if mask.any():
            info["base_reward"] = np.where(mask, T["base_reward"].cpu().numpy(), np.float32(0))
            info["_base_reward"] = mask.copy()
            tgt = np.where(mask[:, None], T["target"].cpu().numpy(), np.float32(0))
            loss = np.where(mask, T["loss"].cpu().numpy(), np.float32(0))
            if self.sparse:
                tgt = {"target": tgt, "_target": mask.copy(),
                       "weight": np.where(mask, T["weight"].cpu().numpy(), 0.0), "_weight": mask.copy()}
            info["prediction"] = {"target": tgt, "_target": mask.copy(), "loss": loss, "_loss": mask.copy()}
            info["_prediction"] = mask.copy()
        if self.log_stats:
            lens = T["stats_len"].cpu().numpy()
            done = lens > 0
            if done.any():
                st = T["stats"].cpu().numpy()
                hist = T["stats_hist"].cpu().numpy()
                scalar: dict[str, Any] = {}
                for j, name in enumerate(self.STAT_NAMES):
                    scalar[name] = np.where(done, st[j].astype(np.float64), 0.0)
                    scalar["_" + name] = done.copy()
                vector: dict[str, Any] = {}
                for m, name in enumerate(("euclidean_distance", "mse")):
                    arr = np.full(n, None, dtype=object)
                    for i in np.nonzero(done)[0]:
                        arr[i] = list(hist[i, m, :lens[i]])
                    vector[name] = arr
                    vector["_" + name] = done.copy()
                info["stats"] = {"scalar": scalar, "_scalar": done.copy(), "vector": vector, "_vector": done.copy()}
                info["_stats"] = done.copy()
        self._autoreset_host = term | trunc
        return obs, reward, term, trunc, info

    def _torch_step(self):
        T = self._t
        mask = T["info_mask"]
        c = (lambda x: x.clone()) if self.copy else (lambda x: x)
        target = c(T["target"])
        if self.sparse:
            target = {"target": target, "_target": c(mask), "weight": c(T["weight"]), "_weight": c(mask)}
        info = {"base_reward": c(T["base_reward"]), "_base_reward": c(mask),
                "prediction": {"target": target, "_target": c(mask), "loss": c(T["loss"]), "_loss": c(mask)},
                "_prediction": c(mask)}
        if self.log_stats:
            if self._stats_view is None:
                done = T["terminated"]
                scalar = {}
                for j, name in enumerate(self.STAT_NAMES):
                    scalar[name] = T["stats"][j]
                    scalar["_" + name] = done
                vector = {"euclidean_distance": T["stats_hist"][:, 0], "_euclidean_distance": done,
                          "mse": T["stats_hist"][:, 1], "_mse": done, "length": T["stats_len"]}
                self._stats_view = {"stats": {"scalar": scalar, "_scalar": done, "vector": vector, "_vector": done},
                                    "_stats": done}
            if self.copy:
                def clone(d):
                    return {k: clone(v) if isinstance(v, dict) else v.clone() for k, v in d.items()}

                info.update(clone(self._stats_view))
            else:
                info.update(self._stats_view)
        return self._torch_obs(), c(T["reward"]), c(T["terminated"]), c(T["truncated"]), info

    # ------------------------------------------------------------------ render
    def _track_render(self, prediction):
        """Host copy of the render-only state of the tracked sub-envs (light_dark.py:102-150): position,
        last observation, last pos / prediction and the (last_pos, prediction_quality) trajectory."""
        if not len(self.render_envs):
            return
        import torch

        T = self._t
        idx = torch.as_tensor(self.render_envs, dtype=torch.int64, device=self.device)
        pos = T["pos"][idx].cpu().numpy()
        noisy = T["noisy_position"][idx].cpu().numpy()
        if prediction is None:  # reset(): every sub-env reset
            reset = np.ones(len(self.render_envs), dtype=bool)
        else:
            reset = T["reset_mask"][idx].cpu().numpy()
            tgt = T["target"][idx].cpu().numpy()
            pred = (prediction[idx].cpu().numpy() if isinstance(prediction, torch.Tensor)
                    else np.asarray(prediction)[self.render_envs])
        for j, r in enumerate(self._render_state):
            if reset[j]:  # trajectory.clear(); last_pred = last_pos = None (:119-120)
                r["traj"] = []
                r["last_pos"] = r["last_pred"] = None
            else:  # :129-130, :146-149
                last_pos, last_pred = tgt[j].copy(), pred[j].copy()
                quality = np.maximum(1 - np.linalg.norm(last_pred - last_pos) / 0.5, 0)
                r["traj"].append((last_pos, quality))
                r["last_pos"], r["last_pred"] = last_pos, last_pred
            r["pos"], r["last_obs"] = pos[j].copy(), noisy[j].copy()

    def render(self):
        """SyncVectorEnv.render(): one rgb_array frame per tracked sub-env, drawn like LightDarkEnv.render
        (light_dark.py:152-243)."""
        from .render import light_dark_frame, no_tracked_error

        if not len(self.render_envs):
            raise no_tracked_error()
        if not self._seeded:
            raise RuntimeError("render() needs reset() first")
        return tuple(light_dark_frame(r["pos"], r["last_obs"], r["last_pos"], r["last_pred"], r["traj"])
                     for r in self._render_state)

    def close(self, **kwargs):
        if not getattr(self, "_closed", True):
            self._closed = True
            self.closed = True
            self._t = {}

    def __repr__(self):
        return f"LightDarkVectorEnv(num_envs={self.num_envs}, device={self.device})"
