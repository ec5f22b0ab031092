"""Drop-in probe: the reference's own registration + make_vec with ap_gym_amd registered into it.

TEST INFRASTRUCTURE (build container only; run by tests/test_integration.py in a child process so
that the gymnasium stub does not leak into other tests).  It loads the reference's unmodified
registration.py / active_perception_vector_env.py through tests/golden/refload.py, runs the
reference's register_envs(), then ap_gym_amd.integration.register_with_ap_gym(), and checks what
the reference's `ap_gym.make_vec` now returns.  The GPU env cannot run here, so the LIDAR ids are
served by an oracle-backed stand-in with the same constructor, spaces and loss (the C oracle in
oracle/, the checker of every LIDAR parity test).
"""

from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests", "golden"), ROOT, os.path.join(ROOT, "active-perception-gym_amd")]

import refload  # noqa: E402

refload.install_stubs()
import gymnasium as gym  # noqa: E402  (the stub)

ap = refload.load_core()
for _m, _names in [("vector_to_single_wrapper", ["VectorToSingleWrapper", "ActivePerceptionVectorToSingleWrapper"]),
                   ("logit_space", ["LogitSpace"]), ("sparsify_wrapper", ["SparsifyWrapper", "SparsifyVectorWrapper"])]:
    _mod = refload.load(_m)
    for _n in _names:
        setattr(ap, _n, getattr(_mod, _n))
reg = refload.load("envs.registration")
ap.make_vec, ap.register = reg.make_vec, reg.register
reg.register_envs()

import ap_gym_amd  # noqa: E402
from ap_gym_amd import integration  # noqa: E402
from ap_gym_amd.lidar_env import lidar_spaces  # noqa: E402
from ap_gym_amd.vector_env import VectorEnv  # noqa: E402
from oracle import oracle  # noqa: E402


class OracleLidarStandIn(VectorEnv):
    """LIDARLocalization2DVectorEnv's constructor, spaces and loss over the C oracle (numpy out)."""

    metadata = {"render_modes": ["rgb_array"], "render_fps": 4, "autoreset_mode": "NextStep"}

    def __init__(self, num_envs=1, dataset=None, static_map=False, lidar_beam_count=8, lidar_range=5,
                 max_episode_steps=100, log_stats=False, sparse=False, render_mode="rgb_array", **_backend):
        self.num_envs, self.render_mode, self.dataset = num_envs, render_mode, dataset
        sp = lidar_spaces(num_envs, dataset.map_height, dataset.map_width, lidar_beam_count, static_map, sparse)
        sp.pop("inner_loss")
        for k, v in sp.items():
            setattr(self, k, v)
        self.kind = "maze" if isinstance(dataset, ap_gym_amd.FloorMapDatasetMaze) else "rooms"
        self.o = oracle.OracleLidarVectorEnv(num_envs, self.kind, dataset.map_width, static_map, 0, lidar_beam_count,
                                             lidar_range, max_episode_steps, sparse=sparse)

    def _obs(self):
        o = self.o
        obs = {"lidar": o.lidar.copy(), "odometry": o.odometry.copy()}
        if o.map is not None:
            obs["map"] = o.map[..., None].copy()
        obs["time_step"] = o.time_step.copy()
        return obs

    def reset(self, *, seed=None, options=None):
        self.o.reset(seed)
        return self._obs(), {}

    def step(self, actions):
        self.o.step(actions["action"], actions["prediction"])
        o = self.o
        return self._obs(), o.reward.copy(), o.terminated.astype(bool), o.truncated.astype(bool), {}


def make_impl(env_id, num_envs=1, **kw):
    if env_id.startswith("LIDARLoc"):
        for k in ("device", "array_backend"):
            kw.pop(k, None)
        spec = ap_gym_amd.registry[env_id]  # what ap_gym_amd.make_vec would merge in
        kw = {**{k: v for k, v in spec.kwargs.items() if k in ("sparse", "log_stats", "static_map")}, **kw}
        return OracleLidarStandIn(num_envs=num_envs, **kw)
    raise RuntimeError(f"no CPU stand-in for {env_id}")


def main():
    lidar_ids = [i for i in gym.registry if i.startswith("LIDARLoc")]
    # 1. the round-1 INTEGRATION.md pattern (vector entry point + additional_wrappers) is refused
    old = gym.registry["LIDARLocRooms-v0"]
    gym.register(id="Probe-v0", entry_point=old.entry_point, vector_entry_point=lambda num_envs=1, **k: None,
                 additional_wrappers=old.additional_wrappers, kwargs=old.kwargs)
    try:
        gym.make_vec("Probe-v0", 2)
        raise AssertionError("gymnasium accepted a vector entry point with additional_wrappers")
    except gym.envs.registration.Error as e:
        assert "additional_wrappers" in str(e)
    del gym.registry["Probe-v0"]
    assert all(len(gym.registry[i].additional_wrappers) == 2 for i in lidar_ids if "sparse" not in i)

    # 2. register the backend under the reference's ids
    switched = integration.register_with_ap_gym(ap, make_impl=make_impl, device="cuda:0")
    ours = set(ap_gym_amd.registry)
    both = {i for i in gym.registry if i in ours}
    assert set(switched) == both, sorted(both - set(switched))
    for want in ("LIDARLocRooms-v0", "LIDARLocMaze-sparse-v0", "MNIST-v0", "TinyImageNetLoc-v0", "LightDark-v0",
                 "CircleSquare-v0", "CircleSquareHideAndSeek-v0"):
        assert want in switched, want
    for i in switched:
        spec = gym.registry[i]
        assert spec.additional_wrappers == () and spec.vector_entry_point is not None, i

    # 3. the reference's make_vec now returns the backend env itself (no restore/pseudo wrapper)
    for env_id, ds in (("LIDARLocRooms-v0", reg.FloorMapDatasetRooms(32, 32)),
                       ("LIDARLocMaze-v0", reg.FloorMapDatasetMaze(21, 21))):
        env = ap.make_vec(env_id, num_envs=6, lidar_beam_count=8, dataset=ds)
        assert isinstance(env, ap.BaseActivePerceptionVectorEnv), type(env)
        assert type(env).__name__ == "ApGymAmdVectorEnv"
        assert ap.ensure_active_perception_vector_env(env) is env
        loss, single_t, batch_t = refload.load("active_perception_vector_env").find_loss_and_pred_space_vec(env)
        assert loss is env.env_impl.loss_fn
        assert single_t.shape == (2,) and batch_t.shape == (6, 2)
        assert isinstance(env.single_action_space, ap.ActivePerceptionActionSpace)
        assert env.prediction_space.shape == (6, 2) and env.inner_action_space.shape == (6, 2)
        assert isinstance(env.single_observation_space["map"], ap.ImageSpace)
        assert env.single_observation_space["map"].shape == (ds.map_height, ds.map_width, 1)
        assert isinstance(env.dataset, ap_gym_amd.FloorMapDataset)  # reference dataset converted
        # the stand-in is driven through the adapter exactly like the GPU env; values are the oracle's
        ref = oracle.OracleLidarVectorEnv(6, env.env_impl.kind, ds.map_width, False, 0, 8)
        obs, _ = env.reset(seed=3)
        ref.reset(3)
        assert np.array_equal(obs["lidar"], ref.lidar)
        rng = np.random.default_rng(0)
        for _ in range(110):
            a = rng.uniform(-1, 1, (6, 2)).astype(np.float32)
            p = rng.uniform(-1, 1, (6, 2)).astype(np.float32)
            obs, rew, term, trunc, _ = env.step({"action": a, "prediction": p})
            ref.step(a, p)
            assert np.array_equal(obs["lidar"], ref.lidar) and np.array_equal(rew, ref.reward)
        # the loss the user trains with is the build's normalized MSE
        pred = rng.uniform(-1, 1, (6, 2)).astype(np.float32)
        tgt = rng.uniform(-1, 1, (6, 2)).astype(np.float32)
        ref_loss = refload.load("active_regression_env")._make_mse_loss_fn_and_target_space(2, -1, 1)[0]
        assert np.array_equal(env.loss_fn(pred, tgt, (6,)), ref_loss(pred, tgt, (6,)))
        env.close()

    # 4. sparse ids keep the weighted loss and the {"target", "weight"} target space
    env = ap.make_vec("LIDARLocRooms-sparse-v0", num_envs=3, lidar_beam_count=8, dataset=reg.FloorMapDatasetRooms())
    assert type(env.loss_fn).__name__ == "WeightedLossFn"
    assert set(env.single_prediction_target_space.spaces) == {"target", "weight"}

    # 5. single-env ids still apply TimeLimit and the log wrapper (now inside the entry point)
    single = gym.make("LIDARLocRoomsStatic-v0")
    names = []
    e = single
    while e is not None:
        names.append(type(e).__name__)
        e = getattr(e, "env", None)
    assert names[0] == "ActiveRegressionLogWrapper" and "TimeLimit" in names, names
    assert names[-1] == "LIDARLocalization2DEnv", names

    # 6. image configs with reference datasets convert to device-pool configs
    cfg = gym.registry["CircleSquare-v0"].kwargs["image_perception_config"]
    kw = integration.convert_kwargs({"image_perception_config": cfg})
    c2 = kw["image_perception_config"]
    assert isinstance(c2, ap_gym_amd.ImagePerceptionConfig)
    assert isinstance(c2.dataset, ap_gym_amd.CircleSquareDataset)
    assert tuple(c2.sensor_size) == tuple(cfg.sensor_size) and c2.step_limit == cfg.step_limit
    import ap_gym_amd.vector_env as ve
    assert ve.HAVE_GYMNASIUM and issubclass(ap_gym_amd.LIDARLocalization2DVectorEnv, gym.vector.VectorEnv)
    print("integration probe OK:", len(switched), "ids switched")


if __name__ == "__main__":
    main()
