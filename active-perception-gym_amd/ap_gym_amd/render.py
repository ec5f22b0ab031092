"""rgb_array frames of the reference's render() methods, drawn on the host from state kept on the GPU.

Rendering is not on the hot path.  The envs keep, for the sub-envs chosen with the
constructor's `render_envs`, the render-only state the reference accumulates per sub-env, and render()
copies that state to the host and draws it with PIL the way the reference's render methods do:

  LIDARLocalization2DEnv.render   ap_gym/envs/lidar_localization2d.py:391-494
  LightDarkEnv.render             ap_gym/envs/light_dark.py:152-243
  colours / quality_color         ap_gym/envs/style.py:5-19

Coordinates keep the reference's dtypes (float32 positions times Python-float scales stay float32 under
NEP 50), so frames are pixel-identical to the reference's for the same state.
"""

from __future__ import annotations

import numpy as np

COLOR_AGENT = (0, 85, 255)
COLOR_OBS_PRIMARY = (55, 255, 0)
COLOR_OBS_SECONDARY = (255, 55, 0)
COLOR_PRED = (200, 0, 200)
COLOR_GOOD = (0, 200, 0)
COLOR_BAD = (200, 0, 0)

DEFAULT_TRACKED = 64  # render_envs=None tracks every sub-env when num_envs <= this


def tracked_envs(render_envs, num_envs: int) -> np.ndarray:
    """Indices of the sub-envs whose render state is kept (None: all of them up to DEFAULT_TRACKED)."""
    if render_envs is None:
        render_envs = range(num_envs) if num_envs <= DEFAULT_TRACKED else ()
    idx = np.asarray(list(render_envs), dtype=np.int64).reshape(-1)
    if idx.size and (idx.min() < 0 or idx.max() >= num_envs):
        raise ValueError(f"render_envs must index sub-envs in [0, {num_envs})")
    return idx


def no_tracked_error() -> RuntimeError:
    return RuntimeError("no sub-env is tracked for rendering: pass render_envs=[...] to the constructor "
                        f"(default: every sub-env when num_envs <= {DEFAULT_TRACKED})")


def quality_color(quality):
    """style.py:13-19: COLOR_GOOD / COLOR_BAD blended by clip(quality, 0, 1), truncated to int."""
    q = np.clip(quality, 0, 1)[..., None]
    return tuple((q * np.array(COLOR_GOOD) + (1 - q) * np.array(COLOR_BAD)).astype(np.int_))


def _disc(draw, c, r, scale, fill):
    draw.ellipse(((c[0] - r) * scale, (c[1] - r) * scale, (c[0] + r) * scale, (c[1] + r) * scale), fill=fill)


def lidar_frame(occ, seen, traj, lidar_dist, lidar_directions, pos, last_pos, last_pred) -> np.ndarray:
    """One LIDARLocalization2DEnv frame (500 px wide).

    occ, seen          bool [H, W]: the map and the observation_map
    traj               float32 [k, 3]: trajectory rows (last_pos x, y, min(prediction_quality, 1))
    lidar_dist         float32 [B]: distances of the last observation
    lidar_directions   float32 [B, 2]: beam vectors scaled by the range
    pos                float32 [2]; last_pos / last_pred float32 [2] or None (right after a reset)
    """
    from PIL import Image, ImageDraw

    h, w = occ.shape
    scale = 500 / w
    alpha = 0.25 + 0.75 * seen.astype(np.float32)
    grey = (alpha * (~occ).astype(np.float32) + (1.0 - alpha) * 0.5) * 255
    size = (int(round(w * scale)), int(round(h * scale)))
    img = Image.fromarray(grey).resize(size, resample=Image.Resampling.NEAREST).convert("RGB")
    draw = ImageDraw.Draw(img, mode="RGBA")
    radius = 0.2
    for a, b in zip(traj[:-1], traj[1:]):
        draw.line((a[0] * scale, a[1] * scale, b[0] * scale, b[1] * scale), width=2, fill=quality_color(b[2]))
    if lidar_dist is not None:
        unit = lidar_directions / np.linalg.norm(lidar_directions, axis=-1, keepdims=True)
        for dist, u in zip(lidar_dist, unit):
            end = pos + u * dist
            draw.line((pos[0] * scale, pos[1] * scale, end[0] * scale, end[1] * scale), width=2,
                      fill=COLOR_OBS_PRIMARY)
            _disc(draw, end, radius, scale, COLOR_OBS_SECONDARY)
    if last_pred is not None:
        draw.line((last_pos[0] * scale, last_pos[1] * scale, last_pred[0] * scale, last_pred[1] * scale),
                  fill=COLOR_PRED + (80,))
        _disc(draw, last_pred, radius, scale, COLOR_PRED)
        _disc(draw, last_pos, radius, scale, COLOR_AGENT + (100,))
    _disc(draw, pos, radius, scale, COLOR_AGENT)
    return np.array(img)


# ---------------------------------------------------------------------------------------- LightDark
LIGHT_POS = np.array([0, -0.7], dtype=np.float32)
LIGHT_HEIGHT = 0.2
_light_dark_base = None


def light_dark_brightness(pos):
    """light_dark.py:96-100: h^2 / (|pos - light|^2 + h^2)."""
    return LIGHT_HEIGHT**2 / (np.sum((pos - LIGHT_POS) ** 2, axis=-1) + LIGHT_HEIGHT**2)


def light_dark_base() -> np.ndarray:
    """light_dark.py:72-81: the 500 x 500 brightness background (0.1 ambient), computed once."""
    global _light_dark_base
    if _light_dark_base is None:
        res = 500
        gx, gy = np.meshgrid(np.linspace(-1, 1, res), np.linspace(-1, 1, res), indexing="ij")
        b = light_dark_brightness(np.stack([gy, gx], axis=-1))
        _light_dark_base = np.broadcast_to(((b * 0.9 + 0.1) * 255).astype(np.uint8)[..., None], (res, res, 3))
    return _light_dark_base


def light_dark_frame(pos, last_obs, last_pos, last_pred, traj) -> np.ndarray:
    """One LightDarkEnv frame: noise disc, trajectory coloured by prediction quality, observation and
    prediction markers.  pos / last_obs / last_pos / last_pred float32 [2] (the last two None after a
    reset); traj: list of (last_pos float32 [2], quality float32)."""
    from PIL import Image, ImageDraw

    img = Image.fromarray(light_dark_base())
    draw = ImageDraw.Draw(img, mode="RGBA")
    dot = 0.01 * img.size[0]
    size = np.array(img.size[::-1])

    def px(p):
        return (p + 1) / 2 * size

    c = px(pos)
    std = (1 - light_dark_brightness(pos)) * 0.3 / 2 * size
    draw.ellipse([tuple(c - std), tuple(c + std)], fill=COLOR_OBS_PRIMARY + (30,), outline=None)
    for (pa, _), (pb, qb) in zip(traj[:-1], traj[1:]):
        a, b = px(pa), px(pb)
        draw.line((a[0], a[1], b[0], b[1]), width=2, fill=quality_color(qb))
    o = px(last_obs)
    draw.line((tuple(c), tuple(o)), fill=COLOR_OBS_PRIMARY + (80,))
    draw.ellipse([tuple(o - dot), tuple(o + dot)], fill=COLOR_OBS_PRIMARY + (100,), outline=None)
    if last_pred is not None:
        lp, ls = px(last_pred), px(last_pos)
        draw.line((tuple(ls), tuple(lp)), fill=COLOR_PRED + (80,))
        draw.ellipse([tuple(lp - dot), tuple(lp + dot)], fill=COLOR_PRED + (100,), outline=None)
        draw.ellipse([tuple(ls - dot), tuple(ls + dot)], fill=COLOR_AGENT + (100,), outline=None)
    draw.ellipse([tuple(c - dot), tuple(c + dot)], fill=COLOR_AGENT, outline=None)
    return np.array(img)
