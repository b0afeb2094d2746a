"""Synthetic photometric / geometric BA problems (SURVEY.md §8d generator).

The reference has no synthetic generator of its own (its inputs come from the OpenCV frontend,
src/sfm.cpp:1117-1167, which cannot run here).  This module builds problems with the reference's data
model restated as SoA arrays:

* keyframes  ``T_w_k`` as Sophus ``[qx qy qz qw tx ty tz]`` (common_types.h:174-179, se3.hpp:70)
* points     anchored in a host keyframe with inverse *distance* ρ along the unit bearing of
             ``u_ref`` (common_types.h:188-217, reprojection.h:105-108)
* blocks     one per (point, later observing keyframe), the anchor itself excluded
             (map_utils.h:347-375)

Trajectory ``T_w_k = (exp([0, 0.002k, 0]), [0.05k, 0, 0])``; every point is observed by the K keyframes
after its host, so ``n_blocks = K·n_points``.

Three image sources:
* ``texture="render"`` ray-casts every keyframe onto a textured plane, so the photometric residual of the
  unperturbed state is ~0 (for solver / convergence tests);
* ``texture="euroc"`` does the same with real image content: the plane carries a 2×2 mosaic of the reference's own
  EuRoC V1 cam0 frames (tests/golden/euroc_texture.npz, made by tests/golden/make_euroc_texture.py), and points
  are placed on high-gradient host pixels (as a direct-method front end selects them);
* ``texture="noise"`` gives each keyframe an independent smooth random texture (for throughput, where
  image content is irrelevant).  ``bench.py`` builds those on the GPU with torch.
"""
from __future__ import annotations

import dataclasses
import math
from typing import Optional

import numpy as np

PHOTOMETRIC, GEOMETRIC = 0, 1
PINHOLE, DOUBLE_SPHERE, EUCM, KB4 = 0, 1, 2, 3
MODEL_IDS = {"pinhole": PINHOLE, "ds": DOUBLE_SPHERE, "eucm": EUCM, "kb4": KB4}
KIND_IDS = {"photometric": PHOTOMETRIC, "geometric": GEOMETRIC}

# EuRoC-like 752×480 intrinsics per model, vector layout of camera_models.h ([fx fy cx cy p1 p2 0 0]).
DEFAULT_INTRINSICS = {
    PINHOLE: [458.654, 457.296, 367.215, 248.375, 0, 0, 0, 0],
    DOUBLE_SPHERE: [349.7, 349.9, 365.9, 249.0, -0.28, 0.57, 0, 0],
    EUCM: [460.0, 459.0, 365.5, 249.5, 0.59, 1.1, 0, 0],
    # Kannala-Brandt 4: the distortion of camera_models.h getTestProjections (:302-306) with a 752×480 camera
    KB4: [379.045, 379.008, 375.5, 239.5, 0.00693023, -0.0013828, -0.000272596, -0.000452646],
}

# DSO-style 8-pixel residual pattern (du, dv) — SURVEY.md §8d.
PATTERN8 = np.array([(0, -2), (-1, -1), (1, -1), (-2, 0), (0, 0), (2, 0), (-1, 1), (0, 2)], np.float32)


@dataclasses.dataclass
class Problem:
    kind: int
    model: int
    width: int
    height: int
    intrinsics: np.ndarray          # (n_cams, 8) float64
    frame_cam: np.ndarray           # (n_frames,) int32
    images: Optional[np.ndarray]    # (n_frames, H, W) uint8, photometric only
    pattern: np.ndarray             # (P, 2) float32
    point_host: np.ndarray          # (n_points,) int32
    u_ref: np.ndarray               # (n_points, 2) float64
    host_intensity: Optional[np.ndarray]  # (n_points, P) float32
    block_point: np.ndarray         # (n_blocks,) int32
    block_target: np.ndarray        # (n_blocks,) int32
    u_obs: Optional[np.ndarray]     # (n_blocks, 2) float64, geometric only
    poses: np.ndarray               # (n_frames, 7) float64 — current state
    rho: np.ndarray                 # (n_points,) float64 — current state
    poses_gt: Optional[np.ndarray] = None
    rho_gt: Optional[np.ndarray] = None
    interp: int = 0                 # image interpolator: 0 bilinear, 1 Ceres' bicubic (pba_set_interpolator)

    @property
    def n_frames(self) -> int:
        return int(self.frame_cam.shape[0])

    @property
    def n_points(self) -> int:
        return int(self.point_host.shape[0])

    @property
    def n_blocks(self) -> int:
        return int(self.block_point.shape[0])

    @property
    def P(self) -> int:
        return int(self.pattern.shape[0]) if self.kind == PHOTOMETRIC else 2

    @property
    def R(self) -> int:
        """Residuals per block."""
        return self.P if self.kind == PHOTOMETRIC else 2

    @property
    def record(self) -> int:
        """Floats per block record [r | J_host | J_target | J_rho]."""
        return 14 * self.R


# ------------------------------------------------------------------------------------------------
# SE3 / camera helpers (numpy, vectorised, double).  Same conventions as Sophus.
# ------------------------------------------------------------------------------------------------
def quat_to_rot(q: np.ndarray) -> np.ndarray:
    x, y, z, w = q[..., 0], q[..., 1], q[..., 2], q[..., 3]
    R = np.empty(q.shape[:-1] + (3, 3))
    R[..., 0, 0] = 1 - 2 * (y * y + z * z)
    R[..., 0, 1] = 2 * (x * y - w * z)
    R[..., 0, 2] = 2 * (x * z + w * y)
    R[..., 1, 0] = 2 * (x * y + w * z)
    R[..., 1, 1] = 1 - 2 * (x * x + z * z)
    R[..., 1, 2] = 2 * (y * z - w * x)
    R[..., 2, 0] = 2 * (x * z - w * y)
    R[..., 2, 1] = 2 * (y * z + w * x)
    R[..., 2, 2] = 1 - 2 * (x * x + y * y)
    return R


def quat_mul(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    ax, ay, az, aw = np.moveaxis(a, -1, 0)
    bx, by, bz, bw = np.moveaxis(b, -1, 0)
    return np.stack([aw * bx + ax * bw + ay * bz - az * by,
                     aw * by + ay * bw + az * bx - ax * bz,
                     aw * bz + az * bw + ax * by - ay * bx,
                     aw * bw - ax * bx - ay * by - az * bz], -1)


def so3_exp(w: np.ndarray) -> np.ndarray:
    th = np.linalg.norm(w, axis=-1, keepdims=True)
    small = th < 1e-10
    th_s = np.where(small, 1.0, th)
    imag = np.where(small, 0.5 - th * th / 48.0, np.sin(0.5 * th_s) / th_s)
    real = np.where(small, 1.0 - th * th / 8.0, np.cos(0.5 * th_s))
    return np.concatenate([imag * w, real], -1)


def se3_exp(d: np.ndarray) -> np.ndarray:
    """Sophus SE3::exp for tangent [υ, ω] (se3.hpp:763-784), vectorised."""
    d = np.asarray(d, np.float64)
    v, w = d[..., :3], d[..., 3:]
    q = so3_exp(w)
    th = np.linalg.norm(w, axis=-1)[..., None, None]
    Om = np.zeros(d.shape[:-1] + (3, 3))
    Om[..., 0, 1], Om[..., 0, 2], Om[..., 1, 2] = -w[..., 2], w[..., 1], -w[..., 0]
    Om[..., 1, 0], Om[..., 2, 0], Om[..., 2, 1] = w[..., 2], -w[..., 1], w[..., 0]
    Om2 = Om @ Om
    ths = np.where(th < 1e-10, 1.0, th)
    a = np.where(th < 1e-10, 0.5, (1 - np.cos(ths)) / ths ** 2)
    b = np.where(th < 1e-10, 1.0 / 6.0, (ths - np.sin(ths)) / ths ** 3)
    V = np.eye(3) + a * Om + b * Om2
    t = (V @ v[..., None])[..., 0]
    return np.concatenate([q, t], -1)


def se3_mul(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    q = quat_mul(a[..., :4], b[..., :4])
    q = q / np.linalg.norm(q, axis=-1, keepdims=True)
    t = a[..., 4:] + (quat_to_rot(a[..., :4]) @ b[..., 4:, None])[..., 0]
    return np.concatenate([q, t], -1)


def se3_plus(T: np.ndarray, d: np.ndarray) -> np.ndarray:
    """LocalParameterizationSE3::Plus — T · exp(δ) (local_parameterization_se3.hpp:43-50)."""
    return se3_mul(T, se3_exp(d))


def unproject(model: int, k: np.ndarray, uv: np.ndarray) -> np.ndarray:
    """Unit bearings (camera_models.h unproject + normalize), vectorised over uv (..., 2)."""
    k = np.asarray(k, np.float64)
    mx = (uv[..., 0] - k[..., 2]) / k[..., 0]
    my = (uv[..., 1] - k[..., 3]) / k[..., 1]
    r2 = mx * mx + my * my
    if model == PINHOLE:
        b = np.stack([mx, my, np.ones_like(mx)], -1)
    elif model == DOUBLE_SPHERE:
        xi, al = k[..., 4], k[..., 5]
        mz = (1 - al * al * r2) / (al * np.sqrt(1 - (2 * al - 1) * r2) + 1 - al)
        fac = (mz * xi + np.sqrt(mz * mz + (1 - xi * xi) * r2)) / (mz * mz + r2)
        b = np.stack([fac * mx, fac * my, fac * mz - xi], -1)
    elif model == EUCM:
        al, be = k[..., 4], k[..., 5]
        mz = (1 - be * al * al * r2) / (al * np.sqrt(1 - (2 * al - 1) * be * r2) + (1 - al))
        b = np.stack([mx, my, mz], -1)
    else:  # KB4: 5 Newton steps on d(θ) = r_u from θ = 0 (camera_models.h:352-380)
        k1, k2, k3, k4 = k[..., 4], k[..., 5], k[..., 6], k[..., 7]
        ru = np.sqrt(r2)
        th = np.zeros_like(ru)
        for _ in range(5):
            t2 = th * th
            f = th + t2 * th * (k1 + t2 * (k2 + t2 * (k3 + t2 * k4))) - ru
            df = 1 + t2 * (3 * k1 + t2 * (5 * k2 + t2 * (7 * k3 + t2 * 9 * k4)))
            th = th - f / df
        safe = np.where(ru > 0, ru, 1.0)
        b = np.stack([np.sin(th) * mx / safe, np.sin(th) * my / safe, np.cos(th)], -1)
    return b / np.linalg.norm(b, axis=-1, keepdims=True)


def project(model: int, k: np.ndarray, p: np.ndarray) -> np.ndarray:
    k = np.asarray(k, np.float64)
    x, y, z = p[..., 0], p[..., 1], p[..., 2]
    if model == PINHOLE:
        den = z
    elif model == DOUBLE_SPHERE:
        xi, al = k[..., 4], k[..., 5]
        d1 = np.sqrt(x * x + y * y + z * z)
        xz = xi * d1 + z
        d2 = np.sqrt(x * x + y * y + xz * xz)
        den = al * d2 + (1 - al) * xz
    elif model == EUCM:
        al, be = k[..., 4], k[..., 5]
        d = np.sqrt(be * (x * x + y * y) + z * z)
        den = al * d + (1 - al) * z
    else:  # KB4 (camera_models.h:316-348): u = fx·d(θ)·x/r + cx, θ = atan2(r, z)
        k1, k2, k3, k4 = k[..., 4], k[..., 5], k[..., 6], k[..., 7]
        r = np.sqrt(x * x + y * y)
        th = np.arctan2(r, z)
        t2 = th * th
        d = th + t2 * th * (k1 + t2 * (k2 + t2 * (k3 + t2 * k4)))
        den = np.where(r > 0, r / np.where(d != 0, d, 1.0), z)
    return np.stack([k[..., 0] * x / den + k[..., 2], k[..., 1] * y / den + k[..., 3]], -1)


def bilinear(img: np.ndarray, u: np.ndarray, v: np.ndarray) -> np.ndarray:
    """Bilinear + edge clamp (the oracle's interpolator), vectorised over one image."""
    H, W = img.shape
    u = np.clip(u, -2, W + 1)
    v = np.clip(v, -2, H + 1)
    x0 = np.floor(u)
    y0 = np.floor(v)
    a, b = u - x0, v - y0
    x0 = x0.astype(np.int64)
    y0 = y0.astype(np.int64)
    xa, xb = np.clip(x0, 0, W - 1), np.clip(x0 + 1, 0, W - 1)
    ya, yb = np.clip(y0, 0, H - 1), np.clip(y0 + 1, 0, H - 1)
    I = img.astype(np.float64)
    return ((1 - b) * ((1 - a) * I[ya, xa] + a * I[ya, xb]) + b * ((1 - a) * I[yb, xa] + a * I[yb, xb]))


# ------------------------------------------------------------------------------------------------
# Scene
# ------------------------------------------------------------------------------------------------
def trajectory(n_frames: int, step: float = 0.05, yaw: float = 0.002) -> np.ndarray:
    k = np.arange(n_frames, dtype=np.float64)
    w = np.stack([np.zeros_like(k), yaw * k, np.zeros_like(k)], -1)
    q = so3_exp(w)
    t = np.stack([step * k, np.zeros_like(k), np.zeros_like(k)], -1)
    return np.concatenate([q, t], -1)


class PlaneTexture:
    """Smooth intensity field on the world plane Z = z0 (sum of random sinusoids), range ~[20, 235]."""

    def __init__(self, rng: np.random.Generator, z0: float = 6.0, n_waves: int = 12):
        self.z0 = z0
        ang = rng.uniform(0, np.pi, n_waves)
        freq = rng.uniform(0.8, 7.0, n_waves) * 2 * np.pi  # rad / m
        self.kx, self.ky = freq * np.cos(ang), freq * np.sin(ang)
        self.phase = rng.uniform(0, 2 * np.pi, n_waves)
        self.amp = rng.uniform(0.5, 1.0, n_waves)
        self.amp /= self.amp.sum()

    def __call__(self, X: np.ndarray, Y: np.ndarray) -> np.ndarray:
        s = np.zeros_like(X)
        for i in range(len(self.kx)):
            s += self.amp[i] * np.sin(self.kx[i] * X + self.ky[i] * Y + self.phase[i])
        return 127.5 + 107.5 * s

    def render(self, model: int, k: np.ndarray, pose: np.ndarray, W: int, H: int) -> np.ndarray:
        uu, vv = np.meshgrid(np.arange(W, dtype=np.float64), np.arange(H, dtype=np.float64))
        b = unproject(model, k, np.stack([uu, vv], -1))
        R = quat_to_rot(pose[:4])
        d = b @ R.T
        lam = (self.z0 - pose[6]) / d[..., 2]
        X = pose[4] + lam * d[..., 0]
        Y = pose[5] + lam * d[..., 1]
        return np.clip(np.rint(self(X, Y)), 0, 255).astype(np.uint8)

    def depth(self, pose: np.ndarray, b: np.ndarray) -> np.ndarray:
        """Distance along bearings b (camera frame) to the plane."""
        d = (quat_to_rot(pose[..., :4]) @ b[..., None])[..., 0]
        return (self.z0 - pose[..., 6]) / d[..., 2]


class ImageTexture(PlaneTexture):
    """A u8 image on the world plane Z = z0 (texel `texel` metres, centred on (x0, y0), mirrored beyond its edges),
    bilinearly sampled — real image content for rendered keyframes."""

    def __init__(self, image: np.ndarray, z0: float = 6.0, texel: float = 0.017, x0: float = 1.0, y0: float = 0.0):
        self.z0, self.img, self.texel = z0, image.astype(np.float64), texel
        self.x0 = x0 - 0.5 * texel * image.shape[1]
        self.y0 = y0 - 0.5 * texel * image.shape[0]

    def __call__(self, X: np.ndarray, Y: np.ndarray) -> np.ndarray:
        H, W = self.img.shape
        u = (X - self.x0) / self.texel
        v = (Y - self.y0) / self.texel
        u = _mirror(u, W)
        v = _mirror(v, H)
        return bilinear(self.img, u, v)


def _mirror(x: np.ndarray, n: int) -> np.ndarray:
    """Mirrored repeat of coordinates into [0, n−1]."""
    p = 2.0 * (n - 1)
    y = np.mod(x, p)
    return np.where(y > n - 1, p - y, y)


def euroc_texture_image() -> np.ndarray:
    import os
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    return np.load(os.path.join(here, "tests", "golden", "euroc_texture.npz"))["texture"]


def noise_images(rng: np.random.Generator, n: int, W: int, H: int, cell: int = 8) -> np.ndarray:
    """Independent smooth random textures (bilinear upsample of a coarse random grid)."""
    gh, gw = H // cell + 2, W // cell + 2
    g = rng.uniform(20, 235, (n, gh, gw))
    ys = np.arange(H) / cell
    xs = np.arange(W) / cell
    y0 = np.floor(ys).astype(int)
    x0 = np.floor(xs).astype(int)
    fy = (ys - y0)[None, :, None]
    fx = (xs - x0)[None, None, :]
    a = g[:, y0][:, :, x0]
    b = g[:, y0][:, :, x0 + 1]
    c = g[:, y0 + 1][:, :, x0]
    d = g[:, y0 + 1][:, :, x0 + 1]
    img = (1 - fy) * ((1 - fx) * a + fx * b) + fy * ((1 - fx) * c + fx * d)
    img += rng.normal(0, 2.0, img.shape)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def make_problem(n_frames: int = 8, n_points: int = 64, K: int = 4, width: int = 752, height: int = 480,
                 model: int | str = PINHOLE, kind: int | str = PHOTOMETRIC, pattern: Optional[np.ndarray] = None,
                 seed: int = 42, texture: str = "render", perturb: bool = True, pose_sigma: float = 0.003,
                 rho_sigma: float = 0.02, border: int = 24, obs_sigma: float = 0.5,
                 with_images: bool = True, intrinsics: Optional[np.ndarray] = None,
                 frame_cam: Optional[np.ndarray] = None, poses_gt: Optional[np.ndarray] = None) -> Problem:
    """Build a synthetic problem.  ``poses``/``rho`` hold the perturbed state.  ``intrinsics``
    ((n_cams, 8), quoted for width × height) overrides the model's default camera, ``frame_cam`` assigns cameras to
    keyframes (a stereo rig: alternating 0/1) and ``poses_gt`` replaces the default trajectory."""
    model = MODEL_IDS.get(model, model) if isinstance(model, str) else model
    kind = KIND_IDS.get(kind, kind) if isinstance(kind, str) else kind
    if n_frames < K + 1:
        raise ValueError("need at least K+1 keyframes")
    rng = np.random.default_rng(seed)
    if intrinsics is not None:
        intr = np.asarray(intrinsics, np.float64).reshape(-1, 8).copy()
    else:
        intr = np.array([DEFAULT_INTRINSICS[model]], np.float64)
        intr[0, :4] *= width / 752.0  # intrinsics are quoted for 752×480; rescale for other sizes
    frame_cam = np.zeros(n_frames, np.int32) if frame_cam is None else np.asarray(frame_cam, np.int32)
    poses_gt = trajectory(n_frames) if poses_gt is None else np.asarray(poses_gt, np.float64)
    kf = intr[frame_cam]  # per-keyframe intrinsics
    pat = PATTERN8 if pattern is None else np.asarray(pattern, np.float32)

    point_host = rng.integers(0, n_frames - K, n_points).astype(np.int32)
    u_ref = np.stack([rng.integers(border, width - border, n_points),
                      rng.integers(border, height - border, n_points)], -1).astype(np.float64)

    tex = None
    rendered = None
    if texture == "euroc":
        tex = ImageTexture(euroc_texture_image())
        rendered = np.stack([tex.render(model, kf[f], poses_gt[f], width, height) for f in range(n_frames)])
        # high-gradient host pixels: of 6 candidates per point keep the one with the largest |∇I|
        cand = 6
        ch = rng.integers(0, n_frames - K, n_points * cand).astype(np.int32)
        cu = rng.integers(border, width - border, n_points * cand)
        cv = rng.integers(border, height - border, n_points * cand)
        img = rendered.astype(np.float64)
        g = np.abs(img[ch, cv, cu + 1] - img[ch, cv, cu - 1]) + np.abs(img[ch, cv + 1, cu] - img[ch, cv - 1, cu])
        best = np.argmax(g.reshape(n_points, cand), 1) + cand * np.arange(n_points)
        point_host = ch[best]
        u_ref = np.stack([cu[best], cv[best]], -1).astype(np.float64)
    b = unproject(model, kf[point_host], u_ref)

    if texture in ("render", "euroc"):
        if tex is None:
            tex = PlaneTexture(rng)
        dist = tex.depth(poses_gt[point_host], b)
    else:
        dist = np.clip(6.0 + rng.normal(0, 1.0, n_points), 3.0, 12.0)
    rho_gt = 1.0 / dist

    block_point = np.repeat(np.arange(n_points, dtype=np.int32), K)
    block_target = (np.repeat(point_host, K) + np.tile(np.arange(1, K + 1, dtype=np.int32), n_points)).astype(np.int32)

    images = host_int = u_obs = None
    if kind == PHOTOMETRIC and with_images:
        if rendered is not None:
            images = rendered
        elif texture == "render":
            images = np.stack([tex.render(model, kf[f], poses_gt[f], width, height) for f in range(n_frames)])
        else:
            images = noise_images(rng, n_frames, width, height)
        host_int = np.empty((n_points, len(pat)), np.float32)
        for f in np.unique(point_host):
            sel = np.nonzero(point_host == f)[0]
            uu = u_ref[sel, None, 0] + pat[None, :, 0]
            vv = u_ref[sel, None, 1] + pat[None, :, 1]
            host_int[sel] = bilinear(images[f], uu, vv).astype(np.float32)
    if kind == GEOMETRIC:
        ph = b / rho_gt[:, None]
        Th, Tt = poses_gt[point_host[block_point]], poses_gt[block_target]
        pw = (quat_to_rot(Th[:, :4]) @ ph[block_point, :, None])[..., 0] + Th[:, 4:]
        pt = (np.swapaxes(quat_to_rot(Tt[:, :4]), -1, -2) @ (pw - Tt[:, 4:])[..., None])[..., 0]
        u_obs = project(model, kf[block_target], pt) + rng.normal(0, obs_sigma, (len(block_point), 2))

    poses, rho = poses_gt.copy(), rho_gt.copy()
    if perturb:
        poses = se3_plus(poses_gt, pose_sigma * rng.normal(0, 1, (n_frames, 6)))
        rho = rho_gt * (1 + rho_sigma * rng.normal(0, 1, n_points))
    return Problem(kind=kind, model=model, width=width, height=height, intrinsics=intr, frame_cam=frame_cam,
                   images=images, pattern=pat, point_host=point_host, u_ref=u_ref, host_intensity=host_int,
                   block_point=block_point, block_target=block_target, u_obs=u_obs, poses=poses, rho=rho,
                   poses_gt=poses_gt, rho_gt=rho_gt)


# ------------------------------------------------------------------------------------------------
# Image pyramid (DSO convention, csrc/pba_pyramid.hip) — numpy restatement for tests.
# ------------------------------------------------------------------------------------------------
def downsample(images: np.ndarray) -> np.ndarray:
    """u8 (n, H, W) → (n, ⌊H/2⌋, ⌊W/2⌋), round(mean of each 2×2 block)."""
    n, H, W = images.shape
    h, w = H // 2, W // 2
    a = images[:, :2 * h, :2 * w].astype(np.uint32).reshape(n, h, 2, w, 2)
    return ((a.sum(axis=(2, 4)) + 2) >> 2).astype(np.uint8)


def level_problem(pb: "Problem", level: int, host_intensity: Optional[np.ndarray] = None) -> "Problem":
    """The problem the engine solves at pyramid `level`: images downsampled `level` times, cameras and u_ref
    scaled (c_l = (c + 0.5)/2^l − 0.5), I_h,k re-sampled (double bilinear) unless given."""
    s = 0.5 ** level
    imgs = pb.images
    for _ in range(level):
        imgs = downsample(imgs)
    k = pb.intrinsics.copy()
    k[:, 0] *= s
    k[:, 1] *= s
    k[:, 2] = (k[:, 2] + 0.5) * s - 0.5
    k[:, 3] = (k[:, 3] + 0.5) * s - 0.5
    ur = (pb.u_ref + 0.5) * s - 0.5
    if host_intensity is None:
        host_intensity = np.empty((pb.n_points, pb.pattern.shape[0]), np.float32)
        for f in np.unique(pb.point_host):
            sel = np.nonzero(pb.point_host == f)[0]
            host_intensity[sel] = bilinear(imgs[f], ur[sel, None, 0] + pb.pattern[None, :, 0],
                                           ur[sel, None, 1] + pb.pattern[None, :, 1]).astype(np.float32)
    return dataclasses.replace(pb, width=imgs.shape[2], height=imgs.shape[1], images=imgs, intrinsics=k, u_ref=ur,
                               host_intensity=host_intensity)


# ------------------------------------------------------------------------------------------------
# BASELINE.json configurations that the tests and the bench build
# ------------------------------------------------------------------------------------------------
def euroc_ds_intrinsics() -> np.ndarray:
    """(2, 8) double-sphere intrinsics of the EuRoC stereo pair from the reference's own calibration data file
    (data/euroc_calib/calibration-double-sphere.json, copied to tests/golden/map_small/)."""
    import json
    import os
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(here, "tests", "golden", "map_small", "euroc_calibration-double-sphere.json")) as f:
        cams = json.load(f)["value0"]["cam.intrinsics"]
    return np.array([[c["fx"], c["fy"], c["cx"], c["cy"], c["xi"], c["alpha"], 0.0, 0.0] for c in cams], np.float64)


def stereo_trajectory(n_keyframes: int, baseline: float = 0.11) -> np.ndarray:
    """Keyframe i → frames 2i (cam0) and 2i+1 (cam1): T_w_c = T_w_i · T_i_c with T_i_c0 = I and T_i_c1 a
    `baseline` shift along x (EuRoC's stereo rig; the sfm map's FrameCamId order, common_types.h:87-90)."""
    T_w_i = trajectory(n_keyframes, step=0.15)
    out = np.empty((2 * n_keyframes, 7))
    out[0::2] = T_w_i
    out[1::2] = se3_mul(T_w_i, np.array([0, 0, 0, 1, baseline, 0, 0], np.float64)[None].repeat(n_keyframes, 0))
    return out


def c1_problem(seed: int = 42, n_keyframes: int = 20, n_points: int = 2000, K: int = 4, **kw) -> Problem:
    """configs[0] (C1): EuRoC-sized geometric BA — 20 stereo keyframes (40 frames, double-sphere cameras with the
    reference's EuRoC calibration), ~2k landmarks each seen by the K frames after its anchor (stereo partner
    included), 752×480; as bundle_adjustment() builds it (map_utils.h:322-375).  Fixed frames {0, 1} = the
    reference's fixed cameras {(0,0), (0,1)} (sfm.cpp:1903)."""
    nf = 2 * n_keyframes
    return make_problem(n_frames=nf, n_points=n_points, K=K, kind=GEOMETRIC, model=DOUBLE_SPHERE, seed=seed,
                        intrinsics=euroc_ds_intrinsics(), frame_cam=np.arange(nf, dtype=np.int32) % 2,
                        poses_gt=stereo_trajectory(n_keyframes), **kw)


def c2_problem(seed: int = 42, n_frames: int = 50, n_points: int = 5000, K: int = 4, **kw) -> Problem:
    """configs[1] (C2): EuRoC-sized photometric BA — 50 keyframes of real EuRoC V1 image content (texture="euroc"),
    cam0's double-sphere calibration, 8-px pattern, ~5k points on high-gradient pixels × K = 4 targets."""
    return make_problem(n_frames=n_frames, n_points=n_points, K=K, kind=PHOTOMETRIC, model=DOUBLE_SPHERE, seed=seed,
                        texture="euroc", intrinsics=euroc_ds_intrinsics()[:1], **kw)


def render_torch(tex: PlaneTexture, K: np.ndarray, poses: np.ndarray, W: int, H: int, device, chunk: int = 64):
    """PlaneTexture.render for a pinhole camera on the GPU (torch, fp64 rays): (n, H, W) u8 tensor."""
    import torch
    n = poses.shape[0]
    out = torch.empty((n, H, W), dtype=torch.uint8, device=device)
    v, u = torch.meshgrid(torch.arange(H, dtype=torch.float64, device=device),
                          torch.arange(W, dtype=torch.float64, device=device), indexing="ij")
    b = torch.stack([(u - K[2]) / K[0], (v - K[3]) / K[1], torch.ones_like(u)], -1)
    b = b / torch.linalg.norm(b, dim=-1, keepdim=True)
    kx = torch.tensor(tex.kx, device=device)
    ky = torch.tensor(tex.ky, device=device)
    ph = torch.tensor(tex.phase, device=device)
    amp = torch.tensor(tex.amp, device=device)
    for s in range(0, n, chunk):
        P = torch.tensor(poses[s:s + chunk], dtype=torch.float64, device=device)
        R = torch.tensor(quat_to_rot(poses[s:s + chunk, :4]), device=device)
        d = torch.einsum("hwj,nij->nhwi", b, R)
        lam = (tex.z0 - P[:, 6, None, None]) / d[..., 2]
        X = P[:, 4, None, None] + lam * d[..., 0]
        Y = P[:, 5, None, None] + lam * d[..., 1]
        acc = torch.zeros_like(X)
        for i in range(kx.shape[0]):
            acc += amp[i] * torch.sin(kx[i] * X + ky[i] * Y + ph[i])
        out[s:s + chunk] = torch.clamp(torch.round(127.5 + 107.5 * acc), 0, 255).to(torch.uint8)
    return out


def c4_shard(device, rank: int = 0, world: int = 1, n_frames: int = 1000, n_points: int = 100000, K: int = 4,
             width: int = 752, height: int = 480, texture: str = "noise", seed: int = 42, block_order: str = "point"):
    """configs[3] (C4) shard of `rank`: hosts [rank·F, (rank+1)·F) of a world·F + K keyframe trajectory, n_points
    points each seen by the K keyframes after its host (n_blocks = K·n_points), pinhole 752×480, 8-px pattern.
    Images are built on the GPU (torch): "noise" (independent smooth textures; throughput) or "render" (one
    textured plane seen by every keyframe, so the residual at the true state is ~0 and LM converges).  Returns
    (problem with images=None and host intensities filled, images as a device tensor of all world·F + K frames).
    block_order: "point" (each point's K blocks together, hosts in order) or "morton" (within each host by target, then
    by the Morton code of u_ref — the image-locality order of the round-4 FETCH A/B)."""
    import torch
    import torch.nn.functional as F_
    F = n_frames
    NF = world * F + K
    off = rank * F
    pb = make_problem(n_frames=F + K, n_points=n_points, K=K, width=width, height=height, kind=PHOTOMETRIC,
                      model=PINHOLE, texture="noise", with_images=False, seed=seed + rank)
    pb.point_host = (pb.point_host + off).astype(np.int32)
    pb.block_target = (pb.block_target + off).astype(np.int32)
    pb.frame_cam = np.zeros(NF, np.int32)
    prng = np.random.default_rng(99)  # the same global poses on every rank
    pb.poses_gt = trajectory(NF)
    images = torch.zeros((NF, height, width), dtype=torch.uint8, device=device)
    if texture == "render":
        tex = PlaneTexture(np.random.default_rng(seed))
        b = unproject(PINHOLE, pb.intrinsics[0], pb.u_ref)
        pb.rho_gt = 1.0 / tex.depth(pb.poses_gt[pb.point_host], b)
        pb.rho = pb.rho_gt * (1 + 0.02 * np.random.default_rng(seed + 1).normal(0, 1, n_points))
        images[off:off + F + K] = render_torch(tex, pb.intrinsics[0], pb.poses_gt[off:off + F + K], width, height,
                                               device)
    else:
        g = torch.Generator(device=device)
        g.manual_seed(1234 + rank)
        for s in range(0, F + K, 100):
            m = min(100, F + K - s)
            coarse = torch.rand((m, 1, height // 8 + 2, width // 8 + 2), generator=g, device=device) * 215 + 20
            img = F_.interpolate(coarse, size=(height + 16, width + 16), mode="bilinear",
                                 align_corners=False)[:, 0, :height, :width]
            img = img + torch.randn((m, height, width), generator=g, device=device) * 2.0
            images[off + s:off + s + m] = img.round().clamp(0, 255).to(torch.uint8)
    pb.poses = se3_plus(pb.poses_gt, 3e-3 * prng.normal(0, 1, (NF, 6)))
    host = torch.from_numpy(pb.point_host.astype(np.int64)).to(device)
    uu = torch.from_numpy(pb.u_ref[:, 0].astype(np.int64)).to(device)[:, None] + \
        torch.from_numpy(pb.pattern[:, 0].astype(np.int64)).to(device)
    vv = torch.from_numpy(pb.u_ref[:, 1].astype(np.int64)).to(device)[:, None] + \
        torch.from_numpy(pb.pattern[:, 1].astype(np.int64)).to(device)
    # integer u_ref and integer pattern → the bilinear host sample is exactly the pixel value
    pb.host_intensity = images[host[:, None], vv, uu].float().cpu().numpy()
    if block_order == "morton":
        def spread(x):  # 16-bit interleave for the Morton code
            x = x.astype(np.uint64) & np.uint64(0xFFFF)
            x = (x | (x << np.uint64(8))) & np.uint64(0x00FF00FF)
            x = (x | (x << np.uint64(4))) & np.uint64(0x0F0F0F0F)
            x = (x | (x << np.uint64(2))) & np.uint64(0x33333333)
            return (x | (x << np.uint64(1))) & np.uint64(0x55555555)
        ur = pb.u_ref[pb.block_point].astype(np.int64)
        code = spread(ur[:, 0]) | (spread(ur[:, 1]) << np.uint64(1))
        order = np.lexsort((code, pb.block_target, pb.point_host[pb.block_point]))
        pb.block_point = np.ascontiguousarray(pb.block_point[order])
        pb.block_target = np.ascontiguousarray(pb.block_target[order])
    return pb, images
