"""NumPy reference of the on-device SimCLR augmentation (``csrc/augment.hip``).

Same counter-based RNG (splitmix64 keyed by seed / step counter / view / dataset index), same
parameter samplers (torchvision's RandomResizedCrop / ColorJitter / RandomGrayscale /
RandomHorizontalFlip logic, ``/root/reference/dataset.py:19-38``) and the same PIL-style pixel
math.  It is the CPU data path (gloo tests, CPU runs) and the parity oracle of the HIP kernel.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import numpy as np

M64 = (1 << 64) - 1


def splitmix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M64
    return x ^ (x >> 31)


class Rng:
    def __init__(self, key: int):
        self.key = key
        self.ctr = 0

    def _next(self) -> int:
        self.ctr += 1
        return splitmix64(self.key ^ ((0xD1B54A32D192ED03 * self.ctr) & M64))

    def uniform(self, a: float = 0.0, b: float = 1.0) -> float:
        u = np.float32((self._next() >> 40) * (1.0 / 16777216.0))
        return float(np.float32(a) + (np.float32(b) - np.float32(a)) * u)

    def randint(self, lo: int, hi_excl: int) -> int:
        return lo + int(self._next() % (hi_excl - lo))


def image_key(seed: int, counter: int, view: int, idx: int) -> int:
    a = splitmix64((counter * 0x9E3779B97F4A7C15 + view) & M64)
    b = splitmix64((idx + 0x632BE59BD9B4E019) & M64)
    return splitmix64((seed ^ a ^ b) & M64)


def sample_params(rng: Rng, H: int, W: int, strength: float) -> dict:
    f32 = np.float32
    area = f32(H * W)
    lr0, lr1 = f32(math.log(3 / 4)), f32(math.log(4 / 3))
    P = {}
    found = False
    for _ in range(10):
        target = area * f32(rng.uniform(0.08, 1.0))
        ar = f32(math.exp(rng.uniform(lr0, lr1)))
        w = int(np.rint(np.sqrt(f32(target * ar))))
        h = int(np.rint(np.sqrt(f32(target / ar))))
        if 0 < w <= W and 0 < h <= H:
            P["ci"] = rng.randint(0, H - h + 1)
            P["cj"] = rng.randint(0, W - w + 1)
            P["ch"], P["cw"] = h, w
            found = True
            break
    if not found:
        in_ratio = W / H
        if in_ratio < 3 / 4:
            w = W
            h = int(np.rint(w / (3 / 4)))
        elif in_ratio > 4 / 3:
            h = H
            w = int(np.rint(h * (4 / 3)))
        else:
            w, h = W, H
        P.update(ci=(H - h) // 2, cj=(W - w) // 2, ch=h, cw=w)
    P["flip"] = rng.uniform() < 0.5
    P["jitter"] = not (0.8 < rng.uniform())
    order = [0, 1, 2, 3]
    for i in range(3, 0, -1):
        j = rng.randint(0, i + 1)
        order[i], order[j] = order[j], order[i]
    P["order"] = order
    b = c = s = 0.8 * strength
    hh = 0.2 * strength
    P["fb"] = rng.uniform(max(0.0, 1 - b), 1 + b)
    P["fc"] = rng.uniform(max(0.0, 1 - c), 1 + c)
    P["fs"] = rng.uniform(max(0.0, 1 - s), 1 + s)
    P["fh"] = rng.uniform(-hh, hh)
    P["gray"] = rng.uniform() < 0.2
    return P


def _clip_trunc(v):
    return np.clip(np.floor(v), 0, 255)


def _luma(r, g, b):
    return (r.astype(np.int64) * 19595 + g.astype(np.int64) * 38470 + b.astype(np.int64) * 7471
            + 0x8000) >> 16


def _rgb2hsv(r, g, b):
    mx = np.maximum(r, np.maximum(g, b))
    mn = np.minimum(r, np.minimum(g, b))
    d = mx - mn
    v = mx
    s = np.where(mx > 0, d / np.where(mx > 0, mx, 1), 0)
    dd = np.where(d > 0, d, 1)
    h = np.where(mx == r, (g - b) / dd, np.where(mx == g, 2 + (b - r) / dd, 4 + (r - g) / dd))
    h = np.where(d > 0, h / 6.0, 0.0)
    h = h - np.floor(h)
    return h, s, v


def _hsv2rgb(h, s, v):
    h6 = h * 6.0
    i = np.floor(h6).astype(np.int64) % 6
    f = h6 - np.floor(h6)
    p, q, t = v * (1 - s), v * (1 - s * f), v * (1 - s * (1 - f))
    r = np.select([i == 0, i == 1, i == 2, i == 3, i == 4], [v, q, p, p, t], v)
    g = np.select([i == 0, i == 1, i == 2, i == 3, i == 4], [t, v, v, q, p], p)
    b = np.select([i == 0, i == 1, i == 2, i == 3, i == 4], [p, p, t, v, v], q)
    return r, g, b


def apply_params(img: np.ndarray, P: dict, OH: int, OW: int) -> np.ndarray:
    """img uint8 [H, W, 3] -> float32 [OH, OW, 3] in [0, 255] (before /255)."""
    f32 = np.float32
    ch, cw, ci, cj = P["ch"], P["cw"], P["ci"], P["cj"]
    oy, ox = np.meshgrid(np.arange(OH), np.arange(OW), indexing="ij")
    if P["flip"]:
        ox = OW - 1 - ox
    fy = np.clip((oy + f32(0.5)) * f32(ch / OH) - f32(0.5), 0, ch - 1).astype(f32)
    fx = np.clip((ox + f32(0.5)) * f32(cw / OW) - f32(0.5), 0, cw - 1).astype(f32)
    y0 = np.floor(fy).astype(np.int64)
    x0 = np.floor(fx).astype(np.int64)
    y1 = np.minimum(y0 + 1, ch - 1)
    x1 = np.minimum(x0 + 1, cw - 1)
    wy = (fy - y0)[..., None]
    wx = (fx - x0)[..., None]
    src = img.astype(f32)
    p00 = src[ci + y0, cj + x0]
    p01 = src[ci + y0, cj + x1]
    p10 = src[ci + y1, cj + x0]
    p11 = src[ci + y1, cj + x1]
    top = p00 + wx * (p01 - p00)
    bot = p10 + wx * (p11 - p10)
    out = np.clip(np.floor(top + wy * (bot - top) + 0.5), 0, 255).astype(f32)
    R, G, B = out[..., 0], out[..., 1], out[..., 2]
    if P["jitter"]:
        for op in P["order"]:
            if op == 0:
                R, G, B = (_clip_trunc(R * f32(P["fb"])), _clip_trunc(G * f32(P["fb"])),
                           _clip_trunc(B * f32(P["fb"])))
            elif op == 1:
                mean = np.floor(_luma(R, G, B).sum() / (OH * OW) + 0.5)
                fc = f32(P["fc"])
                R, G, B = (_clip_trunc(mean + fc * (R - mean)), _clip_trunc(mean + fc * (G - mean)),
                           _clip_trunc(mean + fc * (B - mean)))
            elif op == 2:
                l = _luma(R, G, B).astype(f32)
                fs = f32(P["fs"])
                R, G, B = (_clip_trunc(l + fs * (R - l)), _clip_trunc(l + fs * (G - l)),
                           _clip_trunc(l + fs * (B - l)))
            else:
                h, s, v = _rgb2hsv(R / 255.0, G / 255.0, B / 255.0)
                h = h + P["fh"]
                h = h - np.floor(h)
                r, g, b = _hsv2rgb(h, s, v)
                R = np.clip(np.floor(r * 255 + 0.5), 0, 255)
                G = np.clip(np.floor(g * 255 + 0.5), 0, 255)
                B = np.clip(np.floor(b * 255 + 0.5), 0, 255)
    if P["gray"]:
        l = _luma(R, G, B).astype(f32)
        R = G = B = l
    return np.stack([R, G, B], axis=-1).astype(f32)


def augment_batch(images: np.ndarray, indices: np.ndarray, views: int, OH: int, OW: int,
                  strength: float, seed: int, counter: int, view_offset: int = 0,
                  augment: bool = True) -> np.ndarray:
    """-> float32 [views * n, 3, OH, OW] in [0, 1] (view-major, like the kernel)."""
    n = len(indices)
    H, W = images.shape[1], images.shape[2]
    out = np.empty((views * n, 3, OH, OW), dtype=np.float32)
    for v in range(views):
        for b, idx in enumerate(indices):
            img = images[int(idx)]
            if augment:
                P = sample_params(Rng(image_key(seed, counter, v + view_offset, int(idx))), H, W,
                                  strength)
                pix = apply_params(img, P, OH, OW)
            else:
                pix = img.astype(np.float32)
            out[v * n + b] = pix.transpose(2, 0, 1) / 255.0
    return out
