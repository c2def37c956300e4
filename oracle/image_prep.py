"""TEST INFRASTRUCTURE — CPU oracle of the image pipeline.

Only tests/ may import this module, as the checker of frh_image_preprocess; the
product package never imports it.

Restates, per image and with plain numpy, what configs/faster_rcnn_r50_fpn.py:120-139
asks mmdet v1 / mmcv / OpenCV to do (those libraries are absent here and not vendored
in the reference, so this row is "parity unpinned": the restatement follows their
published algorithms, pinned by hand-computed cases in tests/test_image_pipeline.py):

* mmcv.imrescale (keep_ratio): scale = min(max(scale)/max(h, w), min(scale)/min(h, w)),
  new size int(w*scale + 0.5), int(h*scale + 0.5);
* cv2.resize INTER_LINEAR on uint8 (OpenCV imgproc/resize.cpp, scalar path):
  per destination coordinate f = float((d + 0.5)*scale - 0.5) with scale = 1/(dst/src),
  s = floor(f), f -= s, clamped at both borders (f = 0); weights lrint((1 - f)*2048),
  lrint(f*2048); horizontal int pass, vertical (b0*h0 + b1*h1 + 2^21) >> 22, saturated;
  an exact 2x downscale becomes INTER_AREA ((sum of 2x2 + 2) >> 2, the SIMD rounding);
* mmcv.imflip horizontal; mmdet Normalize: (float32(v) - mean) / std in float32 after
  BGR -> RGB; mmcv.impad_to_multiple(size_divisor) with zeros; collate zero-pads to the
  batch's largest padded shape; HWC -> CHW.
"""
import numpy as np


def rescale_size(h, w, scale):
    """mmcv.imrescale's size rule for a (long, short) tuple scale."""
    s = min(max(scale) / max(h, w), min(scale) / min(h, w))
    return int(w * float(s) + 0.5), int(h * float(s) + 0.5), s


def _coef(dst, src):
    scale = 1.0 / (float(dst) / float(src))
    d = np.arange(dst, dtype=np.float64)
    f = ((d + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    lo = s < 0
    f[lo], s[lo] = 0.0, 0
    hi = s >= src - 1
    f[hi], s[hi] = 0.0, src - 1
    a0 = np.rint((np.float32(1.0) - f) * np.float32(2048.0)).astype(np.int64)
    a1 = np.rint(f * np.float32(2048.0)).astype(np.int64)
    return s, np.minimum(s + 1, src - 1), a0, a1


def resize_linear_u8(img, nh, nw):
    """cv2.resize(img, (nw, nh), interpolation=INTER_LINEAR) for uint8 HxWx3 (scalar path)."""
    h, w = img.shape[:2]
    src = img.astype(np.int64)
    if w == 2 * nw and h == 2 * nh:
        s = src[0::2, 0::2] + src[0::2, 1::2] + src[1::2, 0::2] + src[1::2, 1::2]
        return ((s + 2) >> 2).astype(np.uint8)
    x0, x1, a0, a1 = _coef(nw, w)
    y0, y1, b0, b1 = _coef(nh, h)
    hrow = lambda rows: src[rows][:, x0] * a0[None, :, None] + src[rows][:, x1] * a1[None, :, None]
    t = (b0[:, None, None] * hrow(y0) + b1[:, None, None] * hrow(y1) + (1 << 21)) >> 22
    return np.clip(t, 0, 255).astype(np.uint8)


def normalize(img, mean, std, to_rgb):
    x = img.astype(np.float32)
    if to_rgb:
        x = x[..., ::-1]
    return (x - np.asarray(mean, np.float32)) / np.asarray(std, np.float32)


def preprocess(imgs, dst_sizes, flips, mean, std, to_rgb, out_h, out_w):
    """Batch tensor [B, 3, out_h, out_w] float32 of frh_image_preprocess."""
    out = np.zeros((len(imgs), 3, out_h, out_w), np.float32)
    for b, (img, (nh, nw), fl) in enumerate(zip(imgs, dst_sizes, flips)):
        r = resize_linear_u8(img, nh, nw)
        if fl:
            r = r[:, ::-1]
        out[b, :, :nh, :nw] = normalize(r, mean, std, to_rgb).transpose(2, 0, 1)
    return out
