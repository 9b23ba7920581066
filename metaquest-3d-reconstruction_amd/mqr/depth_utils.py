"""Quest depth decoding: FOV tangents -> pinhole, NDC depth buffer -> metric depth.

Mirror of the reference's ``scripts/utils/depth_utils.py:4-46`` (float32 decode; numpy's
weak-scalar promotion keeps the whole decode in float32).  Pinned by
tests/golden/decode_golden.npz, generated from the reference.
"""
from __future__ import annotations

import numpy as np


def compute_depth_camera_params(left, right, top, bottom, width, height):
    """FOV half-angle tangents -> (fx, fy, cx, cy) in the descriptor convention."""
    fx = width / (right + left)
    fy = height / (top + bottom)
    cx = width * right / (right + left)
    cy = height * top / (top + bottom)
    return fx, fy, cx, cy


def compute_ndc_to_linear_depth_params(near, far):
    if np.isinf(far) or far < near:
        return -2.0 * near, -1.0
    return -2.0 * far * near / (far - near), -(far + near) / (far - near)


def to_linear_depth(d, x, y):
    ndc = d * 2.0 - 1.0
    denom = ndc + y
    return np.divide(x, denom, out=np.zeros_like(d), where=denom != 0)


def convert_depth_to_linear(depth_buffer: np.ndarray, near: float, far: float) -> np.ndarray:
    x, y = compute_ndc_to_linear_depth_params(near, far)
    return to_linear_depth(depth_buffer, x, y).astype(np.float32)


def encode_linear_to_ndc(z: np.ndarray, near: float, far: float) -> np.ndarray:
    """Inverse of convert_depth_to_linear (synthetic-capture generator): metric z -> raw buffer.

    z <= 0 (no return) encodes to 1.0, which the reference decodes to 0 (denominator 0)."""
    x, y = compute_ndc_to_linear_depth_params(near, far)
    z = np.asarray(z, dtype=np.float64)
    with np.errstate(divide="ignore", invalid="ignore"):
        ndc = np.where(z > 0, x / np.where(z > 0, z, 1.0) - y, 1.0)
    return np.clip((ndc + 1.0) * 0.5, 0.0, 1.0).astype(np.float32)
