"""Drop-in for the reference's ``processing/reconstruction/utils/o3d_utils.py`` fusion entry points.

    compute_o3d_intrinsic_matrices(dataset)          o3d_utils.py:14-19
    load_depth_map(...)                              o3d_utils.py:109-150
    integrate(dataset, depth_data_io, side, ...)     o3d_utils.py:153-238

``integrate`` keeps the reference signature, frame order, skip rules (missing / invalid frames
dropped, confidence masking with the same thresholds) and error behaviour (a frame touching no
block raises RuntimeError), but hands the frames to the MI355X in batches: host decode of the
next chunk overlaps the device work of the current one, and the device integrates each batch
with one touch launch + one integrate launch (bit-identical to per-frame calls).
The swap in the reference is one import line:
    from processing.reconstruction.utils.o3d_utils import integrate   ->   from mqr.o3d_utils import integrate
"""
from __future__ import annotations

import sys
from concurrent.futures import ThreadPoolExecutor
from typing import Optional

import numpy as np

from .geometry import Image
from .vbg import VoxelBlockGrid

CHUNK = 64  # frames per host->device hand-off (device batches are <= 32 frames)


def compute_o3d_intrinsic_matrices(dataset) -> np.ndarray:
    """(N,3,3) float32 with the Quest->Open3D principal-point flip cx := W - cx."""
    widths = dataset.widths
    k = dataset.get_intrinsic_matrices()
    k[:, 0, 2] = widths - k[:, 0, 2]
    return k


def _masked_depth(depth_data_io, side, index, dataset, use_confidence_filtered_depth, confidence_threshold,
                  valid_count_threshold) -> Optional[np.ndarray]:
    depth = depth_data_io.load_depth_map(side=side, timestamp=dataset.timestamps[index],
                                         width=dataset.widths[index], height=dataset.heights[index],
                                         near=dataset.nears[index], far=dataset.fars[index])
    if depth is None:
        return None
    if use_confidence_filtered_depth:
        cm = depth_data_io.load_confidence_map(side=side, timestamp=dataset.timestamps[index])
        if cm is None:
            print(f"[Warning] Confidence map not found for timestamp {dataset.timestamps[index]}")
        else:
            depth[cm.confidence_map < confidence_threshold] = 0.0
            depth[cm.valid_count < valid_count_threshold] = 0.0
    return depth


def load_depth_map(depth_data_io, side, index: int, dataset, device, use_confidence_filtered_depth: bool,
                   confidence_threshold: float, valid_count_threshold: int) -> Optional[Image]:
    d = _masked_depth(depth_data_io, side, index, dataset, use_confidence_filtered_depth, confidence_threshold,
                      valid_count_threshold)
    return None if d is None else Image(d, device=device)


def integrate(dataset, depth_data_io, side, use_confidence_filtered_depth: bool, confidence_threshold: float,
              valid_count_threshold: int, voxel_size: float, block_resolution: int, block_count: int,
              depth_max: float, trunc_voxel_multiplier: float, device, show_progress: bool = False,
              desc: Optional[str] = None, vbg_opt: Optional[VoxelBlockGrid] = None) -> VoxelBlockGrid:
    vbg = vbg_opt if vbg_opt is not None else VoxelBlockGrid(
        attr_names=("tsdf", "weight"), attr_dtypes=("float32", "float32"), attr_channels=((1), (1)),
        voxel_size=voxel_size, block_resolution=block_resolution, block_count=block_count, device=device)
    n = len(dataset.timestamps)
    extrinsic_wc = dataset.transforms.extrinsics_wc
    intrinsics = compute_o3d_intrinsic_matrices(dataset)

    def load_chunk(lo):
        hi = min(n, lo + CHUNK)
        frames, ok = [], []
        for i in range(lo, hi):
            d = _masked_depth(depth_data_io, side, i, dataset, use_confidence_filtered_depth, confidence_threshold,
                              valid_count_threshold)
            ok.append(d is not None)
            frames.append(d)
        return lo, hi, frames, ok

    bar = None
    if show_progress:
        from tqdm import tqdm
        bar = tqdm(total=n, desc=desc, file=sys.stderr, dynamic_ncols=True, mininterval=0.1)
    with ThreadPoolExecutor(max_workers=1) as pool:
        fut = pool.submit(load_chunk, 0) if n else None
        while fut is not None:
            lo, hi, frames, ok = fut.result()
            fut = pool.submit(load_chunk, hi) if hi < n else None
            shapes = {f.shape for f in frames if f is not None}
            for shape in shapes:  # frames of one capture share a size; group defensively
                sel = [j for j, f in enumerate(frames) if f is not None and f.shape == shape]
                depths = np.stack([frames[j] for j in sel])
                idx = np.array([lo + j for j in sel])
                vbg.integrate_frames(depths, intrinsics[idx].astype(np.float64), extrinsic_wc[idx].astype(np.float64),
                                     depth_scale=1.0, depth_max=float(depth_max),
                                     trunc_voxel_multiplier=float(trunc_voxel_multiplier))
            if bar is not None:
                bar.update(hi - lo)
    if bar is not None:
        bar.close()
    return vbg
