"""Drop-in for the reference's fragment integration (the second caller of ``integrate``):

    integrate_fragment_point_cloud(depth_data_io, frag_dataset, side, config)
        scripts/processing/reconstruction/depth_optimization/refine_fragment_poses.py:14-58
    integrate_fragment_point_clouds(depth_data_io, fragment_dataset_map, config, workers)
        the parallel part of integrate_and_save_fragment_point_clouds (:61-119), without the saving

Each fragment (``fragment_size`` = 100 frames, pipeline_config.yml:38) is integrated into a FRESH
volume (``vbg_opt=None``) and its point cloud extracted with the default weight threshold 3.0; a
failure or an empty cloud gives ``None`` with the reference's messages.  With
``use_multi_threading`` the reference runs the fragments on a spawn Pool of cpu_count - 1 workers
(utils/paralell_utils.py:55-67): here every worker process opens its own HIP context on the same
GPU (one HIP runtime per process, mqr._lib), so several fragments integrate concurrently on one
MI355X.  Worker results cross the process boundary as (side, positions, normals) arrays.
"""
from __future__ import annotations

import multiprocessing
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np

from .models import Side


@dataclass
class FragmentPoseRefinementConfig:
    """The integration fields of reconstruction_config.py:60-84 (defaults; the pipeline's values are
    in config/pipeline_config.yml:50-58)."""
    device: object = "CUDA:0"
    use_confidence_filtered_depth: bool = True
    confidence_threshold: float = 0.05
    valid_count_threshold: int = 4
    voxel_size: float = 0.01
    block_resolution: int = 16
    block_count: int = 50_000
    depth_max: float = 1.5
    trunc_voxel_multiplier: float = 8.0
    use_multi_threading: bool = False


def integrate_fragment_point_cloud(depth_data_io, frag_dataset, side: Side, config: FragmentPoseRefinementConfig):
    """refine_fragment_poses.py:14-58: fresh volume, integrate, extract_point_cloud(); None on an
    empty cloud or an error (printed as the reference prints it)."""
    from .o3d_utils import integrate
    try:
        vbg = integrate(dataset=frag_dataset, depth_data_io=depth_data_io, side=side,
                        use_confidence_filtered_depth=config.use_confidence_filtered_depth,
                        confidence_threshold=config.confidence_threshold,
                        valid_count_threshold=config.valid_count_threshold, voxel_size=config.voxel_size,
                        block_resolution=config.block_resolution, block_count=config.block_count,
                        depth_max=config.depth_max, trunc_voxel_multiplier=config.trunc_voxel_multiplier,
                        device=config.device, show_progress=False, desc=None, vbg_opt=None)
        pcd = vbg.extract_point_cloud()
        del vbg
        if pcd.point.positions.shape[0] == 0:
            print(f"[Warning] Fragment point cloud for {side.name} is empty (no valid points). "
                  f"Dataset has {len(frag_dataset.timestamps)} frames. "
                  f"This may indicate insufficient depth data or overly strict filtering.")
            return None
        return side, pcd
    except Exception as e:  # noqa: BLE001 -- the reference catches everything per fragment
        ts = frag_dataset.timestamps
        print(f"[Error] integrate_fragment_point_cloud failed for {side.name}: {e}")
        print(f"[Error] Fragment dataset info: {len(ts)} frames, "
              f"timestamps range: {ts.min() if len(ts) > 0 else 'N/A'} - {ts.max() if len(ts) > 0 else 'N/A'}")
        return None


def _worker(args):
    """Pool task: (index, depth_data_io, frag_dataset, side, config) -> (index, result arrays, seconds)."""
    import time
    i, io, ds, side, config = args
    t0 = time.perf_counter()
    # the reference's ParallelWorker (paralell_utils.py:11-19) turns ANY failure of a task into None
    # for that task: library load / HIP context creation in a spawned worker or reading the cloud
    # back must not abort the other fragments
    try:
        r = integrate_fragment_point_cloud(io, ds, side, config)
        if r is None:
            return i, None, time.perf_counter() - t0
        side, pcd = r
        return i, (side, pcd.points, pcd.normals), time.perf_counter() - t0
    except Exception as e:  # noqa: BLE001
        print(f"[Error] integrate_fragment_point_cloud failed for {getattr(side, 'name', side)}: {e}")
        return i, None, time.perf_counter() - t0


def _warm(_):
    """Pool warm-up task: load the library and open the HIP context in the worker."""
    from . import _lib
    _lib.load()
    return os.getpid()


def integrate_fragment_point_clouds(depth_data_io, fragment_dataset_map, config: FragmentPoseRefinementConfig,
                                    workers: Optional[int] = None, pool=None):
    """Every fragment of every side through integrate_fragment_point_cloud, in the reference's
    argument order (sides, then fragments).  With config.use_multi_threading: a spawn Pool of
    `workers` processes (default cpu_count - 1, at most 15: one GPU holds a bounded number of
    contexts), or the caller's `pool`.  Returns [(side, positions, normals) | None] in argument order."""
    args = [(i, depth_data_io, ds, side, config)
            for i, (side, ds) in enumerate((s, d) for s, dss in fragment_dataset_map.items() for d in dss)]
    if not config.use_multi_threading:
        out = [_worker(a) for a in args]
    elif pool is not None:
        out = pool.map(_worker, args)
    else:
        n = workers or max(1, min(multiprocessing.cpu_count() - 1, 15, len(args)))
        os.environ["OMP_NUM_THREADS"] = "1"
        with multiprocessing.get_context("spawn").Pool(processes=n) as p:
            out = p.map(_worker, args)
    res = [None] * len(args)
    for i, r, _ in out:
        res[i] = r
    return res


def fragment_datasets(dataset, fragment_size: int = 100):
    """Consecutive fragment_size-frame slices of a dataset (make_fragments.py's fragment layout;
    its odometry and loop closure are out of scope)."""
    n = len(dataset)
    return [dataset[list(range(a, min(n, a + fragment_size)))] for a in range(0, n, fragment_size)]
