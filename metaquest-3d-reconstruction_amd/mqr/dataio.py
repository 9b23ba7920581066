"""Capture-directory access for the fusion path (Quest layout).

Mirror of the reference's ``DepthDataIO`` (scripts/dataio/depth_data_io.py:14-261) and of the
path layout in ``config/project_path_config.py:39-61, 148-196``:

    <project>/left_depth/<timestamp>.raw          float32 little-endian NDC depth buffer (H*W)
    <project>/left_depth_descriptors.csv          one row per frame (timestamp, size, near/far,
                                                  FOV tangents, UNITY pose)
    <project>/left_depth_confidence/<ts>.npz      {confidence_map f64, valid_count i32}
    <project>/dataset/left_depth_dataset.npz      DepthDataset cache

Same skip rules as the reference: missing file or invalid buffer (all 0, all 1, any NaN, any
negative) -> ``None`` and the frame is dropped.
"""
from __future__ import annotations

from pathlib import Path
from typing import Optional

import numpy as np

from .depth_utils import compute_depth_camera_params, convert_depth_to_linear
from .models import ConfidenceMap, CoordinateSystem, DepthDataset, Side, Transforms

DESCRIPTOR_COLUMNS = [
    "timestamp_ms", "width", "height", "near_z", "far_z",
    "fov_left_angle_tangent", "fov_right_angle_tangent", "fov_top_angle_tangent", "fov_down_angle_tangent",
    "create_pose_location_x", "create_pose_location_y", "create_pose_location_z",
    "create_pose_rotation_x", "create_pose_rotation_y", "create_pose_rotation_z", "create_pose_rotation_w",
]


class DepthPaths:
    def __init__(self, project_dir: Path):
        self.project_dir = Path(project_dir).resolve()

    def depth_dir(self, side: Side) -> Path:
        return self.project_dir / f"{side.value}_depth"

    def depth_map_path(self, side: Side, timestamp: int) -> Path:
        return self.depth_dir(side) / f"{int(timestamp)}.raw"

    def descriptor_path(self, side: Side) -> Path:
        return self.project_dir / f"{side.value}_depth_descriptors.csv"

    def confidence_dir(self, side: Side) -> Path:
        return self.project_dir / f"{side.value}_depth_confidence"

    def confidence_path(self, side: Side, timestamp: int) -> Path:
        return self.confidence_dir(side) / f"{int(timestamp)}.npz"

    def dataset_path(self, side: Side) -> Path:
        return self.project_dir / "dataset" / f"{side.value}_depth_dataset.npz"


class DepthDataIO:
    def __init__(self, project_dir: Path):
        self.paths = DepthPaths(project_dir)
        self.depth_datasets: dict = {}

    # -- descriptors / datasets --------------------------------------------------------
    def load_depth_descriptors(self, side: Side):
        import pandas as pd
        return pd.read_csv(self.paths.descriptor_path(side))

    def build_depth_dataset(self, side: Side) -> DepthDataset:
        df = self.load_depth_descriptors(side)
        cols = {c: [] for c in ("ts", "fx", "fy", "cx", "cy", "pos", "rot", "w", "h", "n", "f", "names")}
        for _, row in df.iterrows():
            ts, w, h = int(row["timestamp_ms"]), int(row["width"]), int(row["height"])
            near, far = float(row["near_z"]), float(row["far_z"])
            fx, fy, cx, cy = compute_depth_camera_params(
                float(row["fov_left_angle_tangent"]), float(row["fov_right_angle_tangent"]),
                float(row["fov_top_angle_tangent"]), float(row["fov_down_angle_tangent"]), w, h)
            if self.load_depth_map(side, ts, w, h, near, far) is None:
                continue
            cols["names"].append(f"{ts}.raw")
            cols["ts"].append(ts)
            cols["fx"].append(fx)
            cols["fy"].append(fy)
            cols["cx"].append(cx)
            cols["cy"].append(cy)
            cols["pos"].append(np.array([row["create_pose_location_x"], row["create_pose_location_y"],
                                         row["create_pose_location_z"]]))
            cols["rot"].append(np.array([row["create_pose_rotation_x"], row["create_pose_rotation_y"],
                                         row["create_pose_rotation_z"], row["create_pose_rotation_w"]]))
            cols["w"].append(w)
            cols["h"].append(h)
            cols["n"].append(near)
            cols["f"].append(far)
        rel = str(self.paths.depth_dir(side).relative_to(self.paths.project_dir))
        return DepthDataset(
            directory_relative_path=rel, image_file_names=np.array(cols["names"]), timestamps=np.array(cols["ts"]),
            fx=np.array(cols["fx"]), fy=np.array(cols["fy"]), cx=np.array(cols["cx"]), cy=np.array(cols["cy"]),
            transforms=Transforms(CoordinateSystem.UNITY, np.array(cols["pos"]), np.array(cols["rot"])),
            widths=np.array(cols["w"]), heights=np.array(cols["h"]), nears=np.array(cols["n"]),
            fars=np.array(cols["f"]))

    def load_depth_dataset(self, side: Side, use_cache: bool = True) -> DepthDataset:
        if side in self.depth_datasets:
            return self.depth_datasets[side]
        path = self.paths.dataset_path(side)
        if use_cache and path.exists():
            ds = DepthDataset.load(path)
        else:
            ds = self.build_depth_dataset(side)
            ds.save(path)
        self.depth_datasets[side] = ds
        return ds

    # -- depth maps -----------------------------------------------------------------------
    @staticmethod
    def is_depth_map_valid(depth_map: np.ndarray) -> bool:
        ok = (depth_map != 0).any() and (depth_map != 1).any()
        ok = ok and not np.isnan(depth_map).any()
        ok = ok and (depth_map >= 0).all()
        return bool(ok)

    def load_raw_depth(self, side: Side, timestamp: int, width: int, height: int) -> Optional[np.ndarray]:
        path = self.paths.depth_map_path(side, timestamp)
        if not path.exists():
            return None
        return np.fromfile(path, dtype="<f4").reshape((int(height), int(width)))

    def load_depth_map(self, side: Side, timestamp: int, width: int, height: int, near: float,
                       far: float) -> Optional[np.ndarray]:
        raw = self.load_raw_depth(side, timestamp, width, height)
        if raw is None or not self.is_depth_map_valid(raw):
            return None
        return convert_depth_to_linear(raw, near, far)

    def load_depth_map_by_index(self, side: Side, dataset: DepthDataset, index: int) -> Optional[np.ndarray]:
        if index < 0 or index >= len(dataset.timestamps):
            return None
        return self.load_depth_map(side, dataset.timestamps[index], dataset.widths[index], dataset.heights[index],
                                   dataset.nears[index], dataset.fars[index])

    # -- confidence maps --------------------------------------------------------------------
    def exists_depth_confidence_map_dir(self, side: Side) -> bool:
        return self.paths.confidence_dir(side).exists()

    def load_confidence_map(self, side: Side, timestamp: int) -> Optional[ConfidenceMap]:
        path = self.paths.confidence_path(side, timestamp)
        if not path.exists():
            return None
        try:
            data = np.load(path)
            return ConfidenceMap(confidence_map=data["confidence_map"], valid_count=data["valid_count"])
        except Exception as e:  # the reference logs and returns None (depth_data_io.py:100-103)
            print(f"[Error] Failed to load confidence map for {side.name} at timestamp {timestamp}: {e}")
            return None

    def save_confidence_map(self, side: Side, timestamp: int, confidence_map: ConfidenceMap) -> None:
        path = self.paths.confidence_path(side, timestamp)
        path.parent.mkdir(parents=True, exist_ok=True)
        np.savez(path, confidence_map=confidence_map.confidence_map, valid_count=confidence_map.valid_count)
