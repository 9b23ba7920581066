"""Pose / camera / confidence containers feeding the fusion path.

Host-side mirror of the reference's ``scripts/models`` surface that the TSDF path consumes:
``Transforms`` (models/transforms.py:42-220), ``CameraDataset`` / ``DepthDataset``
(models/camera_dataset.py:13-214), ``ConfidenceMap`` (models/confidence_map.py:7-32) and
``Side`` (models/side.py).  The arithmetic order (float32 4x4 extrinsics, ``np.linalg.inv``
for world->camera, scipy quaternions in (x, y, z, w) order) follows the reference so the
matrices handed to the kernels are bit-identical to what the reference hands to Open3D
(pinned by the dataset fields in tests/golden/confidence_golden.npz, tests/test_dataio_golden.py).
"""
from __future__ import annotations

from dataclasses import dataclass
from enum import Enum
from pathlib import Path
from typing import Iterator

import numpy as np
from scipy.spatial.transform import Rotation


class Side(Enum):
    LEFT = "left"
    RIGHT = "right"


class CoordinateSystem(Enum):
    """World/camera axis conventions (reference transforms.py:8-32)."""
    UNITY = "Unity"        # world Y-up left-handed; camera X-right, Y-up, Z-forward
    OPEN3D = "Open3D"      # world Y-up right-handed; camera X-right, Y-down, Z-forward
    NERFSTUDIO = "NerfStudio"
    COLMAP = "COLMAP"


class ExtrinsicMode(Enum):
    CameraToWorld = "camera_to_world"
    WorldToCamera = "world_to_camera"


def _world_basis(cs: CoordinateSystem) -> np.ndarray:
    if cs == CoordinateSystem.UNITY:
        return np.eye(3)
    if cs == CoordinateSystem.OPEN3D:
        return np.diag((1, 1, -1))
    if cs == CoordinateSystem.NERFSTUDIO:
        return np.array([[1, 0, 0], [0, 0, 1], [0, 1, 0]])
    if cs == CoordinateSystem.COLMAP:
        return np.diag((1, -1, 1))
    raise ValueError(f"Unknown coordinate system: {cs}")


def _camera_basis(cs: CoordinateSystem) -> np.ndarray:
    if cs == CoordinateSystem.UNITY:
        return np.eye(3)
    if cs == CoordinateSystem.OPEN3D:
        return np.diag((1, -1, -1))
    if cs == CoordinateSystem.NERFSTUDIO:
        return np.array([[1, 0, 0], [0, 0, 1], [0, -1, 0]])
    if cs == CoordinateSystem.COLMAP:
        return np.eye(3)
    raise ValueError(f"Unknown coordinate system: {cs}")


@dataclass
class Transforms:
    """Camera poses: positions (N,3) camera centres, rotations (N,4) camera->world quaternions (x,y,z,w)."""
    coordinate_system: CoordinateSystem
    positions: np.ndarray
    rotations: np.ndarray

    @property
    def extrinsics_wc(self) -> np.ndarray:
        """(N,4,4) float32 world->camera (the extrinsic Open3D integrate takes)."""
        return self.to_extrinsic_matrices(ExtrinsicMode.WorldToCamera)

    @property
    def extrinsics_cw(self) -> np.ndarray:
        """(N,4,4) float32 camera->world."""
        return self.to_extrinsic_matrices(ExtrinsicMode.CameraToWorld)

    def to_extrinsic_matrices(self, mode: ExtrinsicMode = ExtrinsicMode.WorldToCamera) -> np.ndarray:
        n = len(self.positions)
        m = np.zeros((n, 4, 4), dtype=np.float32)
        m[:, :3, :3] = Rotation.from_quat(self.rotations).as_matrix()
        m[:, :3, 3] = self.positions
        m[:, 3, 3] = 1.0
        if mode == ExtrinsicMode.CameraToWorld:
            return m
        if mode == ExtrinsicMode.WorldToCamera:
            return np.linalg.inv(m)
        raise ValueError(f"Unsupported extrinsic mode: {mode}")

    def convert_coordinate_system(self, target_coordinate_system: CoordinateSystem, is_camera: bool = False,
                                  skip_rotation: bool = False) -> "Transforms":
        src = self.coordinate_system
        if src == target_coordinate_system:
            return self
        conv = _world_basis(target_coordinate_system) @ _world_basis(src).T
        positions = (conv @ self.positions.T).T
        if skip_rotation:
            return Transforms(target_coordinate_system, positions, self.rotations)
        rot = Rotation.from_quat(self.rotations).as_matrix()
        if is_camera:
            rot = rot @ _camera_basis(src).T
        rot = conv @ rot @ conv.T
        if is_camera:
            rot = rot @ _camera_basis(target_coordinate_system)
        return Transforms(target_coordinate_system, positions, Rotation.from_matrix(rot).as_quat())

    def to_dict(self) -> dict:
        return {"coordinate_system": self.coordinate_system, "positions": self.positions,
                "rotations": self.rotations}

    def __len__(self) -> int:
        return len(self.positions)


@dataclass
class CameraDataset:
    directory_relative_path: str
    image_file_names: np.ndarray
    timestamps: np.ndarray
    fx: np.ndarray
    fy: np.ndarray
    cx: np.ndarray
    cy: np.ndarray
    transforms: Transforms
    widths: np.ndarray
    heights: np.ndarray

    def __post_init__(self):
        n = self.timestamps.shape[0]
        for v in self.to_dict().values():
            if isinstance(v, np.ndarray) and v.ndim > 0:
                assert v.shape[0] == n

    def to_dict(self) -> dict:
        return {
            "directory_relative_path": self.directory_relative_path,
            "image_file_names": self.image_file_names,
            "timestamps": self.timestamps,
            "fx": self.fx, "fy": self.fy, "cx": self.cx, "cy": self.cy,
            "coordinate_system": self.transforms.coordinate_system.name,
            "positions": self.transforms.positions,
            "rotations": self.transforms.rotations,
            "widths": self.widths, "heights": self.heights,
        }

    @classmethod
    def from_dict(cls, data: dict):
        data = dict(data)
        if "coordinate_system" in data:
            data["transforms"] = Transforms(CoordinateSystem[str(data.pop("coordinate_system"))],
                                            data.pop("positions"), data.pop("rotations"))
        return cls(**data)

    def __len__(self) -> int:
        return len(self.timestamps)

    def __getitem__(self, idx):
        data = self.to_dict()
        if isinstance(idx, (int, np.integer)):
            return {k: (v[idx] if isinstance(v, np.ndarray) and v.ndim > 0 else v) for k, v in data.items()}
        if isinstance(idx, (slice, list, np.ndarray)):
            return self.__class__.from_dict(
                {k: (v[idx] if isinstance(v, np.ndarray) and v.ndim > 0 else v) for k, v in data.items()})
        raise TypeError(f"Unsupported index type: {type(idx)}")

    def __iter__(self) -> Iterator[dict]:
        for i in range(len(self)):
            yield self[i]

    def get_intrinsic_matrices(self) -> np.ndarray:
        """(N,3,3) float32 pinhole matrices in the descriptor's (un-flipped) convention."""
        k = np.zeros((len(self.fx), 3, 3), dtype=np.float32)
        k[:, 0, 0] = self.fx
        k[:, 1, 1] = self.fy
        k[:, 2, 2] = 1.0
        k[:, 0, 2] = self.cx
        k[:, 1, 2] = self.cy
        return k

    def split(self, fragment_size: int):
        return [self[i:i + fragment_size] for i in range(0, len(self), fragment_size)]

    def save(self, path: Path):
        path = Path(path)
        path.parent.mkdir(parents=True, exist_ok=True)
        np.savez(path, **self.to_dict())

    @classmethod
    def load(cls, path: Path):
        return cls.from_dict(dict(np.load(path, allow_pickle=False)))


@dataclass
class DepthDataset(CameraDataset):
    nears: np.ndarray
    fars: np.ndarray

    def to_dict(self) -> dict:
        d = super().to_dict()
        d["nears"] = self.nears
        d["fars"] = self.fars
        return d


@dataclass
class ConfidenceMap:
    """Per-pixel multi-view consistency: confidence_map f64 (H,W), valid_count i32 (H,W)."""
    confidence_map: np.ndarray
    valid_count: np.ndarray

    def __post_init__(self):
        if self.confidence_map.shape != self.valid_count.shape:
            raise ValueError("Confidence map and valid mask must have the same shape.")
        if self.confidence_map.ndim != 2:
            raise ValueError("Confidence map must be a 2D array.")

    @property
    def shape(self):
        return self.confidence_map.shape
