"""Generate the golden fixtures in tests/golden/ by running the REFERENCE's own Python code.

Run here (this container) only:  python tests/golden/make_golden.py [decode | ragged]
It imports /root/reference/scripts (read-only) with ``open3d`` and ``cv2`` stubbed by
MagicMock (neither is installed; the functions exercised never touch them), feeds it synthetic
captures, and stores inputs + reference outputs as .npz data.  Nothing from the reference is
copied; the GPU box never sees the reference -- only these vectors.

Fixtures:
  decode_golden.npz      raw NDC buffers x (near, far) -> convert_depth_to_linear (depth_utils.py:21-46)
                         + is_depth_map_valid verdicts (depth_data_io.py:80-85)
  confidence_golden.npz  per sequence (sphere / room): the capture (raw buffers + descriptor rows), the
                         DepthDataset fields and compute_o3d_intrinsic_matrices (o3d_utils.py:14-19,
                         <seq>_fx / _cx / _K), the OPEN3D extrinsics_wc / _cw (transforms.py:57-72,
                         164-220) and np.linalg.inv(extrinsics_cw), the decoded depth; then
                         build_confidence_map (estimate_depth_confidences.py:15-79) for every ref frame
                         under two parameter sets (_conf_a/_valid_a, _conf_b/_valid_b) and
                         compute_pixel_error_map (compute_pixel_error_map.py:120-220) for frame pairs
  confidence_ragged_golden.npz  a capture with frames of two sizes (per-row width / height in the
                         descriptor CSV), build_confidence_map for every ref frame, two parameter sets
"""
from __future__ import annotations

import os
import sys
import tempfile
from pathlib import Path
from unittest.mock import MagicMock

import numpy as np

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
REF = Path("/root/reference/scripts")


def import_reference():
    for m in ("open3d", "open3d.core", "cv2"):
        sys.modules[m] = MagicMock()
    sys.path.insert(0, str(REF))
    from config.project_path_config import DepthPathConfig
    from dataio.depth_data_io import DepthDataIO
    from models.side import Side
    from models.transforms import CoordinateSystem
    from processing.reconstruction.confidence_estimation.compute_pixel_error_map import compute_pixel_error_map
    from processing.reconstruction.confidence_estimation.estimate_depth_confidences import build_confidence_map
    from processing.reconstruction.utils.o3d_utils import compute_o3d_intrinsic_matrices
    from utils.depth_utils import convert_depth_to_linear
    return dict(DepthPathConfig=DepthPathConfig, DepthDataIO=DepthDataIO, Side=Side, CoordinateSystem=CoordinateSystem,
                compute_pixel_error_map=compute_pixel_error_map, build_confidence_map=build_confidence_map,
                compute_o3d_intrinsic_matrices=compute_o3d_intrinsic_matrices,
                convert_depth_to_linear=convert_depth_to_linear)


def make_decode(ref):
    rng = np.random.default_rng(7)
    raw = rng.random((6, 24, 32)).astype(np.float32)
    raw[0, 0, :4] = [0.0, 1.0, 0.5, 0.999999]
    raw[1] = 0.0                      # invalid: all zero
    raw[2] = 1.0                      # invalid: all one
    raw[3, 5, 5] = np.nan             # invalid: NaN
    raw[4, 2, 2] = -0.25              # invalid: negative
    params = np.array([[0.1, np.inf], [0.1, 10.0], [0.5, 0.2], [0.05, 100.0]])
    io = ref["DepthDataIO"](depth_path_config=None)
    valid = np.array([io.is_depth_map_valid(r) for r in raw])
    out = np.stack([np.stack([ref["convert_depth_to_linear"](r, float(n), float(f)) for r in raw]) for n, f in params])
    # the pipeline passes DepthDataset.nears[i] / fars[i], numpy float64 scalars: under numpy >= 2
    # (NEP 50) they are strongly typed and the decode's division runs in float64 -> separate vectors
    out64 = np.stack([np.stack([ref["convert_depth_to_linear"](r, np.float64(n), np.float64(f)) for r in raw])
                      for n, f in params])
    np.savez_compressed(HERE / "decode_golden.npz", raw=raw, params=params, valid=valid, linear=out,
                        linear64=out64, numpy_version=np.array(np.__version__))


def capture_to_reference(ref, project_dir):
    io = ref["DepthDataIO"](depth_path_config=ref["DepthPathConfig"](project_dir=Path(project_dir)))
    side = ref["Side"].LEFT
    ds = io.build_depth_dataset(side=side)
    K = ref["compute_o3d_intrinsic_matrices"](dataset=ds)
    o3d = ds.transforms.convert_coordinate_system(target_coordinate_system=ref["CoordinateSystem"].OPEN3D,
                                                  is_camera=True)
    T_cw = o3d.extrinsics_cw
    T_wc = o3d.extrinsics_wc
    T_cw_inv = np.linalg.inv(T_cw)
    depths = np.stack([io.load_depth_map_by_index(side=side, dataset=ds, index=i) for i in range(len(ds))])
    return io, ds, K, T_cw, T_wc, T_cw_inv, depths


def make_dataset_and_confidence(ref):
    sys.path.insert(0, str(REPO / "metaquest-3d-reconstruction_amd"))
    from mqr import synthetic

    seqs = {
        "sphere": synthetic.make_sequence("sphere", n=12, height=120, width=160, f=131.25, noise=True, seed=3),
        "room": synthetic.make_sequence("room", n=8, height=96, width=128, f=105.0, noise=True, seed=4),
    }
    out = {}
    for name, seq in seqs.items():
        with tempfile.TemporaryDirectory() as td:
            synthetic.write_capture(td, seq)
            import pandas as pd
            csv = pd.read_csv(Path(td) / "left_depth_descriptors.csv")
            io, ds, K, T_cw, T_wc, T_cw_inv, depths = capture_to_reference(ref, td)
            out[f"{name}_raw"] = seq["raw"]
            out[f"{name}_descriptor"] = csv.to_numpy(dtype=np.float64)
            out[f"{name}_descriptor_cols"] = np.array(list(csv.columns))
            out[f"{name}_fx"] = ds.fx
            out[f"{name}_cx"] = ds.cx
            out[f"{name}_K"] = K
            out[f"{name}_T_cw"] = T_cw
            out[f"{name}_T_wc"] = T_wc
            out[f"{name}_T_cw_inv"] = T_cw_inv
            out[f"{name}_depth"] = depths
            # confidence for every reference frame, two parameter sets
            for tag, (r, dmax, thr) in {"a": (3, 3.0, 0.05), "b": (10, 4.0, 0.08)}.items():
                confs, valids = [], []
                for i in range(len(ds)):
                    cm = ref["build_confidence_map"](io, ds, K, T_cw, T_cw_inv, ref["Side"].LEFT, i,
                                                     target_frame_range=r, depth_max=dmax, error_threshold=thr)
                    confs.append(cm.confidence_map)
                    valids.append(cm.valid_count)
                out[f"{name}_conf_{tag}"] = np.stack(confs)
                out[f"{name}_valid_{tag}"] = np.stack(valids)
            pairs = [(0, 1), (2, 5), (5, 2), (len(ds) - 1, 0)]
            out[f"{name}_pairs"] = np.array(pairs)
            out[f"{name}_err"] = np.stack([
                ref["compute_pixel_error_map"](K, T_cw, T_cw_inv, a, depths[a], b, depths[b], depth_max=3.0)
                for a, b in pairs])
    np.savez_compressed(HERE / "confidence_golden.npz", **out)


def make_ragged_confidence(ref):
    """confidence_ragged_golden.npz: one capture whose frames have two sizes (the descriptor CSV
    gives each frame's width / height, depth_data_io.py:187-188) along one room walk; the
    reference's build_confidence_map for every reference frame (windows mixing both sizes: its
    bilinear_interpolate_depth bounds-checks against the target's own h, w).  Per-frame arrays are
    stored under indexed keys (raw_<i>, conf_<tag>_<i>, valid_<tag>_<i>)."""
    sys.path.insert(0, str(REPO / "metaquest-3d-reconstruction_amd"))
    import pandas as pd
    from mqr import synthetic
    poses = synthetic.room_loop_poses(40)[::3][:12]
    parts = [(0, 5, 120, 160, 131.25), (5, 9, 96, 128, 105.0), (9, 12, 120, 160, 131.25)]
    out = {}
    with tempfile.TemporaryDirectory() as td:
        td = Path(td)
        (td / "left_depth").mkdir()
        rows = []
        raws = []
        for k, (a, b, h, w, f) in enumerate(parts):
            seq = synthetic.make_sequence("room", poses=poses[a:b], height=h, width=w, f=f, noise=True, seed=30 + k)
            sub = td / f"part{k}"
            synthetic.write_capture(sub, seq, t0=1_000_000 + 33 * a)
            rows.append(pd.read_csv(sub / "left_depth_descriptors.csv"))
            for raw in sorted((sub / "left_depth").glob("*.raw")):
                raw.rename(td / "left_depth" / raw.name)
            raws.extend(seq["raw"])
        csv = pd.concat(rows)
        csv.to_csv(td / "left_depth_descriptors.csv", index=False)
        io, ds, K, T_cw, T_wc, T_cw_inv, _ = capture_to_reference_ragged(ref, td)
        out["descriptor"] = csv.to_numpy(dtype=np.float64)
        out["descriptor_cols"] = np.array(list(csv.columns))
        out["n"] = np.array(len(ds))
        out["K"], out["T_cw"], out["T_cw_inv"] = K, T_cw, T_cw_inv
        for i, r in enumerate(raws):
            out[f"raw_{i}"] = r
        for tag, (r, dmax, thr) in {"a": (3, 3.0, 0.05), "b": (10, 4.0, 0.08)}.items():
            for i in range(len(ds)):
                cm = ref["build_confidence_map"](io, ds, K, T_cw, T_cw_inv, ref["Side"].LEFT, i, target_frame_range=r,
                                                 depth_max=dmax, error_threshold=thr)
                out[f"conf_{tag}_{i}"] = cm.confidence_map
                out[f"valid_{tag}_{i}"] = cm.valid_count
    np.savez_compressed(HERE / "confidence_ragged_golden.npz", **out)


def capture_to_reference_ragged(ref, project_dir):
    io = ref["DepthDataIO"](depth_path_config=ref["DepthPathConfig"](project_dir=Path(project_dir)))
    ds = io.build_depth_dataset(side=ref["Side"].LEFT)
    K = ref["compute_o3d_intrinsic_matrices"](dataset=ds)
    o3d = ds.transforms.convert_coordinate_system(target_coordinate_system=ref["CoordinateSystem"].OPEN3D,
                                                  is_camera=True)
    return io, ds, K, o3d.extrinsics_cw, o3d.extrinsics_wc, np.linalg.inv(o3d.extrinsics_cw), None


if __name__ == "__main__":
    ref = import_reference()
    if "ragged" in sys.argv[1:]:
        make_ragged_confidence(ref)
    else:
        make_decode(ref)
        if "decode" not in sys.argv[1:]:
            make_dataset_and_confidence(ref)
            make_ragged_confidence(ref)
    for f in sorted(HERE.glob("*.npz")):
        print(f.name, os.path.getsize(f))
