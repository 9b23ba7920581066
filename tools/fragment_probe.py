"""Fragment path phases (tools/: integrate() per 100-frame fragment into a fresh 50 000-block volume, then\nextract_point_cloud) on the bench's 500-frame capture, across o3d_utils.FIRST_CHUNK values."""
import os, sys, time, json, tempfile, shutil
sys.path.insert(0, "metaquest-3d-reconstruction_amd")
import numpy as np
from mqr import synthetic, o3d_utils
from mqr.confidence import DepthConfidenceEstimationConfig, estimate_depth_confidences
from mqr.dataio import DepthDataIO
from mqr.models import CoordinateSystem, Side
from mqr.fragments import FragmentPoseRefinementConfig, fragment_datasets, integrate_fragment_point_cloud
seq = synthetic.make_sequence_fast("room", poses=synthetic.room_loop_poses(500), device="cuda:0")
cap = {"raw": seq["raw_t"].cpu().numpy(), "unity": seq["unity"], "tangents": seq["tangents"], "near": seq["near"], "far": seq["far"], "width": seq["width"], "height": seq["height"]}
tmp = tempfile.mkdtemp()
synthetic.write_capture(tmp, cap)
io = DepthDataIO(tmp)
estimate_depth_confidences(io, DepthConfidenceEstimationConfig(target_frame_range=10, depth_max=4.0, error_threshold=0.08, skip_if_output_dir_exists=False, device=0), sides=[Side.LEFT])
ds = io.load_depth_dataset(Side.LEFT)
ds.transforms = ds.transforms.convert_coordinate_system(target_coordinate_system=CoordinateSystem.OPEN3D, is_camera=True)
frags = fragment_datasets(ds, 100)
cfg = FragmentPoseRefinementConfig(device="CUDA:0", confidence_threshold=0.02, valid_count_threshold=2, voxel_size=0.01, block_count=50_000, depth_max=4.0, trunc_voxel_multiplier=10.0)
from mqr.vbg import VoxelBlockGrid
res = {}
for rep in range(4):
    for first in (127, 32, 16):
        o3d_utils.FIRST_CHUNK = first
        t0 = time.perf_counter()
        out = []
        for fd in frags:
            ta = time.perf_counter()
            vbg = o3d_utils.integrate(dataset=fd, depth_data_io=io, side=Side.LEFT, use_confidence_filtered_depth=True, confidence_threshold=0.02, valid_count_threshold=2, voxel_size=0.01, block_resolution=16, block_count=50000, depth_max=4.0, trunc_voxel_multiplier=10.0, device="CUDA:0")
            tb = time.perf_counter()
            pcd = vbg.extract_point_cloud()
            n = pcd.points.shape[0]
            tc = time.perf_counter()
            del vbg, pcd
            td = time.perf_counter()
            out.append({"integrate": (tb-ta)*1e3, "extract+host": (tc-tb)*1e3, "release": (td-tc)*1e3, "split": {k: round(v*1e3,2) if isinstance(v,float) else v for k,v in o3d_utils.last_integrate_times.__dict__.items()}})
        if rep:
            res.setdefault(first, []).append({"total_ms": (time.perf_counter()-t0)*1e3, "fragments": out})
print(json.dumps({"first_chunk_ab": {f: {"total_ms": sorted(x["total_ms"] for x in v), "last": v[-1]["fragments"]} for f, v in res.items()}}))
t0 = time.perf_counter(); v = VoxelBlockGrid(attr_names=("tsdf","weight"), attr_dtypes=("float32","float32"), attr_channels=((1),(1)), voxel_size=0.01, block_resolution=16, block_count=50000, device="CUDA:0"); t1=time.perf_counter(); del v; t2=time.perf_counter()
print(json.dumps({"create_ms": (t1-t0)*1e3, "delete_ms": (t2-t1)*1e3}))
shutil.rmtree(tmp)
