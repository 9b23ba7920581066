"""The fragment path (refine_fragment_poses.py:14-58, 81-90): every fragment of a capture into a
FRESH volume through the drop-in integrate (confidence-masked, pipeline_config.yml:50-58 values),
then extract_point_cloud() -- on a spawn Pool of 4 worker processes sharing one GPU, each with its
own HIP context.  Every fragment's point cloud equals the oracle's (volume of the same masked
frames, points at weight 3.0), and the pool's results equal the in-process sequential run."""
import numpy as np
import pytest

import oracle
from gpu_helpers import compare_points_fast

pytestmark = pytest.mark.gpu


def test_fragments_on_a_process_pool_match_oracle(tmp_path):
    from mqr import _lib, synthetic
    from mqr.confidence import DepthConfidenceEstimationConfig, estimate_depth_confidences
    from mqr.dataio import DepthDataIO
    from mqr.fragments import FragmentPoseRefinementConfig, fragment_datasets, integrate_fragment_point_clouds
    from mqr.models import CoordinateSystem, Side
    from mqr.o3d_utils import _masked_depth, compute_o3d_intrinsic_matrices
    _lib.load()
    seq = synthetic.make_sequence("room", n=180, height=240, width=320, f=262.5, noise=True, seed=17)
    synthetic.write_capture(tmp_path, seq)
    io = DepthDataIO(tmp_path)
    estimate_depth_confidences(io, DepthConfidenceEstimationConfig(target_frame_range=10, depth_max=4.0,
                                                                   error_threshold=0.08,
                                                                   skip_if_output_dir_exists=False),
                               sides=[Side.LEFT])
    ds = io.load_depth_dataset(Side.LEFT)
    ds.transforms = ds.transforms.convert_coordinate_system(target_coordinate_system=CoordinateSystem.OPEN3D,
                                                            is_camera=True)
    frags = fragment_datasets(ds, 30)
    assert len(frags) == 6
    cfg = FragmentPoseRefinementConfig(device="CUDA:0", confidence_threshold=0.02, valid_count_threshold=2,
                                       voxel_size=0.01, block_count=50_000, depth_max=4.0,
                                       trunc_voxel_multiplier=10.0, use_multi_threading=True)
    pooled = integrate_fragment_point_clouds(io, {Side.LEFT: frags}, cfg, workers=4)
    cfg.use_multi_threading = False
    seq_res = integrate_fragment_point_clouds(io, {Side.LEFT: frags}, cfg)
    kw = dict(use_confidence_filtered_depth=True, confidence_threshold=0.02, valid_count_threshold=2)
    for fd, r, r2 in zip(frags, pooled, seq_res):
        assert r is not None and r2 is not None
        side, p, n = r
        assert side == Side.LEFT
        # the point order follows the pool's block order, which the parallel touch allocates in
        # arrival order (as Open3D's hash map does): equal as sets of (position, normal) rows
        a, b = np.concatenate([p, n], 1), np.concatenate([r2[1], r2[2]], 1)
        assert np.array_equal(a[np.lexsort(a.T[::-1])], b[np.lexsort(b.T[::-1])])
        ref = oracle.OracleVBG(0.01, 16, 4096)
        K = compute_o3d_intrinsic_matrices(fd).astype(np.float64)
        T = fd.transforms.extrinsics_wc.astype(np.float64)
        for i in range(len(fd)):
            d = _masked_depth(io, Side.LEFT, i, fd, **kw)
            ref.integrate_frame(d, K[i], T[i], 1.0, 4.0, 10.0)
        op, on = ref.extract_points(3.0)
        assert len(op) > 1000
        compare_points_fast(p, n, op, on, tol=1e-6)
