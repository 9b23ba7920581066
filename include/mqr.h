/*
 * mqr.h -- C ABI of libmqr_hip.so, the MI355X (gfx950) TSDF fusion path.
 *
 * Drop-in boundary for the reference's Open3D VoxelBlockGrid usage and its numpy confidence
 * estimator (lszmer/metaquest-3d-reconstruction).  Each entry point names the reference
 * interface it replaces.  Conventions:
 *   - every function returns 0 on success, non-zero on error; mqr_last_error() returns a
 *     thread-local message (the Python layer raises RuntimeError with it, as Open3D does);
 *   - plain pointers and sizes only; `loc` arguments say where a buffer lives:
 *     MQR_HOST (caller-owned host memory, read/written during the call only) or
 *     MQR_DEVICE (device pointer on the volume's device, e.g. from mqr_device_alloc);
 *   - stream ordering of MQR_DEVICE buffers: the library runs on its own non-blocking HIP streams.
 *     Every call that reads or writes caller device buffers first makes those streams wait for all
 *     work enqueued so far on the calling thread's CALLER STREAM (mqr_set_stream; default: the null
 *     stream), so a kernel or copy the caller enqueued there that writes an input -- or still reads a
 *     buffer the call overwrites -- is complete before the library touches it.  No host wait is
 *     involved (an event and a stream wait).  Every call but one has finished with its buffers when
 *     it returns: outputs are complete and visible to any stream afterwards.  The exception is
 *     mqr_integrate_frames on MQR_DEVICE frames, which returns once its last integrate is queued:
 *     the caller stream is then made to wait (device-side) for that integrate, so whatever the
 *     caller enqueues there next -- overwriting or freeing the frames included -- runs after the
 *     library's reads; every later call on the volume orders itself behind it (a host-side reader
 *     of the frames synchronizes the caller stream first, as it would for a kernel of its own).
 *     mqr_integrate_frames also takes MQR_DEVICE_RESIDENT frames: device frames the caller keeps
 *     allocated and unchanged until the device (or the volume, by any call that drains it) has been
 *     synchronized -- e.g. a capture uploaded once and integrated pass after pass.  Reads are ordered
 *     after the caller stream as for MQR_DEVICE, but the caller stream is not made to wait for the
 *     call's integrates, so the next call's first touch -- itself behind the caller stream -- can run
 *     beside this call's last integrate instead of after it;
 *   - matrices are row-major: K = 3x3 intrinsic (Open3D convention, cx already flipped),
 *     T_wc = 4x4 world->camera extrinsic, both float64 as the reference passes them
 *     (o3d_utils.py:203-210);
 *   - a volume handle is not re-entrant; several handles per process/device are fine.
 */
#ifndef MQR_H
#define MQR_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MQR_HOST 0
#define MQR_DEVICE 1
#define MQR_DEVICE_RESIDENT 2 /* mqr_integrate_frames only: see "stream ordering" above */

typedef struct mqr_vbg mqr_vbg;    /* voxel-block-hashed TSDF volume resident in HBM */
typedef struct mqr_geom mqr_geom;  /* extracted point cloud or triangle mesh (device-resident) */
typedef struct mqr_scene mqr_scene;  /* triangle-mesh ray-casting scene (device BVH) */
typedef struct mqr_comm mqr_comm;    /* RCCL communicator of one rank (one process per GPU) */

int mqr_version(void);
/* Build tags: which 0 = a hash of the integrate sources (vbg.hip, vbg_kernels.hpp, mqr_common.hpp),
 * 1 = of the confidence sources, as compiled into this library; counter records under profiles/ carry
 * the tag of the build they measured (bench.py quotes only matching ones).  mqr_vbg_last_kernel: the
 * integrate variant (mqr_vbg_set_variant numbering) the volume's last launch actually used.
 * mqr_vbg_flips: how many mqr_vbg_reset calls swapped in the volume's second table / pool set instead of
 * waiting for an integrate still in flight (see mqr_vbg_reset). */
int mqr_build_tag(int which, char* buf, int cap);
int mqr_vbg_last_kernel(mqr_vbg* v, int* variant);
/* The name of the main kernel the volume's last integrate launch ran (e.g. "k_integrate_wt<7, 1>"). */
int mqr_vbg_last_kernel_name(mqr_vbg* v, char* buf, int cap);
int mqr_vbg_flips(mqr_vbg* v, int64_t* n);
const char* mqr_last_error(void);
int mqr_device_count(int* n);
/* The calling thread's caller stream (a hipStream_t; NULL = the null stream, the default): see
 * "stream ordering" above.  A PyTorch caller passes torch.cuda.current_stream().cuda_stream (the
 * Python layer does this by itself).  A caller stream of another device than the call's is drained on
 * the host instead (hipStreamSynchronize; no cross-device stream wait); an invalid one is status 2.
 * mqr_get_stream reads the current setting. */
int mqr_set_stream(void* stream);
int mqr_get_stream(void** stream);

/* Device memory helpers (so callers can keep inputs resident in HBM without any framework).
 * mqr_device_free waits for the device first (work in flight may still read the buffer). */
int mqr_device_alloc(int device, int64_t bytes, void** ptr);
int mqr_device_free(int device, void* ptr);
int mqr_memcpy(void* dst, int dst_loc, const void* src, int src_loc, int64_t bytes, int device);
int mqr_device_synchronize(int device);
/* hipMemGetInfo of `device`: free and total HBM bytes (the Python layer keeps a released volume for
 * reuse only while enough stays free). */
int mqr_device_mem_info(int device, int64_t* free_bytes, int64_t* total_bytes);

/* o3d.t.geometry.VoxelBlockGrid(attr_names=('tsdf','weight'), attr_dtypes=(f32,f32), attr_channels=(1,1),
 *                               voxel_size, block_resolution, block_count, device)
 * -- reference call site scripts/processing/reconstruction/utils/o3d_utils.py:170-179.
 * block_count is the initial capacity; the volume grows automatically like Open3D's hash map. */
int mqr_vbg_create(float voxel_size, int block_resolution, int64_t block_count, int device, mqr_vbg** out);
int mqr_vbg_destroy(mqr_vbg* v);
/* Empty the volume in place (keeps its allocations): the state of a freshly created grid.  Ordered on the
 * device: when an integrate of an asynchronously returning mqr_integrate_frames is still in flight, the
 * volume swaps in a second hash table / block pool set (allocated once, at the current capacities, while the
 * volume's pool is within 2 GiB and a quarter of the device's HBM stays free) and clears that one, so the
 * next call's first touch overlaps the unfinished integrate; otherwise the clear queues behind it. */
int mqr_vbg_reset(mqr_vbg* v);
int mqr_vbg_size(mqr_vbg* v, int64_t* n_blocks);
int mqr_vbg_capacity(mqr_vbg* v, int64_t* block_capacity);
int mqr_vbg_params(mqr_vbg* v, float* voxel_size, int* block_resolution, int* device);

/* vbg.compute_unique_block_coordinates(depth, intrinsic, extrinsic, depth_scale, depth_max,
 *                                      trunc_voxel_multiplier)  -- o3d_utils.py:212-219.
 * keys_out (host) must hold 4*(H/4)*(W/4) int32 triplets.  Returns 3 ("no block is touched")
 * when nothing is touched, like upstream.  The main volume is not modified. */
int mqr_touch(mqr_vbg* v, const float* depth, int depth_loc, int H, int W, const double* K, const double* T_wc,
              float depth_scale, float depth_max, float trunc_mult, int32_t* keys_out, int64_t* n_out);

/* vbg.integrate(block_coords, depth, intrinsic, extrinsic, depth_scale, depth_max,
 *               trunc_voxel_multiplier)  -- o3d_utils.py:221-229.  keys: n int32 triplets (host). */
int mqr_integrate(mqr_vbg* v, const int32_t* keys, int64_t n, const float* depth, int depth_loc, int H, int W,
                  const double* K, const double* T_wc, float depth_scale, float depth_max, float trunc_mult);

/* The whole per-frame loop of o3d_utils.integrate (:188-236): touch + integrate for B frames in
 * order, batched on device (results identical to B sequential touch+integrate calls).
 * depths: B*H*W float32 metric depth (0 = invalid), K: B*9, T_wc: B*16 (host float64).
 * frame_ok (host, may be NULL): frames with frame_ok[i]==0 are skipped (missing/invalid loads).
 * Returns 3 if a valid frame touches no block (upstream raises).  Every batch's touch counters are
 * read on the host before its integrate is launched, so errors are reported by this call; with
 * MQR_DEVICE / MQR_DEVICE_RESIDENT frames the call returns with the last integrate still running (see
 * "stream ordering" above), with MQR_HOST frames after it has finished. */
int mqr_integrate_frames(mqr_vbg* v, const float* depths, int depth_loc, int B, int H, int W, const double* K,
                         const double* T_wc, const uint8_t* frame_ok, float depth_scale, float depth_max,
                         float trunc_mult);

/* Volume contents (VoxelBlockGrid.save / load payload, and the multi-GPU merge).  Blocks are in
 * buffer order: keys n*3 int32, tsdf / weight n*R^3 float32 ([z][y][x] within a block). */
int mqr_vbg_export(mqr_vbg* v, int32_t* keys, float* tsdf, float* weight, int loc);
int mqr_vbg_import(mqr_vbg* v, const int32_t* keys, const float* tsdf, const float* weight, int64_t n, int loc);

/* Multi-GPU merge: pack the volume against a shared, sorted union key table into
 * [U][R^3][2] = (weight*tsdf, weight) float32 (zeros where a block is absent), and the inverse
 * after a sum-reduce: tsdf = sum(w*tsdf)/sum(w), weight = sum(w).  Device pointers. */
int mqr_vbg_pack_weighted(mqr_vbg* v, const int32_t* union_keys, int64_t U, float* packed);
int mqr_vbg_unpack_weighted(mqr_vbg* v, const int32_t* union_keys, int64_t U, const float* packed);

/* The single exchange step of frame-sharded fusion (SURVEY §8(b) mqr_reduce_rccl, §8(e)); the
 * reference has no distributed path -- this replaces running its integrate() loop
 * (o3d_utils.py:153-238) over all frames in one process.  One process per GPU: rank 0 makes an id
 * (mqr_comm_unique_id), the caller distributes it (e.g. a gloo / TCP store), every rank calls
 * mqr_comm_init.  RCCL (librccl.so.1) is resolved at run time.
 * mqr_reduce_rccl merges every rank's `local` volume into `out` (emptied first):
 *   MQR_MERGE_ROOT     `out` on `root` holds the whole merged volume (others: empty);
 *   MQR_MERGE_SHARDED  `out` holds this rank's owned slice of the sorted block union first
 *                      (*n_owned blocks), then the one-block halo; extract it with
 *                      mqr_extract_mesh_owned(out, thr, *n_owned): shard meshes concatenate to the
 *                      single-volume mesh (triangle counts add exactly).
 * Voxels seen by one rank keep its (tsdf, weight) bit for bit; others merge in rank order:
 * tsdf = (w_a tsdf_a + w_b tsdf_b) / (w_a + w_b), weight = w_a + w_b.  `out` must not be `local`.
 * The plan (sorted block union, owner slices, halo sets, send / receive lists) is computed on the
 * device; the host reads only block counts and list lengths.
 * mqr_comm_timing: the last merge's phases in ms -- [0] count + key all-gathers and the plan,
 * [1] output volume + gather of the outgoing blocks, [2] the RCCL exchange, [3] the merge kernels.
 * mqr_merge_local: the same exchange for n volumes of one process on one device, with device copies
 * as the transport: every rank builds its own plan, packs its own send segments and merges its
 * receive segments in rank order exactly as mqr_reduce_rccl does on that rank; before a byte moves,
 * each sender's segment for d is checked against d's receive segment from it (length, and the
 * source buffers both sides list, entry for entry; mismatch = status 4).  Tests and timing.
 * mqr_merge_local_timing: the last mqr_merge_local's wall time per rank in ms (its plan, output
 * volume, send-segment gather and merge kernels: one rank's share of a merge, without the transfer).
 *
 * mqr_xchg_*: the same exchange with the transport left to the caller (one process per rank; the
 * tests carry the segments over gloo through host buffers).  gathered_keys: world*mx packed block
 * keys (rank r's keys in buffer order at r*mx, padded with 0xFFFF...FF; packing as the int32 keys
 * of mqr_vbg_export: ((x+2^20)<<42)|((y+2^20)<<21)|(z+2^20)).  create = plan + output volume
 * (emptied) + send segments (+ the self segment in place); counts[world] = blocks per send segment
 * (to each peer) and per receive segment (from each peer), floats_per_block = 2*R^3 ((tsdf,
 * weight) interleaved); send_segment copies the segment for `peer` out, recv_segment copies the
 * segment from `peer` in (peer != rank); finish merges in rank order.  `out` must outlive the
 * handle. */
#define MQR_MERGE_ROOT 0
#define MQR_MERGE_SHARDED 1
int mqr_comm_unique_id(uint8_t* id_out /* 128 bytes */);
int mqr_comm_init(int device, int rank, int world, const uint8_t* id /* 128 bytes */, mqr_comm** out);
int mqr_comm_destroy(mqr_comm* comm);
int mqr_reduce_rccl(mqr_vbg* local, mqr_comm* comm, int mode, int root, mqr_vbg* out, int64_t* n_owned);
int mqr_merge_local(mqr_vbg** locals, int n, int mode, int root, mqr_vbg** outs, int64_t* n_owned);
int mqr_comm_timing(mqr_comm* comm, float* ms4);
/* Segment sizes of the last mqr_reduce_rccl on `comm`: blocks sent to / received from each rank
 * (world entries each; the own rank's entry is the local self segment, not carried by RCCL) and the
 * 4-byte words per block (2 R^3, or 1.5 R^3 with uint16 weights).  Zeros before the first merge. */
int mqr_comm_counts(mqr_comm* comm, int64_t* send_blocks, int64_t* recv_blocks, int64_t* floats_per_block);
int mqr_merge_local_timing(float* ms, int n);
/* Merge A/B and test hooks (process-wide).  Bit 0: how every transport merges the received segments --
 * 0 (default) one fused pass per output block folding its entries in rank order in registers, 1 the
 * round-5 form, one pass over the output per source rank.  Bit 1: mqr_merge_local sends float32 weights
 * even where uint16 would hold them.  Segment format: a block travels as its R^3 (tsdf, weight) float32
 * pairs, or -- when every rank's weights are integers <= 65535, which the library knows from each volume's
 * frame count (volumes filled by import or unpack count as unknown) -- as R^3 float32 tsdf then R^3
 * uint16 weights (6 B instead of 8 B per voxel); mqr_comm_counts / mqr_xchg_counts report the 4-byte
 * words per block of the format used (2 R^3 or 1.5 R^3; the caller-carried transport always uses float32
 * pairs).  Every combination gives the same bits. */
int mqr_merge_set_per_source(int on);
typedef struct mqr_xchg mqr_xchg;
int mqr_xchg_create(mqr_vbg* local, int world, int rank, int mode, int root, const uint64_t* gathered_keys,
                    int64_t mx, int keys_loc, mqr_vbg* out, mqr_xchg** h);
int mqr_xchg_counts(mqr_xchg* h, int64_t* send_blocks, int64_t* recv_blocks, int64_t* n_owned,
                    int64_t* floats_per_block);
int mqr_xchg_send_segment(mqr_xchg* h, int peer, float* dst, int loc);
int mqr_xchg_recv_segment(mqr_xchg* h, int peer, const float* src, int loc);
int mqr_xchg_finish(mqr_xchg* h, int64_t* n_owned);
int mqr_xchg_destroy(mqr_xchg* h);

/* vbg.extract_point_cloud(weight_threshold=3.0)   -- reconstruct_scene.py:90, refine_fragment_poses.py:39
 * vbg.extract_triangle_mesh(weight_threshold)       -- reconstruct_scene.py:105-108, 186-189 */
int mqr_extract_points(mqr_vbg* v, float weight_threshold, mqr_geom** out);
int mqr_extract_mesh(mqr_vbg* v, float weight_threshold, mqr_geom** out);
/* Triangles only of cubes whose origin voxel lies in blocks [0, n_owned) (a shard from
 * mqr_reduce_rccl MQR_MERGE_SHARDED); vertices of every block (unreferenced ones may remain). */
int mqr_extract_mesh_owned(mqr_vbg* v, float weight_threshold, int64_t n_owned, mqr_geom** out);
int mqr_geom_counts(mqr_geom* g, int64_t* n_vertices, int64_t* n_triangles);
/* Copy to caller buffers (positions / normals n*3 float32, triangles n*3 int32); NULL skips. */
int mqr_geom_copy(mqr_geom* g, float* positions, float* normals, int32_t* triangles, int loc);
int mqr_geom_free(mqr_geom* g);
/* The geometry's arrays in place (device pointers on its device, null when empty; valid until
 * mqr_geom_free, and only after the call that produced it returned): positions / normals float32
 * [nv][3], triangles int32 [nt][3].  Lets a caller keep the result in HBM, as Open3D's tensor geometry
 * on a CUDA device stays there, and hand it to MQR_DEVICE inputs (mqr_scene_add_triangles,
 * mqr_mesh_filter_components, mqr_color_map) without a host round trip. */
int mqr_geom_device_ptrs(mqr_geom* g, void** positions, void** normals, void** triangles);

/* build_confidence_map / compute_pixel_error_map
 * (confidence_estimation/estimate_depth_confidences.py:15-79, compute_pixel_error_map.py:120-220)
 * for reference frames [ref_begin, ref_end) of an N-frame sequence, all on the device at once.
 * depths: N*H*W float32 metric; K: N*9, T_cw: N*16, T_cw_inv: N*16 float32 (host);
 * frame_ok: N bytes (host, may be NULL).  conf: (ref_end-ref_begin)*H*W float64,
 * valid: same int32, both in `out_loc` memory.  float64 arithmetic as numpy does it. */
int mqr_confidence(int device, const float* depths, int depth_loc, int N, int H, int W, const float* K,
                   const float* T_cw, const float* T_cw_inv, const uint8_t* frame_ok, int ref_begin, int ref_end,
                   int frame_range, double depth_max, double error_threshold, double* conf, int32_t* valid,
                   int out_loc);
/* mqr_confidence for host output as two bytes per pixel: counts[r][y][x] = valid_count | consistent_count
 * << 8 of reference frame ref_begin + r (csrc/confpack.hip: the maps computed into HBM, reduced on the device,
 * each pair checked to give back the map's exact float64 bits; 2 bytes cross the link instead of 12).
 * *packed = 1 on success; 0 when a pixel does not fit (more than 255 valid neighbours) -- counts is then
 * unspecified and the caller uses mqr_confidence.  The pairs expand to the maps in
 * mqr_write_confidence_npz_counts. */
int mqr_confidence_counts(int device, const float* depths, int depth_loc, int N, int H, int W, const float* K,
                          const float* T_cw, const float* T_cw_inv, const uint8_t* frame_ok, int ref_begin,
                          int ref_end, int frame_range, double depth_max, double error_threshold, uint16_t* counts,
                          int* packed);
/* Diagnostic: enable (1) / disable (0) / keep (-1) per-pair stage counting of mqr_confidence on this
 * device (a slower kernel build); 2 = a timing-only build without the tap loads (wrong maps); last4 (nullable) = the last counted call's (pixel, neighbour) pairs
 * with a valid reference pixel, and how many the float32 prefilter, the float64 band filter and the
 * float64 back-projection decided. */
int mqr_confidence_stats(int device, int enable, int64_t* last4);
int mqr_pixel_error_map(int device, const float* ref_depth, const float* tgt_depth, int H, int W, const float* K_ref,
                        const float* K_tgt, const float* T_cw_ref, const float* T_cw_inv_tgt, const float* T_cw_tgt,
                        double depth_max, float* err_out);

/* Device-side depth ingestion.  N raw Quest NDC buffers (H*W float32, raw_loc
 * MQR_HOST / MQR_DEVICE) -> metric depth (depth_out, out_loc) + per-frame validity frame_ok[N]
 * (host).  Replaces DepthDataIO.load_depth_map + is_depth_map_valid
 * (scripts/dataio/depth_data_io.py:33-53, 80-85), convert_depth_to_linear
 * (scripts/utils/depth_utils.py:21-46) and the confidence mask of load_depth_map
 * (processing/reconstruction/utils/o3d_utils.py:131-142).  strong[f] (nullable): bit 0 / bit 1 =
 * near / far were numpy float64 scalars (numpy >= 2 then divides in float64; Python floats keep
 * the decode in float32).  has_mask[f] (nullable) selects frames whose conf (float64) /
 * valid_count (int32) maps, laid out like the depth, are applied: depth = 0 where
 * conf < conf_thr or valid_count < count_thr. */
int mqr_decode_depth(int device, const float* raw, int raw_loc, int N, int H, int W, const double* nears,
                     const double* fars, const uint8_t* strong, const double* conf, const int32_t* valid_count,
                     const uint8_t* has_mask, int mask_loc, double conf_thr, int count_thr, float* depth_out,
                     int out_loc, uint8_t* frame_ok);
/* The same decode with the confidence mask given as one byte per pixel (mask[N][H][W], mask_loc; nonzero =
 * depth 0 where has_mask[f]), e.g. as mqr_read_frames_masked computes it from the npz: 1 byte per pixel to
 * stage instead of 12. */
int mqr_decode_depth_masked(int device, const float* raw, int raw_loc, int N, int H, int W, const double* nears,
                            const double* fars, const uint8_t* strong, const uint8_t* mask, const uint8_t* has_mask,
                            int mask_loc, float* depth_out, int out_loc, uint8_t* frame_ok);

/* Host reads of the drop-in integrate.  Replaces, for n frames, the raw depth
 * read of DepthDataIO.load_depth_map (np.fromfile of H*W little-endian float32,
 * scripts/dataio/depth_data_io.py:33-53) and load_confidence_map (np.load of the np.savez npz:
 * confidence_map <f8 HxW, valid_count <i4 HxW; depth_data_io.py:91-104): `threads` native threads pread
 * the files straight into raw_out[n][H][W] and, when conf_paths is non-null, conf_out / vc_out[n][H][W]
 * (conf_paths[f] may be null: no confidence read for that frame).  Host-only (no device work).
 * status[f] is a set of MQR_FRAME_* bits.  A missing or unreadable raw file leaves zeros in raw_out
 * (decoded invalid); *_OTHER (wrong size, a compressed / non-standard npz, another dtype or shape, a read
 * error) is left to the caller's own loader, which then raises or logs exactly as the reference does. */
#define MQR_FRAME_RAW_OK 1
#define MQR_FRAME_RAW_MISSING 2
#define MQR_FRAME_RAW_OTHER 4
#define MQR_FRAME_CONF_OK 8
#define MQR_FRAME_CONF_MISSING 16
#define MQR_FRAME_CONF_OTHER 32
int mqr_read_frames(int n, const char* const* raw_paths, const char* const* conf_paths, int H, int W,
                    float* raw_out, double* conf_out, int32_t* vc_out, uint8_t* status, int threads);
/* The same reads with the confidence maps reduced while they are read to the mask byte the decode applies:
 * mask_out[f][y][x] = (confidence_map < conf_thr) | (valid_count < count_thr) (o3d_utils.py:131-142),
 * for mqr_decode_depth_masked. */
int mqr_read_frames_masked(int n, const char* const* raw_paths, const char* const* conf_paths, int H, int W,
                           double conf_thr, int count_thr, float* raw_out, uint8_t* mask_out, uint8_t* status,
                           int threads);

/* The confidence maps' writer (SURVEY §8 C3 outputs): for n frames, np.savez(paths[f],
 * confidence_map=conf[f], valid_count=valid[f]) as the reference saves them
 * (scripts/dataio/depth_data_io.py:106-115) -- a zip of stored members confidence_map.npy (<f8 H x W) and
 * valid_count.npy (<i4 H x W), .npy format 1.0 headers, zip64 local extra fields and CRC-32 like
 * np.savez's -- written by `threads` native threads from the caller's arrays.  Host-only.
 * paths[f] may be null (no file for that frame).  status[f]: 0, or the errno of the failed open / write
 * (the caller reports that frame). */
int mqr_write_confidence_npz(int n, const char* const* paths, const double* conf, const int32_t* valid, int H, int W,
                             int32_t* status, int threads);
/* The same files from the confidence maps' two counts per pixel: counts[f][y][x] = valid_count |
 * consistent_count << 8 (as mqr_confidence_counts downloads them); confidence_map = consistent / valid in
 * float64, 0 where valid is 0 (estimate_depth_confidences.py:72-74), expanded by the writer threads. */
int mqr_write_confidence_npz_counts(int n, const char* const* paths, const uint16_t* counts, int H, int W,
                                    int32_t* status, int threads);
/* CRC-32 (zip / zlib) of len bytes continuing from crc (0 to start): the writer's checksum, exported for
 * its tests. */
uint32_t mqr_crc32(uint32_t crc, const void* data, int64_t len);

/* Kernel timing (HIP events on the volume's own stream).  enable=1 starts recording every
 * integrate-kernel launch; stats: launches, total kernel ms, union blocks, frame-blocks
 * (sum of per-frame touched blocks), frames, and the same for touch. */
typedef struct mqr_stats {
    int64_t integrate_launches;
    double integrate_ms;
    int64_t union_blocks;
    int64_t frame_blocks;
    int64_t frames;
    int64_t touch_launches;
    double touch_ms;
    int64_t pixels;
    int64_t table_retries; /* batches touched again after the probe-limited table filled up */
} mqr_stats;
/* enable: 0 off, 1 time every integrate launch (two events per batch on the integrate stream), 2 also
 * every touch launch (two more on the touch stream); results in mqr_vbg_stats. */
int mqr_vbg_profile(mqr_vbg* v, int enable);

/* Test / tuning hooks.  mqr_vbg_set_variant: low byte = integrate kernel (0 default = lean kernel
 * where its preconditions hold, 1 generic, 2 exact R-specialised, 3 lean with the plate map, 5 depth
 * from LDS tiles; all bit-identical, see launch_integrate in csrc/vbg.hip); bit 8 serialises touch and integrate, bit 9 keeps touch
 * order instead of longest-first, bit 10 uses 32-frame batches instead of 127 (bit 20: 64-frame
 * batches; bits 21 / 22 / 23: a first batch of 64 / 32 / 16 frames), bit 11 records
 * system-scope ordering events, bit 12 probes one table slot per new key in the batch touch (forces
 * the full-table undo-and-retry path; test hook), bit 13 sizes the table for the worst case, bit 14 makes
 * every integrate launch wait on a touch-stream event, bit 15 runs the batch in spatial per-XCD groups
 * (k_xcd_order; A/Bs), bit 16 gives the touch one stride-4 pixel per thread instead of two, bit 18 turns
 * off the speculative first-batch integrate (k_gate; A/B), bit 24 makes mqr_integrate_frames on device frames
 * drain its streams before returning (A/B), bit 25 makes mqr_vbg_reset wait for an integrate in flight
 * instead of swapping in the second table / pool set (A/B), bit 26 runs the default integrate without its LDS
 * table of (w, 1 / (w + 1)) (k_integrate_win instead of k_integrate_wt; A/B), bit 27 keeps k_integrate_wt's two
 * Markstein corrections of s / sdf_trunc where one is verified exact for the volume's sdf_trunc (A/B).
 * mqr_check_division: exhaustive bit-pattern check of the division shortcuts used on device against
 * IEEE division (which=0: 1/b via rcp_rn, 1: a/b via div_rn, 2: a/b via the bare core, 3: 1/b via
 * rcp_nm, 4: 1/b via rcp_m, over float bit patterns [lo_bits, lo_bits+count) as b or a); returns
 * the mismatch count and the first bad pattern. */
int mqr_vbg_set_variant(mqr_vbg* v, int variant);
int mqr_check_division(int device, int which, float b, uint32_t lo_bits, uint64_t count, uint32_t* mismatches,
                       uint32_t* first_bad);
/* mqr_check_div64: the confidence kernel's float64 quotients against IEEE division on `count`
 * hashed pairs (a in [-a_max, a_max], b log-uniform in [b_lo, b_hi]); mode 0 = shared refined
 * reciprocal (quotients by Z), 1 = host-rounded reciprocal + Markstein correction (by fx / fy).
 * first_bad: 2 doubles (a, b) of a mismatch. */
int mqr_check_div64(int device, int mode, uint64_t seed, uint64_t count, double a_max, double b_lo, double b_hi,
                    uint64_t* mismatches, double* first_bad);
int mqr_vbg_stats(mqr_vbg* v, mqr_stats* out, int reset);

/* Ray casting: replaces o3d.t.geometry.RaycastingScene as used for colour-aligned
 * depth (reconstruct_scene.py:197-201, o3d_utils.py:324-341, optimize_color_pose.py:24-47).
 * add_triangles ~ RaycastingScene.add_triangles (vertices float32 (nv,3), triangles int32 (nt,3),
 * loc MQR_HOST/MQR_DEVICE; returns the geometry id); the device BVH is (re)built on the first
 * query after a change (mqr_scene_build forces it).  cast_pinhole ~ create_rays_pinhole(K, T_wc,
 * W, H) + cast_rays for n_frames cameras (K (n,3,3) and T_wc (n,4,4) float64 row-major);
 * cast_rays takes explicit rays (n,6) float32 (origin, direction).  Outputs: t_hit (inf on miss)
 * and the optional geometry / primitive ids (0xffffffff on miss), barycentric uvs (n,2) and unit
 * geometric normals (n,3); out_loc says where all output buffers live. */
/* Per-vertex colour from keyframes: the colour averaging of Open3D's
 * colour-map pipeline fed by the reference (optimize_color_pose.py:24-73 -> run_rigid_optimizer;
 * upstream ColorMapUtils.cpp CreateVertexAndImageVisibility + SetGeometryColorAverage, VERIFY).
 * vertices nv*3 float32; images N*H*W*3 uint8 RGB; depths N*H*W float32 colour-aligned depth
 * (ray-cast, raycast_in_color_view); K N*9, T_wc N*16 float64 host.  colors_out nv*3 float32 in
 * [0, 1] (0 where no keyframe sees the vertex), counts_out nv int32 (nullable).  Open3D defaults:
 * max_depth 2.5, visibility_threshold 0.03, margin 10. */
int mqr_color_vertices(int device, const float* vertices, int64_t nv, int vertices_loc, const uint8_t* images,
                       const float* depths, int images_loc, int N, int H, int W, const double* K, const double* T_wc,
                       double max_depth, double visibility_threshold, int margin, float* colors_out,
                       int32_t* counts_out, int out_loc);
/* mqr_color_map: the complete vertex colouring of run_rigid_optimizer with the keyframe poses as
 * given (optimize_color_pose.py:70-73; pose refinement OUT of scope): t_hit = raycast_in_color_view
 * depth (o3d_utils.py:324-341), RGBD depth truncated at depth_trunc (3.0), depth-discontinuity
 * masks (Sobel magnitude > disc_threshold 0.1, dilated by half_dilation 3), visibility, float64
 * colour means, and vertices no keyframe samples filled with the mean of their knn (3) nearest
 * sampled vertices.  counts: keyframes averaged (0 for filled vertices). */
int mqr_color_map(int device, const float* vertices, int64_t nv, int vloc, const uint8_t* images, const float* t_hit,
                  int img_loc, int N, int H, int W, const double* K, const double* T_wc, double max_depth,
                  double visibility_threshold, int margin, double disc_threshold, int half_dilation, double depth_trunc,
                  int knn, float* colors_out, int32_t* counts_out, int out_loc);

int mqr_scene_create(int device, mqr_scene** out);
int mqr_scene_destroy(mqr_scene* s);
int mqr_scene_add_triangles(mqr_scene* s, const float* vertices, int64_t nv, const int32_t* triangles, int64_t nt,
                            int loc, uint32_t* geom_id);
int mqr_scene_build(mqr_scene* s);
int mqr_scene_triangle_count(mqr_scene* s, int64_t* n);
int mqr_scene_cast_pinhole(mqr_scene* s, const double* K, const double* T_wc, int n_frames, int H, int W,
                           float* t_hit, uint32_t* geom_ids, uint32_t* prim_ids, float* uvs, float* normals,
                           int out_loc);
int mqr_scene_cast_rays(mqr_scene* s, const float* rays, int64_t nrays, int rays_loc, float* t_hit,
                        uint32_t* geom_ids, uint32_t* prim_ids, float* uvs, float* normals, int out_loc);

/* filter_mesh_components (processing/reconstruction/utils/o3d_utils.py:241-321) on the device:
 * edge-connected triangle clusters (Open3D cluster_connected_triangles order), keep clusters with
 * >= min_triangle_count triangles (else the largest), then remove_unreferenced_vertices,
 * remove_degenerate_triangles, remove_duplicated_triangles, remove_duplicated_vertices and
 * remove_non_manifold_edges with Open3D's legacy semantics (non-manifold edges visited in
 * ascending vertex-pair order).  vertices / normals (nullable) nv*3 float32, triangles nt*3 int32
 * in `loc` memory.  Result: a device geometry (mqr_geom_counts / _copy / _free).  stats[8]:
 * input triangles, clusters, kept clusters, triangles removed with small clusters, largest
 * cluster, triangles removed by the non-manifold pass, final triangles, final vertices. */
int mqr_mesh_filter_components(int device, const float* vertices, const float* normals, int64_t nv,
                               const int32_t* triangles, int64_t nt, int loc, int64_t min_triangle_count,
                               mqr_geom** out, int64_t* stats);

#ifdef __cplusplus
}
#endif
#endif /* MQR_H */
