// merge.hip -- the single exchange step of frame-sharded fusion across the GPUs of one node
// (SURVEY §8(e)): every rank integrated a contiguous frame range into its own volume; this merges
// them, over RCCL (xGMI) or, for tests on one device, over device-to-device copies.
//
// The reference's unit-weight running average makes partial volumes mergeable:
//   tsdf = (w_a tsdf_a + w_b tsdf_b) / (w_a + w_b),  weight = w_a + w_b     (App. A.3)
// applied source by source in rank order (deterministic); a voxel that only one rank saw keeps
// that rank's (tsdf, weight) bit for bit.
//
// Plan (identical on every rank, computed ON THE DEVICE from the all-gathered block keys):
//   union U = sorted distinct keys (packed order = lexicographic x, y, z; a radix sort of the W
//   ranks' padded key arrays); owner slices = [U r / W, U (r+1) / W); each union block goes to a
//   destination set:
//     MQR_MERGE_ROOT     the root only (the root's output holds the whole volume)
//     MQR_MERGE_SHARDED  its owner and the owners of its 26 neighbours (binary search in the
//                        sorted union) -- so every rank holds its owned blocks plus a one-block
//                        halo, and extracts exactly the cubes whose origin lies in an owned block
//                        (mqr_extract_mesh_owned): triangle counts of the shards add up to the
//                        single-volume count.
//   Every rank sends each of its blocks once per destination (grouped ncclSend / ncclRecv: a
//   sparse all-to-all, per-link traffic ~ own blocks + halo instead of the dense union).  The
//   send and receive lists of one rank are the segments of one sorted record array (kind, peer,
//   entry), so a sender's segment for d and d's segment from that sender list the same blocks in
//   the same (union) order.  The host reads two small count arrays per merge (block counts after
//   the first all-gather, list lengths after the plan); nothing else leaves the device.
//
// Transports.  One rank's side of the exchange (plan, output volume, send segments, rank-ordered
// merge of the receive segments) is `Exchange`; three transports move its segments:
//   mqr_reduce_rccl   ncclSend / ncclRecv between processes (one per GPU);
//   mqr_merge_local   device copies between the n volumes of one process (every rank still builds
//                     its OWN plan and packs its OWN send segments; the pair lists are checked);
//   mqr_xchg_*        the caller (host buffers over gloo, one process per rank, any device).
// Only the ncclSend / ncclRecv call differs between them.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

#include "mqr_common.hpp"

// ------------------------------------------------------------------ RCCL, resolved at run time
namespace {
struct RcclApi {
    bool tried = false, ok = false;
    std::string err;
    ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

std::mutex g_rccl_mu;
RcclApi g_rccl;

// librccl.so.1 by SONAME: the copy torch already mapped if torch is loaded (one RCCL per process),
// else the one on this library's RUNPATH (/opt/rocm/lib).
RcclApi* rccl() {
    std::lock_guard<std::mutex> lk(g_rccl_mu);
    if (g_rccl.tried) return g_rccl.ok ? &g_rccl : nullptr;
    g_rccl.tried = true;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
        g_rccl.err = std::string("RCCL not found: ") + dlerror();
        return nullptr;
    }
#define MQR_SYM(field, name)                                                  \
    g_rccl.field = reinterpret_cast<decltype(g_rccl.field)>(dlsym(h, name));  \
    if (!g_rccl.field) {                                                      \
        g_rccl.err = "RCCL symbol missing: " name;                            \
        return nullptr;                                                       \
    }
    MQR_SYM(GetUniqueId, "ncclGetUniqueId")
    MQR_SYM(CommInitRank, "ncclCommInitRank")
    MQR_SYM(CommDestroy, "ncclCommDestroy")
    MQR_SYM(AllGather, "ncclAllGather")
    MQR_SYM(Send, "ncclSend")
    MQR_SYM(Recv, "ncclRecv")
    MQR_SYM(GroupStart, "ncclGroupStart")
    MQR_SYM(GroupEnd, "ncclGroupEnd")
    MQR_SYM(GetErrorString, "ncclGetErrorString")
#undef MQR_SYM
    g_rccl.ok = true;
    return &g_rccl;
}
}  // namespace

#define MQR_CHECK_NCCL(api, expr)                                                                  \
    do {                                                                                           \
        ncclResult_t _r = (expr);                                                                  \
        if (_r != ncclSuccess) {                                                                   \
            ::mqr::set_error(std::string(#expr) + ": " + (api)->GetErrorString(_r));               \
            return 1;                                                                              \
        }                                                                                          \
    } while (0)

namespace mqr {
// Grow-only device scratch of the merge plan (hipFree synchronises the device: no allocation per
// merge once the block counts stop growing) and the pinned summary the host reads.
struct PlanScratch {
    void* buf = nullptr;
    size_t cap = 0;
    void* h_sum = nullptr;  // pinned PlanSummary
    ~PlanScratch() {
        if (buf) (void)hipFree(buf);
        if (h_sum) (void)hipHostFree(h_sum);
    }
};
}  // namespace mqr

namespace mqr {
struct Exchange;
}

struct mqr_comm {
    int device = 0, rank = 0, world = 1;
    ncclComm_t nc = nullptr;
    hipStream_t s = nullptr;
    void* small = nullptr;  // counts, padded keys
    size_t small_cap = 0;
    mqr::Exchange* x = nullptr;  // plan, send / receive buffers (grow-only, reused across merges)
    // phase timing of the last merge (mqr_comm_timing): start, plan done, gathered, exchanged, merged
    hipEvent_t ev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    float last_ms[4] = {0.f, 0.f, 0.f, 0.f};
    hipEvent_t order = nullptr;  // the local volume's touch stream, waited for on `s` (no host wait)
};

namespace mqr {

// ------------------------------------------------------------------ kernels
// Segment formats.  PK = 0: a block is its R3 (tsdf, weight) float2 pairs, the pool's own layout (8 B per
// voxel).  PK = 1: R3 float tsdf, then R3 uint16 weights (6 B per voxel) -- used when every rank's
// weights are integers <= 65535 (each rank's wbound; all ranks decide alike from the gathered bounds),
// which uint16 holds exactly, so the merge reads the same values either way.
template <int PK>
__device__ __forceinline__ float2 seg_load(const char* __restrict__ blk, int p, int R3) {
    if constexpr (PK == 0) {
        return reinterpret_cast<const float2*>(blk)[p];
    } else {
        return make_float2(reinterpret_cast<const float*>(blk)[p],
                           (float)reinterpret_cast<const uint16_t*>(blk + 4 * (size_t)R3)[p]);
    }
}
__host__ __device__ constexpr size_t seg_block_bytes(int pk, int R3) { return (size_t)R3 * (pk ? 6 : 8); }

// (tsdf, weight) of listed local buffers into consecutive segment blocks.
template <int PK>
__global__ void k_gather_blocks(const int32_t* __restrict__ bufs, int64_t n, const float2* __restrict__ pool, int R3,
                                char* __restrict__ out) {
    const int64_t j = blockIdx.x;
    if (j >= n) return;
    const float2* src = pool + (int64_t)bufs[j] * R3;
    char* dst = out + j * seg_block_bytes(PK, R3);
    for (int p = threadIdx.x; p < R3; p += blockDim.x) {
        const float2 v = src[p];
        if constexpr (PK == 0) {
            reinterpret_cast<float2*>(dst)[p] = v;
        } else {
            reinterpret_cast<float*>(dst)[p] = v.x;
            reinterpret_cast<uint16_t*>(dst + 4 * (size_t)R3)[p] = (uint16_t)v.y;
        }
    }
}

// Merge received entries into destination buffers: a voxel with no weight yet takes the entry as
// is, one with weight merges by the running-average identity; entries with zero weight change
// nothing.  One launch per source rank, in rank order; a buffer appears at most once per source.
template <int PK>
__global__ void k_merge_blocks(const int32_t* __restrict__ dst, int64_t n, const char* __restrict__ in, int R3,
                               float2* __restrict__ pool) {
    const int64_t j = blockIdx.x;
    if (j >= n) return;
    const char* src = in + j * seg_block_bytes(PK, R3);
    float2* out = pool + (int64_t)dst[j] * R3;
    for (int p = threadIdx.x; p < R3; p += blockDim.x) {
        const float2 a = out[p], b = seg_load<PK>(src, p, R3);
        if (b.y == 0.f) continue;
        if (a.y == 0.f) {
            out[p] = b;
        } else {
            const float w = a.y + b.y;
            out[p] = make_float2((a.y * a.x + b.y * b.x) / w, w);
        }
    }
}

// Fused merge (the default): one workgroup per output buffer folds all of its received entries in
// source-rank order in registers -- the same operations in the same order as the k_merge_blocks launch per
// source, so the same bits -- reading each entry once and writing the buffer once, where the per-source
// launches read and rewrite the output buffer for every source that holds it (at 8 ranks a buffer has ~4).
// A buffer gets at most one entry per source, so its entries sit in a dense [n_out][W] table of receive
// indices (-1: none), filled by one scatter over the receive lists (k_merge_entries); the rank's own
// entries are read straight from its send segment (receive indices [roff[me], roff[me+1]) <-> send index
// soff[me] + j - roff[me]), so the self segment is not copied.  Every output buffer gets at least one entry
// (it is in the plan because some rank holds the block), so every voxel is written and the output pool
// needs no zeroing.
static std::atomic<bool> g_merge_per_source{false};  // A/B and test hook: mqr_merge_set_per_source
static std::atomic<bool> g_merge_f32_segments{false};  // A/B and test hook: mqr_merge_set_per_source bit 1
constexpr int kMergeMaxEntries = 64;                  // a buffer gets at most one entry per rank (kMaxRanks)

struct SegOffsets {
    int64_t off[kMergeMaxEntries + 1];  // receive segment s = [off[s], off[s + 1])
};

__global__ void k_merge_entries(const int32_t* __restrict__ dst, int64_t n, SegOffsets seg, int W,
                                int32_t* __restrict__ ent) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    int s = 0;
    while (s + 1 < W && seg.off[s + 1] <= j) ++s;
    ent[(int64_t)dst[j] * W + s] = (int32_t)j;
}

template <int PK>
__global__ __launch_bounds__(256) void k_merge_fused(const int32_t* __restrict__ ent, int W, int64_t n_out,
                                                     const char* __restrict__ recv, const char* __restrict__ send,
                                                     int64_t self_lo, int64_t self_hi, int64_t self_send, int R3,
                                                     float2* __restrict__ pool) {
    __shared__ int32_t e[kMergeMaxEntries];
    __shared__ int n_e;
    const int64_t d = blockIdx.x;
    if (d >= n_out) return;
    if (threadIdx.x == 0) {  // the buffer's entries in source order
        int m = 0;
        for (int s = 0; s < W; ++s) {
            const int32_t j = ent[d * W + s];
            if (j >= 0) e[m++] = j;
        }
        n_e = m;
    }
    __syncthreads();
    const int m = n_e;
    float2* out = pool + d * R3;
    for (int p = threadIdx.x; p < R3; p += blockDim.x) {
        float2 a = make_float2(0.f, 0.f);  // the buffer as the per-source form starts it (zeroed)
        for (int k = 0; k < m; ++k) {
            const int64_t j = e[k];
            const size_t bb = seg_block_bytes(PK, R3);
            const char* blk = (j >= self_lo && j < self_hi) ? send + (self_send + (j - self_lo)) * bb : recv + j * bb;
            const float2 b = seg_load<PK>(blk, p, R3);
            if (b.y == 0.f) continue;
            if (a.y == 0.f) {
                a = b;
            } else {
                const float w = a.y + b.y;
                a = make_float2((a.y * a.x + b.y * b.x) / w, w);
            }
        }
        out[p] = a;
    }
}

// ------------------------------------------------------------------ device plan
// Entries: the W x mx all-gathered keys (rank r's block b at r mx + b, padding = kEmpty).
// After the sort, entry p of the sorted order has key ks[p] and origin vs[p] = r mx + b.
constexpr int kMaxRanks = 64;  // destination sets are 64-bit masks

struct PlanSummary {
    int64_t U;          // union blocks
    int64_t n_owned;    // this rank's owned blocks (the first n_owned output buffers)
    int64_t n_out;      // owned + halo output blocks
    int64_t total;      // send + receive records
    int64_t cnt[2][kMaxRanks];  // [0][d] blocks sent to d, [1][s] blocks received from s
};

__device__ __forceinline__ int64_t slice_lo(int64_t U, int W, int r) { return U * r / W; }
// rank owning union index u (the r with U r / W <= u < U (r + 1) / W)
__device__ __forceinline__ int owner_of(int64_t u, int64_t U, int W) {
    int r = (int)((u * W) / (U > 0 ? U : 1));
    while (r > 0 && slice_lo(U, W, r) > u) --r;
    while (r + 1 < W && slice_lo(U, W, r + 1) <= u) ++r;
    return r;
}

__global__ void k_plan_iota(int32_t* __restrict__ v, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = (int32_t)i;
}

// head[p] = 1 at the first entry of each distinct key
__global__ void k_plan_heads(const uint64_t* __restrict__ ks, int64_t n, int32_t* __restrict__ head) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint64_t k = ks[p];
    head[p] = (k != kEmpty && (p == 0 || ks[p - 1] != k)) ? 1 : 0;
}

// uidx (inclusive head scan) - 1 = union index of entry p; the union keys, the sorted position of
// each union block's first entry; U
__global__ void k_plan_union(const uint64_t* __restrict__ ks, const int32_t* __restrict__ incl, int64_t n,
                             uint64_t* __restrict__ uni, int32_t* __restrict__ first, PlanSummary* __restrict__ sum) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const uint64_t k = ks[p];
    if (k != kEmpty && (p == 0 || ks[p - 1] != k)) {
        uni[incl[p] - 1] = k;
        first[incl[p] - 1] = (int32_t)p;
    }
    if (p == n - 1) sum->U = incl[p];
}

__device__ __forceinline__ int64_t find_union(const uint64_t* __restrict__ uni, int64_t U, uint64_t k) {
    int64_t lo = 0, hi = U;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (uni[mid] < k) lo = mid + 1;
        else hi = mid;
    }
    return lo < U && uni[lo] == k ? lo : -1;
}

// The plan's lists come from per-union-block flags on 2W + 1 channels, in union order within each:
//   channel d < W        send u to rank d       (I hold u, d in dmask[u])
//   channel W + s        receive u from rank s  (s holds u, I am in dmask[u])
//   channel 2W           u is halo for me       (I am in dmask[u], u outside my owned slice)
// Sender and receiver both list a block pair in union order, so their segments match.  Positions:
// one exclusive scan over the per-workgroup channel counts laid out channel-major, so channel c's
// entries start at the sum of the earlier channels' totals: sends [0, ns), receives [ns, ns + nr),
// halo [ns + nr, ...).
constexpr int kPlanThreads = 256;
constexpr int kPlanChannels = 2 * kMaxRanks + 1;

__device__ __forceinline__ bool plan_flag(int c, int W, int me, uint64_t dm, uint64_t hm, bool owned) {
    if (c < W) return ((hm >> me) & 1) && ((dm >> c) & 1);
    if (c < 2 * W) return ((hm >> (c - W)) & 1) && ((dm >> me) & 1);
    return ((dm >> me) & 1) && !owned;
}

__device__ __forceinline__ bool plan_owned(int64_t u, int64_t U, int W, int mode, int root, int me) {
    return mode == MQR_MERGE_ROOT ? me == root : owner_of(u, U, W) == me;
}

// Destination ranks (owner + owners of the 26 neighbours, or the root), holder ranks (the union
// block's run of sorted entries; the sort is stable, so the run is in rank order) and the
// workgroup's channel counts wcnt[c * gridDim.x + blockIdx.x].
__global__ __launch_bounds__(kPlanThreads) void k_plan_masks(const uint64_t* __restrict__ uni,
                                                             const int32_t* __restrict__ first,
                                                             const uint64_t* __restrict__ ks,
                                                             const int32_t* __restrict__ vs, int64_t n, int64_t mx,
                                                             const PlanSummary* __restrict__ sum, int W, int mode,
                                                             int root, int me, uint64_t* __restrict__ dmask,
                                                             uint64_t* __restrict__ hmask, int32_t* __restrict__ wcnt) {
    __shared__ int cnt[kPlanChannels];
    const int NC = 2 * W + 1;
    for (int c = threadIdx.x; c < NC; c += blockDim.x) cnt[c] = 0;
    __syncthreads();
    const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t U = sum->U;
    const bool act = u < U;
    uint64_t dm = 0, hm = 0;
    bool owned = false;
    if (act) {
        const uint64_t k = uni[u];
        if (mode == MQR_MERGE_ROOT) {
            dm = 1ull << root;
        } else {
            dm = 1ull << owner_of(u, U, W);
            int x, y, z;
            unpack_key(k, x, y, z);
            for (int q = 0; q < 27; ++q) {
                const int nx = x + q % 3 - 1, ny = y + (q / 3) % 3 - 1, nz = z + q / 9 - 1;
                if (q == 13 || !key_in_range(nx, ny, nz)) continue;
                const int64_t j = find_union(uni, U, pack_key(nx, ny, nz));
                if (j >= 0) dm |= 1ull << owner_of(j, U, W);  // the neighbour's owner needs u as halo
            }
        }
        for (int64_t p = first[u]; p < n && ks[p] == k; ++p) hm |= 1ull << (vs[p] / mx);
        dmask[u] = dm;
        hmask[u] = hm;
        owned = plan_owned(u, U, W, mode, root, me);
    }
    const int lane = threadIdx.x & 63;
    for (int c = 0; c < NC; ++c) {
        const uint64_t bl = __ballot(act && plan_flag(c, W, me, dm, hm, owned));
        if (lane == 0 && bl) atomicAdd(&cnt[c], __popcll(bl));
    }
    __syncthreads();
    for (int c = threadIdx.x; c < NC; c += blockDim.x) wcnt[(int64_t)c * gridDim.x + blockIdx.x] = cnt[c];
}

// Lists at the scanned positions (wbase = exclusive scan of wcnt): send_idx (my buffer of u, by
// destination), recv_dst / recv_src (output position of u and the source's buffer of u, by source),
// output positions (owned slice first, then halo, both in union order), output keys, the summary.
__global__ __launch_bounds__(kPlanThreads) void k_plan_lists(
    const uint64_t* __restrict__ uni, const int32_t* __restrict__ first, const int32_t* __restrict__ vs, int64_t mx,
    const uint64_t* __restrict__ dmask, const uint64_t* __restrict__ hmask, const int32_t* __restrict__ wcnt,
    const int32_t* __restrict__ wbase, PlanSummary* __restrict__ sum, int W, int mode, int root, int me,
    int32_t* __restrict__ send_idx, int32_t* __restrict__ recv_dst, int32_t* __restrict__ recv_src,
    uint64_t* __restrict__ out_keys) {
    constexpr int NW = kPlanThreads / 64;
    __shared__ int wc[NW][kPlanChannels];  // per-wave channel counts, then their prefix over waves
    const int NC = 2 * W + 1;
    const int64_t nwg = gridDim.x, U = sum->U;
    const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool act = u < U;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t below = (1ull << lane) - 1;
    const uint64_t dm = act ? dmask[u] : 0, hm = act ? hmask[u] : 0;
    const bool owned = act && plan_owned(u, U, W, mode, root, me);
    for (int c = 0; c < NC; ++c) {
        const uint64_t bl = __ballot(act && plan_flag(c, W, me, dm, hm, owned));
        if (lane == 0) wc[wave][c] = __popcll(bl);
    }
    __syncthreads();
    for (int c = threadIdx.x; c < NC; c += blockDim.x) {
        int run = 0;
        for (int w = 0; w < NW; ++w) {
            const int t = wc[w][c];
            wc[w][c] = run;
            run += t;
        }
    }
    __syncthreads();
    const int64_t ns = wbase[(int64_t)W * nwg], nsr = wbase[(int64_t)2 * W * nwg];
    auto pos_of = [&](int c, uint64_t bl) {
        return (int64_t)wbase[(int64_t)c * nwg + blockIdx.x] + wc[wave][c] + __popcll(bl & below);
    };
    int64_t lo, hi;
    if (mode == MQR_MERGE_ROOT) {
        lo = 0;
        hi = me == root ? U : 0;
    } else {
        lo = slice_lo(U, W, me);
        hi = slice_lo(U, W, me + 1);
    }
    int32_t op = -1;  // output position of u
    {
        const bool f = act && plan_flag(2 * W, W, me, dm, hm, owned);
        const uint64_t bl = __ballot(f);
        if (act && u >= lo && u < hi) op = (int32_t)(u - lo);
        else if (f) op = (int32_t)((hi - lo) + (pos_of(2 * W, bl) - nsr));
    }
    if (op >= 0) out_keys[op] = uni[u];
    const int64_t f0 = act ? first[u] : 0;
    for (int d = 0; d < W; ++d) {
        const bool f = act && plan_flag(d, W, me, dm, hm, owned);
        const uint64_t bl = __ballot(f);
        if (f) send_idx[pos_of(d, bl)] = (int32_t)(vs[f0 + __popcll(hm & ((1ull << me) - 1))] % mx);
    }
    for (int s = 0; s < W; ++s) {
        const bool f = act && plan_flag(W + s, W, me, dm, hm, owned);
        const uint64_t bl = __ballot(f);
        if (f) {
            const int64_t j = pos_of(W + s, bl) - ns;
            recv_dst[j] = op;
            recv_src[j] = (int32_t)(vs[f0 + __popcll(hm & ((1ull << s) - 1))] % mx);
        }
    }
    if (blockIdx.x == 0)
        for (int c = threadIdx.x; c < NC; c += blockDim.x) {
            const int64_t last = (int64_t)NC * nwg - 1;
            const int64_t start = wbase[(int64_t)c * nwg];
            const int64_t end = c + 1 < NC ? wbase[(int64_t)(c + 1) * nwg] : wbase[last] + wcnt[last];
            if (c < W) sum->cnt[0][c] = end - start;
            else if (c < 2 * W) sum->cnt[1][c - W] = end - start;
            else {
                sum->n_owned = hi - lo;
                sum->n_out = (hi - lo) + (end - start);
                sum->total = start;  // send + receive records
            }
        }
}

// One rank's plan over the gathered keys dkeys[W * mx] (device).  Host results in `H` (pinned
// summary, read after one stream sync); device lists in the scratch: send_idx (segments by
// destination), recv_dst / recv_src (segments by source), out_keys.
struct PlanView {
    const PlanSummary* H = nullptr;
    int32_t* send_idx = nullptr;
    int32_t* recv_dst = nullptr;
    int32_t* recv_src = nullptr;
    uint64_t* out_keys = nullptr;
};

static size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

static int device_plan(PlanScratch& S, hipStream_t st, const uint64_t* dkeys, int W, int64_t mx, int me, int mode,
                       int root, PlanView& out) {
    const int64_t n = (int64_t)W * mx;
    MQR_REQUIRE(n < (int64_t{1} << 31), "merge plan: too many blocks");
    const int NC = 2 * W + 1;
    const int64_t nwg = (n + kPlanThreads - 1) / kPlanThreads;  // over union indices (U <= n)
    const int64_t nsend = n * (int64_t)std::min(W, 27);         // each union block goes to <= 27 ranks
    size_t tb_sort = 0, tb_scan = 0, tb_wscan = 0;
    MQR_CHECK_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tb_sort, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                                     (const int32_t*)nullptr, (int32_t*)nullptr, (int)n, 0, 64, st));
    MQR_CHECK_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, tb_scan, (const int32_t*)nullptr, (int32_t*)nullptr,
                                                   (int)n, st));
    MQR_CHECK_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tb_wscan, (const int32_t*)nullptr, (int32_t*)nullptr,
                                                   (int)(NC * nwg), st));
    const size_t tb = std::max(tb_sort, std::max(tb_scan, tb_wscan));
    // carve the scratch
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off += align_up(bytes);
        return o;
    };
    const size_t o_ks = take(8 * n), o_vi = take(4 * n), o_vs = take(4 * n), o_head = take(4 * n),
                 o_incl = take(4 * n), o_uni = take(8 * n), o_first = take(4 * n), o_dm = take(8 * n),
                 o_hm = take(8 * n), o_wcnt = take(4 * NC * nwg), o_wbase = take(4 * NC * nwg),
                 o_send = take(4 * nsend), o_rdst = take(4 * n), o_rsrc = take(4 * n), o_okeys = take(8 * n),
                 o_sum = take(sizeof(PlanSummary)), o_tmp = take(tb);
    if (S.cap < off) {
        const size_t want = std::max(off, S.cap + S.cap / 2);
        if (S.buf) MQR_CHECK_HIP(hipFree(S.buf));
        S.buf = nullptr;
        S.cap = 0;
        MQR_CHECK_HIP(hipMalloc(&S.buf, want));
        S.cap = want;
    }
    if (!S.h_sum) MQR_CHECK_HIP(hipHostMalloc(&S.h_sum, sizeof(PlanSummary), hipHostMallocDefault));
    char* b = static_cast<char*>(S.buf);
    auto U64 = [&](size_t o) { return reinterpret_cast<uint64_t*>(b + o); };
    auto I32 = [&](size_t o) { return reinterpret_cast<int32_t*>(b + o); };
    PlanSummary* dsum = reinterpret_cast<PlanSummary*>(b + o_sum);
    void* tmp = b + o_tmp;
    const unsigned g = (unsigned)((n + 255) / 256);
    MQR_CHECK_HIP(hipMemsetAsync(dsum, 0, sizeof(PlanSummary), st));
    hipLaunchKernelGGL(k_plan_iota, dim3(g), dim3(256), 0, st, I32(o_vi), n);
    size_t t = tb;
    MQR_CHECK_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, t, dkeys, U64(o_ks), I32(o_vi), I32(o_vs), (int)n, 0, 64, st));
    hipLaunchKernelGGL(k_plan_heads, dim3(g), dim3(256), 0, st, U64(o_ks), n, I32(o_head));
    t = tb;
    MQR_CHECK_HIP(hipcub::DeviceScan::InclusiveSum(tmp, t, I32(o_head), I32(o_incl), (int)n, st));
    hipLaunchKernelGGL(k_plan_union, dim3(g), dim3(256), 0, st, U64(o_ks), I32(o_incl), n, U64(o_uni), I32(o_first),
                       dsum);
    hipLaunchKernelGGL(k_plan_masks, dim3((unsigned)nwg), dim3(kPlanThreads), 0, st, U64(o_uni), I32(o_first),
                       U64(o_ks), I32(o_vs), n, mx, dsum, W, mode, root, me, U64(o_dm), U64(o_hm), I32(o_wcnt));
    t = tb;
    MQR_CHECK_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, t, I32(o_wcnt), I32(o_wbase), (int)(NC * nwg), st));
    hipLaunchKernelGGL(k_plan_lists, dim3((unsigned)nwg), dim3(kPlanThreads), 0, st, U64(o_uni), I32(o_first),
                       I32(o_vs), mx, U64(o_dm), U64(o_hm), I32(o_wcnt), I32(o_wbase), dsum, W, mode, root, me,
                       I32(o_send), I32(o_rdst), I32(o_rsrc), U64(o_okeys));
    MQR_CHECK_HIP(hipGetLastError());
    MQR_CHECK_HIP(hipMemcpyAsync(S.h_sum, dsum, sizeof(PlanSummary), hipMemcpyDeviceToHost, st));
    MQR_CHECK_HIP(hipStreamSynchronize(st));
    out.H = static_cast<const PlanSummary*>(S.h_sum);
    out.send_idx = I32(o_send);
    out.recv_dst = I32(o_rdst);
    out.recv_src = I32(o_rsrc);
    out.out_keys = U64(o_okeys);
    return 0;
}

static int grow(void** p, size_t* cap, size_t need) {
    if (*cap >= need) return 0;
    const size_t want = std::max(need, *cap + *cap / 2);  // 1.5x: few reallocations as counts vary
    if (*p) MQR_CHECK_HIP(hipFree(*p));
    *p = nullptr;
    *cap = 0;
    MQR_CHECK_HIP(hipMalloc(p, want));
    *cap = want;
    return 0;
}

// Output volume of one rank: empty it, activate its keys in order (owned first).
static int prepare_out(mqr_vbg* out, const uint64_t* dk, int64_t n, bool fused) {
    if (mqr_vbg_reset(out)) return 1;
    return activate_ordered(out, dk, n, fused);
}

// One rank's side of the exchange, whatever carries the bytes (RCCL, device copies between the
// volumes of one process, or host buffers over gloo): its plan, its output volume, the send
// buffer (segments by destination, packed from the local pool by k_gather_blocks) and the receive
// buffer (segments by source, merged in rank order by k_merge_blocks).  The segment accessors are
// the ONLY description of what a transport moves: mqr_reduce_rccl hands them to ncclSend /
// ncclRecv, mqr_merge_local to hipMemcpyAsync, mqr_xchg_* to the caller.
struct Exchange {
    PlanScratch plan;
    PlanView pv;
    PlanSummary H{};
    int W = 1, me = 0, R3 = 0;
    int pk = 0;                       // segment format (seg_load): 0 float2 pairs, 1 uint16 weights
    std::vector<size_t> soff, roff;  // block offsets of the segments
    void* sendbuf = nullptr;
    size_t send_cap = 0;
    void* recvbuf = nullptr;
    size_t recv_cap = 0;
    void* csr = nullptr;  // fused merge: the [n_out][W] entry table
    size_t csr_cap = 0;
    bool fused = true;    // k_merge_fused (false: one k_merge_blocks launch per source, mqr_merge_set_per_source)
    Exchange() = default;
    Exchange(const Exchange&) = delete;
    Exchange& operator=(const Exchange&) = delete;
    ~Exchange() {
        if (sendbuf) (void)hipFree(sendbuf);
        if (recvbuf) (void)hipFree(recvbuf);
        if (csr) (void)hipFree(csr);
    }
    size_t send_blocks(int d) const { return soff[d + 1] - soff[d]; }
    size_t recv_blocks(int s) const { return roff[s + 1] - roff[s]; }
    size_t block_bytes() const { return seg_block_bytes(pk, R3); }
    char* send_seg(int d) const { return static_cast<char*>(sendbuf) + soff[d] * block_bytes(); }
    char* recv_seg(int s) const { return static_cast<char*>(recvbuf) + roff[s] * block_bytes(); }
    size_t seg_bytes(size_t blocks) const { return blocks * block_bytes(); }
};

// `st` waits (on the device) for the integrates still in flight on a volume: integrate_frames on device
// frames returns with its last integrate queued, and the merge overlaps its all-gathers, plan and output
// activation with it -- only the send gather, the first reader of the pool, waits.  (After a sync_all,
// as in mqr_merge_local and mqr_xchg_create, nothing is pending and this enqueues nothing.)
static int order_after_volume_integrates(mqr_vbg* v, hipStream_t st) {
    for (int p = 0; p < 2; ++p)
        if (v->int_pending[p]) MQR_CHECK_HIP(hipStreamWaitEvent(st, v->int_done[p], 0));
    return 0;
}

// Plan (identical on every rank) from the gathered keys dkeys[W * mx] (device), output volume,
// send segments gathered from `local`, and the self segment copied into the receive buffer.
// ev_plan / ev_gathered (nullable) are recorded after the plan and after the gather.
static int xchg_prepare(Exchange& x, hipStream_t st, const uint64_t* dkeys, int W, int64_t mx, int me, int mode,
                        int root, mqr_vbg* local, mqr_vbg* out, hipEvent_t ev_plan, hipEvent_t ev_gathered, int pk) {
    x.W = W;
    x.me = me;
    x.R3 = (int)local->R3;
    x.pk = pk;
    if (device_plan(x.plan, st, dkeys, W, mx, me, mode, root, x.pv)) return 1;
    if (ev_plan) MQR_CHECK_HIP(hipEventRecord(ev_plan, st));
    x.H = *x.pv.H;
    x.soff.assign(W + 1, 0);
    x.roff.assign(W + 1, 0);
    for (int r = 0; r < W; ++r) {
        x.soff[r + 1] = x.soff[r] + (size_t)x.H.cnt[0][r];
        x.roff[r + 1] = x.roff[r] + (size_t)x.H.cnt[1][r];
    }
    const size_t ns = x.soff[W], nr = x.roff[W];
    const size_t eb = x.block_bytes();
    x.fused = !g_merge_per_source.load();
    // (fused: the output's activation is not waited for -- the merge writes only pool buffers, and
    // activate_ordered_check reads its table-full flag after the merge)
    if (prepare_out(out, x.pv.out_keys, x.H.n_out, x.fused)) return 1;
    if (grow(&x.sendbuf, &x.send_cap, std::max<size_t>(ns, 1) * eb) ||
        grow(&x.recvbuf, &x.recv_cap, std::max<size_t>(nr, 1) * eb))
        return 1;
    if (order_after_volume_integrates(local, st)) return 1;
    if (ns) {
        if (x.pk)
            hipLaunchKernelGGL(k_gather_blocks<1>, dim3((unsigned)ns), dim3(256), 0, st, x.pv.send_idx, (int64_t)ns,
                               local->pool, x.R3, static_cast<char*>(x.sendbuf));
        else
            hipLaunchKernelGGL(k_gather_blocks<0>, dim3((unsigned)ns), dim3(256), 0, st, x.pv.send_idx, (int64_t)ns,
                               local->pool, x.R3, static_cast<char*>(x.sendbuf));
    }
    MQR_CHECK_HIP(hipGetLastError());
    if (ev_gathered) MQR_CHECK_HIP(hipEventRecord(ev_gathered, st));
    MQR_REQUIRE(x.send_blocks(me) == x.recv_blocks(me), "merge plan: self segment lengths differ");
    if (x.send_blocks(me) && !x.fused)  // (the fused merge reads the rank's own entries from its send segment)
        MQR_CHECK_HIP(hipMemcpyAsync(x.recv_seg(me), x.send_seg(me), eb * x.send_blocks(me), hipMemcpyDeviceToDevice,
                                     st));
    return 0;
}

// Segment format from every rank's weight bound (wbound: -1 unknown): uint16 weights when all are known
// and <= 65535 (and R^3 even, so a segment is whole 4-byte words); the output's bound is their sum.
static int seg_format(const int64_t* wb, int W, int R3, int64_t* out_bound) {
    bool known = true;
    int64_t mxb = 0, sum = 0;
    for (int r = 0; r < W; ++r) {
        known = known && wb[r] >= 0;
        mxb = std::max(mxb, wb[r]);
        sum += std::max<int64_t>(wb[r], 0);
    }
    *out_bound = known ? sum : -1;
    return (known && mxb <= 65535 && R3 % 2 == 0) ? 1 : 0;
}

// Received segments into the output volume, source by source in rank order (deterministic sums).
static int xchg_merge(Exchange& x, hipStream_t st, mqr_vbg* out) {
    if (x.fused) {
        const int64_t n_out = x.H.n_out, nr = (int64_t)x.roff[x.W];
        if (n_out == 0) return 0;
        MQR_REQUIRE(x.W <= kMergeMaxEntries, "merge: too many ranks");
        if (grow(&x.csr, &x.csr_cap, sizeof(int32_t) * (size_t)n_out * x.W)) return 1;
        int32_t* ent = static_cast<int32_t*>(x.csr);
        MQR_CHECK_HIP(hipMemsetAsync(ent, 0xff, sizeof(int32_t) * (size_t)n_out * x.W, st));
        SegOffsets seg{};
        for (int r = 0; r <= x.W; ++r) seg.off[r] = (int64_t)x.roff[r];
        if (nr)
            hipLaunchKernelGGL(k_merge_entries, dim3((unsigned)((nr + 255) / 256)), dim3(256), 0, st, x.pv.recv_dst, nr,
                               seg, x.W, ent);
        const int me = x.me;
        auto fused = x.pk ? k_merge_fused<1> : k_merge_fused<0>;
        hipLaunchKernelGGL(fused, dim3((unsigned)n_out), dim3(256), 0, st, ent, x.W, n_out,
                           static_cast<const char*>(x.recvbuf), static_cast<const char*>(x.sendbuf),
                           (int64_t)x.roff[me], (int64_t)x.roff[me + 1], (int64_t)x.soff[me], x.R3, out->pool);
        MQR_CHECK_HIP(hipGetLastError());
        return 0;
    }
    for (int src = 0; src < x.W; ++src)
        if (x.recv_blocks(src)) {
            auto per_source = x.pk ? k_merge_blocks<1> : k_merge_blocks<0>;
            hipLaunchKernelGGL(per_source, dim3((unsigned)x.recv_blocks(src)), dim3(256), 0, st,
                               x.pv.recv_dst + x.roff[src], (int64_t)x.recv_blocks(src), x.recv_seg(src), x.R3,
                               out->pool);
        }
    MQR_CHECK_HIP(hipGetLastError());
    return 0;
}

// Every exit of an exchange waits for its stream first: async copies read host memory of the
// call (counts, the pinned plan summary) and a failing rank must not leave kernels in flight.
struct StreamDrain {
    hipStream_t s;
    ~StreamDrain() { (void)hipStreamSynchronize(s); }
};
// A stream the call created: drained, then destroyed (one guard, so the order cannot invert).
struct OwnedStream {
    hipStream_t s = nullptr;
    ~OwnedStream() {
        if (s) {
            (void)hipStreamSynchronize(s);
            (void)hipStreamDestroy(s);
        }
    }
};

}  // namespace mqr

// Split-phase exchange with a caller-carried transport (the gloo / host-staged twin of
// mqr_reduce_rccl, one process per rank): the same plan, segments and merge.
struct mqr_xchg {
    int device = 0, world = 1, rank = 0;
    mqr_vbg* out = nullptr;
    mqr::OwnedStream st;
    mqr::Exchange x;
    void* dkeys = nullptr;
    bool finished = false;
    ~mqr_xchg() {
        if (st.s) (void)hipStreamSynchronize(st.s);
        if (dkeys) (void)hipFree(dkeys);
    }
};

using namespace mqr;

extern "C" {

int mqr_comm_unique_id(uint8_t* id_out) {
    MQR_REQUIRE(id_out, "null argument");
    RcclApi* api = rccl();
    MQR_REQUIRE(api, g_rccl.err.c_str());
    ncclUniqueId id;
    MQR_CHECK_NCCL(api, api->GetUniqueId(&id));
    std::memcpy(id_out, id.internal, NCCL_UNIQUE_ID_BYTES);
    return 0;
}

int mqr_comm_init(int device, int rank, int world, const uint8_t* id, mqr_comm** out) {
    MQR_REQUIRE(id && out, "null argument");
    MQR_REQUIRE(world >= 1 && world <= kMaxRanks && rank >= 0 && rank < world,
                "rank / world out of range (world <= 64)");
    RcclApi* api = rccl();
    MQR_REQUIRE(api, g_rccl.err.c_str());
    MQR_CHECK_HIP(hipSetDevice(device));
    mqr_comm* c = new mqr_comm();
    c->device = device;
    c->rank = rank;
    c->world = world;
    c->x = new Exchange();
    ncclUniqueId uid;
    std::memcpy(uid.internal, id, NCCL_UNIQUE_ID_BYTES);
    ncclResult_t r = api->CommInitRank(&c->nc, world, uid, rank);
    if (r != ncclSuccess) {
        set_error(std::string("ncclCommInitRank: ") + api->GetErrorString(r));
        c->nc = nullptr;
        mqr_comm_destroy(c);
        return 1;
    }
    bool ok = hipStreamCreateWithFlags(&c->s, hipStreamNonBlocking) == hipSuccess;
    for (int i = 0; i < 5 && ok; ++i) ok = hipEventCreate(&c->ev[i]) == hipSuccess;
    if (!ok) {
        set_error("mqr_comm_init: stream / event creation failed");
        mqr_comm_destroy(c);
        return 1;
    }
    *out = c;
    return 0;
}

int mqr_comm_destroy(mqr_comm* c) {
    if (!c) return 0;
    (void)hipSetDevice(c->device);
    if (c->s) (void)hipStreamSynchronize(c->s);
    RcclApi* api = rccl();
    if (api && c->nc) api->CommDestroy(c->nc);
    delete c->x;
    if (c->small) (void)hipFree(c->small);
    for (hipEvent_t e : c->ev)
        if (e) (void)hipEventDestroy(e);
    if (c->order) (void)hipEventDestroy(c->order);
    if (c->s) (void)hipStreamDestroy(c->s);
    delete c;
    return 0;
}

int mqr_comm_timing(mqr_comm* c, float* ms4) {
    MQR_REQUIRE(c && ms4, "null argument");
    for (int i = 0; i < 4; ++i) ms4[i] = c->last_ms[i];
    return 0;
}

int mqr_comm_counts(mqr_comm* c, int64_t* send_blocks, int64_t* recv_blocks, int64_t* floats_per_block) {
    MQR_REQUIRE(c, "null argument");
    const Exchange& x = *c->x;
    const bool run = (int)x.soff.size() == c->world + 1;  // a merge has run on this communicator
    for (int p = 0; p < c->world; ++p) {
        if (send_blocks) send_blocks[p] = run ? (int64_t)x.send_blocks(p) : 0;
        if (recv_blocks) recv_blocks[p] = run ? (int64_t)x.recv_blocks(p) : 0;
    }
    if (floats_per_block) *floats_per_block = (int64_t)(x.block_bytes() / 4);
    return 0;
}

int mqr_reduce_rccl(mqr_vbg* local, mqr_comm* c, int mode, int root, mqr_vbg* out, int64_t* n_owned) {
    MQR_REQUIRE(local && c && out && n_owned, "null argument");
    MQR_REQUIRE(local != out, "mqr_reduce_rccl: `out` must be a different volume than `local` (it is emptied first)");
    MQR_REQUIRE(mode == MQR_MERGE_ROOT || mode == MQR_MERGE_SHARDED, "unknown merge mode");
    MQR_REQUIRE(root >= 0 && root < c->world, "root out of range");
    MQR_REQUIRE(local->device == c->device && out->device == c->device, "volumes and communicator on one device");
    MQR_REQUIRE(local->R == out->R && local->voxel_size == out->voxel_size, "volume geometry differs");
    RcclApi* api = rccl();
    MQR_REQUIRE(api, g_rccl.err.c_str());
    MQR_CHECK_HIP(hipSetDevice(c->device));
    *n_owned = 0;
    const int W = c->world, me = c->rank;
    // host state the stream's async copies read: declared before the drain guard, so it outlives it
    int64_t mine[2] = {0, 0};
    std::vector<int64_t> cnt(2 * W);
    StreamDrain drain{c->s};
    // The local volume's block set is final once its integrate_frames returned (the host read every
    // batch's touch counters), but its last integrate may still be running: `s` waits here for the
    // volume's touch stream only (keys, and anything else enqueued there, e.g. a reset), and for the
    // integrates just before the send gather (xchg_prepare), so the exchange's first half overlaps them.
    if (!c->order) MQR_CHECK_HIP(hipEventCreateWithFlags(&c->order, hipEventDisableTiming | hipEventDisableSystemFence));
    MQR_CHECK_HIP(hipEventRecord(c->order, local->stream));
    MQR_CHECK_HIP(hipStreamWaitEvent(c->s, c->order, 0));
    mine[0] = local->pool_count;
    mine[1] = local->wbound;
    const int64_t n_me = mine[0];
    MQR_CHECK_HIP(hipEventRecord(c->ev[0], c->s));
    // 1. all-gather (block count, weight bound) pairs (host: the padding, the segment format), then the
    //    padded packed keys
    if (grow(&c->small, &c->small_cap, sizeof(int64_t) * 2 * (W + 1))) return 1;
    int64_t* dcnt = static_cast<int64_t*>(c->small);
    MQR_CHECK_HIP(hipMemcpyAsync(dcnt + 2 * W, mine, sizeof(mine), hipMemcpyHostToDevice, c->s));
    MQR_CHECK_NCCL(api, api->AllGather(dcnt + 2 * W, dcnt, 2, ncclInt64, c->nc, c->s));
    MQR_CHECK_HIP(hipMemcpyAsync(cnt.data(), dcnt, sizeof(int64_t) * 2 * W, hipMemcpyDeviceToHost, c->s));
    MQR_CHECK_HIP(hipStreamSynchronize(c->s));
    int64_t mx = 1;
    std::vector<int64_t> wb(W);
    for (int r = 0; r < W; ++r) {
        mx = std::max(mx, cnt[2 * r]);
        wb[r] = cnt[2 * r + 1];
    }
    int64_t out_bound = -1;
    const int pk = seg_format(wb.data(), W, (int)local->R3, &out_bound);
    if (grow(&c->small, &c->small_cap, sizeof(uint64_t) * mx * (W + 1))) return 1;
    uint64_t* dkeys = static_cast<uint64_t*>(c->small);
    uint64_t* dmine = dkeys + mx * W;
    MQR_CHECK_HIP(hipMemsetAsync(dmine, 0xff, sizeof(uint64_t) * mx, c->s));
    if (n_me)
        MQR_CHECK_HIP(hipMemcpyAsync(dmine, local->bkeys, sizeof(uint64_t) * n_me, hipMemcpyDeviceToDevice, c->s));
    MQR_CHECK_NCCL(api, api->AllGather(dmine, dkeys, mx, ncclUint64, c->nc, c->s));
    // 2. plan (on the device, identical on every rank), output volume, send segments
    Exchange& x = *c->x;
    if (xchg_prepare(x, c->s, dkeys, W, mx, me, mode, root, local, out, c->ev[1], c->ev[2], pk)) return 1;
    out->wbound = out_bound;
    // 3. the sparse all-to-all: segment for p -> p, segment from p <- p (the self segment is local)
    {
        ncclResult_t r = api->GroupStart();
        for (int p = 0; p < W && r == ncclSuccess; ++p) {
            if (p == me) continue;
            if (x.send_blocks(p))
                r = api->Send(x.send_seg(p), x.seg_bytes(x.send_blocks(p)), ncclUint8, p, c->nc, c->s);
            if (r == ncclSuccess && x.recv_blocks(p))
                r = api->Recv(x.recv_seg(p), x.seg_bytes(x.recv_blocks(p)), ncclUint8, p, c->nc, c->s);
        }
        const ncclResult_t r2 = api->GroupEnd();
        if (r != ncclSuccess || r2 != ncclSuccess) {
            set_error(std::string("RCCL exchange: ") + api->GetErrorString(r != ncclSuccess ? r : r2));
            return 1;
        }
    }
    MQR_CHECK_HIP(hipEventRecord(c->ev[3], c->s));
    // 4. merge the received segments source by source (rank order)
    if (xchg_merge(x, c->s, out)) return 1;
    MQR_CHECK_HIP(hipEventRecord(c->ev[4], c->s));
    if (hipStreamSynchronize(c->s) != hipSuccess) {
        set_error("mqr_reduce_rccl: merge kernels failed");
        return 1;
    }
    if (activate_ordered_check(out)) return 1;
    for (int i = 0; i < 4; ++i)
        if (hipEventElapsedTime(&c->last_ms[i], c->ev[i], c->ev[i + 1]) != hipSuccess) c->last_ms[i] = -1.f;
    *n_owned = x.H.n_owned;
    return 0;
}

static thread_local std::vector<float> t_local_ms;  // mqr_merge_local_timing

int mqr_merge_local(mqr_vbg** locals, int n, int mode, int root, mqr_vbg** outs, int64_t* n_owned) {
    MQR_REQUIRE(locals && outs && n_owned && n >= 1 && n <= kMaxRanks, "bad arguments");
    MQR_REQUIRE(mode == MQR_MERGE_ROOT || mode == MQR_MERGE_SHARDED, "unknown merge mode");
    MQR_REQUIRE(root >= 0 && root < n, "root out of range");
    for (int r = 0; r < n; ++r) {
        MQR_REQUIRE(locals[r] && outs[r], "null volume");
        MQR_REQUIRE(locals[r]->device == locals[0]->device && outs[r]->device == locals[0]->device,
                    "mqr_merge_local: all volumes on one device");
        MQR_REQUIRE(locals[r]->R == locals[0]->R && outs[r]->R == locals[0]->R &&
                        locals[r]->voxel_size == locals[0]->voxel_size &&
                        outs[r]->voxel_size == locals[0]->voxel_size,
                    "volume geometry differs");
        for (int q = 0; q < n; ++q) MQR_REQUIRE(outs[r] != locals[q], "mqr_merge_local: an output aliases an input");
        for (int q = 0; q < r; ++q) MQR_REQUIRE(outs[r] != outs[q], "mqr_merge_local: two outputs are one volume");
    }
    MQR_CHECK_HIP(hipSetDevice(locals[0]->device));
    int64_t mx = 1;
    for (int r = 0; r < n; ++r) {
        if (sync_all(locals[r])) return 1;
        mx = std::max<int64_t>(mx, locals[r]->pool_count);
    }
    OwnedStream os;
    MQR_CHECK_HIP(hipStreamCreateWithFlags(&os.s, hipStreamNonBlocking));
    const hipStream_t st = os.s;
    // the all-gather, as device copies: rank r's keys at r mx, padded with kEmpty
    uint64_t* dkeys = nullptr;
    MQR_CHECK_HIP(hipMalloc(&dkeys, sizeof(uint64_t) * mx * n));
    struct DevFree {
        void* p;
        ~DevFree() {
            if (p) (void)hipFree(p);
        }
    } kfree{dkeys};
    MQR_CHECK_HIP(hipMemsetAsync(dkeys, 0xff, sizeof(uint64_t) * mx * n, st));
    for (int r = 0; r < n; ++r)
        if (locals[r]->pool_count)
            MQR_CHECK_HIP(hipMemcpyAsync(dkeys + r * mx, locals[r]->bkeys, sizeof(uint64_t) * locals[r]->pool_count,
                                         hipMemcpyDeviceToDevice, st));
    MQR_CHECK_HIP(hipStreamSynchronize(st));
    t_local_ms.assign(n, 0.f);
    std::vector<int64_t> wb(n);
    for (int r = 0; r < n; ++r) wb[r] = locals[r]->wbound;
    int64_t out_bound = -1;
    const int pk = g_merge_f32_segments.load() ? 0 : seg_format(wb.data(), n, (int)locals[0]->R3, &out_bound);
    if (g_merge_f32_segments.load()) seg_format(wb.data(), n, (int)locals[0]->R3, &out_bound);  // (the bound only)
    // 1. every rank's own side, exactly as mqr_reduce_rccl runs it on that rank: its plan (me = s),
    //    its output volume, its send segments packed from its own pool
    // the ranks' Exchange objects (plan scratch, send / receive buffers: grow-only) are kept per device
    // across calls, so a repeated merge allocates nothing and the per-rank times exclude hipMalloc; never
    // destroyed (a static destructor could run after the HIP runtime's teardown)
    static std::mutex cache_mu;
    static auto* cache = new std::map<int, std::vector<std::unique_ptr<Exchange>>>();
    std::lock_guard<std::mutex> cache_lock(cache_mu);
    std::vector<std::unique_ptr<Exchange>>& X = (*cache)[locals[0]->device];
    if ((int)X.size() < n) X.resize(n);
    for (int s = 0; s < n; ++s) {
        if (!X[s]) X[s].reset(new Exchange());
    }
    for (int s = 0; s < n; ++s) {
        const auto t0 = std::chrono::steady_clock::now();
        if (xchg_prepare(*X[s], st, dkeys, n, mx, s, mode, root, locals[s], outs[s], nullptr, nullptr, pk)) return 1;
        outs[s]->wbound = out_bound;
        MQR_CHECK_HIP(hipStreamSynchronize(st));
        t_local_ms[s] += std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    // 2. the transport: sender s's segment for d into d's segment from s.  Both ranks planned the
    //    pair independently, so the segment lengths and the source buffers each side lists (s's
    //    send_idx for d, d's recv_src for s) must agree entry for entry -- checked here, before any
    //    byte moves.
    std::vector<int32_t> a, b;
    for (int d = 0; d < n; ++d)
        for (int s = 0; s < n; ++s) {
            const size_t m = X[s]->send_blocks(d);
            if (m != X[d]->recv_blocks(s)) {
                set_error("mqr_merge_local: rank " + std::to_string(s) + " sends " + std::to_string(m) +
                          " blocks to rank " + std::to_string(d) + ", which expects " +
                          std::to_string(X[d]->recv_blocks(s)));
                return 4;
            }
            if (!m) continue;
            a.resize(m);
            b.resize(m);
            MQR_CHECK_HIP(hipMemcpyAsync(a.data(), X[s]->pv.send_idx + X[s]->soff[d], 4 * m, hipMemcpyDeviceToHost, st));
            MQR_CHECK_HIP(hipMemcpyAsync(b.data(), X[d]->pv.recv_src + X[d]->roff[s], 4 * m, hipMemcpyDeviceToHost, st));
            MQR_CHECK_HIP(hipStreamSynchronize(st));
            if (a != b) {
                set_error("mqr_merge_local: rank " + std::to_string(s) + "'s segment for rank " + std::to_string(d) +
                          " lists other blocks (or another order) than rank " + std::to_string(d) + " expects");
                return 4;
            }
            if (s != d)
                MQR_CHECK_HIP(hipMemcpyAsync(X[d]->recv_seg(s), X[s]->send_seg(d), X[s]->seg_bytes(m),
                                             hipMemcpyDeviceToDevice, st));
        }
    MQR_CHECK_HIP(hipStreamSynchronize(st));
    // 3. every rank merges what it received, in source-rank order
    for (int d = 0; d < n; ++d) {
        const auto t0 = std::chrono::steady_clock::now();
        if (xchg_merge(*X[d], st, outs[d])) return 1;
        MQR_CHECK_HIP(hipStreamSynchronize(st));
        if (activate_ordered_check(outs[d])) return 1;
        n_owned[d] = X[d]->H.n_owned;
        t_local_ms[d] += std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return 0;
}

int mqr_merge_set_per_source(int on) {
    g_merge_per_source.store((on & 1) != 0);
    g_merge_f32_segments.store((on & 2) != 0);
    return 0;
}

int mqr_merge_local_timing(float* ms, int n) {
    MQR_REQUIRE(ms && n >= 0, "bad arguments");
    MQR_REQUIRE((size_t)n <= t_local_ms.size(), "fewer destinations in the last mqr_merge_local");
    for (int i = 0; i < n; ++i) ms[i] = t_local_ms[i];
    return 0;
}

int mqr_xchg_create(mqr_vbg* local, int world, int rank, int mode, int root, const uint64_t* gathered_keys,
                    int64_t mx, int keys_loc, mqr_vbg* out, mqr_xchg** h) {
    MQR_REQUIRE(local && out && gathered_keys && h, "null argument");
    MQR_REQUIRE(local != out, "mqr_xchg_create: `out` must be a different volume than `local` (it is emptied first)");
    MQR_REQUIRE(world >= 1 && world <= kMaxRanks && rank >= 0 && rank < world, "rank / world out of range (world <= 64)");
    MQR_REQUIRE(mode == MQR_MERGE_ROOT || mode == MQR_MERGE_SHARDED, "unknown merge mode");
    MQR_REQUIRE(root >= 0 && root < world, "root out of range");
    MQR_REQUIRE(mx >= 1, "mx (padded keys per rank) must be >= 1");
    MQR_REQUIRE(local->device == out->device, "volumes on one device");
    MQR_REQUIRE(local->R == out->R && local->voxel_size == out->voxel_size, "volume geometry differs");
    *h = nullptr;
    MQR_CHECK_HIP(hipSetDevice(local->device));
    if (sync_all(local)) return 1;
    MQR_REQUIRE(local->pool_count <= mx, "mqr_xchg_create: mx is smaller than this rank's block count");
    std::unique_ptr<mqr_xchg> xh(new mqr_xchg());
    xh->device = local->device;
    xh->world = world;
    xh->rank = rank;
    xh->out = out;
    MQR_CHECK_HIP(hipStreamCreateWithFlags(&xh->st.s, hipStreamNonBlocking));
    if (keys_loc == MQR_DEVICE && order_after_caller(xh->device, xh->st.s)) return 2;
    const size_t kb = sizeof(uint64_t) * (size_t)mx * world;
    MQR_CHECK_HIP(hipMalloc(&xh->dkeys, kb));
    MQR_CHECK_HIP(hipMemcpyAsync(xh->dkeys, gathered_keys, kb,
                                 keys_loc == MQR_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, xh->st.s));
    // This rank's row must be its own keys in buffer order, padded with kEmpty: the plan's send lists
    // index the local pool through it (k_gather_blocks reads buffer `send_idx`), so a foreign or
    // reordered row would read past pool_count or merge blocks into the wrong places.
    {
        const int64_t n = local->pool_count;
        std::vector<uint64_t> row((size_t)mx), mine((size_t)n);
        MQR_CHECK_HIP(hipMemcpyAsync(row.data(), static_cast<const uint64_t*>(xh->dkeys) + (size_t)rank * mx,
                                     sizeof(uint64_t) * mx, hipMemcpyDeviceToHost, xh->st.s));
        if (n) MQR_CHECK_HIP(hipMemcpyAsync(mine.data(), local->bkeys, sizeof(uint64_t) * n, hipMemcpyDeviceToHost,
                                            xh->st.s));
        MQR_CHECK_HIP(hipStreamSynchronize(xh->st.s));
        bool ok = std::equal(mine.begin(), mine.end(), row.begin());
        for (int64_t i = n; ok && i < mx; ++i) ok = row[(size_t)i] == kEmpty;
        if (!ok) {
            set_error("mqr_xchg_create: row " + std::to_string(rank) + " of gathered_keys is not this rank's " +
                      std::to_string(n) + " block keys in buffer order padded with 0xFF..FF");
            return 4;
        }
    }
    if (xchg_prepare(xh->x, xh->st.s, static_cast<const uint64_t*>(xh->dkeys), world, mx, rank, mode, root, local,
                     out, nullptr, nullptr, 0))  // (the caller carries float32 pairs)
        return 1;
    out->wbound = -1;  // (the caller's transport does not carry the ranks' bounds)
    MQR_CHECK_HIP(hipStreamSynchronize(xh->st.s));
    *h = xh.release();
    return 0;
}

int mqr_xchg_counts(mqr_xchg* h, int64_t* send_blocks, int64_t* recv_blocks, int64_t* n_owned, int64_t* floats_per_block) {
    MQR_REQUIRE(h, "null argument");
    for (int p = 0; p < h->world; ++p) {
        if (send_blocks) send_blocks[p] = (int64_t)h->x.send_blocks(p);
        if (recv_blocks) recv_blocks[p] = (int64_t)h->x.recv_blocks(p);
    }
    if (n_owned) *n_owned = h->x.H.n_owned;
    if (floats_per_block) *floats_per_block = (int64_t)(h->x.block_bytes() / 4);
    return 0;
}

int mqr_xchg_send_segment(mqr_xchg* h, int peer, float* dst, int loc) {
    MQR_REQUIRE(h && peer >= 0 && peer < h->world, "bad arguments");
    MQR_REQUIRE(!h->finished, "mqr_xchg_send_segment: exchange already finished");
    const size_t m = h->x.send_blocks(peer);
    if (!m) return 0;
    MQR_REQUIRE(dst, "null destination");
    MQR_CHECK_HIP(hipSetDevice(h->device));
    if (loc == MQR_DEVICE && order_after_caller(h->device, h->st.s)) return 2;
    MQR_CHECK_HIP(hipMemcpyAsync(dst, h->x.send_seg(peer), h->x.seg_bytes(m),
                                 loc == MQR_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, h->st.s));
    MQR_CHECK_HIP(hipStreamSynchronize(h->st.s));
    return 0;
}

int mqr_xchg_recv_segment(mqr_xchg* h, int peer, const float* src, int loc) {
    MQR_REQUIRE(h && peer >= 0 && peer < h->world, "bad arguments");
    MQR_REQUIRE(peer != h->rank, "mqr_xchg_recv_segment: the self segment is already in place");
    MQR_REQUIRE(!h->finished, "mqr_xchg_recv_segment: exchange already finished");
    const size_t m = h->x.recv_blocks(peer);
    if (!m) return 0;
    MQR_REQUIRE(src, "null source");
    MQR_CHECK_HIP(hipSetDevice(h->device));
    if (loc == MQR_DEVICE && order_after_caller(h->device, h->st.s)) return 2;
    MQR_CHECK_HIP(hipMemcpyAsync(h->x.recv_seg(peer), src, h->x.seg_bytes(m),
                                 loc == MQR_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, h->st.s));
    MQR_CHECK_HIP(hipStreamSynchronize(h->st.s));
    return 0;
}

int mqr_xchg_finish(mqr_xchg* h, int64_t* n_owned) {
    MQR_REQUIRE(h, "null argument");
    MQR_REQUIRE(!h->finished, "mqr_xchg_finish: called twice");
    MQR_CHECK_HIP(hipSetDevice(h->device));
    if (xchg_merge(h->x, h->st.s, h->out)) return 1;
    MQR_CHECK_HIP(hipStreamSynchronize(h->st.s));
    if (activate_ordered_check(h->out)) return 1;
    h->finished = true;
    if (n_owned) *n_owned = h->x.H.n_owned;
    return 0;
}

int mqr_xchg_destroy(mqr_xchg* h) {
    if (!h) return 0;
    (void)hipSetDevice(h->device);
    delete h;
    return 0;
}

}  // extern "C"
