// merge.hip -- the single exchange step of frame-sharded fusion across the GPUs of one node
// (SURVEY §8(e)): every rank integrated a contiguous frame range into its own volume; this merges
// them, over RCCL (xGMI) or, for tests on one device, over device-to-device copies.
//
// The reference's unit-weight running average makes partial volumes mergeable:
//   tsdf = (w_a tsdf_a + w_b tsdf_b) / (w_a + w_b),  weight = w_a + w_b     (App. A.3)
// applied source by source in rank order (deterministic); a voxel that only one rank saw keeps
// that rank's (tsdf, weight) bit for bit.
//
// Plan (identical on every rank, computed on the host from the all-gathered block keys):
//   union U = sorted distinct keys (packed order = lexicographic x, y, z); owner slices =
//   [U r / N, U (r+1) / N); each union block goes to a destination set:
//     MQR_MERGE_ROOT     the root only (the root's output holds the whole volume)
//     MQR_MERGE_SHARDED  its owner and the owners of its 26 neighbours -- so every rank holds its
//                        owned blocks plus a one-block halo, and extracts exactly the cubes whose
//                        origin lies in an owned block (mqr_extract_mesh_owned): triangle counts of
//                        the shards add up to the single-volume count.
//   Every rank sends each of its blocks once per destination (grouped ncclSend / ncclRecv: a
//   sparse all-to-all, per-link traffic ~ own blocks + halo instead of the dense union).
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <climits>
#include <cstring>
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

struct mqr_comm {
    int device = 0, rank = 0, world = 1;
    ncclComm_t nc = nullptr;
    hipStream_t s = nullptr;
    // grow-only exchange buffers
    void* sendbuf = nullptr;
    size_t send_cap = 0;
    void* recvbuf = nullptr;
    size_t recv_cap = 0;
    void* small = nullptr;  // counts, padded keys
    size_t small_cap = 0;
    void* lists = nullptr;  // send / receive index lists, output keys (no allocation per merge:
    size_t lists_cap = 0;   // hipFree synchronises the device)
};

namespace mqr {

// ------------------------------------------------------------------ kernels
// (tsdf, weight) of listed local buffers into consecutive [R3] float2 entries.
__global__ void k_gather_blocks(const int32_t* __restrict__ bufs, int64_t n, const float2* __restrict__ pool, int R3,
                                float2* __restrict__ out) {
    const int64_t j = blockIdx.x;
    if (j >= n) return;
    const float2* src = pool + (int64_t)bufs[j] * R3;
    float2* dst = out + j * R3;
    for (int p = threadIdx.x; p < R3; p += blockDim.x) dst[p] = src[p];
}

// Merge received entries into destination buffers: a voxel with no weight yet takes the entry as
// is, one with weight merges by the running-average identity; entries with zero weight change
// nothing.  One launch per source rank, in rank order; a buffer appears at most once per source.
__global__ void k_merge_blocks(const int32_t* __restrict__ dst, int64_t n, const float2* __restrict__ in, int R3,
                               float2* __restrict__ pool) {
    const int64_t j = blockIdx.x;
    if (j >= n) return;
    const float2* src = in + j * R3;
    float2* out = pool + (int64_t)dst[j] * R3;
    for (int p = threadIdx.x; p < R3; p += blockDim.x) {
        const float2 a = out[p], b = src[p];
        if (b.y == 0.f) continue;
        if (a.y == 0.f) {
            out[p] = b;
        } else {
            const float w = a.y + b.y;
            out[p] = make_float2((a.y * a.x + b.y * b.x) / w, w);
        }
    }
}

// ------------------------------------------------------------------ host plan
struct MergePlan {
    int world = 1;
    std::vector<uint64_t> uni;     // sorted union
    std::vector<int64_t> bounds;   // owner slices of the union (indices), world + 1
    std::vector<uint64_t> lokey;   // first key of each slice (world entries)
    std::vector<uint64_t> dmask;   // destination ranks of each union block
    int owner(int64_t u) const {
        return (int)(std::upper_bound(bounds.begin(), bounds.end(), u) - bounds.begin()) - 1;
    }
    int owner_of_key(uint64_t k) const {  // the slice whose key range holds k (k in the union)
        return std::max(0, (int)(std::upper_bound(lokey.begin(), lokey.end(), k) - lokey.begin()) - 1);
    }
    int64_t index(uint64_t k) const {  // union index of k, -1 if absent
        const auto it = std::lower_bound(uni.begin(), uni.end(), k);
        return it != uni.end() && *it == k ? (int64_t)(it - uni.begin()) : -1;
    }
};

static int build_plan(const std::vector<std::vector<uint64_t>>& keys, int mode, int root, MergePlan& P) {
    const int W = (int)keys.size();
    P.world = W;
    size_t tot = 0;
    for (auto& k : keys) tot += k.size();
    P.uni.clear();
    P.uni.reserve(tot);
    for (auto& k : keys) P.uni.insert(P.uni.end(), k.begin(), k.end());
    std::sort(P.uni.begin(), P.uni.end());
    P.uni.erase(std::unique(P.uni.begin(), P.uni.end()), P.uni.end());
    const int64_t U = (int64_t)P.uni.size();
    P.bounds.resize(W + 1);
    for (int r = 0; r <= W; ++r) P.bounds[r] = U * r / W;
    P.lokey.resize(W);
    for (int r = 0; r < W; ++r) P.lokey[r] = P.bounds[r] < U ? P.uni[P.bounds[r]] : kEmpty;
    P.dmask.assign(U, 0);
    for (int64_t u = 0; u < U; ++u) {
        if (mode == MQR_MERGE_ROOT) {
            P.dmask[u] = 1ull << root;
            continue;
        }
        const int own = P.owner(u);
        uint64_t m = 1ull << own;
        int x, y, z;
        unpack_key(P.uni[u], x, y, z);
        // keys pack x-major, so every neighbour key lies in [pack(x-1,y-1,z-1), pack(x+1,y+1,z+1)]:
        // a block whose neighbourhood range sits inside its own slice's key range needs no lookup
        const bool inside = key_in_range(x - 1, y - 1, z - 1) && key_in_range(x + 1, y + 1, z + 1) &&
                            pack_key(x - 1, y - 1, z - 1) >= P.lokey[own] &&
                            (own + 1 == W || pack_key(x + 1, y + 1, z + 1) < P.lokey[own + 1]);
        if (!inside) {
            for (int k = 0; k < 27; ++k) {
                const int nx = x + k % 3 - 1, ny = y + (k / 3) % 3 - 1, nz = z + k / 9 - 1;
                if (k == 13 || !key_in_range(nx, ny, nz)) continue;
                const uint64_t nk = pack_key(nx, ny, nz);
                if (P.index(nk) >= 0) m |= 1ull << P.owner_of_key(nk);  // n's owner needs u as halo
            }
        }
        P.dmask[u] = m;
    }
    return 0;
}

// What rank `me` sends to each destination (local buffer indices, by union index) and receives
// from each source (destination buffer of each entry), and the keys of its output volume (owned
// union blocks first, then halo, each by union index).
struct RankLists {
    std::vector<std::vector<int32_t>> send;  // [dest] local buffers
    std::vector<std::vector<int32_t>> recv;  // [source] output buffers
    std::vector<uint64_t> out_keys;
    int64_t n_owned = 0;
};

static void rank_lists(const MergePlan& P, const std::vector<std::vector<uint64_t>>& keys, int me, int mode,
                       RankLists& L) {
    const int W = P.world;
    const int64_t U = (int64_t)P.uni.size();
    const uint64_t bit = 1ull << me;
    std::vector<int64_t> outpos(U, -1);
    L.out_keys.clear();
    const int64_t lo = mode == MQR_MERGE_ROOT ? 0 : P.bounds[me], hi = mode == MQR_MERGE_ROOT ? U : P.bounds[me + 1];
    for (int64_t u = lo; u < hi; ++u)
        if (P.dmask[u] & bit) {
            outpos[u] = (int64_t)L.out_keys.size();
            L.out_keys.push_back(P.uni[u]);
        }
    L.n_owned = (int64_t)L.out_keys.size();
    for (int64_t u = 0; u < U; ++u)
        if ((P.dmask[u] & bit) && outpos[u] < 0) {
            outpos[u] = (int64_t)L.out_keys.size();
            L.out_keys.push_back(P.uni[u]);
        }
    // sends: my blocks by union index
    const auto& mine = keys[me];
    std::vector<std::pair<int64_t, int32_t>> ub(mine.size());
    for (size_t b = 0; b < mine.size(); ++b) ub[b] = {P.index(mine[b]), (int32_t)b};
    std::sort(ub.begin(), ub.end());
    L.send.assign(W, {});
    for (auto& e : ub)
        for (int d = 0; d < W; ++d)
            if (P.dmask[e.first] & (1ull << d)) L.send[d].push_back(e.second);
    // receives: each source's blocks that come to me, in the order that source sends them
    L.recv.assign(W, {});
    for (int s = 0; s < W; ++s) {
        std::vector<int64_t> us;
        for (uint64_t k : keys[s]) {
            const int64_t u = P.index(k);
            if (P.dmask[u] & bit) us.push_back(u);
        }
        std::sort(us.begin(), us.end());
        for (int64_t u : us) L.recv[s].push_back((int32_t)outpos[u]);
    }
}

static int grow(void** p, size_t* cap, size_t need) {
    if (*cap >= need) return 0;
    if (*p) MQR_CHECK_HIP(hipFree(*p));
    *p = nullptr;
    *cap = 0;
    const size_t want = std::max(need, *cap + *cap / 2);
    MQR_CHECK_HIP(hipMalloc(p, want));
    *cap = want;
    return 0;
}

static int local_keys(mqr_vbg* v, std::vector<uint64_t>& out) {
    if (sync_all(v)) return 1;
    out.resize(v->pool_count);
    if (v->pool_count)
        MQR_CHECK_HIP(hipMemcpy(out.data(), v->bkeys, sizeof(uint64_t) * v->pool_count, hipMemcpyDeviceToHost));
    return 0;
}

// Upload an int32 list to `dst` (device) on stream s.
static int upload(const std::vector<int32_t>& h, int32_t* dst, hipStream_t s) {
    if (!h.empty()) MQR_CHECK_HIP(hipMemcpyAsync(dst, h.data(), sizeof(int32_t) * h.size(), hipMemcpyHostToDevice, s));
    return 0;
}

static size_t total(const std::vector<std::vector<int32_t>>& l) {
    size_t n = 0;
    for (auto& x : l) n += x.size();
    return n;
}

// Output volume of one rank: empty it, activate its keys in order (owned first).  `dk`: device
// scratch for the keys (>= out_keys.size() entries), or null to allocate one here.
static int prepare_out(mqr_vbg* out, const RankLists& L, uint64_t* dk) {
    if (mqr_vbg_reset(out)) return 1;
    if (L.out_keys.empty()) return 0;
    uint64_t* own = nullptr;
    if (!dk) {
        MQR_CHECK_HIP(hipMalloc(&own, sizeof(uint64_t) * L.out_keys.size()));
        dk = own;
    }
    MQR_CHECK_HIP(hipMemcpyAsync(dk, L.out_keys.data(), sizeof(uint64_t) * L.out_keys.size(), hipMemcpyHostToDevice,
                                 out->stream));
    const int rc = activate_ordered(out, dk, (int64_t)L.out_keys.size());
    if (own) (void)hipFree(own);
    return rc;
}

}  // namespace mqr

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
    MQR_REQUIRE(world >= 1 && world <= 64 && rank >= 0 && rank < world, "rank / world out of range (world <= 64)");
    RcclApi* api = rccl();
    MQR_REQUIRE(api, g_rccl.err.c_str());
    MQR_CHECK_HIP(hipSetDevice(device));
    mqr_comm* c = new mqr_comm();
    c->device = device;
    c->rank = rank;
    c->world = world;
    ncclUniqueId uid;
    std::memcpy(uid.internal, id, NCCL_UNIQUE_ID_BYTES);
    ncclResult_t r = api->CommInitRank(&c->nc, world, uid, rank);
    if (r != ncclSuccess) {
        set_error(std::string("ncclCommInitRank: ") + api->GetErrorString(r));
        delete c;
        return 1;
    }
    if (hipStreamCreateWithFlags(&c->s, hipStreamNonBlocking) != hipSuccess) {
        set_error("mqr_comm_init: stream creation failed");
        api->CommDestroy(c->nc);
        delete c;
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
    if (c->sendbuf) (void)hipFree(c->sendbuf);
    if (c->recvbuf) (void)hipFree(c->recvbuf);
    if (c->small) (void)hipFree(c->small);
    if (c->lists) (void)hipFree(c->lists);
    if (c->s) (void)hipStreamDestroy(c->s);
    delete c;
    return 0;
}

int mqr_reduce_rccl(mqr_vbg* local, mqr_comm* c, int mode, int root, mqr_vbg* out, int64_t* n_owned) {
    MQR_REQUIRE(local && c && out && n_owned, "null argument");
    MQR_REQUIRE(mode == MQR_MERGE_ROOT || mode == MQR_MERGE_SHARDED, "unknown merge mode");
    MQR_REQUIRE(root >= 0 && root < c->world, "root out of range");
    MQR_REQUIRE(local->device == c->device && out->device == c->device, "volumes and communicator on one device");
    MQR_REQUIRE(local->R == out->R && local->voxel_size == out->voxel_size, "volume geometry differs");
    RcclApi* api = rccl();
    MQR_REQUIRE(api, g_rccl.err.c_str());
    MQR_CHECK_HIP(hipSetDevice(c->device));
    const int W = c->world, me = c->rank;
    const int R3 = (int)local->R3;
    // 1. all-gather block counts, then the padded packed keys
    std::vector<uint64_t> mine;
    if (local_keys(local, mine)) return 1;
    const int64_t n_me = (int64_t)mine.size();
    if (grow(&c->small, &c->small_cap, sizeof(int64_t) * 2 * W)) return 1;
    int64_t* dcnt = static_cast<int64_t*>(c->small);
    MQR_CHECK_HIP(hipMemcpyAsync(dcnt + W, &n_me, sizeof(int64_t), hipMemcpyHostToDevice, c->s));
    MQR_CHECK_NCCL(api, api->AllGather(dcnt + W, dcnt, 1, ncclInt64, c->nc, c->s));
    std::vector<int64_t> cnt(W);
    MQR_CHECK_HIP(hipMemcpyAsync(cnt.data(), dcnt, sizeof(int64_t) * W, hipMemcpyDeviceToHost, c->s));
    MQR_CHECK_HIP(hipStreamSynchronize(c->s));
    const int64_t mx = std::max<int64_t>(1, *std::max_element(cnt.begin(), cnt.end()));
    if (grow(&c->small, &c->small_cap, sizeof(uint64_t) * mx * (W + 1))) return 1;
    uint64_t* dkeys = static_cast<uint64_t*>(c->small);
    uint64_t* dmine = dkeys + mx * W;
    MQR_CHECK_HIP(hipMemsetAsync(dmine, 0xff, sizeof(uint64_t) * mx, c->s));
    if (n_me) MQR_CHECK_HIP(hipMemcpyAsync(dmine, mine.data(), sizeof(uint64_t) * n_me, hipMemcpyHostToDevice, c->s));
    MQR_CHECK_NCCL(api, api->AllGather(dmine, dkeys, mx, ncclUint64, c->nc, c->s));
    std::vector<uint64_t> flat(mx * W);
    MQR_CHECK_HIP(hipMemcpyAsync(flat.data(), dkeys, sizeof(uint64_t) * mx * W, hipMemcpyDeviceToHost, c->s));
    MQR_CHECK_HIP(hipStreamSynchronize(c->s));
    std::vector<std::vector<uint64_t>> keys(W);
    for (int r = 0; r < W; ++r) keys[r].assign(flat.begin() + r * mx, flat.begin() + r * mx + cnt[r]);
    // 2. plan (identical everywhere) and this rank's lists
    MergePlan P;
    build_plan(keys, mode, root, P);
    RankLists L;
    rank_lists(P, keys, me, mode, L);
    const size_t ns = total(L.send), nr = total(L.recv);
    // index lists, then (8-byte aligned) the output keys
    const size_t lbytes = (sizeof(int32_t) * (ns + nr) + 7) & ~size_t(7);
    if (grow(&c->lists, &c->lists_cap, std::max<size_t>(lbytes + sizeof(uint64_t) * L.out_keys.size(), 8))) return 1;
    int32_t* dlists = static_cast<int32_t*>(c->lists);
    if (prepare_out(out, L, reinterpret_cast<uint64_t*>(static_cast<char*>(c->lists) + lbytes))) return 1;
    // 3. gather my outgoing blocks (segments by destination), post the sparse all-to-all
    const size_t eb = sizeof(float2) * R3;
    if (grow(&c->sendbuf, &c->send_cap, std::max<size_t>(ns, 1) * eb) ||
        grow(&c->recvbuf, &c->recv_cap, std::max<size_t>(nr, 1) * eb))
        return 1;
    std::vector<int32_t> sidx, ridx;
    for (auto& l : L.send) sidx.insert(sidx.end(), l.begin(), l.end());
    for (auto& l : L.recv) ridx.insert(ridx.end(), l.begin(), l.end());
    int rc = upload(sidx, dlists, c->s) || upload(ridx, dlists + ns, c->s);
    if (!rc && ns)
        hipLaunchKernelGGL(k_gather_blocks, dim3((unsigned)ns), dim3(256), 0, c->s, dlists, (int64_t)ns, local->pool,
                           R3, static_cast<float2*>(c->sendbuf));
    float2* sb = static_cast<float2*>(c->sendbuf);
    float2* rb = static_cast<float2*>(c->recvbuf);
    std::vector<size_t> soff(W + 1, 0), roff(W + 1, 0);
    for (int r = 0; r < W; ++r) {
        soff[r + 1] = soff[r] + L.send[r].size();
        roff[r + 1] = roff[r] + L.recv[r].size();
    }
    if (!rc) {
        if (L.send[me].size())
            rc = hipMemcpyAsync(rb + roff[me] * R3, sb + soff[me] * R3, eb * L.send[me].size(),
                                hipMemcpyDeviceToDevice, c->s) != hipSuccess;
        ncclResult_t r = api->GroupStart();
        for (int p = 0; p < W && r == ncclSuccess; ++p) {
            if (p == me) continue;
            if (L.send[p].size())
                r = api->Send(sb + soff[p] * R3, L.send[p].size() * R3 * 2, ncclFloat32, p, c->nc, c->s);
            if (r == ncclSuccess && L.recv[p].size())
                r = api->Recv(rb + roff[p] * R3, L.recv[p].size() * R3 * 2, ncclFloat32, p, c->nc, c->s);
        }
        const ncclResult_t r2 = api->GroupEnd();
        if (r != ncclSuccess || r2 != ncclSuccess) {
            set_error(std::string("RCCL exchange: ") + api->GetErrorString(r != ncclSuccess ? r : r2));
            rc = 1;
        }
    }
    // 4. merge the received entries source by source (rank order)
    for (int s = 0; s < W && !rc; ++s)
        if (L.recv[s].size())
            hipLaunchKernelGGL(k_merge_blocks, dim3((unsigned)L.recv[s].size()), dim3(256), 0, c->s,
                               dlists + ns + roff[s], (int64_t)L.recv[s].size(), rb + roff[s] * R3, R3, out->pool);
    if (!rc && (hipGetLastError() != hipSuccess || hipStreamSynchronize(c->s) != hipSuccess)) {
        set_error("mqr_reduce_rccl: merge kernels failed");
        rc = 1;
    }
    *n_owned = rc ? 0 : L.n_owned;
    return rc;
}

int mqr_merge_local(mqr_vbg** locals, int n, int mode, int root, mqr_vbg** outs, int64_t* n_owned) {
    MQR_REQUIRE(locals && outs && n_owned && n >= 1 && n <= 64, "bad arguments");
    MQR_REQUIRE(mode == MQR_MERGE_ROOT || mode == MQR_MERGE_SHARDED, "unknown merge mode");
    MQR_REQUIRE(root >= 0 && root < n, "root out of range");
    for (int r = 0; r < n; ++r) MQR_REQUIRE(locals[r] && outs[r], "null volume");
    const int R3 = (int)locals[0]->R3;
    std::vector<std::vector<uint64_t>> keys(n);
    for (int r = 0; r < n; ++r)
        if (local_keys(locals[r], keys[r])) return 1;
    MergePlan P;
    build_plan(keys, mode, root, P);
    std::vector<RankLists> L(n);
    for (int r = 0; r < n; ++r) rank_lists(P, keys, r, mode, L[r]);
    const size_t eb = sizeof(float2) * R3;
    // every source gathers its outgoing segments; every destination merges them in source order
    std::vector<float2*> send(n, nullptr);
    std::vector<std::vector<size_t>> soff(n, std::vector<size_t>(n + 1, 0));
    int rc = 0;
    for (int s = 0; s < n && !rc; ++s) {
        MQR_CHECK_HIP(hipSetDevice(locals[s]->device));
        const size_t ns = total(L[s].send);
        for (int d = 0; d < n; ++d) soff[s][d + 1] = soff[s][d] + L[s].send[d].size();
        std::vector<int32_t> sidx;
        for (auto& l : L[s].send) sidx.insert(sidx.end(), l.begin(), l.end());
        int32_t* di = nullptr;
        rc = hipMalloc(&send[s], std::max<size_t>(ns, 1) * eb) != hipSuccess ||
             hipMalloc(&di, sizeof(int32_t) * std::max<size_t>(ns, 1)) != hipSuccess;
        if (!rc && ns) {
            rc = upload(sidx, di, locals[s]->stream);
            hipLaunchKernelGGL(k_gather_blocks, dim3((unsigned)ns), dim3(256), 0, locals[s]->stream, di, (int64_t)ns,
                               locals[s]->pool, R3, send[s]);
            rc = rc || hipStreamSynchronize(locals[s]->stream) != hipSuccess;
        }
        if (di) (void)hipFree(di);
        if (rc) set_error("mqr_merge_local: gather failed");
    }
    for (int d = 0; d < n && !rc; ++d) {
        mqr_vbg* o = outs[d];
        MQR_CHECK_HIP(hipSetDevice(o->device));
        if (prepare_out(o, L[d], nullptr)) {
            rc = 1;
            break;
        }
        for (int s = 0; s < n && !rc; ++s) {
            const size_t m = L[d].recv[s].size();
            if (!m) continue;
            float2* rb = nullptr;
            int32_t* di = nullptr;
            rc = hipMalloc(&rb, m * eb) != hipSuccess || hipMalloc(&di, sizeof(int32_t) * m) != hipSuccess ||
                 // on the merge's stream: a plain device-to-device hipMemcpy is not ordered before
                 // work on a non-blocking stream
                 hipMemcpyAsync(rb, send[s] + soff[s][d] * R3, m * eb, hipMemcpyDefault, o->stream) != hipSuccess ||
                 upload(L[d].recv[s], di, o->stream);
            if (!rc) {
                hipLaunchKernelGGL(k_merge_blocks, dim3((unsigned)m), dim3(256), 0, o->stream, di, (int64_t)m, rb, R3,
                                   o->pool);
                rc = hipGetLastError() != hipSuccess || hipStreamSynchronize(o->stream) != hipSuccess;
            }
            if (rb) (void)hipFree(rb);
            if (di) (void)hipFree(di);
            if (rc) set_error("mqr_merge_local: merge failed");
        }
        n_owned[d] = L[d].n_owned;
    }
    for (int s = 0; s < n; ++s)
        if (send[s]) (void)hipFree(send[s]);
    return rc;
}

}  // extern "C"
