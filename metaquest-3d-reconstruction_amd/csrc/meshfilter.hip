// meshfilter.hip -- filter_mesh_components on the device.
//
// Reference: processing/reconstruction/utils/o3d_utils.py:241-321, run after every mesh
// extraction (reconstruct_scene.py:110-122, 191-195; optimize_color_pose.py:16-22).  It calls
// Open3D legacy TriangleMesh methods; their semantics are restated here:
//   cluster_connected_triangles  triangles sharing an edge (by vertex index) are connected;
//                                cluster ids in order of each cluster's lowest triangle index
//   keep clusters with >= min_triangle_count triangles (none: the largest, first on ties)
//   remove_triangles_by_mask + remove_unreferenced_vertices   (only if something was removed)
//   remove_degenerate_triangles   repeated vertex index
//   remove_duplicated_triangles   same rotation-canonical index triple, first occurrence kept
//   remove_duplicated_vertices    identical coordinates, first occurrence kept, triangles remapped
//   remove_non_manifold_edges     per edge with > 2 triangles drop the smallest-area ones until 2
//                                 remain, repeat until manifold; zero-area triangles are dropped
// Order is preserved everywhere (stable compactions), so the output is deterministic.  The one
// deviation: Open3D visits non-manifold edges in std::unordered_map order; this visits them in
// ascending (v_min, v_max) order (the result differs only where two non-manifold edges share a
// triangle).
//
// Device work: edge keys (u64) -> hipcub radix sort -> union-find over triangles (hook larger
// root under smaller, so the root is the component's lowest triangle index) -> per-cluster
// counts; stable compactions with hipcub::DeviceSelect; duplicate detection by two stable radix
// passes over the canonical keys.  Only the short list of non-manifold edges goes to the host.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <limits>
#include <map>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "mqr_common.hpp"

namespace mqr {
namespace mf {

// ------------------------------------------------------------------ kernels
__global__ void k_iota(int32_t* a, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) a[i] = (int32_t)i;
}

__global__ void k_edge_keys(const int32_t* __restrict__ tri, int64_t nt, uint64_t* keys, int32_t* slot) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 3 * nt) return;
    const int64_t t = i / 3;
    const int k = (int)(i % 3);
    const uint32_t a = (uint32_t)tri[3 * t + k], b = (uint32_t)tri[3 * t + (k + 1) % 3];
    keys[i] = a < b ? ((uint64_t)a << 32 | b) : ((uint64_t)b << 32 | a);
    slot[i] = (int32_t)i;
}

__device__ inline int32_t uf_find(int32_t* p, int32_t x) {
    while (true) {
        const int32_t px = p[x];
        if (px == x) return x;
        const int32_t gx = p[px];
        if (gx != px) p[x] = gx;  // path halving (benign race: any ancestor is a valid parent)
        x = gx;
    }
}

__global__ void k_union_edges(const uint64_t* __restrict__ keys, const int32_t* __restrict__ slot, int64_t m,
                              int32_t* parent) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0 || i >= m || keys[i] != keys[i - 1]) return;
    int32_t a = slot[i - 1] / 3, b = slot[i] / 3;
    while (true) {
        a = uf_find(parent, a);
        b = uf_find(parent, b);
        if (a == b) return;
        if (a > b) {
            const int32_t t = a;
            a = b;
            b = t;
        }
        if (atomicCAS(&parent[b], b, a) == b) return;
    }
}

// Cluster sizes: lanes of a wave mostly share one root (neighbouring triangles), so the wave adds
// each distinct root's lane count with one atomic (per-lane atomics on the root of a 2 M-triangle
// cluster serialised this kernel to ~20 ms).
__global__ void k_roots(int32_t* parent, int64_t n, int32_t* count, int32_t* is_root) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & 63;
    int32_t r = -1;
    if (i < n) {
        r = uf_find(parent, (int32_t)i);
        is_root[i] = r == (int32_t)i;
    }
    bool todo = i < n;
    while (true) {
        const uint64_t pending = __ballot(todo);
        if (!pending) break;
        const int leader = __ffsll((unsigned long long)pending) - 1;
        const int32_t lr = __shfl(r, leader, 64);
        const bool same = todo && r == lr;
        const uint64_t peers = __ballot(same);
        if (lane == leader) atomicAdd(&count[lr], __popcll(peers));
        if (same) todo = false;
    }
}

// Read-only final find into a separate array: compressing `parent` in place here would race with
// other threads' path halving (a halving write can land after a final write and leave a non-root).
__global__ void k_final_root(const int32_t* __restrict__ parent, int64_t n, int32_t* root) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int32_t x = (int32_t)i;
    while (parent[x] != x) x = parent[x];
    root[i] = x;
}

__global__ void k_cluster_table(const int32_t* __restrict__ is_root, const int32_t* __restrict__ cid,
                                const int32_t* __restrict__ count, int64_t n, int32_t* ccount) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && is_root[i]) ccount[cid[i]] = count[i];
}

__global__ void k_keep_by_cluster(const int32_t* __restrict__ root, const int32_t* __restrict__ cid,
                                  const uint8_t* __restrict__ keep_cluster, int64_t n, uint8_t* keep) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) keep[i] = keep_cluster[cid[root[i]]];
}

__global__ void k_gather_tris(const int32_t* __restrict__ tri, const int32_t* __restrict__ sel, int64_t m,
                              int32_t* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const int64_t s = sel[i];
    out[3 * i] = tri[3 * s];
    out[3 * i + 1] = tri[3 * s + 1];
    out[3 * i + 2] = tri[3 * s + 2];
}

__global__ void k_mark_vertices(const int32_t* __restrict__ tri, int64_t nt, int32_t* used) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < 3 * nt) used[tri[i]] = 1;
}

__global__ void k_remap(int32_t* tri, int64_t nt, const int32_t* __restrict__ map) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < 3 * nt) tri[i] = map[tri[i]];
}

__global__ void k_gather_vertices(const float* __restrict__ pos, const float* __restrict__ nrm,
                                  const int32_t* __restrict__ sel, int64_t m, float* pos_out, float* nrm_out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const int64_t s = sel[i];
    for (int a = 0; a < 3; ++a) {
        pos_out[3 * i + a] = pos[3 * s + a];
        if (nrm) nrm_out[3 * i + a] = nrm[3 * s + a];
    }
}

__global__ void k_not_degenerate(const int32_t* __restrict__ tri, int64_t nt, uint8_t* keep) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nt) return;
    const int32_t a = tri[3 * i], b = tri[3 * i + 1], c = tri[3 * i + 2];
    keep[i] = a != b && b != c && c != a;
}

// Open3D RemoveDuplicatedTriangles' canonical rotation (smallest index first, orientation kept)
__device__ inline void canon(const int32_t* t, uint32_t& k0, uint32_t& k1, uint32_t& k2) {
    const uint32_t a = (uint32_t)t[0], b = (uint32_t)t[1], c = (uint32_t)t[2];
    if (a <= b) {
        if (a <= c) k0 = a, k1 = b, k2 = c;
        else k0 = c, k1 = a, k2 = b;
    } else {
        if (b <= c) k0 = b, k1 = c, k2 = a;
        else k0 = c, k1 = a, k2 = b;
    }
}

__global__ void k_tri_key_lo(const int32_t* __restrict__ tri, int64_t nt, uint32_t* k2, int32_t* idx) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nt) return;
    uint32_t a, b, c;
    canon(tri + 3 * i, a, b, c);
    k2[i] = c;
    idx[i] = (int32_t)i;
}

__global__ void k_tri_key_hi(const int32_t* __restrict__ tri, const int32_t* __restrict__ idx, int64_t nt,
                             uint64_t* k01) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nt) return;
    uint32_t a, b, c;
    canon(tri + 3 * (int64_t)idx[i], a, b, c);
    k01[i] = (uint64_t)a << 32 | b;
}

__global__ void k_first_of_run_tri(const int32_t* __restrict__ tri, const int32_t* __restrict__ idx, int64_t nt,
                                   uint8_t* keep) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nt) return;
    uint32_t a, b, c;
    canon(tri + 3 * (int64_t)idx[i], a, b, c);
    bool first = i == 0;
    if (!first) {
        uint32_t pa, pb, pc;
        canon(tri + 3 * (int64_t)idx[i - 1], pa, pb, pc);
        first = a != pa || b != pb || c != pc;
    }
    keep[idx[i]] = first;
}

// vertex coordinate keys as double-equality classes: +0 and -0 equal, NaN never equal
__device__ inline uint32_t coord_bits(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x7fffffffu) == 0 ? 0u : u;
}
__device__ inline bool has_nan(const float* p) { return p[0] != p[0] || p[1] != p[1] || p[2] != p[2]; }

__global__ void k_vtx_key_lo(const float* __restrict__ pos, int64_t nv, uint32_t* kz, int32_t* idx) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nv) return;
    kz[i] = coord_bits(pos[3 * i + 2]);
    idx[i] = (int32_t)i;
}

__global__ void k_vtx_key_hi(const float* __restrict__ pos, const int32_t* __restrict__ idx, int64_t nv,
                             uint64_t* kxy) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nv) return;
    const float* p = pos + 3 * (int64_t)idx[i];
    kxy[i] = (uint64_t)coord_bits(p[0]) << 32 | coord_bits(p[1]);
}

// head[i] = i if sorted position i starts a run of equal coordinates, else 0 (max-scan -> run start)
__global__ void k_vtx_heads(const float* __restrict__ pos, const int32_t* __restrict__ idx, int64_t nv,
                            int32_t* head) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nv) return;
    const float* p = pos + 3 * (int64_t)idx[i];
    bool first = i == 0 || has_nan(p);
    if (!first) {
        const float* q = pos + 3 * (int64_t)idx[i - 1];
        first = has_nan(q) || coord_bits(p[0]) != coord_bits(q[0]) || coord_bits(p[1]) != coord_bits(q[1]) ||
                coord_bits(p[2]) != coord_bits(q[2]);
    }
    head[i] = first ? (int32_t)i : 0;
}

__global__ void k_vtx_rep(const int32_t* __restrict__ idx, const int32_t* __restrict__ start, int64_t nv,
                          int32_t* rep, int32_t* keepv) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nv) return;
    const int32_t v = idx[i], r = idx[start[i]];
    rep[v] = r;
    keepv[v] = r == v;
}

__global__ void k_vtx_map(const int32_t* __restrict__ rep, const int32_t* __restrict__ newidx, int64_t nv,
                          int32_t* map) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nv) map[i] = newidx[rep[i]];
}

// Open3D ComputeTriangleArea in float64: x = p0 - p1, y = p0 - p2, 0.5 * |x cross y|
__global__ void k_areas(const float* __restrict__ pos, const int32_t* __restrict__ tri, int64_t nt, double* area) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nt) return;
    const float* p0 = pos + 3 * (int64_t)tri[3 * i];
    const float* p1 = pos + 3 * (int64_t)tri[3 * i + 1];
    const float* p2 = pos + 3 * (int64_t)tri[3 * i + 2];
    const double x0 = (double)p0[0] - p1[0], x1 = (double)p0[1] - p1[1], x2 = (double)p0[2] - p1[2];
    const double y0 = (double)p0[0] - p2[0], y1 = (double)p0[1] - p2[1], y2 = (double)p0[2] - p2[2];
    const double c0 = x1 * y2 - x2 * y1, c1 = x2 * y0 - x0 * y2, c2 = x0 * y1 - x1 * y0;
    area[i] = 0.5 * sqrt((c0 * c0 + c1 * c1) + c2 * c2);
}

// sorted edge entries inside a run of more than two equal keys (the entries of non-manifold edges)
__global__ void k_nonmanifold_members(const uint64_t* __restrict__ keys, int64_t m, uint8_t* flag) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const uint64_t k = keys[i];
    const bool p1 = i >= 1 && keys[i - 1] == k, p2 = i >= 2 && keys[i - 2] == k;
    const bool n1 = i + 1 < m && keys[i + 1] == k, n2 = i + 2 < m && keys[i + 2] == k;
    flag[i] = (p1 && p2) || (p1 && n1) || (n1 && n2);
}

// key, triangle and area of each member entry (for the host's resolution pass)
__global__ void k_gather_members(const uint64_t* __restrict__ keys, const int32_t* __restrict__ slot,
                                 const double* __restrict__ area, const int32_t* __restrict__ mem, int64_t n,
                                 uint64_t* okey, int32_t* otri, double* oarea) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int32_t e = mem[i], t = slot[e] / 3;
    okey[i] = keys[e];
    otri[i] = t;
    oarea[i] = area[t];
}

__global__ void k_drop_tris(const int32_t* __restrict__ del, int64_t n, double* area) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) area[del[i]] = -1.0;
}

__global__ void k_keep_positive(const double* __restrict__ area, int64_t nt, uint8_t* keep) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nt) keep[i] = area[i] > 0;
}

__global__ void k_gather_f64(const double* __restrict__ a, const int32_t* __restrict__ sel, int64_t m, double* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < m) out[i] = a[sel[i]];
}

// ------------------------------------------------------------------ host helpers
inline unsigned nb(int64_t n) { return (unsigned)std::max<int64_t>((n + 255) / 256, 1); }

// Scratch: a bump arena over one grow-only device buffer cached per device (the ~40 buffers of a
// filter pass cost no hipMalloc / hipFree -- each hipFree synchronises the device, and the
// stream-ordered pool still spent ~66 us per hipFreeAsync); release() pops the top allocation.
// Requests past the arena fall back to hipMallocAsync.  One call owns the cached arena at a time
// (a concurrent call on another thread gets a private one).
struct Arena {
    char* base = nullptr;
    size_t cap = 0;
    bool busy = false;
    hipStream_t s = nullptr;  // cached with the arena: creating a stream costs ~2 ms
};
static std::mutex g_arena_mu;
static Arena g_arena[64];

struct Ctx {
    hipStream_t s = nullptr;
    int device = 0;
    Arena* ar = nullptr;
    Arena priv;
    size_t top = 0;
    std::vector<std::pair<size_t, size_t>> stack;  // (offset, size) of live arena allocations
    std::vector<void*> owned;                        // fallback allocations

    int open(int dev, size_t want) {
        device = dev;
        {
            std::lock_guard<std::mutex> lk(g_arena_mu);
            if (dev >= 0 && dev < 64 && !g_arena[dev].busy) {
                ar = &g_arena[dev];
                ar->busy = true;
            }
        }
        if (!ar) ar = &priv;
        if (!ar->s && hipStreamCreateWithFlags(&ar->s, hipStreamNonBlocking) != hipSuccess) return 1;
        s = ar->s;
        if (ar->cap < want) {
            if (ar->base) (void)hipFree(ar->base);
            ar->base = nullptr;
            ar->cap = 0;
            if (hipMalloc(&ar->base, want) != hipSuccess) return 1;
            ar->cap = want;
        }
        return 0;
    }
    template <class T>
    T* alloc(int64_t n) {
        const size_t bytes = (sizeof(T) * (size_t)std::max<int64_t>(n, 1) + 255) & ~(size_t)255;
        if (ar && top + bytes <= ar->cap) {
            stack.emplace_back(top, bytes);
            void* p = ar->base + top;
            top += bytes;
            return static_cast<T*>(p);
        }
        void* p = nullptr;
        if (hipMallocAsync(&p, bytes, s) != hipSuccess) return nullptr;
        owned.push_back(p);
        return static_cast<T*>(p);
    }
    void release(void* p) {
        if (ar && p >= (void*)ar->base && p < (void*)(ar->base + ar->cap)) {
            const size_t off = static_cast<char*>(p) - ar->base;
            for (size_t i = stack.size(); i-- > 0;)
                if (stack[i].first == off) {
                    stack.erase(stack.begin() + (std::ptrdiff_t)i);
                    break;
                }
            top = stack.empty() ? 0 : stack.back().first + stack.back().second;  // pops freed tops
            return;
        }
        auto it = std::find(owned.begin(), owned.end(), p);
        if (it != owned.end()) {
            (void)hipFreeAsync(p, s);
            owned.erase(it);
        }
    }
    ~Ctx() {
        if (!s) return;
        for (void* p : owned) (void)hipFreeAsync(p, s);
        (void)hipStreamSynchronize(s);
        if (ar == &priv) {
            if (priv.base) (void)hipFree(priv.base);
            (void)hipStreamDestroy(priv.s);
        } else if (ar) {
            std::lock_guard<std::mutex> lk(g_arena_mu);
            ar->busy = false;
        }
    }
};

#define MF_CHECK(expr)                                                           \
    do {                                                                         \
        hipError_t _e = (expr);                                                  \
        if (_e != hipSuccess) {                                                  \
            set_error(std::string(#expr) + ": " + hipGetErrorString(_e));        \
            return 1;                                                            \
        }                                                                        \
    } while (0)
#define MF_ALLOC(var, T, n)                                                      \
    T* var = c.alloc<T>(n);                                                      \
    if (!var) {                                                                  \
        set_error("mesh filter: device allocation failed");                      \
        return 1;                                                                \
    }

// order-preserving list of indices i in [0, n) with flag[i] != 0
template <class F>
static int select_flagged(Ctx& c, const F* flags, int64_t n, int32_t* out, int64_t* count) {
    hipcub::CountingInputIterator<int32_t> it(0);
    int32_t* d_num = c.alloc<int32_t>(1);
    size_t tb = 0;
    MF_CHECK(hipcub::DeviceSelect::Flagged(nullptr, tb, it, flags, out, d_num, (int)n, c.s));
    void* tmp = c.alloc<char>((int64_t)tb + 16);
    if (!d_num || !tmp) {
        set_error("mesh filter: device allocation failed");
        return 1;
    }
    MF_CHECK(hipcub::DeviceSelect::Flagged(tmp, tb, it, flags, out, d_num, (int)n, c.s));
    int32_t h = 0;
    MF_CHECK(hipMemcpyAsync(&h, d_num, sizeof(int32_t), hipMemcpyDeviceToHost, c.s));
    MF_CHECK(hipStreamSynchronize(c.s));
    c.release(tmp);
    c.release(d_num);
    *count = h;
    return 0;
}

static int exclusive_sum(Ctx& c, const int32_t* in, int32_t* out, int64_t n) {
    size_t tb = 0;
    MF_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, in, out, (int)n, c.s));
    void* tmp = c.alloc<char>((int64_t)tb + 16);
    if (!tmp) {
        set_error("mesh filter: device allocation failed");
        return 1;
    }
    MF_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp, tb, in, out, (int)n, c.s));
    c.release(tmp);  // stream-ordered reuse: later work on c.s runs after the scan
    return 0;
}

template <class K>
static int sort_pairs(Ctx& c, const K* kin, K* kout, const int32_t* vin, int32_t* vout, int64_t n, int bits) {
    size_t tb = 0;
    MF_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, tb, kin, kout, vin, vout, (int)n, 0, bits, c.s));
    void* tmp = c.alloc<char>((int64_t)tb + 16);
    if (!tmp) {
        set_error("mesh filter: device allocation failed");
        return 1;
    }
    MF_CHECK(hipcub::DeviceRadixSort::SortPairs(tmp, tb, kin, kout, vin, vout, (int)n, 0, bits, c.s));
    c.release(tmp);
    return 0;
}

// Mesh under edit: device arrays owned by the Ctx (replaced as steps compact them).
struct Mesh {
    float* pos = nullptr;
    float* nrm = nullptr;
    int32_t* tri = nullptr;
    int64_t nv = 0, nt = 0;
};

static int keep_triangles(Ctx& c, Mesh& m, const uint8_t* keep) {
    MF_ALLOC(sel, int32_t, m.nt);
    int64_t k = 0;
    if (select_flagged(c, keep, m.nt, sel, &k)) return 1;
    if (k == m.nt) {
        c.release(sel);
        return 0;
    }
    MF_ALLOC(tri2, int32_t, 3 * k);
    if (k) hipLaunchKernelGGL(k_gather_tris, dim3(nb(k)), dim3(256), 0, c.s, m.tri, sel, k, tri2);
    MF_CHECK(hipGetLastError());
    c.release(sel);
    c.release(m.tri);
    m.tri = tri2;
    m.nt = k;
    return 0;
}

// keep vertices with keepv != 0 (order kept); map[old] = new index for every old vertex
static int keep_vertices(Ctx& c, Mesh& m, const int32_t* keepv, const int32_t* map) {
    MF_ALLOC(sel, int32_t, m.nv);
    int64_t k = 0;
    if (select_flagged(c, keepv, m.nv, sel, &k)) return 1;
    if (m.nt) hipLaunchKernelGGL(k_remap, dim3(nb(3 * m.nt)), dim3(256), 0, c.s, m.tri, m.nt, map);
    MF_CHECK(hipGetLastError());
    if (k != m.nv) {
        MF_ALLOC(pos2, float, 3 * k);
        float* nrm2 = nullptr;
        if (m.nrm) {
            nrm2 = c.alloc<float>(3 * k);
            if (!nrm2) {
                set_error("mesh filter: device allocation failed");
                return 1;
            }
        }
        if (k) hipLaunchKernelGGL(k_gather_vertices, dim3(nb(k)), dim3(256), 0, c.s, m.pos, m.nrm, sel, k, pos2, nrm2);
        MF_CHECK(hipGetLastError());
        c.release(m.pos);
        if (m.nrm) c.release(m.nrm);
        m.pos = pos2;
        m.nrm = nrm2;
        m.nv = k;
    }
    c.release(sel);
    return 0;
}

static int remove_unreferenced_vertices(Ctx& c, Mesh& m) {
    MF_ALLOC(used, int32_t, m.nv);
    MF_ALLOC(newidx, int32_t, m.nv);
    MF_CHECK(hipMemsetAsync(used, 0, sizeof(int32_t) * m.nv, c.s));
    if (m.nt) hipLaunchKernelGGL(k_mark_vertices, dim3(nb(3 * m.nt)), dim3(256), 0, c.s, m.tri, m.nt, used);
    MF_CHECK(hipGetLastError());
    if (exclusive_sum(c, used, newidx, m.nv)) return 1;
    if (keep_vertices(c, m, used, newidx)) return 1;
    c.release(used);
    c.release(newidx);
    return 0;
}

static int remove_duplicated_triangles(Ctx& c, Mesh& m) {
    if (m.nt < 2) return 0;
    const int64_t n = m.nt;
    MF_ALLOC(k2, uint32_t, n);
    MF_ALLOC(k2s, uint32_t, n);
    MF_ALLOC(idx, int32_t, n);
    MF_ALLOC(idx1, int32_t, n);
    MF_ALLOC(k01, uint64_t, n);
    MF_ALLOC(k01s, uint64_t, n);
    MF_ALLOC(idx2, int32_t, n);
    MF_ALLOC(keep, uint8_t, n);
    hipLaunchKernelGGL(k_tri_key_lo, dim3(nb(n)), dim3(256), 0, c.s, m.tri, n, k2, idx);
    MF_CHECK(hipGetLastError());
    if (sort_pairs(c, k2, k2s, idx, idx1, n, 32)) return 1;
    hipLaunchKernelGGL(k_tri_key_hi, dim3(nb(n)), dim3(256), 0, c.s, m.tri, idx1, n, k01);
    MF_CHECK(hipGetLastError());
    if (sort_pairs(c, k01, k01s, idx1, idx2, n, 64)) return 1;
    hipLaunchKernelGGL(k_first_of_run_tri, dim3(nb(n)), dim3(256), 0, c.s, m.tri, idx2, n, keep);
    MF_CHECK(hipGetLastError());
    if (keep_triangles(c, m, keep)) return 1;
    for (void* p : {(void*)k2, (void*)k2s, (void*)idx, (void*)idx1, (void*)k01, (void*)k01s, (void*)idx2, (void*)keep})
        c.release(p);
    return 0;
}

struct MaxOp {
    __device__ __host__ int32_t operator()(int32_t a, int32_t b) const { return a > b ? a : b; }
};

static int remove_duplicated_vertices(Ctx& c, Mesh& m) {
    if (m.nv < 2) return 0;
    const int64_t n = m.nv;
    MF_ALLOC(kz, uint32_t, n);
    MF_ALLOC(kzs, uint32_t, n);
    MF_ALLOC(idx, int32_t, n);
    MF_ALLOC(idx1, int32_t, n);
    MF_ALLOC(kxy, uint64_t, n);
    MF_ALLOC(kxys, uint64_t, n);
    MF_ALLOC(idx2, int32_t, n);
    MF_ALLOC(head, int32_t, n);
    MF_ALLOC(start, int32_t, n);
    MF_ALLOC(rep, int32_t, n);
    MF_ALLOC(keepv, int32_t, n);
    MF_ALLOC(newidx, int32_t, n);
    MF_ALLOC(map, int32_t, n);
    hipLaunchKernelGGL(k_vtx_key_lo, dim3(nb(n)), dim3(256), 0, c.s, m.pos, n, kz, idx);
    MF_CHECK(hipGetLastError());
    if (sort_pairs(c, kz, kzs, idx, idx1, n, 32)) return 1;
    hipLaunchKernelGGL(k_vtx_key_hi, dim3(nb(n)), dim3(256), 0, c.s, m.pos, idx1, n, kxy);
    MF_CHECK(hipGetLastError());
    if (sort_pairs(c, kxy, kxys, idx1, idx2, n, 64)) return 1;
    hipLaunchKernelGGL(k_vtx_heads, dim3(nb(n)), dim3(256), 0, c.s, m.pos, idx2, n, head);
    MF_CHECK(hipGetLastError());
    {
        size_t tb = 0;
        MF_CHECK(hipcub::DeviceScan::InclusiveScan(nullptr, tb, head, start, MaxOp(), (int)n, c.s));
        void* tmp = c.alloc<char>((int64_t)tb + 16);
        if (!tmp) {
            set_error("mesh filter: device allocation failed");
            return 1;
        }
        MF_CHECK(hipcub::DeviceScan::InclusiveScan(tmp, tb, head, start, MaxOp(), (int)n, c.s));
        MF_CHECK(hipStreamSynchronize(c.s));
        c.release(tmp);
    }
    hipLaunchKernelGGL(k_vtx_rep, dim3(nb(n)), dim3(256), 0, c.s, idx2, start, n, rep, keepv);
    MF_CHECK(hipGetLastError());
    if (exclusive_sum(c, keepv, newidx, n)) return 1;
    hipLaunchKernelGGL(k_vtx_map, dim3(nb(n)), dim3(256), 0, c.s, rep, newidx, n, map);
    MF_CHECK(hipGetLastError());
    if (keep_vertices(c, m, keepv, map)) return 1;
    for (void* p : {(void*)kz, (void*)kzs, (void*)idx, (void*)idx1, (void*)kxy, (void*)kxys, (void*)idx2, (void*)head,
                    (void*)start, (void*)rep, (void*)keepv, (void*)newidx, (void*)map})
        c.release(p);
    return 0;
}

// RemoveNonManifoldEdges: edge map on the device; only the entries of non-manifold edges (key,
// triangle, area) go to the host, which resolves the edges in ascending key order with Open3D's
// rule and returns the dropped triangles; triangles with area <= 0 are dropped each round.
static int remove_non_manifold_edges(Ctx& c, Mesh& m, int64_t* removed) {
    *removed = 0;
    const int64_t nt0 = m.nt;
    for (int round = 0; round < 1000; ++round) {
        const int64_t n = m.nt;
        if (n == 0) break;
        MF_ALLOC(area, double, n);
        hipLaunchKernelGGL(k_areas, dim3(nb(n)), dim3(256), 0, c.s, m.pos, m.tri, n, area);
        MF_CHECK(hipGetLastError());
        const int64_t ne = 3 * n;
        MF_ALLOC(keys, uint64_t, ne);
        MF_ALLOC(keys_s, uint64_t, ne);
        MF_ALLOC(slot, int32_t, ne);
        MF_ALLOC(slot_s, int32_t, ne);
        MF_ALLOC(flag, uint8_t, ne);
        MF_ALLOC(mem, int32_t, ne);
        hipLaunchKernelGGL(k_edge_keys, dim3(nb(ne)), dim3(256), 0, c.s, m.tri, n, keys, slot);
        MF_CHECK(hipGetLastError());
        if (sort_pairs(c, keys, keys_s, slot, slot_s, ne, 64)) return 1;
        hipLaunchKernelGGL(k_nonmanifold_members, dim3(nb(ne)), dim3(256), 0, c.s, keys_s, ne, flag);
        MF_CHECK(hipGetLastError());
        int64_t nm = 0;
        if (select_flagged(c, flag, ne, mem, &nm)) return 1;
        const bool manifold = nm == 0;
        if (!manifold) {
            MF_ALLOC(mkey, uint64_t, nm);
            MF_ALLOC(mtri, int32_t, nm);
            MF_ALLOC(marea, double, nm);
            hipLaunchKernelGGL(k_gather_members, dim3(nb(nm)), dim3(256), 0, c.s, keys_s, slot_s, area, mem, nm, mkey,
                               mtri, marea);
            MF_CHECK(hipGetLastError());
            std::vector<uint64_t> hk(nm);
            std::vector<int32_t> ht(nm);
            std::vector<double> ha(nm);
            MF_CHECK(hipMemcpyAsync(hk.data(), mkey, sizeof(uint64_t) * nm, hipMemcpyDeviceToHost, c.s));
            MF_CHECK(hipMemcpyAsync(ht.data(), mtri, sizeof(int32_t) * nm, hipMemcpyDeviceToHost, c.s));
            MF_CHECK(hipMemcpyAsync(ha.data(), marea, sizeof(double) * nm, hipMemcpyDeviceToHost, c.s));
            MF_CHECK(hipStreamSynchronize(c.s));
            std::unordered_map<int32_t, double> cur;  // current area of every triangle involved
            cur.reserve((size_t)nm);
            for (int64_t j = 0; j < nm; ++j) cur.emplace(ht[j], ha[j]);
            std::vector<int32_t> del;
            for (int64_t s0 = 0; s0 < nm;) {  // runs in ascending edge-key order
                int64_t e = s0;
                while (e < nm && hk[e] == hk[s0]) ++e;
                int cnt = 0;
                for (int64_t j = s0; j < e; ++j) cnt += cur[ht[j]] > 0;
                for (int to_delete = cnt - 2; to_delete > 0; --to_delete) {
                    int32_t mt = -1;
                    double ma = std::numeric_limits<double>::max();
                    for (int64_t j = s0; j < e; ++j) {
                        const double a = cur[ht[j]];
                        if (a > 0 && a < ma) mt = ht[j], ma = a;
                    }
                    cur[mt] = -1;
                    del.push_back(mt);
                }
                s0 = e;
            }
            if (!del.empty()) {
                MF_ALLOC(ddel, int32_t, (int64_t)del.size());
                MF_CHECK(hipMemcpyAsync(ddel, del.data(), sizeof(int32_t) * del.size(), hipMemcpyHostToDevice, c.s));
                hipLaunchKernelGGL(k_drop_tris, dim3(nb((int64_t)del.size())), dim3(256), 0, c.s, ddel,
                                   (int64_t)del.size(), area);
                MF_CHECK(hipGetLastError());
                MF_CHECK(hipStreamSynchronize(c.s));  // `del` is pageable host memory
                c.release(ddel);
            }
            c.release(marea);
            c.release(mtri);
            c.release(mkey);
        }
        MF_ALLOC(keep, uint8_t, n);
        hipLaunchKernelGGL(k_keep_positive, dim3(nb(n)), dim3(256), 0, c.s, area, n, keep);
        MF_CHECK(hipGetLastError());
        if (keep_triangles(c, m, keep)) return 1;
        for (void* p : {(void*)area, (void*)keys, (void*)keys_s, (void*)slot, (void*)slot_s, (void*)flag, (void*)mem,
                        (void*)keep})
            c.release(p);
        if (manifold) break;
    }
    *removed = nt0 - m.nt;
    return 0;
}

}  // namespace mf
}  // namespace mqr

using namespace mqr;
using namespace mqr::mf;

extern "C" {

int mqr_mesh_filter_components(int device, const float* vertices, const float* normals, int64_t nv,
                               const int32_t* triangles, int64_t nt, int loc, int64_t min_triangle_count,
                               mqr_geom** out, int64_t* stats) {
    MQR_REQUIRE(out && stats && (nv == 0 || vertices) && (nt == 0 || triangles), "null argument");
    MQR_REQUIRE(nv >= 0 && nt >= 0 && nv < ((int64_t)1 << 31) && nt < ((int64_t)1 << 31) / 3, "mesh too large");
    MQR_CHECK_HIP(hipSetDevice(device));
    for (int i = 0; i < 8; ++i) stats[i] = 0;
    stats[0] = nt;
    Ctx c;
    // arena: ~110 B per triangle + ~90 B per vertex covers the largest stage (edge sort + keys)
    MQR_REQUIRE(c.open(device, (size_t)(128 * nt + 96 * nv) + ((size_t)32 << 20)) == 0,
                "mesh filter: device allocation failed");
    const hipMemcpyKind k = loc == MQR_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    if (loc == MQR_DEVICE && order_after_caller(device, c.s)) return 2;
    Mesh m;
    m.nv = nv;
    m.nt = nt;
    m.pos = c.alloc<float>(3 * nv);
    m.nrm = normals ? c.alloc<float>(3 * nv) : nullptr;
    m.tri = c.alloc<int32_t>(3 * nt);
    MQR_REQUIRE(m.pos && m.tri && (!normals || m.nrm), "mesh filter: device allocation failed");
    if (loc == MQR_DEVICE) {
        if (nv) MQR_CHECK_HIP(hipMemcpyAsync(m.pos, vertices, sizeof(float) * 3 * nv, k, c.s));
        if (nv && normals) MQR_CHECK_HIP(hipMemcpyAsync(m.nrm, normals, sizeof(float) * 3 * nv, k, c.s));
        if (nt) MQR_CHECK_HIP(hipMemcpyAsync(m.tri, triangles, sizeof(int32_t) * 3 * nt, k, c.s));
    } else if (copy_to_device(device, m.pos, vertices, sizeof(float) * 3 * nv, c.s) ||
               (normals && copy_to_device(device, m.nrm, normals, sizeof(float) * 3 * nv, c.s)) ||
               copy_to_device(device, m.tri, triangles, sizeof(int32_t) * 3 * nt, c.s)) {
        return 1;
    }
    if (nt > 0) {
        // ---- cluster_connected_triangles
        const int64_t ne = 3 * nt;
        int32_t* parent = c.alloc<int32_t>(nt);
        uint64_t* keys = c.alloc<uint64_t>(ne);
        uint64_t* keys_s = c.alloc<uint64_t>(ne);
        int32_t* slot = c.alloc<int32_t>(ne);
        int32_t* slot_s = c.alloc<int32_t>(ne);
        int32_t* count = c.alloc<int32_t>(nt);
        int32_t* is_root = c.alloc<int32_t>(nt);
        int32_t* cid = c.alloc<int32_t>(nt);
        MQR_REQUIRE(parent && keys && keys_s && slot && slot_s && count && is_root && cid,
                    "mesh filter: device allocation failed");
        hipLaunchKernelGGL(k_iota, dim3(nb(nt)), dim3(256), 0, c.s, parent, nt);
        hipLaunchKernelGGL(k_edge_keys, dim3(nb(ne)), dim3(256), 0, c.s, m.tri, nt, keys, slot);
        MQR_CHECK_HIP(hipGetLastError());
        if (sort_pairs(c, keys, keys_s, slot, slot_s, ne, 64)) return 1;
        hipLaunchKernelGGL(k_union_edges, dim3(nb(ne)), dim3(256), 0, c.s, keys_s, slot_s, ne, parent);
        MQR_CHECK_HIP(hipMemsetAsync(count, 0, sizeof(int32_t) * nt, c.s));
        hipLaunchKernelGGL(k_roots, dim3(nb(nt)), dim3(256), 0, c.s, parent, nt, count, is_root);
        int32_t* root = c.alloc<int32_t>(nt);
        MQR_REQUIRE(root, "mesh filter: device allocation failed");
        hipLaunchKernelGGL(k_final_root, dim3(nb(nt)), dim3(256), 0, c.s, parent, nt, root);
        MQR_CHECK_HIP(hipGetLastError());
        if (exclusive_sum(c, is_root, cid, nt)) return 1;
        int32_t last_root = 0, last_cid = 0;
        MQR_CHECK_HIP(hipMemcpyAsync(&last_root, is_root + nt - 1, sizeof(int32_t), hipMemcpyDeviceToHost, c.s));
        MQR_CHECK_HIP(hipMemcpyAsync(&last_cid, cid + nt - 1, sizeof(int32_t), hipMemcpyDeviceToHost, c.s));
        MQR_CHECK_HIP(hipStreamSynchronize(c.s));
        const int64_t C = (int64_t)last_root + last_cid;
        int32_t* ccount = c.alloc<int32_t>(C);
        MQR_REQUIRE(ccount, "mesh filter: device allocation failed");
        hipLaunchKernelGGL(k_cluster_table, dim3(nb(nt)), dim3(256), 0, c.s, is_root, cid, count, nt, ccount);
        MQR_CHECK_HIP(hipGetLastError());
        std::vector<int32_t> h_cc(C);
        MQR_CHECK_HIP(hipMemcpyAsync(h_cc.data(), ccount, sizeof(int32_t) * C, hipMemcpyDeviceToHost, c.s));
        MQR_CHECK_HIP(hipStreamSynchronize(c.s));
        // ---- keep clusters with >= min triangles (none: the first largest)
        std::vector<uint8_t> keepc(C, 0);
        int64_t kept = 0, largest = 0, kept_tris = 0;
        for (int64_t i = 0; i < C; ++i) {
            largest = std::max<int64_t>(largest, h_cc[i]);
            if (h_cc[i] >= min_triangle_count) keepc[i] = 1, ++kept, kept_tris += h_cc[i];
        }
        if (kept == 0) {
            const int64_t arg = std::max_element(h_cc.begin(), h_cc.end()) - h_cc.begin();
            keepc[arg] = 1;
            kept = 1;
            kept_tris = h_cc[arg];
        }
        stats[1] = C;
        stats[2] = kept;
        stats[3] = nt - kept_tris;
        stats[4] = largest;
        if (kept_tris < nt) {
            uint8_t* d_keepc = c.alloc<uint8_t>(C);
            uint8_t* keep = c.alloc<uint8_t>(nt);
            MQR_REQUIRE(d_keepc && keep, "mesh filter: device allocation failed");
            MQR_CHECK_HIP(hipMemcpyAsync(d_keepc, keepc.data(), C, hipMemcpyHostToDevice, c.s));
            hipLaunchKernelGGL(k_keep_by_cluster, dim3(nb(nt)), dim3(256), 0, c.s, root, cid, d_keepc, nt, keep);
            MQR_CHECK_HIP(hipGetLastError());
            if (keep_triangles(c, m, keep)) return 1;
            if (remove_unreferenced_vertices(c, m)) return 1;
            c.release(d_keepc);
            c.release(keep);
        }
        for (void* p : {(void*)parent, (void*)root, (void*)keys, (void*)keys_s, (void*)slot, (void*)slot_s,
                        (void*)count, (void*)is_root, (void*)cid, (void*)ccount})
            c.release(p);
        // ---- clean-up sequence of the reference
        if (m.nt) {
            uint8_t* keep = c.alloc<uint8_t>(m.nt);
            MQR_REQUIRE(keep, "mesh filter: device allocation failed");
            hipLaunchKernelGGL(k_not_degenerate, dim3(nb(m.nt)), dim3(256), 0, c.s, m.tri, m.nt, keep);
            MQR_CHECK_HIP(hipGetLastError());
            if (keep_triangles(c, m, keep)) return 1;
            c.release(keep);
        }
        if (remove_duplicated_triangles(c, m)) return 1;
        if (remove_duplicated_vertices(c, m)) return 1;
        int64_t nm_removed = 0;
        if (remove_non_manifold_edges(c, m, &nm_removed)) return 1;
        stats[5] = nm_removed;
    }
    stats[6] = m.nt;
    stats[7] = m.nv;
    // copy the result out of the scratch arena into one allocation owned by the geometry object
    mqr_geom* g = new mqr_geom();
    g->device = device;
    g->nv = m.nv;
    g->nt = m.nt;
    const size_t sv = (sizeof(float) * 3 * (size_t)std::max<int64_t>(m.nv, 1) + 255) & ~(size_t)255;
    const size_t stb = (sizeof(int32_t) * 3 * (size_t)std::max<int64_t>(m.nt, 1) + 255) & ~(size_t)255;
    g->blk = geom_block_alloc(device, 2 * sv + stb, &g->blk_cap);
    if (!g->blk) {
        delete g;
        set_error("mesh filter: device allocation failed");
        return 1;
    }
    g->pos = reinterpret_cast<float*>(g->blk);
    g->nrm = reinterpret_cast<float*>(static_cast<char*>(g->blk) + sv);
    g->tri = reinterpret_cast<int32_t*>(static_cast<char*>(g->blk) + 2 * sv);
    if (m.nv) MQR_CHECK_HIP(hipMemcpyAsync(g->pos, m.pos, sizeof(float) * 3 * m.nv, hipMemcpyDeviceToDevice, c.s));
    if (m.nv && m.nrm)
        MQR_CHECK_HIP(hipMemcpyAsync(g->nrm, m.nrm, sizeof(float) * 3 * m.nv, hipMemcpyDeviceToDevice, c.s));
    else
        MQR_CHECK_HIP(hipMemsetAsync(g->nrm, 0, sv, c.s));
    if (m.nt) MQR_CHECK_HIP(hipMemcpyAsync(g->tri, m.tri, sizeof(int32_t) * 3 * m.nt, hipMemcpyDeviceToDevice, c.s));
    MQR_CHECK_HIP(hipStreamSynchronize(c.s));
    *out = g;
    return 0;
}

}  // extern "C"
