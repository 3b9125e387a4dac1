// rtx_bvh.hip — the reference's BVH build on the GPU.
//
// NewBVHFromWorld (bvh.go:138-185) over a World of spheres: every NewBVH call draws
// axis = rand.Intn(3) from the global source (before its size switch), then a list of
// 1 is a leaf (left == right), a list of 2 is ordered by the axis comparator, and a
// longer list is sorted by it (descending box minimum, HittableCompare{X,Y,Z},
// bvh.go:187-218) and split at len/2.  The shape of that recursion depends only on
// the list sizes, so the pre-order index of every NewBVH call — which global-rand draw
// it makes — and the position of every node in the threaded pre-order layout
// (rtx_layout.h) are known before any sorting.  The build therefore runs level by
// level: all sorts of one recursion depth are one stable radix sort of the prims by
// (block, descending key), where the blocks partition the list into that depth's
// nodes and the leaves finished above it; box unions run bottom-up afterwards, and the
// entries are written straight into the device layout.
//
// Equivalences with the reference: the sort is stable (the host mirror's choice for
// x/exp/slices' unstable pdqsort) and b.min - a.min > 0 is exactly
// b.min > a.min for IEEE float32 (with subnormals the difference is zero only for
// equal values; -0 and +0 compare equal and are canonicalised before the radix sort).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <functional>
#include <map>
#include <vector>

#include "rtx_bvh.h"
#include "rtx_layout.h"

namespace rtxd {

namespace {

// ---- host: Philox4x32-10 word n of host stream `stream` ---------------
uint32_t host_stream_word(uint64_t seed, uint32_t stream, uint64_t n) {
    const uint64_t blk = n >> 2;
    uint32_t c[4] = {(uint32_t)blk, (uint32_t)(blk >> 32), 0u, 0x80000000u | stream};
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    for (int r = 0; r < 10; ++r) {
        if (r > 0) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
        c[1] = (uint32_t)p1;
        c[3] = (uint32_t)p0;
        c[0] = n0;
        c[2] = n2;
    }
    return c[n & 3u];
}

// One NewBVH call.
struct Node {
    uint32_t off, n;       // its slice of the (permuted) prim list
    uint32_t entry;        // position of its node entry in the threaded layout
    uint32_t esc;          // entry + entries of its subtree
    int32_t left, right;   // child nodes (n >= 3), else -1
    uint32_t depth;
    uint32_t axis;         // Intn(3)
};

// ---- device ---------------------------------------------------------------------------
__device__ __forceinline__ float go_min(float x, float y) {  // math.Min via float64 (math.go:38)
    if ((__builtin_isinf(x) && x < 0) || (__builtin_isinf(y) && y < 0)) return -__builtin_inff();
    if (x != x || y != y) return __builtin_nanf("");
    if (x == 0 && x == y) return __builtin_signbit(x) ? x : y;
    return x < y ? x : y;
}
__device__ __forceinline__ float go_max(float x, float y) {  // math.Max (math.go:42)
    if ((__builtin_isinf(x) && x > 0) || (__builtin_isinf(y) && y > 0)) return __builtin_inff();
    if (x != x || y != y) return __builtin_nanf("");
    if (x == 0 && x == y) return __builtin_signbit(x) ? y : x;
    return x > y ? x : y;
}

// NewSphere's box (hittables.go:85-94): NewAabb(center + (-r), center + r).
__global__ void prim_boxes(const rtx_sphere* __restrict__ sp, uint32_t n, float* __restrict__ bmin,
                           float* __restrict__ bmax) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float r = sp[i].radius, nr = r * -1.0f;
    for (int a = 0; a < 3; ++a) {
        const float p1 = sp[i].center[a] + nr, p2 = sp[i].center[a] + r;
        bmin[3 * i + a] = go_min(p1, p2);
        bmax[3 * i + a] = go_max(p1, p2);
    }
}

// Sort key of list position i: (block, descending box minimum along the block's axis).
__global__ void level_keys(uint32_t n, const uint32_t* __restrict__ perm, const float* __restrict__ bmin,
                           const uint32_t* __restrict__ block_off, const uint8_t* __restrict__ block_axis,
                           uint32_t n_blocks, unsigned long long* __restrict__ keys) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint32_t lo = 0, hi = n_blocks;  // last block with offset <= i
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) / 2;
        if (block_off[mid] <= i) lo = mid;
        else hi = mid;
    }
    const uint32_t ax = block_axis[lo];
    uint32_t k = 0;
    if (ax < 3) {
        const float v = bmin[3 * perm[i] + ax] + 0.0f;  // -0 -> +0 (they compare equal)
        uint32_t u = __float_as_uint(v);
        u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);  // ascending order of floats
        k = ~u;                                           // descending
    }
    keys[i] = ((unsigned long long)lo << 32) | k;
}

struct DevNode {
    uint32_t off, n, entry, esc;
    int32_t left, right;
};

// Boxes of one depth's nodes: NewAabbFromBoxes(left, right) (bvh.go:44-50, 182).
__global__ void node_boxes(const DevNode* __restrict__ nodes, const uint32_t* __restrict__ ids, uint32_t count,
                           const uint32_t* __restrict__ perm, const float* __restrict__ pmin,
                           const float* __restrict__ pmax, float* __restrict__ nmin, float* __restrict__ nmax) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    if (t >= count) return;
    const uint32_t id = ids[t];
    const DevNode nd = nodes[id];
    const float *lmin, *lmax, *rmin, *rmax;
    if (nd.n >= 3) {
        lmin = nmin + 3 * nd.left;
        lmax = nmax + 3 * nd.left;
        rmin = nmin + 3 * nd.right;
        rmax = nmax + 3 * nd.right;
    } else {
        const uint32_t a = perm[nd.off], b = perm[nd.off + nd.n - 1];  // n == 1: left == right
        lmin = pmin + 3 * a;
        lmax = pmax + 3 * a;
        rmin = pmin + 3 * b;
        rmax = pmax + 3 * b;
    }
    for (int k = 0; k < 3; ++k) {
        nmin[3 * id + k] = go_min(lmin[k], rmin[k]);
        nmax[3 * id + k] = go_max(lmax[k], rmax[k]);
    }
}

__device__ __forceinline__ void put_prim(rtx_entry* e, const rtx_sphere& s, uint32_t rank) {
    e->a[0] = s.center[0];
    e->a[1] = s.center[1];
    e->a[2] = s.center[2];
    e->a[3] = s.radius;
    e->b[0] = s.radius * s.radius;  // hittables.go:100
    e->b[1] = __int_as_float((int)rank);
    e->b[2] = 0.0f;
    e->b[3] = __int_as_float((int)s.material);
}

// The threaded pre-order entries (rtx_layout.h), as rtx_scene_create's emit() writes
// them for the same tree: a leaf of one prim is emitted once (left == right).
__global__ void emit_entries(const DevNode* __restrict__ nodes, uint32_t n_nodes, const uint32_t* __restrict__ perm,
                             const rtx_sphere* __restrict__ sp, const float* __restrict__ nmin,
                             const float* __restrict__ nmax, rtx_entry* __restrict__ out) {
    const uint32_t id = blockIdx.x * 256 + threadIdx.x;
    if (id >= n_nodes) return;
    const DevNode nd = nodes[id];
    rtx_entry e;
    e.a[0] = nmin[3 * id];
    e.a[1] = nmin[3 * id + 1];
    e.a[2] = nmin[3 * id + 2];
    e.a[3] = __int_as_float((int)nd.esc);
    e.b[0] = nmax[3 * id];
    e.b[1] = nmax[3 * id + 1];
    e.b[2] = nmax[3 * id + 2];
    e.b[3] = __int_as_float(RTX_E_NODE);
    out[nd.entry] = e;
    if (nd.n <= 2) {
        for (uint32_t k = 0; k < nd.n; ++k) {
            rtx_entry p;
            put_prim(&p, sp[perm[nd.off + k]], nd.off + k);
            out[nd.entry + 1 + k] = p;
        }
    }
}

}  // namespace

#define BVH_TRY(expr)                          \
    do {                                       \
        hipError_t e_ = (expr);                \
        if (e_ != hipSuccess) return fail(e_); \
    } while (0)

hipError_t build_sphere_bvh(const rtx_sphere* spheres, uint32_t n, uint64_t seed, uint64_t draw0,
                            std::vector<rtx_entry>& out, double* build_ms) {
    const auto t0 = std::chrono::steady_clock::now();
    // ---- the recursion's shape (sizes only): nodes in pre-order ------------------------
    std::map<uint32_t, uint64_t> calls_memo, entries_memo;
    std::function<uint64_t(uint32_t)> calls = [&](uint32_t m) -> uint64_t {  // NewBVH calls of a list of m
        if (m <= 2) return 1;
        auto it = calls_memo.find(m);
        if (it != calls_memo.end()) return it->second;
        const uint64_t v = 1 + calls(m / 2) + calls(m - m / 2);
        return calls_memo[m] = v;
    };
    std::function<uint64_t(uint32_t)> entries = [&](uint32_t m) -> uint64_t {  // threaded entries
        if (m <= 2) return 1 + m;
        auto it = entries_memo.find(m);
        if (it != entries_memo.end()) return it->second;
        const uint64_t v = 1 + entries(m / 2) + entries(m - m / 2);
        return entries_memo[m] = v;
    };
    std::vector<Node> nodes;
    nodes.reserve(n);
    struct Todo {
        uint32_t off, n, entry, depth;
        uint64_t draw;
        int32_t parent;
        int side;
    };
    std::vector<Todo> stack{{0, n, 0, 0, 0, -1, 0}};
    uint32_t max_depth = 0;
    while (!stack.empty()) {  // pre-order: a node, then its left subtree, then its right
        const Todo t = stack.back();
        stack.pop_back();
        const int32_t id = (int32_t)nodes.size();
        Node nd{t.off, t.n, t.entry, (uint32_t)(t.entry + entries(t.n)), -1, -1, t.depth, 0};
        nd.axis = (uint32_t)(((uint64_t)host_stream_word(seed, 1, draw0 + t.draw) * 3u) >> 32);  // Intn(3), :147
        nodes.push_back(nd);
        if (t.parent >= 0) (t.side == 0 ? nodes[t.parent].left : nodes[t.parent].right) = id;
        max_depth = std::max(max_depth, t.depth);
        if (t.n >= 3) {
            const uint32_t mid = t.n / 2;  // :178
            stack.push_back({t.off + mid, t.n - mid, (uint32_t)(t.entry + 1 + entries(mid)), t.depth + 1,
                             t.draw + 1 + calls(mid), id, 1});
            stack.push_back({t.off, mid, t.entry + 1, t.depth + 1, t.draw + 1, id, 0});
        }
    }
    const uint64_t n_entries = entries(n);
    // ---- device buffers ----------------------------------------------------------------
    rtx_sphere* d_sp = nullptr;
    float *d_pmin = nullptr, *d_pmax = nullptr, *d_nmin = nullptr, *d_nmax = nullptr;
    uint32_t *d_perm = nullptr, *d_perm2 = nullptr, *d_off = nullptr, *d_ids = nullptr;
    uint8_t* d_axis = nullptr;
    unsigned long long *d_keys = nullptr, *d_keys2 = nullptr;
    DevNode* d_nodes = nullptr;
    rtx_entry* d_out = nullptr;
    void* d_tmp = nullptr;
    auto release = [&]() {
        for (void* p : {(void*)d_sp, (void*)d_pmin, (void*)d_pmax, (void*)d_nmin, (void*)d_nmax, (void*)d_perm,
                        (void*)d_perm2, (void*)d_off, (void*)d_ids, (void*)d_axis, (void*)d_keys, (void*)d_keys2,
                        (void*)d_nodes, (void*)d_out, d_tmp})
            if (p) (void)hipFree(p);
    };
    auto fail = [&](hipError_t e) {
        release();
        return e;
    };
    const size_t N = n, M = nodes.size();
    BVH_TRY(hipMalloc(&d_sp, N * sizeof(rtx_sphere)));
    BVH_TRY(hipMalloc(&d_pmin, N * 12));
    BVH_TRY(hipMalloc(&d_pmax, N * 12));
    BVH_TRY(hipMalloc(&d_nmin, M * 12));
    BVH_TRY(hipMalloc(&d_nmax, M * 12));
    BVH_TRY(hipMalloc(&d_perm, N * 4));
    BVH_TRY(hipMalloc(&d_perm2, N * 4));
    BVH_TRY(hipMalloc(&d_off, (N + M + 1) * 4));
    BVH_TRY(hipMalloc(&d_ids, M * 4));
    BVH_TRY(hipMalloc(&d_axis, N + M + 1));
    BVH_TRY(hipMalloc(&d_keys, N * 8));
    BVH_TRY(hipMalloc(&d_keys2, N * 8));
    BVH_TRY(hipMalloc(&d_nodes, M * sizeof(DevNode)));
    BVH_TRY(hipMalloc(&d_out, n_entries * sizeof(rtx_entry)));
    size_t tmp_bytes = 0;
    BVH_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, d_keys, d_keys2, d_perm, d_perm2, (int)N));
    BVH_TRY(hipMalloc(&d_tmp, tmp_bytes));
    BVH_TRY(hipMemcpy(d_sp, spheres, N * sizeof(rtx_sphere), hipMemcpyHostToDevice));
    std::vector<uint32_t> iota(N);
    for (uint32_t i = 0; i < n; ++i) iota[i] = i;  // the World's order (:144-145 copies it)
    BVH_TRY(hipMemcpy(d_perm, iota.data(), N * 4, hipMemcpyHostToDevice));
    const uint32_t grid_n = (uint32_t)((N + 255) / 256);
    hipLaunchKernelGGL(prim_boxes, dim3(grid_n), dim3(256), 0, 0, d_sp, n, d_pmin, d_pmax);
    BVH_TRY(hipGetLastError());
    // ---- one stable sort per recursion depth -------------------------------------------
    std::vector<std::vector<uint32_t>> by_depth(max_depth + 1);
    for (uint32_t i = 0; i < M; ++i) by_depth[nodes[i].depth].push_back(i);
    std::vector<uint32_t> done_leaves;  // leaves of the depths above, as fixed blocks
    std::vector<uint32_t> boff;
    std::vector<uint8_t> bax;
    for (uint32_t d = 0; d <= max_depth; ++d) {
        std::vector<std::pair<uint32_t, uint8_t>> blocks;
        bool any = false;
        for (uint32_t id : by_depth[d]) {
            const Node& nd = nodes[id];
            const bool sorts = nd.n >= 2;  // n == 2 orders its pair (:166-174), n >= 3 sorts (:176)
            blocks.push_back({nd.off, (uint8_t)(sorts ? nd.axis : 3)});
            any |= sorts;
        }
        for (uint32_t id : done_leaves) blocks.push_back({nodes[id].off, (uint8_t)3});
        for (uint32_t id : by_depth[d])
            if (nodes[id].n <= 2) done_leaves.push_back(id);
        if (!any) continue;
        std::sort(blocks.begin(), blocks.end());
        boff.resize(blocks.size());
        bax.resize(blocks.size());
        for (size_t b = 0; b < blocks.size(); ++b) {
            boff[b] = blocks[b].first;
            bax[b] = blocks[b].second;
        }
        BVH_TRY(hipMemcpy(d_off, boff.data(), boff.size() * 4, hipMemcpyHostToDevice));
        BVH_TRY(hipMemcpy(d_axis, bax.data(), bax.size(), hipMemcpyHostToDevice));
        hipLaunchKernelGGL(level_keys, dim3(grid_n), dim3(256), 0, 0, n, d_perm, d_pmin, d_off, d_axis,
                           (uint32_t)blocks.size(), d_keys);
        BVH_TRY(hipGetLastError());
        int end_bit = 32;
        while ((1ull << (end_bit - 32)) < blocks.size()) ++end_bit;
        BVH_TRY(hipcub::DeviceRadixSort::SortPairs(d_tmp, tmp_bytes, d_keys, d_keys2, d_perm, d_perm2, (int)N, 0,
                                                   end_bit));
        std::swap(d_perm, d_perm2);
    }
    // ---- boxes bottom-up, then the entries ---------------------------------------------
    std::vector<DevNode> dn(M);
    for (size_t i = 0; i < M; ++i)
        dn[i] = DevNode{nodes[i].off, nodes[i].n, nodes[i].entry, nodes[i].esc, nodes[i].left, nodes[i].right};
    BVH_TRY(hipMemcpy(d_nodes, dn.data(), M * sizeof(DevNode), hipMemcpyHostToDevice));
    for (int d = (int)max_depth; d >= 0; --d) {
        const auto& ids = by_depth[d];
        if (ids.empty()) continue;
        BVH_TRY(hipMemcpy(d_ids, ids.data(), ids.size() * 4, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(node_boxes, dim3((uint32_t)((ids.size() + 255) / 256)), dim3(256), 0, 0, d_nodes, d_ids,
                           (uint32_t)ids.size(), d_perm, d_pmin, d_pmax, d_nmin, d_nmax);
        BVH_TRY(hipGetLastError());
    }
    hipLaunchKernelGGL(emit_entries, dim3((uint32_t)((M + 255) / 256)), dim3(256), 0, 0, d_nodes, (uint32_t)M, d_perm,
                       d_sp, d_nmin, d_nmax, d_out);
    BVH_TRY(hipGetLastError());
    out.resize(n_entries);
    BVH_TRY(hipMemcpy(out.data(), d_out, n_entries * sizeof(rtx_entry), hipMemcpyDeviceToHost));
    release();
    if (build_ms)
        *build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return hipSuccess;
}

}  // namespace rtxd
