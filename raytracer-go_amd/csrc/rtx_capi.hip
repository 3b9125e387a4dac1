// rtx_capi.hip — the C-ABI of librtx.so (include/rtx.h).
//
// Host-side half of the drop-in boundary: validates the flattened Hittable tree the
// caller hands over (what a cgo Render would pass), converts it once into the
// threaded pre-order device layout (rtx_layout.h), keeps it resident in HBM per
// device, and launches the megakernel.  Errors are returned as codes with a
// thread-local message; nothing throws across the ABI.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>  // types only: librccl is loaded on first use (rccl_api)

#include <algorithm>
#include <array>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/rtx.h"
#include "rtx_device.h"
#include "rtx_kernel.h"
#include "rtx_layout.h"
#include "rtx_ppm.h"
#include "rtx_bvh.h"
#include "rtx_collapse.h"
#include "rtx_topology.h"

namespace {

thread_local std::string g_last_error;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

#define HIP_TRY(expr)                                                                             \
    do {                                                                                          \
        hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess)                                                                     \
            return fail(e_ == hipErrorOutOfMemory ? RTX_ERR_OOM : RTX_ERR_HIP, "%s failed: %s (%s:%d)", \
                        #expr, hipGetErrorString(e_), __FILE__, __LINE__);                        \
    } while (0)

// One threaded layout of the walk on a device (rtx_layout.h): a scene keeping the caller's
// topology has one; a rebuilt one (rtx_topology.h) one per camera octant, uploaded on first use.
struct DeviceLayout {
    rtx_entry* entries = nullptr;
    uint32_t hot = 0;       // entries stored first and cached in LDS by v3 (scenes too big for the LDS copy)
    uint32_t start = 0;     // walk position of the first entry of the walk (the root)
    uint32_t prim_end = 0;  // scenes in the LDS copy: primitives stored first, below this position
    uint32_t n_entries = 0; // device entries before the sentinel (the paired walk's: twice its records)
    uint32_t w2 = 0;        // 1: the paired walk's records (build_w2)
};

struct DeviceCopy {
    int device = -1;
    DeviceLayout lay[16];  // [0, 8): the walk of each camera octant; [8, 16): the near walks of a tiered scene
    rtx_material* materials = nullptr;
    rtx_texture* textures = nullptr;
    uint32_t* texels = nullptr;
    unsigned long long* counters = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    uint32_t n_textures = 0;  // device textures: those materials read (checkered, image, noise)
    uint32_t placement = 0;   // the last enqueued render's rtxd::scene_placement
};

// Sample-colour scratch, one per device, shared by all scenes (grown on demand).  `last`
// marks its latest use, so a render on another stream waits for the previous one before
// reusing it — which also serialises every render on a device on the GPU (the per-scene
// counters and unit queue rely on that).  `scenes` counts the scene copies on the
// device: the last rtx_scene_destroy there frees the scratch (rtx_release_device_memory
// frees it at any time).
struct Scratch {
    float* ptr = nullptr;
    size_t bytes = 0;
    float4* defer = nullptr;  // the tiered walk's queue of deferred paths (64 B per record)
    size_t defer_bytes = 0;
    uint32_t* drain = nullptr;  // the near pass's drain: a record count and a unit cursor per workgroup (Params::drain_count)
    uint32_t* redo = nullptr;  // the tiered walk's redo bits: one per sample of a chunk
    size_t redo_bytes = 0;
    size_t redo_zero = 0;      // bytes at the start of `redo` known to be zero (reduce_samples keeps them so)
    hipEvent_t last = nullptr;
    int scenes = 0;
};
std::mutex g_scratch_mu;
std::map<int, Scratch> g_scratch;

// The PPM encoder's per-device scratch (line lengths and offsets), reused across calls;
// g_ppm_mu is held for a whole (blocking) encode.
struct PpmScratch {
    void* ptr = nullptr;
    size_t bytes = 0;
};
std::mutex g_ppm_mu;
std::map<int, PpmScratch> g_ppm;

// Two pinned host stages for copies into the caller's (pageable) buffer, allocated on first
// use and freed by rtx_release_device_memory(-1): the DMA of chunk k+1 runs while the CPU copies
// chunk k out.  (hipMemcpy into pageable memory stages through the runtime's own buffers: the
// 24.9 MB image of C2 cost ~7 ms that way.)
struct HostStage {
    void* buf[2] = {nullptr, nullptr};
    hipEvent_t ev[2] = {nullptr, nullptr};
};
constexpr size_t kStageBytes = 4u << 20;
std::mutex g_stage_mu;
HostStage g_stage;

hipError_t copy_to_host(void* dst, const void* src, size_t bytes, hipStream_t st) {
    std::lock_guard<std::mutex> lk(g_stage_mu);
    hipError_t e = hipSuccess;
    for (int i = 0; i < 2 && e == hipSuccess; ++i) {
        if (!g_stage.buf[i]) e = hipHostMalloc(&g_stage.buf[i], kStageBytes, hipHostMallocDefault);
        if (e == hipSuccess && !g_stage.ev[i]) e = hipEventCreateWithFlags(&g_stage.ev[i], hipEventDisableTiming);
    }
    const size_t n = (bytes + kStageBytes - 1) / kStageBytes;
    auto len = [&](size_t k) { return std::min(kStageBytes, bytes - k * kStageBytes); };
    for (size_t k = 0; k <= n && e == hipSuccess; ++k) {
        if (k < n) {  // chunk k into stage k % 2 (its previous chunk, k - 2, is already copied out)
            e = hipMemcpyAsync(g_stage.buf[k % 2], static_cast<const char*>(src) + k * kStageBytes, len(k),
                               hipMemcpyDeviceToHost, st);
            if (e == hipSuccess) e = hipEventRecord(g_stage.ev[k % 2], st);
        }
        if (k >= 1 && e == hipSuccess) {  // chunk k - 1 out of its stage while chunk k is in flight
            e = hipEventSynchronize(g_stage.ev[(k - 1) % 2]);
            if (e == hipSuccess)
                std::memcpy(static_cast<char*>(dst) + (k - 1) * kStageBytes, g_stage.buf[(k - 1) % 2], len(k - 1));
        }
    }
    // on a failure no copy into a stage may still be in flight when the lock is released
    if (e != hipSuccess) (void)hipStreamSynchronize(st);
    return e;
}

void release_stage_locked() {
    for (int i = 0; i < 2; ++i) {
        if (g_stage.ev[i]) (void)hipEventDestroy(g_stage.ev[i]);
        if (g_stage.buf[i]) (void)hipHostFree(g_stage.buf[i]);
    }
    g_stage = HostStage{};
}

// The sticky error word of a device: rtxd::KERR_WORDS counters the kernels only add to — waves
// stopped by the watchdog, lanes of waves that found a partial wave at a claim.  No render zeroes them (the stats
// slots are zeroed by every render, so a flag there was wiped by the next render enqueued behind a failed one):
// `seen` is what the host has already reported, and a change since is the error of some render after that report.
// collect_on (every render that returns stats) and rtx_device_check (any number of renders enqueued without
// stats, e.g. a pipelined benchmark) read it.  8 bytes per device, kept for the process's life.
struct KernErr {
    uint32_t* d = nullptr;
    uint32_t seen[rtxd::KERR_WORDS] = {0, 0};
};
std::mutex g_kerr_mu;
std::map<int, KernErr> g_kerr;

// The device's word (allocated and zeroed on first use, synchronously), or nullptr.
uint32_t* kerr_word(int device) {
    std::lock_guard<std::mutex> lk(g_kerr_mu);
    KernErr& k = g_kerr[device];
    if (!k.d) {
        void* p = nullptr;
        if (hipMalloc(&p, rtxd::KERR_WORDS * sizeof(uint32_t)) != hipSuccess) return nullptr;
        if (hipMemset(p, 0, rtxd::KERR_WORDS * sizeof(uint32_t)) != hipSuccess) {
            (void)hipFree(p);
            return nullptr;
        }
        k.d = static_cast<uint32_t*>(p);
    }
    return k.d;
}

// Read the current device's word (the renders to report must have completed) and report what changed since the
// last read: RTX_OK, or RTX_ERR_HIP naming the failure.  The change is then acknowledged.
int kerr_take(int device) {
    std::lock_guard<std::mutex> lk(g_kerr_mu);
    auto it = g_kerr.find(device);
    if (it == g_kerr.end() || !it->second.d) return RTX_OK;  // nothing ever rendered on it
    KernErr& k = it->second;
    uint32_t h[rtxd::KERR_WORDS] = {0, 0};
    HIP_TRY(hipMemcpy(h, k.d, sizeof(h), hipMemcpyDeviceToHost));
    const uint32_t wd = h[rtxd::KERR_WATCHDOG] - k.seen[rtxd::KERR_WATCHDOG];
    const uint32_t pw = h[rtxd::KERR_PARTIAL_WAVE] - k.seen[rtxd::KERR_PARTIAL_WAVE];
    std::memcpy(k.seen, h, sizeof(h));
    if (pw)
        return fail(RTX_ERR_HIP, "render kernel: a wave-level claim was reached without the whole wave (partial EXEC; "
                                 "%u lanes on device %d): output invalid", pw, device);
    if (wd)
        return fail(RTX_ERR_HIP, "render kernel watchdog fired (RTX_WATCHDOG_S; %u waves on device %d): output "
                                 "incomplete", wd, device);
    return RTX_OK;
}

// Free a device's scratch buffers (g_scratch_mu held).
void release_scratch_locked(int device) {
    auto it = g_scratch.find(device);
    if (it == g_scratch.end()) return;
    Scratch& sc = it->second;
    int cur = 0;
    (void)hipGetDevice(&cur);
    if (hipSetDevice(device) == hipSuccess) {
        if (sc.last) (void)hipEventSynchronize(sc.last);
        if (sc.ptr) (void)hipFree(sc.ptr);
        if (sc.defer) (void)hipFree(sc.defer);
        if (sc.redo) (void)hipFree(sc.redo);
        if (sc.drain) (void)hipFree(sc.drain);
        if (sc.last) (void)hipEventDestroy(sc.last);
    }
    (void)hipSetDevice(cur);
    const int scenes = sc.scenes;
    sc = Scratch{};
    sc.scenes = scenes;
}

// ---- RCCL, loaded on first use (rtx_render with n_gpus > 1) --------------------------
struct RcclApi {
    bool tried = false, ok = false;
    std::string err;
    ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    ncclResult_t (*Gather)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    const char* (*GetErrorString)(ncclResult_t) = nullptr;
};
std::mutex g_rccl_mu;
RcclApi g_rccl;
std::map<int, std::vector<ncclComm_t>> g_comms;  // devices 0..n-1 -> communicators (ncclCommInitAll)

const RcclApi* rccl_api() {  // g_rccl_mu held
    if (g_rccl.tried) return g_rccl.ok ? &g_rccl : nullptr;
    g_rccl.tried = true;
    void* h = nullptr;
    for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
        if ((h = dlopen(name, RTLD_NOW | RTLD_GLOBAL))) break;
    if (!h) {
        g_rccl.err = std::string("cannot load librccl: ") + dlerror();
        return nullptr;
    }
    bool ok = true;
    auto sym = [&](auto& fn, const char* name) {
        fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
        ok = ok && fn != nullptr;
    };
    sym(g_rccl.CommInitAll, "ncclCommInitAll");
    sym(g_rccl.CommDestroy, "ncclCommDestroy");
    sym(g_rccl.GroupStart, "ncclGroupStart");
    sym(g_rccl.GroupEnd, "ncclGroupEnd");
    sym(g_rccl.Gather, "ncclGather");
    sym(g_rccl.GetErrorString, "ncclGetErrorString");
    if (!ok) g_rccl.err = "librccl lacks ncclGather / ncclCommInitAll";
    g_rccl.ok = ok;
    return ok ? &g_rccl : nullptr;
}

void release_comms_locked() {  // g_rccl_mu held
    for (auto& kv : g_comms)
        for (ncclComm_t c : kv.second)
            if (c && g_rccl.CommDestroy) (void)g_rccl.CommDestroy(c);
    g_comms.clear();
}

// rtx_render's per-device buffers (bands, the gathered bands, the assembled image), stream and
// gather events, kept between calls and freed by rtx_release_device_memory; g_render_mu is held
// for a whole rtx_render.  Keyed by (device, slot): slot d >= 0 is band d, -1 the gather, -2 the
// image.
struct RenderBuf {
    void* ptr = nullptr;
    size_t bytes = 0;
};
std::mutex g_render_mu;
std::map<std::pair<int, int>, RenderBuf> g_render_bufs;
std::map<int, hipStream_t> g_render_streams;
std::map<std::pair<int, int>, hipEvent_t> g_render_events;

void* render_buffer(int device, int slot, size_t bytes) {  // current device = device
    RenderBuf& b = g_render_bufs[{device, slot}];
    if (b.bytes < bytes) {
        if (b.ptr) (void)hipFree(b.ptr);
        b = RenderBuf{};
        if (hipMalloc(&b.ptr, bytes) != hipSuccess) return b.ptr = nullptr;
        b.bytes = bytes;
    }
    return b.ptr;
}
hipStream_t render_stream(int device) {  // current device = device
    hipStream_t& st = g_render_streams[device];
    if (!st && hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) st = nullptr;
    return st;
}
hipEvent_t render_event(int device, int k) {  // current device = device
    hipEvent_t& ev = g_render_events[{device, k}];
    if (!ev && hipEventCreate(&ev) != hipSuccess) ev = nullptr;
    return ev;
}
void release_render_locked(int device) {  // g_render_mu held; device -1: all
    int cur = 0;
    (void)hipGetDevice(&cur);
    for (auto it = g_render_bufs.begin(); it != g_render_bufs.end();) {
        if ((device < 0 || it->first.first == device) && hipSetDevice(it->first.first) == hipSuccess) {
            (void)hipDeviceSynchronize();
            if (it->second.ptr) (void)hipFree(it->second.ptr);
            it = g_render_bufs.erase(it);
        } else {
            ++it;
        }
    }
    for (auto it = g_render_streams.begin(); it != g_render_streams.end();) {
        if ((device < 0 || it->first == device) && hipSetDevice(it->first) == hipSuccess) {
            if (it->second) (void)hipStreamDestroy(it->second);
            it = g_render_streams.erase(it);
        } else {
            ++it;
        }
    }
    for (auto it = g_render_events.begin(); it != g_render_events.end();) {
        if ((device < 0 || it->first.first == device) && hipSetDevice(it->first.first) == hipSuccess) {
            if (it->second) (void)hipEventDestroy(it->second);
            it = g_render_events.erase(it);
        } else {
            ++it;
        }
    }
    (void)hipSetDevice(cur);
}

}  // namespace

struct rtx_scene {
    // The caller's tree as threaded entries in the reference's visit order (bvh.go:220-249).
    std::vector<rtx_entry> base;
    // The walk as threaded entries: layouts[0] for a scene that keeps the caller's topology; a
    // rebuilt scene (topo) has one per camera octant.  Each is planned on first use, for the
    // camera of that render: the tree's entries less the box tests the collapsed walk leaves
    // out (rtx_collapse.h; skips[k]: per node entry of the uncollapsed walk, 1 = left out).
    // Slots [8, 16) hold the near walks of a tiered scene (near_topo).
    std::vector<rtx_entry> layouts[16];
    std::vector<uint8_t> skips[16];
    std::vector<double> reads[16];  // estimated reads per entry of layouts[k] (the hot set of a big scene)
    bool planned[16] = {};
    bool rebuilt = false;
    bool tiered = false;     // near_topo built: renders whose camera lies in its near region walk in two tiers
    rtxd::Topology near_topo;
    std::vector<uint32_t> sphere_rank;  // each sphere's place in the reference walk (base): the tie rule
    bool every_box = false;  // RTX_SCENE_EVERY_BOX: no box test left out
    rtxd::Topology topo;
    std::vector<float> quadtab;  // 16 floats per quad (rtx_layout.h)
    std::vector<rtx_material> materials;
    std::vector<rtx_texture> textures;
    std::vector<uint32_t> texels;
    std::map<int, DeviceCopy> copies;
    bool has_image = false;  // some texture is an ImageTexture: hits need UV
    bool has_noise = false;  // some texture is a Perlin NoiseTexture
    std::mutex mu;
};

namespace {

int check_ref(const rtx_scene_desc* d, int32_t ref) {
    if (ref >= 0) {
        if ((uint32_t)ref >= d->n_nodes) return fail(RTX_ERR_INVALID_ARG, "node ref %d out of range (%u nodes)", ref, d->n_nodes);
        return RTX_OK;
    }
    const uint32_t p = (uint32_t)(~ref);
    const uint32_t type = p >> 28, idx = p & 0x0FFFFFFFu;
    if (type == RTX_PRIM_SPHERE) {
        if (idx >= d->n_spheres) return fail(RTX_ERR_INVALID_ARG, "sphere ref %u out of range (%u spheres)", idx, d->n_spheres);
        return RTX_OK;
    }
    if (type == RTX_PRIM_QUAD) {
        if (idx >= d->n_quads) return fail(RTX_ERR_INVALID_ARG, "quad ref %u out of range (%u quads)", idx, d->n_quads);
        return RTX_OK;
    }
    if (type == RTX_PRIM_LIST) {  // a nested World (ABI 5)
        if (idx >= d->n_lists || !d->lists) return fail(RTX_ERR_INVALID_ARG, "list ref %u out of range (%u lists)", idx, d->n_lists);
        const rtx_list& l = d->lists[idx];
        // (an empty World is a well-defined miss, hittables.go:55-72: it emits no entries)
        if (l.count && (!d->list_refs || (uint64_t)l.first + l.count > d->n_list_refs))
            return fail(RTX_ERR_INVALID_ARG, "list %u items out of range (%u list refs)", idx, d->n_list_refs);
        return RTX_OK;
    }
    return fail(RTX_ERR_INVALID_ARG, "unknown primitive type %u", type);
}

// Graph vertex of a ref for check_acyclic: nodes 0..n_nodes-1, lists after them; -1 for a leaf.
int64_t vertex_of(const rtx_scene_desc* d, int32_t ref) {
    if (ref >= 0) return ref;
    const uint32_t p = (uint32_t)(~ref);
    return (p >> 28) == RTX_PRIM_LIST ? (int64_t)d->n_nodes + (p & 0x0FFFFFFFu) : -1;
}

// Reject a node / list graph with a cycle (a Go BVH cannot have one, a hand-built table can).
int check_acyclic(const rtx_scene_desc* d) {
    std::vector<uint8_t> state((size_t)d->n_nodes + d->n_lists, 0);  // 0 new, 1 on path, 2 done
    struct F { int64_t v; uint32_t child; };
    auto n_children = [&](int64_t v) -> uint32_t {
        return v < (int64_t)d->n_nodes ? 2u : d->lists[v - d->n_nodes].count;
    };
    auto child = [&](int64_t v, uint32_t k) -> int32_t {
        if (v < (int64_t)d->n_nodes) return k == 0 ? d->nodes[v].left : d->nodes[v].right;
        const rtx_list& l = d->lists[v - d->n_nodes];
        return d->list_refs[l.first + k];
    };
    for (uint32_t r = 0; r < d->n_roots; ++r) {
        if (int rc = check_ref(d, d->roots[r])) return rc;
        const int64_t v0 = vertex_of(d, d->roots[r]);
        if (v0 < 0 || state[v0] == 2) continue;
        std::vector<F> st{{v0, 0}};
        state[v0] = 1;
        while (!st.empty()) {
            F& f = st.back();
            if (f.child == n_children(f.v)) { state[f.v] = 2; st.pop_back(); continue; }
            const int32_t ref = child(f.v, f.child++);
            if (int rc = check_ref(d, ref)) return rc;
            const int64_t v = vertex_of(d, ref);
            if (v < 0 || state[v] == 2) continue;
            if (state[v] == 1) return fail(RTX_ERR_INVALID_ARG, "BVH node / list graph has a cycle through ref %d", ref);
            state[v] = 1;
            st.push_back({v, 0});
        }
    }
    return RTX_OK;
}

// Emit the reference's visit order (bvh.go:220-249) as threaded pre-order entries.
int emit(const rtx_scene_desc* d, int32_t root, std::vector<rtx_entry>& out) {
    struct Frame {
        int32_t ref;
        int64_t node_entry;  // >= 0: close this node's escape when popped
    };
    std::vector<Frame> stack;
    stack.push_back({root, -1});
    const size_t limit = (size_t)1 << 26;  // 2 GiB of entries
    while (!stack.empty()) {
        Frame f = stack.back();
        stack.pop_back();
        if (f.node_entry >= 0) {  // subtree finished
            const int32_t esc = (int32_t)out.size();
            std::memcpy(&out[(size_t)f.node_entry].a[3], &esc, 4);
            continue;
        }
        if (int rc = check_ref(d, f.ref)) return rc;
        if (out.size() >= limit) return fail(RTX_ERR_INVALID_ARG, "BVH expands to more than %zu entries", limit);
        rtx_entry e;
        std::memset(&e, 0, sizeof(e));
        if (f.ref < 0 && (((uint32_t)(~f.ref)) >> 28) == RTX_PRIM_LIST) {
            // a nested World (hittables.go:55-72): its items one after another, each against the
            // running bound — the walk simply continues into the next item's entries
            const rtx_list& l = d->lists[((uint32_t)(~f.ref)) & 0x0FFFFFFFu];
            for (uint32_t k = l.count; k-- > 0;) stack.push_back({d->list_refs[l.first + k], -1});
        } else if (f.ref >= 0) {
            const rtx_bvh_node& n = d->nodes[f.ref];
            e.a[0] = n.bmin[0]; e.a[1] = n.bmin[1]; e.a[2] = n.bmin[2];
            e.b[0] = n.bmax[0]; e.b[1] = n.bmax[1]; e.b[2] = n.bmax[2];
            const int32_t tag = RTX_E_NODE;
            std::memcpy(&e.b[3], &tag, 4);
            const int64_t me = (int64_t)out.size();
            out.push_back(e);
            // visit order: left, then right (skipped when left == right, see rtx_layout.h)
            stack.push_back({0, me});
            if (n.right != n.left) stack.push_back({n.right, -1});
            stack.push_back({n.left, -1});
        } else if ((((uint32_t)(~f.ref)) >> 28) == RTX_PRIM_QUAD) {  // (normal, D | quad, tag)
            const uint32_t idx = ((uint32_t)(~f.ref)) & 0x0FFFFFFFu;
            const rtx_quad& q = d->quads[idx];
            e.a[0] = q.normal[0]; e.a[1] = q.normal[1]; e.a[2] = q.normal[2]; e.a[3] = q.d;
            const int32_t qi = (int32_t)idx, tag = RTX_E_QUAD;
            std::memcpy(&e.b[0], &qi, 4);
            std::memcpy(&e.b[3], &tag, 4);
            out.push_back(e);
        } else {
            const uint32_t idx = ((uint32_t)(~f.ref)) & 0x0FFFFFFFu;
            const rtx_sphere& s = d->spheres[idx];
            e.a[0] = s.center[0]; e.a[1] = s.center[1]; e.a[2] = s.center[2]; e.a[3] = s.radius;
            e.b[0] = s.radius * s.radius;  // hittables.go:100
            const int32_t si = (int32_t)idx, mi = (int32_t)s.material;
            std::memcpy(&e.b[1], &si, 4);
            std::memcpy(&e.b[3], &mi, 4);
            out.push_back(e);
        }
    }
    return RTX_OK;
}

uint32_t env_knob(const char* name, long dflt, long lo, long hi);

void free_copy(DeviceCopy& c);

int upload_copy(rtx_scene* s, DeviceCopy& c);

// The scene's copy on `device` (materials, textures, texels, counters), uploaded on first
// use; a failed upload frees what it had allocated.  Every copy is counted in the device's
// Scratch::scenes.  Walk layouts are uploaded separately (ensure_layout).
int ensure_device(rtx_scene* s, int device, DeviceCopy** out) {
    auto it = s->copies.find(device);
    if (it != s->copies.end()) {
        *out = &it->second;
        return RTX_OK;
    }
    DeviceCopy c;
    c.device = device;
    HIP_TRY(hipSetDevice(device));
    if (int rc = upload_copy(s, c)) {
        free_copy(c);
        return rc;
    }
    {
        std::lock_guard<std::mutex> lk(g_scratch_mu);
        ++g_scratch[device].scenes;
    }
    auto res = s->copies.emplace(device, c);
    *out = &res.first->second;
    return RTX_OK;
}

// Whether walks leave box tests out (rtx_collapse.h): RTX_COLLAPSE=0 in the environment (read
// per plan) or the scene flag RTX_SCENE_EVERY_BOX keep every test.
bool collapse_enabled(bool every_box) {
    if (every_box) return false;
    const char* e = std::getenv("RTX_COLLAPSE");
    return !(e && std::strcmp(e, "0") == 0);
}

// The walk of one tree for one camera: `base` (the caller's tree) or `topo` oriented for octant
// `oct`, less the box tests the collapsed walk leaves out for paths from `cam`.
void plan_walk(const std::vector<rtx_entry>& base, const rtxd::Topology* topo, uint32_t oct,
               const std::vector<float>& quadtab, const rtx_camera& cam, bool collapse, std::vector<rtx_entry>& out,
               std::vector<uint8_t>& skip, std::vector<double>* reads) {
    std::vector<rtx_entry> full;
    if (topo) rtxd::emit_topology(*topo, oct, full);
    const std::vector<rtx_entry>& E = topo ? full : base;
    std::vector<double> pass;
    double walks = 0.0;
    rtxd::sample_node_passes(E, quadtab, cam, pass, &walks);
    rtxd::collapse_layout(E, pass, walks, collapse, out, skip, reads);
}

// Layout slot of a camera: its octant for a rebuilt scene, else 0; near walks of a tiered scene
// at 8 + octant.
uint32_t layout_slot(const rtx_scene* s, const rtx_camera* cam, bool near = false) {
    return near ? 8u + rtxd::camera_octant(*cam) : (s->rebuilt ? rtxd::camera_octant(*cam) : 0u);
}

// The walk for `cam` as threaded entries (s->mu held), planned on the slot's first use.
int scene_layout(rtx_scene* s, const rtx_camera* cam, const std::vector<rtx_entry>** out, bool near = false) {
    const uint32_t k = layout_slot(s, cam, near);
    if (near && !s->tiered) return fail(RTX_ERR_INVALID_ARG, "scene has no near walk");
    if (!s->planned[k]) {
        const rtxd::Topology* t = near ? &s->near_topo : (s->rebuilt ? &s->topo : nullptr);
        plan_walk(s->base, t, k & 7u, s->quadtab, *cam, collapse_enabled(s->every_box), s->layouts[k], s->skips[k],
                  &s->reads[k]);
        s->planned[k] = true;
    }
    *out = &s->layouts[k];
    return RTX_OK;
}

// The paired walk of a layout in HBM: the threaded walk E (host form, escapes as entry indices)
// as RECORDS of two entries — an entry p and the entry the walk takes after p when p does not descend (a node's
// escape, a primitive's successor: its fail successor q(p)).  A lane at a record tests p; if p is a node whose box
// passes it goes to the record of p + 1, else it tests q(p) in the same step and goes to the record of q(p) + 1
// (q(p) a passing node) or of q(q(p)).  So the lane takes exactly the threaded walk's tests, in its order, with its
// bounds — every result and every work counter is the walk's — in up to half the dependent reads: a record holds a
// node's two children (the left child's fail successor is its sibling), so a box that fails costs no read of its
// own.  The slots are entries in the device format (rtx_layout.h) with their successors as record positions: slot 0
// a node's next (b.w) only, slot 1 its escape too (a.w) or a primitive's next (b.z); the sentinel as slot 1 where the
// walk ends.  A record starts at every entry the walk can arrive at (the root, a node's first child, q(q(p)) of a
// record): at most one per entry.  The records the walk reads most (R: the plan's estimate for the record's first
// entry) are stored first, for the LDS cache (hot = 2 x their count entries).
struct W2Layout {
    std::vector<float> soa;  // 'a' halves, 'b' halves (n_entries + 1 each, the sentinel last), the quad table
    uint32_t n_entries = 0, hot = 0, start = 0;
};
void build_w2(const std::vector<rtx_entry>& E, const std::vector<double>* R, uint32_t cap, const std::vector<uint32_t>& rank,
              const std::vector<float>& quadtab, W2Layout& out) {
    const uint32_t n = (uint32_t)E.size();
    auto tag = [&](uint32_t i) {
        int32_t t;
        std::memcpy(&t, &E[i].b[3], 4);
        return t;
    };
    auto q = [&](uint32_t i) -> uint32_t {  // the fail successor (n: the sentinel)
        if (i >= n) return n;
        if (tag(i) != RTX_E_NODE) return i + 1;
        int32_t esc;
        std::memcpy(&esc, &E[i].a[3], 4);
        return (uint32_t)esc;
    };
    std::vector<int64_t> rec_of(n + 1, -1);
    std::vector<uint32_t> first;  // record -> its first entry
    auto need = [&](uint32_t i) {
        if (i < n && rec_of[i] < 0) {
            rec_of[i] = (int64_t)first.size();
            first.push_back(i);
        }
    };
    need(0);
    for (size_t k = 0; k < first.size(); ++k) {  // (first grows as records are found)
        const uint32_t p = first[k], u = q(p);
        if (tag(p) == RTX_E_NODE) need(p + 1);
        if (u < n) {
            if (tag(u) == RTX_E_NODE) need(u + 1);
            need(q(u));
        }
    }
    const uint32_t nr = (uint32_t)first.size();
    // storage order: the hot records (most reads first when estimated, else walk order), then the rest, each in walk
    // order.  A record's reads are its first entry's (R, the threaded walk's) less the arrivals there that a record
    // before it takes as its slot 1 — those of a record whose first entry does not descend (a node's fail fraction
    // 1 - R[p + 1] / R[p]: p + 1, its first child, is read once per pass of p; a primitive always goes on).
    std::vector<uint32_t> order(nr);
    for (uint32_t r = 0; r < nr; ++r) order[r] = r;
    std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return first[a] < first[b]; });
    const uint32_t take = std::min<uint32_t>(cap / 2, nr);
    std::vector<uint8_t> in_hot(nr, 0);
    if (R && R->size() == n) {
        std::vector<double> absorbed(n + 1, 0.0), reads(nr, 0.0);
        for (uint32_t r : order) {  // (q(p) > p: every record taking arrivals at p comes before p's)
            const uint32_t p = first[r], u = q(p);
            reads[r] = std::max(0.0, (*R)[p] - absorbed[p]);
            const double f = tag(p) != RTX_E_NODE ? 1.0
                             : (*R)[p] > 0.0    ? std::max(0.0, 1.0 - (p + 1 < n ? (*R)[p + 1] : 0.0) / (*R)[p])
                                                : 1.0;
            absorbed[u] += reads[r] * f;
        }
        std::vector<uint32_t> idx(order);
        std::partial_sort(idx.begin(), idx.begin() + take, idx.end(), [&](uint32_t a, uint32_t b) {
            return reads[a] != reads[b] ? reads[a] > reads[b] : first[a] < first[b];
        });
        for (uint32_t k = 0; k < take; ++k) in_hot[idx[k]] = 1;
    } else {
        for (uint32_t k = 0; k < take; ++k) in_hot[order[k]] = 1;
    }
    std::vector<uint32_t> slot(nr);
    uint32_t k = 0;
    for (uint32_t r : order)
        if (in_hot[r]) slot[r] = k++;
    for (uint32_t r : order)
        if (!in_hot[r]) slot[r] = k++;
    out.n_entries = 2 * nr;
    out.hot = 2 * take;
    const uint32_t m = out.n_entries + 1;
    const int32_t end = (int32_t)(16 * out.n_entries);
    auto P = [&](uint32_t i) -> int32_t { return i >= n ? end : (int32_t)(32 * slot[(size_t)rec_of[i]]); };
    out.start = (uint32_t)P(0);
    out.soa.assign((size_t)m * 8 + quadtab.size(), 0.0f);
    auto put = [&](uint32_t j, const float a[4], const float b[4]) {  // entry j's halves
        std::memcpy(&out.soa[4 * (size_t)j], a, 16);
        std::memcpy(&out.soa[4 * ((size_t)m + j)], b, 16);
    };
    auto word = [](float* f, int32_t v) { std::memcpy(f, &v, 4); };
    const float inf = std::numeric_limits<float>::infinity();
    const float sa[4] = {inf, inf, inf, 0.0f}, sb[4] = {-inf, -inf, -inf, 0.0f};
    for (uint32_t r = 0; r < nr; ++r) {
        const uint32_t p = first[r], u = q(p);
        for (uint32_t s2 = 0; s2 < 2; ++s2) {
            const uint32_t i = s2 == 0 ? p : u, j = 2 * slot[r] + s2;
            float a[4], b[4];
            if (i >= n) {  // the walk's end as slot 1: the sentinel (empty box, escape = next = the end)
                std::memcpy(a, sa, 16);
                std::memcpy(b, sb, 16);
                word(&a[3], end);
                word(&b[3], end);
                put(j, a, b);
                continue;
            }
            std::memcpy(a, E[i].a, 16);
            std::memcpy(b, E[i].b, 16);
            const int32_t t = tag(i);
            if (t == RTX_E_NODE) {
                word(&b[3], P(i + 1));                 // the box passes: the record of the first child
                word(&a[3], s2 ? P(q(i)) : -1);        // slot 1 fails: the record of its escape (slot 0: slot 1)
            } else {
                word(&b[2], s2 ? P(i + 1) : 0);        // slot 1: the record of its successor (slot 0: slot 1)
                if (t >= 0) {
                    word(&b[3], RTX_DEV_SPHERE(t));
                    int32_t si;  // the sphere's rank word (sphere_test RANK_WORD) in place of its index
                    std::memcpy(&si, &E[i].b[1], 4);
                    word(&b[1], (int32_t)rank[(uint32_t)si]);
                }
            }
            put(j, a, b);
        }
    }
    float a[4], b[4];  // the sentinel entry after the records
    std::memcpy(a, sa, 16);
    std::memcpy(b, sb, 16);
    word(&a[3], end);
    word(&b[3], end);
    put(out.n_entries, a, b);
    if (!quadtab.empty()) std::memcpy(&out.soa[8 * (size_t)m], quadtab.data(), quadtab.size() * sizeof(float));
}

// Upload the walk layout for `cam` to copy c (current device = c's; s->mu held).
int ensure_layout(rtx_scene* s, DeviceCopy* c, const rtx_camera* cam, bool near = false) {
    const uint32_t oct = layout_slot(s, cam, near);
    if (c->lay[oct].entries) return RTX_OK;
    const std::vector<rtx_entry>* E = nullptr;
    if (int rc = scene_layout(s, cam, &E, near)) return rc;
    DeviceLayout& lay = c->lay[oct];
    // RTX_W2=1: a layout in HBM with an LDS cache (config 4's) as the paired walk's records.
    // (Scenes with Perlin noise, or without a cache, walk HBM without the cache kernels, which read entries only.)
    // RTX_W2=2 (tests): records for any layout — walked only from HBM (RTX_FLAG_NO_LDS), else the launch fails.
    const uint32_t cap = env_knob("RTX_HOT_ENTRIES", rtxd::HOT_ENTRIES_MAX, 0, rtxd::HOT_ENTRIES_MAX) & ~1u;
    const uint32_t w2k = env_knob("RTX_W2", 0, 0, 2);  // (off by default: config 4 +6.5 %)
    if (cap > 0 && !s->has_noise && (w2k == 2 || (w2k == 1 && (E->size() + 1) * 16 > rtxd::LDS_B))) {
        W2Layout w;
        build_w2(*E, &s->reads[oct], cap, s->sphere_rank, s->quadtab, w);
        // (+64 B: a lane's record read at the walk's end may touch the sentinel's neighbour; its result is unused)
        HIP_TRY(hipMalloc(&lay.entries, w.soa.size() * sizeof(float) + 64));
        HIP_TRY(hipMemcpy(lay.entries, w.soa.data(), w.soa.size() * sizeof(float), hipMemcpyHostToDevice));
        lay.n_entries = w.n_entries;
        lay.hot = w.hot;
        lay.start = w.start;
        lay.w2 = 1;
        return RTX_OK;
    }
    lay.n_entries = (uint32_t)E->size();
    HIP_TRY(hipMalloc(&lay.entries, (E->size() + 1) * sizeof(rtx_entry) + s->quadtab.size() * sizeof(float)));
    {  // device layout: all 'a' halves, then all 'b' halves (rtxd::SceneRef), each ending
       // with the sentinel entry (rtx_layout.h).  Every entry names its successor (node: next
       // and escape, primitive: next), so the storage order is free: a scene too big for the
       // LDS copy stores its top levels first (lay.hot entries), which v3 caches in LDS; a scene
       // in the LDS copy stores its primitives first (below lay.prim_end), so the asm walk knows
       // an entry's kind from its position before the entry's read returns (walk_phase_asm).
        const size_t n = E->size(), m = n + 1;
        std::vector<uint32_t> pos(m);  // storage index of entry i; the sentinel stays last
        for (size_t i = 0; i <= n; ++i) pos[i] = (uint32_t)i;
        if (m * 16 > rtxd::LDS_B) {
            std::vector<uint32_t> depth(n), ends, per_depth;
            for (size_t i = 0; i < n; ++i) {  // depth = nodes whose subtree holds entry i
                while (!ends.empty() && ends.back() <= i) ends.pop_back();
                depth[i] = (uint32_t)ends.size();
                if (per_depth.size() <= depth[i]) per_depth.resize(depth[i] + 1, 0);
                ++per_depth[depth[i]];
                int32_t tag, esc;
                std::memcpy(&tag, &(*E)[i].b[3], 4);
                if (tag == RTX_E_NODE) {
                    std::memcpy(&esc, &(*E)[i].a[3], 4);
                    ends.push_back((uint32_t)esc);
                }
            }
            const uint32_t cap = env_knob("RTX_HOT_ENTRIES", rtxd::HOT_ENTRIES_MAX, 0, rtxd::HOT_ENTRIES_MAX);
            const std::vector<double>& R = s->reads[oct];
            std::vector<uint8_t> in_hot(n, 0);
            uint32_t hot = 0;
            if (R.size() == n && env_knob("RTX_HOT_BY_READS", 1, 0, 1)) {
                // the entries the walk reads most (the plan's sample estimate), in walk order
                std::vector<uint32_t> idx(n);
                for (size_t i = 0; i < n; ++i) idx[i] = (uint32_t)i;
                const size_t take = std::min<size_t>(cap, n);
                std::partial_sort(idx.begin(), idx.begin() + take, idx.end(), [&](uint32_t a, uint32_t b) {
                    return R[a] != R[b] ? R[a] > R[b] : depth[a] != depth[b] ? depth[a] < depth[b] : a < b;
                });
                for (size_t q = 0; q < take; ++q) in_hot[idx[q]] = 1;
                hot = (uint32_t)take;
            } else {  // the top levels
                uint32_t levels = 0;
                while (levels < per_depth.size() && hot + per_depth[levels] <= cap) hot += per_depth[levels++];
                for (size_t i = 0; i < n; ++i) in_hot[i] = depth[i] < levels;
            }
            uint32_t k = 0;
            for (size_t i = 0; i < n; ++i)
                if (in_hot[i]) pos[i] = k++;
            for (size_t i = 0; i < n; ++i)
                if (!in_hot[i]) pos[i] = k++;
            lay.hot = hot;
        } else {
            // primitives first, in the reference walk's order (the caller's tree walks them in that
            // order; a rebuilt tree's are sorted back into it): the walk's tie rule compares entry
            // indices for that order (sphere_test RANKED, rtx_device.h)
            std::vector<uint32_t> prims;
            for (size_t i = 0; i < n; ++i) {
                int32_t tag;
                std::memcpy(&tag, &(*E)[i].b[3], 4);
                if (tag != RTX_E_NODE) prims.push_back((uint32_t)i);
            }
            // quads before the spheres (in the walk's order: they have no tie rule), so a sphere never wins a tie
            // with a quad by the entry-index rule, as in the oracle (hit_rank: a quad's hit ranks 0)
            auto rank = [&](uint32_t i) -> int64_t {
                int32_t tag, si;
                std::memcpy(&tag, &(*E)[i].b[3], 4);
                if (tag < 0) return -1;
                std::memcpy(&si, &(*E)[i].b[1], 4);
                return (int64_t)s->sphere_rank[(uint32_t)si];
            };
            std::stable_sort(prims.begin(), prims.end(), [&](uint32_t a, uint32_t b) { return rank(a) < rank(b); });
            uint32_t k = 0;
            for (uint32_t i : prims) pos[i] = k++;
            for (size_t i = 0; i < n; ++i) {
                int32_t tag;
                std::memcpy(&tag, &(*E)[i].b[3], 4);
                if (tag == RTX_E_NODE) pos[i] = k++;
            }
            for (size_t i = 0; i < n; ++i) {
                int32_t tag;
                std::memcpy(&tag, &(*E)[i].b[3], 4);
                if (tag != RTX_E_NODE) lay.prim_end = 16 * (pos[i] + 1) > lay.prim_end ? 16 * (pos[i] + 1) : lay.prim_end;
            }
        }
        lay.start = 16 * pos[0];
        std::vector<float> soa(m * 8 + s->quadtab.size(), 0.0f);
        for (size_t i = 0; i < n; ++i) {
            const size_t j = pos[i];
            std::memcpy(&soa[4 * j], (*E)[i].a, 16);
            std::memcpy(&soa[4 * (m + j)], (*E)[i].b, 16);
            int32_t tag, esc;  // the device recoding, rtx_layout.h
            std::memcpy(&tag, &(*E)[i].b[3], 4);
            const int32_t next = (int32_t)(16 * pos[i + 1]);
            if (tag == RTX_E_NODE) {
                std::memcpy(&esc, &(*E)[i].a[3], 4);
                esc = (int32_t)(16 * pos[esc]);
                std::memcpy(&soa[4 * j + 3], &esc, 4);
                std::memcpy(&soa[4 * (m + j) + 3], &next, 4);
            } else {
                std::memcpy(&soa[4 * (m + j) + 2], &next, 4);  // a primitive's successor
                if (tag >= 0) {
                    const int32_t sph = RTX_DEV_SPHERE(tag);
                    std::memcpy(&soa[4 * (m + j) + 3], &sph, 4);
                    int32_t si;  // the sphere's rank word (sphere_test RANK_WORD) in place of its index
                    std::memcpy(&si, &(*E)[i].b[1], 4);
                    std::memcpy(&soa[4 * (m + j) + 1], &s->sphere_rank[(uint32_t)si], 4);
                }
            }
        }
        // the sentinel: box min +inf, max -inf, escape = next = its own position
        const float inf = std::numeric_limits<float>::infinity();
        const int32_t self = (int32_t)(16 * n);
        for (int k = 0; k < 3; ++k) {
            soa[4 * n + k] = inf;
            soa[4 * (m + n) + k] = -inf;
        }
        std::memcpy(&soa[4 * n + 3], &self, 4);
        std::memcpy(&soa[4 * (m + n) + 3], &self, 4);
        if (!s->quadtab.empty()) std::memcpy(&soa[8 * m], s->quadtab.data(), s->quadtab.size() * sizeof(float));
        HIP_TRY(hipMemcpy(lay.entries, soa.data(), soa.size() * sizeof(float), hipMemcpyHostToDevice));
    }
    return RTX_OK;
}

int upload_copy(rtx_scene* s, DeviceCopy& c) {
    // device materials: a Lambertian or DiffuseLight with a SolidColor texture carries the
    // colour itself (rtxd::RTX_DEV_TEX_INLINE), so shading reads no texture record; the other
    // textures they read are numbered anew in the device texture table, which holds only those
    // (small enough for the LDS copy: randSpheres' 488 SolidColors leave one checkered texture)
    std::vector<rtx_texture> dt;
    {
        std::vector<rtx_material> dm(s->materials);
        std::vector<int64_t> renum(s->textures.size(), -1);
        for (rtx_material& m : dm) {
            if ((m.type == RTX_MAT_LAMBERTIAN || m.type == RTX_MAT_DIFFUSE_LIGHT) &&
                s->textures[m.texture].type == RTX_TEX_SOLID) {
                std::memcpy(m.albedo, s->textures[m.texture].even, sizeof(m.albedo));
                m.texture = rtxd::RTX_DEV_TEX_INLINE;
            } else if (m.type == RTX_MAT_LAMBERTIAN || m.type == RTX_MAT_DIFFUSE_LIGHT) {
                if (renum[m.texture] < 0) {
                    renum[m.texture] = (int64_t)dt.size();
                    dt.push_back(s->textures[m.texture]);
                }
                m.texture = (uint32_t)renum[m.texture];
            }
            if (m.type == RTX_MAT_DIELECTRIC) {  // (albedo unused: attenuation is (1,1,1))
                // per-material float32 quotients of materials.go:98, 116-117, computed once here
                // (IEEE division: the same bits the kernel's correctly rounded divide gave)
                const float inv = 1.0f / m.ior;
                const float rf = (1.0f - inv) / (1.0f + inv), rb = (1.0f - m.ior) / (1.0f + m.ior);
                m.albedo[0] = inv;      // eta of a front-face hit
                m.albedo[1] = rf * rf;  // r0 for eta = 1/ior
                m.albedo[2] = rb * rb;  // r0 for eta = ior
            }
        }
        HIP_TRY(hipMalloc(&c.materials, std::max<size_t>(1, dm.size()) * sizeof(rtx_material)));
        if (!dm.empty()) HIP_TRY(hipMemcpy(c.materials, dm.data(), dm.size() * sizeof(rtx_material), hipMemcpyHostToDevice));
    }
    {  // device textures: a Checkered carries invScale = float32(1 / scale) (materials.go:128) in `pad`,
       // the IEEE quotient computed once here instead of per lookup
        for (rtx_texture& t : dt)
            if (t.type == RTX_TEX_CHECKERED) t.pad = 1.0f / t.scale;
        HIP_TRY(hipMalloc(&c.textures, std::max<size_t>(1, dt.size()) * sizeof(rtx_texture)));
        if (!dt.empty()) HIP_TRY(hipMemcpy(c.textures, dt.data(), dt.size() * sizeof(rtx_texture), hipMemcpyHostToDevice));
        c.n_textures = (uint32_t)dt.size();
    }
    HIP_TRY(hipMalloc(&c.texels, std::max<size_t>(1, s->texels.size()) * sizeof(uint32_t)));
    if (!s->texels.empty())
        HIP_TRY(hipMemcpy(c.texels, s->texels.data(), s->texels.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    HIP_TRY(hipMalloc(&c.counters, rtxd::COUNTER_SLOTS * sizeof(unsigned long long)));
    HIP_TRY(hipEventCreate(&c.ev0));
    HIP_TRY(hipEventCreate(&c.ev1));
    return RTX_OK;
}

void free_copy(DeviceCopy& c) {
    if (hipSetDevice(c.device) != hipSuccess) return;
    (void)hipDeviceSynchronize();  // no render of this copy still running
    for (DeviceLayout& l : c.lay) (void)hipFree(l.entries);
    (void)hipFree(c.materials);
    (void)hipFree(c.textures);
    (void)hipFree(c.texels);
    (void)hipFree(c.counters);
    if (c.ev0) (void)hipEventDestroy(c.ev0);
    if (c.ev1) (void)hipEventDestroy(c.ev1);
}

// Free a scene's copy; the last copy on a device also frees the device's scratch.
void drop_copy(DeviceCopy& c) {
    free_copy(c);
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    Scratch& sc = g_scratch[c.device];
    if (sc.scenes > 0 && --sc.scenes == 0) release_scratch_locked(c.device);
}

// The walk's tree (rtx_topology.h): 0 = the caller's, 1 = guarded, 2 = unguarded.  Default:
// guarded when the spheres pass rtxd::precise_enough, else the caller's.  RTX_SCENE_REFERENCE_BVH
// or the environment variable RTX_BVH=reference (read per scene) keep the caller's;
// RTX_BVH=guarded / sah force the guarded / unguarded tree (A/B).
int topology_mode(uint32_t flags, const std::vector<rtx_entry>& ref) {
    if (flags & RTX_SCENE_REFERENCE_BVH) return 0;
    const char* e = std::getenv("RTX_BVH");
    if (e && std::strcmp(e, "reference") == 0) return 0;
    if (e && std::strcmp(e, "sah") == 0) return 2;
    if (e && std::strcmp(e, "guarded") == 0) return 1;
    return rtxd::precise_enough(ref) ? 1 : 0;
}

// The tiered walk: a scene of spheres under one tree also gets a near tree (spheres
// behind their own boxes grown for origins in the near region), unless RTX_SCENE_NO_TIER,
// RTX_SCENE_REFERENCE_BVH or RTX_TIER=0, or a node box does not contain the boxes of the spheres
// below it (the hit check's argument needs that; NewBVH's always do).  Its far tree is the walk's
// other tree: the guarded rebuild, or the caller's.  The region is the core box grown by
// RTX_NEAR_GROW percent of its largest extent: 150 for scenes that pass precise_enough (randSpheres,
// C2 at 100 spp, round 4's margins and FMA walk: 50 / 100 / 150 / 200 / 300 % -> 21.73 / 21.02 / 20.65 /
// 20.73 / 21.05 ms; round 3: 10 / 25 / 40 / 60 / 100 % -> 23.73 / 23.43 / 23.21 / 22.89 / 22.67 ms),
// 1 for the others (config 4's 316-unit slab, whose far corners set every margin anyway: 0 (untiered) /
// 1 / 2 / 5 % -> 100.9 / 76.6 / 77.2 / 78.9 ms).
void quad_table(const rtx_scene_desc* d, std::vector<float>& tab);

// Quads in a near tree: the walk over another tree meets two quads that report the same t (two
// coplanar quads that overlap: the Cornell box's box bottoms on its floor) in another order than the reference, and
// the quad test has no tie rule.  Such a pair is admitted only when either answer gives the same path and colour:
// the same material (not an image texture, which reads the hit's u, v) and the same normal; else no near tree.
bool quad_ties_harmless(const rtx_scene_desc* d, const std::vector<float>& quadtab) {
    const uint32_t n = d->n_quads;
    if (n > 4096) return false;  // (pairs checked one by one)
    std::vector<std::array<float, 6>> box(n);
    for (uint32_t i = 0; i < n; ++i) rtxd::quad_own_box(&quadtab[16 * (size_t)i], &box[i][0], &box[i][3]);
    for (uint32_t i = 0; i < n; ++i)
        for (uint32_t j = i + 1; j < n; ++j) {
            const rtx_quad &a = d->quads[i], &b = d->quads[j];
            bool same = true, opp = true;
            for (int k = 0; k < 3; ++k) {
                same &= a.normal[k] == b.normal[k];
                opp &= a.normal[k] == -b.normal[k];
            }
            const bool coplanar = (same && a.d == b.d) || (opp && a.d == -b.d);
            bool overlap = coplanar;
            for (int k = 0; k < 3 && overlap; ++k) overlap = box[i][k] <= box[j][3 + k] && box[j][k] <= box[i][3 + k];
            if (!overlap) continue;
            if (!same || a.material != b.material) return false;
            const rtx_material& m = d->materials[a.material];
            if ((m.type == RTX_MAT_LAMBERTIAN || m.type == RTX_MAT_DIFFUSE_LIGHT) &&
                d->textures[m.texture].type == RTX_TEX_IMAGE)
                return false;
        }
    return true;
}

bool tier_topology(uint32_t flags, const std::vector<rtx_entry>& base, const rtx_scene_desc* d, rtxd::Topology& near) {
    if (flags & (RTX_SCENE_NO_TIER | RTX_SCENE_REFERENCE_BVH)) return false;
    const char* e = std::getenv("RTX_TIER");
    if (e && std::strcmp(e, "0") == 0) return false;
    // quads join a near tree with RTX_TIER_QUADS=1 when their coplanar ties are harmless — off by
    // default: a ray through the edge two quads share ties them too, and the quad test has no rank rule yet (the GPU
    // parity test found 11 of 4.7 M Cornell segments that then differ from the caller's tree)
    std::vector<float> quadtab;
    quad_table(d, quadtab);
    const bool quads = d->n_quads > 0;
    if (quads && (env_knob("RTX_TIER_QUADS", 0, 0, 1) == 0 || !quad_ties_harmless(d, quadtab))) return false;
    if (!rtxd::own_boxes_nested(base, quads ? &quadtab : nullptr)) return false;
    float box[6];
    // a scene with quads grows its region by 150 % too: it must hold the camera (the Cornell box's is 800 units
    // in front of its 555-unit room)
    const double grow = env_knob("RTX_NEAR_GROW", rtxd::precise_enough(base) || quads ? 150 : 1, 0, 1000) / 100.0;
    return rtxd::near_region(base, box, grow, quads ? &quadtab : nullptr) &&
           rtxd::build_topology(base, false, near, box, quads ? &quadtab : nullptr);
}

// A tiered scene walks in two tiers for a camera whose rays all start in the near region (the
// defocus disk's box, with room for rounding, inside it): else the guarded walk alone.
bool camera_in_box(const float* b, const rtx_camera* cam) {
    for (int k = 0; k < 3; ++k) {
        const double c = cam->center[k];
        const double rad = cam->defocus_angle > 0.0f
                               ? std::fabs((double)cam->defocus_disk_u[k]) + std::fabs((double)cam->defocus_disk_v[k])
                               : 0.0;
        const double pad = rad * 1.0e-3 + std::fabs(c) * 1.0e-6 + 1.0e-6;
        if (!(c - rad - pad > (double)b[k] && c + rad + pad < (double)b[3 + k])) return false;
    }
    return true;
}
bool camera_in_near(const rtx_scene* s, const rtx_camera* cam) {
    return s->tiered && camera_in_box(s->near_topo.near_box, cam);
}

// Each sphere's place in the reference walk of the caller's tree (its first entry in `base`): the walk's
// tie rule (sphere_test RANKED / RANK_WORD) for walks over another tree or in another storage order.
void rank_spheres(rtx_scene* s) {
    s->sphere_rank.clear();
    uint32_t k = 0;
    for (const rtx_entry& e : s->base) {
        int32_t tag, si;
        std::memcpy(&tag, &e.b[3], 4);
        std::memcpy(&si, &e.b[1], 4);
        if (tag < 0) continue;
        if (s->sphere_rank.size() <= (size_t)si) s->sphere_rank.resize((size_t)si + 1, 0xFFFFFFFFu);
        if (s->sphere_rank[(size_t)si] == 0xFFFFFFFFu) s->sphere_rank[(size_t)si] = k;
        ++k;
    }
}

// A scene whose base holds the reference's walk of one tree: take the walk's own tree when it
// qualifies (spheres only; rtxd::build_topology), and its near tree.
void adopt_topology(rtx_scene* s, uint32_t flags, const rtx_scene_desc* d) {
    s->every_box = (flags & RTX_SCENE_EVERY_BOX) != 0;
    const int mode = topology_mode(flags, s->base);
    if (mode != 0 && rtxd::build_topology(s->base, mode == 1, s->topo)) s->rebuilt = true;
    s->tiered = tier_topology(flags, s->base, d, s->near_topo);
}

// The quad table of a scene description (rtx_layout.h): (Q, material), (u, 0), (v, 0), (w, 0).
void quad_table(const rtx_scene_desc* d, std::vector<float>& tab) {
    tab.assign((size_t)d->n_quads * 16, 0.0f);
    for (uint32_t i = 0; i < d->n_quads; ++i) {
        const rtx_quad& q = d->quads[i];
        float* o = &tab[(size_t)i * 16];
        std::memcpy(o, q.q, 12);
        std::memcpy(o + 3, &q.material, 4);
        std::memcpy(o + 4, q.u, 12);
        std::memcpy(o + 8, q.v, 12);
        std::memcpy(o + 12, q.w, 12);
    }
}

uint64_t walk_layout(const rtx_scene* s, const rtx_camera* cam, bool tiered) {
    return (s->rebuilt ? rtxd::camera_octant(*cam) : RTX_LAYOUT_REFERENCE) | (tiered ? RTX_LAYOUT_TIERED : 0u);
}

int check_camera(const rtx_camera* cam) {
    if (!cam) return fail(RTX_ERR_INVALID_ARG, "camera is NULL");
    if (cam->image_width == 0 || cam->image_height == 0) return fail(RTX_ERR_INVALID_ARG, "empty image");
    if (cam->samples_per_pixel == 0) return fail(RTX_ERR_INVALID_ARG, "samples_per_pixel must be > 0");
    if ((uint64_t)cam->image_width * cam->image_height > 0xFFFFFFFFull)
        return fail(RTX_ERR_INVALID_ARG, "image has more than 2^32 pixels (RNG counter is 32-bit)");
    // the kernel's scratch slot of a pixel (64 per tile, tiles padded: at most 64 columns and 64 rows) is 32-bit
    if (((uint64_t)cam->image_width + 64) * ((uint64_t)cam->image_height + 64) > 0xFFFFFFFFull)
        return fail(RTX_ERR_INVALID_ARG, "image too large: its padded tiles exceed 2^32 pixel slots");
    return RTX_OK;
}

int check_region(const rtx_camera* cam, const rtx_region* r) {
    if (!r) return fail(RTX_ERR_INVALID_ARG, "region is NULL");
    if (r->world == 0 || r->rank >= r->world) return fail(RTX_ERR_INVALID_ARG, "bad shard %u/%u", r->rank, r->world);
    if (r->stripe > 4096 || (r->stripe & (r->stripe - 1)) != 0)
        return fail(RTX_ERR_INVALID_ARG, "stripe %u: 0 or a power of two up to 4096", r->stripe);
    if ((uint64_t)r->x0 + r->width > cam->image_width || (uint64_t)r->y0 + r->height > cam->image_height)
        return fail(RTX_ERR_INVALID_ARG, "region [%u+%u, %u+%u] outside %ux%u image", r->x0, r->width, r->y0, r->height,
                    cam->image_width, cam->image_height);
    return RTX_OK;
}

uint32_t region_rows(const rtx_region* r) {
    if (r->world == 0 || r->rank >= r->world) return 0;
    const uint32_t S = r->stripe > 1u ? r->stripe : 1u;
    const uint32_t nst = (r->height + S - 1) / S;  // stripes, the last one maybe partial
    if (r->rank >= nst) return 0;
    const uint32_t k = (nst - r->rank + r->world - 1) / r->world;  // this shard's stripes
    uint32_t rows = k * S;
    if ((nst - 1) % r->world == r->rank && r->height % S) rows -= S - r->height % S;  // it holds the partial one
    return rows;
}

// Stripe rows for the bands of rtx_render(n_gpus > 1): single rows (RTX_STRIPE = 2^k for A/B).  Every rank of
// the 4- and 8-GPU headline measured slowest-rank-fastest with single rows (profiles/r05_stripe_sweep.jsonl:
// N = 8 12.55 ms against 12.78 / 12.83 / 13.05 for 2 / 4 / 8-row stripes).
uint32_t band_stripe(int n) {
    const uint32_t v = n > 1 ? env_knob("RTX_STRIPE", 1, 1, 4096) : 1u;
    return 1u << (31 - __builtin_clz(v));  // a power of two
}

// Integer knob from the environment (read per call), clamped to [lo, hi].
uint32_t env_knob(const char* name, long dflt, long lo, long hi) {
    const char* e = std::getenv(name);
    const long x = e ? std::strtol(e, nullptr, 10) : dflt;
    return (uint32_t)(x < lo ? lo : (x > hi ? hi : x));
}

// Lanes of a wave that wait before it shades (v1-v3); RTX_SHADE_THRESH.  48 measured
// best for v3 at the headline config with primitive batching (44 the same, 40 +1.3 %,
// 56 +4.6 %) and for v1.
uint32_t shade_thresh() {
    static const uint32_t v = [] {
        const char* e = std::getenv("RTX_SHADE_THRESH");
        const long x = e ? std::strtol(e, nullptr, 10) : 48;
        return (uint32_t)(x < 1 ? 1 : (x > 64 ? 64 : x));
    }();
    return v;
}

// Per-wave time limit of the persistent kernel (RTX_WATCHDOG_S, default 300 s): a bug
// can never keep the GPU busy forever; the launch then fails with RTX_ERR_HIP.
uint64_t watchdog_ticks() {
    static const uint64_t v = [] {
        const char* e = std::getenv("RTX_WATCHDOG_S");
        double s = e ? std::strtod(e, nullptr) : 300.0;
        if (!(s > 0)) s = 300.0;
        return (uint64_t)(s * 1.0e8);  // s_memrealtime runs at 100 MHz
    }();
    return v;
}

rtxd::Params make_params(const rtx_scene* s, const DeviceCopy* c, uint32_t oct, const rtx_camera* cam, uint64_t seed,
                         const rtx_region* r, float* d_out) {
    rtxd::Params p;
    std::memset(&p, 0, sizeof(p));
    const DeviceLayout& lay = c->lay[oct];
    p.entries = reinterpret_cast<const float4*>(lay.entries);
    p.n_entries = lay.n_entries;
    p.n_quads = (uint32_t)(s->quadtab.size() / 16);
    p.n_materials = (uint32_t)s->materials.size();
    p.materials = c->materials;
    p.textures = c->textures;
    p.n_textures = c->n_textures;
    p.texels = c->texels;
    p.cam = *cam;
    p.seed = seed;
    p.x0 = r->x0;
    p.y0 = r->y0;
    p.width = r->width;
    p.rows = region_rows(r);
    p.rank = r->rank;
    p.world = r->world;
    p.stripe_log2 = r->stripe > 1 ? (uint32_t)__builtin_ctz(r->stripe) : 0u;
    // RTX_TILE_W = 8 / 16 / 32 overrides the tile width (A/B)
    const uint32_t tw = env_knob("RTX_TILE_W", 0, 0, 32);
    p.tile_w_log2 = tw >= 32 ? 5u : (tw >= 16 ? 4u : (tw >= 8 ? 3u : rtxd::tile_w_log2_for(r->world, r->stripe)));
    p.tile_w_log2 = std::max(p.tile_w_log2, rtxd::tile_w_log2_min(p.stripe_log2));  // a tile within one stripe
    p.out = d_out;
    p.counters = c->counters;
    p.tile_counter = reinterpret_cast<uint32_t*>(c->counters + 7);  // slot 7 low: unit queue head
    p.error_flag = nullptr;  // the device's sticky error word (KernErr), set by enqueue_on
    p.watchdog_ticks = watchdog_ticks();
    p.shade_thresh = shade_thresh();
    p.has_uv = s->has_image ? 1u : 0u;
    p.has_noise = s->has_noise ? 1u : 0u;
    p.n_hot = lay.hot;
    p.start = lay.start;
    p.prim_end = lay.prim_end;
    p.w2 = lay.w2;
    return p;
}

// Enqueue one region on the current device, bracketed by HIP events on `stream`.
// *chunks receives the number of sample chunks (render kernel launches).
// *tiered: whether the render walks in two tiers.
int enqueue_on(rtx_scene* s, DeviceCopy* c, const rtx_camera* cam, uint64_t seed, const rtx_region* r, float* d_out,
               hipStream_t stream, uint32_t flags, bool timed, uint32_t* chunks, bool* tiered) {
    const uint32_t oct = layout_slot(s, cam);  // the walk's layout (rtx_topology.h, rtx_collapse.h)
    if (int rc = ensure_layout(s, c, cam)) return rc;
    rtxd::Params p = make_params(s, c, oct, cam, seed, r, d_out);
    if (!(p.error_flag = kerr_word(c->device))) return fail(RTX_ERR_OOM, "the error word on device %d", c->device);
    // the tiered walk: a camera in the near region of a sphere scene (rtx_scene_near_region's rule)
    bool tier = camera_in_near(s, cam) && !p.has_noise;
    rtxd::Params pn;
    if (tier) {
        if (int rc = ensure_layout(s, c, cam, true)) return rc;
        pn = make_params(s, c, layout_slot(s, cam, true), cam, seed, r, d_out);
        // the paired walk's records are read by the LDS-cache kernels only: two layouts placed unalike walk alone
        if ((p.w2 || pn.w2) && rtxd::tier_placement(pn, p, flags) != RTX_SCENE_LDS_CACHE) tier = false;
        // a scene with quads walks in tiers in single-row shards, with the timed or the counting kernel
        if (p.n_quads && (r->stripe > 1 || ((flags & RTX_FLAG_TIMING) && !(flags & RTX_FLAG_COUNTERS)))) tier = false;
    }
    *tiered = false;
    const uint32_t th = (flags >> 8) & 0x7Fu;  // RTX_FLAG_SHADE_THRESH(n) override
    if (th) p.shade_thresh = th > 64 ? 64 : th;
    *chunks = 0;
    std::unique_lock<std::mutex> scr_lock(g_scratch_mu);
    Scratch* scr = &g_scratch[c->device];
    if (!scr->last) HIP_TRY(hipEventCreateWithFlags(&scr->last, hipEventDisableTiming));
    // Every render on this device waits for the previous one (the shared scratch, and the
    // scene's counters / unit queue, are reused).
    HIP_TRY(hipStreamWaitEvent(stream, scr->last, 0));
    if (p.width > 0 && p.rows > 0) {
        // Sample scratch: up to RTX_SCRATCH_MB (default 16 GiB of the 288 GB HBM) of sample
        // colours, 12 B each; the samples run in chunks that fit.
        // tile-major: every tile of 64 pixels whole (render_items / reduce_samples), 12 B per pixel
        const uint64_t per_sample =
            (uint64_t)rtxd::tiles_x_of(p.width, p.tile_w_log2) * rtxd::tiles_y_of(p.rows, p.tile_w_log2) * 64 * 12;
        const uint64_t budget = (uint64_t)env_knob("RTX_SCRATCH_MB", 16384, 1, 1 << 20) << 20;
        uint64_t chunk = budget / per_sample;
        if (chunk > cam->samples_per_pixel) chunk = cam->samples_per_pixel;
        // the tiered walk names a chunk's samples by 32-bit ids ((k - k0) * tiles * 64 + slot: the redo
        // list, the redo bits' index): at most 2^32 scratch slots per chunk
        if (tier) chunk = std::min<uint64_t>(chunk, 0xFFFFFFFFull / (per_sample / 12));
        if (chunk < 1) return fail(RTX_ERR_OOM, "RTX_SCRATCH_MB too small for one sample of the region");
        const size_t need = (size_t)(chunk * per_sample);
        if (scr->bytes < need) {
            HIP_TRY(hipEventSynchronize(scr->last));
            if (scr->ptr) HIP_TRY(hipFree(scr->ptr));
            scr->ptr = nullptr;
            scr->bytes = 0;
            HIP_TRY(hipMalloc(&scr->ptr, need));
            scr->bytes = need;
        }
        p.scratch = scr->ptr;
        p.kn = (uint32_t)chunk;
        *chunks = (uint32_t)((cam->samples_per_pixel + chunk - 1) / chunk);
        p.sub = env_knob("RTX_ITEM_SUB", 0, 0, 4096);  // 0: chosen per chunk by launch_items
        // the redo pass skips a unit by one vote over its samples' bit words, one sample per lane
        if (tier && p.sub > 64) p.sub = 64;
        p.debug_partial = env_knob("RTX_DEBUG_PARTIAL_SITE", 0, 0, 3);  // (read by librtx_dbgclaim.so only)
        p.cam_pool = env_knob("RTX_CAM_POOL", 1, 0, 1);  // the near pass's camera-ray pool (A/B: 0 = off)
        p.refill_hits = env_knob("RTX_REFILL_HITS", 0, 0, 64);  // its miss phases (untiered: off by default)
        p.item_waves = env_knob("RTX_ITEM_WAVES", 8, 4, 8) >= 8 ? 8u : 4u;
        p.grid_pct = env_knob("RTX_ITEM_GRID", 100, 1, 100);
        p.debug_launch = env_knob("RTX_DEBUG_LAUNCH", 0, 0, 1);
        p.prim_batch = env_knob("RTX_PRIM_BATCH", 16, 1, 65);  // 65: primitive tests only when no node is left
        if (tier) {
            // The queue of deferred paths, per device: an eighth of the chunk's items (measured:
            // 3.2 % of randSpheres' paths leave the near region), at least 2^21 records (the near
            // pass's waves take slots in blocks of 64), at most RTX_DEFER_MB (default 4 GiB) of
            // records; RTX_DEFER_CAP overrides (tests).  A chunk that overflows it is rendered
            // again whole by the redo pass.
            // A sample whose record does not fit is flagged in a bitmap of the chunk's samples (one bit
            // per scratch slot) and rendered again from its camera ray by the redo pass.
            const uint64_t items = chunk * (per_sample / 12);
            uint64_t cap = std::max<uint64_t>(items / 8, 1u << 21);
            if (const char* e = std::getenv("RTX_DEFER_CAP")) cap = std::strtoull(e, nullptr, 10);
            cap = std::min<uint64_t>(cap, ((uint64_t)env_knob("RTX_DEFER_MB", 4096, 1, 1 << 20) << 20) / 64);
            cap = std::min<uint64_t>(cap, 0xFFFFFFFFull / 2);
            const size_t need = (size_t)std::max<uint64_t>(cap, 1) * 64;
            if (scr->defer_bytes < need) {
                HIP_TRY(hipEventSynchronize(scr->last));
                if (scr->defer) HIP_TRY(hipFree(scr->defer));
                scr->defer = nullptr;
                scr->defer_bytes = 0;
                HIP_TRY(hipMalloc(&scr->defer, need));
                scr->defer_bytes = need;
            }
            // the bits (chunk x tiles x 64 slots, 8 per byte), then as many bytes of 4-byte sample ids: the
            // redo list holds up to 1/32 of the chunk's samples (C2 defers 0.9 % of its paths)
            const size_t bits = (size_t)(items / 8);
            if (scr->redo_bytes < 2 * bits) {
                HIP_TRY(hipEventSynchronize(scr->last));
                if (scr->redo) HIP_TRY(hipFree(scr->redo));
                scr->redo = nullptr;
                scr->redo_bytes = 0;
                scr->redo_zero = 0;
                HIP_TRY(hipMalloc(&scr->redo, 2 * bits));
                scr->redo_bytes = 2 * bits;
            }
            // The bits [0, bits) must be zero at the first chunk's start; reduce_samples keeps them so after
            // every chunk.  Past them this render's redo list may leave ids, so only [0, bits) stays known zero.
            if (scr->redo_zero < bits) HIP_TRY(hipMemsetAsync(scr->redo, 0, bits, stream));
            scr->redo_zero = bits;
            rtxd::Params lay = pn;  // the near pass: every setting of p, the near walk's layout
            pn = p;
            pn.entries = lay.entries;
            pn.n_entries = lay.n_entries;
            pn.n_hot = lay.n_hot;
            pn.start = lay.start;
            pn.prim_end = lay.prim_end;
            pn.tier = 1;
            p.tier = 2;
            // the near pass's walk is cheaper: it shades in larger batches and tests primitives in
            // smaller ones (C2 at 100 spp: 56 / 12 lanes 23.15 ms, 48 / 16 23.49 ms; the far pass keeps
            // the defaults), unless RTX_SHADE_THRESH / RTX_SHADE_THRESH(n) / RTX_PRIM_BATCH say otherwise
            // With the camera-ray pool and its miss phases the near pass shades at 52 waiting lanes
            // and takes a miss phase when fewer than 36 of them hit (C2: 90.9 ms against 91.8 at 56 / 36, 92.2 at
            // 52 / 40; profiles/r05_refill_sweep.jsonl)
            const bool pooled = rtxd::tier_placement(pn, p, flags) == RTX_SCENE_IN_LDS && rtxd::pool_fits(pn);
            if (!th && !std::getenv("RTX_SHADE_THRESH")) pn.shade_thresh = pooled ? 52 : 56;
            if (!std::getenv("RTX_REFILL_HITS")) pn.refill_hits = 36;
            if (!std::getenv("RTX_PRIM_BATCH")) pn.prim_batch = 12;
            pn.defer = p.defer = scr->defer;
            pn.redo_bits = p.redo_bits = scr->redo;
            pn.redo_ids = p.redo_ids = scr->redo + bits / 4;
            uint64_t rcap = std::min<uint64_t>(bits / 4, 0xFFFFFFFFull);
            if (const char* e = std::getenv("RTX_REDO_CAP")) rcap = std::min<uint64_t>(rcap, std::strtoull(e, nullptr, 10));
            pn.redo_cap = p.redo_cap = (uint32_t)rcap;  // (RTX_REDO_CAP: tests of the bits' path)
            pn.redo_count = p.redo_count = reinterpret_cast<uint32_t*>(c->counters + 25);
            pn.defer_cap = p.defer_cap = (uint32_t)cap;
            pn.defer_count = p.defer_count = reinterpret_cast<uint32_t*>(c->counters + 22);  // low: records
            // the drain's per-workgroup words: 2 x the near grid (launch_tiered drains only when they fit)
            if (!scr->drain) HIP_TRY(hipMalloc(&scr->drain, rtxd::DRAIN_WORDS * sizeof(uint32_t)));
            pn.drain_count = p.drain_count = scr->drain;
            pn.drain = p.drain = env_knob("RTX_DRAIN", 1, 0, 1);
            std::memcpy(pn.near_min, s->near_topo.near_box, 3 * sizeof(float));
            std::memcpy(pn.near_max, s->near_topo.near_box + 3, 3 * sizeof(float));
            *tiered = true;
        }
    }
    c->placement = *tiered ? rtxd::tier_placement(pn, p, flags) : rtxd::scene_placement(p, flags);
    // every stats slot and the unit queue head start at 0 for every render (a tiered render's first chunk_start
    // launch zeroes them: one launch fewer); the sticky error word is not among them
    if (!*tiered) HIP_TRY(hipMemsetAsync(c->counters, 0, rtxd::COUNTER_SLOTS * sizeof(unsigned long long), stream));
    if (timed) HIP_TRY(hipEventRecord(c->ev0, stream));
    if (const hipError_t e = *tiered ? rtxd::launch_render(pn, flags, stream, &p) : rtxd::launch_render(p, flags, stream)) {
        scr->redo_zero = 0;  // a chunk may have stopped between setting redo bits and clearing them
        return fail(e == hipErrorOutOfMemory ? RTX_ERR_OOM : RTX_ERR_HIP, "render launch failed: %s", hipGetErrorString(e));
    }
    if (timed) HIP_TRY(hipEventRecord(c->ev1, stream));
    HIP_TRY(hipEventRecord(scr->last, stream));
    return RTX_OK;
}

// Wait for an enqueue_on(timed=true) and read its time and counters.
int collect_on(DeviceCopy* c, bool count, uint64_t samples, uint32_t chunks, rtx_stats* st) {
    HIP_TRY(hipEventSynchronize(c->ev1));
    float ms = 0.0f;
    HIP_TRY(hipEventElapsedTime(&ms, c->ev0, c->ev1));
    unsigned long long h[rtxd::COUNTER_SLOTS] = {0};
    HIP_TRY(hipMemcpy(h, c->counters, rtxd::COUNTER_SLOTS * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    // any render on the device since the last report (this one, or one enqueued without stats before it)
    if (int rc = kerr_take(c->device)) return rc;
    std::memset(st, 0, sizeof(*st));
    st->samples = count ? h[0] : samples;
    st->segments = h[1];
    st->node_visits = h[2];
    st->prim_tests = h[3];
    st->hits = h[4];
    st->texel_fetches = h[5];
    st->rng_draws = h[6];
    st->wave_iters = h[8];
    st->lane_steps = h[9];
    st->shade_phases = h[10];
    st->shade_lanes = h[11];
    st->trav_cycles = h[12];
    st->shade_cycles = h[13];
    st->idle_lanes = h[14];
    st->cache_hits = h[15];
    st->parked_lanes = h[16];
    st->deferred_lanes = h[17];
    for (int q = 0; q < 4; ++q) st->shade_split_cycles[q] = h[18 + q];
    st->sample_chunks = chunks;
    st->deferred_paths = h[23];
    st->redo_chunks = h[24];
    st->kernel_ms = ms;
    st->scene_placement = c->placement;
    return RTX_OK;
}

// Checks of the tables every scene shares (materials, textures, texels, primitives).
int validate_tables(const rtx_scene_desc* d) {
    if (d->n_spheres && !d->spheres) return fail(RTX_ERR_INVALID_ARG, "spheres is NULL");
    if (d->n_materials && !d->materials) return fail(RTX_ERR_INVALID_ARG, "materials is NULL");
    if (d->n_textures && !d->textures) return fail(RTX_ERR_INVALID_ARG, "textures is NULL");
    if (d->n_texels && !d->texels) return fail(RTX_ERR_INVALID_ARG, "texels is NULL");
    if (d->n_quads && !d->quads) return fail(RTX_ERR_INVALID_ARG, "quads is NULL");
    if (d->n_quads > (1u << 26)) return fail(RTX_ERR_INVALID_ARG, "too many quads");
    for (uint32_t i = 0; i < d->n_quads; ++i)
        if (d->quads[i].material >= d->n_materials)
            return fail(RTX_ERR_INVALID_ARG, "quad %u material %u out of range", i, d->quads[i].material);
    for (uint32_t i = 0; i < d->n_spheres; ++i)
        if (d->spheres[i].material >= d->n_materials)
            return fail(RTX_ERR_INVALID_ARG, "sphere %u material %u out of range", i, d->spheres[i].material);
    for (uint32_t i = 0; i < d->n_materials; ++i) {
        const rtx_material& m = d->materials[i];
        if (m.type > RTX_MAT_DIFFUSE_LIGHT) return fail(RTX_ERR_INVALID_ARG, "material %u: unknown type %u", i, m.type);
        if ((m.type == RTX_MAT_LAMBERTIAN || m.type == RTX_MAT_DIFFUSE_LIGHT) && m.texture >= d->n_textures)
            return fail(RTX_ERR_INVALID_ARG, "material %u texture %u out of range", i, m.texture);
    }
    for (uint32_t i = 0; i < d->n_textures; ++i) {
        const rtx_texture& t = d->textures[i];
        if (t.type == RTX_TEX_NOISE) {
            if ((uint64_t)t.texel_offset + RTX_NOISE_TEXELS > d->n_texels)
                return fail(RTX_ERR_INVALID_ARG, "texture %u: Perlin tables out of range", i);
            for (uint32_t k = 768; k < RTX_NOISE_TEXELS; ++k)
                if (d->texels[t.texel_offset + k] > 255)
                    return fail(RTX_ERR_INVALID_ARG, "texture %u: Perlin permutation entry out of range", i);
        }
        if (t.type > RTX_TEX_NOISE) return fail(RTX_ERR_INVALID_ARG, "texture %u: unknown type %u", i, t.type);
        if (t.type == RTX_TEX_IMAGE && (int32_t)t.height > 0) {  // RGBA16 raster + border texel (rtx.h)
            if (t.texel_offset & 1u) return fail(RTX_ERR_INVALID_ARG, "texture %u: texel_offset must be even", i);
            if ((uint64_t)t.texel_offset + RTX_IMAGE_TEXEL_WORDS * ((uint64_t)t.width * t.height + 1) > d->n_texels)
                return fail(RTX_ERR_INVALID_ARG, "texture %u texels out of range", i);
        }
    }
    return RTX_OK;
}

// Quad table, materials, textures and texels of a scene whose entries are built; then
// the copy on the current device.  Takes ownership of s (deleted on failure).
int finish_scene(rtx_scene* s, const rtx_scene_desc* d, rtx_scene** out) {
    quad_table(d, s->quadtab);
    s->materials.assign(d->materials, d->materials + d->n_materials);
    s->textures.assign(d->textures, d->textures + d->n_textures);
    for (const rtx_texture& t : s->textures) {
        s->has_image |= t.type == RTX_TEX_IMAGE;
        s->has_noise |= t.type == RTX_TEX_NOISE;
    }
    if (d->n_texels) s->texels.assign(d->texels, d->texels + d->n_texels);
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess) {
        delete s;
        return fail(RTX_ERR_NO_DEVICE, "no HIP device");
    }
    DeviceCopy* c = nullptr;
    if (int rc = ensure_device(s, cur, &c)) {
        for (auto& kv : s->copies) drop_copy(kv.second);
        delete s;
        return rc;
    }
    *out = s;
    return RTX_OK;
}

// rtx_render's band assembly on device 0: the RCCL-gathered bands g[d][r][:] (n bands
// of R rows, row_floats = 3 W floats each; band d holds image rows y = d + r n) -> img[y][:].
__global__ __launch_bounds__(256) void deinterleave_bands(const float* __restrict__ g, float* __restrict__ img,
                                                          uint32_t n, uint32_t R, uint32_t H, uint32_t row_floats,
                                                          uint32_t S) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (uint64_t)H * row_floats) return;
    const uint32_t y = (uint32_t)(i / row_floats), x = (uint32_t)(i % row_floats);
    const uint32_t st = y / S, d = st % n, lr = (st / n) * S + y % S;  // stripe st of band d: its row lr
    img[i] = g[((uint64_t)d * R + lr) * row_floats + x];
}

void add_stats(rtx_stats* acc, const rtx_stats& s) {
    acc->samples += s.samples;
    acc->segments += s.segments;
    acc->node_visits += s.node_visits;
    acc->prim_tests += s.prim_tests;
    acc->hits += s.hits;
    acc->texel_fetches += s.texel_fetches;
    acc->rng_draws += s.rng_draws;
    acc->kernel_ms = std::max(acc->kernel_ms, s.kernel_ms);
    acc->wave_iters += s.wave_iters;
    acc->lane_steps += s.lane_steps;
    acc->shade_phases += s.shade_phases;
    acc->shade_lanes += s.shade_lanes;
    acc->trav_cycles += s.trav_cycles;
    acc->shade_cycles += s.shade_cycles;
    acc->idle_lanes += s.idle_lanes;
    acc->cache_hits += s.cache_hits;
    acc->parked_lanes += s.parked_lanes;
    acc->deferred_lanes += s.deferred_lanes;
    for (int q = 0; q < 4; ++q) acc->shade_split_cycles[q] += s.shade_split_cycles[q];
    acc->sample_chunks = std::max(acc->sample_chunks, s.sample_chunks);
    acc->deferred_paths += s.deferred_paths;
    acc->redo_chunks += s.redo_chunks;
    acc->scene_placement = s.scene_placement;
}

}  // namespace

extern "C" {

int rtx_version(void) { return RTX_ABI_VERSION; }

// (No build date: the library's bytes depend on its sources only, so the PMC profiles bench.py ties to the
// library's hash stay valid across rebuilds of the same sources.)
const char* rtx_build_info(void) {
    return "librtx gfx950 megakernel (ABI 9: persistent (pixel, sample) item waves, LDS scene, threaded pre-order BVH "
           "(binned-SAH walk trees per camera octant: tiered near / guarded, or the caller's), collapsed walk, "
           "RGBA16 image texels, RCCL band gather, PPM on device 0 for any band count)";
}

const char* rtx_last_error(void) { return g_last_error.c_str(); }

int rtx_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

uint32_t rtx_region_rows(const rtx_region* region) { return region ? region_rows(region) : 0; }
uint32_t rtx_region_row(const rtx_region* region, uint32_t i) {
    if (!region || region->world == 0) return 0;
    const uint32_t S = region->stripe > 1u ? region->stripe : 1u;
    return ((i / S) * region->world + region->rank) * S + i % S;
}

int rtx_scene_create(const rtx_scene_desc* d, rtx_scene** out) { return rtx_scene_create_ex(d, 0u, out); }

int rtx_scene_create_ex(const rtx_scene_desc* d, uint32_t flags, rtx_scene** out) {
    g_last_error.clear();
    if (!d || !out) return fail(RTX_ERR_INVALID_ARG, "NULL argument");
    *out = nullptr;
    if (d->n_roots == 0 || !d->roots) return fail(RTX_ERR_INVALID_ARG, "scene has no root");
    if (d->n_nodes && !d->nodes) return fail(RTX_ERR_INVALID_ARG, "nodes is NULL");
    if (d->n_lists && !d->lists) return fail(RTX_ERR_INVALID_ARG, "lists is NULL");
    if (d->n_list_refs && !d->list_refs) return fail(RTX_ERR_INVALID_ARG, "list_refs is NULL");
    if (int rc = validate_tables(d)) return rc;
    if (int rc = check_acyclic(d)) return rc;
    rtx_scene* s = new rtx_scene();
    for (uint32_t i = 0; i < d->n_roots; ++i) {
        if (int rc = emit(d, d->roots[i], s->base)) {
            delete s;
            return rc;
        }
    }
    rank_spheres(s);
    if (d->n_roots == 1) adopt_topology(s, flags, d);
    else s->every_box = (flags & RTX_SCENE_EVERY_BOX) != 0;
    return finish_scene(s, d, out);
}

int rtx_scene_create_spheres(const rtx_sphere* spheres, uint32_t n_spheres, const rtx_material* materials,
                             uint32_t n_materials, const rtx_texture* textures, uint32_t n_textures,
                             const uint32_t* texels, uint64_t n_texels, uint64_t bvh_seed, uint64_t bvh_draw0,
                             rtx_scene** out, double* build_ms) {
    g_last_error.clear();
    if (!out || !spheres) return fail(RTX_ERR_INVALID_ARG, "NULL argument");
    *out = nullptr;
    if (n_spheres == 0) return fail(RTX_ERR_INVALID_ARG, "empty World (NewBVH indexes h[0], bvh.go:164)");
    if (n_spheres > (1u << 25)) return fail(RTX_ERR_INVALID_ARG, "too many spheres for the GPU BVH build");
    rtx_scene_desc d{};
    d.spheres = spheres;
    d.n_spheres = n_spheres;
    d.materials = materials;
    d.n_materials = n_materials;
    d.textures = textures;
    d.n_textures = n_textures;
    d.texels = texels;
    d.n_texels = n_texels;
    if (int rc = validate_tables(&d)) return rc;
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess) return fail(RTX_ERR_NO_DEVICE, "no HIP device");
    rtx_scene* s = new rtx_scene();
    double ms = 0;
    hipError_t e = rtxd::build_sphere_bvh(spheres, n_spheres, bvh_seed, bvh_draw0, s->base, &ms);
    if (e != hipSuccess) {
        delete s;
        return fail(e == hipErrorOutOfMemory ? RTX_ERR_OOM : RTX_ERR_HIP, "GPU BVH build: %s", hipGetErrorString(e));
    }
    if (build_ms) *build_ms = ms;
    rank_spheres(s);
    adopt_topology(s, 0u, &d);
    return finish_scene(s, &d, out);
}

uint64_t rtx_scene_export(const rtx_scene* s, void* out, uint64_t cap) {
    if (!s) return 0;
    const uint64_t bytes = s->base.size() * sizeof(rtx_entry);
    if (out && cap >= bytes) std::memcpy(out, s->base.data(), bytes);
    return bytes;
}

int rtx_scene_topology(const rtx_scene* s, uint32_t octant, rtx_bvh_node* nodes, uint32_t cap, uint32_t* n_nodes,
                       int32_t* root) {
    g_last_error.clear();
    const bool near = (octant & RTX_TREE_NEAR) != 0;
    octant &= ~RTX_TREE_NEAR;
    if (!s || !n_nodes || !root || octant > 7) return fail(RTX_ERR_INVALID_ARG, "bad argument");
    if (near ? !s->tiered : !s->rebuilt) {
        *n_nodes = 0;
        *root = -1;
        return RTX_OK;
    }
    const rtxd::Topology& t = near ? s->near_topo : s->topo;
    std::vector<rtx_bvh_node> v;
    rtxd::orient_topology(t, octant, v);
    *n_nodes = (uint32_t)v.size();
    *root = t.root;
    if (nodes && cap >= v.size()) std::memcpy(nodes, v.data(), v.size() * sizeof(rtx_bvh_node));
    return RTX_OK;
}

uint32_t rtx_camera_octant(const rtx_camera* cam) { return cam ? rtxd::camera_octant(*cam) : 0u; }

namespace {
int copy_skip(const std::vector<uint8_t>& v, uint8_t* skip, uint32_t cap, uint32_t* n) {
    *n = (uint32_t)v.size();
    if (skip && cap >= v.size() && !v.empty()) std::memcpy(skip, v.data(), v.size());
    return RTX_OK;
}
}  // namespace

int rtx_scene_walk_skip(rtx_scene* s, const rtx_camera* cam, uint8_t* skip, uint32_t cap, uint32_t* n) {
    g_last_error.clear();
    if (!s || !n) return fail(RTX_ERR_INVALID_ARG, "bad argument");
    if (int rc = check_camera(cam)) return rc;
    std::lock_guard<std::mutex> lk(s->mu);
    const std::vector<rtx_entry>* E = nullptr;
    if (int rc = scene_layout(s, cam, &E)) return rc;
    return copy_skip(s->skips[layout_slot(s, cam)], skip, cap, n);
}

int rtx_scene_near_skip(rtx_scene* s, const rtx_camera* cam, uint8_t* skip, uint32_t cap, uint32_t* n) {
    g_last_error.clear();
    if (!s || !n) return fail(RTX_ERR_INVALID_ARG, "bad argument");
    if (int rc = check_camera(cam)) return rc;
    std::lock_guard<std::mutex> lk(s->mu);
    const std::vector<rtx_entry>* E = nullptr;
    if (int rc = scene_layout(s, cam, &E, true)) return rc;
    return copy_skip(s->skips[layout_slot(s, cam, true)], skip, cap, n);
}

int rtx_scene_near_region(rtx_scene* s, const rtx_camera* cam, float box[6], uint32_t* active) {
    g_last_error.clear();
    if (!s || !box || !active) return fail(RTX_ERR_INVALID_ARG, "bad argument");
    if (int rc = check_camera(cam)) return rc;
    std::lock_guard<std::mutex> lk(s->mu);
    *active = 0;
    if (!s->tiered) return RTX_OK;
    std::memcpy(box, s->near_topo.near_box, 6 * sizeof(float));
    *active = camera_in_near(s, cam) && !s->has_noise;
    return RTX_OK;
}

int rtx_walk_near_region(const rtx_scene_desc* d, uint32_t flags, const rtx_camera* cam, float box[6],
                         uint32_t* active) {
    g_last_error.clear();
    if (!d || !box || !active) return fail(RTX_ERR_INVALID_ARG, "bad argument");
    if (int rc = check_camera(cam)) return rc;
    if (d->n_roots == 0 || !d->roots) return fail(RTX_ERR_INVALID_ARG, "scene has no root");
    if (d->n_nodes && !d->nodes) return fail(RTX_ERR_INVALID_ARG, "nodes is NULL");
    if (int rc = validate_tables(d)) return rc;
    if (int rc = check_acyclic(d)) return rc;
    std::vector<rtx_entry> base;
    for (uint32_t i = 0; i < d->n_roots; ++i)
        if (int rc = emit(d, d->roots[i], base)) return rc;
    *active = 0;
    rtxd::Topology nt;
    if (d->n_roots != 1 || !tier_topology(flags, base, d, nt)) return RTX_OK;
    std::memcpy(box, nt.near_box, 6 * sizeof(float));
    bool noise = false;
    for (uint32_t i = 0; i < d->n_textures; ++i) noise |= d->textures[i].type == RTX_TEX_NOISE;
    *active = camera_in_box(nt.near_box, cam) && !noise;
    return RTX_OK;
}

int rtx_walk_skip(const rtx_scene_desc* d, uint32_t flags, const rtx_camera* cam, uint8_t* skip, uint32_t cap,
                  uint32_t* n) {
    g_last_error.clear();
    if (!d || !n) return fail(RTX_ERR_INVALID_ARG, "bad argument");
    if (int rc = check_camera(cam)) return rc;
    if (d->n_roots == 0 || !d->roots) return fail(RTX_ERR_INVALID_ARG, "scene has no root");
    if (d->n_nodes && !d->nodes) return fail(RTX_ERR_INVALID_ARG, "nodes is NULL");
    if (int rc = validate_tables(d)) return rc;
    if (int rc = check_acyclic(d)) return rc;
    std::vector<rtx_entry> base;
    for (uint32_t i = 0; i < d->n_roots; ++i)
        if (int rc = emit(d, d->roots[i], base)) return rc;
    rtxd::Topology t;
    const bool rebuilt = d->n_roots == 1 && topology_mode(flags, base) != 0 &&
                         rtxd::build_topology(base, topology_mode(flags, base) == 1, t);
    std::vector<float> quadtab;
    quad_table(d, quadtab);
    std::vector<rtx_entry> walk;
    std::vector<uint8_t> v;
    plan_walk(base, rebuilt ? &t : nullptr, rtxd::camera_octant(*cam), quadtab, *cam,
              collapse_enabled((flags & RTX_SCENE_EVERY_BOX) != 0), walk, v, nullptr);
    return copy_skip(v, skip, cap, n);
}

int rtx_walk_tree(const rtx_scene_desc* d, uint32_t flags, uint32_t octant, rtx_bvh_node* nodes, uint32_t cap,
                  uint32_t* n_nodes, int32_t* root) {
    g_last_error.clear();
    const bool near = (octant & RTX_TREE_NEAR) != 0;
    octant &= ~RTX_TREE_NEAR;
    if (!d || !n_nodes || !root || octant > 7) return fail(RTX_ERR_INVALID_ARG, "bad argument");
    if (d->n_roots == 0 || !d->roots) return fail(RTX_ERR_INVALID_ARG, "scene has no root");
    if (d->n_nodes && !d->nodes) return fail(RTX_ERR_INVALID_ARG, "nodes is NULL");
    if (int rc = validate_tables(d)) return rc;
    if (int rc = check_acyclic(d)) return rc;
    std::vector<rtx_entry> ref;
    for (uint32_t i = 0; i < d->n_roots; ++i)
        if (int rc = emit(d, d->roots[i], ref)) return rc;
    rtxd::Topology t;
    const int mode = topology_mode(flags, ref);
    if (d->n_roots != 1 || (near ? !tier_topology(flags, ref, d, t) : (mode == 0 || !rtxd::build_topology(ref, mode == 1, t)))) {
        *n_nodes = 0;
        *root = -1;
        return RTX_OK;
    }
    std::vector<rtx_bvh_node> v;
    rtxd::orient_topology(t, octant, v);
    *n_nodes = (uint32_t)v.size();
    *root = t.root;
    if (nodes && cap >= v.size()) std::memcpy(nodes, v.data(), v.size() * sizeof(rtx_bvh_node));
    return RTX_OK;
}

void rtx_scene_destroy(rtx_scene* s) {
    if (!s) return;
    int cur = 0;
    (void)hipGetDevice(&cur);
    for (auto& kv : s->copies) drop_copy(kv.second);
    (void)hipSetDevice(cur);
    delete s;
}

uint64_t rtx_scene_device_bytes(const rtx_scene* s) {
    if (!s) return 0;
    return s->base.size() * sizeof(rtx_entry) + s->quadtab.size() * sizeof(float) +
           s->materials.size() * sizeof(rtx_material) +
           s->textures.size() * sizeof(rtx_texture) + s->texels.size() * sizeof(uint32_t);
}

namespace {
// rtx_render_region_device with s->mu held by the caller.  Lock order everywhere: s->mu, then
// g_render_mu (rtx_render_ex, rtx_render_ppm), then g_scratch_mu (enqueue_on).
int render_region_locked(rtx_scene* s, const rtx_camera* cam, uint64_t seed, const rtx_region* region, float* d_out,
                         void* hip_stream, uint32_t flags, rtx_stats* stats) {
    int cur = 0;
    HIP_TRY(hipGetDevice(&cur));
    DeviceCopy* c = nullptr;
    if (int rc = ensure_device(s, cur, &c)) return rc;
    HIP_TRY(hipSetDevice(cur));
    const bool count = (flags & RTX_FLAG_COUNTERS) != 0;
    uint32_t chunks = 0;
    bool tiered = false;
    if (int rc = enqueue_on(s, c, cam, seed, region, d_out, (hipStream_t)hip_stream, flags, stats != nullptr, &chunks,
                            &tiered))
        return rc;
    if (!stats) return RTX_OK;
    const int rc = collect_on(c, count, (uint64_t)region_rows(region) * region->width * cam->samples_per_pixel, chunks, stats);
    stats->walk_layout = walk_layout(s, cam, tiered);
    return rc;
}
}  // namespace

int rtx_render_region_device(rtx_scene* s, const rtx_camera* cam, uint64_t seed, const rtx_region* region,
                             float* d_out, void* hip_stream, uint32_t flags, rtx_stats* stats) {
    g_last_error.clear();
    if (!s || !d_out) return fail(RTX_ERR_INVALID_ARG, "NULL argument");
    if (int rc = check_camera(cam)) return rc;
    if (int rc = check_region(cam, region)) return rc;
    std::lock_guard<std::mutex> lk(s->mu);
    return render_region_locked(s, cam, seed, region, d_out, hip_stream, flags, stats);
}

int rtx_render(rtx_scene* s, const rtx_camera* cam, uint64_t seed, int n_gpus, float* out_rgb, rtx_stats* stats) {
    return rtx_render_ex(s, cam, seed, n_gpus, 0u, out_rgb, stats);
}

namespace {
int render_bands_locked(rtx_scene* s, const rtx_camera* cam, uint64_t seed, int n_gpus, uint32_t flags, float* out_rgb,
                        float** dev_img, hipStream_t* dev_stream, rtx_stats* stats);
}  // namespace

int rtx_render_ex(rtx_scene* s, const rtx_camera* cam, uint64_t seed, int n_gpus, uint32_t flags, float* out_rgb,
                  rtx_stats* stats) {
    g_last_error.clear();
    if (!s || !out_rgb) return fail(RTX_ERR_INVALID_ARG, "NULL argument");
    if (int rc = check_camera(cam)) return rc;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(RTX_ERR_NO_DEVICE, "no HIP device");
    if (n_gpus <= 0) n_gpus = 1;
    if (n_gpus > ndev) return fail(RTX_ERR_INVALID_ARG, "n_gpus=%d but %d devices visible", n_gpus, ndev);
    std::lock_guard<std::mutex> lk(s->mu);
    std::lock_guard<std::mutex> bl(g_render_mu);  // the cached band / gather / image buffers
    return render_bands_locked(s, cam, seed, n_gpus, flags, out_rgb, nullptr, nullptr, stats);
}

namespace {
// rtx_render_ex's bands (rows y % n == d on device d) and their assembly, with s->mu and g_render_mu
// held by the caller.  out_rgb: the caller's host buffer.  Or out_rgb == nullptr: the assembled image
// stays on device 0 in *dev_img (a cached render buffer, valid until the next render under
// g_render_mu), written by *dev_stream (rtx_render_ppm_ex encodes it there).
int render_bands_locked(rtx_scene* s, const rtx_camera* cam, uint64_t seed, int n_gpus, uint32_t flags, float* out_rgb,
                        float** dev_img, hipStream_t* dev_stream, rtx_stats* stats) {
    // RTX_SIM_BANDS=k (tests, one device): k bands, all on device 0, gathered by device copies
    const uint32_t sim = n_gpus == 1 ? env_knob("RTX_SIM_BANDS", 1, 1, 64) : 1u;
    int n = sim > 1 ? (int)sim : n_gpus;
    if ((uint32_t)n > cam->image_height) n = (int)cam->image_height;
    auto dev_of = [&](int d) { return sim > 1 ? 0 : d; };
    // the gather: RCCL for more than one device (RTX_FORCE_RCCL=1: also for one, a 1-rank gather);
    // per-band copies into the caller's rows when RCCL is unavailable or fails (RTX_NO_RCCL=1: always)
    const bool want_rccl = sim == 1 && (n > 1 || env_knob("RTX_FORCE_RCCL", 0, 0, 1) == 1);
    const bool no_rccl = env_knob("RTX_NO_RCCL", 0, 0, 1) == 1;
    const uint32_t kflags = flags & RTX_FLAG_COUNTERS;
    int cur = 0;
    HIP_TRY(hipGetDevice(&cur));
    const uint32_t W = cam->image_width, H = cam->image_height;
    const uint32_t S = band_stripe(n);  // rows per stripe (single rows unless RTX_STRIPE says otherwise)
    rtx_region reg0{0, 0, W, H, 0, (uint32_t)n, S};
    const uint32_t R = region_rows(&reg0);  // rows of band 0, the longest: every band is sent padded to R
    const size_t band_floats = (size_t)R * W * 3, band_bytes = std::max<size_t>(band_floats, 1) * sizeof(float);
    const size_t img_bytes = (size_t)H * W * 3 * sizeof(float);
    std::vector<float*> bufs(n, nullptr);
    std::vector<hipStream_t> streams(n, nullptr);
    std::vector<rtx_region> regs(n);
    std::vector<uint32_t> chunks(n, 0);
    rtx_stats total;
    std::memset(&total, 0, sizeof(total));
    int rc = RTX_OK;
    bool tiered = false;
    // 1. Each band (rows y % n == d) renders on its device, the devices concurrently.
    for (int d = 0; d < n && rc == RTX_OK; ++d) {
        const int dv = dev_of(d);
        DeviceCopy* c = nullptr;
        if ((rc = ensure_device(s, dv, &c))) break;
        if (hipSetDevice(dv) != hipSuccess) { rc = fail(RTX_ERR_HIP, "hipSetDevice(%d)", dv); break; }
        regs[d] = rtx_region{0, 0, W, H, (uint32_t)d, (uint32_t)n, S};
        if (!(streams[d] = render_stream(dv))) { rc = fail(RTX_ERR_HIP, "stream on device %d", dv); break; }
        if (!(bufs[d] = static_cast<float*>(render_buffer(dv, d, band_bytes)))) {
            rc = fail(RTX_ERR_OOM, "hipMalloc band %zu B", band_bytes);
            break;
        }
        rc = enqueue_on(s, c, cam, seed, &regs[d], bufs[d], streams[d], kflags, true, &chunks[d], &tiered);
        if (rc == RTX_OK && sim > 1) {  // simulated bands share device 0's counters and events: read each now
            rtx_stats st;
            rc = collect_on(c, kflags != 0, (uint64_t)region_rows(&regs[d]) * W * cam->samples_per_pixel, chunks[d], &st);
            if (rc == RTX_OK) add_stats(&total, st);
        }
    }
    // 2. Wait for every band (and read its counters), so gather_ms times only the gather.
    for (int d = 0; d < n && rc == RTX_OK && sim == 1; ++d) {
        if (hipSetDevice(dev_of(d)) != hipSuccess) { rc = fail(RTX_ERR_HIP, "hipSetDevice(%d)", dev_of(d)); break; }
        rtx_stats st;
        uint64_t samples = (uint64_t)region_rows(&regs[d]) * W * cam->samples_per_pixel;
        if ((rc = collect_on(&s->copies[dev_of(d)], kflags != 0, samples, chunks[d], &st))) break;
        add_stats(&total, st);
    }
    // 3. Assemble on device 0: the padded bands gathered (one ncclGather over xGMI, or device
    //    copies of simulated bands), de-interleaved by a kernel, copied into the caller's buffer;
    //    or, without RCCL, each band's rows copied straight into the caller's rows.
    uint32_t kind = n == 1 && !want_rccl ? RTX_GATHER_NONE : (sim > 1 ? RTX_GATHER_DEVICE : RTX_GATHER_RCCL);
    std::vector<ncclComm_t>* comms = nullptr;
    const RcclApi* api = nullptr;
    std::unique_lock<std::mutex> rl(g_rccl_mu, std::defer_lock);
    if (rc == RTX_OK && kind == RTX_GATHER_RCCL) {
        rl.lock();
        api = no_rccl ? nullptr : rccl_api();
        if (api) {
            auto it = g_comms.find(n);
            if (it == g_comms.end()) {
                std::vector<ncclComm_t> cs(n, nullptr);
                std::vector<int> devs(n);
                for (int d = 0; d < n; ++d) devs[d] = d;
                if (api->CommInitAll(cs.data(), n, devs.data()) == ncclSuccess) it = g_comms.emplace(n, cs).first;
            }
            if (it != g_comms.end()) comms = &it->second;
        }
        if (!comms) kind = RTX_GATHER_HOST;  // RCCL unavailable: per-band copies
    }
    if (rc == RTX_OK && sim > 1 && no_rccl) kind = RTX_GATHER_HOST;
    hipEvent_t g0 = nullptr, g1 = nullptr;
    if (rc == RTX_OK && kind != RTX_GATHER_NONE) {
        (void)hipSetDevice(0);
        g0 = render_event(0, 0);
        g1 = render_event(0, 1);
        if (!g0 || !g1 || hipEventRecord(g0, streams[0]) != hipSuccess) rc = fail(RTX_ERR_HIP, "gather events");
    }
    float* gathered = nullptr;
    float* img = nullptr;
    if (rc == RTX_OK && (kind == RTX_GATHER_RCCL || kind == RTX_GATHER_DEVICE)) {
        (void)hipSetDevice(0);
        gathered = static_cast<float*>(render_buffer(0, -1, (size_t)n * band_bytes));
        img = static_cast<float*>(render_buffer(0, -2, img_bytes));
        if (!gathered || !img) rc = fail(RTX_ERR_OOM, "device-0 buffers for the gather of %d bands", n);
    }
    if (rc == RTX_OK && kind == RTX_GATHER_RCCL) {
        ncclResult_t e = api->GroupStart();
        for (int d = 0; d < n && e == ncclSuccess; ++d)
            e = api->Gather(bufs[d], d == 0 ? gathered : nullptr, band_floats, ncclFloat, 0, (*comms)[d], streams[d]);
        const ncclResult_t e2 = api->GroupEnd();
        if (e == ncclSuccess) e = e2;
        if (e != ncclSuccess) {  // degrade to per-band copies (the bands are intact)
            for (int d = 0; d < n; ++d)
                if (hipSetDevice(d) == hipSuccess) (void)hipStreamSynchronize(streams[d]);
            (void)hipSetDevice(0);
            (void)hipEventRecord(g0, streams[0]);
            kind = RTX_GATHER_HOST;
        }
    }
    if (rc == RTX_OK && kind == RTX_GATHER_DEVICE) {
        for (int d = 0; d < n && rc == RTX_OK; ++d)
            if (hipMemcpyAsync(gathered + (size_t)d * (band_bytes / sizeof(float)), bufs[d], band_bytes,
                               hipMemcpyDeviceToDevice, streams[0]) != hipSuccess)
                rc = fail(RTX_ERR_HIP, "band copy %d", d);
    }
    if (rc == RTX_OK && (kind == RTX_GATHER_RCCL || kind == RTX_GATHER_DEVICE)) {
        (void)hipSetDevice(0);
        const uint64_t total_floats = (uint64_t)H * W * 3;
        hipLaunchKernelGGL(deinterleave_bands, dim3((uint32_t)((total_floats + 255) / 256)), dim3(256), 0, streams[0],
                           gathered, img, (uint32_t)n, R, H, W * 3, S);
        hipError_t e = hipGetLastError();
        if (e == hipSuccess) e = hipEventRecord(g1, streams[0]);
        if (e == hipSuccess && out_rgb) e = copy_to_host(out_rgb, img, total_floats * sizeof(float), streams[0]);
        for (int d = 1; d < n && e == hipSuccess; ++d)
            if ((e = hipSetDevice(dev_of(d))) == hipSuccess) e = hipStreamSynchronize(streams[d]);
        if (e != hipSuccess) rc = fail(RTX_ERR_HIP, "band assembly: %s", hipGetErrorString(e));
        if (rc == RTX_OK && !out_rgb) *dev_img = img;
    } else if (rc == RTX_OK && kind == RTX_GATHER_HOST) {
        // band d holds the stripes d, d + n, ... (S rows each): one strided copy per band of its whole stripes
        // into the caller's rows, the partial last stripe separately (for a device image, rows of a host image that
        // then goes to device 0 in one copy: RCCL's fallback only)
        std::vector<float> host_img(out_rgb ? 0 : (size_t)H * W * 3);
        float* dst = out_rgb ? out_rgb : host_img.data();
        const size_t row_b = (size_t)W * 3 * sizeof(float);
        for (int d = 0; d < n && rc == RTX_OK; ++d) {
            const uint32_t rows = region_rows(&regs[d]);
            if (!rows) continue;
            const uint32_t full = rows / S, part = rows % S;  // whole stripes, rows of a partial last one
            hipError_t e = hipSetDevice(dev_of(d));
            if (e == hipSuccess && full)
                e = hipMemcpy2DAsync(dst + (size_t)d * S * W * 3, (size_t)n * S * row_b, bufs[d], S * row_b, S * row_b,
                                     full, hipMemcpyDeviceToHost, streams[d]);
            if (e == hipSuccess && part)
                e = hipMemcpyAsync(dst + (size_t)((size_t)full * n + d) * S * W * 3, bufs[d] + (size_t)full * S * W * 3,
                                   part * row_b, hipMemcpyDeviceToHost, streams[d]);
            if (e != hipSuccess) rc = fail(RTX_ERR_HIP, "band %d copy to the host", d);
        }
        for (int d = 0; d < n; ++d)
            if (hipSetDevice(dev_of(d)) == hipSuccess && hipStreamSynchronize(streams[d]) != hipSuccess && rc == RTX_OK)
                rc = fail(RTX_ERR_HIP, "band %d copy to the host", d);
        if (rc == RTX_OK && !out_rgb) {
            (void)hipSetDevice(0);
            if (!(img = static_cast<float*>(render_buffer(0, -2, img_bytes)))) rc = fail(RTX_ERR_OOM, "device-0 image");
            else if (hipMemcpyAsync(img, dst, img_bytes, hipMemcpyHostToDevice, streams[0]) != hipSuccess)
                rc = fail(RTX_ERR_HIP, "image copy to device 0");
            else *dev_img = img;
        }
        if (rc == RTX_OK && (hipSetDevice(0) != hipSuccess || hipEventRecord(g1, streams[0]) != hipSuccess ||
                             hipEventSynchronize(g1) != hipSuccess))
            rc = fail(RTX_ERR_HIP, "gather event");
    } else if (rc == RTX_OK) {  // one device, no gather: the band is the image
        (void)hipSetDevice(0);
        if (out_rgb) {
            hipError_t e = copy_to_host(out_rgb, bufs[0], img_bytes, streams[0]);
            if (e != hipSuccess) rc = fail(RTX_ERR_HIP, "copy image: %s", hipGetErrorString(e));
        } else {
            *dev_img = bufs[0];
        }
    }
    if (rc == RTX_OK && dev_stream) *dev_stream = streams[0];
    if (rc == RTX_OK && kind != RTX_GATHER_NONE) {
        float ms = 0.0f;
        if (hipSetDevice(0) == hipSuccess && hipEventElapsedTime(&ms, g0, g1) == hipSuccess) total.gather_ms = ms;
    }
    for (int d = 0; d < n; ++d)  // nothing of this call still in flight when the buffers are reused
        if (streams[d] && hipSetDevice(dev_of(d)) == hipSuccess) (void)hipStreamSynchronize(streams[d]);
    (void)hipSetDevice(cur);
    total.walk_layout = walk_layout(s, cam, tiered);
    total.gather_kind = kind;
    if (rc == RTX_OK && stats) *stats = total;
    return rc;
}
}  // namespace

int rtx_release_device_memory(int device) {
    g_last_error.clear();
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess) return fail(RTX_ERR_NO_DEVICE, "no HIP device");
    if (device < -1 || device >= ndev) return fail(RTX_ERR_INVALID_ARG, "device %d of %d", device, ndev);
    {
        std::lock_guard<std::mutex> lk(g_scratch_mu);
        for (auto& kv : g_scratch)
            if (device < 0 || kv.first == device) release_scratch_locked(kv.first);
    }
    {
        std::lock_guard<std::mutex> lk(g_ppm_mu);
        int cur = 0;
        (void)hipGetDevice(&cur);
        for (auto& kv : g_ppm)
            if ((device < 0 || kv.first == device) && kv.second.ptr && hipSetDevice(kv.first) == hipSuccess) {
                (void)hipFree(kv.second.ptr);
                kv.second = PpmScratch{};
            }
        (void)hipSetDevice(cur);
    }
    if (device < 0) {
        std::lock_guard<std::mutex> lk(g_stage_mu);
        release_stage_locked();
    }
    {
        std::lock_guard<std::mutex> lk(g_render_mu);
        release_render_locked(device);
    }
    {  // communicators span devices 0..n-1: any release drops them all
        std::lock_guard<std::mutex> lk(g_rccl_mu);
        release_comms_locked();
    }
    return RTX_OK;
}

int rtx_device_check(int device) {
    g_last_error.clear();
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(RTX_ERR_NO_DEVICE, "no HIP device");
    if (device < 0 || device >= ndev) return fail(RTX_ERR_INVALID_ARG, "device %d of %d", device, ndev);
    int cur = 0;
    HIP_TRY(hipGetDevice(&cur));
    HIP_TRY(hipSetDevice(device));
    const hipError_t e = hipDeviceSynchronize();  // every render enqueued on the device has ended
    const int rc = e == hipSuccess ? kerr_take(device)
                                   : fail(RTX_ERR_HIP, "hipDeviceSynchronize(%d): %s", device, hipGetErrorString(e));
    (void)hipSetDevice(cur);
    return rc;
}

uint64_t rtx_device_scratch_bytes(int device) {
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    auto it = g_scratch.find(device);
    return it == g_scratch.end() ? 0 : (uint64_t)it->second.bytes;
}

uint64_t rtx_ppm_max_bytes(uint32_t width, uint32_t height) { return rtxd::ppm_max_bytes(width, height); }

int rtx_encode_ppm_device(const float* d_rgb, uint32_t width, uint32_t height, char* d_text, uint64_t capacity,
                          uint64_t* out_len, void* hip_stream) {
    g_last_error.clear();
    if (!d_text || !out_len || (!d_rgb && (uint64_t)width * height)) return fail(RTX_ERR_INVALID_ARG, "NULL argument");
    const uint64_t n = (uint64_t)width * height;
    if (n > 0x7FFFFFFFull) return fail(RTX_ERR_INVALID_ARG, "image too large for the PPM encoder");
    const uint64_t need = rtxd::ppm_max_bytes(width, height);
    if (capacity < need) return fail(RTX_ERR_INVALID_ARG, "capacity %llu < rtx_ppm_max_bytes %llu",
                                     (unsigned long long)capacity, (unsigned long long)need);
    hipStream_t st = (hipStream_t)hip_stream;
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    char header[64];
    const uint64_t hl = rtxd::ppm_header(width, height, header);
    HIP_TRY(hipMemcpyAsync(d_text, header, hl, hipMemcpyHostToDevice, st));
    HIP_TRY(hipStreamSynchronize(st));  // the header's stack buffer must outlive the copy
    uint64_t total = hl;
    if (n) {
        size_t sb = 0;
        HIP_TRY(rtxd::ppm_scratch_bytes(n, &sb));
        std::lock_guard<std::mutex> lk(g_ppm_mu);  // held until the encode has finished
        PpmScratch& ps = g_ppm[dev];
        if (ps.bytes < sb) {
            if (ps.ptr) HIP_TRY(hipFree(ps.ptr));
            ps = PpmScratch{};
            HIP_TRY(hipMalloc(&ps.ptr, sb));
            ps.bytes = sb;
        }
        uint64_t last_off = 0;
        uint32_t last_len = 0;
        hipError_t e = rtxd::ppm_encode(d_rgb, width, height, d_text, ps.ptr, ps.bytes, hl, st);
        if (e == hipSuccess) e = hipMemcpyAsync(&last_off, rtxd::ppm_last_offset(ps.ptr, n), 8, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipMemcpyAsync(&last_len, rtxd::ppm_last_length(ps.ptr, n), 4, hipMemcpyDeviceToHost, st);
        const hipError_t es = hipStreamSynchronize(st);  // always: the copies target this frame
        HIP_TRY(e);
        HIP_TRY(es);
        total += last_off + last_len;
    }
    *out_len = total;
    return RTX_OK;
}

int rtx_render_ppm(rtx_scene* s, const rtx_camera* cam, uint64_t seed, char* out_text, uint64_t capacity,
                   uint64_t* out_len, rtx_stats* stats) {
    g_last_error.clear();
    if (!s || !out_text || !out_len) return fail(RTX_ERR_INVALID_ARG, "NULL argument");
    if (int rc = check_camera(cam)) return rc;
    const uint32_t W = cam->image_width, H = cam->image_height;
    const uint64_t need = rtxd::ppm_max_bytes(W, H);
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(s->mu);  // (lock order: the scene, then the render buffers)
    std::lock_guard<std::mutex> bl(g_render_mu);  // the cached image / text buffers and stream
    hipStream_t st = render_stream(dev);
    float* rgb = static_cast<float*>(render_buffer(dev, -3, std::max<size_t>(1, (size_t)W * H * 3 * sizeof(float))));
    char* text = static_cast<char*>(render_buffer(dev, -4, need));
    if (!st) return fail(RTX_ERR_HIP, "stream on device %d", dev);
    if (!rgb || !text) return fail(RTX_ERR_OOM, "device buffers for a %ux%u PPM", W, H);
    rtx_region reg{0, 0, W, H, 0, 1};
    rtx_stats local;
    int rc = render_region_locked(s, cam, seed, &reg, rgb, st, 0, stats ? stats : &local);
    uint64_t len = 0;
    if (rc == RTX_OK) rc = rtx_encode_ppm_device(rgb, W, H, text, need, &len, st);
    if (rc == RTX_OK && len > capacity) rc = fail(RTX_ERR_INVALID_ARG, "capacity %llu < PPM length %llu",
                                                  (unsigned long long)capacity, (unsigned long long)len);
    if (rc == RTX_OK && copy_to_host(out_text, text, len, st) != hipSuccess)
        rc = fail(RTX_ERR_HIP, "copying the PPM text to the host");
    (void)hipStreamSynchronize(st);
    if (rc == RTX_OK) *out_len = len;
    return rc;
}

int rtx_render_ppm_ex(rtx_scene* s, const rtx_camera* cam, uint64_t seed, int n_gpus, char* out_text, uint64_t capacity,
                      uint64_t* out_len, rtx_stats* stats) {
    g_last_error.clear();
    if (!s || !out_text || !out_len) return fail(RTX_ERR_INVALID_ARG, "NULL argument");
    if (int rc = check_camera(cam)) return rc;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(RTX_ERR_NO_DEVICE, "no HIP device");
    if (n_gpus <= 0) n_gpus = 1;
    if (n_gpus > ndev) return fail(RTX_ERR_INVALID_ARG, "n_gpus=%d but %d devices visible", n_gpus, ndev);
    const uint32_t W = cam->image_width, H = cam->image_height;
    const uint64_t need = rtxd::ppm_max_bytes(W, H);
    int cur = 0;
    HIP_TRY(hipGetDevice(&cur));
    std::lock_guard<std::mutex> lk(s->mu);  // (lock order: the scene, then the render buffers)
    std::lock_guard<std::mutex> bl(g_render_mu);
    float* img = nullptr;
    hipStream_t st = nullptr;
    rtx_stats local;
    // the bands rendered and assembled on device 0 as rtx_render_ex does, the image left there
    int rc = render_bands_locked(s, cam, seed, n_gpus, 0u, nullptr, &img, &st, stats ? stats : &local);
    if (rc == RTX_OK && hipSetDevice(0) != hipSuccess) rc = fail(RTX_ERR_HIP, "hipSetDevice(0)");
    char* text = rc == RTX_OK ? static_cast<char*>(render_buffer(0, -4, need)) : nullptr;
    if (rc == RTX_OK && !text) rc = fail(RTX_ERR_OOM, "device-0 buffer for a %ux%u PPM", W, H);
    uint64_t len = 0;
    if (rc == RTX_OK) rc = rtx_encode_ppm_device(img, W, H, text, need, &len, st);
    if (rc == RTX_OK && len > capacity) rc = fail(RTX_ERR_INVALID_ARG, "capacity %llu < PPM length %llu",
                                                  (unsigned long long)capacity, (unsigned long long)len);
    if (rc == RTX_OK && copy_to_host(out_text, text, len, st) != hipSuccess)
        rc = fail(RTX_ERR_HIP, "copying the PPM text to the host");
    if (st) (void)hipStreamSynchronize(st);
    (void)hipSetDevice(cur);
    if (rc == RTX_OK) *out_len = len;
    return rc;
}

}  // extern "C"
