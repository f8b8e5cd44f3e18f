// runtime.hip — host side of libpathtracer.so: the C ABI of include/pt_api.h.
//
// Replaces the reference's Vulkan integrator host (src/integrator/basic.cpp,
// src/integrator/integrator.cpp:15-87) and scene upload
// (src/scene/scene.cpp:1643-2006) with HIP: device buffers for the packed
// scene, a float4 sample buffer, SoA slot buffers, and kernel launches on one
// stream per device.  Scene packs are validated on the host before upload so
// that no index in them can send a kernel out of bounds or into a cycle.
#include "pt_device.hpp"
#include "kernels.hpp"
#include "../../../include/pt_api.h"

#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

thread_local std::string g_last_error;

void SetError(const char* fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
}

#define PT_HIP(call)                                                                         \
    do {                                                                                     \
        hipError_t e_ = (call);                                                              \
        if (e_ != hipSuccess) {                                                              \
            SetError("%s failed: %s (%s:%d)", #call, hipGetErrorString(e_), __FILE__, __LINE__); \
            return (int)e_;                                                                  \
        }                                                                                    \
    } while (0)

template <class T>
struct dbuf {
    T* ptr = nullptr;
    size_t count = 0;
    void release() { if (ptr) (void)hipFree(ptr); ptr = nullptr; count = 0; }
    hipError_t upload(const T* src, size_t n)
    {
        // An empty array still gets one zeroed element, so that kernels which
        // read a first record unconditionally (the TLAS root in LaneBegin)
        // read defined memory in a scene without shapes.
        if (!ptr || n > count) {
            release();
            hipError_t e = hipMalloc(&ptr, std::max<size_t>(n, 1) * sizeof(T));
            if (e != hipSuccess) { ptr = nullptr; return e; }
            count = n;
        }
        if (n == 0) return hipMemset(ptr, 0, sizeof(T));
        return hipMemcpy(ptr, src, n * sizeof(T), hipMemcpyHostToDevice);
    }
    hipError_t alloc(size_t n)
    {
        if (n <= count && ptr) return hipSuccess;
        release();
        hipError_t e = hipMalloc(&ptr, std::max<size_t>(n, 1) * sizeof(T));
        if (e != hipSuccess) { ptr = nullptr; return e; }
        count = n;
        return hipSuccess;
    }
};

struct event_pair { hipEvent_t a, b; int kernel; uint32_t rounds; hipStream_t stream; };

}  // namespace

struct pt_device {
    int id = 0;
    hipStream_t stream = nullptr;
    uint32_t cu_count = 256;
    bool profiling = false;
    uint32_t profile_period = 1;   // time every period-th Run call
    uint64_t run_tick = 0;
    std::vector<event_pair> pending;
    std::vector<event_pair> free_events;
    // Live RCCL communicators on this device: while one exists, the blocking
    // calls wait for the stream by polling it together with RCCL's
    // asynchronous error state and a deadline (DeviceWait), so a collective
    // whose peer died returns an error instead of hanging.
    std::vector<pt_comm*> comms;
    bool comm_failed = false;      // a communicator was aborted: waits keep a short deadline
    uint64_t launches[PT_KERNEL_COUNT] = {};
    uint64_t rounds[PT_KERNEL_COUNT] = {};    // rounds the timed launches covered (a batch: its rounds)
    double total_ms[PT_KERNEL_COUNT] = {};
    // Tile-group streams (ptSetBasicRendererSplit): groups 1.. of a batch of
    // rounds run on these, forked from `stream` and joined back into it, so
    // every wait on `stream` covers them.  Created on first use.
    hipStream_t group_stream[PT_MAX_SPLIT - 1] = {};
    hipEvent_t fork_event = nullptr;
    hipEvent_t join_event[PT_MAX_SPLIT - 1] = {};
};

struct pt_scene {
    pt_device* dev = nullptr;
    ptd::dscene d{};
    dbuf<pt_packed_texture> textures;
    dbuf<uint32_t> material;
    dbuf<pt_packed_shape> shapes;        // device copy: Pad0 = PT_SHAPE_FLAG_UV when the material reads UVs
    dbuf<pt_packed_shape_node> shape_nodes;
    dbuf<pt_packed_mesh_face> faces;
    dbuf<pt_packed_mesh_vertex> vertices;
    dbuf<float4> vertex_attr;            // decoded vertex normals + U (vertex_decode_kernel)
    dbuf<float> vertex_v;                // decoded V
    dbuf<pt_packed_mesh_node> mesh_nodes;
    dbuf<pt_packed_camera> cameras;
    dbuf<float> atlas;
    bool atlas_tiled = false;    // atlas in AtlasIndex 4x2-texel blocks
    uint32_t camera_count = 0;
    uint32_t stack_needed = 0;   // max traversal stack entries (TLAS + BLAS)
    uint32_t mats = PT_MATS_ALL | PT_MATS_SCENE; // SceneMaterialMask (shade specialisation)
    uint32_t stack_format = PT_STACK_FORMAT_AUTO;   // ptSetSceneStackFormat (applied at the next update)
    uint32_t hit_record = PT_HIT_RECORD_AUTO;       // ptSetSceneHitRecordForm (applied at the next update)
    uint32_t cached_pairs = 0;   // BLAS child pairs at the front of the device node array (NodeCacheLayout)
    bool blas_packable = false;  // BlasWordsPackable / BlasWords16FirstBits of the device node layout
    uint32_t blas16_bits = 0;
    bool valid = false;
};

struct pt_sample_buffer {
    pt_device* dev = nullptr;
    uint32_t width = 0, height = 0;
    float4* accum = nullptr;
    dbuf<float4> display;      // resolved image (ptRenderSampleBuffer)
    dbuf<uint32_t> display8;   // its sRGB8 encoding
    bool resolved = false;
    uint32_t rank = 0, nranks = 1;   // pixel bands of the last partitioned renderer created on it
};

struct pt_preview {
    pt_device* dev = nullptr;
    pt_scene* scene = nullptr;           // non-owning (preview_render.hpp:20)
    uint32_t width = 0, height = 0;
    dbuf<float4> image;
    dbuf<pt_preview_aov> aov;
    dbuf<uint32_t> spill;
    dbuf<float> observe;                 // ObserveUnderD65's per-sample constants (preview.hip)
    uint32_t* query = nullptr;
    bool rendered = false;
};

namespace {
// Automatic mode's batch for a renderer whose tiles all fit on the GPU at
// once (RoundFused's condition): one launch per AUTO_BATCH rounds.
constexpr uint32_t AUTO_BATCH = 16;
}  // namespace

struct pt_basic_renderer {
    pt_basic_renderer_params params{};
    pt_device* dev = nullptr;
    pt_scene* scene = nullptr;          // non-owning (basic.hpp:8,21)
    pt_sample_buffer* buffer = nullptr; // non-owning
    uint32_t rank = 0, nranks = 1;
    uint32_t tiles_x = 0;
    ptd::dslots slots{};
    dbuf<float4> ray, hit, thr, prob;
    dbuf<float> prob1;                  // grey record form's Probability (kernels.hip StorePathVertex)
    bool grey = false;                  // the live paths are in the grey record form (slots.prob1 set)
    bool grey_blocked = false;          // some live path cannot take it (until the next Reset / state write)
    dbuf<uint32_t> grey_count;          // pt_launch_grey_check's result word
    dbuf<uint32_t> cq_counts, cq_list;  // class-pure shade lists (ClassLists)
    uint32_t cq_parity = 0;
    uint32_t class_lists = 0;           // ptSetBasicRendererClassLists: 0 automatic, 1 off
    dbuf<float> lam;                    // lambda0 per slot (Sample is 0 between rounds)
    dbuf<float2> uv;
    dbuf<uint2> act;
    dbuf<uint16_t> pos;                 // TileOrder positions (kernels.hip)
    dbuf<uint8_t> slotof;               // position -> slot within the tile
    dbuf<uint64_t> outcome;             // ShadeOrder: outcome-class bits per tile (extend -> shade)
    dbuf<uint32_t> tilecost, order;     // longest-first tile order (extend -> tile_order -> extend)
    uint64_t order_tick = 0;            // rounds since creation (tile-order re-sort period)
    dbuf<uint32_t> done;                // per wave: completed paths since the last Reset (ptGetStats)
    int fused = 1;                      // fused rounds mode (ptSetBasicRendererFusedRounds)
    int openpbr = 0;                    // shade OpenPBR materials (ptSetBasicRendererOpenPBR)
    uint32_t round_batch = 0;           // rounds per launch of consecutive Run(1) rounds (0: automatic)
    uint32_t split = 0;                 // tile groups of consecutive rounds (ptSetBasicRendererSplit): 0 auto, 1 off
    dbuf<uint32_t> guard;               // guarded rounds' {stop, rounds run} (ptRenderFrame)
    uint32_t order_groups = 1;          // the group structure the order array holds (tile_order_kernel)
    uint64_t pixels = 0;                // image pixels owned
    uint32_t streams = 1;               // path streams per owned pixel (ptCreateBasicRendererStreams)
    uint32_t stream_tiles = 0;          // tiles per stream
    uint64_t valid_slots = 0;           // streams x pixels: the paths of one round
    dbuf<float4> accx;                  // streams > 1: each stream's accumulator (streams x width x height)
    uint64_t rays = 0;                  // rays traced since the last Reset
    dbuf<uint32_t> spill;
};

struct pt_comm {
    pt_device* dev = nullptr;
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
    double timeout_s = 600.0;     // ptCommSetTimeout
    bool aborted = false;
    int* flag = nullptr;          // device word of the collective argument check (CommAgree)
    int* host_flag = nullptr;     // its pinned host copy: the readback stays an asynchronous copy
                                  // that DeviceWait polls, and outlives a wait that times out
};

namespace {

// Aborts every communicator of the device (ncclCommAbort: RCCL stops their
// kernels) after a failed or overdue collective.
void AbortComms(pt_device* dev)
{
    for (pt_comm* c : dev->comms) {
        if (c->comm) (void)ncclCommAbort(c->comm);
        c->comm = nullptr;
        c->aborted = true;
    }
    dev->comms.clear();
    dev->comm_failed = true;
}

// Waits until the device stream is idle.  With no communicator: one
// hipStreamSynchronize.  With live communicators: polls the stream, each
// communicator's asynchronous error (ncclCommGetAsyncError) and the shortest
// communicator deadline; on an RCCL error or at the deadline every
// communicator is aborted and PT_ERROR_COMM_ABORTED / PT_ERROR_TIMEOUT
// returned.  After an abort, waits give up after 10 s (PT_ERROR_TIMEOUT).
int DeviceWait(pt_device* dev)
{
    if (dev->comms.empty() && !dev->comm_failed) {
        PT_HIP(hipStreamSynchronize(dev->stream));
        return 0;
    }
    double limit = dev->comm_failed ? 10.0 : 1e30;
    for (pt_comm* c : dev->comms) limit = std::min(limit, c->timeout_s);
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 0;; spin++) {
        hipError_t q = hipStreamQuery(dev->stream);
        if (q == hipSuccess) {
            if (dev->comms.empty()) dev->comm_failed = false;   // drained since the abort
            return 0;
        }
        if (q != hipErrorNotReady) {
            SetError("device stream: %s", hipGetErrorString(q));
            return (int)q;
        }
        for (pt_comm* c : dev->comms) {
            ncclResult_t st = ncclSuccess;
            ncclResult_t r = ncclCommGetAsyncError(c->comm, &st);
            if (r != ncclSuccess || (st != ncclSuccess && st != ncclInProgress)) {
                SetError("RCCL communicator (rank %d of %d) failed: %s; communicators aborted", c->rank, c->nranks,
                         ncclGetErrorString(r != ncclSuccess ? r : st));
                AbortComms(dev);
                return PT_ERROR_COMM_ABORTED;
            }
        }
        const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (el > limit) {
            SetError("device stream not idle after %.1f s with a live communicator (a peer rank failed or stalled); "
                     "communicators aborted", el);
            AbortComms(dev);
            return PT_ERROR_TIMEOUT;
        }
        if (spin > 64) std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

#define PT_WAIT(dev)                                    \
    do {                                                \
        if (int w_ = DeviceWait(dev)) return w_;        \
    } while (0)

int BeginTimed(pt_device* dev, int kernel, event_pair& ep, bool sampled = true, uint32_t rounds = 1)
{
    ep.kernel = -1;
    if (!dev->profiling || !sampled) return 0;
    if (!dev->free_events.empty()) { ep = dev->free_events.back(); dev->free_events.pop_back(); }
    else {
        PT_HIP(hipEventCreate(&ep.a));
        PT_HIP(hipEventCreate(&ep.b));
    }
    ep.kernel = kernel;
    ep.rounds = rounds;
    ep.stream = dev->stream;
    PT_HIP(hipEventRecord(ep.a, ep.stream));
    return 0;
}

int EndTimed(pt_device* dev, event_pair& ep)
{
    if (!dev->profiling || ep.kernel < 0) return 0;
    PT_HIP(hipEventRecord(ep.b, ep.stream));
    dev->pending.push_back(ep);
    return 0;
}

int CollectTimes(pt_device* dev)
{
    if (dev->pending.empty()) return 0;
    PT_WAIT(dev);
    for (event_pair& ep : dev->pending) {
        float ms = 0;
        PT_HIP(hipEventElapsedTime(&ms, ep.a, ep.b));
        dev->launches[ep.kernel] += 1;
        dev->rounds[ep.kernel] += ep.rounds;
        dev->total_ms[ep.kernel] += ms;
        dev->free_events.push_back(ep);
    }
    dev->pending.clear();
    return 0;
}

// --- pack validation --------------------------------------------------------------

bool TexOk(uint32_t t, uint32_t n) { return t == PT_TEXTURE_INDEX_NONE || t < n; }

// Depth (edges on the longest root-leaf path) of the TLAS, or -1 if malformed.
int TlasDepth(const pt_scene_packs* p)
{
    uint32_t n = p->shape_node_count;
    struct item { uint32_t node, depth; };
    std::vector<item> st{{0, 0}};
    int maxd = 0;
    size_t visits = 0;
    while (!st.empty()) {
        item it = st.back(); st.pop_back();
        if (++visits > (size_t)n) return -1;   // cycle or shared children
        const pt_packed_shape_node& N = p->shape_nodes[it.node];
        maxd = std::max<int>(maxd, (int)it.depth);
        if (N.ChildNodeIndices == 0) {
            if (N.ShapeIndex >= p->shape_count) return -1;
        } else {
            uint32_t a = N.ChildNodeIndices & 0xFFFF, b = N.ChildNodeIndices >> 16;
            if (a >= n || b >= n) return -1;
            st.push_back({a, it.depth + 1});
            st.push_back({b, it.depth + 1});
        }
    }
    return maxd;
}

int BlasDepth(const pt_scene_packs* p, uint32_t root)
{
    uint32_t n = p->mesh_node_count;
    if (root >= n) return -1;
    struct item { uint32_t node, depth; };
    std::vector<item> st{{root, 0}};
    int maxd = 0;
    size_t visits = 0;
    while (!st.empty()) {
        item it = st.back(); st.pop_back();
        if (++visits > (size_t)n) return -1;
        const pt_packed_mesh_node& N = p->mesh_nodes[it.node];
        maxd = std::max<int>(maxd, (int)it.depth);
        if (N.FaceEndIndex > 0) {
            if (N.FaceBeginOrNodeIndex > N.FaceEndIndex || N.FaceEndIndex > p->mesh_face_count) return -1;
        } else {
            uint32_t c = N.FaceBeginOrNodeIndex;
            if (c + 1 >= n || c + 1 < c) return -1;
            st.push_back({c, it.depth + 1});
            st.push_back({c + 1, it.depth + 1});
        }
    }
    return maxd;
}

bool MaterialOk(const pt_scene_packs* p, uint32_t m)
{
    if ((uint64_t)m * 32 + 32 > p->material_word_count) return false;
    const uint32_t* A = p->material_data + 32 * m;
    uint32_t nt = p->texture_count;
    switch (A[0]) {
        case PT_MATERIAL_TYPE_BASIC_DIFFUSE: return TexOk(A[PT_BASIC_DIFFUSE_BASE_SPECTRUM + 3], nt);
        case PT_MATERIAL_TYPE_BASIC_METAL:
            return TexOk(A[PT_BASIC_METAL_BASE_SPECTRUM + 3], nt) && TexOk(A[PT_BASIC_METAL_SPECULAR_SPECTRUM + 3], nt) &&
                   TexOk(A[PT_BASIC_METAL_ROUGHNESS + 1], nt) && TexOk(A[PT_BASIC_METAL_ROUGHNESS_ANISOTROPY + 1], nt);
        case PT_MATERIAL_TYPE_BASIC_TRANSLUCENT:
            return TexOk(A[PT_BASIC_TRANSLUCENT_ROUGHNESS + 1], nt) && TexOk(A[PT_BASIC_TRANSLUCENT_ROUGHNESS_ANISOTROPY + 1], nt);
        default: return true;   // not shaded by the integrator
    }
}

int ValidatePacks(const pt_scene_packs* p, uint32_t* stack_needed)
{
    if (!p || !p->globals) { SetError("packs: globals missing"); return -1; }
    const pt_packed_scene_globals& g = *p->globals;
    if (g.ShapeCount != 0) {
        if (g.ShapeCount != p->shape_count) { SetError("packs: ShapeCount %u != shape_count %u", g.ShapeCount, p->shape_count); return -1; }
        if (p->shape_node_count == 0) { SetError("packs: no shape nodes"); return -1; }
    }
    if (p->shape_count > 65535 || p->shape_node_count > 65536) { SetError("packs: more than 65535 shapes (16-bit indices)"); return -1; }
    if (!TexOk(g.SkyboxTextureIndex, p->texture_count)) { SetError("packs: bad skybox texture"); return -1; }
    if (p->texture_count > 0 && (!p->atlas || p->atlas_layer_count == 0 || p->atlas_width == 0 || p->atlas_height == 0)) {
        SetError("packs: textures without atlas"); return -1;
    }
    for (uint32_t i = 0; i < p->mesh_face_count; i++) {
        const pt_packed_mesh_face& F = p->mesh_faces[i];
        if (F.VertexIndex0 >= p->mesh_vertex_count || F.VertexIndex1 >= p->mesh_vertex_count ||
            F.VertexIndex2 >= p->mesh_vertex_count) { SetError("packs: face %u vertex out of range", i); return -1; }
    }
    int blas = 0;
    for (uint32_t i = 0; i < p->shape_count; i++) {
        const pt_packed_shape& S = p->shapes[i];
        if (S.Type < 0 || S.Type > 3) { SetError("packs: shape %u bad type", i); return -1; }
        if (!MaterialOk(p, S.MaterialIndex)) { SetError("packs: shape %u bad material %u", i, S.MaterialIndex); return -1; }
        if (S.Type == PT_SHAPE_TYPE_MESH_INSTANCE) {
            int d = BlasDepth(p, S.MeshRootNodeIndex);
            if (d < 0) { SetError("packs: shape %u mesh BVH malformed", i); return -1; }
            blas = std::max(blas, d);
        }
    }
    int tlas = 0;
    if (g.ShapeCount != 0) {
        tlas = TlasDepth(p);
        if (tlas < 0) { SetError("packs: shape BVH malformed"); return -1; }
    }
    *stack_needed = (uint32_t)(std::min(tlas, 32) + std::min(blas, 32));
    return 0;
}

ptd::dframe Frame(pt_basic_renderer* r)
{
    ptd::dframe F;
    F.accum = r->buffer->accum;
    F.width = r->buffer->width;
    F.height = r->buffer->height;
    F.rank = r->rank;
    F.nranks = r->nranks;
    F.tiles_x = r->tiles_x;
    F.tiles_x_magic = r->tiles_x > 1 ? (uint32_t)(((1ull << 32) + r->tiles_x - 1) / r->tiles_x) : 0u;
    F.streams = r->streams;
    F.stream_tiles = r->stream_tiles;
    F.stream_magic = r->streams > 1 ? (uint32_t)(((1ull << 32) + r->stream_tiles - 1) / r->stream_tiles) : 0u;
    F.accx = r->accx.ptr;
    return F;
}

ptd::dparams Params(pt_basic_renderer* r, uint32_t seed)
{
    ptd::dparams P;
    P.camera_index = r->params.CameraIndex;
    P.render_flags = r->params.RenderFlags;
    P.termination_probability = r->params.PathTerminationProbability;
    P.seed = seed;
    return P;
}

// Traversal stack entries beyond the kernel's LDS capacity live in a global
// buffer of (needed - capacity) rows x one column per ray.
int EnsureSpill(pt_basic_renderer* r)
{
    uint32_t need = r->scene->stack_needed, cap = pt_extend_stack_cap();
    if (need <= cap) { r->slots.spill = nullptr; return 0; }
    size_t rows = need - cap;
    PT_HIP(r->spill.alloc(rows * (size_t)r->slots.n));
    r->slots.spill = r->spill.ptr;
    return 0;
}

int CheckReady(pt_basic_renderer* r)
{
    if (!r || !r->scene || !r->buffer) { SetError("renderer: null"); return -1; }
    if (!r->scene->valid) { SetError("renderer: scene has no valid packs (call ptUpdateScene)"); return -1; }
    if (r->params.CameraIndex >= r->scene->camera_count) {
        SetError("renderer: CameraIndex %u >= camera count %u", r->params.CameraIndex, r->scene->camera_count);
        return -1;
    }
    return 0;
}

}  // namespace

extern "C" {

const char* ptGetLastError(void) { return g_last_error.c_str(); }

int ptGetDeviceCount(int* count)
{
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    *count = n;
    return 0;
}

pt_device* ptCreateDevice(int hip_device)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) { SetError("no HIP device available"); return nullptr; }
    if (hip_device < 0 || hip_device >= n) { SetError("device %d out of range (%d devices)", hip_device, n); return nullptr; }
    if (hipSetDevice(hip_device) != hipSuccess) { SetError("hipSetDevice(%d) failed", hip_device); return nullptr; }
    pt_device* d = new pt_device;
    d->id = hip_device;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, hip_device) == hipSuccess && prop.multiProcessorCount > 0)
        d->cu_count = (uint32_t)prop.multiProcessorCount;
    if (hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking) != hipSuccess) {
        SetError("device stream creation failed");
        if (d->stream) (void)hipStreamDestroy(d->stream);
        delete d;
        return nullptr;
    }
    return d;
}

void ptDestroyDevice(pt_device* d)
{
    if (!d) return;
    (void)hipSetDevice(d->id);
    (void)DeviceWait(d);
    // Communicators outliving their device: detached (ptCommDestroy still
    // releases them; every exchange on them fails).
    for (pt_comm* c : d->comms) c->dev = nullptr;
    d->comms.clear();
    for (auto& ep : d->pending) { (void)hipEventDestroy(ep.a); (void)hipEventDestroy(ep.b); }
    for (auto& ep : d->free_events) { (void)hipEventDestroy(ep.a); (void)hipEventDestroy(ep.b); }
    for (uint32_t g = 0; g + 1 < PT_MAX_SPLIT; g++) {
        if (d->group_stream[g]) (void)hipStreamDestroy(d->group_stream[g]);
        if (d->join_event[g]) (void)hipEventDestroy(d->join_event[g]);
    }
    if (d->fork_event) (void)hipEventDestroy(d->fork_event);
    (void)hipStreamDestroy(d->stream);
    delete d;
}

int ptSynchronize(pt_device* d)
{
    if (!d) { SetError("null device"); return -1; }
    PT_HIP(hipSetDevice(d->id));
    PT_WAIT(d);
    return 0;
}

pt_scene* ptCreateScene(pt_device* d)
{
    if (!d) { SetError("null device"); return nullptr; }
    pt_scene* s = new pt_scene;
    s->dev = d;
    return s;
}

void ptDestroyScene(pt_device* d, pt_scene* s)
{
    if (!s) return;
    if (d) (void)hipSetDevice(d->id);
    s->textures.release(); s->material.release(); s->shapes.release(); s->shape_nodes.release();
    s->faces.release(); s->vertices.release(); s->vertex_attr.release(); s->vertex_v.release(); s->mesh_nodes.release(); s->cameras.release(); s->atlas.release();
    delete s;
}

int ptSetSceneStackFormat(pt_scene* s, uint32_t format)
{
    if (!s || format > PT_STACK_FORMAT_NODE_INDEX) { SetError("ptSetSceneStackFormat: bad argument"); return -1; }
    s->stack_format = format;
    return 0;
}

int ptSetSceneHitRecordForm(pt_scene* s, uint32_t form)
{
    if (!s || form > PT_HIT_RECORD_FACE_INDEX) { SetError("ptSetSceneHitRecordForm: bad argument"); return -1; }
    s->hit_record = form;
    return 0;
}

// UpdateVulkanScene (scene.cpp:1692-2006): synchronous upload of the packs.
// Box-coordinate condition of the extend kernel's exact fast slab division
// (pt_device.hpp, IntersectBoundingBox): every TLAS / BLAS bound is 0 or has
// magnitude in [2^-50, 2^40].  Scenes outside it trace with IEEE division.
static bool FastDivBoxes(const pt_scene_packs* p)
{
    auto ok = [](float c) {
        float m = std::fabs(c);
        return m == 0.0f || (m >= 0x1p-50f && m <= 0x1p40f);
    };
    for (uint32_t i = 0; i < p->shape_node_count; i++)
        for (int k = 0; k < 3; k++)
            if (!ok(p->shape_nodes[i].Minimum[k]) || !ok(p->shape_nodes[i].Maximum[k])) return false;
    for (uint32_t i = 0; i < p->mesh_node_count; i++)
        for (int k = 0; k < 3; k++)
            if (!ok(p->mesh_nodes[i].Minimum[k]) || !ok(p->mesh_nodes[i].Maximum[k])) return false;
    return true;
}

// Whether every BLAS node's index words fit one packed stack entry
// (PackBlasEntry): leaves with <= 31 faces starting below 2^26, child-pair
// indices below 2^31.
static bool BlasWordsPackable(const pt_scene_packs* p)
{
    for (uint32_t i = 0; i < p->mesh_node_count; i++) {
        const pt_packed_mesh_node& n = p->mesh_nodes[i];
        if (n.FaceEndIndex > 0) {
            if (n.FaceBeginOrNodeIndex >= (1u << 26) || n.FaceEndIndex < n.FaceBeginOrNodeIndex ||
                n.FaceEndIndex - n.FaceBeginOrNodeIndex > 31)
                return false;
        } else if (n.FaceBeginOrNodeIndex >= 0x80000000u) {
            return false;
        }
    }
    return true;
}

// The 16-bit stack format (PackBlasEntry16): returns the bits F of a leaf's
// first face index, or 0 if some entry does not fit.  Internal entries are
// child-pair indices < 2^15; a leaf needs first < 2^F and count < 2^(15-F)
// for one F; TLAS entries are node indices < 2^16 (ValidatePacks).
static uint32_t BlasWords16FirstBits(const pt_scene_packs* p)
{
    if (p->shape_node_count > 65536) return 0;
    uint32_t max_first = 0, max_count = 0;
    for (uint32_t i = 0; i < p->mesh_node_count; i++) {
        const pt_packed_mesh_node& n = p->mesh_nodes[i];
        if (n.FaceEndIndex > 0) {
            if (n.FaceEndIndex < n.FaceBeginOrNodeIndex) return 0;
            max_first = std::max(max_first, n.FaceBeginOrNodeIndex);
            max_count = std::max(max_count, n.FaceEndIndex - n.FaceBeginOrNodeIndex);
        } else if (n.FaceBeginOrNodeIndex >= 0x8000u) {
            return 0;
        }
    }
    for (uint32_t F = 1; F < 15; F++)
        if (max_first < (1u << F) && max_count < (1u << (15 - F))) return F;
    return 0;
}

// Whether shading a hit on material m reads the hit's texture coordinates:
// some texture index among the fields its BSDF reads (MaterialOk's list, and
// OpenPBR's base colour and specular roughness textures) is set.  Hits on
// other materials skip computing their UV (HitAttributesV).
static bool MaterialReadsUV(const pt_scene_packs* p, uint32_t m)
{
    const uint32_t* A = p->material_data + 32 * (size_t)m;
    auto tx = [&](uint32_t w) { return A[w] != PT_TEXTURE_INDEX_NONE; };
    switch (A[0]) {
        case PT_MATERIAL_TYPE_BASIC_DIFFUSE: return tx(PT_BASIC_DIFFUSE_BASE_SPECTRUM + 3);
        case PT_MATERIAL_TYPE_BASIC_METAL:
            return tx(PT_BASIC_METAL_BASE_SPECTRUM + 3) || tx(PT_BASIC_METAL_SPECULAR_SPECTRUM + 3) ||
                   tx(PT_BASIC_METAL_ROUGHNESS + 1) || tx(PT_BASIC_METAL_ROUGHNESS_ANISOTROPY + 1);
        case PT_MATERIAL_TYPE_BASIC_TRANSLUCENT:
            return tx(PT_BASIC_TRANSLUCENT_ROUGHNESS + 1) || tx(PT_BASIC_TRANSLUCENT_ROUGHNESS_ANISOTROPY + 1);
        case PT_MATERIAL_TYPE_OPENPBR:
            return tx(PT_OPENPBR_BASE_SPECTRUM_TEXTURE_INDEX) || tx(PT_OPENPBR_SPECULAR_ROUGHNESS_TEXTURE_INDEX);
        default: return false;   // not shaded: the path ends
    }
}

// LDS node cache layout (the extend kernel's NodeCacheFill, pt_device.hpp
// PT_NODE_CACHE_PAIRS): the BLAS child pairs in breadth-first order from every
// mesh root -- the top levels, which most node fetches of a frame read (C3:
// the first 6 levels, 120 pairs, take 59 % of the internal-node visits) --
// the first PT_NODE_CACHE_PAIRS of them moved to the front of the device node
// array (pair j at nodes 2j, 2j+1), every other node after them in its
// original order, child-pair and root indices remapped.  The numbering enters
// no result: the traversal's decisions read only the nodes' bounds and face
// ranges, so a renumbered BVH is traversed in the same order to the same
// hits.  Returns the cached pair count, 0 (and the identity layout) when some
// node is the first child of one pair and the second of another, which no
// layout of adjacent pairs can hold.
static uint32_t NodeCacheLayout(const pt_scene_packs* p, std::vector<pt_packed_mesh_node>& out,
                                std::vector<uint32_t>& remap)
{
    const uint32_t n = p->mesh_node_count;
    const pt_packed_mesh_node* in = p->mesh_nodes;
    out.assign(in, in + n);
    remap.resize(n);
    for (uint32_t i = 0; i < n; i++) remap[i] = i;
    if (n < 3) return 0;
    std::vector<uint8_t> role(n, 0);   // 1: first node of a child pair, 2: second
    for (uint32_t i = 0; i < n; i++) {
        if (in[i].FaceEndIndex > 0) continue;
        const uint32_t c = in[i].FaceBeginOrNodeIndex;
        if (c + 1 >= n) return 0;
        role[c] |= 1;
        role[c + 1] |= 2;
    }
    for (uint32_t i = 0; i < n; i++)
        if (role[i] == 3) return 0;
    std::vector<uint32_t> cached, queue;
    std::vector<uint8_t> seen(n, 0);
    for (uint32_t k = 0; k < p->shape_count; k++) {
        if (p->shapes[k].Type != PT_SHAPE_TYPE_MESH_INSTANCE) continue;
        const uint32_t r = p->shapes[k].MeshRootNodeIndex;
        if (r < n && in[r].FaceEndIndex == 0) queue.push_back(in[r].FaceBeginOrNodeIndex);
    }
    for (size_t h = 0; h < queue.size() && cached.size() < PT_NODE_CACHE_PAIRS; h++) {
        const uint32_t c = queue[h];
        if (seen[c]) continue;
        seen[c] = 1;
        cached.push_back(c);
        for (uint32_t m = c; m <= c + 1; m++)
            if (in[m].FaceEndIndex == 0) queue.push_back(in[m].FaceBeginOrNodeIndex);
    }
    if (cached.empty()) return 0;
    std::vector<uint8_t> moved(n, 0);
    for (uint32_t j = 0; j < cached.size(); j++) {
        remap[cached[j]] = 2 * j;
        remap[cached[j] + 1] = 2 * j + 1;
        moved[cached[j]] = moved[cached[j] + 1] = 1;
    }
    uint32_t next = 2 * (uint32_t)cached.size();
    for (uint32_t i = 0; i < n; i++)
        if (!moved[i]) remap[i] = next++;
    for (uint32_t i = 0; i < n; i++) {
        pt_packed_mesh_node N = in[i];
        if (N.FaceEndIndex == 0) N.FaceBeginOrNodeIndex = remap[N.FaceBeginOrNodeIndex];
        out[remap[i]] = N;
    }
    return (uint32_t)cached.size();
}

// Material types reachable by a hit (every shape's material), whether any
// medium can scatter, whether any shape is not a mesh instance and whether sky
// light sampling is on: selects the shade kernel instantiation (kernels.hip
// pt_shade_mats).
static uint32_t SceneMaterialMask(const pt_scene_packs* p)
{
    uint32_t m = 0;
    for (uint32_t i = 0; i < p->shape_count; i++) {
        uint32_t type = p->material_data[32 * p->shapes[i].MaterialIndex];
        if (type == PT_MATERIAL_TYPE_BASIC_DIFFUSE) m |= PT_MATS_DIFFUSE;
        else if (type == PT_MATERIAL_TYPE_BASIC_METAL) m |= PT_MATS_METAL;
        else if (type == PT_MATERIAL_TYPE_BASIC_TRANSLUCENT) m |= PT_MATS_TRANSLUCENT;
        else if (type == PT_MATERIAL_TYPE_OPENPBR) m |= PT_MATS_OPENPBR;
    }
    if ((m & PT_MATS_TRANSLUCENT) || p->globals->SceneScatterRate > 0.0f) m |= PT_MATS_SCATTER;
    for (uint32_t i = 0; i < p->shape_count; i++)
        if (p->shapes[i].Type != PT_SHAPE_TYPE_MESH_INSTANCE) m |= PT_MATS_PRIMS;
    // PT_MATS_SKY clear: the light is never chosen and its pdf term is an
    // exact +0, so the shade kernel drops the sky lobe and the sky pdf
    // (SampleSurfaceIntegrand).  That needs SkyboxSamplingProbability == +0
    // (bit pattern 0: LP * pdf is then +0) and a finite pdf for every
    // direction: the constant 1/(4 pi) below PT_EPSILON, else a finite norm,
    // Kappa <= 1000 and |SkyboxMeanDirection|^2 <= 1.01 (so Kappa (Mu.In - 1)
    // stays far below exp's overflow).
    {
        const pt_packed_scene_globals& G = *p->globals;
        const float K = G.SkyboxConcentration;
        const float* D = G.SkyboxMeanDirection;
        const float norm = ptd::VmfConstants(K).norm;
        const bool pdf_finite = (K < PT_EPSILON) || (std::isfinite(norm) && K <= 1000.0f &&
                                                     D[0] * D[0] + D[1] * D[1] + D[2] * D[2] <= 1.01f);
        uint32_t ssp;
        std::memcpy(&ssp, &G.SkyboxSamplingProbability, 4);
        if (ssp != 0u || !pdf_finite) m |= PT_MATS_SKY;
    }
    // The lean instantiation's two-select texel wrap is exact when every
    // atlas placement lies in [0, 1] (the atlas packer's always do).
    for (uint32_t i = 0; i < p->texture_count; i++)
        for (int k = 0; k < 2; k++) {
            const float a = p->textures[i].AtlasPlacementMinimum[k], b = p->textures[i].AtlasPlacementMaximum[k];
            if (!((a >= 0.0f) & (a <= 1.0f) & (b >= 0.0f) & (b <= 1.0f))) m |= PT_MATS_TEXWRAP;
        }
    return m;
}

int ptUpdateScene(pt_device* d, pt_scene* s, const pt_scene_packs* p, uint32_t dirty)
{
    if (!d || !s) { SetError("null device/scene"); return -1; }
    uint32_t need = 0;
    if (ValidatePacks(p, &need) != 0) { s->valid = false; return -1; }
    PT_HIP(hipSetDevice(d->id));
    PT_WAIT(d);   // like vkDeviceWaitIdle (scene.cpp:1704)
    bool first = !s->valid;
    if (first || (dirty & PT_SCENE_DIRTY_TEXTURES)) {
        PT_HIP(s->textures.upload(p->textures, p->texture_count));
        size_t atlas_floats = (size_t)p->atlas_width * p->atlas_height * 4 * p->atlas_layer_count;
        s->atlas_tiled = p->atlas && p->atlas_width % 4 == 0 && p->atlas_height % 2 == 0;
        if (s->atlas_tiled) {
            // Upload row-major, then re-lay the texels in 4x2 blocks
            // (AtlasIndex, pt_device.hpp) on the device.
            dbuf<float> stage;
            struct release_stage { dbuf<float>& b; ~release_stage() { b.release(); } } guard{stage};
            PT_HIP(stage.upload(p->atlas, atlas_floats));
            PT_HIP(s->atlas.alloc(atlas_floats));
            PT_HIP(pt_launch_atlas_tile(reinterpret_cast<const float4*>(stage.ptr), reinterpret_cast<float4*>(s->atlas.ptr),
                                        p->atlas_width, p->atlas_height, p->atlas_layer_count, d->stream));
            PT_WAIT(d);
        } else {
            PT_HIP(s->atlas.upload(p->atlas, p->atlas ? atlas_floats : 0));
        }
    }
    if (first || (dirty & PT_SCENE_DIRTY_MATERIALS)) PT_HIP(s->material.upload(p->material_data, p->material_word_count));
    if (first || (dirty & PT_SCENE_DIRTY_SHAPES)) PT_HIP(s->shape_nodes.upload(p->shape_nodes, p->shape_node_count));
    // The device BLAS node array in the LDS node cache's layout (the shapes'
    // root indices follow it).
    const bool relayout = first || (dirty & (PT_SCENE_DIRTY_SHAPES | PT_SCENE_DIRTY_MATERIALS | PT_SCENE_DIRTY_MESHES));
    std::vector<pt_packed_mesh_node> nodes;
    std::vector<uint32_t> remap;
    if (relayout) s->cached_pairs = NodeCacheLayout(p, nodes, remap);
    if (relayout) {
        // The device's shape records carry, in their unused Pad0 word, whether
        // the shape's material reads texture coordinates (HitAttributesV).
        std::vector<pt_packed_shape> sh(p->shapes, p->shapes + p->shape_count);
        for (pt_packed_shape& S : sh) {
            S.Pad0 = MaterialReadsUV(p, S.MaterialIndex) ? ptd::PT_SHAPE_FLAG_UV : 0u;
            if (S.Type == PT_SHAPE_TYPE_MESH_INSTANCE) S.MeshRootNodeIndex = remap[S.MeshRootNodeIndex];
        }
        PT_HIP(s->shapes.upload(sh.data(), sh.size()));
        PT_HIP(s->mesh_nodes.upload(nodes.data(), nodes.size()));
    }
    if (first || (dirty & PT_SCENE_DIRTY_MESHES)) {
        // Device face records carry {Position0, Edge1, Edge2} (traverse.hpp
        // LaneMeshFace): the reference's per-test edge subtractions
        // (scene.glsl.inc:307-308) done once here, same IEEE f32 operations.
        std::vector<pt_packed_mesh_face> ef(p->mesh_faces, p->mesh_faces + p->mesh_face_count);
        for (pt_packed_mesh_face& F : ef)
            for (int k = 0; k < 3; k++) {
                float p0 = F.Position0[k];
                F.Position1[k] = F.Position1[k] - p0;
                F.Position2[k] = F.Position2[k] - p0;
            }
        PT_HIP(s->faces.upload(ef.data(), ef.size()));
        PT_HIP(s->vertices.upload(p->mesh_vertices, p->mesh_vertex_count));
        PT_HIP(s->vertex_attr.alloc(std::max<size_t>(p->mesh_vertex_count, 1)));
        PT_HIP(s->vertex_v.alloc(std::max<size_t>(p->mesh_vertex_count, 1)));
        PT_HIP(pt_launch_vertex_decode(reinterpret_cast<const uint2*>(s->vertices.ptr), p->mesh_vertex_count,
                                       s->vertex_attr.ptr, s->vertex_v.ptr, d->stream));
    }
    if (first || (dirty & PT_SCENE_DIRTY_CAMERAS)) PT_HIP(s->cameras.upload(p->cameras, p->camera_count));

    ptd::dscene& D = s->d;
    D.g = *p->globals;
    {
        ptd::vmf_consts K = ptd::VmfConstants(D.g.SkyboxConcentration);
        D.vmf_inv_kappa = K.inv_kappa;
        D.vmf_exp_m2k = K.exp_m2k;
        D.vmf_norm = K.norm;
        D.sky_flat = ptd::SkyFlat();
    }
    D.textures = s->textures.ptr;
    D.material = s->material.ptr;
    D.shapes = s->shapes.ptr;
    D.shape_nodes = reinterpret_cast<const float4*>(s->shape_nodes.ptr);
    D.mesh_faces = reinterpret_cast<const float4*>(s->faces.ptr);
    D.mesh_vertices = reinterpret_cast<const uint2*>(s->vertices.ptr);
    D.vertex_attr = s->vertex_attr.ptr;
    D.vertex_v = s->vertex_v.ptr;
    D.mesh_nodes = reinterpret_cast<const float4*>(s->mesh_nodes.ptr);
    D.cameras = s->cameras.ptr;
    D.atlas = reinterpret_cast<const float4*>(s->atlas.ptr);
    D.atlas_w = p->atlas_width;
    D.atlas_h = p->atlas_height;
    D.atlas_layers = p->atlas ? p->atlas_layer_count : 0;
    D.atlas_tiled = s->atlas_tiled ? 1u : 0u;
    D.fast_div = FastDivBoxes(p) ? 1u : 0u;
    s->mats = SceneMaterialMask(p);
    uint32_t types = s->mats & (PT_MATS_DIFFUSE | PT_MATS_METAL | PT_MATS_TRANSLUCENT | PT_MATS_OPENPBR);
    D.mat_classes = (types & (types - 1)) != 0 ? 1u : 0u;   // more than one material type
    // Hit records carry a mesh face's vertex indices when every index fits
    // 21 bits (PackVertexIndices, traverse.hpp); ptSetSceneHitRecordForm can
    // force the face-index form that larger scenes use.
    D.vidx21 = (p->mesh_vertex_count <= (1u << 21) && s->hit_record != PT_HIT_RECORD_FACE_INDEX) ? 1u : 0u;
    // Traversal stack entries: 16-bit when every entry fits, else packed
    // 32-bit BLAS words, else node indices (ptSetSceneStackFormat can force
    // the wider forms, which larger scenes need).
    // (On the device node layout: its child-pair indices are what the
    // stack entries hold.)
    pt_scene_packs pd = *p;
    if (relayout) pd.mesh_nodes = nodes.data();
    D.blas_words = (s->stack_format != PT_STACK_FORMAT_NODE_INDEX && (relayout ? BlasWordsPackable(&pd) : s->blas_packable)) ? 1u : 0u;
    D.blas_firstbits = 0;
    D.stack16 = 0;
    uint32_t F16 = s->stack_format == PT_STACK_FORMAT_AUTO ? (relayout ? BlasWords16FirstBits(&pd) : s->blas16_bits) : 0u;
    if (relayout) {
        s->blas_packable = BlasWordsPackable(&pd);
        s->blas16_bits = BlasWords16FirstBits(&pd);
    }
    if (uint32_t F = F16) {   // every stack entry fits 16 bits
        D.blas_words = 2;
        D.blas_firstbits = F;
        D.stack16 = 1;
    }
    // The LDS node cache rides with the u16 stack (kernels.hip LaunchExtendE).
    D.node_cache = D.stack16 ? 2 * s->cached_pairs : 0u;
    s->camera_count = p->camera_count;
    s->stack_needed = need;
    s->valid = true;
    return 0;
}

pt_sample_buffer* ptCreateSampleBuffer(pt_device* d, uint32_t w, uint32_t h)
{
    if (!d || w == 0 || h == 0) { SetError("bad sample buffer arguments"); return nullptr; }
    if (hipSetDevice(d->id) != hipSuccess) { SetError("hipSetDevice failed"); return nullptr; }
    pt_sample_buffer* b = new pt_sample_buffer;
    b->dev = d;
    b->width = w;
    b->height = h;
    size_t bytes = (size_t)w * h * sizeof(float4);
    if (hipMalloc(&b->accum, bytes) != hipSuccess || hipMemset(b->accum, 0, bytes) != hipSuccess) {
        SetError("sample buffer allocation failed (%zu bytes)", bytes);
        if (b->accum) (void)hipFree(b->accum);
        delete b;
        return nullptr;
    }
    return b;
}

void ptDestroySampleBuffer(pt_device* d, pt_sample_buffer* b)
{
    if (!b) return;
    if (d) (void)hipSetDevice(d->id);
    if (b->accum) (void)hipFree(b->accum);
    b->display.release();
    b->display8.release();
    delete b;
}

int ptReadSampleBuffer(pt_device* d, pt_sample_buffer* b, float* rgba)
{
    if (!d || !b || !rgba) { SetError("null argument"); return -1; }
    PT_HIP(hipSetDevice(d->id));
    PT_HIP(hipMemcpyAsync(rgba, b->accum, (size_t)b->width * b->height * sizeof(float4), hipMemcpyDeviceToHost, d->stream));
    PT_WAIT(d);
    return 0;
}

int ptWriteSampleBuffer(pt_device* d, pt_sample_buffer* b, const float* rgba)
{
    if (!d || !b || !rgba) { SetError("null argument"); return -1; }
    PT_HIP(hipSetDevice(d->id));
    PT_HIP(hipMemcpyAsync(b->accum, rgba, (size_t)b->width * b->height * sizeof(float4), hipMemcpyHostToDevice, d->stream));
    PT_WAIT(d);
    return 0;
}

// RenderSampleBuffer (integrator.cpp:105-159 + resolve.glsl:112-128)
int ptRenderSampleBuffer(pt_device* d, pt_sample_buffer* b, const pt_resolve_parameters* p)
{
    if (!d || !b || !p) { SetError("null argument"); return -1; }
    if (p->ToneMappingMode > PT_TONE_MAPPING_ACES) { SetError("bad tone mapping mode %u", p->ToneMappingMode); return -1; }
    PT_HIP(hipSetDevice(d->id));
    size_t n = (size_t)b->width * b->height;
    PT_HIP(b->display.alloc(n));
    PT_HIP(b->display8.alloc(n));
    event_pair ep{};
    if (int e = BeginTimed(d, PT_KERNEL_RESOLVE, ep)) return e;
    PT_HIP(pt_launch_resolve(b->accum, (uint32_t)n, p->Brightness, p->ToneMappingMode, p->ToneMappingWhiteLevel,
                             b->display.ptr, b->display8.ptr, d->stream));
    if (int e = EndTimed(d, ep)) return e;
    b->resolved = true;
    return 0;
}

int ptReadResolvedImage(pt_device* d, pt_sample_buffer* b, float* rgba)
{
    if (!d || !b || !rgba) { SetError("null argument"); return -1; }
    if (!b->resolved) { SetError("sample buffer not resolved (call ptRenderSampleBuffer)"); return -1; }
    PT_HIP(hipSetDevice(d->id));
    PT_HIP(hipMemcpyAsync(rgba, b->display.ptr, (size_t)b->width * b->height * sizeof(float4), hipMemcpyDeviceToHost,
                          d->stream));
    PT_WAIT(d);
    return 0;
}

int ptReadResolvedImageSRGB8(pt_device* d, pt_sample_buffer* b, uint8_t* rgba8)
{
    if (!d || !b || !rgba8) { SetError("null argument"); return -1; }
    if (!b->resolved) { SetError("sample buffer not resolved (call ptRenderSampleBuffer)"); return -1; }
    PT_HIP(hipSetDevice(d->id));
    PT_HIP(hipMemcpyAsync(rgba8, b->display8.ptr, (size_t)b->width * b->height * 4, hipMemcpyDeviceToHost, d->stream));
    PT_WAIT(d);
    return 0;
}

// Rounds between two longest-first tile-order sorts (C3 / C5 / C2 at 4:
// +3.4 / +4.9 / -1.4 %, at 16: +3.9 / +5.3 / 0 % vs natural order; period 1
// C3 -2.4 %: DESIGN.md §4).
#ifndef PT_TILE_ORDER_PERIOD
#define PT_TILE_ORDER_PERIOD 16   // experiment builds may change it
#endif
constexpr uint32_t TILE_ORDER_PERIOD = PT_TILE_ORDER_PERIOD;

pt_basic_renderer* ptCreateBasicRendererStreams(pt_device* d, pt_scene* s, pt_sample_buffer* b, uint32_t rank,
                                                uint32_t nranks, uint32_t streams)
{
    if (!d || !s || !b) { SetError("null argument"); return nullptr; }
    if (nranks == 0 || rank >= nranks) { SetError("bad partition %u/%u", rank, nranks); return nullptr; }
    if (streams == 0 || streams > 256) { SetError("bad stream count %u (1..256)", streams); return nullptr; }
    if (hipSetDevice(d->id) != hipSuccess) { SetError("hipSetDevice failed"); return nullptr; }
    pt_basic_renderer* r = new pt_basic_renderer;
    r->dev = d;
    r->scene = s;
    r->buffer = b;
    r->rank = rank;
    r->nranks = nranks;
    r->tiles_x = (b->width + 15) / 16;
    uint32_t bands = (b->height + 15) / 16;
    uint32_t owned = bands > rank ? (bands - rank + nranks - 1) / nranks : 0;
    const uint64_t T = (uint64_t)owned * r->tiles_x;   // tiles per stream
    uint64_t n = T * streams * 256;
    // TileRow's and TileStream's reciprocal divisions are exact while every
    // tile index t has t * divisor < 2^32.
    if (T * r->tiles_x >= (1ull << 32) || (streams > 1 && T * T * streams >= (1ull << 32))) {
        SetError("frame too large");
        delete r;
        return nullptr;
    }
    if (n > 0xFFFFFFFFull / 2) { SetError("too many slots"); delete r; return nullptr; }
    uint32_t ns = (uint32_t)n;
    bool ok = r->ray.alloc(ns) == hipSuccess && r->hit.alloc(ns) == hipSuccess && r->thr.alloc(ns) == hipSuccess &&
              r->prob.alloc(ns) == hipSuccess && r->prob1.alloc(ns) == hipSuccess && r->grey_count.alloc(1) == hipSuccess &&
              r->lam.alloc(ns) == hipSuccess && r->uv.alloc(ns) == hipSuccess &&
              r->act.alloc(ns) == hipSuccess && r->pos.alloc(ns) == hipSuccess && r->slotof.alloc(ns) == hipSuccess &&
              r->outcome.alloc((size_t)(ns / 256) * 4 * ptd::PT_OUTCOME_CLASSES + 1) == hipSuccess &&
              r->tilecost.alloc((size_t)(ns / 256) * 4 + 1) == hipSuccess && r->order.alloc(ns / 256 + 1) == hipSuccess &&
              r->done.alloc(ns / 64 + 1) == hipSuccess;
    const size_t frame_px = (size_t)b->width * b->height;
    if (ok && streams > 1)
        ok = r->accx.alloc((size_t)streams * frame_px) == hipSuccess &&
             hipMemset(r->accx.ptr, 0, (size_t)streams * frame_px * 16) == hipSuccess;
    if (ok && ns) {
        ok = hipMemset(r->ray.ptr, 0, (size_t)ns * 16) == hipSuccess && hipMemset(r->hit.ptr, 0, (size_t)ns * 16) == hipSuccess &&
             hipMemset(r->thr.ptr, 0, (size_t)ns * 16) == hipSuccess && hipMemset(r->prob.ptr, 0, (size_t)ns * 16) == hipSuccess &&
             hipMemset(r->prob1.ptr, 0, (size_t)ns * 4) == hipSuccess &&
             hipMemset(r->lam.ptr, 0, (size_t)ns * 4) == hipSuccess && hipMemset(r->uv.ptr, 0, (size_t)ns * 8) == hipSuccess &&
             hipMemset(r->act.ptr, 0, (size_t)ns * 8) == hipSuccess && hipMemset(r->done.ptr, 0, (size_t)(ns / 64 + 1) * 4) == hipSuccess &&
             hipMemset(r->outcome.ptr, 0, ((size_t)(ns / 256) * 4 * ptd::PT_OUTCOME_CLASSES + 1) * 8) == hipSuccess;
        // Identity TileOrder until the first Reset sorts the rays.
        std::vector<uint16_t> pos(ns);
        std::vector<uint8_t> slotof(ns);
        for (uint32_t i = 0; i < ns; i++) { pos[i] = (uint16_t)(((i & 255u) << 8) | (i & 255u)); slotof[i] = (uint8_t)(i & 255u); }
        std::vector<uint32_t> order(ns / 256);
        for (uint32_t t = 0; t < ns / 256; t++) order[t] = t;   // natural order until a round is timed
        ok = ok && hipMemcpy(r->pos.ptr, pos.data(), (size_t)ns * 2, hipMemcpyHostToDevice) == hipSuccess &&
             hipMemcpy(r->slotof.ptr, slotof.data(), ns, hipMemcpyHostToDevice) == hipSuccess &&
             hipMemset(r->tilecost.ptr, 0, ((size_t)(ns / 256) * 4 + 1) * 4) == hipSuccess &&
             hipMemcpy(r->order.ptr, order.data(), (size_t)(ns / 256) * 4, hipMemcpyHostToDevice) == hipSuccess;
    }
    if (!ok) {
        SetError("renderer slot allocation failed (%u slots)", ns);
        r->ray.release(); r->hit.release(); r->thr.release(); r->prob.release(); r->prob1.release(); r->grey_count.release();
        r->lam.release(); r->uv.release(); r->act.release();
        r->pos.release(); r->slotof.release(); r->outcome.release(); r->tilecost.release(); r->order.release();
        r->done.release(); r->accx.release();
        delete r;
        return nullptr;
    }
    r->streams = streams;
    r->stream_tiles = (uint32_t)T;
    r->slots.ray = r->ray.ptr;
    r->slots.hit = r->hit.ptr;
    r->slots.uv = r->uv.ptr;
    r->slots.thr = r->thr.ptr;
    r->slots.prob = r->prob.ptr;
    r->slots.lam = r->lam.ptr;
    r->slots.act = r->act.ptr;
    r->slots.pos = r->pos.ptr;
    r->slots.slotof = r->slotof.ptr;
    r->slots.outcome = r->outcome.ptr;
    r->slots.tilecost = r->tilecost.ptr;
    r->slots.order = ns ? r->order.ptr : nullptr;
    r->slots.done = r->done.ptr;
    r->slots.spill = nullptr;
    r->slots.n = ns;
    r->slots.tile_count = ns / 256;
    for (uint32_t band = rank; band < bands; band += nranks)
        r->pixels += (uint64_t)b->width * std::min<uint32_t>(16u, b->height - band * 16u);
    r->valid_slots = r->pixels * streams;
    b->rank = rank;
    b->nranks = nranks;
    return r;
}

pt_basic_renderer* ptCreateBasicRendererPartitioned(pt_device* d, pt_scene* s, pt_sample_buffer* b, uint32_t rank,
                                                    uint32_t nranks)
{
    return ptCreateBasicRendererStreams(d, s, b, rank, nranks, 1);
}

// The sample buffer's owned pixels := the streams' accumulators summed in
// stream order, ((A0 + A1) + A2) ...; the streams keep accumulating, so a
// later merge gives the new totals.
int ptMergeBasicRendererStreams(pt_device* d, pt_basic_renderer* r)
{
    if (!d || !r || !r->buffer) { SetError("null argument"); return -1; }
    if (r->streams == 1) return 0;
    PT_HIP(hipSetDevice(d->id));
    PT_HIP(pt_launch_merge_streams(r->buffer->accum, r->accx.ptr, r->buffer->width, r->buffer->height, r->rank,
                                   r->nranks, r->streams, d->stream));
    return 0;
}

uint32_t ptBasicRendererStreams(pt_basic_renderer* r) { return r ? r->streams : 0; }

pt_basic_renderer* ptCreateBasicRenderer(pt_device* d, pt_scene* s, pt_sample_buffer* b)
{
    return ptCreateBasicRendererPartitioned(d, s, b, 0, 1);
}

void ptDestroyBasicRenderer(pt_device* d, pt_basic_renderer* r)
{
    if (!r) return;
    if (d) { (void)hipSetDevice(d->id); (void)DeviceWait(d); }
    r->ray.release(); r->hit.release(); r->thr.release(); r->prob.release(); r->prob1.release(); r->grey_count.release();
    r->cq_counts.release(); r->cq_list.release();
    r->lam.release();
    r->uv.release(); r->act.release(); r->pos.release(); r->slotof.release(); r->outcome.release();
    r->tilecost.release(); r->order.release();
    r->done.release();
    r->spill.release();
    r->guard.release();
    r->accx.release();
    delete r;
}

pt_basic_renderer_params* ptBasicRendererParams(pt_basic_renderer* r) { return r ? &r->params : nullptr; }
uint32_t ptBasicRendererSlotCount(pt_basic_renderer* r) { return r ? r->slots.n : 0; }

// Material mask the renderer shades with (shade / round instantiation): the
// scene's OpenPBR shapes, and the media they bring, join it only when OpenPBR
// shading is enabled (ptSetBasicRendererOpenPBR); otherwise their hits end
// the path as in the reference.
static uint32_t ShadeMats(const pt_basic_renderer* r)
{
    uint32_t m = r->scene->mats;
    if (!(m & PT_MATS_OPENPBR)) return m;
    if (!r->openpbr) return m & ~(uint32_t)PT_MATS_OPENPBR;
    return m | PT_MATS_SCATTER;
}

// Whether the live paths take the grey record form.  Decided on the shade
// instantiation's mask (pt_shade_mats), the same mask ShadeSlot tests as MATS:
// a scene mask without glass can still map to an instantiation that has it
// (diffuse + metal + fog -> PT_MATS_ALL), and that kernel reads the
// four-float record.
static bool GreyForm(const pt_basic_renderer* r) { return pt_grey_mats(pt_shade_mats(ShadeMats(r))); }

// The record form of the renderer's live paths (GreyRecord, kernels.hip
// StorePathVertex): grey while the shade mask keeps every Probability
// wavelength-uniform and every active-shape stack empty.  A mask change
// between rounds (a scene update without Reset, ptSetBasicRendererOpenPBR)
// converts the live paths: to the four-float form always; to the grey form
// only if every live path satisfies its invariants (checked on the device:
// paths that crossed into a glass keep a non-empty stack), else the renderer
// stays in the four-float form until the next Reset or state write.
static int SyncRecordForm(pt_device* d, pt_basic_renderer* r)
{
    const bool want = GreyForm(r);
    if (want != r->grey && r->slots.n) {
        const ptd::dframe F = Frame(r);
        if (!want) {
            PT_HIP(pt_launch_grey_convert(r->slots, F, r->prob1.ptr, false, d->stream));
            r->grey = false;
        } else if (!r->grey_blocked) {
            PT_HIP(hipMemsetAsync(r->grey_count.ptr, 0, sizeof(uint32_t), d->stream));
            PT_HIP(pt_launch_grey_check(r->slots, F, r->grey_count.ptr, d->stream));
            PT_WAIT(d);
            uint32_t bad = 0;
            PT_HIP(hipMemcpy(&bad, r->grey_count.ptr, sizeof(bad), hipMemcpyDeviceToHost));
            if (bad == 0) {
                PT_HIP(pt_launch_grey_convert(r->slots, F, r->prob1.ptr, true, d->stream));
                r->grey = true;
            } else {
                r->grey_blocked = true;
            }
        }
    }
    r->slots.prob1 = r->grey ? r->prob1.ptr : nullptr;
    return 0;
}

// ResetBasicRenderer (basic.cpp:285-304)
int ptResetBasicRenderer(pt_device* d, pt_basic_renderer* r)
{
    if (!d) { SetError("null device"); return -1; }
    if (CheckReady(r) != 0) return -1;
    PT_HIP(hipSetDevice(d->id));
    // Every live path is replaced: the record form follows the shade mask.
    r->grey = GreyForm(r);
    r->grey_blocked = false;
    r->slots.prob1 = r->grey ? r->prob1.ptr : nullptr;
    event_pair ep{};
    if (int e = BeginTimed(d, PT_KERNEL_RAYGEN, ep)) return e;
    PT_HIP(pt_launch_raygen(r->scene->d, r->slots, Frame(r), Params(r, r->params.FrameIndex), d->stream));
    if (int e = EndTimed(d, ep)) return e;
    PT_HIP(hipMemsetAsync(r->done.ptr, 0, (size_t)(r->slots.n / 64 + 1) * 4, d->stream));
    r->rays = 0;
    return 0;
}

// RunBasicRenderer (basic.cpp:306-332)
// Fused rounds (round_kernel) when every tile of the launch fits on the GPU
// at once -- a rank's share of a strongly scaled frame -- and the scene needs
// no spilled stack (renderer mode 1); mode 0 never fuses, mode 2 fuses
// whenever the kernel applies (tests and A/B).

// Completion queue of the shade kernel (kernels.hip ShadeTile): worth its
// barriers when paths also end at surfaces -- sky light sampling (a sample
// below the horizon ends the path), roulette, or metal / translucent /
// OpenPBR BSDFs (failed samples) -- so that completions are scattered over
// the hit waves.  Measured (profiles/r04_ab3): C2 shade -3.7 %, C5 -3.0 %;
// C3 (diffuse, no light sampling, no roulette: every completion is an escape,
// already grouped by ShadeOrder) +3 % with it, so it stays off there.
static bool ShadeCompact(const pt_basic_renderer* r)
{
    const uint32_t m = ShadeMats(r);
    return (m & (PT_MATS_METAL | PT_MATS_TRANSLUCENT | PT_MATS_OPENPBR)) != 0 ||
           r->scene->d.g.SkyboxSamplingProbability > 0.0f || r->params.PathTerminationProbability > 0.0f;
}

static bool RoundFused(const pt_basic_renderer* r, const ptd::dslots& g)
{
    const int mode = r->fused;
    if (mode == 0 || g.spill || g.tile_count == 0) return false;
    uint32_t cap = pt_round_capacity(ShadeMats(r), r->scene->d.stack16 != 0, r->dev->cu_count);
    if (cap == 0) return false;
    return mode == 2 || g.tile_count <= cap;
}

// Class-list region of one tile group of K: classes x CQ_SUB sub-lists of
// the largest group's capacity (group g holds at most ceil(T / K) tiles).
static size_t ClassListStride(uint32_t tiles, uint32_t K)
{
    return (size_t)ptd::PT_OUTCOME_CLASSES * CQ_SUB * pt_classq_sub_capacity((tiles + K - 1) / K);
}

// Class-list buffers: the counters of PT_MAX_SPLIT tile groups (2 parities x
// classes x CQ_SUB each) plus those of single-stream rounds (region
// PT_MAX_SPLIT, kept zero by its own parity), allocated on first use and
// zeroed; the lists sized for the K groups in use (K regions of
// ClassListStride) or for a single-stream round over every tile, whichever
// is larger (about 20 B per slot), grown when K grows.  A growth waits for
// the device stream: the old lists may still be read by queued launches.
static int ClassListBuffers(pt_device* d, pt_basic_renderer* r, uint32_t K)
{
    const size_t nc = (size_t)ptd::PT_OUTCOME_CLASSES * CQ_SUB;
    const uint32_t T = r->slots.tile_count;
    if (!r->cq_counts.ptr) {
        if (r->cq_counts.alloc((PT_MAX_SPLIT + 1) * 2 * nc) != hipSuccess ||
            hipMemset(r->cq_counts.ptr, 0, (PT_MAX_SPLIT + 1) * 2 * nc * sizeof(uint32_t)) != hipSuccess) {
            SetError("class list allocation failed");
            return -1;
        }
    }
    const size_t need = std::max(ClassListStride(T, 1), K * ClassListStride(T, K));
    if (need > r->cq_list.count) {
        if (r->cq_list.ptr) PT_WAIT(d);
        if (r->cq_list.alloc(need) != hipSuccess) {
            SetError("class list allocation failed");
            return -1;
        }
    }
    return 0;
}

static bool ClassListRounds(const pt_basic_renderer* r);

// Class-pure shade of one single-stream round over every tile (the
// renderer's rounds outside tile groups: Run(2), single rounds, guarded
// rounds), with the single-stream counter region.  A renderer whose tile
// groups use the lists takes them for every round: a tile-local shade's
// TileOrder would leave the slots permuted within their tiles against the
// positions, and the class lists' gathers by slot lose their coherence
// (C2 -4 % measured, profiles/r05_exp2).
static int ClassListShade(pt_device* d, pt_basic_renderer* r, const ptd::dslots& L, const ptd::dframe& F,
                          const ptd::dparams& P, hipStream_t st)
{
    if (int e = ClassListBuffers(d, r, 1)) return e;
    const size_t nc = (size_t)ptd::PT_OUTCOME_CLASSES * CQ_SUB;
    uint32_t* cnt = r->cq_counts.ptr + PT_MAX_SPLIT * 2 * nc;
    uint32_t* cq = cnt + nc * r->cq_parity;
    uint32_t* cq_next = cnt + nc * (r->cq_parity ^ 1u);
    r->cq_parity ^= 1u;
    PT_HIP(pt_launch_shade_classq(r->scene->d, L, F, P, ShadeMats(r), ShadeCompact(r), cq, cq_next, r->cq_list.ptr,
                                  st));
    return 0;
}

int ptRunBasicRenderer(pt_device* d, pt_basic_renderer* r, uint32_t rounds)
{
    if (!d) { SetError("null device"); return -1; }
    if (CheckReady(r) != 0) return -1;
    PT_HIP(hipSetDevice(d->id));
    if (int e = EnsureSpill(r)) return e;
    if (int e = SyncRecordForm(d, r)) return e;
    r->params.FrameIndex += 1;
    ptd::dparams P = Params(r, r->params.FrameIndex);
    ptd::dframe F = Frame(r);
    const ptd::dslots& L = r->slots;
    const bool fused = RoundFused(r, L);
    // Run(R >= 2) where round batches apply (RunRounds' rule): the R rounds
    // with the one seed as batches of the rounds kernel (seed_step 0), one
    // launch instead of R -- the application's Run(2) after a restart.
    const uint32_t B = r->round_batch ? r->round_batch : (fused && r->fused == 1 ? AUTO_BATCH : 1u);
    if (fused && rounds >= 2 && B >= 2 && pt_rounds_available(L)) {
        for (uint32_t left = rounds; left > 0;) {
            const uint32_t n = std::min(left, B);
            ptd::dparams Pb = P;
            Pb.rounds = n;
            Pb.seed_step = 0;
            const uint64_t t = d->run_tick % d->profile_period;
            const bool sampled = d->profiling && (t == 0 || t + n > d->profile_period);
            d->run_tick += n;
            event_pair ep{};
            if (int e = BeginTimed(d, PT_KERNEL_ROUNDS, ep, sampled, n)) return e;
            PT_HIP(pt_launch_rounds(r->scene->d, L, F, Pb, ShadeMats(r), d->stream));
            if (int e = EndTimed(d, ep)) return e;
            for (uint32_t g = 0; g < r->order_groups; g++)
                PT_HIP(pt_launch_tile_order(L, d->stream, r->order_groups, g));
            r->rays += r->valid_slots * n;
            left -= n;
        }
        return 0;
    }
    for (uint32_t i = 0; i < rounds; i++) {
        // Kernel timing samples every profile_period-th round.
        const bool sampled = d->profiling && (d->run_tick++ % d->profile_period) == 0;
        // Tiles keep their relative cost for many rounds: re-sort every
        // TILE_ORDER_PERIOD rounds (one small launch).
        const bool sort = L.order && (r->order_tick++ % TILE_ORDER_PERIOD) == 0;
        event_pair ep{};
        if (fused) {
            if (int e = BeginTimed(d, PT_KERNEL_ROUND, ep, sampled)) return e;
            PT_HIP(pt_launch_round(r->scene->d, L, F, P, ShadeMats(r), d->stream));
            if (int e = EndTimed(d, ep)) return e;
        } else {
            if (int e = BeginTimed(d, PT_KERNEL_EXTEND, ep, sampled)) return e;
            PT_HIP(pt_launch_extend(r->scene->d, L, F, L.spill, d->stream));
            if (int e = EndTimed(d, ep)) return e;
            if (int e = BeginTimed(d, PT_KERNEL_SHADE, ep, sampled)) return e;
            if (ClassListRounds(r)) {
                if (int e = ClassListShade(d, r, L, F, P, d->stream)) return e;
            } else {
                PT_HIP(pt_launch_shade(r->scene->d, L, F, P, ShadeMats(r), ShadeCompact(r), d->stream));
            }
            if (int e = EndTimed(d, ep)) return e;
        }
        if (sort)
            for (uint32_t g = 0; g < r->order_groups; g++) PT_HIP(pt_launch_tile_order(L, d->stream, r->order_groups, g));
        r->rays += r->valid_slots;
    }
    return 0;
}

// Tile groups on concurrent streams (ptSetBasicRendererSplit).  A batch of
// consecutive rounds over a whole frame ends each extend and shade launch
// with a tail of a few long blocks while most CUs idle.  Split into K groups
// of tiles (t = g, g + K, ...), each running its own sequence of rounds on
// its own stream, the launches of one group fill the CUs another group's
// tail leaves idle.  A slot's round depends only on its own previous round
// and the round's FrameIndex, so the results are those of the unsplit
// rounds, bit for bit.  Measured (bench.py A/B, profiles/r05_split,
// r05_splitk): K = 2 / 3 / 4 against 1 -- C3 +4.8 / +6.8 / -8 %, C2 +17 /
// +17 / -3 %, C5 +15 / +16 / -11 %, C4 +1.3 / +1.7 / -1 %; halving the
// launches on ONE stream costs 14-20 % (tools/exp_two_streams.py), so the
// gain is the overlap.  Four groups take every hardware queue of the
// process (GPU_MAX_HW_QUEUES = 4) and lose.
constexpr uint32_t SPLIT_MIN_TILES = 2048;   // automatic mode: whole frames (C2 has 4 096 tiles)
constexpr uint32_t SPLIT_AUTO_GROUPS = 3;

static uint32_t SplitGroups(const pt_basic_renderer* r)
{
    const ptd::dslots& L = r->slots;
    if (!L.order || L.tile_count < 2 || r->split == 1) return 1;
    if (r->split >= 2) return std::min(r->split, L.tile_count);
    return (!RoundFused(r, L) && L.tile_count >= SPLIT_MIN_TILES) ? SPLIT_AUTO_GROUPS : 1u;
}

// Class-pure shade inside tile groups (kernels.hip shade_classq_kernel):
// scenes with more than one material type whose shade instantiation has a
// class-pure form.  In tile groups the lists' latency and the gathers' extra
// bytes overlap the other groups' launches (C2 +6 %, C5 +6 %); alone on one
// stream they cost more than the lanes gain, so single-stream rounds keep
// the tile-local shade.
static bool ClassLists(const pt_basic_renderer* r)
{
    return r->class_lists != 1 && r->scene->d.mat_classes != 0 && pt_class_lists_supported(ShadeMats(r));
}

// Rounds of this renderer shade through class lists (tile groups and
// single-stream rounds alike).
static bool ClassListRounds(const pt_basic_renderer* r) { return SplitGroups(r) > 1 && ClassLists(r); }

// The dispatch order holds each group's tiles in its own segment; a change of
// K restarts it from the natural order of each group.
static int EnsureOrderGroups(pt_device* d, pt_basic_renderer* r, uint32_t K)
{
    if (r->order_groups == K || !r->slots.order) return 0;
    const uint32_t T = r->slots.tile_count;
    std::vector<uint32_t> order(T);
    uint32_t i = 0;
    for (uint32_t g = 0; g < K; g++)
        for (uint32_t j = 0; j < pt_tile_group_count(T, K, g); j++) order[i++] = pt_tile_group_tile(T, K, g, j);
    PT_WAIT(d);
    PT_HIP(hipMemcpy(r->order.ptr, order.data(), (size_t)T * 4, hipMemcpyHostToDevice));
    r->order_groups = K;
    return 0;
}

static int EnsureGroupStreams(pt_device* d, uint32_t K)
{
    if (!d->fork_event) PT_HIP(hipEventCreateWithFlags(&d->fork_event, hipEventDisableTiming));
    for (uint32_t g = 0; g + 1 < K; g++) {
        if (!d->group_stream[g]) PT_HIP(hipStreamCreateWithFlags(&d->group_stream[g], hipStreamNonBlocking));
        if (!d->join_event[g]) PT_HIP(hipEventCreateWithFlags(&d->join_event[g], hipEventDisableTiming));
    }
    return 0;
}

// k consecutive rounds (FrameIndex + 1 ... + k) in K tile groups.  Group 0
// runs on the device stream (its launches are the ones profiling times);
// the others wait for everything enqueued before (fork) and the device
// stream waits for them at the end (join), on every path out.
static int RunRoundsSplit(pt_device* d, pt_basic_renderer* r, uint64_t k, uint32_t K)
{
    PT_HIP(hipSetDevice(d->id));
    if (int e = EnsureSpill(r)) return e;
    if (int e = SyncRecordForm(d, r)) return e;
    if (int e = EnsureOrderGroups(d, r, K)) return e;
    if (int e = EnsureGroupStreams(d, K)) return e;
    const ptd::dframe F = Frame(r);
    const uint32_t mats = ShadeMats(r);
    const bool compact = ShadeCompact(r);
    ptd::dslots G[PT_MAX_SPLIT];
    hipStream_t S[PT_MAX_SPLIT];
    for (uint32_t g = 0; g < K; g++) {
        G[g] = r->slots;
        G[g].order = r->slots.order + pt_tile_group_start(r->slots.tile_count, K, g);
        G[g].tile_count = pt_tile_group_count(r->slots.tile_count, K, g);
        S[g] = g ? d->group_stream[g - 1] : d->stream;
    }
    const bool lists = ClassLists(r);
    if (lists) {
        // Per group: 2 parities x classes counters (zero at the batch
        // start) and a list region of ClassListStride words.
        if (int e = ClassListBuffers(d, r, K)) return e;
        PT_HIP(hipMemsetAsync(r->cq_counts.ptr, 0, PT_MAX_SPLIT * 2 * ptd::PT_OUTCOME_CLASSES * CQ_SUB * sizeof(uint32_t),
                              d->stream));
    }
    PT_HIP(hipEventRecord(d->fork_event, d->stream));
    for (uint32_t g = 1; g < K; g++) PT_HIP(hipStreamWaitEvent(S[g], d->fork_event, 0));
    auto rounds = [&]() -> int {
        for (uint64_t i = 0; i < k; i++) {
            r->params.FrameIndex += 1;
            const ptd::dparams P = Params(r, r->params.FrameIndex);
            const bool sampled = d->profiling && (d->run_tick++ % d->profile_period) == 0;
            const bool sort = (r->order_tick++ % TILE_ORDER_PERIOD) == 0;
            for (uint32_t g = 0; g < K; g++) {
                event_pair ep{};
                if (g == 0)
                    if (int e = BeginTimed(d, PT_KERNEL_EXTEND, ep, sampled)) return e;
                PT_HIP(pt_launch_extend(r->scene->d, G[g], F, r->slots.spill, S[g]));
                if (g == 0) {
                    if (int e = EndTimed(d, ep)) return e;
                    if (int e = BeginTimed(d, PT_KERNEL_SHADE, ep, sampled)) return e;
                }
                if (lists) {
                    // Class-pure shade: the group's own counters (parity per
                    // round) and list region.
                    const size_t nc = (size_t)ptd::PT_OUTCOME_CLASSES * CQ_SUB;
                    uint32_t* cnt = r->cq_counts.ptr + g * 2 * nc;
                    PT_HIP(pt_launch_shade_classq(r->scene->d, G[g], F, P, mats, compact, cnt + nc * (i & 1u),
                                                  cnt + nc * ((i & 1u) ^ 1u),
                                                  r->cq_list.ptr + g * ClassListStride(r->slots.tile_count, K), S[g],
                                                  r->slots.tile_count, K, g));
                } else {
                    PT_HIP(pt_launch_shade(r->scene->d, G[g], F, P, mats, compact, S[g]));
                }
                if (g == 0)
                    if (int e = EndTimed(d, ep)) return e;
                if (sort) PT_HIP(pt_launch_tile_order(r->slots, S[g], K, g));
            }
            r->rays += r->valid_slots;
        }
        return 0;
    };
    const int rc = rounds();
    for (uint32_t g = 1; g < K; g++) {
        PT_HIP(hipEventRecord(d->join_event[g - 1], S[g]));
        PT_HIP(hipStreamWaitEvent(d->stream, d->join_event[g - 1], 0));
    }
    return rc;
}

// k consecutive Run(1) calls: the same rounds with the same seeds (FrameIndex
// + 1 ... + k), as round batches (rounds_kernel) when the renderer allows
// them, else one ptRunBasicRenderer(1) per round.  round_batch: 0 automatic
// (AUTO_BATCH rounds per launch when every tile fits on the GPU at once, where
// the per-round launches cost most: C1 256x256 round 0.0176 -> 0.0055 ms;
// whole frames that do not fit run slower batched -- C3 0.431 vs 0.47-0.53
// ms per round, C2 -22 %: extend then runs at the shade kernel's occupancy and
// the block's waves wait at the round's barriers), 1 never, R >= 2 always R.
static int RunRounds(pt_device* d, pt_basic_renderer* r, uint64_t k)
{
    if (!r || CheckReady(r) != 0) return -1;
    uint32_t B = r->round_batch;
    if (B == 0) B = RoundFused(r, r->slots) && r->fused == 1 ? AUTO_BATCH : 1u;
    if (B > 1) {
        PT_HIP(hipSetDevice(d->id));
        if (int e = EnsureSpill(r)) return e;
        if (int e = SyncRecordForm(d, r)) return e;
        if (pt_rounds_available(r->slots)) {
            const ptd::dframe F = Frame(r);
            while (k > 0) {
                const uint32_t n = (uint32_t)std::min<uint64_t>(k, B);
                ptd::dparams P = Params(r, r->params.FrameIndex + 1);
                P.rounds = n;
                P.seed_step = 1;
                r->params.FrameIndex += n;
                // The profiling period counts rounds: a batch is timed when
                // one of its n rounds is a sampled one.
                const uint64_t t = d->run_tick % d->profile_period;
                const bool sampled = d->profiling && (t == 0 || t + n > d->profile_period);
                d->run_tick += n;
                event_pair ep{};
                if (int e = BeginTimed(d, PT_KERNEL_ROUNDS, ep, sampled, n)) return e;
                PT_HIP(pt_launch_rounds(r->scene->d, r->slots, F, P, ShadeMats(r), d->stream));
                if (int e = EndTimed(d, ep)) return e;
                // The batch's block times order the next batch.
                for (uint32_t g = 0; g < r->order_groups; g++)
                    PT_HIP(pt_launch_tile_order(r->slots, d->stream, r->order_groups, g));
                r->rays += r->valid_slots * n;
                k -= n;
            }
            return 0;
        }
    }
    const uint32_t K = SplitGroups(r);
    if (K > 1 && k > 1) return RunRoundsSplit(d, r, k, K);
    for (uint64_t i = 0; i < k; i++)
        if (int e = ptRunBasicRenderer(d, r, 1)) return e;
    return 0;
}

int ptRunBasicRendererRounds(pt_device* d, pt_basic_renderer* r, uint32_t count)
{
    if (!d) { SetError("null device"); return -1; }
    if (CheckReady(r) != 0) return -1;
    return RunRounds(d, r, count);
}

int ptSetBasicRendererRoundBatch(pt_basic_renderer* r, uint32_t rounds)
{
    if (!r) { SetError("ptSetBasicRendererRoundBatch: null renderer"); return -1; }
    r->round_batch = rounds;
    return 0;
}

int ptSetBasicRendererClassLists(pt_basic_renderer* r, uint32_t mode)
{
    if (!r || mode > 1) { SetError("ptSetBasicRendererClassLists: bad argument (0 automatic, 1 off)"); return -1; }
    r->class_lists = mode;
    return 0;
}

int ptGetBasicRendererClassLists(const pt_basic_renderer* r, uint32_t* used)
{
    if (!r || !used) { SetError("ptGetBasicRendererClassLists: null argument"); return -1; }
    *used = ClassListRounds(r) ? 1u : 0u;
    return 0;
}

int ptSetBasicRendererSplit(pt_basic_renderer* r, uint32_t groups)
{
    if (!r || groups > PT_MAX_SPLIT) {
        SetError("ptSetBasicRendererSplit: bad argument (groups 0..%u)", PT_MAX_SPLIT);
        return -1;
    }
    r->split = groups;
    return 0;
}

int ptGetBasicRendererSplit(const pt_basic_renderer* r, uint32_t* groups, uint32_t* timed_tiles, uint32_t* tiles)
{
    if (!r) { SetError("ptGetBasicRendererSplit: null renderer"); return -1; }
    const uint32_t K = SplitGroups(r);
    if (groups) *groups = K;
    if (timed_tiles) *timed_tiles = pt_tile_group_count(r->slots.tile_count, K, 0);
    if (tiles) *tiles = r->slots.tile_count;
    return 0;
}

int ptSetBasicRendererFusedRounds(pt_basic_renderer* r, int mode)
{
    if (!r || mode < 0 || mode > 2) { SetError("ptSetBasicRendererFusedRounds: bad argument"); return -1; }
    r->fused = mode;
    return 0;
}

int ptSetBasicRendererOpenPBR(pt_basic_renderer* r, int enable)
{
    if (!r || enable < 0 || enable > 1) { SetError("ptSetBasicRendererOpenPBR: bad argument"); return -1; }
    r->openpbr = enable;
    return 0;
}

// Counters of the work done since the last Reset: rays traced (every owned
// pixel's slot traces one ray per round, K3) and paths completed (the
// accumulator increments of basic_scatter.glsl:350-359, counted whether or
// not RENDER_FLAG_ACCUMULATE is set).  Synchronises the device stream.
int ptGetStats(pt_device* d, pt_basic_renderer* r, uint64_t* rays, uint64_t* samples)
{
    if (!d || !r) { SetError("null argument"); return -1; }
    PT_HIP(hipSetDevice(d->id));
    PT_WAIT(d);
    if (rays) *rays = r->rays;
    if (samples) {
        std::vector<uint32_t> w(r->slots.n / 64 + 1);
        PT_HIP(hipMemcpy(w.data(), r->done.ptr, w.size() * 4, hipMemcpyDeviceToHost));
        uint64_t sum = 0;
        for (uint32_t v : w) sum += v;
        *samples = sum;
    }
    return 0;
}

// n guarded Run(1) rounds (FrameIndex + 1 ... + n) on the device stream:
// each preceded by guard_kernel, the launches of a round past the target
// returning at once.  Returns the rounds that ran in *ran and leaves
// FrameIndex and the ray count as those rounds left them.
static int RunGuardedRounds(pt_device* d, pt_basic_renderer* r, uint32_t n, uint64_t target, uint32_t* ran)
{
    PT_HIP(hipSetDevice(d->id));
    if (int e = EnsureSpill(r)) return e;
    if (int e = SyncRecordForm(d, r)) return e;
    if (!r->guard.ptr) PT_HIP(r->guard.alloc(2));
    PT_HIP(hipMemsetAsync(r->guard.ptr, 0, 2 * sizeof(uint32_t), d->stream));
    ptd::dslots L = r->slots;
    L.stop = r->guard.ptr;
    const ptd::dframe F = Frame(r);
    const bool fused = RoundFused(r, L);
    const uint32_t mats = ShadeMats(r);
    const bool compact = ShadeCompact(r);
    const uint64_t base = r->params.FrameIndex;
    const bool lists = !fused && ClassListRounds(r);
    const uint32_t parity0 = r->cq_parity;
    for (uint32_t i = 0; i < n; i++) {
        PT_HIP(pt_launch_guard(r->done.ptr, r->slots.n / 64 + 1, target, r->guard.ptr, d->stream));
        const ptd::dparams P = Params(r, base + i + 1);
        if (fused) {
            PT_HIP(pt_launch_round(r->scene->d, L, F, P, mats, d->stream));
        } else {
            PT_HIP(pt_launch_extend(r->scene->d, L, F, L.spill, d->stream));
            if (lists) {
                if (int e = ClassListShade(d, r, L, F, P, d->stream)) return e;
            } else {
                PT_HIP(pt_launch_shade(r->scene->d, L, F, P, mats, compact, d->stream));
            }
        }
    }
    uint32_t flags[2] = {0, 0};
    PT_WAIT(d);
    PT_HIP(hipMemcpy(flags, r->guard.ptr, sizeof(flags), hipMemcpyDeviceToHost));
    *ran = flags[1];
    // A skipped round left the class-list counters alone: the parity
    // follows the rounds that ran.
    if (lists) r->cq_parity = parity0 ^ (flags[1] & 1u);
    r->params.FrameIndex = base + flags[1];
    r->rays += r->valid_slots * flags[1];
    d->run_tick += flags[1];
    r->order_tick += flags[1];
    return 0;
}

constexpr double GUARD_PREDICTED = 8.0;   // rounds left, by the last batch's rate, for the guarded end

// Benchmark-mode frame: Reset, Run(2) as after a restart
// (application.cpp:109-110), then Run(1) rounds -- one new seed each, as the
// application's frame loop issues them (application.cpp:100-115,
// basic.cpp:306-332) -- until the paths completed since the Reset reach
// target_samples (the accumulator's alpha sum) or max_rounds rounds ran.
//
// The frame ends at the reference's round -- the first whose total reaches
// the target -- unconditionally.  A round completes at most one path per
// owned pixel (px), so with `remaining` paths to go the first
// ceil(remaining / px) - 1 rounds cannot reach the target: every batch of
// rounds enqueued without a look at the count is at most ceil(remaining /
// px) long, its last round the first that may reach it.  The count is read
// back between batches.  When the last batch's completion rate says at most
// GUARD_PREDICTED rounds are left, the rounds run guarded instead: a device
// check before each round returns the round's launches at once when the
// target is already reached (RunGuardedRounds), so a rate that changes can
// cost a read-back but never a round.  The guarded end starts with the
// rounds that cannot overshoot, batched, and guards only the rest.  The
// rate decides only how the rounds are issued, never how many run.
// Measured on the C3 1024-spp frame (tools/exp_frame_end.py,
// profiles/r06_frame_end): 16 batches, +1.7 ms (0.16 %) against the same
// 2 760 rounds in one call with no read-back.
int ptRenderFrame(pt_device* d, pt_basic_renderer* r, uint64_t target_samples, uint32_t max_rounds,
                  uint32_t* rounds_out, uint64_t* samples_out)
{
    if (!d || !r) { SetError("null argument"); return -1; }
    if (max_rounds < 2) { SetError("ptRenderFrame: max_rounds must be >= 2"); return -1; }
    if (int e = ptResetBasicRenderer(d, r)) return e;
    if (int e = ptRunBasicRenderer(d, r, 2)) return e;
    uint32_t rounds = 2;
    uint64_t samples = 0, prev = 0;
    uint32_t last_batch = 0;
    const uint64_t px = std::max<uint64_t>(r->valid_slots, 1);   // paths one round can complete
    // The two rounds of Run(2) complete at most 2 px paths: the first batch
    // needs no read-back.
    if (target_samples > 2 * px) {
        const uint64_t k = std::min<uint64_t>((target_samples - 2 * px + px - 1) / px, max_rounds - rounds);
        if (k >= 1) {
            if (int e = RunRounds(d, r, k)) return e;
            rounds += (uint32_t)k;
            last_batch = rounds;   // the rate below: completions since the Reset per round
        }
    }
    for (;;) {
        if (int e = ptGetStats(d, r, nullptr, &samples)) return e;
        if (samples >= target_samples || rounds >= max_rounds) break;
        const uint64_t remaining = target_samples - samples;
        if (last_batch > 0 && samples > prev) {
            const double rate = (double)(samples - prev) / last_batch;   // completions per round
            const double predicted = (double)remaining / rate;
            if (predicted <= GUARD_PREDICTED) {
                // The last few rounds, with one read-back after them: first
                // the rounds that cannot overshoot, as one batch (its last
                // round may reach the target), then guarded single rounds
                // for the rest the rate predicts -- each returns at once
                // when the target is already reached, so the frame still
                // ends at the first round that reaches it.
                const uint64_t ks = std::min<uint64_t>((remaining + px - 1) / px, max_rounds - rounds);
                if (int e = RunRounds(d, r, ks)) return e;
                rounds += (uint32_t)ks;
                const double left = std::max(predicted - (double)ks, 0.0);
                const uint32_t n = (uint32_t)std::min<uint64_t>((uint64_t)(1.25 * left) + 2, max_rounds - rounds);
                uint32_t ran = 0;
                if (n >= 1)
                    if (int e = RunGuardedRounds(d, r, n, target_samples, &ran)) return e;
                rounds += ran;
                prev = samples;
                last_batch = (uint32_t)ks + ran;
                continue;
            }
        }
        const uint64_t k = std::min<uint64_t>((remaining + px - 1) / px, max_rounds - rounds);   // cannot overshoot
        if (int e = RunRounds(d, r, k)) return e;
        rounds += (uint32_t)k;
        prev = samples;
        last_batch = (uint32_t)k;
    }
    if (rounds_out) *rounds_out = rounds;
    if (samples_out) *samples_out = samples;
    return 0;
}

int ptReadBasicRendererStreamState(pt_device* d, pt_basic_renderer* r, uint32_t stream, pt_pixel_state* out)
{
    if (!d || !r || !out) { SetError("null argument"); return -1; }
    if (stream >= r->streams) { SetError("stream %u >= the renderer's %u streams", stream, r->streams); return -1; }
    PT_HIP(hipSetDevice(d->id));
    PT_WAIT(d);
    uint32_t n = r->slots.n;
    std::vector<float4> ray(n), hit(n), thr(n), prob(n);
    std::vector<float> lam(n);
    std::vector<float2> uv(n);
    std::vector<uint2> act(n);
    std::vector<uint16_t> pos(n);
    if (n && r->scene->valid) {
        // The slots hold compact hits; rebuild the reference's packed trace
        // records (normal, tangent, uv, material) for the readback.
        dbuf<float4> rec;
        dbuf<float2> ruv;
        PT_HIP(rec.alloc(n));
        PT_HIP(ruv.alloc(n));
        hipError_t e = pt_launch_finalize(r->scene->d, n, r->hit.ptr, r->uv.ptr, rec.ptr, ruv.ptr, d->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(d->stream);
        if (e == hipSuccess) e = hipMemcpy(hit.data(), rec.ptr, (size_t)n * 16, hipMemcpyDeviceToHost);
        if (e == hipSuccess) e = hipMemcpy(uv.data(), ruv.ptr, (size_t)n * 8, hipMemcpyDeviceToHost);
        rec.release();
        ruv.release();
        PT_HIP(e);
    }
    PT_HIP(hipMemcpy(ray.data(), r->ray.ptr, (size_t)n * 16, hipMemcpyDeviceToHost));
    PT_HIP(hipMemcpy(thr.data(), r->thr.ptr, (size_t)n * 16, hipMemcpyDeviceToHost));
    if (r->grey) {
        // Grey record form: the one stored Probability is all four components.
        std::vector<float> p1(n);
        PT_HIP(hipMemcpy(p1.data(), r->prob1.ptr, (size_t)n * 4, hipMemcpyDeviceToHost));
        for (uint32_t i = 0; i < n; i++) prob[i] = make_float4(p1[i], p1[i], p1[i], p1[i]);
    } else {
        PT_HIP(hipMemcpy(prob.data(), r->prob.ptr, (size_t)n * 16, hipMemcpyDeviceToHost));
    }
    PT_HIP(hipMemcpy(lam.data(), r->lam.ptr, (size_t)n * 4, hipMemcpyDeviceToHost));
    PT_HIP(hipMemcpy(act.data(), r->act.ptr, (size_t)n * 8, hipMemcpyDeviceToHost));
    PT_HIP(hipMemcpy(pos.data(), r->pos.ptr, (size_t)n * 2, hipMemcpyDeviceToHost));
    uint32_t W = r->buffer->width, H = r->buffer->height;
    auto bits = [](float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; };
    const uint32_t s0 = stream * r->stream_tiles * 256, s1 = s0 + r->stream_tiles * 256;
    for (uint32_t s = s0; s < s1; s++) {
        uint32_t t = (s >> 8) - stream * r->stream_tiles, l = s & 255u, k = t / r->tiles_x, tx = t - k * r->tiles_x;
        uint32_t x = tx * 16 + (l & 15u), y = (r->rank + k * r->nranks) * 16 + (l >> 4);
        if (x >= W || y >= H) continue;
        pt_pixel_state& O = out[(size_t)y * W + x];
        // Ray and hit records live at the slot's TileOrder positions.
        uint32_t qr = (s & ~255u) | (pos[s] >> 8u), qh = (s & ~255u) | (pos[s] & 255u);
        O.origin[0] = ray[qr].x; O.origin[1] = ray[qr].y; O.origin[2] = ray[qr].z;
        O.packed_velocity = bits(ray[qr].w);
        O.hit.time = hit[qh].x;
        O.hit.shape_material = bits(hit[qh].y);
        O.hit.packed_normal = bits(hit[qh].z);
        O.hit.packed_tangent = bits(hit[qh].w);
        O.hit.u = uv[qh].x;
        O.hit.v = uv[qh].y;
        O.lambda0 = lam[s];
        O.throughput[0] = thr[s].x; O.throughput[1] = thr[s].y; O.throughput[2] = thr[s].z; O.throughput[3] = thr[s].w;
        O.probability[0] = prob[s].x; O.probability[1] = prob[s].y; O.probability[2] = prob[s].z; O.probability[3] = prob[s].w;
        O.sample[0] = O.sample[1] = O.sample[2] = 0.0f;   // StorePathVertex (kernels.hip)
        O.active01 = act[s].x;
        O.active23 = act[s].y;
    }
    return 0;
}

int ptReadBasicRendererState(pt_device* d, pt_basic_renderer* r, pt_pixel_state* out)
{
    return ptReadBasicRendererStreamState(d, r, 0, out);
}

// Resume: the live path of every owned pixel of one stream from
// a saved pt_pixel_state (what ptReadBasicRendererStreamState returned between
// rounds).  Restored: the next ray (origin, packed velocity) and the path
// record (basic.glsl.inc:159-198: lambda0, throughput, probability, active
// stack).  Not restored: the trace record -- each round traces before it
// scatters (basic_trace.glsl then basic_scatter.glsl), so the next Run's
// extend replaces it before anything reads it; until then the readback
// reports a miss.  Sample must be 0: a live path's Sample is 0 between rounds
// (StorePathVertex, kernels.hip).  Checked before anything is written: every
// active-stack entry is 0xFFFF or a shape of the scene, lambda0 lies in
// [0, 1].
int ptWriteBasicRendererStreamState(pt_device* d, pt_basic_renderer* r, uint32_t stream, const pt_pixel_state* in)
{
    if (!d || !in) { SetError("null argument"); return -1; }
    if (CheckReady(r) != 0) return -1;
    if (stream >= r->streams) { SetError("stream %u >= the renderer's %u streams", stream, r->streams); return -1; }
    const uint32_t W = r->buffer->width, H = r->buffer->height;
    const uint32_t shapes = r->scene->d.g.ShapeCount;
    const uint32_t T = r->stream_tiles, s0 = stream * T * 256;
    std::vector<float4> ray((size_t)T * 256), thr((size_t)T * 256), prob((size_t)T * 256);
    std::vector<float> lam((size_t)T * 256);
    std::vector<uint2> act((size_t)T * 256);
    for (uint32_t i = 0; i < T * 256; i++) {
        const uint32_t t = i >> 8, l = i & 255u, k = t / r->tiles_x, tx = t - k * r->tiles_x;
        const uint32_t x = tx * 16 + (l & 15u), y = (r->rank + k * r->nranks) * 16 + (l >> 4);
        ray[i] = make_float4(0, 0, 0, 0);
        thr[i] = prob[i] = make_float4(0, 0, 0, 0);
        lam[i] = 0.0f;
        act[i] = make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);
        if (x >= W || y >= H) continue;
        const pt_pixel_state& S = in[(size_t)y * W + x];
        if (S.sample[0] != 0.0f || S.sample[1] != 0.0f || S.sample[2] != 0.0f) {
            SetError("pixel (%u, %u): a live path's sample is 0 between rounds", x, y);
            return -1;
        }
        if (!(S.lambda0 >= 0.0f && S.lambda0 <= 1.0f)) {   // R01() of basic_scatter.glsl:40 (can round to 1)
            SetError("pixel (%u, %u): lambda0 %g outside [0, 1]", x, y, (double)S.lambda0);
            return -1;
        }
        const uint32_t e[4] = {S.active01 & 0xFFFFu, S.active01 >> 16, S.active23 & 0xFFFFu, S.active23 >> 16};
        for (uint32_t v : e)
            if (v != 0xFFFFu && v >= shapes) {
                SetError("pixel (%u, %u): active shape %u >= the scene's %u shapes", x, y, v, shapes);
                return -1;
            }
        float w;
        std::memcpy(&w, &S.packed_velocity, 4);
        ray[i] = make_float4(S.origin[0], S.origin[1], S.origin[2], w);
        thr[i] = make_float4(S.throughput[0], S.throughput[1], S.throughput[2], S.throughput[3]);
        prob[i] = make_float4(S.probability[0], S.probability[1], S.probability[2], S.probability[3]);
        lam[i] = S.lambda0;
        act[i] = make_uint2(S.active01, S.active23);
    }
    PT_HIP(hipSetDevice(d->id));
    // The written records are four-float ones: the other streams' live paths
    // leave the grey form too; the next Run converts back when it can.
    if (r->grey) PT_HIP(pt_launch_grey_convert(r->slots, Frame(r), r->prob1.ptr, false, d->stream));
    r->grey = false;
    r->grey_blocked = false;
    r->slots.prob1 = nullptr;
    PT_WAIT(d);
    const size_t n = (size_t)T * 256;
    PT_HIP(hipMemcpy(r->thr.ptr + s0, thr.data(), n * 16, hipMemcpyHostToDevice));
    PT_HIP(hipMemcpy(r->prob.ptr + s0, prob.data(), n * 16, hipMemcpyHostToDevice));
    PT_HIP(hipMemcpy(r->lam.ptr + s0, lam.data(), n * 4, hipMemcpyHostToDevice));
    PT_HIP(hipMemcpy(r->act.ptr + s0, act.data(), n * 8, hipMemcpyHostToDevice));
    dbuf<float4> stage;
    hipError_t e = stage.upload(ray.data(), n);
    if (e == hipSuccess) e = pt_launch_restore_rays(r->slots, Frame(r), stage.ptr, s0 / 256, T, d->stream);
    if (e != hipSuccess) {
        stage.release();
        PT_HIP(e);
    }
    const int w = DeviceWait(d);
    stage.release();
    return w;
}

int ptWriteBasicRendererState(pt_device* d, pt_basic_renderer* r, const pt_pixel_state* in)
{
    return ptWriteBasicRendererStreamState(d, r, 0, in);
}

// A stream's own accumulator (width x height rgba32f; one stream: the sample
// buffer itself), for saving and restoring a multi-stream render.
static float4* StreamAccumulator(pt_basic_renderer* r, uint32_t stream)
{
    return r->streams == 1 ? r->buffer->accum : r->accx.ptr + (size_t)stream * r->buffer->width * r->buffer->height;
}

int ptReadBasicRendererStreamAccumulator(pt_device* d, pt_basic_renderer* r, uint32_t stream, float* rgba)
{
    if (!d || !r || !r->buffer || !rgba) { SetError("null argument"); return -1; }
    if (stream >= r->streams) { SetError("stream %u >= the renderer's %u streams", stream, r->streams); return -1; }
    PT_HIP(hipSetDevice(d->id));
    PT_HIP(hipMemcpyAsync(rgba, StreamAccumulator(r, stream), (size_t)r->buffer->width * r->buffer->height * 16,
                          hipMemcpyDeviceToHost, d->stream));
    PT_WAIT(d);
    return 0;
}

int ptWriteBasicRendererStreamAccumulator(pt_device* d, pt_basic_renderer* r, uint32_t stream, const float* rgba)
{
    if (!d || !r || !r->buffer || !rgba) { SetError("null argument"); return -1; }
    if (stream >= r->streams) { SetError("stream %u >= the renderer's %u streams", stream, r->streams); return -1; }
    PT_HIP(hipSetDevice(d->id));
    PT_HIP(hipMemcpyAsync(StreamAccumulator(r, stream), rgba, (size_t)r->buffer->width * r->buffer->height * 16,
                          hipMemcpyHostToDevice, d->stream));
    PT_WAIT(d);
    return 0;
}

static_assert(PT_SHADE_DIFFUSE == PT_MATS_DIFFUSE && PT_SHADE_METAL == PT_MATS_METAL &&
              PT_SHADE_TRANSLUCENT == PT_MATS_TRANSLUCENT && PT_SHADE_SCATTER == PT_MATS_SCATTER &&
              PT_SHADE_OPENPBR == PT_MATS_OPENPBR && PT_SHADE_PRIMS == PT_MATS_PRIMS && PT_SHADE_SKY == PT_MATS_SKY &&
              PT_SHADE_TEXWRAP == PT_MATS_TEXWRAP, "pt_api.h shade mask bits");

int ptGetBasicRendererShadeInfo(pt_basic_renderer* r, pt_shade_info* info)
{
    if (!r || !info) { SetError("null argument"); return -1; }
    if (!r->scene || !r->scene->valid) { SetError("renderer: scene has no valid packs (call ptUpdateScene)"); return -1; }
    info->scene_mask = ShadeMats(r);
    info->kernel_mask = pt_shade_mats(ShadeMats(r));
    info->completion_queue = ShadeCompact(r) ? 1u : 0u;
    info->grey_records = r->grey ? 1u : 0u;
    return 0;
}

pt_preview* ptCreatePreviewRenderContext(pt_device* d, pt_scene* s)
{
    if (!d || !s) { SetError("null argument"); return nullptr; }
    if (hipSetDevice(d->id) != hipSuccess) { SetError("hipSetDevice failed"); return nullptr; }
    pt_preview* c = new pt_preview;
    c->dev = d;
    c->scene = s;
    uint32_t none = 0xFFFFFFFFu;
    if (hipMalloc(&c->query, sizeof(uint32_t)) != hipSuccess ||
        hipMemcpy(c->query, &none, sizeof(none), hipMemcpyHostToDevice) != hipSuccess) {
        SetError("preview query buffer allocation failed");
        if (c->query) (void)hipFree(c->query);
        delete c;
        return nullptr;
    }
    if (c->observe.alloc(PT_OBSERVE_TABLE_FLOATS) != hipSuccess || pt_launch_observe_table(c->observe.ptr, d->stream) != hipSuccess) {
        SetError("preview table set-up failed");
        c->observe.release();
        (void)hipFree(c->query);
        delete c;
        return nullptr;
    }
    return c;
}

void ptDestroyPreviewRenderContext(pt_device* d, pt_preview* c)
{
    if (!c) return;
    if (d) (void)hipSetDevice(d->id);
    c->image.release();
    c->aov.release();
    c->spill.release();
    c->observe.release();
    if (c->query) (void)hipFree(c->query);
    delete c;
}

// RenderPreview (preview_render.cpp:118-181)
int ptRenderPreview(pt_device* d, pt_preview* c, const pt_preview_parameters* p)
{
    if (!d || !c || !p) { SetError("null argument"); return -1; }
    if (!c->scene->valid) { SetError("preview: scene has no valid packs (call ptUpdateScene)"); return -1; }
    if (p->RenderMode > PT_PREVIEW_RENDER_MODE_SCENE_COMPLEXITY) { SetError("bad preview mode %u", p->RenderMode); return -1; }
    if (p->RenderSizeX == 0 || p->RenderSizeY == 0 || p->RenderSizeX > 32768 || p->RenderSizeY > 32768) {
        SetError("bad preview size %ux%u", p->RenderSizeX, p->RenderSizeY);
        return -1;
    }
    PT_HIP(hipSetDevice(d->id));
    size_t n = (size_t)p->RenderSizeX * p->RenderSizeY;
    PT_HIP(c->image.alloc(n));
    PT_HIP(c->aov.alloc(n));
    uint32_t need = c->scene->stack_needed, cap = pt_preview_stack_cap();
    uint32_t* spill = nullptr;
    if (need > cap) {
        size_t threads = (size_t)((p->RenderSizeX + 15) / 16) * ((p->RenderSizeY + 15) / 16) * 256;
        PT_HIP(c->spill.alloc((need - cap) * threads));
        spill = c->spill.ptr;
    }
    event_pair ep{};
    if (int e = BeginTimed(d, PT_KERNEL_PREVIEW, ep)) return e;
    PT_HIP(pt_launch_preview(c->scene->d, p, spill, c->image.ptr, c->aov.ptr, c->query, c->observe.ptr, d->stream));
    if (int e = EndTimed(d, ep)) return e;
    c->width = p->RenderSizeX;
    c->height = p->RenderSizeY;
    c->rendered = true;
    return 0;
}

// RetrievePreviewQueryResult (preview_render.cpp:96-116)
int ptRetrievePreviewQueryResult(pt_device* d, pt_preview* c, uint32_t* hit_shape_index)
{
    if (!d || !c || !hit_shape_index) { SetError("null argument"); return -1; }
    PT_HIP(hipSetDevice(d->id));
    PT_HIP(hipMemcpyAsync(hit_shape_index, c->query, sizeof(uint32_t), hipMemcpyDeviceToHost, d->stream));
    PT_WAIT(d);
    return 0;
}

int ptReadPreviewImage(pt_device* d, pt_preview* c, float* rgba)
{
    if (!d || !c || !rgba) { SetError("null argument"); return -1; }
    if (!c->rendered) { SetError("preview not rendered"); return -1; }
    PT_HIP(hipSetDevice(d->id));
    PT_HIP(hipMemcpyAsync(rgba, c->image.ptr, (size_t)c->width * c->height * sizeof(float4), hipMemcpyDeviceToHost,
                          d->stream));
    PT_WAIT(d);
    return 0;
}

int ptReadPreviewAOVs(pt_device* d, pt_preview* c, pt_preview_aov* aov)
{
    if (!d || !c || !aov) { SetError("null argument"); return -1; }
    if (!c->rendered) { SetError("preview not rendered"); return -1; }
    PT_HIP(hipSetDevice(d->id));
    PT_HIP(hipMemcpyAsync(aov, c->aov.ptr, (size_t)c->width * c->height * sizeof(pt_preview_aov),
                          hipMemcpyDeviceToHost, d->stream));
    PT_WAIT(d);
    return 0;
}

int ptTraceRays(pt_device* d, pt_scene* s, uint32_t n, const float* origins, const uint32_t* vel, const float* dur,
                pt_hit_record* out)
{
    if (!d || !s || (n && (!origins || !vel || !dur || !out))) { SetError("null argument"); return -1; }
    if (!s->valid) { SetError("scene has no valid packs"); return -1; }
    if (n == 0) return 0;
    PT_HIP(hipSetDevice(d->id));
    bool spill = s->stack_needed > pt_extend_stack_cap();
    dbuf<float> d_o, d_t;
    dbuf<uint32_t> d_v, d_spill;
    dbuf<float4> d_hit, d_rec;
    dbuf<float2> d_hc, d_uv;
    hipError_t e = hipSuccess;
    do {
        if ((e = d_o.upload(origins, (size_t)n * 3)) != hipSuccess) break;
        if ((e = d_t.upload(dur, n)) != hipSuccess) break;
        if ((e = d_v.upload(vel, n)) != hipSuccess) break;
        if ((e = d_hit.alloc(n)) != hipSuccess || (e = d_rec.alloc(n)) != hipSuccess) break;
        if ((e = d_hc.alloc(n)) != hipSuccess || (e = d_uv.alloc(n)) != hipSuccess) break;
        if (spill && (e = d_spill.alloc((size_t)(s->stack_needed - pt_extend_stack_cap()) * n)) != hipSuccess) break;
        e = pt_launch_trace_rays(s->d, n, d_o.ptr, d_v.ptr, d_t.ptr, d_hit.ptr, d_hc.ptr, d_rec.ptr, d_uv.ptr,
                                 spill ? d_spill.ptr : nullptr, d->stream);
        if (e != hipSuccess) break;
        if ((e = hipStreamSynchronize(d->stream)) != hipSuccess) break;
        std::vector<float4> rec(n);
        std::vector<float2> uv(n);
        if ((e = hipMemcpy(rec.data(), d_rec.ptr, (size_t)n * 16, hipMemcpyDeviceToHost)) != hipSuccess) break;
        if ((e = hipMemcpy(uv.data(), d_uv.ptr, (size_t)n * 8, hipMemcpyDeviceToHost)) != hipSuccess) break;
        for (uint32_t i = 0; i < n; i++) {
            std::memcpy(&out[i].time, &rec[i].x, 4);
            std::memcpy(&out[i].shape_material, &rec[i].y, 4);
            std::memcpy(&out[i].packed_normal, &rec[i].z, 4);
            std::memcpy(&out[i].packed_tangent, &rec[i].w, 4);
            out[i].u = uv[i].x;
            out[i].v = uv[i].y;
        }
    } while (0);
    d_o.release(); d_t.release(); d_v.release(); d_spill.release();
    d_hit.release(); d_rec.release(); d_hc.release(); d_uv.release();
    if (e != hipSuccess) { SetError("ptTraceRays: %s", hipGetErrorString(e)); return (int)e; }
    return 0;
}

// Diagnostic: ptExtendStats's traversal counters for caller-given rays (the
// ptTraceRays inputs), plus each ray's step count (order-independent: a ray's
// traversal does not depend on its neighbours).
int ptTraceRaysStats(pt_device* d, pt_scene* s, uint32_t n, const float* origins, const uint32_t* vel,
                     const float* dur, uint64_t out[PT_EXTEND_STATS_COUNT], uint32_t* steps)
{
    if (!d || !s || !out || (n && (!origins || !vel || !dur))) { SetError("null argument"); return -1; }
    if (!s->valid) { SetError("scene has no valid packs"); return -1; }
    for (int i = 0; i < PT_EXTEND_STATS_COUNT; i++) out[i] = 0;
    if (n == 0) return 0;
    PT_HIP(hipSetDevice(d->id));
    bool spill = s->stack_needed > pt_extend_stack_cap();
    dbuf<float> d_o, d_t;
    dbuf<uint32_t> d_v, d_spill, d_steps;
    dbuf<float4> d_hit;
    dbuf<float2> d_hc;
    dbuf<unsigned long long> d_out;
    hipError_t e = hipSuccess;
    unsigned long long h[PT_EXTEND_STATS_COUNT] = {};
    do {
        if ((e = d_o.upload(origins, (size_t)n * 3)) != hipSuccess) break;
        if ((e = d_t.upload(dur, n)) != hipSuccess) break;
        if ((e = d_v.upload(vel, n)) != hipSuccess) break;
        if ((e = d_hit.alloc(n)) != hipSuccess || (e = d_hc.alloc(n)) != hipSuccess) break;
        if ((e = d_out.alloc(PT_EXTEND_STATS_COUNT)) != hipSuccess) break;
        if (steps && (e = d_steps.alloc(n)) != hipSuccess) break;
        if (spill && (e = d_spill.alloc((size_t)(s->stack_needed - pt_extend_stack_cap()) * n)) != hipSuccess) break;
        if ((e = hipMemsetAsync(d_out.ptr, 0, sizeof(h), d->stream)) != hipSuccess) break;
        e = pt_launch_trace_rays_stats(s->d, n, d_o.ptr, d_v.ptr, d_t.ptr, d_hit.ptr, d_hc.ptr,
                                       spill ? d_spill.ptr : nullptr, d_out.ptr, steps ? d_steps.ptr : nullptr,
                                       d->stream);
        if (e != hipSuccess) break;
        if ((e = hipMemcpyAsync(h, d_out.ptr, sizeof(h), hipMemcpyDeviceToHost, d->stream)) != hipSuccess) break;
        if (steps && (e = hipMemcpyAsync(steps, d_steps.ptr, (size_t)n * 4, hipMemcpyDeviceToHost, d->stream)) != hipSuccess)
            break;
        e = hipStreamSynchronize(d->stream);
    } while (0);
    d_o.release(); d_t.release(); d_v.release(); d_spill.release(); d_steps.release();
    d_hit.release(); d_hc.release(); d_out.release();
    if (e != hipSuccess) { SetError("ptTraceRaysStats: %s", hipGetErrorString(e)); return (int)e; }
    for (int i = 0; i < PT_EXTEND_STATS_COUNT; i++) out[i] = h[i];
    return 0;
}

int ptCheckFastDivision(pt_device* d, uint64_t n, uint32_t seed, uint64_t* mismatches)
{
    if (!d || !mismatches) { SetError("null argument"); return -1; }
    PT_HIP(hipSetDevice(d->id));
    unsigned long long* dm = nullptr;
    PT_HIP(hipMalloc(&dm, sizeof(unsigned long long)));
    hipError_t e = hipMemsetAsync(dm, 0, sizeof(unsigned long long), d->stream);
    if (e == hipSuccess) e = pt_launch_xdiv_check(n, seed, dm, d->stream);
    unsigned long long h = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&h, dm, sizeof(h), hipMemcpyDeviceToHost, d->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(d->stream);
    (void)hipFree(dm);
    if (e != hipSuccess) { SetError("ptCheckFastDivision: %s", hipGetErrorString(e)); return (int)e; }
    *mismatches = h;
    return 0;
}

int ptCheckFastReciprocal(pt_device* d, uint64_t* mismatches)
{
    if (!d || !mismatches) { SetError("null argument"); return -1; }
    PT_HIP(hipSetDevice(d->id));
    unsigned long long* dm = nullptr;
    PT_HIP(hipMalloc(&dm, sizeof(unsigned long long)));
    hipError_t e = hipMemsetAsync(dm, 0, sizeof(unsigned long long), d->stream);
    if (e == hipSuccess) e = pt_launch_rcp_check(dm, d->stream);
    unsigned long long h = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&h, dm, sizeof(h), hipMemcpyDeviceToHost, d->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(d->stream);
    (void)hipFree(dm);
    if (e != hipSuccess) { SetError("ptCheckFastReciprocal: %s", hipGetErrorString(e)); return (int)e; }
    *mismatches = h;
    return 0;
}

static int ExtendStats(pt_device* d, pt_basic_renderer* r, uint64_t* out, uint32_t* steps_out, const char* what)
{
    if (!d || (!out && !steps_out)) { SetError("null argument"); return -1; }
    if (CheckReady(r) != 0) return -1;
    PT_HIP(hipSetDevice(d->id));
    if (int e = EnsureSpill(r)) return e;
    unsigned long long* dm = nullptr;
    uint32_t* ds = nullptr;
    PT_HIP(hipMalloc(&dm, PT_EXTEND_STATS_COUNT * sizeof(unsigned long long)));
    hipError_t e = steps_out ? hipMalloc(&ds, (size_t)r->slots.n * 4) : hipSuccess;
    if (e == hipSuccess) e = hipMemsetAsync(dm, 0, PT_EXTEND_STATS_COUNT * sizeof(unsigned long long), d->stream);
    if (e == hipSuccess)
        e = pt_launch_extend_stats(r->scene->d, r->slots, Frame(r), r->slots.spill, dm, ds, d->stream);
    unsigned long long h[PT_EXTEND_STATS_COUNT] = {};
    if (e == hipSuccess) e = hipMemcpyAsync(h, dm, sizeof(h), hipMemcpyDeviceToHost, d->stream);
    if (e == hipSuccess && ds) e = hipMemcpyAsync(steps_out, ds, (size_t)r->slots.n * 4, hipMemcpyDeviceToHost, d->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(d->stream);
    (void)hipFree(dm);
    if (ds) (void)hipFree(ds);
    if (e != hipSuccess) { SetError("%s: %s", what, hipGetErrorString(e)); return (int)e; }
    if (out)
        for (int i = 0; i < PT_EXTEND_STATS_COUNT; i++) out[i] = h[i];
    return 0;
}

int ptExtendStats(pt_device* d, pt_basic_renderer* r, uint64_t out[PT_EXTEND_STATS_COUNT])
{
    return ExtendStats(d, r, out, nullptr, "ptExtendStats");
}

int ptExtendStepCounts(pt_device* d, pt_basic_renderer* r, uint32_t* steps)
{
    return ExtendStats(d, r, nullptr, steps, "ptExtendStepCounts");
}

int ptSetProfiling(pt_device* d, int enable)
{
    if (!d) { SetError("null device"); return -1; }
    if (int e = CollectTimes(d)) return e;
    d->profiling = enable != 0;
    return 0;
}

int ptSetProfilingPeriod(pt_device* d, uint32_t period)
{
    if (!d || period == 0) { SetError("bad argument"); return -1; }
    d->profile_period = period;
    d->run_tick = 0;
    return 0;
}

int ptGetKernelStats(pt_device* d, int kernel, uint64_t* launches, double* total_ms)
{
    if (!d || kernel < 0 || kernel >= PT_KERNEL_COUNT) { SetError("bad argument"); return -1; }
    PT_HIP(hipSetDevice(d->id));
    if (int e = CollectTimes(d)) return e;
    if (launches) *launches = d->launches[kernel];
    if (total_ms) *total_ms = d->total_ms[kernel];
    return 0;
}

int ptGetKernelRounds(pt_device* d, int kernel, uint64_t* rounds)
{
    if (!d || !rounds || kernel < 0 || kernel >= PT_KERNEL_COUNT) { SetError("bad argument"); return -1; }
    PT_HIP(hipSetDevice(d->id));
    if (int e = CollectTimes(d)) return e;
    *rounds = d->rounds[kernel];
    return 0;
}

int ptResetKernelStats(pt_device* d)
{
    if (!d) { SetError("null device"); return -1; }
    if (int e = CollectTimes(d)) return e;
    for (int k = 0; k < PT_KERNEL_COUNT; k++) { d->launches[k] = 0; d->rounds[k] = 0; d->total_ms[k] = 0; }
    return 0;
}

// --- RCCL ------------------------------------------------------------------------

int ptSceneStackNeeded(pt_scene* s, uint32_t* entries)
{
    if (!s || !entries) { SetError("null argument"); return -1; }
    *entries = s->stack_needed;
    return 0;
}

int ptSceneNodeCache(pt_scene* s, uint32_t* pairs)
{
    if (!s || !pairs) { SetError("null argument"); return -1; }
    *pairs = s->valid ? s->d.node_cache / 2 : 0u;
    return 0;
}

int ptCommGetUniqueId(uint8_t id[128])
{
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    ncclUniqueId u;
    ncclResult_t e = ncclGetUniqueId(&u);
    if (e != ncclSuccess) { SetError("ncclGetUniqueId: %s", ncclGetErrorString(e)); return (int)e; }
    std::memcpy(id, &u, 128);
    return 0;
}

pt_comm* ptCommCreate(pt_device* d, int nranks, int rank, const uint8_t id[128])
{
    if (!d || nranks < 1 || rank < 0 || rank >= nranks) { SetError("bad comm arguments"); return nullptr; }
    if (hipSetDevice(d->id) != hipSuccess) { SetError("hipSetDevice failed"); return nullptr; }
    ncclUniqueId u;
    std::memcpy(&u, id, 128);
    pt_comm* c = new pt_comm;
    c->dev = d;
    c->nranks = nranks;
    c->rank = rank;
    if (hipMalloc(&c->flag, sizeof(int)) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&c->host_flag), sizeof(int), hipHostMallocDefault) != hipSuccess) {
        SetError("comm flag allocation failed");
        if (c->flag) (void)hipFree(c->flag);
        delete c;
        return nullptr;
    }
    ncclResult_t e = ncclCommInitRank(&c->comm, nranks, u, rank);
    if (e != ncclSuccess) {
        SetError("ncclCommInitRank: %s", ncclGetErrorString(e));
        (void)hipFree(c->flag);
        (void)hipHostFree(c->host_flag);
        delete c;
        return nullptr;
    }
    d->comms.push_back(c);
    return c;
}

void ptCommDestroy(pt_comm* c)
{
    if (!c) return;
    if (pt_device* d = c->dev) {
        (void)hipSetDevice(d->id);
        auto& v = d->comms;
        v.erase(std::remove(v.begin(), v.end(), c), v.end());
        // A CommAgree readback left queued by a wait that failed (which
        // aborted the communicator) lands before the pinned word is freed:
        // the abort stops RCCL's kernels, and after an abort a wait gives up
        // within 10 s.
        if (c->aborted) (void)DeviceWait(d);
    }
    if (c->comm) (void)ncclCommDestroy(c->comm);
    if (c->flag) (void)hipFree(c->flag);
    if (c->host_flag) (void)hipHostFree(c->host_flag);
    delete c;
}

int ptCommSetTimeout(pt_comm* c, double seconds)
{
    if (!c || !(seconds > 0.0)) { SetError("ptCommSetTimeout: bad argument"); return -1; }
    c->timeout_s = seconds;
    return 0;
}

namespace {

int CommUsable(pt_device* d, pt_comm* c)
{
    if (!d || !c) { SetError("null argument"); return -1; }
    if (!c->dev) { SetError("communicator's device was destroyed"); return -1; }
    if (c->aborted || !c->comm) {
        SetError("communicator aborted after an earlier failure (rank %d of %d)", c->rank, c->nranks);
        return PT_ERROR_COMM_ABORTED;
    }
    if (c->dev != d) { SetError("communicator belongs to another device"); return -1; }
    return 0;
}

// A collective was just enqueued: its synchronous result and the
// communicator's asynchronous error state (non-blocking).  Any failure aborts
// the device's communicators, so no rank is left inside a collective whose
// peers have given up.
int CommEnqueued(pt_device* d, pt_comm* c, ncclResult_t e, const char* what)
{
    ncclResult_t st = ncclSuccess;
    if (e == ncclSuccess && ncclCommGetAsyncError(c->comm, &st) == ncclSuccess && (st == ncclSuccess || st == ncclInProgress))
        return 0;
    SetError("%s: %s; communicators aborted", what, ncclGetErrorString(e != ncclSuccess ? e : st));
    AbortComms(d);
    return PT_ERROR_COMM_ABORTED;
}

// Collective agreement on the caller's argument checks before a collective:
// every rank contributes `bad` (non-zero = its check failed) to a one-word
// max all-reduce and waits for it, so either every rank enters the
// collective or none does (a check failing on one rank only would otherwise
// leave the others blocked inside it).  Returns 0 when every rank passed.
int CommAgree(pt_device* d, pt_comm* c, int bad, const char* what)
{
    if (c->nranks == 1) return bad ? -1 : 0;
    // Pinned host word both ways: the copies are truly asynchronous, so a
    // hung peer is seen by DeviceWait's polling (a pageable copy would block
    // inside hipMemcpyAsync), and a readback still queued when the wait gives
    // up writes into memory that lives until ptCommDestroy.
    *c->host_flag = bad ? 1 : 0;
    PT_HIP(hipMemcpyAsync(c->flag, c->host_flag, sizeof(int), hipMemcpyHostToDevice, d->stream));
    ncclResult_t e = ncclAllReduce(c->flag, c->flag, 1, ncclInt32, ncclMax, c->comm, d->stream);
    if (int r = CommEnqueued(d, c, e, what)) return r;
    PT_HIP(hipMemcpyAsync(c->host_flag, c->flag, sizeof(int), hipMemcpyDeviceToHost, d->stream));
    PT_WAIT(d);
    const int h = *c->host_flag;
    if (h && !bad) {
        SetError("%s: the arguments failed their check on another rank; nothing was exchanged", what);
        return -1;
    }
    return h ? -1 : 0;
}

}  // namespace

int ptCommReduceSampleBuffer(pt_device* d, pt_comm* c, pt_sample_buffer* b, int root)
{
    if (int e = CommUsable(d, c)) return e;
    PT_HIP(hipSetDevice(d->id));
    // Argument checks, agreed on by every rank (CommAgree).  The rows zeroed
    // below are those outside the buffer's partition, so the partition must
    // be this communicator's rank of nranks.  A whole-frame buffer on a
    // multi-rank communicator is a sample shard: reducing it in place would
    // add the root's previous totals again on a repeated call.  (A one-rank
    // communicator sums nothing across ranks; it may reduce any partition --
    // the zeroing alone is then observable.)
    int bad = 0;
    if (!b) { SetError("null sample buffer"); bad = 1; }
    else if (root < 0 || root >= c->nranks) { SetError("bad root %d", root); bad = 1; }
    else if (b->nranks == 1 && c->nranks > 1) {
        SetError("ptCommReduceSampleBuffer: whole-frame buffer on a %d-rank communicator (sample shards: use "
                 "ptCommReduceSampleBufferInto)", c->nranks);
        bad = 1;
    } else if (c->nranks > 1 && b->nranks > 1 && ((int)b->nranks != c->nranks || (int)b->rank != c->rank)) {
        SetError("sample buffer partition %u/%u does not match communicator rank %d of %d", b->rank, b->nranks,
                 c->rank, c->nranks);
        bad = 1;
    }
    if (int e = CommAgree(d, c, bad, "ptCommReduceSampleBuffer")) return e;
    size_t count = (size_t)b->width * b->height * 4;
    // Only the bands this rank renders may enter the sum: at the root the
    // other rows hold the previous reduce's totals (a progressive frame
    // reduces again after more rounds), so they are zeroed first and the
    // in-place sum stays exact on every call.
    PT_HIP(pt_launch_zero_unowned(b->accum, b->width, b->height, b->rank, b->nranks, d->stream));
    ncclResult_t e = ncclReduce(b->accum, b->accum, count, ncclFloat32, ncclSum, root, c->comm, d->stream);
    return CommEnqueued(d, c, e, "ncclReduce");
}

int ptCommReduceSampleBufferInto(pt_device* d, pt_comm* c, pt_sample_buffer* b, pt_sample_buffer* total, int root)
{
    if (int e = CommUsable(d, c)) return e;
    PT_HIP(hipSetDevice(d->id));
    const bool is_root = c->rank == root;
    int bad = 0;
    if (!b) { SetError("null sample buffer"); bad = 1; }
    else if (root < 0 || root >= c->nranks) { SetError("bad root %d", root); bad = 1; }
    else if (is_root && (!total || total->width != b->width || total->height != b->height)) {
        SetError("ptCommReduceSampleBufferInto: the root needs a total buffer of the same size");
        bad = 1;
    }
    if (int e = CommAgree(d, c, bad, "ptCommReduceSampleBufferInto")) return e;
    size_t count = (size_t)b->width * b->height * 4;
    ncclResult_t e = ncclReduce(b->accum, is_root ? total->accum : b->accum, count, ncclFloat32, ncclSum, root, c->comm,
                                d->stream);
    return CommEnqueued(d, c, e, "ncclReduce");
}

// The same frame-end exchange with 1/N of the traffic: the bands are
// disjoint, so the root needs only each band's owner's rows.  Band b (rows
// [16b, 16b+16), contiguous in the row-major buffer) is owned by rank
// b % nranks; every non-root owner sends its bands to the root, which
// receives them in place.  One group of point-to-point transfers: each peer
// pushes ~1/N of the frame over its own xGMI link to the root concurrently,
// instead of a ring reduction of the whole buffer.
int ptCommGatherSampleBuffer(pt_device* d, pt_comm* c, pt_sample_buffer* b, int root)
{
    if (int e = CommUsable(d, c)) return e;
    PT_HIP(hipSetDevice(d->id));
    int bad = 0;
    if (!b) { SetError("null sample buffer"); bad = 1; }
    else if (root < 0 || root >= c->nranks) { SetError("bad root %d", root); bad = 1; }
    else if ((int)b->nranks != c->nranks || (int)b->rank != c->rank) {
        SetError("sample buffer partition %u/%u does not match communicator rank %d of %d", b->rank, b->nranks,
                 c->rank, c->nranks);
        bad = 1;
    }
    if (int e = CommAgree(d, c, bad, "ptCommGatherSampleBuffer")) return e;
    if (c->nranks == 1) return 0;
    uint32_t bands = (b->height + 15) / 16;
    ncclResult_t e = ncclGroupStart();
    for (uint32_t band = 0; band < bands && e == ncclSuccess; band++) {
        int owner = (int)(band % (uint32_t)c->nranks);
        if (owner == root) continue;
        uint32_t rows = std::min<uint32_t>(16u, b->height - band * 16u);
        float* p = reinterpret_cast<float*>(b->accum + (size_t)band * 16 * b->width);
        size_t count = (size_t)rows * b->width * 4;
        if (c->rank == owner) e = ncclSend(p, count, ncclFloat32, root, c->comm, d->stream);
        else if (c->rank == root) e = ncclRecv(p, count, ncclFloat32, owner, c->comm, d->stream);
    }
    ncclResult_t g = ncclGroupEnd();
    if (e == ncclSuccess) e = g;
    return CommEnqueued(d, c, e, "band gather");
}

}  // extern "C"
