/*
 * pt_api.h — C ABI of the MI355X wavefront path tracer (libpathtracer.so).
 *
 * Drop-in for the reference's integrator boundary.  Each entry point names the
 * reference interface it replaces (paths relative to the reference root):
 *
 *   ptCreateDevice            src/core/vulkan.hpp  CreateVulkan (device + queue)
 *   ptCreateScene             src/scene/scene.hpp:440  CreateVulkanScene
 *   ptUpdateScene             src/scene/scene.hpp:441  UpdateVulkanScene
 *   ptDestroyScene            src/scene/scene.hpp:442  DestroyVulkanScene
 *   ptCreateSampleBuffer      src/integrator/integrator.hpp:51  CreateSampleBuffer
 *   ptDestroySampleBuffer     src/integrator/integrator.hpp:53  DestroySampleBuffer
 *   ptCreateBasicRenderer     src/integrator/basic.hpp:28  CreateBasicRenderer
 *   ptDestroyBasicRenderer    src/integrator/basic.hpp:29  DestroyBasicRenderer
 *   ptResetBasicRenderer      src/integrator/basic.hpp:31  ResetBasicRenderer
 *   ptRunBasicRenderer        src/integrator/basic.hpp:32  RunBasicRenderer
 *   ptRenderSampleBuffer      src/integrator/integrator.hpp:55-60  RenderSampleBuffer
 *                             (resolve.glsl: XYZ -> sRGB, tone mapping)
 *   ptCreatePreviewRenderContext  src/application/preview_render.hpp:65-70
 *   ptDestroyPreviewRenderContext preview_render.hpp:72-76
 *   ptRenderPreview           preview_render.hpp:85-90  RenderPreview
 *   ptRetrievePreviewQueryResult  preview_render.hpp:78-83
 *   ptBasicRendererParams     src/integrator/basic.hpp:6-26  (the caller-written
 *                             CameraIndex / RenderFlags / PathLengthLimit /
 *                             PathTerminationProbability fields, FrameIndex)
 *
 * Additions (no reference counterpart): sample-buffer readback, explicit
 * synchronisation, a bit-exact ray query (ptTraceRays), slot-state readback,
 * per-kernel timing, pixel-band partitioning and an RCCL frame-end reduce for
 * one-process-per-GPU rendering.
 *
 * Conventions: creators return NULL on failure and set ptGetLastError();
 * other calls return 0 on success or a non-zero status (HIP / RCCL error
 * codes are forwarded).  ptDestroy* accept NULL.  Reset/Run enqueue work on
 * the device's stream and return immediately (the reference records into a
 * command buffer that executes after submit); reads and ptSynchronize block.
 */
#ifndef PT_API_H
#define PT_API_H

#include <stdint.h>
#include "pt_packed.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pt_device pt_device;
typedef struct pt_scene pt_scene;
typedef struct pt_sample_buffer pt_sample_buffer;
typedef struct pt_basic_renderer pt_basic_renderer;
typedef struct pt_comm pt_comm;
typedef struct pt_preview pt_preview;

/* Mutable renderer state (src/integrator/basic.hpp:18-25).  The caller writes
 * CameraIndex, RenderFlags, PathLengthLimit and PathTerminationProbability
 * before Reset/Run, exactly like application.cpp:104-107.  FrameIndex is the
 * seed schedule: Reset seeds with the current value, Run increments it first
 * and all rounds of one Run share the seed (basic.cpp:285-332). */
typedef struct pt_basic_renderer_params {
    uint32_t FrameIndex;
    uint32_t CameraIndex;
    uint32_t RenderFlags;                 /* PT_RENDER_FLAG_ACCUMULATE | _SAMPLE_JITTER */
    uint32_t PathLengthLimit;             /* unused by the reference integrator */
    float    PathTerminationProbability;
} pt_basic_renderer_params;

/* One trace result (src/integrator/basic.glsl.inc:32-38).  On a miss only
 * shape_material (= 0xFFFFFFFF) is meaningful, as in StoreTraceHit. */
typedef struct pt_hit_record {
    float    time;
    uint32_t shape_material;              /* shape << 16 | material */
    uint32_t packed_normal;               /* octahedral snorm16x2 */
    uint32_t packed_tangent;
    float    u, v;
} pt_hit_record;

/* Per-pixel integrator state (trace_buffer + path_buffer of
 * src/integrator/basic.glsl.inc:23-59), in image order.  Duration is not
 * stored: every producer writes HIT_TIME_LIMIT (scene.glsl.inc:617,
 * basic_scatter.glsl:163,307). */
typedef struct pt_pixel_state {
    float    origin[3];
    uint32_t packed_velocity;
    pt_hit_record hit;
    float    lambda0;
    float    throughput[4];
    float    probability[4];
    float    sample[3];
    uint32_t active01, active23;          /* 4 x u16 active shape stack, 0xFFFF = none */
} pt_pixel_state;

enum {
    PT_KERNEL_RAYGEN  = 0,
    PT_KERNEL_EXTEND  = 1,
    PT_KERNEL_SHADE   = 2,
    PT_KERNEL_RESOLVE = 3,
    PT_KERNEL_PREVIEW = 4,
    PT_KERNEL_ROUND   = 5,   /* fused extend + shade of a small partition (one launch per round) */
    PT_KERNEL_ROUNDS  = 6,   /* a round batch: several rounds of every tile in one launch */
    PT_KERNEL_COUNT   = 7,
};

/* resolve_parameters (src/integrator/integrator.hpp:12-48). */
enum {
    PT_TONE_MAPPING_CLAMP    = 0,
    PT_TONE_MAPPING_REINHARD = 1,
    PT_TONE_MAPPING_HABLE    = 2,
    PT_TONE_MAPPING_ACES     = 3,
};

/* preview_render_mode (src/application/preview_render.hpp:3-13). */
enum {
    PT_PREVIEW_RENDER_MODE_BASE_COLOR        = 0,
    PT_PREVIEW_RENDER_MODE_BASE_COLOR_SHADED = 1,
    PT_PREVIEW_RENDER_MODE_NORMAL            = 2,
    PT_PREVIEW_RENDER_MODE_MATERIAL_INDEX    = 3,
    PT_PREVIEW_RENDER_MODE_PRIMITIVE_INDEX   = 4,
    PT_PREVIEW_RENDER_MODE_MESH_COMPLEXITY   = 5,
    PT_PREVIEW_RENDER_MODE_SCENE_COMPLEXITY  = 6,
};

/* preview_parameters (preview_render.hpp:22-33). */
typedef struct pt_preview_parameters {
    pt_packed_transform CameraTransform;
    uint32_t RenderMode;
    float    Brightness;
    uint32_t SelectedShapeIndex;          /* 0xFFFFFFFF = none */
    uint32_t RenderSizeX, RenderSizeY;
    uint32_t MouseX, MouseY;
} pt_preview_parameters;

/* Per-pixel primary-hit AOVs of the preview: Trace()'s hit (scene.glsl.inc:
 * 102-119) for the pixel's primary ray. */
typedef struct pt_preview_aov {
    float    time;
    uint32_t shape_index;                 /* 0xFFFFFFFF on a miss (other fields 0) */
    uint32_t material_index;
    uint32_t primitive_index;
    uint32_t mesh_complexity;             /* BLAS nodes visited (Hit.MeshComplexity) */
    uint32_t scene_complexity;            /* TLAS nodes visited (Hit.SceneComplexity) */
    float    normal[3];                   /* world normal, not quantised */
    float    u, v;
    uint32_t reserved;
} pt_preview_aov;

typedef struct pt_resolve_parameters {
    float    Brightness;                  /* default 1 */
    uint32_t ToneMappingMode;             /* PT_TONE_MAPPING_*, default CLAMP */
    float    ToneMappingWhiteLevel;       /* Reinhard white level, default 1 */
} pt_resolve_parameters;

const char* ptGetLastError(void);

pt_device* ptCreateDevice(int hip_device);
void       ptDestroyDevice(pt_device* device);
int        ptSynchronize(pt_device* device);
int        ptGetDeviceCount(int* count);

pt_scene* ptCreateScene(pt_device* device);
int       ptUpdateScene(pt_device* device, pt_scene* scene, const pt_scene_packs* packs, uint32_t dirty_flags);
void      ptDestroyScene(pt_device* device, pt_scene* scene);
/* Encodings chosen per scene at ptUpdateScene (no effect on results; the
 * wider forms are what larger scenes need, so tests force them on small
 * ones).  Stack format: AUTO = 16-bit entries when every TLAS / BLAS entry
 * fits, else packed 32-bit BLAS words when every node fits, else node
 * indices; WORDS32 / NODE_INDEX force the wider forms.  Hit record: AUTO =
 * the hit face's vertex indices when they fit 21 bits, else its face index;
 * FACE_INDEX forces the latter.  Take effect at the next ptUpdateScene. */
enum {
    PT_STACK_FORMAT_AUTO       = 0,
    PT_STACK_FORMAT_WORDS32    = 1,
    PT_STACK_FORMAT_NODE_INDEX = 2,
    PT_HIT_RECORD_AUTO         = 0,
    PT_HIT_RECORD_FACE_INDEX   = 1,
};
int       ptSetSceneStackFormat(pt_scene* scene, uint32_t format);
int       ptSetSceneHitRecordForm(pt_scene* scene, uint32_t form);
/* Traversal stack entries the uploaded scene can need (TLAS depth + deepest
 * BLAS depth, each capped at the reference's Stack[32]); the extend kernel keeps
 * 20 in LDS and spills the rest to a per-ray global buffer. */
int       ptSceneStackNeeded(pt_scene* scene, uint32_t* entries);
/* BLAS child pairs the extend kernel keeps in LDS for the uploaded scene
 * (the top levels of its BLASes, laid out first in the device node array;
 * 0 = no cache: scenes whose stack entries need 32 bits, or no mesh). */
int       ptSceneNodeCache(pt_scene* scene, uint32_t* pairs);

pt_sample_buffer* ptCreateSampleBuffer(pt_device* device, uint32_t width, uint32_t height);
void              ptDestroySampleBuffer(pt_device* device, pt_sample_buffer* buffer);
/* rgba = width*height*4 floats: CIE XYZ sums + sample count, row-major. */
int               ptReadSampleBuffer(pt_device* device, pt_sample_buffer* buffer, float* rgba);
/* Overwrites the accumulator (e.g. to resume accumulation from a saved one). */
int               ptWriteSampleBuffer(pt_device* device, pt_sample_buffer* buffer, const float* rgba);
/* RenderSampleBuffer: resolves the accumulator into the buffer's display
 * image on the device stream (resolve.glsl:112-128). */
int               ptRenderSampleBuffer(pt_device* device, pt_sample_buffer* buffer, const pt_resolve_parameters* params);
/* Display image of the last ptRenderSampleBuffer: the fragment shader's
 * OutColor (rgba32f, alpha 1) ... */
int               ptReadResolvedImage(pt_device* device, pt_sample_buffer* buffer, float* rgba);
/* ... and its 8-bit sRGB encoding as a B8G8R8A8_SRGB swapchain stores it
 * (bytes R,G,B,A per pixel). */
int               ptReadResolvedImageSRGB8(pt_device* device, pt_sample_buffer* buffer, uint8_t* rgba8);

pt_basic_renderer* ptCreateBasicRenderer(pt_device* device, pt_scene* scene, pt_sample_buffer* buffer);
/* Renderer owning only the 16-row pixel bands b with b % nranks == rank. */
pt_basic_renderer* ptCreateBasicRendererPartitioned(pt_device* device, pt_scene* scene, pt_sample_buffer* buffer,
                                                    uint32_t rank, uint32_t nranks);
/* Path streams for a partition too small to fill the GPU:
 * the renderer carries `streams` independent paths per owned pixel, stream k
 * seeded with FrameIndex + (k << 24) -- the sample shards' offsets -- so one
 * launch holds streams x the partition's slots.  With more than one stream
 * each stream accumulates into an accumulator of its own, and
 * ptMergeBasicRendererStreams writes their sum, in stream order, into the
 * sample buffer's owned pixels (call it before reading or exchanging a
 * frame; it may repeat as the rounds go on).  Each stream's state and
 * accumulator equal a one-stream renderer's started at its FrameIndex
 * offset. */
pt_basic_renderer* ptCreateBasicRendererStreams(pt_device* device, pt_scene* scene, pt_sample_buffer* buffer,
                                                uint32_t rank, uint32_t nranks, uint32_t streams);
int                ptMergeBasicRendererStreams(pt_device* device, pt_basic_renderer* renderer);
uint32_t           ptBasicRendererStreams(pt_basic_renderer* renderer);
void               ptDestroyBasicRenderer(pt_device* device, pt_basic_renderer* renderer);
pt_basic_renderer_params* ptBasicRendererParams(pt_basic_renderer* renderer);
int                ptResetBasicRenderer(pt_device* device, pt_basic_renderer* renderer);
int                ptRunBasicRenderer(pt_device* device, pt_basic_renderer* renderer, uint32_t rounds);
uint32_t           ptBasicRendererSlotCount(pt_basic_renderer* renderer);
/* Fused rounds: 0 = never (extend then shade launches), 1 = automatic (one
 * extend+shade launch per round when every tile of the renderer fits on the
 * GPU at once: a rank's share of a strongly scaled frame), 2 = whenever the
 * scene allows (no spilled traversal stack).  Results are identical in every
 * mode.  Default 1. */
int                ptSetBasicRendererFusedRounds(pt_basic_renderer* renderer, int mode);
/* Consecutive rounds: ptRunBasicRendererRounds(d, r, k) is k calls of
 * ptRunBasicRenderer(d, r, 1) -- the application's frame loop, one new
 * FrameIndex per round (application.cpp:100-115) -- with identical results.
 * Round batches run up to R of those rounds in one launch, each tile
 * advancing through them without a grid-wide barrier between rounds (a slot's
 * round depends only on its own previous round).  ptSetBasicRendererRoundBatch:
 * 0 = automatic (16 rounds per launch when every tile of the renderer fits on
 * the GPU at once and fused rounds are automatic, else one round per launch
 * pair), 1 = never, R >= 2 = R whenever the scene allows (no spilled stack).
 * Default 0.  ptRenderFrame runs its Run(1) rounds this way. */
int                ptRunBasicRendererRounds(pt_device* device, pt_basic_renderer* renderer, uint32_t count);
int                ptSetBasicRendererRoundBatch(pt_basic_renderer* renderer, uint32_t rounds);
/* Tile groups on concurrent streams (no reference counterpart: a launch
 * schedule).  Consecutive rounds that run one launch pair per round
 * (ptRunBasicRendererRounds, ptRenderFrame) split the renderer's tiles into K
 * groups (tile t in group t % K); each group runs the batch's rounds on its
 * own HIP stream, so one group's launches fill the CUs another group's
 * kernel tail leaves idle.  The device stream forks before the batch and
 * joins after it, and every wait covers the groups.  Results are identical
 * for every K.  groups: 0 = automatic (3 when the rounds run unfused over at
 * least 2 048 tiles, else 1), 1 = off, 2..PT_MAX_SPLIT = that many (4 takes
 * every hardware queue of the process and measured slower).
 * ptGetBasicRendererSplit reports the K that consecutive rounds use now, the
 * tiles of group 0 (the launches kernel profiling times) and all tiles; any
 * pointer may be NULL.  Default 0. */
#define PT_MAX_SPLIT 4
/* Class-pure shade inside tile groups (no reference counterpart: a launch
 * schedule).  In scenes with more than one material type, the rounds of a
 * tile group shade through per-class lists of the round's rays, so that each
 * wave shades one material class. Results are identical.  mode: 0 =
 * automatic (on for such scenes in tile groups), 1 = off.
 * ptGetBasicRendererClassLists sets *used to 1 when consecutive rounds use
 * them now.  Default 0. */
int                ptSetBasicRendererClassLists(pt_basic_renderer* renderer, uint32_t mode);
int                ptGetBasicRendererClassLists(const pt_basic_renderer* renderer, uint32_t* used);
int                ptSetBasicRendererSplit(pt_basic_renderer* renderer, uint32_t groups);
int                ptGetBasicRendererSplit(const pt_basic_renderer* renderer, uint32_t* groups, uint32_t* timed_tiles,
                                           uint32_t* tiles);
/* OpenPBR shading (opt-in extension, no reference counterpart): 0 (default)
 * = an OpenPBR hit ends its path with no contribution, as in the reference,
 * whose integrator does not compile its OpenPBR BSDF (scene.glsl.inc:685);
 * 1 = shade OpenPBR materials with the layered sampler and medium of
 * src/scene/openpbr.glsl.inc (deviations in DESIGN.md §6). */
int                ptSetBasicRendererOpenPBR(pt_basic_renderer* renderer, int enable);
/* Work done since the last Reset: rays traced (one per owned pixel per round)
 * and paths completed (accumulator sample increments, basic_scatter.glsl:
 * 350-359).  Either pointer may be NULL.  Synchronises the device stream. */
int                ptGetStats(pt_device* device, pt_basic_renderer* renderer, uint64_t* rays, uint64_t* samples);
/* Benchmark-mode frame (no reference entry point: the
 * application loop of application.cpp:100-115 with an spp target): Reset,
 * Run(2), then Run(1) rounds until the paths completed since the Reset reach
 * target_samples (e.g. spp * pixels owned) or max_rounds (>= 2) rounds ran.
 * The frame always ends at the first round whose total reaches the target,
 * as the loop issued one round at a time would (the rounds are batched only
 * where they cannot overshoot, the last few guarded on the device).
 * Blocks until done.  rounds_out / samples_out (either may be NULL): rounds
 * run and paths completed. */
int                ptRenderFrame(pt_device* device, pt_basic_renderer* renderer, uint64_t target_samples,
                                 uint32_t max_rounds, uint32_t* rounds_out, uint64_t* samples_out);
/* out = width*height states in image order; pixels outside the renderer's
 * partition are left untouched.  Stream 0's paths (ptReadBasicRendererStreamState:
 * any stream's). */
int                ptReadBasicRendererState(pt_device* device, pt_basic_renderer* renderer, pt_pixel_state* out);
int                ptReadBasicRendererStreamState(pt_device* device, pt_basic_renderer* renderer, uint32_t stream,
                                                  pt_pixel_state* out);
/* Resume (no reference counterpart; the reference restarts paths on Reset,
 * basic_scatter.glsl:330-336): restores the live path of every owned pixel
 * of stream 0 (or `stream`) from `in` (width*height states in image order, as
 * ptReadBasicRendererState returned them between rounds; other pixels are not
 * read): the next ray and the path record (lambda0, throughput, probability,
 * active shapes).  The trace record is not restored -- the next Run traces
 * the restored ray before it scatters, so it is not needed; the readback shows
 * a miss until then.  With the accumulator (ptWriteSampleBuffer) and
 * FrameIndex restored too, the following Runs equal the uninterrupted
 * render's bit for bit.  Fails, writing nothing, if a sample is non-zero (a
 * live path's is 0 between rounds), a lambda0 lies outside [0, 1] or an
 * active entry is neither 0xFFFF nor a shape of the scene.  Synchronises. */
int                ptWriteBasicRendererState(pt_device* device, pt_basic_renderer* renderer, const pt_pixel_state* in);
int                ptWriteBasicRendererStreamState(pt_device* device, pt_basic_renderer* renderer, uint32_t stream,
                                                   const pt_pixel_state* in);
/* A path stream's own accumulator (width*height*4 floats, as
 * ptReadSampleBuffer): with one stream it is the sample buffer; with several,
 * the per-stream sums ptMergeBasicRendererStreams adds up.  Saving and
 * restoring every stream's accumulator and state resumes a multi-stream
 * render bit for bit. */
int                ptReadBasicRendererStreamAccumulator(pt_device* device, pt_basic_renderer* renderer, uint32_t stream,
                                                        float* rgba);
int                ptWriteBasicRendererStreamAccumulator(pt_device* device, pt_basic_renderer* renderer,
                                                         uint32_t stream, const float* rgba);

/* Diagnostic: the shade variant the renderer runs (chosen on the host from
 * the scene's packs at ptUpdateScene and from the renderer's options; no
 * effect on results).  Mask bits: material types present, a scattering
 * medium, analytic shapes, sky light sampling that matters (the host cannot
 * prove SkyboxSamplingProbability * pdf an exact +0), texture placements
 * outside the unit square. */
enum {
    PT_SHADE_DIFFUSE     = 1,
    PT_SHADE_METAL       = 2,
    PT_SHADE_TRANSLUCENT = 4,
    PT_SHADE_SCATTER     = 8,
    PT_SHADE_OPENPBR     = 16,
    PT_SHADE_PRIMS       = 32,
    PT_SHADE_SKY         = 64,
    PT_SHADE_TEXWRAP     = 128,
};
typedef struct pt_shade_info {
    uint32_t scene_mask;        /* PT_SHADE_* of the scene as the renderer shades it */
    uint32_t kernel_mask;       /* the instantiation launched: the smallest superset built
                                   (PT_SHADE_DIFFUSE alone = the lean diffuse-mesh kernel) */
    uint32_t completion_queue;  /* 1: completed paths restart through the block's queue
                                   (the separate extend / shade launches; fused rounds do not queue) */
    uint32_t grey_records;      /* 1: live paths keep one Probability float and no stack
                                   (as of the last Reset / Run / state write) */
} pt_shade_info;
int                ptGetBasicRendererShadeInfo(pt_basic_renderer* renderer, pt_shade_info* info);

/* Editor preview (preview_render.glsl:96-178): one primary ray per pixel of
 * RenderSizeX x RenderSizeY through the same Trace() as the integrator.
 * RenderPreview enqueues; the reads synchronise.  The query result is the
 * shape index under (MouseX, MouseY) of the last render (0xFFFFFFFF = sky or
 * no render yet; a mouse position outside the image leaves it unchanged, as
 * the reference's query buffer). */
pt_preview* ptCreatePreviewRenderContext(pt_device* device, pt_scene* scene);
void        ptDestroyPreviewRenderContext(pt_device* device, pt_preview* context);
int         ptRenderPreview(pt_device* device, pt_preview* context, const pt_preview_parameters* params);
int         ptRetrievePreviewQueryResult(pt_device* device, pt_preview* context, uint32_t* hit_shape_index);
/* rgba: RenderSizeX * RenderSizeY * 4 floats (OutColor); aov: one record per pixel. */
int         ptReadPreviewImage(pt_device* device, pt_preview* context, float* rgba);
int         ptReadPreviewAOVs(pt_device* device, pt_preview* context, pt_preview_aov* aov);

/* Bit-exact Trace() (scene.glsl.inc:522-611) of n rays: origins (3n floats),
 * packed unit velocities (n), durations (n) -> n hit records. */
int ptTraceRays(pt_device* device, pt_scene* scene, uint32_t n, const float* origins,
                const uint32_t* packed_velocities, const float* durations, pt_hit_record* out);

/* Diagnostic: evaluates the device's exact fast division helper (XDiv: an
 * FMA-corrected reciprocal, no longer on the traversal path since the slab
 * test's reciprocal convention) against IEEE division on n
 * device-generated operand pairs; returns the number of bit mismatches
 * (must be 0). */
int ptCheckFastDivision(pt_device* device, uint64_t n, uint32_t seed, uint64_t* mismatches);

/* Diagnostic: evaluates the device's fast reciprocal (hardware rcp + one
 * FMA Newton step) on every float d with 2^-126 <= |d| < 2^126 against the
 * IEEE quotient 1.0f / d; returns the number of bit mismatches (must be 0). */
int ptCheckFastReciprocal(pt_device* device, uint64_t* mismatches);

/* Diagnostic: runs the extend step on the renderer's current rays with
 * traversal counters.  It writes the same hit records the next Run's extend
 * writes first, so the render is not perturbed.  out = {rays, lane steps, wave steps x 64, internal nodes,
 * BLAS leaves, faces tested, stack pops, TLAS leaves, waves, then the internal
 * BLAS wave steps by the number of distinct nodes among the wave's lanes
 * taking them: 1, 2, 3-4, 5-8, more than 8}. */
#define PT_EXTEND_STATS_COUNT 14
int ptExtendStats(pt_device* device, pt_basic_renderer* renderer, uint64_t out[PT_EXTEND_STATS_COUNT]);
/* Diagnostic, same pass: the traversal step count of every ray, per ray
 * POSITION (steps[q], q < width-rounded slot count; 0 where no ray). */
int ptExtendStepCounts(pt_device* device, pt_basic_renderer* renderer, uint32_t* steps);

/* Diagnostic, caller-given rays (the ptTraceRays inputs): the counters of
 * ptExtendStats and, if steps != NULL, each ray's traversal step count. */
int ptTraceRaysStats(pt_device* device, pt_scene* scene, uint32_t n, const float* origins,
                     const uint32_t* packed_velocities, const float* durations,
                     uint64_t out[PT_EXTEND_STATS_COUNT], uint32_t* steps);

/* Per-kernel device time, measured with HIP events on the renderer stream. */
int ptSetProfiling(pt_device* device, int enable);
/* Time only the kernels of every period-th round (default 1; rounds counted
 * across ptRunBasicRenderer calls): each event pair around a kernel costs
 * issue time, so a timed loop can sample its kernels' durations instead of
 * bracketing every launch. */
int ptSetProfilingPeriod(pt_device* device, uint32_t period);
int ptGetKernelStats(pt_device* device, int kernel, uint64_t* launches, double* total_ms);
/* Rounds covered by the timed launches of `kernel` (one per launch, except a
 * round batch, PT_KERNEL_ROUNDS, which covers its rounds): total_ms / rounds
 * is the kernel's time per round. */
int ptGetKernelRounds(pt_device* device, int kernel, uint64_t* rounds);
int ptResetKernelStats(pt_device* device);

/* RCCL communicator over one process per GPU (xGMI).
 *
 * Failure contract: every ptComm* exchange first agrees
 * on its argument checks across the ranks (a one-word all-reduce), so a
 * check that fails on any rank fails the call on every rank and nothing is
 * exchanged.  While a communicator is live, every call that waits for the
 * device stream (ptSynchronize, the reads, ptGetStats, ptRenderFrame,
 * ptUpdateScene, the comm calls' own checks) polls the stream, RCCL's
 * asynchronous error state and the communicator's deadline instead of
 * blocking: on an RCCL error it aborts the device's communicators
 * (ncclCommAbort) and returns PT_ERROR_COMM_ABORTED, at the deadline
 * PT_ERROR_TIMEOUT.  An aborted communicator fails every later call with
 * PT_ERROR_COMM_ABORTED; destroy it (and the process normally exits). */
enum {
    PT_ERROR_COMM_ABORTED = -2,
    PT_ERROR_TIMEOUT      = -3,
};
int      ptCommGetUniqueId(uint8_t id[128]);
pt_comm* ptCommCreate(pt_device* device, int nranks, int rank, const uint8_t id[128]);
void     ptCommDestroy(pt_comm* comm);
/* Deadline of a wait on the device stream while the communicator is live
 * (default 600 s: longer than any frame of the benchmark configurations). */
int      ptCommSetTimeout(pt_comm* comm, double seconds);
/* Frame-end ncclReduce(sum) of the float4 accumulator to `root` (exact: the
 * ranks' pixel bands are disjoint).  Each rank first zeroes the rows outside
 * the bands of the last partitioned renderer created on the buffer, so the
 * root's buffer may be reduced again after further rounds (progressive
 * frames): after every call it holds the sum of the ranks' own bands. */
int      ptCommReduceSampleBuffer(pt_device* device, pt_comm* comm, pt_sample_buffer* buffer, int root);
/* The same frame-end exchange at 1/N of the traffic: every rank's own bands
 * go point-to-point to `root`, which stores them in place (grouped
 * ncclSend/ncclRecv).  Requires the buffer's partition (the last partitioned
 * renderer created on it) to be this communicator's rank of nranks.  After
 * the call the root's buffer holds every rank's bands; other ranks' buffers
 * are unchanged.  Repeatable after further rounds. */
int      ptCommGatherSampleBuffer(pt_device* device, pt_comm* comm, pt_sample_buffer* buffer, int root);
/* Sample sharding (north_star: "pixels/samples shard ... RCCL reduce of the
 * per-pixel radiance and sample-count buffers at frame end"): every rank
 * renders the whole frame with its own RNG stream (a FrameIndex offset per
 * rank) and keeps its own running accumulator; this out-of-place
 * ncclReduce(sum) leaves in `total` on `root` the sum over ranks of their
 * XYZ radiance sums and sample counts, which the resolve averages.  The
 * ranks' own accumulators are unchanged, so the call may repeat after more
 * rounds (progressive frames).  `total` is read only on `root` (may be NULL
 * elsewhere) and must match `buffer`'s size. */
int      ptCommReduceSampleBufferInto(pt_device* device, pt_comm* comm, pt_sample_buffer* buffer,
                                      pt_sample_buffer* total, int root);

#ifdef __cplusplus
}
#endif

#endif /* PT_API_H */
