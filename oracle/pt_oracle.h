/*
 * pt_oracle.h — CPU oracle for the wavefront path tracer.  TEST
 * INFRASTRUCTURE ONLY: linked by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py, never by the product library.
 *
 * A scalar, per-pixel restatement of the reference integrator
 * (src/integrator/basic_trace.glsl, basic_scatter.glsl, basic.glsl.inc,
 * src/scene/scene.glsl.inc, basic_{diffuse,metal,translucent}.glsl.inc,
 * src/core/{common,spectrum}.glsl.inc) and of its dispatch / seed schedule
 * (src/integrator/basic.cpp:285-332), under the numerics convention of
 * include/pt_fp.h.  Parity against the reference binary itself is unpinned:
 * the reference (Vulkan + glslc + glm) cannot be built or run in this
 * environment and ships no tests or golden data.
 */
#ifndef PT_ORACLE_H
#define PT_ORACLE_H

#include "../include/pt_api.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_renderer oracle_renderer;

/* Deep-copies the packs. threads = 0: OMP_NUM_THREADS, else hardware concurrency (<= 64). */
oracle_renderer* oracle_create(const pt_scene_packs* packs, uint32_t width, uint32_t height,
                               uint32_t rank, uint32_t nranks, int threads);
void oracle_destroy(oracle_renderer* r);
pt_basic_renderer_params* oracle_params(oracle_renderer* r);
/* OpenPBR shading on/off (ptSetBasicRendererOpenPBR); off by default. */
void oracle_set_openpbr(oracle_renderer* r, int enable);
void oracle_set_threads(oracle_renderer* r, int threads);
/* Slab-test division convention for every later Trace() in this process:
 * 1 = correctly rounded IEEE (Min-O) / V (default: the HIP kernels' and
 * SURVEY.md §7/§8(c)'s convention), 0 = reciprocal multiply
 * RN((Min-O) * RN(1/V)) (measurement only). */
void oracle_set_slab_division(int ieee);
int oracle_slab_division(void);
/* IntersectBoundingBox (common.glsl.inc:153-185) in the current convention: entry t or 1e30. */
float oracle_intersect_bounding_box(const float origin[3], const float velocity[3], float reach, const float mn[3],
                                    const float mx[3]);
void oracle_reset(oracle_renderer* r);
void oracle_run(oracle_renderer* r, uint32_t rounds);
void oracle_read_accum(oracle_renderer* r, float* rgba);
void oracle_read_state(oracle_renderer* r, pt_pixel_state* out);
/* Counters: rays traced and paths completed since creation. */
void oracle_counters(oracle_renderer* r, uint64_t* rays, uint64_t* samples);

/* Trace() of n rays against the packed scene. */
void oracle_trace_rays(const pt_scene_packs* packs, uint32_t n, const float* origins,
                       const uint32_t* packed_velocities, const float* durations, pt_hit_record* out);

/* RenderSampleBuffer (resolve.glsl:60-130) of n accumulator pixels:
 * out = OutColor (rgba32f), out8 = sRGB8 swapchain bytes (R,G,B,A). */
void oracle_resolve(const float* accum, uint32_t n, const pt_resolve_parameters* params, float* out, uint8_t* out8);

/* RenderPreview (preview_render.glsl:96-178) over RenderSizeX x RenderSizeY
 * pixels: OutColor rgba (4 floats/px), primary-hit AOVs, and the pick query
 * result (HitShapeIndex at MouseX, MouseY; untouched if outside). */
void oracle_preview(const pt_scene_packs* packs, const pt_preview_parameters* params, float* rgba, pt_preview_aov* aov,
                    uint32_t* hit_shape_index);

/* Convention kernels, exposed for known-answer tests. */
float oracle_fp_exp(float x);
float oracle_fp_log(float x);
float oracle_fp_sin(float x);
float oracle_fp_cos(float x);
float oracle_fp_atan2(float y, float x);
float oracle_fp_asin(float x);
uint32_t oracle_pcg(uint32_t* state);
uint32_t oracle_pack_unit_vector(const float v[3]);
float oracle_unpack_snorm16(uint32_t bits);
void oracle_unpack_unit_vector(uint32_t packed, float out[3]);
void oracle_sample_observer(float lambda, float out[3]);

#ifdef __cplusplus
}
#endif

#endif /* PT_ORACLE_H */
