// kernels.hpp — launch interface between runtime.cpp and kernels.hip.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../../include/pt_packed.h"
#include "../../../include/pt_api.h"

namespace ptd {

struct dscene;

// ShadeOrder outcome classes of a traced ray (kernels.hip).
constexpr uint32_t PT_OUTCOME_CLASSES = 5;   // hit: diffuse, metal, translucent, other material; miss

// Per-slot state, SoA of 16-byte records.
struct dslots {
    float4* ray;        // origin.xyz, packed velocity
    float4* hit;        // compact hit: time, shape index, primitive index, coords.x
    float2* uv;         // compact hit: coords.y, coords.z
    float4* thr;        // throughput[4]
    float4* prob;       // probability[4]
    float* prob1;       // grey record form (non-null): the path's Probability, whose four components
                        // are equal, as one float; prob and act are then not read (GreyRecord, kernels.hip)
    float* lam;         // normalized lambda0 (a live path's Sample is always 0: StorePathVertex)
    uint2* act;         // active-shape stack (2 x u16 pairs)
    uint16_t* pos;      // per slot: position of its current ray (high byte) and of
                        // its last traced hit (low byte) within its tile (TileOrder)
    uint8_t* slotof;    // per position: the slot (within the tile) whose ray sits there
    uint64_t* outcome;  // ShadeOrder, per tile [class][4 words]: bit t set iff the ray at position t
                        // ended in that class (extend): hit diffuse / metal / translucent / other, miss
    uint32_t* tilecost; // per tile and wave: the wave's extend time (s_memtime ticks)
    uint32_t* order;    // extend's block -> tile map (longest previous extend first), or null
    uint32_t* done;     // per wave of 64 slots: paths completed by shade since the last Reset (ptGetStats)
    uint32_t* spill;    // traversal stack spill: (needed - LDS capacity) rows x n
    const uint32_t* stop = nullptr;   // guarded rounds (ptRenderFrame's last rounds): set -> the launch returns
    uint32_t n;
    uint32_t tile_count;    // n / 256: one block per tile
};

struct dframe {
    float4* accum;      // width x height, XYZ sum + count
    uint32_t width, height;
    uint32_t rank, nranks;
    uint32_t tiles_x;
    uint32_t tiles_x_magic;   // ceil(2^32 / tiles_x): t / tiles_x = umulhi(t, magic)
                              // for t * tiles_x < 2^32 (checked at renderer creation)
    // Path streams (ptCreateBasicRendererStreams): the renderer's tiles are
    // `streams` copies of its owned tiles, stream k's seeds offset by k << 24
    // and its paths accumulated in accx[k] (one stream: in accum itself).
    uint32_t streams;         // 1: one path per owned pixel
    uint32_t stream_tiles;    // tiles per stream
    uint32_t stream_magic;    // ceil(2^32 / stream_tiles) (streams > 1)
    float4* accx;             // streams x width x height (streams > 1)
};

struct dparams {
    uint32_t camera_index;
    uint32_t render_flags;
    float termination_probability;
    uint32_t seed;
    // Round batches (rounds_kernel): rounds per launch, and the seed step
    // between them (1: consecutive Run(1) calls, 0: one Run(R)).
    uint32_t rounds = 1;
    uint32_t seed_step = 0;
};

}  // namespace ptd

hipError_t pt_launch_raygen(const ptd::dscene& S, const ptd::dslots& L, const ptd::dframe& F, const ptd::dparams& P,
                            hipStream_t st);
hipError_t pt_launch_extend(const ptd::dscene& S, const ptd::dslots& L, const ptd::dframe& F, uint32_t* spill,
                            hipStream_t st);
hipError_t pt_launch_extend_stats(const ptd::dscene& S, const ptd::dslots& L, const ptd::dframe& F, uint32_t* spill,
                                  unsigned long long* out, uint32_t* steps, hipStream_t st);
// Material-type mask of a scene (shade kernel specialisation).
enum : uint32_t {
    PT_MATS_DIFFUSE = 1,
    PT_MATS_METAL = 2,
    PT_MATS_TRANSLUCENT = 4,
    PT_MATS_SCATTER = 8,
    PT_MATS_ALL = 15,
    PT_MATS_OPENPBR = 16,     // OpenPBR shapes shaded (ptSetBasicRendererOpenPBR); instantiated as ALL | OPENPBR
    PT_MATS_PRIMS = 32,       // some shape is a plane, sphere or cube (else every shape is a mesh instance)
    PT_MATS_SKY = 64,         // SkyboxSamplingProbability != 0 (sky light sampling can be drawn)
    PT_MATS_SCENE = PT_MATS_PRIMS | PT_MATS_SKY,
    PT_MATS_TEXWRAP = 128,    // some texture's atlas placement lies outside [0, 1] (host mask only: no lean kernel)
};
uint32_t pt_shade_mats(uint32_t scene_mats);
// Grey record form (kernels.hip GreyRecord): the shade mask keeps every path's
// Probability wavelength-uniform and its active-shape stack empty.
constexpr bool pt_grey_mats(uint32_t shade_mats) { return !(shade_mats & (PT_MATS_TRANSLUCENT | PT_MATS_OPENPBR)); }
// Record-form conversions of a renderer's live paths (between rounds):
// counts the valid slots whose Probability components differ or whose stack
// is not empty (a path that cannot take the grey form); converts every valid
// slot's record to the grey form (to_grey) or back to the four-float form.
// State write: rays[i] = the restored ray of slot tile0 * 256 + i, for
// `tiles` tiles; stored at their TileOrder positions, every hit a miss.
hipError_t pt_launch_restore_rays(const ptd::dslots& L, const ptd::dframe& F, const float4* rays, uint32_t tile0,
                                  uint32_t tiles, hipStream_t st);
hipError_t pt_launch_grey_check(const ptd::dslots& L, const ptd::dframe& F, uint32_t* count, hipStream_t st);
hipError_t pt_launch_grey_convert(const ptd::dslots& L, const ptd::dframe& F, float* prob1, bool to_grey,
                                  hipStream_t st);
// Preview base-colour tables: the 16 sample constants of ObserveUnderD65
// (preview.hip), filled once per preview context.
constexpr uint32_t PT_OBSERVE_TABLE_FLOATS = 16 * 5;
hipError_t pt_launch_observe_table(float* table, hipStream_t st);
hipError_t pt_launch_preview(const ptd::dscene& S, const pt_preview_parameters* p, uint32_t* spill, float4* out,
                             pt_preview_aov* aov, uint32_t* query, const float* observe_table, hipStream_t st);
uint32_t pt_preview_stack_cap();
hipError_t pt_launch_resolve(const float4* accum, uint32_t n, float brightness, uint32_t mode, float white, float4* out,
                             uint32_t* out8, hipStream_t st);
// compact: the completion-queue instantiation (ShadeTile), for scenes whose
// paths also end at surfaces.
hipError_t pt_launch_shade(const ptd::dscene& S, const ptd::dslots& L, const ptd::dframe& F, const ptd::dparams& P,
                           uint32_t scene_mats, bool compact, hipStream_t st);
// Class-pure shade (kernels.hip shade_classq_kernel): per-class lists of the
// round's positions built by class_list_kernel, each class's list CQ_SUB
// sub-lists of pt_classq_sub_capacity words; counts: the PT_OUTCOME_CLASSES x
// CQ_SUB counters of this round (zero at the launch), next_counts: the other
// parity's, cleared for the next round.  L is a tile group's slots (the
// group's tile_count; tiles_all, groups, group: pt_tile_group_tile).  For the
// shade instantiations pt_class_lists_supported accepts.
constexpr uint32_t CQ_SUB = 1;
inline uint32_t pt_classq_sub_capacity(uint32_t tiles) { return (tiles + CQ_SUB - 1) / CQ_SUB * 256; }
bool pt_class_lists_supported(uint32_t scene_mats);
hipError_t pt_launch_shade_classq(const ptd::dscene& S, const ptd::dslots& L, const ptd::dframe& F,
                                  const ptd::dparams& P, uint32_t scene_mats, bool compact, uint32_t* counts,
                                  uint32_t* next_counts, uint32_t* list, hipStream_t st, uint32_t tiles_all = 0,
                                  uint32_t groups = 1, uint32_t group = 0);
hipError_t pt_launch_vertex_decode(const uint2* v, uint32_t n, float4* attr, float* vv, hipStream_t st);
// Tile groups (ptSetBasicRendererSplit): group g of K owns tiles g, g + K, ...
// (pt_tile_group_count of them) and the dispatch-order segment starting at
// pt_tile_group_start.  pt_launch_tile_order sorts one group's segment
// longest-first (groups = 1: the whole frame).
__host__ __device__ inline uint32_t pt_tile_group_count(uint32_t tiles, uint32_t groups, uint32_t group)
{
    return group < tiles ? (tiles - group + groups - 1) / groups : 0u;
}
// The i-th tile of a group.
__host__ __device__ inline uint32_t pt_tile_group_tile(uint32_t tiles, uint32_t groups, uint32_t group, uint32_t i)
{
    return group + i * groups;
}
__host__ __device__ inline uint32_t pt_tile_group_start(uint32_t tiles, uint32_t groups, uint32_t group)
{
    uint32_t s = 0;
    for (uint32_t h = 0; h < group; h++) s += pt_tile_group_count(tiles, groups, h);
    return s;
}
hipError_t pt_launch_tile_order(const ptd::dslots& L, hipStream_t st, uint32_t groups = 1, uint32_t group = 0);
// Guarded rounds (ptRenderFrame): flags[0] := 1 once the done words' sum (the
// paths completed since the Reset, ptGetStats) reaches target; while it is
// 0, flags[1] counts the rounds that run.
hipError_t pt_launch_guard(const uint32_t* done, uint32_t words, uint64_t target, uint32_t* flags, hipStream_t st);
// Fused round (extend + shade per tile in one launch, round_kernel): the
// tiles the GPU can hold at once for this scene (0: not available), and the
// launch (hipErrorNotSupported when the scene needs a spilled stack).
uint32_t pt_round_capacity(uint32_t scene_mats, bool stack16, uint32_t cu_count);
hipError_t pt_launch_round(const ptd::dscene& S, const ptd::dslots& L, const ptd::dframe& F, const ptd::dparams& P,
                           uint32_t scene_mats, hipStream_t st);
// Round batch: P.rounds rounds (extend + shade) of every tile in one launch,
// each block running its own tile through all of them (rounds_kernel).
hipError_t pt_launch_rounds(const ptd::dscene& S, const ptd::dslots& L, const ptd::dframe& F, const ptd::dparams& P,
                            uint32_t scene_mats, hipStream_t st);
bool pt_rounds_available(const ptd::dslots& L);
// Zeroes the rows of a sample buffer outside a renderer's 16-row bands
// (b % nranks != rank) before a frame-end reduce.
hipError_t pt_launch_zero_unowned(float4* accum, uint32_t width, uint32_t height, uint32_t rank, uint32_t nranks,
                                  hipStream_t st);
// Path streams' merge into the sample buffer's accumulator (owned bands).
hipError_t pt_launch_merge_streams(float4* accum, float4* accx, uint32_t width, uint32_t height, uint32_t rank,
                                   uint32_t nranks, uint32_t streams, hipStream_t st);
// Packed row-major atlas (w x h texels per layer) -> AtlasIndex block layout;
// needs w % 4 == 0 and h % 2 == 0.
hipError_t pt_launch_atlas_tile(const float4* src, float4* dst, uint32_t w, uint32_t h, uint32_t layers, hipStream_t st);
hipError_t pt_launch_rcp_check(unsigned long long* mismatches, hipStream_t st);
hipError_t pt_launch_xdiv_check(uint64_t n, uint32_t seed, unsigned long long* mismatches, hipStream_t st);
// Diagnostic: the traversal counters of ptExtendStats for caller-given rays.
hipError_t pt_launch_trace_rays_stats(const ptd::dscene& S, uint32_t n, const float* origins, const uint32_t* vel,
                                      const float* dur, float4* hit, float2* hc, uint32_t* spill,
                                      unsigned long long* out, uint32_t* steps, hipStream_t st);
hipError_t pt_launch_trace_rays(const ptd::dscene& S, uint32_t n, const float* origins, const uint32_t* vel,
                                const float* dur, float4* hit, float2* hc, float4* rec, float2* uv, uint32_t* spill,
                                hipStream_t st);
hipError_t pt_launch_finalize(const ptd::dscene& S, uint32_t n, const float4* hit, const float2* hc, float4* rec,
                              float2* uv, hipStream_t st);
uint32_t pt_extend_stack_cap();
