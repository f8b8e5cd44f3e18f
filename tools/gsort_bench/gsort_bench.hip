// Microbenchmark of the global ray sort pass (kernels.hip "Global ray sort")
// on real keys (dump_keys.py): where do count / scan / scatter spend their
// time, and do cheaper formulations exist?
//
//   base     the renderer's pass: count (LDS histogram per chunk, one global
//            atomic per nonzero bin), scan, scatter (recount, one returning
//            global atomic per nonzero bin reserves the chunk's range, LDS
//            atomics assign positions);
//   noatom   count with plain stores instead of the global atomics (timing
//            only: how much of count is the atomics);
//   ticket   count takes the chunk's offset inside each bin from a RETURNING
//            global atomic (stored per chunk and bin) and each slot's rank
//            inside its (chunk, bin) from the LDS atomic (stored per slot);
//            the scatter is then a stream: q = cursor[k] + chunkoff + rank;
//   ticket16 the same with 16 384-slot chunks.
// Build: hipcc --offload-arch=gfx950 -O3 -o gsort_bench gsort_bench.hip
// Run:   ./gsort_bench keys.bin
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } \
    } while (0)

constexpr uint32_t BINS = 4096;
constexpr uint32_t TH = 1024;

__global__ void empty_kernel() {}

template <uint32_t CHUNK>
__global__ __launch_bounds__(TH) void count_base(const uint16_t* key, uint32_t n, uint32_t* hist)
{
    __shared__ uint32_t cnt[BINS];
    for (uint32_t b = threadIdx.x; b < BINS; b += TH) cnt[b] = 0;
    __syncthreads();
    const uint32_t s0 = blockIdx.x * CHUNK;
#pragma unroll
    for (uint32_t i = 0; i < CHUNK / TH; i++) {
        uint32_t s = s0 + i * TH + threadIdx.x;
        if (s < n) atomicAdd(&cnt[key[s]], 1u);
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < BINS; b += TH)
        if (uint32_t c = cnt[b]) atomicAdd(&hist[b], c);
}

template <uint32_t CHUNK>
__global__ __launch_bounds__(TH) void count_noatom(const uint16_t* key, uint32_t n, uint32_t* dummy)
{
    __shared__ uint32_t cnt[BINS];
    for (uint32_t b = threadIdx.x; b < BINS; b += TH) cnt[b] = 0;
    __syncthreads();
    const uint32_t s0 = blockIdx.x * CHUNK;
#pragma unroll
    for (uint32_t i = 0; i < CHUNK / TH; i++) {
        uint32_t s = s0 + i * TH + threadIdx.x;
        if (s < n) atomicAdd(&cnt[key[s]], 1u);
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < BINS; b += TH)
        if (uint32_t c = cnt[b]) dummy[(size_t)blockIdx.x * BINS + b] = c;
}

template <uint32_t CHUNK>
__global__ __launch_bounds__(TH) void count_ticket(const uint16_t* key, uint32_t n, uint32_t* hist, uint32_t* chunkoff,
                                                   uint16_t* rank)
{
    __shared__ uint32_t cnt[BINS];
    for (uint32_t b = threadIdx.x; b < BINS; b += TH) cnt[b] = 0;
    __syncthreads();
    const uint32_t s0 = blockIdx.x * CHUNK;
#pragma unroll
    for (uint32_t i = 0; i < CHUNK / TH; i++) {
        uint32_t s = s0 + i * TH + threadIdx.x;
        if (s < n) rank[s] = (uint16_t)atomicAdd(&cnt[key[s]], 1u);
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < BINS; b += TH)
        if (uint32_t c = cnt[b]) chunkoff[(size_t)blockIdx.x * BINS + b] = atomicAdd(&hist[b], c);
}

__global__ __launch_bounds__(TH) void scan(uint32_t* hist, uint32_t* cursor, uint32_t* nvalid)
{
    constexpr uint32_t PER = BINS / TH;
    __shared__ uint32_t wsum[TH / 64];
    const uint32_t t = threadIdx.x, b0 = t * PER;
    uint32_t local[PER], sum = 0;
    for (uint32_t i = 0; i < PER; i++) { local[i] = hist[b0 + i]; sum += local[i]; }
    uint32_t incl = sum;
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t v = (uint32_t)__shfl_up((int)incl, o, 64);
        if ((t & 63u) >= (uint32_t)o) incl += v;
    }
    if ((t & 63u) == 63u) wsum[t >> 6] = incl;
    __syncthreads();
    uint32_t before = 0;
    for (uint32_t w = 0; w < (t >> 6); w++) before += wsum[w];
    uint32_t run = before + incl - sum;
    for (uint32_t i = 0; i < PER; i++) { cursor[b0 + i] = run; run += local[i]; hist[b0 + i] = 0; }
    if (t == TH - 1) *nvalid = run;
}

template <uint32_t CHUNK>
__global__ __launch_bounds__(TH) void scatter_base(const uint16_t* key, uint32_t n, uint32_t* cursor, uint32_t* gpos,
                                                   uint32_t* perm)
{
    __shared__ uint32_t cnt[BINS];
    for (uint32_t b = threadIdx.x; b < BINS; b += TH) cnt[b] = 0;
    __syncthreads();
    const uint32_t s0 = blockIdx.x * CHUNK;
    uint32_t k[CHUNK / TH];
#pragma unroll
    for (uint32_t i = 0; i < CHUNK / TH; i++) {
        uint32_t s = s0 + i * TH + threadIdx.x;
        k[i] = s < n ? key[s] : 0u;
        if (s < n) atomicAdd(&cnt[k[i]], 1u);
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < BINS; b += TH)
        if (uint32_t c = cnt[b]) cnt[b] = atomicAdd(&cursor[b], c);
    __syncthreads();
#pragma unroll
    for (uint32_t i = 0; i < CHUNK / TH; i++) {
        uint32_t s = s0 + i * TH + threadIdx.x;
        if (s >= n) continue;
        uint32_t q = atomicAdd(&cnt[k[i]], 1u);
        gpos[s] = q;
        perm[q] = s;
    }
}

template <uint32_t CHUNK>
__global__ __launch_bounds__(256) void scatter_ticket(const uint16_t* key, uint32_t n, const uint32_t* cursor,
                                                      const uint32_t* chunkoff, const uint16_t* rank, uint32_t* gpos,
                                                      uint32_t* perm)
{
    uint32_t s = blockIdx.x * 256 + threadIdx.x;
    if (s >= n) return;
    uint32_t k = key[s];
    uint32_t q = cursor[k] + chunkoff[(size_t)(s / CHUNK) * BINS + k] + rank[s];
    gpos[s] = q;
    perm[q] = s;
}


// Block-shape variants of base's count / scatter (NT threads, CHUNK slots).
template <uint32_t CHUNK, uint32_t NT>
__global__ __launch_bounds__(NT) void count_nt(const uint16_t* key, uint32_t n, uint32_t* hist)
{
    __shared__ uint32_t cnt[BINS];
    for (uint32_t b = threadIdx.x; b < BINS; b += NT) cnt[b] = 0;
    __syncthreads();
    const uint32_t s0 = blockIdx.x * CHUNK;
#pragma unroll
    for (uint32_t i = 0; i < CHUNK / NT; i++) {
        uint32_t s = s0 + i * NT + threadIdx.x;
        if (s < n) atomicAdd(&cnt[key[s]], 1u);
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < BINS; b += NT)
        if (uint32_t c = cnt[b]) atomicAdd(&hist[b], c);
}

// LDS histogram in 4 copies (lane & 3): same-key lanes of a wave conflict 4x less.
template <uint32_t CHUNK>
__global__ __launch_bounds__(TH) void count_copies(const uint16_t* key, uint32_t n, uint32_t* hist)
{
    __shared__ uint32_t cnt[4 * BINS];
    for (uint32_t b = threadIdx.x; b < 4 * BINS; b += TH) cnt[b] = 0;
    __syncthreads();
    const uint32_t s0 = blockIdx.x * CHUNK, c = threadIdx.x & 3u;
#pragma unroll
    for (uint32_t i = 0; i < CHUNK / TH; i++) {
        uint32_t s = s0 + i * TH + threadIdx.x;
        if (s < n) atomicAdd(&cnt[key[s] * 4 + c], 1u);
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < BINS; b += TH) {
        uint4 v = *reinterpret_cast<const uint4*>(&cnt[b * 4]);
        if (uint32_t t = v.x + v.y + v.z + v.w) atomicAdd(&hist[b], t);
    }
}

// Keys loaded 8 per thread as one uint4 (contiguous slots per thread).
template <uint32_t CHUNK>
__global__ __launch_bounds__(TH) void count_vec(const uint16_t* key, uint32_t n, uint32_t* hist)
{
    __shared__ uint32_t cnt[BINS];
    for (uint32_t b = threadIdx.x; b < BINS; b += TH) cnt[b] = 0;
    __syncthreads();
    const uint32_t s0 = blockIdx.x * CHUNK + threadIdx.x * 8;
    if (s0 + 8 <= n) {
        uint4 v = *reinterpret_cast<const uint4*>(key + s0);
        uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; j++) {
            atomicAdd(&cnt[w[j] & 0xFFFFu], 1u);
            atomicAdd(&cnt[w[j] >> 16], 1u);
        }
    } else {
        for (uint32_t s = s0; s < n && s < s0 + 8; s++) atomicAdd(&cnt[key[s]], 1u);
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < BINS; b += TH)
        if (uint32_t c = cnt[b]) atomicAdd(&hist[b], c);
}

template <uint32_t CHUNK, uint32_t NT>
__global__ __launch_bounds__(NT) void scatter_nt(const uint16_t* key, uint32_t n, uint32_t* cursor, uint32_t* perm)
{
    __shared__ uint32_t cnt[BINS];
    for (uint32_t b = threadIdx.x; b < BINS; b += NT) cnt[b] = 0;
    __syncthreads();
    const uint32_t s0 = blockIdx.x * CHUNK;
    uint32_t k[CHUNK / NT];
#pragma unroll
    for (uint32_t i = 0; i < CHUNK / NT; i++) {
        uint32_t s = s0 + i * NT + threadIdx.x;
        k[i] = s < n ? key[s] : 0u;
        if (s < n) atomicAdd(&cnt[k[i]], 1u);
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < BINS; b += NT)
        if (uint32_t c = cnt[b]) cnt[b] = atomicAdd(&cursor[b], c);
    __syncthreads();
#pragma unroll
    for (uint32_t i = 0; i < CHUNK / NT; i++) {
        uint32_t s = s0 + i * NT + threadIdx.x;
        if (s >= n) continue;
        perm[atomicAdd(&cnt[k[i]], 1u)] = s;
    }
}

static bool check(const std::vector<uint16_t>& keys, const uint32_t* dperm, uint32_t n);

template <class CountF, class ScatterF>
static void run_variant(const char* name, const std::vector<uint16_t>& keys, CountF count, ScatterF scatter,
                        uint32_t* hist, uint32_t* cursor, uint32_t* nvalid, uint32_t* perm, hipEvent_t* ev, int reps)
{
    const uint32_t n = (uint32_t)keys.size();
    float tc = 0, ts = 0, tx = 0;
    bool ok = true;
    for (int it = 0; it < reps + 2; it++) {
        float m;
        CK(hipEventRecord(ev[0]));
        count();
        CK(hipEventRecord(ev[1]));
        hipLaunchKernelGGL(scan, dim3(1), dim3(TH), 0, 0, hist, cursor, nvalid);
        CK(hipEventRecord(ev[2]));
        scatter();
        CK(hipEventRecord(ev[3]));
        CK(hipEventSynchronize(ev[3]));
        if (it == 0) ok = check(keys, perm, n);
        if (it >= 2) {
            CK(hipEventElapsedTime(&m, ev[0], ev[1])); tc += m;
            CK(hipEventElapsedTime(&m, ev[1], ev[2])); ts += m;
            CK(hipEventElapsedTime(&m, ev[2], ev[3])); tx += m;
        }
    }
    printf("  %-22s count %.2f scan %.2f scatter %.2f us | valid %d\n", name, tc / reps * 1e3, ts / reps * 1e3,
           tx / reps * 1e3, (int)ok);
}

static bool check(const std::vector<uint16_t>& keys, const uint32_t* dperm, uint32_t n)
{
    std::vector<uint32_t> perm(n);
    CK(hipMemcpy(perm.data(), dperm, n * 4, hipMemcpyDeviceToHost));
    std::vector<char> seen(n, 0);
    uint32_t prev = 0;
    for (uint32_t q = 0; q < n; q++) {
        uint32_t s = perm[q];
        if (s >= n || seen[s]) return false;
        seen[s] = 1;
        if (keys[s] < prev) return false;
        prev = keys[s];
    }
    return true;
}

int main(int argc, char** argv)
{
    if (argc < 2) { fprintf(stderr, "usage: gsort_bench keys.bin\n"); return 2; }
    FILE* f = fopen(argv[1], "rb");
    if (!f) { perror("keys"); return 2; }
    std::vector<uint16_t> all;
    uint16_t buf[65536];
    size_t got;
    while ((got = fread(buf, 2, 65536, f)) > 0) all.insert(all.end(), buf, buf + got);
    fclose(f);
    const uint32_t rounds = 3, n = (uint32_t)(all.size() / rounds);
    printf("n=%u rounds=%u\n", n, rounds);
    uint16_t *key, *rank;
    uint32_t *hist, *cursor, *nvalid, *gpos, *perm, *chunkoff, *dummy;
    const uint32_t maxchunks = (n + 8191) / 8192;
    CK(hipMalloc(&key, (size_t)n * 2));
    CK(hipMalloc(&rank, (size_t)n * 2));
    CK(hipMalloc(&hist, BINS * 4));
    CK(hipMalloc(&cursor, BINS * 4));
    CK(hipMalloc(&nvalid, 4));
    CK(hipMalloc(&gpos, (size_t)n * 4));
    CK(hipMalloc(&perm, (size_t)n * 4));
    CK(hipMalloc(&chunkoff, (size_t)maxchunks * BINS * 4));
    CK(hipMalloc(&dummy, (size_t)maxchunks * BINS * 4));
    CK(hipMemset(hist, 0, BINS * 4));
    hipEvent_t ev[8];
    for (auto& e : ev) CK(hipEventCreate(&e));
    const int reps = 20;
    for (uint32_t r = 0; r < rounds; r++) {
        std::vector<uint16_t> keys(all.begin() + (size_t)r * n, all.begin() + (size_t)(r + 1) * n);
        CK(hipMemcpy(key, keys.data(), (size_t)n * 2, hipMemcpyHostToDevice));
        const uint32_t c8 = (n + 8191) / 8192, c16 = (n + 16383) / 16384, b256 = (n + 255) / 256;
        float t[6] = {0, 0, 0, 0, 0, 0};
        bool ok_base = true, ok_t8 = true, ok_t16 = true;
        for (int it = 0; it < reps + 2; it++) {
            float m;
            // base
            CK(hipEventRecord(ev[0]));
            hipLaunchKernelGGL(count_base<8192>, dim3(c8), dim3(TH), 0, 0, key, n, hist);
            CK(hipEventRecord(ev[1]));
            hipLaunchKernelGGL(scan, dim3(1), dim3(TH), 0, 0, hist, cursor, nvalid);
            CK(hipEventRecord(ev[2]));
            hipLaunchKernelGGL(scatter_base<8192>, dim3(c8), dim3(TH), 0, 0, key, n, cursor, gpos, perm);
            CK(hipEventRecord(ev[3]));
            // noatom
            hipLaunchKernelGGL(count_noatom<8192>, dim3(c8), dim3(TH), 0, 0, key, n, dummy);
            CK(hipEventRecord(ev[4]));
            CK(hipEventSynchronize(ev[4]));
            if (it == 0) ok_base = check(keys, perm, n);
            if (it >= 2) {
                CK(hipEventElapsedTime(&m, ev[0], ev[1])); t[0] += m;
                CK(hipEventElapsedTime(&m, ev[1], ev[2])); t[1] += m;
                CK(hipEventElapsedTime(&m, ev[2], ev[3])); t[2] += m;
                CK(hipEventElapsedTime(&m, ev[3], ev[4])); t[3] += m;
            }
        }
        printf("round %u base: count %.2f scan %.2f scatter %.2f us | noatom count %.2f us | valid %d\n", r,
               t[0] / reps * 1e3, t[1] / reps * 1e3, t[2] / reps * 1e3, t[3] / reps * 1e3, (int)ok_base);
        for (int v = 0; v < 2; v++) {
            float tc = 0, ts = 0, tx = 0;
            for (int it = 0; it < reps + 2; it++) {
                float m;
                CK(hipEventRecord(ev[0]));
                if (v == 0) hipLaunchKernelGGL(count_ticket<8192>, dim3(c8), dim3(TH), 0, 0, key, n, hist, chunkoff, rank);
                else hipLaunchKernelGGL(count_ticket<16384>, dim3(c16), dim3(TH), 0, 0, key, n, hist, chunkoff, rank);
                CK(hipEventRecord(ev[1]));
                hipLaunchKernelGGL(scan, dim3(1), dim3(TH), 0, 0, hist, cursor, nvalid);
                CK(hipEventRecord(ev[2]));
                if (v == 0) hipLaunchKernelGGL(scatter_ticket<8192>, dim3(b256), dim3(256), 0, 0, key, n, cursor, chunkoff, rank, gpos, perm);
                else hipLaunchKernelGGL(scatter_ticket<16384>, dim3(b256), dim3(256), 0, 0, key, n, cursor, chunkoff, rank, gpos, perm);
                CK(hipEventRecord(ev[3]));
                CK(hipEventSynchronize(ev[3]));
                if (it == 0) (v == 0 ? ok_t8 : ok_t16) = check(keys, perm, n);
                if (it >= 2) {
                    CK(hipEventElapsedTime(&m, ev[0], ev[1])); tc += m;
                    CK(hipEventElapsedTime(&m, ev[1], ev[2])); ts += m;
                    CK(hipEventElapsedTime(&m, ev[2], ev[3])); tx += m;
                }
            }
            printf("round %u ticket%s: count %.2f scan %.2f scatter %.2f us | valid %d\n", r, v ? "16" : "8",
                   tc / reps * 1e3, ts / reps * 1e3, tx / reps * 1e3, (int)(v ? ok_t16 : ok_t8));
        }
        const uint32_t c2 = (n + 2047) / 2048, c4 = (n + 4095) / 4096;
        run_variant("nt256_chunk2048", keys,
                    [&] { hipLaunchKernelGGL((count_nt<2048, 256>), dim3(c2), dim3(256), 0, 0, key, n, hist); },
                    [&] { hipLaunchKernelGGL((scatter_nt<2048, 256>), dim3(c2), dim3(256), 0, 0, key, n, cursor, perm); },
                    hist, cursor, nvalid, perm, ev, reps);
        run_variant("nt512_chunk4096", keys,
                    [&] { hipLaunchKernelGGL((count_nt<4096, 512>), dim3(c4), dim3(512), 0, 0, key, n, hist); },
                    [&] { hipLaunchKernelGGL((scatter_nt<4096, 512>), dim3(c4), dim3(512), 0, 0, key, n, cursor, perm); },
                    hist, cursor, nvalid, perm, ev, reps);
        run_variant("nt256_chunk4096", keys,
                    [&] { hipLaunchKernelGGL((count_nt<4096, 256>), dim3(c4), dim3(256), 0, 0, key, n, hist); },
                    [&] { hipLaunchKernelGGL((scatter_nt<4096, 256>), dim3(c4), dim3(256), 0, 0, key, n, cursor, perm); },
                    hist, cursor, nvalid, perm, ev, reps);
        run_variant("nt1024_chunk8192", keys,
                    [&] { hipLaunchKernelGGL((count_nt<8192, 1024>), dim3(c8), dim3(1024), 0, 0, key, n, hist); },
                    [&] { hipLaunchKernelGGL((scatter_nt<8192, 1024>), dim3(c8), dim3(1024), 0, 0, key, n, cursor, perm); },
                    hist, cursor, nvalid, perm, ev, reps);
        run_variant("copies4_chunk8192", keys,
                    [&] { hipLaunchKernelGGL((count_copies<8192>), dim3(c8), dim3(TH), 0, 0, key, n, hist); },
                    [&] { hipLaunchKernelGGL((scatter_nt<8192, 1024>), dim3(c8), dim3(1024), 0, 0, key, n, cursor, perm); },
                    hist, cursor, nvalid, perm, ev, reps);
        run_variant("vec8_chunk8192", keys,
                    [&] { hipLaunchKernelGGL((count_vec<8192>), dim3(c8), dim3(TH), 0, 0, key, n, hist); },
                    [&] { hipLaunchKernelGGL((scatter_nt<8192, 1024>), dim3(c8), dim3(1024), 0, 0, key, n, cursor, perm); },
                    hist, cursor, nvalid, perm, ev, reps);
        // Empty kernels: the launch + event overhead floor.
        run_variant("empty", keys, [&] { hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, 0); },
                    [&] { hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, 0); }, hist, cursor, nvalid, perm, ev, reps);
    }
    printf("done\n");
    return 0;
}
