// chase_probe.hip -- dependent-fetch ceiling for the traversal's access pattern (diagnostics).
//
// Every lane (or lane group) follows a chain of 64-B records: the next record's index is read
// from the record just fetched, exactly like a BVH step (one dependent round trip per step).
// Records are uniformly random over an array of N records, so the array size decides where
// they are served from (L2 4 MiB per XCD, Infinity Cache 256 MiB, HBM beyond).
//
// modes (argv[1]):
//   lane4  one chain per lane, the record as four 16-B loads (the traversal's fetch)
//   lane1  one chain per lane, one 16-B load per step (a 16-B record)
//   quad   one chain per 4 lanes, each lane loads one 16-B quarter (one load instruction per
//          step covers 16 records), the next index comes from the quad's lane 3
//   dual4  two chains per lane, both records' loads issued before either is waited for
//   lane3 / lane3d / lane2  48 B as 3 loads / 3 loads + a 4-B link / 32 B as 2 loads
//   act2 / act4  lane4 with every 2nd / 4th lane following a chain (steps/s counts active chains)
//   coop4  one chain per lane; the 4 lanes {c, c+16, c+32, c+48} fetch each other's records
//          cooperatively (load k: every lane of the group reads quarter `row` of the record of
//          the group's row-k chain, so one load instruction touches 16 records, not 64), then a
//          4x4 transpose (v_permlane32_swap + v_permlane16_swap) hands every lane its own record
// usage: chase_probe MODE RECORDS STEPS [WAVES_PER_CU=32] [REPS=3]
// prints one JSON line: dependent steps per second over all chains, and per chain.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(2);                                                               \
        }                                                                          \
    } while (0)

__global__ void k_init(int4* rec, unsigned n, unsigned seed) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    const unsigned nxt = h % n;
    for (int q = 0; q < 4; ++q) rec[4 * i + q] = make_int4((int)nxt, (int)(nxt ^ 1), (int)(nxt ^ 2), (int)nxt);
}

__device__ __forceinline__ unsigned start_of(unsigned chain, unsigned n) {
    unsigned h = chain * 0x9E3779B9u + 12345u;
    h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13;
    return h % n;
}

__global__ __launch_bounds__(64) void k_lane4(const int4* __restrict__ rec, unsigned n, int steps, unsigned* sink) {
    const unsigned chain = blockIdx.x * 64 + threadIdx.x;
    unsigned idx = start_of(chain, n);
    unsigned acc = 0;
    for (int s = 0; s < steps; ++s) {
        const int4 a = rec[4 * (size_t)idx + 0], b = rec[4 * (size_t)idx + 1];
        const int4 c = rec[4 * (size_t)idx + 2], d = rec[4 * (size_t)idx + 3];
        asm volatile("" ::"v"(a.y), "v"(b.y), "v"(c.y));
        acc += (unsigned)(a.z ^ b.z ^ c.z);
        idx = (unsigned)d.w;
    }
    if (acc == 0xdeadbeefu) sink[0] = idx;
}

__global__ __launch_bounds__(64) void k_lane1(const int4* __restrict__ rec, unsigned n, int steps, unsigned* sink) {
    const unsigned chain = blockIdx.x * 64 + threadIdx.x;
    unsigned idx = start_of(chain, n);
    for (int s = 0; s < steps; ++s) idx = (unsigned)rec[4 * (size_t)idx + 3].w;
    if (idx == 0xdeadbeefu) sink[0] = idx;
}

__global__ __launch_bounds__(64) void k_quad(const int4* __restrict__ rec, unsigned n, int steps, unsigned* sink) {
    const unsigned lane = threadIdx.x, q = lane & 3;
    const unsigned chain = blockIdx.x * 16 + (lane >> 2);
    unsigned idx = start_of(chain, n);
    unsigned acc = 0;
    for (int s = 0; s < steps; ++s) {
        const int4 v = rec[4 * (size_t)idx + q];
        acc += (unsigned)v.z;
        // the quad's lane 3 holds the link (DPP quad permute: broadcast lane 3 of each quad)
        idx = (unsigned)__builtin_amdgcn_mov_dpp(v.w, 0xFF, 0xF, 0xF, false);
    }
    if (acc == 0xdeadbeefu) sink[0] = idx;
}

__global__ __launch_bounds__(64) void k_dual4(const int4* __restrict__ rec, unsigned n, int steps, unsigned* sink) {
    const unsigned chain = (blockIdx.x * 64 + threadIdx.x) * 2;
    unsigned i0 = start_of(chain, n), i1 = start_of(chain + 1, n);
    unsigned acc = 0;
    for (int s = 0; s < steps; ++s) {
        const int4 a0 = rec[4 * (size_t)i0 + 0], b0 = rec[4 * (size_t)i0 + 1];
        const int4 c0 = rec[4 * (size_t)i0 + 2], d0 = rec[4 * (size_t)i0 + 3];
        const int4 a1 = rec[4 * (size_t)i1 + 0], b1 = rec[4 * (size_t)i1 + 1];
        const int4 c1 = rec[4 * (size_t)i1 + 2], d1 = rec[4 * (size_t)i1 + 3];
        asm volatile("" ::"v"(a0.y), "v"(b0.y), "v"(c0.y), "v"(a1.y), "v"(b1.y), "v"(c1.y));
        acc += (unsigned)(a0.z ^ b0.z ^ c0.z ^ a1.z ^ b1.z ^ c1.z);
        i0 = (unsigned)d0.w;
        i1 = (unsigned)d1.w;
    }
    if (acc == 0xdeadbeefu) sink[0] = i0 ^ i1;
}

// lane3: the record as three 16-B loads (link in the third); lane3d: three 16-B loads plus one
// 4-B load of the link word at offset 48; lane2: two 16-B loads (link in the second).
__global__ __launch_bounds__(64) void k_lane3(const int4* __restrict__ rec, unsigned n, int steps, unsigned* sink) {
    const unsigned chain = blockIdx.x * 64 + threadIdx.x;
    unsigned idx = start_of(chain, n);
    unsigned acc = 0;
    for (int s = 0; s < steps; ++s) {
        const int4 a = rec[4 * (size_t)idx + 0], b = rec[4 * (size_t)idx + 1], c = rec[4 * (size_t)idx + 2];
        asm volatile("" ::"v"(a.y), "v"(b.y), "v"(c.y));
        acc += (unsigned)(a.z ^ b.z ^ c.x);
        idx = (unsigned)c.w;
    }
    if (acc == 0xdeadbeefu) sink[0] = idx;
}
__global__ __launch_bounds__(64) void k_lane3d(const int4* __restrict__ rec, unsigned n, int steps, unsigned* sink) {
    const unsigned chain = blockIdx.x * 64 + threadIdx.x;
    unsigned idx = start_of(chain, n);
    unsigned acc = 0;
    for (int s = 0; s < steps; ++s) {
        const int4 a = rec[4 * (size_t)idx + 0], b = rec[4 * (size_t)idx + 1], c = rec[4 * (size_t)idx + 2];
        const int d = reinterpret_cast<const int*>(rec + 4 * (size_t)idx + 3)[0];
        asm volatile("" ::"v"(a.y), "v"(b.y), "v"(c.y), "v"(c.w));
        acc += (unsigned)(a.z ^ b.z ^ c.x);
        idx = (unsigned)d;
    }
    if (acc == 0xdeadbeefu) sink[0] = idx;
}
__global__ __launch_bounds__(64) void k_lane3q(const int4* __restrict__ rec, unsigned n, int steps, unsigned* sink) {
    const unsigned chain = blockIdx.x * 64 + threadIdx.x;
    unsigned idx = start_of(chain, n);
    unsigned acc = 0;
    for (int s = 0; s < steps; ++s) {
        const int4 a = rec[4 * (size_t)idx + 0], b = rec[4 * (size_t)idx + 1], c = rec[4 * (size_t)idx + 2];
        const int2 d = reinterpret_cast<const int2*>(rec + 4 * (size_t)idx + 3)[0];
        asm volatile("" ::"v"(a.y), "v"(b.y), "v"(c.y), "v"(c.w), "v"(d.y));
        acc += (unsigned)(a.z ^ b.z ^ c.x);
        idx = (unsigned)d.x;
    }
    if (acc == 0xdeadbeefu) sink[0] = idx;
}
__global__ __launch_bounds__(64) void k_lane2(const int4* __restrict__ rec, unsigned n, int steps, unsigned* sink) {
    const unsigned chain = blockIdx.x * 64 + threadIdx.x;
    unsigned idx = start_of(chain, n);
    unsigned acc = 0;
    for (int s = 0; s < steps; ++s) {
        const int4 a = rec[4 * (size_t)idx + 0], b = rec[4 * (size_t)idx + 1];
        asm volatile("" ::"v"(a.y), "v"(b.y));
        acc += (unsigned)(a.z ^ b.x);
        idx = (unsigned)b.w;
    }
    if (acc == 0xdeadbeefu) sink[0] = idx;
}
// lane4 with only every ACT-th lane of a wave following a chain (the others idle in the loop,
// exec-masked): does a gather cost by the lanes it serves or by the instruction?
template <int ACT>
__global__ __launch_bounds__(64) void k_lane4_act(const int4* __restrict__ rec, unsigned n, int steps, unsigned* sink) {
    const unsigned chain = blockIdx.x * 64 + threadIdx.x;
    unsigned idx = start_of(chain, n);
    unsigned acc = 0;
    const bool on = (threadIdx.x % ACT) == 0;
    for (int s = 0; s < steps; ++s) {
        if (on) {
            const int4 a = rec[4 * (size_t)idx + 0], b = rec[4 * (size_t)idx + 1];
            const int4 c = rec[4 * (size_t)idx + 2], d = rec[4 * (size_t)idx + 3];
            asm volatile("" ::"v"(a.y), "v"(b.y), "v"(c.y));
            acc += (unsigned)(a.z ^ b.z ^ c.z);
            idx = (unsigned)d.w;
        }
        __builtin_amdgcn_s_barrier();   // keep the idle lanes' wave in the loop (one wave per block)
    }
    if (acc == 0xdeadbeefu) sink[0] = idx;
}

// 4x4 transpose across the lane group {c, c+16, c+32, c+48}: element (row r, register k) <->
// (row k, register r).  permlane32_swap(vdst, src0) swaps lanes 32-63 of vdst with lanes 0-31 of
// src0; permlane16_swap swaps the odd 16-lane rows of vdst with the even rows of src0.
__device__ __forceinline__ void transpose4(unsigned& a0, unsigned& a1, unsigned& a2, unsigned& a3) {
    auto p = __builtin_amdgcn_permlane32_swap(a0, a2, false, false);
    a0 = p[0]; a2 = p[1];
    p = __builtin_amdgcn_permlane32_swap(a1, a3, false, false);
    a1 = p[0]; a3 = p[1];
    p = __builtin_amdgcn_permlane16_swap(a0, a1, false, false);
    a0 = p[0]; a1 = p[1];
    p = __builtin_amdgcn_permlane16_swap(a2, a3, false, false);
    a2 = p[0]; a3 = p[1];
}
__device__ __forceinline__ void transpose4(int4& a0, int4& a1, int4& a2, int4& a3) {
#define T4(f) { unsigned x0 = a0.f, x1 = a1.f, x2 = a2.f, x3 = a3.f; transpose4(x0, x1, x2, x3); \
                a0.f = (int)x0; a1.f = (int)x1; a2.f = (int)x2; a3.f = (int)x3; }
    T4(x) T4(y) T4(z) T4(w)
#undef T4
}

__global__ void k_ttest(unsigned* out) {
    const unsigned l = threadIdx.x;
    unsigned a0 = l * 4 + 0, a1 = l * 4 + 1, a2 = l * 4 + 2, a3 = l * 4 + 3;
    transpose4(a0, a1, a2, a3);
    out[4 * l + 0] = a0; out[4 * l + 1] = a1; out[4 * l + 2] = a2; out[4 * l + 3] = a3;
}

__global__ __launch_bounds__(64) void k_coop4(const int4* __restrict__ rec, unsigned n, int steps, unsigned* sink) {
    const unsigned lane = threadIdx.x, row = lane >> 4;
    const unsigned chain = blockIdx.x * 64 + lane;
    unsigned idx = start_of(chain, n);
    unsigned acc = 0;
    for (int s = 0; s < steps; ++s) {
        unsigned n0 = idx, n1 = idx, n2 = idx, n3 = idx;
        transpose4(n0, n1, n2, n3);   // n_k = the index of this group's row-k chain
        int4 v0 = rec[4 * (size_t)n0 + row], v1 = rec[4 * (size_t)n1 + row];
        int4 v2 = rec[4 * (size_t)n2 + row], v3 = rec[4 * (size_t)n3 + row];
        transpose4(v0, v1, v2, v3);   // v_k = quarter k of this lane's own record
        asm volatile("" ::"v"(v0.y), "v"(v1.y), "v"(v2.y));
        acc += (unsigned)(v0.z ^ v1.z ^ v2.z);
        idx = (unsigned)v3.w;
    }
    if (acc == 0xdeadbeefu) sink[0] = idx;
}

int main(int argc, char** argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s lane4|lane1|quad|dual4 RECORDS STEPS [WAVES_PER_CU] [REPS]\n", argv[0]);
        return 1;
    }
    const char* mode = argv[1];
    const unsigned n = (unsigned)strtoul(argv[2], nullptr, 10);
    const int steps = atoi(argv[3]);
    const int wpc = argc > 4 ? atoi(argv[4]) : 32;
    const int reps = argc > 5 ? atoi(argv[5]) : 3;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    int4* rec = nullptr;
    unsigned* sink = nullptr;
    CK(hipMalloc(&rec, (size_t)n * 64));
    CK(hipMalloc(&sink, 4));
    k_init<<<(n + 255) / 256, 256>>>(rec, n, 777u);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    const unsigned waves = (unsigned)(cus * wpc);
    int chainsPerWave = 64;
    void (*kern)(const int4*, unsigned, int, unsigned*) = k_lane4;
    if (!strcmp(mode, "lane1")) kern = k_lane1;
    else if (!strcmp(mode, "quad")) { kern = k_quad; chainsPerWave = 16; }
    else if (!strcmp(mode, "dual4")) { kern = k_dual4; chainsPerWave = 128; }
    else if (!strcmp(mode, "coop4")) kern = k_coop4;
    else if (!strcmp(mode, "lane3")) kern = k_lane3;
    else if (!strcmp(mode, "lane3d")) kern = k_lane3d;
    else if (!strcmp(mode, "lane2")) kern = k_lane2;
    else if (!strcmp(mode, "lane3q")) kern = k_lane3q;
    else if (!strcmp(mode, "act2")) { kern = k_lane4_act<2>; chainsPerWave = 32; }
    else if (!strcmp(mode, "act4")) { kern = k_lane4_act<4>; chainsPerWave = 16; }
    else if (!strcmp(mode, "ttest")) {
        unsigned* d;
        CK(hipMalloc(&d, 256 * 4));
        k_ttest<<<1, 64>>>(d);
        std::vector<unsigned> h(256);
        CK(hipMemcpy(h.data(), d, 1024, hipMemcpyDeviceToHost));
        int bad = 0;
        for (unsigned l = 0; l < 64; ++l)
            for (unsigned k = 0; k < 4; ++k) {
                const unsigned r = l >> 4, c = l & 15, src = c + 16 * k;   // (row k, register r)
                if (h[4 * l + k] != src * 4 + r) ++bad;
            }
        printf("{\"mode\": \"ttest\", \"bad\": %d}\n", bad);
        return bad ? 3 : 0;
    }
    else if (strcmp(mode, "lane4")) { fprintf(stderr, "bad mode\n"); return 1; }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    kern<<<waves, 64>>>(rec, n, steps / 4 > 0 ? steps / 4 : 1, sink);   // warm (TLB, caches)
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0));
        kern<<<waves, 64>>>(rec, n, steps, sink);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
    }
    const double chains = (double)waves * chainsPerWave;
    const double stepsTotal = chains * steps;
    printf("{\"mode\": \"%s\", \"records\": %u, \"array_mb\": %.1f, \"steps\": %d, \"waves_per_cu\": %d, "
           "\"chains\": %.0f, \"ms\": %.4f, \"gsteps_per_s\": %.2f, \"ns_per_step_per_chain\": %.1f}\n",
           mode, n, n * 64.0 / 1048576.0, steps, wpc, chains, best, stepsTotal / (best * 1e-3) / 1e9,
           best * 1e6 / steps);
    CK(hipFree(rec));
    CK(hipFree(sink));
    return 0;
}
