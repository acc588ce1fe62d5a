// k1_shape_probe.hip — where does K1's fixed cost at shard size come from?
// Standalone measurement tool (not part of the product).  Streams ≈300 MB (one rank's
// config-4 shard at N = 8) in K1's tile shapes and reports median µs per launch over 4
// rotating buffer sets (so the 256 MB MALL cannot serve them):
//   soa    : K1's layout — 4 SoA arrays (flags u32, cpu u32, mem u64, pair u32); a tile is
//            256 pods = 5 16-B loads per lane from 4 arrays; tiles interleaved over the
//            workgroup's waves (tile a + w, a + w + 8, ...), DS tiles in flight per wave
//   soaws  : the same arrays, every wave its own contiguous tile range
//   tile   : tile-major (AoSoA) — a tile's 5 KB contiguous, same interleave as soa
//   flat   : one contiguous stream per workgroup (the shard_probe floor)
// Each with or without 160 KB of dynamic LDS (K1's occupancy: one workgroup per CU).
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/k1_shape_probe scripts/k1_shape_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
constexpr int TILE = 256;              // pods per tile
constexpr int NW = 8;                  // waves per workgroup

__device__ __forceinline__ v4u ld(const v4u* p) { return __builtin_nontemporal_load(p); }

struct Arr {
    const uint32_t* flags;
    const uint32_t* cpu;
    const uint64_t* mem;
    const uint32_t* pair;
    const uint8_t* tiles;              // tile-major copy: 5 KB per tile
    int64_t n_tiles;
};

struct T5 { v4u a, b, c, d, e; };

// MODE 0 soa interleaved, 1 soa per-wave contiguous, 2 tile-major interleaved
template <int MODE>
__device__ __forceinline__ void load_tile(const Arr& A, int64_t t, uint32_t lane, T5& r) {
    if constexpr (MODE == 2) {
        const v4u* b = reinterpret_cast<const v4u*>(A.tiles + t * 5120) + lane;
        r.a = ld(b); r.b = ld(b + 64); r.c = ld(b + 128); r.d = ld(b + 192); r.e = ld(b + 256);
    } else {
        const int64_t p = t * TILE + lane * 4;
        r.a = ld(reinterpret_cast<const v4u*>(A.flags + p));
        r.b = ld(reinterpret_cast<const v4u*>(A.cpu + p));
        r.c = ld(reinterpret_cast<const v4u*>(A.mem + t * TILE + lane * 2));
        r.d = ld(reinterpret_cast<const v4u*>(A.mem + t * TILE + 128 + lane * 2));
        r.e = ld(reinterpret_cast<const v4u*>(A.pair + p));
    }
}

template <int MODE, int DS>
__global__ __launch_bounds__(512) void k_tiles(Arr A, uint32_t* out) {
    extern __shared__ uint32_t lds[];
    const uint32_t lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    int64_t a, b, st;
    if constexpr (MODE == 1) {
        const int64_t nwv = (int64_t)gridDim.x * NW, w = (int64_t)blockIdx.x * NW + wid;
        a = A.n_tiles * w / nwv; b = A.n_tiles * (w + 1) / nwv; st = 1;
    } else {
        a = A.n_tiles * blockIdx.x / gridDim.x + wid; b = A.n_tiles * (blockIdx.x + 1) / gridDim.x; st = NW;
    }
    uint32_t acc = 0;
    if (a < b) {
        T5 T[DS];
#pragma unroll
        for (int d = 0; d < DS; ++d) {
            const int64_t u = a + d * st;
            load_tile<MODE>(A, u < b ? u : a, lane, T[d]);
            __builtin_amdgcn_sched_barrier(0);
        }
        for (int64_t t = a; t < b; t += DS * st) {
#pragma unroll
            for (int d = 0; d < DS; ++d) {
                const int64_t u = t + d * st;
                if (u < b) {
                    const v4u x = T[d].a ^ T[d].b ^ T[d].c ^ T[d].d ^ T[d].e;
                    acc ^= x.x ^ x.y ^ x.z ^ x.w;
                }
                __builtin_amdgcn_sched_barrier(0);
                const int64_t nu = u + DS * st;
                load_tile<MODE>(A, nu < b ? nu : (u < b ? u : a), lane, T[d]);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    }
    if (acc == 0x12345678u) { lds[threadIdx.x] = acc; out[0] = lds[(threadIdx.x + 1) & 511]; }
}

template <int U>
__global__ __launch_bounds__(512) void k_flat(const uint8_t* base, int64_t bytes, uint32_t* out) {
    extern __shared__ uint32_t lds[];
    const v4u* p = reinterpret_cast<const v4u*>(base);
    const int64_t n16 = bytes / 16;
    const int64_t per = (n16 + gridDim.x - 1) / gridDim.x;
    const int64_t lo = (int64_t)blockIdx.x * per;
    const int64_t hi = lo + per < n16 ? lo + per : n16;
    uint32_t acc = 0;
    for (int64_t b = lo + threadIdx.x; b < hi; b += 512 * U) {
        v4u v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = b + (int64_t)u * 512;
            v[u] = ld(p + (i < hi ? i : lo));
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (acc == 0x12345678u) { lds[threadIdx.x] = acc; out[0] = lds[(threadIdx.x + 1) & 511]; }
}

int main(int argc, char** argv) {
    const int64_t pods = (argc > 1 ? atoll(argv[1]) : 12500000) / TILE * TILE;
    const int64_t n_tiles = pods / TILE;
    const int R = 4;
    std::vector<Arr> sets(R);
    std::vector<uint8_t*> flatb(R);
    const int64_t soa_bytes = pods * 20;
    for (int r = 0; r < R; ++r) {
        uint8_t* b;
        CK(hipMalloc(&b, soa_bytes));
        CK(hipMemset(b, r + 1, soa_bytes));
        Arr& A = sets[r];
        A.flags = (const uint32_t*)b;
        A.cpu = (const uint32_t*)(b + pods * 4);
        A.mem = (const uint64_t*)(b + pods * 8);
        A.pair = (const uint32_t*)(b + pods * 16);
        uint8_t* t;
        CK(hipMalloc(&t, n_tiles * 5120));
        CK(hipMemset(t, r + 1, n_tiles * 5120));
        A.tiles = t;
        A.n_tiles = n_tiles;
        flatb[r] = b;
    }
    uint32_t* out;
    CK(hipMalloc(&out, 4));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    printf("{\"pods\": %lld, \"bytes\": %lld, \"cus\": %d, \"us\": {", (long long)pods, (long long)soa_bytes, cus);
    bool first = true;
    auto run = [&](const char* name, auto launch) {
        for (int r = 0; r < R; ++r) launch(r);
        CK(hipDeviceSynchronize());
        std::vector<float> ts;
        for (int rep = 0; rep < 40; ++rep) {
            CK(hipEventRecord(e0));
            launch(rep % R);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        printf("%s\"%s\": %.1f", first ? "" : ", ", name, ts[ts.size() / 2] * 1e3);
        first = false;
        fflush(stdout);
    };
    const size_t big = 160 << 10;
    CK(hipFuncSetAttribute((const void*)k_tiles<0, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, big));
    CK(hipFuncSetAttribute((const void*)k_tiles<0, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, big));
    CK(hipFuncSetAttribute((const void*)k_tiles<1, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, big));
    CK(hipFuncSetAttribute((const void*)k_tiles<2, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, big));
    CK(hipFuncSetAttribute((const void*)k_flat<4>, hipFuncAttributeMaxDynamicSharedMemorySize, big));
#define KT(MODE, DS, LDS, NAME)                                                                  \
    run(NAME, [&](int r) {                                                                       \
        hipLaunchKernelGGL((k_tiles<MODE, DS>), dim3(cus), dim3(512), LDS, 0, sets[r], out);     \
    })
    KT(0, 4, 0, "soa_ds4");
    KT(0, 4, big, "soa_ds4_lds160k");
    KT(0, 2, big, "soa_ds2_lds160k");
    KT(1, 4, big, "soaws_ds4_lds160k");
    KT(2, 4, 0, "tile_ds4");
    KT(2, 4, big, "tile_ds4_lds160k");
    run("flat_u4", [&](int r) { hipLaunchKernelGGL((k_flat<4>), dim3(cus), dim3(512), 0, 0, flatb[r], soa_bytes, out); });
    run("flat_u4_lds160k", [&](int r) { hipLaunchKernelGGL((k_flat<4>), dim3(cus), dim3(512), big, 0, flatb[r], soa_bytes, out); });
    printf("}}\n");
    return 0;
}
