// stream_probe.hip — practical HBM read ceiling on this MI355X for the access shapes K1 uses.
// Standalone measurement tool (not part of the product): reads a 2.4 GB buffer with
// 16-B-per-lane loads in several launch shapes and prints GB/s per shape as JSON.
//   hipcc --offload-arch=gfx950 -O3 -o stream_probe scripts/stream_probe.hip
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

// Contiguous share per workgroup; waves interleave 1-KB wave tiles; U loads per lane in flight.
template <int THREADS, int U, bool NT>
__global__ __launch_bounds__(THREADS) void k_chunk(const uint4* __restrict__ p, int64_t n16, uint32_t* out) {
    const int64_t per = (n16 + gridDim.x - 1) / gridDim.x;
    const int64_t lo = (int64_t)blockIdx.x * per;
    const int64_t hi = lo + per < n16 ? lo + per : n16;
    uint32_t acc = 0;
    for (int64_t b = lo + threadIdx.x; b < hi; b += (int64_t)THREADS * U) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = b + (int64_t)u * THREADS;
            const int64_t j = i < hi ? i : lo;
            if constexpr (NT) {
                const v4u t = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p + j));
                v[u] = make_uint4(t.x, t.y, t.z, t.w);
            } else {
                v[u] = p[j];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// S parallel streams (struct-of-arrays fields): the buffer is S equal arrays and every
// workgroup reads the same relative share of each, U rounds of S loads in flight — the
// K1 K-tile shape (flags, cpu0, pair0, mem0 x2, records) against one contiguous stream.
template <int THREADS, int S, int U>
__global__ __launch_bounds__(THREADS) void k_multi(const uint4* __restrict__ p, int64_t n16, uint32_t* out) {
    const int64_t na = n16 / S;
    const int64_t per = (na + gridDim.x - 1) / gridDim.x;
    const int64_t lo = (int64_t)blockIdx.x * per;
    const int64_t hi = lo + per < na ? lo + per : na;
    uint32_t acc = 0;
    for (int64_t b = lo + threadIdx.x; b < hi; b += (int64_t)THREADS * U) {
        uint4 v[U][S];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = b + (int64_t)u * THREADS;
            const int64_t j = i < hi ? i : lo;
#pragma unroll
            for (int k = 0; k < S; ++k) {
                const v4u t = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p + (int64_t)k * na + j));
                v[u][k] = make_uint4(t.x, t.y, t.z, t.w);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int k = 0; k < S; ++k) acc ^= v[u][k].x ^ v[u][k].y ^ v[u][k].z ^ v[u][k].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// As k_multi, but stream k starts at k * (sp16 + ex16) (16-B units): power-of-two spacing
// between the SoA arrays (ex16 = 0) against skewed bases — do separately allocated
// arrays read at the same tile offset collide on HBM channels?
template <int THREADS, int S, int U>
__global__ __launch_bounds__(THREADS) void k_multi_sp(const uint4* __restrict__ p, int64_t na, int64_t sp16,
                                                      int64_t ex16, uint32_t* out) {
    const int64_t per = (na + gridDim.x - 1) / gridDim.x;
    const int64_t lo = (int64_t)blockIdx.x * per;
    const int64_t hi = lo + per < na ? lo + per : na;
    uint32_t acc = 0;
    for (int64_t b = lo + threadIdx.x; b < hi; b += (int64_t)THREADS * U) {
        uint4 v[U][S];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = b + (int64_t)u * THREADS;
            const int64_t j = i < hi ? i : lo;
#pragma unroll
            for (int k = 0; k < S; ++k) {
                const v4u t = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p + (int64_t)k * (sp16 + ex16) + j));
                v[u][k] = make_uint4(t.x, t.y, t.z, t.w);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int k = 0; k < S; ++k) acc ^= v[u][k].x ^ v[u][k].y ^ v[u][k].z ^ v[u][k].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// Grid-stride (every wave walks the whole buffer at a stride of the grid).
template <int THREADS, int U>
__global__ __launch_bounds__(THREADS) void k_stride(const uint4* __restrict__ p, int64_t n16, uint32_t* out) {
    const int64_t stride = (int64_t)gridDim.x * THREADS;
    uint32_t acc = 0;
    for (int64_t b = (int64_t)blockIdx.x * THREADS + threadIdx.x; b < n16; b += stride * U) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = b + (int64_t)u * stride;
            v[u] = p[i < n16 ? i : b];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <class F>
static float time_ms(F&& launch, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    launch();
    CK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(a));
        launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

int main() {
    const int64_t bytes = 2400ll << 20;
    const int64_t big = 3200ll << 20;                  // room for 5 streams 512 MB apart + skew
    const int64_t n16 = bytes / 16;
    uint4* p;
    uint32_t* out;
    CK(hipMalloc(&p, big));
    CK(hipMalloc(&out, 4));
    CK(hipMemset(p, 1, big));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    printf("{\"bytes\": %lld, \"cus\": %d, \"GBps\": {", (long long)bytes, cus);
    bool first = true;
    auto rep = [&](const char* name, float ms) {
        printf("%s\"%s\": %.0f", first ? "" : ", ", name, bytes / (ms * 1e-3) / 1e9);
        first = false;
        fflush(stdout);
    };
#define RUN_CHUNK(T, U, NT, WPC)                                                                         \
    rep("chunk_t" #T "_u" #U "_nt" #NT "_wgpercu" #WPC,                                                   \
        time_ms([&] { hipLaunchKernelGGL((k_chunk<T, U, NT>), dim3(cus * WPC), dim3(T), 0, 0, p, n16, out); }, 10))
    RUN_CHUNK(1024, 2, false, 1);
    RUN_CHUNK(1024, 4, false, 1);
    RUN_CHUNK(1024, 8, false, 1);
    RUN_CHUNK(1024, 4, true, 1);
    RUN_CHUNK(1024, 4, false, 2);
    RUN_CHUNK(512, 4, false, 2);
    RUN_CHUNK(512, 4, false, 4);
    RUN_CHUNK(256, 4, false, 8);
    RUN_CHUNK(256, 8, false, 8);
    RUN_CHUNK(256, 4, false, 16);
    RUN_CHUNK(256, 4, false, 64);
    RUN_CHUNK(512, 4, true, 1);
    RUN_CHUNK(512, 8, true, 1);
#define RUN_MULTI(T, S, U)                                                                                \
    rep("multi_t" #T "_s" #S "_u" #U,                                                                    \
        time_ms([&] { hipLaunchKernelGGL((k_multi<T, S, U>), dim3(cus), dim3(T), 0, 0, p, n16, out); }, 10))
    RUN_MULTI(512, 1, 4);
    RUN_MULTI(512, 5, 1);
    RUN_MULTI(512, 5, 2);
    RUN_MULTI(512, 5, 4);
    RUN_MULTI(512, 9, 2);
    RUN_MULTI(1024, 5, 2);
    {   // 5 streams of 448 MB (2240 MB read) at 512 MB spacing + skew
        const int64_t na = (448ll << 20) / 16, sp = (512ll << 20) / 16;
        const int64_t mb = 2240ll << 20;
        auto rep2 = [&](const char* name, float ms) {
            printf("%s\"%s\": %.0f", first ? "" : ", ", name, mb / (ms * 1e-3) / 1e9);
            first = false;
            fflush(stdout);
        };
        for (int64_t ex : {0ll, 256ll, 4096ll, 65536ll, (1ll << 20) + 4096}) {
            char name[64];
            snprintf(name, sizeof name, "multi_sp512M_skew%lld_t512_s5_u2", (long long)ex);
            rep2(name, time_ms([&] { hipLaunchKernelGGL((k_multi_sp<512, 5, 2>), dim3(cus), dim3(512), 0, 0, p, na, sp,
                                                         ex / 16, out); }, 10));
        }
        // K1-like: arrays of 100M x 4 B rounded up to 2 MB (191 x 2 MB apart)
        const int64_t sp191 = (191ll << 21) / 16, na191 = (382ll << 20) / 16;
        const int64_t mb191 = 5 * (382ll << 20);
        for (int64_t ex : {0ll, 4096ll}) {
            char name[64];
            snprintf(name, sizeof name, "multi_sp191x2M_skew%lld_t512_s5_u2", (long long)ex);
            const float ms = time_ms([&] { hipLaunchKernelGGL((k_multi_sp<512, 5, 2>), dim3(cus), dim3(512), 0, 0, p, na191,
                                                              sp191, ex / 16, out); }, 10);
            printf(", \"%s\": %.0f", name, mb191 / (ms * 1e-3) / 1e9);
        }
    }
#define RUN_STRIDE(T, U, WPC)                                                                             \
    rep("stride_t" #T "_u" #U "_wgpercu" #WPC,                                                           \
        time_ms([&] { hipLaunchKernelGGL((k_stride<T, U>), dim3(cus * WPC), dim3(T), 0, 0, p, n16, out); }, 10))
    RUN_STRIDE(1024, 4, 1);
    RUN_STRIDE(256, 4, 8);
    RUN_STRIDE(256, 8, 8);
    printf("}}\n");
    return 0;
}
