// shard_probe.hip — the read floor at one rank's shard size (≈300 MB: 12.5 M config-4 pods).
// Standalone measurement tool (not part of the product).  Reads R rotating buffers of B
// bytes (so the 256 MB MALL cannot serve them) in several launch shapes and reports the
// median time per launch, with and without a per-workgroup flush of W bytes at the end
// (K1's LDS-partials flush: 256 x 160 KB = 41 MB at 10 k groups).
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/shard_probe scripts/shard_probe.hip
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

// Contiguous share per workgroup, U 16-B nontemporal loads per lane in flight; optional
// flush of `wb` bytes per workgroup (uint4 stores) after the stream.
template <int THREADS, int U>
__global__ __launch_bounds__(THREADS) void k_read(const uint4* __restrict__ p, int64_t n16, uint4* __restrict__ flush,
                                                  int64_t wb16, uint32_t* out) {
    const int64_t per = (n16 + gridDim.x - 1) / gridDim.x;
    const int64_t lo = (int64_t)blockIdx.x * per;
    const int64_t hi = lo + per < n16 ? lo + per : n16;
    uint32_t acc = 0;
    for (int64_t b = lo + threadIdx.x; b < hi; b += (int64_t)THREADS * U) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = b + (int64_t)u * THREADS;
            const v4u t = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p + (i < hi ? i : lo)));
            v[u] = make_uint4(t.x, t.y, t.z, t.w);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (wb16) {
        uint4* f = flush + (int64_t)blockIdx.x * wb16;
        for (int64_t i = threadIdx.x; i < wb16; i += THREADS) f[i] = make_uint4(acc, acc, acc, i);
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char** argv) {
    const int64_t B = (argc > 1 ? atoll(argv[1]) : 300) << 20;
    const int R = 4;
    std::vector<uint4*> bufs(R);
    for (auto& b : bufs) {
        CK(hipMalloc(&b, B));
        CK(hipMemset(b, 1, B));
    }
    uint4* flush;
    uint32_t* out;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int64_t wb = 160 << 10;                         // per workgroup
    CK(hipMalloc(&flush, (int64_t)cus * 4 * wb));
    CK(hipMalloc(&out, 4));
    const int64_t n16 = B / 16;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    printf("{\"bytes\": %lld, \"cus\": %d, \"us\": {", (long long)B, cus);
    bool first = true;
    auto run = [&](const char* name, auto launch) {
        for (int r = 0; r < R; ++r) launch(bufs[r]);
        CK(hipDeviceSynchronize());
        std::vector<float> ts;
        for (int rep = 0; rep < 40; ++rep) {
            CK(hipEventRecord(a));
            launch(bufs[rep % R]);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        printf("%s\"%s\": %.1f", first ? "" : ", ", name, ts[ts.size() / 2] * 1e3);
        first = false;
        fflush(stdout);
    };
#define K(T, U, WPC, W)                                                                                   \
    run("t" #T "_u" #U "_wgpercu" #WPC "_flush" #W, [&](uint4* p) {                                      \
        hipLaunchKernelGGL((k_read<T, U>), dim3(cus * WPC), dim3(T), 0, 0, p, n16, flush, W ? wb / 16 : 0, out); \
    })
    K(512, 4, 1, 0);
    K(512, 8, 1, 0);
    K(512, 4, 1, 1);
    K(1024, 4, 1, 0);
    K(512, 4, 2, 0);
    K(256, 4, 4, 0);
    K(256, 8, 4, 0);
    K(256, 4, 8, 0);
    K(512, 4, 2, 1);
    printf("}}\n");
    return 0;
}
