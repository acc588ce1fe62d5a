// size_probe.hip — streaming-read time against size on this MI355X: what a K1-shaped
// kernel (one 512-thread workgroup per CU, 16-B nontemporal loads, contiguous share per
// workgroup) can reach for one rank's shard (~300 MB at N = 8) vs the whole snapshot.
// Standalone measurement tool (not part of the product).  Rotates over buffers totalling
// >= 2.4 GB so that every launch reads from HBM, not from the 256 MB Infinity Cache.
//   hipcc --offload-arch=gfx950 -O3 -o size_probe scripts/size_probe.hip
// Prints one JSON object: per size the median kernel time (HIP events) and GB/s, for
//   read   : loads only (U = 4 tiles in flight per lane),
//   flush  : loads + a 160 KB per-workgroup store at the end (K1's partial flush),
//   empty  : a launch that reads nothing (launch + drain floor).
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

template <int U, bool FLUSH>
__global__ __launch_bounds__(512) void k_read(const uint4* __restrict__ p, int64_t n16, uint4* __restrict__ part,
                                              uint32_t* out) {
    const int64_t per = (n16 + gridDim.x - 1) / gridDim.x;
    const int64_t lo = (int64_t)blockIdx.x * per;
    const int64_t hi = lo + per < n16 ? lo + per : n16;
    uint32_t acc = 0;
    for (int64_t b = lo + threadIdx.x; b < hi; b += (int64_t)512 * U) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = b + (int64_t)u * 512;
            const int64_t j = i < hi ? i : lo;
            const v4u t = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p + j));
            v[u] = make_uint4(t.x, t.y, t.z, t.w);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if constexpr (FLUSH) {
        // 160 KB per workgroup = 10240 x 16 B, as K1's per-workgroup slot partials
        uint4* o = part + (int64_t)blockIdx.x * 10240;
        for (int i = threadIdx.x; i < 10240; i += 512) o[i] = make_uint4(acc, i, 0, 0);
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_empty(uint32_t* out) {
    if (threadIdx.x == 1234567) out[0] = 1;
}

int main() {
    const int64_t total = 2400ll << 20;
    uint4* base;
    uint4* part;
    uint32_t* out;
    CK(hipMalloc(&base, total));
    CK(hipMalloc(&part, 1024ll * 10240 * 16));
    CK(hipMalloc(&out, 4));
    CK(hipMemset(base, 1, total));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto med = [&](auto&& launch) {
        std::vector<float> ts;
        for (int r = 0; r < 24; ++r) {
            CK(hipEventRecord(a));
            launch(r);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (r >= 4) ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        return ts[ts.size() / 2];
    };
    printf("{\"cus\": %d, \"empty_ms\": %.4f, \"sizes\": [", cus,
           med([&](int) { hipLaunchKernelGGL(k_empty, dim3(cus), dim3(512), 0, 0, out); }));
    bool first = true;
    for (int64_t mb : {32ll, 64ll, 124ll, 248ll, 500ll, 1000ll, 2400ll}) {
        const int64_t bytes = mb << 20, n16 = bytes / 16, nbuf = std::max<int64_t>(1, total / bytes);
        auto at = [&](int r) { return base + (r % nbuf) * n16; };
        const float r4 = med([&](int r) { hipLaunchKernelGGL((k_read<4, false>), dim3(cus), dim3(512), 0, 0, at(r), n16, part, out); });
        const float r8 = med([&](int r) { hipLaunchKernelGGL((k_read<8, false>), dim3(cus), dim3(512), 0, 0, at(r), n16, part, out); });
        const float f4 = med([&](int r) { hipLaunchKernelGGL((k_read<4, true>), dim3(cus), dim3(512), 0, 0, at(r), n16, part, out); });
        const float r4x2 = med([&](int r) { hipLaunchKernelGGL((k_read<4, false>), dim3(2 * cus), dim3(512), 0, 0, at(r), n16, part, out); });
        printf("%s{\"MB\": %lld, \"buffers\": %lld, \"read_u4_ms\": %.4f, \"read_u8_ms\": %.4f, \"flush_u4_ms\": %.4f, "
               "\"read_u4_2wg_ms\": %.4f, \"read_u4_GBps\": %.0f, \"read_u8_GBps\": %.0f}",
               first ? "" : ", ", (long long)mb, (long long)nbuf, r4, r8, f4, r4x2, bytes / (r4 * 1e-3) / 1e9,
               bytes / (r8 * 1e-3) / 1e9);
        first = false;
        fflush(stdout);
    }
    printf("]}\n");
    return 0;
}
