// esc_list.hip — the per-call drop-ins of the Go signatures over a slice of objects:
//   CalculatePodsRequestsTotal(pods)   pkg/k8s/util.go:27-38 (+ ComputePodResourceRequest,
//                                      pkg/k8s/scheduler/types.go:72-89, per pod)
//   CalculateNodesCapacityTotal(nodes) pkg/k8s/util.go:41-51
//
// The batched decision (esc_run) works on a resident snapshot; these calls get a fresh
// slice every time (SURVEY.md §7 hard part 6), typically ~1000 objects.  A per-call snapshot
// (class layout, work plan, touch lists) costs ~1 ms, so this path keeps per-context
// reusable pinned buffers instead and does the least a call can:
//   host: one walk over the objects writes each one's container records (cpu, mem; an
//         absent init key as INT64_MIN, which the max skips) and a u32 shape word into
//         pinned host memory;
//   GPU:  one launch of k_list_sum reads them straight from pinned memory (zero-copy: the
//         whole slice is a few tens of KB, less than a DMA setup costs), computes every
//         item's effective request with Go's wrapping int64 adds and signed max, sums the
//         items exactly (lo32 / hi split words: no intermediate wrap), and the last
//         workgroup writes the four words to pinned host memory;
//   host: spins on a completion word the kernel writes after the sums (pinned memory,
//         the call's sequence number behind a system-scope fence) instead of a stream
//         synchronisation, whose wake-up alone cost more than the whole slice (VERDICT r4
//         item 7), then joins the exact sums and range-checks them (a sum outside int64 is
//         where the reference's Quantity would move to inf.Dec: ESC_E_LIMIT, as for the
//         resident path).  A kernel that never signals (a HIP error) is caught by the
//         stream synchronisation the spin falls back to after 1 s.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>

#include "esc_internal.h"

namespace esc {

namespace {

// One item per thread and every thread's loads independent of the others' (the meta and
// offset words together, then the records): the items are read from pinned host memory, so
// each dependent round trip is a PCIe latency, and a grid-stride loop over few threads had
// stacked ~8 of them (0.027 ms for 949 pods).
constexpr int LS_THREADS = 1024;
constexpr uint32_t LS_REG_MAX = 0xFFFF, LS_INIT_MAX = 0x7FFF;
constexpr uint32_t LS_OVH = 1u << 31;

// acc: [0] cpu lo32 sum, [1] cpu hi sum, [2] mem lo32 sum, [3] mem hi sum, [4] workgroups done.
// out (pinned host): the four sum words, then out[4] = seq once they are visible.
__global__ __launch_bounds__(LS_THREADS) void k_list_sum(const uint32_t* __restrict__ meta,
                                                         const uint32_t* __restrict__ off,
                                                         const int64_t* __restrict__ rec, int64_t n,
                                                         unsigned long long* __restrict__ acc,
                                                         unsigned long long* __restrict__ out, unsigned long long seq) {
    unsigned long long cl = 0, ml = 0;
    long long ch = 0, mh = 0;
    for (int64_t i = (int64_t)blockIdx.x * LS_THREADS + threadIdx.x; i < n; i += (int64_t)gridDim.x * LS_THREADS) {
        const uint32_t m = meta[i];
        const int64_t* r = rec + 2 * (int64_t)off[i];
        const uint32_t nreg = m & LS_REG_MAX, ninit = (m >> 16) & LS_INIT_MAX;
        uint64_t c = 0, mm = 0;                         // Resource.Add: int64 += (wraps), types.go:14-27
        for (uint32_t k = 0; k < nreg; ++k) {
            c += (uint64_t)r[2 * k];
            mm += (uint64_t)r[2 * k + 1];
        }
        r += 2 * nreg;
        for (uint32_t k = 0; k < ninit; ++k) {          // SetMaxResource over present keys, :30-43
            const int64_t x = r[2 * k], y = r[2 * k + 1];
            if (x > (int64_t)c) c = (uint64_t)x;
            if (y > (int64_t)mm) mm = (uint64_t)y;
        }
        if (m & LS_OVH) {                               // Spec.Overhead != nil, :84
            c += (uint64_t)r[2 * ninit];
            mm += (uint64_t)r[2 * ninit + 1];
        }
        cl += c & 0xFFFFFFFFull;
        ch += (long long)(int64_t)c >> 32;
        ml += mm & 0xFFFFFFFFull;
        mh += (long long)(int64_t)mm >> 32;
    }
    for (int o = 32; o > 0; o >>= 1) {
        cl += __shfl_xor(cl, o);
        ch += __shfl_xor(ch, o);
        ml += __shfl_xor(ml, o);
        mh += __shfl_xor(mh, o);
    }
    __shared__ unsigned long long s[LS_THREADS / 64][4];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) {
        s[wid][0] = cl; s[wid][1] = (unsigned long long)ch; s[wid][2] = ml; s[wid][3] = (unsigned long long)mh;
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        unsigned long long v = 0;
        for (int w = 0; w < LS_THREADS / 64; ++w) v += s[w][threadIdx.x];
        if (gridDim.x == 1) out[threadIdx.x] = v;       // one workgroup: straight to the host
        else atomicAdd(acc + threadIdx.x, v);
    }
    if (gridDim.x == 1) {
        __syncthreads();
        if (threadIdx.x == 0) {                         // the sums first, then the completion word
            __threadfence_system();
            __hip_atomic_store(out + 4, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        return;
    }
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long t = atomicAdd(acc + 4, 1ull);
        if (t == gridDim.x - 1) {                       // last workgroup: every add is in
            __threadfence();
            for (int k = 0; k < 4; ++k) {
                out[k] = atomicExch(acc + k, 0ull);
            }
            atomicExch(acc + 4, 0ull);
            __threadfence_system();
            __hip_atomic_store(out + 4, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

}  // namespace

struct ListReducer {
    int device = -1;
    int64_t cap_items = 0, cap_rec = 0;
    uint32_t* h_meta = nullptr;         // pinned: per item, n_reg | n_init << 16 | overhead << 31
    uint32_t* h_off = nullptr;          // pinned: its first record
    int64_t* h_rec = nullptr;           // pinned: (cpu, mem) per record
    unsigned long long* h_out = nullptr;// pinned: the four sum words + the completion word
    unsigned long long seq = 0;         // calls so far (the completion word's value)
    unsigned long long* d_acc = nullptr;// device: multi-workgroup accumulators (zero at rest)
    int max_blocks = 64;

    ~ListReducer() {
        if (h_meta) hipHostFree(h_meta);
        if (h_off) hipHostFree(h_off);
        if (h_rec) hipHostFree(h_rec);
        if (h_out) hipHostFree(h_out);
        if (d_acc) hipFree(d_acc);
    }
    hipError_t reserve(int64_t items, int64_t recs) {
        hipError_t e = hipSuccess;
        if (items > cap_items) {
            const int64_t c = std::max<int64_t>(items, 2 * cap_items);
            if (h_meta) hipHostFree(h_meta);
            if (h_off) hipHostFree(h_off);
            h_meta = nullptr;
            h_off = nullptr;
            cap_items = 0;
            if ((e = hipHostMalloc(reinterpret_cast<void**>(&h_meta), (size_t)c * 4))) return e;
            if ((e = hipHostMalloc(reinterpret_cast<void**>(&h_off), (size_t)c * 4))) return e;
            cap_items = c;
        }
        if (recs > cap_rec) {
            const int64_t c = std::max<int64_t>(recs, 2 * cap_rec);
            if (h_rec) hipHostFree(h_rec);
            h_rec = nullptr;
            cap_rec = 0;
            if ((e = hipHostMalloc(reinterpret_cast<void**>(&h_rec), (size_t)c * 16))) return e;
            cap_rec = c;
        }
        return e;
    }
};

namespace {

inline void put(int64_t* r, int64_t k, const esc_request& q, int64_t absent) {
    r[2 * k] = q.has_cpu ? q.cpu_m : absent;
    r[2 * k + 1] = q.has_mem ? q.mem_b : absent;
}

int32_t get_reducer(ListReducer*& r, int device) {
    if (r) return ESC_OK;
    ListReducer* x = new (std::nothrow) ListReducer();
    if (!x) return ESC_E_NOMEM;
    x->device = device;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess) x->max_blocks = std::max(1, prop.multiProcessorCount);
    if (hipHostMalloc(reinterpret_cast<void**>(&x->h_out), 8 * sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&x->d_acc), 5 * sizeof(unsigned long long)) != hipSuccess ||
        hipMemset(x->d_acc, 0, 5 * sizeof(unsigned long long)) != hipSuccess) {
        delete x;
        return ESC_E_HIP;
    }
    r = x;
    return ESC_OK;
}

// exact sum of the split words; false when it leaves int64
bool join(unsigned long long lo, unsigned long long hi, int64_t& v) {
    const __int128 t = (__int128)lo + ((__int128)(long long)hi << 32);
    if (t < (__int128)INT64_MIN || t > (__int128)INT64_MAX) return false;
    v = (int64_t)t;
    return true;
}

int32_t run(ListReducer* r, hipStream_t st, int64_t n, int64_t* mem_b, int64_t* cpu_m) {
    if (n == 0) {                                       // the Go loop's zero Quantities
        *mem_b = 0;
        *cpu_m = 0;
        return ESC_OK;
    }
    const int64_t want = (n + LS_THREADS - 1) / LS_THREADS;
    const int nblk = (int)std::min<int64_t>(std::max<int64_t>(want, 1), r->max_blocks);
    const unsigned long long seq = ++r->seq;
    hipLaunchKernelGGL(k_list_sum, dim3(nblk), dim3(LS_THREADS), 0, st, r->h_meta, r->h_off, r->h_rec, n, r->d_acc,
                       r->h_out, seq);
    if (hipGetLastError() != hipSuccess) return ESC_E_HIP;
    // wait for the completion word (the kernel's last store); give up spinning after 1 s and
    // let the stream synchronisation report whatever stopped the kernel
    const volatile unsigned long long* o = r->h_out;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t k = 0; __atomic_load_n(&r->h_out[4], __ATOMIC_ACQUIRE) != seq; ++k) {
        __builtin_ia32_pause();
        if ((k & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(1)) {
            if (hipStreamSynchronize(st) != hipSuccess) return ESC_E_HIP;
            if (__atomic_load_n(&r->h_out[4], __ATOMIC_ACQUIRE) != seq) return ESC_E_HIP;
            break;
        }
    }
    int64_t cpu, mem;
    if (!join(o[0], o[1], cpu) || !join(o[2], o[3], mem)) return ESC_E_LIMIT;
    *cpu_m = cpu;
    *mem_b = mem;
    return ESC_OK;
}

}  // namespace

int32_t list_pods_requests_total(ListReducer*& r, int device, void* stream, const esc_pod_obj* pods, int64_t n,
                                 int64_t* mem_b, int64_t* cpu_m) {
    if (int32_t rc = get_reducer(r, device)) return rc;
    int64_t nrec = 0;
    for (int64_t i = 0; i < n; ++i) {
        const esc_pod_obj& p = pods[i];
        if (p.n_containers < 0 || p.n_init_containers < 0 || (uint32_t)p.n_containers > LS_REG_MAX ||
            (uint32_t)p.n_init_containers > LS_INIT_MAX || (p.n_containers && !p.containers) ||
            (p.n_init_containers && !p.init_containers))
            return ESC_E_INVAL;
        nrec += p.n_containers + p.n_init_containers + (p.has_overhead ? 1 : 0);
    }
    if (hipSetDevice(device) != hipSuccess || r->reserve(n, nrec) != hipSuccess) return ESC_E_HIP;
    int64_t at = 0;
    for (int64_t i = 0; i < n; ++i) {
        const esc_pod_obj& p = pods[i];
        r->h_meta[i] = (uint32_t)p.n_containers | (uint32_t)p.n_init_containers << 16 | (p.has_overhead ? LS_OVH : 0u);
        r->h_off[i] = (uint32_t)at;
        int64_t* q = r->h_rec + 2 * at;
        for (int32_t k = 0; k < p.n_containers; ++k) put(q, k, p.containers[k], 0);            // absent adds 0
        q += 2 * (int64_t)p.n_containers;
        for (int32_t k = 0; k < p.n_init_containers; ++k) put(q, k, p.init_containers[k], INT64_MIN);  // absent: no max
        q += 2 * (int64_t)p.n_init_containers;
        if (p.has_overhead) put(q, 0, p.overhead, 0);
        at += p.n_containers + p.n_init_containers + (p.has_overhead ? 1 : 0);
    }
    if (at >= (int64_t)UINT32_MAX) return ESC_E_LIMIT;
    return run(r, (hipStream_t)stream, n, mem_b, cpu_m);
}

int32_t list_nodes_capacity_total(ListReducer*& r, int device, void* stream, const esc_node_obj* nodes, int64_t n,
                                  int64_t* mem_b, int64_t* cpu_m) {
    if (int32_t rc = get_reducer(r, device)) return rc;
    if (n >= (int64_t)UINT32_MAX) return ESC_E_LIMIT;
    if (hipSetDevice(device) != hipSuccess || r->reserve(n, n) != hipSuccess) return ESC_E_HIP;
    for (int64_t i = 0; i < n; ++i) {                   // Allocatable.Cpu() / .Memory(): absent = zero Quantity
        r->h_meta[i] = 1;
        r->h_off[i] = (uint32_t)i;
        put(r->h_rec, i, nodes[i].allocatable, 0);
    }
    return run(r, (hipStream_t)stream, n, mem_b, cpu_m);
}

void list_reducer_free(ListReducer*& r) {
    delete r;
    r = nullptr;
}

// ------------------------------------------------------------------ HBM read probe
namespace {
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
constexpr int HP_THREADS = 512, HP_U = 8;

// a contiguous share per workgroup, waves interleaved over 8-KB rounds, HP_U nontemporal
// 16-B loads per lane in flight (K1's K-tile stream shape); the XOR keeps the loads live
__global__ __launch_bounds__(HP_THREADS) void k_hbm_probe(const v4u* __restrict__ p, int64_t n16,
                                                          uint32_t* __restrict__ out) {
    const int64_t per = (n16 + gridDim.x - 1) / gridDim.x;
    const int64_t lo = (int64_t)blockIdx.x * per;
    const int64_t hi = lo + per < n16 ? lo + per : n16;
    uint32_t acc = 0;
    for (int64_t b = lo + threadIdx.x; b < hi; b += (int64_t)HP_THREADS * HP_U) {
        v4u v[HP_U];
#pragma unroll
        for (int u = 0; u < HP_U; ++u) {
            const int64_t i = b + (int64_t)u * HP_THREADS;
            v[u] = __builtin_nontemporal_load(p + (i < hi ? i : lo));
        }
#pragma unroll
        for (int u = 0; u < HP_U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (acc == 0x9E3779B9u) out[blockIdx.x & 255] = acc;     // (never, in practice)
}
}  // namespace

int32_t hbm_probe(int device, void* stream, int64_t bytes, int32_t reps, double* gbps) {
    if (bytes < (1 << 20) || reps < 1 || !gbps) return ESC_E_INVAL;
    hipStream_t st = (hipStream_t)stream;
    if (hipSetDevice(device) != hipSuccess) return ESC_E_HIP;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return ESC_E_HIP;
    const int64_t n16 = bytes / 16;
    v4u* buf = nullptr;
    uint32_t* out = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int32_t rc = ESC_OK;
    if (hipMalloc(reinterpret_cast<void**>(&buf), (size_t)n16 * 16) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&out), 256 * 4) != hipSuccess)
        rc = ESC_E_NOMEM;
    if (!rc && (hipMemsetAsync(buf, 0x5A, (size_t)n16 * 16, st) != hipSuccess || hipEventCreate(&e0) != hipSuccess ||
                hipEventCreate(&e1) != hipSuccess))
        rc = ESC_E_HIP;
    double best = 0;
    const int nblk = prop.multiProcessorCount;                  // one workgroup per CU, as K1
    for (int r = 0; !rc && r <= reps; ++r) {                    // launch 0 warms up
        hipEventRecord(e0, st);
        hipLaunchKernelGGL(k_hbm_probe, dim3(nblk), dim3(HP_THREADS), 0, st, buf, n16, out);
        hipEventRecord(e1, st);
        float ms = 0;
        if (hipGetLastError() != hipSuccess || hipEventSynchronize(e1) != hipSuccess ||
            hipEventElapsedTime(&ms, e0, e1) != hipSuccess) {
            rc = ESC_E_HIP;
            break;
        }
        if (r && ms > 0) best = std::max(best, (double)n16 * 16 / (ms * 1e-3) / 1e9);
    }
    if (e0) hipEventDestroy(e0);
    if (e1) hipEventDestroy(e1);
    if (buf) hipFree(buf);
    if (out) hipFree(out);
    *gbps = best;
    return rc;
}

}  // namespace esc
