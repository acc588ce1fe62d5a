// esc_common.h — internal definitions shared by the packer, the generator, the HIP
// kernels and the host runtime.  The decision arithmetic here is compiled twice:
// into the K4 kernel (device) and into the scalar C-ABI entry points (host).  Both
// builds use -ffp-contract=off so every float64 operation is the single IEEE-754
// operation the Go source performs.
#pragma once

#include <stdint.h>
#include "escalator_hip.h"

#if defined(__HIPCC__)
#define ESC_HD __host__ __device__ __forceinline__
#else
#define ESC_HD static inline
#endif

namespace esc {

constexpr uint32_t NONE = ESC_NONE;
constexpr int TILE = 256;                 // S tile: 64 lanes x 4 pods
constexpr int PODS_PER_LANE = 4;
constexpr int CTILE = 64;                 // C tile: 64 lanes x 1 pod
constexpr uint32_t CODE_MULTI = 0x80000000u;   // pair code: offset of a [count, g...] list
constexpr uint32_t NODE_DRY_BIT = 0x40000000u; // node membership entry: the group is in dry mode
constexpr uint32_t NODE_GROUP_MASK = 0x3FFFFFFFu;

// Fast-path packing ranges of K1's LDS partials.  A pod outside them is
// spilled by the same kernel to the exact "wide" global accumulators, so every input
// stays exact.  (Node sums are exact for any int64 input: K2 keeps them split lo32/hi.)
constexpr int64_t POD_CPU_LIMIT  = int64_t(1) << 20;   // per-pod effective millicores
constexpr int64_t POD_MEM_LIMIT  = int64_t(1) << 44;   // per-pod effective bytes
constexpr int64_t PODS_PER_BLOCK_MAX  = int64_t(1) << 20;  // keeps cpu|count<<40 exact
constexpr int CNT_SHIFT = 40;
constexpr uint64_t CPU_MASK = (uint64_t(1) << CNT_SHIFT) - 1;

// Per-group pod words, reduce-scattered with SUM across ranks to each group's owner
// (DESIGN.md §7).  Every sum travels split as
// lo = v & 0xffffffff, hi = v >> 32 (arithmetic) so the cross-rank SUM cannot wrap and
// the exact total is recoverable (Quantity.Add's overflow check).
enum PodWord : int { PW_CPU_LO = 0, PW_CPU_HI, PW_MEM_LO, PW_MEM_HI, PW_N, PW_K };
// Per-group node words (final, exact): untainted capacity sums and the filterNodes counts;
// NW_FLAGS carries ESC_TF_NODE_OVERFLOW.  One rank owns each group's node side (its pair's
// entries) and computes these words exactly; they are never exchanged.
enum NodeWord : int { NW_CPU = 0, NW_MEM, NW_N_UNT, NW_N_TAINT, NW_N_CORD, NW_FLAGS, NW_K };

// Device-side per-group parameters (from esc_group_spec + esc_group_state).
struct GroupParams {
    int32_t min_nodes, max_nodes;
    int32_t taint_upper, taint_lower, scale_up;
    int32_t slow_rate, fast_rate;
    int32_t dry;
    int32_t locked, requested;
    int64_t cached_cpu, cached_mem;
};

struct Totals {
    int64_t pod_cpu, pod_mem, n_pods;
    int64_t node_cpu, node_mem;
    int64_t n_nodes, n_unt, n_taint, n_cord;
    int64_t first, first_cpu, first_mem;
    int64_t flags;
};

// ------------------------------------------------------------- Go float helpers
ESC_HD uint64_t dbits(double x) { union { double d; uint64_t u; } v; v.d = x; return v.u; }
ESC_HD double bitsd(uint64_t x) { union { double d; uint64_t u; } v; v.u = x; return v.d; }
ESC_HD bool is_nan(double x) { return (dbits(x) & 0x7fffffffffffffffull) > 0x7ff0000000000000ull; }
ESC_HD bool is_pinf(double x) { return dbits(x) == 0x7ff0000000000000ull; }
ESC_HD bool is_inf(double x) { return (dbits(x) & 0x7fffffffffffffffull) == 0x7ff0000000000000ull; }
ESC_HD bool sign_bit(double x) { return (dbits(x) >> 63) != 0; }

constexpr double MAX_FLOAT64 = 1.7976931348623157e308;

// math.Max (Go stdlib): +Inf wins, then NaN, then the signed-zero rule.
ESC_HD double go_max(double x, double y) {
    if (is_pinf(x) || is_pinf(y)) return bitsd(0x7ff0000000000000ull);
    if (is_nan(x) || is_nan(y)) return bitsd(0x7ff8000000000001ull);
    if (x == 0.0 && x == y) return sign_bit(x) ? y : x;
    return x > y ? x : y;
}

// math.Ceil for finite |x| < 2^52 via truncation; NaN/Inf/huge pass through.
ESC_HD double go_ceil(double x) {
    if (is_nan(x) || is_inf(x)) return x;
    const double two52 = 4503599627370496.0;
    if (x >= two52 || x <= -two52) return x;
    double t = (double)(int64_t)x;            // exact truncation toward zero
    if (t < x) t += 1.0;
    if (t == 0.0 && sign_bit(x)) return -0.0; // ceil(-0.5) = -0
    return t;
}

// int(float64) on amd64 (CVTTSD2SQ): NaN, Inf and out-of-range give INT64_MIN.
ESC_HD int64_t go_int(double x) {
    if (is_nan(x) || !(x < 9223372036854775808.0) || !(x >= -9223372036854775808.0))
        return INT64_MIN;
    return (int64_t)x;
}

// Quantity.MilliValue() of a scale-0 memory amount: value*1000 with int64 wrap.
ESC_HD int64_t milli_mem(int64_t b) { return (int64_t)((uint64_t)b * 1000ull); }

// IEEE division that never traps (host C and device agree on x/0 already; kept explicit).
ESC_HD double fdiv(double a, double b) { return a / b; }

// calcPercentUsage — pkg/controller/util.go:58-81.
ESC_HD int32_t percent_usage(int64_t cpu_req, int64_t mem_req, int64_t cpu_cap, int64_t mem_cap,
                             int64_t n_unt, double* cpu, double* mem) {
    const int64_t a = cpu_req, b = milli_mem(mem_req), c = cpu_cap, d = milli_mem(mem_cap);
    if (a == 0 && b == 0 && c == 0 && d == 0 && n_unt == 0) { *cpu = 0.0; *mem = 0.0; return ESC_ST_OK; }
    if (c == 0 || d == 0) {
        if (n_unt == 0) { *cpu = MAX_FLOAT64; *mem = MAX_FLOAT64; return ESC_ST_OK; }
        *cpu = 0.0; *mem = 0.0; return ESC_ST_ERR_DIV_ZERO;
    }
    *cpu = fdiv((double)a, (double)c) * 100.0;
    *mem = fdiv((double)b, (double)d) * 100.0;
    return ESC_ST_OK;
}

// calcScaleUpDelta — pkg/controller/util.go:13-46.
ESC_HD int32_t scale_up_delta(int64_t n_unt, double cpu_pct, double mem_pct, int64_t cpu_req,
                              int64_t mem_req, int64_t cached_cpu, int64_t cached_mem,
                              int32_t scale_up_pct, int64_t* delta) {
    const double node_count = (double)n_unt;
    const double t = (double)scale_up_pct;
    double need_cpu, need_mem;
    if (cpu_pct == MAX_FLOAT64 || mem_pct == MAX_FLOAT64) {
        if (cached_cpu == 0 || cached_mem == 0) { *delta = 1; return ESC_ST_OK; }
        need_cpu = go_ceil(fdiv(fdiv((double)cpu_req, (double)cached_cpu), t) * 100.0);
        need_mem = go_ceil(fdiv(fdiv((double)milli_mem(mem_req), (double)milli_mem(cached_mem)), t) * 100.0);
    } else {
        const double pc = fdiv(cpu_pct - t, t);
        const double pm = fdiv(mem_pct - t, t);
        need_cpu = go_ceil(node_count * pc);
        need_mem = go_ceil(node_count * pm);
    }
    const int64_t d = go_int(go_max(need_cpu, need_mem));
    *delta = d;
    return d < 0 ? ESC_ST_ERR_NEG_DELTA : ESC_ST_OK;
}

// scaleNodeGroup's decision arithmetic — pkg/controller/controller.go:192-397 (the
// actuation calls at :367-383 stay with the host); scaleDownTaint clamp
// scale_down.go:138-158.
ESC_HD void decide_one(const GroupParams& p, const Totals& t, esc_group_decision& d) {
    d.cpu_pct = 0.0; d.mem_pct = 0.0; d.delta = 0; d.n_to_taint = 0;
    d.status = ESC_ST_OK; d.branch = ESC_BR_NONE; d.taint_status = ESC_ST_OK; d.reserved = 0;
    // :207-211 cache allNodes[0]'s allocatable (persisting host state)
    d.cached_cpu_m = t.n_nodes > 0 ? t.first_cpu : p.cached_cpu;
    d.cached_mem_b = t.n_nodes > 0 ? t.first_mem : p.cached_mem;
    if (t.n_nodes == 0 && t.n_pods == 0) { d.branch = ESC_BR_EMPTY; return; }          // :233
    if (t.n_nodes < p.min_nodes) { d.branch = ESC_BR_GATE; d.status = ESC_ST_ERR_MIN_NODES; return; } // :238
    if (t.n_nodes > p.max_nodes) { d.branch = ESC_BR_GATE; d.status = ESC_ST_ERR_MAX_NODES; return; } // :247
    if (t.flags & (ESC_TF_POD_OVERFLOW | ESC_TF_NODE_OVERFLOW)) {
        d.branch = ESC_BR_GATE; d.status = ESC_ST_ERR_OVERFLOW; return;
    }
    if (t.n_unt < p.min_nodes) { d.branch = ESC_BR_BELOW_MIN; d.delta = p.min_nodes - t.n_unt; return; } // :281
    double cpu, mem;
    int32_t st = percent_usage(t.pod_cpu, t.pod_mem, t.node_cpu, t.node_mem, t.n_unt, &cpu, &mem);
    d.cpu_pct = cpu; d.mem_pct = mem;
    if (st != ESC_ST_OK) { d.branch = ESC_BR_PCT_ERR; d.status = st; return; }        // :300
    if (p.locked) { d.branch = ESC_BR_LOCKED; d.delta = p.requested; return; }          // :317
    const double mx = go_max(cpu, mem);                                                 // :328
    if (mx < (double)p.taint_lower) { d.branch = ESC_BR_FAST_DOWN; d.delta = -(int64_t)p.fast_rate; }
    else if (mx < (double)p.taint_upper) { d.branch = ESC_BR_SLOW_DOWN; d.delta = -(int64_t)p.slow_rate; }
    else if (mx > (double)p.scale_up) {
        d.branch = ESC_BR_SCALE_UP;
        int64_t delta;
        st = scale_up_delta(t.n_unt, cpu, mem, t.pod_cpu, t.pod_mem, d.cached_cpu_m, d.cached_mem_b,
                            p.scale_up, &delta);
        d.delta = delta;
        if (st != ESC_ST_OK) { d.status = st; return; }                                 // :347
    }
    if (d.delta < 0) {                                                                   // :368
        int64_t n = -d.delta;
        if (t.n_unt - n < p.min_nodes) {
            n = t.n_unt - p.min_nodes;
            if (n < 0) { d.taint_status = ESC_ST_ERR_TAINT_MIN; n = 0; }
        }
        d.n_to_taint = n;
    }
}

// The gauges scaleNodeGroup sets in this run — controller.go:224-228 (before any gate),
// :275-278 (after the min/max gates), :309-315 (after calcPercentUsage succeeded; 0 when
// scaling up from 0).  Memory gauges are float64(Quantity.MilliValue() / 1000): the
// wrapped ×1000 product, integer-divided (truncating) by 1000.
ESC_HD void metrics_one(const Totals& t, const esc_group_decision& d, esc_group_metrics& m) {
    m.nodes = (double)t.n_nodes;
    m.nodes_cordoned = (double)t.n_cord;
    m.nodes_untainted = (double)t.n_unt;
    m.nodes_tainted = (double)t.n_taint;
    m.pods = (double)t.n_pods;
    m.cpu_request = m.cpu_capacity = m.mem_capacity = m.mem_request = 0.0;
    m.cpu_percent = m.mem_percent = 0.0;
    m.reserved = 0;
    m.set_mask = ESC_M_NODES | ESC_M_NODES_CORDONED | ESC_M_NODES_UNTAINTED | ESC_M_NODES_TAINTED | ESC_M_PODS;
    if (d.branch == ESC_BR_EMPTY || d.branch == ESC_BR_GATE) return;                    // :233-255
    m.cpu_request = (double)t.pod_cpu;
    m.cpu_capacity = (double)t.node_cpu;
    m.mem_capacity = (double)(milli_mem(t.node_mem) / 1000);
    m.mem_request = (double)(milli_mem(t.pod_mem) / 1000);
    m.set_mask |= ESC_M_CPU_REQUEST | ESC_M_CPU_CAPACITY | ESC_M_MEM_CAPACITY | ESC_M_MEM_REQUEST;
    if (d.branch == ESC_BR_BELOW_MIN || d.branch == ESC_BR_PCT_ERR) return;             // :281, :300
    const bool from_zero = d.cpu_pct == MAX_FLOAT64 || d.mem_pct == MAX_FLOAT64;
    m.cpu_percent = from_zero ? 0.0 : d.cpu_pct;
    m.mem_percent = from_zero ? 0.0 : d.mem_pct;
    m.set_mask |= ESC_M_CPU_PERCENT | ESC_M_MEM_PERCENT;
}

// ---------------------------------------------------------- pod flag helpers
ESC_HD uint32_t pf_xreg(uint32_t f)  { return (f >> ESC_PF_XREG_SHIFT) & ESC_PF_CNT_MASK; }
ESC_HD uint32_t pf_xinit(uint32_t f) { return (f >> ESC_PF_XINIT_SHIFT) & ESC_PF_CNT_MASK; }
ESC_HD uint32_t pf_xctr(uint32_t f)  { return pf_xreg(f) + pf_xinit(f) + ((f & ESC_PF_HAS_OVH) ? 1u : 0u); }
ESC_HD uint32_t pf_xpair(uint32_t f) { return (f >> ESC_PF_XPAIR_SHIFT) & ESC_PF_PAIR_MASK; }
ESC_HD bool pf_default_ok(uint32_t f) {
    return (f & (ESC_PF_DAEMONSET | ESC_PF_STATIC | ESC_PF_HAS_SEL | ESC_PF_AFF_BLOCK)) == 0;
}
ESC_HD uint32_t nf_xlbl(uint32_t f) { return (f >> ESC_NF_XLBL_SHIFT) & ESC_PF_CNT_MASK; }

}  // namespace esc
