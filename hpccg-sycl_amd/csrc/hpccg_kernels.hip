// hpccg_kernels.hip -- hand-written CDNA4 (gfx950) kernels for the HPCCG hot
// path. Memory-bound throughout (fp64, ~0.16 flop/byte): no MFMA; the design
// goals are coalesced 16 B/lane streams, one pass per fused step, XCD-local
// slice ownership, and bitwise-reproducible reductions.
//
// Numerics contract (tests/test_gpu_parity.py): compiled with
// -ffp-contract=off, SpMV and waxpby are BITWISE equal to the reference
// (HPC_sparsemv.cpp:76-87, waxpby.cpp:73-90: same per-row entry order, no
// FMA); dot products use a fixed-shape two-stage tree (per-slice partials,
// then one 1024-thread block in fixed order), so they are reproducible run to
// run and differ from the reference's sequential sum only by rounding.
#include <climits>
#include <type_traits>

#include "hpccg_internal.h"

#pragma clang fp contract(off)

namespace hpccg {

namespace {

constexpr int kWave = 64;

__device__ __forceinline__ unsigned long long now_ticks()
{
    return __builtin_amdgcn_s_memrealtime();  // 100 MHz constant clock
}

// Block b of a grid dealt round-robin over the 8 XCDs -> logical slice, so
// that every XCD walks one contiguous 1/8 of the rows (x re-reads of the
// stencil's neighbouring planes then hit that XCD's L2).
__device__ __forceinline__ int xcd_slice(int grid)
{
    const int b = blockIdx.x;
    const int per = grid / kNumXcd;
    return (b % kNumXcd) * per + (b / kNumXcd);
}

// Same XCD ownership, each XCD's slices in reverse order: a kernel that follows
// a forward sweep starts on the rows its predecessor wrote last (still in the
// XCD's L2 / the Infinity Cache).
__device__ __forceinline__ int xcd_slice_rev(int grid)
{
    const int b = blockIdx.x;
    const int per = grid / kNumXcd;
    return (b % kNumXcd) * per + (per - 1 - b / kNumXcd);
}

// The SpMV launches cover up to two slice ranges ([s0, s0 + n0) then
// [s1, s1 + n1)): all slices, or the interior / halo-dependent slices of a
// multi-rank iteration that overlaps its halo exchange. -1: no slice.
__device__ __forceinline__ int spmv_slice(const CgArgs& a)
{
    const int i = xcd_slice(a.sgrid);
    if (i >= a.sn0 + a.sn1) return -1;
    return i < a.sn0 ? a.s0 + i : a.s1 + (i - a.sn0);
}

// Lane l < off receives lane l + off (gfx950 lane moves, no LDS traffic):
// permlane32/16_swap for the cross-row steps, DPP row_shl inside a row.
template <int kOff>
__device__ __forceinline__ double from_lane_plus(double v)
{
    const int lo = __double2loint(v), hi = __double2hiint(v);
    int rlo, rhi;
    if constexpr (kOff == 32) {
        rlo = __builtin_amdgcn_permlane32_swap(lo, lo, false, false)[1];
        rhi = __builtin_amdgcn_permlane32_swap(hi, hi, false, false)[1];
    } else if constexpr (kOff == 16) {
        rlo = __builtin_amdgcn_permlane16_swap(lo, lo, false, false)[1];
        rhi = __builtin_amdgcn_permlane16_swap(hi, hi, false, false)[1];
    } else {
        static_assert(kOff >= 1 && kOff <= 8, "row_shl range");
        rlo = __builtin_amdgcn_update_dpp(0, lo, 0x100 + kOff, 0xF, 0xF, false);
        rhi = __builtin_amdgcn_update_dpp(0, hi, 0x100 + kOff, 0xF, 0xF, false);
    }
    return __hiloint2double(rhi, rlo);
}

// Wave sum, result valid in LANE 0 only. Fixed tree: the butterfly's lane 0,
// v_l += v_{l+off} for off = 32, 16, 8, 4, 2, 1 (lanes >= off are don't-care).
__device__ __forceinline__ double wave_sum(double v)
{
    v += from_lane_plus<32>(v);
    v += from_lane_plus<16>(v);
    v += from_lane_plus<8>(v);
    v += from_lane_plus<4>(v);
    v += from_lane_plus<2>(v);
    v += from_lane_plus<1>(v);
    return v;
}

// Deterministic block reduction (fixed shape): waves by shfl_xor, then the
// wave sums in wave order by thread 0. Result valid in thread 0.
template <int kThreads>
__device__ __forceinline__ double block_sum(double v)
{
    constexpr int kWaves = kThreads / kWave;
    __shared__ double wsum[kWaves];
    v = wave_sum(v);
    const int lane = threadIdx.x & (kWave - 1);
    const int w = threadIdx.x / kWave;
    if (lane == 0) wsum[w] = v;
    __syncthreads();
    double s = 0.0;
    if (threadIdx.x == 0) {
#pragma unroll
        for (int i = 0; i < kWaves; i++) s += wsum[i];
    }
    return s;
}

__device__ __forceinline__ void stamp(const CgArgs& a, int slot)
{
    const int idx = atomicAdd(&a.kst[2], 1);
    if (idx < a.stamp_cap) {
        a.stamps[2 * idx] = now_ticks();
        a.stamps[2 * idx + 1] = (unsigned long long)slot;
    }
}

// First kernel that finds the solve finished records the end time once.
__device__ __forceinline__ void mark_end(const CgArgs& a)
{
    if (atomicCAS(&a.kst[1], 0, 1) == 0) stamp(a, kStampEnd);
}

// HPCCG.cpp:358 loop condition for iteration k: k < max_iter && normr > tol,
// where normr is the value computed in iteration k-1, i.e. sqrt(r_{k-2}.r_{k-2})
// (sqrt(r_0.r_0) for k = 1). hist[j] = r_j.r_j is filled by the p-update
// kernel of iteration j+1; that kernel itself reads r_{k-1}.r_{k-1} from g.
__device__ __forceinline__ bool cg_run(const CgArgs& a, int k, bool in_p_update, double rr = 0.0)
{
    if (k >= a.max_iter) return false;
    double chk;
    if (k == 1)
        chk = in_p_update ? rr : a.hist[0];
    else
        chk = a.hist[k - 2];
    return sqrt(chk) > a.tol;
}

// ---------------------------------------------------------------------------
// Row-blocked vector access: each thread owns kRpt consecutive rows of the
// block's 512-row slice; kRpt = 2 gives 16 B per lane per stream.
// ---------------------------------------------------------------------------
template <int kRpt>
struct Rows {
    double v[kRpt];
};

template <int kRpt>
__device__ __forceinline__ Rows<kRpt> ld(const double* __restrict__ p)
{
    Rows<kRpt> r;
    if constexpr (kRpt == 1) {
        r.v[0] = p[0];
    } else {
#pragma unroll
        for (int i = 0; i < kRpt; i += 2) {
            const double2 t = *reinterpret_cast<const double2*>(p + i);
            r.v[i] = t.x;
            r.v[i + 1] = t.y;
        }
    }
    return r;
}

template <int kRpt>
__device__ __forceinline__ void st(double* __restrict__ p, const Rows<kRpt>& r)
{
    if constexpr (kRpt == 1) {
        p[0] = r.v[0];
    } else {
#pragma unroll
        for (int i = 0; i < kRpt; i += 2) *reinterpret_cast<double2*>(p + i) = make_double2(r.v[i], r.v[i + 1]);
    }
}

template <int kRpt>
__device__ __forceinline__ void ld_cols(const int* __restrict__ p, int (&c)[kRpt]);

typedef double d2v __attribute__((ext_vector_type(2)));
typedef int i2v __attribute__((ext_vector_type(2)));
typedef int i4v __attribute__((ext_vector_type(4)));

// Matrix streams: optionally non-temporal (read once per SpMV; keeps L2 for x).
template <int kRpt, bool kNT>
__device__ __forceinline__ Rows<kRpt> ld_m(const double* __restrict__ p)
{
    if constexpr (!kNT) {
        return ld<kRpt>(p);
    } else {
        Rows<kRpt> r;
        if constexpr (kRpt == 1) {
            r.v[0] = __builtin_nontemporal_load(p);
        } else {
#pragma unroll
            for (int i = 0; i < kRpt; i += 2) {
                const d2v t = __builtin_nontemporal_load(reinterpret_cast<const d2v*>(p + i));
                r.v[i] = t.x;
                r.v[i + 1] = t.y;
            }
        }
        return r;
    }
}

template <int kRpt, bool kNT>
__device__ __forceinline__ void ld_cols_m(const int* __restrict__ p, int (&c)[kRpt])
{
    if constexpr (!kNT) {
        ld_cols<kRpt>(p, c);
    } else if constexpr (kRpt == 1) {
        c[0] = __builtin_nontemporal_load(p);
    } else if constexpr (kRpt == 2) {
        const i2v t = __builtin_nontemporal_load(reinterpret_cast<const i2v*>(p));
        c[0] = t.x;
        c[1] = t.y;
    } else {
#pragma unroll
        for (int i = 0; i < kRpt; i += 4) {
            const i4v t = __builtin_nontemporal_load(reinterpret_cast<const i4v*>(p + i));
            c[i] = t.x;
            c[i + 1] = t.y;
            c[i + 2] = t.z;
            c[i + 3] = t.w;
        }
    }
}

template <int kRpt>
__device__ __forceinline__ void ld_cols(const int* __restrict__ p, int (&c)[kRpt])
{
    if constexpr (kRpt == 1) {
        c[0] = p[0];
    } else if constexpr (kRpt == 2) {
        const int2 t = *reinterpret_cast<const int2*>(p);
        c[0] = t.x;
        c[1] = t.y;
    } else {
#pragma unroll
        for (int i = 0; i < kRpt; i += 4) {
            const int4 t = *reinterpret_cast<const int4*>(p + i);
            c[i] = t.x;
            c[i + 1] = t.y;
            c[i + 2] = t.z;
            c[i + 3] = t.w;
        }
    }
}

// Vectors are allocated padded to a multiple of 512 rows, so full-width loads
// are always in bounds; rows >= n are masked on store and in the dots.

// p of iteration k lives in ring buffer k % nring: the update of p reads
// p_{k-1} from the previous buffer, and with x deferral the last nring p's
// stay available for the batched x update.
__device__ __forceinline__ double* cur_p(const CgArgs& a, int k)
{
    return a.p + (size_t)(k % a.nring) * (size_t)a.pstride;
}

template <int kRpt>
__device__ __forceinline__ void st_rows(double* __restrict__ base, int row, int n, const Rows<kRpt>& o)
{
    if (row + kRpt <= n) {
        st<kRpt>(base + row, o);
    } else {
        for (int i = 0; i < kRpt; i++)
            if (row + i < n) base[row + i] = o.v[i];
    }
}

// ---------------------------------------------------------------------------
// Dot-product completion, fixed two-level shape (bitwise identical whoever
// runs it): slice partials are summed in groups of kGroup by a 64-lane
// butterfly (group g = slices [64g, 64g+64)); the group sums are then added by
// kTopThreads "virtual" threads (virtual thread t adds group sums t, t+256, ...
// in order), a butterfly per virtual wave, and the 4 wave sums in order.
// which = kPAP: p.Ap (HPCCG.cpp:381); kRR: r.r (HPCCG.cpp:353, 367), which
// closes iteration k and advances kst[0].
//
// a.fold = 1 (default): completed inside the producing kernel. Every block
// publishes its partial with a write-through (sc1) store, waits for it
// (s_waitcnt vmcnt(0)) and takes a relaxed agent-scope ticket on its group;
// the group's last arriver (told by the ticket value) acquires, reads the
// group's partials with sc1 loads, publishes the group sum the same way and
// takes a ticket on the top counter; the last group reducer forms the total.
// This is the guide's in-launch split-K form (cdna_hip_programming.md 5,
// "In-launch split-K reduction", sc1 slab stores, no release fence): a
// per-block agent release (buffer_wbl2) instead measured 57 -> 653 us on the
// update kernel, and one block reading all 15625 partials took 8.9 us.
// a.fold = 0: a separate one-block k_finalize computes the same two levels.
// ---------------------------------------------------------------------------
constexpr int kGroup = 64;
constexpr int kTopThreads = 256;

__device__ __forceinline__ void st_sc1(double* p, double v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ int ngroups_of(const CgArgs& a) { return (a.nslices + kGroup - 1) / kGroup; }

// group sum by one wave (lane l reads slice partial 64g + l)
__device__ __forceinline__ double group_sum(const CgArgs& a, int g, int lane)
{
    const int i = g * kGroup + lane;
    const double v = (i < a.nslices) ? ld_sc1(a.partial + i) : 0.0;
    return wave_sum(v);
}

// The same fixed shape computed by one wave (virtual waves in order); valid in
// lane 0. ld(i) reads group sum i. All loads are issued before the sums.
template <class Ld>
__device__ __forceinline__ double top_sum_wave(Ld ld, int ng, int lane)
{
    constexpr int kVWaves = kTopThreads / kWave;
    double v[kVWaves];
#pragma unroll
    for (int vw = 0; vw < kVWaves; vw++) v[vw] = 0.0;
    for (int i0 = 0; i0 < ng; i0 += kTopThreads) {
        double t[kVWaves];
#pragma unroll
        for (int vw = 0; vw < kVWaves; vw++) {
            const int i = i0 + vw * kWave + lane;
            t[vw] = i < ng ? ld(i) : 0.0;
        }
#pragma unroll
        for (int vw = 0; vw < kVWaves; vw++)
            if (i0 + vw * kWave < ng) v[vw] += t[vw];
    }
    double s = 0.0;
#pragma unroll
    for (int vw = 0; vw < kVWaves; vw++) s += wave_sum(v[vw]);
    return s;
}

// r_{k-1}.r_{k-1} from the update's group sums, in every thread (redund mode),
// else g[kRR].
__device__ __forceinline__ double cur_rr(const CgArgs& a)
{
    if (!a.redund) return a.g[kRR];
    const int ng = ngroups_of(a);
    const double* gp = a.partial + a.nslices + kRR * ng;
    const int lane = threadIdx.x & (kWave - 1);
    const double v = top_sum_wave([gp](int i) { return gp[i]; }, ng, lane);
    return __shfl(v, 0, kWave);
}

__device__ __forceinline__ void finish_dot(const CgArgs& a, double s, int which, int kfinal)
{
    a.loc[which] = s;
    if (a.nranks == 1) a.g[which] = s;
    if (which == kRR) a.kst[0] = kfinal;
    // multi-rank: the local sum is done, the all-reduce comes next (t4 class)
    if (a.nranks > 1) stamp(a, which == kRR ? kStampArRR : kStampArPAP);
}

// Partials of slices s0 .. s0 + cnt - 1 (one group: s0 % kGroup + cnt <=
// kGroup), the partial of slice s0 + j in lane j of wave 0; called by wave 0
// only. The lanes publish their partials together, lane 0 takes one ticket of
// cnt arrivals on the group; the group's last arriver then sums the group and
// takes a ticket on the top counter, whose last arriver forms the total.
__device__ __forceinline__ void complete_dot_lanes(const CgArgs& a, int s0, int cnt, double bs, int which,
                                                   int kfinal)
{
    const int ng = ngroups_of(a);
    double* gp = a.partial + a.nslices + which * ng;       // group sums of this dot
    unsigned* gt = a.tickets + which * (ng + 1);          // group tickets, then the top one
    const int lane = threadIdx.x;
    if (!fold_of(a, which)) {
        double* dst = (which == kPAP && a.pap_upd) ? a.ppart : a.partial;
        if (lane < cnt) dst[s0 + lane] = bs;
        return;
    }
    const int g = s0 / kGroup;
    int role = 0;
    if (lane < cnt) st_sc1(a.partial + s0 + lane, bs);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) {
        const unsigned glen = (unsigned)min(kGroup, a.nslices - g * kGroup);
        const unsigned t =
            __hip_atomic_fetch_add(gt + g, (unsigned)cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        role = (t + (unsigned)cnt == glen) ? 1 : 0;
        if (role) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
    role = __shfl(role, 0, kWave);
    if (role == 0) return;
    // group reducer (this wave): sc1 loads of the group's partials
    const double v = group_sum(a, g, lane);
    if (lane == 0) {
        st_sc1(gp + g, v);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(gt + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
        const unsigned t = __hip_atomic_fetch_add(gt + ng, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        role = (t == (unsigned)ng - 1u) ? 2 : 0;
        if (role == 2) {
            stamp(a, which == kRR ? kStampFinRR : kStampFinPAP);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
    role = __shfl(role, 0, kWave);
    if (role != 2) return;
    const double tot = top_sum_wave([gp](int i) { return ld_sc1(gp + i); }, ng, lane);
    if (lane == 0) {
        finish_dot(a, tot, which, kfinal);
        __hip_atomic_store(gt + ng, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
    }
}

// bs valid in thread 0. Only wave 0 takes part in the hand-off: the other waves
// of the block return right away (the publish round trip then holds one wave,
// not the block).
template <int kThreads>
__device__ __forceinline__ void complete_dot(const CgArgs& a, int s, double bs, int which, int kfinal)
{
    if (threadIdx.x >= kWave) return;
    complete_dot_lanes(a, s, 1, bs, which, kfinal);
}

// ---------------------------------------------------------------------------
// Prologue: p = x + 0.0*x   (HPCCG.cpp:347, waxpby(nrow, 1.0, x, 0.0, x, p))
// ---------------------------------------------------------------------------
template <int kRpt>
__global__ __launch_bounds__(kSliceRows / kRpt) void k_prologue_copy(CgArgs a)
{
    const int s = xcd_slice(a.grid);
    if (blockIdx.x == 0 && threadIdx.x == 0) stamp(a, kStampPrologue);
    if (s >= a.nslices) return;
    const int row = s * kSliceRows + threadIdx.x * kRpt;
    Rows<kRpt> xv = ld<kRpt>(a.x + row), o;
#pragma unroll
    for (int i = 0; i < kRpt; i++) o.v[i] = xv.v[i] + 0.0 * xv.v[i];
    st_rows<kRpt>(a.p, row, a.n, o);
}

// ---------------------------------------------------------------------------
// p = r + beta*p  (HPCCG.cpp:362 for k == 1: p = r + 0*r; :366-369 otherwise)
// Separate kernel only when the update is not fused into the SpMV (multi-rank:
// the halo of p must be exchanged between the two).
// ---------------------------------------------------------------------------
template <int kRpt>
__global__ __launch_bounds__(kSliceRows / kRpt) void k_p_update(CgArgs a)
{
    const int k = a.kst[0];
    const double rr = cur_rr(a);
    const bool run = cg_run(a, k, true, rr);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (k == 1 || run) a.hist[k - 1] = rr;
        if (run)
            stamp(a, kStampPUpdate);
        else
            mark_end(a);
    }
    if (!run) return;
    const int s = xcd_slice(a.grid);
    if (s >= a.nslices) return;
    const int row = s * kSliceRows + threadIdx.x * kRpt;
    const double beta = (k == 1) ? 0.0 : rr / a.hist[k - 2];
    const Rows<kRpt> rv = ld<kRpt>(a.r + row);
    const Rows<kRpt> yv = (k == 1) ? rv : ld<kRpt>(cur_p(a, k - 1) + row);
    Rows<kRpt> o;
#pragma unroll
    for (int i = 0; i < kRpt; i++) o.v[i] = rv.v[i] + beta * yv.v[i];
    st_rows<kRpt>(cur_p(a, k), row, a.n, o);
}

// Multi-rank with the p update fused into the SpMV: the rows the neighbours
// need (the first nlo and last nhi local rows) are updated first, by this
// kernel, so the halo can move p_k before the SpMV computes the rest. Same
// expression as k_p_update; the SpMV later stores the same bits there again.
__global__ __launch_bounds__(256) void k_p_boundary(CgArgs a, int nlo, int nhi)
{
    const int k = a.kst[0];
    const double rr = cur_rr(a);
    if (!cg_run(a, k, true, rr)) return;
    if (blockIdx.x == 0 && threadIdx.x == 0) stamp(a, kStampHalo);  // halo class from here
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= nlo + nhi) return;
    const int row = i < nlo ? i : a.n - nhi + (i - nlo);
    const double beta = (k == 1) ? 0.0 : rr / a.hist[k - 2];
    const double rv = a.r[row];
    const double yv = (k == 1) ? rv : cur_p(a, k - 1)[row];
    cur_p(a, k)[row] = rv + beta * yv;
}

// Gather halo plan: pack p_k at the rows the requesting ranks need
// (exchange_externals.cpp:100-118 fills send_buffer the same way). With the p
// update fused into the SpMV, p_k is computed here with k_p_update's exact
// expression (the SpMV stores the same bits at those rows later).
__global__ __launch_bounds__(256) void k_pack(CgArgs a, const int* __restrict__ idx, int cnt,
                                              double* __restrict__ buf, bool prologue)
{
    int k = 0;
    double rr = 0.0;
    if (!prologue) {
        k = a.kst[0];
        rr = cur_rr(a);
        if (!cg_run(a, k, true, rr)) return;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) stamp(a, kStampHalo);  // halo class from here
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= cnt) return;
    const int e = idx[i];
    double v;
    if (prologue) {
        v = a.p[e];
    } else if (a.fuse_p) {
        const double beta = (k == 1) ? 0.0 : rr / a.hist[k - 2];
        const double rv = a.r[e];
        const double yv = (k == 1) ? rv : cur_p(a, k - 1)[e];
        v = rv + beta * yv;
    } else {
        v = cur_p(a, k)[e];
    }
    buf[i] = v;
}

// ---------------------------------------------------------------------------
// SpMV over SELL-512 (HPC_sparsemv.cpp:68-89) + fused p.Ap slice partial
// (ddot.cpp:60-73), optionally + the p update (waxpby, HPCCG.cpp:362/369).
//
// Thread t of slice s owns rows s*512 + t*kRpt + [0, kRpt). Slot j of the
// slice is a contiguous 512-entry run: lane loads are 16 B (vals) / 8 B (cols)
// and a wave reads 1 KiB + 512 B per slot. x is gathered through L1/L2/MALL;
// for the stencil the 64 lanes of a wave hit consecutive x.
// Gather source G(c): p[c] (plain), or r[c] + beta*p_old[c] (fused p update:
// the exact expression k_p_update stores, so every row sum is unchanged).
// kW > 0: slice width known at compile time (27 / 7), fully unrolled.
// ---------------------------------------------------------------------------
struct GatherP {
    const double* __restrict__ x;
    __device__ __forceinline__ double operator()(int c) const { return x[c]; }
};
struct GatherRP {
    const double* __restrict__ r;
    const double* __restrict__ pold;
    double beta;
    __device__ __forceinline__ double operator()(int c) const { return r[c] + beta * pold[c]; }
};

template <int kRpt, int kW, bool kNT, class G>
__device__ __forceinline__ void spmv_rows(const CgArgs& a, const G& gat, int s, double (&sum)[kRpt])
{
    // kW > 0: every slice has exactly kW slots (host padded the image to a
    // uniform width), so slice s starts at s*kW and the loop fully unrolls.
    const size_t b0 = (kW > 0) ? (size_t)s * kW : (size_t)a.slice_base[s];
    const int w = (kW > 0) ? kW : (int)(a.slice_base[s + 1] - a.slice_base[s]);
    const size_t base = b0 * kSliceRows + (size_t)threadIdx.x * kRpt;
    const double* __restrict__ vp = a.vals + base;
    const int* __restrict__ cp = a.cols + base;
#pragma unroll
    for (int i = 0; i < kRpt; i++) sum[i] = 0.0;
    if constexpr (kW > 0) {
#pragma unroll
        for (int j = 0; j < kW; j++) {
            int c[kRpt];
            ld_cols_m<kRpt, kNT>(cp + (size_t)j * kSliceRows, c);
            const Rows<kRpt> v = ld_m<kRpt, kNT>(vp + (size_t)j * kSliceRows);
#pragma unroll
            for (int i = 0; i < kRpt; i++) {
                const double xv = (c[i] >= 0) ? gat(c[i]) : 0.0;
                sum[i] = sum[i] + v.v[i] * xv;
            }
        }
    } else {
#pragma unroll 3
        for (int j = 0; j < w; j++) {
            int c[kRpt];
            ld_cols_m<kRpt, kNT>(cp + (size_t)j * kSliceRows, c);
            const Rows<kRpt> v = ld_m<kRpt, kNT>(vp + (size_t)j * kSliceRows);
#pragma unroll
            for (int i = 0; i < kRpt; i++) {
                const double xv = (c[i] >= 0) ? gat(c[i]) : 0.0;
                sum[i] = sum[i] + v.v[i] * xv;
            }
        }
    }
}

// Padding slots add v*x = 0*0 = +0: a sum that starts at +0.0 is never -0 under
// round-to-nearest, so +0 leaves every row sum bit-identical to skipping it.

// SELL-512-C: per slice a dictionary of the distinct (column - row) offsets
// (at most 255; stencils have 7 or 27), and per stored entry a 1-byte code
// (kCodePad = padding). The stream is 8 B value + 1 B code per slot. The plain
// kernel gathers x[row + dict[code]]; the LDS kernel reads its staged window
// at lane + ldsc[code], a per-slice constant for every code (checked at
// build). Same products in the same order as SELL-512.
template <int kRpt, bool kNT>
__device__ __forceinline__ void ld_codes(const unsigned char* __restrict__ p, unsigned (&c)[kRpt])
{
    if constexpr (kRpt == 1) {
        c[0] = kNT ? __builtin_nontemporal_load(p) : p[0];
    } else if constexpr (kRpt == 2) {
        const unsigned short t = kNT ? __builtin_nontemporal_load(reinterpret_cast<const unsigned short*>(p))
                                     : *reinterpret_cast<const unsigned short*>(p);
        c[0] = t & 0xFFu;
        c[1] = t >> 8;
    } else {
#pragma unroll
        for (int i = 0; i < kRpt; i += 4) {
            const unsigned t = kNT ? __builtin_nontemporal_load(reinterpret_cast<const unsigned*>(p + i))
                                   : *reinterpret_cast<const unsigned*>(p + i);
#pragma unroll
            for (int q = 0; q < 4; q++) c[i + q] = (t >> (8 * q)) & 0xFFu;
        }
    }
}

template <int kRpt, bool kNT, bool kFuse, int kW = 0, bool kVal = false>
__global__ __launch_bounds__(kSliceRows / kRpt) void k_spmv_c(CgArgs a, bool prologue)
{
    __shared__ int sdict[kCodes];
    __shared__ double sval[kVal ? kCodes : 1];
    int k = 0;
    double rr = 0.0;  // r_{k-1}.r_{k-1}: the fused p update needs it
    if (!prologue) {
        k = a.kst[0];
        if (kFuse) rr = cur_rr(a);
        const bool run = cg_run(a, k, kFuse, rr);
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            if (kFuse && (k == 1 || run)) a.hist[k - 1] = rr;
            if (run)
                stamp(a, kStampSpmv);
            else
                mark_end(a);
        }
        if (!run) return;
    }
    const int s = spmv_slice(a);
    if (s < 0) return;
    {
        const int nc = a.ccount[s];  // codes in use; kCodePad has value 0
        for (int i = threadIdx.x; i < nc; i += kSliceRows / kRpt) {
            sdict[i] = a.cdict[(size_t)s * kCodes + i];
            if constexpr (kVal) sval[i] = a.cval[(size_t)s * kCodes + i];
        }
        if (kVal && threadIdx.x == 0) sval[kCodePad] = 0.0;
    }
    __syncthreads();
    const int row = s * kSliceRows + threadIdx.x * kRpt;
    double* __restrict__ p = cur_p(a, k);
    // kW > 0: uniform image of width kW, the slot loop fully unrolled
    const size_t b0 = kW > 0 ? (size_t)s * kW : (size_t)a.slice_base[s];
    const int w = kW > 0 ? kW : (int)(a.slice_base[s + 1] - b0);
    const size_t base = b0 * kSliceRows + (size_t)threadIdx.x * kRpt;
    const double* __restrict__ vp = a.vals + base;
    const unsigned char* __restrict__ cp = a.ccodes + base;
    double beta = 0.0;
    const double* pold = a.r;
    if constexpr (kFuse) {
        beta = (k == 1) ? 0.0 : rr / a.hist[k - 2];
        pold = (k == 1) ? a.r : cur_p(a, k - 1);
    }
    const double* __restrict__ xext = p - a.ghost_lo;
    double sum[kRpt];
#pragma unroll
    for (int i = 0; i < kRpt; i++) sum[i] = 0.0;
#pragma unroll kW > 0 ? kW : 3
    for (int j = 0; j < w; j++) {
        unsigned c[kRpt];
        ld_codes<kRpt, kNT>(cp + (size_t)j * kSliceRows, c);
        Rows<kRpt> v;
        if constexpr (kVal) {
#pragma unroll
            for (int i = 0; i < kRpt; i++) v.v[i] = sval[c[i]];
        } else {
            v = ld_m<kRpt, kNT>(vp + (size_t)j * kSliceRows);
        }
#pragma unroll
        for (int i = 0; i < kRpt; i++) {
            double xv = 0.0;
            if (c[i] != kCodePad) {
                const int col = row + i + sdict[c[i]];
                if constexpr (kFuse) xv = a.r[col - a.ghost_lo] + beta * pold[col - a.ghost_lo];
                else xv = xext[col];
            }
            sum[i] = sum[i] + v.v[i] * xv;
        }
    }
    Rows<kRpt> pv;
    if constexpr (kFuse) {
        const Rows<kRpt> rv = ld<kRpt>(a.r + row);
        const Rows<kRpt> yv = ld<kRpt>(pold + row);
#pragma unroll
        for (int i = 0; i < kRpt; i++) pv.v[i] = rv.v[i] + beta * yv.v[i];
        st_rows<kRpt>(p, row, a.n, pv);
    } else {
        pv = ld<kRpt>(p + row);
    }
    Rows<kRpt> o;
#pragma unroll
    for (int i = 0; i < kRpt; i++) o.v[i] = sum[i];
    st_rows<kRpt>(a.Ap, row, a.n, o);
    if (prologue) return;
    double d = 0.0;
#pragma unroll
    for (int i = 0; i < kRpt; i++)
        if (row + i < a.n) d += pv.v[i] * o.v[i];
    const double bs = block_sum<kSliceRows / kRpt>(d);
    complete_dot<kSliceRows / kRpt>(a, s, bs, kPAP, 0);
}

// ---------------------------------------------------------------------------
// SELL-512-V4: the SELL-512-V codes regrouped in chunks of kVC = 4 slots, row
// by row inside a chunk (a row's 4 codes are one dword; 2 rows one qword), so
// a thread fetches 4 slots per load instead of 1. Chunk padding is kCodePad.
// The kernel gathers x[row + dict[code]] from global memory (L1/L2 hits) with
// every gather of a chunk in flight; the values come from the slice's LDS
// dictionary. Same products in the same order as SELL-512. With one row per
// thread, the p.Ap partial is formed on thread pairs and reduced in the
// 256-thread tree of the two-rows-per-thread kernels: the same bits.
// ---------------------------------------------------------------------------
constexpr int kVC = 4;

__global__ __launch_bounds__(256) void k_interleave_v4(const unsigned int* __restrict__ slice_base,
                                                       const unsigned int* __restrict__ vbase4, int nslices,
                                                       const unsigned char* __restrict__ codes,
                                                       unsigned char* __restrict__ out)
{
    const int s = blockIdx.x;
    if (s >= nslices) return;
    const size_t e0 = (size_t)slice_base[s] * kSliceRows, e1 = (size_t)slice_base[s + 1] * kSliceRows;
    unsigned char* o = out + (size_t)vbase4[s] * (kSliceRows * kVC);
    for (size_t e = e0 + threadIdx.x; e < e1; e += 256) {
        const int j = (int)((e - e0) / kSliceRows), lane = (int)((e - e0) % kSliceRows);
        o[(size_t)(j / kVC) * (kSliceRows * kVC) + lane * kVC + j % kVC] = codes[e];
    }
}

template <int kRpt, bool kNT>
__device__ __forceinline__ void ld_chunk(const unsigned char* __restrict__ p, unsigned (&c)[kRpt])
{
    if constexpr (kRpt == 1) {
        c[0] = kNT ? __builtin_nontemporal_load(reinterpret_cast<const unsigned*>(p))
                   : *reinterpret_cast<const unsigned*>(p);
    } else {
        static_assert(kRpt == 2, "1 or 2 rows per thread");
        typedef unsigned u2v __attribute__((ext_vector_type(2)));
        const u2v t = kNT ? __builtin_nontemporal_load(reinterpret_cast<const u2v*>(p))
                          : *reinterpret_cast<const u2v*>(p);
        c[0] = t.x;
        c[1] = t.y;
    }
}

// kPre > 0: the first kPre chunks of codes are loaded before the dictionary
// barrier (the whole row for widths <= 4 kPre).
template <int kRpt, bool kNT, bool kFuse, int kW, int kPre = 0>
__global__ __launch_bounds__(kSliceRows / kRpt) void k_spmv_v4(CgArgs a, bool prologue)
{
    __shared__ int sdict[kCodes];
    __shared__ double sval[kCodes];
    __shared__ double spair[kRpt == 1 ? kSliceRows / 2 : 1];
    __shared__ double wsum[4];
    int k = 0;
    double rr = 0.0;  // r_{k-1}.r_{k-1}: the fused p update needs it
    if (!prologue) {
        k = a.kst[0];
        if (kFuse) rr = cur_rr(a);
        const bool run = cg_run(a, k, kFuse, rr);
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            if (kFuse && (k == 1 || run)) a.hist[k - 1] = rr;
            if (run)
                stamp(a, kStampSpmv);
            else
                mark_end(a);
        }
        if (!run) return;
    }
    const int s = spmv_slice(a);
    if (s < 0) return;
    const unsigned c0 = a.vbase4[s];
    const int nch = kW > 0 ? (kW + kVC - 1) / kVC : (int)(a.vbase4[s + 1] - c0);
    const unsigned char* __restrict__ cp =
        a.vcodes4 + (size_t)c0 * (kSliceRows * kVC) + (size_t)threadIdx.x * (kRpt * kVC);
    // dictionary loads first (the first kDict entries without waiting for the
    // count), then the code prefetch: vmcnt retires in order
    constexpr int kDict = 32;
    const int nc = a.ccount[s];  // codes in use; kCodePad has value 0
    int dk = 0;
    double dv = 0.0;
    if (threadIdx.x < kDict) {
        dk = a.cdict[(size_t)s * kCodes + threadIdx.x];
        dv = a.cval[(size_t)s * kCodes + threadIdx.x];
    }
    constexpr int kP = kPre > 0 ? kPre : 1;
    unsigned cpre[kP][kRpt];
#pragma unroll
    for (int q = 0; q < kPre; q++)
        if (q < nch) ld_chunk<kRpt, kNT>(cp + (size_t)q * (kSliceRows * kVC), cpre[q]);
    if (threadIdx.x < kDict) {
        sdict[threadIdx.x] = dk;
        sval[threadIdx.x] = dv;
    }
    for (int i = kDict + threadIdx.x; i < nc; i += kSliceRows / kRpt) {
        sdict[i] = a.cdict[(size_t)s * kCodes + i];
        sval[i] = a.cval[(size_t)s * kCodes + i];
    }
    if (threadIdx.x == 0) sval[kCodePad] = 0.0;
    __syncthreads();
    const int row = s * kSliceRows + threadIdx.x * kRpt;
    double* __restrict__ p = cur_p(a, k);
    double beta = 0.0;
    const double* pold = a.r;
    if constexpr (kFuse) {
        beta = (k == 1) ? 0.0 : rr / a.hist[k - 2];
        pold = (k == 1) ? a.r : cur_p(a, k - 1);
    }
    const double* __restrict__ xext = p - a.ghost_lo;
    double sum[kRpt];
#pragma unroll
    for (int i = 0; i < kRpt; i++) sum[i] = 0.0;
    auto chunk = [&](const unsigned (&cw)[kRpt]) {
#pragma unroll
        for (int jj = 0; jj < kVC; jj++) {
#pragma unroll
            for (int i = 0; i < kRpt; i++) {
                const unsigned c = (cw[i] >> (8 * jj)) & 0xFFu;
                double xv = 0.0;
                if (c != kCodePad) {
                    const int col = row + i + sdict[c];
                    if constexpr (kFuse) xv = a.r[col - a.ghost_lo] + beta * pold[col - a.ghost_lo];
                    else xv = xext[col];
                }
                sum[i] = sum[i] + sval[c] * xv;
            }
        }
    };
#pragma unroll
    for (int q = 0; q < kPre; q++)
        if (q < nch) chunk(cpre[q]);
#pragma unroll kW > 0 ? (kW + kVC - 1) / kVC : 2
    for (int q = kPre; q < nch; q++) {
        unsigned cw[kRpt];
        ld_chunk<kRpt, kNT>(cp + (size_t)q * (kSliceRows * kVC), cw);
        chunk(cw);
    }
    Rows<kRpt> pv;
    if constexpr (kFuse) {
        const Rows<kRpt> rv = ld<kRpt>(a.r + row);
        const Rows<kRpt> yv = ld<kRpt>(pold + row);
#pragma unroll
        for (int i = 0; i < kRpt; i++) pv.v[i] = rv.v[i] + beta * yv.v[i];
        st_rows<kRpt>(p, row, a.n, pv);
    } else {
        pv = ld<kRpt>(p + row);
    }
    Rows<kRpt> o;
#pragma unroll
    for (int i = 0; i < kRpt; i++) o.v[i] = sum[i];
    st_rows<kRpt>(a.Ap, row, a.n, o);
    if (prologue) return;
    double bs;
    if constexpr (kRpt == 2) {
        double d = 0.0;
#pragma unroll
        for (int i = 0; i < kRpt; i++)
            if (row + i < a.n) d += pv.v[i] * o.v[i];
        bs = block_sum<kSliceRows / kRpt>(d);
    } else {
        // (0 + p_2t Ap_2t) + p_2t+1 Ap_2t+1 on the even lane (an absent row
        // adds +0: the sum is never -0), then block_sum<256>'s tree
        const double t = (row < a.n) ? pv.v[0] * o.v[0] : 0.0;
        const double u = from_lane_plus<1>(t);
        if ((threadIdx.x & 1) == 0) spair[threadIdx.x >> 1] = (0.0 + t) + u;
        __syncthreads();
        double v = 0.0;
        if (threadIdx.x < kSliceRows / 2) v = wave_sum(spair[threadIdx.x]);
        if (threadIdx.x < kSliceRows / 2 && (threadIdx.x & (kWave - 1)) == 0) wsum[threadIdx.x / kWave] = v;
        __syncthreads();
        bs = 0.0;
        if (threadIdx.x == 0) {
#pragma unroll
            for (int i = 0; i < 4; i++) bs += wsum[i];
        }
    }
    complete_dot<kSliceRows / kRpt>(a, s, bs, kPAP, 0);
}

// SELL-512-C / -V build: one block per slice. An LDS hash of the slice's
// distinct keys gives the codes: the (column - row) offset (C), or the pair
// (offset, value) (V; the values get their own hash first, so a pair is one
// 64-bit key: offset, value code). With windows, ldsc[code] is the LDS
// position of row 0's column for that offset, and every entry must agree.
// ok[0] = 0: more than 255 keys in a slice; ok[1] = 0: no LDS form.
__global__ __launch_bounds__(256) void k_build_c(const unsigned int* __restrict__ slice_base, int nslices,
                                                 const int* __restrict__ cols, const double* __restrict__ vals,
                                                 const int* __restrict__ win_ptr,
                                                 const int* __restrict__ win_start, const int* __restrict__ win_off,
                                                 const int* __restrict__ win_len,
                                                 unsigned char* __restrict__ codes, int* __restrict__ cdict,
                                                 double* __restrict__ cval, int* __restrict__ ldsc,
                                                 int* __restrict__ ccount, int* ok)
{
    typedef unsigned long long u64;
    constexpr int kH = 1024;
    constexpr u64 kEmpty = ~0ull;  // neither a pair key (value code <= 254) nor, checked, a value
    constexpr int kEmptyPos = INT_MIN;
    __shared__ u64 keys[kH];
    __shared__ int code_of[kH];
    __shared__ u64 vkeys[kH];
    __shared__ int vcode_of[kH];
    __shared__ double svals[kCodePad];
    __shared__ int sldsc[kCodes];
    __shared__ int cnt, vcnt;
    const int s = blockIdx.x;
    if (s >= nslices) return;
    for (int h = threadIdx.x; h < kH; h += 256) {
        keys[h] = kEmpty;
        vkeys[h] = kEmpty;
    }
    if (threadIdx.x == 0) {
        cnt = 0;
        vcnt = 0;
    }
    for (int i = threadIdx.x; i < kCodes; i += 256) {
        cdict[(size_t)s * kCodes + i] = 0;
        if (cval) cval[(size_t)s * kCodes + i] = 0.0;  // code kCodePad: value 0
        sldsc[i] = kEmptyPos;
    }
    __syncthreads();
    const int row0 = s * kSliceRows;
    const size_t e0 = (size_t)slice_base[s] * kSliceRows, e1 = (size_t)slice_base[s + 1] * kSliceRows;
    auto slot_of = [](u64 k) { return (int)(((k ^ (k >> 29)) * 0x9E3779B97F4A7C15ull) >> 54); };  // 10 bits
    auto insert = [&](u64* tab, u64 key) {
        int h = slot_of(key);
        for (int probe = 0; probe < kH; probe++) {
            const u64 old = atomicCAS(&tab[h], kEmpty, key);
            if (old == kEmpty || old == key) return;
            h = (h + 1) & (kH - 1);
        }
    };
    auto find = [&](const u64* tab, u64 key) {
        int h = slot_of(key);
        for (int probe = 0; probe < kH && tab[h] != key; probe++) h = (h + 1) & (kH - 1);
        return tab[h] == key ? h : -1;
    };
    // values (V only)
    if (cval) {
        for (size_t e = e0 + threadIdx.x; e < e1; e += 256) {
            if (cols[e] < 0) continue;
            const u64 vb = (u64)__double_as_longlong(vals[e]);
            if (vb == kEmpty) ok[0] = 0;  // that NaN pattern is the empty marker
            else insert(vkeys, vb);
        }
        __syncthreads();
        for (int h = threadIdx.x; h < kH; h += 256)
            if (vkeys[h] != kEmpty) {
                const int vc = atomicAdd(&vcnt, 1);
                vcode_of[h] = vc;
                if (vc < kCodePad) svals[vc] = __longlong_as_double((long long)vkeys[h]);
            }
        __syncthreads();
        if (vcnt > kCodePad) {
            if (threadIdx.x == 0) ok[0] = 0;
            return;
        }
    }
    auto key_of = [&](size_t e, int d) -> u64 {
        u64 vc = 0;
        if (cval) {
            const int h = find(vkeys, (u64)__double_as_longlong(vals[e]));
            vc = h < 0 ? 0xFFFFull : (u64)vcode_of[h];
        }
        return ((u64)(unsigned)d << 32) | vc;
    };
    for (size_t e = e0 + threadIdx.x; e < e1; e += 256) {
        const int c = cols[e];
        if (c < 0) continue;
        insert(keys, key_of(e, c - (row0 + (int)((e - e0) % kSliceRows))));
    }
    __syncthreads();
    for (int h = threadIdx.x; h < kH; h += 256) {
        if (keys[h] == kEmpty) continue;
        const int code = atomicAdd(&cnt, 1);
        code_of[h] = code;
        if (code < kCodePad) {
            cdict[(size_t)s * kCodes + code] = (int)(unsigned)(keys[h] >> 32);
            if (cval) {
                const unsigned vc = (unsigned)(keys[h] & 0xFFFFFFFFull);
                if (vc < kCodePad) cval[(size_t)s * kCodes + code] = svals[vc];
                else ok[0] = 0;
            }
        }
    }
    __syncthreads();
    if (cnt > kCodePad) {
        if (threadIdx.x == 0) ok[0] = 0;
        return;
    }
    if (threadIdx.x == 0) ccount[s] = cnt;
    const int w0 = win_ptr ? win_ptr[s] : 0, w1 = win_ptr ? win_ptr[s + 1] : 0;
    for (size_t e = e0 + threadIdx.x; e < e1; e += 256) {
        const int c = cols[e];
        if (c < 0) {
            codes[e] = (unsigned char)kCodePad;
            continue;
        }
        const int lane = (int)((e - e0) % kSliceRows);
        const int h = find(keys, key_of(e, c - (row0 + lane)));  // present: <= 255 keys inserted
        if (h < 0) {
            ok[0] = 0;
            continue;
        }
        const int code = code_of[h];
        codes[e] = (unsigned char)code;
        if (ldsc) {
            int w = w0;
            while (w + 1 < w1 && win_start[w + 1] <= c) w++;
            if (w >= w1 || c < win_start[w] || c >= win_start[w] + win_len[w]) {
                ok[1] = 0;
                continue;
            }
            const int pos0 = win_off[w] + (c - win_start[w]) - lane;  // position of lane 0's column
            const int old = atomicCAS(&sldsc[code], kEmptyPos, pos0);
            if (old != kEmptyPos && old != pos0) ok[1] = 0;
        }
    }
    if (ldsc) {
        __syncthreads();
        for (int i = threadIdx.x; i < kCodes; i += 256) ldsc[(size_t)s * kCodes + i] = sldsc[i];
    }
}

// ---------------------------------------------------------------------------
// SELL-512-P: per-row pattern ids over the SELL-512-C codes. Rows of a slice
// whose code sequences (slot 0..w-1) are equal share one pattern; a stencil
// slice has a handful (interior, x/y/z faces, edges). The SpMV streams the
// values (8 B per slot) and one byte per row; the offsets come from a
// per-slice table in LDS. Pass 1 (one block of 512 lanes per slice): hash
// each lane's code sequence, one representative lane per pattern (the lowest),
// ids in representative order, every lane verified against its
// representative. ok[0] = 0 when a slice has more than kMaxPat patterns, a
// table over kPatCap entries, or a hash collision.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kSliceRows) void k_build_p(const unsigned int* __restrict__ slice_base, int nslices,
                                                        const unsigned char* __restrict__ codes,
                                                        unsigned char* __restrict__ prow, int* __restrict__ prep,
                                                        int* __restrict__ pcount, int* ok)
{
    typedef unsigned long long u64;
    constexpr int kH = 1024;
    constexpr u64 kEmpty = ~0ull;
    __shared__ u64 keys[kH];
    __shared__ int rep[kH];
    __shared__ short rid[kSliceRows];  // pattern id of a representative lane, else -1
    __shared__ int cnt;
    const int s = blockIdx.x;
    if (s >= nslices) return;
    for (int h = threadIdx.x; h < kH; h += kSliceRows) {
        keys[h] = kEmpty;
        rep[h] = INT_MAX;
    }
    __syncthreads();
    const int lane = threadIdx.x;
    const size_t e0 = (size_t)slice_base[s] * kSliceRows;
    const int w = (int)(slice_base[s + 1] - slice_base[s]);
    u64 hsh = 0xcbf29ce484222325ull ^ (u64)w;
    for (int j = 0; j < w; j++) {
        hsh = (hsh ^ codes[e0 + (size_t)j * kSliceRows + lane]) * 0x100000001b3ull;
        hsh ^= hsh >> 31;
    }
    if (hsh == kEmpty) hsh = 0;
    int h = (int)((hsh * 0x9E3779B97F4A7C15ull) >> 54);
    for (int probe = 0; probe < kH; probe++) {
        const u64 old = atomicCAS(&keys[h], kEmpty, hsh);
        if (old == kEmpty || old == hsh) break;
        h = (h + 1) & (kH - 1);
    }
    atomicMin(&rep[h], lane);
    __syncthreads();
    rid[lane] = rep[h] == lane ? 1 : -1;
    __syncthreads();
    if (threadIdx.x == 0) {  // ids in lane order of the representatives
        int n = 0;
        for (int l = 0; l < kSliceRows; l++)
            if (rid[l] > 0) {
                if (n < kMaxPat) prep[(size_t)s * kMaxPat + n] = l;
                rid[l] = (short)n++;
            }
        cnt = n;
        pcount[s] = n;
        if (n > kMaxPat || n * w > kPatCap) ok[0] = 0;
    }
    __syncthreads();
    if (cnt > kMaxPat || cnt * w > kPatCap) return;
    const int r = rep[h];
    for (int j = 0; j < w; j++)
        if (codes[e0 + (size_t)j * kSliceRows + lane] != codes[e0 + (size_t)j * kSliceRows + r]) ok[0] = 0;
    prow[(size_t)s * kSliceRows + lane] = (unsigned char)rid[r];
}

// Pass 2: the pattern tables, slice s at pbase[s]: entry (id, j) = the
// offset of slot j of pattern id -- column - row (tab_g, gathering kernels)
// or the LDS position relative to the row's lane (tab_l) -- or kPatPad.
__global__ __launch_bounds__(256) void k_fill_p(const unsigned int* __restrict__ slice_base, int nslices,
                                                const unsigned char* __restrict__ codes,
                                                const int* __restrict__ prep, const int* __restrict__ pcount,
                                                const int* __restrict__ pbase, const int* __restrict__ cdict,
                                                const int* __restrict__ ldsc, int* __restrict__ tab_g,
                                                int* __restrict__ tab_l)
{
    const int s = blockIdx.x;
    if (s >= nslices) return;
    const size_t e0 = (size_t)slice_base[s] * kSliceRows;
    const int w = (int)(slice_base[s + 1] - slice_base[s]);
    const int n = pcount[s] * w;
    for (int i = threadIdx.x; i < n; i += 256) {
        const int id = i / w, j = i % w;
        const unsigned c = codes[e0 + (size_t)j * kSliceRows + prep[(size_t)s * kMaxPat + id]];
        const size_t o = (size_t)pbase[s] + i;
        tab_g[o] = c == kCodePad ? kPatPad : cdict[(size_t)s * kCodes + c];
        if (tab_l) tab_l[o] = c == kCodePad ? kPatPad : ldsc[(size_t)s * kCodes + c];
    }
}

// ---------------------------------------------------------------------------
// SELL-512-A: offset-aligned slots. Slot j of slice s holds, for every row,
// its entry at the slice's j-th smallest (column - row) offset, 0.0 where the
// row has none. A row's entries keep their order (required ascending), and a
// hole adds 0 * x = +-0, which never changes a sum that starts at +0.0: the
// row sums are the reference's bits. Every row of a slice then reads x at the
// same offsets, so a thread's two rows take one 16-byte x load per slot and
// the offsets are per-slice scalars. One block of 512 lanes per slice.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kSliceRows) void k_build_a(const unsigned int* __restrict__ slice_base, int nslices,
                                                        const unsigned char* __restrict__ codes,
                                                        const double* __restrict__ vals,
                                                        const int* __restrict__ cdict, const int* __restrict__ ccount,
                                                        const unsigned int* __restrict__ abase,
                                                        double* __restrict__ aval, int* __restrict__ aoff, int* ok,
                                                        int* maxabs)
{
    __shared__ int soff[kAMax];
    __shared__ int srank[kAMax];
    const int s = blockIdx.x;
    if (s >= nslices) return;
    const int K = ccount[s];
    const int lane = threadIdx.x;
    if (K > kAMax) {
        if (lane == 0) ok[0] = 0;
        return;
    }
    if (lane < K) soff[lane] = cdict[(size_t)s * kCodes + lane];
    __syncthreads();
    if (lane < K) {
        const int o = soff[lane];
        int r = 0;
        for (int c = 0; c < K; c++) r += soff[c] < o ? 1 : 0;
        srank[lane] = r;
        aoff[(size_t)s * kAMax + r] = o;
        atomicMax(maxabs, o < 0 ? -o : o);
    } else if (lane < kAMax) {
        aoff[(size_t)s * kAMax + lane] = 0;
    }
    __syncthreads();
    const size_t e0 = (size_t)slice_base[s] * kSliceRows;
    const int w = (int)(slice_base[s + 1] - slice_base[s]);
    double* out = aval + (size_t)abase[s] * kSliceRows + lane;
    int prev = -1;
    for (int j = 0; j < w; j++) {
        const unsigned c = codes[e0 + (size_t)j * kSliceRows + lane];
        if (c == kCodePad) continue;
        const int r = srank[c];
        if (r <= prev) ok[0] = 0;  // entries out of offset order: no A image
        prev = r;
        out[(size_t)r * kSliceRows] = vals[e0 + (size_t)j * kSliceRows + lane];
    }
}

template <int kRpt, int kW, int kMinW, bool kNT, bool kFuse>
__global__ __launch_bounds__(kSliceRows / kRpt, kMinW) void k_spmv(CgArgs a, bool prologue)
{
    int k = 0;
    double rr = 0.0;  // r_{k-1}.r_{k-1}: the fused p update needs it
    if (!prologue) {
        k = a.kst[0];
        if (kFuse) rr = cur_rr(a);
        const bool run = cg_run(a, k, kFuse, rr);
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            if (kFuse && (k == 1 || run)) a.hist[k - 1] = rr;
            if (run)
                stamp(a, kStampSpmv);
            else
                mark_end(a);
        }
        if (!run) return;
    }
    const int s = spmv_slice(a);
    if (s < 0) return;
    const int row = s * kSliceRows + threadIdx.x * kRpt;
    double* __restrict__ p = cur_p(a, k);
    double sum[kRpt];
    Rows<kRpt> pv;
    if constexpr (kFuse) {
        // beta and p_{k-1} exactly as k_p_update uses them
        const double beta = (k == 1) ? 0.0 : rr / a.hist[k - 2];
        const double* pold = (k == 1) ? a.r : cur_p(a, k - 1);
        const GatherRP gat{a.r, pold, beta};
        spmv_rows<kRpt, kW, kNT>(a, gat, s, sum);
        const Rows<kRpt> rv = ld<kRpt>(a.r + row);
        const Rows<kRpt> yv = ld<kRpt>(pold + row);
#pragma unroll
        for (int i = 0; i < kRpt; i++) pv.v[i] = rv.v[i] + beta * yv.v[i];
        st_rows<kRpt>(p, row, a.n, pv);
    } else {
        const GatherP gat{p - a.ghost_lo};
        spmv_rows<kRpt, kW, kNT>(a, gat, s, sum);
        pv = ld<kRpt>(p + row);
    }
    Rows<kRpt> o;
#pragma unroll
    for (int i = 0; i < kRpt; i++) o.v[i] = sum[i];
    st_rows<kRpt>(a.Ap, row, a.n, o);
    if (prologue) return;  // HPCCG.cpp:351: the prologue SpMV has no p.Ap
    double d = 0.0;
#pragma unroll
    for (int i = 0; i < kRpt; i++)
        if (row + i < a.n) d += pv.v[i] * o.v[i];
    const double bs = block_sum<kSliceRows / kRpt>(d);
    complete_dot<kSliceRows / kRpt>(a, s, bs, kPAP, 0);
}

// ---------------------------------------------------------------------------
// SELL-512-L SpMV: the slice's x windows (host-computed union of the column
// ranges the slice touches; 3 windows of 512 + 2(nx+1) for the stencils) are
// staged into LDS with coalesced loads, then every entry reads x from LDS
// through a 16-bit slice-local index. Same per-row order and products as
// k_spmv, so the same bits; 10 B per stored entry instead of 12.
// ---------------------------------------------------------------------------
template <int kRpt, bool kNT>
__device__ __forceinline__ void ld_lcols(const unsigned short* __restrict__ p, unsigned (&c)[kRpt])
{
    if constexpr (kRpt == 1) {
        c[0] = kNT ? __builtin_nontemporal_load(p) : p[0];
    } else if constexpr (kRpt == 2) {
        const unsigned t = kNT ? __builtin_nontemporal_load(reinterpret_cast<const unsigned*>(p))
                               : *reinterpret_cast<const unsigned*>(p);
        c[0] = t & 0xFFFFu;
        c[1] = t >> 16;
    } else {
#pragma unroll
        for (int i = 0; i < kRpt; i += 4) {
            typedef unsigned u2v __attribute__((ext_vector_type(2)));
            const u2v t = kNT ? __builtin_nontemporal_load(reinterpret_cast<const u2v*>(p + i))
                              : *reinterpret_cast<const u2v*>(p + i);
            c[i] = t.x & 0xFFFFu;
            c[i + 1] = t.x >> 16;
            c[i + 2] = t.y & 0xFFFFu;
            c[i + 3] = t.y >> 16;
        }
    }
}


// Index stream of the LDS kernels: 16-bit LDS positions (SELL-512-L) or 1-byte
// offset codes (SELL-512-C, position = lane + ldsc[code]).
template <bool kCode>
struct LdsIdx {
    using T = typename std::conditional<kCode, unsigned char, unsigned short>::type;
    static constexpr unsigned kPad = kCode ? kCodePad : kLdsPad;
};

template <int kRpt, bool kNT, bool kCode>
__device__ __forceinline__ void ld_idx(const typename LdsIdx<kCode>::T* __restrict__ p, unsigned (&c)[kRpt])
{
    if constexpr (kCode)
        ld_codes<kRpt, kNT>(p, c);
    else
        ld_lcols<kRpt, kNT>(p, c);
}

template <bool kCode>
__device__ __forceinline__ int lds_pos(unsigned c, int lrow, const int* sldsc)
{
    if constexpr (kCode)
        return lrow + sldsc[c];
    else
        return (int)c;
}

// kVal (SELL-512-V): no value stream; the value of code c is sval[c].
template <int kRpt, bool kNT, bool kCode, bool kVal, int kPre, int kP>
__device__ __forceinline__ void lds_prefetch(const double* __restrict__ vp,
                                             const typename LdsIdx<kCode>::T* __restrict__ cp, int wdt,
                                             Rows<kRpt> (&vpre)[kP], unsigned (&cpre)[kP][kRpt])
{
#pragma unroll
    for (int j = 0; j < kPre; j++) {
        if (j < wdt) {
            ld_idx<kRpt, kNT, kCode>(cp + (size_t)j * kSliceRows, cpre[j]);
            if constexpr (!kVal) vpre[j] = ld_m<kRpt, kNT>(vp + (size_t)j * kSliceRows);
        }
    }
}

template <int kRpt, bool kNT, bool kCode, bool kVal>
__device__ __forceinline__ void lds_stream(const double* __restrict__ vp,
                                           const typename LdsIdx<kCode>::T* __restrict__ cp, int j0, int wdt,
                                           const double* xs, const int* sldsc, const double* sval,
                                           double (&sum)[kRpt])
{
    const int lrow = threadIdx.x * kRpt;
#pragma unroll kVal ? 4 : 3
    for (int j = j0; j < wdt; j++) {
        unsigned c[kRpt];
        ld_idx<kRpt, kNT, kCode>(cp + (size_t)j * kSliceRows, c);
        Rows<kRpt> v;
        if constexpr (kVal) {
#pragma unroll
            for (int i = 0; i < kRpt; i++) v.v[i] = sval[c[i]];
        } else {
            v = ld_m<kRpt, kNT>(vp + (size_t)j * kSliceRows);
        }
#pragma unroll
        for (int i = 0; i < kRpt; i++) {
            const double xv = (c[i] != LdsIdx<kCode>::kPad) ? xs[lds_pos<kCode>(c[i], lrow + i, sldsc)] : 0.0;
            sum[i] = sum[i] + v.v[i] * xv;
        }
    }
}

// kPre > 0: the first kPre slots of the matrix stream are loaded before the
// window staging and its barrier, so the block's HBM stream starts at once.
// kFmt: 0 SELL-512-L (16-bit LDS indices + values), 1 SELL-512-C (offset
// codes + values), 2 SELL-512-V (codes of (offset, value) pairs only).
template <int kRpt, bool kNT, bool kFuse, int kPre, int kFmt = 0>
__global__ __launch_bounds__(kSliceRows / kRpt) void k_spmv_lds(CgArgs a, bool prologue)
{
    constexpr bool kCode = kFmt != 0;
    constexpr bool kVal = kFmt == 2;
    extern __shared__ __attribute__((aligned(16))) double xs[];
    __shared__ int sldsc[kCode ? kCodes : 1];
    __shared__ double sval[kVal ? kCodes : 1];
    using IdxT = typename LdsIdx<kCode>::T;
    int k = 0;
    double rr = 0.0;  // r_{k-1}.r_{k-1}: the fused p update needs it
    if (!prologue) {
        k = a.kst[0];
        if (kFuse) rr = cur_rr(a);
        const bool run = cg_run(a, k, kFuse, rr);
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            if (kFuse && (k == 1 || run)) a.hist[k - 1] = rr;
            if (run)
                stamp(a, kStampSpmv);
            else
                mark_end(a);
        }
        if (!run) return;
    }
    const int s = spmv_slice(a);
    if (s < 0) return;
    double* __restrict__ p = cur_p(a, k);
    const double* __restrict__ xext = p - a.ghost_lo;
    const size_t base = (size_t)a.slice_base[s] * kSliceRows + (size_t)threadIdx.x * kRpt;
    const int wdt = (int)(a.slice_base[s + 1] - a.slice_base[s]);
    const double* __restrict__ vp = a.vals + base;
    const IdxT* __restrict__ cp = (kCode ? (const IdxT*)(const void*)a.ccodes : (const IdxT*)(const void*)a.lcols) + base;
    constexpr int kP = kPre > 0 ? kPre : 1;
    unsigned cpre[kP][kRpt];
    Rows<kRpt> vpre[kP];
    // the first nt_split slices of every XCD's eighth stream with the default
    // policy (they may stay resident in the Infinity Cache between iterations,
    // spread evenly over the XCDs), the rest non-temporal
    const bool nt = kNT && (xcd_slice(a.sgrid) % (a.sgrid / kNumXcd)) >= a.nt_split;
    if (nt)
        lds_prefetch<kRpt, true, kCode, kVal, kPre>(vp, cp, wdt, vpre, cpre);
    else
        lds_prefetch<kRpt, false, kCode, kVal, kPre>(vp, cp, wdt, vpre, cpre);
    if constexpr (kCode)
    {
        // C: the whole dictionary (no dependent count load ahead of the staging);
        // V: the codes in use, kCodePad has value 0
        const int nc = kVal ? a.ccount[s] : kCodes;
        for (int i = threadIdx.x; i < nc; i += kSliceRows / kRpt) {
            sldsc[i] = a.ldsc[(size_t)s * kCodes + i];
            if constexpr (kVal) sval[i] = a.cval[(size_t)s * kCodes + i];
        }
        if (kVal && threadIdx.x == 0) sval[kCodePad] = 0.0;
    }
    // stage the windows; with kFuse the staged value of an own row is
    // p_k = r + beta*p_{k-1}, the exact expression k_p_update stores
    double beta = 0.0;
    const double* __restrict__ pold = a.r;
    if constexpr (kFuse) {
        beta = (k == 1) ? 0.0 : rr / a.hist[k - 2];
        pold = (k == 1) ? a.r : cur_p(a, k - 1);
    }
    const int w0 = a.win_ptr[s], w1 = a.win_ptr[s + 1];
    for (int w = w0; w < w1; w++) {
        const int st0 = a.win_start[w], len = a.win_len[w], off = a.win_off[w];
        for (int i = threadIdx.x; i < len; i += kSliceRows / kRpt) {
            if constexpr (kFuse) {
                // own rows: p_k computed here; ghost planes: p_k from the halo
                const int l = st0 + i - a.ghost_lo;
                xs[off + i] = ((unsigned)l < (unsigned)a.n) ? a.r[l] + beta * pold[l] : xext[st0 + i];
            } else {
                xs[off + i] = xext[st0 + i];
            }
        }
    }
    __syncthreads();
    double sum[kRpt];
#pragma unroll
    for (int i = 0; i < kRpt; i++) sum[i] = 0.0;
#pragma unroll
    for (int j = 0; j < kPre; j++) {
        if (j < wdt) {
#pragma unroll
            for (int i = 0; i < kRpt; i++) {
                const double xv = (cpre[j][i] != LdsIdx<kCode>::kPad)
                                      ? xs[lds_pos<kCode>(cpre[j][i], threadIdx.x * kRpt + i, sldsc)]
                                      : 0.0;
                const double v = kVal ? sval[cpre[j][i]] : vpre[j].v[i];
                sum[i] = sum[i] + v * xv;
            }
        }
    }
    if (nt)
        lds_stream<kRpt, true, kCode, kVal>(vp, cp, kPre, wdt, xs, sldsc, sval, sum);
    else
        lds_stream<kRpt, false, kCode, kVal>(vp, cp, kPre, wdt, xs, sldsc, sval, sum);
    const int row = s * kSliceRows + threadIdx.x * kRpt;
    Rows<kRpt> o;
#pragma unroll
    for (int i = 0; i < kRpt; i++) o.v[i] = sum[i];
    st_rows<kRpt>(a.Ap, row, a.n, o);
    if (prologue) return;
    Rows<kRpt> pv;
    if constexpr (kFuse) {
        const Rows<kRpt> rv = ld<kRpt>(a.r + row);
        const Rows<kRpt> yv = ld<kRpt>(pold + row);
#pragma unroll
        for (int i = 0; i < kRpt; i++) pv.v[i] = rv.v[i] + beta * yv.v[i];
        st_rows<kRpt>(p, row, a.n, pv);
    } else {
        pv = ld<kRpt>(p + row);
    }
    double d = 0.0;
#pragma unroll
    for (int i = 0; i < kRpt; i++)
        if (row + i < a.n) d += pv.v[i] * o.v[i];
    const double bs = block_sum<kSliceRows / kRpt>(d);
    complete_dot<kSliceRows / kRpt>(a, s, bs, kPAP, 0);
}

// ---------------------------------------------------------------------------
// SELL-512-P SpMV kernels: values streamed as in SELL-512 (8 B per slot), one
// pattern-id byte per row, the slice's pattern table (kPatCap ints) in LDS.
// k_spmv_lp reads x from the staged windows (the SELL-512-L staging, p update
// fused as in k_spmv_lds); k_spmv_pp gathers x from global memory. Same
// products in the same slot order as SELL-512, same p.Ap tree per kRpt.
// ---------------------------------------------------------------------------
template <int kRpt>
__device__ __forceinline__ void ld_pids(const unsigned char* __restrict__ p, int (&pid)[kRpt])
{
    if constexpr (kRpt == 1) {
        pid[0] = p[0];
    } else {
        static_assert(kRpt == 2, "1 or 2 rows per thread");
        const unsigned t = *reinterpret_cast<const unsigned short*>(p);
        pid[0] = t & 0xFFu;
        pid[1] = t >> 8;
    }
}

template <int kRpt, bool kNT, int kU>
__device__ __forceinline__ void lp_stream(const double* __restrict__ vp, int j0, int wdt, const int (&pr)[kRpt],
                                          const double* xs, const int* spat, double (&sum)[kRpt])
{
    const int lrow = threadIdx.x * kRpt;
#pragma unroll kU
    for (int j = j0; j < wdt; j++) {
        const Rows<kRpt> v = ld_m<kRpt, kNT>(vp + (size_t)j * kSliceRows);
#pragma unroll
        for (int i = 0; i < kRpt; i++) {
            const int c = spat[pr[i] + j];
            const double xv = c != kPatPad ? xs[lrow + i + c] : 0.0;
            sum[i] = sum[i] + v.v[i] * xv;
        }
    }
}

// Dynamic LDS: the windows (a.lds_doubles doubles), then the pattern table
// (a.pat_max ints, the largest over slices).
// kEarly: the slice's pattern ids and first kPre value slots (they depend
// only on blockIdx) are loaded before the iteration test.
template <int kRpt, bool kNT, bool kFuse, int kPre, int kU = 3, bool kEarly = false>
__global__ __launch_bounds__(kSliceRows / kRpt) void k_spmv_lp(CgArgs a, bool prologue)
{
    extern __shared__ __attribute__((aligned(16))) double xs[];
    int* const spat = reinterpret_cast<int*>(xs + a.lds_doubles);
    constexpr int kP = kPre > 0 ? kPre : 1;
    Rows<kRpt> vpre[kP];
    int pid[kRpt];
    const int s = spmv_slice(a);
    const size_t base = s >= 0 ? (size_t)a.slice_base[s] * kSliceRows + (size_t)threadIdx.x * kRpt : 0;
    const int wdt = s >= 0 ? (int)(a.slice_base[s + 1] - a.slice_base[s]) : 0;
    const double* __restrict__ vp = a.vals + base;
    const bool nt = kNT && (xcd_slice(a.sgrid) % (a.sgrid / kNumXcd)) >= a.nt_split;
    auto load_early = [&]() {
        ld_pids<kRpt>(a.prow + (size_t)s * kSliceRows + threadIdx.x * kRpt, pid);
#pragma unroll
        for (int j = 0; j < kPre; j++)
            if (j < wdt)
                vpre[j] = nt ? ld_m<kRpt, true>(vp + (size_t)j * kSliceRows) : ld_m<kRpt, false>(vp + (size_t)j * kSliceRows);
    };
    if (kEarly && s >= 0) load_early();
    int k = 0;
    double rr = 0.0;  // r_{k-1}.r_{k-1}: the fused p update needs it
    if (!prologue) {
        k = a.kst[0];
        if (kFuse) rr = cur_rr(a);
        const bool run = cg_run(a, k, kFuse, rr);
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            if (kFuse && (k == 1 || run)) a.hist[k - 1] = rr;
            if (run)
                stamp(a, kStampSpmv);
            else
                mark_end(a);
        }
        if (!run) return;
    }
    if (s < 0) return;
    double* __restrict__ p = cur_p(a, k);
    const double* __restrict__ xext = p - a.ghost_lo;
    if (!kEarly) load_early();
    {
        const int np = a.pcount[s] * wdt;
        const int* __restrict__ tab = a.ptab_l + a.pbase[s];
        for (int i = threadIdx.x; i < np; i += kSliceRows / kRpt) spat[i] = tab[i];
    }
    double beta = 0.0;
    const double* __restrict__ pold = a.r;
    if constexpr (kFuse) {
        beta = (k == 1) ? 0.0 : rr / a.hist[k - 2];
        pold = (k == 1) ? a.r : cur_p(a, k - 1);
    }
    const int w0 = a.win_ptr[s], w1 = a.win_ptr[s + 1];
    for (int w = w0; w < w1; w++) {
        const int st0 = a.win_start[w], len = a.win_len[w], off = a.win_off[w];
        for (int i = threadIdx.x; i < len; i += kSliceRows / kRpt) {
            if constexpr (kFuse) {
                const int l = st0 + i - a.ghost_lo;
                xs[off + i] = ((unsigned)l < (unsigned)a.n) ? a.r[l] + beta * pold[l] : xext[st0 + i];
            } else {
                xs[off + i] = xext[st0 + i];
            }
        }
    }
    __syncthreads();
    int pr[kRpt];
#pragma unroll
    for (int i = 0; i < kRpt; i++) pr[i] = pid[i] * wdt;
    double sum[kRpt];
#pragma unroll
    for (int i = 0; i < kRpt; i++) sum[i] = 0.0;
    const int lrow = threadIdx.x * kRpt;
#pragma unroll
    for (int j = 0; j < kPre; j++) {
        if (j < wdt) {
#pragma unroll
            for (int i = 0; i < kRpt; i++) {
                const int c = spat[pr[i] + j];
                const double xv = c != kPatPad ? xs[lrow + i + c] : 0.0;
                sum[i] = sum[i] + vpre[j].v[i] * xv;
            }
        }
    }
    if (nt)
        lp_stream<kRpt, true, kU>(vp, kPre, wdt, pr, xs, spat, sum);
    else
        lp_stream<kRpt, false, kU>(vp, kPre, wdt, pr, xs, spat, sum);
    const int row = s * kSliceRows + threadIdx.x * kRpt;
    Rows<kRpt> o;
#pragma unroll
    for (int i = 0; i < kRpt; i++) o.v[i] = sum[i];
    st_rows<kRpt>(a.Ap, row, a.n, o);
    if (prologue) return;
    Rows<kRpt> pv;
    if constexpr (kFuse) {
        const Rows<kRpt> rv = ld<kRpt>(a.r + row);
        const Rows<kRpt> yv = ld<kRpt>(pold + row);
#pragma unroll
        for (int i = 0; i < kRpt; i++) pv.v[i] = rv.v[i] + beta * yv.v[i];
        st_rows<kRpt>(p, row, a.n, pv);
    } else {
        pv = ld<kRpt>(p + row);
    }
    double d = 0.0;
#pragma unroll
    for (int i = 0; i < kRpt; i++)
        if (row + i < a.n) d += pv.v[i] * o.v[i];
    const double bs = block_sum<kSliceRows / kRpt>(d);
    complete_dot<kSliceRows / kRpt>(a, s, bs, kPAP, 0);
}

// Dynamic LDS: the pattern table (a.pat_max ints). kW > 0: uniform width,
// slot loop fully unrolled.
template <int kRpt, bool kNT, bool kFuse, int kW = 0>
__global__ __launch_bounds__(kSliceRows / kRpt) void k_spmv_pp(CgArgs a, bool prologue)
{
    extern __shared__ int spat[];
    int k = 0;
    double rr = 0.0;
    if (!prologue) {
        k = a.kst[0];
        if (kFuse) rr = cur_rr(a);
        const bool run = cg_run(a, k, kFuse, rr);
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            if (kFuse && (k == 1 || run)) a.hist[k - 1] = rr;
            if (run)
                stamp(a, kStampSpmv);
            else
                mark_end(a);
        }
        if (!run) return;
    }
    const int s = spmv_slice(a);
    if (s < 0) return;
    const int wdt = kW > 0 ? kW : (int)(a.slice_base[s + 1] - a.slice_base[s]);
    int pid[kRpt];
    ld_pids<kRpt>(a.prow + (size_t)s * kSliceRows + threadIdx.x * kRpt, pid);
    {
        const int np = a.pcount[s] * wdt;
        const int* __restrict__ tab = a.ptab_g + a.pbase[s];
        for (int i = threadIdx.x; i < np; i += kSliceRows / kRpt) spat[i] = tab[i];
    }
    __syncthreads();
    const int row = s * kSliceRows + threadIdx.x * kRpt;
    double* __restrict__ p = cur_p(a, k);
    const size_t base = (size_t)a.slice_base[s] * kSliceRows + (size_t)threadIdx.x * kRpt;
    const double* __restrict__ vp = a.vals + base;
    double beta = 0.0;
    const double* pold = a.r;
    if constexpr (kFuse) {
        beta = (k == 1) ? 0.0 : rr / a.hist[k - 2];
        pold = (k == 1) ? a.r : cur_p(a, k - 1);
    }
    const double* __restrict__ xext = p - a.ghost_lo;
    int pr[kRpt];
#pragma unroll
    for (int i = 0; i < kRpt; i++) pr[i] = pid[i] * wdt;
    double sum[kRpt];
#pragma unroll
    for (int i = 0; i < kRpt; i++) sum[i] = 0.0;
#pragma unroll kW > 0 ? kW : 3
    for (int j = 0; j < wdt; j++) {
        const Rows<kRpt> v = ld_m<kRpt, kNT>(vp + (size_t)j * kSliceRows);
#pragma unroll
        for (int i = 0; i < kRpt; i++) {
            const int off = spat[pr[i] + j];
            double xv = 0.0;
            if (off != kPatPad) {
                const int col = row + i + off;
                if constexpr (kFuse) xv = a.r[col - a.ghost_lo] + beta * pold[col - a.ghost_lo];
                else xv = xext[col];
            }
            sum[i] = sum[i] + v.v[i] * xv;
        }
    }
    Rows<kRpt> pv;
    if constexpr (kFuse) {
        const Rows<kRpt> rv = ld<kRpt>(a.r + row);
        const Rows<kRpt> yv = ld<kRpt>(pold + row);
#pragma unroll
        for (int i = 0; i < kRpt; i++) pv.v[i] = rv.v[i] + beta * yv.v[i];
        st_rows<kRpt>(p, row, a.n, pv);
    } else {
        pv = ld<kRpt>(p + row);
    }
    Rows<kRpt> o;
#pragma unroll
    for (int i = 0; i < kRpt; i++) o.v[i] = sum[i];
    st_rows<kRpt>(a.Ap, row, a.n, o);
    if (prologue) return;
    double d = 0.0;
#pragma unroll
    for (int i = 0; i < kRpt; i++)
        if (row + i < a.n) d += pv.v[i] * o.v[i];
    const double bs = block_sum<kSliceRows / kRpt>(d);
    complete_dot<kSliceRows / kRpt>(a, s, bs, kPAP, 0);
}

// kRpt consecutive doubles from an 8-byte aligned address: one 16-byte load
// for two rows (global loads need only dword alignment on gfx950).
template <int kRpt>
__device__ __forceinline__ Rows<kRpt> ld_rows_u(const double* __restrict__ p)
{
    Rows<kRpt> o;
    if constexpr (kRpt == 2) {
        typedef double d2u __attribute__((ext_vector_type(2), aligned(8)));
        const d2u t = *reinterpret_cast<const d2u*>(p);
        o.v[0] = t.x;
        o.v[1] = t.y;
    } else {
#pragma unroll
        for (int i = 0; i < kRpt; i++) o.v[i] = p[i];
    }
    return o;
}

// SELL-512-A SpMV: per slot one value load and one x load per thread at the
// slice's offset for that slot. Holes read x inside the zeroed guard zones of
// the p buffers (and of r) or at a real neighbour; their value is 0.0.
// kW > 0: uniform width, slot loop fully unrolled. kFuse (single rank, never
// the prologue): x = r + beta*p_{k-1} formed per load, k_p_update's exact
// expression, so every row sum is unchanged; the thread's own rows of p_k
// are stored for the update kernel and the next iteration.
template <int kRpt, bool kNT, int kW = 0, bool kFuse = false, int kPre = 0>
__global__ __launch_bounds__(kSliceRows / kRpt) void k_spmv_pa(CgArgs a, bool prologue)
{
    static_assert(kPre == 0 || (kW > 0 && kPre <= kW), "early loads need the uniform width");
    // kPre > 0: the slice, its first kPre value slots and its offsets depend
    // only on blockIdx, so they are loaded before the iteration count and
    // r.r (two dependent scalar loads) decide whether the block runs
    const int s = spmv_slice(a);
    constexpr int kP = kPre > 0 ? kPre : 1;
    Rows<kRpt> vpre[kP];
    int offp[kPre > 0 ? kW : 1];
    if constexpr (kPre > 0) {
        if (s >= 0) {
            const double* __restrict__ vp0 = a.aval + (size_t)s * kW * kSliceRows + (size_t)threadIdx.x * kRpt;
#pragma unroll
            for (int j = 0; j < kPre; j++) vpre[j] = ld_m<kRpt, kNT>(vp0 + (size_t)j * kSliceRows);
#pragma unroll
            for (int j = 0; j < kW; j++) offp[j] = a.aoff[(size_t)s * kAMax + j];
        }
    }
    int k = 0;
    double rr = 0.0;  // r_{k-1}.r_{k-1}: the fused p update needs it
    if (!prologue) {
        k = a.kst[0];
        if (kFuse) rr = cur_rr(a);
        const bool run = cg_run(a, k, kFuse, rr);
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            if (kFuse && (k == 1 || run)) a.hist[k - 1] = rr;
            if (run)
                stamp(a, kStampSpmv);
            else
                mark_end(a);
        }
        if (!run) return;
    }
    if (s < 0) return;
    const int wdt = kW > 0 ? kW : (int)(a.abase[s + 1] - a.abase[s]);
    const int row = s * kSliceRows + threadIdx.x * kRpt;
    double* __restrict__ p = cur_p(a, k);
    const double* __restrict__ xr = p - a.ghost_lo + row;  // x of column row + off at xr[off]
    double beta = 0.0;
    const double* __restrict__ rr_ = a.r - a.ghost_lo + row;
    const double* __restrict__ py = rr_;
    if constexpr (kFuse) {
        beta = (k == 1) ? 0.0 : rr / a.hist[k - 2];
        py = ((k == 1) ? a.r : cur_p(a, k - 1)) - a.ghost_lo + row;
    }
    // uniform width: slice s starts at slot row s * kW
    const size_t vb = kW > 0 ? (size_t)s * kW : (size_t)a.abase[s];
    const double* __restrict__ vp = a.aval + vb * kSliceRows + (size_t)threadIdx.x * kRpt;
    const int* __restrict__ off = a.aoff + (size_t)s * kAMax;
    double sum[kRpt];
#pragma unroll
    for (int i = 0; i < kRpt; i++) sum[i] = 0.0;
#pragma unroll kW > 0 ? kW : 4
    for (int j = 0; j < wdt; j++) {
        Rows<kRpt> v;
        int oj;
        if constexpr (kPre > 0) {
            v = j < kPre ? vpre[j] : ld_m<kRpt, kNT>(vp + (size_t)j * kSliceRows);
            oj = offp[j];
        } else {
            v = ld_m<kRpt, kNT>(vp + (size_t)j * kSliceRows);
            oj = off[j];
        }
        Rows<kRpt> xv;
        if constexpr (kFuse) {
            const Rows<kRpt> rv = ld_rows_u<kRpt>(rr_ + oj);
            const Rows<kRpt> yv = ld_rows_u<kRpt>(py + oj);
#pragma unroll
            for (int i = 0; i < kRpt; i++) xv.v[i] = rv.v[i] + beta * yv.v[i];
        } else {
            xv = ld_rows_u<kRpt>(xr + oj);
        }
#pragma unroll
        for (int i = 0; i < kRpt; i++) sum[i] = sum[i] + v.v[i] * xv.v[i];
    }
    Rows<kRpt> o;
#pragma unroll
    for (int i = 0; i < kRpt; i++) o.v[i] = sum[i];
    st_rows<kRpt>(a.Ap, row, a.n, o);
    if (prologue) return;
    Rows<kRpt> pv;
    if constexpr (kFuse) {
        const Rows<kRpt> rv = ld<kRpt>(rr_ + a.ghost_lo);
        const Rows<kRpt> yv = ld<kRpt>(py + a.ghost_lo);
#pragma unroll
        for (int i = 0; i < kRpt; i++) pv.v[i] = rv.v[i] + beta * yv.v[i];
        st_rows<kRpt>(p, row, a.n, pv);
    } else {
        pv = ld<kRpt>(p + row);
    }
    double d = 0.0;
#pragma unroll
    for (int i = 0; i < kRpt; i++)
        if (row + i < a.n) d += pv.v[i] * o.v[i];
    const double bs = block_sum<kSliceRows / kRpt>(d);
    complete_dot<kSliceRows / kRpt>(a, s, bs, kPAP, 0);
}

// SELL-512-A with x from LDS windows: the windows of the slice (one per
// z-plane for the 27-pt stencil, holes included) are staged first, with
// kFuse p_k = r + beta*p_{k-1} computed per staged own row (k_p_update's
// exact expression; ghost rows come from the halo as in k_spmv_lp). Slot j
// then reads xs[lane row + alds[j]]: one per-slice scalar per slot, no index
// or pattern stream, no table lookup. kPre value slots are loaded before the
// staging barrier. kW > 0: uniform width, slot loop fully unrolled.
template <int kRpt, bool kNT, bool kFuse, int kPre, int kW = 0>
__global__ __launch_bounds__(kSliceRows / kRpt) void k_spmv_la(CgArgs a, bool prologue)
{
    extern __shared__ __attribute__((aligned(16))) double xs[];
    int k = 0;
    double rr = 0.0;  // r_{k-1}.r_{k-1}: the fused p update needs it
    if (!prologue) {
        k = a.kst[0];
        if (kFuse) rr = cur_rr(a);
        const bool run = cg_run(a, k, kFuse, rr);
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            if (kFuse && (k == 1 || run)) a.hist[k - 1] = rr;
            if (run)
                stamp(a, kStampSpmv);
            else
                mark_end(a);
        }
        if (!run) return;
    }
    const int s = spmv_slice(a);
    if (s < 0) return;
    double* __restrict__ p = cur_p(a, k);
    const int wdt = kW > 0 ? kW : (int)(a.abase[s + 1] - a.abase[s]);
    const double* __restrict__ vp = a.aval + (size_t)a.abase[s] * kSliceRows + (size_t)threadIdx.x * kRpt;
    const bool nt = kNT && (xcd_slice(a.sgrid) % (a.sgrid / kNumXcd)) >= a.nt_split;
    constexpr int kP = kPre > 0 ? kPre : 1;
    Rows<kRpt> vpre[kP];
#pragma unroll
    for (int j = 0; j < kPre; j++)
        if (j < wdt)
            vpre[j] = nt ? ld_m<kRpt, true>(vp + (size_t)j * kSliceRows) : ld_m<kRpt, false>(vp + (size_t)j * kSliceRows);
    double beta = 0.0;
    const double* __restrict__ pold = a.r;
    if constexpr (kFuse) {
        beta = (k == 1) ? 0.0 : rr / a.hist[k - 2];
        pold = (k == 1) ? a.r : cur_p(a, k - 1);
    }
    const int srow = s * kSliceRows;
    {
        const int nw = a.awn[s];
        const int* __restrict__ win = a.awin + (size_t)s * kAWin * 3;
        for (int w = 0; w < nw; w++) {
            // offsets are in the [ghost_lo | n | ghost_hi] column numbering
            const int st0 = srow + win[3 * w] - a.ghost_lo, len = win[3 * w + 1], base = win[3 * w + 2];
            for (int i = threadIdx.x; i < len; i += kSliceRows / kRpt) {
                const int l = st0 + i;  // local row (< 0 / >= n: ghosts, guard or padding zeros)
                if constexpr (kFuse)
                    xs[base + i] = ((unsigned)l < (unsigned)a.n) ? a.r[l] + beta * pold[l] : p[l];
                else
                    xs[base + i] = p[l];
            }
        }
    }
    __syncthreads();
    const int* __restrict__ cl = a.alds + (size_t)s * kAMax;
    const int lrow = threadIdx.x * kRpt;
    double sum[kRpt];
#pragma unroll
    for (int i = 0; i < kRpt; i++) sum[i] = 0.0;
#pragma unroll
    for (int j = 0; j < kPre; j++) {
        if (j < wdt) {
            const int c = lrow + cl[j];
#pragma unroll
            for (int i = 0; i < kRpt; i++) sum[i] = sum[i] + vpre[j].v[i] * xs[c + i];
        }
    }
    if (nt) {
#pragma unroll kW > 0 ? kW : 6
        for (int j = kPre; j < wdt; j++) {
            const Rows<kRpt> v = ld_m<kRpt, true>(vp + (size_t)j * kSliceRows);
            const int c = lrow + cl[j];
#pragma unroll
            for (int i = 0; i < kRpt; i++) sum[i] = sum[i] + v.v[i] * xs[c + i];
        }
    } else {
#pragma unroll kW > 0 ? kW : 6
        for (int j = kPre; j < wdt; j++) {
            const Rows<kRpt> v = ld_m<kRpt, false>(vp + (size_t)j * kSliceRows);
            const int c = lrow + cl[j];
#pragma unroll
            for (int i = 0; i < kRpt; i++) sum[i] = sum[i] + v.v[i] * xs[c + i];
        }
    }
    const int row = srow + lrow;
    Rows<kRpt> o;
#pragma unroll
    for (int i = 0; i < kRpt; i++) o.v[i] = sum[i];
    st_rows<kRpt>(a.Ap, row, a.n, o);
    if (prologue) return;
    Rows<kRpt> pv;
    if constexpr (kFuse) {
        const Rows<kRpt> rv = ld<kRpt>(a.r + row);
        const Rows<kRpt> yv = ld<kRpt>(pold + row);
#pragma unroll
        for (int i = 0; i < kRpt; i++) pv.v[i] = rv.v[i] + beta * yv.v[i];
        st_rows<kRpt>(p, row, a.n, pv);
    } else {
        pv = ld<kRpt>(p + row);
    }
    double d = 0.0;
#pragma unroll
    for (int i = 0; i < kRpt; i++)
        if (row + i < a.n) d += pv.v[i] * o.v[i];
    const double bs = block_sum<kSliceRows / kRpt>(d);
    complete_dot<kSliceRows / kRpt>(a, s, bs, kPAP, 0);
}

// SELL-512-A LDS windows over slice pairs (single rank): block P owns slices
// 2P and 2P + 1 with 512 threads (waves 0-3 slice 2P, 4-7 slice 2P + 1, two
// rows per thread as everywhere). The pair's windows cover both slices, so a
// stencil plane is staged once for 1024 rows (27-pt 200^3: 4.2 instead of 5.4
// doubles per row) and the p.Ap hand-off takes one ticket per two slices.
// Each half forms its slice's partial with block_sum<256>'s shape (wave sums,
// then the 4 in order), so the dot is bitwise the one-slice kernels'.
template <bool kNT, bool kFuse, int kPre, int kMinW = 1, int kS = 2, int kSU = 1>
__global__ __launch_bounds__(kS * kSliceRows / 2, kMinW) void k_spmv_la2(CgArgs a, bool prologue)
{
    static_assert(kS == 2 || kS == 4, "slices per block");
    constexpr int kRpt = 2;
    constexpr int kHalf = kSliceRows / kRpt;  // threads per slice
    constexpr int kThr = kS * kHalf;
    extern __shared__ __attribute__((aligned(16))) double xs[];
    __shared__ double wsum[kThr / kWave];
    const int* __restrict__ g_lds = kS == 2 ? a.alds2 : a.alds4;
    const int* __restrict__ g_win = kS == 2 ? a.awin2 : a.awin4;
    const int* __restrict__ g_wn = kS == 2 ? a.awn2 : a.awn4;
    int P = xcd_slice(kS == 2 ? a.pgrid : a.qgrid);  // group: all, or the interior / halo runs
    P = P < a.gn0 ? a.gs0 + P : (P < a.gn0 + a.gn1 ? a.gs1 + (P - a.gn0) : -1);
    const int half = threadIdx.x / kHalf;  // slice of the group
    const int s = P < 0 ? a.nslices : kS * P + half;
    const bool have = s < a.nslices;
    const int lrow = (threadIdx.x % kHalf) * kRpt;  // row within the slice
    const int wdt = have ? (int)(a.abase[s + 1] - a.abase[s]) : 0;
    const double* __restrict__ vp = a.aval + (have ? (size_t)a.abase[s] * kSliceRows : 0) + lrow;
    constexpr int kP = kPre > 0 ? kPre : 1;
    Rows<kRpt> vpre[kP];
#pragma unroll
    for (int j = 0; j < kPre; j++)
        if (j < wdt) vpre[j] = ld_m<kRpt, kNT>(vp + (size_t)j * kSliceRows);
    int k = 0;
    double rr = 0.0;  // r_{k-1}.r_{k-1}: the fused p update needs it
    if (!prologue) {
        k = a.kst[0];
        if (kFuse) rr = cur_rr(a);
        const bool run = cg_run(a, k, kFuse, rr);
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            if (kFuse && (k == 1 || run)) a.hist[k - 1] = rr;
            if (run)
                stamp(a, kStampSpmv);
            else
                mark_end(a);
        }
        if (!run) return;
    }
    if (P < 0 || kS * P >= a.nslices) return;
    double* __restrict__ p = cur_p(a, k);
    double beta = 0.0;
    const double* __restrict__ pold = a.r;
    if constexpr (kFuse) {
        beta = (k == 1) ? 0.0 : rr / a.hist[k - 2];
        pold = (k == 1) ? a.r : cur_p(a, k - 1);
    }
    const int prow0 = kS * P * kSliceRows;  // first row of the group
    {
        const int nw = g_wn[P];
        const int* __restrict__ win = g_win + (size_t)P * kAWin * 3;
        for (int w = 0; w < nw; w++) {
            const int st0 = prow0 + win[3 * w] - a.ghost_lo, len = win[3 * w + 1], base = win[3 * w + 2];
            int i = threadIdx.x;
            if constexpr (kSU > 1) {
                // kSU positions per thread with every load issued before the stores
                for (; i + (kSU - 1) * kThr < len; i += kSU * kThr) {
                    double v[kSU];
#pragma unroll
                    for (int u = 0; u < kSU; u++) {
                        const int l = st0 + i + u * kThr;
                        if constexpr (kFuse)
                            v[u] = ((unsigned)l < (unsigned)a.n) ? a.r[l] + beta * pold[l] : p[l];
                        else
                            v[u] = p[l];
                    }
#pragma unroll
                    for (int u = 0; u < kSU; u++) xs[base + i + u * kThr] = v[u];
                }
            }
            for (; i < len; i += kThr) {
                const int l = st0 + i;  // local row (< 0 / >= n: guard or padding zeros)
                if constexpr (kFuse)
                    xs[base + i] = ((unsigned)l < (unsigned)a.n) ? a.r[l] + beta * pold[l] : p[l];
                else
                    xs[base + i] = p[l];
            }
        }
    }
    __syncthreads();
    double sum[kRpt];
#pragma unroll
    for (int i = 0; i < kRpt; i++) sum[i] = 0.0;
    const int row = s * kSliceRows + lrow;
    double d = 0.0;
    if (have) {
        const int* __restrict__ cl = g_lds + (size_t)s * kAMax;
        const int prow = half * kSliceRows + lrow;  // row within the pair
#pragma unroll
        for (int j = 0; j < kPre; j++) {
            if (j < wdt) {
                const int c = prow + cl[j];
#pragma unroll
                for (int i = 0; i < kRpt; i++) sum[i] = sum[i] + vpre[j].v[i] * xs[c + i];
            }
        }
#pragma unroll 6
        for (int j = kPre; j < wdt; j++) {
            const Rows<kRpt> v = ld_m<kRpt, kNT>(vp + (size_t)j * kSliceRows);
            const int c = prow + cl[j];
#pragma unroll
            for (int i = 0; i < kRpt; i++) sum[i] = sum[i] + v.v[i] * xs[c + i];
        }
        Rows<kRpt> o;
#pragma unroll
        for (int i = 0; i < kRpt; i++) o.v[i] = sum[i];
        st_rows<kRpt>(a.Ap, row, a.n, o);
        if (!prologue) {
            Rows<kRpt> pv;
            if constexpr (kFuse) {
                const Rows<kRpt> rv = ld<kRpt>(a.r + row);
                const Rows<kRpt> yv = ld<kRpt>(pold + row);
#pragma unroll
                for (int i = 0; i < kRpt; i++) pv.v[i] = rv.v[i] + beta * yv.v[i];
                st_rows<kRpt>(p, row, a.n, pv);
            } else {
                pv = ld<kRpt>(p + row);
            }
#pragma unroll
            for (int i = 0; i < kRpt; i++)
                if (row + i < a.n) d += pv.v[i] * o.v[i];
        }
    }
    if (prologue) return;
    // per-slice partials with block_sum<256>'s shape
    const double wv = wave_sum(d);
    const int lane = threadIdx.x & (kWave - 1);
    if (lane == 0) wsum[threadIdx.x / kWave] = wv;
    __syncthreads();
    if (threadIdx.x >= kWave) return;
    constexpr int kWh = kHalf / kWave;
    double bs = 0.0;
    if (lane < kS) {
#pragma unroll
        for (int i = 0; i < kWh; i++) bs += wsum[lane * kWh + i];
    }
    complete_dot_lanes(a, kS * P, min(kS, a.nslices - kS * P), bs, kPAP, 0);
}

// Plain SpMV on arbitrary x (kernel-level C ABI): same body, no dot.
template <int kRpt>
__global__ __launch_bounds__(kSliceRows / kRpt) void k_spmv_plain(CgArgs a, const double* xext,
                                                                  double* y)
{
    const int s = xcd_slice(a.grid);
    if (s >= a.nslices) return;
    double sum[kRpt];
    spmv_rows<kRpt, 0, true>(a, GatherP{xext}, s, sum);
    const int row = s * kSliceRows + threadIdx.x * kRpt;
    for (int i = 0; i < kRpt; i++)
        if (row + i < a.n) y[row + i] = sum[i];
}

// Diagnostic only (never in the CG path): streams the SELL image like the
// SpMV but without the x gather -- the matrix-streaming ceiling.
template <int kW>
__global__ __launch_bounds__(256) void k_stream_diag(CgArgs a)
{
    const int s = xcd_slice(a.grid);
    if (s >= a.nslices) return;
    const size_t base = (size_t)s * kW * kSliceRows + (size_t)threadIdx.x * 2;
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int j = 0; j < kW; j++) {
        int c[2];
        ld_cols<2>(a.cols + base + (size_t)j * kSliceRows, c);
        const Rows<2> v = ld<2>(a.vals + base + (size_t)j * kSliceRows);
        s0 = s0 + v.v[0] * (double)c[0];
        s1 = s1 + v.v[1] * (double)c[1];
    }
    const int row = s * kSliceRows + threadIdx.x * 2;
    if (row + 2 <= a.n) {
        Rows<2> o;
        o.v[0] = s0;
        o.v[1] = s1;
        st<2>(a.Ap + row, o);
    }
}

// Separate final reduction (a.fold == 0): the same two levels and order as the
// folded completion, so fold on/off give the same bits.
constexpr int kFinalizeThreads = 1024;
constexpr int kFinLdsGroups = 4096;  // group sums kept in LDS up to 2M slices

__global__ __launch_bounds__(kFinalizeThreads) void k_finalize(CgArgs a, int which, bool prologue)
{
    __shared__ double gs[kFinLdsGroups];
    const int k = a.kst[0];
    const bool run = prologue || cg_run(a, k, false);
    if (threadIdx.x == 0) {
        if (run)
            stamp(a, which == kRR ? kStampFinRR : kStampFinPAP);
        else
            mark_end(a);
    }
    if (!run) return;
    const int ng = ngroups_of(a);
    const bool in_lds = ng <= kFinLdsGroups;
    double* gp = a.partial + a.nslices + which * ng;
    const int lane = threadIdx.x & (kWave - 1);
    constexpr int kWaves = kFinalizeThreads / kWave;
    constexpr int kBatch = 16;  // groups per wave per round, loads in flight together
    for (int g0 = threadIdx.x / kWave; g0 < ng; g0 += kWaves * kBatch) {
        double v[kBatch];
#pragma unroll
        for (int b = 0; b < kBatch; b++) {
            const int i = (g0 + b * kWaves) * kGroup + lane;
            v[b] = (g0 + b * kWaves < ng && i < a.nslices) ? a.partial[i] : 0.0;
        }
#pragma unroll
        for (int b = 0; b < kBatch; b++) {
            const double w = wave_sum(v[b]);
            const int g = g0 + b * kWaves;
            if (lane == 0 && g < ng) {
                if (in_lds)
                    gs[g] = w;
                else
                    gp[g] = w;
            }
        }
    }
    __syncthreads();  // group sums written by this block
    if (threadIdx.x < kWave) {
        const double tot = in_lds ? top_sum_wave([&](int i) { return gs[i]; }, ng, lane)
                                  : top_sum_wave([gp](int i) { return gp[i]; }, ng, lane);
        if (lane == 0) finish_dot(a, tot, which, prologue ? 1 : k + 1);
    }
}

// x += alpha_j p_j for j = j0..j1 in order (HPCCG.cpp:383, one rounding per
// term as in the reference); alpha_kcur comes from the caller (the update's own
// alpha, not yet in ahist for the reader). Four p loads are issued before their
// adds, so a long ring does not serialise one HBM latency per term.
template <int kRpt>
__device__ __forceinline__ void x_accumulate(const CgArgs& a, int row, int j0, int j1, int kcur, double alpha_kcur,
                                             Rows<kRpt>& xn)
{
    constexpr int kB = 4;
    int j = j0;
    for (; j + kB - 1 <= j1; j += kB) {
        Rows<kRpt> pj[kB];
        double aj[kB];
#pragma unroll
        for (int b = 0; b < kB; b++) {
            pj[b] = ld<kRpt>(cur_p(a, j + b) + row);
            aj[b] = (j + b == kcur) ? alpha_kcur : a.ahist[j + b];
        }
#pragma unroll
        for (int b = 0; b < kB; b++)
#pragma unroll
            for (int i = 0; i < kRpt; i++) xn.v[i] = xn.v[i] + aj[b] * pj[b].v[i];
    }
    for (; j <= j1; j++) {
        const double aj = (j == kcur) ? alpha_kcur : a.ahist[j];
        const Rows<kRpt> pj = ld<kRpt>(cur_p(a, j) + row);
#pragma unroll
        for (int i = 0; i < kRpt; i++) xn.v[i] = xn.v[i] + aj * pj.v[i];
    }
}

// ---------------------------------------------------------------------------
// Fused update + r.r partial.
// prologue: r = b + (-1)*Ap                (HPCCG.cpp:352)
// loop:     x = x + alpha*p; r = r + (-alpha)*Ap   (HPCCG.cpp:382-384),
//           alpha = rtrans / (p.Ap); then the r.r partial that the next
//           iteration's ddot(r, r) (HPCCG.cpp:367) would compute.
// ---------------------------------------------------------------------------
// One slice's share of the update for the thread owning rows lt*kRpt.. of
// slice s (HPCCG.cpp:352 in the prologue; :382-384 with the deferred x
// update); returns the thread's r.r contribution.
template <int kRpt, bool kPrologue>
__device__ __forceinline__ double update_slice(const CgArgs& a, int s, int lt, int k, double alpha)
{
    const int row = s * kSliceRows + lt * kRpt;
    const Rows<kRpt> apv = ld<kRpt>(a.Ap + row);
    Rows<kRpt> rn;
    if constexpr (kPrologue) {
        const Rows<kRpt> bv = ld<kRpt>(a.b + row);
#pragma unroll
        for (int i = 0; i < kRpt; i++) rn.v[i] = bv.v[i] + (-1.0) * apv.v[i];
    } else {
        const Rows<kRpt> rv = ld<kRpt>(a.r + row);
#pragma unroll
        for (int i = 0; i < kRpt; i++) rn.v[i] = rv.v[i] + (-alpha) * apv.v[i];
        if (!a.xdefer) {
            const Rows<kRpt> xv = ld<kRpt>(a.x + row);
            const Rows<kRpt> pv = ld<kRpt>(cur_p(a, k) + row);
            Rows<kRpt> xn;
#pragma unroll
            for (int i = 0; i < kRpt; i++) xn.v[i] = xv.v[i] + alpha * pv.v[i];
            st_rows<kRpt>(a.x, row, a.n, xn);
        } else if (k % a.nring == 0) {
            // deferred x update (HPCCG.cpp:383 for iterations k-nring+1 .. k): the same
            // x + alpha_j p_j roundings in the same order, one pass over x
            Rows<kRpt> xn = ld<kRpt>(a.x + row);
            x_accumulate<kRpt>(a, row, k - a.nring + 1, k, k, alpha, xn);
            st_rows<kRpt>(a.x, row, a.n, xn);
        }
    }
    st_rows<kRpt>(a.r, row, a.n, rn);
    double d = 0.0;
#pragma unroll
    for (int i = 0; i < kRpt; i++)
        if (row + i < a.n) d += rn.v[i] * rn.v[i];
    return d;
}

template <int kRpt, bool kPrologue>
__global__ __launch_bounds__(kSliceRows / kRpt) void k_update(CgArgs a)
{
    int k = 0;
    if constexpr (!kPrologue) {
        k = a.kst[0];
        const bool run = cg_run(a, k, false);
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            if (run)
                stamp(a, kStampUpdate);
            else
                mark_end(a);
        }
        if (!run) return;
    }
    const int s = a.rev ? xcd_slice_rev(a.grid) : xcd_slice(a.grid);
    if (s >= a.nslices) return;
    double alpha = 0.0;
    if constexpr (!kPrologue) {
        alpha = a.g[kRR] / a.g[kPAP];
        if (blockIdx.x == 0 && threadIdx.x == 0) a.ahist[k] = alpha;
    }
    const double d = update_slice<kRpt, kPrologue>(a, s, threadIdx.x, k, alpha);
    const double bs = block_sum<kSliceRows / kRpt>(d);
    complete_dot<kSliceRows / kRpt>(a, s, bs, kRR, kPrologue ? 1 : k + 1);
}

// The loop update with the slice's Ap and r loaded before the iteration test
// and alpha, which need two and three dependent scalar loads (a.uearly): the
// same values and the same partial tree as k_update.
template <int kRpt>
__global__ __launch_bounds__(kSliceRows / kRpt) void k_update_e(CgArgs a)
{
    const int s = a.rev ? xcd_slice_rev(a.grid) : xcd_slice(a.grid);
    const bool have = s < a.nslices;
    const int row = s * kSliceRows + threadIdx.x * kRpt;
    Rows<kRpt> apv, rv;
    if (have) {
        apv = ld<kRpt>(a.Ap + row);
        rv = ld<kRpt>(a.r + row);
    }
    const int k = a.kst[0];
    const bool run = cg_run(a, k, false);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (run)
            stamp(a, kStampUpdate);
        else
            mark_end(a);
    }
    if (!run || !have) return;
    const double alpha = a.g[kRR] / a.g[kPAP];
    if (blockIdx.x == 0 && threadIdx.x == 0) a.ahist[k] = alpha;
    Rows<kRpt> rn;
#pragma unroll
    for (int i = 0; i < kRpt; i++) rn.v[i] = rv.v[i] + (-alpha) * apv.v[i];
    if (!a.xdefer) {
        const Rows<kRpt> xv = ld<kRpt>(a.x + row);
        const Rows<kRpt> pv = ld<kRpt>(cur_p(a, k) + row);
        Rows<kRpt> xn;
#pragma unroll
        for (int i = 0; i < kRpt; i++) xn.v[i] = xv.v[i] + alpha * pv.v[i];
        st_rows<kRpt>(a.x, row, a.n, xn);
    } else if (k % a.nring == 0) {
        Rows<kRpt> xn = ld<kRpt>(a.x + row);
        x_accumulate<kRpt>(a, row, k - a.nring + 1, k, k, alpha, xn);
        st_rows<kRpt>(a.x, row, a.n, xn);
    }
    st_rows<kRpt>(a.r, row, a.n, rn);
    double d = 0.0;
#pragma unroll
    for (int i = 0; i < kRpt; i++)
        if (row + i < a.n) d += rn.v[i] * rn.v[i];
    const double bs = block_sum<kSliceRows / kRpt>(d);
    complete_dot<kSliceRows / kRpt>(a, s, bs, kRR, k + 1);
}

// The loop update over kM consecutive slices per workgroup (a.um = kM): the
// same per-slice values, partials and partial tree as k_update (each slice's
// block_sum shape), but one publish round trip and one ticket per kM slices,
// so folding r.r into the update costs a quarter of the tickets at kM = 4.
template <int kRpt, int kM>
__global__ __launch_bounds__(kSliceRows / kRpt) void k_update_m(CgArgs a)
{
    constexpr int kThreads = kSliceRows / kRpt;
    constexpr int kWaves = kThreads / kWave;
    static_assert(kGroup % kM == 0, "a workgroup's slices stay in one group");
    __shared__ double wsum[kM][kWaves];
    const int k = a.kst[0];
    const bool run = cg_run(a, k, false);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (run)
            stamp(a, kStampUpdate);
        else
            mark_end(a);
    }
    if (!run) return;
    const int S = a.rev ? xcd_slice_rev(a.umgrid) : xcd_slice(a.umgrid);
    const int s0 = S * kM;
    if (s0 >= a.nslices) return;
    const int cnt = min(kM, a.nslices - s0);
    const double alpha = a.g[kRR] / a.g[kPAP];
    if (blockIdx.x == 0 && threadIdx.x == 0) a.ahist[k] = alpha;
    double d[kM];
    if (a.xdefer && k % a.nring != 0) {
        // r = r - alpha Ap only (x deferred): every slice's loads first
        Rows<kRpt> apv[kM], rv[kM];
#pragma unroll
        for (int j = 0; j < kM; j++) {
            const int row = (s0 + j) * kSliceRows + threadIdx.x * kRpt;
            if (j < cnt) {
                apv[j] = ld<kRpt>(a.Ap + row);
                rv[j] = ld<kRpt>(a.r + row);
            }
        }
#pragma unroll
        for (int j = 0; j < kM; j++) {
            d[j] = 0.0;
            if (j < cnt) {
                const int row = (s0 + j) * kSliceRows + threadIdx.x * kRpt;
                Rows<kRpt> rn;
#pragma unroll
                for (int i = 0; i < kRpt; i++) rn.v[i] = rv[j].v[i] + (-alpha) * apv[j].v[i];
                st_rows<kRpt>(a.r, row, a.n, rn);
#pragma unroll
                for (int i = 0; i < kRpt; i++)
                    if (row + i < a.n) d[j] += rn.v[i] * rn.v[i];
            }
        }
    } else {
#pragma unroll
        for (int j = 0; j < kM; j++)
            d[j] = j < cnt ? update_slice<kRpt, false>(a, s0 + j, threadIdx.x, k, alpha) : 0.0;
    }
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
#pragma unroll
    for (int j = 0; j < kM; j++) {
        const double v = wave_sum(d[j]);
        if (lane == 0) wsum[j][w] = v;
    }
    __syncthreads();
    if (threadIdx.x >= kWave) return;
    double bs = 0.0;  // block_sum's order: 0 + wave 0 + wave 1 + ...
    if (lane < cnt) {
#pragma unroll
        for (int i = 0; i < kWaves; i++) bs += wsum[lane][i];
    }
    complete_dot_lanes(a, s0, cnt, bs, kRR, k + 1);
}

// ---------------------------------------------------------------------------
// Redundant dot completion (single rank, a.redund): no finalize kernels and no
// tickets between workgroups. The update runs one workgroup per 64-slice group
// (1024 threads, four slices at a time); each workgroup first sums ALL p.Ap
// slice partials itself (the fixed two-level shape of k_finalize), keeps its
// slices' r.r partials in LDS and stores its group's r.r sum; every SpMV
// workgroup then sums the group sums itself (cur_rr). One arrival counter per
// update workgroup advances k.
// ---------------------------------------------------------------------------
constexpr int kUGThreads = 1024;

// p.Ap (which = kPAP) or r.r total from the slice partials, in every thread.
__device__ double total_from_partials(const CgArgs& a, int which, double* gs_lds, const double* part = nullptr)
{
    const int ng = ngroups_of(a);
    (void)which;
    if (!part) part = a.partial;  // the producing kernel's slice partials
    const int lane = threadIdx.x & (kWave - 1);
    const int nw = blockDim.x / kWave;
    constexpr int kB = 8;
    for (int g0 = threadIdx.x / kWave; g0 < ng; g0 += nw * kB) {
        double v[kB];
#pragma unroll
        for (int b = 0; b < kB; b++) {
            const int i = (g0 + b * nw) * kGroup + lane;
            v[b] = (g0 + b * nw < ng && i < a.nslices) ? part[i] : 0.0;
        }
#pragma unroll
        for (int b = 0; b < kB; b++) {
            const double w = wave_sum(v[b]);
            if (lane == 0 && g0 + b * nw < ng) gs_lds[g0 + b * nw] = w;
        }
    }
    __syncthreads();
    __shared__ double tot;
    if (threadIdx.x < kWave) {
        const double t = top_sum_wave([gs_lds](int i) { return gs_lds[i]; }, ng, lane);
        if (lane == 0) tot = t;
    }
    __syncthreads();
    return tot;
}

// Loop update that forms p.Ap itself (a.pap_upd: one rank, at most kPapGroups
// groups): every workgroup sums all SpMV slice partials with k_finalize's
// fixed two-level shape (total_from_partials), so the SpMV publishes its
// partials without tickets and no p.Ap finalize runs. Ap and r are loaded
// before that sum. Same values as k_update.
constexpr int kPapGroups = 64;

template <int kRpt>
__global__ __launch_bounds__(kSliceRows / kRpt) void k_update_pr(CgArgs a)
{
    __shared__ double gs[kPapGroups];
    const int s = a.rev ? xcd_slice_rev(a.grid) : xcd_slice(a.grid);
    const bool have = s < a.nslices;
    const int row = s * kSliceRows + threadIdx.x * kRpt;
    Rows<kRpt> apv, rv;
    if (have) {
        apv = ld<kRpt>(a.Ap + row);
        rv = ld<kRpt>(a.r + row);
    }
    const int k = a.kst[0];
    const bool run = cg_run(a, k, false);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (run)
            stamp(a, kStampUpdate);
        else
            mark_end(a);
    }
    if (!run) return;
    const double pap = total_from_partials(a, kPAP, gs, a.ppart);  // every thread; block-wide barriers
    if (!have) return;
    const double alpha = a.g[kRR] / pap;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        a.ahist[k] = alpha;
        a.g[kPAP] = pap;
        a.loc[kPAP] = pap;
    }
    Rows<kRpt> rn;
#pragma unroll
    for (int i = 0; i < kRpt; i++) rn.v[i] = rv.v[i] + (-alpha) * apv.v[i];
    if (!a.xdefer) {
        const Rows<kRpt> xv = ld<kRpt>(a.x + row);
        const Rows<kRpt> pv = ld<kRpt>(cur_p(a, k) + row);
        Rows<kRpt> xn;
#pragma unroll
        for (int i = 0; i < kRpt; i++) xn.v[i] = xv.v[i] + alpha * pv.v[i];
        st_rows<kRpt>(a.x, row, a.n, xn);
    } else if (k % a.nring == 0) {
        Rows<kRpt> xn = ld<kRpt>(a.x + row);
        x_accumulate<kRpt>(a, row, k - a.nring + 1, k, k, alpha, xn);
        st_rows<kRpt>(a.x, row, a.n, xn);
    }
    st_rows<kRpt>(a.r, row, a.n, rn);
    double d = 0.0;
#pragma unroll
    for (int i = 0; i < kRpt; i++)
        if (row + i < a.n) d += rn.v[i] * rn.v[i];
    const double bs = block_sum<kSliceRows / kRpt>(d);
    complete_dot<kSliceRows / kRpt>(a, s, bs, kRR, k + 1);
}

template <int kRpt, bool kPrologue>
__global__ __launch_bounds__(kUGThreads) void k_update_g(CgArgs a)
{
    __shared__ double gs[kFinLdsGroups];
    __shared__ double wsum[kUGThreads / kWave];
    __shared__ double spart[kGroup];
    int k = 0;
    if constexpr (!kPrologue) {
        k = a.kst[0];
        const bool run = cg_run(a, k, false);
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            if (run)
                stamp(a, kStampUpdate);
            else
                mark_end(a);
        }
        if (!run) return;
    }
    const int ng = ngroups_of(a);
    const int per = a.ugrid / kNumXcd;
    const int b = blockIdx.x;
    const int g = (b % kNumXcd) * per + (a.rev ? per - 1 - b / kNumXcd : b / kNumXcd);
    double alpha = 0.0;
    if constexpr (!kPrologue) {
        const double pap = total_from_partials(a, kPAP, gs);
        alpha = a.hist[k - 1] / pap;  // rtrans / (p.Ap), HPCCG.cpp:380
        if (b == 0 && threadIdx.x == 0) a.ahist[k] = alpha;
    }
    if (g >= ng) return;
    constexpr int kTps = kSliceRows / kRpt;       // threads per slice
    constexpr int kSpp = kUGThreads / kTps;       // slices per pass
    const int q = threadIdx.x / kTps, lt = threadIdx.x % kTps;
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    const int s0 = g * kGroup, cnt = min(kGroup, a.nslices - s0);
    for (int j0 = 0; j0 < cnt; j0 += kSpp) {
        const int j = j0 + q;
        double d = 0.0;
        if (j < cnt) d = update_slice<kRpt, kPrologue>(a, s0 + j, lt, k, alpha);
        // the block_sum<kTps> shape per slice: wave sums, then in wave order
        d = wave_sum(d);
        if (lane == 0) wsum[w] = d;
        __syncthreads();
        if (lt == 0 && j < cnt) {
            double bs = 0.0;
#pragma unroll
            for (int i = 0; i < kTps / kWave; i++) bs += wsum[q * (kTps / kWave) + i];
            spart[j] = bs;
        }
        __syncthreads();
    }
    if (threadIdx.x < kWave) {
        const double v = wave_sum(lane < cnt ? spart[lane] : 0.0);  // group_sum's shape
        if (lane == 0) {
            a.partial[a.nslices + kRR * ng + g] = v;
            __threadfence();
            const unsigned t = atomicAdd(a.tickets, 1u);
            if (t == (unsigned)ng - 1u) {  // every group stored: advance k
                stamp(a, kStampFinRR);
                a.kst[0] = kPrologue ? 1 : k + 1;
                atomicExch(a.tickets, 0u);
            }
        }
    }
}


// Timestamp-only kernel around RCCL calls (multi-rank): one lane, one store.
__global__ void k_stamp(CgArgs a, int slot, bool prologue)
{
    if (!prologue) {
        // The r.r all-reduce follows the finalize that already advanced k.
        const int k = a.kst[0] - (slot == kStampArRR ? 1 : 0);
        if (!cg_run(a, k, false)) {
            mark_end(a);
            return;
        }
    }
    stamp(a, slot);
}

__global__ void k_end(CgArgs a) { mark_end(a); }

// After the loop: x += alpha_j p_j for the iterations since the last batched
// update (niters = kst[0] - 1 is final here).
template <int kRpt>
__global__ __launch_bounds__(kSliceRows / kRpt) void k_xflush(CgArgs a)
{
    const int niters = a.kst[0] - 1;
    const int first = (niters / a.nring) * a.nring + 1;
    if (!a.xdefer || first > niters) return;
    const int s = xcd_slice(a.grid);
    if (s >= a.nslices) return;
    const int row = s * kSliceRows + threadIdx.x * kRpt;
    Rows<kRpt> xn = ld<kRpt>(a.x + row);
    x_accumulate<kRpt>(a, row, first, niters, -1, 0.0, xn);
    st_rows<kRpt>(a.x, row, a.n, xn);
}

// ---------------------------------------------------------------------------
// Kernel-level ops on arbitrary device pointers.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_waxpby(int n, double alpha, const double* x, double beta,
                                                const double* y, double* w)
{
    // waxpby.cpp:73-90 branches (alpha == 1 / beta == 1 only drop an exact
    // multiply by one, so every branch rounds like the general expression).
    const int stride = gridDim.x * blockDim.x;
    if (alpha == 1.0) {
        for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) w[i] = x[i] + beta * y[i];
    } else if (beta == 1.0) {
        for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) w[i] = alpha * x[i] + y[i];
    } else {
        for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
            w[i] = alpha * x[i] + beta * y[i];
    }
}

constexpr int kDotChunk = 4096;  // rows per partial: fixed shape, deterministic
constexpr int kDotFinalThreads = 1024;

__global__ __launch_bounds__(256) void k_dot_partial(int n, const double* x, const double* y,
                                                     double* partial)
{
    const int base = blockIdx.x * kDotChunk;
    const int end = min(n, base + kDotChunk);
    double d = 0.0;
    for (int i = base + threadIdx.x; i < end; i += 256) d += x[i] * y[i];
    const double s = block_sum<256>(d);
    if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

__global__ __launch_bounds__(kDotFinalThreads) void k_dot_final(const double* partial, int nparts,
                                                                double* out)
{
    double v = 0.0;
    for (int i = threadIdx.x; i < nparts; i += kDotFinalThreads) v += partial[i];
    const double s = block_sum<kDotFinalThreads>(v);
    if (threadIdx.x == 0) *out = s;
}

// ---------------------------------------------------------------------------
// Device generator: generate_matrix.cpp:251-289 written straight into the
// SELL-512 image. One thread per row; entries in (sz, sy, sx) order; slots
// past the row length padded with col = -1, val = 0. Local columns are
// global - col_base (col_base = start_row - ghost_lo).
// ---------------------------------------------------------------------------
__device__ __forceinline__ unsigned short lds_index(int lc, const int* win_start, const int* win_len,
                                                    const int* win_off, int w0, int w1)
{
    for (int w = w0; w < w1; w++)
        if (lc >= win_start[w] && lc < win_start[w] + win_len[w])
            return (unsigned short)(win_off[w] + lc - win_start[w]);
    return kLdsPad;  // not reached: windows cover every column of the slice
}

__global__ __launch_bounds__(256) void k_generate(int nx, int ny, int nz, int rank, int size,
                                                  int use_7pt, long long col_base,
                                                  const unsigned int* slice_base, int* cols,
                                                  double* vals, double* b, double* xexact, int nrow,
                                                  const int* win_ptr, const int* win_start,
                                                  const int* win_len, const int* win_off,
                                                  unsigned short* lcols)
{
    const int lrow = blockIdx.x * blockDim.x + threadIdx.x;
    if (lrow >= nrow) return;
    const long long nxy = (long long)nx * ny;
    const long long total_nrow = (long long)nrow * size;
    const long long start_row = (long long)nrow * rank;
    const int iz = (int)(lrow / nxy);
    const int iy = (int)((lrow - (long long)iz * nxy) / nx);
    const int ix = (int)(lrow - (long long)iz * nxy - (long long)iy * nx);
    const long long currow = start_row + lrow;
    const int s = lrow / kSliceRows;
    const int lane = lrow - s * kSliceRows;
    const unsigned int b0 = slice_base[s];
    const int w = (int)(slice_base[s + 1] - b0);
    const size_t base = (size_t)b0 * kSliceRows + lane;
    int j = 0;
    for (int sz = -1; sz <= 1; sz++)
        for (int sy = -1; sy <= 1; sy++)
            for (int sx = -1; sx <= 1; sx++) {
                const long long curcol = currow + sz * nxy + (long long)sy * nx + sx;
                if (ix + sx >= 0 && ix + sx < nx && iy + sy >= 0 && iy + sy < ny && curcol >= 0 &&
                    curcol < total_nrow && (!use_7pt || sz * sz + sy * sy + sx * sx <= 1)) {
                    vals[base + (size_t)j * kSliceRows] = (curcol == currow) ? 27.0 : -1.0;
                    cols[base + (size_t)j * kSliceRows] = (int)(curcol - col_base);
                    if (lcols)
                        lcols[base + (size_t)j * kSliceRows] =
                            lds_index((int)(curcol - col_base), win_start, win_len, win_off,
                                      win_ptr[s], win_ptr[s + 1]);
                    j++;
                }
            }
    b[lrow] = 27.0 - ((double)(j - 1));
    xexact[lrow] = 1.0;
    for (; j < w; j++) {
        vals[base + (size_t)j * kSliceRows] = 0.0;
        cols[base + (size_t)j * kSliceRows] = -1;
        if (lcols) lcols[base + (size_t)j * kSliceRows] = kLdsPad;
    }
}

// Rows of the last slice past nrow: all slots padding.
__global__ void k_generate_tail(int nrow, int nslices, const unsigned int* slice_base, int* cols,
                                double* vals, unsigned short* lcols)
{
    const int s = nslices - 1;
    const int lane = threadIdx.x;
    if (s * kSliceRows + lane < nrow) return;
    const unsigned int b0 = slice_base[s];
    const int w = (int)(slice_base[s + 1] - b0);
    for (int j = 0; j < w; j++) {
        vals[(size_t)b0 * kSliceRows + (size_t)j * kSliceRows + lane] = 0.0;
        cols[(size_t)b0 * kSliceRows + (size_t)j * kSliceRows + lane] = -1;
        if (lcols) lcols[(size_t)b0 * kSliceRows + (size_t)j * kSliceRows + lane] = kLdsPad;
    }
}

constexpr int kRpt = 2;
constexpr int kBlock = kSliceRows / kRpt;

}  // namespace

// ---- launch wrappers ------------------------------------------------------
void launch_cg_prologue_copy(const CgArgs& a, hipStream_t s)
{
    hipLaunchKernelGGL(k_prologue_copy<kRpt>, dim3(a.grid), dim3(kBlock), 0, s, a);
}

void launch_cg_p_update(const CgArgs& a, hipStream_t s)
{
    hipLaunchKernelGGL(k_p_update<kRpt>, dim3(a.grid), dim3(kBlock), 0, s, a);
}

void launch_interleave_v4(const unsigned int* slice_base, const unsigned int* vbase4, int nslices,
                          const unsigned char* codes, unsigned char* out, hipStream_t s)
{
    if (nslices <= 0) return;
    hipLaunchKernelGGL(k_interleave_v4, dim3(nslices), dim3(256), 0, s, slice_base, vbase4, nslices, codes, out);
}

void launch_build_p(const unsigned int* slice_base, int nslices, const unsigned char* codes, unsigned char* prow,
                    int* prep, int* pcount, int* ok, hipStream_t s)
{
    if (nslices <= 0) return;
    hipLaunchKernelGGL(k_build_p, dim3(nslices), dim3(kSliceRows), 0, s, slice_base, nslices, codes, prow, prep,
                       pcount, ok);
}

void launch_build_a(const unsigned int* slice_base, int nslices, const unsigned char* codes, const double* vals,
                    const int* cdict, const int* ccount, const unsigned int* abase, double* aval, int* aoff,
                    int* ok, int* maxabs, hipStream_t s)
{
    if (nslices <= 0) return;
    hipLaunchKernelGGL(k_build_a, dim3(nslices), dim3(kSliceRows), 0, s, slice_base, nslices, codes, vals, cdict,
                       ccount, abase, aval, aoff, ok, maxabs);
}

void launch_fill_p(const unsigned int* slice_base, int nslices, const unsigned char* codes, const int* prep,
                   const int* pcount, const int* pbase, const int* cdict, const int* ldsc, int* tab_g, int* tab_l,
                   hipStream_t s)
{
    if (nslices <= 0) return;
    hipLaunchKernelGGL(k_fill_p, dim3(nslices), dim3(256), 0, s, slice_base, nslices, codes, prep, pcount, pbase,
                       cdict, ldsc, tab_g, tab_l);
}

void launch_build_c(const unsigned int* slice_base, int nslices, const int* cols, const double* vals,
                    const int* win_ptr, const int* win_start, const int* win_off, const int* win_len,
                    unsigned char* codes, int* cdict, double* cval, int* ldsc, int* ccount, int* ok,
                    hipStream_t s)
{
    if (nslices <= 0) return;
    hipLaunchKernelGGL(k_build_c, dim3(nslices), dim3(256), 0, s, slice_base, nslices, cols, vals, win_ptr,
                       win_start, win_off, win_len, codes, cdict, cval, ldsc, ccount, ok);
}

void launch_cg_pack(const CgArgs& a, const int* idx, int cnt, double* buf, bool prologue, hipStream_t s)
{
    if (cnt <= 0) return;
    hipLaunchKernelGGL(k_pack, dim3((cnt + 255) / 256), dim3(256), 0, s, a, idx, cnt, buf, prologue);
}

void launch_cg_p_boundary(const CgArgs& a, int nlo, int nhi, hipStream_t s)
{
    if (nlo + nhi <= 0) return;
    hipLaunchKernelGGL(k_p_boundary, dim3((nlo + nhi + 255) / 256), dim3(256), 0, s, a, nlo, nhi);
}

// SpMV variants. All compute every row bitwise identically; the p.Ap
// partial's summation tree depends only on rows-per-thread (kRpt), so
// variants with equal kRpt give bitwise-equal CG traces.
//   0 runtime width, 2 rows/thread      1 runtime width, 1 row/thread
//   2 runtime width, 4 rows/thread
//   27 / 7  uniform width, fully unrolled, 2 rows/thread
//   327 / 427: same with __launch_bounds__ min waves/SIMD 3 / 4
//   +1000: non-temporal loads of vals/cols (1000 = the default: runtime
//   width, 2 rows/thread, nt -- within ~3 % of the matrix-streaming ceiling)
//   2000 / 2001 / 2002 / 2100: SELL-512-L (x windows staged in LDS, 16-bit
//   slice-local indices) with 2 / 1 / 4 rows per thread, nt; 2100 = 2 rows, no nt
//   3xxx / 4xxx: SELL-512-C (1-byte offset codes), plain gather / LDS windows
//   5xxx / 6xxx / 7xxx: SELL-512-V (codes of (offset, value) pairs; opt-in)
//   8000 / 8200 / 8208 / 8300 / 8201: SELL-512-P with LDS windows (per-row
//   pattern ids; prefetch 0 / 4 / 8 slots, 8300 no nt, 8201 1 row/thread);
//   8216 / 8219 / 8226: prefetch 8 / 8 / 4, stream unrolled 6 / 9 / 6;
//   8308 / 8316 / 8326: no nt, prefetch 8 / 8 / 4, unrolled 3 / 6 / 6
//   8507 / 8527 / 8607: plain SELL-512-P, uniform width 7 / 27 / 7 fully
//   unrolled (8607 no nt)
//   8500 / 8501 / 8600: SELL-512-P, plain gather (2 rows nt, 1 row nt, 2 rows)
//   8700 / 8707 / 8727 / 8800 / 8807: SELL-512-A (offset-aligned slots, one
//   16-byte x load per thread and slot), nt dynamic width / 7 / 27, no nt
//   dynamic / 7
//   8236 / 8246 / 8336: 8226 (nt, prefetch 4 / 8) and 8326 (default policy)
//   with the pattern ids and the prefetched slots loaded before the run test
//   8717 / 8817: width 7 unrolled, all 7 value slots and the offsets loaded
//   before the run test (nt / default policy); 8737 / 8757 / 8837 / 8857:
//   width 27, 4 / 8 value slots early (nt, nt, default, default)
//   8900 / 8902 / 8910 / 8927 / 8947: SELL-512-A with LDS windows, nt prefetch
//   4 / nt prefetch 2 / no nt prefetch 4 / nt prefetch 4 width 27 unrolled /
//   nt no prefetch width 27
//   8960 / 8962 / 8970: SELL-512-A pair windows (two slices per 512-thread
//   block, single rank), nt prefetch 4 / nt prefetch 2 / default policy 4;
//   8961 / 8963 / 8965: nt prefetch 1 / 3 / 0; 8966 / 8967 / 8968: nt
//   prefetch 2 / 1 / 4 with at most 64 VGPRs (8 waves per SIMD)
//   8972 / 8973: 8963 with 2 / 3 staged positions per thread, loads before
//   stores; 8974: 8963 with at most 64 VGPRs (8 waves per SIMD)
//   8980 / 8982 / 8983: four slices per 1024-thread block (quad windows),
//   nt prefetch 0 / 2 / 3
//   9999: diagnostic matrix stream without the gather (not an SpMV)
#define HPCCG_SPMV(RPT, W, MINW, NT)                                                                \
    do {                                                                                            \
        if (a.fuse_p && !prologue)                                                                  \
            hipLaunchKernelGGL((k_spmv<RPT, W, MINW, NT, true>), dim3(a.sgrid), dim3(kSliceRows / RPT), \
                               0, s, a, prologue);                                                  \
        else                                                                                        \
            hipLaunchKernelGGL((k_spmv<RPT, W, MINW, NT, false>), dim3(a.sgrid),                   \
                               dim3(kSliceRows / RPT), 0, s, a, prologue);                          \
    } while (0)
#define HPCCG_SPMV_CWV(RPT, NT, W, VAL)                                                            \
    do {                                                                                           \
        if (a.fuse_p && !prologue)                                                                 \
            hipLaunchKernelGGL((k_spmv_c<RPT, NT, true, W, VAL>), dim3(a.sgrid), dim3(kSliceRows / RPT), 0, s, \
                               a, prologue);                                                       \
        else                                                                                       \
            hipLaunchKernelGGL((k_spmv_c<RPT, NT, false, W, VAL>), dim3(a.sgrid), dim3(kSliceRows / RPT), 0, \
                               s, a, prologue);                                                    \
    } while (0)
#define HPCCG_SPMV_V4P(RPT, NT, W, PRE)                                                            \
    do {                                                                                           \
        if (a.fuse_p && !prologue)                                                                 \
            hipLaunchKernelGGL((k_spmv_v4<RPT, NT, true, W, PRE>), dim3(a.sgrid), dim3(kSliceRows / RPT), 0, s, \
                               a, prologue);                                                       \
        else                                                                                       \
            hipLaunchKernelGGL((k_spmv_v4<RPT, NT, false, W, PRE>), dim3(a.sgrid), dim3(kSliceRows / RPT), 0, \
                               s, a, prologue);                                                    \
    } while (0)
#define HPCCG_SPMV_V4(RPT, NT, W) HPCCG_SPMV_V4P(RPT, NT, W, 0)
#define HPCCG_SPMV_CW(RPT, NT, W) HPCCG_SPMV_CWV(RPT, NT, W, false)
#define HPCCG_SPMV_C(RPT, NT) HPCCG_SPMV_CW(RPT, NT, 0)
#define HPCCG_SPMV_V(RPT, NT) HPCCG_SPMV_CWV(RPT, NT, 0, true)
#define HPCCG_SPMV_LDSX(RPT, NT, PRE, CODE)                                                        \
    do {                                                                                           \
        const size_t smem = (size_t)a.lds_doubles * sizeof(double);                                \
        if (a.fuse_p && !prologue)                                                                 \
            hipLaunchKernelGGL((k_spmv_lds<RPT, NT, true, PRE, CODE>), dim3(a.sgrid), dim3(kSliceRows / RPT), \
                               smem, s, a, prologue);                                              \
        else                                                                                       \
            hipLaunchKernelGGL((k_spmv_lds<RPT, NT, false, PRE, CODE>), dim3(a.sgrid), dim3(kSliceRows / RPT), \
                               smem, s, a, prologue);                                              \
    } while (0)
#define HPCCG_SPMV_LDS(RPT, NT, PRE) HPCCG_SPMV_LDSX(RPT, NT, PRE, 0)
#define HPCCG_SPMV_LPE(RPT, NT, PRE, U, E)                                                         \
    do {                                                                                           \
        const size_t smem = (size_t)a.lds_doubles * sizeof(double) + (size_t)a.pat_max * sizeof(int); \
        if (a.fuse_p && !prologue)                                                                 \
            hipLaunchKernelGGL((k_spmv_lp<RPT, NT, true, PRE, U, E>), dim3(a.sgrid), dim3(kSliceRows / RPT), smem, \
                               s, a, prologue);                                                    \
        else                                                                                       \
            hipLaunchKernelGGL((k_spmv_lp<RPT, NT, false, PRE, U, E>), dim3(a.sgrid), dim3(kSliceRows / RPT), \
                               smem, s, a, prologue);                                              \
    } while (0)
#define HPCCG_SPMV_LPU(RPT, NT, PRE, U) HPCCG_SPMV_LPE(RPT, NT, PRE, U, false)
#define HPCCG_SPMV_LP(RPT, NT, PRE) HPCCG_SPMV_LPU(RPT, NT, PRE, 3)
#define HPCCG_SPMV_PAP(RPT, NT, W, PRE)                                                            \
    do {                                                                                           \
        if (a.fuse_p && !prologue)                                                                 \
            hipLaunchKernelGGL((k_spmv_pa<RPT, NT, W, true, PRE>), dim3(a.sgrid), dim3(kSliceRows / RPT), 0, \
                               s, a, prologue);                                                    \
        else                                                                                       \
            hipLaunchKernelGGL((k_spmv_pa<RPT, NT, W, false, PRE>), dim3(a.sgrid), dim3(kSliceRows / RPT), 0, \
                               s, a, prologue);                                                    \
    } while (0)
#define HPCCG_SPMV_PA(RPT, NT, W) HPCCG_SPMV_PAP(RPT, NT, W, 0)
#define HPCCG_SPMV_LA(RPT, NT, PRE, W)                                                             \
    do {                                                                                           \
        const size_t smem = (size_t)a.alds_doubles * sizeof(double);                               \
        if (a.fuse_p && !prologue)                                                                 \
            hipLaunchKernelGGL((k_spmv_la<RPT, NT, true, PRE, W>), dim3(a.sgrid), dim3(kSliceRows / RPT), smem, \
                               s, a, prologue);                                                    \
        else                                                                                       \
            hipLaunchKernelGGL((k_spmv_la<RPT, NT, false, PRE, W>), dim3(a.sgrid), dim3(kSliceRows / RPT), \
                               smem, s, a, prologue);                                              \
    } while (0)
#define HPCCG_SPMV_LA2W(NT, PRE, MINW)                                                             \
    do {                                                                                           \
        const size_t smem = (size_t)a.alds2_doubles * sizeof(double);                              \
        if (a.fuse_p && !prologue)                                                                 \
            hipLaunchKernelGGL((k_spmv_la2<NT, true, PRE, MINW>), dim3(a.pgrid), dim3(kSliceRows), smem, s, a, \
                               prologue);                                                          \
        else                                                                                       \
            hipLaunchKernelGGL((k_spmv_la2<NT, false, PRE, MINW>), dim3(a.pgrid), dim3(kSliceRows), smem, s, a, \
                               prologue);                                                          \
    } while (0)
#define HPCCG_SPMV_LA2(NT, PRE) HPCCG_SPMV_LA2W(NT, PRE, 1)
#define HPCCG_SPMV_LA2U(NT, PRE, SU)                                                               \
    do {                                                                                           \
        const size_t smem = (size_t)a.alds2_doubles * sizeof(double);                              \
        if (a.fuse_p && !prologue)                                                                 \
            hipLaunchKernelGGL((k_spmv_la2<NT, true, PRE, SU == 4 ? 8 : 1, 2, SU == 4 ? 1 : SU>), dim3(a.pgrid), dim3(kSliceRows), smem, s, \
                               a, prologue);                                                       \
        else                                                                                       \
            hipLaunchKernelGGL((k_spmv_la2<NT, false, PRE, SU == 4 ? 8 : 1, 2, SU == 4 ? 1 : SU>), dim3(a.pgrid), dim3(kSliceRows), smem, \
                               s, a, prologue);                                                    \
    } while (0)
#define HPCCG_SPMV_LA4(NT, PRE)                                                                    \
    do {                                                                                           \
        const size_t smem = (size_t)a.alds4_doubles * sizeof(double);                              \
        if (a.fuse_p && !prologue)                                                                 \
            hipLaunchKernelGGL((k_spmv_la2<NT, true, PRE, 8, 4>), dim3(a.qgrid), dim3(2 * kSliceRows), smem, s, \
                               a, prologue);                                                       \
        else                                                                                       \
            hipLaunchKernelGGL((k_spmv_la2<NT, false, PRE, 8, 4>), dim3(a.qgrid), dim3(2 * kSliceRows), smem, \
                               s, a, prologue);                                                    \
    } while (0)
#define HPCCG_SPMV_PPW(RPT, NT, W)                                                                 \
    do {                                                                                           \
        if (a.fuse_p && !prologue)                                                                 \
            hipLaunchKernelGGL((k_spmv_pp<RPT, NT, true, W>), dim3(a.sgrid), dim3(kSliceRows / RPT),         \
                               (size_t)a.pat_max * sizeof(int), s, a, prologue);                   \
        else                                                                                       \
            hipLaunchKernelGGL((k_spmv_pp<RPT, NT, false, W>), dim3(a.sgrid), dim3(kSliceRows / RPT),        \
                               (size_t)a.pat_max * sizeof(int), s, a, prologue);                   \
    } while (0)
#define HPCCG_SPMV_PP(RPT, NT) HPCCG_SPMV_PPW(RPT, NT, 0)
bool spmv_variant_ok(int v)
{
    switch (v) {
    case 0: case 1: case 2: case 27: case 7: case 327: case 427:
    case 1000: case 1001: case 1002: case 1027: case 1007: case 9999:
    case 2000: case 2001: case 2002: case 2100: case 2200: case 2208: case 2300: case 2308:
    case 3000: case 3001: case 3002: case 3100: case 3007: case 3027: case 4000: case 4200: case 4300: case 4202: case 4206: case 4208:
    case 5000: case 5100: case 5200: case 5208: case 5300: case 5308: case 5401: case 5404: case 5204:
    case 6000: case 6100: case 6104: case 6001:
    case 7001: case 7101: case 7002: case 7102: case 7027: case 7127: case 7007: case 7107:
    case 7201: case 7202: case 7301: case 7302: case 7204:
    case 8000: case 8200: case 8208: case 8300: case 8201: case 8500: case 8501: case 8600:
    case 8216: case 8219: case 8226: case 8308: case 8316: case 8326: case 8507: case 8527: case 8607:
    case 8700: case 8707: case 8727: case 8800: case 8807:
    case 8900: case 8927: case 8910: case 8902: case 8947:
    case 8236: case 8246: case 8336: case 8960: case 8962: case 8970:
    case 8961: case 8963: case 8965: case 8966: case 8967: case 8968:
    case 8980: case 8982: case 8983: case 8972: case 8973: case 8974:
    case 8717: case 8737: case 8757: case 8837: case 8857: case 8817:
        return true;
    default:
        return false;
    }
}

void launch_cg_spmv(const CgArgs& a, int variant, bool prologue, hipStream_t s)
{
    switch (variant) {
    case 1: HPCCG_SPMV(1, 0, 1, false); break;
    case 2: HPCCG_SPMV(4, 0, 1, false); break;
    case 27: HPCCG_SPMV(2, 27, 1, false); break;
    case 327: HPCCG_SPMV(2, 27, 3, false); break;
    case 427: HPCCG_SPMV(2, 27, 4, false); break;
    case 7: HPCCG_SPMV(2, 7, 1, false); break;
    case 1000: HPCCG_SPMV(2, 0, 1, true); break;
    case 1001: HPCCG_SPMV(1, 0, 1, true); break;
    case 1002: HPCCG_SPMV(4, 0, 1, true); break;
    case 1027: HPCCG_SPMV(2, 27, 1, true); break;
    case 1007: HPCCG_SPMV(2, 7, 1, true); break;
    case 9999: hipLaunchKernelGGL(k_stream_diag<27>, dim3(a.grid), dim3(256), 0, s, a); break;
    case 2000: HPCCG_SPMV_LDS(2, true, 0); break;
    case 2001: HPCCG_SPMV_LDS(1, true, 0); break;
    case 2002: HPCCG_SPMV_LDS(4, true, 0); break;
    case 2100: HPCCG_SPMV_LDS(2, false, 0); break;
    case 2200: HPCCG_SPMV_LDS(2, true, 4); break;
    case 2208: HPCCG_SPMV_LDS(2, true, 8); break;
    case 2300: HPCCG_SPMV_LDS(2, false, 4); break;
    case 2308: HPCCG_SPMV_LDS(2, false, 8); break;
    case 4200: HPCCG_SPMV_LDSX(2, true, 4, 1); break;
    case 4202: HPCCG_SPMV_LDSX(2, true, 2, 1); break;
    case 4206: HPCCG_SPMV_LDSX(2, true, 6, 1); break;
    case 4208: HPCCG_SPMV_LDSX(2, true, 8, 1); break;
    case 4300: HPCCG_SPMV_LDSX(2, false, 4, 1); break;
    case 4000: HPCCG_SPMV_LDSX(2, true, 0, 1); break;
    case 5200: HPCCG_SPMV_LDSX(2, true, 4, 2); break;
    case 5208: HPCCG_SPMV_LDSX(2, true, 8, 2); break;
    case 5300: HPCCG_SPMV_LDSX(2, false, 4, 2); break;
    case 5308: HPCCG_SPMV_LDSX(2, false, 8, 2); break;
    case 5000: HPCCG_SPMV_LDSX(2, true, 0, 2); break;
    case 5100: HPCCG_SPMV_LDSX(2, false, 0, 2); break;
    case 5401: HPCCG_SPMV_LDSX(1, false, 8, 2); break;
    case 5404: HPCCG_SPMV_LDSX(4, false, 4, 2); break;
    case 5204: HPCCG_SPMV_LDSX(4, true, 4, 2); break;
    case 6000: HPCCG_SPMV_V(2, true); break;
    case 6100: HPCCG_SPMV_V(2, false); break;
    case 6104: HPCCG_SPMV_V(4, false); break;
    case 6001: HPCCG_SPMV_V(1, true); break;
    case 7001: HPCCG_SPMV_V4(1, true, 0); break;
    case 7101: HPCCG_SPMV_V4(1, false, 0); break;
    case 7002: HPCCG_SPMV_V4(2, true, 0); break;
    case 7102: HPCCG_SPMV_V4(2, false, 0); break;
    case 7027: HPCCG_SPMV_V4(1, true, 27); break;
    case 7127: HPCCG_SPMV_V4(1, false, 27); break;
    case 7007: HPCCG_SPMV_V4(1, true, 7); break;
    case 7107: HPCCG_SPMV_V4(1, false, 7); break;
    case 7201: HPCCG_SPMV_V4P(1, true, 0, 8); break;
    case 7202: HPCCG_SPMV_V4P(2, true, 0, 8); break;
    case 7301: HPCCG_SPMV_V4P(1, false, 0, 8); break;
    case 7302: HPCCG_SPMV_V4P(2, false, 0, 8); break;
    case 7204: HPCCG_SPMV_V4P(2, true, 0, 4); break;
    case 8000: HPCCG_SPMV_LP(2, true, 0); break;
    case 8200: HPCCG_SPMV_LP(2, true, 4); break;
    case 8208: HPCCG_SPMV_LP(2, true, 8); break;
    case 8300: HPCCG_SPMV_LP(2, false, 4); break;
    case 8201: HPCCG_SPMV_LP(1, true, 4); break;
    case 8216: HPCCG_SPMV_LPU(2, true, 8, 6); break;
    case 8219: HPCCG_SPMV_LPU(2, true, 8, 9); break;
    case 8226: HPCCG_SPMV_LPU(2, true, 4, 6); break;
    case 8308: HPCCG_SPMV_LP(2, false, 8); break;
    case 8316: HPCCG_SPMV_LPU(2, false, 8, 6); break;
    case 8326: HPCCG_SPMV_LPU(2, false, 4, 6); break;
    case 8507: HPCCG_SPMV_PPW(2, true, 7); break;
    case 8700: HPCCG_SPMV_PA(2, true, 0); break;
    case 8236: HPCCG_SPMV_LPE(2, true, 4, 6, true); break;
    case 8246: HPCCG_SPMV_LPE(2, true, 8, 6, true); break;
    case 8336: HPCCG_SPMV_LPE(2, false, 4, 6, true); break;
    case 8717: HPCCG_SPMV_PAP(2, true, 7, 7); break;
    case 8817: HPCCG_SPMV_PAP(2, false, 7, 7); break;
    case 8737: HPCCG_SPMV_PAP(2, true, 27, 4); break;
    case 8757: HPCCG_SPMV_PAP(2, true, 27, 8); break;
    case 8837: HPCCG_SPMV_PAP(2, false, 27, 4); break;
    case 8857: HPCCG_SPMV_PAP(2, false, 27, 8); break;
    case 8900: HPCCG_SPMV_LA(2, true, 4, 0); break;
    case 8960: HPCCG_SPMV_LA2(true, 4); break;
    case 8962: HPCCG_SPMV_LA2(true, 2); break;
    case 8961: HPCCG_SPMV_LA2(true, 1); break;
    case 8972: HPCCG_SPMV_LA2U(true, 3, 2); break;
    case 8973: HPCCG_SPMV_LA2U(true, 3, 3); break;
    case 8974: HPCCG_SPMV_LA2U(true, 3, 4); break;
    case 8980: HPCCG_SPMV_LA4(true, 0); break;
    case 8982: HPCCG_SPMV_LA4(true, 2); break;
    case 8983: HPCCG_SPMV_LA4(true, 3); break;
    case 8965: HPCCG_SPMV_LA2(true, 0); break;
    case 8963: HPCCG_SPMV_LA2(true, 3); break;
    case 8966: HPCCG_SPMV_LA2W(true, 2, 8); break;
    case 8967: HPCCG_SPMV_LA2W(true, 1, 8); break;
    case 8968: HPCCG_SPMV_LA2W(true, 4, 8); break;
    case 8970: HPCCG_SPMV_LA2(false, 4); break;
    case 8902: HPCCG_SPMV_LA(2, true, 2, 0); break;
    case 8910: HPCCG_SPMV_LA(2, false, 4, 0); break;
    case 8927: HPCCG_SPMV_LA(2, true, 4, 27); break;
    case 8947: HPCCG_SPMV_LA(2, true, 0, 27); break;
    case 8707: HPCCG_SPMV_PA(2, true, 7); break;
    case 8727: HPCCG_SPMV_PA(2, true, 27); break;
    case 8800: HPCCG_SPMV_PA(2, false, 0); break;
    case 8807: HPCCG_SPMV_PA(2, false, 7); break;
    case 8527: HPCCG_SPMV_PPW(2, true, 27); break;
    case 8607: HPCCG_SPMV_PPW(2, false, 7); break;
    case 8500: HPCCG_SPMV_PP(2, true); break;
    case 8501: HPCCG_SPMV_PP(1, true); break;
    case 8600: HPCCG_SPMV_PP(2, false); break;
    case 3000: HPCCG_SPMV_C(2, true); break;
    case 3001: HPCCG_SPMV_C(1, true); break;
    case 3002: HPCCG_SPMV_C(4, true); break;
    case 3100: HPCCG_SPMV_C(2, false); break;
    case 3007: HPCCG_SPMV_CW(2, true, 7); break;
    case 3027: HPCCG_SPMV_CW(2, true, 27); break;
    default: HPCCG_SPMV(2, 0, 1, false); break;
    }
}
#undef HPCCG_SPMV
#undef HPCCG_SPMV_LDS
#undef HPCCG_SPMV_LDSX
#undef HPCCG_SPMV_C
#undef HPCCG_SPMV_CW
#undef HPCCG_SPMV_CWV
#undef HPCCG_SPMV_V
#undef HPCCG_SPMV_V4
#undef HPCCG_SPMV_V4P
#undef HPCCG_SPMV_LP
#undef HPCCG_SPMV_LPU
#undef HPCCG_SPMV_PP
#undef HPCCG_SPMV_PPW

void launch_cg_finalize(const CgArgs& a, int which, bool prologue, hipStream_t s)
{
    hipLaunchKernelGGL(k_finalize, dim3(1), dim3(kFinalizeThreads), 0, s, a, which, prologue);
}

void launch_cg_update(const CgArgs& a, bool prologue, hipStream_t s)
{
    if (a.redund) {
        if (prologue)
            hipLaunchKernelGGL((k_update_g<kRpt, true>), dim3(a.ugrid), dim3(kUGThreads), 0, s, a);
        else
            hipLaunchKernelGGL((k_update_g<kRpt, false>), dim3(a.ugrid), dim3(kUGThreads), 0, s, a);
        return;
    }
    if (prologue)
        hipLaunchKernelGGL((k_update<kRpt, true>), dim3(a.grid), dim3(kBlock), 0, s, a);
    else if (a.um == 2)
        hipLaunchKernelGGL((k_update_m<kRpt, 2>), dim3(a.umgrid), dim3(kBlock), 0, s, a);
    else if (a.um == 4)
        hipLaunchKernelGGL((k_update_m<kRpt, 4>), dim3(a.umgrid), dim3(kBlock), 0, s, a);
    else if (a.um == 8)
        hipLaunchKernelGGL((k_update_m<kRpt, 8>), dim3(a.umgrid), dim3(kBlock), 0, s, a);
    else if (a.pap_upd)
        hipLaunchKernelGGL(k_update_pr<kRpt>, dim3(a.grid), dim3(kBlock), 0, s, a);
    else if (a.uearly)
        hipLaunchKernelGGL(k_update_e<kRpt>, dim3(a.grid), dim3(kBlock), 0, s, a);
    else
        hipLaunchKernelGGL((k_update<kRpt, false>), dim3(a.grid), dim3(kBlock), 0, s, a);
}

void launch_cg_stamp(const CgArgs& a, int slot, bool prologue, hipStream_t s)
{
    hipLaunchKernelGGL(k_stamp, dim3(1), dim3(64), 0, s, a, slot, prologue);
}

void launch_cg_end(const CgArgs& a, hipStream_t s)
{
    hipLaunchKernelGGL(k_end, dim3(1), dim3(64), 0, s, a);
}

__global__ void k_group_sum(GroupSum gs)
{
    double v = 0.0;
    for (int r = 0; r < gs.nranks; r++) v += gs.loc[r][gs.which];
    for (int r = 0; r < gs.nranks; r++) gs.g[r][gs.which] = v;
}

void launch_group_sum(const GroupSum& gs, hipStream_t s)
{
    hipLaunchKernelGGL(k_group_sum, dim3(1), dim3(1), 0, s, gs);
}

void launch_cg_xflush(const CgArgs& a, hipStream_t s)
{
    if (a.xdefer) hipLaunchKernelGGL(k_xflush<kRpt>, dim3(a.grid), dim3(kBlock), 0, s, a);
}

void launch_waxpby(int n, double alpha, const double* x, double beta, const double* y, double* w,
                   hipStream_t s)
{
    if (n <= 0) return;
    int grid = (n + 255) / 256;
    if (grid > 8192) grid = 8192;
    hipLaunchKernelGGL(k_waxpby, dim3(grid), dim3(256), 0, s, n, alpha, x, beta, y, w);
}

int ddot_nparts(int n) { return n <= 0 ? 1 : (n + kDotChunk - 1) / kDotChunk; }

void launch_ddot(int n, const double* x, const double* y, double* partial, int nparts, double* out,
                 hipStream_t s)
{
    if (n > 0) hipLaunchKernelGGL(k_dot_partial, dim3(nparts), dim3(256), 0, s, n, x, y, partial);
    hipLaunchKernelGGL(k_dot_final, dim3(1), dim3(kDotFinalThreads), 0, s, partial,
                       n > 0 ? nparts : 0, out);
}

void launch_sparsemv(const CgArgs& a, const double* xext, double* y, int variant, hipStream_t s)
{
    (void)variant;
    hipLaunchKernelGGL(k_spmv_plain<kRpt>, dim3(a.grid), dim3(kBlock), 0, s, a, xext, y);
}

void launch_generate(int nx, int ny, int nz, int rank, int size, int use_7pt, long long col_base,
                     const unsigned int* slice_base, int* cols, double* vals, double* b,
                     double* xexact, int nrow, const int* win_ptr, const int* win_start,
                     const int* win_len, const int* win_off, unsigned short* lcols, hipStream_t s)
{
    const int nslices = (nrow + kSliceRows - 1) / kSliceRows;
    hipLaunchKernelGGL(k_generate, dim3((nrow + 255) / 256), dim3(256), 0, s, nx, ny, nz, rank, size,
                       use_7pt, col_base, slice_base, cols, vals, b, xexact, nrow, win_ptr,
                       win_start, win_len, win_off, lcols);
    hipLaunchKernelGGL(k_generate_tail, dim3(1), dim3(kSliceRows), 0, s, nrow, nslices, slice_base,
                       cols, vals, lcols);
}

}  // namespace hpccg
