// hpccg_kernels.hip -- hand-written CDNA4 (gfx950) kernels for the HPCCG hot
// path. Memory-bound throughout (fp64, ~0.16 flop/byte): no MFMA; the design
// goals are coalesced 16 B/lane streams, one pass per fused step, XCD-local
// slice ownership, and bitwise-reproducible reductions.
//
// Numerics contract (tests/test_gpu_parity.py): compiled with
// -ffp-contract=off, SpMV and waxpby are BITWISE equal to the reference
// (HPC_sparsemv.cpp:76-87, waxpby.cpp:73-90: same per-row entry order, no
// FMA); dot products use a fixed-shape tree (per-slice partials, groups of 64
// slices, one top level), so they are reproducible run to run and differ from
// the reference's sequential sum only by rounding.
//
// Kernels of one CG iteration (HPCCG.cpp:358-386), one workgroup per 512-row
// slice (two for the pair kernel), XCD-aware slice order:
//   SpMV      k_spmv_a2r (SELL-512-A, LDS windows shared by slice pairs, the
//             values streamed HBM -> LDS by per-wave LDS-DMA rings) |
//             k_spmv_a2 (the same with register loads: non-uniform widths) |
//             k_spmv_a (SELL-512-A, x read at the slice's offsets) |
//             k_spmv_sell (SELL-512, int32 columns: any matrix)
//             + p = r + beta p formed on the fly (fused) + p.Ap, completed
//             in the kernel (self-validating slots); trailing blocks apply
//             the deferred x terms of 1/(x_ring-1) of the slices (side_flush)
//   update    k_update: r = r - alpha Ap (x too with x_defer 0 / 1), r.r
//             completed the same way
//   finalize  k_finalize: the fixed-shape total of a dot (fold 0 only)
#include <climits>

#include "hpccg_internal.h"

#pragma clang fp contract(off)

namespace hpccg {

namespace {

constexpr int kWave = 64;
constexpr int kRpt = 2;                    // rows per thread in every slice kernel
constexpr int kBlock = kSliceRows / kRpt;  // 256 threads per slice

__device__ __forceinline__ unsigned long long now_ticks()
{
    return __builtin_amdgcn_s_memrealtime();  // 100 MHz constant clock
}

// Block b of a grid dealt round-robin over the 8 XCDs -> logical slice, so
// that every XCD walks one contiguous 1/8 of the rows (x re-reads of the
// stencil's neighbouring planes then hit that XCD's L2). Speed only: no
// result depends on the placement.
__device__ __forceinline__ int xcd_slice(int grid)
{
    const int b = blockIdx.x;
    const int per = grid / kNumXcd;
    return (b % kNumXcd) * per + (b / kNumXcd);
}

// Same XCD ownership, each XCD's slices in reverse order: a kernel that follows
// a forward sweep starts on the rows its predecessor wrote last.
__device__ __forceinline__ int xcd_slice_rev(int grid)
{
    const int b = blockIdx.x;
    const int per = grid / kNumXcd;
    return (b % kNumXcd) * per + (per - 1 - b / kNumXcd);
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

// Whole-wave lane shifts (DPP wave_shr:1 / wave_shl:1): lane l receives lane
// l - 1 / l + 1; lane 0 / lane 63 receive 0.0 (the caller loads those itself).
__device__ __forceinline__ double wave_shr1(double v)
{
    const int lo = __double2loint(v), hi = __double2hiint(v);
    return __hiloint2double(__builtin_amdgcn_update_dpp(0, hi, 0x138, 0xF, 0xF, false),
                            __builtin_amdgcn_update_dpp(0, lo, 0x138, 0xF, 0xF, false));
}
__device__ __forceinline__ double wave_shl1(double v)
{
    const int lo = __double2loint(v), hi = __double2hiint(v);
    return __hiloint2double(__builtin_amdgcn_update_dpp(0, hi, 0x130, 0xF, 0xF, false),
                            __builtin_amdgcn_update_dpp(0, lo, 0x130, 0xF, 0xF, false));
}

// Wave sum, result valid in LANE 0 only. Fixed tree: v_l += v_{l+off} for
// off = 32, 16, 8, 4, 2, 1 (lanes >= off are don't-care).
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

// Deterministic block reduction (fixed shape): wave sums, then the wave sums
// in wave order by thread 0. Result valid in thread 0.
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

// Timer stamps (HPCCG.cpp:71-72 TICK/TOCK classes): one plain store per
// (iteration, class) slot, no allocation, so stamping adds no dependency to
// any kernel. The host orders the stamps by time (stamps_to_times).
__device__ __forceinline__ void stamp(const CgArgs& a, int k, int slot)
{
    if (k >= 0 && k <= a.max_iter) a.stamps[(size_t)k * kNumStampSlots + slot] = now_ticks();
}

// The first kernel that finds the solve finished records the end time once.
__device__ __forceinline__ void mark_end(const CgArgs& a)
{
    if (atomicCAS(&a.kst[1], 0, 1) == 0) a.stamps[(size_t)(a.max_iter + 1) * kNumStampSlots + kStampEnd] = now_ticks();
}

// HPCCG.cpp:358 loop condition for iteration k: k < max_iter && normr > tol,
// where normr is the value computed in iteration k-1, i.e. sqrt(r_{k-2}.r_{k-2})
// (sqrt(r_0.r_0) for k = 1). hist[j] = r_j.r_j is filled by the kernel that
// forms p_{j+1}; that kernel itself reads r_{k-1}.r_{k-1} from g.
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
// Row-blocked vector access: thread t owns rows 2t, 2t + 1 of its slice, so
// every vector stream is 16 B per lane.
// ---------------------------------------------------------------------------
struct Rows {
    double v[kRpt];
};

typedef double d2v __attribute__((ext_vector_type(2)));
typedef double d2u __attribute__((ext_vector_type(2), aligned(8)));

__device__ __forceinline__ Rows ld(const double* __restrict__ p)
{
    const d2v t = *reinterpret_cast<const d2v*>(p);
    return Rows{{t.x, t.y}};
}

// 8-byte aligned pair (SELL-512-A reads x at odd offsets)
__device__ __forceinline__ Rows ld_u(const double* __restrict__ p)
{
    const d2u t = *reinterpret_cast<const d2u*>(p);
    return Rows{{t.x, t.y}};
}

// Load through the constant address space: a scalar load (s_load) for a
// wave-uniform address. Only for data no kernel of the same launch writes.
template <class T>
__device__ __forceinline__ T sld(const T* p)
{
    return *(const __attribute__((address_space(4))) T*)(p);
}

// Matrix streams: non-temporal when the image is far beyond the Infinity
// Cache (read once per SpMV; keeps L2 for the vectors).
template <bool kNT>
__device__ __forceinline__ Rows ld_m(const double* __restrict__ p)
{
    if constexpr (!kNT) {
        return ld(p);
    } else {
        const d2v t = __builtin_nontemporal_load(reinterpret_cast<const d2v*>(p));
        return Rows{{t.x, t.y}};
    }
}

template <bool kNT>
__device__ __forceinline__ void ld_cols_m(const int* __restrict__ p, int (&c)[kRpt])
{
    typedef int i2v __attribute__((ext_vector_type(2)));
    const i2v t = kNT ? __builtin_nontemporal_load(reinterpret_cast<const i2v*>(p))
                      : *reinterpret_cast<const i2v*>(p);
    c[0] = t.x;
    c[1] = t.y;
}

// Vectors are allocated padded to a multiple of 512 rows, so full-width loads
// are always in bounds; rows >= n are masked on store and in the dots.
__device__ __forceinline__ void st_rows(double* __restrict__ base, int row, int n, const Rows& o)
{
    if (row + kRpt <= n) {
        *reinterpret_cast<d2v*>(base + row) = d2v{o.v[0], o.v[1]};
    } else {
        for (int i = 0; i < kRpt; i++)
            if (row + i < n) base[row + i] = o.v[i];
    }
}

// The CG vectors (Ap, p_k, r, x) as streams: non-temporal stores when
// a.nt_store, so they do not sit dirty in L2 when the kernel ends (every
// kernel boundary writes back what is dirty, ~B / 6 TB/s).
__device__ __forceinline__ void st_vec(const CgArgs& a, double* __restrict__ base, int row, const Rows& o)
{
    if (!a.nt_store) {
        st_rows(base, row, a.n, o);
    } else if (row + kRpt <= a.n) {
        __builtin_nontemporal_store(d2v{o.v[0], o.v[1]}, reinterpret_cast<d2v*>(base + row));
    } else {
        for (int i = 0; i < kRpt; i++)
            if (row + i < a.n) base[row + i] = o.v[i];
    }
}

// halo_pull: is slice s among the rows the neighbours pull from this rank's r
// (the first rsend_lo, the last rsend_hi)? Its r is stored write-through (one
// 16-B sc1 store, the rows past n masked: the ghost_hi plane follows them) and
// drained before the block's r.r partial, so a neighbour's pull -- ordered
// after this rank's r.r contribution -- reads it from memory.
__device__ __forceinline__ bool pulled_slice(const CgArgs& a, int s)
{
    return (a.rsend_lo > 0 && s * kSliceRows < a.rsend_lo) ||
           (a.rsend_hi > 0 && (s + 1) * kSliceRows > a.n - a.rsend_hi);
}
__device__ __forceinline__ void st_r_through(const CgArgs& a, int row, const Rows& o)
{
    if (row + kRpt <= a.n) {
        const d2v v = {o.v[0], o.v[1]};
        asm volatile("global_store_dwordx4 %0, %1, off sc1" : : "v"(a.r + row), "v"(v) : "memory");
    } else {
        for (int i = 0; i < kRpt; i++)
            if (row + i < a.n) asm volatile("global_store_dwordx2 %0, %1, off sc1" : : "v"(a.r + row + i), "v"(o.v[i]) : "memory");
    }
}

// p of iteration k lives in ring buffer k % nring: the update of p reads
// p_{k-1} from the previous buffer, and with x deferral the last nring p's
// stay available for the batched x update.
__device__ __forceinline__ double* cur_p(const CgArgs& a, int k)
{
    return a.p + (size_t)(k % a.nring) * (size_t)a.pstride;
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
// Folded (fold_of): completed inside the producing kernel through
// self-validating slots. Every partial and group-sum slot holds kSlotEmpty (a
// NaN payload no arithmetic produces) until its value is stored. Producers
// store their partial with an agent-scope (sc1) store and leave -- no drain,
// no atomic. The group's member with the largest block index, i.e. the one
// dispatched last (group_last_unit), waits for the group's slots to fill, sums
// them, resets them to empty and stores the group sum; the group whose last
// member has the largest block index of all (top_group) then waits for every
// group sum and forms the total. A waiter only waits for blocks dispatched
// before it (dispatch is in block order on every XCD), so the wait always ends.
// Otherwise k_finalize computes the same two levels in a separate launch (and
// resets the slots). Same shape every way: bitwise the same total.
// (An arrival-ticket completion -- atomics, a drain per block -- lost: the
// ticket's round trip made every block of the short 100^3 update kernel wait,
// 10.3 -> 23.6 us; it served only the dropped eager halo overlap and is gone.)
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

__device__ __forceinline__ int ld_sc1_i(const int* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1_i(int* p, int v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ int ngroups_of(const CgArgs& a) { return (a.nslices + kGroup - 1) / kGroup; }

// Slot layout: each dot has its own slice-partial slots (p.Ap, then r.r) and
// its own group sums after both. The fused update completes both dots in one
// launch: with separate ranges no slot is reused within a launch, so a
// waiter's resets need no drain before it publishes (they only have to land
// before the next launch, which the kernel boundary guarantees). This is the
// one invariant the slot completion relies on; round 3's drains before each
// publish cost the 100^3 fused launch ~1 us on its critical path
// (profiles/r04_carry/ab100_drains.log) and are gone.
__device__ __forceinline__ double* slice_slots(const CgArgs& a, int which) { return a.partial + which * a.nslices; }
__device__ __forceinline__ double* group_slots(const CgArgs& a, int which, int ng)
{
    return a.partial + 2 * a.nslices + which * ng;
}

__device__ __forceinline__ bool slot_full(double v) { return __double_as_longlong(v) != (long long)kSlotEmpty; }
__device__ __forceinline__ double slot_empty() { return __longlong_as_double((long long)kSlotEmpty); }

// Every in-kernel wait is bounded (HIP promises no dispatch order; the slot
// protocol below relies on the order observed on gfx950). Called after a
// failed poll, wave-uniform: true once another waiter has given up (the solve
// is void, leave at once) or this wait has outlived a.spin_ticks.
// The iteration state as the waits see it: derived from a.partial, which every
// waiter holds anyway (a.kst would be one more live register pair).
__device__ __forceinline__ int* kst_of(const CgArgs& a) { return reinterpret_cast<int*>(a.partial - kKstDoubles); }

__device__ __forceinline__ bool wait_expired(const CgArgs& a, unsigned& t0)
{
    const int* err = kst_of(a) + kErrBase;
    if (ld_sc1_i(err) != kErrNone) return true;
    const unsigned t = (unsigned)now_ticks() | 1u;  // 32 bits of the 100 MHz clock (42 s wrap), never 0
    if (t0 == 0) {
        t0 = t;
        return false;
    }
    return t - t0 > (unsigned)err[kErrBudget];
}

// One lane: record the first failed wait and end the solve. k >= max_iter
// fails every later loop test, and the iteration's published run flag is
// cleared so the kernels that follow this launch in the same iteration (the
// unfused update, k_finalize) do nothing either. The host reads err after the
// solve (HPCCG_HIP_EHIP) and empties every slot before the next one.
__device__ __forceinline__ void abort_solve(const CgArgs& a, int code, int slot, int k, int which)
{
    int* const kst = kst_of(a);
    int* const err = kst + kErrBase;
    int none = kErrNone;  // relaxed: the record is read by the host after the solve
    if (__hip_atomic_compare_exchange_strong(err, &none, code, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT)) {
        st_sc1_i(err + 1, (int)blockIdx.x);
        st_sc1_i(err + 2, slot);
        st_sc1_i(err + 3, k);
        st_sc1_i(err + 4, which);
    }
    st_sc1_i(kst + 0, a.max_iter);
    st_sc1_i(kst + 2, a.max_iter);
    st_sc1_i(kst + 5, 0);
}

// How a launch deals its units (slices, or slice pairs: spu slices per unit)
// to blocks: unit u = the x-th XCD eighth's i-th unit, run by block
// kNumXcd * i + x (xcd_slice), or kNumXcd * (per - 1 - i) + x (xcd_slice_rev).
struct UnitMap {
    int units, per, spu;
    bool rev;
};
__host__ __device__ constexpr int min_i(int a, int b) { return a < b ? a : b; }
__host__ __device__ __forceinline__ int unit_block(const UnitMap& m, int u)
{
    const int x = u / m.per, i = u % m.per;
    return kNumXcd * (m.rev ? m.per - 1 - i : i) + x;
}
// Within one eighth the block index is monotone in u, so the largest is at an
// end of the group or of an eighth inside it.
__host__ __device__ __forceinline__ int group_last_unit(const UnitMap& m, int g)
{
    const int upg = kGroup / m.spu;
    const int u0 = g * upg, u1 = min_i(m.units, u0 + upg) - 1;
    int best = u0, bb = unit_block(m, u0);
    auto cand = [&](int u) {
        if (u >= u0 && u <= u1) {
            const int b = unit_block(m, u);
            if (b > bb) bb = b, best = u;
        }
    };
    cand(u1);
    for (int c = u0 / m.per + 1; c * m.per <= u1; c++) {
        cand(c * m.per - 1);
        cand(c * m.per);
    }
    return best;
}
__host__ __device__ __forceinline__ int top_group(const UnitMap& m)
{
    int best = 0, bb = -1;
    for (int c = 0; c < kNumXcd && c * m.per < m.units; c++) {
        const int us[2] = {c * m.per, min_i(m.units - 1, c * m.per + m.per - 1)};
        for (int u : us) {
            const int b = unit_block(m, u);
            if (b > bb) bb = b, best = u;
        }
    }
    return best * m.spu / kGroup;
}


// The same fixed top-level shape computed by one wave (virtual waves in order);
// valid in lane 0. ld(i) reads group sum i. All loads are issued before the sums.
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

// The same sum from values already polled (ng <= kTopThreads: lane l of chunk
// c holds group c * kWave + l in w[c]): top_sum_wave's exact operations,
// without loading the group sums a second time after the poll that found them
// all full (one round trip less on the dot's critical path).
constexpr int kTopChunks = kTopThreads / kWave;
__device__ __forceinline__ double top_sum_polled(const double (&w)[kTopChunks], int ng, int lane)
{
    double v[kTopChunks];
#pragma unroll
    for (int vw = 0; vw < kTopChunks; vw++) {
        v[vw] = 0.0;
        const double t = vw * kWave + lane < ng ? w[vw] : 0.0;
        if (vw * kWave < ng) v[vw] += t;
    }
    double s = 0.0;
#pragma unroll
    for (int vw = 0; vw < kTopChunks; vw++) s += wave_sum(v[vw]);
    return s;
}

// Peer-memory all-reduce of one CG scalar (MPI_Allreduce in ddot.cpp:79-80),
// one lane: this rank's local sum into slot [which][k & 1][prank] of every
// rank's mailbox (system-scope stores: the mailboxes of other GPUs are
// IPC-mapped), then -- bounded -- until all pranks slots of its own mailbox
// are full, and the sum in rank order from 0.0 (k_group_sum's order: bitwise
// the in-process group's all-reduce), summed from the poll that found them
// all full (no second round trip). Its slots are emptied for iteration k + 2,
// the next user of this parity; a rank writes them again only after it has
// this rank's contribution to iteration k + 1 of the same dot, which a later
// launch stores (each dot's all-reduce runs once per launch), and a launch's
// stores have landed when it ends: so no drain after the reset, except where
// one kernel runs several rounds of one dot (drain: the self-test).
// Returns NaN when the wait gave up (the solve is void then).
__device__ __forceinline__ double peer_allreduce(const CgArgs& a, double s, int which, int k, bool drain = false)
{
    const int base = (which * 2 + (k & 1)) * kMboxRanks;
    for (int q = 0; q < a.pranks; q++)
        __hip_atomic_store(a.peers[q] + base + a.prank, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    double* const mb = a.mbox + base;
    unsigned t0 = 0, polls = 0;
    double tot;
    for (;;) {
        bool full = true;
        tot = 0.0;
        for (int q = 0; q < a.pranks; q++) {
            const double v = __hip_atomic_load(mb + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            full = full && slot_full(v);
            tot += v;
        }
        if (full) break;
        if ((++polls & 15) == 0 && wait_expired(a, t0)) {
            abort_solve(a, kErrPeerWait, which * 2 + (k & 1), k, which);
            return __longlong_as_double(0x7FF8000000000000ll);
        }
        __builtin_amdgcn_s_sleep(1);
    }
    for (int q = 0; q < a.pranks; q++)
        __hip_atomic_store(mb + q, slot_empty(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (drain) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return tot;
}

// Group fold (CgArgs::gfw, the last member of a phase of an in-process group
// run in member order): every other member's launch of this phase has ended,
// so their local totals are final; summed in rank order from 0.0 (k_group_sum's
// sum) and stored into every member's g. Not inlined: one lane of one block
// runs it, and inlined it cost the direct kernel a VGPR and a spill.
// r.r also goes to the parity slot iteration k + 1 reads (a member that runs
// the fused update reads it there; harmless for the others).
__device__ __noinline__ double group_fold_sum(double* const* gtab, int gn, int grank, double s, int which, int k)
{
    double v = 0.0;
    for (int q = 0; q < gn; q++) v += q == grank ? s : gtab[q][which];
    for (int q = 0; q < gn; q++) {
        gtab[gn + q][which] = v;
        if (which == kRR) gtab[gn + q][kRRPar + ((k + 1) & 1)] = v;
    }
    return v;
}

// The local total of a dot is known: publish it (k = the iteration it belongs
// to). r.r closes iteration k: the next iteration is k + 1.
// stamp_fin: the folded completion stamps the DDOT class here (k_finalize
// stamps it when it starts).
__device__ __forceinline__ void finish_dot(const CgArgs& a, double s, int which, int k, bool stamp_fin = true)
{
    a.loc[which] = s;
    if (a.peer_ar) {  // the global sum, in this kernel (the all-reduce class starts here)
        stamp(a, k, which == kRR ? kStampArRR : kStampArPAP);
        s = peer_allreduce(a, s, which, k);
        a.g[which] = s;
    } else if (!a.allreduce) {
        a.g[which] = s;
    } else if (a.gfw & (which == kPAP ? 1 : 2)) {
        s = group_fold_sum(a.gtab, a.gn, a.grank, s, which, k);
    }
    // the r.r iteration k + 1 reads, by its parity (fused update: kRRPar)
    if (which == kRR && a.fupd) a.g[kRRPar + ((k + 1) & 1)] = s;
    // (write-through: an in-launch pull's blocks on other XCDs wait for it)
    if (which == kRR) st_sc1_i(a.kst + (a.fupd && ((k + 1) & 1) ? 2 : 0), k + 1);
    if (a.fupd) {  // one copy per XCD group of update blocks, 128 B apart (no single hot line)
        for (int j = 0; j < kNumXcd; j++)
            st_sc1(a.pready + kReadyStride * j, which == kPAP ? s : slot_empty());  // p.Ap: the update blocks
                                                                                       // wait for it; r.r: all read it
    }
    if (stamp_fin) stamp(a, k, which == kRR ? kStampFinRR : kStampFinPAP);
    // the local sum is done, the all-reduce comes next (t4 class)
    if (a.allreduce) stamp(a, k, which == kRR ? kStampArRR : kStampArPAP);
}

// Partials of slices s0 .. s0 + cnt - 1 (one group: s0 % kGroup + cnt <=
// kGroup), the partial of slice s0 + j in lane j of wave 0; called by wave 0
// only; u: this block's unit under m. Not folded: plain stores for k_finalize.
__device__ __forceinline__ void complete_dot_lanes(const CgArgs& a, const UnitMap& m, int u, int s0, int cnt, double bs,
                                                   int which, int k)
{
    const int lane = threadIdx.x;
    double* const sp = slice_slots(a, which);
    if (!fold_of(a, which)) {
        if (lane < cnt) sp[s0 + lane] = bs;
        return;
    }
    const int ng = ngroups_of(a);
    double* const gp = group_slots(a, which, ng);
    const int g = s0 / kGroup;
    const int i = g * kGroup + lane;  // the group's slot of this lane
    {
        // (a.dbg_withhold: the guard test's missing partial)
        if (lane < cnt && !(which == kPAP && s0 + lane == a.dbg_withhold - 1)) st_sc1(sp + s0 + lane, bs);
        if (u != group_last_unit(m, g)) return;
        double v;
        unsigned t0 = 0, polls = 0;
        for (;;) {  // the group's other members were dispatched before this block
            v = i < a.nslices ? ld_sc1(sp + i) : 0.0;
            if (__all(i >= a.nslices || slot_full(v))) break;
            if ((++polls & 15) == 0 && wait_expired(a, t0)) {  // every 16th failed poll
                if (lane == 0) abort_solve(a, kErrGroupWait, g, k, which);
                return;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        // the resets need no drain: each dot owns its slot range (slice_slots,
        // group_slots), so no slot is read again within this launch, and the
        // next launch starts after the kernel boundary (k_rearm at solve start)
        if (i < a.nslices) st_sc1(sp + i, slot_empty());
        v = wave_sum(v);
        if (lane == 0) st_sc1(gp + g, v);
        if (g != top_group(m)) return;
        double wp[kTopChunks] = {0.0, 0.0, 0.0, 0.0};  // (the polled group sums, ng <= kTopThreads)
        static_assert(kTopChunks == 4, "wp");
        for (int j0 = 0; j0 < ng; j0 += kWave) {  // every other group's reducer came before
            for (;;) {
                const int j = j0 + lane;
                const double w = j < ng ? ld_sc1(gp + j) : 0.0;
                if (__all(j >= ng || slot_full(w))) {
                    if (j0 == 0) wp[0] = w;
                    else if (j0 == kWave) wp[1] = w;
                    else if (j0 == 2 * kWave) wp[2] = w;
                    else if (j0 == 3 * kWave) wp[3] = w;
                    break;
                }
                if ((++polls & 15) == 0 && wait_expired(a, t0)) {
                    if (lane == 0) abort_solve(a, kErrTopWait, j0, k, which);
                    return;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        const double tot = ng <= kTopThreads ? top_sum_polled(wp, ng, lane)
                                             : top_sum_wave([gp](int j) { return ld_sc1(gp + j); }, ng, lane);
        for (int j = lane; j < ng; j += kWave) st_sc1(gp + j, slot_empty());
        if (lane == 0) finish_dot(a, tot, which, k);
    }
}

// One slice's partial, valid in thread 0 (block_sum<256> shape). Only wave 0
// takes part in the hand-off: the other waves of the block return right away.
__device__ __forceinline__ void complete_dot(const CgArgs& a, const UnitMap& m, int u, int s, double bs, int which,
                                             int k)
{
    if (threadIdx.x >= kWave) return;
    complete_dot_lanes(a, m, u, s, 1, bs, which, k);
}

// The unit maps of the SpMV launches (all units, xcd_slice over sgrid; the
// slot completion runs only on such launches) and of the update.
__device__ __forceinline__ UnitMap spmv_units(const CgArgs& a, int spu)
{
    return UnitMap{a.sn0 + a.sn1, a.sgrid / kNumXcd, spu, false};
}
__device__ __forceinline__ UnitMap update_units(const CgArgs& a)
{
    return UnitMap{a.nslices, a.grid / kNumXcd, 1, a.rev != 0};
}

// The SpMV of iteration k publishes {k, run} (kst[4..5]) for the kernels that
// follow it in the iteration (update, finalize): one 8-byte load gives them
// both, instead of k and then the history value the loop test depends on.
__device__ __forceinline__ void publish_iter(const CgArgs& a, int k, bool run)
{
    *reinterpret_cast<int2*>(a.kst + 4) = make_int2(k, run ? 1 : 0);
}
__device__ __forceinline__ bool iter_of(const CgArgs& a, int& k)
{
    const int2 v = *reinterpret_cast<const int2*>(a.kst + 4);
    k = v.x;
    return v.y != 0;
}

// The iteration a launch runs. Fused update (a.fupd): the launch's own r.r
// completion writes the next k, so k is kept in two slots by parity (kst[0]
// even, kst[2] odd; a.kpar from the host's count): no block of a launch can
// read the value its launch writes. kst[1] (end stamped) makes every later
// launch a no-op (max_iter fails the loop test).
template <bool kFU>
__device__ __forceinline__ int iter_k(const CgArgs& a)
{
    if constexpr (!kFU) {
        return a.kst[0];
    } else {
        if (a.kst[1]) return a.max_iter;
        return a.kst[a.kpar ? 2 : 0];
    }
}

// Iteration state every SpMV kernel reads first: k, and for the fused p update
// r_{k-1}.r_{k-1} and beta. Returns false when the solve has ended.
struct IterState {
    int k;
    double rr;
    double beta;
};

// kScalar: the state through the scalar cache (s_load counts on lgkmcnt, so it
// does not wait behind the early value loads on the in-order vmcnt; written by
// earlier launches only -- with the fused update the parity slots keep this
// launch's writes apart). Direct kernel timeline, 7-pt 256^3: a unit block
// spent 4.3 of its 10.1 us waiting for its vector-loaded state.
template <bool kFU>
__device__ __forceinline__ int iter_k_s(const CgArgs& a)
{
    if constexpr (!kFU) {
        return sld(a.kst);
    } else {
        if (sld(a.kst + 1)) return a.max_iter;
        return sld(a.kst + (a.kpar ? 2 : 0));
    }
}

template <bool kFuse, bool kFU = false, bool kScalar = false>
__device__ __forceinline__ bool spmv_begin(const CgArgs& a, bool prologue, IterState& st)
{
    st.k = 0;
    st.rr = 0.0;
    st.beta = 0.0;
    if (prologue) return true;
    bool run;
    if constexpr (kScalar) {
        st.k = iter_k_s<kFU>(a);
        if (kFuse) st.rr = sld(a.g + (kFU ? kRRPar + a.kpar : kRR));
        const double h1 = sld(a.hist + max(st.k - 2, 0));  // r_{k-2}.r_{k-2} (k >= 2)
        run = st.k < a.max_iter && sqrt(st.k == 1 ? (kFuse ? st.rr : sld(a.hist)) : h1) > a.tol;
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            publish_iter(a, st.k, run);
            if (kFuse && (st.k == 1 || run)) a.hist[st.k - 1] = st.rr;
            if (run)
                stamp(a, st.k, kStampSpmv);
            else
                mark_end(a);
        }
        if (kFuse && run) st.beta = (st.k == 1) ? 0.0 : st.rr / h1;
        return run;
    }
    st.k = iter_k<kFU>(a);
    if (kFuse) st.rr = a.g[kFU ? kRRPar + a.kpar : kRR];
    run = cg_run(a, st.k, kFuse, st.rr);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        publish_iter(a, st.k, run);
        if (kFuse && (st.k == 1 || run)) a.hist[st.k - 1] = st.rr;
        if (run)
            stamp(a, st.k, kStampSpmv);
        else
            mark_end(a);
    }
    if (kFuse && run) st.beta = (st.k == 1) ? 0.0 : st.rr / a.hist[st.k - 2];
    return run;
}

// ---------------------------------------------------------------------------
// Prologue: p = x + 0.0*x   (HPCCG.cpp:347, waxpby(nrow, 1.0, x, 0.0, x, p))
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_prologue_copy(CgArgs a)
{
    const int s = xcd_slice(a.grid);
    if (blockIdx.x == 0 && threadIdx.x == 0) stamp(a, 0, kStampPrologue);
    if (s >= a.nslices) return;
    const int row = s * kSliceRows + threadIdx.x * kRpt;
    const Rows xv = ld(a.x + row);
    Rows o;
#pragma unroll
    for (int i = 0; i < kRpt; i++) o.v[i] = xv.v[i] + 0.0 * xv.v[i];
    st_rows(a.p, row, a.n, o);
}

// ---------------------------------------------------------------------------
// p = r + beta*p  (HPCCG.cpp:362 for k == 1: p = r + 0*r; :366-369 otherwise)
// as its own pass: the general (SELL-512) path, whose SpMV gathers p_k.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_p_update(CgArgs a)
{
    const int k = a.kst[0];
    const double rr = a.g[kRR];
    const bool run = cg_run(a, k, true, rr);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (k == 1 || run) a.hist[k - 1] = rr;
        if (run)
            stamp(a, k, kStampPUpdate);
        else
            mark_end(a);
    }
    if (!run) return;
    const int s = xcd_slice(a.grid);
    if (s >= a.nslices) return;
    const int row = s * kSliceRows + threadIdx.x * kRpt;
    const double beta = (k == 1) ? 0.0 : rr / a.hist[k - 2];
    const Rows rv = ld(a.r + row);
    const Rows yv = (k == 1) ? rv : ld(cur_p(a, k - 1) + row);
    Rows o;
#pragma unroll
    for (int i = 0; i < kRpt; i++) o.v[i] = rv.v[i] + beta * yv.v[i];
    st_rows(cur_p(a, k), row, a.n, o);
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
        rr = a.g[kRR];
        if (!cg_run(a, k, true, rr)) return;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) stamp(a, k, kStampHalo);  // halo class from here
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

// SpMV launches cover up to two slice (or pair) ranges ([s0, s0 + n0) then
// [s1, s1 + n1)): all, or the interior / halo-dependent units of a multi-rank
// iteration that overlaps its halo exchange. -1: no unit.
__device__ __forceinline__ int unit_of(const CgArgs& a)
{
    if ((int)blockIdx.x >= a.sgrid) return -1;  // x_defer 2: a side-flush block
    const int i = xcd_slice(a.sgrid);
    if (i >= a.sn0 + a.sn1) return -1;
    return i < a.sn0 ? a.s0 + i : a.s1 + (i - a.sn0);
}

// The epilogue every SpMV kernel shares for its two rows: store Ap; p_k
// (fused: r + beta p_{k-1}, k_p_update's expression, stored for the update's
// deferred x and the next iteration); the rows' p.Ap terms in order.
// pk (optional): the rows' p_k as the caller already holds it (the pair
// kernel's staged window; fused, the same expression, so the same bits).
template <bool kFuse, bool kFU = false>
__device__ __forceinline__ double spmv_rows_out(const CgArgs& a, const IterState& st, bool prologue, int row,
                                                const double (&sum)[kRpt], const Rows* pk = nullptr)
{
    if (kFU) {  // read by this launch's update blocks on any XCD: write-through
        // one 16-B sc1 store (rows past n are padding; their holes sum to 0);
        // inline asm: the agent-scope atomic stores of st_sc1 made the
        // compiler hoist the unrolled slot loop's loads (255 VGPRs)
        const d2v v = {sum[0], sum[1]};
        if (a.nt_store)  // streamed once: keep it out of the L2 the x reads live on
            asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" : : "v"(a.Ap + row), "v"(v));
        else
            asm volatile("global_store_dwordx4 %0, %1, off sc1" : : "v"(a.Ap + row), "v"(v));
    } else {
        st_vec(a, a.Ap, row, Rows{{sum[0], sum[1]}});
    }
    if (prologue) return 0.0;  // HPCCG.cpp:351: the prologue SpMV has no p.Ap
    double* __restrict__ p = cur_p(a, st.k);
    Rows pv;
    if (pk) {
        pv = *pk;
        if constexpr (kFuse) st_vec(a, p, row, pv);
    } else if constexpr (kFuse) {
        const double* __restrict__ pold = (st.k == 1) ? a.r : cur_p(a, st.k - 1);
        const Rows rv = ld(a.r + row);
        const Rows yv = ld(pold + row);
#pragma unroll
        for (int i = 0; i < kRpt; i++) pv.v[i] = rv.v[i] + st.beta * yv.v[i];
        st_vec(a, p, row, pv);
    } else {
        pv = ld(p + row);
    }
    double d = 0.0;
#pragma unroll
    for (int i = 0; i < kRpt; i++)
        if (row + i < a.n) d += pv.v[i] * sum[i];
    return d;
}

// ---------------------------------------------------------------------------
// SpMV over SELL-512 (HPC_sparsemv.cpp:68-89) + p.Ap slice partial
// (ddot.cpp:60-73): the general path for any matrix (the gather halo plan,
// rows that are not in ascending column order, more than kAMax distinct
// offsets per slice). Slot j of a slice is a contiguous 512-entry run; x is
// gathered through L1/L2/MALL from p_k (computed by k_p_update). Padding slots
// (col -1, value 0) add +0, which never changes a row sum that starts at +0.
// ---------------------------------------------------------------------------
// ---------------------------------------------------------------------------
// x_defer 2: the deferred x update beside the SpMV. The SpMV launch of
// iteration k carries trailing blocks (index >= sgrid: dispatched last, they
// take the CUs the SpMV's last blocks leave idle) that apply x += alpha_j p_j
// for j = max(1, k - q) .. k - 1 (q = nring - 1) to the slices whose turn it
// is (s % q == k % q), in order, one rounding per term (HPCCG.cpp:383). The
// SpMV writes only ring buffer k % nring, which holds none of those p_j, and
// alpha_j (j < k) is in ahist; k_xflush applies the rest after the loop. Per
// row the same terms in the same order as every iteration's waxpby: same bits.
// kSpu: slices per block (512-thread pair kernels 2, else 1); kB: p loads in
// flight per thread, as many as the host kernel's occupancy leaves VGPRs for
// (the ring pair kernel's is set by its LDS, 2 blocks per CU: 16; the direct
// kernel keeps its own VGPR count: 8 at width 7, 4 at width 27).
// ---------------------------------------------------------------------------
__host__ __device__ constexpr int side_blocks(int nslices, int nring, int spu)
{
    return ((nslices + nring - 2) / (nring - 1) + spu - 1) / spu;
}

template <int kSpu, int kB, bool kFU = false>
__device__ __forceinline__ bool side_flush(const CgArgs& a, bool prologue)
{
    if ((int)blockIdx.x < a.sgrid || (int)blockIdx.x >= a.send) return false;
    if (prologue) return true;
    const int k = iter_k<kFU>(a);
    if (k < 2 || !cg_run(a, k, false)) return true;
    const int q = a.nring - 1;
    const int s = k % q + q * (kSpu * ((int)blockIdx.x - a.sgrid) + (int)threadIdx.x / kBlock);
    if (s >= a.nslices) return true;
    const int row = s * kSliceRows + (threadIdx.x % kBlock) * kRpt;
    // streamed once: non-temporal, so they do not displace the SpMV's window rows from L2
    Rows xn = ld_m<true>(a.x + row);
    for (int j0 = max(1, k - q); j0 < k; j0 += kB) {
        Rows pj[kB];
        double aj[kB];
#pragma unroll
        for (int b = 0; b < kB; b++) {
            const int j = min(j0 + b, k - 1);
            pj[b] = ld_m<true>(cur_p(a, j) + row);
            aj[b] = sld(a.ahist + j);  // written by earlier updates: scalar loads
        }
#pragma unroll
        for (int b = 0; b < kB; b++)
            if (j0 + b < k)
#pragma unroll
                for (int i = 0; i < kRpt; i++) xn.v[i] = xn.v[i] + aj[b] * pj[b].v[i];
    }
    if (row + kRpt <= a.n)
        __builtin_nontemporal_store(d2v{xn.v[0], xn.v[1]}, reinterpret_cast<d2v*>(a.x + row));
    else
        st_rows(a.x, row, a.n, xn);
    return true;
}

// ---------------------------------------------------------------------------
// r-halo (a.rhalo): the ghost blocks of the SpMV launch (index >= a.gbase,
// the launch's last blocks) store p_k = r + beta p_{k-1} at the ghost
// rows, k_p_update's expression on the received r planes and the p_{k-1}
// ghosts the previous launch stored (k == 1: p_1 = r + 0 r). The neighbour
// forms the same rows of its own p_k with the same expression and the same
// all-reduced beta: the same bits the reference's halo would carry
// (exchange_externals.cpp:87-126). Read as p_{k-1} by the next launch only.
// ---------------------------------------------------------------------------
// kFU: the launch's instantiation (a.fupd is set only with the direct kernel;
// a run-time choice here cost the 7-pt fused instantiation 26 VGPRs)
//
// In-launch pull (a.pull_in): once the iteration's r.r completion -- in this
// launch (fused update) or in k_update -- has published k + 1 (after the peer
// all-reduce: every rank's r_k is final, its boundary rows stored
// write-through and drained before its r.r partial, pulled_slice), the
// neighbours' boundary rows of r_k are read with system-scope loads into this
// rank's ghost rows of r, which the next launch reads (k_pull's work, without
// k_pull's launch). Nothing in this launch reads those ghost rows afterwards:
// the unit blocks read r_{k-1}'s ghosts for p_k before their p.Ap partials,
// which the r.r completion waits behind, and ghost_store's thread that reads
// a ghost row is the thread that rewrites it (same index sequence, program
// order). The neighbour overwrites its rows only after this rank's next p.Ap
// contribution, which follows this launch. bl / nbl: this block among the
// pull blocks.
// Rows [0, lo) of src_lo and [0, hi) of src_hi into dst_lo / dst_hi, block bl
// of nbl: system-scope loads (another GPU's or member's memory, stored
// write-through there), plain stores (read by the next launch).
__device__ __forceinline__ void copy_rows(const double* src_lo, double* dst_lo, int lo, const double* src_hi,
                                          double* dst_hi, int hi, int bl, int nbl)
{
    constexpr int kU = 4;  // loads in flight per thread
    const int tot = lo + hi;
    const int nth = nbl * (int)blockDim.x;
    for (int i0 = bl * (int)blockDim.x + (int)threadIdx.x; i0 < tot; i0 += kU * nth) {
        double w[kU];
#pragma unroll
        for (int u = 0; u < kU; u++) {
            const int i = i0 + u * nth;
            w[u] = i < tot ? __hip_atomic_load(i < lo ? src_lo + i : src_hi + (i - lo), __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_SYSTEM)
                           : 0.0;
        }
#pragma unroll
        for (int u = 0; u < kU; u++) {
            const int i = i0 + u * nth;
            if (i < tot) (i < lo ? dst_lo[i] : dst_hi[i - lo]) = w[u];
        }
    }
}

// kSeg: the caller may carry the group fold's segment table (k_update only:
// the fused SpMV kernel's registers stay as they are).
template <bool kSeg = false>
__device__ __forceinline__ void pull_rows(const CgArgs& a, int k, int bl, int nbl)
{
    if (k + 1 >= a.max_iter) return;  // no SpMV reads them
    const int* const slot = a.kst + ((a.fupd && ((k + 1) & 1)) ? 2 : 0);
    unsigned t0 = 0, polls = 0;
    int v;
    while ((v = ld_sc1_i(slot)) < k + 1) {
        if ((++polls & 15) == 0 && wait_expired(a, t0)) {
            if ((threadIdx.x & (kWave - 1)) == 0) abort_solve(a, kErrPullWait, bl, k, kRR);
            return;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    if (v != k + 1) return;  // the solve was aborted
    if (bl == 0 && threadIdx.x == 0) stamp(a, k + 1, kStampHalo);
    if constexpr (kSeg) {
        if (a.npseg) {
            for (int g = 0; g < a.npseg; g++)
                copy_rows(a.psegs[g].src, a.psegs[g].dst, (int)a.psegs[g].cnt, nullptr, nullptr, 0, bl, nbl);
            return;
        }
    }
    copy_rows(a.pl_src_lo, a.pl_dst_lo, a.pl_lo, a.pl_src_hi, a.pl_dst_hi, a.pl_hi, bl, nbl);
}

template <bool kFU>
__device__ __forceinline__ bool ghost_store(const CgArgs& a, bool prologue)
{
    if ((int)blockIdx.x < a.gbase) return false;
    if (prologue) return true;
    const int k = iter_k<kFU>(a);
    // fused update: this launch's r.r completion rewrites g[kRR] while ghost
    // blocks may still start (they are outside its chain): the parity slot
    const double rr = a.g[kFU ? kRRPar + a.kpar : kRR];
    if (!cg_run(a, k, true, rr)) return true;
    const double beta = (k == 1) ? 0.0 : rr / a.hist[k - 2];
    const double* __restrict__ pold = (k == 1) ? a.r : cur_p(a, k - 1);
    double* __restrict__ pk = cur_p(a, k);
    const int nlo = a.ghost_lo, tot = a.ghost_lo + a.ghost_hi;
    const int bl = (int)blockIdx.x - a.gbase, nbl = (int)gridDim.x - a.gbase;  // (the last blocks)
    for (int i = bl * (int)blockDim.x + (int)threadIdx.x; i < tot; i += nbl * (int)blockDim.x) {
        const int row = i < nlo ? i - nlo : a.n + (i - nlo);
        pk[row] = a.r[row] + beta * pold[row];
    }
    if constexpr (kFU)
        if (a.pull_in) pull_rows(a, k, bl, nbl);
    return true;
}

// ---------------------------------------------------------------------------
// Fused update (a.fupd; one rank, direct kernel): the SpMV launch of iteration
// k ends with a.grid update blocks (index a.ubase .. a.gbase - 1, dispatched
// after every unit and side block; ghost blocks follow them) that do k_update's work -- r = r - alpha Ap and the r.r
// partial (HPCCG.cpp:382-384, 367), the same expressions in the same order --
// once the launch's p.Ap total is in its self-validating slots (a.pready:
// kNumXcd copies 128 B apart, block b polls copy b mod kNumXcd, so no single
// line takes every poll). Every unit block is dispatched before them and none
// waits on them, so the wait ends. Ap comes from this launch's unit blocks on
// any XCD: stored write-through, drained (an explicit vmcnt(0) in every wave
// before the block sum) before their partials are published, read with
// agent-scope loads. r is prefetched before the wait.
// Saves the update's launch and ramp; bitwise the unfused iteration.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool fused_update(const CgArgs& a, bool prologue, unsigned long long* tw = nullptr)
{
    if ((int)blockIdx.x < a.ubase || (int)blockIdx.x >= a.gbase) return false;
    if (prologue) return true;
    const int bl = (int)blockIdx.x - a.ubase;  // a.ubase is a multiple of kNumXcd
    constexpr int spu = 2;  // two slices per update block (one measured slower: DESIGN.md 4)
    const int units = (a.nslices + spu - 1) / spu;
    const int ugrid = (units + kNumXcd - 1) / kNumXcd * kNumXcd;
    const int per = ugrid / kNumXcd;
    const int u = (bl % kNumXcd) * per + (a.rev ? per - 1 - bl / kNumXcd : bl / kNumXcd);
    if (u >= units) return true;
    const int s = u * spu;  // first slice of the unit
    const int nsl = min(spu, a.nslices - s);
    const int row = s * kSliceRows + threadIdx.x * kRpt;
    // the state through the scalar cache and r's rows (they need no state)
    // issued together: the loop test no longer holds the prefetch back (block
    // timeline, 7-pt 256^3: update blocks spent 3.5 of their 5.6 us before the
    // p.Ap total was in hand). A no-op launch after the end loads r for nothing.
    const int k = iter_k_s<true>(a);
    const double rr = sld(a.g + kRRPar + a.kpar);  // r_{k-1}.r_{k-1}: the previous launch's
    const Rows rv = ld(a.r + row);
    const Rows rv2 = nsl > 1 ? ld(a.r + row + kSliceRows) : Rows{{0.0, 0.0}};
    asm volatile("" ::: "memory");  // the prefetch stays ahead of the test
    if (k >= a.max_iter || !(sqrt(k == 1 ? rr : sld(a.hist + k - 2)) > a.tol)) return true;  // cg_run
    __shared__ double pap_s;
    __shared__ int gave_up;
    if (threadIdx.x == 0) {  // one poller per block
        double v;
        const double* slot = a.pready + kReadyStride * (bl % kNumXcd);
        unsigned t0 = 0, polls = 0;
        int bail = 0;
        while (!slot_full(v = ld_sc1(slot))) {
            if ((++polls & 15) == 0 && wait_expired(a, t0)) {
                abort_solve(a, kErrReadyWait, bl % kNumXcd, k, kPAP);
                bail = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(8);
        }
        pap_s = v;
        gave_up = bail;
    }
    __syncthreads();
    if (gave_up) return true;
    if (tw && threadIdx.x == 0) *tw = now_ticks();  // diagnostics (the timeline instantiation)
    const double alpha = rr / pap_s;
    if (bl == 0 && threadIdx.x == 0) {
        a.ahist[k] = alpha;
        stamp(a, k, kStampUpdate);
    }
    // one 16-B agent-coherent load (sc1: not served by a stale L2 line); the
    // compiler does not count an asm load, so its wait is explicit
    d2v apw, apw2 = {0.0, 0.0};
    if (nsl > 1)
        asm volatile("global_load_dwordx4 %0, %2, off sc1\n\tglobal_load_dwordx4 %1, %3, off sc1\n\t"
                     "s_waitcnt vmcnt(0)"
                     : "=&v"(apw), "=&v"(apw2) : "v"(a.Ap + row), "v"(a.Ap + row + kSliceRows) : "memory");
    else
        asm volatile("global_load_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(apw) : "v"(a.Ap + row) : "memory");
    // each slice exactly as k_update forms it: r, its partial with block_sum<256>'s shape
    // (wave sums, then the four in wave order), both slices through one barrier
    const bool wt = pulled_slice(a, s) || (nsl > 1 && pulled_slice(a, s + 1));  // (block-uniform)
    auto slice = [&](const Rows& r_, const d2v& ap_, int rw) -> double {
        Rows rn;
        rn.v[0] = r_.v[0] + (-alpha) * ap_.x;
        rn.v[1] = r_.v[1] + (-alpha) * ap_.y;
        if (wt)
            st_r_through(a, rw, rn);
        else
            st_vec(a, a.r, rw, rn);
        double d = 0.0;
#pragma unroll
        for (int i = 0; i < kRpt; i++)
            if (rw + i < a.n) d += rn.v[i] * rn.v[i];
        return wave_sum(d);
    };
    __shared__ double ws2[2][kBlock / kWave];
    const double wa = slice(rv, apw, row);
    const double wb = nsl > 1 ? slice(rv2, apw2, row + kSliceRows) : 0.0;
    const int lane = threadIdx.x & (kWave - 1);
    if (lane == 0) {
        ws2[0][threadIdx.x / kWave] = wa;
        ws2[1][threadIdx.x / kWave] = wb;
    }
    if (wt) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (pulled rows landed before the partial)
    __syncthreads();
    if (threadIdx.x >= kWave) return true;
    double bsj = 0.0;  // lane j: slice s + j's partial
    if (lane < 2) {
#pragma unroll
        for (int i = 0; i < kBlock / kWave; i++) bsj += ws2[lane][i];
    }
    complete_dot_lanes(a, UnitMap{units, per, spu, a.rev != 0}, u, s, nsl, bsj, kRR, k);
    return true;
}

template <bool kNT>
__global__ __launch_bounds__(kBlock) void k_spmv_sell(CgArgs a, bool prologue)
{
    IterState st;
    if (!spmv_begin<false>(a, prologue, st)) return;
    const int s = unit_of(a);
    if (s < 0) return;
    const double* __restrict__ x = cur_p(a, st.k) - a.ghost_lo;  // local columns include the ghosts
    const size_t base = (size_t)a.slice_base[s] * kSliceRows + (size_t)threadIdx.x * kRpt;
    const int w = (int)(a.slice_base[s + 1] - a.slice_base[s]);
    const double* __restrict__ vp = a.vals + base;
    const int* __restrict__ cp = a.cols + base;
    double sum[kRpt] = {0.0, 0.0};
#pragma unroll 3
    for (int j = 0; j < w; j++) {
        int c[kRpt];
        ld_cols_m<kNT>(cp + (size_t)j * kSliceRows, c);
        const Rows v = ld_m<kNT>(vp + (size_t)j * kSliceRows);
#pragma unroll
        for (int i = 0; i < kRpt; i++) {
            const double xv = (c[i] >= 0) ? x[c[i]] : 0.0;
            sum[i] = sum[i] + v.v[i] * xv;
        }
    }
    const int row = s * kSliceRows + threadIdx.x * kRpt;
    const double d = spmv_rows_out<false>(a, st, prologue, row, sum);
    if (prologue) return;
    const double bs = block_sum<kBlock>(d);
    complete_dot(a, spmv_units(a, 1), s, s, bs, kPAP, st.k);
}

// ---------------------------------------------------------------------------
// SELL-512-A SpMV, x read directly: slot j of slice s holds, for every row,
// the entry at the slice's j-th smallest offset (0.0 where the row has none:
// a hole); x of row i's slot j is at p + i + aoff[s][j], one 16-B load per
// thread and slot. Holes read x inside the zeroed guard zones around every p
// buffer and r, or at a real neighbour; 0.0 * finite adds +-0 and never
// changes the sum. kW > 0: uniform width, slot loop unrolled, the first kPre
// value slots and the offsets loaded before the iteration test. kFuse (single
// rank, never the prologue): x = r + beta*p_{k-1} formed per load, k_p_update's
// exact expression, so every row sum is unchanged.
// ---------------------------------------------------------------------------
// Triple plan of the 7-point width: slot groups in slot order -- z-, y-, the
// x triple (offsets -1, 0, +1), y+, z+. A slice whose offsets group exactly so
// (atri[s], checked on the host) reads x once for the triple: its centre pair,
// the neighbours' rows from the adjacent lanes (wave_shr1 / wave_shl1), lanes
// 0 and 63 loading their one outside value. Same x values, same products,
// same order: same bits. 7-pt 256^3 same-process A/B: 2679 vs 2641 it/s. (The
// 27-wide plan, nine triples, needs 83+ VGPRs and measured 52 vs 45 us at 100^3.)
__host__ __device__ constexpr int tri_groups(int w) { return w == 7 ? 5 : 0; }
__host__ __device__ constexpr int tri_first(int w, int g) { return g <= 2 ? g : g + 2; }
__host__ __device__ constexpr int tri_size(int w, int g) { return g == 2 ? 3 : 1; }

// Block timeline of the direct kernel (dbg_timeline, the kTL instantiations
// of the 100^3 and 7-pt defaults): per block of the launch, kTlWords words --
// block | HW_ID << 32, entry, state read (unit) / p.Ap ready (update block),
// slot loop done (unit), end, role (0 unit, 1 side, 2 ghost, 3 update), XCC.
// Each stamp is stored when it is taken, by every lane to the same word (one
// store, no branch) through an asm store the compiler does not treat as a
// memory operation: the diagnostic then holds no register across the kernel
// and moves no load (a plain store, or a branch around it, cost occupancy
// steps: 77 -> 255 VGPRs). No-op launches leave rows half written: read it
// after an eager solve.
__device__ __forceinline__ void tl_stamp(const CgArgs& a, int word)
{
    const unsigned long long t = now_ticks();
    asm volatile("global_store_dwordx2 %0, %1, off" : : "v"(a.dbg_tl + (size_t)blockIdx.x * kTlWords + word), "v"(t));
}
__device__ __forceinline__ void tl_end(const CgArgs& a, int role)
{
    if (threadIdx.x != 0) return;
    unsigned long long* o = a.dbg_tl + (size_t)blockIdx.x * kTlWords;
    o[4] = now_ticks();
    o[0] = (unsigned long long)blockIdx.x |
           ((unsigned long long)__builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11)) << 32);  // HW_ID
    o[5] = (unsigned long long)role;
    o[6] = __builtin_amdgcn_s_getreg(20 | (0 << 6) | (15 << 11));  // XCC_ID
}

template <int kW, bool kNT, bool kFuse, int kPre, bool kTri = false, bool kFU = false, bool kTL = false>
__global__ __launch_bounds__(kBlock) void k_spmv_a(CgArgs a, bool prologue)
{
    static_assert(kPre == 0 || (kW > 0 && kPre <= kW), "early loads need the uniform width");
    const int s = unit_of(a);
    constexpr int kP = kPre > 0 ? kPre : 1;
    Rows vpre[kP];
    int offp[kPre > 0 ? kW : 1];
    if constexpr (kPre > 0) {
        if (s >= 0) {
            const double* __restrict__ vp0 = a.aval + (size_t)s * kW * kSliceRows + (size_t)threadIdx.x * kRpt;
#pragma unroll
            for (int j = 0; j < kPre; j++) vpre[j] = ld_m<kNT>(vp0 + (size_t)j * kSliceRows);
#pragma unroll
            for (int j = 0; j < kW; j++) offp[j] = a.aoff[(size_t)s * kAMax + j];
        }
    }
    if constexpr (kTL) tl_stamp(a, 1);  // entry (after the early loads: before them it cost 24 VGPRs)
    if constexpr (kFU && kTL) {
        if (fused_update(a, prologue, a.dbg_tl + (size_t)blockIdx.x * kTlWords + 2)) {
            tl_end(a, 3);
            return;
        }
    } else if constexpr (kFU) {
        if (fused_update(a, prologue)) return;
    }
    if (side_flush<1, kW == 7 ? 8 : 4, kFU>(a, prologue)) {
        if constexpr (kTL) tl_end(a, 1);
        return;
    }
    if (ghost_store<kFU>(a, prologue)) {
        if constexpr (kTL) tl_end(a, 2);
        return;
    }
    IterState st;
    if (!spmv_begin<kFuse, kFU, true>(a, prologue, st)) return;
    if (s < 0) return;
    if constexpr (kTL) tl_stamp(a, 2);
    const int wdt = kW > 0 ? kW : (int)(a.abase[s + 1] - a.abase[s]);
    const int row = s * kSliceRows + threadIdx.x * kRpt;
    const double* __restrict__ xr = cur_p(a, st.k) + row;  // x of column row + off at xr[off]
    const double* __restrict__ rr_ = a.r + row;
    const double* __restrict__ py = rr_;
    if constexpr (kFuse) py = ((st.k == 1) ? a.r : cur_p(a, st.k - 1)) + row;
    const size_t vb = kW > 0 ? (size_t)s * kW : (size_t)a.abase[s];
    const double* __restrict__ vp = a.aval + vb * kSliceRows + (size_t)threadIdx.x * kRpt;
    const int* __restrict__ off = a.aoff + (size_t)s * kAMax;
    double sum[kRpt] = {0.0, 0.0};
    if constexpr (kTri && tri_groups(kW) > 0 && kPre > 0) {
        if (a.atri[s]) {
            auto xpair = [&](int o) -> Rows {
                if constexpr (kFuse) {
                    const Rows rv = ld_u(rr_ + o);
                    const Rows yv = ld_u(py + o);
                    return Rows{{rv.v[0] + st.beta * yv.v[0], rv.v[1] + st.beta * yv.v[1]}};
                } else {
                    return ld_u(xr + o);
                }
            };
            auto x1 = [&](int o) -> double {
                if constexpr (kFuse)
                    return rr_[o] + st.beta * py[o];
                else
                    return xr[o];
            };
            auto val = [&](int j) -> Rows { return j < kPre ? vpre[j] : ld_m<kNT>(vp + (size_t)j * kSliceRows); };
            const int lane = threadIdx.x & (kWave - 1);
            Rows ctr{{0.0, 0.0}};  // the triple's centre pair: x at the rows themselves when its offset is 0
            auto triple = [&](const Rows& v0, const Rows& v1, const Rows& v2, int o) {
                const Rows c = xpair(o);
                ctr = c;
                double left = wave_shr1(c.v[1]);
                double right = wave_shl1(c.v[0]);
                if (lane == 0) left = x1(o - 1);
                if (lane == kWave - 1) right = x1(o + 2);
                sum[0] = sum[0] + v0.v[0] * left;
                sum[1] = sum[1] + v0.v[1] * c.v[0];
                sum[0] = sum[0] + v1.v[0] * c.v[0];
                sum[1] = sum[1] + v1.v[1] * c.v[1];
                sum[0] = sum[0] + v2.v[0] * c.v[1];
                sum[1] = sum[1] + v2.v[1] * right;
            };
#pragma unroll
            for (int g = 0; g < tri_groups(kW); g++) {
                const int j0 = tri_first(kW, g);
                if (tri_size(kW, g) == 1) {
                    const Rows v = val(j0);
                    const Rows xv = xpair(offp[j0]);
#pragma unroll
                    for (int i = 0; i < kRpt; i++) sum[i] = sum[i] + v.v[i] * xv.v[i];
                } else {
                    triple(val(j0), val(j0 + 1), val(j0 + 2), offp[j0 + 1]);
                }
            }
            if constexpr (kTL) tl_stamp(a, 3);
            // the rows' p_k is the triple's centre (offset 0: the same expression,
            // so the same bits): no second read of r and p_{k-1} for the epilogue
            constexpr int kCtr = tri_first(kW, 2) + 1;
            const double d = offp[kCtr] == 0 ? spmv_rows_out<kFuse, kFU>(a, st, prologue, row, sum, &ctr)
                                             : spmv_rows_out<kFuse, kFU>(a, st, prologue, row, sum);
            if (prologue) return;
            if constexpr (kFU) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // Ap landed before the partial
            const double bs = block_sum<kBlock>(d);
            complete_dot(a, spmv_units(a, 1), s, s, bs, kPAP, st.k);
            if constexpr (kTL) tl_end(a, 0);
            return;
        }
    }
#pragma unroll kW > 0 ? kW : 4
    for (int j = 0; j < wdt; j++) {
        Rows v;
        int oj;
        if constexpr (kPre > 0) {
            v = j < kPre ? vpre[j] : ld_m<kNT>(vp + (size_t)j * kSliceRows);
            oj = offp[j];
        } else {
            v = ld_m<kNT>(vp + (size_t)j * kSliceRows);
            oj = off[j];
        }
        Rows xv;
        if constexpr (kFuse) {
            const Rows rv = ld_u(rr_ + oj);
            const Rows yv = ld_u(py + oj);
#pragma unroll
            for (int i = 0; i < kRpt; i++) xv.v[i] = rv.v[i] + st.beta * yv.v[i];
        } else {
            xv = ld_u(xr + oj);
        }
#pragma unroll
        for (int i = 0; i < kRpt; i++) sum[i] = sum[i] + v.v[i] * xv.v[i];
    }
    if constexpr (kTL) tl_stamp(a, 3);
    const double d = spmv_rows_out<kFuse, kFU>(a, st, prologue, row, sum);
    if (prologue) return;
    // fused update: this wave's write-through Ap has landed before the block's
    // partial can be published (the update blocks read it once the p.Ap total
    // is out); explicit, not left to how __syncthreads() lowers
    if constexpr (kFU) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const double bs = block_sum<kBlock>(d);
    complete_dot(a, spmv_units(a, 1), s, s, bs, kPAP, st.k);
    if constexpr (kTL) tl_end(a, 0);
}

// ---------------------------------------------------------------------------
// Resident fused update (option resident_update; one rank, direct kernel,
// width 27): one 256-thread block per slice PAIR, four
// rows per thread -- rows 2t, 2t + 1 of each slice, the direct kernel's rows,
// both slices' loads interleaved in one slot loop -- and every unit block
// resident at once (the host sizes the launch to the chip: hipOccupancy x
// CUs >= units, else this kernel is not used). A block keeps its rows' Ap
// and the r it read for p_k in registers, publishes its two p.Ap partials,
// waits for the launch's p.Ap total (the pready slots the dot completion
// fills) and applies the update itself: no Ap stream (stored, then read back
// by update blocks) and no second read of r -- 24 B per row less than the
// unit + update-block launch. Same expressions in the same order as the
// direct kernel and fused_update (HPCCG.cpp:377-385): the same bits. The side
// blocks (deferred x) trail the units as in every direct launch.
// Co-residency is not promised by HIP: a launch that could not fit (another
// process on the GPU) ends in the bounded pready wait, an error, not a hang.
// ---------------------------------------------------------------------------
// 4 blocks per CU (4 waves per SIMD, <= 128 VGPRs): 1024 resident blocks, the
// 977 pair units of 100^3 fit at once.
template <bool kNT, int kPre = 3, int kStep = 2>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_spmv_ar(CgArgs a,
                                                                                                  bool prologue)
{
    constexpr int kW = 27;  // kPre early slots, then kW - kPre slots in steps of kStep, a step's loads issued first
    static_assert((kW - kPre) % kStep == 0, "slot steps");
    if (side_flush<1, 4, true>(a, prologue)) return;
    const int P = unit_of(a);
    IterState st;
    if (!spmv_begin<true, true, true>(a, prologue, st)) return;
    if (P < 0) return;
    const int s0 = 2 * P;
    const int nsl = min(2, a.nslices - s0);
    const int s1 = nsl > 1 ? s0 + 1 : s0;  // (an odd last slice: its twin repeats it, masked below)
    const int lr = threadIdx.x * kRpt;     // row within each slice
    const int row0 = s0 * kSliceRows + lr, row1 = s1 * kSliceRows + lr;
    const double* __restrict__ vp0 = a.aval + (size_t)s0 * kW * kSliceRows + lr;
    const double* __restrict__ vp1 = a.aval + (size_t)s1 * kW * kSliceRows + lr;
    Rows pre0[kPre], pre1[kPre];
#pragma unroll
    for (int j = 0; j < kPre; j++) {
        pre0[j] = ld_m<kNT>(vp0 + (size_t)j * kSliceRows);
        pre1[j] = ld_m<kNT>(vp1 + (size_t)j * kSliceRows);
    }
    const int* __restrict__ off0 = a.aoff + (size_t)s0 * kAMax;
    const int* __restrict__ off1 = a.aoff + (size_t)s1 * kAMax;
    const double* __restrict__ r0 = a.r + row0;
    const double* __restrict__ r1 = a.r + row1;
    const double* __restrict__ pold = (st.k == 1) ? a.r : cur_p(a, st.k - 1);
    const double* __restrict__ y0 = pold + row0;
    const double* __restrict__ y1 = pold + row1;
    double sum0[kRpt] = {0.0, 0.0}, sum1[kRpt] = {0.0, 0.0};
    // one slot of both slices: x = r + beta p_{k-1} at the offset, in slot order
    auto slot = [&](const Rows& v0, const Rows& v1, const Rows& ra, const Rows& ya, const Rows& rb, const Rows& yb) {
#pragma unroll
        for (int i = 0; i < kRpt; i++) {
            sum0[i] = sum0[i] + v0.v[i] * (ra.v[i] + st.beta * ya.v[i]);
            sum1[i] = sum1[i] + v1.v[i] * (rb.v[i] + st.beta * yb.v[i]);
        }
    };
#pragma unroll
    for (int j = 0; j < kPre; j++) {
        const int o0 = sld(off0 + j), o1 = sld(off1 + j);
        slot(pre0[j], pre1[j], ld_u(r0 + o0), ld_u(y0 + o0), ld_u(r1 + o1), ld_u(y1 + o1));
    }
#pragma unroll 1
    for (int j0 = kPre; j0 < kW; j0 += kStep) {
        Rows v0[kStep], v1[kStep], ra[kStep], ya[kStep], rb[kStep], yb[kStep];
#pragma unroll
        for (int u = 0; u < kStep; u++) {
            const int o0 = sld(off0 + j0 + u), o1 = sld(off1 + j0 + u);
            v0[u] = ld_m<kNT>(vp0 + (size_t)(j0 + u) * kSliceRows);
            v1[u] = ld_m<kNT>(vp1 + (size_t)(j0 + u) * kSliceRows);
            ra[u] = ld_u(r0 + o0);
            ya[u] = ld_u(y0 + o0);
            rb[u] = ld_u(r1 + o1);
            yb[u] = ld_u(y1 + o1);
        }
#pragma unroll
        for (int u = 0; u < kStep; u++) slot(v0[u], v1[u], ra[u], ya[u], rb[u], yb[u]);
    }
    // p_k at the rows (k_p_update's expression), kept with r for the update
    const Rows rv0 = ld(a.r + row0), rv1 = ld(a.r + row1);
    const Rows yv0 = ld(pold + row0), yv1 = ld(pold + row1);
    Rows pk0, pk1;
#pragma unroll
    for (int i = 0; i < kRpt; i++) {
        pk0.v[i] = rv0.v[i] + st.beta * yv0.v[i];
        pk1.v[i] = rv1.v[i] + st.beta * yv1.v[i];
    }
    double* __restrict__ p = cur_p(a, st.k);
    st_vec(a, p, row0, pk0);
    if (nsl > 1) st_vec(a, p, row1, pk1);
    double d0 = 0.0, d1 = 0.0;
#pragma unroll
    for (int i = 0; i < kRpt; i++) {
        if (row0 + i < a.n) d0 += pk0.v[i] * sum0[i];
        if (nsl > 1 && row1 + i < a.n) d1 += pk1.v[i] * sum1[i];
    }
    // the two slices' p.Ap partials with block_sum<256>'s shape
    __shared__ double ws2[2][kBlock / kWave];
    __shared__ double pap_s;
    __shared__ int gave_up;
    const int lane = threadIdx.x & (kWave - 1);
    const double w0 = wave_sum(d0), w1 = wave_sum(d1);
    if (lane == 0) {
        ws2[0][threadIdx.x / kWave] = w0;
        ws2[1][threadIdx.x / kWave] = w1;
    }
    __syncthreads();
    if (threadIdx.x < kWave) {
        double bsj = 0.0;  // lane j: slice s0 + j's partial
        if (lane < 2) {
#pragma unroll
            for (int i = 0; i < kBlock / kWave; i++) bsj += ws2[lane][i];
        }
        complete_dot_lanes(a, spmv_units(a, 2), P, s0, nsl, bsj, kPAP, st.k);
    }
    // the launch's p.Ap total (every unit block is resident: no wait depends
    // on a block that has not started)
    if (threadIdx.x == 0) {
        double v;
        const double* slot = a.pready + kReadyStride * (blockIdx.x % kNumXcd);
        unsigned t0 = 0, polls = 0;
        int bail = 0;
        // (dbg_resident_stall: the wait of a launch that could not be resident)
        while (!slot_full(v = ld_sc1(slot)) || a.dbg_resident_stall) {
            if ((++polls & 15) == 0 && wait_expired(a, t0)) {
                abort_solve(a, kErrReadyWait, blockIdx.x % kNumXcd, st.k, kPAP);
                bail = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(8);
        }
        pap_s = v;
        gave_up = bail;
    }
    __syncthreads();
    if (gave_up) return;
    const double alpha = st.rr / pap_s;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        a.ahist[st.k] = alpha;
        stamp(a, st.k, kStampUpdate);
    }
    // r = r - alpha Ap (fused_update's expression) and the r.r partials
    Rows rn0, rn1;
#pragma unroll
    for (int i = 0; i < kRpt; i++) {
        rn0.v[i] = rv0.v[i] + (-alpha) * sum0[i];
        rn1.v[i] = rv1.v[i] + (-alpha) * sum1[i];
    }
    st_vec(a, a.r, row0, rn0);
    if (nsl > 1) st_vec(a, a.r, row1, rn1);
    double e0 = 0.0, e1 = 0.0;
#pragma unroll
    for (int i = 0; i < kRpt; i++) {
        if (row0 + i < a.n) e0 += rn0.v[i] * rn0.v[i];
        if (nsl > 1 && row1 + i < a.n) e1 += rn1.v[i] * rn1.v[i];
    }
    const double x0 = wave_sum(e0), x1 = wave_sum(e1);
    __syncthreads();  // (ws2 reused)
    if (lane == 0) {
        ws2[0][threadIdx.x / kWave] = x0;
        ws2[1][threadIdx.x / kWave] = x1;
    }
    __syncthreads();
    if (threadIdx.x >= kWave) return;
    double bsj = 0.0;
    if (lane < 2) {
#pragma unroll
        for (int i = 0; i < kBlock / kWave; i++) bsj += ws2[lane][i];
    }
    complete_dot_lanes(a, spmv_units(a, 2), P, s0, nsl, bsj, kRR, st.k);
}

// ---------------------------------------------------------------------------
// Persistent CG (option resident_update 6; the k_spmv_ar setting, one launch
// per solve): after the prologue, ONE launch runs every iteration. Each pair
// block keeps its rows' x, r_{k-1} and p_{k-1} in registers (x += alpha p_k
// there: no deferred-x side blocks, x stored once at the end), and the two
// dots of every iteration complete through slots of their own (a.pslots:
// iteration k's slice partials, group sums and kPersBcast broadcast copies of the
// total, all emptied before the launch), so no slot is reused within the
// launch. Neighbour values of r_{k-1} and p_{k-1} are read with sc1 buffer
// loads (L1 bypassed: another CU rewrote them during this launch) after the
// r.r total that orders them; r_k and p_k are stored sc1 and drained by every
// wave before its block's r.r partial. r_k overwrites r_{k-1} only after the
// p.Ap total, i.e. after every block's slot loop. Same expressions in the same
// order as k_spmv_ar / the unfused kernels (HPCCG.cpp:358-385): the same bits.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void vm_wait(int n)  // n: a constant after unrolling
{
    switch (n) {
#define HPCCG_VMW(i) \
    case i: asm volatile("s_waitcnt vmcnt(" #i ")" ::: "memory"); break;
        HPCCG_VMW(0) HPCCG_VMW(1) HPCCG_VMW(2) HPCCG_VMW(3) HPCCG_VMW(4) HPCCG_VMW(5) HPCCG_VMW(6) HPCCG_VMW(7)
#undef HPCCG_VMW
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}
typedef __attribute__((address_space(3))) void lds_void;
constexpr int kCpolSc1 = 16;  // buffer instruction cache policy: sc1

__device__ __forceinline__ __amdgpu_buffer_rsrc_t vec_rsrc(const double* base)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(base), (short)0, 0x7FFFFFF0, 0x00020000);
}
__device__ __forceinline__ Rows ld_rs(__amdgpu_buffer_rsrc_t rs, int byte)
{
    const d2v t = __builtin_bit_cast(d2v, __builtin_amdgcn_raw_buffer_load_b128(rs, byte, 0, kCpolSc1));
    return Rows{{t.x, t.y}};
}
// rows >= n stay untouched (the padding rows hold zeros)
__device__ __forceinline__ void st_rs(__amdgpu_buffer_rsrc_t rs, int byte, int row, int n, const Rows& o)
{
    if (row + kRpt <= n) {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int,
                                                                  d2v{o.v[0], o.v[1]}),
                                               rs, byte, 0, kCpolSc1);
    } else {
        for (int i = 0; i < kRpt; i++)
            if (row + i < n)
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned int,
                                                                         o.v[i]),
                                                      rs, byte + 8 * i, 0, kCpolSc1);
    }
}

// Iteration k's slots: [which][nslices] partials, [which][ngroups] group sums,
// [which][kPersBcast x kReadyStride] broadcast copies of the total.
__device__ __forceinline__ double* pers_slots(const CgArgs& a, int k)
{
    return a.pslots + (size_t)(k - a.pk0) * a.pslot_stride;  // (the launch's window starts at pk0)
}
__device__ __forceinline__ double* pers_bcast(const CgArgs& a, int k, int which)
{
    const int ng = ngroups_of(a);
    return pers_slots(a, k) + 2 * a.nslices + 2 * ng + which * kPersBcast * kReadyStride;
}

// complete_dot_lanes' slot protocol on iteration k's own slots (no resets):
// wave 0, lane j holds slice s0 + j's partial.
// role: bit 0 this block waits for its group's partials, bit 1 (with bit 0)
// its group is the top group (group_last_unit / top_group, once per launch)
template <bool kMR>
__device__ __forceinline__ void pers_dot(const CgArgs& a, int role, int s0, int cnt, double bs, int which, int k)
{
    const int lane = threadIdx.x;
    double* const base = pers_slots(a, k);
    const int ng = ngroups_of(a);
    double* const sp = base + which * a.nslices;
    double* const gp = base + 2 * a.nslices + which * ng;
    const int g = s0 / kGroup;
    const int i = g * kGroup + lane;
    if (lane < cnt && !(which == kPAP && s0 + lane == a.dbg_withhold - 1)) st_sc1(sp + s0 + lane, bs);
    if (!(role & 1)) return;
    double v;
    unsigned t0 = 0, polls = 0;
    for (;;) {
        v = i < a.nslices ? ld_sc1(sp + i) : 0.0;
        if (__all(i >= a.nslices || slot_full(v))) break;
        if ((++polls & 15) == 0 && wait_expired(a, t0)) {
            if (lane == 0) abort_solve(a, kErrGroupWait, g, k, which);
            return;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    v = wave_sum(v);
    if (lane == 0) st_sc1(gp + g, v);
    if (!(role & 2)) return;
    double wp[kTopChunks] = {0.0, 0.0, 0.0, 0.0};  // (the polled group sums, ng <= kTopThreads)
    for (int j0 = 0; j0 < ng; j0 += kWave) {
        for (;;) {
            const int j = j0 + lane;
            const double w = j < ng ? ld_sc1(gp + j) : 0.0;
            if (__all(j >= ng || slot_full(w))) {
                if (j0 == 0) wp[0] = w;
                else if (j0 == kWave) wp[1] = w;
                else if (j0 == 2 * kWave) wp[2] = w;
                else if (j0 == 3 * kWave) wp[3] = w;
                break;
            }
            if ((++polls & 15) == 0 && wait_expired(a, t0)) {
                if (lane == 0) abort_solve(a, kErrTopWait, j0, k, which);
                return;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    // top_sum_wave's shape from the polled values: no second round trip
    double tot = ng <= kTopThreads ? top_sum_polled(wp, ng, lane)
                                   : top_sum_wave([gp](int j) { return ld_sc1(gp + j); }, ng, lane);
    if constexpr (kMR) {
        // several ranks: the job's total (MPI_Allreduce, ddot.cpp:79-80) -- this
        // rank's sum into every rank's mailbox, the contributions summed in rank
        // order (peer_allreduce; drained: one launch runs every iteration)
        int bad = 0;
        if (lane == 0) {
            stamp(a, k, which == kRR ? kStampArRR : kStampArPAP);
            tot = peer_allreduce(a, tot, which, k, true);
            bad = ld_sc1_i(kst_of(a) + kErrBase) != kErrNone;
        }
        if (__shfl(bad, 0, kWave)) return;  // (the solve was given up: the waiters see the error record)
    }
    tot = __shfl(tot, 0, kWave);
    for (int c = lane; c < kPersBcast; c += kWave) st_sc1(pers_bcast(a, k, which) + kReadyStride * c, tot);
    if (lane == 0) stamp(a, k, which == kRR ? kStampFinRR : kStampFinPAP);
}

// One lane per block: iteration k's total of dot `which` (bounded wait).
// Returns false when the solve was abandoned.
__device__ __forceinline__ bool pers_wait(const CgArgs& a, int k, int which, double& out, bool stall)
{
    const double* slot = pers_bcast(a, k, which) + kReadyStride * (blockIdx.x % kPersBcast);
    unsigned t0 = 0, polls = 0;
    double v;
    while (!slot_full(v = ld_sc1(slot)) || stall) {
        if ((++polls & 15) == 0 && wait_expired(a, t0)) {
            abort_solve(a, kErrReadyWait, blockIdx.x % kPersBcast, k, which);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    out = v;
    return true;
}

// kMR: several ranks (z-slabs of a process-per-GPU job): the dots summed over
// the ranks in the kernel, r's ghost rows pulled from the neighbours at the
// top of every iteration. Its own instantiation: the one-rank kernel keeps
// its registers.
template <bool kNT, bool kMR = false, int kPre = 3, int kStep = 2, int kL = 3>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_cg_persist(CgArgs a)
{
    constexpr int kW = 27;
    // kL > 0: the first kL value slots come through LDS (kPre == kL), loaded by
    // LDS-DMA during the previous iteration's two waits; else kPre register slots
    static_assert((kW - kPre) % kStep == 0 && (kL == 0 || kL == kPre), "slot steps");
    const int P = unit_of(a);
    if (P < 0) return;
    // an earlier window ended the solve, or gave it up
    if (a.pk0 > 1 && (sld(a.kst + 1) || sld(a.kst + kErrBase) != kErrNone)) return;
    // several ranks (z-slabs): the ghost rows of r this pair reads -- its
    // windows (awin2: one per offset cluster, holes included) cut to the ghost
    // planes [-ghost_lo, 0) and [n, n + ghost_hi) -- as segments of one index
    // range [0, gtot), pulled from the neighbours at the top of every iteration
    __shared__ int gseg_row[kMR ? 2 * kAWin : 1], gseg_end[kMR ? 2 * kAWin : 1];
    __shared__ int gseg_tot;
    if constexpr (kMR) {
        if (threadIdx.x == 0) {
            const int prow0 = 2 * P * kSliceRows, nw = a.awn2[P];
            const int* win = a.awin2 + (size_t)P * kAWin * 3;
            int ns = 0, tot = 0;
            for (int w = 0; w < nw; w++) {
                const int w0 = prow0 + win[3 * w], w1 = w0 + win[3 * w + 1];
                const int lo0 = max(w0, -a.ghost_lo), lo1 = min(w1, 0);
                const int hi0 = max(w0, a.n), hi1 = min(w1, a.n + a.ghost_hi);
                if (lo1 > lo0) {
                    gseg_row[ns] = lo0;
                    tot += lo1 - lo0;
                    gseg_end[ns++] = tot;
                }
                if (hi1 > hi0) {
                    gseg_row[ns] = hi0;
                    tot += hi1 - hi0;
                    gseg_end[ns++] = tot;
                }
            }
            for (int j = ns; j < 2 * kAWin; j++) gseg_end[j] = INT_MAX;
            gseg_tot = tot;
        }
        __syncthreads();  // (before the first ring DMAs: nothing to drain yet)
    }
    const int gtot = kMR ? gseg_tot : 0;  // block-uniform
    const int s0 = 2 * P;
    const int nsl = min(2, a.nslices - s0);
    const int s1 = nsl > 1 ? s0 + 1 : s0;
    const int lr = threadIdx.x * kRpt;
    const int row0 = s0 * kSliceRows + lr, row1 = s1 * kSliceRows + lr;
    const double* __restrict__ vp0 = a.aval + (size_t)s0 * kW * kSliceRows + lr;
    const double* __restrict__ vp1 = a.aval + (size_t)s1 * kW * kSliceRows + lr;
    const int* __restrict__ off0 = a.aoff + (size_t)s0 * kAMax;
    const int* __restrict__ off1 = a.aoff + (size_t)s1 * kAMax;
    constexpr int kR = kL > 0 ? 0 : kPre;  // register slots
    Rows pre0[kR > 0 ? kR : 1], pre1[kR > 0 ? kR : 1];
#pragma unroll
    for (int j = 0; j < kR; j++) {
        pre0[j] = ld_m<kNT>(vp0 + (size_t)j * kSliceRows);
        pre1[j] = ld_m<kNT>(vp1 + (size_t)j * kSliceRows);
    }
    // LDS value ring: slot j of slice half h, wave w at entry ((j * 2 + h) * 4 +
    // w) * 128 doubles, lane l's 16 B at + 2 l (written and read by lane l only)
    __shared__ __attribute__((aligned(16))) double vring[kL > 0 ? kL * 2 * kBlock * kRpt : 2];
    const int wv = threadIdx.x / kWave;
    const int lane_ = threadIdx.x & (kWave - 1);
    // (buffer form: the lane's byte offset in a VGPR, the slot's in an SGPR)
    const __amdgpu_buffer_rsrc_t rsa = vec_rsrc(a.aval);
    const int lb = lr * 8;
    const int sb0 = s0 * kW * kSliceRows * 8, sb1 = s1 * kW * kSliceRows * 8;
    auto dma = [&](int j) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsa, (lds_void*)(vring + ((j * 2 + 0) * 4 + wv) * (2 * kWave)), 16,
                                                 lb, sb0 + j * kSliceRows * 8, 0, kNT ? 2 : 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsa, (lds_void*)(vring + ((j * 2 + 1) * 4 + wv) * (2 * kWave)), 16,
                                                 lb, sb1 + j * kSliceRows * 8, 0, kNT ? 2 : 0);
    };
    auto lds_val = [&](int j, int h) -> Rows {
        const d2v t = *reinterpret_cast<const d2v*>(vring + ((j * 2 + h) * 4 + wv) * (2 * kWave) + 2 * lane_);
        return Rows{{t.x, t.y}};
    };
    constexpr int kA = (kL + 1) / 2;  // ring slots refilled during the p.Ap wait; the rest during the r.r wait

#pragma unroll
    for (int j = 0; j < kL; j++) dma(j);
    // a raw workgroup barrier: __syncthreads() would drain the DMAs (vmcnt(0))
    auto bar = [&]() {
        if constexpr (kL > 0) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
        } else {
            __syncthreads();
        }
    };
    // r and the p ring through buffer resources based at the start of their
    // buffers (guard zone, then the ghost_lo planes of several ranks)
    const __amdgpu_buffer_rsrc_t rsr = vec_rsrc(a.r - a.pguard);
    const __amdgpu_buffer_rsrc_t rsp = vec_rsrc(a.p - a.pguard);
    const int b0 = (row0 + a.pguard) * 8, b1 = (row1 + a.pguard) * 8;
    const int pstr = (int)(a.pstride * 8);
    // the rows' x (in registers for the whole solve)
    Rows xv0 = ld(a.x + row0), xv1 = ld(a.x + row1);
    // r_{k-1}.r_{k-1} and r_{k-2}.r_{k-2}: the prologue's r_0.r_0 (k = 1), else
    // the history the previous window left
    double rr1 = a.pk0 == 1 ? a.g[kRRPar + 1] : a.hist[a.pk0 - 1];
    double rr2 = a.pk0 == 1 ? 0.0 : a.hist[a.pk0 - 2];
    int role;
    {
        const UnitMap m = spmv_units(a, 2);
        const int g = s0 / kGroup;
        role = P == group_last_unit(m, g) ? (g == top_group(m) ? 3 : 1) : 0;
        role = __builtin_amdgcn_readfirstlane(role);
    }
    __shared__ double ws2[2][kBlock / kWave];
    __shared__ double tot_s;
    __shared__ int gave_up;
    const int lane = threadIdx.x & (kWave - 1);
    int k = a.pk0;
    for (;; k++) {
        // HPCCG.cpp:358
        const bool run = k < a.max_iter && sqrt(k == 1 ? rr1 : rr2) > a.tol;
        if (run && k >= a.pk1) {  // the end of this launch's window: the next launch goes on from k
            vm_wait(0);           // (the ring's last refill)
            st_rows(a.x, row0, a.n, xv0);
            if (nsl > 1) st_rows(a.x, row1, a.n, xv1);
            if (blockIdx.x == 0 && threadIdx.x == 0) {
                a.hist[k - 1] = rr1;
                a.kst[0] = k;
                a.kst[2] = k;
            }
            return;
        }
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            if (k == 1 || run) a.hist[k - 1] = rr1;
            if (run) stamp(a, k, kStampSpmv);
        }
        if (!run) break;
        const double beta = (k == 1) ? 0.0 : rr1 / rr2;
        if (kMR && gtot > 0) {
            // r_{k-1}'s ghost rows from the neighbours (exchange_externals.cpp:
            // 84-126): system-scope loads of their r, stored write-through there
            // and drained before their r.r contribution, which the r.r total
            // this iteration started from includes; they overwrite it only
            // after this rank's p.Ap contribution, i.e. after this slot loop.
            // Kept in r's ghost rows, and p_k = r + beta p_{k-1} formed at them
            // (k_p_update's expression; the owner forms the same bits) into
            // ring buffer k & 1 for the next iteration's p_{k-1}. Every block
            // pulls all the ghost rows it reads itself (blocks that share a
            // row store the same value).
            if (P == 0 && threadIdx.x == 0) stamp(a, k, kStampHalo);
            const double* const yg = a.p + (size_t)((k - 1) & 1) * a.pstride;
            double* const pg = a.p + (size_t)(k & 1) * a.pstride;
            constexpr int kPullU = 6;  // remote loads in flight per thread
            for (int e0 = threadIdx.x; e0 < gtot; e0 += kPullU * kBlock) {
                double v[kPullU];
                int g[kPullU];
#pragma unroll
                for (int u = 0; u < kPullU; u++) {
                    const int e = e0 + u * kBlock;
                    g[u] = INT_MIN;
                    v[u] = 0.0;
                    if (e < gtot) {
                        int j = 0;
                        while (e >= gseg_end[j]) j++;
                        const int row = gseg_row[j] + (e - (j ? gseg_end[j - 1] : 0));
                        g[u] = row;
                        const double* src = row < 0 ? a.pl_src_lo + (row + a.ghost_lo) : a.pl_src_hi + (row - a.n);
                        v[u] = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    }
                }
#pragma unroll
                for (int u = 0; u < kPullU; u++) {
                    if (g[u] == INT_MIN) continue;
                    const double y = k == 1 ? v[u] : ld_sc1(yg + g[u]);  // (k = 1: p_1 = r_0 + 0 r_0)
                    st_sc1(a.r + g[u], v[u]);
                    st_sc1(pg + g[u], v[u] + beta * y);
                }
            }
            vm_wait(0);  // this block's ghost rows are in place before any of its waves reads them
            bar();
        }
        // p_{k-1}: ring buffer (k - 1) & 1 (k = 1: r_0, beta 0)
        const __amdgpu_buffer_rsrc_t rsy = k == 1 ? rsr : rsp;
        const int yb = k == 1 ? 0 : ((k - 1) & 1) * pstr;
        double sum0[kRpt] = {0.0, 0.0}, sum1[kRpt] = {0.0, 0.0};
        auto slot = [&](const Rows& v0, const Rows& v1, const Rows& ra, const Rows& ya, const Rows& rb, const Rows& yb_) {
#pragma unroll
            for (int i = 0; i < kRpt; i++) {
                sum0[i] = sum0[i] + v0.v[i] * (ra.v[i] + beta * ya.v[i]);
                sum1[i] = sum1[i] + v1.v[i] * (rb.v[i] + beta * yb_.v[i]);
            }
        };
        if constexpr (kL > 0) vm_wait(0);  // the ring's DMAs (issued during the waits) have landed
#pragma unroll
        for (int j = 0; j < kPre; j++) {
            const int o0 = sld(off0 + j) * 8, o1 = sld(off1 + j) * 8;
            if constexpr (kL > 0)
                slot(lds_val(j, 0), lds_val(j, 1), ld_rs(rsr, b0 + o0), ld_rs(rsy, yb + b0 + o0), ld_rs(rsr, b1 + o1),
                     ld_rs(rsy, yb + b1 + o1));
            else
                slot(pre0[j], pre1[j], ld_rs(rsr, b0 + o0), ld_rs(rsy, yb + b0 + o0), ld_rs(rsr, b1 + o1),
                     ld_rs(rsy, yb + b1 + o1));
        }
#pragma unroll 1
        for (int j0 = kPre; j0 < kW; j0 += kStep) {
            Rows v0[kStep], v1[kStep], ra[kStep], ya[kStep], rb[kStep], yc[kStep];
#pragma unroll
            for (int u = 0; u < kStep; u++) {
                const int o0 = sld(off0 + j0 + u) * 8, o1 = sld(off1 + j0 + u) * 8;
                v0[u] = ld_m<kNT>(vp0 + (size_t)(j0 + u) * kSliceRows);
                v1[u] = ld_m<kNT>(vp1 + (size_t)(j0 + u) * kSliceRows);
                ra[u] = ld_rs(rsr, b0 + o0);
                ya[u] = ld_rs(rsy, yb + b0 + o0);
                rb[u] = ld_rs(rsr, b1 + o1);
                yc[u] = ld_rs(rsy, yb + b1 + o1);
            }
#pragma unroll
            for (int u = 0; u < kStep; u++) slot(v0[u], v1[u], ra[u], ya[u], rb[u], yc[u]);
        }
        // the rows' r_{k-1} and p_k = r + beta p_{k-1} (k_p_update's expression;
        // read again: the slot loop's centre values came through L2 just now)
        const Rows rv0 = ld_rs(rsr, b0), rv1 = ld_rs(rsr, b1);
        const Rows yv0 = ld_rs(rsy, yb + b0), yv1 = ld_rs(rsy, yb + b1);
        Rows pk0, pk1;
#pragma unroll
        for (int i = 0; i < kRpt; i++) {
            pk0.v[i] = rv0.v[i] + beta * yv0.v[i];
            pk1.v[i] = rv1.v[i] + beta * yv1.v[i];
        }
        // p_k at the rows into ring buffer k & 1
        st_rs(rsp, (k & 1) * pstr + b0, row0, a.n, pk0);
        if (nsl > 1) st_rs(rsp, (k & 1) * pstr + b1, row1, a.n, pk1);
        double d0 = 0.0, d1 = 0.0;
#pragma unroll
        for (int i = 0; i < kRpt; i++) {
            if (row0 + i < a.n) d0 += pk0.v[i] * sum0[i];
            if (nsl > 1 && row1 + i < a.n) d1 += pk1.v[i] * sum1[i];
        }
        {
            const double w0 = wave_sum(d0), w1 = wave_sum(d1);
            if (lane == 0) {
                ws2[0][threadIdx.x / kWave] = w0;
                ws2[1][threadIdx.x / kWave] = w1;
            }
        }
        bar();
        if (threadIdx.x < kWave) {
            double bsj = 0.0;
            if (lane < 2) {
#pragma unroll
                for (int i = 0; i < kBlock / kWave; i++) bsj += ws2[lane][i];
            }
            pers_dot<kMR>(a, role, s0, nsl, bsj, kPAP, k);
        }
        // the next iteration's first ring slots, landing during the p.Ap wait
        // (this lane's reads of those entries are done: lgkmcnt)
        if constexpr (kL > 0) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int j = 0; j < kA; j++) dma(j);
        }
        if (threadIdx.x == 0) {
            double v = 0.0;
            gave_up = pers_wait(a, k, kPAP, v, a.dbg_resident_stall != 0) ? 0 : 1;
            tot_s = v;
        }
        bar();
        if (gave_up) {
            vm_wait(0);  // no DMA may land after the block's LDS is released
            return;
        }
        const double alpha = rr1 / tot_s;
        if (blockIdx.x == 0 && threadIdx.x == 0) stamp(a, k, kStampUpdate);
        // x += alpha p_k (waxpby, HPCCG.cpp:377), r = r - alpha Ap (:379), r.r (:384)
        Rows rn0, rn1;
#pragma unroll
        for (int i = 0; i < kRpt; i++) {
            xv0.v[i] = xv0.v[i] + alpha * pk0.v[i];
            xv1.v[i] = xv1.v[i] + alpha * pk1.v[i];
            rn0.v[i] = rv0.v[i] + (-alpha) * sum0[i];
            rn1.v[i] = rv1.v[i] + (-alpha) * sum1[i];
        }
        st_rs(rsr, b0, row0, a.n, rn0);
        if (nsl > 1) st_rs(rsr, b1, row1, a.n, rn1);
        double e0 = 0.0, e1 = 0.0;
#pragma unroll
        for (int i = 0; i < kRpt; i++) {
            if (row0 + i < a.n) e0 += rn0.v[i] * rn0.v[i];
            if (nsl > 1 && row1 + i < a.n) e1 += rn1.v[i] * rn1.v[i];
        }
        {
            const double w0 = wave_sum(e0), w1 = wave_sum(e1);
            // this wave's p_k and r_k have landed before the block's r.r partial
            // (the next iteration's readers are ordered after the r.r total)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (lane == 0) {
                ws2[0][threadIdx.x / kWave] = w0;
                ws2[1][threadIdx.x / kWave] = w1;
            }
        }
        bar();
        if (threadIdx.x < kWave) {
            double bsj = 0.0;
            if (lane < 2) {
#pragma unroll
                for (int i = 0; i < kBlock / kWave; i++) bsj += ws2[lane][i];
            }
            pers_dot<kMR>(a, role, s0, nsl, bsj, kRR, k);
        }
        // the next iteration's early value slots, in flight across the wait
#pragma unroll
        for (int j = 0; j < kR; j++) {
            pre0[j] = ld_m<kNT>(vp0 + (size_t)j * kSliceRows);
            pre1[j] = ld_m<kNT>(vp1 + (size_t)j * kSliceRows);
        }
        if constexpr (kL > 0) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int j = kA; j < kL; j++) dma(j);
        }
        if (threadIdx.x == 0) {
            double v = 0.0;
            gave_up = pers_wait(a, k, kRR, v, false) ? 0 : 1;
            tot_s = v;
        }
        bar();
        if (gave_up) {
            vm_wait(0);
            return;
        }
        // (tot_s is written again only after the next p.Ap barrier -- and only
        // once the next p.Ap total exists, which needs every wave's next partial)
        rr2 = rr1;
        rr1 = tot_s;
    }
    // k: the first iteration not run (niters = k - 1)
    vm_wait(0);  // (the ring's last refill)
    st_rows(a.x, row0, a.n, xv0);
    if (nsl > 1) st_rows(a.x, row1, a.n, xv1);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        a.kst[0] = k;
        a.kst[2] = k;
        mark_end(a);
    }
}


// ---------------------------------------------------------------------------
// SELL-512-A with x from LDS windows shared by slice pairs: block P owns
// slices 2P and 2P + 1 with 512 threads (waves 0-3 slice 2P, 4-7 slice
// 2P + 1, two rows per thread). The pair's windows (one per offset cluster:
// one per z-plane for the 27-pt stencil, holes included) are staged first,
// with kFuse p_k = r + beta*p_{k-1} computed per staged row (k_p_update's
// expression; at ghost rows of a multi-rank slab from r's received planes and
// the p_{k-1} ghosts the ghost blocks stored; guard rows are zeros). Slot j then reads xs[pair row + alds[s][j]]: one per-slice
// scalar per slot. kPre value slots are loaded before the iteration test.
// Each half forms its slice's partial with block_sum<256>'s shape, so the dot
// is bitwise the one-slice kernels'. 27-pt 200^3: a plane window covers 1024
// rows for 1426 staged doubles (4.2 per row).
// ---------------------------------------------------------------------------
// The pair's windows into LDS (xs): fused, p_k = r + beta*p_{k-1} per staged
// row (ghost rows of a multi-rank slab: r's received planes and p_{k-1}'s
// stored ghosts, ghost_store); guard rows are zeros. Every load of a round is
// issued before its LDS stores: the pair's windows are one LDS range [0, tot)
// (pair_windows lays them out back to back, even bases and lengths), each
// thread stages the row pairs e = 2 t + 1024 u of it, kU per round (16-B
// loads and LDS stores; one row at a time measured slower).
template <bool kFuse, int kU = 5>
__device__ __forceinline__ void stage_pair_windows(const CgArgs& a, const IterState& st, int P,
                                                           const double* __restrict__ p, const double* __restrict__ pold,
                                                           double* __restrict__ xs)
{
    const int prow0 = 2 * P * kSliceRows;
    const int nw = sld(a.awn2 + P);  // P is wave-uniform: the tables come through the scalar cache
    const int* __restrict__ win = a.awin2 + (size_t)P * kAWin * 3;
    int wlo[kAWin], wbase[kAWin];
#pragma unroll
    for (int w = 0; w < kAWin; w++) {
        wlo[w] = w < nw ? sld(win + 3 * w) : 0;
        wbase[w] = w < nw ? sld(win + 3 * w + 2) : INT_MAX;
    }
    const int tot = sld(win + 3 * (nw - 1) + 2) + sld(win + 3 * (nw - 1) + 1);
    for (int e0 = 2 * (int)threadIdx.x; e0 < tot; e0 += 4 * kBlock * kU) {
        d2v rv[kU], yv[kU];
#pragma unroll
        for (int u = 0; u < kU; u++) {
            const int e = e0 + 4 * kBlock * u;
            if (e < tot) {
                int lo = wlo[0], base = wbase[0];
#pragma unroll
                for (int w = 1; w < kAWin; w++)
                    if (e >= wbase[w]) lo = wlo[w], base = wbase[w];
                const int l = prow0 + lo + (e - base);  // local rows l, l + 1
                if (!kFuse) {
                    rv[u] = *reinterpret_cast<const d2v*>(p + l);
                } else {  // every row, ghosts and guard zeros included (rhalo)
                    rv[u] = *reinterpret_cast<const d2v*>(a.r + l);
                    yv[u] = *reinterpret_cast<const d2v*>(pold + l);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < kU; u++) {
            const int e = e0 + 4 * kBlock * u;
            if (e < tot) {
                d2v v = rv[u];
                if constexpr (kFuse) {
                    v.x = rv[u].x + st.beta * yv[u].x;
                    v.y = rv[u].y + st.beta * yv[u].y;
                }
                *reinterpret_cast<d2v*>(xs + e) = v;
            }
        }
    }
}

// The pair kernel's epilogue: Ap, p_k (from the window), the two
// slices' p.Ap partials with block_sum<256>'s shape, completed (fold) or stored.
template <bool kFuse>
__device__ __forceinline__ void pair_epilogue(const CgArgs& a, const IterState& st, bool prologue, int P, int s, bool have,
                                              int lrow, const double* __restrict__ xs, const double (&sum)[kRpt])
{
    __shared__ double wsum[2 * kBlock / kWave];
    double d = 0.0;
    if (have) {
        const int prow = (threadIdx.x / kBlock) * kSliceRows + lrow;  // row within the pair
        const int pd = a.adiag2 ? a.adiag2[s] : -1;  // LDS position of the slice's offset 0
        if (pd >= 0) {
            const Rows pk{{xs[prow + pd], xs[prow + pd + 1]}};
            d = spmv_rows_out<kFuse>(a, st, prologue, s * kSliceRows + lrow, sum, &pk);
        } else {
            d = spmv_rows_out<kFuse>(a, st, prologue, s * kSliceRows + lrow, sum);
        }
    }
    if (prologue) return;
    const double wv = wave_sum(d);
    const int lane = threadIdx.x & (kWave - 1);
    if (lane == 0) wsum[threadIdx.x / kWave] = wv;
    __syncthreads();
    if (threadIdx.x >= kWave) return;
    constexpr int kWh = kBlock / kWave;
    double bs = 0.0;
    if (lane < 2) {
#pragma unroll
        for (int i = 0; i < kWh; i++) bs += wsum[lane * kWh + i];
    }
    complete_dot_lanes(a, spmv_units(a, 2), P, 2 * P, min(2, a.nslices - 2 * P), bs, kPAP, st.k);
}

// ---------------------------------------------------------------------------
// SELL-512-A with x from LDS windows shared by slice pairs: block P owns
// slices 2P and 2P + 1 with 512 threads (waves 0-3 slice 2P, 4-7 slice
// 2P + 1, two rows per thread). The pair's windows (one per offset cluster:
// one per z-plane for the 27-pt stencil, holes included) are staged first
// (stage_pair_windows). Slot j then reads xs[pair row + alds[s][j]]: one
// per-slice scalar per slot. kPre value slots are loaded before the iteration
// test. Each half forms its slice's partial with block_sum<256>'s shape, so
// the dot is bitwise the one-slice kernels'. 27-pt 200^3: a plane window
// covers 1024 rows for 1426 staged doubles (4.2 per row).
// ---------------------------------------------------------------------------
template <bool kNT, bool kFuse, int kPre>
__global__ __launch_bounds__(2 * kBlock) void k_spmv_a2(CgArgs a, bool prologue)
{
    if (ghost_store<false>(a, prologue)) return;
    extern __shared__ __attribute__((aligned(16))) double xs[];
    const int P = unit_of(a);  // pair: all, or the interior / halo runs
    const int half = threadIdx.x / kBlock;
    const int s = P < 0 ? a.nslices : 2 * P + half;
    const bool have = s < a.nslices;
    const int lrow = (threadIdx.x % kBlock) * kRpt;  // row within the slice
    const int wdt = have ? (int)(a.abase[s + 1] - a.abase[s]) : 0;
    const double* __restrict__ vp = a.aval + (have ? (size_t)a.abase[s] * kSliceRows : 0) + lrow;
    constexpr int kP = kPre > 0 ? kPre : 1;
    Rows vpre[kP];
#pragma unroll
    for (int j = 0; j < kPre; j++)
        if (j < wdt) vpre[j] = ld_m<kNT>(vp + (size_t)j * kSliceRows);
    IterState st;
    if (!spmv_begin<kFuse>(a, prologue, st)) return;
    if (P < 0 || 2 * P >= a.nslices) return;
    const double* __restrict__ p = cur_p(a, st.k);
    const double* __restrict__ pold = a.r;
    if constexpr (kFuse) pold = (st.k == 1) ? a.r : cur_p(a, st.k - 1);
    stage_pair_windows<kFuse>(a, st, P, p, pold, xs);
    __syncthreads();
    double sum[kRpt] = {0.0, 0.0};
    if (have) {
        const int* __restrict__ cl = a.alds2 + (size_t)s * kAMax;
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
            const Rows v = ld_m<kNT>(vp + (size_t)j * kSliceRows);
            const int c = prow + cl[j];
#pragma unroll
            for (int i = 0; i < kRpt; i++) sum[i] = sum[i] + v.v[i] * xs[c + i];
        }
    }
    pair_epilogue<kFuse>(a, st, prologue, P, s, have, lrow, xs, sum);
}

// ---------------------------------------------------------------------------
// The pair kernel with the value stream through LDS-DMA (uniform width kW):
// every wave owns 128 rows of one slice and streams their value slots from
// HBM straight into a private ring of kR 1-KB LDS entries
// (global_load_lds_dwordx4, non-temporal; lane l's 16 B land at entry + 16 l
// and are read back by lane l). The first kR slots are issued before the
// iteration test, so they land while the windows are staged; each consumed
// entry is refilled with slot j + kR right away, a counted vmcnt wait ahead
// of each read. No value occupies a VGPR across the staging barrier.
// The iteration state and the window/offset tables come through the scalar
// cache, so nothing but the ring is counted on vmcnt in the slot loop.
// 27-pt 200^3, same-process A/B (tools/ab_inproc.py): SpMV 337.8 us at kR = 3
// (2579 CG it/s) against 342.0 / 343.5 us at kR = 2 / 4 and 355.1 us for the
// register pair kernel (2469 it/s); storing Ap and p_k after the p.Ap ticket
// instead measured 341.8 us. Same products in the same order: same bits.
// ---------------------------------------------------------------------------
constexpr int kA2RingMax = 4;


// kTL: the diagnostic instantiation that records the block timeline
// (dbg_timeline, kTlWords); the product launches never write it.
template <bool kFuse, int kW, int kR, bool kTL = false>
__global__ __launch_bounds__(2 * kBlock) void k_spmv_a2r(CgArgs a, bool prologue)
{
    if (side_flush<2, 16>(a, prologue)) return;
    if (ghost_store<false>(a, prologue)) return;
    static_assert(kR >= 1 && kR <= kA2RingMax && kR <= kW, "ring depth");
    extern __shared__ __attribute__((aligned(16))) double xs[];
    const int P = unit_of(a);
    const int half = threadIdx.x / kBlock;
    const int s = P < 0 ? a.nslices : 2 * P + half;
    const bool have = s < a.nslices;
    const int lane = threadIdx.x & (kWave - 1);
    const int lrow = (threadIdx.x % kBlock) * kRpt;  // row within the slice: wave's 128 rows, lane-linear
    // an odd last pair's second half streams its partner's values (never used)
    const double* __restrict__ vp = a.aval + (size_t)(have ? s : s - 1) * kW * kSliceRows + lrow;
    double* __restrict__ ring = xs + ((a.alds2_doubles + 1) & ~1) + (threadIdx.x / kWave) * (kR * 2 * kWave);
    if (P < 0 || 2 * P >= a.nslices) return;
    unsigned long long tl[5] = {0, 0, 0, 0, 0};
    if constexpr (kTL) tl[0] = now_ticks();
#pragma unroll
    for (int j = 0; j < kR; j++)
        __builtin_amdgcn_global_load_lds((const void*)(vp + (size_t)j * kSliceRows), (lds_void*)(ring + j * 2 * kWave),
                                         16, 0, 2 /* nt */);
    // the slot offsets: scalar loads (slice index made wave-uniform), all
    // before the ring is counted, so no vector load lands among the DMAs
    const int su = __builtin_amdgcn_readfirstlane(have ? s : s - 1);
    typedef const __attribute__((address_space(4))) int* cint_p;  // constant space: s_load
    const cint_p cl = (cint_p)(a.alds2 + (size_t)su * kAMax);
    int clv[kW];
#pragma unroll
    for (int j = 0; j < kW; j++) clv[j] = cl[j];
    // iteration state through the scalar cache (s_load counts on lgkmcnt, so
    // it does not queue behind the ring's DMAs on vmcnt); written by earlier
    // kernels only
    IterState st;
    st.k = 0;
    st.rr = 0.0;
    st.beta = 0.0;
    bool run = true;
    if (!prologue) {
        st.k = sld(a.kst);
        if (kFuse) st.rr = sld(a.g + kRR);
        const double h1 = sld(a.hist + max(st.k - 2, 0));  // r_{k-2}.r_{k-2} (k >= 2)
        run = st.k < a.max_iter && sqrt(st.k == 1 ? (kFuse ? st.rr : sld(a.hist)) : h1) > a.tol;
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            publish_iter(a, st.k, run);
            if (kFuse && (st.k == 1 || run)) a.hist[st.k - 1] = st.rr;
            if (run)
                stamp(a, st.k, kStampSpmv);
            else
                mark_end(a);
        }
        if (kFuse && run) st.beta = (st.k == 1) ? 0.0 : st.rr / h1;
    }
    if (!run) {
        vm_wait(0);  // no DMA may land after the block's LDS is released
        return;
    }
    if constexpr (kTL) tl[1] = now_ticks();
    const double* __restrict__ p = cur_p(a, st.k);
    const double* __restrict__ pold = a.r;
    if constexpr (kFuse) pold = (st.k == 1) ? a.r : cur_p(a, st.k - 1);
    stage_pair_windows<kFuse>(a, st, P, p, pold, xs);
    // raw barrier: __syncthreads() would drain the ring (vmcnt(0))
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if constexpr (kTL) tl[2] = now_ticks();
    const int prow = half * kSliceRows + lrow;  // row within the pair
    double sum[kRpt] = {0.0, 0.0};
#pragma unroll
    for (int j = 0; j < kW; j++) {
        vm_wait((j + kR < kW ? j + kR : kW) - j - 1);  // slot j has landed
        const d2v v = *reinterpret_cast<const d2v*>(ring + (j % kR) * 2 * kWave + 2 * lane);
        const int c = prow + clv[j];
        sum[0] = sum[0] + v.x * xs[c];
        sum[1] = sum[1] + v.y * xs[c + 1];
        asm volatile("" : "+v"(sum[0]), "+v"(sum[1]));  // keep the products here (else 220 VGPRs)
        if (j + kR < kW) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // entry read before its refill lands
            __builtin_amdgcn_global_load_lds((const void*)(vp + (size_t)(j + kR) * kSliceRows),
                                             (lds_void*)(ring + (j % kR) * 2 * kWave), 16, 0, 2);
        }
    }
    if constexpr (kTL) tl[3] = now_ticks();
    pair_epilogue<kFuse>(a, st, prologue, P, s, have, lrow, xs, sum);
    if constexpr (kTL) {
        if (threadIdx.x == 0 && a.dbg_tl) {  // wave 0 ran the dot hand-off: the block's last work
            tl[4] = now_ticks();
            const unsigned hwid = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11));    // HW_ID
            const unsigned xcc = __builtin_amdgcn_s_getreg(20 | (0 << 6) | (15 << 11));   // XCC_ID
            unsigned long long* o = a.dbg_tl + (size_t)P * kTlWords;
            o[0] = (unsigned long long)blockIdx.x | ((unsigned long long)hwid << 32);
#pragma unroll
            for (int i = 0; i < 5; i++) o[1 + i] = tl[i];
            o[6] = xcc;
            o[7] = (unsigned long long)st.k;
        }
    }
}

// Plain SpMV on a caller's x (kernel-level C ABI, HPC_sparsemv.cpp:68-89):
// the SELL-512-A image in prologue mode reads p; this one reads xext through
// the SELL-512 image when the matrix keeps one. Same body, no dot.
__global__ __launch_bounds__(kBlock) void k_spmv_plain(CgArgs a, const double* __restrict__ xext,
                                                       double* __restrict__ y)
{
    const int s = xcd_slice(a.grid);
    if (s >= a.nslices) return;
    const size_t base = (size_t)a.slice_base[s] * kSliceRows + (size_t)threadIdx.x * kRpt;
    const int w = (int)(a.slice_base[s + 1] - a.slice_base[s]);
    double sum[kRpt] = {0.0, 0.0};
    for (int j = 0; j < w; j++) {
        int c[kRpt];
        ld_cols_m<false>(a.cols + base + (size_t)j * kSliceRows, c);
        const Rows v = ld(a.vals + base + (size_t)j * kSliceRows);
#pragma unroll
        for (int i = 0; i < kRpt; i++) sum[i] = sum[i] + v.v[i] * ((c[i] >= 0) ? xext[c[i]] : 0.0);
    }
    const int row = s * kSliceRows + threadIdx.x * kRpt;
    for (int i = 0; i < kRpt; i++)
        if (row + i < a.n) y[row + i] = sum[i];
}

// Diagnostic only (never in the CG path): streams the SELL-512-A values like
// the SpMV (16 B non-temporal loads per lane, slot-major) without the x side,
// writing one sum per row -- a known byte count (8 B x slots read, 8 B x n
// written) for the rocprofv3 FETCH_SIZE / WRITE_SIZE calibration.
__global__ __launch_bounds__(kBlock) void k_stream_a(CgArgs a)
{
    const int s = xcd_slice(a.grid);
    if (s >= a.nslices) return;
    const int w = (int)(a.abase[s + 1] - a.abase[s]);
    const double* __restrict__ vp = a.aval + (size_t)a.abase[s] * kSliceRows + (size_t)threadIdx.x * kRpt;
    double sum[kRpt] = {0.0, 0.0};
#pragma unroll 4
    for (int j = 0; j < w; j++) {
        const Rows v = ld_m<true>(vp + (size_t)j * kSliceRows);
        sum[0] = sum[0] + v.v[0];
        sum[1] = sum[1] + v.v[1];
    }
    st_rows(a.Ap, s * kSliceRows + threadIdx.x * kRpt, a.n, Rows{{sum[0], sum[1]}});
}

// ---------------------------------------------------------------------------
// Separate final reduction (dot not folded): the same two levels and order as
// the folded completion, so fold on/off give the same bits. The partials are
// loaded first -- they do not depend on the iteration state -- so the loads
// overlap the k / loop-test chain; one 1024-thread block.
// ---------------------------------------------------------------------------
constexpr int kFinalizeThreads = 1024;
constexpr int kFinLdsGroups = 2048;  // group sums kept in LDS up to 128 K slices (64 M rows)

// kB groups per wave per round, every load of a round issued before the sums
// (one round up to 16 x kB groups: 200^3 has 245, 7-pt 256^3 512).
template <int kB>
__device__ __forceinline__ void finalize_groups(const CgArgs& a, double* sp, int ng, bool in_lds, double* gs,
                                                double* gp)
{
    const int lane = threadIdx.x & (kWave - 1);
    constexpr int kWaves = kFinalizeThreads / kWave;
    for (int g0 = threadIdx.x / kWave; g0 < ng; g0 += kWaves * kB) {
        double v[kB];
#pragma unroll
        for (int b = 0; b < kB; b++) {
            const int i = (g0 + b * kWaves) * kGroup + lane;
            v[b] = (g0 + b * kWaves < ng && i < a.nslices) ? sp[i] : 0.0;
        }
#pragma unroll
        for (int b = 0; b < kB; b++) {  // the slots are empty again for the next producer
            const int i = (g0 + b * kWaves) * kGroup + lane;
            if (g0 + b * kWaves < ng && i < a.nslices) sp[i] = slot_empty();
        }
#pragma unroll
        for (int b = 0; b < kB; b++) {
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
}

__global__ __launch_bounds__(kFinalizeThreads) void k_finalize(CgArgs a, int which, bool prologue)
{
    __shared__ double gs[kFinLdsGroups];
    const int ng = ngroups_of(a);
    const bool in_lds = ng <= kFinLdsGroups;
    double* const sp = slice_slots(a, which);
    double* const gp = group_slots(a, which, ng);
    const int lane = threadIdx.x & (kWave - 1);
    int k = 0;
    bool run = true;
    if (!prologue) run = iter_of(a, k);
    // stamped unconditionally: stamps after the end stamp are dropped on the host
    if (threadIdx.x == 0) stamp(a, k, which == kRR ? kStampFinRR : kStampFinPAP);
    if (ng <= 4 * (kFinalizeThreads / kWave))
        finalize_groups<4>(a, sp, ng, in_lds, gs, gp);
    else if (ng <= 16 * (kFinalizeThreads / kWave))
        finalize_groups<16>(a, sp, ng, in_lds, gs, gp);
    else
        finalize_groups<32>(a, sp, ng, in_lds, gs, gp);
    if (!run) {
        if (threadIdx.x == 0) mark_end(a);
        return;
    }
    if (!in_lds) __threadfence_block();
    __syncthreads();  // group sums written by this block
    if (threadIdx.x < kWave) {
        const double tot = in_lds ? top_sum_wave([&](int i) { return gs[i]; }, ng, lane)
                                  : top_sum_wave([gp](int i) { return gp[i]; }, ng, lane);
        if (!in_lds)
            for (int j = lane; j < ng; j += kWave) gp[j] = slot_empty();
        if (lane == 0) finish_dot(a, tot, which, k, false);
    }
}

// x += alpha_j p_j for j = j0..j1 in order (HPCCG.cpp:383, one rounding per
// term as in the reference); alpha_kcur comes from the caller (the update's own
// alpha, not yet in ahist for the reader). Four p loads are issued before their
// adds, so a long ring does not serialise one HBM latency per term.
__device__ __forceinline__ void x_accumulate(const CgArgs& a, int row, int j0, int j1, int kcur, double alpha_kcur,
                                             Rows& xn)
{
    constexpr int kB = 4;
    int j = j0;
    for (; j + kB - 1 <= j1; j += kB) {
        Rows pj[kB];
        double aj[kB];
#pragma unroll
        for (int b = 0; b < kB; b++) {
            pj[b] = ld(cur_p(a, j + b) + row);
            aj[b] = (j + b == kcur) ? alpha_kcur : a.ahist[j + b];
        }
#pragma unroll
        for (int b = 0; b < kB; b++)
#pragma unroll
            for (int i = 0; i < kRpt; i++) xn.v[i] = xn.v[i] + aj[b] * pj[b].v[i];
    }
    for (; j <= j1; j++) {
        const double aj = (j == kcur) ? alpha_kcur : a.ahist[j];
        const Rows pj = ld(cur_p(a, j) + row);
#pragma unroll
        for (int i = 0; i < kRpt; i++) xn.v[i] = xn.v[i] + aj * pj.v[i];
    }
}

// ---------------------------------------------------------------------------
// Fused update + r.r partial.
// prologue: r = b + (-1)*Ap                (HPCCG.cpp:352)
// loop:     x = x + alpha*p; r = r + (-alpha)*Ap   (HPCCG.cpp:382-384),
//           alpha = rtrans / (p.Ap); then the r.r partial that the next
//           iteration's ddot(r, r) (HPCCG.cpp:367) would compute. With x
//           deferral the x update runs every nring iterations over the ring
//           of p buffers, the same roundings in the same order.
// ---------------------------------------------------------------------------
// In the loop, Ap and r are loaded together with the iteration state, which
// comes through the scalar cache (published by this iteration's SpMV launch):
// the loop test no longer holds the loads back (a no-op launch after the end
// loads them for nothing).
template <bool kPrologue>
__global__ __launch_bounds__(kBlock) void k_update(CgArgs a)
{
    if ((int)blockIdx.x >= a.grid) {  // in-launch pull blocks (a.pull_in), after the update's
        int k = 0;
        if constexpr (!kPrologue) {
            if (!a.kst[5]) return;  // publish_iter's {k, run}
            k = a.kst[4];
        }
        pull_rows<true>(a, k, (int)blockIdx.x - a.grid, (int)gridDim.x - a.grid);
        return;
    }
    int k = 0;
    const int s = a.rev ? xcd_slice_rev(a.grid) : xcd_slice(a.grid);
    const int row = s * kSliceRows + threadIdx.x * kRpt;
    Rows apv, rv;
    if constexpr (!kPrologue) {
        k = sld(a.kst + 4);  // publish_iter's {k, run}
        const bool run = sld(a.kst + 5) != 0;
        if (s < a.nslices) {
            apv = ld(a.Ap + row);
            rv = ld(a.r + row);
        }
        asm volatile("" ::: "memory");  // the loads stay ahead of the test
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            if (run)
                stamp(a, k, kStampUpdate);
            else
                mark_end(a);
        }
        if (!run) return;
    }
    if (s >= a.nslices) return;
    double alpha = 0.0;
    if constexpr (!kPrologue) {
        alpha = sld(a.g + kRR) / sld(a.g + kPAP);
        if (blockIdx.x == 0 && threadIdx.x == 0) a.ahist[k] = alpha;
    }
    Rows rn;
    if constexpr (kPrologue) {
        apv = ld(a.Ap + row);
        const Rows bv = ld(a.b + row);
#pragma unroll
        for (int i = 0; i < kRpt; i++) rn.v[i] = bv.v[i] + (-1.0) * apv.v[i];
    } else {
#pragma unroll
        for (int i = 0; i < kRpt; i++) rn.v[i] = rv.v[i] + (-alpha) * apv.v[i];
        if (!a.xdefer) {
            const Rows xv = ld(a.x + row);
            const Rows pv = ld(cur_p(a, k) + row);
            Rows xn;
#pragma unroll
            for (int i = 0; i < kRpt; i++) xn.v[i] = xv.v[i] + alpha * pv.v[i];
            st_vec(a, a.x, row, xn);
        } else if (a.xdefer == 1 && k % a.nring == 0) {
            // deferred x update (HPCCG.cpp:383 for iterations k-nring+1 .. k)
            Rows xn = ld(a.x + row);
            x_accumulate(a, row, k - a.nring + 1, k, k, alpha, xn);
            st_vec(a, a.x, row, xn);
        }
    }
    const bool wt = pulled_slice(a, s);  // (block-uniform)
    if (wt)
        st_r_through(a, row, rn);
    else
        st_vec(a, a.r, row, rn);
    double d = 0.0;
#pragma unroll
    for (int i = 0; i < kRpt; i++)
        if (row + i < a.n) d += rn.v[i] * rn.v[i];
    if (wt) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // landed before the partial is published
    const double bs = block_sum<kBlock>(d);
    complete_dot(a, update_units(a), s, s, bs, kRR, k);
}

// Timestamp-only kernel around RCCL calls (multi-rank): one lane, one store.
__global__ void k_stamp(CgArgs a, int slot, bool prologue)
{
    int k = 0;
    if (!prologue) {
        // The r.r all-reduce follows the finalize that already advanced k.
        k = a.kst[0] - (slot == kStampArRR ? 1 : 0);
        if (!cg_run(a, k, false)) {
            mark_end(a);
            return;
        }
    }
    stamp(a, k, slot);
}

__global__ void k_end(CgArgs a) { mark_end(a); }

// r-halo by pull (option halo_pull): before the SpMV launch of iteration k
// (k_host's parity as the fused launch reads it), this rank's ghost planes of
// r are read straight from the neighbours' boundary rows -- another GPU's
// memory through IPC, or another group member's buffer -- with system-scope
// loads (sc0 sc1: from memory, never a copy cached in this GPU's L2). The
// neighbour stored those rows write-through and drained them before its r.r
// partial (pulled_slice), and this rank's previous launch waited for that
// contribution (peer all-reduce, or RCCL's after the neighbour's kernel end),
// so the rows are r_{k-1}; the neighbour rewrites them only after this
// rank's p.Ap of iteration k, which follows this kernel. Plain stores here:
// the SpMV launch reading them starts after this kernel ends. A solve that
// has ended leaves them alone.
__global__ __launch_bounds__(256) void k_pull(CgArgs a, const double* __restrict__ lo_src, double* __restrict__ lo_dst,
                                              int lo_cnt, const double* __restrict__ hi_src,
                                              double* __restrict__ hi_dst, int hi_cnt, int mode)
{
    const bool force = mode & 1, pexpr = mode & 2;
    if (!force) {  // (force: the creation-time test and the prologue, outside the iteration test)
        const int k = a.fupd ? (a.kst[1] ? a.max_iter : a.kst[a.kpar ? 2 : 0]) : a.kst[0];
        const double rr = a.g[a.fupd ? kRRPar + a.kpar : kRR];
        if (k >= a.max_iter || !(sqrt(k == 1 ? rr : a.hist[max(k - 2, 0)]) > a.tol)) return;  // cg_run
        if (blockIdx.x == 0 && threadIdx.x == 0) stamp(a, k, kStampHalo);
    }
    constexpr int kU = 4;  // loads in flight per thread
    const int tot = lo_cnt + hi_cnt;
    const int stride = (int)(gridDim.x * blockDim.x) * kU;
    for (int i0 = (int)(blockIdx.x * blockDim.x + threadIdx.x); i0 < tot; i0 += stride) {
        double v[kU];
#pragma unroll
        for (int u = 0; u < kU; u++) {
            const int i = i0 + u * (int)(gridDim.x * blockDim.x);
            v[u] = i < tot ? __hip_atomic_load(i < lo_cnt ? lo_src + i : hi_src + (i - lo_cnt), __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_SYSTEM)
                           : 0.0;
        }
#pragma unroll
        for (int u = 0; u < kU; u++) {
            const int i = i0 + u * (int)(gridDim.x * blockDim.x);
            // (pexpr: k_prologue_copy's p = x + 0.0 x on the neighbour's x)
            if (i < tot) (i < lo_cnt ? lo_dst[i] : hi_dst[i - lo_cnt]) = pexpr ? v[u] + 0.0 * v[u] : v[u];
        }
    }
}

// The prologue's barrier (one lane): a peer all-reduce on the kMboxBarrier
// slots. Every rank stores into it after its p = x (stream order), so once it
// returns every rank's x is in place for the x pull that follows; no rank
// changes its x before this rank's first r.r contribution, which comes after
// that pull. Used once per solve: each rank empties its slots when all
// arrived, long before the next solve's barrier refills them.
__global__ void k_peer_barrier(CgArgs a)
{
    if (threadIdx.x == 0) (void)peer_allreduce(a, 1.0, kMboxBarrier, 0, true);
}

// The peer all-reduce's creation-time self-test (peer_autotest): one lane runs
// `rounds` all-reduces of each scalar slot through the kernels' own
// peer_allreduce, contribution (prank + 1) + 0.5 k + 0.25 which.
__global__ void k_peer_selftest(CgArgs a, int rounds, double* out)
{
    if (threadIdx.x != 0) return;
    for (int k = 0; k < rounds; k++)
        for (int which = 0; which < 2; which++)
            out[2 * k + which] = peer_allreduce(a, (double)(a.prank + 1) + 0.5 * k + 0.25 * which, which, k, true);
}

// Every solve starts here, stream-ordered before its prologue (HPCCG.cpp:
// 342-356 starts from r = b - A x with nothing carried over): the iteration
// state and error record zeroed with the spin budget set, every dot slot --
// slice partials, group sums, the fused update's p.Ap ready slots -- empty.
// No solve then depends on what an earlier solve, an aborted one or the
// placement probe's timed solves left in them.
__global__ __launch_bounds__(256) void k_rearm(int* kst, double* partial, int np, int budget)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < 2 * kKstDoubles) kst[i] = i == kErrBase + kErrBudget ? budget : 0;
    if (i < np) partial[i] = slot_empty();
}

// After the loop: x += alpha_j p_j for the iterations since the last batched
// update (niters = kst[0] - 1 is final here).
__global__ __launch_bounds__(kBlock) void k_xflush(CgArgs a)
{
    if (!a.xdefer) return;
    const int niters = (a.fupd ? max(a.kst[0], a.kst[2]) : a.kst[0]) - 1;
    const int s = xcd_slice(a.grid);
    if (s >= a.nslices) return;
    // the last term already applied to this slice's x (0: none)
    int last;
    if (a.xdefer == 1) {
        last = (niters / a.nring) * a.nring;
    } else {  // beside the SpMV: the SpMV of iteration kp applied terms up to kp - 1
        const int q = a.nring - 1, ph = s % q == 0 ? q : s % q;
        last = niters >= ph ? niters - (niters - ph) % q - 1 : 0;
    }
    const int first = last + 1;
    if (first > niters) return;
    const int row = s * kSliceRows + threadIdx.x * kRpt;
    Rows xn = ld(a.x + row);
    x_accumulate(a, row, first, niters, -1, 0.0, xn);
    st_rows(a.x, row, a.n, xn);
}

__global__ void k_group_sum(GroupSum gs)
{
    double v = 0.0;
    for (int r = 0; r < gs.nranks; r++) v += gs.loc[r][gs.which];
    for (int r = 0; r < gs.nranks; r++) gs.g[r][gs.which] = v;
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

__global__ __launch_bounds__(256) void k_dot_partial(int n, const double* x, const double* y, double* partial)
{
    const int base = blockIdx.x * kDotChunk;
    const int end = min(n, base + kDotChunk);
    double d = 0.0;
    for (int i = base + threadIdx.x; i < end; i += 256) d += x[i] * y[i];
    const double s = block_sum<256>(d);
    if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

__global__ __launch_bounds__(kDotFinalThreads) void k_dot_final(const double* partial, int nparts, double* out)
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
__global__ __launch_bounds__(256) void k_generate(int nx, int ny, int nz, int rank, int size, int use_7pt,
                                                  long long col_base, const unsigned int* slice_base, int* cols,
                                                  double* vals, double* b, double* xexact, int nrow)
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
                    j++;
                }
            }
    b[lrow] = 27.0 - ((double)(j - 1));
    xexact[lrow] = 1.0;
    for (; j < w; j++) {
        vals[base + (size_t)j * kSliceRows] = 0.0;
        cols[base + (size_t)j * kSliceRows] = -1;
    }
}

// Rows of the last slice past nrow: all slots padding.
__global__ void k_generate_tail(int nrow, int nslices, const unsigned int* slice_base, int* cols, double* vals)
{
    const int s = nslices - 1;
    const int lane = threadIdx.x;
    if (s * kSliceRows + lane < nrow) return;
    const unsigned int b0 = slice_base[s];
    const int w = (int)(slice_base[s + 1] - b0);
    for (int j = 0; j < w; j++) {
        vals[(size_t)b0 * kSliceRows + (size_t)j * kSliceRows + lane] = 0.0;
        cols[(size_t)b0 * kSliceRows + (size_t)j * kSliceRows + lane] = -1;
    }
}

// ---------------------------------------------------------------------------
// SELL-512-A from the SELL-512 image, on the device. Pass 1 (k_a_offsets): the
// slice's distinct offsets (local column - ghost_lo - row) in an LDS table --
// one insert per distinct value of a wave (the wave's lanes usually share it),
// at most kAMax per slice -- sorted into aoff[s][0..K), acount[s] = K; ok[0]
// = 0 when a slice has more than kAMax offsets or a row's entries are not in
// strictly ascending column order (the A slots would sum in another order).
// Pass 2 (k_a_fill): every entry goes to the slot of its offset.
// ---------------------------------------------------------------------------
constexpr int kATable = 64;  // LDS hash slots (> kAMax: a full table means too many offsets)
constexpr int kEmpty = INT_MIN;

__global__ __launch_bounds__(kSliceRows) void k_a_offsets(const unsigned int* __restrict__ slice_base, int nslices,
                                                          const int* __restrict__ cols, int ghost_lo,
                                                          int* __restrict__ aoff, int* __restrict__ acount,
                                                          int* ok, int* maxabs)
{
    __shared__ int tab[kATable];
    __shared__ int cnt, over;
    const int s = blockIdx.x;
    if (s >= nslices) return;
    const int lane = threadIdx.x;
    if (lane < kATable) tab[lane] = kEmpty;
    if (lane == 0) cnt = 0, over = 0;
    __syncthreads();
    const size_t e0 = (size_t)slice_base[s] * kSliceRows + lane;
    const int w = (int)(slice_base[s + 1] - slice_base[s]);
    const int row = s * kSliceRows + lane;
    int prev = INT_MIN;
    bool ordered = true;
    for (int j = 0; j < w; j++) {
        const int c = cols[e0 + (size_t)j * kSliceRows];
        const bool has = c >= 0;
        const int o = has ? c - ghost_lo - row : 0;
        if (has) {
            if (o <= prev) ordered = false;
            prev = o;
        }
        // wave-level dedupe: insert the first pending lane's value, drop every
        // lane holding it, repeat
        bool pending = has;
        while (__any(pending)) {
            const unsigned long long m = __ballot(pending);
            const int leader = __ffsll((long long)m) - 1;
            const int key = __shfl(o, leader, kWave);
            if (pending && o == key) pending = false;
            if ((lane & (kWave - 1)) == leader) {
                unsigned h = ((unsigned)key * 2654435761u) >> 26;  // 6 bits
                for (int t = 0; t < kATable; t++, h = (h + 1) & (kATable - 1)) {
                    const int old = atomicCAS(&tab[h], kEmpty, key);
                    if (old == kEmpty) {
                        atomicAdd(&cnt, 1);
                        break;
                    }
                    if (old == key) break;
                    if (t == kATable - 1) atomicExch(&over, 1);
                }
            }
        }
    }
    if (!ordered) atomicExch(&over, 1);
    __syncthreads();
    const int K = cnt;
    if (over || K > kAMax) {
        if (lane == 0) ok[0] = 0;
        return;
    }
    if (lane < kATable) {
        const int o = tab[lane];
        if (o != kEmpty) {
            int r = 0;
            for (int t = 0; t < kATable; t++) r += (tab[t] != kEmpty && tab[t] < o) ? 1 : 0;
            aoff[(size_t)s * kAMax + r] = o;
            atomicMax(maxabs, o < 0 ? -o : o);
        }
    }
    if (lane >= K && lane < kAMax) aoff[(size_t)s * kAMax + lane] = 0;  // padding slots: offset 0, value 0
    if (lane == 0) acount[s] = K;
}

__global__ __launch_bounds__(kSliceRows) void k_a_fill(const unsigned int* __restrict__ slice_base, int nslices,
                                                       const int* __restrict__ cols, const double* __restrict__ vals,
                                                       int ghost_lo, const int* __restrict__ aoff,
                                                       const int* __restrict__ acount,
                                                       const unsigned int* __restrict__ abase, double* __restrict__ aval)
{
    __shared__ int so[kAMax];
    const int s = blockIdx.x;
    if (s >= nslices) return;
    const int lane = threadIdx.x;
    const int K = acount[s];
    if (lane < kAMax) so[lane] = aoff[(size_t)s * kAMax + lane];
    __syncthreads();
    const size_t e0 = (size_t)slice_base[s] * kSliceRows + lane;
    const int w = (int)(slice_base[s + 1] - slice_base[s]);
    const int row = s * kSliceRows + lane;
    double* out = aval + (size_t)abase[s] * kSliceRows + lane;
    int r = 0;
    for (int j = 0; j < w; j++) {
        const int c = cols[e0 + (size_t)j * kSliceRows];
        if (c < 0) continue;
        const int o = c - ghost_lo - row;
        while (r < K && so[r] < o) r++;  // rows ascend: the slot index only grows
        out[(size_t)r * kSliceRows] = vals[e0 + (size_t)j * kSliceRows];
    }
}

}  // namespace

// ---- launch wrappers ------------------------------------------------------
void launch_cg_prologue_copy(const CgArgs& a, hipStream_t s)
{
    hipLaunchKernelGGL(k_prologue_copy, dim3(a.grid), dim3(kBlock), 0, s, a);
}

void launch_cg_p_update(const CgArgs& a, hipStream_t s)
{
    hipLaunchKernelGGL(k_p_update, dim3(a.grid), dim3(kBlock), 0, s, a);
}


void launch_cg_pack(const CgArgs& a, const int* idx, int cnt, double* buf, bool prologue, hipStream_t s)
{
    if (cnt <= 0) return;
    hipLaunchKernelGGL(k_pack, dim3((cnt + 255) / 256), dim3(256), 0, s, a, idx, cnt, buf, prologue);
}

bool spmv_kernel_ok(int kernel) { return kernel >= kSpmvSell && kernel <= kSpmvPairs; }

size_t a2_lds_bytes(int lds_doubles, int ring)
{
    if (ring <= 0) return (size_t)lds_doubles * sizeof(double);
    return (size_t)((lds_doubles + 1) & ~1) * sizeof(double) + (size_t)(2 * kBlock / kWave) * ring * 2 * kWave * sizeof(double);
}

// The ring kernels may need more than the 64 KB default dynamic LDS.
int a2_ring_prepare()
{
    const int lim = 160 * 1024 - 1024;
    hipError_t e = hipSuccess;
#define HPCCG_A2R_ATTR(W, R)                                                                                               \
    if (e == hipSuccess)                                                                                                \
        e = hipFuncSetAttribute((const void*)k_spmv_a2r<true, W, R>, hipFuncAttributeMaxDynamicSharedMemorySize, lim); \
    if (e == hipSuccess)                                                                                                \
        e = hipFuncSetAttribute((const void*)k_spmv_a2r<false, W, R>, hipFuncAttributeMaxDynamicSharedMemorySize, lim);
    HPCCG_A2R_ATTR(27, kA2RingDefault) HPCCG_A2R_ATTR(7, kA2RingDefault)
#undef HPCCG_A2R_ATTR
    if (e == hipSuccess)  // the timeline diagnostic's instantiation
        e = hipFuncSetAttribute((const void*)k_spmv_a2r<true, 27, 3, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                lim);
    return e == hipSuccess ? 0 : -1;
}


// The SpMV of one CG iteration (or of the prologue). Template choice:
//   kSpmvSell   k_spmv_sell, non-temporal above the Infinity Cache (a.nt)
//   kSpmvDirect k_spmv_a: width 27 with 4 value slots and the offsets early,
//               width 7, or any width; a.fuse_p selects the fused p update
//   kSpmvPairs  k_spmv_a2, 3 value slots early
void launch_cg_spmv(const CgArgs& a, int kernel, bool prologue, hipStream_t s)
{
    const bool fuse = a.fuse_p && !prologue;
    // x_defer 2: the side-flush blocks trail the units (one launch per iteration carries them)
    const bool side = !prologue && a.xdefer == 2 && a.xside &&
                      ((kernel == kSpmvPairs && a.a2_ring > 0) || kernel == kSpmvDirect);
    const int spu = kernel == kSpmvPairs ? 2 : 1;
    const int nside = side ? side_blocks(a.nslices, a.nring, spu) : 0;
    // fused update: a.grid update blocks after the side blocks, from a block
    // index that is a multiple of kNumXcd (their XCD-aware slice order)
    const bool fu = !prologue && a.fupd && kernel == kSpmvDirect && fuse;
    // r-halo: ghost blocks, the launch's last, store p_k at the ghost rows
    const int gtot = a.ghost_lo + a.ghost_hi;
    const int gthreads = kernel == kSpmvPairs ? 2 * kBlock : kBlock;
    // (about four rows per thread); the fused launch's also pull r_k (a.pull_in)
    const int ptot = (fu && a.pull_in) ? a.pl_lo + a.pl_hi : 0;
    const int gmax = gtot > ptot ? gtot : ptot;
    const int nghost = (fuse && a.rhalo && gmax > 0) ? (gmax + 4 * gthreads - 1) / (4 * gthreads) : 0;
    CgArgs b = a;
    b.send = a.sgrid + nside;
    // resident fused update (k_spmv_ar, width 27): [pair units | side blocks]
    if (fu && a.resident && a.a_width == 27 && kernel == kSpmvDirect) {
        const int pairs = (a.nslices + 1) / 2;
        b.s0 = 0;
        b.sn0 = pairs;
        b.s1 = b.sn1 = 0;
        b.sgrid = (pairs + kNumXcd - 1) / kNumXcd * kNumXcd;
        b.send = b.sgrid + nside;
        b.ubase = b.gbase = INT_MAX;
        if (a.nt)
            hipLaunchKernelGGL((k_spmv_ar<true>), dim3(b.send), dim3(kBlock), 0, s, b, prologue);
        else
            hipLaunchKernelGGL((k_spmv_ar<false>), dim3(b.send), dim3(kBlock), 0, s, b, prologue);
        return;
    }
    // update units: two slices per block (four rows per thread)
    const int ugrid = ((a.nslices + 1) / 2 + kNumXcd - 1) / kNumXcd * kNumXcd;
    // fused update: [units | side | pad to kNumXcd | update | ghost]; else [units | side | ghost]
    b.ubase = fu ? (b.send + kNumXcd - 1) / kNumXcd * kNumXcd : 0;
    b.gbase = nghost ? (fu ? b.ubase + ugrid : b.send) : INT_MAX;
    const dim3 sg((fu ? b.ubase + ugrid : b.send) + nghost);
    // diagnostics: the block-timeline instantiations of the two fused-update defaults
    if (kernel == kSpmvDirect && fu && a.dbg_tl && a.a_width == 7 && a.nt && a.atri) {
        hipLaunchKernelGGL((k_spmv_a<7, true, true, 7, true, true, true>), sg, dim3(kBlock), 0, s, b, prologue);
        return;
    }
    if (kernel == kSpmvDirect && fu && a.dbg_tl && a.a_width == 27 && !a.nt) {
        hipLaunchKernelGGL((k_spmv_a<27, false, true, 4, false, true, true>), sg, dim3(kBlock), 0, s, b, prologue);
        return;
    }
#define HPCCG_A(W, NT, PRE)                                                                                       \
    do {                                                                                                          \
        if (fu && a.atri && tri_groups(W) > 0 && PRE > 0)                                                       \
            hipLaunchKernelGGL((k_spmv_a<W, NT, true, PRE, true, true>), sg, dim3(kBlock), 0, s, b, prologue); \
        else if (fu)                                                                                              \
            hipLaunchKernelGGL((k_spmv_a<W, NT, true, PRE, false, true>), sg, dim3(kBlock), 0, s, b, prologue); \
        else if (a.atri && tri_groups(W) > 0 && PRE > 0 && fuse)                                                \
            hipLaunchKernelGGL((k_spmv_a<W, NT, true, PRE, true>), sg, dim3(kBlock), 0, s, b, prologue); \
        else if (a.atri && tri_groups(W) > 0 && PRE > 0)                                                        \
            hipLaunchKernelGGL((k_spmv_a<W, NT, false, PRE, true>), sg, dim3(kBlock), 0, s, b, prologue); \
        else if (fuse)                                                                                            \
            hipLaunchKernelGGL((k_spmv_a<W, NT, true, PRE>), sg, dim3(kBlock), 0, s, b, prologue);       \
        else                                                                                                      \
            hipLaunchKernelGGL((k_spmv_a<W, NT, false, PRE>), sg, dim3(kBlock), 0, s, b, prologue);      \
    } while (0)
    switch (kernel) {
    case kSpmvPairs: {
        if (a.a2_ring > 0) {
            const size_t smem = a2_lds_bytes(a.alds2_doubles, a.a2_ring);
            if (fuse && a.dbg_tl && a.a_width == 27 && a.a2_ring == 3) {  // diagnostics: block timeline
                hipLaunchKernelGGL((k_spmv_a2r<true, 27, 3, true>), sg, dim3(2 * kBlock), smem, s, b, prologue);
                break;
            }
#define HPCCG_A2R(W, R)                                                                                           \
    do {                                                                                                          \
        if (fuse)                                                                                                 \
            hipLaunchKernelGGL((k_spmv_a2r<true, W, R>), sg, dim3(2 * kBlock), smem, s, b, prologue); \
        else                                                                                                      \
            hipLaunchKernelGGL((k_spmv_a2r<false, W, R>), sg, dim3(2 * kBlock), smem, s, b, prologue); \
    } while (0)
            // (one ring depth, kA2RingDefault: 1, 2 and 4 measured slower)
            if (a.a_width == 7)
                HPCCG_A2R(7, kA2RingDefault);
            else
                HPCCG_A2R(27, kA2RingDefault);
#undef HPCCG_A2R
            break;
        }
        const size_t smem = (size_t)a.alds2_doubles * sizeof(double);
        if (fuse)
            hipLaunchKernelGGL((k_spmv_a2<true, true, 3>), sg, dim3(2 * kBlock), smem, s, b, prologue);
        else
            hipLaunchKernelGGL((k_spmv_a2<true, false, 3>), sg, dim3(2 * kBlock), smem, s, b, prologue);
        break;
    }
    case kSpmvDirect:
        // value slots loaded before the iteration test: 4 of 27 (the offsets
        // early too), all 7 of 7 (7-pt 256^3 same-process A/B: 2445 vs 2422
        // it/s against 3); other depths measured even or slower
        if (a.a_width == 27) {
            if (a.nt) HPCCG_A(27, true, 4); else HPCCG_A(27, false, 4);
        } else if (a.a_width == 7) {
            if (a.nt) HPCCG_A(7, true, 7); else HPCCG_A(7, false, 7);
        } else {
            if (a.nt) HPCCG_A(0, true, 0); else HPCCG_A(0, false, 0);
        }
        break;
    default:
        if (a.nt)
            hipLaunchKernelGGL((k_spmv_sell<true>), sg, dim3(kBlock), 0, s, b, prologue);
        else
            hipLaunchKernelGGL((k_spmv_sell<false>), sg, dim3(kBlock), 0, s, b, prologue);
        break;
    }
#undef HPCCG_A
}

// Host restatement check of the slot completion's waiter choice (the same
// functions the kernels run): for each group, its waiting unit; the top group.
int slot_plan(int units, int grid, int spu, int rev, int* last_unit, int* top)
{
    if (units < 1 || grid < units || grid % kNumXcd || (spu != 1 && spu != 2)) return -1;
    const UnitMap m{units, grid / kNumXcd, spu, rev != 0};
    const int ng = (units * spu + kGroup - 1) / kGroup;
    for (int g = 0; g < ng; g++) last_unit[g] = group_last_unit(m, g);
    *top = top_group(m);
    return ng;
}

void launch_stream_a(const CgArgs& a, hipStream_t s)
{
    hipLaunchKernelGGL(k_stream_a, dim3(a.grid), dim3(kBlock), 0, s, a);
}

// Blocks of k_spmv_ar the whole chip holds at once (the host's residency
// check), at most 4 per CU -- the occupancy the kernel is built for
// (amdgpu_waves_per_eu(4, 4)). The occupancy API reported 5 once the pruned
// build brought the kernel to 90 VGPRs, yet a 1040-block launch (102^3) then
// timed out in its p.Ap wait on the GPU (not every block was resident):
// residency is only trusted at the designed 4.
constexpr int kResidentPerCu = 4;
int resident_capacity(bool nt)
{
    int per_cu = 0, dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return 0;
    const hipError_t e = nt ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_spmv_ar<true>, kBlock, 0)
                            : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_spmv_ar<false>, kBlock, 0);
    return e == hipSuccess ? (per_cu < kResidentPerCu ? per_cu : kResidentPerCu) * cus : 0;
}

int persist_capacity(bool nt)
{
    int per_cu = 0, dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return 0;
    int per_cu_mr = 0;  // (the multi-rank form's figure too: the smaller counts)
    hipError_t e = nt ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_cg_persist<true>, kBlock, 0)
                      : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_cg_persist<false>, kBlock, 0);
    if (e == hipSuccess)
        e = nt ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu_mr, k_cg_persist<true, true>, kBlock, 0)
               : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu_mr, k_cg_persist<false, true>, kBlock, 0);
    per_cu = per_cu < per_cu_mr ? per_cu : per_cu_mr;
    return e == hipSuccess ? (per_cu < kResidentPerCu ? per_cu : kResidentPerCu) * cus : 0;
}

void launch_cg_persist(const CgArgs& a, hipStream_t s)
{
    const int pairs = (a.nslices + 1) / 2;
    CgArgs b = a;
    b.s0 = 0;
    b.sn0 = pairs;
    b.s1 = b.sn1 = 0;
    b.sgrid = (pairs + kNumXcd - 1) / kNumXcd * kNumXcd;
    b.send = b.sgrid;
    b.ubase = b.gbase = INT_MAX;
    if (a.pranks > 1) {  // (a z-slab rank: the peer all-reduce and the pull in the kernel)
        if (a.nt)
            hipLaunchKernelGGL((k_cg_persist<true, true>), dim3(b.sgrid), dim3(kBlock), 0, s, b);
        else
            hipLaunchKernelGGL((k_cg_persist<false, true>), dim3(b.sgrid), dim3(kBlock), 0, s, b);
    } else if (a.nt) {
        hipLaunchKernelGGL((k_cg_persist<true>), dim3(b.sgrid), dim3(kBlock), 0, s, b);
    } else {
        hipLaunchKernelGGL((k_cg_persist<false>), dim3(b.sgrid), dim3(kBlock), 0, s, b);
    }
}

__global__ __launch_bounds__(256) void k_fill_empty(double* p, long long n)
{
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i < n) p[i] = slot_empty();
}

void launch_fill_empty(double* p, long long n, hipStream_t s)
{
    if (n > 0) hipLaunchKernelGGL(k_fill_empty, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, p, n);
}

void launch_cg_finalize(const CgArgs& a, int which, bool prologue, hipStream_t s)
{
    hipLaunchKernelGGL(k_finalize, dim3(1), dim3(kFinalizeThreads), 0, s, a, which, prologue);
}

void launch_cg_update(const CgArgs& a, bool prologue, hipStream_t s)
{
    // in-launch pull: trailing blocks, about four rows per thread
    const int ptot = a.pull_in ? (a.npseg ? a.pseg_rows : a.pl_lo + a.pl_hi) : 0;
    const dim3 grid(a.grid + (ptot + 4 * kBlock - 1) / (4 * kBlock));
    if (prologue)
        hipLaunchKernelGGL((k_update<true>), grid, dim3(kBlock), 0, s, a);
    else
        hipLaunchKernelGGL((k_update<false>), grid, dim3(kBlock), 0, s, a);
}

void launch_cg_stamp(const CgArgs& a, int slot, bool prologue, hipStream_t s)
{
    hipLaunchKernelGGL(k_stamp, dim3(1), dim3(64), 0, s, a, slot, prologue);
}

void launch_cg_end(const CgArgs& a, hipStream_t s) { hipLaunchKernelGGL(k_end, dim3(1), dim3(64), 0, s, a); }

void launch_pull(const CgArgs& a, const double* lo_src, double* lo_dst, int lo_cnt, const double* hi_src, double* hi_dst,
                 int hi_cnt, hipStream_t s, bool force, bool pexpr)
{
    const int tot = lo_cnt + hi_cnt;
    if (tot <= 0) return;
    const int grid = (tot + 4 * 256 - 1) / (4 * 256);
    hipLaunchKernelGGL(k_pull, dim3(grid), dim3(256), 0, s, a, lo_src, lo_dst, lo_cnt, hi_src, hi_dst, hi_cnt,
                       (force ? 1 : 0) | (pexpr ? 2 : 0));
}

void launch_peer_barrier(const CgArgs& a, hipStream_t s)
{
    hipLaunchKernelGGL(k_peer_barrier, dim3(1), dim3(64), 0, s, a);
}

void launch_peer_selftest(const CgArgs& a, int rounds, double* out, hipStream_t s)
{
    hipLaunchKernelGGL(k_peer_selftest, dim3(1), dim3(64), 0, s, a, rounds, out);
}

void launch_rearm(int* kst, double* partial, int np, int budget, hipStream_t s)
{
    const int cnt = np > 2 * kKstDoubles ? np : 2 * kKstDoubles;
    hipLaunchKernelGGL(k_rearm, dim3((cnt + 255) / 256), dim3(256), 0, s, kst, partial, np, budget);
}

void launch_group_sum(const GroupSum& gs, hipStream_t s)
{
    hipLaunchKernelGGL(k_group_sum, dim3(1), dim3(1), 0, s, gs);
}

void launch_cg_xflush(const CgArgs& a, hipStream_t s)
{
    if (a.xdefer) hipLaunchKernelGGL(k_xflush, dim3(a.grid), dim3(kBlock), 0, s, a);
}

void launch_waxpby(int n, double alpha, const double* x, double beta, const double* y, double* w, hipStream_t s)
{
    if (n <= 0) return;
    int grid = (n + 255) / 256;
    if (grid > 8192) grid = 8192;
    hipLaunchKernelGGL(k_waxpby, dim3(grid), dim3(256), 0, s, n, alpha, x, beta, y, w);
}

int ddot_nparts(int n) { return n <= 0 ? 1 : (n + kDotChunk - 1) / kDotChunk; }

void launch_ddot(int n, const double* x, const double* y, double* partial, int nparts, double* out, hipStream_t s)
{
    if (n > 0) hipLaunchKernelGGL(k_dot_partial, dim3(nparts), dim3(256), 0, s, n, x, y, partial);
    hipLaunchKernelGGL(k_dot_final, dim3(1), dim3(kDotFinalThreads), 0, s, partial, n > 0 ? nparts : 0, out);
}

void launch_sparsemv(const CgArgs& a, const double* xext, double* y, hipStream_t s)
{
    hipLaunchKernelGGL(k_spmv_plain, dim3(a.grid), dim3(kBlock), 0, s, a, xext, y);
}

void launch_generate(int nx, int ny, int nz, int rank, int size, int use_7pt, long long col_base,
                     const unsigned int* slice_base, int* cols, double* vals, double* b, double* xexact, int nrow,
                     hipStream_t s)
{
    if (nrow <= 0) return;
    const int nslices = (nrow + kSliceRows - 1) / kSliceRows;
    hipLaunchKernelGGL(k_generate, dim3((nrow + 255) / 256), dim3(256), 0, s, nx, ny, nz, rank, size, use_7pt,
                       col_base, slice_base, cols, vals, b, xexact, nrow);
    hipLaunchKernelGGL(k_generate_tail, dim3(1), dim3(kSliceRows), 0, s, nrow, nslices, slice_base, cols, vals);
}

void launch_a_offsets(const unsigned int* slice_base, int nslices, const int* cols, int ghost_lo, int* aoff,
                      int* acount, int* ok, int* maxabs, hipStream_t s)
{
    if (nslices <= 0) return;
    hipLaunchKernelGGL(k_a_offsets, dim3(nslices), dim3(kSliceRows), 0, s, slice_base, nslices, cols, ghost_lo, aoff,
                       acount, ok, maxabs);
}

void launch_a_fill(const unsigned int* slice_base, int nslices, const int* cols, const double* vals, int ghost_lo,
                   const int* aoff, const int* acount, const unsigned int* abase, double* aval, hipStream_t s)
{
    if (nslices <= 0) return;
    hipLaunchKernelGGL(k_a_fill, dim3(nslices), dim3(kSliceRows), 0, s, slice_base, nslices, cols, vals, ghost_lo,
                       aoff, acount, abase, aval);
}

}  // namespace hpccg
