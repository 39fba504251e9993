// hpccg_internal.h -- shared between the kernel TU (hpccg_kernels.hip) and the
// host orchestration TU (hpccg_solver.cpp). Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace hpccg {

// SELL-C layout: C rows per slice, slot-major inside a slice. C is fixed so
// that one workgroup owns exactly one slice in every CG kernel, which keeps
// the per-slice dot partials of every kernel aligned (deterministic sums).
constexpr int kSliceRows = 512;
constexpr int kNumXcd = 8;        // MI355X: 8 XCDs, blocks dealt round-robin

// Indices into the device scalar block.
enum Scalar : int { kRR = 0, kPAP = 1 };

// Stamp slots (SURVEY 8(a) TICK/TOCK classes, HPCCG.cpp:71-72).
enum StampSlot : int {
    kStampPUpdate = 0,  // waxpby p = r + beta p       -> WAXPBY
    kStampHalo = 1,     // halo exchange starts         -> exchange (t5)
    kStampSpmv = 2,     // SpMV (+ fused p.Ap partials) -> SPARSEMV
    kStampFinPAP = 3,   // final p.Ap reduction         -> DDOT
    kStampArPAP = 4,    // all-reduce of p.Ap           -> DDOT + all-reduce (t4)
    kStampUpdate = 5,   // x += a p, r -= a Ap (+ r.r)  -> WAXPBY
    kStampFinRR = 6,    // final r.r reduction          -> DDOT
    kStampArRR = 7,     // all-reduce of r.r            -> DDOT + all-reduce (t4)
    kStampPrologue = 8, // p = x, r = b - Ap            -> WAXPBY
    kStampEnd = 9,
    kNumStampSlots = 10
};

// Everything a CG kernel needs, passed by value (graph-capture friendly: all
// per-iteration state lives in device memory, never in kernel arguments).
struct CgArgs {
    int n;                 // local rows
    int nslices;           // ceil(n / kSliceRows)
    int grid;              // nslices rounded up to a multiple of kNumXcd
    int max_iter;
    double tol;
    int nranks;
    int ghost_lo;          // halo rows below (in p only)
    const double* b;
    double* x;
    double* r;
    double* p;             // local rows of p; p - ghost_lo .. p + n + ghost_hi valid
    long long pstride;     // distance between ring buffers of p (doubles)
    int nring;             // p_k lives in ring buffer k % nring (1 = in place)
    int xdefer;            // 1: x += alpha_j p_j applied every nring iterations
    int rev;               // 1: the update kernel walks each XCD's slices backwards
    int redund;            // 1: no finalize kernels: consumers sum the producers' partials themselves
    int ugrid;             // k_update_g grid (groups rounded up to a multiple of kNumXcd)
    int um;                // slices per k_update workgroup (1: k_update, else k_update_m)
    int uearly;            // um = 1: k_update_e (Ap and r loaded before the iteration test)
    int pap_upd;           // one rank, um = 1: k_update_pr forms p.Ap itself (SpMV: partials only)
    double* ppart;         // pap_upd: the SpMV's p.Ap slice partials (apart from the r.r ones)
    int umgrid;            // k_update_m grid (slice blocks of um rounded up to a multiple of kNumXcd)
    int s0, sn0, s1, sn1;  // SpMV launch: slices [s0, s0 + sn0) then [s1, s1 + sn1)
    int sgrid;             // SpMV launch grid (sn0 + sn1 rounded up to a multiple of kNumXcd)
    int nt_split;          // NT matrix kernels: per XCD, this many leading slices use default-policy loads
    double* ahist;         // [max_iter + 1]: alpha_k (for the deferred x update)
    int fuse_p;            // 1: p = r + beta p computed inside the SpMV (single rank)
    int fold;              // dots completed in the producing kernel: 0 none, 1 both, 2 p.Ap only, 3 r.r only
    unsigned int* tickets; // [2 x (ngroups + 1)] arrival counters (fold): groups, top
    double* Ap;
    double* partial;       // [nslices] slice partials, then 2 x ngroups group sums
    double* g;             // [2] dot results after the all-reduce
    double* loc;           // [2] local dot results
    double* hist;          // [max_iter + 1]: hist[j] = r_j . r_j (global)
    int* kst;              // [0] next iteration k, [1] end stamped, [2] stamp count
    unsigned long long* stamps;  // pairs (s_memrealtime, slot)
    int stamp_cap;         // capacity in pairs
    // SELL-512 matrix
    const unsigned int* slice_base;  // [nslices + 1], units of kSliceRows slots
    const int* cols;       // local column (ghost-inclusive base), -1 = padding
    const double* vals;
    // SELL-512-L: per-slice x windows staged in LDS + slice-local indices
    const unsigned short* lcols;  // LDS index of the column, kLdsPad = padding
    const unsigned char* ccodes;  // SELL-512-C: per entry, code of its (column - row) offset
    const int* cdict;             // SELL-512-C: per slice, kCodes offsets
    const int* ldsc;              // SELL-512-C: per slice, LDS position of lane 0's column per code
    const double* cval;           // SELL-512-V: per slice, kCodes values (codes name (offset, value) pairs)
    const int* ccount;            // SELL-512-C / -V: per slice, codes in use (dictionary entries to load)
    const unsigned int* vbase4;   // SELL-512-V4: [nslices + 1] first chunk of each slice (4 slots x 512 rows)
    const unsigned char* vcodes4; // SELL-512-V4: the V codes, a row's 4 codes of a chunk contiguous
    const unsigned char* prow;    // SELL-512-P: per row, its pattern id within the slice
    const int* pcount;            // SELL-512-P: per slice, patterns
    const int* pbase;             // SELL-512-P: per slice, first entry of its pattern table
    const int* ptab_g;            // SELL-512-P: pattern tables, column - row per slot (kPatPad = padding)
    const int* ptab_l;            // SELL-512-P: pattern tables, LDS position - lane per slot
    const double* aval;           // SELL-512-A: values in offset-aligned slots (holes 0.0)
    const int* aoff;              // SELL-512-A: per slice, kAMax offsets (column - row), ascending
    const unsigned int* abase;    // SELL-512-A: [nslices + 1] first slot row of each slice
    const int* alds;              // SELL-512-A LDS: per slice, kAMax LDS positions (minus the lane's row)
    const int* awin;              // SELL-512-A LDS: per slice, kAWin windows (first row - slice row, length, LDS base)
    const int* awn;               // SELL-512-A LDS: windows per slice
    int alds_doubles;             // SELL-512-A LDS: dynamic LDS per block (largest window total)
    const int* alds2;             // SELL-512-A pair windows: per slice, kAMax LDS positions (minus the pair row)
    const int* awin2;             // per slice pair, kAWin windows (first row - pair row, length, LDS base)
    const int* awn2;              // windows per slice pair
    int alds2_doubles;            // dynamic LDS per two-slice block
    int pgrid;                    // two-slice blocks, rounded up to a multiple of kNumXcd
    const int* alds4;             // the same for groups of four slices (k_spmv_la2<..., 4>)
    const int* awin4;
    const int* awn4;
    int alds4_doubles;
    int qgrid;
    // group kernels (pair / quad windows): group ranges [gs0, gs0 + gn0) then
    // [gs1, gs1 + gn1), as s0/sn0/s1/sn1 for the one-slice kernels; pgrid /
    // qgrid cover gn0 + gn1. agroup = slices per group of the variant (0: none)
    int agroup, gs0, gn0, gs1, gn1;
    int pat_max;                  // SELL-512-P: largest table (ints) over slices: dynamic LDS
    const int* win_ptr;    // [nslices + 1] into the window arrays
    const int* win_start;  // first local column of the window
    const int* win_len;    // entries
    const int* win_off;    // LDS offset (doubles)
    int lds_doubles;       // dynamic LDS per block (max staged entries over slices)
};

// Is dot `which` (kRR / kPAP) completed inside its producing kernel?
inline __host__ __device__ bool fold_of(const CgArgs& a, int which)
{
    if (which == kPAP && a.pap_upd) return false;  // the update kernel sums the partials itself
    return a.fold == 1 || (a.fold == 2 && which == kPAP) || (a.fold == 3 && which == kRR);
}


constexpr unsigned short kLdsPad = 0xFFFF;
constexpr int kLdsMaxDoubles = 8192;  // 64 KiB of LDS per block at most
constexpr int kLdsMaxWindows = 16;
// p ring length = x-update deferral depth (option x_ring) for images well
// beyond the Infinity Cache. 32 vs 8, in-CG update kernel: 7-pt 256^3 92.8 vs
// 102.7 us, 200^3 45.4 vs 46.6 us.
constexpr int kXRingDefault = 32;
constexpr int kXRingMax = 64;

// ---- launches (hpccg_kernels.hip) -----------------------------------------
// CG iteration pieces; all take the same CgArgs.
void launch_cg_prologue_copy(const CgArgs& a, hipStream_t s);   // p = x + 0*x
void launch_cg_p_update(const CgArgs& a, hipStream_t s);        // p = r + beta p
void launch_cg_p_boundary(const CgArgs& a, int nlo, int nhi, hipStream_t s);  // same, halo rows only
// gather plan: buf[i] = p_k[idx[i]] (computed when fused; prologue: p = x)
void launch_cg_pack(const CgArgs& a, const int* idx, int cnt, double* buf, bool prologue, hipStream_t s);
void launch_cg_spmv(const CgArgs& a, int variant, bool prologue, hipStream_t s);
bool spmv_variant_ok(int variant);
void launch_cg_finalize(const CgArgs& a, int which, bool prologue, hipStream_t s);
void launch_cg_update(const CgArgs& a, bool prologue, hipStream_t s);
void launch_cg_stamp(const CgArgs& a, int slot, bool prologue, hipStream_t s);
void launch_cg_end(const CgArgs& a, hipStream_t s);
void launch_cg_xflush(const CgArgs& a, hipStream_t s);  // pending deferred x updates

// In-process rank group all-reduce of one CG scalar: g[which] of every rank =
// sum of loc[which] over ranks, in rank order.
constexpr int kMaxGroupRanks = 16;
struct GroupSum {
    int nranks;
    int which;
    const double* loc[kMaxGroupRanks];
    double* g[kMaxGroupRanks];
};
void launch_group_sum(const GroupSum& gs, hipStream_t s);

// Kernel-level ops on arbitrary device pointers.
void launch_waxpby(int n, double alpha, const double* x, double beta, const double* y, double* w,
                   hipStream_t s);
void launch_ddot(int n, const double* x, const double* y, double* partial, int nparts,
                 double* out, hipStream_t s);
int ddot_nparts(int n);
void launch_sparsemv(const CgArgs& a, const double* xext, double* y, int variant, hipStream_t s);

// SELL-512-C from the SELL-512 cols on the device (windows optional); with
// vals and cval non-null, SELL-512-V (codes of (offset, value) pairs, cval[s *
// kCodes + code] = value). ccount[s] = codes in use. ok[0] = 0 if a slice has more than 255 distinct
// keys, ok[1] = 0 if a code's entries fall in different windows (no LDS form).
constexpr int kCodes = 256;
constexpr unsigned kCodePad = 255;
void launch_build_c(const unsigned int* slice_base, int nslices, const int* cols, const double* vals,
                    const int* win_ptr, const int* win_start, const int* win_off, const int* win_len,
                    unsigned char* codes, int* cdict, double* cval, int* ldsc, int* ccount, int* ok,
                    hipStream_t s);
// SELL-512-P (per-row pattern ids over the SELL-512-C codes): pass 1 writes
// prow, prep[s * kMaxPat + id] (representative lane), pcount; ok[0] = 0 when a
// slice does not fit. Pass 2 writes the tables at pbase (host prefix sum of
// pcount * width): tab_g from cdict, tab_l from ldsc (may be null).
constexpr int kMaxPat = 256;
constexpr int kPatCap = 2048;          // table entries per slice at most (LDS ints)
constexpr int kPatPad = -2147483647 - 1;  // padding slot
void launch_build_p(const unsigned int* slice_base, int nslices, const unsigned char* codes, unsigned char* prow,
                    int* prep, int* pcount, int* ok, hipStream_t s);
void launch_fill_p(const unsigned int* slice_base, int nslices, const unsigned char* codes, const int* prep,
                   const int* pcount, const int* pbase, const int* cdict, const int* ldsc, int* tab_g, int* tab_l,
                   hipStream_t s);
// SELL-512-A (offset-aligned slots) from the SELL-512-C codes: slot j of slice
// s holds, for every row, the entry at the slice's j-th smallest offset (0.0
// where the row has none). abase from the host prefix of ccount. aoff[s *
// kAMax + j] = offset. ok[0] = 0 when a slice has more than kAMax offsets or a
// row's entries are not in ascending offset order; maxabs = max |offset|.
constexpr int kAMax = 32;
// SELL-512-A LDS windows: a slice's offsets cut where two neighbours are more
// than a slice apart; each window stages every row of the slice at every
// offset of its range (holes included), at most kAWin windows and kALdsMax
// doubles per slice.
constexpr int kAWin = 8;
constexpr int kALdsMax = 8000;  // + static LDS within the 64 KB default dynamic limit
// Two-slice blocks (k_spmv_la2): windows over both slices' offsets, so
// neighbouring slices share their staged planes.
constexpr int kALdsMax2 = 7936;
constexpr int kALdsMax4 = 7936;
void launch_build_a(const unsigned int* slice_base, int nslices, const unsigned char* codes, const double* vals,
                    const int* cdict, const int* ccount, const unsigned int* abase, double* aval, int* aoff,
                    int* ok, int* maxabs, hipStream_t s);
// SELL-512-V4 regrouping of the V codes (vbase4 in chunks of 4 slots).
void launch_interleave_v4(const unsigned int* slice_base, const unsigned int* vbase4, int nslices,
                          const unsigned char* codes, unsigned char* out, hipStream_t s);
// Device generator: writes the SELL-512 image, b, xexact.
// With win_* non-null it also writes the SELL-512-L index image (lcols).
void launch_generate(int nx, int ny, int nz, int rank, int size, int use_7pt, long long col_base,
                     const unsigned int* slice_base, int* cols, double* vals, double* b,
                     double* xexact, int nrow, const int* win_ptr, const int* win_start,
                     const int* win_len, const int* win_off, unsigned short* lcols, hipStream_t s);

}  // namespace hpccg
