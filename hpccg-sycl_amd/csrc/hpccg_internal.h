// hpccg_internal.h -- shared between the kernel TU (hpccg_kernels.hip) and the
// host orchestration TU (hpccg_solver.cpp). Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace hpccg {

// SELL-C layout: C rows per slice, slot-major inside a slice. C is fixed so
// that one workgroup owns exactly one slice (two for the pair kernel) in every
// CG kernel, which keeps the per-slice dot partials of every kernel aligned
// (deterministic sums).
constexpr int kSliceRows = 512;
constexpr int kNumXcd = 8;  // MI355X: 8 XCDs, blocks dealt round-robin
constexpr int kReadyStride = 16;  // doubles between the fused update's p.Ap ready slots (128 B)
// The persistent launch's broadcast copies of each dot total (blocks poll copy
// blockIdx % kPersBcast): at 100^3, 64 copies measured +0.1-0.2 % over one per
// XCD (12 alternating runs), 128 another +0.25 % over 64 (13 runs, two
// sessions), 256 -0.25 % (profiles/r06_ab/persist_bcast_copies_ab100.log)
#ifndef HPCCG_BCAST
#define HPCCG_BCAST 128
#endif
constexpr int kPersBcast = HPCCG_BCAST;

// Indices into the device scalar block (g = scal[0..], loc = scal[2..]).
// kRRPar: with the fused update (a.fupd) r.r is also kept in two slots by the
// parity of the iteration that reads it, g[kRRPar + (k & 1)] = r_{k-1}.r_{k-1},
// so no block of a launch -- the ghost blocks are outside the launch's
// p.Ap -> update -> r.r chain -- can read the r.r its own launch writes.
enum Scalar : int { kRR = 0, kPAP = 1, kRRPar = 4 };

// Stamp slots (SURVEY 8(a) TICK/TOCK classes, HPCCG.cpp:71-72); stamps are
// stored at [k * kNumStampSlots + slot] for iteration k (0 = the prologue),
// the end stamp at [(max_iter + 1) * kNumStampSlots + kStampEnd].
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

// SpMV kernels (option "spmv_kernel").
enum SpmvKernel : int {
    kSpmvSell = 0,    // SELL-512, int32 columns, x gathered from p_k (any matrix)
    kSpmvDirect = 1,  // SELL-512-A, x read at the slice's offsets
    kSpmvPairs = 2,   // SELL-512-A, x from LDS windows shared by slice pairs
};

// Everything a CG kernel needs, passed by value (graph-capture friendly: all
// per-iteration state lives in device memory, never in kernel arguments).
// One run of rows a pull copies: src (another member's boundary rows) -> dst.
struct PullSeg {
    const double* src;
    double* dst;
    long long cnt;
};

struct CgArgs {
    int n;                 // local rows
    int nslices;           // ceil(n / kSliceRows)
    int grid;              // nslices rounded up to a multiple of kNumXcd
    int max_iter;
    double tol;
    int nranks;
    int allreduce;         // 1: the dot scalars go through an all-reduce (loc -> g) after the local sum
    int ghost_lo;          // halo rows below (in p only)
    const double* b;
    double* x;
    double* r;             // r with zeroed guard zones (the fused A kernels read holes there)
    double* p;             // local rows of ring buffer 0; p - ghost_lo .. p + n + ghost_hi valid
    long long pstride;     // distance between ring buffers of p (doubles)
    int nring;             // p_k lives in ring buffer k % nring
    int xdefer;            // deferred x += alpha_j p_j: 1 every nring-th update, all rows; 2 beside the SpMV (side_flush)
    int rev;               // 1: the update kernel walks each XCD's slices backwards
    int s0, sn0, s1, sn1;  // SpMV launch: units [s0, s0 + sn0) then [s1, s1 + sn1) (slices; pairs for kSpmvPairs)
    int sgrid;             // SpMV launch grid (sn0 + sn1 rounded up to a multiple of kNumXcd)
    int nt;                // non-temporal matrix loads (image beyond the Infinity Cache)
    int a_width;           // SELL-512-A uniform slot count (27, 7, ...), 0 = per-slice widths
    double* ahist;         // [max_iter + 1]: alpha_k (for the deferred x update)
    int fuse_p;            // 1: p = r + beta p computed inside the SpMV
    int fold;              // dots completed in the producing kernel: 0 none, 1 both, 2 p.Ap only, 3 r.r only
    double* Ap;
    double* partial;       // [2 x nslices] slice partials (p.Ap, r.r), then 2 x ngroups group sums
    double* g;             // [2] dot results after the all-reduce
    double* loc;           // [2] local dot results
    double* hist;          // [max_iter + 1]: hist[j] = r_j . r_j (global)
    int* kst;              // [0] next iteration k, [1] end stamped
    unsigned long long* stamps;  // [(max_iter + 2) x kNumStampSlots] s_memrealtime
    // SELL-512 matrix (the general kernel; kept only when no A image exists)
    const unsigned int* slice_base;  // [nslices + 1], units of kSliceRows slots
    const int* cols;       // local column (ghost-inclusive base), -1 = padding
    const double* vals;
    // SELL-512-A: values in per-slice offset-aligned slots (holes 0.0)
    const double* aval;
    const int* aoff;              // per slice, kAMax offsets (local column - row), ascending
    const unsigned int* abase;    // [nslices + 1] first slot row of each slice
    const int* alds2;             // pair windows: per slice, kAMax LDS positions (minus the pair row)
    const int* awin2;             // per pair, kAWin windows (first row - pair row, length, LDS base)
    const int* awn2;              // windows per pair
    const int* adiag2;            // per slice: LDS position of offset 0 (minus the pair row), -1 none
    const unsigned char* atri;    // direct kernel: per slice, 1 = offsets in the width's triple plan (null: off)
    int alds2_doubles;            // dynamic LDS per two-slice block
    int nt_store;                 // CG vector stores non-temporal
    int a2_ring;                  // pair kernel: value slots in flight per wave through its LDS-DMA ring (0: register loads)
    int xside;                    // x_defer 2: this SpMV launch carries the side-flush blocks
    int fupd;                     // fused update: the SpMV launch's trailing blocks run the update (one rank,
                                  // direct kernel); k lives in kst[0] / kst[2] by parity (kpar)
    int kpar;                     // fused update: parity of the iteration this launch runs
    int resident;                 // resident pair kernels: 1 k_spmv_ar, kResidentAuto k_cg_persist (option resident_update)
    int dbg_resident_stall;       // debug (retry test): k_spmv_ar's p.Ap wait never sees the total (it expires)
    int ubase;                    // fused update: first update block of the SpMV launch (set at launch)
    double* pready;               // fused update: self-validating slots of the p.Ap total (kNumXcd, kReadyStride apart)
    double* pslots;               // persistent CG (resident == kResidentAuto): per iteration pslot_stride slots, emptied first
    long long pslot_stride;
    int pk0, pk1;                 // persistent CG: the launch runs iterations [pk0, pk1) (its window)
    int pguard;                   // rows below local row 0 in r and in every p buffer (guard + ghost_lo padding)
    int dbg_withhold;             // debug (guard test): slice + 1 whose p.Ap partial is never published; 0 off
    unsigned long long* dbg_tl;   // diagnostics (option dbg_timeline): per unit 8 words of block clock stamps
                                  // (kTlWords below); null off. Only the timeline instantiation writes it.
    // r-halo exchange (multi-rank z-slabs, fused p update): the halo moves r's
    // boundary planes (with the r.r all-reduce) into r's ghost planes; the SpMV
    // forms p_k = r + beta p_{k-1} at ghost rows itself, and its ghost blocks
    // (index >= gbase) store p_k there for the next iteration's p_{k-1}
    int rhalo;
    int ghost_hi;                 // halo rows above (ghost_lo: below)
    int gbase;                    // first ghost block of the SpMV launch (set at launch; INT_MAX: none)
    // peer-memory all-reduce of the two CG scalars (option peer_allreduce): the
    // lane that completes a local dot stores it into slot [which][k & 1][prank]
    // of every rank's mailbox (peers: device table of the ranks' mailboxes,
    // IPC-mapped across processes), waits for all pranks slots of its own
    // (mbox) and sums them in rank order -- no RCCL call, no launch
    int peer_ar;
    int prank, pranks;
    double* mbox;
    double* const* peers;
    // r-halo by pull (option halo_pull): the neighbours read this rank's first
    // rsend_lo and last rsend_hi rows of r straight from its memory, so the
    // update stores those rows write-through and drains them before its r.r
    // partial (0, 0: off)
    int rsend_lo, rsend_hi;
    // In-launch pull (pull_in; halo_pull 2): the iteration's last launch --
    // the fused SpMV launch's ghost blocks, or trailing blocks of k_update --
    // reads the neighbours' boundary rows of r_k into pl_dst once its own r.r
    // completion (after the peer all-reduce) has published k + 1; pl_lo /
    // pl_hi rows from pl_src_lo / pl_src_hi (an in-process group: the members'
    // buffers; an RCCL job: IPC-mapped; the emulation: its own rows)
    int pull_in;
    // Group fold (an in-process group run in member order, both dots folded):
    // the finishing lane of the phase's last member sums the members' local
    // totals in rank order (k_group_sum's sum) and stores the total into every
    // member's g: gtab[0 .. gn) the members' loc, gtab[gn .. 2 gn) their g;
    // gfw: the dots this member folds (1 p.Ap: the SpMV phase's last, member
    // gn - 1; 2 r.r: the update phase's last, member 0); grank: its index
    int gn, gfw, grank;
    double* const* gtab;
    // the group fold's pull: member 0's update (the last launch of an
    // iteration) pulls every member's ghost planes: npseg segments of
    // pseg_rows rows in all (psegs in device memory); 0: pl_* alone
    const struct PullSeg* psegs;
    int npseg, pseg_rows;
    int send;  // one past the last side-flush block (set per launch)
    int pl_lo, pl_hi;
    const double* pl_src_lo;
    const double* pl_src_hi;
    double* pl_dst_lo;
    double* pl_dst_hi;
};
// Block timeline (dbg_timeline), per unit of the ring pair kernel: [0] block
// index | HW_ID << 32, [1] entry, [2] iteration state read, [3] windows staged
// (after the barrier), [4] slot loop done, [5] epilogue + dot hand-off done
// (s_memrealtime, 100 MHz), [6] XCC id, [7] iteration k.
constexpr int kTlWords = 8;
// Peer mailbox: [kind][k & 1][rank], kind = kRR / kPAP (the two CG scalars) or
// kMboxBarrier (the prologue's barrier before the x pull), up to kMboxRanks ranks
constexpr int kMboxRanks = 16;
constexpr int kMboxBarrier = 2;
constexpr int kMboxSlots = 3 * 2 * kMboxRanks;

// Bounded in-kernel waits: a wait that outlives the spin budget (s_memrealtime
// ticks, 100 MHz) records itself in the device error record and ends the
// solve (later launches fail the loop test); the host turns it into an error
// return. The record lives in device memory behind the iteration state,
// err = kst + kErrBase, and kst is found from a.partial (kKstDoubles below):
// the waits are a cold path and must not hold registers in the hot one.
//   err[0] code, [1] block, [2] group / slot, [3] iteration k, [4] dot (kRR /
//   kPAP), [5] the maximum code over the ranks of an RCCL job (all-reduced
//   after the solve), [6] the spin budget in ticks (u32, at most 42 s; set by the host).
constexpr int kErrBase = 8;
constexpr int kErrWords = 8;
// The state block precedes the dot slots in one allocation: kst = (int*)
// (partial - kKstDoubles). 256 B, so no slot shares a cache line with kst:
// every block reads k there at its start, and the slots' sc1 stores drop
// their line from the XCD's L2.
constexpr int kKstDoubles = 32;
static_assert(kKstDoubles * 2 >= kErrBase + kErrWords, "state block");
constexpr int kErrAllRanks = 5;
constexpr int kErrBudget = 6;
enum DevError : int {
    kErrNone = 0,
    kErrGroupWait = 1,  // a group's waiter: slice partials missing
    kErrTopWait = 2,    // the top waiter: group sums missing
    kErrReadyWait = 3,  // a fused update block: the launch's p.Ap total missing
    kErrPeerWait = 4,   // peer all-reduce: another rank's contribution missing
    kErrPullWait = 5,   // in-launch pull: the launch's r.r completion missing
};
constexpr long long kSpinTicksDefault = 100000000;  // 1 s

// Is dot `which` (kRR / kPAP) completed inside its producing kernel?
inline __host__ __device__ bool fold_of(const CgArgs& a, int which)
{
    return a.fold == 1 || (a.fold == 2 && which == kPAP) || (a.fold == 3 && which == kRR);
}

// SELL-512-A limits: at most kAMax distinct offsets per slice; the pair
// windows cut the union of a pair's offsets where neighbours are more than a
// slice apart, at most kAWin windows and kALdsMax2 staged doubles per pair.
constexpr int kAMax = 32;
// An empty dot-partial / group-sum slot: a NaN payload no arithmetic produces.
constexpr unsigned long long kSlotEmpty = 0x7FF4DEADBEEF0001ull;
constexpr int kAWin = 8;
constexpr int kALdsMax2 = 7936;  // 62 KB: within the 64 KB default dynamic LDS limit
// Zeroed guard zone on each side of every p buffer and of r: a hole of row i
// at offset o reads column i + o, where o is a real offset of some row of the
// same pair, so i + o lies within 1023 of a valid column.
constexpr long long kGuardRows = 4 * kSliceRows;

// p ring length = x-update deferral depth (option x_ring) for images well
// beyond the Infinity Cache. 32 vs 8, in-CG update kernel: 7-pt 256^3 92.8 vs
// 102.7 us, 200^3 45.4 vs 46.6 us.
constexpr int kXRingDefault = 32;
constexpr int kXRingMax = 64;

// ---- launches (hpccg_kernels.hip) -----------------------------------------
void launch_cg_prologue_copy(const CgArgs& a, hipStream_t s);   // p = x
void launch_cg_p_update(const CgArgs& a, hipStream_t s);        // p = r + beta p
// gather plan: buf[i] = p_k[idx[i]] (computed when fused; prologue: p = x)
void launch_cg_pack(const CgArgs& a, const int* idx, int cnt, double* buf, bool prologue, hipStream_t s);
bool spmv_kernel_ok(int kernel);
void launch_cg_spmv(const CgArgs& a, int kernel, bool prologue, hipStream_t s);
// Pair kernel with the LDS-DMA value ring (a2_ring > 0: uniform width 27 or 7):
// dynamic LDS bytes, and the one-time attribute that lets it exceed 64 KB.
constexpr int kA2RingDefault = 3;
size_t a2_lds_bytes(int lds_doubles, int ring);
int a2_ring_prepare();
void launch_cg_finalize(const CgArgs& a, int which, bool prologue, hipStream_t s);
// k_spmv_ar blocks the whole chip holds at once (0: unknown)
int resident_capacity(bool nt);
// persistent CG (one launch runs every iteration after the prologue): its
// capacity, the launch, and the slot fill (kSlotEmpty) that precedes it
constexpr int kResidentPersist = 6;
constexpr int kResidentAuto = 8;  // resident_update -1: the persistent launch with the 3-slot LDS ring
constexpr int kPersistWindow = 512;  // iterations per persistent launch (its slots: 32 MB at 100^3)
int persist_capacity(bool nt);
void launch_cg_persist(const CgArgs& a, hipStream_t s);
void launch_fill_empty(double* p, long long n, hipStream_t s);
// slots per iteration of the persistent launch
inline long long persist_slot_stride(int nslices)
{
    return 2LL * nslices + 2LL * ((nslices + 63) / 64) + 2LL * kPersBcast * kReadyStride;
}
void launch_cg_update(const CgArgs& a, bool prologue, hipStream_t s);
void launch_cg_stamp(const CgArgs& a, int slot, bool prologue, hipStream_t s);
void launch_cg_end(const CgArgs& a, hipStream_t s);
// peer all-reduce self-test: rounds x both scalars through peer_allreduce, results to out[2 * rounds]
void launch_peer_selftest(const CgArgs& a, int rounds, double* out, hipStream_t s);
// r-halo by pull: ghost planes of r read from the neighbours' boundary rows
// (system-scope loads) before the SpMV launch; lo_cnt rows lo_src -> lo_dst, hi likewise.
// force: outside a solve's iteration test (the creation-time test, the prologue);
// pexpr: store v + 0.0 v (the prologue's p = x, HPCCG.cpp:347) instead of v
void launch_pull(const CgArgs& a, const double* lo_src, double* lo_dst, int lo_cnt, const double* hi_src, double* hi_dst,
                 int hi_cnt, hipStream_t s, bool force = false, bool pexpr = false);
// the prologue's barrier (one lane, peer_allreduce on the kMboxBarrier slots):
// every rank's p = x (and its x) is in place before any rank pulls x's rows
void launch_peer_barrier(const CgArgs& a, hipStream_t s);
// solve start: state zeroed (spin budget set), every dot slot empty
void launch_rearm(int* kst, double* partial, int np, int budget, hipStream_t s);
void launch_cg_xflush(const CgArgs& a, hipStream_t s);  // pending deferred x updates

// In-process rank group all-reduce of one CG scalar: g[which] of every rank =
// sum of loc[which] over ranks, in rank order.
constexpr int kMaxGroupRanks = 16;
static_assert(kMaxGroupRanks == kMboxRanks, "mailbox rows");
struct GroupSum {
    int nranks;
    int which;
    const double* loc[kMaxGroupRanks];
    double* g[kMaxGroupRanks];
};
void launch_group_sum(const GroupSum& gs, hipStream_t s);

// Kernel-level ops on arbitrary device pointers.
void launch_waxpby(int n, double alpha, const double* x, double beta, const double* y, double* w, hipStream_t s);
void launch_ddot(int n, const double* x, const double* y, double* partial, int nparts, double* out, hipStream_t s);
int ddot_nparts(int n);
void launch_sparsemv(const CgArgs& a, const double* xext, double* y, hipStream_t s);
// Diagnostic: the SELL-512-A values streamed like the SpMV, known bytes (FETCH calibration).
constexpr int kDiagStreamA = 9;
void launch_stream_a(const CgArgs& a, hipStream_t s);
// Slot completion plan (host): per group the unit that waits, and the top group; returns the group count.
int slot_plan(int units, int grid, int spu, int rev, int* last_unit, int* top);

// Device generator: writes the SELL-512 image, b, xexact.
void launch_generate(int nx, int ny, int nz, int rank, int size, int use_7pt, long long col_base,
                     const unsigned int* slice_base, int* cols, double* vals, double* b, double* xexact, int nrow,
                     hipStream_t s);
// SELL-512-A from the SELL-512 image: per-slice offsets (ok[0] = 0 when a
// slice has more than kAMax or a row is not in ascending column order), then
// the values into their offsets' slots (aval zeroed beforehand).
void launch_a_offsets(const unsigned int* slice_base, int nslices, const int* cols, int ghost_lo, int* aoff,
                      int* acount, int* ok, int* maxabs, hipStream_t s);
void launch_a_fill(const unsigned int* slice_base, int nslices, const int* cols, const double* vals, int ghost_lo,
                   const int* aoff, const int* acount, const unsigned int* abase, double* aval, hipStream_t s);

}  // namespace hpccg
