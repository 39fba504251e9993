// hpccg_solver.cpp -- host side of the MI355X HPCCG path: HPC_Sparse_Matrix ->
// SELL-512 conversion, device residency, the device-resident CG driver
// (HPCCG.cpp:312-402), the z-slab halo exchange and scalar all-reduces over
// RCCL (exchange_externals.cpp:51-131, ddot.cpp:75-85), and the C ABI.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <climits>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <map>
#include <unordered_map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/HPC_Sparse_Matrix.hpp"
#include "../../include/hpccg_hip.h"
#include "hpccg_internal.h"

using namespace hpccg;

// ---------------------------------------------------------------------------
// errors
// ---------------------------------------------------------------------------
namespace {

thread_local std::string g_err;

int set_err(int code, const char* fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

}  // namespace

namespace hpccg {
// error channel for the other host translation units (read_hpc_row.cpp)
int set_error_message(int code, const char* msg) { return set_err(code, "%s", msg); }
}  // namespace hpccg

namespace {

#define HIP_TRY(expr)                                                                              \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess)                                                                      \
            return set_err(e_ == hipErrorOutOfMemory ? HPCCG_HIP_ENOMEM : HPCCG_HIP_EHIP,          \
                           "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__);   \
    } while (0)

#define NCCL_TRY(expr)                                                                             \
    do {                                                                                           \
        ncclResult_t r_ = (expr);                                                                  \
        if (r_ != ncclSuccess)                                                                     \
            return set_err(HPCCG_HIP_ERCCL, "%s: %s (%s:%d)", #expr, ncclGetErrorString(r_),      \
                           __FILE__, __LINE__);                                                    \
    } while (0)

#define TRY(expr)                                                                                  \
    do {                                                                                           \
        int rc_ = (expr);                                                                          \
        if (rc_ != 0) return rc_;                                                                  \
    } while (0)

// ---------------------------------------------------------------------------
// communicator (one rank per GPU per process)
// ---------------------------------------------------------------------------
struct Comm {
    ncclComm_t comm = nullptr;
    int nranks = 1;
    int rank = 0;
};
Comm g_comm;

// In-process rank group (hpccg_hip_group_*): while a group member is being
// created on this thread, rank/size come from here instead of the RCCL
// communicator, and the halo plan is made by hpccg_hip_group_* afterwards.
// Gather halo plan (make_local_matrix.cpp:58-610, exchange_externals.cpp:51-131)
// for partitions the z-slab plan cannot serve: the external columns get local
// indices n, n+1, ... grouped by owning rank, groups in order of first
// appearance and first appearance inside a group, exactly as
// make_local_matrix.cpp:96-200 numbers them.
struct GatherPlan {
    std::vector<long long> ext_global;              // external j <-> local column n + j
    std::unordered_map<long long, int> ext_of;      // global column -> j
    std::vector<int> recv_rank, recv_off, recv_cnt; // externals owned by recv_rank[i]: [off, off + cnt)
    std::vector<std::vector<int>> req;              // per owner: the global columns we need, our order
    std::vector<int> send_rank, send_off, send_cnt; // per requester: a run of send_idx
    std::vector<int> send_idx;                      // local rows packed for the requesters
};

struct GroupCtx {
    int active = 0, nranks = 1, rank = 0;
    const int* info = nullptr;        // every member's {nrow, ghost_lo, ghost_hi, start_row}, or null
    const GatherPlan* plan = nullptr; // this member's gather plan (gather mode), or null
};
thread_local GroupCtx g_group_ctx;
int g_halo_mode = 0;  // 0 auto (slab when it serves every rank), 1 slab only, 2 gather
int comm_nranks() { return g_group_ctx.active ? g_group_ctx.nranks : g_comm.nranks; }
int comm_rank() { return g_group_ctx.active ? g_group_ctx.rank : g_comm.rank; }

// ---------------------------------------------------------------------------
// SELL-512 build from any row accessor. Entry order per row is preserved.
// ---------------------------------------------------------------------------
// Column map of the slab plan: global column -> index into [ghost_lo | n | ghost_hi].
struct SlabCols {
    long long col_base, ncol_ext;
    long long operator()(long long c) const
    {
        const long long lc = c - col_base;
        return (lc < 0 || lc >= ncol_ext) ? -1 : lc;
    }
};

template <class RowLen, class RowAt, class ColMap>
long long sell_build_impl(int nrow, ColMap colmap, RowLen row_len, RowAt row_at, unsigned int* slice_base,
                          int* sell_cols, double* sell_vals, int uniform_width, int* err)
{
    const int nslices = (nrow + kSliceRows - 1) / kSliceRows;
    // widths
    long long total = 0;
    int wmax = 0;
    std::vector<int> w(nslices, 0);
    for (int s = 0; s < nslices; s++) {
        int m = 0;
        for (int i = s * kSliceRows; i < std::min(nrow, (s + 1) * kSliceRows); i++)
            m = std::max(m, row_len(i));
        w[s] = m;
        wmax = std::max(wmax, m);
    }
    if (uniform_width) std::fill(w.begin(), w.end(), wmax);
    for (int s = 0; s < nslices; s++) {
        if (slice_base) slice_base[s] = (unsigned int)total;
        total += w[s];
    }
    if (slice_base) slice_base[nslices] = (unsigned int)total;
    if (!sell_cols || !sell_vals) return total * kSliceRows;
    // fill, parallel over slices
    std::atomic<int> bad{0};
    const int nth = std::max(1, std::min<int>(16, (int)std::thread::hardware_concurrency()));
    auto work = [&](int t) {
        for (int s = t; s < nslices; s += nth) {
            const size_t b0 = (size_t)slice_base[s] * kSliceRows;
            for (int lane = 0; lane < kSliceRows; lane++) {
                const int i = s * kSliceRows + lane;
                const int len = i < nrow ? row_len(i) : 0;
                for (int j = 0; j < w[s]; j++) {
                    const size_t e = b0 + (size_t)j * kSliceRows + lane;
                    if (j < len) {
                        double v;
                        long long c;
                        row_at(i, j, &c, &v);
                        const long long lc = colmap(c);
                        if (lc < 0) bad.store(1);
                        sell_cols[e] = (int)lc;
                        sell_vals[e] = v;
                    } else {
                        sell_cols[e] = -1;
                        sell_vals[e] = 0.0;
                    }
                }
            }
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nth; t++) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
    if (err) *err = bad.load();
    return total * kSliceRows;
}

}  // namespace

// ---------------------------------------------------------------------------
// device matrix + CG workspace
// ---------------------------------------------------------------------------
struct hpccg_hip_matrix {
    int device = 0;
    int rank = 0, nranks = 1;  // z-slab rank of this matrix (RCCL communicator or in-process group)
    int in_group = 0;          // 1: halo / all-reduce by hpccg_hip_group_solve, not RCCL
    int nrow = 0, start_row = 0, total_nrow = 0;
    int ghost_lo = 0, ghost_hi = 0;
    // what neighbours need from us (filled by the collective plan exchange)
    int send_lo = 0;  // rows to send to rank-1 (its ghost_hi)
    int send_hi = 0;  // rows to send to rank+1 (its ghost_lo)
    // gather plan (partitions the slab plan cannot serve): externals after the
    // local rows (ghost_lo = 0, ghost_hi = number of externals)
    int general = 0;
    std::vector<int> recv_rank, recv_off, recv_cnt, send_rank, send_off, send_cnt;
    int nsend = 0;
    int* d_send_idx = nullptr;
    double* d_send_buf = nullptr;
    // halo / interior overlap (multi-rank slab plan): the leading b_lo and
    // trailing b_hi slices read ghost columns, the rest do not
    int halo_b_lo = -1, halo_b_hi = -1;
    int overlap = 1;
    hipStream_t stream2 = nullptr;
    hipEvent_t ev_pb = nullptr, ev_halo = nullptr;
    long long nnz = 0, nslots = 0, nslots4 = 0;
    int nslices = 0, grid = 0, width = 0, uniform = 0;
    int spmv_variant = 0;
    int use_graph = 1;
    int fuse_p = -1;  // p = r + beta p inside the SpMV: -1 auto (on for the LDS kernels only)
    int fold = -1;   // dots completed inside their producing kernel (two-level, sc1 publish); -1 auto
    unsigned int* d_slice_base = nullptr;
    int* d_cols = nullptr;
    double* d_vals = nullptr;
    // SELL-512-L (LDS-staged x windows)
    int has_lds = 0, lds_doubles = 0, nwin = 0;
    unsigned short* d_lcols = nullptr;
    // SELL-512-C (per-slice offset dictionary + 1-byte codes)
    int has_c = 0, has_c_lds = 0;
    unsigned char* d_ccodes = nullptr;
    int *d_cdict = nullptr, *d_ldsc = nullptr, *d_ccount = nullptr;
    // SELL-512-V (per-slice dictionary of (offset, value) pairs + 1-byte codes)
    int has_v = 0, has_v_lds = 0;
    // SELL-512-P (per-row pattern ids over the C codes, pattern tables per slice)
    int has_p = 0, has_p_lds = 0;
    unsigned char* d_prow = nullptr;
    int *d_prep = nullptr, *d_pcount = nullptr, *d_pbase = nullptr, *d_ptab_g = nullptr, *d_ptab_l = nullptr;
    int pat_max = 0;  // largest pattern table over slices (ints)
    // SELL-512-A (offset-aligned slots, holes 0.0; per-slice offset lists)
    int has_a = 0;
    int a_width = 0;  // slots per slice when uniform (every slice padded to the widest), else 0
    int has_a_lds = 0;  // SELL-512-A LDS windows (27-pt: one per plane, holes included)
    int *d_alds = nullptr, *d_awin = nullptr, *d_awn = nullptr;
    int alds_doubles = 0;
    int has_a_lds2 = 0;  // the same over slice pairs (k_spmv_la2, single rank)
    int *d_alds2 = nullptr, *d_awin2 = nullptr, *d_awn2 = nullptr;
    int alds2_doubles = 0;
    int has_a_lds4 = 0;  // and over groups of four slices
    int *d_alds4 = nullptr, *d_awin4 = nullptr, *d_awn4 = nullptr;
    int alds4_doubles = 0;
    double* d_aval = nullptr;
    int* d_aoff = nullptr;
    unsigned int* d_abase = nullptr;
    long long p_guard = 0;  // zeroed doubles on each side of every p buffer (A kernels read holes there)
    int value_codes = 0;  // opt-in: let choose_variant pick SELL-512-V
    unsigned char* d_vcodes = nullptr;
    int *d_vdict = nullptr, *d_vldsc = nullptr, *d_vcount = nullptr;
    double* d_vval = nullptr;
    unsigned int* d_vbase4 = nullptr;  // SELL-512-V4: the V codes in 4-slot chunks
    unsigned char* d_vcodes4 = nullptr;
    int *d_win_ptr = nullptr, *d_win_start = nullptr, *d_win_len = nullptr, *d_win_off = nullptr;
    // workspace (padded to a multiple of kSliceRows rows)
    size_t npad = 0;
    double* d_pbuf = nullptr;  // ring_alloc buffers of [ghost_lo_pad | npad | ghost_hi_pad]
    int ring_alloc = 0;        // p ring buffers allocated
    double* d_p = nullptr;     // local rows of ring buffer 0
    long long pstride = 0;     // doubles between ring buffers
    double* d_ahist = nullptr;
    int x_defer = 1;           // batched x update every x_ring iterations
    int x_ring = -1;           // p ring length with x_defer (2..kXRingMax; -1 auto, x_ring_effective)
    int rev_update = 1;        // update kernel walks slices backwards (reads the SpMV's latest writes first)
    long long resident_mb = -1; // NT kernels: MB of leading slices on default-policy loads (-1 auto)
    int redund = 0;            // consumers complete the dots themselves, no finalize kernels (measured slower)
    int update_slices = 1;     // slices per loop-update workgroup (1, 2, 4, 8)
    int update_early = 0;      // loop update loads Ap and r before the iteration test
    int pap_upd = 0;           // the loop update forms p.Ap from the SpMV partials (one rank, <= 64 groups)
    double *d_r = nullptr, *d_Ap = nullptr, *d_x = nullptr, *d_b = nullptr;
    double* d_rbuf = nullptr;  // r with p_guard zeroed doubles on each side (fused SELL-512-A reads holes there)
    double* d_partial = nullptr;
    unsigned int* d_tickets = nullptr;
    int ntickets = 0;
    double* d_scal = nullptr;  // g[2], loc[2], scratch[4]
    int* d_kst = nullptr;
    double* d_hist = nullptr;
    unsigned long long* d_stamps = nullptr;
    int hist_cap = 0, stamp_cap = 0;
    double* d_ddot_partial = nullptr;
    int ddot_cap = 0;
    // generated-problem vectors
    double *d_gen_b = nullptr, *d_gen_x0 = nullptr, *d_gen_xexact = nullptr;
    hipStream_t stream = nullptr;
    hipGraphExec_t graph_exec = nullptr;
    int graph_chunk = 0;       // iterations in the captured graph
    int graph_iters = 8;       // option graph_chunk: iterations per captured graph
    CgArgs graph_args{};
    int graph_variant = -1;
    // hipEvent timing (event_timing option)
    int event_timing = 0;
    std::vector<hipEvent_t> ev;   // 4 per iteration slot: spmv start/end, update start/end
    double ktimes[4] = {0, 0, 0, 0};
    // last solve
    std::vector<double> trace;
    int last_niters = 0;
};

namespace {

int free_matrix(hpccg_hip_matrix* M)
{
    if (!M) return 0;
    (void)hipSetDevice(M->device);
    if (M->graph_exec) (void)hipGraphExecDestroy(M->graph_exec);
    void* ptrs[] = {M->d_slice_base, M->d_cols,    M->d_vals,  M->d_pbuf,  M->d_ahist,  M->d_rbuf,
                    M->d_Ap,         M->d_x,       M->d_b,     M->d_partial,      M->d_scal,
                    M->d_tickets,
                    M->d_kst,        M->d_hist,    M->d_stamps, M->d_ddot_partial, M->d_gen_b,
                    M->d_gen_x0,     M->d_gen_xexact, M->d_lcols, M->d_win_ptr, M->d_win_start,
                    M->d_win_len,    M->d_win_off, M->d_send_idx, M->d_send_buf, M->d_ccodes, M->d_cdict, M->d_ldsc,
                    M->d_vcodes,     M->d_vdict,   M->d_vval,  M->d_vldsc, M->d_vbase4, M->d_vcodes4,
                    M->d_ccount,     M->d_vcount,  M->d_prow,  M->d_prep,  M->d_pcount, M->d_pbase,
                    M->d_ptab_g,     M->d_ptab_l,  M->d_aval,  M->d_aoff,  M->d_abase,
                    M->d_alds,       M->d_awin,    M->d_awn,   M->d_alds2, M->d_awin2, M->d_awn2,
                    M->d_alds4,      M->d_awin4,   M->d_awn4};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    for (hipEvent_t e : M->ev) (void)hipEventDestroy(e);
    if (M->stream) (void)hipStreamDestroy(M->stream);
    if (M->stream2) (void)hipStreamDestroy(M->stream2);
    if (M->ev_pb) (void)hipEventDestroy(M->ev_pb);
    if (M->ev_halo) (void)hipEventDestroy(M->ev_halo);
    delete M;
    return 0;
}

// Frees a matrix under construction on every early return; release() on success.
struct MatrixGuard {
    hpccg_hip_matrix* m;
    ~MatrixGuard()
    {
        if (m) free_matrix(m);
    }
    hpccg_hip_matrix* release()
    {
        hpccg_hip_matrix* t = m;
        m = nullptr;
        return t;
    }
};

// Can the z-slab plan serve rank r? (ghosts from rank+-1 only, contiguous,
// the planes those ranks own; the condition hpccg_slab_plan enforces)
bool slab_serves(const int* info, int P, int r)
{
    const int* me = info + 4 * r;
    const int glo = me[1], ghi = me[2];
    if (glo > 0 && (r == 0 || glo > info[4 * (r - 1)])) return false;
    if (ghi > 0 && (r == P - 1 || ghi > info[4 * (r + 1)])) return false;
    if (r > 0 && info[4 * (r - 1) + 3] + info[4 * (r - 1)] != me[3]) return false;
    return true;
}

// 1 = slab plan for every rank, 2 = gather plan for every rank (all ranks decide
// the same from the same all-gathered info).
int choose_halo_mode(const int* info, int P)
{
    if (g_halo_mode == 2) return 2;
    for (int r = 0; r < P; r++)
        if (!slab_serves(info, P, r)) return g_halo_mode == 1 ? -1 : 2;
    return 1;
}

int owner_of(long long c, const int* info, int P)  // make_local_matrix.cpp:165-173
{
    int lo = 0, hi = P - 1;
    while (lo < hi) {  // last rank whose start_row <= c
        const int mid = (lo + hi + 1) / 2;
        if (info[4 * mid + 3] <= c) lo = mid; else hi = mid - 1;
    }
    return lo;
}

template <class RowLen, class RowAt>
void gather_externals(int nrow, long long start, const int* info, int P, RowLen row_len, RowAt row_at,
                      GatherPlan& g)
{
    std::vector<long long> first;  // externals in order of first appearance
    std::unordered_map<long long, int> seen;
    for (int i = 0; i < nrow; i++) {
        const int len = row_len(i);
        for (int j = 0; j < len; j++) {
            long long c;
            double v;
            row_at(i, j, &c, &v);
            if (c >= start && c < start + nrow) continue;
            if (seen.emplace(c, (int)first.size()).second) first.push_back(c);
        }
    }
    std::vector<std::vector<int>> by_owner(P);
    std::vector<int> order;
    for (int i = 0; i < (int)first.size(); i++) {
        const int q = owner_of(first[i], info, P);
        if (by_owner[q].empty()) order.push_back(q);
        by_owner[q].push_back(i);
    }
    g.ext_global.assign(first.size(), 0);
    g.req.assign(P, {});
    int count = 0;
    for (int q : order) {
        g.recv_rank.push_back(q);
        g.recv_off.push_back(count);
        g.recv_cnt.push_back((int)by_owner[q].size());
        for (int i : by_owner[q]) {
            g.ext_global[count] = first[i];
            g.ext_of[first[i]] = count;
            g.req[q].push_back((int)first[i]);
            count++;
        }
    }
}

// What rank r packs for its requesters, from every rank's requests
// (reqs_to_me[q] = the global columns rank q needs from r, q's order).
void gather_sends(long long start, const std::vector<std::vector<int>>& reqs_to_me, GatherPlan& g)
{
    g.send_rank.clear();
    g.send_off.clear();
    g.send_cnt.clear();
    g.send_idx.clear();
    for (int q = 0; q < (int)reqs_to_me.size(); q++) {
        if (reqs_to_me[q].empty()) continue;
        g.send_rank.push_back(q);
        g.send_off.push_back((int)g.send_idx.size());
        g.send_cnt.push_back((int)reqs_to_me[q].size());
        for (int c : reqs_to_me[q]) g.send_idx.push_back((int)(c - start));
    }
}

// RCCL: requests travel to their owners (the handshake of make_local_matrix
// .cpp:286-587): an all-gather of the P x P count matrix, then grouped
// send/recv of the int32 column lists.
int rccl_requests(hpccg_hip_matrix* M, GatherPlan& g)
{
    const int P = g_comm.nranks, r = g_comm.rank;
    std::vector<int> mine(P);
    for (int q = 0; q < P; q++) mine[q] = (int)g.req[q].size();
    int* d = nullptr;
    HIP_TRY(hipMalloc(&d, sizeof(int) * (size_t)P * (P + 1)));
    HIP_TRY(hipMemcpy(d, mine.data(), sizeof(int) * P, hipMemcpyHostToDevice));
    NCCL_TRY(ncclAllGather(d, d + P, P, ncclInt32, g_comm.comm, M->stream));
    std::vector<int> cnt((size_t)P * P);
    HIP_TRY(hipMemcpyAsync(cnt.data(), d + P, sizeof(int) * P * P, hipMemcpyDeviceToHost, M->stream));
    HIP_TRY(hipStreamSynchronize(M->stream));
    (void)hipFree(d);
    long long nout = 0, nin = 0;
    for (int q = 0; q < P; q++) {
        nout += cnt[(size_t)r * P + q];
        nin += cnt[(size_t)q * P + r];
    }
    int* dout = nullptr;
    int* din = nullptr;
    HIP_TRY(hipMalloc(&dout, sizeof(int) * std::max(1LL, nout)));
    HIP_TRY(hipMalloc(&din, sizeof(int) * std::max(1LL, nin)));
    std::vector<int> flat;
    for (int q = 0; q < P; q++) flat.insert(flat.end(), g.req[q].begin(), g.req[q].end());
    if (nout) HIP_TRY(hipMemcpy(dout, flat.data(), sizeof(int) * nout, hipMemcpyHostToDevice));
    NCCL_TRY(ncclGroupStart());
    long long oo = 0, oi = 0;
    for (int q = 0; q < P; q++) {
        const int co = cnt[(size_t)r * P + q], ci = cnt[(size_t)q * P + r];
        if (co) NCCL_TRY(ncclSend(dout + oo, co, ncclInt32, q, g_comm.comm, M->stream));
        if (ci) NCCL_TRY(ncclRecv(din + oi, ci, ncclInt32, q, g_comm.comm, M->stream));
        oo += co;
        oi += ci;
    }
    NCCL_TRY(ncclGroupEnd());
    std::vector<int> got(std::max(1LL, nin));
    HIP_TRY(hipMemcpyAsync(got.data(), din, sizeof(int) * std::max(1LL, nin), hipMemcpyDeviceToHost, M->stream));
    HIP_TRY(hipStreamSynchronize(M->stream));
    (void)hipFree(dout);
    (void)hipFree(din);
    std::vector<std::vector<int>> to_me(P);
    oi = 0;
    for (int q = 0; q < P; q++) {
        const int ci = cnt[(size_t)q * P + r];
        to_me[q].assign(got.begin() + oi, got.begin() + oi + ci);
        oi += ci;
    }
    gather_sends(M->start_row, to_me, g);
    return 0;
}

// Install a gather plan on M (host tables + device send list/buffer).
int install_gather(hpccg_hip_matrix* M, const GatherPlan& g)
{
    M->general = 1;
    M->ghost_lo = 0;
    M->ghost_hi = (int)g.ext_global.size();
    M->recv_rank = g.recv_rank;
    M->recv_off = g.recv_off;
    M->recv_cnt = g.recv_cnt;
    M->send_rank = g.send_rank;
    M->send_off = g.send_off;
    M->send_cnt = g.send_cnt;
    M->nsend = (int)g.send_idx.size();
    HIP_TRY(hipMalloc(&M->d_send_idx, sizeof(int) * std::max(1, M->nsend)));
    HIP_TRY(hipMalloc(&M->d_send_buf, sizeof(double) * std::max(1, M->nsend)));
    if (M->nsend)
        HIP_TRY(hipMemcpy(M->d_send_idx, g.send_idx.data(), sizeof(int) * M->nsend, hipMemcpyHostToDevice));
    return 0;
}

// Plan exchange: every rank learns what its neighbours need. For z-slabs it is
// one all-gather of {nrow, ghost_lo, ghost_hi, start_row}; when the slab plan
// cannot serve every rank, *mode is set to 2 and the caller builds the gather
// plan (the general make_local_matrix.cpp:58-610 handshake).
int exchange_plan(hpccg_hip_matrix* M, int* mode = nullptr, std::vector<int>* all_out = nullptr)
{
    M->send_lo = M->send_hi = 0;
    M->rank = comm_rank();
    M->nranks = comm_nranks();
    if (mode) *mode = 1;
    if (g_group_ctx.active) {  // in-process group: planned by the group functions
        M->in_group = 1;
        if (g_group_ctx.info) {
            const int P = g_group_ctx.nranks;
            const int md = P == 1 ? 1 : choose_halo_mode(g_group_ctx.info, P);
            if (md < 0) return set_err(HPCCG_HIP_EPLAN, "the z-slab halo plan cannot serve this partition");
            if (mode) *mode = md;
            if (all_out) all_out->assign(g_group_ctx.info, g_group_ctx.info + 4 * P);
        }
        return 0;
    }
    if (g_comm.nranks == 1) {
        if (M->ghost_lo || M->ghost_hi)
            return set_err(HPCCG_HIP_EPLAN, "columns outside the local rows on a single rank");
        return 0;
    }
    int* d = nullptr;
    HIP_TRY(hipMalloc(&d, sizeof(int) * 4 * (g_comm.nranks + 1)));
    int mine[4] = {M->nrow, M->ghost_lo, M->ghost_hi, M->start_row};
    HIP_TRY(hipMemcpy(d, mine, sizeof mine, hipMemcpyHostToDevice));
    NCCL_TRY(ncclAllGather(d, d + 4, 4, ncclInt32, g_comm.comm, M->stream));
    std::vector<int> all(4 * g_comm.nranks);
    HIP_TRY(hipMemcpyAsync(all.data(), d + 4, sizeof(int) * 4 * g_comm.nranks, hipMemcpyDeviceToHost,
                           M->stream));
    HIP_TRY(hipStreamSynchronize(M->stream));
    (void)hipFree(d);
    const int md = choose_halo_mode(all.data(), g_comm.nranks);
    if (md < 0) return set_err(HPCCG_HIP_EPLAN, "the z-slab halo plan cannot serve this partition");
    if (all_out) *all_out = all;
    if (md == 2) {
        if (!mode) return set_err(HPCCG_HIP_EPLAN, "gather halo plan needs the matrix rows");
        *mode = 2;
        return 0;
    }
    int sends[2];
    TRY(hpccg_slab_plan(g_comm.nranks, g_comm.rank, all.data(), sends));
    M->send_lo = sends[0];
    M->send_hi = sends[1];
    return 0;
}

// SELL-512-C and SELL-512-V from the uploaded SELL-512 image (and windows, if
// any) on the device. A format is dropped when a slice has more than 255
// distinct keys (C: offsets; V: (offset, value) pairs), its LDS form when a
// code's entries fall in different windows.
int build_code_image(hpccg_hip_matrix* M, bool with_vals, unsigned char** codes, int** dict, double** val,
                     int** ldsc, int** count, int* has, int* has_lds)
{
    const size_t ndict = (size_t)std::max(1, M->nslices) * kCodes;
    HIP_TRY(hipMalloc(codes, std::max<size_t>(1, (size_t)M->nslots)));
    HIP_TRY(hipMalloc(count, sizeof(int) * std::max(1, M->nslices)));
    HIP_TRY(hipMalloc(dict, sizeof(int) * ndict));
    if (with_vals) HIP_TRY(hipMalloc(val, sizeof(double) * ndict));
    if (M->has_lds) HIP_TRY(hipMalloc(ldsc, sizeof(int) * ndict));
    int* d_ok = nullptr;
    HIP_TRY(hipMalloc(&d_ok, sizeof(int) * 2));
    const int ones[2] = {1, 1};
    HIP_TRY(hipMemcpyAsync(d_ok, ones, sizeof ones, hipMemcpyHostToDevice, M->stream));
    launch_build_c(M->d_slice_base, M->nslices, M->d_cols, with_vals ? M->d_vals : nullptr,
                   M->has_lds ? M->d_win_ptr : nullptr, M->d_win_start, M->d_win_off, M->d_win_len, *codes, *dict,
                   with_vals ? *val : nullptr, M->has_lds ? *ldsc : nullptr, *count, d_ok, M->stream);
    HIP_TRY(hipGetLastError());
    int ok[2] = {0, 0};
    HIP_TRY(hipMemcpyAsync(ok, d_ok, sizeof ok, hipMemcpyDeviceToHost, M->stream));
    HIP_TRY(hipStreamSynchronize(M->stream));
    (void)hipFree(d_ok);
    *has = ok[0];
    *has_lds = ok[0] && ok[1] && M->has_lds;
    auto drop = [](auto** q) {
        if (*q) (void)hipFree(*q);
        *q = nullptr;
    };
    if (!*has_lds) drop(ldsc);
    if (!*has) {
        drop(codes);
        drop(dict);
        drop(count);
        if (val) drop(val);
    }
    return 0;
}

// SELL-512-P from the SELL-512-C codes: pattern ids per row, tables per slice.
int build_p_image(hpccg_hip_matrix* M)
{
    const int S = M->nslices;
    if (!M->has_c || S < 1) return 0;
    HIP_TRY(hipMalloc(&M->d_prow, (size_t)S * kSliceRows));
    HIP_TRY(hipMalloc(&M->d_prep, sizeof(int) * (size_t)S * kMaxPat));
    HIP_TRY(hipMalloc(&M->d_pcount, sizeof(int) * S));
    int* d_ok = nullptr;
    HIP_TRY(hipMalloc(&d_ok, sizeof(int)));
    const int one = 1;
    HIP_TRY(hipMemcpyAsync(d_ok, &one, sizeof one, hipMemcpyHostToDevice, M->stream));
    launch_build_p(M->d_slice_base, S, M->d_ccodes, M->d_prow, M->d_prep, M->d_pcount, d_ok, M->stream);
    HIP_TRY(hipGetLastError());
    int ok = 0;
    std::vector<int> cnt(S);
    std::vector<unsigned int> sb(S + 1);
    HIP_TRY(hipMemcpyAsync(&ok, d_ok, sizeof ok, hipMemcpyDeviceToHost, M->stream));
    HIP_TRY(hipMemcpyAsync(cnt.data(), M->d_pcount, sizeof(int) * S, hipMemcpyDeviceToHost, M->stream));
    HIP_TRY(hipMemcpyAsync(sb.data(), M->d_slice_base, sizeof(unsigned int) * sb.size(), hipMemcpyDeviceToHost,
                           M->stream));
    HIP_TRY(hipStreamSynchronize(M->stream));
    (void)hipFree(d_ok);
    std::vector<int> base(S + 1, 0);
    M->pat_max = 0;
    for (int i = 0; i < S && ok; i++) {
        M->pat_max = std::max<int>(M->pat_max, cnt[i] * (int)(sb[i + 1] - sb[i]));
        const long long e = (long long)base[i] + (long long)cnt[i] * (sb[i + 1] - sb[i]);
        if (e > INT_MAX) ok = 0;
        else base[i + 1] = (int)e;
    }
    if (ok) {
        HIP_TRY(hipMalloc(&M->d_pbase, sizeof(int) * base.size()));
        HIP_TRY(hipMemcpy(M->d_pbase, base.data(), sizeof(int) * base.size(), hipMemcpyHostToDevice));
        const size_t ne = std::max(1, base[S]);
        HIP_TRY(hipMalloc(&M->d_ptab_g, sizeof(int) * ne));
        if (M->has_c_lds) HIP_TRY(hipMalloc(&M->d_ptab_l, sizeof(int) * ne));
        launch_fill_p(M->d_slice_base, S, M->d_ccodes, M->d_prep, M->d_pcount, M->d_pbase, M->d_cdict,
                      M->has_c_lds ? M->d_ldsc : nullptr, M->d_ptab_g, M->d_ptab_l, M->stream);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipStreamSynchronize(M->stream));
    }
    (void)hipFree(M->d_prep);  // representatives: build only
    M->d_prep = nullptr;
    M->has_p = ok;
    // the LDS kernels keep the table after the windows in one dynamic allocation
    M->has_p_lds = ok && M->has_c_lds && (size_t)M->lds_doubles * 8 + (size_t)M->pat_max * 4 <= 65536;
    if (!ok) {
        for (int** q : {&M->d_pcount, &M->d_pbase, &M->d_ptab_g, &M->d_ptab_l}) {
            if (*q) (void)hipFree(*q);
            *q = nullptr;
        }
        (void)hipFree(M->d_prow);
        M->d_prow = nullptr;
    }
    return 0;
}

int alloc_ring(hpccg_hip_matrix* M, int nbuf);
int alloc_r(hpccg_hip_matrix* M);
int x_ring_effective(const hpccg_hip_matrix* M);

// Windows of a group of slices [s0, s0 + ns) over the union of their
// ascending offsets (cut where neighbours are more than a slice apart):
// window [o_a, o_b] stages rows s0*512 + o_a .. (s0 + ns)*512 - 1 + o_b, so
// every row of every slice of the group finds every offset of the range,
// holes included. lds[s][j] = LDS position of slot j minus the row's index
// in the group; padding slots (offset 0, value 0.0) read slot 0's. Returns
// the doubles staged, or -1 when it needs more than kAWin windows.
int group_windows(const std::vector<int>& off, const std::vector<int>& cnt, int s0, int ns, int* win, int* nwin,
                  std::vector<int>& lds)
{
    std::vector<int> u;
    for (int t = 0; t < ns; t++)
        for (int j = 0; j < cnt[s0 + t]; j++) u.push_back(off[(size_t)(s0 + t) * kAMax + j]);
    std::sort(u.begin(), u.end());
    u.erase(std::unique(u.begin(), u.end()), u.end());
    const int rows = ns * kSliceRows;
    int nw = 0, base = 0;
    std::vector<int> wlo, wbase;
    if (u.empty()) {  // empty rows only: one window of the group's own rows
        win[0] = 0, win[1] = rows, win[2] = 0;
        wlo.push_back(0), wbase.push_back(0);
        nw = 1, base = rows;
    }
    for (size_t j = 0; j < u.size();) {
        size_t e = j;
        while (e + 1 < u.size() && u[e + 1] - u[e] <= kSliceRows) e++;
        if (nw == kAWin) return -1;
        win[3 * nw] = u[j];
        win[3 * nw + 1] = rows + u[e] - u[j];
        win[3 * nw + 2] = base;
        wlo.push_back(u[j]);
        wbase.push_back(base);
        base += rows + u[e] - u[j];
        nw++;
        j = e + 1;
    }
    for (int t = 0; t < ns; t++) {
        const int s = s0 + t;
        int* l = &lds[(size_t)s * kAMax];
        for (int j = 0; j < cnt[s]; j++) {
            const int o = off[(size_t)s * kAMax + j];
            int w = 0;
            while (w + 1 < nw && wlo[w + 1] <= o) w++;
            l[j] = wbase[w] + o - wlo[w];
        }
        // padding slots read slot 0's position; a slice without entries reads
        // its own rows in the group's single window (position = group row)
        if (cnt[s] == 0) l[0] = 0;
        for (int j = std::max(cnt[s], 1); j < kAMax; j++) l[j] = l[0];
    }
    *nwin = nw;
    return base;
}

// SELL-512-A group windows (k_spmv_la2): slices G*g .. G*g + G - 1 share
// one set (G = 2 or 4).
int build_a_windows_g(hpccg_hip_matrix* M, const std::vector<int>& off, const std::vector<int>& cnt, int G,
                      int cap, int** d_lds, int** d_win, int** d_wn, int* doubles, int* has)
{
    const int S = M->nslices;
    const int NG = (S + G - 1) / G;
    std::vector<int> lds((size_t)S * kAMax, 0), win((size_t)NG * kAWin * 3, 0), wn(NG, 0);
    int maxd = 0;
    for (int P = 0; P < NG; P++) {
        const int d = group_windows(off, cnt, G * P, std::min(G, S - G * P), &win[(size_t)P * kAWin * 3], &wn[P], lds);
        if (d < 0 || d > cap) return 0;
        maxd = std::max(maxd, d);
    }
    HIP_TRY(hipMalloc(d_lds, sizeof(int) * lds.size()));
    HIP_TRY(hipMalloc(d_win, sizeof(int) * win.size()));
    HIP_TRY(hipMalloc(d_wn, sizeof(int) * wn.size()));
    HIP_TRY(hipMemcpy(*d_lds, lds.data(), sizeof(int) * lds.size(), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(*d_win, win.data(), sizeof(int) * win.size(), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(*d_wn, wn.data(), sizeof(int) * wn.size(), hipMemcpyHostToDevice));
    *doubles = maxd;
    *has = 1;
    return 0;
}

int build_a_windows2(hpccg_hip_matrix* M, const std::vector<int>& off, const std::vector<int>& cnt)
{
    TRY(build_a_windows_g(M, off, cnt, 2, kALdsMax2, &M->d_alds2, &M->d_awin2, &M->d_awn2, &M->alds2_doubles,
                          &M->has_a_lds2));
    return build_a_windows_g(M, off, cnt, 4, kALdsMax4, &M->d_alds4, &M->d_awin4, &M->d_awn4, &M->alds4_doubles,
                             &M->has_a_lds4);
}

// SELL-512-A LDS windows (host, from the per-slice offsets): the ascending
// offsets are cut where neighbours are more than a slice apart (staging the
// gap would cost more than a second window); window [o_a, o_b] stages rows
// s*512 + o_a .. s*512 + 511 + o_b, so every row of the slice finds every
// offset of the range in it, holes included, and slot j reads LDS position
// lane row + alds[j]. Padding slots (offset 0, value 0.0) read slot 0's.
int build_a_windows(hpccg_hip_matrix* M, const std::vector<int>& cnt)
{
    const int S = M->nslices;
    std::vector<int> off((size_t)S * kAMax);
    HIP_TRY(hipMemcpy(off.data(), M->d_aoff, sizeof(int) * off.size(), hipMemcpyDeviceToHost));
    std::vector<int> lds((size_t)S * kAMax, 0), win((size_t)S * kAWin * 3, 0), wn(S, 0);
    int maxd = 0;
    for (int s = 0; s < S; s++) {
        const int K = cnt[s];
        const int* o = &off[(size_t)s * kAMax];
        int* w = &win[(size_t)s * kAWin * 3];
        int nw = 0, base = 0;
        if (K == 0) {  // empty rows only: one window of the slice's own rows
            w[0] = 0, w[1] = kSliceRows, w[2] = 0;
            nw = 1, base = kSliceRows;
        }
        for (int j = 0; j < K;) {
            int e = j;
            while (e + 1 < K && o[e + 1] - o[e] <= kSliceRows) e++;
            if (nw == kAWin) return 0;
            w[3 * nw] = o[j];
            w[3 * nw + 1] = kSliceRows + o[e] - o[j];
            w[3 * nw + 2] = base;
            for (int q = j; q <= e; q++) lds[(size_t)s * kAMax + q] = base + o[q] - o[j];
            base += kSliceRows + o[e] - o[j];
            nw++;
            j = e + 1;
        }
        if (base > kALdsMax) return 0;
        for (int q = std::max(K, 1); q < kAMax; q++) lds[(size_t)s * kAMax + q] = lds[(size_t)s * kAMax];
        wn[s] = nw;
        maxd = std::max(maxd, base);
    }
    HIP_TRY(hipMalloc(&M->d_alds, sizeof(int) * lds.size()));
    HIP_TRY(hipMalloc(&M->d_awin, sizeof(int) * win.size()));
    HIP_TRY(hipMalloc(&M->d_awn, sizeof(int) * wn.size()));
    HIP_TRY(hipMemcpy(M->d_alds, lds.data(), sizeof(int) * lds.size(), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(M->d_awin, win.data(), sizeof(int) * win.size(), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(M->d_awn, wn.data(), sizeof(int) * wn.size(), hipMemcpyHostToDevice));
    M->alds_doubles = maxd;
    M->has_a_lds = 1;
    return build_a_windows2(M, off, cnt);
}

// SELL-512-A from the SELL-512-C codes (k_build_a), then the p ring again
// with zeroed guard zones of max |offset| + a slice on each side, so a hole's
// x load stays inside the buffer.
int build_a_image(hpccg_hip_matrix* M)
{
    const int S = M->nslices;
    if (!M->has_c || S < 1) return 0;
    std::vector<int> cnt(S);
    HIP_TRY(hipMemcpy(cnt.data(), M->d_ccount, sizeof(int) * S, hipMemcpyDeviceToHost));
    std::vector<unsigned int> ab(S + 1, 0);
    int wmax = 0;
    for (int i = 0; i < S; i++) {
        if (cnt[i] > kAMax) return 0;
        ab[i + 1] = ab[i] + (unsigned)cnt[i];
        wmax = std::max(wmax, cnt[i]);
    }
    // uniform slot count when padding every slice to the widest costs < 4 %
    // (stencils: only the first and last planes' slices are narrower); the
    // padding slots are holes at offset 0 (value 0.0, x of the row itself)
    M->a_width = 0;
    if ((double)wmax * S <= 1.04 * (double)ab[S]) {
        for (int i = 0; i <= S; i++) ab[i] = (unsigned)i * (unsigned)wmax;
        M->a_width = wmax;
    }
    HIP_TRY(hipMalloc(&M->d_abase, sizeof(unsigned int) * ab.size()));
    HIP_TRY(hipMemcpy(M->d_abase, ab.data(), sizeof(unsigned int) * ab.size(), hipMemcpyHostToDevice));
    const size_t na = std::max<size_t>(1, (size_t)ab[S] * kSliceRows);
    HIP_TRY(hipMalloc(&M->d_aval, sizeof(double) * na));
    HIP_TRY(hipMemsetAsync(M->d_aval, 0, sizeof(double) * na, M->stream));
    HIP_TRY(hipMalloc(&M->d_aoff, sizeof(int) * (size_t)S * kAMax));
    int* d_flags = nullptr;  // ok, maxabs
    HIP_TRY(hipMalloc(&d_flags, sizeof(int) * 2));
    const int init[2] = {1, 0};
    HIP_TRY(hipMemcpyAsync(d_flags, init, sizeof init, hipMemcpyHostToDevice, M->stream));
    launch_build_a(M->d_slice_base, S, M->d_ccodes, M->d_vals, M->d_cdict, M->d_ccount, M->d_abase, M->d_aval,
                   M->d_aoff, d_flags, d_flags + 1, M->stream);
    HIP_TRY(hipGetLastError());
    int fl[2] = {0, 0};
    HIP_TRY(hipMemcpyAsync(fl, d_flags, sizeof fl, hipMemcpyDeviceToHost, M->stream));
    HIP_TRY(hipStreamSynchronize(M->stream));
    (void)hipFree(d_flags);
    if (!fl[0]) {
        for (void** q : {(void**)&M->d_aval, (void**)&M->d_aoff, (void**)&M->d_abase}) {
            (void)hipFree(*q);
            *q = nullptr;
        }
        return 0;
    }
    // A hole of row i at offset o reads column i + o; o is a real offset of
    // some row of the same slice (of the same group of four slices for the
    // group windows), so i + o lies within 2047 of a valid column: four
    // slices of zeros on each side cover every hole, whatever max |o|.
    const long long guard = 4 * kSliceRows;
    if (guard > M->p_guard) {
        M->p_guard = guard;
        const size_t glo_pad = ((size_t)M->ghost_lo + kSliceRows - 1) / kSliceRows * kSliceRows;
        const size_t ghi_pad = ((size_t)M->ghost_hi + 2 + kSliceRows - 1) / kSliceRows * kSliceRows;
        M->pstride = (long long)(M->p_guard + glo_pad + M->npad + ghi_pad + M->p_guard);
        if (M->d_pbuf) TRY(alloc_ring(M, std::max(M->ring_alloc, x_ring_effective(M))));
        if (M->d_rbuf) TRY(alloc_r(M));
    }
    M->has_a = 1;
    return build_a_windows(M, cnt);
}

int build_c_image(hpccg_hip_matrix* M)
{
    TRY(build_code_image(M, false, &M->d_ccodes, &M->d_cdict, nullptr, &M->d_ldsc, &M->d_ccount, &M->has_c,
                         &M->has_c_lds));
    TRY(build_p_image(M));
    TRY(build_a_image(M));
    TRY(build_code_image(M, true, &M->d_vcodes, &M->d_vdict, &M->d_vval, &M->d_vldsc, &M->d_vcount, &M->has_v,
                         &M->has_v_lds));
    if (!M->has_v || M->nslices < 1) return 0;
    // SELL-512-V4: slice s owns chunks [vbase4[s], vbase4[s + 1]) of 4 slots
    std::vector<unsigned int> sb(M->nslices + 1), vb(M->nslices + 1, 0);
    HIP_TRY(hipMemcpy(sb.data(), M->d_slice_base, sizeof(unsigned int) * sb.size(), hipMemcpyDeviceToHost));
    for (int i = 0; i < M->nslices; i++) vb[i + 1] = vb[i] + (sb[i + 1] - sb[i] + 3) / 4;
    const size_t bytes = (size_t)vb[M->nslices] * kSliceRows * 4;
    M->nslots4 = (long long)vb[M->nslices] * 4 * kSliceRows;
    HIP_TRY(hipMalloc(&M->d_vbase4, sizeof(unsigned int) * vb.size()));
    HIP_TRY(hipMemcpy(M->d_vbase4, vb.data(), sizeof(unsigned int) * vb.size(), hipMemcpyHostToDevice));
    HIP_TRY(hipMalloc(&M->d_vcodes4, std::max<size_t>(1, bytes)));
    HIP_TRY(hipMemsetAsync(M->d_vcodes4, (int)kCodePad, bytes, M->stream));
    launch_interleave_v4(M->d_slice_base, M->d_vbase4, M->nslices, M->d_vcodes, M->d_vcodes4, M->stream);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(M->stream));
    return 0;
}

// x_ring auto: the long ring where the matrix image is far beyond the 256 MB
// Infinity Cache (7-pt 256^3 update 93 vs 103 us with 32 vs 8); near it, the 32
// p buffers cycled through the cache evict the image (100^3: 14290 vs 14160
// it/s with 8 vs 32).
int x_ring_effective(const hpccg_hip_matrix* M)
{
    if (M->x_ring > 0) return M->x_ring;
    return (double)M->nslots * 8.0 > 512e6 ? kXRingDefault : 8;
}

// The p ring: nbuf buffers of pstride doubles, local rows 512-row aligned.
int alloc_ring(hpccg_hip_matrix* M, int nbuf)
{
    // the new ring first: on failure the matrix keeps its old one
    const size_t glo_pad = ((size_t)M->ghost_lo + kSliceRows - 1) / kSliceRows * kSliceRows;
    const size_t ptotal = (size_t)M->pstride * nbuf;
    double* buf = nullptr;
    HIP_TRY(hipMalloc(&buf, sizeof(double) * ptotal));
    if (hipMemset(buf, 0, sizeof(double) * ptotal) != hipSuccess) {
        (void)hipFree(buf);
        return set_err(HPCCG_HIP_EHIP, "hipMemset of the p ring failed");
    }
    if (M->d_pbuf) (void)hipFree(M->d_pbuf);
    M->d_pbuf = buf;
    M->d_p = M->d_pbuf + M->p_guard + glo_pad;
    M->ring_alloc = nbuf;
    return 0;
}

// r = [p_guard zeros | npad rows | p_guard zeros]; only rows < n are ever
// written. Reallocated (zeroed) when the guard grows: r is recomputed by every
// solve's prologue.
int alloc_r(hpccg_hip_matrix* M)
{
    const size_t total = M->npad + 2 * (size_t)M->p_guard;
    double* buf = nullptr;
    HIP_TRY(hipMalloc(&buf, sizeof(double) * total));
    if (hipMemset(buf, 0, sizeof(double) * total) != hipSuccess) {
        (void)hipFree(buf);
        return set_err(HPCCG_HIP_EHIP, "hipMemset of r failed");
    }
    if (M->d_rbuf) (void)hipFree(M->d_rbuf);
    M->d_rbuf = buf;
    M->d_r = buf + M->p_guard;
    return 0;
}

int alloc_workspace(hpccg_hip_matrix* M)
{
    M->npad = (size_t)M->nslices * kSliceRows;
    if (M->npad == 0) M->npad = kSliceRows;
    // p = [ghost_lo | n | ghost_hi]; local rows start 512-row aligned
    const size_t glo_pad = ((size_t)M->ghost_lo + kSliceRows - 1) / kSliceRows * kSliceRows;
    const size_t ghi_pad = ((size_t)M->ghost_hi + 2 + kSliceRows - 1) / kSliceRows * kSliceRows;
    M->pstride = (long long)(M->p_guard + glo_pad + M->npad + ghi_pad + M->p_guard);
    TRY(alloc_ring(M, x_ring_effective(M)));
    TRY(alloc_r(M));
    double** vecs[] = {&M->d_Ap, &M->d_x, &M->d_b};
    for (double** v : vecs) {
        HIP_TRY(hipMalloc(v, sizeof(double) * M->npad));
        HIP_TRY(hipMemset(*v, 0, sizeof(double) * M->npad));
    }
    const int ngroups = (M->nslices + 63) / 64;  // kGroup in hpccg_kernels.hip
    // slice partials, group sums of both dots, 8 spare, then the p.Ap slice
    // partials of the pap_upd mode
    HIP_TRY(hipMalloc(&M->d_partial, sizeof(double) * (2 * std::max(1, M->nslices) + 2 * ngroups + 8)));
    M->ntickets = 2 * (ngroups + 1);
    HIP_TRY(hipMalloc(&M->d_tickets, sizeof(unsigned int) * M->ntickets));
    HIP_TRY(hipMemset(M->d_tickets, 0, sizeof(unsigned int) * M->ntickets));
    HIP_TRY(hipMalloc(&M->d_scal, sizeof(double) * 8));
    HIP_TRY(hipMemset(M->d_scal, 0, sizeof(double) * 8));
    HIP_TRY(hipMalloc(&M->d_kst, sizeof(int) * 8));  // kst[0..3] + tickets[2] (+pad)
    HIP_TRY(hipMemset(M->d_kst, 0, sizeof(int) * 8));
    return 0;
}

int ensure_hist(hpccg_hip_matrix* M, int max_iter)
{
    const int need = std::max(2, max_iter + 1);
    if (need > M->hist_cap) {
        if (M->d_hist) (void)hipFree(M->d_hist);
        if (M->d_ahist) (void)hipFree(M->d_ahist);
        HIP_TRY(hipMalloc(&M->d_hist, sizeof(double) * need));
        HIP_TRY(hipMalloc(&M->d_ahist, sizeof(double) * need));
        M->hist_cap = need;
    }
    const int scap = 16 + (max_iter + 2) * kNumStampSlots;
    if (scap > M->stamp_cap) {
        if (M->d_stamps) (void)hipFree(M->d_stamps);
        HIP_TRY(hipMalloc(&M->d_stamps, sizeof(unsigned long long) * 2 * scap));
        M->stamp_cap = scap;
    }
    return 0;
}

// Default SpMV kernel for a matrix (measured r01, profiles/r01/spmv_sweep_*.jsonl):
// SELL-512-L when the staged x per row is small against the row length (27-pt:
// 5.4 staged doubles vs 26.7 entries per row -> 1.33x faster; 7-pt: 6 vs 7 ->
// 1.14x slower), non-temporal matrix loads once the image outgrows the 256 MB
// Infinity Cache (>= 128^3: nt 5-12 % faster; <= 100^3: default policy 2-20 %
// faster). The LDS kernels prefetch 4 matrix slots ahead of the window staging
// barrier (2200/2300; in-CG 200^3: 409-415 vs 420-441 us per SpMV, 100^3 even).
// Which image variant v needs that M lacks (nullptr: none).
const char* variant_unavailable(const hpccg_hip_matrix* M, int v)
{
    if (v >= 2000 && v < 3000 && !M->has_lds) return "the SELL-512-L windows";
    if (v >= 3000 && v < 4000 && !M->has_c) return "the SELL-512-C image";
    if (v >= 4000 && v < 5000 && !M->has_c_lds) return "the SELL-512-C LDS image";
    if (v >= 5000 && v < 6000 && !M->has_v_lds) return "the SELL-512-V LDS image";
    if (v >= 6000 && v < 8000 && !M->has_v) return "the SELL-512-V image";
    if (v >= 8000 && v < 8500 && !M->has_p_lds) return "the SELL-512-P LDS image";
    if (v >= 8500 && v < 8700 && !M->has_p) return "the SELL-512-P image";
    if (v >= 8700 && v < 8900 && !M->has_a) return "the SELL-512-A image";
    if (v >= 8900 && v < 8960 && !M->has_a_lds) return "the SELL-512-A LDS windows";
    if (v >= 8960 && v < 8980 && !M->has_a_lds2) return "the SELL-512-A pair windows";
    if (v >= 8980 && v < 9000 && !M->has_a_lds4) return "the SELL-512-A quad windows";
    if (v >= 8960 && v < 9000 && M->general) return "the slab halo plan (SELL-512-A group windows)";
    return nullptr;
}

// Slots per slice a fixed-width variant unrolls (0: any width): xx07 / xx27,
// 9999 = 27, and the SELL-512-A early-load variants.
int required_width(int v)
{
    switch (v) {
    case 8717: case 8817: return 7;
    case 8737: case 8757: case 8837: case 8857: case 9999: return 27;
    default: break;
    }
    const int w = v % 100;
    return (w == 27 || w == 7) ? w : 0;
}

// Fixed-width variants unroll the slot loop: every slice must have exactly
// that many slots (SELL-512-A: that many offsets).
bool fixed_width_ok(const hpccg_hip_matrix* M, int v)
{
    const int w = required_width(v);
    if (w == 0) return true;
    if (v >= 8700 && v < 9000) return M->has_a && M->a_width == w;
    return M->uniform && M->width == w;
}

int choose_variant(const hpccg_hip_matrix* M)
{
    const double rows = std::max(1, M->nrow);
    const bool lds = M->has_lds && (double)M->nnz / rows >= 2.5 * M->lds_doubles / (double)kSliceRows;
    const double image = (double)M->nslots * (lds ? 10.0 : 12.0);
    const bool big = image > 180e6;
    // SELL-512-C (1-byte offset codes, 9 B per slot) where the image allows it:
    // 200^3 in-CG SpMV 407-414 vs 433 us (LDS), 7-pt 256^3 265-272 vs 328-340 us
    // SELL-512-V4 (1-byte (offset, value) codes in 4-slot chunks, values from
    // the slice dictionary; ~1 B per slot) wherever it fits: in-CG SpMV 200^3
    // 155 vs 407 us (SELL-512-C LDS), 100^3 32 vs 58 us, 7-pt 256^3 187 vs
    // 284 us. Non-temporal code loads above ~100 MB of codes. Opt-in
    // ("value_codes"): it stops reading every stored value from HBM per
    // iteration, which the headline bench keeps.
    if (M->value_codes && M->has_v) return (double)M->nslots4 > 100e6 ? 7201 : 7301;
    // SELL-512-P (8 B value per slot + 1 B pattern id per row) wherever a
    // slice's row patterns fit: in-CG SpMV 200^3 377 vs 408 us (8226 vs 4200),
    // 100^3 53.4 vs 58.2 us (8300), 7-pt 256^3 252 vs 277 us (8500 vs 3000).
    // Non-temporal value loads once the image outgrows the 256 MB Infinity Cache.
    const bool big_p = (double)M->nslots * 8.0 > 256e6;
    // One rank, 27-pt beyond the Infinity Cache: SELL-512-A pair windows (two
    // slices per 512-thread block share their staged planes, 4.2 instead of
    // 5.4 staged doubles per row; one ticket per two slices), 3 value slots
    // early: 200^3 2461-2468 vs 2330-2387 it/s (8236) on one box.
    if (lds && big_p && M->has_p_lds && !M->general && M->has_a_lds2) return 8963;
    // SELL-512-A (values in offset-aligned slots, x read directly at the
    // slice's offsets, p = r + beta*p_{k-1} formed per load on one rank)
    // everywhere except the 27-pt images beyond the Infinity Cache, where the
    // LDS windows compute p once per staged entry: 100^3 SpMV 49.7 us and
    // no k_p_update vs 53.0 (14789 vs 14113 it/s); 7-pt 256^3 2397 vs 2319
    // it/s (8707 fused); 200^3 fused 423 us, separate p update 365 + 30 us vs
    // 381 us (8226).
    if (M->has_a && !(lds && big_p && M->has_p_lds)) {
        // width 27: 4 value slots and the offsets loaded before the run
        // test, 100^3 SpMV 44.6 vs 49.3-50.1 us (15983 vs 14737-14901 it/s)
        if (!big_p) return M->a_width == 27 ? 8837 : 8800;
        return M->a_width == 7 ? 8707 : 8700;
    }
    // 8236 = 8226 with the pattern ids and the 4 prefetched value slots
    // loaded before the iteration test: 200^3 2412-2416 vs 2385-2391 it/s
    if (lds && M->has_p_lds) return big_p ? 8236 : 8300;
    if (!lds && M->has_p) {
        if (M->uniform && M->width == 7 && big_p) return 8507;  // 7-pt 256^3: 248 vs 253 us
        return big_p ? 8500 : 8600;
    }
    if (lds) return M->has_c_lds ? 4200 : (big ? 2200 : 2300);
    if (M->has_c) return big ? 3000 : 3100;
    return big ? 1000 : 0;
}

// SELL-512-V kernels: 5xxx (LDS), 6xxx (plain), 7xxx (plain, 4-slot chunks).
bool variant_is_v(int v) { return v >= 5000 && v < 8000; }

// Matrix-stream bytes per stored slot of the kernel in use.
double slot_bytes(const hpccg_hip_matrix* M)
{
    const int v = M->spmv_variant;
    if (v >= 7000 && v < 8000) return (double)M->nslots4 / std::max<long long>(1, M->nslots);
    if (variant_is_v(v)) return 1.0;
    if ((v >= 3000 && v < 5000)) return 9.0;
    if (v >= 8700 && v < 9000) return 8.0;
    if (v >= 8000 && v < 9000) return 8.0 + (double)M->nslices * kSliceRows / std::max<long long>(1, M->nslots);
    if (v >= 2000 && v < 3000) return 10.0;
    return 12.0;
}

// resident_mb auto: an NT image not far above the 256 MB Infinity Cache keeps
// 128 MB of itself on default-policy loads, which then survive to the next
// iteration (100^3, 270 MB: SpMV 59.6 vs 62.3 us); a multi-GB stream evicts
// everything, and default-policy loads only cost there (200^3: 449 vs 432 us).
long long resident_mb_effective(const hpccg_hip_matrix* M)
{
    if (M->resident_mb >= 0) return M->resident_mb;
    const double image = (double)M->nslots * slot_bytes(M);
    return image <= 400e6 ? 128 : 0;
}

// fuse_p (single rank): measured slower in the plain SELL-512 kernels, where it
// doubles every gather (561 -> 744 us at 200^3), so "auto" enables it only for
// the SELL-512-L kernels, which compute p_k once per staged window entry.
// Multi-rank: only the SELL-512-L kernels, which stage ghost planes from the
// halo and compute own rows (the halo rows first, by k_p_boundary).
bool fuse_p_effective(const hpccg_hip_matrix* M)
{
    if (M->spmv_variant == 9999) return false;
    const int v = M->spmv_variant;
    const bool lds = (v >= 2000 && v < 3000) || (v >= 4000 && v < 6000) || (v >= 8000 && v < 8500) ||
                     (v >= 8900 && v < 9000);
    const bool aligned = v >= 8700 && v < 8900;  // SELL-512-A: x = r + beta*p per coalesced load
    if (M->nranks != 1 && !lds) return false;
    if (M->fuse_p < 0) return lds || aligned;
    return M->fuse_p != 0;
}

// fold auto (measured): completing p.Ap inside the SpMV saves the k_finalize
// launch (7-14 us incl. its boundary) but holds each block's wave 0 for the
// publish round trip. 100^3 (1954 slices): 13062 vs 12475 it/s (C format);
// SELL-512-P: 7-pt 256^3 (32768 slices) 2326-2432 vs 2275-2410, 200^3 (15625)
// 2277-2293 vs 2279-2286 (even). r.r in the update kernel: slower at every
// size (every block of a short kernel waits for its ticket).
int fold_effective(const hpccg_hip_matrix* M)
{
    if (M->fold >= 0 && M->fold <= 3) return M->fold;
    return 2;
}

// p.Ap formed by every loop-update workgroup (k_update_pr): one rank, one
// slice per update workgroup, no redundant mode, at most 64 groups of slice
// partials (32 K slices: 16 M rows) to sum per workgroup.
bool pap_upd_effective(const hpccg_hip_matrix* M)
{
    if (M->pap_upd <= 0 || M->nranks != 1 || M->update_slices != 1 || M->redund > 0) return false;
    return (M->nslices + 63) / 64 <= 64;
}

// Redundant dot completion (k_update_g + cur_rr): single rank, group sums that
// fit the update's LDS, at least one iteration (trace[0] then comes from hist).
bool redund_effective(const hpccg_hip_matrix* M, int max_iter)
{
    if (M->nranks != 1 || max_iter < 2 || M->nslices < 1) return false;
    if ((M->nslices + 63) / 64 > 4096) return false;  // kFinLdsGroups
    return M->redund > 0;
}

CgArgs make_args(hpccg_hip_matrix* M, const double* b, double* x, int max_iter, double tol)
{
    CgArgs a;
    std::memset(&a, 0, sizeof a);  // graph cache compares bytes
    a.n = M->nrow;
    a.nslices = M->nslices;
    a.grid = M->grid;
    a.max_iter = max_iter;
    a.tol = tol;
    a.nranks = M->nranks;
    a.ghost_lo = M->ghost_lo;
    a.b = b;
    a.x = x;
    a.r = M->d_r;
    a.p = M->d_p;
    a.pstride = M->pstride;
    a.fuse_p = fuse_p_effective(M) ? 1 : 0;
    a.xdefer = M->x_defer ? 1 : 0;
    a.rev = M->rev_update ? 1 : 0;
    a.s0 = 0;
    a.sn0 = M->nslices;
    a.s1 = 0;
    a.sn1 = 0;
    a.sgrid = M->grid;
    {
        const double per_slice = (double)M->nslots / std::max(1, M->nslices) * slot_bytes(M);
        const double sl = (double)resident_mb_effective(M) * 1e6 / std::max(1.0, per_slice);
        a.nt_split = (int)std::min<double>(M->grid / kNumXcd, sl / kNumXcd);
    }
    a.nring = a.xdefer ? x_ring_effective(M) : (a.fuse_p ? 2 : 1);
    a.ahist = M->d_ahist;
    a.fold = fold_effective(M);
    a.redund = redund_effective(M, max_iter) ? 1 : 0;
    if (a.redund) a.fold = 0;
    {
        const int ng = (M->nslices + 63) / 64;
        a.ugrid = std::max(kNumXcd, (ng + kNumXcd - 1) / kNumXcd * kNumXcd);
        a.um = M->update_slices;
        a.uearly = M->update_early ? 1 : 0;
        a.pap_upd = pap_upd_effective(M) ? 1 : 0;
        a.ppart = M->d_partial + std::max(1, M->nslices) + 2 * ng + 8;
        const int nb = (M->nslices + a.um - 1) / a.um;
        a.umgrid = std::max(kNumXcd, (nb + kNumXcd - 1) / kNumXcd * kNumXcd);
    }
    a.tickets = M->d_tickets;
    a.Ap = M->d_Ap;
    a.partial = M->d_partial;
    a.g = M->d_scal;
    a.loc = M->d_scal + 2;
    a.hist = M->d_hist;
    a.kst = M->d_kst;
    a.stamps = M->d_stamps;
    a.stamp_cap = M->stamp_cap;
    a.slice_base = M->d_slice_base;
    a.cols = M->d_cols;
    a.vals = M->d_vals;
    a.lcols = M->d_lcols;
    const bool v = variant_is_v(M->spmv_variant);
    a.ccodes = v ? M->d_vcodes : M->d_ccodes;
    a.cdict = v ? M->d_vdict : M->d_cdict;
    a.ldsc = v ? M->d_vldsc : M->d_ldsc;
    a.cval = v ? M->d_vval : nullptr;
    a.ccount = v ? M->d_vcount : M->d_ccount;
    a.vbase4 = M->d_vbase4;
    a.vcodes4 = M->d_vcodes4;
    a.prow = M->d_prow;
    a.pcount = M->d_pcount;
    a.pbase = M->d_pbase;
    a.ptab_g = M->d_ptab_g;
    a.ptab_l = M->d_ptab_l;
    a.aval = M->d_aval;
    a.aoff = M->d_aoff;
    a.abase = M->d_abase;
    a.alds = M->d_alds;
    a.awin = M->d_awin;
    a.awn = M->d_awn;
    a.alds_doubles = std::max(1, M->alds_doubles);
    a.alds2 = M->d_alds2;
    a.awin2 = M->d_awin2;
    a.awn2 = M->d_awn2;
    a.alds2_doubles = std::max(1, M->alds2_doubles);
    a.pgrid = std::max(kNumXcd, ((M->nslices + 1) / 2 + kNumXcd - 1) / kNumXcd * kNumXcd);
    a.alds4 = M->d_alds4;
    a.awin4 = M->d_awin4;
    a.awn4 = M->d_awn4;
    a.alds4_doubles = std::max(1, M->alds4_doubles);
    a.qgrid = std::max(kNumXcd, ((M->nslices + 3) / 4 + kNumXcd - 1) / kNumXcd * kNumXcd);
    {
        const int v = M->spmv_variant;
        a.agroup = (v >= 8960 && v < 8980) ? 2 : ((v >= 8980 && v < 9000) ? 4 : 0);
        a.gs0 = 0;
        a.gn0 = a.agroup ? (M->nslices + a.agroup - 1) / a.agroup : 0;
        a.gs1 = a.gn1 = 0;
    }
    a.pat_max = std::max(1, M->pat_max);
    a.win_ptr = M->d_win_ptr;
    a.win_start = M->d_win_start;
    a.win_len = M->d_win_len;
    a.win_off = M->d_win_off;
    a.lds_doubles = M->lds_doubles;
    return a;
}

// Halo exchange of p (exchange_externals.cpp:51-131): the z-slab ghosts are
// contiguous, so no pack: rank r sends its first send_lo rows down and its
// last send_hi rows up, and receives straight into the ghost regions.
int enqueue_halo(hpccg_hip_matrix* M, double* p, hipStream_t st = nullptr)
{
    if (g_comm.nranks == 1) return 0;
    if (!st) st = M->stream;
    const int r = g_comm.rank;
    NCCL_TRY(ncclGroupStart());
    if (r > 0) {
        if (M->ghost_lo) NCCL_TRY(ncclRecv(p - M->ghost_lo, M->ghost_lo, ncclFloat64, r - 1, g_comm.comm, st));
        if (M->send_lo) NCCL_TRY(ncclSend(p, M->send_lo, ncclFloat64, r - 1, g_comm.comm, st));
    }
    if (r < g_comm.nranks - 1) {
        if (M->ghost_hi) NCCL_TRY(ncclRecv(p + M->nrow, M->ghost_hi, ncclFloat64, r + 1, g_comm.comm, st));
        if (M->send_hi)
            NCCL_TRY(ncclSend(p + M->nrow - M->send_hi, M->send_hi, ncclFloat64, r + 1, g_comm.comm, st));
    }
    NCCL_TRY(ncclGroupEnd());
    return 0;
}

// Gather plan over RCCL (exchange_externals.cpp:51-131): pack what each
// requester needs, then one grouped send/recv per neighbour; the externals
// arrive contiguously after the local rows.
int enqueue_halo_gather(hpccg_hip_matrix* M, const CgArgs& a, double* p, bool prologue)
{
    if (g_comm.nranks == 1) return 0;
    launch_cg_pack(a, M->d_send_idx, M->nsend, M->d_send_buf, prologue, M->stream);
    NCCL_TRY(ncclGroupStart());
    for (size_t i = 0; i < M->recv_rank.size(); i++)
        NCCL_TRY(ncclRecv(p + M->nrow + M->recv_off[i], M->recv_cnt[i], ncclFloat64, M->recv_rank[i],
                          g_comm.comm, M->stream));
    for (size_t i = 0; i < M->send_rank.size(); i++)
        NCCL_TRY(ncclSend(M->d_send_buf + M->send_off[i], M->send_cnt[i], ncclFloat64, M->send_rank[i],
                          g_comm.comm, M->stream));
    NCCL_TRY(ncclGroupEnd());
    return 0;
}

int enqueue_allreduce(hpccg_hip_matrix* M, const CgArgs& a, int which)
{
    if (g_comm.nranks == 1) return 0;
    NCCL_TRY(ncclAllReduce(a.loc + which, a.g + which, 1, ncclFloat64, ncclSum, g_comm.comm, M->stream));
    return 0;
}

int ensure_events(hpccg_hip_matrix* M, int slots)
{
    while ((int)M->ev.size() < 4 * slots) {
        hipEvent_t e;
        HIP_TRY(hipEventCreate(&e));
        M->ev.push_back(e);
    }
    return 0;
}

// p_k's ring buffer (local rows), as the kernels' cur_p computes it.
// p_k's ring buffer (local rows), as the kernels' cur_p computes it.
double* ring_p(const CgArgs& a, int k) { return a.p + (size_t)(k % a.nring) * (size_t)a.pstride; }

// The ranks one host thread enqueues: one matrix (a process of an RCCL job, or
// a single GPU), or every member of an in-process group (hpccg_hip_group_*).
struct Ranks {
    hpccg_hip_matrix* const* M;
    const CgArgs* a;
    int P;
    hipEvent_t* ev;  // group: P "ready" events + 1 "reduced" event
};

int use_device(const Ranks& R, int r)
{
    if (R.P > 1) HIP_TRY(hipSetDevice(R.M[r]->device));
    return 0;
}

// In-process halo: rank r's ghost planes are copied from its neighbours' p_k
// rows once their streams have produced them (the same rows enqueue_halo moves
// with RCCL). Rank r-1 cannot overwrite p_k's ring slot before the copy: its
// next write there comes after at least one all-reduce, which waits for rank
// r's update kernel, which follows rank r's SpMV on the same stream.
int group_halo(const Ranks& R, int k_host, bool prologue)
{
    for (int r = 0; r < R.P; r++) {
        TRY(use_device(R, r));
        HIP_TRY(hipEventRecord(R.ev[r], R.M[r]->stream));
    }
    auto p_of = [&](int r) { return prologue ? R.a[r].p : ring_p(R.a[r], k_host); };
    for (int r = 0; r < R.P; r++) {
        hpccg_hip_matrix* M = R.M[r];
        TRY(use_device(R, r));
        if (r > 0 && M->ghost_lo) {
            const hpccg_hip_matrix* L = R.M[r - 1];
            HIP_TRY(hipStreamWaitEvent(M->stream, R.ev[r - 1], 0));
            HIP_TRY(hipMemcpyPeerAsync(p_of(r) - M->ghost_lo, M->device, p_of(r - 1) + L->nrow - M->ghost_lo,
                                       L->device, sizeof(double) * M->ghost_lo, M->stream));
        }
        if (r < R.P - 1 && M->ghost_hi) {
            const hpccg_hip_matrix* U = R.M[r + 1];
            HIP_TRY(hipStreamWaitEvent(M->stream, R.ev[r + 1], 0));
            HIP_TRY(hipMemcpyPeerAsync(p_of(r) + M->nrow, M->device, p_of(r + 1), U->device,
                                       sizeof(double) * M->ghost_hi, M->stream));
        }
    }
    return 0;
}

// In-process gather halo: every member packs for its requesters; each
// receiver copies its runs out of the owners' send buffers. An owner's next
// pack (next iteration) follows an all-reduce that waits for the receiver's
// SpMV, which follows the copy.
int group_halo_gather(const Ranks& R, int k_host, bool prologue)
{
    for (int r = 0; r < R.P; r++) {
        hpccg_hip_matrix* M = R.M[r];
        TRY(use_device(R, r));
        launch_cg_pack(R.a[r], M->d_send_idx, M->nsend, M->d_send_buf, prologue, M->stream);
        HIP_TRY(hipEventRecord(R.ev[r], M->stream));
    }
    for (int r = 0; r < R.P; r++) {
        hpccg_hip_matrix* M = R.M[r];
        double* p = prologue ? R.a[r].p : ring_p(R.a[r], k_host);
        TRY(use_device(R, r));
        for (size_t i = 0; i < M->recv_rank.size(); i++) {
            const int q = M->recv_rank[i];
            const hpccg_hip_matrix* Q = R.M[q];
            size_t j = 0;
            while (j < Q->send_rank.size() && Q->send_rank[j] != r) j++;
            if (j == Q->send_rank.size() || Q->send_cnt[j] != M->recv_cnt[i])
                return set_err(HPCCG_HIP_EPLAN, "rank %d: no matching send run on rank %d", r, q);
            HIP_TRY(hipStreamWaitEvent(M->stream, R.ev[q], 0));
            HIP_TRY(hipMemcpyPeerAsync(p + M->nrow + M->recv_off[i], M->device, Q->d_send_buf + Q->send_off[j],
                                       Q->device, sizeof(double) * M->recv_cnt[i], M->stream));
        }
    }
    return 0;
}

// In-process all-reduce of loc[which]: one lane on rank 0's stream adds the
// ranks' values in rank order and writes g[which] of every rank.
int group_allreduce(const Ranks& R, int which)
{
    GroupSum gs;
    std::memset(&gs, 0, sizeof gs);
    gs.nranks = R.P;
    gs.which = which;
    for (int r = 0; r < R.P; r++) {
        gs.loc[r] = R.a[r].loc;
        gs.g[r] = R.a[r].g;
        TRY(use_device(R, r));
        HIP_TRY(hipEventRecord(R.ev[r], R.M[r]->stream));
    }
    TRY(use_device(R, 0));
    for (int r = 1; r < R.P; r++) HIP_TRY(hipStreamWaitEvent(R.M[0]->stream, R.ev[r], 0));
    launch_group_sum(gs, R.M[0]->stream);
    HIP_TRY(hipEventRecord(R.ev[R.P], R.M[0]->stream));
    for (int r = 1; r < R.P; r++) {
        TRY(use_device(R, r));
        HIP_TRY(hipStreamWaitEvent(R.M[r]->stream, R.ev[R.P], 0));
    }
    return 0;
}

int exch_halo(const Ranks& R, int k_host, bool prologue)
{
    // k_pack (gather plan) and k_p_boundary (fused slab) stamp the halo class
    // themselves; otherwise a one-lane stamp kernel does
    const bool stamped = R.M[0]->general || (!prologue && R.a[0].fuse_p);
    for (int r = 0; r < R.P && !stamped; r++) {
        TRY(use_device(R, r));
        launch_cg_stamp(R.a[r], kStampHalo, prologue, R.M[r]->stream);
    }
    if (R.M[0]->general) {
        if (R.P > 1) return group_halo_gather(R, k_host, prologue);
        return enqueue_halo_gather(R.M[0], R.a[0], prologue ? R.a[0].p : ring_p(R.a[0], k_host), prologue);
    }
    if (R.P > 1) return group_halo(R, k_host, prologue);
    return enqueue_halo(R.M[0], prologue ? R.a[0].p : ring_p(R.a[0], k_host));
}

int exch_allreduce(const Ranks& R, int which, bool prologue)
{
    (void)prologue;  // the all-reduce class is stamped where the local sum completes (finish_dot)
    if (R.P > 1) return group_allreduce(R, which);
    return enqueue_allreduce(R.M[0], R.a[0], which);
}

// One CG iteration k (HPCCG.cpp:358-386), fully device resident, for every
// rank of R. slot >= 0 (single matrix): bracket the SpMV and the fused update
// with that slot's hipEvents. k_host is the iteration being enqueued: it
// addresses p_k's ring slot for the halo.
// SpMV launch arguments over a slice subset (interior or halo-dependent runs).
CgArgs spmv_range(const CgArgs& a, int s0, int n0, int s1, int n1)
{
    CgArgs b = a;
    b.s0 = s0;
    b.sn0 = n0;
    b.s1 = s1;
    b.sn1 = n1;
    b.sgrid = std::max(kNumXcd, (n0 + n1 + kNumXcd - 1) / kNumXcd * kNumXcd);
    return b;
}

// The same for the group kernels, in groups of a.agroup slices.
CgArgs group_range(const CgArgs& a, int g0, int n0, int g1, int n1)
{
    CgArgs b = a;
    b.gs0 = g0;
    b.gn0 = n0;
    b.gs1 = g1;
    b.gn1 = n1;
    const int grid = std::max(kNumXcd, (n0 + n1 + kNumXcd - 1) / kNumXcd * kNumXcd);
    if (a.agroup == 2)
        b.pgrid = grid;
    else
        b.qgrid = grid;
    return b;
}

// Multi-rank slab iteration with the halo exchange overlapped (SURVEY 5,
// "overlap the halo with the interior-row SpMV"): the halo rows of p_k first
// (k_p_boundary), then the exchange on the second stream while the main stream
// runs the SpMV over the slices that read no ghost column; the ghost-reading
// slices follow once the halo has landed. Same values, same partial slots.
bool overlap_ok(const Ranks& R)
{
    for (int r = 0; r < R.P; r++) {
        const hpccg_hip_matrix* M = R.M[r];
        if (!M->overlap || M->general || M->halo_b_lo < 0 || !R.a[r].fuse_p) return false;
    }
    return true;
}

int enqueue_spmv_overlapped(const Ranks& R, int slot, int k_host)
{
    for (int r = 0; r < R.P; r++) {
        hpccg_hip_matrix* M = R.M[r];
        TRY(use_device(R, r));
        launch_cg_p_boundary(R.a[r], M->send_lo, M->send_hi, M->stream);  // stamps the halo class
        HIP_TRY(hipEventRecord(M->ev_pb, M->stream));
    }
    for (int r = 0; r < R.P; r++) {
        hpccg_hip_matrix* M = R.M[r];
        TRY(use_device(R, r));
        double* p = ring_p(R.a[r], k_host);
        if (R.P == 1) {
            HIP_TRY(hipStreamWaitEvent(M->stream2, M->ev_pb, 0));
            TRY(enqueue_halo(M, p, M->stream2));
        } else {
            if (r > 0 && M->ghost_lo) {
                const hpccg_hip_matrix* L = R.M[r - 1];
                HIP_TRY(hipStreamWaitEvent(M->stream2, L->ev_pb, 0));
                HIP_TRY(hipMemcpyPeerAsync(p - M->ghost_lo, M->device,
                                           ring_p(R.a[r - 1], k_host) + L->nrow - M->ghost_lo, L->device,
                                           sizeof(double) * M->ghost_lo, M->stream2));
            }
            if (r < R.P - 1 && M->ghost_hi) {
                const hpccg_hip_matrix* U = R.M[r + 1];
                HIP_TRY(hipStreamWaitEvent(M->stream2, U->ev_pb, 0));
                HIP_TRY(hipMemcpyPeerAsync(p + M->nrow, M->device, ring_p(R.a[r + 1], k_host), U->device,
                                           sizeof(double) * M->ghost_hi, M->stream2));
            }
        }
        HIP_TRY(hipEventRecord(M->ev_halo, M->stream2));
    }
    for (int r = 0; r < R.P; r++) {
        hpccg_hip_matrix* M = R.M[r];
        const CgArgs& a = R.a[r];
        TRY(use_device(R, r));
        const int lo = M->halo_b_lo, hi = M->halo_b_hi, mid = M->nslices - lo - hi;
        if (slot >= 0) HIP_TRY(hipEventRecord(M->ev[4 * slot], M->stream));
        if (a.agroup) {
            // groups holding a ghost-reading slice run after the halo: the
            // first ceil(lo / G) and every group from floor((S - hi) / G)
            const int G = a.agroup, NG = (M->nslices + G - 1) / G;
            const int glo = std::min(NG, (lo + G - 1) / G);
            const int ghi0 = std::max(glo, (M->nslices - hi) / G);
            launch_cg_spmv(group_range(a, glo, ghi0 - glo, 0, 0), M->spmv_variant, false, M->stream);
            HIP_TRY(hipStreamWaitEvent(M->stream, M->ev_halo, 0));
            if (glo + (NG - ghi0) > 0)
                launch_cg_spmv(group_range(a, 0, glo, ghi0, NG - ghi0), M->spmv_variant, false, M->stream);
        } else {
            launch_cg_spmv(spmv_range(a, lo, mid, 0, 0), M->spmv_variant, false, M->stream);
            HIP_TRY(hipStreamWaitEvent(M->stream, M->ev_halo, 0));
            if (lo + hi > 0)
                launch_cg_spmv(spmv_range(a, 0, lo, M->nslices - hi, hi), M->spmv_variant, false, M->stream);
        }
        if (slot >= 0) HIP_TRY(hipEventRecord(M->ev[4 * slot + 1], M->stream));
        if (!a.redund && !a.pap_upd && !fold_of(a, kPAP)) launch_cg_finalize(a, kPAP, false, M->stream);
    }
    return 0;
}

int enqueue_iteration(const Ranks& R, int slot = -1, int k_host = 1)
{
    const bool multi = R.a[0].nranks > 1;
    if (multi && overlap_ok(R)) {
        TRY(enqueue_spmv_overlapped(R, slot, k_host));
        TRY(exch_allreduce(R, kPAP, false));
        for (int r = 0; r < R.P; r++) {
            hpccg_hip_matrix* M = R.M[r];
            const CgArgs& a = R.a[r];
            TRY(use_device(R, r));
            if (slot >= 0) HIP_TRY(hipEventRecord(M->ev[4 * slot + 2], M->stream));
            launch_cg_update(a, false, M->stream);
            if (slot >= 0) HIP_TRY(hipEventRecord(M->ev[4 * slot + 3], M->stream));
            if (!a.redund && !fold_of(a, kRR)) launch_cg_finalize(a, kRR, false, M->stream);
        }
        TRY(exch_allreduce(R, kRR, false));
        HIP_TRY(hipGetLastError());
        return 0;
    }
    for (int r = 0; r < R.P; r++) {
        TRY(use_device(R, r));
        if (!R.a[r].fuse_p)
            launch_cg_p_update(R.a[r], R.M[r]->stream);
        else if (multi && !R.M[r]->general)  // gather plan: k_pack computes the halo rows
            launch_cg_p_boundary(R.a[r], R.M[r]->send_lo, R.M[r]->send_hi, R.M[r]->stream);
    }
    if (multi) TRY(exch_halo(R, k_host, false));
    for (int r = 0; r < R.P; r++) {
        hpccg_hip_matrix* M = R.M[r];
        const CgArgs& a = R.a[r];
        TRY(use_device(R, r));
        if (slot >= 0) HIP_TRY(hipEventRecord(M->ev[4 * slot], M->stream));
        launch_cg_spmv(a, M->spmv_variant, false, M->stream);
        if (slot >= 0) HIP_TRY(hipEventRecord(M->ev[4 * slot + 1], M->stream));
        if (!a.redund && !a.pap_upd && !fold_of(a, kPAP)) launch_cg_finalize(a, kPAP, false, M->stream);
    }
    if (multi) TRY(exch_allreduce(R, kPAP, false));
    for (int r = 0; r < R.P; r++) {
        hpccg_hip_matrix* M = R.M[r];
        const CgArgs& a = R.a[r];
        TRY(use_device(R, r));
        if (slot >= 0) HIP_TRY(hipEventRecord(M->ev[4 * slot + 2], M->stream));
        launch_cg_update(a, false, M->stream);
        if (slot >= 0) HIP_TRY(hipEventRecord(M->ev[4 * slot + 3], M->stream));
        if (!a.redund && !fold_of(a, kRR)) launch_cg_finalize(a, kRR, false, M->stream);
    }
    if (multi) TRY(exch_allreduce(R, kRR, false));
    HIP_TRY(hipGetLastError());
    return 0;
}

int enqueue_prologue(const Ranks& R, bool events)
{
    const bool multi = R.a[0].nranks > 1;
    for (int r = 0; r < R.P; r++) {
        TRY(use_device(R, r));
        launch_cg_prologue_copy(R.a[r], R.M[r]->stream);  // p = x
    }
    if (multi) TRY(exch_halo(R, 0, true));
    for (int r = 0; r < R.P; r++) {
        hpccg_hip_matrix* M = R.M[r];
        const CgArgs& a = R.a[r];
        hipStream_t s = M->stream;
        TRY(use_device(R, r));
        if (events) HIP_TRY(hipEventRecord(M->ev[0], s));
        launch_cg_spmv(a, M->spmv_variant, true, s);  // Ap = A p
        if (events) HIP_TRY(hipEventRecord(M->ev[1], s));
        if (events) HIP_TRY(hipEventRecord(M->ev[2], s));
        launch_cg_update(a, true, s);                  // r = b - Ap (+ r.r partials)
        if (events) HIP_TRY(hipEventRecord(M->ev[3], s));
        if (!a.redund && !fold_of(a, kRR)) launch_cg_finalize(a, kRR, true, s);  // rtrans, k = 1
    }
    if (multi) TRY(exch_allreduce(R, kRR, true));
    HIP_TRY(hipGetLastError());
    return 0;
}



int build_graph(hpccg_hip_matrix* M, const CgArgs& a)
{
    if (M->graph_exec) {
        (void)hipGraphExecDestroy(M->graph_exec);
        M->graph_exec = nullptr;
    }
    hipGraph_t g = nullptr;
    HIP_TRY(hipStreamBeginCapture(M->stream, hipStreamCaptureModeThreadLocal));
    int rc = 0;
    const Ranks R{&M, &a, 1, nullptr};
    for (int i = 0; i < M->graph_iters && rc == 0; i++) rc = enqueue_iteration(R, -1, i + 1);
    hipError_t e = hipStreamEndCapture(M->stream, &g);
    if (rc) return rc;
    if (e != hipSuccess) return set_err(HPCCG_HIP_EHIP, "graph capture failed: %s", hipGetErrorString(e));
    e = hipGraphInstantiate(&M->graph_exec, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (e != hipSuccess) return set_err(HPCCG_HIP_EHIP, "graph instantiate failed: %s", hipGetErrorString(e));
    M->graph_chunk = M->graph_iters;
    return 0;
}

// Turns the device stamp sequence into the reference's timer classes.
void stamps_to_times(const std::vector<unsigned long long>& st, int count, double* times)
{
    double t1 = 0, t2 = 0, t3 = 0, t4 = 0, t5 = 0;
    for (int i = 0; i + 1 < count; i++) {
        const int slot = (int)st[2 * i + 1];
        if (slot == kStampEnd) break;
        const double d = (double)(st[2 * (i + 1)] - st[2 * i]) * 1e-8;  // 100 MHz
        switch (slot) {
        case kStampPUpdate:
        case kStampUpdate:
        case kStampPrologue: t2 += d; break;
        case kStampSpmv: t3 += d; break;
        case kStampFinPAP:
        case kStampFinRR: t1 += d; break;
        case kStampArPAP:
        case kStampArRR:
            t1 += d;
            t4 += d;
            break;
        case kStampHalo: t5 += d; break;
        default: break;
        }
    }
    times[1] = t1;
    times[2] = t2;
    times[3] = t3;
    times[4] = t4;
    times[5] = t5;
}

// Solve on the ranks Ms[0..P) (P > 1: an in-process group; P == 1: this
// process's matrix, exchanging through RCCL when the communicator has peers).
int solve_ranks(hpccg_hip_matrix* const* Ms, int P, const double* const* b_dev, double* const* x_dev,
                int max_iter, double tol, int* niters_out, double* normr_out, double* times, int print)
{
    hpccg_hip_matrix* M = Ms[0];
    std::vector<CgArgs> av(P);
    std::vector<hipEvent_t> gev;
    struct EvFree {
        std::vector<hipEvent_t>& v;
        ~EvFree() { for (hipEvent_t e : v) (void)hipEventDestroy(e); }
    } ev_free{gev};
    const int iters = std::max(0, max_iter - 1);
    const bool events = P == 1 && M->event_timing != 0;
    for (int r = 0; r < P; r++) {
        HIP_TRY(hipSetDevice(Ms[r]->device));
        TRY(ensure_hist(Ms[r], max_iter));
        // a variant this matrix cannot run (e.g. a one-rank kernel on a rank of a group)
        if (variant_unavailable(Ms[r], Ms[r]->spmv_variant)) Ms[r]->spmv_variant = choose_variant(Ms[r]);
    }
    if (P > 1) {
        gev.resize(P + 1);
        for (int r = 0; r <= P; r++) {
            HIP_TRY(hipSetDevice(Ms[r < P ? r : 0]->device));
            HIP_TRY(hipEventCreateWithFlags(&gev[r], hipEventDisableTiming));
        }
    }
    HIP_TRY(hipSetDevice(M->device));
    const auto t_begin = std::chrono::steady_clock::now();
    for (int r = 0; r < P; r++) {
        HIP_TRY(hipSetDevice(Ms[r]->device));
        av[r] = make_args(Ms[r], b_dev[r], x_dev[r], max_iter, tol);
        HIP_TRY(hipMemsetAsync(Ms[r]->d_kst, 0, sizeof(int) * 8, Ms[r]->stream));  // iteration state
        HIP_TRY(hipMemsetAsync(Ms[r]->d_tickets, 0, sizeof(unsigned int) * Ms[r]->ntickets, Ms[r]->stream));
    }
    const CgArgs& a = av[0];
    const Ranks R{Ms, av.data(), P, gev.data()};
    if (events) TRY(ensure_events(M, iters + 1));
    TRY(enqueue_prologue(R, events));
    const int chunk = std::max(1, M->graph_iters);
    const bool graph = P == 1 && !events && M->use_graph && M->nranks == 1 && iters >= chunk;
    int done = 0;
    if (graph) {
        // kernel arguments are baked into the graph: rebuild only when they change
        if (!M->graph_exec || std::memcmp(&M->graph_args, &a, sizeof a) != 0 ||
            M->graph_variant != M->spmv_variant || M->graph_chunk != chunk) {
            TRY(build_graph(M, a));
            M->graph_args = a;
            M->graph_variant = M->spmv_variant;
        }
        for (; done + chunk <= iters; done += chunk)
            HIP_TRY(hipGraphLaunch(M->graph_exec, M->stream));
    }
    for (; done < iters; done++) TRY(enqueue_iteration(R, events ? done + 1 : -1, done + 1));
    for (int r = P - 1; r >= 0; r--) {
        TRY(use_device(R, r));
        launch_cg_end(av[r], Ms[r]->stream);
        launch_cg_xflush(av[r], Ms[r]->stream);  // x += alpha_j p_j still pending (x_defer)
        HIP_TRY(hipGetLastError());
        if (r > 0) HIP_TRY(hipStreamSynchronize(Ms[r]->stream));
    }
    // results
    int kst[4];
    HIP_TRY(hipMemcpyAsync(kst, M->d_kst, sizeof kst, hipMemcpyDeviceToHost, M->stream));
    double scal[8];
    HIP_TRY(hipMemcpyAsync(scal, M->d_scal, sizeof scal, hipMemcpyDeviceToHost, M->stream));
    HIP_TRY(hipStreamSynchronize(M->stream));
    const auto t_end = std::chrono::steady_clock::now();
    const int niters = std::max(0, kst[0] - 1);
    std::vector<double> hist(std::max(1, niters));
    if (niters > 0)
        HIP_TRY(hipMemcpy(hist.data(), M->d_hist, sizeof(double) * niters, hipMemcpyDeviceToHost));
    const int nst = std::min(kst[2], M->stamp_cap);
    std::vector<unsigned long long> st(2 * std::max(1, nst));
    if (nst > 0)
        HIP_TRY(hipMemcpy(st.data(), M->d_stamps, sizeof(unsigned long long) * 2 * nst,
                          hipMemcpyDeviceToHost));
    // normr after iteration k is sqrt(r_{k-1}.r_{k-1}) (HPCCG.cpp:371)
    M->trace.assign(niters + 1, 0.0);
    M->trace[0] = std::sqrt(niters > 0 ? hist[0] : scal[kRR]);
    for (int k = 1; k <= niters; k++) M->trace[k] = std::sqrt(hist[k - 1]);
    M->last_niters = niters;
    for (int r = 1; r < P; r++) {  // every group member reports the same solve
        Ms[r]->trace = M->trace;
        Ms[r]->last_niters = niters;
    }
    const double normr = M->trace[niters];
    if (events) {
        double sp = 0, up = 0;
        for (int i = 0; i <= niters; i++) {
            float ms = 0.f;
            HIP_TRY(hipEventElapsedTime(&ms, M->ev[4 * i], M->ev[4 * i + 1]));
            sp += ms;
            HIP_TRY(hipEventElapsedTime(&ms, M->ev[4 * i + 2], M->ev[4 * i + 3]));
            up += ms;
        }
        M->ktimes[0] = sp;
        M->ktimes[1] = niters + 1;
        M->ktimes[2] = up;
        M->ktimes[3] = niters + 1;
    }
    if (print && M->rank == 0) {
        int pf = max_iter / 10;
        if (pf > 50) pf = 50;
        if (pf < 1) pf = 1;
        std::cout << "Initial Residual = " << M->trace[0] << std::endl;
        for (int k = 1; k <= niters; k++)
            if (k % pf == 0 || k + 1 == max_iter)
                std::cout << "Iteration = " << k << "   Residual = " << M->trace[k] << std::endl;
    }
    if (times) {
        stamps_to_times(st, nst, times);
        times[0] = std::chrono::duration<double>(t_end - t_begin).count();
    }
    *niters_out = niters;
    *normr_out = normr;
    return 0;
}

int solve_impl(hpccg_hip_matrix* M, const double* b_dev, double* x_dev, int max_iter, double tol,
               int* niters_out, double* normr_out, double* times, int print)
{
    HIP_TRY(hipSetDevice(M->device));
    if (M->in_group) return set_err(HPCCG_HIP_EINVAL, "group member: solve with hpccg_hip_group_solve");
    return solve_ranks(&M, 1, &b_dev, &x_dev, max_iter, tol, niters_out, normr_out, times, print);
}

// ---------------------------------------------------------------------------
// SELL-512-L windows. Per slice: the sorted distinct columns the slice reads,
// merged into windows when the gap is <= kWinGap entries (staging a few unused
// x is cheaper than another window). A matrix qualifies when every slice fits
// kLdsMaxDoubles entries in <= kLdsMaxWindows windows; otherwise the plain
// SELL-512 kernels are used.
// ---------------------------------------------------------------------------
constexpr int kWinGap = 16;

struct Windows {
    std::vector<int> ptr, start, len, off;
    int max_staged = 0;
};

bool windows_from_cols(std::vector<int>& cols, Windows& W)
{
    std::sort(cols.begin(), cols.end());
    cols.erase(std::unique(cols.begin(), cols.end()), cols.end());
    int staged = 0, nw = 0;
    size_t i = 0;
    while (i < cols.size()) {
        const int st = cols[i];
        int last = st;
        size_t j = i + 1;
        while (j < cols.size() && cols[j] - last <= kWinGap) last = cols[j++];
        W.start.push_back(st);
        W.len.push_back(last - st + 1);
        W.off.push_back(staged);
        staged += last - st + 1;
        nw++;
        i = j;
    }
    W.ptr.push_back((int)W.start.size());
    W.max_staged = std::max(W.max_staged, staged);
    return staged <= kLdsMaxDoubles && nw <= kLdsMaxWindows;
}

// From the host SELL image (local columns, -1 padding). Fills lcols.
bool build_windows_from_image(int nslices, const std::vector<unsigned int>& sb, const std::vector<int>& hc,
                              Windows& W, std::vector<unsigned short>& lcols)
{
    W = Windows();
    W.ptr.push_back(0);
    std::vector<int> cols;
    for (int s = 0; s < nslices; s++) {
        cols.clear();
        const size_t e0 = (size_t)sb[s] * kSliceRows, e1 = (size_t)sb[s + 1] * kSliceRows;
        for (size_t e = e0; e < e1; e++)
            if (hc[e] >= 0) cols.push_back(hc[e]);
        if (!windows_from_cols(cols, W)) return false;
    }
    lcols.assign(hc.size(), kLdsPad);
    const int nth = std::max(1, std::min<int>(16, (int)std::thread::hardware_concurrency()));
    auto work = [&](int t) {
        for (int s = t; s < nslices; s += nth) {
            const int w0 = W.ptr[s], w1 = W.ptr[s + 1];
            const size_t e0 = (size_t)sb[s] * kSliceRows, e1 = (size_t)sb[s + 1] * kSliceRows;
            for (size_t e = e0; e < e1; e++) {
                const int c = hc[e];
                if (c < 0) continue;
                int w = w0;
                while (w + 1 < w1 && W.start[w + 1] <= c) w++;
                lcols[e] = (unsigned short)(W.off[w] + c - W.start[w]);
            }
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nth; t++) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
    return true;
}

// Stencil slabs, analytically: a superset of the columns a slice of rows
// [r0, r1) can touch -- the three z-planes' ranges widened by nx + 1.
bool build_windows_stencil(int nslices, int nrow, int nx, int nxy, int ghost_lo, long long ncol_ext,
                           Windows& W, bool use_7pt = false)
{
    W = Windows();
    W.ptr.push_back(0);
    for (int s = 0; s < nslices; s++) {
        const long long r0 = (long long)s * kSliceRows, r1 = std::min<long long>(nrow, r0 + kSliceRows);
        std::vector<std::pair<long long, long long>> iv;
        for (int sz = -1; sz <= 1; sz++) {
            // 27-pt: every plane +-(nx+1); 7-pt: the +-1 planes only straight across,
            // the own plane +-nx (generate_matrix.cpp:259-281)
            const long long m = use_7pt ? (sz == 0 ? nx : 0) : nx + 1;
            long long lo = ghost_lo + r0 + (long long)sz * nxy - m;
            long long hi = ghost_lo + r1 - 1 + (long long)sz * nxy + m;
            lo = std::max(0LL, lo);
            hi = std::min(ncol_ext - 1, hi);
            if (lo <= hi) iv.push_back({lo, hi});
        }
        std::sort(iv.begin(), iv.end());
        int staged = 0, nw = 0;
        long long cs = -1, ce = -2;
        auto flush = [&]() {
            if (cs < 0) return;
            W.start.push_back((int)cs);
            W.len.push_back((int)(ce - cs + 1));
            W.off.push_back(staged);
            staged += (int)(ce - cs + 1);
            nw++;
        };
        for (auto& p : iv) {
            if (cs >= 0 && p.first <= ce + kWinGap) {
                ce = std::max(ce, p.second);
            } else {
                flush();
                cs = p.first;
                ce = p.second;
            }
        }
        flush();
        W.ptr.push_back((int)W.start.size());
        W.max_staged = std::max(W.max_staged, staged);
        if (staged > kLdsMaxDoubles || nw > kLdsMaxWindows) return false;
    }
    return true;
}

// Which slices read ghost columns (their windows reach outside [ghost_lo,
// ghost_lo + n)): a leading and a trailing run for slab plans, else no overlap.
void halo_runs(hpccg_hip_matrix* M, const Windows& W)
{
    M->halo_b_lo = M->halo_b_hi = -1;
    if (M->nslices < 1 || (int)W.ptr.size() != M->nslices + 1) return;
    const long long lo = M->ghost_lo, hi = (long long)M->ghost_lo + M->nrow;
    std::vector<char> t(M->nslices, 0);
    for (int s = 0; s < M->nslices; s++)
        for (int w = W.ptr[s]; w < W.ptr[s + 1]; w++)
            if (W.start[w] < lo || (long long)W.start[w] + W.len[w] > hi) t[s] = 1;
    int a = 0, b = 0;
    while (a < M->nslices && t[a]) a++;
    while (b < M->nslices - a && t[M->nslices - 1 - b]) b++;
    for (int s = a; s < M->nslices - b; s++)
        if (t[s]) return;  // a ghost reader in the middle: no overlap
    if (a + b >= M->nslices) return;
    M->halo_b_lo = a;
    M->halo_b_hi = b;
}

int upload_windows(hpccg_hip_matrix* M, const Windows& W)
{
    halo_runs(M, W);
    M->nwin = (int)W.start.size();
    const size_t nw = std::max<size_t>(1, W.start.size());
    HIP_TRY(hipMalloc(&M->d_win_ptr, sizeof(int) * W.ptr.size()));
    HIP_TRY(hipMemcpy(M->d_win_ptr, W.ptr.data(), sizeof(int) * W.ptr.size(), hipMemcpyHostToDevice));
    int** dst[] = {&M->d_win_start, &M->d_win_len, &M->d_win_off};
    const std::vector<int>* src[] = {&W.start, &W.len, &W.off};
    for (int i = 0; i < 3; i++) {
        HIP_TRY(hipMalloc(dst[i], sizeof(int) * nw));
        if (!src[i]->empty())
            HIP_TRY(hipMemcpy(*dst[i], src[i]->data(), sizeof(int) * src[i]->size(), hipMemcpyHostToDevice));
    }
    M->lds_doubles = std::max(1, W.max_staged);
    M->has_lds = 1;
    return 0;
}

template <class RowLen, class RowAt>
int create_from_rows(hpccg_hip_matrix** out, int nrow, int start_row, int total_nrow, RowLen row_len,
                     RowAt row_at)
{
    if (!out) return set_err(HPCCG_HIP_EINVAL, "out is NULL");
    if (nrow < 0) return set_err(HPCCG_HIP_EINVAL, "nrow < 0");
    MatrixGuard guard{new hpccg_hip_matrix()};
    hpccg_hip_matrix* M = guard.m;
    HIP_TRY(hipGetDevice(&M->device));
    M->nrow = nrow;
    M->start_row = start_row;
    M->total_nrow = total_nrow;
    // halo plan from the column range
    long long mn = start_row, mx = (long long)start_row + nrow - 1, nnz = 0;
    for (int i = 0; i < nrow; i++) {
        const int len = row_len(i);
        nnz += len;
        for (int j = 0; j < len; j++) {
            long long c;
            double v;
            row_at(i, j, &c, &v);
            mn = std::min(mn, c);
            mx = std::max(mx, c);
        }
    }
    M->nnz = nnz;
    M->ghost_lo = (int)std::max(0LL, (long long)start_row - mn);
    M->ghost_hi = (int)std::max(0LL, mx - ((long long)start_row + nrow - 1));
    if (mn < 0 || mx >= total_nrow) return set_err(HPCCG_HIP_EPLAN, "column outside [0, total_nrow)");
    HIP_TRY(hipStreamCreateWithFlags(&M->stream, hipStreamDefault));
    {
        // halo stream at the highest priority: its small transfer kernels get CUs
        // while the interior SpMV fills the chip
        int least = 0, greatest = 0;
        HIP_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
        HIP_TRY(hipStreamCreateWithPriority(&M->stream2, hipStreamDefault, greatest));
    }
    HIP_TRY(hipEventCreateWithFlags(&M->ev_pb, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&M->ev_halo, hipEventDisableTiming));
    int mode = 1;
    std::vector<int> all;
    GatherPlan gp_local;
    const GatherPlan* gp = nullptr;
    int rc = exchange_plan(M, &mode, &all);
    if (rc == 0 && mode == 2) {
        // gather plan: externals after the local rows (make_local_matrix.cpp:58-610)
        if (g_group_ctx.active) {
            gp = g_group_ctx.plan;
            if (!gp) rc = set_err(HPCCG_HIP_EPLAN, "group member without a gather plan");
        } else {
            gather_externals(nrow, start_row, all.data(), M->nranks, row_len, row_at, gp_local);
            rc = rccl_requests(M, gp_local);
            gp = &gp_local;
        }
        if (rc == 0) rc = install_gather(M, *gp);
    } else if (rc == 0 && g_group_ctx.active && g_group_ctx.info && M->nranks > 1) {
        int sends[2];
        rc = hpccg_slab_plan(M->nranks, M->rank, g_group_ctx.info, sends);
        M->send_lo = sends[0];
        M->send_hi = sends[1];
    }
    if (rc) {
        return rc;
    }
    M->nslices = (nrow + kSliceRows - 1) / kSliceRows;
    M->grid = std::max(kNumXcd, (M->nslices + kNumXcd - 1) / kNumXcd * kNumXcd);
    const long long col_base = (long long)start_row - M->ghost_lo;
    const long long ncol_ext = (long long)M->ghost_lo + nrow + M->ghost_hi;
    // uniform width when padding to the max costs < 4 % (stencils)
    std::vector<unsigned int> sb(M->nslices + 1);
    std::vector<int> hc;
    std::vector<double> hv;
    int bad = 0;
    auto build = [&](auto colmap) {
        const long long slots_var = sell_build_impl(nrow, colmap, row_len, row_at, sb.data(), nullptr, nullptr, 0,
                                                    nullptr);
        const long long slots_uni = sell_build_impl(nrow, colmap, row_len, row_at, sb.data(), nullptr, nullptr, 1,
                                                    nullptr);
        M->uniform = (slots_uni <= slots_var + slots_var / 25) ? 1 : 0;
        M->nslots = sell_build_impl(nrow, colmap, row_len, row_at, sb.data(), nullptr, nullptr, M->uniform,
                                    nullptr);
        M->width = M->nslices ? (int)(M->nslots / kSliceRows / M->nslices) : 0;
        hc.assign((size_t)std::max(1LL, M->nslots), 0);
        hv.assign((size_t)std::max(1LL, M->nslots), 0.0);
        sell_build_impl(nrow, colmap, row_len, row_at, sb.data(), hc.data(), hv.data(), M->uniform, &bad);
    };
    if (M->general) {
        // own columns -> c - start_row; externals -> n + j (ghost_lo = 0)
        const std::unordered_map<long long, int>& ext = gp->ext_of;
        const long long s0 = start_row, n0 = nrow;
        build([&ext, s0, n0](long long c) -> long long {
            if (c >= s0 && c < s0 + n0) return c - s0;
            const auto it = ext.find(c);
            return it == ext.end() ? -1 : n0 + it->second;
        });
    } else {
        build(SlabCols{col_base, ncol_ext});
    }
    if (bad) {
        return set_err(HPCCG_HIP_EPLAN, "column index outside the halo plan");
    }
    Windows W;
    std::vector<unsigned short> lc;
    const bool lds_ok = nrow > 0 && build_windows_from_image(M->nslices, sb, hc, W, lc);
    rc = [&]() -> int {
        HIP_TRY(hipMalloc(&M->d_slice_base, sizeof(unsigned int) * sb.size()));
        HIP_TRY(hipMemcpy(M->d_slice_base, sb.data(), sizeof(unsigned int) * sb.size(), hipMemcpyHostToDevice));
        HIP_TRY(hipMalloc(&M->d_cols, sizeof(int) * hc.size()));
        HIP_TRY(hipMemcpy(M->d_cols, hc.data(), sizeof(int) * hc.size(), hipMemcpyHostToDevice));
        HIP_TRY(hipMalloc(&M->d_vals, sizeof(double) * hv.size()));
        HIP_TRY(hipMemcpy(M->d_vals, hv.data(), sizeof(double) * hv.size(), hipMemcpyHostToDevice));
        if (lds_ok) {
            TRY(upload_windows(M, W));
            HIP_TRY(hipMalloc(&M->d_lcols, sizeof(unsigned short) * lc.size()));
            HIP_TRY(hipMemcpy(M->d_lcols, lc.data(), sizeof(unsigned short) * lc.size(), hipMemcpyHostToDevice));
        }
        TRY(build_c_image(M));
        M->spmv_variant = choose_variant(M);
        return alloc_workspace(M);
    }();
    if (rc) {
        return rc;
    }
    *out = guard.release();
    return 0;
}

// scratch for kernel-level ddot without a matrix
struct Scratch {
    double* partial = nullptr;
    int cap = 0;
    double* out = nullptr;
    hipStream_t s = nullptr;
    int device = -1;
};
thread_local Scratch g_scratch;

int scratch_for(int nparts)
{
    int dev;
    HIP_TRY(hipGetDevice(&dev));
    if (g_scratch.device != dev) {
        g_scratch = Scratch();
        g_scratch.device = dev;
        HIP_TRY(hipStreamCreateWithFlags(&g_scratch.s, hipStreamDefault));
        HIP_TRY(hipMalloc(&g_scratch.out, sizeof(double) * 2));
    }
    if (nparts > g_scratch.cap) {
        if (g_scratch.partial) (void)hipFree(g_scratch.partial);
        HIP_TRY(hipMalloc(&g_scratch.partial, sizeof(double) * (nparts + 8)));
        g_scratch.cap = nparts;
    }
    return 0;
}

std::mutex g_dropin_mu;
std::map<const void*, hpccg_hip_matrix*> g_dropin_cache;

}  // namespace

// ---- in-process rank group -------------------------------------------------
namespace {

template <class Make>
int group_make(int nranks, const int* devices, hpccg_hip_matrix** out, Make make, const int* info = nullptr,
               const std::vector<GatherPlan>* plans = nullptr)
{
    if (!out) return set_err(HPCCG_HIP_EINVAL, "out is NULL");
    if (nranks < 1 || nranks > kMaxGroupRanks)
        return set_err(HPCCG_HIP_EINVAL, "group size must be 1..%d", kMaxGroupRanks);
    if (g_comm.nranks > 1) return set_err(HPCCG_HIP_EINVAL, "in-process group inside an RCCL job");
    int cur = 0;
    HIP_TRY(hipGetDevice(&cur));
    for (int r = 0; r < nranks; r++) out[r] = nullptr;
    int rc = 0;
    for (int r = 0; r < nranks && rc == 0; r++) {
        const int dev = devices ? devices[r] : cur;
        if (hipSetDevice(dev) != hipSuccess) {
            rc = set_err(HPCCG_HIP_EHIP, "hipSetDevice(%d) failed", dev);
            break;
        }
        g_group_ctx = GroupCtx{1, nranks, r, info, plans ? &(*plans)[r] : nullptr};
        rc = make(r, &out[r]);
        g_group_ctx = GroupCtx();
    }
    // slab plan from every member's {nrow, ghost_lo, ghost_hi, start_row}
    std::vector<int> minfo(4 * nranks);
    for (int r = 0; r < nranks && rc == 0; r++) {
        const hpccg_hip_matrix* M = out[r];
        int mine[4] = {M->nrow, M->ghost_lo, M->ghost_hi, M->start_row};
        std::memcpy(&minfo[4 * r], mine, sizeof mine);
    }
    for (int r = 0; r < nranks && rc == 0 && !out[0]->general; r++) {
        int sends[2];
        rc = hpccg_slab_plan(nranks, r, minfo.data(), sends);
        if (rc == 0) {
            out[r]->send_lo = sends[0];
            out[r]->send_hi = sends[1];
        }
    }
    // peer access between the members' distinct devices
    for (int r = 0; r < nranks && rc == 0; r++)
        for (int q = 0; q < nranks; q++) {
            if (out[r]->device == out[q]->device) continue;
            int can = 0;
            (void)hipDeviceCanAccessPeer(&can, out[r]->device, out[q]->device);
            if (!can) {
                rc = set_err(HPCCG_HIP_EHIP, "device %d cannot access device %d", out[r]->device,
                             out[q]->device);
                break;
            }
            (void)hipSetDevice(out[r]->device);
            const hipError_t e = hipDeviceEnablePeerAccess(out[q]->device, 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
                rc = set_err(HPCCG_HIP_EHIP, "hipDeviceEnablePeerAccess: %s", hipGetErrorString(e));
                break;
            }
            (void)hipGetLastError();
        }
    (void)hipSetDevice(cur);
    if (rc) {
        for (int r = 0; r < nranks; r++) {
            free_matrix(out[r]);
            out[r] = nullptr;
        }
    }
    return rc;
}

}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

int hpccg_hip_abi_version(void) { return 1; }

const char* hpccg_hip_last_error(void) { return g_err.c_str(); }

int hpccg_hip_device_count(int* count)
{
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) c = 0;
    *count = c;
    return c > 0 ? 0 : set_err(HPCCG_HIP_ENODEV, "no HIP device");
}

int hpccg_hip_set_device(int device)
{
    HIP_TRY(hipSetDevice(device));
    return 0;
}

int hpccg_hip_comm_unique_id(unsigned char id_out[128])
{
    ncclUniqueId id;
    NCCL_TRY(ncclGetUniqueId(&id));
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    std::memcpy(id_out, &id, 128);
    return 0;
}

int hpccg_hip_comm_init(const unsigned char id[128], int nranks, int rank)
{
    if (nranks < 1 || rank < 0 || rank >= nranks) return set_err(HPCCG_HIP_EINVAL, "bad nranks/rank");
    if (g_comm.comm) {
        ncclCommDestroy(g_comm.comm);
        g_comm = Comm();
    }
    // a 1-rank communicator is created too (bootstrap + RCCL check on one GPU);
    // the solver still takes its single-rank path when nranks == 1
    ncclUniqueId uid;
    std::memcpy(&uid, id, 128);
    NCCL_TRY(ncclCommInitRank(&g_comm.comm, nranks, uid, rank));
    g_comm.nranks = nranks;
    g_comm.rank = rank;
    return 0;
}

int hpccg_hip_comm_destroy(void)
{
    if (g_comm.comm) ncclCommDestroy(g_comm.comm);
    g_comm = Comm();
    return 0;
}

int hpccg_hip_comm_size(int* nranks, int* rank)
{
    if (nranks) *nranks = g_comm.nranks;
    if (rank) *rank = g_comm.rank;
    return 0;
}

int hpccg_hip_comm_allreduce_host(double* vals, int n, int op)
{
    if (!vals || n < 0 || op < 0 || op > 2) return set_err(HPCCG_HIP_EINVAL, "bad argument");
    if (!g_comm.comm || n == 0) return 0;
    double* d = nullptr;
    hipStream_t s = nullptr;
    HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamDefault));
    HIP_TRY(hipMalloc(&d, sizeof(double) * n));
    HIP_TRY(hipMemcpy(d, vals, sizeof(double) * n, hipMemcpyHostToDevice));
    const ncclRedOp_t ops[3] = {ncclSum, ncclMin, ncclMax};
    NCCL_TRY(ncclAllReduce(d, d, n, ncclFloat64, ops[op], g_comm.comm, s));
    HIP_TRY(hipStreamSynchronize(s));
    HIP_TRY(hipMemcpy(vals, d, sizeof(double) * n, hipMemcpyDeviceToHost));
    (void)hipFree(d);
    (void)hipStreamDestroy(s);
    return 0;
}

int hpccg_hip_device_name(char* buf, int cap, int* cus)
{
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, dev));
    if (buf && cap > 0) {
        std::snprintf(buf, cap, "%s (%s)", prop.name[0] ? prop.name : "AMD Instinct GPU", prop.gcnArchName);
    }
    if (cus) *cus = prop.multiProcessorCount;
    return 0;
}

int hpccg_hip_matrix_create(const HPC_Sparse_Matrix* A, hpccg_hip_matrix** out)
{
    if (!A) return set_err(HPCCG_HIP_EINVAL, "A is NULL");
    const int n = A->local_nrow;
    return create_from_rows(
        out, n, A->start_row, A->total_nrow, [A](int i) { return A->nnz_in_row[i]; },
        [A](int i, int j, long long* c, double* v) {
            *c = A->ptr_to_inds_in_row[i][j];
            *v = A->ptr_to_vals_in_row[i][j];
        });
}

int hpccg_hip_matrix_create_csr(int nrow, int start_row, int total_nrow, const long long* row_ptr,
                                const int* cols, const double* vals, hpccg_hip_matrix** out)
{
    if (nrow > 0 && (!row_ptr || !cols || !vals)) return set_err(HPCCG_HIP_EINVAL, "NULL CSR array");
    return create_from_rows(
        out, nrow, start_row, total_nrow, [row_ptr](int i) { return (int)(row_ptr[i + 1] - row_ptr[i]); },
        [row_ptr, cols, vals](int i, int j, long long* c, double* v) {
            *c = cols[row_ptr[i] + j];
            *v = vals[row_ptr[i] + j];
        });
}

int hpccg_hip_matrix_generate(int nx, int ny, int nz, int use_7pt, hpccg_hip_matrix** out)
{
    if (nx < 1 || ny < 1 || nz < 1) return set_err(HPCCG_HIP_EINVAL, "nx, ny, nz must be >= 1");
    const long long n64 = (long long)nx * ny * nz;
    if (n64 * comm_nranks() >= (1LL << 31)) return set_err(HPCCG_HIP_EINVAL, "global rows exceed int32");
    const int n = (int)n64, rank = comm_rank(), size = comm_nranks();
    MatrixGuard guard{new hpccg_hip_matrix()};
    hpccg_hip_matrix* M = guard.m;
    HIP_TRY(hipGetDevice(&M->device));
    M->nrow = n;
    M->start_row = n * rank;
    M->total_nrow = n * size;
    const int nxy = nx * ny;
    M->ghost_lo = rank > 0 ? std::min(nxy, n) : 0;
    M->ghost_hi = rank < size - 1 ? std::min(nxy, n) : 0;
    // rows per z-plane beyond one plane would need rank+-2 (nz >= 1 keeps it at +-1)
    HIP_TRY(hipStreamCreateWithFlags(&M->stream, hipStreamDefault));
    {
        // halo stream at the highest priority: its small transfer kernels get CUs
        // while the interior SpMV fills the chip
        int least = 0, greatest = 0;
        HIP_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
        HIP_TRY(hipStreamCreateWithPriority(&M->stream2, hipStreamDefault, greatest));
    }
    HIP_TRY(hipEventCreateWithFlags(&M->ev_pb, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&M->ev_halo, hipEventDisableTiming));
    int rc = exchange_plan(M);
    if (rc) {
        return rc;
    }
    M->nslices = (n + kSliceRows - 1) / kSliceRows;
    M->grid = std::max(kNumXcd, (M->nslices + kNumXcd - 1) / kNumXcd * kNumXcd);
    // row lengths analytically (generate_matrix.cpp:259-281 acceptance test)
    auto axis = [](int i, int nn) { return 1 + (i > 0) + (i < nn - 1); };
    const long long total = (long long)n * size;
    const long long start = (long long)n * rank;
    auto row_len = [&](int lrow) -> int {
        const int iz = lrow / nxy, iy = (lrow % nxy) / nx, ix = lrow % nx;
        const long long grow = start + lrow;
        const int zl = grow - nxy >= 0, zh = grow + nxy < total;
        if (use_7pt) return 1 + (ix > 0) + (ix < nx - 1) + (iy > 0) + (iy < ny - 1) + zl + zh;
        (void)iz;
        return axis(ix, nx) * axis(iy, ny) * (1 + zl + zh);
    };
    std::vector<int> w(M->nslices, 0);
    long long nnz = 0;
    for (int i = 0; i < n; i++) {
        const int l = row_len(i);
        nnz += l;
        w[i / kSliceRows] = std::max(w[i / kSliceRows], l);
    }
    M->nnz = nnz;
    int wmax = 0;
    long long var = 0;
    for (int s = 0; s < M->nslices; s++) {
        wmax = std::max(wmax, w[s]);
        var += w[s];
    }
    M->uniform = ((long long)wmax * M->nslices <= var + var / 25) ? 1 : 0;
    std::vector<unsigned int> sb(M->nslices + 1);
    long long acc = 0;
    for (int s = 0; s < M->nslices; s++) {
        sb[s] = (unsigned int)acc;
        acc += M->uniform ? wmax : w[s];
    }
    sb[M->nslices] = (unsigned int)acc;
    M->nslots = acc * kSliceRows;
    M->width = M->uniform ? wmax : 0;
    Windows W;
    const long long ncol_ext = (long long)M->ghost_lo + n + M->ghost_hi;
    const bool lds_ok = build_windows_stencil(M->nslices, n, nx, nxy, M->ghost_lo, ncol_ext, W, use_7pt != 0);
    rc = [&]() -> int {
        HIP_TRY(hipMalloc(&M->d_slice_base, sizeof(unsigned int) * sb.size()));
        HIP_TRY(hipMemcpy(M->d_slice_base, sb.data(), sizeof(unsigned int) * sb.size(), hipMemcpyHostToDevice));
        if (lds_ok) {
            TRY(upload_windows(M, W));
            HIP_TRY(hipMalloc(&M->d_lcols, sizeof(unsigned short) * std::max(1LL, M->nslots)));
        }
        HIP_TRY(hipMalloc(&M->d_cols, sizeof(int) * std::max(1LL, M->nslots)));
        HIP_TRY(hipMalloc(&M->d_vals, sizeof(double) * std::max(1LL, M->nslots)));
        TRY(alloc_workspace(M));
        HIP_TRY(hipMalloc(&M->d_gen_b, sizeof(double) * M->npad));
        HIP_TRY(hipMalloc(&M->d_gen_x0, sizeof(double) * M->npad));
        HIP_TRY(hipMalloc(&M->d_gen_xexact, sizeof(double) * M->npad));
        HIP_TRY(hipMemset(M->d_gen_b, 0, sizeof(double) * M->npad));
        HIP_TRY(hipMemset(M->d_gen_x0, 0, sizeof(double) * M->npad));
        HIP_TRY(hipMemset(M->d_gen_xexact, 0, sizeof(double) * M->npad));
        launch_generate(nx, ny, nz, rank, size, use_7pt, start - M->ghost_lo, M->d_slice_base, M->d_cols,
                        M->d_vals, M->d_gen_b, M->d_gen_xexact, n, M->d_win_ptr, M->d_win_start,
                        M->d_win_len, M->d_win_off, M->d_lcols, M->stream);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipStreamSynchronize(M->stream));
        TRY(build_c_image(M));
        M->spmv_variant = choose_variant(M);
        return 0;
    }();
    if (rc) {
        return rc;
    }
    *out = guard.release();
    return 0;
}


int hpccg_hip_group_generate(int nx, int ny, int nz, int use_7pt, int nranks, const int* devices,
                             hpccg_hip_matrix** out)
{
    return group_make(nranks, devices, out, [&](int, hpccg_hip_matrix** m) {
        return hpccg_hip_matrix_generate(nx, ny, nz, use_7pt, m);
    });
}

int hpccg_hip_group_create_csr(int nranks, const int* devices, const int* nrow, const int* start_row,
                               int total_nrow, const long long* const* row_ptr, const int* const* cols,
                               const double* const* vals, hpccg_hip_matrix** out)
{
    if (!nrow || !start_row || !row_ptr || !cols || !vals) return set_err(HPCCG_HIP_EINVAL, "NULL argument");
    if (nranks < 1 || nranks > kMaxGroupRanks)
        return set_err(HPCCG_HIP_EINVAL, "group size must be 1..%d", kMaxGroupRanks);
    // what the all-gather of exchange_plan would give every member
    std::vector<int> info(4 * nranks);
    for (int r = 0; r < nranks; r++) {
        if (nrow[r] < 0 || (nrow[r] > 0 && (!row_ptr[r] || !cols[r] || !vals[r])))
            return set_err(HPCCG_HIP_EINVAL, "member %d: bad CSR", r);
        long long mn = start_row[r], mx = (long long)start_row[r] + nrow[r] - 1;
        for (long long e = 0; e < (nrow[r] > 0 ? row_ptr[r][nrow[r]] : 0); e++) {
            mn = std::min<long long>(mn, cols[r][e]);
            mx = std::max<long long>(mx, cols[r][e]);
        }
        if (mn < 0 || mx >= total_nrow) return set_err(HPCCG_HIP_EPLAN, "member %d: column outside [0, total_nrow)", r);
        info[4 * r] = nrow[r];
        info[4 * r + 1] = (int)std::max(0LL, (long long)start_row[r] - mn);
        info[4 * r + 2] = (int)std::max(0LL, mx - ((long long)start_row[r] + nrow[r] - 1));
        info[4 * r + 3] = start_row[r];
    }
    const int mode = nranks == 1 ? 1 : choose_halo_mode(info.data(), nranks);
    if (mode < 0) return set_err(HPCCG_HIP_EPLAN, "the z-slab halo plan cannot serve this partition");
    std::vector<GatherPlan> plans;
    if (mode == 2) {  // the requests every member would send its owners, then the send runs
        plans.resize(nranks);
        for (int r = 0; r < nranks; r++) {
            const long long* rp = row_ptr[r];
            const int* cl = cols[r];
            const double* vl = vals[r];
            gather_externals(nrow[r], start_row[r], info.data(), nranks,
                             [rp](int i) { return (int)(rp[i + 1] - rp[i]); },
                             [rp, cl, vl](int i, int j, long long* c, double* v) {
                                 *c = cl[rp[i] + j];
                                 *v = vl[rp[i] + j];
                             },
                             plans[r]);
        }
        for (int r = 0; r < nranks; r++) {
            std::vector<std::vector<int>> to_me(nranks);
            for (int q = 0; q < nranks; q++) to_me[q] = plans[q].req[r];
            gather_sends(start_row[r], to_me, plans[r]);
        }
    }
    return group_make(
        nranks, devices, out,
        [&](int r, hpccg_hip_matrix** m) {
            return hpccg_hip_matrix_create_csr(nrow[r], start_row[r], total_nrow, row_ptr[r], cols[r], vals[r], m);
        },
        info.data(), mode == 2 ? &plans : nullptr);
}

int hpccg_hip_group_solve(hpccg_hip_matrix* const* Ms, int nranks, const double* const* b_dev,
                          double* const* x_dev, int max_iter, double tolerance, int* niters, double* normr,
                          double* times)
{
    if (!Ms || !b_dev || !x_dev || !niters || !normr || nranks < 1 || nranks > kMaxGroupRanks)
        return set_err(HPCCG_HIP_EINVAL, "bad argument");
    for (int r = 0; r < nranks; r++) {
        if (!Ms[r] || !b_dev[r] || !x_dev[r]) return set_err(HPCCG_HIP_EINVAL, "NULL member %d", r);
        if (Ms[r]->nranks != nranks || Ms[r]->rank != r || (nranks > 1 && !Ms[r]->in_group))
            return set_err(HPCCG_HIP_EINVAL, "member %d is not rank %d of a %d-rank group", r, r, nranks);
    }
    int cur = 0;
    HIP_TRY(hipGetDevice(&cur));
    const int rc = solve_ranks(Ms, nranks, b_dev, x_dev, max_iter, tolerance, niters, normr, times, 0);
    (void)hipSetDevice(cur);
    return rc;
}

int hpccg_hip_set_halo_mode(int mode)
{
    if (mode < 0 || mode > 2) return set_err(HPCCG_HIP_EINVAL, "halo mode must be 0, 1 or 2");
    g_halo_mode = mode;
    return 0;
}

int hpccg_hip_matrix_destroy(hpccg_hip_matrix* M) { return free_matrix(M); }

int hpccg_hip_matrix_info(const hpccg_hip_matrix* M, long long info[8])
{
    if (!M) return set_err(HPCCG_HIP_EINVAL, "M is NULL");
    info[0] = M->nrow;
    info[1] = (long long)M->ghost_lo + M->nrow + M->ghost_hi;
    info[2] = M->nnz;
    info[3] = M->nslots;
    info[4] = M->ghost_lo;
    info[5] = M->ghost_hi;
    info[6] = M->spmv_variant;
    info[7] = M->uniform ? M->width : 0;
    return 0;
}

int hpccg_hip_matrix_vectors(hpccg_hip_matrix* M, double** b, double** x0, double** xexact)
{
    if (!M || !M->d_gen_b) return set_err(HPCCG_HIP_EINVAL, "not a device-generated matrix");
    if (b) *b = M->d_gen_b;
    if (x0) *x0 = M->d_gen_x0;
    if (xexact) *xexact = M->d_gen_xexact;
    return 0;
}

int hpccg_hip_set_option(hpccg_hip_matrix* M, const char* key, long long value)
{
    if (!M || !key) return set_err(HPCCG_HIP_EINVAL, "NULL argument");
    if (!std::strcmp(key, "use_graph")) {
        M->use_graph = (int)value;
    } else if (!std::strcmp(key, "event_timing")) {
        M->event_timing = (int)value;
    } else if (!std::strcmp(key, "fuse_p")) {
        M->fuse_p = (int)value;
    } else if (!std::strcmp(key, "x_defer")) {
        M->x_defer = (int)value;
    } else if (!std::strcmp(key, "x_ring")) {
        if (value != -1 && (value < 2 || value > kXRingMax))
            return set_err(HPCCG_HIP_EINVAL, "x_ring must be -1 (auto) or 2..%d", kXRingMax);
        const int prev = M->x_ring;
        M->x_ring = (int)value;
        if (x_ring_effective(M) > M->ring_alloc) {
            HIP_TRY(hipSetDevice(M->device));
            HIP_TRY(hipStreamSynchronize(M->stream));
            const int rc = alloc_ring(M, x_ring_effective(M));
            if (rc) {
                M->x_ring = prev;
                return rc;
            }
        }
    } else if (!std::strcmp(key, "rev_update")) {
        M->rev_update = (int)value;
    } else if (!std::strcmp(key, "redund")) {
        M->redund = (int)value;
    } else if (!std::strcmp(key, "update_early")) {
        M->update_early = value != 0;
    } else if (!std::strcmp(key, "pap_in_update")) {
        M->pap_upd = (int)value;
    } else if (!std::strcmp(key, "update_slices")) {
        if (value != 1 && value != 2 && value != 4 && value != 8)
            return set_err(HPCCG_HIP_EINVAL, "update_slices must be 1, 2, 4 or 8");
        M->update_slices = (int)value;
    } else if (!std::strcmp(key, "overlap")) {
        M->overlap = (int)value;
    } else if (!std::strcmp(key, "graph_chunk")) {
        if (value < 1 || value > 4096) return set_err(HPCCG_HIP_EINVAL, "graph_chunk must be 1..4096");
        M->graph_iters = (int)value;
    } else if (!std::strcmp(key, "resident_mb")) {
        M->resident_mb = value < 0 ? -1 : value;
    } else if (!std::strcmp(key, "fold")) {
        M->fold = (int)value;
    } else if (!std::strcmp(key, "value_codes")) {
        M->value_codes = value != 0;
        M->spmv_variant = choose_variant(M);
    } else if (!std::strcmp(key, "spmv_variant")) {
        const int v = (int)value;
        const int w = required_width(v);
        if (!spmv_variant_ok(v) || v == 9999)
            return set_err(HPCCG_HIP_EINVAL, "unknown spmv variant %lld", value);
        if (w && !fixed_width_ok(M, v))
            return set_err(HPCCG_HIP_EINVAL, "variant %d needs a uniform width-%d SELL image", v, w);
        if (const char* why = variant_unavailable(M, v))
            return set_err(HPCCG_HIP_EINVAL, "variant %d needs %s (not built)", v, why);
        M->spmv_variant = v;
    } else {
        return set_err(HPCCG_HIP_EINVAL, "unknown option '%s'", key);
    }
    return 0;
}

int hpccg_hip_solve_device(hpccg_hip_matrix* M, const double* b_dev, double* x_dev, int max_iter,
                           double tolerance, int* niters, double* normr, double* times, int print)
{
    if (!M || !b_dev || !x_dev || !niters || !normr) return set_err(HPCCG_HIP_EINVAL, "NULL argument");
    // The vectorised kernels need 512-row padded buffers: x is staged through
    // the workspace (x_dev may be any length-n buffer); b likewise unless it
    // is the generated b, which is already padded.
    HIP_TRY(hipSetDevice(M->device));
    double* x = M->d_x;
    HIP_TRY(hipMemcpyAsync(x, x_dev, sizeof(double) * M->nrow, hipMemcpyDeviceToDevice, M->stream));
    const double* b = b_dev;
    if (b_dev != M->d_gen_b && b_dev != M->d_b) {
        HIP_TRY(hipMemcpyAsync(M->d_b, b_dev, sizeof(double) * M->nrow, hipMemcpyDeviceToDevice, M->stream));
        b = M->d_b;
    }
    TRY(solve_impl(M, b, x, max_iter, tolerance, niters, normr, times, print));
    HIP_TRY(hipMemcpyAsync(x_dev, x, sizeof(double) * M->nrow, hipMemcpyDeviceToDevice, M->stream));
    HIP_TRY(hipStreamSynchronize(M->stream));
    return 0;
}

int hpccg_hip_solve(hpccg_hip_matrix* M, const double* b, double* x, int max_iter, double tolerance,
                    int* niters, double* normr, double* times, int print)
{
    if (!M || !b || !x || !niters || !normr) return set_err(HPCCG_HIP_EINVAL, "NULL argument");
    HIP_TRY(hipSetDevice(M->device));
    const auto t0 = std::chrono::steady_clock::now();
    HIP_TRY(hipMemcpyAsync(M->d_b, b, sizeof(double) * M->nrow, hipMemcpyHostToDevice, M->stream));
    HIP_TRY(hipMemcpyAsync(M->d_x, x, sizeof(double) * M->nrow, hipMemcpyHostToDevice, M->stream));
    HIP_TRY(hipStreamSynchronize(M->stream));
    const double setup = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    TRY(solve_impl(M, M->d_b, M->d_x, max_iter, tolerance, niters, normr, times, print));
    HIP_TRY(hipMemcpy(x, M->d_x, sizeof(double) * M->nrow, hipMemcpyDeviceToHost));
    if (times) times[6] = setup;
    return 0;
}

int hpccg_hip_diag_spmv(hpccg_hip_matrix* M, int variant, int reps, double* avg_us)
{
    if (!M || !avg_us || reps < 1) return set_err(HPCCG_HIP_EINVAL, "bad argument");
    const int w = required_width(variant);
    if (!spmv_variant_ok(variant)) return set_err(HPCCG_HIP_EINVAL, "unknown variant %d", variant);
    if (const char* why = variant_unavailable(M, variant))
        return set_err(HPCCG_HIP_EINVAL, "variant %d needs %s", variant, why);
    if (w && !fixed_width_ok(M, variant))
        return set_err(HPCCG_HIP_EINVAL, "variant %d needs a uniform SELL image of that width", variant);
    HIP_TRY(hipSetDevice(M->device));
    TRY(ensure_hist(M, 2));
    const int keep = M->spmv_variant;
    M->spmv_variant = variant;  // make_args picks that variant's image
    CgArgs a = make_args(M, M->d_b, M->d_x, 2, 0.0);
    M->spmv_variant = keep;
    hipEvent_t e0, e1;
    HIP_TRY(hipEventCreate(&e0));
    HIP_TRY(hipEventCreate(&e1));
    launch_cg_spmv(a, variant, true, M->stream);  // warm
    HIP_TRY(hipEventRecord(e0, M->stream));
    for (int i = 0; i < reps; i++) launch_cg_spmv(a, variant, true, M->stream);
    HIP_TRY(hipEventRecord(e1, M->stream));
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventSynchronize(e1));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    *avg_us = 1e3 * ms / reps;
    return 0;
}

int hpccg_hip_get_option(const hpccg_hip_matrix* M, const char* key, long long* value)
{
    if (!M || !key || !value) return set_err(HPCCG_HIP_EINVAL, "NULL argument");
    if (!std::strcmp(key, "use_graph")) *value = M->use_graph;
    else if (!std::strcmp(key, "spmv_variant")) *value = M->spmv_variant;
    else if (!std::strcmp(key, "event_timing")) *value = M->event_timing;
    else if (!std::strcmp(key, "fuse_p")) *value = fuse_p_effective(M) ? 1 : 0;
    else if (!std::strcmp(key, "fold")) *value = fold_effective(M);
    else if (!std::strcmp(key, "x_defer")) *value = M->x_defer;
    else if (!std::strcmp(key, "x_ring")) *value = x_ring_effective(M);
    else if (!std::strcmp(key, "update_slices")) *value = M->update_slices;
    else if (!std::strcmp(key, "update_early")) *value = M->update_early;
    else if (!std::strcmp(key, "pap_in_update")) *value = pap_upd_effective(M) ? 1 : 0;
    else if (!std::strcmp(key, "rev_update")) *value = M->rev_update;
    else if (!std::strcmp(key, "resident_mb")) *value = resident_mb_effective(M);
    else if (!std::strcmp(key, "redund")) *value = redund_effective(M, 2) ? 1 : 0;  // off unless set
    else if (!std::strcmp(key, "halo_mode")) *value = M->nranks == 1 ? 0 : (M->general ? 2 : 1);
    else if (!std::strcmp(key, "graph_chunk")) *value = M->graph_iters;
    else if (!std::strcmp(key, "value_codes")) *value = variant_is_v(M->spmv_variant) ? 1 : 0;
    else if (!std::strcmp(key, "value_codes_available")) *value = M->has_v;
    else if (!std::strcmp(key, "overlap"))
        *value = (M->overlap && M->nranks > 1 && !M->general && M->halo_b_lo >= 0) ? 1 : 0;
    else if (!std::strcmp(key, "num_external")) *value = M->general ? M->ghost_hi : M->ghost_lo + M->ghost_hi;
    else if (!std::strcmp(key, "lds_doubles")) *value = M->has_lds ? M->lds_doubles : 0;
    else if (!std::strcmp(key, "windows")) *value = M->nwin;
    else return set_err(HPCCG_HIP_EINVAL, "unknown option '%s'", key);
    return 0;
}

int hpccg_hip_kernel_times(const hpccg_hip_matrix* M, double out[4])
{
    if (!M || !out) return set_err(HPCCG_HIP_EINVAL, "NULL argument");
    for (int i = 0; i < 4; i++) out[i] = M->ktimes[i];
    return 0;
}

int hpccg_hip_last_trace(const hpccg_hip_matrix* M, double* out, int cap)
{
    if (!M || !out) return set_err(HPCCG_HIP_EINVAL, "NULL argument");
    const int n = std::min<int>(cap, (int)M->trace.size());
    for (int i = 0; i < n; i++) out[i] = M->trace[i];
    return n;
}

int hpccg_hip_sparsemv(hpccg_hip_matrix* M, const double* x_dev, double* y_dev)
{
    if (!M || !x_dev || !y_dev) return set_err(HPCCG_HIP_EINVAL, "NULL argument");
    HIP_TRY(hipSetDevice(M->device));
    // stage x into p (the halo-carrying buffer), exchange, multiply
    if (M->in_group && M->nranks > 1)
        return set_err(HPCCG_HIP_EINVAL, "group member: the halo needs hpccg_hip_group_solve");
    HIP_TRY(hipMemcpyAsync(M->d_p, x_dev, sizeof(double) * M->nrow, hipMemcpyDeviceToDevice, M->stream));
    CgArgs a = make_args(M, nullptr, nullptr, 0, 0.0);
    if (M->general)
        TRY(enqueue_halo_gather(M, a, M->d_p, true));
    else
        TRY(enqueue_halo(M, M->d_p));
    launch_sparsemv(a, M->d_p - M->ghost_lo, y_dev, 0, M->stream);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(M->stream));
    return 0;
}

int hpccg_hip_ddot(int n, const double* x_dev, const double* y_dev, double* result)
{
    if (n < 0 || !result || (n > 0 && (!x_dev || !y_dev))) return set_err(HPCCG_HIP_EINVAL, "bad argument");
    const int nparts = ddot_nparts(n);
    TRY(scratch_for(nparts));
    launch_ddot(n, x_dev, y_dev, g_scratch.partial, nparts, g_scratch.out, g_scratch.s);
    HIP_TRY(hipGetLastError());
    if (g_comm.nranks > 1)
        NCCL_TRY(ncclAllReduce(g_scratch.out, g_scratch.out + 1, 1, ncclFloat64, ncclSum, g_comm.comm,
                               g_scratch.s));
    HIP_TRY(hipMemcpyAsync(result, g_scratch.out + (g_comm.nranks > 1 ? 1 : 0), sizeof(double),
                           hipMemcpyDeviceToHost, g_scratch.s));
    HIP_TRY(hipStreamSynchronize(g_scratch.s));
    return 0;
}

int hpccg_hip_waxpby(int n, double alpha, const double* x_dev, double beta, const double* y_dev,
                     double* w_dev)
{
    if (n < 0 || (n > 0 && (!x_dev || !y_dev || !w_dev))) return set_err(HPCCG_HIP_EINVAL, "bad argument");
    TRY(scratch_for(1));
    launch_waxpby(n, alpha, x_dev, beta, y_dev, w_dev, g_scratch.s);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(g_scratch.s));
    return 0;
}

int hpccg_hip_HPCCG(HPC_Sparse_Matrix* A, double* b, double* x, int max_iter, double tolerance,
                    int* niters, double* normr, double* times)
{
    hpccg_hip_matrix* M = nullptr;
    double setup = 0.0;
    {
        std::lock_guard<std::mutex> lk(g_dropin_mu);
        auto it = g_dropin_cache.find(A);
        if (it != g_dropin_cache.end()) {
            M = it->second;
        } else {
            const auto t0 = std::chrono::steady_clock::now();
            TRY(hpccg_hip_matrix_create(A, &M));
            setup = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            g_dropin_cache[A] = M;
        }
    }
    TRY(hpccg_hip_solve(M, b, x, max_iter, tolerance, niters, normr, times, 1));
    if (times) times[6] += setup;
    return 0;
}

long long hpccg_sell_build(int nrow, long long col_base, long long ncol_ext, const long long* row_ptr,
                           const int* cols, const double* vals, unsigned int* slice_base, int* sell_cols,
                           double* sell_vals)
{
    auto row_len = [row_ptr](int i) { return (int)(row_ptr[i + 1] - row_ptr[i]); };
    auto row_at = [row_ptr, cols, vals](int i, int j, long long* c, double* v) {
        *c = cols[row_ptr[i] + j];
        *v = vals ? vals[row_ptr[i] + j] : 0.0;
    };
    std::vector<unsigned int> tmp;
    if (!slice_base) {
        tmp.resize((nrow + kSliceRows - 1) / kSliceRows + 1);
        slice_base = tmp.data();
    }
    const long long var = sell_build_impl(nrow, SlabCols{col_base, ncol_ext}, row_len, row_at, slice_base, nullptr,
                                          nullptr, 0, nullptr);
    const long long uni = sell_build_impl(nrow, SlabCols{col_base, ncol_ext}, row_len, row_at, slice_base, nullptr,
                                          nullptr, 1, nullptr);
    const int uniform = (uni <= var + var / 25) ? 1 : 0;
    int bad = 0;
    const long long r = sell_build_impl(nrow, SlabCols{col_base, ncol_ext}, row_len, row_at, slice_base, sell_cols,
                                        sell_vals, uniform, &bad);
    return bad ? HPCCG_HIP_EPLAN : r;
}

int hpccg_gather_plan(int nranks, const int* info, int nrow, int start_row, const long long* row_ptr,
                      const int* cols, int cap, int* ext_global, int* num_external, int* nrecv, int* recv_rank,
                      int* recv_off, int* recv_cnt)
{
    if (nranks < 1 || !info || nrow < 0 || (nrow > 0 && (!row_ptr || !cols)) || !num_external || !nrecv)
        return set_err(HPCCG_HIP_EINVAL, "bad argument");
    GatherPlan g;
    gather_externals(
        nrow, start_row, info, nranks, [row_ptr](int i) { return (int)(row_ptr[i + 1] - row_ptr[i]); },
        [row_ptr, cols](int i, int j, long long* c, double* v) {
            *c = cols[row_ptr[i] + j];
            *v = 0.0;
        },
        g);
    *num_external = (int)g.ext_global.size();
    *nrecv = (int)g.recv_rank.size();
    if (ext_global && cap >= *num_external)
        for (int j = 0; j < *num_external; j++) ext_global[j] = (int)g.ext_global[j];
    if (recv_rank && recv_off && recv_cnt && cap >= *nrecv)
        for (int i = 0; i < *nrecv; i++) {
            recv_rank[i] = g.recv_rank[i];
            recv_off[i] = g.recv_off[i];
            recv_cnt[i] = g.recv_cnt[i];
        }
    return 0;
}

int hpccg_slab_plan(int nranks, int rank, const int* info, int sends[2])
{
    if (nranks < 1 || rank < 0 || rank >= nranks || !info || !sends)
        return set_err(HPCCG_HIP_EINVAL, "bad argument");
    const int r = rank, P = nranks;
    const int* me = info + 4 * r;
    const int nrow = me[0], ghost_lo = me[1], ghost_hi = me[2], start_row = me[3];
    // ghosts must come from the adjacent ranks only, contiguously
    if (ghost_lo > 0 && (r == 0 || ghost_lo > info[4 * (r - 1)]))
        return set_err(HPCCG_HIP_EPLAN, "rank %d: ghost_lo %d not owned by rank %d", r, ghost_lo, r - 1);
    if (ghost_hi > 0 && (r == P - 1 || ghost_hi > info[4 * (r + 1)]))
        return set_err(HPCCG_HIP_EPLAN, "rank %d: ghost_hi %d not owned by rank %d", r, ghost_hi, r + 1);
    if (r > 0 && info[4 * (r - 1) + 3] + info[4 * (r - 1)] != start_row)
        return set_err(HPCCG_HIP_EPLAN, "rank %d: row ranges are not contiguous", r);
    sends[0] = (r > 0) ? info[4 * (r - 1) + 2] : 0;      // rank-1's ghost_hi: our first rows
    sends[1] = (r < P - 1) ? info[4 * (r + 1) + 1] : 0;  // rank+1's ghost_lo: our last rows
    if (sends[0] > nrow || sends[1] > nrow)
        return set_err(HPCCG_HIP_EPLAN, "rank %d: neighbour needs more rows than owned", r);
    return 0;
}

int hpccg_halo_plan(int nrow, int start_row, int total_nrow, const long long* row_ptr, const int* cols,
                    int plan_out[4])
{
    long long mn = start_row, mx = (long long)start_row + nrow - 1;
    for (long long e = 0; e < (nrow > 0 ? row_ptr[nrow] : 0); e++) {
        mn = std::min<long long>(mn, cols[e]);
        mx = std::max<long long>(mx, cols[e]);
    }
    if (mn < 0 || mx >= total_nrow) return set_err(HPCCG_HIP_EPLAN, "column outside [0, total_nrow)");
    plan_out[0] = (int)(start_row - mn);
    plan_out[1] = (int)(mx - ((long long)start_row + nrow - 1));
    plan_out[2] = (int)mn;
    plan_out[3] = (int)mx;
    return 0;
}

}  // extern "C"
