// hpccg_solver.cpp -- host side of the MI355X HPCCG path: HPC_Sparse_Matrix ->
// SELL-512 / SELL-512-A conversion, device residency, the device-resident CG
// driver (HPCCG.cpp:312-402) replayed from hipGraphs, the z-slab halo exchange
// and scalar all-reduces over RCCL (exchange_externals.cpp:51-131,
// ddot.cpp:75-85), the in-process rank group, and the C ABI.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <map>
#include <mutex>
#include <string>
#include <system_error>
#include <thread>
#include <unordered_map>
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
    // host-bootstrapped (hpccg_hip_comm_init_host): no RCCL communicator; the
    // setup exchanges go through the caller's all-gather, and the iteration
    // must run without a collective (peer all-reduce + halo pull)
    hpccg_hip_allgather_fn ag = nullptr;
    void* ag_ctx = nullptr;
    // RCCL: the setup collectives' stream and staging buffer
    hipStream_t stream = nullptr;
    unsigned char* d_buf = nullptr;
    size_t buf_bytes = 0;
};
Comm g_comm;
bool comm_host() { return g_comm.ag != nullptr; }
bool comm_up() { return g_comm.comm != nullptr || g_comm.ag != nullptr; }

void comm_reset()
{
    if (g_comm.comm) ncclCommDestroy(g_comm.comm);
    if (g_comm.d_buf) (void)hipFree(g_comm.d_buf);
    if (g_comm.stream) (void)hipStreamDestroy(g_comm.stream);
    g_comm = Comm();
}

// All-gather of `bytes` host bytes per rank into all[nranks * bytes] (rank
// order): RCCL staged through device memory, or the host bootstrap's
// callback. The setup-time exchanges of make_local_matrix.cpp:185-201 /
// :286-587 and the self-tests' verdicts go through here.
int comm_allgather(const void* mine, void* all, size_t bytes)
{
    if (g_comm.nranks == 1 || !comm_up()) {
        std::memcpy(all, mine, bytes);
        return 0;
    }
    if (g_comm.ag) {
        if (g_comm.ag(mine, all, (unsigned long long)bytes, g_comm.ag_ctx) != 0)
            return set_err(HPCCG_HIP_EINVAL, "the host all-gather callback failed (%zu B per rank)", bytes);
        return 0;
    }
    const size_t need = bytes * (size_t)(g_comm.nranks + 1);
    if (!g_comm.stream) HIP_TRY(hipStreamCreateWithFlags(&g_comm.stream, hipStreamNonBlocking));
    if (need > g_comm.buf_bytes) {
        if (g_comm.d_buf) (void)hipFree(g_comm.d_buf);
        g_comm.d_buf = nullptr;
        g_comm.buf_bytes = 0;
        HIP_TRY(hipMalloc(&g_comm.d_buf, need));
        g_comm.buf_bytes = need;
    }
    unsigned char* d = g_comm.d_buf;
    HIP_TRY(hipMemcpyAsync(d + bytes * g_comm.nranks, mine, bytes, hipMemcpyHostToDevice, g_comm.stream));
    NCCL_TRY(ncclAllGather(d + bytes * g_comm.nranks, d, bytes, ncclUint8, g_comm.comm, g_comm.stream));
    HIP_TRY(hipStreamSynchronize(g_comm.stream));
    HIP_TRY(hipMemcpy(all, d, bytes * g_comm.nranks, hipMemcpyDeviceToHost));
    return 0;
}

// Minimum over the ranks of one int (the self-tests' verdicts).
int comm_min(int v, int* out)
{
    std::vector<int> all(std::max(1, g_comm.nranks));
    TRY(comm_allgather(&v, all.data(), sizeof v));
    *out = *std::min_element(all.begin(), all.end());
    return 0;
}

// The job's in-kernel transport verdicts from every rank's own self-test
// results (collective; hpccg_hip_transport_verdict): local = {peer all-reduce,
// halo pull, production protocol} as this rank saw them. The peer all-reduce
// and the pull each stay on only where every rank passed; the protocol test
// counts only where both did, and a protocol failure on any rank turns both
// off on every rank (RCCL then carries the scalars and r's planes). Every
// rank computes the same three values from the same gathered table.
int transport_verdict(const int local[3], int out[3])
{
    TRY(comm_min(local[0] ? 1 : 0, &out[0]));
    TRY(comm_min(local[1] ? 1 : 0, &out[1]));
    TRY(comm_min((out[0] && out[1] && local[2]) ? 1 : 0, &out[2]));
    if (out[0] && out[1] && !out[2]) out[0] = out[1] = 0;
    return 0;
}

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

// In-process rank group (hpccg_hip_group_*): while a group member is being
// created on this thread, rank/size come from here instead of the RCCL
// communicator, and the halo plan is made by hpccg_hip_group_* afterwards.
struct GroupCtx {
    int active = 0, nranks = 1, rank = 0;
    const int* info = nullptr;        // every member's {nrow, ghost_lo, ghost_hi, start_row}, or null
    const GatherPlan* plan = nullptr; // this member's gather plan (gather mode), or null
};
thread_local GroupCtx g_group_ctx;
int g_halo_mode = 0;  // 0 auto (slab when it serves every rank), 1 slab only, 2 gather
int g_keep_sell = 0;  // keep the SELL-512 image beside SELL-512-A (kernel A/B, diagnostics)
// placement probe at creation: -1 auto (images over kPlaceMinBytes), 0 off, n
// candidates. Off by default since round 4: the probe's gain is
// box-dependent and it is asked for explicitly (bench.py --placement).
int g_place_tries = 0;
constexpr int kPlaceAuto = 6;        // candidates of the automatic probe
constexpr int kPlacePhases = 4;      // values, p ring, r, Ap
constexpr double kPlaceMinBytes = 512e6;  // auto: only images that stream from HBM
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
    long long total = 0;
    int wmax = 0;
    std::vector<int> w(nslices, 0);
    for (int s = 0; s < nslices; s++) {
        int m = 0;
        for (int i = s * kSliceRows; i < std::min(nrow, (s + 1) * kSliceRows); i++) m = std::max(m, row_len(i));
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
    int send_lo = 0;  // rows to send to rank-1 (its ghost_hi)
    int send_hi = 0;  // rows to send to rank+1 (its ghost_lo)
    // gather plan (partitions the slab plan cannot serve): externals after the
    // local rows (ghost_lo = 0, ghost_hi = number of externals)
    int general = 0;
    std::vector<int> recv_rank, recv_off, recv_cnt, send_rank, send_off, send_cnt;
    int nsend = 0;
    int* d_send_idx = nullptr;
    double* d_send_buf = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t ev_flush = nullptr;  // flush_stream's marker (default flags: system-scope release)
    hipEvent_t ev_mid = nullptr;    // wait_matrix: blocking-sync marker before a solve's last graph chunk
    int mid_pending = 0;            // ev_mid was recorded for the solve in flight
    long long nnz = 0, nslots = 0;
    int nslices = 0, grid = 0, width = 0, uniform = 0;
    int kernel = 0;       // SpMV kernel in use (SpmvKernel)
    int kernel_opt = -1;  // option spmv_kernel (-1 auto)
    int use_graph = 1;
    int fuse_p = -1;      // -1 auto: on where the kernel forms p_k itself
    int fuse_update = -1; // the update as trailing blocks of the SpMV launch; -1 auto (fuse_update_effective)
    int resident_update = -1;     // the resident pair kernels (k_spmv_ar, k_cg_persist; resident_of, persist_ok)
    int resident_retries = 0;     // solves re-run after a resident launch's wait expired (resident_retry)
    int resident_failed = 0;      // a resident launch's wait expired (GPU shared): the unit + update launch from then on
    int resident_used = 0;        // the last solve ran k_spmv_ar
    int last_dev_err = 0;         // the device error code the last failed solve recorded (DevError)
    int last_dev_err_all = 0;     // ... its maximum over a job's ranks (all-reduced: the same on every rank)
    size_t npartial = 0;  // dot slots (the last one: the fused update's p.Ap total)
    int a2_ring = kA2RingDefault;  // pair kernel: LDS-DMA value ring depth per wave (0: register loads; uniform widths 27 and 7)
    int fold = -1;        // -1 auto: 1 (both dots completed in their producers); 0 k_finalize
    int force_comm = 0;   // diagnostics: 1 scalars through the RCCL communicator even at one rank;
                          // 2 also the multi-rank iteration with a self send/recv as its halo
    // SELL-512 (the general kernel; freed once SELL-512-A exists unless kept)
    int has_sell = 0;
    unsigned int* d_slice_base = nullptr;
    int* d_cols = nullptr;
    double* d_vals = nullptr;
    // SELL-512-A
    int has_a = 0, a_width = 0;
    int a_reject = 0;  // SELL-512-A not built (diagnostics): 2 its flag read late, 3 rejected although
                       // the device's columns fit (a kernel fault), 4 rejected and they do not
    long long a_slots = 0;
    double* d_aval = nullptr;
    int* d_aoff = nullptr;
    unsigned int* d_abase = nullptr;
    int has_pairs = 0, alds2_doubles = 0;
    int *d_alds2 = nullptr, *d_awin2 = nullptr, *d_awn2 = nullptr, *d_adiag2 = nullptr;
    unsigned char* d_atri = nullptr;  // direct kernel: slices in the width's triple plan
    // workspace (padded to a multiple of kSliceRows rows)
    size_t npad = 0;
    double* d_pbuf = nullptr;  // ring_alloc buffers of [guard | ghost_lo_pad | npad | ghost_hi_pad | guard]
    int ring_alloc = 0;
    double* d_p = nullptr;     // local rows of ring buffer 0
    long long pstride = 0;
    double* d_ahist = nullptr;
    double* d_pslots = nullptr;   // persistent CG (persist_of): per-iteration dot slots
    long long pslots_cap = 0;     // doubles
    int x_defer = 2;      // deferred x: beside the SpMV where the kernel carries it, else batched (x_defer_effective)
    int x_ring = -1;
    double *d_r = nullptr, *d_Ap = nullptr, *d_x = nullptr, *d_b = nullptr;
    double* d_rbuf = nullptr;
    double* d_partial = nullptr;  // inside the d_kst block (not freed on its own)
    double* d_scal = nullptr;  // g[2], loc[2], spare
    double** d_gtab = nullptr;  // group fold (last member): the members' loc, then their g
    std::vector<double*> h_gtab;
    PullSeg* d_pseg = nullptr;  // group fold (member 0): every member's pull, done by its update
    std::vector<PullSeg> h_pseg;
    int gfold_used = 0;         // the last group solve summed its dots in the last member's kernels
    int* d_kst = nullptr;      // [0, kErrBase) iteration state, then the device error record (kErrWords)
    long long spin_us = kSpinTicksDefault / 100;  // bound of every in-kernel wait (option spin_budget_us)
    int dbg_withhold = 0;      // debug: slice + 1 whose p.Ap partial is withheld (guard test)
    int dbg_resident_stall = 0;  // debug: the resident launch's p.Ap wait expires (the retry test)
    unsigned long long* d_tl = nullptr;  // diagnostics (dbg_timeline): per unit kTlWords block stamps
    int tl_units = 0;
    int solve_dirty = 0;       // a solve started and did not finish cleanly: reset the dot slots first
    // peer-memory all-reduce of the CG scalars (option peer_allreduce)
    int peer_ar = -1;                  // option peer_allreduce: -1 auto (peer_ar_of), 0 off, 1 on
    int peer_auto_ok = 0;              // auto: the creation-time self-test passed on every rank
    // r-halo by pull (option halo_pull: -1 auto, 0 the RCCL / peer-copy planes, 1 k_pull, 2 in-launch)
    int halo_pull = -1;
    int pull_auto_ok = 0;              // RCCL job: the creation-time pull test passed on every rank
    int proto_auto_ok = 0;             // ... and the production-protocol test (protocol_autotest)
    int persist_auto_ok = 0;           // ... and its persistent-launch run (every rank's blocks co-resident, same bits)
    std::string selftest_note;         // why a creation-time self-test failed on this rank (diagnostics)
    double* d_pull_lo = nullptr;       // rank - 1's r (its local row 0), mapped here (RCCL job)
    double* d_pull_hi = nullptr;       // rank + 1's r
    double* d_pullx_lo = nullptr;      // rank - 1's x workspace (d_x, its local row 0): the prologue's p = x halo
    double* d_pullx_hi = nullptr;      // rank + 1's x
    int pull_lo_n = 0;                 // rank - 1's row count
    std::vector<void*> ipc_r_opened;   // the neighbours' r buffers mapped from other processes
    double* d_mbox = nullptr;          // this rank's mailbox (kMboxSlots, uncached / fine-grained)
    double** d_peers = nullptr;        // device table: every rank's mailbox, as this rank addresses it
    int peers_for = 0;                 // ranks the table was built for (0: none)
    std::vector<void*> ipc_opened;     // peers' mailboxes mapped from other processes
    double* d_hist = nullptr;
    unsigned long long* d_stamps = nullptr;
    double* d_emul = nullptr;  // force_comm 2: self-exchange receive buffer (two planes)
    int emul_plane = 0;        // force_comm 2: rows per plane (the largest column offset; 0 unknown)
    int hist_cap = 0;
    long long stamp_cap = 0;
    // pinned readback of a solve's results (state, scalars, r.r history, timer
    // stamps): one batch of async copies and one wait per solve
    char* h_rb = nullptr;
    size_t h_rb_bytes = 0;
    std::vector<void*> graveyard;  // diagnostics: buffers moved by hpccg_hip_diag_realloc, held until destroy
    struct Vmm {
        void* va;  // the mapping (aligned inside the reservation)
        size_t bytes;
        hipMemGenericAllocationHandle_t h;
        void* res;  // the reservation
        size_t res_bytes;
    };
    std::vector<Vmm> vmm;  // diagnostics: hpccg_hip_diag_realloc's VMM mappings (unmapped at destroy)
    std::vector<double> place_us;  // placement probe: SpMV us per candidate (0 = the creation placement)
    int place_pick = 0;            // the candidate kept
    double *d_gen_b = nullptr, *d_gen_x0 = nullptr, *d_gen_xexact = nullptr;
    long long bytes = 0;       // device bytes held
    // hipGraph of graph_chunk iterations (kernel arguments are baked in)
    hipGraphExec_t graph_exec = nullptr;
    int graph_chunk = 0;
    int graph_iters = 32;  // 100^3 same-process A/B: 20 442 vs 20 198 it/s at 8 (200^3 +0.15 %); 499 (one graph per solve) 20 033
    std::vector<CgArgs> graph_args;
    int graph_kernel = -1;
    int graph_failed = 0;      // capture refused here (e.g. RCCL inside a graph): eager from then on
    int graph_used = 0;        // the last solve replayed graphs
    // hipEvent timing (event_timing option)
    int event_timing = 0;
    std::vector<hipEvent_t> ev;
    double ktimes[4] = {0, 0, 0, 0};
    std::vector<double> kiter;  // event_timing: per iteration {SpMV ms, update ms}
    std::vector<double> trace;
    int last_niters = 0;
};

namespace {

// Canary debug mode (HPCCG_CANARY=1 in the environment when the library first
// allocates): every matrix buffer gets kCanaryBytes of a NaN
// pattern no kernel stores (0x7FF5C0DE in every 32-bit word) before and after
// it, registered here, and every canary of the process is checked after each
// solve (and by hpccg_hip_diag_canary_check). A store that runs past a buffer
// trips the canary next to it and names the buffer and the offset. Off: one
// plain hipMalloc per buffer, nothing registered.
constexpr size_t kCanaryBytes = size_t(64) << 10;
constexpr unsigned kCanaryWord = 0x7FF5C0DEu;
struct CanaryRec {
    char* base;    // the allocation: [canary | user bytes, rounded up to 256 B | canary]
    size_t bytes;  // user bytes rounded up to 256 (the tail canary's offset: dword-aligned for its fill)
};
std::mutex g_canary_mu;
std::unordered_map<void*, CanaryRec> g_canary;  // user pointer -> allocation
bool canary_on()
{
    static const bool on = [] {
        const char* e = std::getenv("HPCCG_CANARY");
        return e && e[0] == '1';
    }();
    return on;
}

// Large device buffers. Never physically contiguous allocations
// (hipDeviceMallocContiguous): on this stack they corrupted OTHER live
// buffers and later allocations -- wrong b / x0 seen by the next solve, a
// matrix image whose uploaded columns the A pass rejected -- even while the
// contiguous buffers were held and never freed (DESIGN.md 4,
// tools/diag_carry.py, profiles/r04_carry/). The product library has no path
// to them at all; the diagnostics variant (-DHPCCG_DIAG_CONTIG) keeps one.
hipError_t big_malloc(void** p, size_t b, unsigned flags = hipDeviceMallocDefault)
{
    if (!canary_on()) return flags == hipDeviceMallocDefault ? hipMalloc(p, b) : hipExtMallocWithFlags(p, b, flags);
    void* base = nullptr;
    b = (b + 255) & ~size_t(255);  // (a byte-sized buffer would leave the tail canary unaligned)
    const size_t tot = b + 2 * kCanaryBytes;
    hipError_t e = flags == hipDeviceMallocDefault ? hipMalloc(&base, tot) : hipExtMallocWithFlags(&base, tot, flags);
    if (e != hipSuccess) return e;
    // both canaries written and landed before the buffer is handed out
    const size_t words = kCanaryBytes / 4;
    char* c = static_cast<char*>(base);
    if ((e = hipMemsetD32(reinterpret_cast<hipDeviceptr_t>(c), (int)kCanaryWord, words)) != hipSuccess ||
        (e = hipMemsetD32(reinterpret_cast<hipDeviceptr_t>(c + kCanaryBytes + b), (int)kCanaryWord, words)) !=
            hipSuccess ||
        (e = hipDeviceSynchronize()) != hipSuccess) {
        (void)hipFree(base);
        return e;
    }
    *p = c + kCanaryBytes;
    std::lock_guard<std::mutex> lk(g_canary_mu);
    g_canary[*p] = CanaryRec{c, b};
    return hipSuccess;
}

// Frees what big_malloc handed out (any other device pointer: plain hipFree).
void big_free(void* p)
{
    if (!p) return;
    if (canary_on()) {
        std::lock_guard<std::mutex> lk(g_canary_mu);
        const auto it = g_canary.find(p);
        if (it != g_canary.end()) {
            p = it->second.base;
            g_canary.erase(it);
        }
    }
    (void)hipFree(p);
}

// Every registered canary checked (device-wide sync first). Returns the number
// of tripped canaries; the first few are described in *report.
int canary_check(std::string* report)
{
    if (!canary_on()) return 0;
    if (hipDeviceSynchronize() != hipSuccess) (void)hipGetLastError();
    std::lock_guard<std::mutex> lk(g_canary_mu);
    std::vector<unsigned> buf(kCanaryBytes / 4);
    int bad = 0;
    for (const auto& kv : g_canary) {
        const CanaryRec& c = kv.second;
        for (int side = 0; side < 2; side++) {
            const char* src = side == 0 ? c.base : c.base + kCanaryBytes + c.bytes;
            if (hipMemcpy(buf.data(), src, kCanaryBytes, hipMemcpyDeviceToHost) != hipSuccess) {
                (void)hipGetLastError();
                continue;
            }
            size_t first = buf.size(), last = 0, n = 0;
            for (size_t i = 0; i < buf.size(); i++)
                if (buf[i] != kCanaryWord) {
                    first = std::min(first, i);
                    last = i;
                    n++;
                }
            if (!n) continue;
            bad++;
            if (report && bad <= 8) {
                char line[256];
                // head canary: offsets before the buffer (negative); tail: past its end
                const long long b0 = side == 0 ? -(long long)kCanaryBytes + 4 * (long long)first
                                               : (long long)c.bytes + 4 * (long long)first;
                const long long b1 = side == 0 ? -(long long)kCanaryBytes + 4 * (long long)last
                                               : (long long)c.bytes + 4 * (long long)last;
                std::snprintf(line, sizeof line,
                              "canary %s of buffer %p (%zu B): %zu words changed, bytes [%lld, %lld] relative to "
                              "the buffer, first word 0x%08x\n",
                              side == 0 ? "head" : "tail", kv.first, c.bytes, n, b0, b1 + 3, buf[first]);
                *report += line;
            }
        }
    }
    return bad;
}

// Host-to-device copy ordered on stream s (no matrix: the kernel-level API's
// scratch); waits, so the source may go away.
int h2d_stream(hipStream_t s, void* dst, const void* src, size_t bytes)
{
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
    HIP_TRY(hipStreamSynchronize(s));
    return 0;
}

// Device-to-host copy into pageable memory after the work queued on stream s:
// a synchronous copy once s has drained, so the data is in dst on return
// (an async copy into pageable memory gives no such guarantee at the stream
// sync).
int d2h(hipStream_t s, void* dst, const void* src, size_t bytes)
{
    HIP_TRY(hipStreamSynchronize(s));
    HIP_TRY(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return 0;
}

template <class T>
int dev_alloc(hpccg_hip_matrix* M, T** p, size_t count, bool zero = false)
{
    const size_t b = sizeof(T) * std::max<size_t>(1, count);
    HIP_TRY(big_malloc(reinterpret_cast<void**>(p), b));
    if (zero) HIP_TRY(hipMemsetAsync(*p, 0, b, M->stream));  // ordered before M's kernels and copies
    M->bytes += (long long)b;
    return 0;
}

// A marker with a system-scope release on M's stream, waited for: what the
// kernels left dirty in the L2s is in memory before a buffer is freed (and
// reused by the next allocation) or read by the host's copy engine. Needed
// after event-timed work: the timing events are created without that release
// (ensure_events), and without it a line written back later lands in
// whatever buffer owns the memory by then.
int flush_stream(hpccg_hip_matrix* M)
{
    if (!M->stream) return 0;
    if (!M->ev_flush) HIP_TRY(hipEventCreateWithFlags(&M->ev_flush, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(M->ev_flush, M->stream));
    HIP_TRY(hipEventSynchronize(M->ev_flush));
    return 0;
}

// Host-to-device copy into a buffer of M, ordered on M's stream where the
// kernels (or RCCL calls) that read it run (a plain hipMemcpy is ordered on
// the null stream, which the library's non-blocking streams do not wait
// for). Flushed on both sides: a zero fill of the same memory still dirty in
// an L2 must not be written back over the copied data later, and the copy
// must be in memory for every XCD. Waits, so the source may go away.
int h2d(hpccg_hip_matrix* M, void* dst, const void* src, size_t bytes)
{
    TRY(flush_stream(M));
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, M->stream));
    return flush_stream(M);
}

template <class T>
void dev_free(hpccg_hip_matrix* M, T** p, size_t count)
{
    if (*p) {
        (void)flush_stream(M);
        big_free(*p);
        M->bytes -= (long long)(sizeof(T) * std::max<size_t>(1, count));
    }
    *p = nullptr;
}

int free_matrix(hpccg_hip_matrix* M)
{
    if (!M) return 0;
    // Nothing may write into this matrix's memory once it is freed and reused:
    // its own streams, and in a group the other members' kernels, which store
    // into its mailbox (peer all-reduce) or read its planes -- every device of
    // a group is drained, not just this one
    if (M->in_group) {
        int nd = 0;
        if (hipGetDeviceCount(&nd) == hipSuccess)
            for (int d = 0; d < nd; d++)
                if (hipSetDevice(d) == hipSuccess) (void)hipDeviceSynchronize();
    }
    (void)hipSetDevice(M->device);
    (void)hipDeviceSynchronize();
    (void)flush_stream(M);
    if (M->graph_exec) (void)hipGraphExecDestroy(M->graph_exec);
    for (const auto& v : M->vmm)  // diagnostics' VMM mappings: released below, not hipFree'd
        for (double** q : {&M->d_aval, &M->d_pbuf, &M->d_rbuf, &M->d_Ap, &M->d_x})
            if (*q == v.va) *q = nullptr;
    void* ptrs[] = {M->d_slice_base, M->d_cols,   M->d_vals,      M->d_aval,    M->d_aoff,     M->d_abase,
                    M->d_alds2,      M->d_awin2,  M->d_awn2,      M->d_adiag2,     M->d_atri,      M->d_pbuf,    M->d_ahist,    M->d_pslots,  M->d_rbuf,
                    M->d_Ap,         M->d_x,      M->d_b,         M->d_scal,
                    M->d_kst,        M->d_hist,   M->d_stamps,    M->d_gen_b,   M->d_gen_x0,   M->d_gen_xexact,
                    M->d_send_idx,   M->d_send_buf,  M->d_emul,  M->d_tl};
    for (void* p : ptrs) big_free(p);
    for (void* p : M->ipc_opened) (void)hipIpcCloseMemHandle(p);
    for (void* p : M->ipc_r_opened) (void)hipIpcCloseMemHandle(p);
    if (M->h_rb) (void)hipHostFree(M->h_rb);
    for (void* p : M->graveyard) big_free(p);
    for (const auto& v : M->vmm) {
        (void)hipMemUnmap(v.va, v.bytes);
        (void)hipMemRelease(v.h);
        (void)hipMemAddressFree(v.res, v.res_bytes);
    }
    for (void* p : {(void*)M->d_mbox, (void*)M->d_gtab, (void*)M->d_pseg, (void*)M->d_peers}) big_free(p);
    for (hipEvent_t e : M->ev) (void)hipEventDestroy(e);
    if (M->ev_flush) (void)hipEventDestroy(M->ev_flush);
    if (M->ev_mid) (void)hipEventDestroy(M->ev_mid);
    if (M->stream) (void)hipStreamDestroy(M->stream);
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

int make_streams(hpccg_hip_matrix* M)
{
    HIP_TRY(hipStreamCreateWithFlags(&M->stream, hipStreamNonBlocking));
    return 0;
}

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
        if (info[4 * mid + 3] <= c)
            lo = mid;
        else
            hi = mid - 1;
    }
    return lo;
}

template <class RowLen, class RowAt>
void gather_externals(int nrow, long long start, const int* info, int P, RowLen row_len, RowAt row_at, GatherPlan& g)
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
    TRY(h2d(M, d, mine.data(), sizeof(int) * P));
    NCCL_TRY(ncclAllGather(d, d + P, P, ncclInt32, g_comm.comm, M->stream));
    std::vector<int> cnt((size_t)P * P);
    TRY(d2h(M->stream, cnt.data(), d + P, sizeof(int) * P * P));
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
    if (nout) TRY(h2d(M, dout, flat.data(), sizeof(int) * nout));
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
    TRY(d2h(M->stream, got.data(), din, sizeof(int) * std::max(1LL, nin)));
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
    TRY(dev_alloc(M, &M->d_send_idx, M->nsend));
    TRY(dev_alloc(M, &M->d_send_buf, M->nsend));
    if (M->nsend)
        TRY(h2d(M, M->d_send_idx, g.send_idx.data(), sizeof(int) * M->nsend));
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
    int mine[4] = {M->nrow, M->ghost_lo, M->ghost_hi, M->start_row};
    std::vector<int> all(4 * g_comm.nranks);
    TRY(comm_allgather(mine, all.data(), sizeof mine));
    const int md = choose_halo_mode(all.data(), g_comm.nranks);
    if (md < 0) return set_err(HPCCG_HIP_EPLAN, "the z-slab halo plan cannot serve this partition");
    if (all_out) *all_out = all;
    if (md == 2) {
        if (!mode) return set_err(HPCCG_HIP_EPLAN, "gather halo plan needs the matrix rows");
        // (every rank decides this from the same all-gathered rows)
        if (comm_host())
            return set_err(HPCCG_HIP_EPLAN, "the gather halo plan moves p through RCCL; a host-bootstrapped "
                                            "communicator serves z-slab partitions only");
        *mode = 2;
        return 0;
    }
    int sends[2];
    TRY(hpccg_slab_plan(g_comm.nranks, g_comm.rank, all.data(), sends));
    M->send_lo = sends[0];
    M->send_hi = sends[1];
    return 0;
}

// ---------------------------------------------------------------------------
// SELL-512-A and its pair windows
// ---------------------------------------------------------------------------
// Windows of the pair of slices [2P, 2P + ns) over the union of their
// ascending offsets, cut where neighbours are more than a slice apart: window
// [o_a, o_b] stages rows pair_row + o_a .. pair_row + ns*512 - 1 + o_b, so
// every row of the pair finds every offset of the range in it, holes
// included. lds[s][j] = LDS position of slot j minus the row's index in the
// pair; padding slots (offset 0, value 0.0) read slot 0's. Returns the
// doubles staged, or -1 when it needs more than kAWin windows.
int pair_windows(const std::vector<int>& off, const std::vector<int>& cnt, int s0, int ns, int* win, int* nwin,
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
    if (u.empty()) {  // empty rows only: one window of the pair's own rows
        win[0] = 0, win[1] = rows, win[2] = 0;
        wlo.push_back(0), wbase.push_back(0);
        nw = 1, base = rows;
    }
    for (size_t j = 0; j < u.size();) {
        size_t e = j;
        while (e + 1 < u.size() && u[e + 1] - u[e] <= kSliceRows) e++;
        if (nw == kAWin) return -1;
        // even first row and length: the kernel stages row pairs with 16-B
        // loads and stores (one extra row at most at either end)
        const int lo = u[j] - (u[j] & 1);
        const int len = (rows + u[e] - lo + 1) & ~1;
        win[3 * nw] = lo;
        win[3 * nw + 1] = len;
        win[3 * nw + 2] = base;
        wlo.push_back(lo);
        wbase.push_back(base);
        base += len;
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
        if (cnt[s] == 0) l[0] = 0;
        for (int j = std::max(cnt[s], 1); j < kAMax; j++) l[j] = l[0];
    }
    *nwin = nw;
    return base;
}

// SELL-512-A from the SELL-512 image on the device (k_a_offsets, k_a_fill),
// the pair windows on the host from the per-slice offsets. No A image when a slice has more than kAMax offsets
// or a row is not in ascending column order (the general kernel stays).
int build_a_image(hpccg_hip_matrix* M)
{
    const int S = M->nslices;
    if (!M->has_sell || S < 1) return 0;
    int* d_acount = nullptr;
    int* d_flags = nullptr;
    HIP_TRY(hipMalloc(&d_acount, sizeof(int) * S));
    HIP_TRY(hipMalloc(&d_flags, sizeof(int) * 2));
    struct Tmp {
        int* a;
        int* b;
        ~Tmp()
        {
            (void)hipFree(a);
            (void)hipFree(b);
        }
    } tmp{d_acount, d_flags};
    TRY(dev_alloc(M, &M->d_aoff, (size_t)S * kAMax));
    const int init[2] = {1, 0};
    HIP_TRY(hipMemcpyAsync(d_flags, init, sizeof init, hipMemcpyHostToDevice, M->stream));
    launch_a_offsets(M->d_slice_base, S, M->d_cols, M->ghost_lo, M->d_aoff, d_acount, d_flags, d_flags + 1,
                     M->stream);
    HIP_TRY(hipGetLastError());
    int fl[2] = {0, 0};
    std::vector<int> cnt(S);
    TRY(d2h(M->stream, fl, d_flags, sizeof fl));
    TRY(d2h(M->stream, cnt.data(), d_acount, sizeof(int) * S));
    HIP_TRY(hipStreamSynchronize(M->stream));
    if (!fl[0]) {
        // (diagnostics: a second read after a device-wide sync tells a late
        // readback from a real rejection)
        int again[2] = {0, 0};
        HIP_TRY(hipDeviceSynchronize());
        HIP_TRY(hipMemcpy(again, d_flags, sizeof again, hipMemcpyDeviceToHost));
        M->a_reject = again[0] ? 2 : 1;
        if (!again[0]) {  // the device's columns re-checked on the host: 3 they fit (a kernel fault), 4 they do not
            std::vector<unsigned int> sbh(S + 1);
            HIP_TRY(hipMemcpy(sbh.data(), M->d_slice_base, sizeof(unsigned int) * (S + 1), hipMemcpyDeviceToHost));
            std::vector<int> ch((size_t)sbh[S] * kSliceRows);
            HIP_TRY(hipMemcpy(ch.data(), M->d_cols, sizeof(int) * ch.size(), hipMemcpyDeviceToHost));
            bool fits = true;
            for (int sl = 0; sl < S && fits; sl++) {
                std::vector<int> offs;
                for (int lane = 0; lane < kSliceRows; lane++) {
                    int prev = INT_MIN;
                    for (unsigned j = sbh[sl]; j < sbh[sl + 1]; j++) {
                        const int c = ch[(size_t)j * kSliceRows + lane];
                        if (c < 0) continue;
                        const int o = c - M->ghost_lo - (sl * kSliceRows + lane);
                        if (o <= prev) fits = false;
                        prev = o;
                        if (std::find(offs.begin(), offs.end(), o) == offs.end()) offs.push_back(o);
                    }
                }
                if ((int)offs.size() > kAMax) fits = false;
            }
            M->a_reject = fits ? 3 : 4;
        }
        dev_free(M, &M->d_aoff, (size_t)S * kAMax);
        return 0;
    }
    std::vector<unsigned int> ab(S + 1, 0);
    int wmax = 0;
    for (int i = 0; i < S; i++) {
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
    M->a_slots = (long long)ab[S] * kSliceRows;
    TRY(dev_alloc(M, &M->d_abase, ab.size()));
    TRY(h2d(M, M->d_abase, ab.data(), sizeof(unsigned int) * ab.size()));
    TRY(dev_alloc(M, &M->d_aval, (size_t)M->a_slots));
    HIP_TRY(hipMemsetAsync(M->d_aval, 0, sizeof(double) * std::max<long long>(1, M->a_slots), M->stream));
    launch_a_fill(M->d_slice_base, S, M->d_cols, M->d_vals, M->ghost_lo, M->d_aoff, d_acount, M->d_abase,
                  M->d_aval, M->stream);
    HIP_TRY(hipGetLastError());
    std::vector<int> off((size_t)S * kAMax);
    TRY(d2h(M->stream, off.data(), M->d_aoff, sizeof(int) * off.size()));
    HIP_TRY(hipStreamSynchronize(M->stream));
    M->has_a = 1;
    for (int sl = 0; sl < S; sl++)
        if (cnt[sl] > 0) M->emul_plane = std::max(M->emul_plane, off[(size_t)sl * kAMax + cnt[sl] - 1]);
    // 7-pt triple plan of the direct kernel (tri_first / tri_size in hpccg_kernels.hip):
    // the slice's offsets, grouped greedily into runs of three consecutive
    // offsets, form exactly the width's group sequence
    if (M->a_width == 7) {
        std::vector<unsigned char> tri(S, 0);
        for (int s = 0; s < S; s++) {
            if (cnt[s] != M->a_width) continue;
            const int* o = &off[(size_t)s * kAMax];
            std::vector<int> sizes;
            for (int j = 0; j < cnt[s];) {
                const bool t3 = j + 2 < cnt[s] && o[j + 1] == o[j] + 1 && o[j + 2] == o[j] + 2;
                sizes.push_back(t3 ? 3 : 1);
                j += t3 ? 3 : 1;
            }
            const std::vector<int> want{1, 1, 3, 1, 1};
            tri[s] = sizes == want ? 1 : 0;
        }
        TRY(dev_alloc(M, &M->d_atri, tri.size()));
        TRY(h2d(M, M->d_atri, tri.data(), tri.size()));
    }
    // pair windows
    const int NP = (S + 1) / 2;
    std::vector<int> lds((size_t)S * kAMax, 0), win((size_t)NP * kAWin * 3, 0), wn(NP, 0);
    int maxd = 0;
    for (int P = 0; P < NP; P++) {
        const int d = pair_windows(off, cnt, 2 * P, std::min(2, S - 2 * P), &win[(size_t)P * kAWin * 3], &wn[P], lds);
        if (d < 0 || d > kALdsMax2) return 0;  // direct kernel only
        maxd = std::max(maxd, d);
    }
    std::vector<int> diag(S, -1);  // LDS position of offset 0 (the rows' own p_k)
    for (int s = 0; s < S; s++)
        for (int j = 0; j < cnt[s]; j++)
            if (off[(size_t)s * kAMax + j] == 0) diag[s] = lds[(size_t)s * kAMax + j];
    TRY(dev_alloc(M, &M->d_adiag2, diag.size()));
    TRY(h2d(M, M->d_adiag2, diag.data(), sizeof(int) * diag.size()));
    TRY(dev_alloc(M, &M->d_alds2, lds.size()));
    TRY(dev_alloc(M, &M->d_awin2, win.size()));
    TRY(dev_alloc(M, &M->d_awn2, wn.size()));
    TRY(h2d(M, M->d_alds2, lds.data(), sizeof(int) * lds.size()));
    TRY(h2d(M, M->d_awin2, win.data(), sizeof(int) * win.size()));
    TRY(h2d(M, M->d_awn2, wn.data(), sizeof(int) * wn.size()));
    M->alds2_doubles = std::max(1, maxd);
    M->has_pairs = 1;
    return 0;
}

void drop_sell(hpccg_hip_matrix* M)
{
    dev_free(M, &M->d_cols, (size_t)M->nslots);
    dev_free(M, &M->d_vals, (size_t)M->nslots);
    dev_free(M, &M->d_slice_base, (size_t)M->nslices + 1);
    M->has_sell = 0;
}

// SELL-512-A images beyond the 256 MB Infinity Cache stream non-temporally.
bool image_big(const hpccg_hip_matrix* M)
{
    const double bytes = M->has_a ? (double)M->a_slots * 8.0 : (double)M->nslots * 12.0;
    return bytes > 256e6;
}

// The matrix streams' cache policy: non-temporal loads beyond the Infinity
// Cache (a forced policy measured even or slower: DESIGN.md 4, what was dropped)
bool nt_load_of(const hpccg_hip_matrix* M) { return image_big(M); }

bool kernel_available(const hpccg_hip_matrix* M, int k)
{
    if (k == kSpmvSell) return M->has_sell;
    if (k == kSpmvDirect) return M->has_a;
    if (k == kSpmvPairs) return M->has_pairs && !M->general;
    return false;
}

// Default SpMV kernel (measured): the pair windows for 27-point
// images beyond the Infinity Cache (the staged doubles per row are small
// against the row length: 4.2 vs 26.7 at 200^3; 200^3 SpMV 352-372 us against
// 423 us for the direct kernel); x read directly at the slice's offsets
// everywhere else (100^3 44 us; 7-pt 256^3: 6 staged doubles for 7 entries,
// the LDS kernels lose); SELL-512 when there is no A image.
int choose_kernel(const hpccg_hip_matrix* M)
{
    if (M->kernel_opt >= 0 && kernel_available(M, M->kernel_opt)) return M->kernel_opt;
    if (!M->has_a) return kSpmvSell;
    const double per_row = (double)M->nnz / std::max(1, M->nrow);
    const double staged = (double)M->alds2_doubles / (2.0 * kSliceRows);
    if (kernel_available(M, kSpmvPairs) && image_big(M) && per_row >= 2.5 * staged) return kSpmvPairs;
    return kSpmvDirect;
}

// The pair kernel's LDS-DMA value ring (k_spmv_a2r): uniform width 27 or 7, and
// the windows plus the ring within the CU's LDS.
int a2_ring_effective(const hpccg_hip_matrix* M)
{
    if (M->kernel != kSpmvPairs || M->a2_ring <= 0 || (M->a_width != 27 && M->a_width != 7)) return 0;
    if (a2_lds_bytes(M->alds2_doubles, M->a2_ring) > (size_t)(159 * 1024)) return 0;
    static const int prepared = a2_ring_prepare();
    return prepared == 0 ? M->a2_ring : 0;
}

// Non-temporal stores of the CG vectors where the direct kernel streams an
// image beyond the Infinity Cache: its x reads at the +-1-plane offsets live
// on L2 reuse, which dirty Ap / p_k / r lines would crowd out. Same-process
// A/B, 7-pt 256^3: 2888 vs 2712 CG it/s (SpMV 253 vs 274 us); 200^3 (pair
// ring kernel) 2644 vs 2650 and 100^3 19190 vs 19175: left off there.
bool nt_store_effective(const hpccg_hip_matrix* M) { return M->kernel == kSpmvDirect && image_big(M); }

// p = r + beta p formed inside the SpMV: the pair kernel (ghost rows from the
// halo) on any rank count; the direct kernel on one rank, or on z-slab ranks
// with the halo received into r's ghost planes (halo_into_r); never the
// SELL-512 gather (it would double every gather: 561 -> 744 us at 200^3).
bool fuse_p_effective(const hpccg_hip_matrix* M)
{
    if (M->fuse_p == 0) return false;
    if (M->kernel == kSpmvPairs) return true;
    if (M->kernel == kSpmvDirect) return M->nranks == 1 || !M->general;
    return false;
}

bool multi_of(const hpccg_hip_matrix* M);

// The r-halo exchange (z-slab ranks, p update fused into the SpMV): instead of
// p_k's boundary planes before the SpMV (k_p_boundary + a send/recv of its
// own), r's boundary planes move right after the update, in the same RCCL
// group as the r.r all-reduce, into r's ghost planes. The fused kernels form
// p_k = r + beta p_{k-1} at every row they read, ghost rows included (the
// p_{k-1} ghosts stored by the previous launch's ghost blocks), so the direct
// kernel runs fused on any rank count and an iteration makes two RCCL calls
// (p.Ap all-reduce; r.r all-reduce + r planes) and one launch less. The
// neighbour forms the same p_k rows with the same expression and the same
// all-reduced beta: the values the reference's exchange_externals delivers
// (exchange_externals.cpp:87-126), bitwise.
bool rhalo_of(const hpccg_hip_matrix* M)
{
    return multi_of(M) && !M->general && fuse_p_effective(M) &&
           (M->kernel == kSpmvDirect || M->kernel == kSpmvPairs);
}

// The peer-memory all-reduce (option peer_allreduce; RCCL stays the default):
// on several ranks, or the 1-rank force_comm emulation. In an in-process group
// the members' kernels wait for each other inside the GPU, so they must run
// side by side: eager launches on their own streams, at most two members
// (GPU_MAX_HW_QUEUES = 4 queues hold two members' two streams each).
// Auto (-1, the default): a process's rank of an RCCL job whose creation-time
// self-test passed on every rank (peer_autotest), and the 1-rank emulation;
// never an in-process group (its members would have to run side by side,
// eagerly, instead of in one graph).
bool emulated_multi(const hpccg_hip_matrix* M);
bool peer_ar_of(const hpccg_hip_matrix* M)
{
    if (!multi_of(M) || M->peer_ar == 0) return false;
    if (M->peer_ar > 0) return !M->in_group || M->nranks <= 2;
    return !M->in_group && (emulated_multi(M) || M->peer_auto_ok);
}

// The r-halo by pull (option halo_pull, -1 auto the default): each rank reads
// its ghost planes of r from the neighbours' boundary rows -- in the
// iteration's last launch (pull_in_of) or in a k_pull launch before the SpMV
// launch (an in-process group's members' buffers; another process's
// through IPC, when the creation-time test passed on every rank; the 1-rank
// emulation pulls its own rows into scratch) instead of the RCCL send/recv
// group (or peer copies) after the update: no RCCL call left in the iteration
// when the scalars are summed in the kernels.
bool rhalo_of(const hpccg_hip_matrix* M);
bool pull_of(const hpccg_hip_matrix* M)
{
    if (!rhalo_of(M) || M->halo_pull == 0) return false;
    if (M->in_group || emulated_multi(M)) return true;
    return M->pull_auto_ok != 0;  // (an RCCL job: its neighbours' r mapped and tested at creation)
}

// In-launch pull (halo_pull 2, and auto): no k_pull launch -- the
// iteration's last launch pulls r_k once its own r.r completion is in, which
// needs the global sum inside the kernel (the peer all-reduce) and r.r folded
// into its producer (no k_finalize after it). Emulated (force_comm 2, one
// GPU), per iteration against k_pull: 100^3 +3.0 vs +4.8-5.2 us, 200^3
// +3.9-4.0 vs +5.5, 7-pt 256^3 +3.6-3.7 vs +5.6-5.7 (profiles/r04_inlaunch).
bool pull_in_of(const hpccg_hip_matrix* M, const CgArgs& a)
{
    return pull_of(M) && M->halo_pull != 1 && a.peer_ar && fold_of(a, kRR);
}

// Both dots folded into their producing kernels (slot completion, no
// k_finalize launch): same-process A/B against p.Ap folded + r.r through
// k_finalize, 100^3 19249 vs 17814 CG it/s, 200^3 2619 vs 2543, 7-pt 256^3
// 2531 vs 2425 (with the older ticket completion, folding r.r into the short
// update kernel lost: every block waited for its ticket).
int fold_effective(const hpccg_hip_matrix* M) { return M->fold == 0 ? 0 : 1; }

// x_ring auto: the long ring where the matrix image is far beyond the 256 MB
// Infinity Cache (7-pt 256^3 update 93 vs 103 us with 32 vs 8); near it, the 32
// p buffers cycled through the cache evict the image (100^3: 14290 vs 14160
// it/s with 8 vs 32). A ring of 2 at 100^3 looked +4 % in one process (the
// ring buffers of an 8-ring allocation) and measured -2.8 % across fresh
// processes (tools/ab_bench_opts.sh: 18361 vs 18899 it/s, 4 rounds each).
int x_ring_effective(const hpccg_hip_matrix* M)
{
    if (M->x_ring > 0) return M->x_ring;
    const double bytes = M->has_a ? (double)M->a_slots * 8.0 : (double)M->nslots * 12.0;
    return bytes > 512e6 ? kXRingDefault : 8;
}

// The p ring: nbuf buffers of pstride doubles, local rows 512-row aligned,
// zeroed guard zones on both sides (the A kernels read holes there).
int alloc_ring(hpccg_hip_matrix* M, int nbuf)
{
    const size_t glo_pad = ((size_t)M->ghost_lo + kSliceRows - 1) / kSliceRows * kSliceRows;
    const size_t ptotal = (size_t)M->pstride * nbuf;
    double* buf = nullptr;
    HIP_TRY(big_malloc(reinterpret_cast<void**>(&buf), sizeof(double) * ptotal));
    if (hipMemsetAsync(buf, 0, sizeof(double) * ptotal, M->stream) != hipSuccess) {
        big_free(buf);
        return set_err(HPCCG_HIP_EHIP, "hipMemset of the p ring failed");
    }
    dev_free(M, &M->d_pbuf, (size_t)M->pstride * M->ring_alloc);
    M->d_pbuf = buf;
    M->bytes += (long long)(sizeof(double) * ptotal);
    M->d_p = M->d_pbuf + kGuardRows + glo_pad;
    M->ring_alloc = nbuf;
    return 0;
}

int alloc_workspace(hpccg_hip_matrix* M)
{
    M->npad = (size_t)M->nslices * kSliceRows;
    if (M->npad == 0) M->npad = kSliceRows;
    const size_t glo_pad = ((size_t)M->ghost_lo + kSliceRows - 1) / kSliceRows * kSliceRows;
    const size_t ghi_pad = ((size_t)M->ghost_hi + 2 + kSliceRows - 1) / kSliceRows * kSliceRows;
    M->pstride = (long long)(kGuardRows + glo_pad + M->npad + ghi_pad + kGuardRows);
    TRY(alloc_ring(M, x_ring_effective(M)));
    // r as one p buffer: zeroed guard zones and ghost planes (halo_into_r)
    TRY(dev_alloc(M, &M->d_rbuf, (size_t)M->pstride, true));
    M->d_r = M->d_rbuf + kGuardRows + glo_pad;
    TRY(dev_alloc(M, &M->d_Ap, M->npad, true));
    TRY(dev_alloc(M, &M->d_x, M->npad, true));
    TRY(dev_alloc(M, &M->d_b, M->npad, true));
    const int ngroups = (M->nslices + 63) / 64;  // kGroup in hpccg_kernels.hip
    {
        const size_t np = 2 * (size_t)std::max(1, M->nslices) + 2 * ngroups + 8 + kNumXcd * kReadyStride;
        M->npartial = np;
        // one block: the iteration state and error record (kKstDoubles), then
        // the slots -- the kernels' bounded waits find the record from
        // a.partial, which they hold anyway (kst_of in hpccg_kernels.hip)
        double* blk = nullptr;
        TRY(dev_alloc(M, &blk, kKstDoubles + np, true));
        M->d_kst = reinterpret_cast<int*>(blk);
        M->d_partial = blk + kKstDoubles;
        const std::vector<unsigned long long> empty(np, kSlotEmpty);  // every dot slot starts empty
        TRY(h2d(M, M->d_partial, empty.data(), np * sizeof(double)));
    }
    TRY(dev_alloc(M, &M->d_scal, 8, true));
    TRY(flush_stream(M));  // every fill landed and written back: other streams and peers may read them
    return 0;
}

// force_comm 2 on a 1-rank communicator: the multi-rank iteration shape
// (halo fork/join, RCCL send/recv, all-reduced scalars) on one GPU, to time
// what the RCCL path adds per iteration where only one GPU is available.
bool emulated_multi(const hpccg_hip_matrix* M)
{
    return M->nranks == 1 && M->force_comm == 2 && g_comm.comm && g_comm.nranks == 1 && !M->in_group;
}
// The plane an interior z-slab rank of this problem exchanges with each
// neighbour: the stencil's largest column offset (nx ny + nx + 1 for the
// 27-point stencil, from the A image's offsets), else a 200^2 plane.
size_t emul_rows(const hpccg_hip_matrix* M)
{
    return std::min<size_t>(M->nrow, M->emul_plane > 0 ? (size_t)M->emul_plane : 40000);
}
bool multi_of(const hpccg_hip_matrix* M) { return M->nranks > 1 || emulated_multi(M); }

// Pinned readback layout: kst + error record (64 B), the scalars (64 B), then
// hist (hist_cap doubles), then the stamps (stamp_cap words).
constexpr size_t kRbScal = 64;
constexpr size_t kRbHist = 128;
static_assert(sizeof(int) * (kErrBase + kErrWords) <= kRbScal, "readback layout");

int ensure_hist(hpccg_hip_matrix* M, int max_iter)
{
    if (emulated_multi(M) && !M->d_emul) TRY(dev_alloc(M, &M->d_emul, 2 * emul_rows(M), true));
    const int need = std::max(2, max_iter + 1);
    if (need > M->hist_cap) {
        dev_free(M, &M->d_hist, M->hist_cap);
        dev_free(M, &M->d_ahist, M->hist_cap);
        TRY(dev_alloc(M, &M->d_hist, need));
        TRY(dev_alloc(M, &M->d_ahist, need));
        M->hist_cap = need;
    }
    const long long scap = (long long)(max_iter + 2) * kNumStampSlots;
    if (scap > M->stamp_cap) {
        dev_free(M, &M->d_stamps, (size_t)M->stamp_cap);
        TRY(dev_alloc(M, &M->d_stamps, (size_t)scap));
        M->stamp_cap = scap;
    }
    const size_t rb = kRbHist + sizeof(double) * (size_t)M->hist_cap + sizeof(unsigned long long) * (size_t)M->stamp_cap;
    if (rb > M->h_rb_bytes) {
        if (M->h_rb) HIP_TRY(hipHostFree(M->h_rb));
        M->h_rb = nullptr;
        M->h_rb_bytes = 0;
        HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&M->h_rb), rb, hipHostMallocDefault));
        M->h_rb_bytes = rb;
    }
    return 0;
}

// Wait for a stream by polling it: a blocking wait on a solve-long stream
// sleeps, and its wake-up cost 120-820 us per synchronous readback at the end
// of a 200^3 solve (rocprof kernel trace, profiles/r03_200); polling returns
// within microseconds.
// The end of a solve: a marker with a system-scope release (flush_stream's
// event) behind the solve's work, polled rather than blocked on (a blocking
// wait adds tens of us of wake-up). The release writes back what the kernels
// left dirty in the L2s before the caller frees, reuses or copies anything.
int wait_matrix(hpccg_hip_matrix* M)
{
    if (!M->ev_flush) HIP_TRY(hipEventCreateWithFlags(&M->ev_flush, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(M->ev_flush, M->stream));
    // a long solve: sleep (blocking sync) until its last graph chunk starts,
    // then poll only that tail -- a whole solve's spin held a host core
    // (under the box's CPU quota an RCCL job's ranks would starve
    // its proxy threads), while the blocking wait's late wake-up is hidden
    // behind the chunk still running
    if (M->mid_pending) {
        M->mid_pending = 0;
        HIP_TRY(hipEventSynchronize(M->ev_mid));
    }
    for (;;) {
        const hipError_t e = hipEventQuery(M->ev_flush);
        if (e == hipSuccess) return 0;
        if (e != hipErrorNotReady) return set_err(HPCCG_HIP_EHIP, "hipEventQuery: %s", hipGetErrorString(e));
        std::this_thread::yield();
    }
}

int grid_of(int units) { return std::max(kNumXcd, (units + kNumXcd - 1) / kNumXcd * kNumXcd); }

// x_defer 2 (x terms applied by trailing blocks of the SpMV launch) is built
// into the LDS-DMA ring pair kernel and the direct kernel; elsewhere it means 1.
int x_defer_effective(const hpccg_hip_matrix* M)
{
    const bool side = (M->kernel == kSpmvPairs && a2_ring_effective(M) > 0) || M->kernel == kSpmvDirect;
    if (M->x_defer == 2 && !side) return 1;
    return M->x_defer;
}

// Fused update: one rank (no all-reduce between p.Ap and the update), the
// direct kernel with the p update fused, both dots completed in-kernel
// through slots, x deferred beside the SpMV. On by default: same-process
// A/B with two slices per update block (fused_update_slices 2), 100^3
// 21 485 vs 20 261 CG it/s, 7-pt 256^3 2838 vs 2807 (one slice per update
// block: 20 865 / 2748 -- the update blocks inherit the SpMV's occupancy, so
// each needs more rows in flight).
bool fuse_update_effective(const hpccg_hip_matrix* M)
{
    const bool want = M->fuse_update != 0;
    // several ranks: only with the in-kernel peer all-reduce (the update needs
    // the global p.Ap inside the launch), and not in an in-process group
    // (2: also an in-process group -- tests only, members small enough to be
    // resident side by side: the update blocks wait for the other member's p.Ap)
    const bool ranks_ok = (M->nranks == 1 && !M->force_comm) || (peer_ar_of(M) && (!M->in_group || M->fuse_update == 2));
    return want && ranks_ok && M->kernel == kSpmvDirect && fuse_p_effective(M) && fold_effective(M) == 1 &&
           x_defer_effective(M) == 2;
}

// Option resident_update (-1 auto, the default: the persistent launch where
// it holds, else k_spmv_ar; 1 k_spmv_ar only; 0 off): one rank, the direct kernel at width 27 with the fused update, and the chip
// holds every pair unit of the launch at once (hipOccupancy x CUs: 27-pt up
// to ~101^3), else the unit + update-block launch stays. 100^3, alternating
// processes, 3 rounds: 19.6-19.8k -> 20.8-21.2k CG it/s, SpMV launch 49.3-49.8
// -> 46.1-46.9 us (profiles/r05_ab/resident_update_ab100.log). A solve whose
// resident wait expired (another process holding part of the GPU) is re-run
// without it (resident_retry, counted, at most kResidentMaxRetries). Not
// with the block-timeline diagnostics (their instantiation is the other launch).
bool resident_of(const hpccg_hip_matrix* M)
{
    if (!M->resident_update || M->resident_failed || M->d_tl || M->nranks != 1 || M->force_comm || M->in_group ||
        M->kernel != kSpmvDirect || M->a_width != 27 || !fuse_update_effective(M))
        return false;
    const int pairs = (M->nslices + 1) / 2;
    return resident_capacity(nt_load_of(M)) >= grid_of(pairs);
}

// The persistent CG launch (k_cg_persist; option resident_update -1 auto):
// every iteration after the prologue in one launch, where resident_of holds
// and the chip holds every pair block of it at once. Its slot loop: three
// LDS-ring slots + steps of 2 (four other shapes measured even or slower and
// are gone: DESIGN.md 4). a.resident = kResidentAuto marks it.
int persist_shape(const hpccg_hip_matrix* M) { return M->resident_update == -1 ? kResidentAuto : 0; }
// Several ranks: a process's z-slab rank whose in-kernel
// transport passed every creation-time test -- the peer all-reduce, the
// pull, the production protocol and its persistent run on every rank --
// runs the persistent launch too (its multi-rank instantiation: the dots
// summed over the ranks in the kernel, r's ghost rows pulled at the top of
// every iteration), so a 100^3-per-GPU job keeps one launch per solve. The
// per-iteration resident kernel (k_spmv_ar) has no multi-rank form.
bool persist_multi_of(const hpccg_hip_matrix* M)
{
    return M->nranks > 1 && !M->in_group && M->resident_update == -1 && !M->resident_failed && !M->d_tl &&
           M->persist_auto_ok && peer_ar_of(M) && pull_of(M) && M->halo_pull != 1 && !M->general && M->has_pairs &&
           M->kernel == kSpmvDirect && M->a_width == 27 && fuse_update_effective(M);
}
bool persist_ok(const hpccg_hip_matrix* M)
{
    if (!(persist_shape(M) && resident_of(M)) && !persist_multi_of(M)) return false;
    // (byte offsets of the p ring in 32 bits)
    if (M->pstride * 2 * (long long)sizeof(double) >= (1LL << 31)) return false;
    return persist_capacity(nt_load_of(M)) >= grid_of((M->nslices + 1) / 2);
}
// ... and its per-iteration slots are allocated: one window of kPersistWindow
// iterations per launch (a longer solve runs several launches)
long long persist_slots_needed(const hpccg_hip_matrix* M, int max_iter)
{
    return (long long)std::min(std::max(max_iter - 1, 1), kPersistWindow) * persist_slot_stride((int)M->nslices);
}
bool persist_of(const hpccg_hip_matrix* M, int max_iter)
{
    return persist_ok(M) && M->d_pslots && M->pslots_cap >= persist_slots_needed(M, max_iter);
}
int ensure_pslots(hpccg_hip_matrix* M, int max_iter)
{
    if (!persist_ok(M)) return 0;
    const long long need = persist_slots_needed(M, max_iter);
    if (need > M->pslots_cap) {
        dev_free(M, &M->d_pslots, (size_t)M->pslots_cap);
        M->pslots_cap = 0;
        // no memory for the slots: not an error -- persist_of is false without
        // them and the per-iteration resident launch runs
        if (dev_alloc(M, &M->d_pslots, (size_t)need)) {
            (void)hipGetLastError();
            M->d_pslots = nullptr;
            std::fprintf(stderr, "hpccg_hip: no device memory for the persistent launch's slots (%lld doubles); "
                                 "per-iteration launches\n", need);
            return 0;
        }
        M->pslots_cap = need;
    }
    return 0;
}

CgArgs make_args(hpccg_hip_matrix* M, const double* b, double* x, int max_iter, double tol)
{
    CgArgs a;
    std::memset(&a, 0, sizeof a);  // the graph cache compares bytes
    a.n = M->nrow;
    a.nslices = M->nslices;
    a.grid = M->grid;
    a.max_iter = max_iter;
    a.tol = tol;
    a.nranks = M->nranks;
    a.allreduce = (M->nranks > 1 || (M->force_comm && g_comm.comm && !M->in_group)) ? 1 : 0;
    a.ghost_lo = M->ghost_lo;
    a.b = b;
    a.x = x;
    a.r = M->d_r;
    a.p = M->d_p;
    a.pstride = M->pstride;
    a.pguard = (int)(kGuardRows + ((size_t)M->ghost_lo + kSliceRows - 1) / kSliceRows * kSliceRows);
    a.fuse_p = fuse_p_effective(M) ? 1 : 0;
    a.xdefer = x_defer_effective(M);
    a.xside = 1;
    a.fupd = fuse_update_effective(M) ? 1 : 0;
    // (1: k_spmv_ar; kResidentAuto: the persistent launch)
    a.resident = 0;
    if (a.fupd && resident_of(M))
        a.resident = persist_of(M, max_iter) ? persist_shape(M) : 1;
    else if (a.fupd && persist_multi_of(M) && persist_of(M, max_iter))
        a.resident = kResidentAuto;
    a.pready = M->d_partial + (M->npartial - kNumXcd * kReadyStride);
    if (a.resident >= kResidentPersist) {
        a.pslots = M->d_pslots;
        a.pslot_stride = persist_slot_stride((int)M->nslices);
    }
    a.rev = 1;
    a.nring = a.xdefer ? x_ring_effective(M) : (a.fuse_p ? 2 : 1);
    if (a.resident >= kResidentPersist) {  // x lives in the persistent blocks' registers: nothing deferred
        a.xdefer = 0;
        a.nring = 2;
    }
    const int units = M->kernel == kSpmvPairs ? (M->nslices + 1) / 2 : M->nslices;
    a.s0 = 0;
    a.sn0 = units;
    a.s1 = a.sn1 = 0;
    a.sgrid = grid_of(units);
    a.nt = nt_load_of(M) ? 1 : 0;
    a.a_width = M->a_width;
    a.ahist = M->d_ahist;
    a.fold = fold_effective(M);
    a.Ap = M->d_Ap;
    a.partial = M->d_partial;
    a.g = M->d_scal;
    a.loc = M->d_scal + 2;
    a.hist = M->d_hist;
    a.kst = M->d_kst;
    a.dbg_withhold = M->dbg_withhold;
    a.dbg_resident_stall = M->dbg_resident_stall;
    a.dbg_tl = M->d_tl;
    a.rhalo = rhalo_of(M) ? 1 : 0;
    a.ghost_hi = M->ghost_hi;
    a.gbase = INT_MAX;  // set per launch
    a.peer_ar = peer_ar_of(M) && M->d_peers ? 1 : 0;
    if (a.peer_ar) {  // the scalars are summed inside the kernels: no RCCL all-reduce, no group sum
        a.allreduce = 0;
        a.prank = M->nranks > 1 ? M->rank : 0;
        a.pranks = M->nranks;
        a.mbox = M->d_mbox;
        a.peers = M->d_peers;
    }
    a.stamps = M->d_stamps;
    if (pull_of(M)) {  // the rows the neighbours pull go write-through (pulled_slice)
        a.rsend_lo = emulated_multi(M) ? (int)emul_rows(M) : M->send_lo;
        a.rsend_hi = emulated_multi(M) ? (int)emul_rows(M) : M->send_hi;
        a.pull_in = pull_in_of(M, a) ? 1 : 0;  // (pl_*: pull_plan, once the ranks' r are known)
    }
    a.slice_base = M->d_slice_base;
    a.cols = M->d_cols;
    a.vals = M->d_vals;
    a.aval = M->d_aval;
    a.aoff = M->d_aoff;
    a.abase = M->d_abase;
    a.alds2 = M->d_alds2;
    a.adiag2 = M->d_adiag2;
    a.atri = M->d_atri;
    a.awin2 = M->d_awin2;
    a.awn2 = M->d_awn2;
    a.alds2_doubles = std::max(1, M->alds2_doubles);
    a.a2_ring = a2_ring_effective(M);
    a.nt_store = nt_store_effective(M) ? 1 : 0;
    if (std::getenv("HPCCG_DEBUG_ADDR"))
        std::fprintf(stderr, "hpccg_hip addr: aval %p p %p pstride_B %lld r %p Ap %p x %p b %p\n", (void*)a.aval,
                     (void*)a.p, a.pstride * 8, (void*)a.r, (void*)a.Ap, (void*)a.x, (void*)a.b);
    return a;
}

// ---------------------------------------------------------------------------
// exchanges
// ---------------------------------------------------------------------------
// Halo exchange of p (exchange_externals.cpp:51-131): the z-slab ghosts are
// contiguous, so no pack: rank r sends its first send_lo rows down and its
// last send_hi rows up, and receives straight into the ghost regions.
// The RCCL data path asked for on a host-bootstrapped communicator (solve_ranks
// refuses such an iteration up front; this guards every other caller).
int need_rccl(const char* what)
{
    return set_err(HPCCG_HIP_EINVAL, "%s needs RCCL: the host-bootstrapped communicator runs the peer all-reduce "
                                     "and the halo pull only", what);
}

int enqueue_halo(hpccg_hip_matrix* M, double* p, hipStream_t st, double* dst = nullptr)
{
    // dst: where the ghost planes land (local row 0 of that buffer; p's own by default)
    if (!dst) dst = p;
    if (g_comm.nranks == 1) {
        if (!emulated_multi(M)) return 0;
        // force_comm 2: an interior rank's two planes (its first and last
        // rows) sent to itself, through the same RCCL calls and streams
        const size_t cnt = emul_rows(M);
        NCCL_TRY(ncclGroupStart());
        NCCL_TRY(ncclRecv(M->d_emul, cnt, ncclFloat64, 0, g_comm.comm, st));
        NCCL_TRY(ncclSend(p, cnt, ncclFloat64, 0, g_comm.comm, st));
        NCCL_TRY(ncclRecv(M->d_emul + cnt, cnt, ncclFloat64, 0, g_comm.comm, st));
        NCCL_TRY(ncclSend(p + M->nrow - cnt, cnt, ncclFloat64, 0, g_comm.comm, st));
        NCCL_TRY(ncclGroupEnd());
        return 0;
    }
    if (!g_comm.comm) return need_rccl("the p halo exchange");
    const int r = g_comm.rank;
    NCCL_TRY(ncclGroupStart());
    if (r > 0) {
        if (M->ghost_lo) NCCL_TRY(ncclRecv(dst - M->ghost_lo, M->ghost_lo, ncclFloat64, r - 1, g_comm.comm, st));
        if (M->send_lo) NCCL_TRY(ncclSend(p, M->send_lo, ncclFloat64, r - 1, g_comm.comm, st));
    }
    if (r < g_comm.nranks - 1) {
        if (M->ghost_hi) NCCL_TRY(ncclRecv(dst + M->nrow, M->ghost_hi, ncclFloat64, r + 1, g_comm.comm, st));
        if (M->send_hi) NCCL_TRY(ncclSend(p + M->nrow - M->send_hi, M->send_hi, ncclFloat64, r + 1, g_comm.comm, st));
    }
    NCCL_TRY(ncclGroupEnd());
    return 0;
}

// The z-slab halo of p through the host bootstrap (the kernel-level sparsemv
// of a host-bootstrapped job; its solver pulls r's planes in the kernels):
// every rank contributes its first send_lo and last send_hi rows and takes its
// ghost planes from its neighbours' contributions (exchange_externals.cpp
// :87-126, staged through the host). Local failures are recorded, not
// returned, until both all-gathers are done.
int host_halo(hpccg_hip_matrix* M, double* p)
{
    const int P = g_comm.nranks, r = g_comm.rank;
    const int mine[2] = {M->send_lo, M->send_hi};
    std::vector<int> sz(2 * P);
    TRY(comm_allgather(mine, sz.data(), sizeof mine));
    int S = 1;
    for (int q = 0; q < P; q++) S = std::max(S, sz[2 * q] + sz[2 * q + 1]);
    std::vector<double> out(S, 0.0), all((size_t)S * P);
    int rc = 0;
    if (M->send_lo) rc = d2h(M->stream, out.data(), p, sizeof(double) * M->send_lo);
    if (!rc && M->send_hi) rc = d2h(M->stream, out.data() + M->send_lo, p + M->nrow - M->send_hi, sizeof(double) * M->send_hi);
    TRY(comm_allgather(out.data(), all.data(), sizeof(double) * S));
    if (rc) return rc;
    if (r > 0 && M->ghost_lo) {  // rank r-1's last rows: its contribution after its first send_lo
        if (sz[2 * (r - 1) + 1] != M->ghost_lo) return set_err(HPCCG_HIP_EPLAN, "host halo: rank %d sends %d rows, %d needed", r - 1, sz[2 * (r - 1) + 1], M->ghost_lo);
        TRY(h2d(M, p - M->ghost_lo, all.data() + (size_t)S * (r - 1) + sz[2 * (r - 1)], sizeof(double) * M->ghost_lo));
    }
    if (r < P - 1 && M->ghost_hi) {  // rank r+1's first rows
        if (sz[2 * (r + 1)] != M->ghost_hi) return set_err(HPCCG_HIP_EPLAN, "host halo: rank %d sends %d rows, %d needed", r + 1, sz[2 * (r + 1)], M->ghost_hi);
        TRY(h2d(M, p + M->nrow, all.data() + (size_t)S * (r + 1), sizeof(double) * M->ghost_hi));
    }
    return 0;
}

// Gather plan over RCCL (exchange_externals.cpp:51-131): pack what each
// requester needs, then one grouped send/recv per neighbour; the externals
// arrive contiguously after the local rows.
int enqueue_halo_gather(hpccg_hip_matrix* M, const CgArgs& a, double* p, bool prologue)
{
    if (g_comm.nranks == 1) return 0;
    if (!g_comm.comm) return need_rccl("the gather halo exchange");
    launch_cg_pack(a, M->d_send_idx, M->nsend, M->d_send_buf, prologue, M->stream);
    NCCL_TRY(ncclGroupStart());
    for (size_t i = 0; i < M->recv_rank.size(); i++)
        NCCL_TRY(ncclRecv(p + M->nrow + M->recv_off[i], M->recv_cnt[i], ncclFloat64, M->recv_rank[i], g_comm.comm,
                          M->stream));
    for (size_t i = 0; i < M->send_rank.size(); i++)
        NCCL_TRY(ncclSend(M->d_send_buf + M->send_off[i], M->send_cnt[i], ncclFloat64, M->send_rank[i], g_comm.comm,
                          M->stream));
    NCCL_TRY(ncclGroupEnd());
    return 0;
}

// MPI_Allreduce of one scalar (ddot.cpp:79-80): loc[which] -> g[which].
int enqueue_allreduce(hpccg_hip_matrix* M, const CgArgs& a, int which)
{
    if (!a.allreduce) return 0;
    if (!g_comm.comm) return comm_host() ? need_rccl("the scalar all-reduce") : 0;
    NCCL_TRY(ncclAllReduce(a.loc + which, a.g + which, 1, ncclFloat64, ncclSum, g_comm.comm, M->stream));
    return 0;
}

int ensure_events(hpccg_hip_matrix* M, int slots)
{
    static const bool fence = [] {  // diagnostics: HPCCG_EVENT_FENCE=1 keeps the release
        const char* e = std::getenv("HPCCG_EVENT_FENCE");
        return e && e[0] == '1';
    }();
    while ((int)M->ev.size() < 4 * slots) {
        hipEvent_t e;
        // no system-scope release at the record: a timed kernel's interval
        // would otherwise include writing back the caches it left dirty
        HIP_TRY(hipEventCreateWithFlags(&e, fence ? hipEventDefault : hipEventDisableSystemFence));
        M->ev.push_back(e);
    }
    return 0;
}

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

// copy between two members (same device: a plain D2D copy, graph-capturable)
int member_copy(hpccg_hip_matrix* dst_m, double* dst, const hpccg_hip_matrix* src_m, const double* src, size_t n,
                hipStream_t s)
{
    if (n == 0) return 0;
    if (dst_m->device == src_m->device)
        HIP_TRY(hipMemcpyAsync(dst, src, sizeof(double) * n, hipMemcpyDeviceToDevice, s));
    else
        HIP_TRY(hipMemcpyPeerAsync(dst, dst_m->device, src, src_m->device, sizeof(double) * n, s));
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
    auto dst_of = p_of;
    for (int r = 0; r < R.P; r++) {
        hpccg_hip_matrix* M = R.M[r];
        TRY(use_device(R, r));
        if (r > 0 && M->ghost_lo) {
            const hpccg_hip_matrix* L = R.M[r - 1];
            HIP_TRY(hipStreamWaitEvent(M->stream, R.ev[r - 1], 0));
            TRY(member_copy(M, dst_of(r) - M->ghost_lo, L, p_of(r - 1) + L->nrow - M->ghost_lo, M->ghost_lo,
                            M->stream));
        }
        if (r < R.P - 1 && M->ghost_hi) {
            const hpccg_hip_matrix* U = R.M[r + 1];
            HIP_TRY(hipStreamWaitEvent(M->stream, R.ev[r + 1], 0));
            TRY(member_copy(M, dst_of(r) + M->nrow, U, p_of(r + 1), M->ghost_hi, M->stream));
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
            TRY(member_copy(M, p + M->nrow + M->recv_off[i], Q, Q->d_send_buf + Q->send_off[j], M->recv_cnt[i],
                            M->stream));
        }
    }
    return 0;
}

// In-process all-reduce of loc[which]: one lane on rank 0's stream adds the
// ranks' values in rank order and writes g[which] of every rank.
// Group fold (CgArgs::gfw): the phase's last member's kernel sums the dot;
// the others' streams only wait for it. The SpMV phase runs the members
// 0 .. P-1 and member P-1 folds p.Ap; the update phase runs them in reverse and
// member 0 folds r.r, so member 0's next SpMV follows its own update (its r
// and p still in the MALL: the 2 x 100^3 group's SpMV ran 56-58 us after the
// other member's launches against 42 us after its own).
// group_gather_join runs before the folding member's launch: its stream waits
// for every other member's.
bool gfold_of(const Ranks& R) { return R.P > 1 && R.a[0].gn > 0; }
int fold_member(const Ranks& R, int which) { return which == kPAP ? R.P - 1 : 0; }

int group_gather_join(const Ranks& R, int last)
{
    for (int r = 0; r < R.P; r++) {
        if (r == last) continue;
        TRY(use_device(R, r));
        HIP_TRY(hipEventRecord(R.ev[r], R.M[r]->stream));
    }
    TRY(use_device(R, last));
    for (int r = 0; r < R.P; r++)
        if (r != last) HIP_TRY(hipStreamWaitEvent(R.M[last]->stream, R.ev[r], 0));
    return 0;
}

int group_allreduce(const Ranks& R, int which)
{
    if (gfold_of(R)) {  // summed by the folding member's launch: its end releases the others
        const int f = fold_member(R, which);
        TRY(use_device(R, f));
        HIP_TRY(hipEventRecord(R.ev[R.P], R.M[f]->stream));
        for (int r = 0; r < R.P; r++) {
            if (r == f) continue;
            TRY(use_device(R, r));
            HIP_TRY(hipStreamWaitEvent(R.M[r]->stream, R.ev[R.P], 0));
        }
        return 0;
    }
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
    return enqueue_halo(R.M[0], prologue ? R.a[0].p : ring_p(R.a[0], k_host), R.M[0]->stream);
}

int exch_allreduce(const Ranks& R, int which)
{
    if (!R.a[0].allreduce) return 0;
    if (R.P > 1) return group_allreduce(R, which);
    return enqueue_allreduce(R.M[0], R.a[0], which);
}

// r-halo (rhalo_of): after the update, the r.r all-reduce and r's boundary
// planes into the neighbours' r ghost planes. One RCCL group on a process's
// communicator (force_comm 2: a plane-sized self send/recv of r, the shape of
// the multi-rank iteration on one GPU); peer copies in an in-process group,
// after the rank-ordered sum (whose stream waited for every member's update).
int exch_rr_rhalo(const Ranks& R)
{
    if (pull_of(R.M[0])) {  // the planes are pulled before the next SpMV: the r.r all-reduce only
        if (!R.a[0].allreduce) return 0;  // (peer all-reduce: summed in the kernels)
        return R.P > 1 ? group_allreduce(R, kRR) : enqueue_allreduce(R.M[0], R.a[0], kRR);
    }
    if (R.P > 1) {
        if (R.a[0].allreduce) {
            TRY(group_allreduce(R, kRR));
        } else {  // peer all-reduce (in the kernels): only the copies' order on the members' streams
            for (int r = 0; r < R.P; r++) {
                TRY(use_device(R, r));
                HIP_TRY(hipEventRecord(R.ev[r], R.M[r]->stream));
            }
            for (int r = 0; r < R.P; r++) {
                TRY(use_device(R, r));
                if (r > 0) HIP_TRY(hipStreamWaitEvent(R.M[r]->stream, R.ev[r - 1], 0));
                if (r < R.P - 1) HIP_TRY(hipStreamWaitEvent(R.M[r]->stream, R.ev[r + 1], 0));
            }
        }
        for (int r = 0; r < R.P; r++) {
            hpccg_hip_matrix* M = R.M[r];
            double* rr = R.a[r].r;
            TRY(use_device(R, r));
            if (r > 0 && M->ghost_lo)
                TRY(member_copy(M, rr - M->ghost_lo, R.M[r - 1], R.a[r - 1].r + R.M[r - 1]->nrow - M->ghost_lo,
                                M->ghost_lo, M->stream));
            if (r < R.P - 1 && M->ghost_hi)
                TRY(member_copy(M, rr + M->nrow, R.M[r + 1], R.a[r + 1].r, M->ghost_hi, M->stream));
        }
        return 0;
    }
    hpccg_hip_matrix* M = R.M[0];
    const CgArgs& a = R.a[0];
    if (!g_comm.comm) return comm_host() ? need_rccl("r's plane exchange") : 0;
    // the all-reduce and the planes in one RCCL group
    NCCL_TRY(ncclGroupStart());
    if (a.allreduce)
        NCCL_TRY(ncclAllReduce(a.loc + kRR, a.g + kRR, 1, ncclFloat64, ncclSum, g_comm.comm, M->stream));
    if (g_comm.nranks == 1) {  // force_comm 2: an interior rank's two planes, to itself
        const size_t cnt = emul_rows(M);
        NCCL_TRY(ncclRecv(M->d_emul, cnt, ncclFloat64, 0, g_comm.comm, M->stream));
        NCCL_TRY(ncclSend(a.r, cnt, ncclFloat64, 0, g_comm.comm, M->stream));
        NCCL_TRY(ncclRecv(M->d_emul + cnt, cnt, ncclFloat64, 0, g_comm.comm, M->stream));
        NCCL_TRY(ncclSend(a.r + M->nrow - cnt, cnt, ncclFloat64, 0, g_comm.comm, M->stream));
    } else {
        const int r = g_comm.rank;
        if (r > 0) {
            if (M->ghost_lo) NCCL_TRY(ncclRecv(a.r - M->ghost_lo, M->ghost_lo, ncclFloat64, r - 1, g_comm.comm, M->stream));
            if (M->send_lo) NCCL_TRY(ncclSend(a.r, M->send_lo, ncclFloat64, r - 1, g_comm.comm, M->stream));
        }
        if (r < g_comm.nranks - 1) {
            if (M->ghost_hi) NCCL_TRY(ncclRecv(a.r + M->nrow, M->ghost_hi, ncclFloat64, r + 1, g_comm.comm, M->stream));
            if (M->send_hi)
                NCCL_TRY(ncclSend(a.r + M->nrow - M->send_hi, M->send_hi, ncclFloat64, r + 1, g_comm.comm, M->stream));
        }
    }
    NCCL_TRY(ncclGroupEnd());
    return 0;
}

// The r-halo by pull (pull_of): where rank r's ghost planes of r come from,
// into av[r].pl_* (k_pull's operands, or the in-launch pull's).
int pull_plan(hpccg_hip_matrix* const* Ms, CgArgs* av, int P, int r)
{
    hpccg_hip_matrix* M = Ms[r];
    CgArgs& a = av[r];
    const double *lo_src = nullptr, *hi_src = nullptr;
    double *lo_dst = a.r - M->ghost_lo, *hi_dst = a.r + M->nrow;
    int lo = 0, hi = 0;
    if (P > 1) {  // an in-process group: the members' own buffers
        if (r > 0 && M->ghost_lo) {
            lo = M->ghost_lo;
            lo_src = av[r - 1].r + Ms[r - 1]->nrow - lo;
        }
        if (r < P - 1 && M->ghost_hi) {
            hi = M->ghost_hi;
            hi_src = av[r + 1].r;
        }
    } else if (emulated_multi(M)) {  // an interior rank's two planes: its own rows into scratch
        // (halo_pull 3, diagnostics: none -- the iteration's cost without its halo)
        lo = hi = M->halo_pull == 3 ? 0 : (int)emul_rows(M);
        lo_src = a.r;
        hi_src = a.r + M->nrow - hi;
        lo_dst = M->d_emul;
        hi_dst = M->d_emul + lo;
    } else {  // an RCCL job: the neighbours' r, IPC-mapped at creation
        if (M->ghost_lo) {
            lo = M->ghost_lo;
            lo_src = M->d_pull_lo ? M->d_pull_lo + M->pull_lo_n - lo : nullptr;
        }
        if (M->ghost_hi) {
            hi = M->ghost_hi;
            hi_src = M->d_pull_hi;
        }
        if ((lo && !lo_src) || (hi && !hi_src)) return set_err(HPCCG_HIP_EINVAL, "halo_pull: a neighbour's r is not mapped");
    }
    a.pl_lo = lo;
    a.pl_hi = hi;
    a.pl_src_lo = lo_src;
    a.pl_src_hi = hi_src;
    a.pl_dst_lo = lo_dst;
    a.pl_dst_hi = hi_dst;
    return 0;
}

// k_pull: rank r's ghost planes right before its SpMV launch, on its stream.
void enqueue_pull(const Ranks& R, int r, const CgArgs& a)
{
    launch_pull(a, a.pl_src_lo, a.pl_dst_lo, a.pl_lo, a.pl_src_hi, a.pl_dst_hi, a.pl_hi, R.M[r]->stream);
}

// One CG iteration k (HPCCG.cpp:358-386), fully device resident, for every
// rank of R. slot >= 0 (single matrix): bracket the SpMV and the update with
// that slot's hipEvents. k_host is the iteration being enqueued: it addresses
// p_k's ring slot for the halo.
int enqueue_iteration(const Ranks& R, int slot = -1, int k_host = 1)
{
    const bool multi = multi_of(R.M[0]);
    // (fused p update on z-slab ranks: always the r-halo, rhalo_of; the gather
    // plan's k_pack forms the halo rows itself)
    for (int r = 0; r < R.P; r++) {
        TRY(use_device(R, r));
        if (!R.a[r].fuse_p) launch_cg_p_update(R.a[r], R.M[r]->stream);
    }
    if (multi && !R.a[0].rhalo) TRY(exch_halo(R, k_host, false));  // (rhalo: r's planes came with r.r)
    const bool pull = multi && pull_of(R.M[0]);
    for (int r = 0; r < R.P; r++) {
        hpccg_hip_matrix* M = R.M[r];
        CgArgs a = R.a[r];
        a.kpar = k_host & 1;  // fused update: the parity slot of k (iter_k)
        TRY(use_device(R, r));
        if (gfold_of(R) && r == R.P - 1) TRY(group_gather_join(R, r));  // (use_device(R, r) after it)
        TRY(use_device(R, r));
        if (pull && !a.pull_in && !a.npseg) enqueue_pull(R, r, a);  // r's ghost planes for this SpMV
        if (slot >= 0) HIP_TRY(hipEventRecord(M->ev[4 * slot], M->stream));
        launch_cg_spmv(a, M->kernel, false, M->stream);
        if (slot >= 0) HIP_TRY(hipEventRecord(M->ev[4 * slot + 1], M->stream));
        if (!fold_of(a, kPAP)) launch_cg_finalize(a, kPAP, false, M->stream);
    }
    if (R.a[0].fupd) {  // the update ran inside the SpMV launch (one rank, or the peer all-reduce)
        if (slot >= 0) {
            HIP_TRY(hipEventRecord(R.M[0]->ev[4 * slot + 2], R.M[0]->stream));
            HIP_TRY(hipEventRecord(R.M[0]->ev[4 * slot + 3], R.M[0]->stream));
        }
        if (R.a[0].rhalo) TRY(exch_rr_rhalo(R));  // r's planes (the scalars were summed in the launch)
        HIP_TRY(hipGetLastError());
        return 0;
    }
    TRY(exch_allreduce(R, kPAP));
    for (int i = 0; i < R.P; i++) {
        const int r = gfold_of(R) ? R.P - 1 - i : i;  // group fold: the update phase in reverse
        hpccg_hip_matrix* M = R.M[r];
        const CgArgs& a = R.a[r];
        if (a.fupd) continue;  // (group fold: member P-1's update ran in its SpMV launch)
        if (gfold_of(R) && r == fold_member(R, kRR)) TRY(group_gather_join(R, r));
        TRY(use_device(R, r));
        if (slot >= 0) HIP_TRY(hipEventRecord(M->ev[4 * slot + 2], M->stream));
        launch_cg_update(a, false, M->stream);
        if (slot >= 0) HIP_TRY(hipEventRecord(M->ev[4 * slot + 3], M->stream));
        if (!fold_of(a, kRR)) launch_cg_finalize(a, kRR, false, M->stream);
    }
    if (R.a[0].rhalo)
        TRY(exch_rr_rhalo(R));
    else
        TRY(exch_allreduce(R, kRR));
    HIP_TRY(hipGetLastError());
    return 0;
}

// The prologue's p = x halo by pull (exchange_externals.cpp:51-131 at
// HPCCG.cpp:349) for a process's rank of a job whose pull tests passed, x in
// the mapped workspace: after a one-lane peer barrier (every rank's x is in
// place), the neighbours' boundary rows of x are read with system-scope loads
// into p's ghost rows through k_prologue_copy's expression. With it a solve
// makes no RCCL call at all (the host-bootstrapped job has none to make).
// Only state every rank shares decides it (the creation-time verdicts, the
// options): a process's multi-rank solve always runs on the
// matrix's own x workspace, the buffer the neighbours mapped (solve_ranks
// refuses anything else), so no rank can pick the pull while its neighbour
// posts RCCL sends.
bool xpull_of(const hpccg_hip_matrix* M, const CgArgs& a)
{
    return M->nranks > 1 && !M->in_group && pull_of(M) && a.peer_ar && (!M->ghost_lo || M->d_pullx_lo) &&
           (!M->ghost_hi || M->d_pullx_hi);
}

void prologue_pull(hpccg_hip_matrix* M, const CgArgs& a)
{
    launch_cg_stamp(a, kStampHalo, true, M->stream);
    launch_peer_barrier(a, M->stream);
    const int lo = M->ghost_lo, hi = M->ghost_hi;
    launch_pull(a, lo ? M->d_pullx_lo + M->pull_lo_n - lo : nullptr, a.p - lo, lo, M->d_pullx_hi, a.p + M->nrow, hi,
                M->stream, true, true);
}

int enqueue_prologue(const Ranks& R, bool events)
{
    const bool multi = multi_of(R.M[0]);
    for (int r = 0; r < R.P; r++) {
        TRY(use_device(R, r));
        launch_cg_prologue_copy(R.a[r], R.M[r]->stream);  // p = x
    }
    if (multi && R.P == 1 && xpull_of(R.M[0], R.a[0]))
        prologue_pull(R.M[0], R.a[0]);
    else if (multi)
        TRY(exch_halo(R, 0, true));
    for (int r = 0; r < R.P; r++) {
        hpccg_hip_matrix* M = R.M[r];
        const CgArgs& a = R.a[r];
        hipStream_t s = M->stream;
        TRY(use_device(R, r));
        if (events) HIP_TRY(hipEventRecord(M->ev[0], s));
        launch_cg_spmv(a, M->kernel, true, s);  // Ap = A p
        if (events) HIP_TRY(hipEventRecord(M->ev[1], s));
        if (gfold_of(R)) continue;  // the updates below, in reverse (fold_member)
        if (events) HIP_TRY(hipEventRecord(M->ev[2], s));
        launch_cg_update(a, true, s);  // r = b - Ap (+ r.r partials)
        if (events) HIP_TRY(hipEventRecord(M->ev[3], s));
        if (!fold_of(a, kRR)) launch_cg_finalize(a, kRR, true, s);  // rtrans, k = 1
    }
    for (int i = 0; gfold_of(R) && i < R.P; i++) {  // group fold: member 0 last, it folds r.r
        const int r = R.P - 1 - i;
        if (r == fold_member(R, kRR)) TRY(group_gather_join(R, r));
        TRY(use_device(R, r));
        launch_cg_update(R.a[r], true, R.M[r]->stream);
    }
    if (R.a[0].rhalo)
        TRY(exch_rr_rhalo(R));  // r_0's planes: iteration 1 forms p_1 = r_0 at the ghost rows
    else
        TRY(exch_allreduce(R, kRR));
    HIP_TRY(hipGetLastError());
    return 0;
}

// Iterations per captured graph: a multiple of the p ring length when a halo
// is exchanged (the captured copies address p_k's ring slot by k_host, so a
// replay must start on the same slot), else graph_iters.
int graph_chunk_of(const Ranks& R)
{
    int chunk = std::max(1, R.M[0]->graph_iters);
    if (R.a[0].fupd || R.a[R.P - 1].fupd) chunk += chunk & 1;  // the parity of k is baked into each captured launch
    if (multi_of(R.M[0]) && !R.a[0].rhalo) {
        const int ring = R.a[0].nring;
        chunk = (chunk + ring - 1) / ring * ring;
    }
    return chunk;
}

// Capture `chunk` iterations of every rank of R into one hipGraph on rank 0's
// stream. One device only; RCCL calls are captured with the rest. Several
// in-process ranks: their work is captured
// serialised on rank 0's stream -- the ROCm 7.2 runtime crashes capturing a
// stream that waits on events of two other capturing streams
// (tools/probe/capture_probe.hip: 3+ forked streams segfault, 1-2 do not) --
// which costs nothing on one device, where each rank's kernels fill the GPU.
int build_graph(const Ranks& R, int chunk)
{
    hpccg_hip_matrix* M0 = R.M[0];
    if (M0->graph_exec) {
        (void)hipGraphExecDestroy(M0->graph_exec);
        M0->graph_exec = nullptr;
    }
    hipStream_t s0 = M0->stream;
    std::vector<hipStream_t> saved;
    if (R.P > 1)
        for (int r = 0; r < R.P; r++) {
            saved.push_back(R.M[r]->stream);
            R.M[r]->stream = s0;
        }
    struct Restore {
        const Ranks& R;
        std::vector<hipStream_t>& saved;
        ~Restore()
        {
            for (size_t r = 0; r < saved.size(); r++) R.M[r]->stream = saved[r];
        }
    } restore{R, saved};
    hipGraph_t g = nullptr;
    HIP_TRY(hipStreamBeginCapture(s0, hipStreamCaptureModeThreadLocal));
    int rc = 0;
    for (int i = 0; i < chunk && rc == 0; i++) rc = enqueue_iteration(R, -1, i + 1);
    hipError_t e = hipStreamEndCapture(s0, &g);
    if (rc) {
        if (g) (void)hipGraphDestroy(g);
        (void)hipGetLastError();
        return rc;
    }
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return set_err(HPCCG_HIP_EHIP, "graph capture failed: %s", hipGetErrorString(e));
    }
    e = hipGraphInstantiate(&M0->graph_exec, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (e != hipSuccess) {
        M0->graph_exec = nullptr;
        (void)hipGetLastError();
        return set_err(HPCCG_HIP_EHIP, "graph instantiate failed: %s", hipGetErrorString(e));
    }
    M0->graph_chunk = chunk;
    return 0;
}

// Device stamps -> the reference's timer classes: every stamped (time, class)
// in time order up to the end stamp; a class owns the time until the next
// stamp.
void stamps_to_times(const std::vector<unsigned long long>& st, int max_iter, double* times)
{
    const unsigned long long t_end = st[(size_t)(max_iter + 1) * kNumStampSlots + kStampEnd];
    std::vector<std::pair<unsigned long long, int>> ev;
    for (int k = 0; k <= max_iter; k++)
        for (int s = 0; s < kNumStampSlots; s++) {
            const unsigned long long t = st[(size_t)k * kNumStampSlots + s];
            if (t && (!t_end || t <= t_end)) ev.push_back({t, s});
        }
    std::sort(ev.begin(), ev.end());
    if (t_end) ev.push_back({t_end, kStampEnd});
    double t1 = 0, t2 = 0, t3 = 0, t4 = 0, t5 = 0;
    for (size_t i = 0; i + 1 < ev.size(); i++) {
        const double d = (double)(ev[i + 1].first - ev[i].first) * 1e-8;  // 100 MHz
        switch (ev[i].second) {
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

// Iteration state and error record zeroed, the spin budget (ticks) set.
int clear_state(hpccg_hip_matrix* M)
{
    const long long ticks = M->spin_us * 100;  // s_memrealtime: 100 MHz
    HIP_TRY(hipMemsetAsync(M->d_kst, 0, sizeof(int) * (kErrBase + kErrWords), M->stream));
    HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)(M->d_kst + kErrBase + kErrBudget), (int)ticks, 1, M->stream));
    return 0;
}

// A mailbox for the peer all-reduce: uncached device memory where the runtime
// gives it (every load and store goes to memory: other GPUs write it over
// xGMI), else fine-grained; every slot empty. A plain (coarse-grained)
// allocation is not used: nothing makes another GPU's stores into it visible
// to this GPU's polls through its L2. Returns 1 when neither kind
// could be allocated.
int alloc_mbox(hpccg_hip_matrix* M)
{
    const size_t bytes = sizeof(double) * kMboxSlots;
    void* p = nullptr;
    if (hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached) != hipSuccess) {
        (void)hipGetLastError();
        p = nullptr;
        if (hipExtMallocWithFlags(&p, bytes, hipDeviceMallocFinegrained) != hipSuccess) {
            (void)hipGetLastError();
            return 1;
        }
    }
    M->d_mbox = static_cast<double*>(p);
    const std::vector<unsigned long long> empty(kMboxSlots, kSlotEmpty);
    TRY(h2d(M, M->d_mbox, empty.data(), bytes));
    return 0;
}

// Collective over the ranks of a job (RCCL or the host bootstrap): every rank
// exports its mailbox (IPC handle), all-gathers the handles and maps the
// others'. A local failure only clears this rank's flag -- every rank makes
// the same collective calls whatever fails locally -- and
// *all_ok is the minimum over the ranks (0: nothing is mapped).
int map_peer_mailboxes(hpccg_hip_matrix* M, std::vector<double*>& table, int* all_ok)
{
    const int nr = M->nranks;
    int ok = 1;
    if (!M->d_mbox) {
        ok = alloc_mbox(M) == 0;
        if (!ok) M->selftest_note += "mailbox: no uncached or fine-grained memory; ";
        (void)hipGetLastError();
    }
    hipIpcMemHandle_t h;
    std::memset(&h, 0, sizeof h);
    hipError_t e;
    if (ok && (e = hipIpcGetMemHandle(&h, M->d_mbox)) != hipSuccess) {
        M->selftest_note += std::string("mailbox hipIpcGetMemHandle: ") + hipGetErrorString(e) + "; ";
        (void)hipGetLastError();
        ok = 0;
    }
    const size_t hb = sizeof(h), rec = hb + 8;  // handle | ok flag (padded)
    std::vector<unsigned char> mine(rec, 0), all(rec * nr);
    std::memcpy(mine.data(), &h, hb);
    mine[hb] = (unsigned char)ok;
    TRY(comm_allgather(mine.data(), all.data(), rec));
    int mapped = 1;
    for (int q = 0; q < nr; q++) mapped = mapped && all[rec * q + hb] != 0;
    for (int q = 0; q < nr && mapped; q++) {
        if (q == M->rank) {
            table[q] = M->d_mbox;
            continue;
        }
        hipIpcMemHandle_t hq;
        std::memcpy(&hq, all.data() + rec * q, hb);
        void* ptr = nullptr;
        if ((e = hipIpcOpenMemHandle(&ptr, hq, hipIpcMemLazyEnablePeerAccess)) != hipSuccess) {
            M->selftest_note += "rank " + std::to_string(q) + "'s mailbox hipIpcOpenMemHandle: " +
                                hipGetErrorString(e) + "; ";
            (void)hipGetLastError();
            mapped = 0;
            break;
        }
        M->ipc_opened.push_back(ptr);
        table[q] = static_cast<double*>(ptr);
    }
    TRY(comm_min(mapped, all_ok));  // every rank learns whether every rank mapped every mailbox
    if (!*all_ok) {
        for (void* ptr : M->ipc_opened) (void)hipIpcCloseMemHandle(ptr);
        M->ipc_opened.clear();
    }
    return 0;
}

// The peer all-reduce's mailboxes and each rank's table of them (once per
// rank count): an in-process group's members address each other's directly;
// the ranks of a job exchange IPC handles of their mailboxes (one all-gather
// over RCCL or the host bootstrap) and map them (hipIpcOpenMemHandle); the 1-rank
// emulation addresses its own.
int ensure_peers(hpccg_hip_matrix* const* Ms, int P)
{
    hpccg_hip_matrix* M = Ms[0];
    if (!peer_ar_of(M)) return 0;
    const int nr = M->nranks;
    if (nr > kMaxGroupRanks) return set_err(HPCCG_HIP_EINVAL, "peer_allreduce: at most %d ranks", kMaxGroupRanks);
    bool ready = true;
    for (int r = 0; r < P; r++) ready = ready && Ms[r]->peers_for == nr && Ms[r]->d_peers;
    if (ready) return 0;
    std::vector<std::vector<double*>> tables(P, std::vector<double*>(kMaxGroupRanks, nullptr));
    if (P > 1 || nr == 1) {
        for (int r = 0; r < P; r++) {
            HIP_TRY(hipSetDevice(Ms[r]->device));
            if (!Ms[r]->d_mbox && alloc_mbox(Ms[r]))
                return set_err(HPCCG_HIP_EINVAL, "peer_allreduce: no uncached or fine-grained mailbox memory");
        }
        for (int r = 0; r < P; r++)
            for (int q = 0; q < P; q++) tables[r][q] = Ms[q]->d_mbox;
    } else {  // one process per GPU: IPC handles through RCCL
        if (!comm_up()) return set_err(HPCCG_HIP_EINVAL, "peer_allreduce: no communicator");
        int all_ok = 0;
        TRY(map_peer_mailboxes(M, tables[0], &all_ok));
        if (!all_ok)
            return set_err(HPCCG_HIP_EINVAL,
                           "peer_allreduce: a rank's mailbox could not be exported or mapped (uncached or "
                           "fine-grained memory over IPC)");
    }
    for (int r = 0; r < P; r++) {
        hpccg_hip_matrix* Mr = Ms[r];
        HIP_TRY(hipSetDevice(Mr->device));
        if (!Mr->d_peers) HIP_TRY(hipMalloc(&Mr->d_peers, sizeof(double*) * kMaxGroupRanks));
        TRY(h2d(Mr, Mr->d_peers, tables[r].data(), sizeof(double*) * kMaxGroupRanks));
        Mr->peers_for = nr;
    }
    HIP_TRY(hipSetDevice(M->device));
    return 0;
}

// Option peer_allreduce auto (-1, the default): at creation, every rank of a
// job maps the others' mailboxes and runs kPeerTestRounds peer all-reduces of
// both scalars through the kernels' own code (k_peer_selftest, bounded waits),
// each checked bitwise on the host against the rank-ordered sum; when every
// rank passes, protocol_autotest runs the real iteration once more before the
// scalars are summed in the kernels from then on (the iteration is one launch
// with the fused update); otherwise RCCL's all-reduces stay (a host-bootstrapped
// job has no such fallback: its matrices are refused). Collective: every rank
// creates its matrix.
constexpr int kPeerTestRounds = 64;

int reset_dot_state(hpccg_hip_matrix* M);

// Option halo_pull auto (collective, at creation): every rank exports its r
// buffer (IPC handle of the allocation, the offset of local row 0 in it, its
// row count), maps its two neighbours', and tests a pull: each rank stores
// 0.5 g + 1 at every global row g of its first send_lo and last send_hi rows,
// the ranks meet, each pulls its ghost planes with the kernels' own k_pull and
// checks them on the host. Then protocol_autotest. Used only when every rank
// passes; otherwise r's planes stay on RCCL.
int pull_autotest(hpccg_hip_matrix* M)
{
    M->pull_auto_ok = 0;
    const int nr = M->nranks, me = M->rank;
    // r (the iteration's pull) and the x workspace (the prologue's p = x halo):
    // the IPC handle of each allocation and the offset of local row 0 in it
    double* const bufs[2] = {M->d_r, M->d_x};
    hipIpcMemHandle_t h[2];
    long long off[2] = {0, 0};
    std::memset(h, 0, sizeof h);
    int ok = M->d_rbuf != nullptr && M->d_x != nullptr;
    hipError_t e = hipSuccess;
    for (int i = 0; i < 2 && ok; i++) {
        void* base = nullptr;  // the allocation the handle maps (canary mode: before the buffer)
        size_t range = 0;
        if ((e = hipMemGetAddressRange(&base, &range, bufs[i])) != hipSuccess ||
            (e = hipIpcGetMemHandle(&h[i], base)) != hipSuccess) {
            M->selftest_note += std::string(i ? "x" : "r") + " hipIpcGetMemHandle: " + hipGetErrorString(e) + "; ";
            (void)hipGetLastError();
            ok = 0;
        }
        off[i] = (long long)((char*)bufs[i] - (char*)base);
    }
    const size_t hb = sizeof(hipIpcMemHandle_t), rec = 2 * hb + 24;  // handles | offsets (B) | nrow | ok
    std::vector<unsigned char> mine(rec, 0), all(rec * nr);
    std::memcpy(mine.data(), h, 2 * hb);
    std::memcpy(mine.data() + 2 * hb, off, 16);
    std::memcpy(mine.data() + 2 * hb + 16, &M->nrow, 4);
    std::memcpy(mine.data() + 2 * hb + 20, &ok, 4);
    TRY(comm_allgather(mine.data(), all.data(), rec));
    auto field = [&](int q, size_t at, void* out, size_t n) { std::memcpy(out, all.data() + rec * q + at, n); };
    int mapped = 1;
    for (int side = 0; side < 2 && mapped; side++) {
        const int q = side == 0 ? me - 1 : me + 1;
        const int need = side == 0 ? M->ghost_lo : M->ghost_hi;
        if (q < 0 || q >= nr || need == 0) continue;
        int qok = 0, qn = 0;
        long long qoff[2] = {0, 0};
        field(q, 2 * hb + 20, &qok, 4);
        field(q, 2 * hb + 16, &qn, 4);
        field(q, 2 * hb, qoff, 16);
        double* got[2] = {nullptr, nullptr};
        for (int i = 0; i < 2 && mapped; i++) {
            hipIpcMemHandle_t hq;
            field(q, i * hb, &hq, hb);
            void* ptr = nullptr;
            if (!qok || (e = hipIpcOpenMemHandle(&ptr, hq, hipIpcMemLazyEnablePeerAccess)) != hipSuccess) {
                M->selftest_note += "rank " + std::to_string(q) + "'s " + (i ? "x " : "r ") +
                                    (qok ? std::string("hipIpcOpenMemHandle: ") + hipGetErrorString(e)
                                         : std::string("not exported")) + "; ";
                (void)hipGetLastError();
                mapped = 0;
                break;
            }
            M->ipc_r_opened.push_back(ptr);
            got[i] = reinterpret_cast<double*>(static_cast<char*>(ptr) + qoff[i]);
        }
        if (side == 0) {
            M->d_pull_lo = got[0];
            M->d_pullx_lo = got[1];
            M->pull_lo_n = qn;
        } else {
            M->d_pull_hi = got[0];
            M->d_pullx_hi = got[1];
        }
    }
    int all_ok = 0;
    TRY(comm_min(mapped, &all_ok));
    if (all_ok) {
        // the test pattern in this rank's sent rows, then every rank pulls
        auto pattern = [&](long long g) { return 0.5 * (double)g + 1.0; };
        int good = 1;
        std::vector<double> v;
        for (int i = 0; i < M->send_lo; i++) v.push_back(pattern((long long)M->start_row + i));
        if (M->send_lo && h2d(M, M->d_r, v.data(), sizeof(double) * v.size())) good = 0;
        v.clear();
        for (int i = M->nrow - M->send_hi; i < M->nrow; i++) v.push_back(pattern((long long)M->start_row + i));
        if (M->send_hi && h2d(M, M->d_r + M->nrow - M->send_hi, v.data(), sizeof(double) * v.size())) good = 0;
        int dummy = 0;
        TRY(comm_min(1, &dummy));  // every rank's rows are in place
        const int lo = M->d_pull_lo ? M->ghost_lo : 0, hi = M->d_pull_hi ? M->ghost_hi : 0;
        std::vector<double> gl(lo), gh(hi);
        if (good) {
            CgArgs a = make_args(M, M->d_b, M->d_x, 2, 0.0);
            launch_pull(a, M->d_pull_lo ? M->d_pull_lo + M->pull_lo_n - lo : nullptr, M->d_r - M->ghost_lo, lo,
                        M->d_pull_hi, M->d_r + M->nrow, hi, M->stream, true);
            good = hipGetLastError() == hipSuccess;
        }
        if (good && lo && d2h(M->stream, gl.data(), M->d_r - lo, sizeof(double) * lo)) good = 0;
        if (good && hi && d2h(M->stream, gh.data(), M->d_r + M->nrow, sizeof(double) * hi)) good = 0;
        for (int i = 0; i < lo && good; i++) good = gl[i] == pattern((long long)M->start_row - lo + i);
        for (int i = 0; i < hi && good; i++) good = gh[i] == pattern((long long)M->start_row + M->nrow + i);
        if (!good) M->selftest_note += "pull pattern: the pulled ghost rows differ; ";
        TRY(comm_min(good, &all_ok));
        TRY(comm_min(1, &dummy));  // no rank clears its rows while another still pulls
        HIP_TRY(hipMemsetAsync(M->d_rbuf, 0, sizeof(double) * (size_t)M->pstride, M->stream));
        TRY(flush_stream(M));
    }
    if (!all_ok) {
        for (void* ptr : M->ipc_r_opened) (void)hipIpcCloseMemHandle(ptr);
        M->ipc_r_opened.clear();
        M->d_pull_lo = M->d_pull_hi = M->d_pullx_lo = M->d_pullx_hi = nullptr;
        return 0;
    }
    M->pull_auto_ok = 1;
    return 0;
}

int peer_autotest(hpccg_hip_matrix* M)
{
    M->peer_auto_ok = 0;
    const int nr = M->nranks;
    if (nr > kMaxGroupRanks) return 0;
    std::vector<double*> table(kMaxGroupRanks, nullptr);
    int all_ok = 0;
    TRY(map_peer_mailboxes(M, table, &all_ok));
    if (!all_ok) return 0;
    int ok = 1;
    if (!M->d_peers && hipMalloc(&M->d_peers, sizeof(double*) * kMaxGroupRanks) != hipSuccess) ok = 0;
    if (ok && h2d(M, M->d_peers, table.data(), sizeof(double*) * kMaxGroupRanks)) ok = 0;
    double* out = nullptr;
    if (ok && hipMalloc(&out, sizeof(double) * 2 * kPeerTestRounds) != hipSuccess) ok = 0;
    std::vector<double> got(2 * kPeerTestRounds);
    int err[kErrWords] = {kErrNone};
    if (ok) {  // (a rank that cannot run it leaves the others' waits to expire: they fail too)
        M->peers_for = nr;
        CgArgs a = make_args(M, M->d_b, M->d_x, 2, 0.0);
        a.peer_ar = 1;
        a.prank = M->rank;
        a.pranks = nr;
        a.mbox = M->d_mbox;
        a.peers = M->d_peers;
        const long long budget = std::min<long long>(200000000LL, M->spin_us * 100);  // at most 2 s
        launch_rearm(M->d_kst, M->d_partial, (int)M->npartial, (int)budget, M->stream);
        launch_peer_selftest(a, kPeerTestRounds, out, M->stream);
        ok = hipGetLastError() == hipSuccess;
        if (ok && d2h(M->stream, got.data(), out, sizeof(double) * got.size())) ok = 0;
        if (ok && d2h(M->stream, err, M->d_kst + kErrBase, sizeof err)) ok = 0;
    }
    (void)hipGetLastError();
    if (out) (void)hipFree(out);
    if (!ok) M->selftest_note += "peer test: could not run; ";
    if (ok && err[0] != kErrNone) M->selftest_note += "peer test: a wait gave up (code " + std::to_string(err[0]) + "); ";
    ok = ok && err[0] == kErrNone;
    for (int k = 0; k < kPeerTestRounds && ok; k++)
        for (int which = 0; which < 2; which++) {
            double want = 0.0;  // k_peer_selftest's contributions, summed in rank order
            for (int q = 0; q < nr; q++) want += (double)(q + 1) + 0.5 * k + 0.25 * which;
            if (std::memcmp(&want, &got[2 * k + which], sizeof want) != 0) {
                if (ok) M->selftest_note += "peer test: round " + std::to_string(k) + " summed wrong; ";
                ok = 0;
            }
        }
    TRY(comm_min(ok, &all_ok));
    TRY(reset_dot_state(M));  // the test's slots, and a rank's waits may have given up: every mailbox empty
    TRY(comm_min(1, &ok));    // no rank's next kernel stores into a mailbox before its owner has reset it
    M->peer_auto_ok = all_ok;
    return 0;
}

int solve_ranks(hpccg_hip_matrix* const* Ms, int P, const double* const* b_dev, double* const* x_dev, int max_iter,
                double tol, int* niters_out, double* normr_out, double* times, int print);

// The production protocol itself, after the peer and pull tests
// passed on every rank: a short solve of this matrix (kProtoIters iterations,
// a synthetic b and a nonzero x0) launch for launch as the solves will run it -- the peer
// all-reduce inside the kernels, r's boundary rows stored write-through and
// drained before the r.r partial, the neighbours' rows pulled by the
// iteration's last launch -- against the same solve with r's planes moved by
// RCCL (a host-bootstrapped job: by k_pull launches before each SpMV). Both
// must give the same bits (the scalars are summed the same way in both, only
// the plane transport differs), and every rank's trace must be every other
// rank's (all sum the same global dots). The auto modes stay on only if every
// rank passes; otherwise both fall back to RCCL.
constexpr int kProtoIters = 12;

int protocol_autotest(hpccg_hip_matrix* M, int* local_ok)
{
    *local_ok = 0;
    int ok = 1;
    const size_t np = M->npad;
    // b and x: the matrix's own workspace (x is the buffer the neighbours have
    // mapped for the prologue's pull); b = 1 + (global row mod 13) / 8
    // and x0 = ((global row mod 7) - 3) / 4, not zero: the prologue's p = x halo
    // carries values (pulled from the neighbours' x in the in-kernel form)
    std::vector<double> hb(np, 0.0), hx(np, 0.0);
    for (int i = 0; i < M->nrow; i++) {
        hb[i] = 1.0 + (double)(((long long)M->start_row + i) % 13) * 0.125;
        hx[i] = 0.25 * (double)(((long long)M->start_row + i) % 7 - 3);
    }
    if (h2d(M, M->d_b, hb.data(), sizeof(double) * np)) ok = 0;
    struct Run {
        int it = -1;
        double nr = 0.0;
        std::vector<double> trace, x;
    } run[2];
    const int hp0 = M->halo_pull, ug0 = M->use_graph;
    for (int v = 0; v < 2; v++) {  // every rank runs both solves: their RCCL calls and error exchanges are collective
        M->halo_pull = v == 0 ? 2 : (comm_host() ? 1 : 0);
        M->use_graph = 0;
        const double* b = M->d_b;
        double* x = M->d_x;
        if (h2d(M, x, hx.data(), sizeof(double) * np)) ok = 0;
        const int rc = solve_ranks(&M, 1, &b, &x, kProtoIters + 1, 0.0, &run[v].it, &run[v].nr, nullptr, 0);
        if (rc) ok = 0;
        run[v].trace = M->trace;
        run[v].x.assign(M->nrow, 0.0);
        if (rc == 0 && d2h(M->stream, run[v].x.data(), x, sizeof(double) * M->nrow)) ok = 0;
    }
    (void)hipGetLastError();
    M->halo_pull = hp0;
    M->use_graph = ug0;
    M->trace.clear();
    M->last_niters = 0;
    if (!ok) M->selftest_note += "protocol test: a solve failed (" + g_err + "); ";
    const bool ran = ok;
    ok = ok && run[0].it == kProtoIters && run[1].it == run[0].it &&
         std::memcmp(&run[0].nr, &run[1].nr, sizeof(double)) == 0 && run[0].trace.size() == run[1].trace.size() &&
         std::memcmp(run[0].trace.data(), run[1].trace.data(), sizeof(double) * run[0].trace.size()) == 0 &&
         std::memcmp(run[0].x.data(), run[1].x.data(), sizeof(double) * M->nrow) == 0;
    // every rank's trace is every other rank's
    unsigned long long hsh = 0x9e3779b97f4a7c15ULL;
    for (double t : run[0].trace) {
        unsigned long long bits;
        std::memcpy(&bits, &t, 8);
        hsh = (hsh ^ bits) * 0x100000001b3ULL;
    }
    std::vector<unsigned long long> hs(M->nranks);
    TRY(comm_allgather(&hsh, hs.data(), sizeof hsh));
    if (ran && !ok) M->selftest_note += "protocol test: the in-launch pull and the reference transport differ; ";
    for (unsigned long long q : hs)
        if (q != hsh && ok) {
            M->selftest_note += "protocol test: the ranks' traces differ; ";
            ok = 0;
        }
    // debug (the fallback tests): this rank reports a failed protocol test
    if (ok && std::getenv("HPCCG_DBG_FAIL_PROTO")) {
        M->selftest_note += "protocol test: failed on purpose (HPCCG_DBG_FAIL_PROTO); ";
        ok = 0;
    }
    *local_ok = ok;  // (the job's verdict: transport_verdict)
    return 0;
}

// After the protocol test passed on every rank: the persistent launch's
// multi-rank form (persist_multi_of) on the job's own devices -- a short
// solve of this matrix with it against the per-iteration launches, bitwise,
// every rank's blocks co-resident on its GPU for the whole launch (a launch
// that is not ends in a bounded wait: the solve fails, on every rank). Runs
// under the matrix's spin budget (a shorter one could expire while another
// rank's process still loads the kernel's code object); the verdict
// (comm_min) keeps the launch only where every rank passed. Debug:
// HPCCG_DBG_FAIL_PERSIST fails it here.
int persist_autotest(hpccg_hip_matrix* M, int* local_ok)
{
    *local_ok = 0;
    int ok = 1;
    const size_t np = M->npad;
    std::vector<double> hb(np, 0.0), hx(np, 0.0);
    for (int i = 0; i < M->nrow; i++) {
        hb[i] = 1.0 + (double)(((long long)M->start_row + i) % 11) * 0.25;
        hx[i] = 0.125 * (double)(((long long)M->start_row + i) % 5 - 2);
    }
    if (h2d(M, M->d_b, hb.data(), sizeof(double) * np)) ok = 0;
    struct Run {
        int it = -1, resident = 0;
        double nr = 0.0;
        std::vector<double> trace, x;
    } run[2];
    const int ru0 = M->resident_update, pa0 = M->persist_auto_ok, rf0 = M->resident_failed;
    for (int v = 0; v < 2; v++) {  // collective: every rank runs both solves
        M->resident_update = v == 0 ? 0 : -1;
        M->persist_auto_ok = v;
        M->resident_failed = 0;
        const double* b = M->d_b;
        double* x = M->d_x;
        if (h2d(M, x, hx.data(), sizeof(double) * np)) ok = 0;
        const int rc = solve_ranks(&M, 1, &b, &x, kProtoIters + 1, 0.0, &run[v].it, &run[v].nr, nullptr, 0);
        run[v].resident = M->resident_used;
        if (rc) {
            if (ok) M->selftest_note += "persistent test: a solve failed (" + g_err + "); ";
            ok = 0;
        }
        run[v].trace = M->trace;
        run[v].x.assign(M->nrow, 0.0);
        if (rc == 0 && d2h(M->stream, run[v].x.data(), x, sizeof(double) * M->nrow)) ok = 0;
    }
    (void)hipGetLastError();
    M->resident_update = ru0;
    M->persist_auto_ok = pa0;
    M->resident_failed = rf0;
    M->trace.clear();
    M->last_niters = 0;
    if (ok && run[1].resident != kResidentAuto) {
        M->selftest_note += "persistent test: not eligible on this rank (the chip cannot hold its blocks); ";
        ok = 0;
    }
    if (ok && !(run[0].it == kProtoIters && run[1].it == run[0].it &&
                std::memcmp(&run[0].nr, &run[1].nr, sizeof(double)) == 0 &&
                run[0].trace.size() == run[1].trace.size() &&
                std::memcmp(run[0].trace.data(), run[1].trace.data(), sizeof(double) * run[0].trace.size()) == 0 &&
                std::memcmp(run[0].x.data(), run[1].x.data(), sizeof(double) * M->nrow) == 0)) {
        M->selftest_note += "persistent test: the persistent and the per-iteration launches differ; ";
        ok = 0;
    }
    if (ok && std::getenv("HPCCG_DBG_FAIL_PERSIST")) {
        M->selftest_note += "persistent test: failed on purpose (HPCCG_DBG_FAIL_PERSIST); ";
        ok = 0;
    }
    *local_ok = ok;
    return 0;
}

// The reference's residual lines (HPCCG.cpp:342-344, 356, 372-373) from the
// solve's trace, rank 0 only.
void print_trace(const hpccg_hip_matrix* M, int niters, int max_iter)
{
    if (M->rank != 0) return;
    int pf = max_iter / 10;
    if (pf > 50) pf = 50;
    if (pf < 1) pf = 1;
    std::cout << "Initial Residual = " << M->trace[0] << std::endl;
    for (int k = 1; k <= niters; k++)
        if (k % pf == 0 || k + 1 == max_iter)
            std::cout << "Iteration = " << k << "   Residual = " << M->trace[k] << std::endl;
}

// After a failed solve: every dot slot empty again, the
// error record cleared, so the next solve starts from the allocation state.
int reset_dot_state(hpccg_hip_matrix* M)
{
    HIP_TRY(hipSetDevice(M->device));
    HIP_TRY(hipStreamSynchronize(M->stream));
    const std::vector<unsigned long long> empty(M->npartial, kSlotEmpty);
    HIP_TRY(hipMemcpyAsync(M->d_partial, empty.data(), M->npartial * sizeof(double), hipMemcpyHostToDevice, M->stream));
    if (M->d_mbox)
        HIP_TRY(hipMemcpyAsync(M->d_mbox, empty.data(), sizeof(double) * kMboxSlots, hipMemcpyHostToDevice, M->stream));
    TRY(clear_state(M));
    HIP_TRY(hipStreamSynchronize(M->stream));
    return 0;
}

// The device error record of every rank (err0: rank 0's, already on the host):
// a bounded wait that gave up voids the solve (HPCCG_HIP_EHIP). The reference
// aborts on a failed exchange (exchange_externals.cpp:119-125); this returns.
int check_device_error(hpccg_hip_matrix* const* Ms, int P, const int* err0)
{
    static const char* what[] = {"", "slice partials of a dot group", "group sums of a dot",
                                 "the p.Ap total (fused update)",
                                 "another rank's contribution (peer all-reduce)",
                                 "the launch's r.r completion (in-launch pull)"};
    static const char* where[] = {"", "group", "group", "ready slot", "slot (dot * 2 + parity)", "pull block"};
    int bad_rank = -1, e[kErrWords];
    for (int r = 0; r < P && bad_rank < 0; r++) {
        if (r == 0) {
            std::memcpy(e, err0, sizeof e);
        } else {
            HIP_TRY(hipSetDevice(Ms[r]->device));
            HIP_TRY(hipMemcpy(e, Ms[r]->d_kst + kErrBase, sizeof e, hipMemcpyDeviceToHost));
        }
        if (e[0] != kErrNone || (P == 1 && e[kErrAllRanks] != kErrNone)) bad_rank = r;
    }
    if (bad_rank < 0) return 0;
    for (int r = 0; r < P; r++) {
        Ms[r]->last_dev_err = e[0] != kErrNone ? e[0] : e[kErrAllRanks];
        Ms[r]->last_dev_err_all = e[kErrAllRanks];
    }
    for (int r = 0; r < P; r++) {
        TRY(reset_dot_state(Ms[r]));
        Ms[r]->solve_dirty = 0;  // reset here (a second reset at the next solve's start could empty a slot a
                                 // faster rank has already filled for it)
    }
    // a job's ranks all come here (the code is all-reduced): none starts its
    // next solve -- whose first contributions land in the others' mailboxes --
    // before every rank has emptied its own
    if (P == 1 && Ms[0]->nranks > 1 && !Ms[0]->in_group && comm_up()) {
        int dummy = 0;
        TRY(comm_min(1, &dummy));
    }
    HIP_TRY(hipSetDevice(Ms[0]->device));
    const int rank = Ms[bad_rank]->rank;
    if (e[0] == kErrNone)
        return set_err(HPCCG_HIP_EHIP, "rank %d: a device wait timed out on another rank (code %d); solve abandoned",
                       rank, e[kErrAllRanks]);
    return set_err(HPCCG_HIP_EHIP,
                   "rank %d: device wait timed out after %.0f us waiting for %s (block %d, %s %d, iteration %d, "
                   "dot %s); solve abandoned, dot slots reset",
                   rank, (double)Ms[bad_rank]->spin_us, e[0] > 0 && e[0] <= kErrPullWait ? what[e[0]] : "?", e[1],
                   e[0] > 0 && e[0] <= kErrPullWait ? where[e[0]] : "slot", e[2], e[3], e[4] == kPAP ? "p.Ap" : "r.r");
}

// Solve on the ranks Ms[0..P) (P > 1: an in-process group; P == 1: this
// process's matrix, exchanging through RCCL when the communicator has peers).
int solve_ranks(hpccg_hip_matrix* const* Ms, int P, const double* const* b_dev, double* const* x_dev, int max_iter,
                double tol, int* niters_out, double* normr_out, double* times, int print)
{
    hpccg_hip_matrix* M = Ms[0];
    std::vector<CgArgs> av(P);
    std::vector<hipEvent_t> gev;
    struct EvFree {
        std::vector<hipEvent_t>& v;
        ~EvFree()
        {
            for (hipEvent_t e : v) (void)hipEventDestroy(e);
        }
    } ev_free{gev};
    if (max_iter < 1) max_iter = 1;
    const int iters = max_iter - 1;
    const bool events = P == 1 && M->event_timing != 0;
    // a process's rank of a multi-rank job solves in its own x workspace: the
    // prologue's x pull reads the neighbours' d_x (xpull_of)
    if (P == 1 && M->nranks > 1 && !M->in_group && x_dev[0] != M->d_x)
        return set_err(HPCCG_HIP_EINVAL, "multi-rank solve: x must be staged in the matrix's x workspace");
    bool one_device = true;
    for (int r = 0; r < P; r++) {
        HIP_TRY(hipSetDevice(Ms[r]->device));
        TRY(ensure_hist(Ms[r], max_iter));
        Ms[r]->kernel = choose_kernel(Ms[r]);
        if (P == 1) TRY(ensure_pslots(Ms[r], max_iter));
        if (Ms[r]->device != M->device) one_device = false;
    }
    if (P > 1) {
        gev.resize(P + 1);
        for (int r = 0; r <= P; r++) {
            HIP_TRY(hipSetDevice(Ms[r < P ? r : 0]->device));
            HIP_TRY(hipEventCreateWithFlags(&gev[r], hipEventDisableTiming));
        }
    }
    HIP_TRY(hipSetDevice(M->device));
    TRY(ensure_peers(Ms, P));
    const auto t_begin = std::chrono::steady_clock::now();
    for (int r = 0; r < P; r++) {
        HIP_TRY(hipSetDevice(Ms[r]->device));
        av[r] = make_args(Ms[r], b_dev[r], x_dev[r], max_iter, tol);
        // the last solve returned an error part-way: the peer mailbox too
        if (Ms[r]->solve_dirty) TRY(reset_dot_state(Ms[r]));
        Ms[r]->solve_dirty = 1;
        // every solve starts from the same device state: iteration state,
        // error record and spin budget, every dot and ready slot empty,
        // (one stream-ordered launch)
        launch_rearm(Ms[r]->d_kst, Ms[r]->d_partial, (int)Ms[r]->npartial,
                     (int)std::min<long long>(Ms[r]->spin_us * 100, INT_MAX), Ms[r]->stream);
        HIP_TRY(hipMemsetAsync(Ms[r]->d_stamps, 0,
                               sizeof(unsigned long long) * (size_t)(max_iter + 2) * kNumStampSlots, Ms[r]->stream));
    }
    // the members' streams start after every member's reset (the group's
    // kernels read each other's buffers)
    if (P > 1) {
        for (int r = 0; r < P; r++) {
            HIP_TRY(hipSetDevice(Ms[r]->device));
            HIP_TRY(hipEventRecord(gev[r], Ms[r]->stream));
        }
        for (int r = 0; r < P; r++) {
            HIP_TRY(hipSetDevice(Ms[r]->device));
            for (int q = 0; q < P; q++)
                if (q != r) HIP_TRY(hipStreamWaitEvent(Ms[r]->stream, gev[q], 0));
        }
    }
    if (multi_of(M) && pull_of(M))
        for (int r = 0; r < P; r++) TRY(pull_plan(Ms, av.data(), P, r));
    // a host-bootstrapped job has no RCCL: the iteration must make no collective
    // call (the scalars summed in the kernels, r's planes pulled). Every rank
    // holds the same options unless the caller set them differently
    if (P == 1 && M->nranks > 1 && comm_host() && (av[0].allreduce || !av[0].rhalo || !pull_of(M) || !xpull_of(M, av[0])))
        return set_err(HPCCG_HIP_EINVAL,
                       "host-bootstrapped communicator: this solve would need RCCL (peer_allreduce %d, rhalo %d, "
                       "halo_pull %d, x pull %d): leave peer_allreduce, halo_pull, fuse_p and the kernel on auto",
                       av[0].peer_ar, av[0].rhalo, pull_of(M) ? 1 : 0, xpull_of(M, av[0]) ? 1 : 0);
    // group fold: RCCL-style group sums (no peer all-reduce), both dots folded
    if (P > 1 && av[0].allreduce && fold_of(av[0], kPAP) && fold_of(av[0], kRR)) {
        for (int f : {P - 1, 0}) {  // the folding members: p.Ap (the SpMV phase's last), r.r (the update's)
            hpccg_hip_matrix* L = Ms[f];
            HIP_TRY(hipSetDevice(L->device));
            if (!L->d_gtab) TRY(dev_alloc(L, &L->d_gtab, 2 * kMaxGroupRanks));
            L->h_gtab.assign(2 * P, nullptr);
            for (int r = 0; r < P; r++) {
                L->h_gtab[r] = av[r].loc;
                L->h_gtab[P + r] = av[r].g;
            }
            HIP_TRY(hipMemcpyAsync(L->d_gtab, L->h_gtab.data(), sizeof(double*) * 2 * P, hipMemcpyHostToDevice,
                                   L->stream));
            HIP_TRY(hipStreamSynchronize(L->stream));  // (pageable source: done before it can change)
            av[f].gtab = L->d_gtab;
        }
        for (int r = 0; r < P; r++) {
            av[r].gn = P;
            av[r].grank = r;
        }
        av[P - 1].gfw |= 1;
        av[0].gfw |= 2;
        // member P-1 folds p.Ap inside its SpMV launch, after every other
        // member's: with the direct kernel its update runs as trailing blocks of
        // that launch (the fused update; member 0's r.r fold also stores its
        // parity slot), one launch less per group iteration
        {
            hpccg_hip_matrix* L = Ms[P - 1];
            CgArgs& l = av[P - 1];
            if (L->fuse_update != 0 && L->kernel == kSpmvDirect && l.fuse_p && fold_effective(L) == 1 &&
                l.xdefer == 2)
                l.fupd = 1;
        }
        // the r-halo by pull: member 0's update, the iteration's last launch,
        // pulls every member's ghost planes once its r.r fold is in (every
        // other member's update ran before it): no k_pull launch per member
        if (multi_of(M) && pull_of(M) && !Ms[0]->general) {
            hpccg_hip_matrix* L = Ms[0];
            HIP_TRY(hipSetDevice(L->device));
            if (!L->d_pseg) TRY(dev_alloc(L, &L->d_pseg, 2 * kMaxGroupRanks));
            L->h_pseg.clear();
            long long rows = 0;
            for (int r = 0; r < P; r++) {
                if (av[r].pl_lo) L->h_pseg.push_back({av[r].pl_src_lo, av[r].pl_dst_lo, av[r].pl_lo});
                if (av[r].pl_hi) L->h_pseg.push_back({av[r].pl_src_hi, av[r].pl_dst_hi, av[r].pl_hi});
                rows += av[r].pl_lo + av[r].pl_hi;
            }
            if (!L->h_pseg.empty()) {
                HIP_TRY(hipMemcpyAsync(L->d_pseg, L->h_pseg.data(), sizeof(PullSeg) * L->h_pseg.size(),
                                       hipMemcpyHostToDevice, L->stream));
                HIP_TRY(hipStreamSynchronize(L->stream));
                for (int r = 0; r < P; r++) av[r].npseg = -1;  // pulled by member 0: no k_pull
                av[0].pull_in = 1;
                av[0].psegs = L->d_pseg;
                av[0].npseg = (int)L->h_pseg.size();
                av[0].pseg_rows = (int)rows;
            }
        }
    }
    for (int r = 0; r < P; r++) Ms[r]->gfold_used = av[0].gn > 0 ? 1 : 0;
    M->resident_used = av[0].resident;
    M->last_dev_err = M->last_dev_err_all = 0;
    const Ranks R{Ms, av.data(), P, gev.data()};
    if (events) TRY(ensure_events(M, iters + 1));
    TRY(enqueue_prologue(R, events));
    int done = 0;
    M->graph_used = 0;
    const bool persist = P == 1 && av[0].resident >= kResidentPersist;
    if (persist) {  // every iteration in one launch per window (k_cg_persist), its slots emptied first
        if (events && iters > 0) HIP_TRY(hipEventRecord(M->ev[4], M->stream));
        for (int k0 = 1; k0 == 1 || k0 <= iters; k0 += kPersistWindow) {
            CgArgs w = av[0];
            w.pk0 = k0;
            w.pk1 = k0 + kPersistWindow;
            launch_fill_empty(M->d_pslots, (long long)kPersistWindow * w.pslot_stride < M->pslots_cap
                                               ? (long long)kPersistWindow * w.pslot_stride
                                               : M->pslots_cap,
                              M->stream);
            launch_cg_persist(w, M->stream);
        }
        if (events && iters > 0) HIP_TRY(hipEventRecord(M->ev[5], M->stream));
        HIP_TRY(hipGetLastError());
        done = iters;
    }
    const int chunk = graph_chunk_of(R);
    // (an in-process group with the peer all-reduce: its members' kernels wait
    // for each other, so they are never serialised into one graph)
    if (!persist && !events && M->use_graph && !M->graph_failed && one_device && iters >= chunk &&
        !(P > 1 && av[0].peer_ar)) {
        // kernel arguments are baked into the graph: rebuild only when they change
        bool same = M->graph_exec && (int)M->graph_args.size() == P && M->graph_kernel == M->kernel &&
                    M->graph_chunk == chunk;
        for (int r = 0; same && r < P; r++) same = std::memcmp(&M->graph_args[r], &av[r], sizeof(CgArgs)) == 0;
        int rc = 0;
        if (!same) {
            rc = build_graph(R, chunk);
            if (rc == 0) {
                M->graph_args = av;
                M->graph_kernel = M->kernel;
            } else {
                // captured RCCL or peer copies refused here: eager launches from now on
                M->graph_failed = 1;
                std::fprintf(stderr, "hpccg_hip: hipGraph capture unavailable (%s); eager launches\n",
                             g_err.c_str());
            }
        }
        if (rc == 0) {
            HIP_TRY(hipSetDevice(M->device));
            // the graph runs every member's work from rank 0's stream: it starts
            // after the members' eager prologue, and their eager tail after it
            for (int r = 1; r < P; r++) {
                HIP_TRY(hipEventRecord(gev[r], Ms[r]->stream));
                HIP_TRY(hipStreamWaitEvent(M->stream, gev[r], 0));
            }
            for (; done + chunk <= iters; done += chunk) {
                if (done + 2 * chunk > iters && done > 0) {  // before the last chunk: wait_matrix sleeps to here
                    if (!M->ev_mid)
                        HIP_TRY(hipEventCreateWithFlags(&M->ev_mid, hipEventDisableTiming | hipEventBlockingSync));
                    HIP_TRY(hipEventRecord(M->ev_mid, M->stream));
                    M->mid_pending = 1;
                }
                HIP_TRY(hipGraphLaunch(M->graph_exec, M->stream));
            }
            if (P > 1) {
                HIP_TRY(hipEventRecord(gev[0], M->stream));
                for (int r = 1; r < P; r++) HIP_TRY(hipStreamWaitEvent(Ms[r]->stream, gev[0], 0));
            }
            M->graph_used = 1;
        }
    }
    for (; done < iters; done++) TRY(enqueue_iteration(R, events ? done + 1 : -1, done + 1));
    for (int r = P - 1; r >= 0; r--) {
        TRY(use_device(R, r));
        launch_cg_end(av[r], Ms[r]->stream);
        launch_cg_xflush(av[r], Ms[r]->stream);  // x += alpha_j p_j still pending (x_defer)
        HIP_TRY(hipGetLastError());
        if (r > 0) HIP_TRY(hipStreamSynchronize(Ms[r]->stream));
    }
    HIP_TRY(hipSetDevice(M->device));
    // an RCCL job: every rank learns whether any rank gave up a wait (err[7])
    if (P == 1 && M->nranks > 1 && !M->in_group && g_comm.comm)
        NCCL_TRY(ncclAllReduce(M->d_kst + kErrBase, M->d_kst + kErrBase + kErrAllRanks, 1, ncclInt32, ncclMax,
                               g_comm.comm, M->stream));
    // one batch of async copies into the pinned readback buffer, one wait:
    // the state, the scalars, the r.r history and (times) the stamps
    int* const kst = reinterpret_cast<int*>(M->h_rb);
    double* const scal = reinterpret_cast<double*>(M->h_rb + kRbScal);
    double* const hist = reinterpret_cast<double*>(M->h_rb + kRbHist);
    unsigned long long* const stamps =
        reinterpret_cast<unsigned long long*>(M->h_rb + kRbHist + sizeof(double) * (size_t)M->hist_cap);
    const size_t nstamps = (size_t)(max_iter + 2) * kNumStampSlots;
    HIP_TRY(hipMemcpyAsync(kst, M->d_kst, sizeof(int) * (kErrBase + kErrWords), hipMemcpyDeviceToHost, M->stream));
    HIP_TRY(hipMemcpyAsync(scal, M->d_scal, sizeof(double) * 8, hipMemcpyDeviceToHost, M->stream));
    if (max_iter > 0)
        HIP_TRY(hipMemcpyAsync(hist, M->d_hist, sizeof(double) * max_iter, hipMemcpyDeviceToHost, M->stream));
    if (times)
        HIP_TRY(hipMemcpyAsync(stamps, M->d_stamps, sizeof(unsigned long long) * nstamps, hipMemcpyDeviceToHost,
                               M->stream));
    TRY(wait_matrix(M));
    const auto t_end = std::chrono::steady_clock::now();
    // a host-bootstrapped job: every rank learns whether any rank gave up a wait
    // (after the wait: no rank starts its next solve before every rank's last
    // kernels have ended, so no mailbox slot of this solve is written late)
    if (P == 1 && M->nranks > 1 && !M->in_group && comm_host()) {
        std::vector<int> codes(M->nranks);
        TRY(comm_allgather(kst + kErrBase, codes.data(), sizeof(int)));
        kst[kErrBase + kErrAllRanks] = *std::max_element(codes.begin(), codes.end());
    }
    TRY(check_device_error(Ms, P, kst + kErrBase));
    // (the fused update keeps k in kst[0] / kst[2] by parity: the later one is the count)
    const int niters = std::max(0, (av[0].fupd ? std::max(kst[0], kst[2]) : kst[0]) - 1);
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
    if (events && persist) {
        // the prologue's two launches, then the persistent launch's time spread
        // evenly over its iterations (one SpMV-to-r.r period each)
        float ms0 = 0.f, ms1 = 0.f, msp = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms0, M->ev[0], M->ev[1]));
        HIP_TRY(hipEventElapsedTime(&ms1, M->ev[2], M->ev[3]));
        if (iters > 0) HIP_TRY(hipEventElapsedTime(&msp, M->ev[4], M->ev[5]));
        M->kiter.assign(2 * (size_t)(niters + 1), 0.0);
        M->kiter[0] = ms0;
        M->kiter[1] = ms1;
        for (int i = 1; i <= niters; i++) M->kiter[2 * i] = msp / niters;
        M->ktimes[0] = ms0 + msp;
        M->ktimes[1] = niters + 1;
        M->ktimes[2] = ms1;
        M->ktimes[3] = 1;
    } else if (events) {
        double sp = 0, up = 0;
        M->kiter.assign(2 * (size_t)(niters + 1), 0.0);
        for (int i = 0; i <= niters; i++) {
            float ms = 0.f;
            HIP_TRY(hipEventElapsedTime(&ms, M->ev[4 * i], M->ev[4 * i + 1]));
            sp += ms;
            M->kiter[2 * i] = ms;
            HIP_TRY(hipEventElapsedTime(&ms, M->ev[4 * i + 2], M->ev[4 * i + 3]));
            up += ms;
            M->kiter[2 * i + 1] = ms;
        }
        M->ktimes[0] = sp;
        M->ktimes[1] = niters + 1;
        M->ktimes[2] = up;
        M->ktimes[3] = niters + 1;
    }
    if (print) print_trace(M, niters, max_iter);
    if (times) {
        const std::vector<unsigned long long> st(stamps, stamps + nstamps);
        stamps_to_times(st, max_iter, times);
        times[0] = std::chrono::duration<double>(t_end - t_begin).count();
    }
    *niters_out = niters;
    *normr_out = normr;
    for (int r = 0; r < P; r++) Ms[r]->solve_dirty = 0;
    if (canary_on()) {  // debug mode: no store of this solve ran past a buffer
        std::string rep;
        const int bad = canary_check(&rep);
        if (bad) {
            std::fprintf(stderr, "hpccg_hip canary: %d tripped after a solve\n%s", bad, rep.c_str());
            return set_err(HPCCG_HIP_EHIP, "canary: %d tripped after a solve: %s", bad, rep.c_str());
        }
    }
    return 0;
}

// The resident fused update waits inside its launch for blocks HIP does not
// promise to run at the same time: with another process holding part of the
// GPU its p.Ap wait can expire. Such a solve is re-run from the caller's
// inputs with the unit + update-block launch, which needs no co-residency
// (every wait there is on blocks dispatched earlier).
// Every retry is counted (option resident_retries: the bench and the GPU
// suite require 0). After a retry the matrix tries the resident launch again
// at its next solve, until kResidentMaxRetries retries have happened; from
// then on it keeps the other launch (one stderr line says so each time).
constexpr int kResidentMaxRetries = 3;
bool resident_retry(hpccg_hip_matrix* M, int rc)
{
    // (the persistent launch waits on every block at each dot: any of its
    // waits; across ranks also the peer all-reduce's)
    const bool persist_wait = M->resident_used >= kResidentPersist &&
                              (M->last_dev_err == kErrGroupWait || M->last_dev_err == kErrTopWait ||
                               (M->nranks > 1 && M->last_dev_err == kErrPeerWait));
    bool want = rc == HPCCG_HIP_EHIP && M->resident_used && (M->last_dev_err == kErrReadyWait || persist_wait);
    if (M->nranks > 1 && !M->in_group && comm_up()) {
        // a job's ranks re-run together or not at all (every rank returned
        // EHIP: the error code is all-reduced); one rank's expired wait is
        // another's missing peer contribution
        // (a device wait gave up: every rank holds the same all-ranks code and
        // returned EHIP, so every rank comes here)
        int none = 1;
        if (rc != HPCCG_HIP_EHIP || M->last_dev_err_all == kErrNone || comm_min(want ? 0 : 1, &none)) return false;
        want = none == 0;
    }
    if (!want) return false;
    M->resident_failed = 1;
    M->resident_retries++;
    std::fprintf(stderr, "hpccg_hip: the resident launch's wait expired (a shared GPU?); the solve is re-run with "
                         "the unit + update-block launch (retry %d of this matrix%s)\n",
                 M->resident_retries,
                 M->resident_retries >= kResidentMaxRetries ? "; it keeps that launch from now on" : "");
    return true;
}
// After the re-run: the next solve tries the resident launch again, unless the
// retries ran out.
void resident_rearm(hpccg_hip_matrix* M)
{
    if (M->resident_retries < kResidentMaxRetries) M->resident_failed = 0;
}

int solve_impl(hpccg_hip_matrix* M, const double* b_dev, double* x_dev, int max_iter, double tol, int* niters_out,
               double* normr_out, double* times, int print)
{
    HIP_TRY(hipSetDevice(M->device));
    if (M->in_group && M->nranks > 1)
        return set_err(HPCCG_HIP_EINVAL, "group member: solve with hpccg_hip_group_solve");
    return solve_ranks(&M, 1, &b_dev, &x_dev, max_iter, tol, niters_out, normr_out, times, print);
}

// After the SELL-512 image is on the device: SELL-512-A (freeing SELL-512
// unless the general kernel still needs it or it is kept), the kernel, the
// workspace.
int finish_matrix(hpccg_hip_matrix* M)
{
    TRY(build_a_image(M));
    if (M->has_a && !g_keep_sell) drop_sell(M);
    M->kernel = choose_kernel(M);
    TRY(alloc_workspace(M));
    if (g_place_tries != 0 && !M->in_group && M->has_a) {
        const int tries =
            g_place_tries > 0 ? g_place_tries : ((double)M->a_slots * 8.0 >= kPlaceMinBytes ? kPlaceAuto : 0);
        if (tries) TRY(hpccg_hip_probe_placement(M, tries));
    }
    // a job's ranks (collective, after the probe: it may move r): the peer
    // all-reduce and the halo pull self-tests, then the production protocol
    // (protocol_autotest); every rank reaches the same verdicts
    if (M->nranks > 1 && !M->in_group && comm_up()) {
        const bool host = comm_host();
        // a host-bootstrapped job has no RCCL to fall back to: the r-halo
        // iteration (z-slab plan, SELL-512-A kernel with the p update fused) on
        // every rank, or the matrix is refused on every rank
        int can = 1;
        if (host) TRY(comm_min(rhalo_of(M) ? 1 : 0, &can));
        if (host && !can)
            return set_err(HPCCG_HIP_EPLAN, "host-bootstrapped communicator: a rank's matrix cannot run the r-halo "
                                            "iteration (z-slab plan and a SELL-512-A image are needed; RCCL serves "
                                            "the others)");
        const bool peer = M->peer_ar < 0 && (host || !std::getenv("HPCCG_NO_PEER_AUTO"));
        const bool pull = M->halo_pull != 0 && !M->general && (host || !std::getenv("HPCCG_NO_PULL_AUTO"));
        if (peer) TRY(peer_autotest(M));
        if (pull) TRY(pull_autotest(M));
        // (the peer and pull verdicts so far are every rank's)
        const bool both = peer && pull && M->peer_auto_ok && M->pull_auto_ok;
        int local[3] = {M->peer_auto_ok, M->pull_auto_ok, 0}, v[3] = {0, 0, 0};
        if (both) TRY(protocol_autotest(M, &local[2]));
        TRY(transport_verdict(local, v));  // collective: the same on every rank
        M->peer_auto_ok = v[0];
        M->pull_auto_ok = v[1];
        M->proto_auto_ok = v[2];
        if (both && !v[2]) {  // both fall back to RCCL
            for (void* ptr : M->ipc_r_opened) (void)hipIpcCloseMemHandle(ptr);
            M->ipc_r_opened.clear();
            M->d_pull_lo = M->d_pull_hi = M->d_pullx_lo = M->d_pullx_hi = nullptr;
        }
        // the persistent launch across the ranks: only after the protocol
        // passed everywhere (v[2] is every rank's), and only where its own
        // test passed on every rank
        M->persist_auto_ok = 0;
        if (v[2]) {
            M->persist_auto_ok = 1;  // (would the launch be taken on this rank?)
            const int elig = persist_ok(M) ? 1 : 0;
            M->persist_auto_ok = 0;
            int all = 0;
            TRY(comm_min(elig, &all));  // (7-pt, images the chip cannot hold: not tested, stays off)
            if (all) {
                int lp = 0;
                TRY(persist_autotest(M, &lp));
                TRY(comm_min(lp, &M->persist_auto_ok));
            }
        }
        if (host && !(M->peer_auto_ok && M->pull_auto_ok))
            return set_err(HPCCG_HIP_EPLAN, "host-bootstrapped communicator: the %s self-test failed on some rank "
                                            "(peer %d, pull %d, protocol %d); this transport needs all three. "
                                            "This rank: %s",
                           both ? "production-protocol" : !M->peer_auto_ok ? "peer all-reduce" : "halo pull",
                           M->peer_auto_ok, M->pull_auto_ok, M->proto_auto_ok,
                           M->selftest_note.empty() ? "passed" : M->selftest_note.c_str());
        if ((peer && !M->peer_auto_ok) || (pull && !M->pull_auto_ok))  // (an RCCL job falls back; say why)
            std::fprintf(stderr, "hpccg_hip rank %d: in-kernel transport off (peer %d, pull %d, protocol %d): %s\n",
                         M->rank, M->peer_auto_ok, M->pull_auto_ok, M->proto_auto_ok,
                         M->selftest_note.empty() ? "another rank failed" : M->selftest_note.c_str());
    }
    return 0;
}

template <class RowLen, class RowAt>
int create_from_rows(hpccg_hip_matrix** out, int nrow, int start_row, int total_nrow, RowLen row_len, RowAt row_at)
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
    TRY(make_streams(M));
    int mode = 1;
    std::vector<int> all;
    GatherPlan gp_local;
    const GatherPlan* gp = nullptr;
    TRY(exchange_plan(M, &mode, &all));
    if (mode == 2) {
        // gather plan: externals after the local rows (make_local_matrix.cpp:58-610)
        if (g_group_ctx.active) {
            gp = g_group_ctx.plan;
            if (!gp) return set_err(HPCCG_HIP_EPLAN, "group member without a gather plan");
        } else {
            gather_externals(nrow, start_row, all.data(), M->nranks, row_len, row_at, gp_local);
            TRY(rccl_requests(M, gp_local));
            gp = &gp_local;
        }
        TRY(install_gather(M, *gp));
    } else if (g_group_ctx.active && g_group_ctx.info && M->nranks > 1) {
        int sends[2];
        TRY(hpccg_slab_plan(M->nranks, M->rank, g_group_ctx.info, sends));
        M->send_lo = sends[0];
        M->send_hi = sends[1];
    }
    M->nslices = (nrow + kSliceRows - 1) / kSliceRows;
    M->grid = grid_of(M->nslices);
    const long long col_base = (long long)start_row - M->ghost_lo;
    const long long ncol_ext = (long long)M->ghost_lo + nrow + M->ghost_hi;
    std::vector<unsigned int> sb(M->nslices + 1);
    std::vector<int> hc;
    std::vector<double> hv;
    int bad = 0;
    auto build = [&](auto colmap) {
        const long long slots_var = sell_build_impl(nrow, colmap, row_len, row_at, sb.data(), nullptr, nullptr, 0, nullptr);
        const long long slots_uni = sell_build_impl(nrow, colmap, row_len, row_at, sb.data(), nullptr, nullptr, 1, nullptr);
        // uniform width when padding to the max costs < 4 % (stencils)
        M->uniform = (slots_uni <= slots_var + slots_var / 25) ? 1 : 0;
        M->nslots = sell_build_impl(nrow, colmap, row_len, row_at, sb.data(), nullptr, nullptr, M->uniform, nullptr);
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
    if (bad) return set_err(HPCCG_HIP_EPLAN, "column index outside the halo plan");
    TRY(dev_alloc(M, &M->d_slice_base, sb.size()));
    TRY(h2d(M, M->d_slice_base, sb.data(), sizeof(unsigned int) * sb.size()));
    TRY(dev_alloc(M, &M->d_cols, hc.size()));
    TRY(h2d(M, M->d_cols, hc.data(), sizeof(int) * hc.size()));
    TRY(dev_alloc(M, &M->d_vals, hv.size()));
    TRY(h2d(M, M->d_vals, hv.data(), sizeof(double) * hv.size()));
    M->has_sell = 1;
    TRY(finish_matrix(M));
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
        HIP_TRY(hipStreamCreateWithFlags(&g_scratch.s, hipStreamNonBlocking));
        HIP_TRY(hipMalloc(&g_scratch.out, sizeof(double) * 2));
    }
    if (nparts > g_scratch.cap) {
        if (g_scratch.partial) (void)hipFree(g_scratch.partial);
        HIP_TRY(hipMalloc(&g_scratch.partial, sizeof(double) * (nparts + 8)));
        g_scratch.cap = nparts;
    }
    return 0;
}

// ---- drop-in cache (hpccg_hip_HPCCG) ----------------------------------------
// A device matrix per caller HPC_Sparse_Matrix, keyed by its address AND a
// fingerprint of its contents (sizes, row lengths, every column index and
// value), so a matrix destroyed and re-created at the same address, or edited
// in place, is converted again instead of reusing a stale image.
struct DropinEntry {
    unsigned long long fp = 0;
    hpccg_hip_matrix* M = nullptr;
};
std::mutex g_dropin_mu;
std::map<const void*, DropinEntry> g_dropin_cache;

inline unsigned long long mix64(unsigned long long h, unsigned long long v)
{
    h ^= v + 0x9e3779b97f4a7c15ULL + (h << 6) + (h >> 2);
    return h * 0xff51afd7ed558ccdULL;
}

unsigned long long fingerprint(const HPC_Sparse_Matrix* A)
{
    const int n = A->local_nrow;
    unsigned long long head = mix64(0x1234, (unsigned long long)(unsigned)n);
    head = mix64(head, (unsigned long long)(unsigned)A->start_row);
    head = mix64(head, (unsigned long long)(unsigned)A->total_nrow);
    head = mix64(head, (unsigned long long)(unsigned)A->local_ncol);
    const int nth = std::max(1, std::min<int>(16, (int)std::thread::hardware_concurrency()));
    std::vector<unsigned long long> part(nth, 0);
    auto work = [&](int t) {
        const int r0 = (int)((long long)n * t / nth), r1 = (int)((long long)n * (t + 1) / nth);
        unsigned long long h = (unsigned long long)t;
        for (int i = r0; i < r1; i++) {
            const int len = A->nnz_in_row[i];
            h = mix64(h, (unsigned long long)(unsigned)len);
            const double* v = A->ptr_to_vals_in_row[i];
            const int* c = A->ptr_to_inds_in_row[i];
            for (int j = 0; j < len; j++) {
                unsigned long long bits;
                std::memcpy(&bits, v + j, 8);
                h = mix64(h, bits ^ ((unsigned long long)(unsigned)c[j] << 17));
            }
        }
        part[t] = h;
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nth; t++) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
    for (int t = 0; t < nth; t++) head = mix64(head, part[t]);
    return head;
}

}  // namespace

// ---- in-process rank group -------------------------------------------------
namespace {

template <class Make>
int group_make(int nranks, const int* devices, hpccg_hip_matrix** out, Make make, const int* info = nullptr,
               const std::vector<GatherPlan>* plans = nullptr)
{
    if (!out) return set_err(HPCCG_HIP_EINVAL, "out is NULL");
    if (nranks < 1 || nranks > kMaxGroupRanks) return set_err(HPCCG_HIP_EINVAL, "group size must be 1..%d", kMaxGroupRanks);
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
                rc = set_err(HPCCG_HIP_EHIP, "device %d cannot access device %d", out[r]->device, out[q]->device);
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

int hpccg_hip_abi_version(void) { return 2; }

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
    comm_reset();
    // a 1-rank communicator is created too (bootstrap + RCCL check on one GPU);
    // the solver still takes its single-rank path when nranks == 1
    ncclUniqueId uid;
    std::memcpy(&uid, id, 128);
    NCCL_TRY(ncclCommInitRank(&g_comm.comm, nranks, uid, rank));
    g_comm.nranks = nranks;
    g_comm.rank = rank;
    return 0;
}

int hpccg_hip_comm_init_host(int nranks, int rank, hpccg_hip_allgather_fn allgather, void* ctx)
{
    if (nranks < 1 || rank < 0 || rank >= nranks || !allgather)
        return set_err(HPCCG_HIP_EINVAL, "bad nranks/rank or no all-gather callback");
    comm_reset();
    g_comm.nranks = nranks;
    g_comm.rank = rank;
    g_comm.ag = allgather;
    g_comm.ag_ctx = ctx;
    // the callback is collective: every rank must see every rank in order
    std::vector<int> all(nranks, -1);
    int rc = comm_allgather(&rank, all.data(), sizeof rank);
    for (int q = 0; q < nranks && rc == 0; q++)
        if (all[q] != q) rc = set_err(HPCCG_HIP_EINVAL, "host all-gather: slot %d holds rank %d", q, all[q]);
    if (rc) comm_reset();
    return rc;
}

int hpccg_hip_comm_destroy(void)
{
    comm_reset();
    return 0;
}

int hpccg_hip_comm_mode(int* mode)
{
    if (!mode) return set_err(HPCCG_HIP_EINVAL, "mode is NULL");
    *mode = g_comm.comm ? 1 : (g_comm.ag ? 2 : 0);
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
    if (comm_host() && n > 0) {  // every rank's values, reduced in rank order
        std::vector<double> all((size_t)n * g_comm.nranks);
        TRY(comm_allgather(vals, all.data(), sizeof(double) * n));
        for (int i = 0; i < n; i++) {
            double v = op == 0 ? 0.0 : all[i];
            for (int q = 0; q < g_comm.nranks; q++) {
                const double w = all[(size_t)q * n + i];
                v = op == 0 ? v + w : op == 1 ? std::min(v, w) : std::max(v, w);
            }
            vals[i] = v;
        }
        return 0;
    }
    if (!g_comm.comm || n == 0) return 0;
    double* d = nullptr;
    hipStream_t s = nullptr;
    HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    HIP_TRY(hipMalloc(&d, sizeof(double) * n));
    TRY(h2d_stream(s, d, vals, sizeof(double) * n));
    const ncclRedOp_t ops[3] = {ncclSum, ncclMin, ncclMax};
    NCCL_TRY(ncclAllReduce(d, d, n, ncclFloat64, ops[op], g_comm.comm, s));
    HIP_TRY(hipStreamSynchronize(s));
    HIP_TRY(hipMemcpy(vals, d, sizeof(double) * n, hipMemcpyDeviceToHost));
    (void)hipFree(d);
    (void)hipStreamDestroy(s);
    return 0;
}

int hpccg_hip_transport_verdict(const int local[3], int verdict[3])
{
    if (!local || !verdict) return set_err(HPCCG_HIP_EINVAL, "NULL argument");
    if (!comm_up()) return set_err(HPCCG_HIP_EINVAL, "no communicator (hpccg_hip_comm_init / _init_host first)");
    return transport_verdict(local, verdict);
}

int hpccg_hip_runtime_info(int ints_out[6], char* pci_bus_id, int pci_cap, char* rccl_path, char* hip_path,
                           int path_cap)
{
    if (!ints_out) return set_err(HPCCG_HIP_EINVAL, "ints_out is NULL");
    int dev = 0, v = 0;
    HIP_TRY(hipGetDevice(&dev));
    ints_out[0] = ints_out[1] = 0;
    if (g_comm.comm) {
        NCCL_TRY(ncclCommCount(g_comm.comm, &ints_out[0]));
        NCCL_TRY(ncclCommUserRank(g_comm.comm, &ints_out[1]));
    }
    NCCL_TRY(ncclGetVersion(&v));
    ints_out[2] = v;
    HIP_TRY(hipRuntimeGetVersion(&v));
    ints_out[3] = v;
    HIP_TRY(hipDriverGetVersion(&v));
    ints_out[4] = v;
    ints_out[5] = dev;
    if (pci_bus_id && pci_cap > 0) HIP_TRY(hipDeviceGetPCIBusId(pci_bus_id, pci_cap, dev));
    // the files the RCCL and HIP entry points of this library resolved to
    auto where = [](const void* sym, char* out, int cap) {
        Dl_info di;
        if (!out || cap <= 0) return;
        if (dladdr(sym, &di) && di.dli_fname)
            std::snprintf(out, cap, "%s", di.dli_fname);
        else
            std::snprintf(out, cap, "?");
    };
    where(reinterpret_cast<const void*>(&ncclGetVersion), rccl_path, path_cap);
    where(reinterpret_cast<const void*>(&hipRuntimeGetVersion), hip_path, path_cap);
    return 0;
}

int hpccg_hip_device_name(char* buf, int cap, int* cus)
{
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, dev));
    if (buf && cap > 0) std::snprintf(buf, cap, "%s (%s)", prop.name[0] ? prop.name : "AMD Instinct GPU", prop.gcnArchName);
    if (cus) *cus = prop.multiProcessorCount;
    return 0;
}

int hpccg_hip_matrix_create(const HPC_Sparse_Matrix* A, hpccg_hip_matrix** out)
{
    if (!A) return set_err(HPCCG_HIP_EINVAL, "A is NULL");
    // A matrix that has been through make_local_matrix (make_local_matrix.cpp:
    // 595 sets local_ncol = local_nrow + num_external) holds LOCAL column
    // indices; this library plans the halo itself from global columns.
    if (A->local_ncol != A->local_nrow)
        return set_err(HPCCG_HIP_EPLAN,
                       "A has local_ncol %d != local_nrow %d: it has been through make_local_matrix (local column "
                       "indices); pass the matrix with global column indices (generate_matrix / read_HPC_row output)",
                       A->local_ncol, A->local_nrow);
    const int n = A->local_nrow;
    return create_from_rows(
        out, n, A->start_row, A->total_nrow, [A](int i) { return A->nnz_in_row[i]; },
        [A](int i, int j, long long* c, double* v) {
            *c = A->ptr_to_inds_in_row[i][j];
            *v = A->ptr_to_vals_in_row[i][j];
        });
}

int hpccg_hip_matrix_create_csr(int nrow, int start_row, int total_nrow, const long long* row_ptr, const int* cols,
                                const double* vals, hpccg_hip_matrix** out)
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
    if (!out) return set_err(HPCCG_HIP_EINVAL, "out is NULL");
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
    TRY(make_streams(M));
    TRY(exchange_plan(M));
    M->nslices = (n + kSliceRows - 1) / kSliceRows;
    M->grid = grid_of(M->nslices);
    // row lengths analytically (generate_matrix.cpp:259-281 acceptance test)
    auto axis = [](int i, int nn) { return 1 + (i > 0) + (i < nn - 1); };
    const long long total = (long long)n * size;
    const long long start = (long long)n * rank;
    auto row_len = [&](int lrow) -> int {
        const int iy = (lrow % nxy) / nx, ix = lrow % nx;
        const long long grow = start + lrow;
        const int zl = grow - nxy >= 0, zh = grow + nxy < total;
        if (use_7pt) return 1 + (ix > 0) + (ix < nx - 1) + (iy > 0) + (iy < ny - 1) + zl + zh;
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
    TRY(dev_alloc(M, &M->d_slice_base, sb.size()));
    TRY(h2d(M, M->d_slice_base, sb.data(), sizeof(unsigned int) * sb.size()));
    TRY(dev_alloc(M, &M->d_cols, (size_t)M->nslots));
    TRY(dev_alloc(M, &M->d_vals, (size_t)M->nslots));
    M->has_sell = 1;
    const size_t npad = std::max<size_t>(kSliceRows, (size_t)M->nslices * kSliceRows);
    TRY(dev_alloc(M, &M->d_gen_b, npad, true));
    TRY(dev_alloc(M, &M->d_gen_x0, npad, true));
    TRY(dev_alloc(M, &M->d_gen_xexact, npad, true));
    launch_generate(nx, ny, nz, rank, size, use_7pt, start - M->ghost_lo, M->d_slice_base, M->d_cols, M->d_vals,
                    M->d_gen_b, M->d_gen_xexact, n, M->stream);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(M->stream));
    TRY(finish_matrix(M));
    *out = guard.release();
    return 0;
}

int hpccg_hip_group_generate(int nx, int ny, int nz, int use_7pt, int nranks, const int* devices,
                             hpccg_hip_matrix** out)
{
    return group_make(nranks, devices, out,
                      [&](int, hpccg_hip_matrix** m) { return hpccg_hip_matrix_generate(nx, ny, nz, use_7pt, m); });
}

int hpccg_hip_group_create_csr(int nranks, const int* devices, const int* nrow, const int* start_row, int total_nrow,
                               const long long* const* row_ptr, const int* const* cols, const double* const* vals,
                               hpccg_hip_matrix** out)
{
    if (!nrow || !start_row || !row_ptr || !cols || !vals) return set_err(HPCCG_HIP_EINVAL, "NULL argument");
    if (nranks < 1 || nranks > kMaxGroupRanks) return set_err(HPCCG_HIP_EINVAL, "group size must be 1..%d", kMaxGroupRanks);
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
            gather_externals(
                nrow[r], start_row[r], info.data(), nranks, [rp](int i) { return (int)(rp[i + 1] - rp[i]); },
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

int hpccg_hip_group_solve(hpccg_hip_matrix* const* Ms, int nranks, const double* const* b_dev, double* const* x_dev,
                          int max_iter, double tolerance, int* niters, double* normr, double* times)
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
    // the kernels read whole 512-row slices: stage x (and b unless it is the
    // generated, padded b) through each member's padded workspace
    std::vector<const double*> bb(nranks);
    std::vector<double*> xx(nranks);
    for (int r = 0; r < nranks; r++) {
        hpccg_hip_matrix* M = Ms[r];
        HIP_TRY(hipSetDevice(M->device));
        HIP_TRY(hipMemcpyAsync(M->d_x, x_dev[r], sizeof(double) * M->nrow, hipMemcpyDeviceToDevice, M->stream));
        bb[r] = b_dev[r];
        if (b_dev[r] != M->d_gen_b && b_dev[r] != M->d_b) {
            HIP_TRY(hipMemcpyAsync(M->d_b, b_dev[r], sizeof(double) * M->nrow, hipMemcpyDeviceToDevice, M->stream));
            bb[r] = M->d_b;
        }
        xx[r] = M->d_x;
    }
    int rc = solve_ranks(Ms, nranks, bb.data(), xx.data(), max_iter, tolerance, niters, normr, times, 0);
    for (int r = 0; r < nranks && rc == 0; r++) {
        hpccg_hip_matrix* M = Ms[r];
        if (hipSetDevice(M->device) != hipSuccess ||
            hipMemcpyAsync(x_dev[r], M->d_x, sizeof(double) * M->nrow, hipMemcpyDeviceToDevice, M->stream) !=
                hipSuccess ||
            hipStreamSynchronize(M->stream) != hipSuccess)
            rc = set_err(HPCCG_HIP_EHIP, "copying x of member %d back failed", r);
    }
    (void)hipSetDevice(cur);
    return rc;
}

int hpccg_hip_set_halo_mode(int mode)
{
    if (mode < 0 || mode > 2) return set_err(HPCCG_HIP_EINVAL, "halo mode must be 0, 1 or 2");
    g_halo_mode = mode;
    return 0;
}

int hpccg_hip_set_keep_sell(int keep)
{
    g_keep_sell = keep ? 1 : 0;
    return 0;
}

int hpccg_hip_set_placement_probe(int tries)
{
    if (tries < -1 || tries > 16) return set_err(HPCCG_HIP_EINVAL, "placement probe: -1 (auto), 0 (off) or 1..16");
    g_place_tries = tries;
    return 0;
}

int hpccg_hip_matrix_destroy(hpccg_hip_matrix* M) { return free_matrix(M); }

int hpccg_hip_matrix_info(const hpccg_hip_matrix* M, long long info[8])
{
    if (!M || !info) return set_err(HPCCG_HIP_EINVAL, "NULL argument");
    info[0] = M->nrow;
    info[1] = (long long)M->ghost_lo + M->nrow + M->ghost_hi;
    info[2] = M->nnz;
    info[3] = M->has_a ? M->a_slots : M->nslots;
    info[4] = M->ghost_lo;
    info[5] = M->ghost_hi;
    info[6] = M->kernel;
    info[7] = M->has_a ? M->a_width : (M->uniform ? M->width : 0);
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

// Options (hpccg_hip.h documents each): twelve settings of the solve --
// use_graph, spmv_kernel, fuse_p, fold, x_defer, x_ring, fuse_update,
// resident_update, graph_chunk, a2_ring, peer_allreduce, halo_pull -- and
// diagnostics (event_timing, force_comm, spin_budget_us, dbg_*). Variants
// that measured even or slower than the defaults were removed (DESIGN.md 4,
// "What was dropped"); git history keeps them.
int hpccg_hip_set_option(hpccg_hip_matrix* M, const char* key, long long value)
{
    if (!M || !key) return set_err(HPCCG_HIP_EINVAL, "NULL argument");
    if (!std::strcmp(key, "use_graph")) {
        M->use_graph = (int)value;
    } else if (!std::strcmp(key, "event_timing")) {
        M->event_timing = (int)value;
    } else if (!std::strcmp(key, "fuse_p")) {
        M->fuse_p = value < 0 ? -1 : (value ? 1 : 0);
    } else if (!std::strcmp(key, "x_defer")) {
        if (value < 0 || value > 2)
            return set_err(HPCCG_HIP_EINVAL, "x_defer must be 0 (every iteration), 1 (batched in the update) or 2 "
                                             "(beside the SpMV)");
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
    } else if (!std::strcmp(key, "fuse_update")) {
        M->fuse_update = value < 0 ? -1 : (value > 2 ? 2 : (int)value);
    } else if (!std::strcmp(key, "resident_update")) {
        if (value < -1 || value > 1)
            return set_err(HPCCG_HIP_EINVAL, "resident_update: -1 (auto: the persistent launch where it fits), 0 off "
                                             "or 1 (the per-iteration resident launch only)");
        M->resident_update = (int)value;
        if (value) M->resident_failed = 0;
    } else if (!std::strcmp(key, "graph_chunk")) {
        if (value < 1 || value > 4096) return set_err(HPCCG_HIP_EINVAL, "graph_chunk must be 1..4096");
        M->graph_iters = (int)value;
    } else if (!std::strcmp(key, "fold")) {
        if (value < -1 || value > 1)
            return set_err(HPCCG_HIP_EINVAL, "fold must be -1 (auto: both dots in their producers), 1 or 0 (k_finalize)");
        M->fold = (int)value;
    } else if (!std::strcmp(key, "a2_ring")) {
        if (value != -1 && value != 0 && value != kA2RingDefault)
            return set_err(HPCCG_HIP_EINVAL, "a2_ring must be -1 (auto: %d), 0 (register loads) or %d", kA2RingDefault,
                           kA2RingDefault);
        M->a2_ring = value < 0 ? kA2RingDefault : (int)value;
    } else if (!std::strcmp(key, "force_comm")) {
        if (value < 0 || value > 2) return set_err(HPCCG_HIP_EINVAL, "force_comm is 0, 1 or 2");
        M->force_comm = (int)value;
    } else if (!std::strcmp(key, "spin_budget_us")) {
        if (value < 1 || value > 20000000LL) return set_err(HPCCG_HIP_EINVAL, "spin_budget_us must be 1..2e7");
        M->spin_us = value;
    } else if (!std::strcmp(key, "peer_allreduce")) {
        M->peer_ar = value < 0 ? -1 : (value ? 1 : 0);
    } else if (!std::strcmp(key, "halo_pull")) {
        // -1 auto, 0 off (the RCCL / peer-copy planes), 1 k_pull where possible, 2 in-launch where the
        // peer all-reduce runs (else 1); 3 (diagnostics, the 1-rank emulation): in-launch with no rows
        M->halo_pull = value < 0 ? -1 : (value > 3 ? 3 : (int)value);
    } else if (!std::strcmp(key, "dbg_timeline")) {
        if (value != 0 && value != 1) return set_err(HPCCG_HIP_EINVAL, "dbg_timeline must be 0 or 1");
        HIP_TRY(hipSetDevice(M->device));
        if (M->d_tl) {
            dev_free(M, &M->d_tl, (size_t)M->tl_units * kTlWords);
            M->tl_units = 0;
        }
        if (value) {
            M->tl_units = 3 * M->nslices + 1024;  // >= the blocks of any SpMV launch (units, side, ghost, update)
            TRY(dev_alloc(M, &M->d_tl, (size_t)M->tl_units * kTlWords, true));
        }  // the graph cache compares the kernel arguments: a changed dbg_tl re-captures
    } else if (!std::strcmp(key, "dbg_resident_stall")) {
        M->dbg_resident_stall = value ? 1 : 0;
    } else if (!std::strcmp(key, "dbg_withhold")) {
        if (value < 0 || value > M->nslices) return set_err(HPCCG_HIP_EINVAL, "dbg_withhold must be 0..nslices");
        M->dbg_withhold = (int)value;
    } else if (!std::strcmp(key, "spmv_kernel")) {
        if (value != -1 && !spmv_kernel_ok((int)value))
            return set_err(HPCCG_HIP_EINVAL, "spmv_kernel must be -1 (auto), 0 (SELL-512), 1 (SELL-512-A direct) or "
                                             "2 (SELL-512-A pair windows)");
        if (value >= 0 && !kernel_available(M, (int)value))
            return set_err(HPCCG_HIP_EINVAL, "spmv_kernel %lld: its image was not built for this matrix%s", value,
                           value == kSpmvSell ? " (hpccg_hip_set_keep_sell(1) before creation keeps SELL-512)" : "");
        M->kernel_opt = (int)value;
        M->kernel = choose_kernel(M);
    } else {
        return set_err(HPCCG_HIP_EINVAL, "unknown option '%s'", key);
    }
    return 0;
}

int hpccg_hip_get_option(const hpccg_hip_matrix* M, const char* key, long long* value)
{
    if (!M || !key || !value) return set_err(HPCCG_HIP_EINVAL, "NULL argument");
    if (!std::strcmp(key, "use_graph")) *value = M->use_graph;
    else if (!std::strcmp(key, "spmv_kernel")) *value = M->kernel;
    else if (!std::strcmp(key, "event_timing")) *value = M->event_timing;
    else if (!std::strcmp(key, "fuse_p")) *value = fuse_p_effective(M) ? 1 : 0;
    else if (!std::strcmp(key, "fold")) *value = fold_effective(M);
    else if (!std::strcmp(key, "x_defer")) *value = x_defer_effective(M);
    else if (!std::strcmp(key, "x_ring")) *value = x_ring_effective(M);
    else if (!std::strcmp(key, "fuse_update")) *value = fuse_update_effective(M) ? 1 : 0;
    else if (!std::strcmp(key, "resident_update"))
        *value = persist_ok(M) ? kResidentAuto : resident_of(M) ? 1 : 0;
    else if (!std::strcmp(key, "resident_retries")) *value = M->resident_retries;
    else if (!std::strcmp(key, "halo_mode")) *value = M->nranks == 1 ? 0 : (M->general ? 2 : 1);
    else if (!std::strcmp(key, "graph_chunk")) {  // effective: see graph_chunk_of
        long long c = std::max(1, M->graph_iters);
        if (fuse_update_effective(M)) c += c & 1;
        if (multi_of(M) && !rhalo_of(M)) {
            const long long ring = x_defer_effective(M) ? x_ring_effective(M) : (fuse_p_effective(M) ? 2 : 1);
            c = (c + ring - 1) / ring * ring;
        }
        *value = c;
    }
    else if (!std::strcmp(key, "graph_used")) *value = M->graph_used;
    else if (!std::strcmp(key, "force_comm")) *value = M->force_comm;
    else if (!std::strcmp(key, "spin_budget_us")) *value = M->spin_us;
    else if (!std::strcmp(key, "dbg_withhold")) *value = M->dbg_withhold;
    else if (!std::strcmp(key, "dbg_timeline")) *value = M->d_tl ? 1 : 0;
    else if (!std::strcmp(key, "peer_allreduce")) *value = peer_ar_of(M) ? 1 : 0;
    else if (!std::strcmp(key, "group_fold")) *value = M->gfold_used;
    else if (!std::strcmp(key, "rhalo")) *value = rhalo_of(M) ? 1 : 0;
    else if (!std::strcmp(key, "halo_pull")) {
        CgArgs a{};
        a.peer_ar = peer_ar_of(M) ? 1 : 0;
        a.fold = fold_effective(M);
        *value = pull_of(M) ? (pull_in_of(M, a) ? 2 : 1) : 0;
    }
    else if (!std::strcmp(key, "a2_ring")) *value = a2_ring_effective(M);
    else if (!std::strcmp(key, "nt_store")) *value = nt_store_effective(M) ? 1 : 0;
    else if (!std::strcmp(key, "num_external")) *value = M->general ? M->ghost_hi : M->ghost_lo + M->ghost_hi;
    else if (!std::strcmp(key, "has_sell")) *value = M->has_sell;
    else if (!std::strcmp(key, "has_a")) *value = M->has_a;
    else if (!std::strcmp(key, "a_reject")) *value = M->a_reject;
    else if (!std::strcmp(key, "has_pairs")) *value = M->has_pairs;
    else if (!std::strcmp(key, "a_width")) *value = M->a_width;
    else if (!std::strcmp(key, "lds_doubles")) *value = M->has_pairs ? M->alds2_doubles : 0;
    else if (!std::strcmp(key, "nt")) *value = nt_load_of(M) ? 1 : 0;
    else if (!std::strcmp(key, "device_bytes")) *value = M->bytes;
    else if (!std::strcmp(key, "placement_pick")) *value = M->place_pick;
    else if (!std::strcmp(key, "peer_auto_ok")) *value = M->peer_auto_ok;
    else if (!std::strcmp(key, "pull_auto_ok")) *value = M->pull_auto_ok;
    else if (!std::strcmp(key, "proto_auto_ok")) *value = M->proto_auto_ok;
    else if (!std::strcmp(key, "persist_auto_ok")) *value = M->persist_auto_ok;
    else return set_err(HPCCG_HIP_EINVAL, "unknown option '%s'", key);
    return 0;
}

int hpccg_hip_solve_device(hpccg_hip_matrix* M, const double* b_dev, double* x_dev, int max_iter, double tolerance,
                           int* niters, double* normr, double* times, int print)
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
    int rc = solve_impl(M, b, x, max_iter, tolerance, niters, normr, times, print);
    if (resident_retry(M, rc)) {  // from x_dev again
        HIP_TRY(hipMemcpyAsync(x, x_dev, sizeof(double) * M->nrow, hipMemcpyDeviceToDevice, M->stream));
        rc = solve_impl(M, b, x, max_iter, tolerance, niters, normr, times, print);
        resident_rearm(M);
    }
    TRY(rc);
    HIP_TRY(hipMemcpyAsync(x_dev, x, sizeof(double) * M->nrow, hipMemcpyDeviceToDevice, M->stream));
    return wait_matrix(M);
}

namespace {

// The caller's b and x into d_b / d_x: pageable copies straight from the
// caller's memory (the runtime moves them at ~56 GB/s on the box; a pinned
// stage filled by host threads measured 1-3 % slower per solve at 100^3 and
// 200^3, its extra host copy costing more than it saved).
int upload_host(hpccg_hip_matrix* M, const double* b, const double* x, bool with_b)
{
    if (with_b) HIP_TRY(hipMemcpyAsync(M->d_b, b, sizeof(double) * M->nrow, hipMemcpyHostToDevice, M->stream));
    HIP_TRY(hipMemcpyAsync(M->d_x, x, sizeof(double) * M->nrow, hipMemcpyHostToDevice, M->stream));
    HIP_TRY(hipStreamSynchronize(M->stream));
    return 0;
}

int download_x(hpccg_hip_matrix* M, double* x)
{
    HIP_TRY(hipMemcpy(x, M->d_x, sizeof(double) * M->nrow, hipMemcpyDeviceToHost));
    return 0;
}

// hpccg_hip_solve up to (not including) the copy of x back to the caller
int solve_host(hpccg_hip_matrix* M, const double* b, const double* x, int max_iter, double tolerance, int* niters,
               double* normr, double* times, int print)
{
    HIP_TRY(hipSetDevice(M->device));
    const auto t0 = std::chrono::steady_clock::now();
    TRY(upload_host(M, b, x, true));
    const double setup = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    int rc = solve_impl(M, M->d_b, M->d_x, max_iter, tolerance, niters, normr, times, print);
    if (resident_retry(M, rc)) {  // from the caller's x again
        TRY(upload_host(M, b, x, false));
        rc = solve_impl(M, M->d_b, M->d_x, max_iter, tolerance, niters, normr, times, print);
        resident_rearm(M);
    }
    TRY(rc);
    if (times) times[6] = setup;
    return 0;
}

}  // namespace

int hpccg_hip_solve(hpccg_hip_matrix* M, const double* b, double* x, int max_iter, double tolerance, int* niters,
                    double* normr, double* times, int print)
{
    if (!M || !b || !x || !niters || !normr) return set_err(HPCCG_HIP_EINVAL, "NULL argument");
    TRY(solve_host(M, b, x, max_iter, tolerance, niters, normr, times, print));
    return download_x(M, x);
}

int hpccg_hip_diag_spmv(hpccg_hip_matrix* M, int kernel, int reps, double* avg_us)
{
    if (!M || !avg_us || reps < 1) return set_err(HPCCG_HIP_EINVAL, "bad argument");
    const bool stream = kernel == kDiagStreamA && M->has_a;
    if (!stream && (!spmv_kernel_ok(kernel) || !kernel_available(M, kernel)))
        return set_err(HPCCG_HIP_EINVAL, "spmv_kernel %d is not available for this matrix", kernel);
    HIP_TRY(hipSetDevice(M->device));
    TRY(ensure_hist(M, 2));
    const int keep = M->kernel;
    if (!stream) M->kernel = kernel;  // make_args sizes the grid for that kernel
    CgArgs a = make_args(M, M->d_b, M->d_x, 2, 0.0);
    M->kernel = keep;
    auto launch = [&]() {
        if (stream)
            launch_stream_a(a, M->stream);
        else
            launch_cg_spmv(a, kernel, true, M->stream);
    };
    hipEvent_t e0, e1;
    HIP_TRY(hipEventCreate(&e0));
    HIP_TRY(hipEventCreate(&e1));
    launch();  // warm
    HIP_TRY(hipEventRecord(e0, M->stream));
    for (int i = 0; i < reps; i++) launch();
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

// Physical placement probe: the CG iteration rate of a large
// image depends on where in HBM its values and the p ring were placed (306-350
// us per 200^3 SpMV on one box, same code, same virtual layout). Time a few
// CG iterations on the creation placement and on `tries` candidate
// allocations (each allocated while the earlier ones are held, so each lands
// elsewhere), keep the fastest, free the rest. Values are copied, the ring is
// zeroed as alloc_ring leaves it; nothing else moves and no result changes.
// Off unless asked for (hpccg_hip_set_placement_probe / bench.py --placement).
// Round 3's contiguous candidates found the fast placements and corrupted
// other buffers (big_malloc); plain candidates are safe and rarely faster.
constexpr int kPlaceIters = 10;  // CG iterations per candidate (eager, event-timed)

// Median SpMV + update time (us) of iterations 2.. of a short eager solve on
// scratch b, x. A rank of an RCCL job or a group member is timed as one rank
// (no halo, no all-reduce: the probe must not make collective calls that the
// other ranks' probes might not match; the ghost rows it leaves unwritten are
// the ring's zeros).
int probe_time(hpccg_hip_matrix* M, const double* b, double* x, double* us)
{
    const int nr = M->nranks, ev = M->event_timing, gr = M->use_graph;
    M->nranks = 1;
    M->event_timing = 1;
    M->use_graph = 0;
    int it = 0;
    double normr = 0.0;
    int rc = 0;
    if (hipMemsetAsync(x, 0, sizeof(double) * M->npad, M->stream) != hipSuccess)
        rc = set_err(HPCCG_HIP_EHIP, "placement probe: hipMemsetAsync failed");
    if (!rc) rc = solve_ranks(&M, 1, &b, &x, kPlaceIters, 0.0, &it, &normr, nullptr, 0);
    M->nranks = nr;
    M->event_timing = ev;
    M->use_graph = gr;
    if (rc) return rc;
    std::vector<double> v;
    for (int i = 2; i <= it; i++) v.push_back(M->kiter[2 * i] + M->kiter[2 * i + 1]);
    if (v.empty()) return set_err(HPCCG_HIP_EINVAL, "placement probe: the solve ran %d iterations", it);
    std::nth_element(v.begin(), v.begin() + v.size() / 2, v.end());
    *us = 1e3 * v[v.size() / 2];
    return 0;
}

// The probe's candidates are plain allocations (big_malloc's reason). Only
// the diagnostics variant of the library (-DHPCCG_DIAG_CONTIG,
// tools/build_variant.sh) lets tools/diag_carry.py ask for others:
// HPCCG_PROBE_ALLOC = hipExtMallocWithFlags flags (4: contiguous -- this
// corrupted other buffers). HPCCG_PROBE_KEEP=1 holds the dropped candidates
// for the life of the process instead of freeing them.
static unsigned probe_alloc_flags()
{
#ifdef HPCCG_DIAG_CONTIG
    const char* e = std::getenv("HPCCG_PROBE_ALLOC");
    return e && *e ? (unsigned)std::atoi(e) : hipDeviceMallocDefault;
#else
    return hipDeviceMallocDefault;
#endif
}
static bool probe_keep()
{
    const char* e = std::getenv("HPCCG_PROBE_KEEP");
    return e && e[0] == '1';
}
static std::vector<double*> g_probe_held;

int hpccg_hip_probe_placement(hpccg_hip_matrix* M, int tries)
{
    if (!M) return set_err(HPCCG_HIP_EINVAL, "NULL argument");
    if (tries < 0 || tries > 16) return set_err(HPCCG_HIP_EINVAL, "tries must be 0..16");
    M->place_us.clear();
    M->place_pick = 0;
    if (!tries || !M->has_a || !M->d_aval || !M->d_pbuf) return 0;
    HIP_TRY(hipSetDevice(M->device));
    HIP_TRY(hipStreamSynchronize(M->stream));
    // b | x of the timed solves, each padded to npad rows like the solver's
    // own vectors (the slice kernels load whole slices)
    const size_t n = M->npad;
    double* scratch = nullptr;
    HIP_TRY(hipMalloc(&scratch, 2 * sizeof(double) * n));
    auto done = [&](int rc) {
        (void)flush_stream(M);  // the timed solves ran with the timing events (no system-scope release)
        (void)hipFree(scratch);
        (void)hipGetLastError();  // a refused candidate allocation only ends a phase
        M->trace.clear();         // the probe's solves are not the caller's
        M->last_niters = 0;
        M->kiter.clear();
        for (double& t : M->ktimes) t = 0.0;
        return rc;
    };
    // b: every 32-bit word 0x3ff00000 (each double ~1.0000002; only the rate matters)
    if (hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(scratch), 0x3ff00000u, 2 * n, M->stream) != hipSuccess)
        return done(set_err(HPCCG_HIP_EHIP, "placement probe: hipMemsetD32Async failed"));
    double us = 0.0;
    int rc = probe_time(M, scratch, scratch + n, &us);
    if (rc) return done(rc);
    M->place_us.push_back(us);
    double best_us = us;
    // phase 0 places the values (copied), 1 the p ring, 2 r, 3 Ap (zeroed, as
    // workspace allocation leaves them), each against the others' kept placement
    const ptrdiff_t poff = M->d_p - M->d_pbuf, roff = M->d_r - M->d_rbuf;
    for (int phase = 0; phase < kPlacePhases; phase++) {
        if (phase == 2 && M->pull_auto_ok) continue;  // the neighbours have this r mapped (halo_pull)
        double** const slots[kPlacePhases] = {&M->d_aval, &M->d_pbuf, &M->d_rbuf, &M->d_Ap};
        const size_t counts[kPlacePhases] = {(size_t)std::max<long long>(1, M->a_slots),
                                             (size_t)M->pstride * M->ring_alloc, (size_t)M->pstride, M->npad};
        double** slot = slots[phase];
        const size_t bytes = sizeof(double) * counts[phase];
        auto set = [&](double* q) {
            *slot = q;
            if (phase == 1) M->d_p = q + poff;
            if (phase == 2) M->d_r = q + roff;
        };
        std::vector<double*> cand{*slot};
        size_t best = 0;
        for (int t = 0; t < tries && !rc; t++) {
            size_t fr = 0, tot = 0;
            if (hipMemGetInfo(&fr, &tot) != hipSuccess || fr < bytes + (size_t(8) << 30)) break;  // headroom
            double* q = nullptr;
            if (big_malloc(reinterpret_cast<void**>(&q), bytes, probe_alloc_flags()) != hipSuccess)
                break;
            cand.push_back(q);
            const hipError_t e = phase == 0 ? hipMemcpyAsync(q, cand[0], bytes, hipMemcpyDeviceToDevice, M->stream)
                                            : hipMemsetAsync(q, 0, bytes, M->stream);
            if (e != hipSuccess) {
                rc = set_err(HPCCG_HIP_EHIP, "placement probe: filling candidate %d failed", t + 1);
                break;
            }
            set(q);
            rc = probe_time(M, scratch, scratch + n, &us);
            if (rc) break;
            M->place_us.push_back(us);
            if (us < best_us) {
                best_us = us;
                best = cand.size() - 1;
            }
        }
        if (rc) best = 0;
        (void)flush_stream(M);  // no launch reads the others any more, and nothing of theirs is left in cache
        set(cand[best]);
        for (size_t i = 0; i < cand.size(); i++)
            if (i != best) {
                if (probe_keep())
                    g_probe_held.push_back(cand[i]);  // diagnostics: never handed out again
                else
                    big_free(cand[i]);
            }
        if (phase > 0 && hipMemsetAsync(cand[best], 0, bytes, M->stream) != hipSuccess && !rc)
            rc = set_err(HPCCG_HIP_EHIP, "placement probe: hipMemsetAsync failed");  // the solves' values
        M->place_pick |= (int)best << (8 * phase);
        if (rc) break;
    }
    return done(rc);
}

int hpccg_hip_diag_placement(const hpccg_hip_matrix* M, double* us_out, int cap)
{
    if (!M || (!us_out && cap > 0)) return set_err(HPCCG_HIP_EINVAL, "NULL argument");
    const int n = (int)M->place_us.size();
    for (int i = 0; i < std::min(n, cap); i++) us_out[i] = M->place_us[i];
    return n;
}

// Diagnostics: a mapping through the VMM API at a chosen virtual alignment.
int vmm_alloc(hpccg_hip_matrix* M, size_t bytes, size_t align, double** out)
{
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = M->device;
    size_t gran = 0;
    HIP_TRY(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended));
    const size_t sz = (bytes + gran - 1) / gran * gran;
    // reserve align more and map at an aligned address inside (the
    // reservation's own alignment argument is not honoured above 2 MB here)
    align = std::max(align, gran);
    void* res = nullptr;
    HIP_TRY(hipMemAddressReserve(&res, sz + align, gran, nullptr, 0));
    const uintptr_t a0 = (reinterpret_cast<uintptr_t>(res) + align - 1) / align * align;
    void* va = reinterpret_cast<void*>(a0);
    hipMemGenericAllocationHandle_t h;
    HIP_TRY(hipMemCreate(&h, sz, &prop, 0));
    HIP_TRY(hipMemMap(va, sz, 0, h, 0));
    hipMemAccessDesc ad = {};
    ad.location = prop.location;
    ad.flags = hipMemAccessFlagsProtReadWrite;
    HIP_TRY(hipMemSetAccess(va, sz, &ad, 1));
    M->vmm.push_back({va, sz, h, res, sz + align});
    *out = static_cast<double*>(va);
    return 0;
}

int hpccg_hip_diag_realloc(hpccg_hip_matrix* M, int which, unsigned long long* va_out)
{
    if (!M) return set_err(HPCCG_HIP_EINVAL, "NULL argument");
    const int mode = which >> 8;
    which &= 255;
    HIP_TRY(hipSetDevice(M->device));
    HIP_TRY(hipStreamSynchronize(M->stream));
    double** buf;
    size_t n;
    switch (which) {
    case 0: buf = &M->d_aval; n = (size_t)std::max<long long>(1, M->a_slots); break;
    case 1: buf = &M->d_pbuf; n = (size_t)M->pstride * M->ring_alloc; break;
    case 2: buf = &M->d_rbuf; n = (size_t)M->pstride; break;
    case 3: buf = &M->d_Ap; n = M->npad; break;
    case 4: buf = &M->d_x; n = M->npad; break;
    default: return set_err(HPCCG_HIP_EINVAL, "which must be 0..4");
    }
    if (mode < 0 || mode > 6) return set_err(HPCCG_HIP_EINVAL, "mode must be 0..6");
#ifndef HPCCG_DIAG_CONTIG
    if (mode == 1)
        return set_err(HPCCG_HIP_EINVAL, "mode 1 (physically contiguous memory) exists only in the diagnostics "
                                         "variant of the library (-DHPCCG_DIAG_CONTIG): it corrupted other buffers");
#endif
    if (!*buf) return set_err(HPCCG_HIP_EINVAL, "buffer %d not allocated", which);
    // the neighbours pull from this r through their IPC mappings of it (halo_pull):
    // a moved r would leave them reading the old buffer
    if (which == 2 && M->pull_auto_ok)
        return set_err(HPCCG_HIP_EINVAL, "r cannot move: the neighbours have it mapped (halo_pull)");
    double* nb = nullptr;
    const size_t bytes = sizeof(double) * n;
    if (mode == 0) {
        HIP_TRY(big_malloc(reinterpret_cast<void**>(&nb), bytes));
#ifdef HPCCG_DIAG_CONTIG
    } else if (mode == 1) {
        HIP_TRY(big_malloc(reinterpret_cast<void**>(&nb), bytes, hipDeviceMallocContiguous));
#endif
    } else if (mode == 5) {  // fine-grained (coherent) device memory
        HIP_TRY(big_malloc(reinterpret_cast<void**>(&nb), bytes, hipDeviceMallocFinegrained));
    } else if (mode == 6) {
        HIP_TRY(big_malloc(reinterpret_cast<void**>(&nb), bytes, hipDeviceMallocUncached));
    } else {  // VMM at 2 MB, 64 MB or 1 GB virtual alignment
        const size_t align = mode == 2 ? (size_t(1) << 21) : mode == 3 ? (size_t(1) << 26) : (size_t(1) << 30);
        TRY(vmm_alloc(M, bytes, align, &nb));
    }
    HIP_TRY(hipMemcpyAsync(nb, *buf, bytes, hipMemcpyDeviceToDevice, M->stream));
    HIP_TRY(hipStreamSynchronize(M->stream));
    bool mapped = false;  // a VMM mapping is released at destroy, not hipFree'd
    for (const auto& v : M->vmm) mapped = mapped || v.va == *buf;
    if (!mapped) M->graveyard.push_back(*buf);  // held: the new buffer gets other physical memory
    const ptrdiff_t poff = M->d_p - M->d_pbuf, roff = M->d_r - M->d_rbuf;
    *buf = nb;
    if (which == 1) M->d_p = M->d_pbuf + poff;
    if (which == 2) M->d_r = M->d_rbuf + roff;
    if (va_out) *va_out = reinterpret_cast<unsigned long long>(nb);
    return 0;  // the graph cache compares kernel arguments: the next solve re-captures
}

int hpccg_hip_diag_canary_check(int* enabled, char* report, int cap)
{
    if (enabled) *enabled = canary_on() ? 1 : 0;
    std::string rep;
    const int bad = canary_check(&rep);
    if (report && cap > 0) std::snprintf(report, (size_t)cap, "%s", rep.c_str());
    return bad;
}

int hpccg_hip_diag_timeline(const hpccg_hip_matrix* M, unsigned long long* out, int cap)
{
    if (!M || !out) return set_err(HPCCG_HIP_EINVAL, "NULL argument");
    if (!M->d_tl) return set_err(HPCCG_HIP_EINVAL, "dbg_timeline is off");
    const int n = std::min(cap, M->tl_units);
    HIP_TRY(hipSetDevice(M->device));
    HIP_TRY(hipStreamSynchronize(M->stream));
    HIP_TRY(hipMemcpy(out, M->d_tl, (size_t)n * kTlWords * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    return n;
}

int hpccg_hip_diag_slot_plan(int units, int grid, int spu, int rev, int* last_unit, int cap, int* top_group)
{
    if (!last_unit || !top_group || units < 1) return set_err(HPCCG_HIP_EINVAL, "bad argument");
    const int ng = (units * spu + 63) / 64;
    if (ng > cap) return set_err(HPCCG_HIP_EINVAL, "cap %d < %d groups", cap, ng);
    const int r = slot_plan(units, grid, spu, rev, last_unit, top_group);
    if (r < 0) return set_err(HPCCG_HIP_EINVAL, "bad launch shape");
    return r;
}

int hpccg_hip_kernel_times(const hpccg_hip_matrix* M, double out[4])
{
    if (!M || !out) return set_err(HPCCG_HIP_EINVAL, "NULL argument");
    for (int i = 0; i < 4; i++) out[i] = M->ktimes[i];
    return 0;
}

int hpccg_hip_kernel_times_iter(const hpccg_hip_matrix* M, double* out, int cap)
{
    if (!M || !out) return set_err(HPCCG_HIP_EINVAL, "NULL argument");
    const int n = std::min<int>(cap, (int)(M->kiter.size() / 2));
    for (int i = 0; i < 2 * n; i++) out[i] = M->kiter[i];
    return n;
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
    if (M->in_group && M->nranks > 1) return set_err(HPCCG_HIP_EINVAL, "group member: the halo needs hpccg_hip_group_solve");
    TRY(ensure_hist(M, 1));  // the pack kernel stamps the halo class
    // stage x into p (the halo-carrying, guarded buffer), exchange, multiply
    HIP_TRY(hipMemcpyAsync(M->d_p, x_dev, sizeof(double) * M->nrow, hipMemcpyDeviceToDevice, M->stream));
    CgArgs a = make_args(M, nullptr, nullptr, 1, 0.0);
    if (M->general)
        TRY(enqueue_halo_gather(M, a, M->d_p, true));
    else if (comm_host() && g_comm.nranks > 1)
        TRY(host_halo(M, M->d_p));
    else
        TRY(enqueue_halo(M, M->d_p, M->stream));
    if (M->has_sell && (M->kernel == kSpmvSell || !M->has_a)) {
        launch_sparsemv(a, M->d_p - M->ghost_lo, y_dev, M->stream);
    } else {
        // SELL-512-A in prologue mode: Ap = A p (same row sums), then y = Ap
        CgArgs d = a;  // (every slice as a unit of the direct kernel, no side-flush blocks)
        d.s0 = 0;
        d.sn0 = M->nslices;
        d.s1 = d.sn1 = 0;
        d.sgrid = grid_of(M->nslices);
        d.xside = 0;
        launch_cg_spmv(d, kSpmvDirect, true, M->stream);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(y_dev, M->d_Ap, sizeof(double) * M->nrow, hipMemcpyDeviceToDevice, M->stream));
    }
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
    if (comm_host() && g_comm.nranks > 1) {  // every rank's local sum, added in rank order from 0.0
        double loc = 0.0;
        TRY(d2h(g_scratch.s, &loc, g_scratch.out, sizeof(double)));
        std::vector<double> all(g_comm.nranks);
        TRY(comm_allgather(&loc, all.data(), sizeof loc));
        double v = 0.0;
        for (double w : all) v += w;
        *result = v;
        return 0;
    }
    if (g_comm.nranks > 1)
        NCCL_TRY(ncclAllReduce(g_scratch.out, g_scratch.out + 1, 1, ncclFloat64, ncclSum, g_comm.comm, g_scratch.s));
    return d2h(g_scratch.s, result, g_scratch.out + (g_comm.nranks > 1 ? 1 : 0), sizeof(double));
}

int hpccg_hip_waxpby(int n, double alpha, const double* x_dev, double beta, const double* y_dev, double* w_dev)
{
    if (n < 0 || (n > 0 && (!x_dev || !y_dev || !w_dev))) return set_err(HPCCG_HIP_EINVAL, "bad argument");
    TRY(scratch_for(1));
    launch_waxpby(n, alpha, x_dev, beta, y_dev, w_dev, g_scratch.s);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(g_scratch.s));
    return 0;
}

int hpccg_hip_HPCCG(HPC_Sparse_Matrix* A, double* b, double* x, int max_iter, double tolerance, int* niters,
                    double* normr, double* times)
{
    if (!A || !b || !x || !niters || !normr) return set_err(HPCCG_HIP_EINVAL, "NULL argument");
    if (A->local_ncol != A->local_nrow)
        return set_err(HPCCG_HIP_EPLAN,
                       "A has local_ncol %d != local_nrow %d: it has been through make_local_matrix (local column "
                       "indices); pass the matrix with global column indices",
                       A->local_ncol, A->local_nrow);
    // A cached image is solved on at once, while host threads fingerprint A
    // (~23 ms at 200^3, 12 % of the solve); x is written back only if the
    // fingerprint still matches -- otherwise A changed since it was cached, and
    // the image is rebuilt and the solve run again from the caller's x.
    hpccg_hip_matrix* M = nullptr;
    unsigned long long cached_fp = 0;
    {
        std::lock_guard<std::mutex> lk(g_dropin_mu);
        auto it = g_dropin_cache.find(A);
        // (the sizes first: the speculative solve reads nrow values of b and x)
        if (it != g_dropin_cache.end() && it->second.M->nrow == A->local_nrow &&
            it->second.M->start_row == A->start_row && it->second.M->total_nrow == A->total_nrow)
            M = it->second.M, cached_fp = it->second.fp;
    }
    if (M) {
        unsigned long long fp = 0;
        std::thread fth;
        try {
            fth = std::thread([&] { fp = fingerprint(A); });
        } catch (const std::system_error&) {  // no thread to spare: fingerprint first
            fp = fingerprint(A);
        }
        const int rc = solve_host(M, b, x, max_iter, tolerance, niters, normr, times, 0);
        if (fth.joinable()) fth.join();
        if (fp == cached_fp) {
            TRY(rc);
            print_trace(M, *niters, max_iter);
            return download_x(M, x);
        }
        (void)hipGetLastError();
        g_err.clear();
    }
    double setup = 0.0;
    {
        std::lock_guard<std::mutex> lk(g_dropin_mu);
        const auto t0 = std::chrono::steady_clock::now();
        const unsigned long long fp = fingerprint(A);
        auto it = g_dropin_cache.find(A);
        if (it != g_dropin_cache.end() && it->second.fp == fp) {
            M = it->second.M;
        } else {
            if (it != g_dropin_cache.end()) {  // same address, other contents: a new matrix
                free_matrix(it->second.M);
                g_dropin_cache.erase(it);
            }
            TRY(hpccg_hip_matrix_create(A, &M));
            g_dropin_cache[A] = DropinEntry{fp, M};
        }
        setup = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    }
    TRY(hpccg_hip_solve(M, b, x, max_iter, tolerance, niters, normr, times, 1));
    if (times) times[6] += setup;
    return 0;
}

int hpccg_hip_dropin_release(const HPC_Sparse_Matrix* A)
{
    std::lock_guard<std::mutex> lk(g_dropin_mu);
    auto it = g_dropin_cache.find(A);
    if (it == g_dropin_cache.end()) return 0;
    free_matrix(it->second.M);
    g_dropin_cache.erase(it);
    return 1;
}

int hpccg_hip_dropin_cached(const HPC_Sparse_Matrix* A)
{
    std::lock_guard<std::mutex> lk(g_dropin_mu);
    return g_dropin_cache.count(A) ? 1 : 0;
}

long long hpccg_sell_build(int nrow, long long col_base, long long ncol_ext, const long long* row_ptr, const int* cols,
                           const double* vals, unsigned int* slice_base, int* sell_cols, double* sell_vals)
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
    const long long var =
        sell_build_impl(nrow, SlabCols{col_base, ncol_ext}, row_len, row_at, slice_base, nullptr, nullptr, 0, nullptr);
    const long long uni =
        sell_build_impl(nrow, SlabCols{col_base, ncol_ext}, row_len, row_at, slice_base, nullptr, nullptr, 1, nullptr);
    const int uniform = (uni <= var + var / 25) ? 1 : 0;
    int bad = 0;
    const long long r = sell_build_impl(nrow, SlabCols{col_base, ncol_ext}, row_len, row_at, slice_base, sell_cols,
                                        sell_vals, uniform, &bad);
    return bad ? HPCCG_HIP_EPLAN : r;
}

int hpccg_gather_plan(int nranks, const int* info, int nrow, int start_row, const long long* row_ptr, const int* cols,
                      int cap, int* ext_global, int* num_external, int* nrecv, int* recv_rank, int* recv_off,
                      int* recv_cnt)
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
    if (nranks < 1 || rank < 0 || rank >= nranks || !info || !sends) return set_err(HPCCG_HIP_EINVAL, "bad argument");
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
    if (sends[0] > nrow || sends[1] > nrow) return set_err(HPCCG_HIP_EPLAN, "rank %d: neighbour needs more rows than owned", r);
    return 0;
}

int hpccg_halo_plan(int nrow, int start_row, int total_nrow, const long long* row_ptr, const int* cols, int plan_out[4])
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
